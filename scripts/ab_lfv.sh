#!/bin/bash
# A/B of the ring-per-wave less-flat VoxelGrid (LEGO_LFV_WAVE=0: the block
# kernel for every ring), fleet and C2 lines, alternating on one box.
set -euo pipefail
O="--no-cpu --no-handoff --mapping-steps 0 --dense-scans 0 --loop-scans 0"
for r in 1 2; do
  for w in 1 0; do
    LEGO_LFV_WAVE=$w timeout -k 10 200 python bench.py $O > gpurun_out/ablfv_${w}_$r.log 2>&1
  done
done
echo done
