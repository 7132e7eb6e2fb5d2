#!/bin/bash
# Mapping / VoxelGrid checks of this session: the C5, loop and hand-off GPU
# tests, then A/B of the fused LM iteration (LEGO_MO_UNFUSED=1: two kernels)
# on the C5 line and of the ring-per-wave VoxelGrid (LEGO_LFV_WAVE=0) on the
# fleet and C2 lines.
set -euo pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c5.py \
  tests/test_gpu_loop.py tests/test_gpu_handoff.py tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/t_mo.log 2>&1
C5="--no-cpu --steps 2 --warmup 1 --loop-scans 0 --dense-scans 0 --fleet-streams 0 --mapping-steps 15"
timeout -k 10 300 python bench.py $C5 > gpurun_out/c5only.log 2>&1
LEGO_MO_UNFUSED=1 timeout -k 10 300 python bench.py $C5 > gpurun_out/c5only_unf.log 2>&1
bash scripts/ab_lfv.sh
