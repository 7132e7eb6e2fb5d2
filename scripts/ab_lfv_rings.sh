#!/bin/bash
# GPU-box A/B of LEGO_LFV_BLOCK_RINGS (rings per large-ring workgroup of
# k_lf_voxel) on the fleet line, alternating settings on one box.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-abrings}"
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for k in ${SETTINGS:-1 4 2 8}; do
    LEGO_LFV_BLOCK_RINGS=$k timeout -k 10 200 python bench.py --no-cpu --no-handoff --steps 2 --warmup 1 \
      --mapping-steps 0 --dense-scans 0 --loop-scans 0 > "$O/b_${k}_${rep}.json" 2> /dev/null
    python3 -c "import json,sys; d=json.loads(open('$O/b_${k}_${rep}.json').read().strip().splitlines()[-1]); print('rings', $k, 'fleet', round(d['aux']['fleet_vlp16']['scans_per_s']), 'c2', round(d['value']))"
  done
done
