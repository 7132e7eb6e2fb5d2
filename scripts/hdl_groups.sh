#!/bin/bash
# C3 (HDL-64E, seed 2, 200 scans) rate vs the odometry launch's workgroups.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for g in ${GS:-24 48 96 160}; do
  LEGO_ODOM_WORKGROUPS=$g timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.')
import bench
L = bench.load_ffi()
import torch; torch.cuda.init()
print($g, round(bench.dense_bench(L, 200, 20, 0)['scans_per_s']))
" 2>&1 | grep -v amdgpu | tail -1 || exit 1
done
