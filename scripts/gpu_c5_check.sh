#!/bin/bash
# GPU-box: the mapping tests, then the C5 line alone and its kernel trace.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-c5chk}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_loop.py tests/test_gpu_handoff.py \
  tests/test_gpu_parity.py tests/test_gpu_voxel_grid.py -k "c5 or loop or handoff or scan_to_map or keyframe or voxel or pcl or adversarial or nonfinite or overflow or forced" -m gpu -x -v -s --timeout 300 \
  --timeout-method thread > "$O/gpu_tests.log" 2>&1
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python bench.py --no-cpu --no-handoff --steps 1 --warmup 0 --fleet-streams 0 --dense-scans 0 \
  --loop-scans 0 --stream-len 100 --mapping-steps 15 > "$O/bench.json" 2> "$O/bench.err"
TAG=${TAG:-c5chk}/tr STEPS=3 bash "$R/scripts/gpu_c5_trace.sh"
echo done
