#!/bin/bash
# Round 6: k_ip_lds pixel mapping + no bad-word fill: parity subset, then the
# fleet A/B of the two builds (build/ab/A = before, B = after) and one bench line.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r06f}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_front_parts.py tests/test_gpu_presets.py \
  tests/test_gpu_c4.py tests/test_golden.py > "$O/tests.log" 2>&1
ROUNDS=3 AB_ERR="$O/ab.err" bash scripts/ab_fleet_builds.sh > "$O/ab_fleet.txt"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
echo done
