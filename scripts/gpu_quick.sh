#!/bin/bash
# Parity suite + profiled bench (odom phase stamps) on the GPU box.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-quick}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python bench.py --no-cpu --stages --loop-scans 0 --dense-scans 0 > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python bench.py --no-cpu --odom-profile --steps 2 --warmup 1 --loop-scans 0 --dense-scans 0 --fleet-streams 0 --mapping-steps 0 > "$O/bench_prof.json" 2> "$O/prof.txt"
cat "$O/bench.json"
grep -v amdgpu "$O/prof.txt"
