#!/bin/bash
# C3 (HDL-64E) stage and odometry-phase breakdown on the GPU box.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-hdl}"
mkdir -p "$O"
cd "$R"
B="bench.py --sensor HDL-64E --batch 20 --stream-len 120 --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0"
timeout -k 10 300 python $B --stages > "$O/bench.json" 2> "$O/stages.txt"
timeout -k 10 300 python $B --odom-profile --steps 2 --warmup 1 > "$O/bench_prof.json" 2> "$O/prof.txt"
cat "$O/bench.json"
grep -v amdgpu "$O/stages.txt" | tail -16
grep -v amdgpu "$O/prof.txt"
