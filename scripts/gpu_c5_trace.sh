#!/bin/bash
# GPU-box: kernel trace (timestamps) of the C5 mapping line alone, for the
# per-step kernel timeline (scripts/c5_timeline.py reads it).
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-c5trace}"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run \
  -- python3 "$R/bench.py" --no-cpu --no-handoff --steps 1 --warmup 0 --fleet-streams 0 --dense-scans 0 \
  --loop-scans 0 --node-scans 0 --stream-len 100 --mapping-steps ${STEPS:-4} > "$O/bench.log" 2>&1
find "$O" -name '*kernel_trace.csv' | head -1
echo done
