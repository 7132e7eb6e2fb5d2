#!/bin/bash
# rocprofv3 kernel stats of the fleet line alone and the C2 line alone
# (TAG names the output directory under gpurun_out/).
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-pq}"
mkdir -p "$O"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/fleet" -o run \
  -- python3 "$R/bench.py" --no-cpu --no-handoff --steps 1 --warmup 0 --mapping-steps 0 --dense-scans 0 --loop-scans 0 --stream-len 100 > "$O/fleet.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c2" -o run \
  -- python3 "$R/bench.py" --no-cpu --no-handoff --steps 6 --warmup 1 --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 > "$O/c2.log" 2>&1
echo done
