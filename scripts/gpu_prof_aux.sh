#!/bin/bash
# GPU-box: rocprofv3 kernel stats of the C5 mapping aux line and of the fleet
# aux line, each alone (bench.py with the other legs off).  First failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-aux}"
mkdir -p "$O"
cd /tmp
B="$R/bench.py --no-cpu --steps 2 --warmup 1 --loop-scans 0 --dense-scans 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5" -o run \
  -- python3 $B --fleet-streams 0 --mapping-steps ${C5_STEPS:-15} > "$O/c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/fleet" -o run \
  -- python3 $B --fleet-streams 256 --mapping-steps 0 > "$O/fleet.log" 2>&1
echo done
