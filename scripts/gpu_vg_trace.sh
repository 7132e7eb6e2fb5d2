#!/bin/bash
# GPU box: kernel trace of the C5 VoxelGrids one at a time (scripts/vg_probe.py)
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-vgtrace}"
mkdir -p "$O"
cd /tmp
REPS=${REPS:-2} SCANS=${SCANS:-2} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o run \
  -- python3 "$R/scripts/vg_probe.py" > "$O/probe.log" 2>&1
echo done
