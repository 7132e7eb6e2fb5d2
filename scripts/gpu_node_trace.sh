#!/bin/bash
# GPU box: kernel + copy trace of the node-API path (scripts/ab_node.py, SCANS scans)
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-nodetrace}"
mkdir -p "$O"
cd /tmp
SCANS=${SCANS:-30} LABEL=T timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/trace" -o run \
  -- python3 "$R/scripts/ab_node.py" > "$O/node.log" 2>&1
echo done
