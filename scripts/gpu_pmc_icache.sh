#!/bin/bash
# GPU-box: instruction-cache counters of the fleet's kernels over
# scripts/fleet_probe.py (one rocprofv3 pass).  The first failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-pmci}"
mkdir -p "$O"
cd /tmp
P="python3 $R/scripts/fleet_probe.py --streams 64 --steps 2"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  --output-format csv -d "$O/p1" -o run -- $P > "$O/p1.log" 2>&1
echo done
