#!/bin/bash
# GPU-box: instruction-cache and wait counters of the C2 bench command
# (k_odom dominates it; one rocprofv3 pass).  The first failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-pmcio}"
mkdir -p "$O"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  --output-format csv -d "$O/p1" -o run -- python3 "$R/bench.py" --no-cpu --mapping-steps 0 --fleet-streams 0 \
  --dense-scans 0 --loop-scans 0 --steps 2 --warmup 1 > "$O/p1.log" 2>&1
echo done
