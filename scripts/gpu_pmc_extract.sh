#!/bin/bash
# GPU-box: LDS / instruction-mix counters of the fleet's kernels (k_extract
# first of all) over scripts/fleet_probe.py, one rocprofv3 pass per counter
# group.  The first failure ends the session.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-pmcx}"
mkdir -p "$O"
cd /tmp
P="python3 $R/scripts/fleet_probe.py --streams 64 --steps 2"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- $P > "$O/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU \
  --output-format csv -d "$O/p1" -o run -- $P > "$O/p1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$O/p2" -o run -- $P > "$O/p2.log" 2>&1
echo done
