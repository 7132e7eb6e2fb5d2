#!/bin/bash
# GPU-box session, step 2: rocprofv3 passes over the headline bench command
# (no mapping / fleet aux lines, so the kernel table is the C2 stream's):
# --kernel-trace --stats, then one pass per HBM counter (FETCH_SIZE,
# WRITE_SIZE; the guide's separate-pass rule).  The first failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
cd /tmp
B="$R/bench.py --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_stats" -o run \
  -- python3 $B > "$O/prof_stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
  -- python3 $B --steps 2 --warmup 1 > "$O/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
  -- python3 $B --steps 2 --warmup 1 > "$O/pmc_write.log" 2>&1
echo done
