#!/bin/bash
# GPU-box session, step 2: one rocprofv3 pass over the headline bench command
# (no mapping / fleet aux lines, so the kernel table is the C2 stream's).
# MODE=stats: --kernel-trace --stats; MODE=fetch / write: one PMC counter.
# The profiler may exit 139 after writing its outputs (cooperative launch):
# the script reports that and ends; nothing else runs on the GPU after it.
set -uo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
cd /tmp
case "${MODE:-stats}" in
  stats) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_stats" -o run \
           -- python3 "$R/bench.py" --no-cpu --mapping-steps 0 --fleet-streams 0 > "$O/prof_stats.log" 2>&1 ;;
  fetch) timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
           -- python3 "$R/bench.py" --no-cpu --mapping-steps 0 --fleet-streams 0 --steps 2 --warmup 1 > "$O/pmc_fetch.log" 2>&1 ;;
  write) timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
           -- python3 "$R/bench.py" --no-cpu --mapping-steps 0 --fleet-streams 0 --steps 2 --warmup 1 > "$O/pmc_write.log" 2>&1 ;;
esac
rc=$?
echo "rocprofv3 exit $rc"
find "$O" -name "*.csv" | head -20
exit 0
