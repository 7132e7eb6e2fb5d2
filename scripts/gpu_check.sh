#!/bin/bash
# One GPU-box session: parity suite, smoke, bench line, rocprof kernel stats
# and the two HBM PMC passes for k_odom.  Every GPU step has its own time
# limit; the first failure ends the script (set -e).
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rA > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
timeout -k 10 300 python bench.py --stages > "$O/bench.json" 2> "$O/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_stats" -o run \
  -- python3 "$R/bench.py" --no-cpu > "$O/prof_stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
  -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 > "$O/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
  -- python3 "$R/bench.py" --no-cpu --steps 2 --warmup 1 > "$O/pmc_write.log" 2>&1
echo done
