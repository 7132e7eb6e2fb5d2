#!/bin/bash
# GPU-box session, step 1: parity suite, smoke and the bench line (with the
# CPU baselines).  Every GPU step has its own time limit; the first failure
# ends the script (set -e).  The profiles are separate calls
# (scripts/gpu_profile.sh): rocprofv3 exits with SIGSEGV after writing its
# outputs when the program used a cooperative launch.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rA > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
timeout -k 10 400 python bench.py --stages > "$O/bench.json" 2> "$O/bench.err"
echo done
