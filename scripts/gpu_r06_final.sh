#!/bin/bash
# Round-6 record at HEAD: the per-line profiles (scripts/gpu_profile_r06.sh),
# the full GPU suite, smoke() and the default bench line.  The first failure ends it.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
T="${TAG:-r06z}"
O="$R/gpurun_out/$T"
mkdir -p "$O"
TAG=$T PARTS="${PARTS:-c2 c3 fleet c5 node phases}" bash "$R/scripts/gpu_profile_r06.sh"
cd "$R"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
echo done
