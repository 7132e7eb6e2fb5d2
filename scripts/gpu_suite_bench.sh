#!/bin/bash
# GPU-box: the -m gpu suite, then a bench line (args in BENCH_ARGS).  The
# first failure ends the session.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-sb}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
tail -2 "$O/gpu_tests.log"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
echo done
