#!/bin/bash
# GPU-box: the whole -m gpu suite (one process, per-test timeout), then smoke.
# TESTS overrides the selection.  The first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-tests}"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
tail -3 "$O/gpu_tests.log"
