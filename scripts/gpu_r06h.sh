#!/bin/bash
# Round 6: the node call's single-pass check + staged upload.  Node-path GPU
# tests, then the node A/B of the two builds on VLP-16 and VLS-128.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r06h}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_presets.py tests/test_gpu_node_order.py tests/test_gpu_node_overlap.py \
  tests/test_gpu_handoff.py tests/test_golden.py > "$O/tests.log" 2>&1
LIBS="build/ab/A/liblego_hip.so build/ab/B/liblego_hip.so" SCANS=80 bash scripts/ab_node_libs.sh > "$O/ab_vlp16.txt" 2>>"$O/ab.err"
SENSOR=VLS-128 SEED=3 LIBS="build/ab/A/liblego_hip.so build/ab/B/liblego_hip.so" SCANS=30 bash scripts/ab_node_libs.sh > "$O/ab_vls128.txt" 2>>"$O/ab.err"
echo done
