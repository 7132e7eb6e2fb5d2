#!/bin/bash
# Round 6: k_ip_lds without the dead ground-image writes and with the pixel
# rows by reciprocal: projection parity subset (images, gated topics and
# batches), the fleet A/B of the builds, the phase profile.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r06t}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_presets.py tests/test_gpu_streams.py tests/test_gpu_c4.py > "$O/tests.log" 2>&1
ROUNDS=3 AB_ERR="$O/ab.err" bash scripts/ab_fleet_builds.sh > "$O/ab_fleet.txt"
LEGO_HIP_LIB_AB=build/prof/liblego_hip.so timeout -k 10 300 python scripts/ip_phase.py > "$O/ip_phase.txt" 2> "$O/ip_phase.err"
echo done
