#!/bin/bash
# A/B timing of liblego_hip.so builds on the C3 (HDL-64E) stream on one box
# (alternating, three runs each): build/ab/<variant>.  Diagnostic.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2 3; do
  for v in ${VARIANTS:-A B}; do
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so timeout -k 10 120 python bench.py --sensor HDL-64E --batch 20 \
      --stream-len 120 --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), round(d['roofline']['launch_ms'], 3))" || exit 1
  done
done
