#!/bin/bash
# A/B headline timing of two builds of liblego_hip.so on one box (alternating,
# three runs each): build/ab/A and build/ab/B (or the builds named in
# VARIANTS; AB_ARGS: extra bench.py arguments, e.g. "--steps 20 --warmup 5").
# Diagnostic.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2 3; do
  for v in ${VARIANTS:-A B}; do
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so timeout -k 10 120 python bench.py --no-cpu --mapping-steps 0 \
      --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0 ${AB_ARGS:-} 2>>"${AB_ERR:-/dev/null}" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), round(d['roofline']['launch_ms'], 3))" || exit 1
  done
done
