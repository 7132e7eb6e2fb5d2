#!/bin/bash
# C3 A/B over environment settings (GPU box): bench.py's C3 configuration
# alone for each setting in ENVS (space-separated; "-" = none), two rounds.
# Prints scans/s and the k_odom launch ms.  Diagnostic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OFF="--no-cpu --no-handoff --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0"
for r in 1 2; do
  for e in $ENVS; do
    env ${e/#-/LEGO_NONE=1} timeout -k 10 120 python bench.py $OFF --sensor HDL-64E --seed 2 --stream-len 200 --batch 20 \
      --steps 20 --warmup 3 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$e', round(d['value']), round(d['roofline']['launch_ms'], 3))" || exit 1
  done
done
