#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2; do
for g in ${GS:-16 20 24 28 32}; do
  LEGO_ODOM_WORKGROUPS=$g timeout -k 10 120 python bench.py --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('G=$g', round(d['value']), round(d['roofline']['launch_ms'], 3))" || exit 1
done; done
