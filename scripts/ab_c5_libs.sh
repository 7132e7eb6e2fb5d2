#!/bin/bash
# A/B/... of library builds on the C5 mapping line alone (one box, alternating
# runs): LIBS="path1 path2 ...".  Prints the median ms per mapping step
# (per-step map mode) and with the map installed once, per build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2 3; do
for v in $LIBS; do
  LEGO_HIP_LIB_AB=$v timeout -k 10 180 python bench.py --no-cpu --steps 1 --warmup 0 --fleet-streams 0 --dense-scans 0 \
    --loop-scans 0 --node-scans 0 --stream-len 100 --mapping-steps 15 2>>"${AB_ERR:-/dev/null}" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['aux']['scan_to_map_c5']
print('$v', round(c['gpu_ms_per_step'], 3), round(c['gpu_ms_per_step_map_installed_once'], 3), c['iterations'])" || exit 1
done; done
