#!/bin/bash
# C5 A/B (GPU box): bench.py's scan-to-map line alone, alternating the
# environment settings in AB_ENVS (default: the partition rounds persistent /
# four launches a round), three runs each.  Prints per-step and installed-map
# medians (ms).  Diagnostic.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2 3; do
  for e in ${AB_ENVS:-LEGO_VG_PERSIST=1 LEGO_VG_PERSIST=0}; do
    env $e timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 --mapping-steps ${C5_STEPS:-20} \
      --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0 2>>"${AB_ERR:-/dev/null}" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['aux']['scan_to_map_c5']
print('$e', round(d['gpu_ms_per_step'], 3), round(d['gpu_ms_per_step_map_installed_once'], 3))" || exit 1
  done
done
