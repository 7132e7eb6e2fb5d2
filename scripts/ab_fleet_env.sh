#!/bin/bash
# GPU-box A/B of an environment knob on the fleet line (fleet_probe, 256
# streams x 20 scans), alternating: KNOB=<name>, SETTINGS="0 1".
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2 3; do
  for v in ${SETTINGS:-0 1}; do
    env "$KNOB=$v" timeout -k 10 120 python scripts/fleet_probe.py --streams ${STREAMS:-256} --k 20 --steps 3 2>/dev/null \
      | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$KNOB=$v', round(d['scans_per_s']), round(d['ms_per_call'], 2))" || exit 1
  done
done
