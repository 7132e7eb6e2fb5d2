#!/bin/bash
# A/B of one environment knob on the C2 headline (one box, alternating runs):
# VAR=<name> A=<value> B=<value> bash scripts/env_ab.sh.  Prints scans/s, the
# k_odom launch time and the fa.voxel stage per run (STEPS / WARMUP: bench's
# defaults unless set).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2 3; do
for v in "$A" "$B"; do
  env "$VAR=$v" timeout -k 10 120 python bench.py --steps ${STEPS:-6} --warmup ${WARMUP:-2} --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 \
    --loop-scans 0 --node-scans 0 2>>"${AB_ERR:-/dev/null}" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$VAR=$v', round(d['value']), round(d['roofline']['launch_ms'], 3),
      round(d.get('stages_ms_per_step', {}).get('fa.voxel', -1), 3))" || exit 1
done; done
