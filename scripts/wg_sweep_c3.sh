#!/bin/bash
# GPU box: C3 (HDL-64E, 20-scan batches) at several odometry workgroup counts
# per stream (LEGO_ODOM_WORKGROUPS, diagnostic override), two runs each.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2; do
  for g in ${WGS:-48 64 96 128 192}; do
    LEGO_ODOM_WORKGROUPS=$g timeout -k 10 120 python bench.py --no-cpu --mapping-steps 0 --fleet-streams 0 \
      --dense-scans 0 --loop-scans 0 --node-scans 0 --sensor HDL-64E --seed 2 --batch 20 --stream-len 200 \
      --steps 20 --warmup 4 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('G=$g', round(d['value']), round(d['roofline']['launch_ms'], 3), d['pose_delta_vs_oracle'])" || exit 1
  done
done
