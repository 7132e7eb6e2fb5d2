#!/bin/bash
# A/B of two library builds (GPU box) on the node path and the fleet line:
# scripts/ab_node.py (80 scans) and scripts/fleet_parts_ab.py (default parts,
# one round of 10 calls), alternating build/ab/base and build/ab/new, three
# rounds.  Diagnostic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2 3; do
  for v in base new; do
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so SCANS=80 LABEL=$v timeout -k 10 200 python scripts/ab_node.py || exit 1
  done
done
for r in 1 2; do
  for v in base new; do
    echo -n "$v fleet "
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so timeout -k 10 300 python scripts/fleet_parts_ab.py --rounds 1 --parts 2 | grep round || exit 1
  done
done
