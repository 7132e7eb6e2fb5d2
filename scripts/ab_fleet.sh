#!/bin/bash
# A/B fleet-aux timing of library builds on one box (diagnostic): build/ab/A
# vs build/ab/B, or the builds named in VARIANTS; STREAMS streams (256, the
# aux line's) x 20 scans per call.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in 1 2; do
  for v in ${VARIANTS:-A B}; do
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so timeout -k 10 120 python scripts/fleet_probe.py --streams ${STREAMS:-256} --k 20 --steps 3 2>/dev/null | tail -1 | sed "s/^/$v /" || exit 1
  done
done
