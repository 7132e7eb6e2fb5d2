#!/bin/bash
# Fleet A/B of two builds of liblego_hip.so on one box: build/ab/A and
# build/ab/B (or VARIANTS), alternating, ROUNDS rounds of
# scripts/fleet_opts_ab.py with the default options (one process per run).
# Diagnostic.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in ${VARIANTS:-A B}; do
    LEGO_HIP_LIB_AB=build/ab/$v/liblego_hip.so timeout -k 10 240 python scripts/fleet_opts_ab.py --settings "" \
      --rounds 1 --calls "${CALLS:-10}" 2>>"${AB_ERR:-/dev/null}" | sed "s/^/$v /" || exit 1
  done
done
