#!/bin/bash
# Node-path A/B of library builds (GPU box): scripts/ab_node.py with each of
# LIBS in turn, three rounds, SCANS scans (default 80).  Diagnostic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2 3; do
  for v in $LIBS; do
    LEGO_HIP_LIB_AB=$v SCANS=${SCANS:-80} LABEL=$(basename $(dirname $v)) timeout -k 10 200 python scripts/ab_node.py || exit 1
  done
done
