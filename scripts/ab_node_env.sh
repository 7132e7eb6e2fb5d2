#!/bin/bash
# Node-path A/B over environment settings (GPU box): scripts/ab_node.py (80
# scans) with each of ENVS (space-separated VAR=value; "-" = none), three
# rounds.  Diagnostic.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for r in 1 2 3; do
  for e in $ENVS; do
    env ${e/#-/LEGO_NONE=1} SCANS=${SCANS:-80} LABEL=$e timeout -k 10 200 python scripts/ab_node.py || exit 1
  done
done
