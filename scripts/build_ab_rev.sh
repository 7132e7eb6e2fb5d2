#!/bin/bash
# Builds liblego_hip.so of a git revision into build/ab/<name> (for
# scripts/ab.sh: VARIANTS="<name> ..." times it against other builds on one
# box).  CPU side: a temporary worktree, the revision's own Makefile.
#   scripts/build_ab_rev.sh HEAD A        # the committed tree as variant A
#   scripts/build_ab_rev.sh WORK B        # the working tree as variant B
set -euo pipefail
cd "$(dirname "$0")/.."
REV="$1"; NAME="$2"
OUT="$(pwd)/build/ab/$NAME"
rm -rf "$OUT"
if [ "$REV" = WORK ]; then
  make -s -C lego-loam_amd -j8 OUT="$OUT" "$OUT/liblego_hip.so"
else
  WT="$(mktemp -d /tmp/lego_ab_XXXX)"
  git worktree add -q --detach "$WT" "$REV"
  make -s -C "$WT/lego-loam_amd" -j8 OUT="$OUT" "$OUT/liblego_hip.so"
  git worktree remove --force "$WT"
fi
ls -la "$OUT/liblego_hip.so"
