#!/bin/bash
# GPU box: the C5 mapping VoxelGrids' local sorts replayed from segment files
# (scripts/mb/data, written from an oracle key dump), all segments at once and
# the deepest alone, with block 0's phase stamps; each binary in MBSEG_BINS
# (e.g. an old and a new build of the sort), then the ring-shaped and random
# whole-array checks against std::sort.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
D=scripts/mb/data
for b in ${MBSEG_BINS:-mb_vgsort}; do
  echo "== $b"
  for spec in "c5_map_surf_large 26" "c5_map_surf_small 26" "c5_outlier_large 22" "c5_total_large 21"; do
    set -- $spec
    [ -f "$D/$1.bin" ] || continue
    timeout -k 10 60 "./build/$b" seg "$D/$1.bin" "$2" 0
    timeout -k 10 60 "./build/$b" seg "$D/$1.bin" "$2" 1
  done
  timeout -k 10 120 "./build/$b" 1800 1536 3
done
