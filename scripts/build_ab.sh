#!/bin/bash
# Builds two variants of liblego_hip.so for scripts/ab.sh: build/ab/A with
# the compile flags in A_FLAGS, build/ab/B with B_FLAGS (e.g. -DODOM_TOUCH=0).
# CPU side (hipcc cross-compiles); the variants travel with the snapshot.
set -euo pipefail
cd "$(dirname "$0")/../lego-loam_amd"
for v in A B; do
  f="${v}_FLAGS"
  rm -rf "../build/ab/$v"  # the flags are not a make dependency: rebuild every object
  make -s -j8 OUT=../build/ab/$v EXTRA="${!f:-}" ../build/ab/$v/liblego_hip.so
done
ls -la ../build/ab/*/liblego_hip.so
