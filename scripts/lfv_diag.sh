#!/bin/bash
# Diagnostic build of liblego_hip.so with k_lf_voxel's sort output, voxel
# stores and counts checked in the kernel (LFV_DIAG: violations printed and
# the access skipped), for the register-form fault.
# CPU side; the build travels with the snapshot to build/diag/.
set -euo pipefail
cd "$(dirname "$0")/../lego-loam_amd"
rm -rf ../build/diag
make -s -j8 OUT=../build/diag EXTRA="-DLFV_DIAG=1 ${DIAG_FLAGS:-}" ../build/diag/liblego_hip.so
ls -la ../build/diag/liblego_hip.so
