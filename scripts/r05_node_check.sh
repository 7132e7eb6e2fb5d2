#!/bin/bash
# Round-5 node-path check (GPU box): the wave heap sort and the node call's
# side-stream VoxelGrid.  Parity subset, single-scan widths, node latency with
# and without the overlap, C2 A/B of build/ab/A vs B.  Diagnostic.
set -uo pipefail
O=gpurun_out/${TAG:-r05p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_perm.py \
  tests/test_gpu_lfv_forms.py tests/test_gpu_voxel_grid.py tests/test_gpu_parity.py tests/test_gpu_node_order.py \
  tests/test_gpu_ring_slots.py tests/test_gpu_handoff.py > $O/tests.txt 2>&1 || exit 1
LEGO_NODE_OVERLAP=0 timeout -k 10 300 python scripts/lfv_wide_ab.py > $O/lfv_wide.txt 2>&1 || exit 1
for v in 1 0 1 0; do
  LEGO_NODE_OVERLAP=$v SCANS=80 LABEL=ov$v timeout -k 10 200 python scripts/ab_node.py >> $O/node.txt 2>&1 || exit 1
done
AB_ARGS="--steps 20 --warmup 5" timeout -k 10 800 scripts/ab.sh > $O/c2_ab.txt 2>&1 || exit 1
