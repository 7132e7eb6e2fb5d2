#!/bin/bash
# Round 6: k_lf_voxel's single-scan sort with the waves' segments: the sort
# permutation tests (modes 9 / 10 against std::sort), the product paths that
# run it, the sort timing of modes 8 / 10 and the bench line (node paths).
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort_perm.py tests/test_gpu_lfv_forms.py tests/test_gpu_node_overlap.py tests/test_gpu_parity.py tests/test_gpu_presets.py tests/test_gpu_voxel_grid.py tests/test_gpu_streams.py -m gpu -v --timeout 180 --timeout-method thread -rf > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/sort_time.py 8,10 > $O/sort_time.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo ok
# the fleet's k_odom phase split (stream 0's workgroup; stamps on)
timeout -k 10 200 python -u scripts/fleet_probe.py --streams 256 --k 20 --steps 2 --distinct 16 --extract-profile > gpurun_out/r06e/fleet_probe.json 2> gpurun_out/r06e/fleet_probe.err || exit 1
echo ok2
