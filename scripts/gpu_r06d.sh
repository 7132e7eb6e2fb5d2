#!/bin/bash
# Round 6: the fused projection kernel (k_ip_lds) against the four-kernel
# path: parity tests touching batches, then the fleet A/B (fleet_opts_ab.py).
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_c4.py tests/test_gpu_front_parts.py tests/test_gpu_branches.py -m gpu -v --timeout 180 --timeout-method thread -rf > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/fleet_opts_ab.py --settings "ip_fused=1;ip_fused=0" > $O/fleet_ab.txt 2> $O/fleet_ab.err || exit 1
echo ok
