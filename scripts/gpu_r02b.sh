set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_c4.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --cpu-budget 2 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
echo done
