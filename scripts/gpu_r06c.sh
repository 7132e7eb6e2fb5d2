set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -rf > gpurun_out/r06c/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r06c/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r06c/bench.json 2> gpurun_out/r06c/bench.err
