#!/bin/bash
# Round 6: fused-batch preset tests, then the N=2 rehearsal on one GPU
# (two ranks sharing device 0, gloo gather) whose stdout must be one JSON line.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r06q}"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_presets.py \
  > "$O/tests.log" 2>&1
LEGO_BENCH_SHARE_GPU=1 LEGO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu \
  --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0 > "$O/bench2.json" 2> "$O/bench2.err"
echo done
