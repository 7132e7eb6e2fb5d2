#!/bin/bash
# GPU-box rehearsal of the N > 1 bench path on one GPU: two ranks share
# device 0 and gather over gloo (never the driver's configuration), plus a
# short N = 1 line.  Diagnostic.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-n2}"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python bench.py --no-cpu --fleet-streams 0 --dense-scans 0 --loop-scans 0 --mapping-steps 0 \
  > "$O/bench_n1.json" 2> "$O/bench_n1.err"
LEGO_BENCH_SHARE_GPU=1 LEGO_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 \
  > "$O/bench_n2.json" 2> "$O/bench_n2.err"
echo done
