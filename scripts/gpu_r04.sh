#!/bin/bash
# GPU-box session (round 4): the -m gpu suite, a default bench line, and the
# N = 2 rehearsal (two ranks sharing device 0 over gloo: the collective
# transport decision of bench.py's N > 1 path).  The first failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r04}"
mkdir -p "$O"
cd "$R"
git_rev=$(cat "$R/.commit" 2>/dev/null || echo unknown)
echo "$git_rev" > "$O/COMMIT"
if [ -n "${MB:-}" ]; then  # microbenchmarks built in-tree (build/)
  for m in $MB; do timeout -k 10 120 "./build/$m" > "$O/$m.txt" 2>&1; cat "$O/$m.txt"; done
fi
if [ -n "${MBSEG:-}" ]; then  # the C5 local-sort segment replays (scripts/mb_seg.sh)
  bash scripts/mb_seg.sh > "$O/mb_seg.txt" 2>&1; cat "$O/mb_seg.txt"
fi
if [ -n "${FIRST:-}" ]; then  # targeted tests first (fail fast)
  timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v -s --timeout 240 --timeout-method thread \
    > "$O/first_tests.log" 2>&1
  tail -2 "$O/first_tests.log"
fi
if [ -n "${PROBE:-}" ]; then  # diagnostic python scripts (scripts/*.py)
  for p in $PROBE; do timeout -k 10 300 python -u "scripts/$p.py" > "$O/$p.txt" 2>&1; cat "$O/$p.txt"; done
fi
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
  tail -2 "$O/gpu_tests.log"
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
  echo bench ok
fi
if [ -n "${N2:-}" ]; then
  LEGO_BENCH_SHARE_GPU=1 LEGO_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 \
    > "$O/bench_n2.json" 2> "$O/bench_n2.err"
  echo n2 ok
fi
if [ -n "${PROF:-}" ]; then
  PARTS="$PROF" TAG="${TAG}p" bash scripts/gpu_profile_r04.sh
  echo prof ok
fi
if [ -n "${ENVAB:-}" ]; then  # ENVAB="VAR A B"
  set -- $ENVAB
  VAR=$1 A=$2 B=$3 bash scripts/env_ab.sh > "$O/envab_$1.txt" 2>&1
  cat "$O/envab_$1.txt"
fi
if [ -n "${ENVAB5:-}" ]; then  # ENVAB5="VAR A B" on the C5 line
  set -- $ENVAB5
  VAR=$1 A=$2 B=$3 bash scripts/env_ab_c5.sh > "$O/envab5_$1.txt" 2>&1
  cat "$O/envab5_$1.txt"
fi
if [ -n "${NODEAB:-}" ]; then  # NODEAB="VAR VALUE": node-API latency, default (A) vs VAR=VALUE (B), alternating
  set -- $NODEAB
  for k in 1 2 3; do
    LABEL=A timeout -k 10 180 python -u scripts/ab_node.py >> "$O/ab_node.txt" 2>&1
    env "$1=$2" LABEL=B timeout -k 10 180 python -u scripts/ab_node.py >> "$O/ab_node.txt" 2>&1
  done
  cat "$O/ab_node.txt"
fi
if [ -n "${AB:-}" ]; then
  bash scripts/ab.sh > "$O/ab.txt" 2>&1
  cat "$O/ab.txt"
fi
echo done
