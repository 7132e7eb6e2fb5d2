#!/bin/bash
# GPU-box profiling session (round 6).  Every pass profiles only the work of
# its line: bench.py with the other legs off and --no-handoff (no untimed
# mapping hand-off fetches; the warm-up steps are the only untimed kernels).
#   c2/      C2 headline: --kernel-trace --stats, then FETCH_SIZE and
#            WRITE_SIZE passes (one counter block per pass)
#   c3/      the same for the HDL-64E stream (seed 2, 20 scans per step)
#   fleet/   the fleet line alone (--kernel-trace --stats)
#   c5/      the C5 mapping line alone (--kernel-trace --stats)
#   node/    the node-API lines alone (VLP-16 and VLS-128, --kernel-trace --stats)
# The first failure ends it.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-r06p}"
mkdir -p "$O"
cd /tmp
OFF="--no-cpu --no-handoff --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0"
prof() {  # dir, bench args...
  local d="$1"; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$d/prof_stats" -o run \
    -- python3 "$R/bench.py" "$@" > "$O/$d/prof_stats.log" 2>&1
}
pmc() {  # dir, counter, bench args...
  local d="$1" c="$2"; shift 2
  local low
  low=$(echo "$c" | tr 'A-Z' 'a-z' | sed 's/_size//')
  timeout -k 10 300 rocprofv3 --pmc "$c" --output-format csv -d "$O/$d/pmc_$low" -o run \
    -- python3 "$R/bench.py" "$@" > "$O/$d/pmc_$low.log" 2>&1
}
mkdir -p "$O/c2" "$O/c3" "$O/fleet" "$O/c5" "$O/node"
C2="$OFF --steps 20 --warmup 2"
C3="$OFF --sensor HDL-64E --seed 2 --stream-len 200 --batch 20 --steps 8 --warmup 2"
PARTS="${PARTS:-c2 c3 fleet c5 node}"
if [[ " $PARTS " == *" c2 "* ]]; then
prof c2 $C2
pmc c2 FETCH_SIZE $OFF --steps 2 --warmup 1
pmc c2 WRITE_SIZE $OFF --steps 2 --warmup 1
fi
if [[ " $PARTS " == *" c3 "* ]]; then
prof c3 $C3
pmc c3 FETCH_SIZE $OFF --sensor HDL-64E --seed 2 --stream-len 200 --batch 20 --steps 2 --warmup 1
pmc c3 WRITE_SIZE $OFF --sensor HDL-64E --seed 2 --stream-len 200 --batch 20 --steps 2 --warmup 1
fi
if [[ " $PARTS " == *" fleet "* ]]; then
FL="--no-cpu --no-handoff --steps 1 --warmup 0 --mapping-steps 0 --dense-scans 0 --loop-scans 0 --node-scans 0 --stream-len 100"
prof fleet $FL
pmc fleet FETCH_SIZE $FL
pmc fleet WRITE_SIZE $FL
fi
if [[ " $PARTS " == *" c5 "* ]]; then
prof c5 --no-cpu --no-handoff --steps 1 --warmup 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --node-scans 0 --stream-len 100 --mapping-steps 15
fi
if [[ " $PARTS " == *" node "* ]]; then
prof node --no-cpu --no-handoff --steps 1 --warmup 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --mapping-steps 0 --stream-len 100 --node-scans 60
fi
if [[ " $PARTS " == *" phases "* ]]; then  # the in-kernel odometry phase stamps of the C2 line
  mkdir -p "$O/phases"
  cd "$R"
  timeout -k 10 300 python3 bench.py $OFF --steps 6 --warmup 2 --odom-profile > "$O/phases/bench.json" \
    2> "$O/phases/odom_phase_profile.txt"
  cd /tmp
fi
if [[ " $PARTS " == *" c5trace "* ]]; then
  TAG="${TAG}/c5t" bash "$R/scripts/gpu_c5_trace.sh"
fi
echo done
