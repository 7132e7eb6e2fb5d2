#!/bin/bash
# GPU-box session for a profile refresh: the parity suite, smoke and the full
# bench line (gpu_check.sh), the rocprofv3 passes (gpu_profile.sh), the
# in-kernel odometry phase profile, a rocprofv3 kernel summary of the C5
# mapping steps, a kernel summary of the 64-stream fleet, and the FETCH_SIZE calibration of k_pixels' access pattern
# (scripts/mb/mb_gather.hip).  Every GPU step has its own limit; the first
# failure ends the session.
set -euo pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(pwd)}"
T="${TAG:-refresh}"
O="$R/gpurun_out/$T"
mkdir -p "$O" "$R/gpurun_out/${T}_q"
cd "$R"
TAG=$T bash scripts/gpu_check.sh
TAG=$T bash scripts/gpu_profile.sh
timeout -k 10 300 python bench.py --no-cpu --odom-profile --steps 2 --warmup 1 --loop-scans 0 --dense-scans 0 \
  --fleet-streams 0 --mapping-steps 0 > "$R/gpurun_out/${T}_q/bench_prof.json" 2> "$R/gpurun_out/${T}_q/prof.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5" -o run \
  -- python3 "$R/bench.py" --no-cpu --fleet-streams 0 --dense-scans 0 --loop-scans 0 --steps 1 --warmup 1 \
  --mapping-steps 5 > "$O/prof_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_fleet" -o run \
  -- python3 "$R/scripts/fleet_probe.py" --streams 256 --steps 3 > "$O/prof_fleet.log" 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_gather" -o run \
  -- "$R/build/mb_gather" > "$O/pmc_gather.log" 2>&1
echo done
