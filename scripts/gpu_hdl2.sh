#!/bin/bash
# C3 stream-position study: the HDL-64E stream's first vs later scans.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-hdl2}"
mkdir -p "$O"
cd "$R"
B="bench.py --sensor HDL-64E --batch 20 --no-cpu --mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0"
timeout -k 10 300 python $B --stream-len 120 --steps 4 --warmup 1 > "$O/a.json" 2> "$O/a.err"
timeout -k 10 300 python $B --stream-len 200 --steps 9 --warmup 1 --odom-profile > "$O/b.json" 2> "$O/b.err"
python3 -c "
import json
for f in ('a','b'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['roofline']['launch_ms'])
"
grep -v amdgpu "$O/b.err" | tail -22
