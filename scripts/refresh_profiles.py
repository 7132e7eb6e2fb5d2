#!/usr/bin/env python3
"""Copies one GPU session's evidence (scripts/gpu_check.sh + gpu_profile.sh
under gpurun_out/<tag>, the phase profile of gpu_quick.sh under
gpurun_out/<tag>_q) into profiles/r01_* and prints the numbers DESIGN.md
quotes.  Usage: refresh_profiles.py <tag>"""
import json
import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
src = REPO / "gpurun_out" / tag
prof = REPO / "profiles"
shutil.copy(src / "bench.json", prof / "r01_bench.json")
shutil.copy(src / "gpu_tests.log", prof / "r01_gpu_tests.log")
shutil.copy(src / "prof_stats" / "run_kernel_stats.csv", prof / "r01_kernel_stats.csv")
subprocess.run([sys.executable, str(REPO / "scripts" / "pmc_summary.py"), str(src), str(prof / "r01_pmc_summary.json"),
                "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py --no-cpu "
                "--mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --steps 2 --warmup 1 "
                "(3 launches per kernel, 100 VLP-16 scans each; k_odom = 48 workgroups, plain launch)"], check=True)
q = REPO / "gpurun_out" / (tag + "_q") / "prof.txt"
if q.exists():
    (prof / "r01_odom_phase_profile.txt").write_text(
        "".join(line for line in q.read_text().splitlines(True) if "amdgpu" not in line))
d = json.loads((prof / "r01_bench.json").read_text())
import csv  # noqa: E402

rows = list(csv.DictReader(open(prof / "r01_kernel_stats.csv")))
kod = next(r for r in rows if r["Name"].startswith("lego::k_odom"))
pmc = json.loads((prof / "r01_pmc_summary.json").read_text())
print(json.dumps({
    "value": d["value"], "launch_ms": d["roofline"]["launch_ms"], "rocprof_k_odom_ms": float(kod["AverageNs"]) / 1e6,
    "achieved_GBs": d["roofline"]["achieved"], "frac": d["roofline"]["frac"],
    "k_odom_pmc_MB": pmc["k_odom_hbm_bytes_per_launch"] / 1e6, "cpu_1": d["cpu_baseline"]["value"],
    "cpu_16": d["aux"]["cpu_all_cores"]["value"], "fleet": d["aux"]["fleet_vlp16"]["scans_per_s"],
    "c3": d["aux"]["dense_hdl64_c3"]["scans_per_s"], "c5_gpu_ms": d["aux"]["scan_to_map_c5"]["gpu_ms_per_step"],
    "c5_cpu_ms": d["aux"]["scan_to_map_c5"]["cpu_ms_per_step"], "loop": d["aux"]["loop_closure"],
    "pose_delta": d["pose_delta_vs_oracle"]}, indent=1))
