#!/usr/bin/env python3
"""Copies one GPU session's evidence (scripts/gpu_check.sh + gpu_profile.sh
under gpurun_out/<tag>, the phase profile of gpu_quick.sh under
gpurun_out/<tag>_q) into profiles/<round>_*, stamps the summaries with the
commit the session ran, and prints the numbers DESIGN.md quotes.
Usage: refresh_profiles.py <tag> [round (r02)] [commit (HEAD)]"""
import json
import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
rnd = sys.argv[2] if len(sys.argv) > 2 else "r02"
commit = sys.argv[3] if len(sys.argv) > 3 else subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=REPO,
                                                             capture_output=True, text=True).stdout.strip()
src = REPO / "gpurun_out" / tag
prof = REPO / "profiles"
shutil.copy(src / "bench.json", prof / f"{rnd}_bench.json")
shutil.copy(src / "gpu_tests.log", prof / f"{rnd}_gpu_tests.log")
shutil.copy(src / "prof_stats" / "run_kernel_stats.csv", prof / f"{rnd}_kernel_stats.csv")
subprocess.run([sys.executable, str(REPO / "scripts" / "pmc_summary.py"), str(src), str(prof / f"{rnd}_pmc_summary.json"),
                "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py --no-cpu "
                "--mapping-steps 0 --fleet-streams 0 --dense-scans 0 --loop-scans 0 --steps 2 --warmup 1 "
                "(3 launches per kernel, 100 VLP-16 scans each; k_odom = 24 workgroups, plain launch)", commit],
               check=True)
for sub, name in (("prof_fleet", "fleet_kernel_stats.csv"), ("prof_c5", "c5_kernel_stats.csv")):
    f = src / sub / "run_kernel_stats.csv"
    if f.exists():
        shutil.copy(f, prof / f"{rnd}_{name}")
q = REPO / "gpurun_out" / (tag + "_q") / "prof.txt"
if q.exists():
    (prof / f"{rnd}_odom_phase_profile.txt").write_text(
        "".join(line for line in q.read_text().splitlines(True) if "amdgpu" not in line))
d = json.loads((prof / f"{rnd}_bench.json").read_text())
import csv  # noqa: E402

rows = list(csv.DictReader(open(prof / f"{rnd}_kernel_stats.csv")))
kod = next(r for r in rows if r["Name"].startswith("lego::k_odom"))
pmc = json.loads((prof / f"{rnd}_pmc_summary.json").read_text())
(prof / f"{rnd}_COMMIT").write_text(f"{commit}\n")
print(json.dumps({
    "value": d["value"], "launch_ms": d["roofline"]["launch_ms"], "rocprof_k_odom_ms": float(kod["AverageNs"]) / 1e6,
    "achieved_GBs": d["roofline"]["achieved"], "frac": d["roofline"]["frac"],
    "k_odom_pmc_MB": pmc["k_odom_hbm_bytes_per_launch"] / 1e6, "cpu_1": d["cpu_baseline"]["value"],
    "cpu_16": d["aux"]["cpu_all_cores"]["value"], "fleet": d["aux"]["fleet_vlp16"]["scans_per_s"],
    "c3": d["aux"]["dense_hdl64_c3"]["scans_per_s"], "c5_gpu_ms": d["aux"]["scan_to_map_c5"]["gpu_ms_per_step"],
    "c5_cpu_ms": d["aux"]["scan_to_map_c5"]["cpu_ms_per_step"], "loop": d["aux"]["loop_closure"],
    "pose_delta": d["pose_delta_vs_oracle"]}, indent=1))
