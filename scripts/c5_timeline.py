"""Reads a rocprofv3 kernel trace of the C5 line (scripts/gpu_c5_trace.sh) and
prints each mapping step's timeline: every VoxelGrid (k_vg_init .. k_vg_emit)
with its sort phases, the index builds and the LM iterations."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
mo = [r for r in rows if any(k in r["Kernel_Name"] for k in ("k_vg_", "k_mo_", "k_idx_", "k_scan_", "k_kf_"))]
# a step starts at k_mo_associate
steps, cur = [], None
for r in mo:
    n = r["Kernel_Name"].split("(")[0].replace("lego::", "")
    if n == "k_mo_associate":
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for si, st in enumerate(steps):
    t0 = st[0][1]
    print(f"step {si}: {(st[-1][2] - t0) / 1e3:.1f} us, {len(st)} kernels")
    vg, ph = None, defaultdict(float)
    for n, a, b in st:
        if n == "k_vg_init":
            vg = a
            ph = defaultdict(float)
        if vg is not None:
            key = "rounds" if n in ("k_vg_count", "k_vg_decide", "k_vg_swap", "k_vg_plan") else n
            ph[key] += (b - a) / 1e3
        if n == "k_vg_emit" and vg is not None:
            print(f"  VG @{(vg - t0) / 1e3:8.1f}  {(b - vg) / 1e3:7.1f} us  " +
                  " ".join(f"{k.replace('k_vg_', '')}={v:.1f}" for k, v in ph.items()))
            vg = None
        elif vg is None and not n.startswith("k_vg"):
            print(f"  {n:16s} @{(a - t0) / 1e3:8.1f}  {(b - a) / 1e3:7.1f} us")
