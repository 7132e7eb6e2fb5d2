"""Per-stream view of one C5 mapping step from a rocprofv3 kernel trace
(scripts/gpu_c5_trace.sh): for each stream, the spans of its VoxelGrids and
other kernels, relative to the step's k_mo_associate."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
want = int(sys.argv[2]) if len(sys.argv) > 2 else 1
starts = [i for i, r in enumerate(rows) if "k_mo_associate" in r["Kernel_Name"]]
a = starts[want]
b = next(i for i in range(a, len(rows)) if "k_mo_finish" in rows[i]["Kernel_Name"])
t0 = int(rows[a]["Start_Timestamp"])
lo = int(rows[a]["Start_Timestamp"]) - 3000_000
hi = int(rows[b]["End_Timestamp"])
per = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e < t0 - 50_000 or s > hi:
        continue
    n = r["Kernel_Name"].split("(")[0].replace("lego::", "")
    if not any(k in n for k in ("k_vg", "k_mo", "k_idx", "k_scan")):
        continue
    per[r["Queue_Id"]].append((n, s, e))
print(f"step {want}: {(hi - t0) / 1e3:.1f} us from k_mo_associate to k_mo_finish")
for q, ks in per.items():
    out, vg = [], None
    for n, s, e in ks:
        if n == "k_vg_init":
            vg = s
        elif n == "k_vg_emit" and vg is not None:
            out.append(f"VG[{(vg - t0) / 1e3:.0f}..{(e - t0) / 1e3:.0f}]")
            vg = None
        elif vg is None:
            out.append(f"{n}[{(s - t0) / 1e3:.0f}..{(e - t0) / 1e3:.0f}]")
    print(f"queue {q}: " + " ".join(out))
