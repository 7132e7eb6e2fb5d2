"""C5's six VoxelGrids one at a time through lego_voxel_grid (GPU box):
per cloud the sort's shape (rounds, local / slow / heap-sorted segments) and
the device time, median of a few repetitions.  Diagnostic, not a test."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lego-loam_amd"))
import numpy as np  # noqa: E402
import legoffi as L  # noqa: E402

sensor = "VLS-128"
sc = L.synth_cfg(sensor, 3)
surf, corner = L.synth_map(3, 50.0, 1_000_000, 200_000)
cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc)) + 16  # as bench.py's mapping line
eng = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts=L.opts_from_env())
reps = int(os.environ.get("REPS", "5"))


def vg(name, pts, leaf):
    us, st, out = [], None, None
    for _ in range(reps):
        out, st = eng.voxel_grid(pts, leaf)
        us.append(st["device_us"])
    print(f"{name:14s} n={len(pts):8d} leaf={leaf} out={len(out):7d} us={statistics.median(us):8.1f} "
          f"rounds={st['rounds']} local={st['local_segments']} slow={st['slow_segments']} heap={st['heap_segments']}",
          flush=True)
    return out


vg("map_surf", surf, 0.4)
vg("map_corner", corner, 0.2)
for k in range(int(os.environ.get("SCANS", "3"))):
    eng.ip(*L.synth_scan(sc, k))
    fa = eng.fa()
    if not fa["publish_to_mapping"]:
        continue
    vg(f"scan{k}_corner", fa["corner_last"], 0.2)
    s = vg(f"scan{k}_surf", fa["surf_last"], 0.4)
    o = vg(f"scan{k}_outlier", fa["outlier_last"], 0.4)
    vg(f"scan{k}_total", np.concatenate([s, o]), 0.4)
eng.close()
