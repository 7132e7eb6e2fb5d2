"""VLS-128 front end and mapping on a few scans (GPU box, diagnostic): ip + fa
on their own, then the C5 sequence (fixed map installed, ip / fa / mo), each
step's status printed.  LEGO_HIP_LIB_AB selects the library."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lego-loam_amd"))
import legoffi as L  # noqa: E402

sc = L.synth_cfg("VLS-128", 3)
cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc)) + 16
g = L.Lego(L.sensor_cfg("VLS-128", L.hip_lib()), max_points=cap, opts=L.opts_from_env())
for k in range(3):
    g.ip(*L.synth_scan(sc, k))
    fa = g.fa()
    print("front end scan", k, "ok", len(fa["surf_last"]), flush=True)
g.close()
surf, corner = L.synth_map(3, 50.0, 1_000_000, 200_000)
g = L.Lego(L.sensor_cfg("VLS-128", L.hip_lib()), max_points=cap, opts=L.opts_from_env())
g.mo_set_map(corner, surf)
print("map installed", flush=True)
for k in range(3):
    g.ip(*L.synth_scan(sc, k))
    g.fa()
    o = g.mo()
    print("mapping scan", k, "ok", o["processed"], o["iterations"], flush=True)
g.close()
print("done", L.HIP_LIB)
