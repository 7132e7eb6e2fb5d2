"""Single-scan (node-call) A/B of k_lf_voxel's block width (GPU box):
lego_ip_process -> lego_fa_process over SCANS scans of each sensor, with
LEGO_LFV_WIDE=1 (every ring by a 1024-thread workgroup, the default for
launches of <= 128 rings) and =0 (the batch kernel: rings <= 512 by a wave,
larger ones by 256-thread workgroups), alternating per scan.  Prints the
median fa call (host wall clock) and the median fa.voxel stage (device
events: k_lf_voxel) per sensor and width.  Diagnostic, not a test."""
import os
import statistics
import sys
import time

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "lego-loam_amd"))
import ctypes as C  # noqa: E402

import legoffi as L  # noqa: E402

n = int(os.environ.get("SCANS", "24"))
lib = L.hip_lib()
SENS = {"VLP-16": 1, "HDL-64E": 2, "VLS-128": 3}
for sensor in os.environ.get("SENSORS", "VLP-16,HDL-64E,VLS-128").split(","):
    seed = SENS[sensor]
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    g = L.Lego(L.sensor_cfg(sensor, lib), max_points=max(len(p) for p, _ in scans) + 16, opts=L.opts_from_env())
    on = (C.c_float * 1)()
    nn = C.c_int32()
    lib.lego_stage_times(g.h, None, on, 0, C.byref(nn))  # stage events on
    wides = [int(w) for w in os.environ.get("WIDES", "1,0").split(",")]
    res = {w: ([], [], []) for w in wides}
    for k, (p, s) in enumerate(scans):
        wide = wides[k % len(wides)]
        os.environ["LEGO_LFV_WIDE"] = str(wide)
        g.ip(p, s)
        t0 = time.perf_counter()
        g.fa()
        t1 = time.perf_counter()
        if k >= 2:  # past module loading
            res[wide][0].append((t1 - t0) * 1e3)
            st = g.stage_times()
            res[wide][1].append(st.get("fa.voxel", float("nan")))
            res[wide][2].append(st)
    g.close()
    for w in wides:
        print(f"{sensor:8s} wide={w}  fa median {statistics.median(res[w][0]):.3f} ms  "
              f"k_lf_voxel median {statistics.median(res[w][1]) * 1e3:.1f} us  (n={len(res[w][0])})", flush=True)
        print("   stages (us): " + "  ".join(f"{k} {statistics.median(d.get(k, 0.0) for d in res[w][2]) * 1e3:.1f}"
                                          for k in res[w][2][0]), flush=True)
