"""Per-ring time of the device's VoxelGrid block sort (GPU box): every ring of
tests/golden/dense_ring_keys.npz (VLS-128 seed 3 scan 0, HDL-64E seed 2 scan 0)
and C2 scan 465's rings (c2_ring_keys.npz) through lego_sort_permutation in
the modes given (default 8,7: the LDS-id form, 1024 threads, sum order / exact,
k_lf_voxel's node form), host
wall clock per call minus the call's floor (a 2-key sort), min of 5.  Prints
the slowest rings with their heap-sorted piece counts.  Diagnostic."""
import os
import sys
import time

import numpy as np

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "lego-loam_amd"))
import legoffi as L  # noqa: E402

MODES = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "8,7").split(",")]
d = dict(np.load(os.path.join(R, "tests/golden/dense_ring_keys.npz")))
d.update({"c2:" + k: v for k, v in np.load(os.path.join(R, "tests/golden/c2_ring_keys.npz")).items()})
g = L.Lego(L.sensor_cfg("VLS-128", L.hip_lib()), max_points=4096, opts=L.opts_from_env())


def t(keys, mode):
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        _, heap = g.sort_permutation(keys, mode)
        best = min(best, time.perf_counter() - t0)
    return best * 1e6, heap


floor = min(t(np.array([2, 1], np.uint32), m)[0] for m in MODES)
print(f"call floor {floor:.1f} us")
for mode in MODES:
    rows = []
    for k in d:
        us, heap = t(d[k], mode)
        rows.append((us - floor, k, len(d[k]), heap))
    rows.sort(reverse=True)
    print(f"mode {mode}: sum over rings {sum(r[0] for r in rows):.0f} us; slowest:")
    for us, k, n, heap in rows[:8]:
        print(f"  {k:14s} n {n:5d} heap pieces {heap:3d}  {us:8.1f} us")
g.close()
