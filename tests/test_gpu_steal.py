"""The exchanges' steal-on-timeout paths (lego_odom.hip, "exchange" and the
hand-off exchange): nothing assumes the workgroups of an odometry launch are
resident together, so a workgroup that never publishes (LEGO_ODOM_SILENT_WG,
a diagnostic read at context creation) must only cost time: the others wait
kStealTicks, then compute its NN queries and its share of TransformToEnd
themselves.  The records must equal a normal context's byte for byte:
VLP-16 (LDS-resident: NN exchange) and HDL-64E (HBM-resident: NN and
hand-off exchanges)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


@pytest.mark.parametrize("sensor,seed,n,cap", [("VLP-16", 7, 10, 40000), ("HDL-64E", 2, 4, 140000)])
def test_silent_workgroup_is_stolen(L, sensor, seed, n, cap):
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    g = L.Lego(cfg, max_points=cap, max_batch=n)
    want = bytes(g.odom_batch(*_pack(scans)))
    g.close()
    os.environ["LEGO_ODOM_SILENT_WG"] = "3"
    try:
        s = L.Lego(cfg, max_points=cap, max_batch=n)
    finally:
        os.environ.pop("LEGO_ODOM_SILENT_WG", None)
    got = bytes(s.odom_batch(*_pack(scans)))
    s.close()
    assert [got[64 * k:64 * k + 60] for k in range(n)] == [want[64 * k:64 * k + 60] for k in range(n)]
