"""The node call's two streams (lego_fa_process: the per-ring less-flat
VoxelGrid, featureAssociation.cpp:778-782, on the context's second stream
beside the LM, the hand-off waiting for it on the device) are a scheduling
change only: every output of every scan equals, byte for byte, the
single-stream order (LEGO_NODE_OVERLAP=0, read per call) and the oracle's.
Two contexts run the same scans, one per mode; VLP-16 (the LDS-resident
odometry, k_odom<false, true>) and HDL-64E (the ring form, k_odom<true, true>).
Reference: featureAssociation.cpp:1759-1815 (publishCloudsLast, the less-flat
cloud's only reader), :1817-1860 (runFeatureAssociation)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CLOUDS = ("sharp", "less_sharp", "flat", "less_flat", "corner_last", "surf_last", "outlier_last")


@pytest.mark.parametrize("sensor,seed,n", [("VLP-16", 4, 10), ("HDL-64E", 2, 6)])
def test_overlap_is_only_scheduling(L, sensor, seed, n):
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    cap = max(len(p) for p, _ in scans) + 16
    ora = L.Oracle(L.sensor_cfg(sensor))
    ctx = {m: L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap) for m in ("1", "0")}
    old = os.environ.get("LEGO_NODE_OVERLAP")
    try:
        for k, (p, s) in enumerate(scans):
            ora.ip(p, s)
            ref = ora.fa()
            got = {}
            for m, g in ctx.items():
                os.environ["LEGO_NODE_OVERLAP"] = m
                g.ip(p, s)
                got[m] = g.fa()
            for key in CLOUDS:
                a, b = got["1"][key], got["0"][key]
                assert a.tobytes() == b.tobytes(), (k, key, len(a), len(b))
                assert a.tobytes() == ref[key].tobytes(), (k, key, "oracle")
            for key in ("transform_cur", "transform_sum"):
                assert np.array_equal(got["1"][key].view(np.uint32), got["0"][key].view(np.uint32)), (k, key)
                assert np.array_equal(got["1"][key].view(np.uint32), ref[key].view(np.uint32)), (k, key, "oracle")
            assert got["1"]["odom_valid"] == got["0"]["odom_valid"] == ref["odom_valid"], k
    finally:
        if old is None:
            os.environ.pop("LEGO_NODE_OVERLAP", None)
        else:
            os.environ["LEGO_NODE_OVERLAP"] = old
        for g in ctx.values():
            g.close()
