"""The node call's two streams (lego_fa_process: the per-ring less-flat
VoxelGrid, featureAssociation.cpp:778-782, on the context's second stream
beside the LM, the hand-off waiting for it on the device) are a scheduling
change only: every output of every scan equals, byte for byte, the
single-stream order (lego_ctx_opts::node_overlap = 0) and the oracle's.
Two contexts run the same scans, one per mode; VLP-16 (the LDS-resident
odometry, k_odom<false, true>) and HDL-64E (the ring form, k_odom<true, true>).
The hand-off's bounded wait, forced to give up (lf_wait_ms = 0), fails the
call and the context until lego_reset, with every workgroup following the
lead's decision.
Reference: featureAssociation.cpp:1759-1815 (publishCloudsLast, the less-flat
cloud's only reader), :1817-1860 (runFeatureAssociation)."""
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
    ctx = {m: L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts={"node_overlap": m}) for m in (1, 0)}
    try:
        for k, (p, s) in enumerate(scans):
            ora.ip(p, s)
            ref = ora.fa()
            got = {}
            for m, g in ctx.items():
                g.ip(p, s)
                got[m] = g.fa()
            for key in CLOUDS:
                a, b = got[1][key], got[0][key]
                assert a.tobytes() == b.tobytes(), (k, key, len(a), len(b))
                assert a.tobytes() == ref[key].tobytes(), (k, key, "oracle")
            for key in ("transform_cur", "transform_sum"):
                assert np.array_equal(got[1][key].view(np.uint32), got[0][key].view(np.uint32)), (k, key)
                assert np.array_equal(got[1][key].view(np.uint32), ref[key].view(np.uint32)), (k, key, "oracle")
            assert got[1]["odom_valid"] == got[0]["odom_valid"] == ref["odom_valid"], k
    finally:
        for g in ctx.values():
            g.close()


@pytest.mark.parametrize("sensor,seed", [("VLP-16", 4), ("HDL-64E", 2)])
def test_late_voxel_grid_fails_until_reset(L, sensor, seed):
    """lf_wait_ms = 0: the lead never waits, so the hand-off gives up at once
    (kBadLfLate; the initialisation scan publishes its clouds too, so the
    first call reaches the wait).  The call returns LEGO_E_DEVICE, later
    odometry calls LEGO_E_STATE (the stream's state is not trusted), and after
    lego_reset the context's batches equal a fresh context's byte for byte."""
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(4)]
    cap = max(len(p) for p, _ in scans) + 16
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    stamps = np.array([s for _, s in scans])
    g = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, max_batch=4, opts={"lf_wait_ms": 0})
    g.ip(*scans[0])
    with pytest.raises(RuntimeError, match=f"status {L.LEGO_E_DEVICE} .*lego_reset"):
        g.fa()
    g.ip(*scans[1])
    with pytest.raises(RuntimeError, match=f"status {L.LEGO_E_STATE} "):
        g.fa()
    with pytest.raises(RuntimeError, match=f"status {L.LEGO_E_STATE} "):
        g.odom_batch(pts, off, stamps)
    g.reset()
    got = bytes(g.odom_batch(pts, off, stamps))
    g.close()
    f = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, max_batch=4)
    want = bytes(f.odom_batch(pts, off, stamps))
    f.close()
    assert [got[64 * k:64 * k + 60] for k in range(4)] == [want[64 * k:64 * k + 60] for k in range(4)]
