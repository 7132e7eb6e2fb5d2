"""Node-API call order and the resident hand-off (lego_mo_process reading the
context's own last lego_fa_process clouds on the device, lego_api.hip
`resident`): any projection call in between overwrites the slot those
clouds live in, so the step must take the upload path instead.

The order of a ROS deployment whose mapping callback runs late: ip(k) ->
fa(k) -> ip(k+1) -> mo(fa output of k) -> fa(k+1) -> ...  With
lego_ip_process_pc2 as the projection call (the raw-message entry, ADVICE r4:
it had not invalidated the resident hand-off), every mapping step must equal,
bit for bit, the step of a context driven in the plain order ip -> fa -> mo.
Reference: mapOptmization.cpp:1487-1522 (run), featureAssociation.cpp:
1790-1815 (publishCloudsLast)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pc2(L, pts, stamp):
    """a velodyne-layout PointCloud2 (x y z pad intensity ring) over pts"""
    F, U16 = L.PF["FLOAT32"], L.PF["UINT16"]
    raw = np.ascontiguousarray(pts).view(np.uint8).reshape(-1)
    fields = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F, 1), ("ring", 20, U16, 1)]
    return L.pc2_msg(raw, fields, 32, len(pts), stamp=stamp)


@pytest.mark.parametrize("sensor,seed,n", [("VLP-16", 6, 16), ("HDL-64E", 2, 8)])
def test_projection_between_fa_and_mo(L, sensor, seed, n):
    import ctypes as C

    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    cap = max(len(p) for p, _ in scans) + 16
    a = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap)  # late-mapping order, pc2 projection
    b = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap)  # plain order
    steps = 0
    try:
        msgs = [_pc2(L, p, s) for p, s in scans]
        st = a.lib.lego_ip_process_pc2(a.h, C.byref(msgs[0]), 0, C.byref(a._ip))
        assert st == 0, a.lib.lego_last_error()
        for k in range(n):
            a.fa()
            if k + 1 < n:  # the next scan's projection before this scan's mapping step
                st = a.lib.lego_ip_process_pc2(a.h, C.byref(msgs[k + 1]), 0, C.byref(a._ip))
                assert st == 0, a.lib.lego_last_error()
            ra = a.mo()
            b.ip(*scans[k])
            b.fa()
            rb = b.mo()
            assert ra["processed"] == rb["processed"], k
            if not rb["processed"]:
                continue
            steps += 1
            for key in ("transform_aft_mapped", "transform_tobe_mapped", "transform_bef_mapped"):
                assert np.array_equal(ra[key].view(np.uint32), rb[key].view(np.uint32)), (k, key, ra[key], rb[key])
            for key in ("iterations", "n_corner_scan_ds", "n_surf_scan_ds", "n_rows_last"):
                assert ra[key] == rb[key], (k, key)
    finally:
        a.close()
        b.close()
    assert steps >= 2, steps
