"""GPU odometry with scan-line keys out of ring order, vs the oracle.

The odometry's correspondence searches read a point's scan line from
int(intensity) (featureAssociation.cpp:1062-1099, :1173-1220).  Clouds from
the pipeline come ring after ring, so the keys only grow along a cloud and the
device's key tables (first / last index of each key, stored where the key
changes) bound the scan-line windows.  Here two rings' labels are swapped in
the segmented cloud handed to lego_fa_process, so the keys of the new last
clouds decrease somewhere: the index build must mark the clouds irregular and
the searches must take the literal scan-line loops.  Oracle and GPU run on the
same modified input; features exact, poses within the north-star 1e-4."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4


def _swap_rings(L, ip, a, b):
    """A copy of ip's segmented cloud with ring labels a and b exchanged
    (fractional part kept).  Returns the array (keep it alive)."""
    seg = L._arr(ip.segmented_cloud, ip.n_segmented, L.XYZI_DTYPE).copy()
    r = np.floor(seg["intensity"]).astype(np.int64)
    frac = seg["intensity"] - r.astype(np.float32)
    lab = np.where(r == a, b, np.where(r == b, a, r)).astype(np.float32)
    seg["intensity"] = lab + frac
    return seg


def test_swapped_ring_labels_match_oracle(L):
    sc = L.synth_cfg("VLP-16", 4)
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc))
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    worst = 0.0
    for k in range(12):
        pts, stamp = L.synth_scan(sc, k)
        gpu.ip(pts, stamp)
        ora.ip(pts, stamp)
        seg = _swap_rings(L, ora._ip, 3, 10)
        ptr = seg.ctypes.data_as(L.C.POINTER(L.PointXYZI))
        gpu._ip.segmented_cloud = ptr  # not the context's own buffer: uploaded as given
        ora._ip.segmented_cloud = ptr
        g, o = gpu.fa(), ora.fa()
        for key in ("sharp", "less_sharp", "flat", "less_flat"):
            assert np.array_equal(g[key].view(np.uint32), o[key].view(np.uint32)), (k, key)
        assert g["odom_valid"] == o["odom_valid"], k
        d = float(np.max(np.abs(np.asarray(g["transform_sum"], np.float64) - np.asarray(o["transform_sum"], np.float64))))
        assert d <= POSE_TOL, (k, g["transform_sum"], o["transform_sum"])
        assert np.array_equal(np.asarray(g["transform_sum"], np.float32).view(np.uint32),
                              np.asarray(o["transform_sum"], np.float32).view(np.uint32)), k
        worst = max(worst, d)
        del seg
    print(f"swapped ring labels: 12 scans, worst |dpose| {worst:.3g}")
    gpu.close()
