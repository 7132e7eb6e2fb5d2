"""Wire formats: sensor_msgs/PointCloud2 decode
(pcl::fromROSMsg into PointXYZIR) on the device, the PointXYZI encoder and the
ROS1 serialiser of cloud_msgs/cloud_info.

The references here are restatements of the published formats: PCL's field
mapping (a field is copied when name, datatype and count match, else left 0)
and ROS1 message serialisation (little-endian; strings and arrays carry a
uint32 length).  Parity unpinned against PCL / roscpp themselves (absent)."""
import ctypes as C
import struct

import numpy as np
import pytest


def pcl_from_ros_msg(raw: np.ndarray, fields, point_step, width, height, row_step, L):
    """numpy restatement of pcl::fromROSMsg -> PointXYZIR."""
    want = {"x": (0, 7, 4), "y": (4, 7, 4), "z": (8, 7, 4), "intensity": (16, 7, 4), "ring": (20, 4, 2)}
    out = np.zeros(width * height, dtype=L.XYZIR_DTYPE).view(np.uint8).reshape(-1, 32)
    for name, (soff, dt, size) in want.items():
        src = [f for f in fields if f[0] == name and f[2] == dt and f[3] in (0, 1)]
        if not src:
            continue
        off = src[0][1]
        for r in range(height):
            for c in range(width):
                p = r * row_step + c * point_step + off
                out[r * width + c, soff:soff + size] = raw[p:p + size]
    return out.reshape(-1).view(L.XYZIR_DTYPE)


def ros1_cloud_info(seq, sec, nsec, frame, sri, eri, so, eo, od, gflag, col, rng):
    b = struct.pack("<III", seq, sec, nsec) + struct.pack("<I", len(frame)) + frame.encode()
    b += struct.pack("<I", len(sri)) + np.asarray(sri, "<i4").tobytes()
    b += struct.pack("<I", len(eri)) + np.asarray(eri, "<i4").tobytes()
    b += struct.pack("<fff", so, eo, od)
    b += struct.pack("<I", len(gflag)) + np.asarray(gflag, np.uint8).tobytes()
    b += struct.pack("<I", len(col)) + np.asarray(col, "<u4").tobytes()
    b += struct.pack("<I", len(rng)) + np.asarray(rng, "<f4").tobytes()
    return b


def test_cloud_info_serialize(L):
    lib = L.hip_lib()
    N, H = 2, 3
    sri = (C.c_int32 * N)(4, -7)
    eri = (C.c_int32 * N)(9, 11)
    gf = (C.c_uint8 * (N * H))(1, 0, 0, 1, 1, 0)
    col = (C.c_uint32 * (N * H))(0, 5, 1799, 3, 2, 1)
    rng = (C.c_float * (N * H))(1.5, 2.25, 0.0, -0.0, 3.0, 7.125)
    info = L.CloudInfo()
    info.stamp = 12.25
    info.start_ring_index = C.cast(sri, C.POINTER(C.c_int32))
    info.end_ring_index = C.cast(eri, C.POINTER(C.c_int32))
    info.start_orientation, info.end_orientation, info.orientation_diff = -3.0, 3.5, 6.5
    info.segmented_cloud_ground_flag = C.cast(gf, C.POINTER(C.c_uint8))
    info.segmented_cloud_col_ind = C.cast(col, C.POINTER(C.c_uint32))
    info.segmented_cloud_range = C.cast(rng, C.POINTER(C.c_float))
    n = C.c_uint64()
    assert lib.lego_cloud_info_serialize(C.byref(info), N, H, 7, b"base_link", None, 0, C.byref(n)) == 0
    buf = (C.c_uint8 * n.value)()
    assert lib.lego_cloud_info_serialize(C.byref(info), N, H, 7, b"base_link", buf, n.value, C.byref(n)) == 0
    want = ros1_cloud_info(7, 12, 250000000, "base_link", list(sri), list(eri), -3.0, 3.5, 6.5, list(gf),
                           list(col), list(rng))
    assert bytes(buf) == want
    small = (C.c_uint8 * 10)()
    assert lib.lego_cloud_info_serialize(C.byref(info), N, H, 7, b"base_link", small, 10,
                                         C.byref(n)) == L.LEGO_E_CAPACITY
    # ros::Time::fromSec rounding: 0.9999999996 s -> 1 s 0 ns
    info.stamp = 0.9999999996
    assert lib.lego_cloud_info_serialize(C.byref(info), N, H, 0, b"", buf, len(buf), C.byref(n)) == 0
    assert struct.unpack("<III", bytes(buf)[:12]) == (0, 1, 0)


def test_encode_xyzi(L):
    lib = L.hip_lib()
    pts = np.array([(1.0, -2.0, 3.5, 17.25), (0.0, 0.0, -0.0, 0.5)], dtype=L.XYZI_DTYPE)
    out = np.full(64, 0xAB, np.uint8)
    f4 = (L.Pc2Field * 4)()
    assert lib.lego_pc2_encode_xyzi(pts.ctypes.data, 2, out.ctypes.data, f4) == 0
    rec = out.reshape(2, 32)
    for i in range(2):
        v = rec[i].view("<f4")
        assert v[0] == pts["x"][i] and v[1] == pts["y"][i] and v[2] == pts["z"][i]
        assert v[3] == 1.0 and v[4] == pts["intensity"][i] and not rec[i, 20:].any()
    assert [(f.name, f.offset, f.datatype, f.count) for f in f4] == [
        (b"x", 0, 7, 1), (b"y", 4, 7, 1), (b"z", 8, 7, 1), (b"intensity", 16, 7, 1)]


def _layouts(L, pts):
    """(name, fields, point_step, height, row_pad, builder) for a few real
    driver layouts and mismatches."""
    n = len(pts)
    F, U16, U8, F64 = L.PF["FLOAT32"], L.PF["UINT16"], L.PF["UINT8"], L.PF["FLOAT64"]
    std = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F, 1), ("ring", 20, U16, 1)]
    packed = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 12, F, 1), ("ring", 16, U16, 1)]
    ouster = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F, 1), ("t", 20, 6, 1),
              ("reflectivity", 24, U16, 1), ("ring", 26, U16, 1), ("ambient", 28, U16, 1), ("range", 32, 6, 1)]
    ring_u8 = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 12, F, 1), ("ring", 16, U8, 1)]
    inten_f64 = [("x", 0, F, 0), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F64, 1), ("ring", 24, U16, 1)]
    return [("velodyne32", std, 32, 1, 0), ("packed22", packed, 22, 1, 0), ("ouster48_rows", ouster, 48, 16, 8),
            ("ring_uint8", ring_u8, 17, 1, 0), ("count0_intensity_f64", inten_f64, 26, 2, 4)]


def _build(L, pts, fields, ps, height, pad):
    n = len(pts)
    width = n // height
    n = width * height
    row_step = width * ps + pad
    raw = np.zeros(height * row_step, np.uint8)
    src = pts.view(np.uint8).reshape(-1, 32)
    vals = {"x": src[:, 0:4], "y": src[:, 4:8], "z": src[:, 8:12], "intensity": src[:, 16:20],
            "ring": src[:, 20:22]}
    rng = np.random.default_rng(5)
    for i in range(n):
        r, c = divmod(i, width)
        base = r * row_step + c * ps
        raw[base:base + ps] = rng.integers(0, 256, ps, dtype=np.uint8)  # junk in unmapped bytes
        for nm, off, dt, cnt in fields:
            if nm in vals:
                size = {7: 4, 4: 2, 2: 1, 8: 8, 6: 4}[dt]
                v = vals[nm][i]
                raw[base + off:base + off + min(size, len(v))] = v[:size]
    return raw, width, height, row_step


@pytest.mark.gpu
def test_pc2_decode_layouts(L):
    sc = L.synth_cfg("VLP-16", 0)
    pts, st = L.synth_scan(sc, 0)
    pts = pts[:4096]
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    for name, fields, ps, height, pad in _layouts(L, pts):
        raw, width, height, row_step = _build(L, pts, fields, ps, height, pad)
        m = L.pc2_msg(raw, fields, ps, width, height, row_step, stamp=st)
        out = np.zeros(width * height, dtype=L.XYZIR_DTYPE)
        n = C.c_int32()
        assert g.lib.lego_pc2_decode(g.h, C.byref(m), out.ctypes.data, len(out), C.byref(n)) == 0, name
        want = pcl_from_ros_msg(raw, fields, ps, width, height, row_step, L)
        assert n.value == len(want)
        assert np.array_equal(out.view(np.uint8), want.view(np.uint8)), name
    # not dense, big-endian, a field past point_step
    raw, width, height, row_step = _build(L, pts, _layouts(L, pts)[0][1], 32, 1, 0)
    n = C.c_int32()
    out = np.zeros(len(pts), dtype=L.XYZIR_DTYPE)
    m = L.pc2_msg(raw, _layouts(L, pts)[0][1], 32, width, is_dense=0)
    assert g.lib.lego_pc2_decode(g.h, C.byref(m), out.ctypes.data, len(out), C.byref(n)) == L.LEGO_E_NOT_DENSE
    m = L.pc2_msg(raw, _layouts(L, pts)[0][1], 32, width, is_bigendian=1)
    assert g.lib.lego_pc2_decode(g.h, C.byref(m), out.ctypes.data, len(out), C.byref(n)) == L.LEGO_E_ARG
    m = L.pc2_msg(raw, [("x", 30, L.PF["FLOAT32"], 1)], 32, width)
    assert g.lib.lego_pc2_decode(g.h, C.byref(m), out.ctypes.data, len(out), C.byref(n)) == L.LEGO_E_ARG
    g.close()


def _velodyne_msg(L, pts, stamp):
    F, U16 = L.PF["FLOAT32"], L.PF["UINT16"]
    fields = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F, 1), ("ring", 20, U16, 1)]
    raw = np.ascontiguousarray(pts).view(np.uint8).copy()
    return L.pc2_msg(raw, fields, 32, len(pts), stamp=stamp)


@pytest.mark.gpu
def test_ip_process_pc2_equals_ip_process(L):
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 1)
    a = L.Lego(cfg, max_points=40000)
    b = L.Lego(cfg, max_points=40000)
    for k in range(3):
        pts, st = L.synth_scan(sc, k)
        ga = a.ip(pts, st)
        m = _velodyne_msg(L, pts, st)
        out = L.IpOut()
        assert b.lib.lego_ip_process_pc2(b.h, C.byref(m), 0, C.byref(out)) == 0
        gb = L.ip_to_dict(out, cfg)
        b._ip = out  # the node hand-off the wrapper's fa() forwards
        for key in ("segmented", "outlier", "col_ind", "range", "ground_flag", "start_ring_index"):
            assert np.array_equal(np.asarray(ga[key]).view(np.uint8), np.asarray(gb[key]).view(np.uint8)), key
        fa, fb = a.fa(), b.fa()
        assert np.array_equal(fa["transform_sum"].view(np.uint32), fb["transform_sum"].view(np.uint32))
    a.close()
    b.close()


@pytest.mark.gpu
def test_odom_batch_pc2_equals_odom_batch(L):
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 2)
    K = 6
    scans = [L.synth_scan(sc, k) for k in range(K)]
    a = L.Lego(cfg, max_points=40000, max_batch=K)
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(K + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    ra = bytes(a.odom_batch(pts, off, np.array([s for _, s in scans])))
    b = L.Lego(cfg, max_points=40000, max_batch=K)
    msgs = (L.Pc2Msg * K)()
    keep = []
    for k, (p, s) in enumerate(scans):
        m = _velodyne_msg(L, p, s)
        keep.append(m)
        msgs[k] = m
    recs = (L.PoseRec * K)()
    assert b.lib.lego_odom_batch_pc2(b.h, msgs, K, 0, recs) == 0
    rb = bytes(recs)
    for k in range(K):
        assert ra[64 * k:64 * k + 60] == rb[64 * k:64 * k + 60], k
    a.close()
    b.close()
