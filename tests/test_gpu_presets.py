"""GPU parity for the reference's other sensor presets (HDL-32E, OS1-16,
OS1-64: utility.h:70-102) and for the useCloudRing = false projection branch
(imageProjection.cpp:170, 225-233), through the C-ABI against the oracle.

Per preset: one scan's images, clouds, cloud_info and features byte-equal;
an 8-scan stream through the node calls and the same 8 scans as one device
batch, every pose bit-exact.  Ring-less: the vertical-angle row on the
sensors whose synthetic beams sit inside their bins and on the two whose
beams sit on the bins' edges (VLS-128, HDL-64E: float rounding decides the
row, the stress case), the ring channel scrambled, non-finite points removed
(first and last included), a stream's poses, and a raw PointCloud2 without a
ring field and with is_dense = false."""
import ctypes as C

import numpy as np
import pytest

from test_gpu_parity import assert_feat_equal, assert_ip_equal

pytestmark = pytest.mark.gpu

PRESETS = [("HDL-32E", 4), ("OS1-16", 5), ("OS1-64", 6)]


def maxpts(L, sc):
    return L.synth_lib().lego_synth_max_points(C.byref(sc)) + 16


def cfgs(L, name, ring=True):
    g, o = L.sensor_cfg(name, L.hip_lib()), L.sensor_cfg(name)
    if not ring:
        g.use_cloud_ring = 0
        o.use_cloud_ring = 0
    return g, o


def u32(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("sensor,seed", PRESETS)
def test_preset_scan_parity(L, sensor, seed):
    sc = L.synth_cfg(sensor, seed)
    pts, st = L.synth_scan(sc, 0)
    gc, oc = cfgs(L, sensor)
    gpu, ora = L.Lego(gc, max_points=maxpts(L, sc)), L.Oracle(oc)
    assert_ip_equal(gpu.ip(pts, st, images=True), ora.ip(pts, st, images=True))
    assert_feat_equal(gpu.fa(), ora.fa())
    g = gpu.ip(pts, st, gated=True)
    o = L.Oracle(oc).ip(pts, st, gated=True)
    for k in ("full_info_cloud", "ground_cloud", "segmented_cloud_pure"):
        assert np.array_equal(g[k].view(np.uint8), o[k].view(np.uint8)), k
    gpu.close()


@pytest.mark.parametrize("sensor,seed", PRESETS)
def test_preset_stream_node_and_batch(L, sensor, seed):
    K = 8
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(K)]
    gc, oc = cfgs(L, sensor)
    gpu, ora = L.Lego(gc, max_points=maxpts(L, sc)), L.Oracle(oc)
    want = []
    for k, (pts, st) in enumerate(scans):
        assert_ip_equal(gpu.ip(pts, st), ora.ip(pts, st), images=False)
        gf, of = gpu.fa(), ora.fa()
        assert_feat_equal(gf, of)
        assert gf["odom_valid"] == of["odom_valid"]
        assert np.array_equal(u32(gf["transform_sum"]), u32(of["transform_sum"])), (k, gf["transform_sum"],
                                                                                  of["transform_sum"])
        if gf["publish_to_mapping"]:
            for key in ("corner_last", "surf_last", "outlier_last"):
                assert np.array_equal(gf[key].view(np.uint32), of[key].view(np.uint32)), (k, key)
        want.append(of)
    gpu.close()
    # the same scans as one batch: the batch kernels (segmentation, sorts and
    # odometry forms chosen by the batch size)
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(K + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    gb = L.Lego(gc, max_points=maxpts(L, sc), max_batch=K)
    recs = gb.odom_batch(pts, off, np.array([s for _, s in scans]))
    for k in range(K):
        r = recs[k]
        assert (r.n_sharp, r.n_less_sharp, r.n_flat, r.n_less_flat) == tuple(
            len(want[k][n]) for n in ("sharp", "less_sharp", "flat", "less_flat")), k
        assert np.array_equal(u32(list(r.transform_sum)), u32(want[k]["transform_sum"])), k
    gb.close()


@pytest.mark.parametrize("sensor,seed", [("VLP-16", 0), ("HDL-32E", 1), ("OS1-64", 2), ("VLS-128", 3),
                                         ("HDL-64E", 2)])
def test_ringless_scan_parity(L, sensor, seed):
    sc = L.synth_cfg(sensor, seed)
    pts, st = L.synth_scan(sc, 0)
    pts["ring"] = np.random.default_rng(seed).integers(0, 1000, len(pts))  # not read by this branch
    gc, oc = cfgs(L, sensor, ring=False)
    gpu, ora = L.Lego(gc, max_points=maxpts(L, sc)), L.Oracle(oc)
    assert_ip_equal(gpu.ip(pts, st, images=True), ora.ip(pts, st, images=True))
    assert_feat_equal(gpu.fa(), ora.fa())
    gpu.close()


def test_ringless_row_edges(L):
    """The size_t row conversion (:230-233) on the device: rows a half and a
    twentieth of a row below ang_bottom land in row 0, further below and above
    the top row are skipped."""
    from test_presets import _edge_points
    gc, oc = cfgs(L, "VLP-16", ring=False)
    vs = [-0.5, -1.5, 7.5, 15.5, 16.5, -0.05, -0.999, 15.999]
    pts = _edge_points(L, oc, vs)
    # the scene around them, so the segmentation has something to do
    scene, st = L.synth_scan(L.synth_cfg("VLP-16", 7), 0)
    pts = np.concatenate([scene, pts])
    gpu = L.Lego(gc, max_points=len(pts) + 16)
    assert_ip_equal(gpu.ip(pts, st, images=True), L.Oracle(oc).ip(pts, st, images=True))
    gpu.close()


def test_ringless_nan_points_removed(L):
    sc = L.synth_cfg("VLP-16", 4)
    pts, st = L.synth_scan(sc, 0)
    rng = np.random.default_rng(1)
    for idx in ([0, 1, 2, len(pts) - 2, len(pts) - 1], rng.choice(len(pts), 500, replace=False), [7]):
        dirty = pts.copy()
        dirty["x"][idx] = np.nan
        dirty["z"][idx[:1]] = np.inf
        gc, oc = cfgs(L, "VLP-16", ring=False)
        gpu, ora = L.Lego(gc, max_points=len(pts) + 16), L.Oracle(oc)
        assert_ip_equal(gpu.ip(dirty, st, images=True), ora.ip(dirty, st, images=True))
        assert_feat_equal(gpu.fa(), ora.fa())
        gpu.close()
    # the ring branch still rejects the scan; a scan with no finite point is rejected by both
    gr = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=len(pts) + 16)
    with pytest.raises(RuntimeError, match="status 1 "):
        gr.ip(dirty, st)
    gr.close()
    gc, _ = cfgs(L, "VLP-16", ring=False)
    gpu = L.Lego(gc, max_points=len(pts) + 16)
    allnan = pts[:64].copy()
    allnan["y"] = np.nan
    with pytest.raises(RuntimeError, match="status 1 "):
        gpu.ip(allnan, st)
    gpu.ip(pts, st)  # the context still works
    gpu.close()


def test_ringless_stream_node_and_batch(L):
    """Poses of a ring-less VLP-16 stream with non-finite points in every scan,
    node calls and one device batch, bit-exact against the oracle."""
    K = 8
    sc = L.synth_cfg("VLP-16", 1)
    rng = np.random.default_rng(3)
    scans = []
    for k in range(K):
        p, s = L.synth_scan(sc, k)
        p["y"][rng.choice(len(p), 50, replace=False)] = np.nan
        p["ring"] = 0
        scans.append((p, s))
    gc, oc = cfgs(L, "VLP-16", ring=False)
    gpu, ora = L.Lego(gc, max_points=40000), L.Oracle(oc)
    want = []
    for k, (p, s) in enumerate(scans):
        assert_ip_equal(gpu.ip(p, s), ora.ip(p, s), images=False)
        gf, of = gpu.fa(), ora.fa()
        assert_feat_equal(gf, of)
        assert np.array_equal(u32(gf["transform_sum"]), u32(of["transform_sum"])), k
        want.append(of["transform_sum"])
    gpu.close()
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(K + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    gb = L.Lego(gc, max_points=40000, max_batch=K)
    recs = gb.odom_batch(pts, off, np.array([s for _, s in scans]))
    for k in range(K):
        assert np.array_equal(u32(list(recs[k].transform_sum)), u32(want[k])), k
    gb.close()


def test_ringless_pc2_without_ring_field(L):
    """lego_ip_process_pc2 of an XYZI message (no ring field) flagged
    is_dense = false, with NaN points: accepted without useCloudRing (the
    NaNs removed, :170), rejected with it (:173-176)."""
    sc = L.synth_cfg("OS1-16", 2)
    pts, st = L.synth_scan(sc, 0)
    pts["x"][[0, 100, 2000]] = np.nan
    F = L.PF["FLOAT32"]
    fields = [("x", 0, F, 1), ("y", 4, F, 1), ("z", 8, F, 1), ("intensity", 16, F, 1)]
    raw = np.ascontiguousarray(pts).view(np.uint8).copy()
    m = L.pc2_msg(raw, fields, 32, len(pts), stamp=st, is_dense=0)
    gc, oc = cfgs(L, "OS1-16", ring=False)
    gpu = L.Lego(gc, max_points=maxpts(L, sc))
    out = L.IpOut()
    assert gpu.lib.lego_ip_process_pc2(gpu.h, C.byref(m), L.LEGO_IP_IMAGES, C.byref(out)) == 0
    noring = pts.copy()
    noring["ring"] = 0
    assert_ip_equal(L.ip_to_dict(out, gc, True), L.Oracle(oc).ip(noring, st, images=True))
    gpu.close()
    gr = L.Lego(L.sensor_cfg("OS1-16", L.hip_lib()), max_points=maxpts(L, sc))
    assert gr.lib.lego_ip_process_pc2(gr.h, C.byref(m), 0, C.byref(out)) == L.LEGO_E_NOT_DENSE
    gr.close()


@pytest.mark.parametrize("sensor,seed,ring", [("VLP-16", 7, False), ("OS1-16", 5, True), ("OS1-16", 8, False)])
def test_fused_batch_presets(L, sensor, seed, ring):
    """Batches of more than 8 VLP-16-class scans take k_ip_lds (the whole
    projection and segmentation per scan in one workgroup), with the
    ring-less branch's NaN removal and OS1-16's 1024 columns: 12 scans as one
    device batch (non-finite points in every ring-less scan), every scan's
    segmented cloud, cloud_info and features byte-equal and every pose
    bit-exact against the oracle."""
    K = 12
    sc = L.synth_cfg(sensor, seed)
    rng = np.random.default_rng(seed)
    scans = []
    for k in range(K):
        p, s = L.synth_scan(sc, k)
        if not ring:
            p["x"][rng.choice(len(p), 40, replace=False)] = np.nan
            p["ring"] = rng.integers(0, 1000, len(p))  # not read by this branch
        scans.append((p, s))
    gc, oc = cfgs(L, sensor, ring=ring)
    ora = L.Oracle(oc)
    want = []
    for p, s in scans:
        wi = ora.ip(p, s)
        want.append((wi, ora.fa()))
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(K + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    gb = L.Lego(gc, max_points=max(len(p) for p, _ in scans) + 16, max_batch=K)
    recs = gb.odom_batch(pts, off, np.array([s for _, s in scans]))
    for k in range(K):
        gi, gf = gb.batch_fetch(k)
        assert_ip_equal(gi, want[k][0], images=False)
        assert_feat_equal(gf, want[k][1])
        assert np.array_equal(u32(list(recs[k].transform_sum)), u32(want[k][1]["transform_sum"])), k
    gb.close()
