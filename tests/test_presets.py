"""The reference's other sensor presets (utility.h:70-102) and the
useCloudRing = false projection branch (imageProjection.cpp:228-233) on the
CPU oracle: the preset values, the synthetic source for HDL-32E / OS1-16 /
OS1-64, and the vertical-angle row with its size_t conversion."""
import numpy as np
import pytest

NEW_PRESETS = [("HDL-32E", 32, 1800, 20), ("OS1-16", 16, 1024, 7), ("OS1-64", 64, 1024, 15)]


def ringless(L, name, lib=None):
    cfg = L.sensor_cfg(name, lib)
    cfg.use_cloud_ring = 0
    return cfg


@pytest.mark.parametrize("name,n,h,g", NEW_PRESETS)
def test_synth_presets_match_sensor_presets(L, name, n, h, g):
    sc = L.synth_cfg(name, 1)
    cfg = L.sensor_cfg(name)
    assert (sc.n_scan, sc.horizon_scan) == (cfg.n_scan, cfg.horizon_scan) == (n, h)
    assert cfg.ground_scan_ind == g
    pts, _ = L.synth_scan(sc, 0)
    assert len(pts) > 0.5 * n * h  # the downward half of the beams at least
    assert pts["ring"].max() == n - 1


@pytest.mark.parametrize("name", ["VLP-16", "HDL-32E", "OS1-16", "OS1-64"])
def test_ringless_rows_equal_ring_rows(L, name):
    """The synthetic beams sit inside their rows' vertical-angle bins, so both
    branches of :225-231 project every point to the same pixel: the images
    and clouds of the two oracle configurations are equal byte for byte.
    (VLS-128's and HDL-64E's synthetic beams sit exactly on their bins' lower
    edges, so float rounding moves some of them a row down: those sensors are
    the GPU tests' stress case for this branch, not an equality here.)"""
    sc = L.synth_cfg(name, 2)
    pts, st = L.synth_scan(sc, 0)
    a = L.Oracle(L.sensor_cfg(name)).ip(pts, st, images=True)
    b = L.Oracle(ringless(L, name)).ip(pts, st, images=True)
    for k in ("range_image", "label_image", "segmented", "col_ind", "start_ring_index"):
        assert np.array_equal(np.asarray(a[k]).view(np.uint8), np.asarray(b[k]).view(np.uint8)), k


def test_ringless_ignores_ring_channel(L):
    sc = L.synth_cfg("VLP-16", 3)
    pts, st = L.synth_scan(sc, 0)
    scrambled = pts.copy()
    scrambled["ring"] = np.random.default_rng(0).integers(0, 400, len(pts))
    a = L.Oracle(ringless(L, "VLP-16")).ip(pts, st, images=True)
    b = L.Oracle(ringless(L, "VLP-16")).ip(scrambled, st, images=True)
    assert np.array_equal(a["range_image"].view(np.uint8), b["range_image"].view(np.uint8))


def _edge_points(L, cfg, vs):
    """One point per target row value v = (verticalAngle + ang_bottom) /
    ang_res_y, 10 m out, each in its own column (v mid-way between integers,
    so the float rounding of the angle cannot move it across a bin edge)."""
    pts = np.zeros(len(vs), dtype=L.XYZIR_DTYPE)
    for i, v in enumerate(vs):
        el = np.deg2rad(v * cfg.ang_res_y - cfg.ang_bottom)
        az = np.deg2rad(90.0 - 10.0 * (i + 1))  # columns 50, 100, ... apart
        pts[i]["x"] = 10.0 * np.cos(el) * np.sin(az)
        pts[i]["y"] = 10.0 * np.cos(el) * np.cos(az)
        pts[i]["z"] = 10.0 * np.sin(el)
        pts[i]["ring"] = 3  # ignored by this branch
    return pts


def test_ringless_size_t_row_known_answers(L):
    """:230-233 with rowIdn a size_t: v in (-1, 0) truncates to row 0 (the
    reference keeps points up to one row below ang_bottom), v <= -1 wraps past
    N_SCAN and is skipped, v >= N_SCAN is skipped."""
    cfg = ringless(L, "VLP-16")
    N, H = cfg.n_scan, cfg.horizon_scan
    vs = [-0.5, -1.5, 7.5, 15.5, 16.5, -0.05]
    want = [0, None, 7, 15, None, 0]
    pts = _edge_points(L, cfg, vs)
    out = L.Oracle(cfg).ip(pts, 0.0, images=True)
    img = out["range_image"].reshape(N, H)
    hit = {}
    for r, c in zip(*np.nonzero(img != np.float32(np.finfo(np.float32).max))):
        hit[int(c)] = int(r)
    for i, (v, w) in enumerate(zip(vs, want)):
        x, y = float(pts[i]["x"]), float(pts[i]["y"])
        col = int(-round((np.degrees(np.arctan2(x, y)) - 90.0) / cfg.ang_res_x) + H // 2) % H
        assert hit.get(col) == w, (v, col, hit)


def test_ringless_nan_points_removed(L):
    """removeNaNFromPointCloud (:170): non-finite points are dropped, including
    the first and last (findStartEndAngle then reads the first / last finite
    point); the ring branch still rejects them (:173-176)."""
    sc = L.synth_cfg("VLP-16", 4)
    pts, st = L.synth_scan(sc, 0)
    dirty = pts.copy()
    rng = np.random.default_rng(1)
    idx = np.concatenate([[0, 1, len(pts) - 1], rng.choice(len(pts), 300, replace=False)])
    dirty["x"][idx] = np.nan
    clean = np.delete(pts, np.unique(idx))
    a = L.Oracle(ringless(L, "VLP-16")).ip(dirty, st, images=True)
    b = L.Oracle(ringless(L, "VLP-16")).ip(clean, st, images=True)
    for k in ("start_orientation", "end_orientation"):
        assert np.float32(a[k]).tobytes() == np.float32(b[k]).tobytes(), k
    for k in ("range_image", "segmented"):
        assert np.array_equal(np.asarray(a[k]).view(np.uint8), np.asarray(b[k]).view(np.uint8)), k
    with pytest.raises(RuntimeError, match="status 1 "):
        L.Oracle(L.sensor_cfg("VLP-16")).ip(dirty, st)
    allnan = pts[:10].copy()
    allnan["y"] = np.inf
    with pytest.raises(RuntimeError):
        L.Oracle(ringless(L, "VLP-16")).ip(allnan, st)
