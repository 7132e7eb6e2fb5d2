"""Known-answer tests for the CPU oracle, derived by hand from the reference
source (the reference ships no tests or golden data — SURVEY.md §4).  Each
case names the lines whose behaviour it pins."""
import math

import numpy as np
import pytest

H, N, G = 1800, 16, 7  # VLP-16 (utility.h:63-68)


def pt(L, ring, col, rng, elev_deg=None, inten=0.0):
    """A point that projects to (ring, col) at range rng: column centre azimuth
    theta = 0.2*col - 180 deg (imageProjection.cpp:235-237 inverted)."""
    th = math.radians(0.2 * col - 180.0)
    el = math.radians(-15.0 + 2.0 * ring if elev_deg is None else elev_deg)
    p = np.zeros(1, dtype=L.XYZIR_DTYPE)
    p["x"] = rng * math.cos(el) * math.cos(th)
    p["y"] = rng * math.cos(el) * math.sin(th)
    p["z"] = rng * math.sin(el)
    p["intensity"] = inten
    p["ring"] = ring
    return p


def run_ip(L, pts):
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    return ora.ip(np.concatenate(pts), 0.0, images=True)


def idx(r, c):
    return r * H + c


def cloud_projection(L):
    pts = [pt(L, 3, 900, 10.0), pt(L, 3, 900, 20.0),  # same pixel: the second wins
           pt(L, 5, 1000, 0.5),                         # below sensorMinimumRange
           pt(L, 4, 450, 7.0)]
    bad = pt(L, 3, 100, 5.0)
    bad["ring"] = 16                                    # rowIdn >= N_SCAN
    return pts + [bad]


def test_projection_last_writer_wins(L):
    """:219-256 — ring -> row, atan2f -> column, range < 1 m dropped, ring >=
    N_SCAN dropped, later points overwrite earlier ones, intensity = row + col/1e4."""
    out = run_ip(L, cloud_projection(L))
    r = out["range_image"]
    assert r[idx(3, 900)] == pytest.approx(20.0, abs=1e-5)
    assert r[idx(4, 450)] == pytest.approx(7.0, abs=1e-5)
    assert r[idx(5, 1000)] == np.finfo(np.float32).max
    assert r[idx(3, 100)] == np.finfo(np.float32).max
    fc = out["full_cloud"]
    assert fc["intensity"][idx(3, 900)] == np.float32(3 + 900 / 10000.0)
    assert fc["intensity"][idx(4, 450)] == np.float32(4 + 450 / 10000.0)
    assert fc["intensity"][idx(5, 1000)] == -1.0 and np.isnan(fc["x"][idx(5, 1000)])
    assert (r < np.finfo(np.float32).max).sum() == 2


def cloud_ground(L, col=900):
    pts = []
    for ring in range(4):  # rows 0..3 on the plane z = -0.6
        el = math.radians(-15.0 + 2.0 * ring)
        pts.append(pt(L, ring, col, 0.6 / math.sin(-el)))
    for ring in (5, 6, 7):  # a wall at 5 m: steep pairs
        el = math.radians(-15.0 + 2.0 * ring)
        pts.append(pt(L, ring, col, 5.0 / math.cos(el)))
    return pts


def test_ground_overwrite_semantics(L):
    """:267-291 — column walk i = 0..g-1: an invalid pair writes -1 at row i,
    overwriting the 1 the previous (valid, flat) pair wrote there."""
    col = 900
    out = run_ip(L, cloud_ground(L, col))
    g = out["ground_image"].reshape(N, H)[:, col]
    np.testing.assert_array_equal(g[:8], [1, 1, 1, -1, -1, 0, 0, 0])
    assert (g[8:] == 0).all()
    lab = out["label_image"].reshape(N, H)[:, col]
    assert (lab[:3] == -1).all()          # ground
    assert lab[4] == -1                   # empty pixel (range FLT_MAX)


def cloud_segmentation(L):
    pts = []
    # A: 30 pixels in row 10, cols 100..129, range 10 -> valid
    pts += [pt(L, 10, c, 10.0) for c in range(100, 130)]
    # B: seed (9,300) alone on its row, pushed rows {10, 11}: 5 px, 2 lines -> INVALID
    pts += [pt(L, r, c, 10.0) for r, c in [(9, 300), (10, 300), (11, 300), (11, 301), (11, 302)]]
    # C: seed (9,500); pushed rows {9, 10, 11, 12}: 5 px, 4 lines -> valid
    pts += [pt(L, r, c, 10.0) for r, c in [(9, 500), (9, 501), (10, 500), (11, 500), (12, 500)]]
    # D: 4 pixels -> invalid
    pts += [pt(L, 13, c, 10.0) for c in range(700, 704)]
    # E: 30 pixels across the column wrap (row 14, cols 1790..1799 and 0..19) -> valid
    pts += [pt(L, 14, c, 10.0) for c in list(range(1790, 1800)) + list(range(0, 20))]
    # F: range jump breaks the edge test: two singletons
    pts += [pt(L, 15, 900, 10.0), pt(L, 15, 901, 20.0)]
    return pts


def test_segmentation_validity_rules(L):
    """:370-460 — components of the 4-neighbourhood with column wrap; valid if
    size >= 30 or (size >= 5 and >= 3 distinct rows among the PUSHED pixels:
    lineCountFlag is never set for the seed, :431); labels count valid
    components in raster order of their seeds; invalid ones become 999999."""
    out = run_ip(L, cloud_segmentation(L))
    lab = out["label_image"].reshape(N, H)
    # raster order of seeds: C (9,500) < A (10,100) < E (14,0)
    assert (lab[10, 100:130] == 2).all()
    for r, c in [(9, 300), (10, 300), (11, 300), (11, 301), (11, 302)]:
        assert lab[r, c] == 999999
    for r, c in [(9, 500), (9, 501), (10, 500), (11, 500), (12, 500)]:
        assert lab[r, c] == 1
    assert (lab[13, 700:704] == 999999).all()
    assert (lab[14, 1790:1800] == 3).all() and (lab[14, 0:20] == 3).all()
    assert lab[15, 900] == 999999 and lab[15, 901] == 999999
    # segmented cloud = valid labels (no ground here), row-major; outliers: invalid,
    # row > g and col % 5 == 0 (:328-334)
    assert len(out["segmented"]) == 30 + 5 + 30
    outl_cols = sorted(int(round(float(i) % 1 * 1e4)) for i in out["outlier"]["intensity"])
    # B's (9|10|11, 300), D's (13, 700), F's (15, 900)
    assert outl_cols == [300, 300, 300, 700, 900]
    # cloud_info ring indices (:323, :354): start = count_before - 1 + 5, end = count_after - 1 - 5
    sri, eri = out["start_ring_index"], out["end_ring_index"]
    counts = np.bincount(np.floor(out["segmented"]["intensity"]).astype(int), minlength=N)
    before = np.concatenate([[0], np.cumsum(counts)[:-1]])
    np.testing.assert_array_equal(sri, before - 1 + 5)
    np.testing.assert_array_equal(eri, np.cumsum(counts) - 1 - 5)


def test_voxel_grid_centroids(L):
    """pcl::VoxelGrid: ijk = floor(p/leaf) - floor(min/leaf), idx = i + j*dx + k*dx*dy,
    output ordered by idx, centroid = float sum / count (PCL 1.8 voxel_grid.hpp)."""
    import ctypes as C

    pts = np.array([(0.05, 0.05, 0.05, 1.0), (0.15, 0.1, 0.1, 3.0), (0.25, 0.0, 0.0, 5.0),
                    (0.05, 0.45, 0.0, 7.0)], dtype=L.XYZI_DTYPE)
    out = np.zeros(8, dtype=L.XYZI_DTYPE)
    n = C.c_int32()
    lib = L.oracle_lib()
    assert lib.lego_oracle_voxel_grid(pts.ctypes.data, len(pts), 0.2, 0, out.ctypes.data, C.byref(n)) == 0
    f = np.float32
    # voxels (i,j,k): p0,p1 -> (0,0,0); p2 -> (1,0,0); p3 -> (0,2,0); idx = i + j*dx, dx = 2
    exp = [((f(0.05) + f(0.15)) / f(2), (f(0.05) + f(0.1)) / f(2), (f(0.05) + f(0.1)) / f(2), f(2.0)),
           (f(0.25), f(0.0), f(0.0), f(5.0)),
           (f(0.05), f(0.45), f(0.0), f(7.0))]
    got = out[: n.value]
    assert n.value == 3
    for g_, e in zip(got, exp):
        assert tuple(np.float32(v) for v in g_) == tuple(np.float32(v) for v in e)


def cloud_single(L):
    return [pt(L, 8, 1234, 12.0)]


def test_empty_scan_rejected(L):
    """findStartEndAngle reads points[0] and points[size-1]
    (imageProjection.cpp:201-203), so an empty scan is undefined upstream; the
    boundary rejects it with LEGO_E_ARG instead."""
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    with pytest.raises(RuntimeError, match="status 4"):
        ora.ip(np.zeros(0, dtype=L.XYZIR_DTYPE), 0.0)


def test_single_point_scan(L):
    """One point: projected, too small to segment, an outlier only if its column
    is a multiple of 5 (1234 is not), no features."""
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    out = ora.ip(np.concatenate(cloud_single(L)), 0.0, images=True)
    assert (out["range_image"] < np.finfo(np.float32).max).sum() == 1
    assert out["label_image"].reshape(N, H)[8, 1234] == 999999
    assert len(out["segmented"]) == 0 and len(out["outlier"]) == 0
    fa = ora.fa()
    assert all(len(fa[k]) == 0 for k in ("sharp", "less_sharp", "flat", "less_flat"))


@pytest.mark.gpu
def test_product_rejects_empty_scan(L):
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=64)
    with pytest.raises(RuntimeError, match="status 4"):
        gpu.ip(np.zeros(0, dtype=L.XYZIR_DTYPE), 0.0)
    gpu.close()


@pytest.mark.gpu
@pytest.mark.parametrize("make", [cloud_single, cloud_projection, cloud_ground, cloud_segmentation])
def test_product_on_kat_clouds(L, make):
    """The HIP product on the hand-built clouds: every image and cloud equal to
    the oracle's, bit for bit (empty and near-empty scans included)."""
    pts = np.concatenate(make(L))
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    o = ora.ip(pts, 0.0, images=True)
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=len(pts) + 16)
    g = gpu.ip(pts, 0.0, images=True)
    for k, v in o.items():
        a, b = np.asarray(v), np.asarray(g[k])
        if a.ndim == 0:
            a, b = np.array([v], np.float32), np.array([g[k]], np.float32)
        if a.dtype.names:
            a, b = a.view(np.uint8), b.view(np.uint8)
        elif a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        np.testing.assert_array_equal(a, b, err_msg=k)
    gpu.close()


def test_voxel_order_sensitivity_bounded(L):
    """PCL sums each voxel after the unstable std::sort of (idx, point)
    (SURVEY.md §9.9); the oracle and the product reproduce that order.  Summing
    in input order instead (vg_opts=0, rounds 1-2's product) changes only the
    less-flat centroids' last bits: over a 12-scan stream, features of the
    same membership and poses within the north-star 1e-4 — the size of what
    the summation order alone moves."""
    sc = L.synth_cfg("VLP-16", 4)
    a = L.Oracle(L.sensor_cfg("VLP-16"), vg_opts=0)
    b = L.Oracle(L.sensor_cfg("VLP-16"))
    worst = 0.0
    for k in range(12):
        pts, stamp = L.synth_scan(sc, k)
        a.ip(pts, stamp)
        b.ip(pts, stamp)
        fa, fb = a.fa(), b.fa()
        for key in ("sharp", "less_sharp", "flat"):
            np.testing.assert_array_equal(fa[key].view(np.uint8), fb[key].view(np.uint8))
        assert len(fa["less_flat"]) == len(fb["less_flat"])
        worst = max(worst, float(np.max(np.abs(fa["transform_sum"].astype(np.float64) - fb["transform_sum"]))))
    assert worst <= 1e-4, worst


def test_level_stationary_imu(L):
    """KAT: an IMU that reads level, still and gravity only (identity
    orientation, zero gyro, a = +g) leaves every de-skewed point and the
    odometry exactly as without an IMU — all IMU angles, velocities and
    angular increments are 0, so TransformToStartIMU / PluginIMURotation /
    TransformToEnd reduce to identities (sin 0 = 0, cos 0 = 1).  Mapping
    differs only by transformUpdate's blend toward the level attitude
    (mapOptmization.cpp:488-489): at the first optimized step
    aft[0] = (float)(0.998 * aft_noimu[0] + 0.002 * 0), likewise aft[2]."""
    sc = L.synth_cfg("VLP-16", 2)
    cfg = L.sensor_cfg("VLP-16")
    a, b = L.Oracle(cfg), L.Oracle(cfg)
    imu = np.zeros(60, dtype=L.IMU_DTYPE)
    imu["stamp"] = 0.005 + 0.01 * np.arange(60)
    imu["orientation"][:, 3] = 1.0
    imu["linear_acceleration"][:, 2] = 9.81
    j = 0
    blended = False
    for k in range(6):
        pts, st = L.synth_scan(sc, k)
        n = int(np.searchsorted(imu["stamp"], st + 0.1))
        b.imu(imu[j:n])
        j = n
        a.ip(pts, st); fa_a = a.fa(); mo_a = a.mo()
        b.ip(pts, st); fa_b = b.fa(); mo_b = b.mo()
        assert np.array_equal(fa_a["transform_sum"].view(np.uint32), fa_b["transform_sum"].view(np.uint32)), k
        for key in ("sharp", "less_sharp", "flat", "less_flat"):
            assert np.array_equal(fa_a[key].view(np.float32), fa_b[key].view(np.float32)), (k, key)
        if blended:
            continue
        if mo_a["optimized"]:
            ta, tb = mo_a["transform_aft_mapped"], mo_b["transform_aft_mapped"]
            for i in (0, 2):
                assert tb[i] == np.float32(0.998 * np.float64(ta[i]) + 0.002 * 0.0), (k, i)
            for i in (1, 3, 4, 5):
                assert tb[i] == ta[i], (k, i)
            blended = True
        else:
            assert np.array_equal(mo_a["transform_aft_mapped"], mo_b["transform_aft_mapped"]), k
    assert blended


def test_fusion_without_mapping_is_odometry(L):
    """KAT (transformFusion.cpp:94-205): before any /aft_mapped_to_init the
    correction is the identity (aft = bef = 0), so /integrated_to_init
    reproduces /laser_odom_to_init up to float rounding of the composition."""
    sc = L.synth_cfg("VLP-16", 3)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    for k in range(6):
        pts, st = L.synth_scan(sc, k)
        ora.ip(pts, st)
        fa = ora.fa()
        m = ora.fusion()
        assert np.abs(m.astype(np.float64) - fa["transform_sum"]).max() < 2e-6, (k, m, fa["transform_sum"])


def test_oracle_loop_closure_on_a_circle(L):
    """performLoopClosure (mapOptmization.cpp:875-945) restated: on a drive in
    a 3.8 m circle no history keyframe qualifies before 30 s; afterwards the
    closest old keyframe is found, the ICP converges to a near-identity
    correction (the synthetic odometry drifts little) with a fitness below
    historyKeyframeFitnessScore, and the constraint is a proper rigid motion."""
    import numpy as np

    sc = L.synth_cfg("VLP-16", 6, yaw_rate_dps=15.0, speed_mps=1.0)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    for k in range(340):
        ora.ip(*L.synth_scan(sc, k))
        ora.fa()
        ora.mo()
        if k == 289:
            early = ora.loop_closure()
            assert early["detected"] == 0 and early["closest_id"] == -1
    o = ora.loop_closure()
    assert o["detected"] == 1 and o["converged"] == 1 and o["accepted"] == 1
    assert 0 <= o["closest_id"] < o["latest_id"] and o["n_source"] > 100 and o["n_target"] > 1000
    assert 1 <= o["iterations"] < 100 and 0 < o["fitness"] < 0.3
    T = o["icp_transform"].reshape(4, 4)
    assert np.allclose(T[3], [0, 0, 0, 1]) and np.max(np.abs(T[:3, :3] - np.eye(3))) < 0.05
    assert np.max(np.abs(T[:3, 3])) < 0.5
    for key in ("from_rotation", "to_rotation", "between_rotation"):
        R = o[key].reshape(3, 3)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-6) and abs(np.linalg.det(R) - 1) < 1e-6, key


def test_gated_topics_follow_the_images(L):
    """publishCloud's gated topics (imageProjection.cpp:480-506) restated from
    the images they are cut from: /full_cloud_info is the full cloud with
    intensity = range where a point was written (:252-254, else the NaN point
    with intensity -1), /ground_cloud the full-cloud points with groundMat == 1
    in rows <= groundScanInd in row-major order (:301-308), and
    /segmented_cloud_pure the points with a valid label, intensity = label
    (:357-367)."""
    sc = L.synth_cfg("VLP-16", 0)
    pts, stamp = L.synth_scan(sc, 0)
    o = L.Oracle(L.sensor_cfg("VLP-16")).ip(pts, stamp, images=True, gated=True)
    full, rng, gnd, lab = o["full_cloud"], o["range_image"], o["ground_image"], o["label_image"]
    written = rng != np.finfo(np.float32).max
    info = full.copy()
    info["intensity"][written] = rng[written]
    assert np.array_equal(o["full_info_cloud"].view(np.uint8), info.view(np.uint8))
    rows = np.arange(N * H) // H
    assert np.array_equal(o["ground_cloud"].view(np.uint8), full[(gnd == 1) & (rows <= G)].view(np.uint8))
    sel = (lab > 0) & (lab != 999999)
    pure = full[sel].copy()
    pure["intensity"] = lab[sel].astype(np.float32)
    assert np.array_equal(o["segmented_cloud_pure"].view(np.uint8), pure.view(np.uint8))
    assert len(o["ground_cloud"]) > 100 and len(o["segmented_cloud_pure"]) > 100
