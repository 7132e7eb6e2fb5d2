"""GPU parity: the HIP path through the C-ABI vs the CPU oracle on the same
seeded synthetic scans.  Bit-exact for images, labels, the segmented cloud,
cloud_info and feature clouds; poses within the north-star tolerance 1e-4."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4  # BASELINE.json north_star: "within 1e-4 on the 6-DoF pose"


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def assert_ip_equal(g, o, images=True):
    for k in ("start_orientation", "end_orientation", "orientation_diff"):
        assert np.float32(g[k]).tobytes() == np.float32(o[k]).tobytes(), k
    for k in ("start_ring_index", "end_ring_index", "ground_flag", "col_ind", "range",
              "segmented", "outlier"):
        assert g[k].shape == o[k].shape, (k, g[k].shape, o[k].shape)
        assert np.array_equal(bits(g[k]), bits(o[k])), k
    if images:
        for k in ("range_image", "ground_image", "label_image", "full_cloud"):
            assert np.array_equal(bits(g[k]), bits(o[k])), k


def assert_feat_equal(g, o):
    for k in ("sharp", "less_sharp", "flat", "less_flat"):
        assert g[k].shape == o[k].shape, (k, g[k].shape, o[k].shape)
        assert np.array_equal(bits(g[k]), bits(o[k])), k


@pytest.mark.parametrize("sensor,seed,extra", [
    ("VLP-16", 0, {}), ("VLP-16", 1, {}), ("VLP-16", 2, {"dup_frac": 0.05}),
    ("HDL-64E", 2, {}), ("VLS-128", 3, {}),
])
def test_ip_parity(L, sensor, seed, extra):
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    sc = L.synth_cfg(sensor, seed, **extra)
    pts, stamp = L.synth_scan(sc, 0)
    gpu = L.Lego(cfg, max_points=len(pts) + 16)
    ora = L.Oracle(L.sensor_cfg(sensor))
    assert_ip_equal(gpu.ip(pts, stamp, images=True), ora.ip(pts, stamp, images=True))
    gpu.close()


@pytest.mark.parametrize("sensor,seed", [("VLP-16", 0), ("HDL-64E", 2), ("VLS-128", 3)])
def test_gated_topics_parity(L, sensor, seed):
    """LEGO_IP_GATED: /full_cloud_info, /ground_cloud and /segmented_cloud_pure
    (imageProjection.cpp:480-506) byte for byte against the oracle, with the
    regular outputs unchanged."""
    sc = L.synth_cfg(sensor, seed)
    pts, stamp = L.synth_scan(sc, 0)
    gpu = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=len(pts) + 16)
    ora = L.Oracle(L.sensor_cfg(sensor))
    g = gpu.ip(pts, stamp, gated=True)
    o = ora.ip(pts, stamp, gated=True)
    assert_ip_equal(g, o, images=False)
    for k in ("full_info_cloud", "ground_cloud", "segmented_cloud_pure"):
        assert g[k].shape == o[k].shape, (k, g[k].shape, o[k].shape)
        assert np.array_equal(bits(g[k]), bits(o[k])), k
    assert "full_info_cloud" not in gpu.ip(pts, stamp)  # not materialised unless asked
    gpu.close()


@pytest.mark.parametrize("sensor,seed,nscans", [("VLP-16", 1, 12), ("HDL-64E", 2, 3)])
def test_stream_parity_node_api(L, sensor, seed, nscans):
    """ip -> fa per scan through the node-shaped calls; features bit-exact,
    poses within tolerance (and reported when bit-exact)."""
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    sc = L.synth_cfg(sensor, seed)
    gpu = L.Lego(cfg, max_points=L.synth_lib().lego_synth_max_points(L.C.byref(sc)))
    ora = L.Oracle(L.sensor_cfg(sensor))
    worst = 0.0
    for k in range(nscans):
        pts, stamp = L.synth_scan(sc, k)
        assert_ip_equal(gpu.ip(pts, stamp), ora.ip(pts, stamp), images=False)
        gf, of = gpu.fa(), ora.fa()
        assert_feat_equal(gf, of)
        assert gf["odom_valid"] == of["odom_valid"]
        assert gf["publish_to_mapping"] == of["publish_to_mapping"]
        d = float(np.max(np.abs(gf["transform_sum"].astype(np.float64) - of["transform_sum"])))
        worst = max(worst, d)
        assert d <= POSE_TOL, (k, gf["transform_sum"], of["transform_sum"])
        assert np.array_equal(gf["transform_sum"].view(np.uint32), of["transform_sum"].view(np.uint32)), k
        if gf["publish_to_mapping"]:
            for key in ("corner_last", "surf_last", "outlier_last"):
                assert np.array_equal(gf[key].view(np.uint32), of[key].view(np.uint32)), (k, key)
    print(f"{sensor}: worst |dpose| = {worst:.3g}")
    gpu.close()


def test_fa_on_oracle_input(L):
    """GPU feature association fed the ORACLE's cloud_info (host upload path)."""
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 4)
    gpu = L.Lego(cfg, max_points=40000)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    for k in range(3):
        pts, stamp = L.synth_scan(sc, k)
        ora.ip(pts, stamp)
        # feed the oracle's IpOut straight into the product's lego_fa_process
        out = L.FaOut()
        L.check(gpu.lib.lego_fa_process(gpu.h, L.C.byref(ora._ip), L.C.byref(out)), "fa", gpu.lib)
        assert_feat_equal(L.fa_to_dict(out), ora.fa())
    gpu.close()


def test_batch_equals_node_path(L):
    """lego_odom_batch over K scans == K node-shaped calls (same stream state)."""
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 5)
    K = 8
    scans = [L.synth_scan(sc, k) for k in range(K)]
    pts = np.concatenate([s[0] for s in scans])
    off = np.zeros(K + 1, np.int64)
    off[1:] = np.cumsum([len(s[0]) for s in scans])
    stamps = np.array([s[1] for s in scans])
    gb = L.Lego(cfg, max_points=40000, max_batch=K)
    recs = gb.odom_batch(pts, off, stamps)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    for k in range(K):
        ora.ip(*scans[k])
        of = ora.fa()
        gi, gf = gb.batch_fetch(k)
        assert_feat_equal(gf, of)
        r = recs[k]
        assert r.n_sharp == len(of["sharp"]) and r.n_less_flat == len(of["less_flat"])
        assert r.odom_valid == of["odom_valid"]
        d = np.max(np.abs(np.array(list(r.transform_sum), np.float64) - of["transform_sum"]))
        assert d <= POSE_TOL, (k, list(r.transform_sum), of["transform_sum"])
    gb.close()


def test_not_dense_rejected(L):
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 0)
    pts, stamp = L.synth_scan(sc, 0)
    pts = pts.copy()
    pts["x"][10] = np.nan
    gpu = L.Lego(cfg, max_points=len(pts) + 16)
    out = L.IpOut()
    st = gpu.lib.lego_ip_process(gpu.h, pts.ctypes.data, len(pts), stamp, 0, L.C.byref(out))
    assert st == L.LEGO_E_NOT_DENSE
    gpu.close()


def test_batch_argument_checks(L):
    """Empty scans and over-capacity scans are refused before any launch; a
    non-finite point is caught on the device (LEGO_E_NOT_DENSE), on both the
    host-buffer and the device-buffer paths."""
    import torch

    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 0)
    a, sa = L.synth_scan(sc, 0)
    b, sb = L.synth_scan(sc, 1)
    pts = np.concatenate([a, b])
    gpu = L.Lego(cfg, max_points=max(len(a), len(b)) + 16, max_batch=4)
    recs = (L.PoseRec * 3)()
    lib = gpu.lib
    stamps = np.array([sa, sa, sb])

    def call(p, off, on_device=0):
        if on_device:
            dp = torch.from_numpy(p.view(np.uint8)).cuda()
            do = torch.from_numpy(off).cuda()
            return lib.lego_odom_batch(gpu.h, dp.data_ptr(), do.data_ptr(), stamps.ctypes.data, len(off) - 1,
                                       1, recs)
        return lib.lego_odom_batch(gpu.h, p.ctypes.data, off.ctypes.data, stamps.ctypes.data, len(off) - 1, 0,
                                   recs)

    empty = np.array([0, len(a), len(a), len(pts)], np.int64)
    assert call(pts, empty) == L.LEGO_E_ARG
    assert call(pts, empty, 1) == L.LEGO_E_ARG
    small = L.Lego(cfg, max_points=1000, max_batch=4)
    assert small.lib.lego_odom_batch(small.h, pts.ctypes.data, np.array([0, len(a)], np.int64).ctypes.data,
                                     stamps.ctypes.data, 1, 0, recs) == L.LEGO_E_CAPACITY
    small.close()
    bad = pts.copy()
    bad["z"][len(a) + 7] = np.inf
    two = np.array([0, len(a), len(pts)], np.int64)
    assert call(bad, two) == L.LEGO_E_NOT_DENSE
    gpu.reset()
    assert call(bad, two, 1) == L.LEGO_E_NOT_DENSE
    gpu.reset()
    assert call(pts, two, 1) == L.LEGO_OK
    gpu.close()


def test_fused_batch_not_dense_word(L):
    """Batches of more than 8 VLP-16 scans take k_ip_lds, which clears each
    scan's error word itself (no fill before the batch): a non-finite point in
    scan 10 is LEGO_E_NOT_DENSE naming that scan, and after lego_reset clean
    batches through both slots succeed and equal a fresh context's records."""
    import torch

    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 4)
    K = 12
    scans = [L.synth_scan(sc, j) for j in range(3 * K)]
    maxn = max(len(p) for p, _ in scans) + 16

    def batch(lo):
        pts = np.concatenate([p for p, _ in scans[lo:lo + K]])
        off = np.zeros(K + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p, _ in scans[lo:lo + K]])
        return pts, off, np.array([s for _, s in scans[lo:lo + K]])

    def call(g, pts, off, st, recs):
        dp = torch.from_numpy(pts.view(np.uint8)).cuda()
        do = torch.from_numpy(off).cuda()
        return g.lib.lego_odom_batch(g.h, dp.data_ptr(), do.data_ptr(), st.ctypes.data, K, 1, recs)

    gpu = L.Lego(cfg, max_points=maxn, max_batch=K)
    ref = L.Lego(cfg, max_points=maxn, max_batch=K)
    recs, rref = (L.PoseRec * K)(), (L.PoseRec * K)()
    pts, off, st = batch(0)
    bad = pts.copy()
    bad["x"][off[10] + 5] = np.nan
    assert call(gpu, bad, off, st, recs) == L.LEGO_E_NOT_DENSE
    assert "scan 10" in gpu.lib.lego_last_error().decode()
    gpu.reset()
    for w in range(3):
        pts, off, st = batch(w * K)
        assert call(gpu, pts, off, st, recs) == L.LEGO_OK, gpu.lib.lego_last_error()
        assert call(ref, pts, off, st, rref) == L.LEGO_OK
        assert bytes(recs) == bytes(rref), w
    gpu.close()
    ref.close()


@pytest.mark.parametrize("sensor,seed,nscans,n_surf,n_corner", [
    ("VLP-16", 3, 14, 200000, 40000),
])
def test_scan_to_map_parity(L, sensor, seed, nscans, n_surf, n_corner):
    """mapOptimization's scan-to-map step against a fixed synthetic map (config
    C5 shape, smaller): voxel-filtered sizes bit-exact, the same processed /
    optimized decisions and iteration counts, poses within 1e-4."""
    sc = L.synth_cfg(sensor, seed)
    surf, corner = L.synth_map(seed, 50.0, n_surf, n_corner)
    ora = L.Oracle(L.sensor_cfg(sensor))
    ora.mo_set_map(corner, surf)
    gpu = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=40000)
    gpu.mo_set_map(corner, surf)
    steps = optimized = 0
    worst = 0.0
    for k in range(nscans):
        pts, stamp = L.synth_scan(sc, k)
        ora.ip(pts, stamp)
        ora.fa()
        o = ora.mo()
        gpu.ip(pts, stamp)
        gpu.fa()
        g = gpu.mo()
        assert g["processed"] == o["processed"], k
        if not o["processed"]:
            continue
        steps += 1
        for key in ("optimized", "n_corner_map_ds", "n_surf_map_ds", "n_corner_scan_ds", "n_surf_scan_ds"):
            assert g[key] == o[key], (k, key, g[key], o[key])
        optimized += int(o["optimized"])
        d = np.max(np.abs(g["transform_aft_mapped"].astype(np.float64) - o["transform_aft_mapped"]))
        worst = max(worst, float(d))
        assert d <= POSE_TOL, (k, g["transform_aft_mapped"], o["transform_aft_mapped"], g["iterations"],
                               o["iterations"], g["n_rows_last"], o["n_rows_last"])
        assert np.array_equal(g["transform_aft_mapped"].view(np.uint32), o["transform_aft_mapped"].view(np.uint32)), k
    print(f"scan-to-map: {steps} steps, {optimized} optimized, worst |dpose| = {worst:.3g}")
    assert steps >= 2 and optimized >= 1
    gpu.close()


def test_scan_to_map_gates(L):
    """run()'s gates (mapOptmization.cpp:1487-1499): nothing is processed
    before the first odometry hand-off (the initialisation scan)."""
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    sc = L.synth_cfg("VLP-16", 0)
    gpu.ip(*L.synth_scan(sc, 0))
    fa = gpu.fa()
    assert fa["odom_valid"] == 0
    assert gpu.mo()["processed"] == 0
    gpu.close()


def test_scan_to_map_keyframe_parity(L):
    """The reference's default mapping mode: the surrounding map is built from
    the saved keyframes (radius search, 1 m key-pose filter, existing-key
    bookkeeping, transformed clouds, map voxel filter).  Same decisions, sizes
    bit-exact, poses within 1e-4 over a 40-scan stream."""
    sc = L.synth_cfg("VLP-16", 6)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    steps = optimized = 0
    worst = 0.0
    for k in range(40):
        pts, stamp = L.synth_scan(sc, k)
        ora.ip(pts, stamp)
        ora.fa()
        o = ora.mo()
        gpu.ip(pts, stamp)
        gpu.fa()
        g = gpu.mo()
        assert g["processed"] == o["processed"], k
        if not o["processed"]:
            continue
        steps += 1
        for key in ("optimized", "n_corner_map_ds", "n_surf_map_ds", "n_corner_scan_ds", "n_surf_scan_ds"):
            assert g[key] == o[key], (k, key, g[key], o[key])
        optimized += int(o["optimized"])
        d = np.max(np.abs(g["transform_aft_mapped"].astype(np.float64) - o["transform_aft_mapped"]))
        worst = max(worst, float(d))
        assert d <= POSE_TOL, (k, g["transform_aft_mapped"], o["transform_aft_mapped"])
        assert np.array_equal(g["transform_aft_mapped"].view(np.uint32), o["transform_aft_mapped"].view(np.uint32)), k
    print(f"keyframe scan-to-map: {steps} steps, {optimized} optimized, worst |dpose| = {worst:.3g}")
    assert steps >= 5 and optimized >= 3
    gpu.close()


def test_keyframe_store_full_is_reported(L):
    """The keyframe store's capacity (lego_ctx_opts::kf_cap shrinks it,
    diagnostic): the step whose keyframe does not fit returns LEGO_E_CAPACITY
    itself (not a later one), every later step does too (the history is
    incomplete), and lego_reset recovers the context: the stream then matches
    a fresh one."""
    sc = L.synth_cfg("VLP-16", 6)
    scans = [L.synth_scan(sc, k) for k in range(30)]
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, opts={"kf_cap": 3})
    saved_ok, failed_at, msgs = 0, None, []
    for k, (pts, stamp) in enumerate(scans):
        gpu.ip(pts, stamp)
        gpu.fa()
        try:
            saved_ok += gpu.mo()["processed"]
        except RuntimeError as e:
            msgs.append(str(e))
            if failed_at is None:
                failed_at = k
    assert failed_at is not None and "keyframe store is full" in msgs[0], msgs[:1]
    assert "was not saved" in msgs[0] and len(msgs) >= 2, msgs  # reported at its own step, then sticky
    assert f"status {L.LEGO_E_CAPACITY}" in msgs[0]
    gpu.reset()
    got = []
    for pts, stamp in scans[:10]:
        gpu.ip(pts, stamp)
        gpu.fa()
        got.append(gpu.mo()["transform_aft_mapped"])
    gpu.close()
    fresh = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    for (pts, stamp), g in zip(scans[:10], got):
        fresh.ip(pts, stamp)
        fresh.fa()
        assert np.array_equal(fresh.mo()["transform_aft_mapped"], g)
    fresh.close()


def test_concurrent_streams_identical(L):
    """Contexts on one device driven concurrently (one host thread and HIP
    stream each) give the same pose records, byte for byte, as one context at
    a time — also with fewer odometry workgroups than the default (the
    redundant per-workgroup solve makes the count invisible)."""
    import threading

    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    K = 10
    streams = []
    for seed in (4, 5, 6, 7):
        sc = L.synth_cfg("VLP-16", seed)
        scans = [L.synth_scan(sc, k) for k in range(K)]
        pts = np.concatenate([s[0] for s in scans])
        off = np.zeros(K + 1, np.int64)
        off[1:] = np.cumsum([len(s[0]) for s in scans])
        streams.append((pts, off, np.array([s[1] for s in scans])))

    def run(ctx, st):
        pts, off, stamps = st
        h = K // 2  # two batches: the odometry state crosses a launch boundary
        a = bytes(ctx.odom_batch(pts[:off[h]], off[:h + 1], stamps[:h]))
        b = bytes(ctx.odom_batch(pts[off[h]:], off[h:] - off[h], stamps[h:]))
        raw = a + b
        return [raw[64 * k:64 * k + 60] for k in range(K)]  # every field but the pad word

    ref = []
    for st in streams:
        g = L.Lego(cfg, max_points=40000, max_batch=K)
        ref.append(run(g, st))
        g.close()
    ctxs = []
    for wg in (None, 16, 4, 1):
        ctxs.append(L.Lego(cfg, max_points=40000, max_batch=K, opts={"odom_workgroups": wg} if wg else None))
    got = [None] * len(ctxs)
    errs = []

    def worker(i):
        try:
            got[i] = run(ctxs[i], streams[i])
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(ctxs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs:
        c.close()
    assert not errs, errs
    for i in range(len(ctxs)):
        assert got[i] == ref[i], i


@pytest.mark.parametrize("sensor,seeds,K,cap,workgroups", [
    ("VLP-16", (4, 8, 9), 8, 40000, None), ("VLP-16", (4, 8, 9), 8, 40000, 1),
    ("HDL-64E", (2, 5), 4, 140000, None)])
def test_fleet_equals_single_streams(L, sensor, seeds, K, cap, workgroups):
    """A fleet context (lego_fleet_create: S streams, one launch per stage for
    all of them) gives each stream the same pose records, byte for byte, as
    the stream's own context, across two stream-major batches (the states
    and the FA carries cross the launch boundary per stream).  HDL-64E: the
    HBM-resident odometry with its per-stream hand-off exchange."""
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    S = len(seeds)
    streams = []
    for seed in seeds:
        sc = L.synth_cfg(sensor, seed)
        streams.append([L.synth_scan(sc, k) for k in range(K)])

    def pack(scans):
        pts = np.concatenate([p for p, _ in scans])
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p, _ in scans])
        return pts, off, np.array([t for _, t in scans])

    ref = []
    for scans in streams:
        g = L.Lego(cfg, max_points=cap, max_batch=K)
        raw = bytes(g.odom_batch(*pack(scans[:K // 2]))) + bytes(g.odom_batch(*pack(scans[K // 2:])))
        g.close()
        ref.append([raw[64 * k:64 * k + 60] for k in range(K)])
    fl = L.Lego(cfg, max_points=cap, max_batch=K // 2, streams=S,
                opts={"odom_workgroups": workgroups} if workgroups else None)
    got = [[] for _ in range(S)]
    for h in (slice(0, K // 2), slice(K // 2, K)):
        batch = [sc for scans in streams for sc in scans[h]]  # stream-major
        raw = bytes(fl.odom_batch(*pack(batch)))
        for s in range(S):
            for k in range(K // 2):
                r = s * (K // 2) + k
                got[s].append(raw[64 * r:64 * r + 60])
    # a batch that is not S x K scans is refused
    with pytest.raises(RuntimeError):
        fl.odom_batch(*pack([streams[s][0] for s in range(S)] + [streams[0][1]]))
    fl.close()
    for s in range(S):
        assert got[s] == ref[s], s


def test_hbm_reset_clears_handoff_exchange(L):
    """HBM-resident odometry (HDL-64E): after lego_reset the hand-off sequence
    restarts, so the exchange's granules must be cleared with it.  A context
    that ran one stream, was reset and then ran another gives the second
    stream's records byte for byte as a fresh context."""
    cfg = L.sensor_cfg("HDL-64E", L.hip_lib())

    def pack(scans):
        pts = np.concatenate([p for p, _ in scans])
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p, _ in scans])
        return pts, off, np.array([t for _, t in scans])

    a = [L.synth_scan(L.synth_cfg("HDL-64E", 2), k) for k in range(4)]
    b = [L.synth_scan(L.synth_cfg("HDL-64E", 5), k) for k in range(4)]
    g = L.Lego(cfg, max_points=140000, max_batch=4)
    g.odom_batch(*pack(a))
    g.reset()
    got = bytes(g.odom_batch(*pack(b)))
    g.close()
    f = L.Lego(cfg, max_points=140000, max_batch=4)
    want = bytes(f.odom_batch(*pack(b)))
    f.close()
    assert [got[64 * k:64 * k + 60] for k in range(4)] == [want[64 * k:64 * k + 60] for k in range(4)]


def test_async_batches_equal_sync(L):
    """lego_odom_batch_submit / _wait two deep (the second batch's extraction
    overlapping the first one's odometry, the slots alternating) gives the
    same records as synchronous lego_odom_batch calls; misuse is refused."""
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 11)
    K, nb = 5, 4
    scans = [L.synth_scan(sc, k) for k in range(K * nb)]

    def pack(lo, hi):
        pts = np.concatenate([p for p, _ in scans[lo:hi]])
        off = np.zeros(hi - lo + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p, _ in scans[lo:hi]])
        return pts, off, np.array([t for _, t in scans[lo:hi]])

    a = L.Lego(cfg, max_points=40000, max_batch=K)
    ref = [bytes(a.odom_batch(*pack(i * K, (i + 1) * K))) for i in range(nb)]
    a.close()
    b = L.Lego(cfg, max_points=40000, max_batch=K)
    keep, got = [], []
    recs = (L.PoseRec * K)()
    for i in range(nb):
        pts, off, st = pack(i * K, (i + 1) * K)
        keep.append((pts, off, st))
        assert b.lib.lego_odom_batch_submit(b.h, pts.ctypes.data, off.ctypes.data, st.ctypes.data, K, 0,
                                            None, 0, None) == 0
        if i >= 1:
            if i == 1:  # a third batch in flight and a node call are refused
                assert b.lib.lego_odom_batch_submit(b.h, pts.ctypes.data, off.ctypes.data, st.ctypes.data, K,
                                                    0, None, 0, None) == L.LEGO_E_STATE
                out = L.IpOut()
                assert b.lib.lego_fa_process(b.h, C.byref(out), C.byref(L.FaOut())) == L.LEGO_E_STATE
            b.wait(recs)
            got.append(bytes(recs))
    b.wait(recs)
    got.append(bytes(recs))
    assert b.lib.lego_odom_batch_wait(b.h, recs, K, None) == L.LEGO_E_STATE
    b.close()
    for i in range(nb):
        for k in range(K):
            assert ref[i][64 * k:64 * k + 60] == got[i][64 * k:64 * k + 60], (i, k)


def test_reset_in_flight(L):
    """lego_reset with a batch in flight: that batch finishes with the old
    state, the next one starts fresh (== a new context)."""
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    sc = L.synth_cfg("VLP-16", 12)
    K = 4
    scans = [L.synth_scan(sc, k) for k in range(2 * K)]
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(2 * K + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    st = np.array([t for _, t in scans])
    lo, hi = (pts[:off[K]], off[:K + 1], st[:K]), (pts[off[K]:], off[K:] - off[K], st[K:])
    a = L.Lego(cfg, max_points=40000, max_batch=K)
    r1 = bytes(a.odom_batch(*lo))
    a.close()
    a = L.Lego(cfg, max_points=40000, max_batch=K)
    r2 = bytes(a.odom_batch(*hi))  # the second half from a fresh state
    a.close()
    b = L.Lego(cfg, max_points=40000, max_batch=K)
    recs = (L.PoseRec * K)()
    keep = [lo, hi]
    for p, o, s_ in keep:
        assert b.lib.lego_odom_batch_submit(b.h, p.ctypes.data, o.ctypes.data, s_.ctypes.data, K, 0,
                                            None, 0, None) == 0
        if p is lo[0]:
            b.reset()
    b.wait(recs)
    g1 = bytes(recs)
    b.wait(recs)
    g2 = bytes(recs)
    b.close()
    for k in range(K):
        assert r1[64 * k:64 * k + 60] == g1[64 * k:64 * k + 60], k
        assert r2[64 * k:64 * k + 60] == g2[64 * k:64 * k + 60], k


@pytest.mark.parametrize("seed,extra", [(0, {}), (1, {}), (2, {"dup_frac": 0.05})])
def test_seg_lds_equals_hbm_union_find(L, seed, extra):
    """VLP-16 batches of more than kSegHbmMaxScans (8) scans are projected and
    segmented in LDS, by default in one kernel per scan (k_ip_lds), with
    lego_ctx_opts::ip_fused = 0 by k_project / k_pixels / k_ground + k_seg_lds;
    node calls (one scan) and the seg_hbm option (diagnostic) go through the
    HBM union-find (k_ccl_* + k_compact) that the larger sensors use.  All
    equal the oracle, clouds and cloud_info byte for byte on 12 consecutive
    scans (and labels / images through the node calls)."""
    sc = L.synth_cfg("VLP-16", seed, **extra)
    scans = [L.synth_scan(sc, k) for k in range(12)]
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    ref = [ora.ip(p, s, images=True) for p, s in scans]
    cap = max(len(p) for p, _ in scans) + 16
    pts = np.concatenate([p for p, _ in scans])
    offs = np.concatenate([[0], np.cumsum([len(p) for p, _ in scans])]).astype(np.int64)
    stamps = np.array([s for _, s in scans], dtype=np.float64)
    outs = {}
    for mode in ("lds", "lds4", "hbm"):
        gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap, max_batch=len(scans),
                     opts={"seg_hbm": int(mode == "hbm"), "ip_fused": int(mode == "lds")})
        gpu.odom_batch(pts, offs, stamps)
        outs[mode] = [gpu.batch_fetch(k)[0] for k in range(len(scans))]
        gpu.close()
    node = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap)
    outs["node"] = [node.ip(p, s, images=True) for p, s in scans]
    node.close()
    for k in range(len(scans)):
        assert_ip_equal(outs["lds"][k], ref[k], images=False)
        assert_ip_equal(outs["lds4"][k], ref[k], images=False)
        assert_ip_equal(outs["hbm"][k], ref[k], images=False)
        assert_ip_equal(outs["node"][k], ref[k])


def test_node_upload_capacity_and_chunks(L):
    """The node call's staged upload (lego_ip_process): a cloud of exactly
    max_points points, spanning several 32768-point chunks, projects like the
    oracle; one point more is LEGO_E_CAPACITY before any upload; a cloud with
    a non-finite point in its last chunk is refused and the context keeps
    working."""
    sc = L.synth_cfg("HDL-64E", 2)
    pts, st = L.synth_scan(sc, 0)
    n = len(pts)
    assert n > 3 * 32768
    cfg = L.sensor_cfg("HDL-64E", L.hip_lib())
    gpu = L.Lego(cfg, max_points=n)
    ora = L.Oracle(L.sensor_cfg("HDL-64E"))
    assert_ip_equal(gpu.ip(pts, st, images=True), ora.ip(pts, st, images=True))
    big = np.concatenate([pts, pts[:1]])
    out = L.IpOut()
    assert gpu.lib.lego_ip_process(gpu.h, big.ctypes.data, len(big), st, 0, L.C.byref(out)) == L.LEGO_E_CAPACITY
    bad = pts.copy()
    bad["y"][n - 3] = np.inf
    assert gpu.lib.lego_ip_process(gpu.h, bad.ctypes.data, n, st, 0, L.C.byref(out)) == L.LEGO_E_NOT_DENSE
    pts1, st1 = L.synth_scan(sc, 1)
    if len(pts1) <= n:
        assert_ip_equal(gpu.ip(pts1, st1, images=True), L.Oracle(L.sensor_cfg("HDL-64E")).ip(pts1, st1, images=True))
    gpu.close()
