"""The two places where bit-exactness is most likely to break silently, forced
and checked against the oracle, with the pose record's path flags proving the
branch was taken (include/lego_loam.h LEGO_REC_*):

* sector-sort ties.  The product sorts each sector with a wave-local bitonic
  network and falls back to the libstdc++ introsort restatement when two
  curvatures are equal, so equal keys keep std::sort's order
  (featureAssociation.cpp:699, lego_fa.hip).  Ranges quantised to 5 cm make
  equal curvatures in nearly every sector; the records carry
  LEGO_REC_SORT_TIES and the four feature clouds must equal the oracle's byte
  for byte;
* the odometry's switch between LDS-resident and HBM-resident last clouds
  (lego_odom.hip): a VLP-16 stream whose less-flat cloud crosses the 4096-point
  LDS cap downwards and back up mid-stream (a denser far-wall scene, seed 23).
  LEGO_REC_ODOM_HBM must be set exactly on the scans whose previous scan's
  clouds exceeded the caps, and the poses must match the oracle across both
  switches;
* the speculative sector-parallel picking of k_extract (rings other than 0
  walk their six sectors at once and re-walk a sector whose predecessor's
  boundary suppression reached a position it picked): lego_extract_profile's
  counters prove both the parallel walks and re-walks ran, and the four
  feature clouds must equal the oracle's byte for byte;
* starved scans mid-stream (a sensor blocked but for a narrow sector: scans
  with no features at all, or a few): the LM gate on the last clouds' sizes
  and the few-rows guards, in a single-stream context and in a fleet (hashed
  grids over near-empty clouds), every pose equal to the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4  # BASELINE.json north_star
LDS_SURF, LDS_CORNER = 4096, 2048  # k_odom's LDS caps (lego_odom.hip kLdsSurf / kLdsCorner)
REC_SORT_TIES, REC_ODOM_HBM = 4, 8


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def quantise(pts, q):
    """Moves every point along its ray so its range is a multiple of q."""
    p = pts.copy()
    x, y, z = (p[k].astype(np.float64) for k in ("x", "y", "z"))
    r = np.sqrt(x * x + y * y + z * z)
    s = np.round(r / q) * q / r
    for k, v in (("x", x), ("y", y), ("z", z)):
        p[k] = (v * s).astype(np.float32)
    return p


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


def _oracle(L, scans):
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    out = []
    for p, s in scans:
        ora.ip(p, s)
        out.append(ora.fa())
    return out


def _check_recs(recs, ref, label):
    worst, exact = 0.0, 0
    for k, (r, o) in enumerate(zip(recs, ref)):
        ts = np.array(list(r.transform_sum), np.float64)
        assert (r.n_sharp, r.n_less_sharp, r.n_flat, r.n_less_flat, r.odom_valid) == (
            len(o["sharp"]), len(o["less_sharp"]), len(o["flat"]), len(o["less_flat"]), o["odom_valid"]), (label, k)
        d = float(np.max(np.abs(ts - o["transform_sum"].astype(np.float64))))
        assert d <= POSE_TOL, (label, k, ts, o["transform_sum"])
        worst = max(worst, d)
        exact += int(np.array_equal(ts.astype(np.float32).view(np.uint32),
                                    o["transform_sum"].astype(np.float32).view(np.uint32)))
    print(f"{label}: {len(recs)} scans, worst |dpose| {worst:.3g}, bit-exact {exact}/{len(recs)}")
    assert exact == len(recs), f"{label}: only {exact}/{len(recs)} poses bit-exact"


def test_sector_sort_ties_match_oracle(L):
    sc = L.synth_cfg("VLP-16", 0)
    scans = [(quantise(p, 0.05), s) for p, s in (L.synth_scan(sc, k) for k in range(8))]
    ref = _oracle(L, scans)
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for p, _ in scans) + 16
    gpu = L.Lego(cfg, max_points=cap)
    for k, (p, s) in enumerate(scans):  # node-shaped path: the feature clouds themselves
        gpu.ip(p, s)
        g = gpu.fa()
        for key in ("sharp", "less_sharp", "flat", "less_flat"):
            assert np.array_equal(bits(g[key]), bits(ref[k][key])), (k, key)
    gpu.close()
    gpu = L.Lego(cfg, max_points=cap, max_batch=len(scans))
    recs = list(gpu.odom_batch(*_pack(scans)))
    gpu.close()
    assert all(r.flags & REC_SORT_TIES for r in recs), [r.flags for r in recs]
    _check_recs(recs, ref, "quantised ranges (sort ties)")


def test_lds_hbm_switch_mid_stream(L):
    sc = L.synth_cfg("VLP-16", 23, n_walls=10, n_boxes=50, n_cylinders=30, dropout=0.0, speed_mps=3.0)
    scans = [L.synth_scan(sc, k) for k in range(16)]
    ref = _oracle(L, scans)
    over = [len(o["less_flat"]) > LDS_SURF or len(o["less_sharp"]) > LDS_CORNER for o in ref]
    # the stream crosses the cap both ways (the test's premise)
    assert any(over[:7]) and not all(over) and over[-1], [len(o["less_flat"]) for o in ref]
    expect_hbm = [False] + over[:-1]  # scan k's LM runs on scan k-1's clouds
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for p, _ in scans) + 16
    gpu = L.Lego(cfg, max_points=cap, max_batch=8)
    recs = list(gpu.odom_batch(*_pack(scans[:8]))) + list(gpu.odom_batch(*_pack(scans[8:])))
    gpu.close()
    assert [bool(r.flags & REC_ODOM_HBM) for r in recs] == expect_hbm, [r.flags for r in recs]
    _check_recs(recs, ref, "LDS <-> HBM residency switch")


def test_speculative_picking_rewalks_match_oracle(L):
    import ctypes as C

    sc = L.synth_cfg("VLP-16", 12)
    scans = [L.synth_scan(sc, k) for k in range(10)]
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    lib = L.hip_lib()
    gpu = L.Lego(L.sensor_cfg("VLP-16", lib), max_points=max(len(p) for p, _ in scans) + 16)
    L.check(lib.lego_odom_profile(gpu.h, 1, None), "lego_odom_profile", lib)
    for k, (p, s) in enumerate(scans):
        gpu.ip(p, s)
        g = gpu.fa()
        ora.ip(p, s)
        o = ora.fa()
        for key in ("sharp", "less_sharp", "flat", "less_flat"):
            assert np.array_equal(bits(g[key]), bits(o[key])), (k, key)
    xp = (C.c_uint64 * 8)()
    L.check(lib.lego_extract_profile(gpu.h, xp), "lego_extract_profile", lib)
    gpu.close()
    rings, rewalks, parallel = xp[4], xp[5], xp[6]
    print(f"rings {rings}, picked in parallel {parallel}, sector re-walks {rewalks}")
    assert rings >= 10 * 16 and parallel > 0 and rewalks > 0


def wedge(pts, a0_deg, width_deg):
    """The points of a scan whose azimuth lies in [a0, a0 + width) degrees, in
    their firing order (a sensor blocked but for a narrow sector)."""
    az = np.degrees(np.arctan2(pts["y"].astype(np.float64), pts["x"].astype(np.float64))) % 360.0
    keep = (az >= a0_deg) & (az < a0_deg + width_deg)
    assert keep.any()
    return pts[keep]


def _sparse_stream(L):
    """A VLP-16 stream with starved scans mid-stream: the next scans' LM finds
    fewer than 10 corner or 100 surf points in the last clouds and skips the
    update (featureAssociation.cpp:1668 gate), the first scans after the
    blockage run their LM against the starved clouds (few rows: the < 10
    rows guard, :1677 / :1690), and the stream then recovers."""
    sc = L.synth_cfg("VLP-16", 5)
    scans = [L.synth_scan(sc, k) for k in range(14)]
    for k, w in ((4, 6.0), (5, 2.0), (8, 20.0), (11, 1.0)):
        p, s = scans[k]
        scans[k] = (wedge(p, 30.0 * k, w), s)
    return scans


def test_starved_scans_mid_stream(L):
    scans = _sparse_stream(L)
    ref = _oracle(L, scans)
    small = [len(o["less_sharp"]) < 10 or len(o["less_flat"]) < 100 for o in ref]
    assert any(small) and not all(small), [(len(o["less_sharp"]), len(o["less_flat"])) for o in ref]
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for p, _ in scans) + 16
    gpu = L.Lego(cfg, max_points=cap, max_batch=7)  # a batch boundary right after the first blockage
    recs = list(gpu.odom_batch(*_pack(scans[:7]))) + list(gpu.odom_batch(*_pack(scans[7:])))
    gpu.close()
    _check_recs(recs, ref, "starved scans")


def test_starved_scans_in_a_fleet(L):
    """The same stream beside a normal one in a fleet context (a few odometry
    workgroups per stream: the hashed grids over near-empty clouds): every
    record equals the stream's own context byte for byte."""
    starved = _sparse_stream(L)
    sc = L.synth_cfg("VLP-16", 6)
    normal = [L.synth_scan(sc, k) for k in range(len(starved))]
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for p, _ in starved + normal) + 16
    K = len(starved) // 2
    ref = []
    for scans in (starved, normal):
        g = L.Lego(cfg, max_points=cap, max_batch=K)
        raw = bytes(g.odom_batch(*_pack(scans[:K]))) + bytes(g.odom_batch(*_pack(scans[K:])))
        g.close()
        ref.append([raw[64 * k:64 * k + 60] for k in range(2 * K)])
    fl = L.Lego(cfg, max_points=cap, max_batch=K, streams=2)
    got = [[], []]
    for h in (slice(0, K), slice(K, 2 * K)):
        raw = bytes(fl.odom_batch(*_pack(starved[h] + normal[h])))
        for s in range(2):
            got[s] += [raw[64 * (s * K + k):64 * (s * K + k) + 60] for k in range(K)]
    fl.close()
    assert got == ref
    recs = [L.PoseRec.from_buffer_copy(r + bytes(4)) for r in got[0]]
    _check_recs(recs, _oracle(L, starved), "starved scans in a fleet")
