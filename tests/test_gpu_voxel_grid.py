"""The device VoxelGrid (lego_voxel_grid; lego_vg.hip + lego_vgsort.h) against
the oracle's pcl::VoxelGrid restatement with PCL's std::sort (the reference's
order of each voxel's points): bit-exact centroids on clouds from a few
points to the C5 map's size, on adversarial key orders that drive std::sort
into its heap-sort fallback, through the forced single-workgroup partition
path, with non-finite points and in the integer-overflow case.

The adversarial keys (tests/golden/vg_killer.npz) come from McIlroy's
adversary run against libstdc++'s std::sort (tests/golden/make_vg_killer.py);
they become clouds with leaf 1: the point of key k lies in voxel k."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent


def oracle_vg(L, pts, leaf):
    lib = L.oracle_lib()
    pts = np.ascontiguousarray(pts, dtype=L.XYZI_DTYPE)
    out = np.zeros(max(len(pts), 1), L.XYZI_DTYPE)
    n = C.c_int32()
    assert lib.lego_oracle_voxel_grid(pts.ctypes.data, len(pts), leaf, 1, out.ctypes.data, C.byref(n)) == 0
    return out[:n.value]


def cloud(rng, n, extent, dtype):
    p = np.zeros(n, dtype)
    for k in ("x", "y", "z"):
        p[k] = rng.uniform(-extent, extent, n).astype(np.float32)
    p["intensity"] = rng.uniform(0, 100, n).astype(np.float32)
    return p


def keyed_cloud(keys, dtype, seed=0):
    """voxel k of leaf 1 for key k (y, z in voxel 0): jittered inside it so the
    summation order shows in the centroid's last bits"""
    rng = np.random.default_rng(seed)
    n = len(keys)
    p = np.zeros(n, dtype)
    p["x"] = (keys.astype(np.float64) + rng.uniform(0.05, 0.95, n)).astype(np.float32)
    p["y"] = rng.uniform(0.05, 0.95, n).astype(np.float32)
    p["z"] = rng.uniform(0.05, 0.95, n).astype(np.float32)
    p["intensity"] = rng.uniform(0, 100, n).astype(np.float32)
    return p


@pytest.fixture(scope="module")
def gpu(L):
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=1)
    yield g
    g.close()


def _same(a, b, what):
    assert len(a) == len(b), f"{what}: {len(a)} vs {len(b)} voxels"
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=what)


@pytest.mark.parametrize("n,extent,leaf", [(1, 1.0, 0.2), (17, 0.3, 0.2), (300, 1.0, 0.2), (5000, 3.0, 0.4),
                                           (8192, 4.0, 0.4), (9000, 4.0, 0.4), (60000, 10.0, 0.4),
                                           (400000, 30.0, 0.4), (1200000, 60.0, 0.4)])
def test_random_clouds_match_pcl_order(L, gpu, n, extent, leaf):
    rng = np.random.default_rng(n)
    p = cloud(rng, n, extent, L.XYZI_DTYPE)
    got, st = gpu.voxel_grid(p, leaf)
    _same(got, oracle_vg(L, p, leaf), f"n={n}")
    assert st["sorted"] == n and st["voxels"] == len(got)
    print(f"n={n}: {st}")


def test_scan_shaped_clouds_match_pcl_order(L, gpu):
    """a less-flat-like cloud: a VLP-16 scan's segmented points, in scan order"""
    sc = L.synth_cfg("VLP-16", 5)
    pts, _ = L.synth_scan(sc, 3)
    p = np.zeros(len(pts), L.XYZI_DTYPE)
    for k in ("x", "y", "z", "intensity"):
        p[k] = pts[k]
    for leaf in (0.2, 0.4, 1.0):
        got, st = gpu.voxel_grid(p, leaf)
        _same(got, oracle_vg(L, p, leaf), f"leaf {leaf}")


# Which sort path the heap-sorted pieces take (lego_vgsort.h, sumOrder): the
# div3 cases hold keys three times inside their pieces (exact heap sort by one
# lane); n20000_div1's one piece of 19,944 keys exceeds a workgroup's LDS
# (exact heap sort in global memory); n3000_div2 (one piece of 2,956 keys,
# each twice), n512_div1 and n200_div1 (distinct keys) are ranked in parallel,
# which gives the same centroids (two addends commute).
@pytest.mark.parametrize("case", ["n8000_div3", "n30000_div3", "n20000_div1", "n3000_div2", "n512_div1",
                                  "n200_div1"])
def test_adversarial_keys_heap_fallback(L, gpu, case):
    z = np.load(REPO / "tests/golden/vg_killer.npz")
    keys = z[case]
    p = keyed_cloud(keys, L.XYZI_DTYPE)
    got, st = gpu.voxel_grid(p, 1.0)
    _same(got, oracle_vg(L, p, 1.0), case)
    print(f"{case}: {st}")
    # voxel k of leaf 1 for key k: the voxel indices are the keys minus the
    # smallest, so std::sort takes the same heap-sorted pieces
    assert st["heap_segments"] == int(z["heaps_" + case][0]) > 0


def test_nonfinite_points_skipped(L, gpu):
    rng = np.random.default_rng(7)
    p = cloud(rng, 20000, 5.0, L.XYZI_DTYPE)
    bad = rng.choice(len(p), 50, replace=False)
    p["x"][bad[:20]] = np.nan
    p["y"][bad[20:35]] = np.inf
    p["z"][bad[35:]] = -np.inf
    got, st = gpu.voxel_grid(p, 0.4)
    _same(got, oracle_vg(L, p, 0.4), "non-finite")
    assert st["nonfinite"] == 50 and st["sorted"] == len(p) - 50


def test_leaf_overflow_copies_input(L, gpu):
    rng = np.random.default_rng(8)
    p = cloud(rng, 3000, 1000.0, L.XYZI_DTYPE)
    got, _ = gpu.voxel_grid(p, 0.001)  # (2e6)^3 voxels > INT_MAX: PCL returns the cloud
    _same(got, oracle_vg(L, p, 0.001), "overflow")
    _same(got, p, "overflow is a copy")


def test_forced_single_workgroup_partition(L):
    """lego_ctx_opts::vg_rounds = 0 (diagnostic): no multi-workgroup rounds,
    so clouds above the workgroup size are partitioned by one workgroup in
    global memory (the path for segments the rounds leave too large), heap
    sort included."""
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=1, opts={"vg_rounds": 0})
    keys = np.load(REPO / "tests/golden/vg_killer.npz")["n20000_div1"]
    for name, p, leaf in (("random", cloud(np.random.default_rng(3), 150000, 20.0, L.XYZI_DTYPE), 0.4),
                          ("killer", keyed_cloud(keys, L.XYZI_DTYPE), 1.0)):
        got, st = g.voxel_grid(p, leaf)
        _same(got, oracle_vg(L, p, leaf), name)
        assert st["rounds"] == 0 and st["slow_segments"] > 0, (name, st)
    g.close()
