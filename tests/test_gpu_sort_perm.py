"""lego_sort_permutation — the device's libstdc++ std::sort permutation of
(key, index) pairs compared by key (PCL VoxelGrid's sort; lego_vgsort.h's
workgroup sort and lego_vgsort_wave.h's one-wave sort of the per-ring
less-flat VoxelGrid) — against the oracle's real std::sort
(lego_oracle_sort_permutation): the same permutation on random keys with ties,
sorted / reversed / constant / organ-pipe arrays, every size around the
16-key insertion-sort threshold and the one-wave sort's 64-key and 512-key
bounds, and McIlroy-adversary keys (tests/golden/vg_killer.npz, made by
tests/golden/make_vg_killer.py against libstdc++) that drive std::sort into
its heap-sort fallback — the device must take that fallback too.  Every form
of the workgroup sort runs at both block sizes (modes 0 and 2..8)."""
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parent.parent


def ref_perm(L, keys):
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.zeros(max(len(keys), 1), np.int32)
    assert L.oracle_lib().lego_oracle_sort_permutation(keys.ctypes.data, len(keys), perm.ctypes.data) == 0
    return perm[:len(keys)]


@pytest.fixture(scope="module")
def gpu(L):
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=1000, max_batch=1)
    yield g
    g.close()


def shapes(n, rng):
    yield "random_ties", rng.integers(0, max(1, n // 3), n)
    yield "random", rng.integers(0, 1 << 30, n)
    yield "sorted", np.arange(n)
    yield "reversed", np.arange(n)[::-1].copy()
    yield "constant", np.full(n, 7)
    yield "organ_pipe", np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]])
    yield "two_runs", np.concatenate([np.sort(rng.integers(0, 1000, n // 2)), np.sort(rng.integers(0, 1000, n - n // 2))])


SIZES = [0, 1, 2, 15, 16, 17, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256, 300, 511, 512]


@pytest.mark.parametrize("wave", [True, False])
@pytest.mark.parametrize("n", SIZES)
def test_permutation_matches_std_sort(L, gpu, n, wave):
    rng = np.random.default_rng(1000 + n)
    for name, keys in shapes(n, rng):
        got, _ = gpu.sort_permutation(keys, wave=wave)
        np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{name} n={n} wave={wave}")


@pytest.mark.parametrize("n", [600, 1000, 1800, 4096, 8192])
def test_block_sort_larger_arrays(L, gpu, n):
    rng = np.random.default_rng(n)
    for name, keys in shapes(n, rng):
        got, _ = gpu.sort_permutation(keys, wave=False)
        np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{name} n={n}")


@pytest.mark.parametrize("case", ["n64_div1", "n200_div1", "n500_div3", "n512_div1", "n3000_div2"])
def test_adversarial_keys_take_the_heap_fallback(L, gpu, case):
    """the same permutation, and exactly as many heap-sorted pieces as
    std::sort takes (heaps_<case>: counted by tests/native/vgsort_check.cpp's
    restatement, itself checked equal to std::sort on those keys)"""
    z = np.load(REPO / "tests/golden/vg_killer.npz")
    keys, heaps = z[case], int(z["heaps_" + case][0])
    for wave in ([True, False] if len(keys) <= 512 else [False]):
        got, heap = gpu.sort_permutation(keys, wave=wave)
        np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{case} wave={wave}")
        assert heap == heaps, f"{case} wave={wave}: {heap} heap-sorted pieces, std::sort takes {heaps}"
    assert any(int(z["heaps_" + c][0]) > 0 for c in ("n64_div1", "n200_div1", "n512_div1"))


def test_size_limits(L, gpu):
    with pytest.raises(Exception):
        gpu.sort_permutation(np.zeros(513, np.uint32), wave=True)
    with pytest.raises(Exception):
        gpu.sort_permutation(np.zeros(8193, np.uint32), wave=False)
    for mode in (2, 4, 5, 6):
        with pytest.raises(Exception):
            gpu.sort_permutation(np.zeros(2049, np.uint32), wave=mode)
    for mode in (7, 8):
        with pytest.raises(Exception):
            gpu.sort_permutation(np.zeros(8193, np.uint32), wave=mode)
    with pytest.raises(Exception):
        gpu.sort_permutation(np.zeros(10, np.uint32), wave=9)


# Both forms of the workgroup sort (segment ids in registers: vg_block_sort;
# in LDS: vg_block_sort_sid) at both block sizes, each compiled under the
# register budget of the kernel that runs it: 256 threads as k_lf_voxel (its
# LFV_MINB workgroups per CU, the build that spills), 1024 threads as the
# mapping VoxelGrids' k_vg_local.  Round 4's only GPU fault came from a build
# of k_lf_voxel running the register form at 256 threads, a configuration no
# permutation test had covered.
EXACT_MODES = {0: ("reg", 1024), 4: ("reg", 256), 6: ("lds", 256), 7: ("lds", 1024)}
SUM_MODES = {2: ("lds", 256), 3: ("reg", 1024), 5: ("reg", 256), 8: ("lds", 1024)}


def ring_cases():
    """the per-ring less-flat sort keys k_lf_voxel's workgroups sort: C2 scan
    465 (VLP-16) and the dense sensors' > 512-point rings of VLS-128 seed 3
    scan 0 (the scan of round 4's fault record) and HDL-64E seed 2 scan 0
    (tests/golden/make_ring_keys.py)"""
    for f in ("c2_ring_keys.npz", "dense_ring_keys.npz"):
        z = np.load(REPO / "tests/golden" / f)
        for k in z.files:
            yield f"{f[:-4]}:{k}", z[k]


@pytest.mark.parametrize("mode", sorted(EXACT_MODES))
def test_both_forms_both_sizes_exact(L, gpu, mode):
    """std::sort's exact permutation from every form / block size: the ring
    keys, seven shapes around the rows-per-wave bounds (a 256-thread block's
    waves hold 8 rows of 64 at n = 2048, a 1024-thread block's 2 rows at
    n = 2048 and 8 at 8192), and the McIlroy keys with std::sort's exact
    heap-piece counts."""
    form, T = EXACT_MODES[mode]
    cap = 2048 if T == 256 else 8192
    n_checked = 0
    for name, keys in ring_cases():
        got, _ = gpu.sort_permutation(keys, wave=mode)
        np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{name} mode {mode} ({form}/{T})")
        n_checked += 1
    rng = np.random.default_rng(77 + mode)
    for n in (17, 64, 65, 511, 513, 1023, 1025, 1500, 1800, 2047, 2048, 4096, 8192):
        if n > cap:
            continue
        for name, keys in shapes(n, rng):
            got, _ = gpu.sort_permutation(keys, wave=mode)
            np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{name} n={n} mode {mode} ({form}/{T})")
            n_checked += 1
    z = np.load(REPO / "tests/golden/vg_killer.npz")
    for case in ("n64_div1", "n200_div1", "n500_div3", "n512_div1", "n3000_div2", "n8000_div3"):
        keys, heaps = z[case], int(z["heaps_" + case][0])
        if len(keys) > cap:
            continue
        got, heap = gpu.sort_permutation(keys, wave=mode)
        np.testing.assert_array_equal(got, ref_perm(L, keys), err_msg=f"{case} mode {mode}")
        assert heap == heaps, f"{case} mode {mode}: {heap} heap-sorted pieces, std::sort takes {heaps}"
        n_checked += 1
    print(f"mode {mode} ({form}/{T}): {n_checked} arrays equal to std::sort")


def voxel_sums(keys, perm, vals):
    """each key's values summed from 0 in the order perm leaves them (float32,
    one addend at a time: k_vg_emit / lfv_centroid)"""
    out, cur, acc = [], None, np.float32(0)
    for i in perm:
        if keys[i] != cur:
            if cur is not None:
                out.append(acc)
            cur, acc = keys[i], np.float32(0)
        acc = np.float32(acc + vals[i])
    if cur is not None:
        out.append(acc)
    return np.array(out, np.float32)


def sum_order_cases():
    yield from ring_cases()
    zk = np.load(REPO / "tests/golden/vg_killer.npz")
    for k in ("n200_div1", "n512_div1", "n3000_div2", "n8000_div3", "n500_div3"):
        yield k, zk[k]
    rng = np.random.default_rng(5)
    for n in (17, 20, 33, 48, 64, 65, 100, 200, 300, 511, 700, 1800, 5000):
        for name, keys in shapes(n, rng):
            yield f"{name}_{n}", keys


@pytest.mark.parametrize("mode", sorted(SUM_MODES))
def test_sum_order_sort_gives_std_sort_sums(L, gpu, mode):
    """The VoxelGrids' rule of the block sort (lego_vgsort.h sumOrder) in both
    forms at both block sizes (SUM_MODES; mode 2 = k_lf_voxel's LDS-id form,
    3 = the mapping clouds' register form): a permutation, sorted by key,
    every position outside the stably ranked heap pieces as std::sort leaves
    it, and every key's float32 sum from 0 in its order bit-equal to the sum
    in std::sort's order (random values).  The C2 rings are scan 465's
    (tests/golden/make_ring_keys.py); ring6 holds heap pieces of both kinds."""
    cap = 2048 if SUM_MODES[mode][1] == 256 else 8192
    rng = np.random.default_rng(11)
    ranked = 0
    for name, keys in sum_order_cases():
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        if len(keys) > cap:
            continue
        got, heaps = gpu.sort_permutation(keys, wave=mode)
        ref = ref_perm(L, keys)
        assert np.array_equal(np.sort(got), np.arange(len(keys))), name
        assert np.all(np.diff(keys[got].astype(np.int64)) >= 0), name
        vals = rng.uniform(-10, 10, len(keys)).astype(np.float32)
        np.testing.assert_array_equal(voxel_sums(keys, got, vals).view(np.uint32),
                                      voxel_sums(keys, ref, vals).view(np.uint32), err_msg=name)
        _, heaps_exact = gpu.sort_permutation(keys, wave=False) if len(keys) <= 8192 else (None, heaps)
        assert heaps == heaps_exact, name
        ranked += int(not np.array_equal(got, ref))
    print(f"mode {mode}: {ranked} arrays with stably ranked heap pieces")
    assert ranked > 0
