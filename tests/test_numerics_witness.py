"""Breaks the common mode of the solver restatement:
`lego_numerics.h` / `lego_icp.h` are compiled into both the oracle and the
gfx950 kernels, so they are checked here against a second, independently
written restatement of the same published algorithms
(tests/witness_numerics.py, numpy float32) — bit for bit on

* adversarial systems: ill-conditioned, rank-deficient, repeated eigenvalues,
  zero / diagonal / permutation matrices, extreme scales, the QR failure
  branch (|R_ii| < 10 FLT_EPSILON) and the LU pivoting;
* the real systems of the path, logged by the oracle
  (`lego_oracle_log_systems`): the odometry's 3x3 normal equations of the C2
  stream (featureAssociation.cpp:1327,1334,1349 / 1428,1435,1450) and the
  mapping's 6x6 normal equations, 5x3 plane fits and 3x3 corner covariances
  of a C5-shaped step (mapOptmization.cpp:1126,1189,1276,1283,1298);

plus PCL's VoxelGrid against the oracle's, and the Eigen JacobiSVD / umeyama
restatement against numpy's float64 SVD within tolerance (Eigen's float
internals are not reproducible in numpy).  OpenCV / PCL / Eigen themselves are
absent: parity against their binaries stays unpinned."""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tests"))
import witness_numerics as W  # noqa: E402

F32P = C.POINTER(C.c_float)
pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")  # overflow / NaN cases are intended


@pytest.fixture(scope="module")
def capi(tmp_path_factory):
    so = tmp_path_factory.mktemp("capi") / "libnumerics_capi.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    "-I", str(REPO / "include"), "-I", str(REPO / "lego-loam_amd/csrc"),
                    str(REPO / "tests/native/numerics_capi.cpp"), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    for fn in ("lw_solve_qr",):
        getattr(lib, fn).argtypes = [C.c_int, C.c_int, F32P, F32P, F32P]
    lib.lw_eigen.argtypes = [C.c_int, C.c_int, F32P, F32P, F32P]
    lib.lw_inv.argtypes = [C.c_int, F32P, F32P]
    lib.lw_svd3.argtypes = [F32P, F32P, F32P, F32P]
    lib.lw_umeyama.argtypes = [F32P, F32P, F32P, F32P]
    return lib


def _p(a):
    return a.ctypes.data_as(F32P)


def shared_qr(lib, A, b):
    A = np.ascontiguousarray(A, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    x = np.zeros(A.shape[1], np.float32)
    ok = lib.lw_solve_qr(A.shape[0], A.shape[1], _p(A), _p(b), _p(x))
    assert ok >= 0
    return bool(ok), x


def shared_eigen(lib, A, form=0):
    A = np.ascontiguousarray(A, np.float32)
    n = A.shape[0]
    w, v = np.zeros(n, np.float32), np.zeros((n, n), np.float32)
    assert lib.lw_eigen(n, form, _p(A), _p(w), _p(v)) == 0
    return w, v


def shared_inv(lib, A):
    A = np.ascontiguousarray(A, np.float32)
    d = np.zeros_like(A)
    ok = lib.lw_inv(A.shape[0], _p(A), _p(d))
    assert ok >= 0
    return bool(ok), d


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def check_system(lib, A, b=None, eig=True, inv=True, qr=True):
    """Every applicable shared routine vs the witness on one system."""
    n = A.shape[1]
    if qr:
        ok1, x1 = shared_qr(lib, A, b)
        ok2, x2 = W.solve_qr(A, b)
        assert ok1 == ok2 and same_bits(x1, x2), ("qr", A, b, x1, x2)
    if eig and A.shape[0] == n:
        w1, v1 = shared_eigen(lib, A)
        w2, v2 = W.eigen_sym(A)
        assert same_bits(w1, w2) and same_bits(v1, v2), ("eigen", A, w1, w2)
        if n == 3:  # the device's register form
            w3, v3 = shared_eigen(lib, A, form=1)
            assert same_bits(w3, w2) and same_bits(v3, v2), ("eigen3", A)
        if inv:  # the reference inverts the eigenvector matrix (matV.inv())
            ok1, d1 = shared_inv(lib, v1)
            ok2, d2 = W.inv3(v1) if n == 3 else W.inv_lu(v1)
            assert ok1 == ok2 and same_bits(d1, d2), ("inv", v1)
    if inv and A.shape[0] == n:
        ok1, d1 = shared_inv(lib, A)
        ok2, d2 = W.inv3(A) if n == 3 else W.inv_lu(A)
        assert ok1 == ok2 and same_bits(d1, d2), ("inv", A)


def adversarial(n, rng):
    """Systems meant to take every branch of the three solvers."""
    out = []
    for cond in (1.0, 1e2, 1e4, 1e7):
        Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
        ev = np.geomspace(1.0, 1.0 / cond, n) * rng.uniform(0.1, 1e3)
        out.append((Q * ev) @ Q.T)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    out.append((Q * np.r_[np.ones(n - 1), 0.0]) @ Q.T)           # rank deficient
    out.append((Q * np.r_[[5.0] * 2, np.ones(n - 2)]) @ Q.T)       # repeated eigenvalues
    out.append(np.eye(n) * 3.0)                                    # already diagonal
    out.append(np.diag(rng.uniform(-5, 5, n)))                     # indefinite diagonal
    out.append(np.zeros((n, n)))                                   # zero: QR fails, Jacobi no-op
    out.append(np.eye(n)[rng.permutation(n)] * 2.0)                # a symmetric permutation? (pivoting)
    P = np.eye(n)[rng.permutation(n)]
    out.append(P + P.T)
    B = rng.standard_normal((n, n))
    out.append(B + B.T)                                            # indefinite
    out.append((B @ B.T) * 1e-18)                                  # tiny scale
    out.append((B @ B.T) * 1e18)                                   # huge scale
    out.append(np.full((n, n), 2.0) + np.eye(n) * 1e-6)            # nearly rank one
    return [np.asarray(a, np.float32) for a in out]


@pytest.mark.parametrize("n", [3, 6])
def test_adversarial_square_systems(capi, n):
    rng = np.random.default_rng(100 + n)
    for A in adversarial(n, rng) * 1:
        b = rng.standard_normal(n).astype(np.float32)
        check_system(capi, A, b)
    for _ in range(150):  # and plain random symmetric systems
        B = rng.standard_normal((n, n)).astype(np.float32)
        check_system(capi, (B @ B.T).astype(np.float32), rng.standard_normal(n).astype(np.float32))


def test_adversarial_plane_fits(capi):
    """mapOptimization's 5x3 least-squares plane fit (A0 x = -1)."""
    rng = np.random.default_rng(7)
    b = -np.ones(5, np.float32)
    cases = [rng.standard_normal((5, 3)) * 10 for _ in range(200)]
    cases.append(np.outer(np.arange(1, 6), [1.0, 2.0, 3.0]))            # collinear points: rank 1
    cases.append(np.zeros((5, 3)))
    cases.append(np.c_[rng.standard_normal((5, 2)), np.zeros(5)])        # a zero column
    plane = rng.standard_normal((5, 2)) @ rng.standard_normal((2, 3))    # through the origin: rank 2
    cases.append(plane)
    for A in cases:
        check_system(capi, np.asarray(A, np.float32), b, eig=False, inv=False)


@pytest.fixture(scope="module")
def real_systems(L):
    """The oracle's own systems: C2's odometry (40 scans of the headline
    stream) and two C5 mapping steps (VLS-128 seed 3 vs the 1.0 M / 200 k map)."""
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    ora.log_systems(True)
    sc = L.synth_cfg("VLP-16", 1)
    for k in range(40):
        ora.ip(*L.synth_scan(sc, k))
        ora.fa()
    odo = ora.systems(0)
    ora = L.Oracle(L.sensor_cfg("VLS-128"))
    surf, corner = L.synth_map(3, 50.0, 1_000_000, 200_000)
    ora.mo_set_map(corner, surf)
    ora.log_systems(True)
    sc = L.synth_cfg("VLS-128", 3)
    steps, k = 0, 0
    while steps < 2:
        ora.ip(*L.synth_scan(sc, k))
        ora.fa()
        steps += int(ora.mo()["processed"])
        k += 1
    return odo, ora.systems(1), ora.systems(2), ora.systems(3)


def test_real_odometry_systems(capi, real_systems):
    odo = real_systems[0]
    assert len(odo) > 300
    for row in odo:
        check_system(capi, row[:9].reshape(3, 3), row[9:12])
    print(f"{len(odo)} odometry 3x3 systems of the C2 stream: bit-equal")


def test_real_mapping_systems(capi, real_systems):
    _, lm, plane, cov = real_systems
    assert len(lm) >= 2 and len(plane) > 500 and len(cov) > 500
    for row in lm:
        check_system(capi, row[:36].reshape(6, 6), row[36:42])
    b = -np.ones(5, np.float32)
    for row in plane[::4]:
        check_system(capi, row.reshape(5, 3), b, eig=False, inv=False)
    for row in cov[::4]:
        A = row.reshape(3, 3)
        w1, v1 = shared_eigen(capi, A)
        w2, v2 = W.eigen_sym(A)
        w3, v3 = shared_eigen(capi, A, form=1)
        assert same_bits(w1, w2) and same_bits(v1, v2) and same_bits(w3, w2) and same_bits(v3, v2), A
    print(f"C5: {len(lm)} 6x6 LM systems, {len(plane[::4])} plane fits, {len(cov[::4])} corner covariances: "
          "bit-equal")


def test_voxel_grid_witness(L):
    rng = np.random.default_rng(3)
    lib = L.oracle_lib()
    for n, leaf, scale in ((5000, 0.2, 5.0), (20000, 0.4, 30.0), (3000, 1.0, 2.0), (64, 0.2, 0.05)):
        pts = np.zeros(n, L.XYZI_DTYPE)
        for k in ("x", "y", "z"):
            pts[k] = (rng.standard_normal(n) * scale).astype(np.float32)
        pts["intensity"] = rng.uniform(0, 100, n).astype(np.float32)
        pts[n // 3: n // 3 + 20] = pts[:20]  # duplicates
        pts["x"][7] = np.nan                 # dropped by both
        out = np.zeros(n, L.XYZI_DTYPE)
        m = C.c_int32()
        assert lib.lego_oracle_voxel_grid(pts.ctypes.data, n, leaf, 0, out.ctypes.data, C.byref(m)) == 0
        got = np.stack([out[k][:m.value] for k in ("x", "y", "z", "intensity")], axis=1)
        exp = W.voxel_grid(pts, leaf)
        assert got.shape == exp.shape and same_bits(got, exp), (n, leaf)


def test_svd_and_umeyama_within_tolerance(capi):
    rng = np.random.default_rng(11)
    for _ in range(300):
        A = rng.standard_normal((3, 3)).astype(np.float32)
        U, S, V = (np.zeros((3, 3), np.float32), np.zeros(3, np.float32), np.zeros((3, 3), np.float32))
        assert capi.lw_svd3(_p(A), _p(U), _p(S), _p(V)) == 1
        s_ref = np.linalg.svd(A.astype(np.float64), compute_uv=False)
        assert np.allclose(S, s_ref, rtol=0, atol=2e-6 * s_ref[0] + 1e-30), (S, s_ref)
        assert np.allclose((U * S) @ V.T, A, atol=3e-6 * s_ref[0])
    for _ in range(200):  # a rigid motion between two point sets: umeyama recovers it
        src = rng.standard_normal((50, 3)) * 5
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        t = rng.standard_normal(3) * 3
        dst = src @ R.T + t
        sm, dm = src.mean(0).astype(np.float32), dst.mean(0).astype(np.float32)
        sigma = (((dst - dm).T @ (src - sm)) / len(src)).astype(np.float32)
        T = np.zeros((4, 4), np.float32)
        capi.lw_umeyama(_p(sm), _p(dm), _p(np.ascontiguousarray(sigma)), _p(T))
        assert np.allclose(T[:3, :3], R, atol=2e-5) and np.allclose(T[:3, 3], t, atol=2e-4), (T, R, t)
