"""The keyframe pose graph (lego-loam_amd/csrc/lego_pgo_host.h), iSAM2's role
in mapOptimization (mapOptmization.cpp:1372-1420, 930-944, 1456-1478).  GTSAM
is absent, so parity against it is unpinned; this pins the restatement:

* against an independent solver: scipy's trust-region least squares on the
  whitened residuals of the same factors (GTSAM 4's default charts: rotation
  Logmap + translation of measured^-1 h(x)), parameterised independently;
* on a closed square drive with a heading drift and one loop factor: the loop
  residual shrinks and the prior pose stays; with a loop as certain as the
  odometry the loop closes and the correction spreads along the chain;
* the chain-only graph (the reference without loop closure): the estimate is
  the initial values exactly, so the product's keyframe chain needs no solve;
* the camera-frame transform <-> gtsam::Pose3 round trip
  (Rot3::RzRyRx / Rot3::xyz()) returns the same floats, the premise of that
  chain identity."""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest
from scipy.optimize import least_squares
from scipy.spatial.transform import Rotation

REPO = Path(__file__).resolve().parent.parent
D = C.POINTER(C.c_double)
I = C.POINTER(C.c_int)
F = C.POINTER(C.c_float)
VAR_ODOM = np.array([1e-6, 1e-6, 1e-6, 1e-8, 1e-8, 1e-6])  # mapOptmization.cpp:347-350


@pytest.fixture(scope="module")
def pgo(tmp_path_factory):
    so = tmp_path_factory.mktemp("pgo") / "libpgo_capi.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", str(REPO / "lego-loam_amd/csrc"),
                    str(REPO / "tests/native/pgo_capi.cpp"), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    lib.pgo_solve.argtypes = [C.c_int, D, C.c_int, I, I, D, D, I, D]
    lib.pgo_roundtrip.argtypes = [C.c_int, F, F]
    return lib


def pose(R, t):
    return np.concatenate([np.asarray(R, float).ravel(), np.asarray(t, float)])


def inv_mul(a, b):
    """a^-1 b for 12-vector poses."""
    Ra, Rb = a[:9].reshape(3, 3), b[:9].reshape(3, 3)
    return pose(Ra.T @ Rb, Ra.T @ (b[9:] - a[9:]))


def local(z, h):
    d = inv_mul(z, h)
    return np.concatenate([Rotation.from_matrix(d[:9].reshape(3, 3)).as_rotvec(), d[9:]])


def retract(x, d):
    R = x[:9].reshape(3, 3)
    return pose(R @ Rotation.from_rotvec(d[:3]).as_matrix(), x[9:] + R @ d[3:])


def solve_product(lib, init, factors):
    K, nf = len(init), len(factors)
    fi = np.array([f[0] for f in factors], np.int32)
    fj = np.array([f[1] for f in factors], np.int32)
    fz = np.ascontiguousarray([f[2] for f in factors], np.float64)
    fv = np.ascontiguousarray([f[3] for f in factors], np.float64)
    lp = np.array([int(f[4]) for f in factors], np.int32)
    ini = np.ascontiguousarray(init, np.float64)
    est = np.zeros_like(ini)
    its = lib.pgo_solve(K, ini.ctypes.data_as(D), nf, fi.ctypes.data_as(I), fj.ctypes.data_as(I),
                        fz.ctypes.data_as(D), fv.ctypes.data_as(D), lp.ctypes.data_as(I), est.ctypes.data_as(D))
    return est, its


def solve_witness(init, factors):
    """Independent: scipy least_squares over per-pose perturbations of the
    initial values (a different parameterisation than the product's GN)."""
    K = len(init)

    def resid(p):
        x = [retract(init[k], p[6 * k:6 * k + 6]) for k in range(K)]
        r = []
        for i, j, z, var, _ in factors:
            e = local(z, x[i]) if j < 0 else local(z, inv_mul(x[i], x[j]))
            r.append(e / np.sqrt(var))
        return np.concatenate(r)

    sol = least_squares(resid, np.zeros(6 * K), method="trf", xtol=1e-15, ftol=1e-15, gtol=1e-15,
                        x_scale="jac", max_nfev=2000)
    return np.array([retract(init[k], sol.x[6 * k:6 * k + 6]) for k in range(K)])


def square_drive(n_side=8, step=1.0, drift=0.02, seed=0, loop_var=0.02):
    """A closed square path: true poses, odometry measurements with a heading
    drift per step and noise, the dead-reckoned chain as initial values."""
    rng = np.random.default_rng(seed)
    truth = [pose(np.eye(3), np.zeros(3))]
    for s in range(4):
        for k in range(n_side):
            prev = truth[-1]
            turn = np.pi / 2 if k == n_side - 1 else 0.0
            rel = pose(Rotation.from_rotvec([0, 0, turn]).as_matrix(), [step, 0, 0])
            R = prev[:9].reshape(3, 3)
            truth.append(pose(R @ rel[:9].reshape(3, 3), prev[9:] + R @ rel[9:]))
    truth = truth[:-1]  # the last pose coincides with the first: closed by the loop factor
    meas = []
    for a, b in zip(truth, truth[1:]):
        z = inv_mul(a, b)
        d = np.r_[rng.normal(0, 1e-3, 3) + [0, 0, drift], rng.normal(0, 1e-3, 3)]
        meas.append(retract(z, d))
    init = [truth[0]]
    for z in meas:
        R = init[-1][:9].reshape(3, 3)
        init.append(pose(R @ z[:9].reshape(3, 3), init[-1][9:] + R @ z[9:]))
    loop_z = inv_mul(truth[-1], truth[0])  # the true relative pose, as an accepted ICP would give
    factors = [(0, -1, init[0], VAR_ODOM, False)]
    factors += [(k, k + 1, meas[k], VAR_ODOM, False) for k in range(len(meas))]
    factors += [(len(init) - 1, 0, loop_z, np.full(6, loop_var), True)]  # (latest, closest), variance = fitness
    return np.array(truth), np.array(init), factors


def test_chain_without_loops_is_the_initial_estimate(pgo):
    truth, init, factors = square_drive()
    chain = [f for f in factors if not f[4]]
    est, _ = solve_product(pgo, init, chain)
    # the odometry factors were built from the initial values themselves
    z_exact = [(0, -1, init[0], VAR_ODOM, False)] + [(k, k + 1, inv_mul(init[k], init[k + 1]), VAR_ODOM, False)
                                                      for k in range(len(init) - 1)]
    est, its = solve_product(pgo, init, z_exact)
    assert its <= 2 and np.max(np.abs(est - init)) < 1e-12


@pytest.mark.parametrize("loop_var", [0.02, 1e-9])
def test_square_loop_matches_independent_solver(pgo, loop_var):
    """loop_var 0.02: an ICP fitness as the reference's loops carry; the
    odometry's variances (1e-6 / 1e-8) make that factor weak, so the loop
    residual shrinks but stays.  1e-9: a loop as certain as the odometry
    closes almost fully."""
    truth, init, factors = square_drive(loop_var=loop_var)
    est, its = solve_product(pgo, init, factors)
    ref = solve_witness(init, factors)
    assert its < 30
    dt = np.max(np.abs(est[:, 9:] - ref[:, 9:]))
    dr = max(np.linalg.norm(Rotation.from_matrix(a[:9].reshape(3, 3).T @ b[:9].reshape(3, 3)).as_rotvec())
             for a, b in zip(est, ref))
    assert dt < 1e-6 and dr < 1e-7, (dt, dr)
    # the loop closes: the last pose moves to where the loop factor puts it, the
    # prior pose stays, and the drift is spread along the chain
    gap_before = np.linalg.norm(init[-1, 9:] - truth[-1, 9:])
    gap_after = np.linalg.norm(est[-1, 9:] - truth[-1, 9:])
    loop_res = lambda x: np.linalg.norm(local(factors[-1][2], inv_mul(x[-1], x[0])))  # noqa: E731
    assert loop_res(est) < loop_res(init), (loop_res(est), loop_res(init))
    assert np.max(np.abs(est[0] - init[0])) < 1e-6
    if loop_var < 1e-6:
        assert gap_before > 0.5 and gap_after < 0.2 * gap_before, (gap_before, gap_after)
        mid = len(init) // 2
        assert 0.1 < np.linalg.norm(est[mid, 9:] - init[mid, 9:]) < np.linalg.norm(est[-1, 9:] - init[-1, 9:])


def test_two_loops_and_random_graphs(pgo):
    rng = np.random.default_rng(5)
    for trial in range(4):
        truth, init, factors = square_drive(n_side=5, drift=0.01 + 0.01 * trial, seed=trial)
        K = len(init)
        extra = rng.integers(0, K // 2)  # a second loop between two poses far apart
        factors.append((K - 1 - extra, extra, inv_mul(truth[K - 1 - extra], truth[extra]), np.full(6, 0.05), True))
        est, _ = solve_product(pgo, init, factors)
        ref = solve_witness(init, factors)
        assert np.max(np.abs(est[:, 9:] - ref[:, 9:])) < 1e-6, trial
        assert np.max(np.abs(est[:, :9] - ref[:, :9])) < 1e-6, trial


def test_transform_pose_round_trip(pgo):
    rng = np.random.default_rng(9)
    t = np.empty((20000, 6), np.float32)
    t[:, :3] = rng.uniform(-1.5, 1.5, (20000, 3))   # roll / pitch (|pitch| < pi/2) / yaw, camera frame
    t[:, 3:] = rng.uniform(-200, 200, (20000, 3))
    out = np.zeros_like(t)
    pgo.pgo_roundtrip(len(t), t.ctypes.data_as(F), out.ctypes.data_as(F))
    assert np.array_equal(out.view(np.uint32), t.view(np.uint32))
