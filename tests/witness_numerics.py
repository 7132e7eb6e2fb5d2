"""Independent witness of the third-party solver arithmetic on the path.

TEST INFRASTRUCTURE.  `lego-loam_amd/csrc/lego_numerics.h` restates OpenCV's
float solvers once and that one restatement is compiled into both the product
kernels and the oracle, so an error in it could never show up as a parity
failure.  This module codes the same published
algorithms a second time, separately, in numpy float32 scalar arithmetic
(IEEE single, no contraction), so tests/test_numerics_witness.py can compare
the two bit for bit.  OpenCV itself is absent: parity against OpenCV's binary
stays unpinned; this pins the restatement against a second reading of the
algorithm.

Algorithms (OpenCV 3.x `modules/core/src/lapack.cpp`, `hal`):
  * cv::solve(A, b, DECOMP_QR) -> hal::QR32f -> QRImpl: Householder
    reflections column by column (v = x + sign(x0)|x| e0, normalised), the
    reflectors stored below the diagonal scaled by 1/v0 with h = v0^2, then
    the rhs transformed and back substitution; a pivot |R_ii| < 10*FLT_EPSILON
    fails and cv::solve returns zeros.  Reference call sites:
    featureAssociation.cpp:1327,1428 (3x3), mapOptmization.cpp:1189 (5x3
    least squares), :1276 (6x6).
  * cv::eigen(symmetric) -> hal::Jacobi -> JacobiImpl_: cyclic-by-largest
    Jacobi with per-row (indR) / per-column (indC) running maxima of the
    off-diagonal, cv::hypot, stop at |p| <= FLT_EPSILON or n*n*30 rotations,
    then a selection sort (descending, strict <), eigenvectors as rows.  Call
    sites featureAssociation.cpp:1334,1435, mapOptmization.cpp:1126,1283.
  * Mat::inv() -> cv::invert(DECOMP_LU): 3x3 closed form (float det3, double
    cofactors), larger sizes LUImpl with partial pivoting (eps 10*FLT_EPSILON).
    Call sites featureAssociation.cpp:1349,1450 (3x3), mapOptmization.cpp:1298
    (6x6).
  * pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8): bounding box, voxel
    index floor(p * 1/leaf) - min_b, (idx, point) pairs sorted by idx, the
    centroid of each run as float sums divided by the count.  In-voxel order:
    input order (the product's documented choice, DESIGN.md §2 deviation 2).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
FLT_EPS = f32(1.1920928955078125e-07)


def _abs(x):
    return f32(abs(x))


def hypot_cv(a, b):
    a, b = _abs(a), _abs(b)
    if a > b:
        r = b / a
        return a * f32(np.sqrt(f32(1) + r * r))
    if b > 0:
        r = a / b
        return b * f32(np.sqrt(f32(1) + r * r))
    return f32(0)


def solve_qr(A, b):
    """QRImpl on a copy of the m x n float32 matrix A and rhs b (one column).
    Returns (ok, x)."""
    R = [[f32(v) for v in row] for row in np.asarray(A, np.float32)]
    rhs = [f32(v) for v in np.asarray(b, np.float32)]
    m, n = len(R), len(R[0])
    h = [f32(0)] * n
    for col in range(n):
        v = [R[col + i][col] for i in range(m - col)]
        nrm2 = f32(0)
        for e in v:
            nrm2 = nrm2 + e * e
        first = v[0]
        sgn = f32(1) if first >= 0 else f32(-1)
        v[0] = first + sgn * f32(np.sqrt(nrm2))
        nrm = f32(np.sqrt(nrm2 + v[0] * v[0] - first * first))
        v = [e / nrm for e in v]
        for j in range(col, n):
            dot = f32(0)
            for i in range(col, m):
                dot = dot + v[i - col] * R[i][j]
            for i in range(col, m):
                R[i][j] = R[i][j] - f32(2) * v[i - col] * dot
        h[col] = v[0] * v[0]
        for i in range(1, m - col):
            R[col + i][col] = v[i] / v[0]
    for col in range(n):
        v = [f32(1)] + [R[col + i][col] for i in range(1, m - col)]
        dot = f32(0)
        for i in range(col, m):
            dot = dot + v[i - col] * rhs[i]
        for i in range(col, m):
            rhs[i] = rhs[i] - f32(2) * v[i - col] * dot * h[col]
    for i in range(n - 1, -1, -1):
        for j in range(n - 1, i, -1):
            rhs[i] = rhs[i] - rhs[j] * R[i][j]
        if _abs(R[i][i]) < FLT_EPS * f32(10):
            return False, np.zeros(n, np.float32)
        rhs[i] = rhs[i] / R[i][i]
    return True, np.array(rhs[:n], np.float32)


def _row_max(A, r, n):
    """(index, |value|) of the largest |A[r][c]|, c > r (first on ties)."""
    best, bv = r + 1, _abs(A[r][r + 1])
    for c in range(r + 2, n):
        if bv < _abs(A[r][c]):
            best, bv = c, _abs(A[r][c])
    return best


def _col_max(A, c):
    """index of the largest |A[r][c]|, r < c (first on ties)."""
    best, bv = 0, _abs(A[0][c])
    for r in range(1, c):
        if bv < _abs(A[r][c]):
            best, bv = r, _abs(A[r][c])
    return best


def eigen_sym(A):
    """JacobiImpl_ on a copy of the symmetric float32 matrix: (W desc, V rows)."""
    a = [[f32(v) for v in row] for row in np.asarray(A, np.float32)]
    n = len(a)
    V = [[f32(1) if i == j else f32(0) for j in range(n)] for i in range(n)]
    W = [a[i][i] for i in range(n)]
    rmax = [_row_max(a, r, n) if r < n - 1 else 0 for r in range(n)]
    cmax = [_col_max(a, c) if c > 0 else 0 for c in range(n)]
    for _ in range(n * n * 30 if n > 1 else 0):
        k, mv = 0, _abs(a[0][rmax[0]])
        for r in range(1, n - 1):
            if mv < _abs(a[r][rmax[r]]):
                k, mv = r, _abs(a[r][rmax[r]])
        l = rmax[k]
        for c in range(1, n):
            if mv < _abs(a[cmax[c]][c]):
                k, l, mv = cmax[c], c, _abs(a[cmax[c]][c])
        p = a[k][l]
        if _abs(p) <= FLT_EPS:
            break
        y = f32(float(W[l] - W[k]) * 0.5)  # float difference, double product, float store
        t = _abs(y) + hypot_cv(p, y)
        s = hypot_cv(p, t)
        c = t / s
        s = p / s
        t = (p / t) * p
        if y < 0:
            s, t = -s, -t
        a[k][l] = f32(0)
        W[k] = W[k] - t
        W[l] = W[l] + t

        def rot(x0, x1):
            return x0 * c - x1 * s, x0 * s + x1 * c

        for i in range(k):
            a[i][k], a[i][l] = rot(a[i][k], a[i][l])
        for i in range(k + 1, l):
            a[k][i], a[i][l] = rot(a[k][i], a[i][l])
        for i in range(l + 1, n):
            a[k][i], a[l][i] = rot(a[k][i], a[l][i])
        for i in range(n):
            V[k][i], V[l][i] = rot(V[k][i], V[l][i])
        for idx in (k, l):
            if idx < n - 1:
                rmax[idx] = _row_max(a, idx, n)
            if idx > 0:
                cmax[idx] = _col_max(a, idx)
    for k in range(n - 1):
        m = k
        for i in range(k + 1, n):
            if W[m] < W[i]:
                m = i
        if m != k:
            W[m], W[k] = W[k], W[m]
            V[m], V[k] = V[k], V[m]
    return np.array(W, np.float32), np.array(V, np.float32)


def inv3(S):
    """cv::invert(DECOMP_LU) 3x3 closed form: (ok, inverse)."""
    m = np.asarray(S, np.float32)
    g = lambda i, j: f32(m[i, j])  # noqa: E731
    det = (g(0, 0) * (g(1, 1) * g(2, 2) - g(1, 2) * g(2, 1))
           - g(0, 1) * (g(1, 0) * g(2, 2) - g(1, 2) * g(2, 0))
           + g(0, 2) * (g(1, 0) * g(2, 1) - g(1, 1) * g(2, 0)))
    d = float(det)
    if d == 0.0:
        return False, np.zeros((3, 3), np.float32)
    d = 1.0 / d
    G = lambda i, j: float(m[i, j])  # noqa: E731
    cof = [[G(1, 1) * G(2, 2) - G(1, 2) * G(2, 1), G(0, 2) * G(2, 1) - G(0, 1) * G(2, 2),
            G(0, 1) * G(1, 2) - G(0, 2) * G(1, 1)],
           [G(1, 2) * G(2, 0) - G(1, 0) * G(2, 2), G(0, 0) * G(2, 2) - G(0, 2) * G(2, 0),
            G(0, 2) * G(1, 0) - G(0, 0) * G(1, 2)],
           [G(1, 0) * G(2, 1) - G(1, 1) * G(2, 0), G(0, 1) * G(2, 0) - G(0, 0) * G(2, 1),
            G(0, 0) * G(1, 1) - G(0, 1) * G(1, 0)]]
    return True, np.array([[f32(x * d) for x in row] for row in cof], np.float32)


def inv_lu(S):
    """cv::invert(DECOMP_LU) for n > 3: LUImpl with the identity as rhs."""
    A = [[f32(v) for v in row] for row in np.asarray(S, np.float32)]
    n = len(A)
    B = [[f32(1) if i == j else f32(0) for j in range(n)] for i in range(n)]
    for i in range(n):
        piv = i
        for j in range(i + 1, n):
            if _abs(A[j][i]) > _abs(A[piv][i]):
                piv = j
        if _abs(A[piv][i]) < FLT_EPS * f32(10):
            return False, np.zeros((n, n), np.float32)
        if piv != i:
            A[i][i:], A[piv][i:] = A[piv][i:], A[i][i:]
            B[i], B[piv] = B[piv], B[i]
        d = f32(-1) / A[i][i]
        for j in range(i + 1, n):
            alpha = A[j][i] * d
            for q in range(i + 1, n):
                A[j][q] = A[j][q] + alpha * A[i][q]
            for q in range(n):
                B[j][q] = B[j][q] + alpha * B[i][q]
        A[i][i] = -d
    for i in range(n - 1, -1, -1):
        for j in range(n):
            acc = B[i][j]
            for q in range(i + 1, n):
                acc = acc - A[i][q] * B[q][j]
            B[i][j] = acc * A[i][i]
    return True, np.array(B, np.float32)


def voxel_grid(pts, leaf):
    """pcl::VoxelGrid over a structured PointXYZI array (fields x, y, z,
    intensity), in-voxel input order.  Returns float32 (k, 4)."""
    P = np.stack([pts["x"], pts["y"], pts["z"], pts["intensity"]], axis=1).astype(np.float32)
    fin = np.isfinite(P[:, :3]).all(axis=1)
    Q = P[fin]
    if len(Q) == 0:
        return np.zeros((0, 4), np.float32)
    inv = f32(1) / f32(leaf)
    lo, hi = Q[:, :3].min(axis=0), Q[:, :3].max(axis=0)
    span = [int(f32(hi[k] - lo[k]) * inv) + 1 for k in range(3)]
    if span[0] * span[1] * span[2] > 2**31 - 1:
        return P.copy()
    minb = [int(np.floor(f32(lo[k]) * inv)) for k in range(3)]
    maxb = [int(np.floor(f32(hi[k]) * inv)) for k in range(3)]
    d0, d1 = maxb[0] - minb[0] + 1, maxb[1] - minb[1] + 1
    ijk = [(np.floor(Q[:, k] * inv) - np.float32(minb[k])).astype(np.int64) for k in range(3)]
    key = ijk[0] + ijk[1] * d0 + ijk[2] * d0 * d1
    order = np.argsort(key, kind="stable")
    out = []
    i = 0
    while i < len(order):
        j = i
        acc = [f32(0)] * 4
        while j < len(order) and key[order[j]] == key[order[i]]:
            row = Q[order[j]]
            acc = [acc[c] + row[c] for c in range(4)]
            j += 1
        cnt = f32(j - i)
        out.append([a / cnt for a in acc])
        i = j
    return np.array(out, np.float32).reshape(-1, 4)
