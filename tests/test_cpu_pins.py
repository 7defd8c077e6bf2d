"""CPU: independent pins of the oracle restatement.  Parity of the HIP path is
bit-exact against oracle/ (the -m gpu tests); these tests check the oracle itself against textbook
float64 numpy implementations written from the published algorithms, not from the reference text:

* EPnP (Lepetit, Moreno-Noguer, Fua 2009: control points by PCA (axis signs as Eigen's solver), barycentric coordinates, the 2n x 12
  system's 4-dimensional null space, the three beta approximations + Gauss-Newton, Procrustes R, t,
  the smallest reprojection error) on NOISY, Refine-sized correspondence sets (n = 6 .. 400) against
  oracle PnPsolver::compute_pose: pose within 1e-4, CheckInliers sets identical;
* the absolute-orientation step of Sim3Solver::ComputeSim3 (3 points, fixed scale) against an SVD
  (Kabsch/Arun) solution: rotation and translation within 1e-4;
* MLPnP's residual Jacobian: the oracle replaces the reference's machine-generated mlpnpJacs
  (MLPnPsolver.cpp:773-1020) by an analytic derivative of the same residual
  r = n^T (R(w) X + t) / |R(w) X + t|.  Here it is compared with central differences of that
  residual (a derivation independent of both), and a Gauss-Newton run with each Jacobian from the
  same start ends at poses within 1e-4 — the bound on what the substitution can change.
The reference itself cannot be built here (no Eigen/OpenCV headers), so these pins bound the
restatement; they do not replace reference outputs (DESIGN.md "Oracle")."""
import numpy as np
import pytest

import oracle_lib as ol
from rsc import synth

PAIRS = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]


# ---------------------------------------------------------------------------------------------
# EPnP, float64 textbook form
# ---------------------------------------------------------------------------------------------
def _procrustes(pw, pc):
    pw0, pc0 = pw.mean(0), pc.mean(0)
    H = (pc - pc0).T @ (pw - pw0)
    U, _, Vt = np.linalg.svd(H)
    D = np.diag([1.0, 1.0, np.sign(np.linalg.det(U @ Vt))])
    R = U @ D @ Vt
    return R, pc0 - R @ pw0


def _reproj(R, t, pw, uv, K):
    fx, fy, cx, cy = K
    Xc = pw @ R.T + t
    u = cx + fx * Xc[:, 0] / Xc[:, 2]
    v = cy + fy * Xc[:, 1] / Xc[:, 2]
    return np.mean(np.hypot(uv[:, 0] - u, uv[:, 1] - v))


def epnp_numpy(pw, uv, K):
    fx, fy, cx, cy = K
    n = len(pw)
    c0 = pw.mean(0)
    D = pw - c0
    # The principal axes' SIGNS are an implementation detail of Eigen's SelfAdjointEigenSolver (the
    # reference, PnPsolver.cpp:311-319) that changes the noisy EPnP answer (mirrored control points
    # give a different null-space approximation); they are taken from the oracle's restated solver,
    # whose eigenpairs are pinned against numpy in test_cpu_oracle.py.  Everything else is numpy.
    lam, V = np.linalg.eigh(D.T @ D)
    _, Vo, _ = ol.sym_eig(D.T @ D)
    V = V * np.sign(np.sum(V * Vo, axis=0))
    cw = np.vstack([c0] + [c0 + np.sqrt(lam[i] / n) * V[:, i] for i in range(3)])
    a = np.linalg.solve((cw[1:] - c0).T, D.T).T
    al = np.column_stack([1.0 - a.sum(1), a])
    M = np.zeros((2 * n, 12))
    for j in range(4):
        M[0::2, 3 * j] = al[:, j] * fx
        M[0::2, 3 * j + 2] = al[:, j] * (cx - uv[:, 0])
        M[1::2, 3 * j + 1] = al[:, j] * fy
        M[1::2, 3 * j + 2] = al[:, j] * (cy - uv[:, 1])
    _, EV = np.linalg.eigh(M.T @ M)
    v = [EV[:, i] for i in range(4)]  # null-space basis, smallest eigenvalue first
    dv = [[v[i][3 * a:3 * a + 3] - v[i][3 * b:3 * b + 3] for (a, b) in PAIRS] for i in range(4)]
    L = np.zeros((6, 10))
    for j in range(6):
        d = [dv[i][j] for i in range(4)]
        L[j] = [d[0] @ d[0], 2 * d[0] @ d[1], d[1] @ d[1], 2 * d[0] @ d[2], 2 * d[1] @ d[2], d[2] @ d[2],
                2 * d[0] @ d[3], 2 * d[1] @ d[3], 2 * d[2] @ d[3], d[3] @ d[3]]
    rho = np.array([np.sum((cw[a] - cw[b]) ** 2) for (a, b) in PAIRS])

    def quad(b):
        return np.array([b[0] * b[0], b[0] * b[1], b[1] * b[1], b[0] * b[2], b[1] * b[2], b[2] * b[2],
                         b[0] * b[3], b[1] * b[3], b[2] * b[3], b[3] * b[3]])

    def gauss_newton(b):
        b = b.copy()
        for _ in range(5):
            J = np.zeros((6, 4))
            for j in range(6):
                l = L[j]
                J[j] = [2 * l[0] * b[0] + l[1] * b[1] + l[3] * b[2] + l[6] * b[3],
                        l[1] * b[0] + 2 * l[2] * b[1] + l[4] * b[2] + l[7] * b[3],
                        l[3] * b[0] + l[4] * b[1] + 2 * l[5] * b[2] + l[8] * b[3],
                        l[6] * b[0] + l[7] * b[1] + l[8] * b[2] + 2 * l[9] * b[3]]
            r = rho - L @ quad(b)
            b = b + np.linalg.lstsq(J, r, rcond=None)[0]
        return b

    betas = []
    x = np.linalg.lstsq(L[:, [0, 1, 3, 6]], rho, rcond=None)[0]
    b0 = np.sqrt(abs(x[0]))
    s = -1.0 if x[0] < 0 else 1.0
    betas.append(np.array([b0, s * x[1] / b0, s * x[2] / b0, s * x[3] / b0]))
    for cols in ([0, 1, 2], [0, 1, 2, 3, 4]):  # approximations 2 and 3 (published sign rules)
        x = np.linalg.lstsq(L[:, cols], rho, rcond=None)[0]
        if x[0] < 0:
            b0, b1 = np.sqrt(-x[0]), (np.sqrt(-x[2]) if x[2] < 0 else 0.0)
        else:
            b0, b1 = np.sqrt(x[0]), (np.sqrt(x[2]) if x[2] > 0 else 0.0)
        if x[1] < 0:
            b0 = -b0
        betas.append(np.array([b0, b1, x[3] / b0 if len(cols) == 5 else 0.0, 0.0]))
    best = None
    for b in betas:
        b = gauss_newton(b)
        ccs = sum(b[i] * v[i] for i in range(4)).reshape(4, 3)
        pcs = al @ ccs
        if pcs[0, 2] < 0:
            pcs = -pcs
        R, t = _procrustes(pw, pcs)
        e = _reproj(R, t, pw, uv, K)
        if best is None or e < best[0]:
            best = (e, R, t)
    return best[1], best[2]


@pytest.mark.parametrize("n", [6, 10, 30, 100, 400])
def test_epnp_noisy_sets_match_numpy(n):
    rng = np.random.default_rng(100 + n)
    checked = 0
    for _ in range(20):
        sc = synth.make_pnp_scene(rng, 600, 0.7)
        o = ol.OraclePnP(sc, 1)
        inl = np.flatnonzero(sc.inlier_true)
        idx = np.sort(rng.choice(inl, size=n, replace=False)).astype(np.int32)
        Ro, to, _ = o.compute_pose(idx)
        K = (float(sc.fx), float(sc.fy), float(sc.cx), float(sc.cy))
        pw = sc.p3dw[idx].astype(np.float64)
        uv = sc.p2d[idx].astype(np.float64)
        Rn, tn = epnp_numpy(pw, uv, K)
        # a 6-point noisy set can be ill-conditioned (pose error >> noise): compare where the
        # problem is well posed, i.e. where the textbook solution is itself near the truth
        if np.abs(Rn - sc.R_true).max() > 0.05:
            continue
        checked += 1
        assert np.abs(Ro - Rn).max() < 1e-4, (n, np.abs(Ro - Rn).max())
        assert np.abs(to - tn).max() < 1e-4 * max(1.0, np.abs(tn).max()), (n, np.abs(to - tn).max())
        co, io = o.check_inliers(Ro, to, sc.n)
        cn, inn = o.check_inliers(Rn.astype(np.float32), tn.astype(np.float32), sc.n)
        assert co == cn and np.array_equal(io, inn)
    assert checked >= 10


# ---------------------------------------------------------------------------------------------
# Sim3Solver::ComputeSim3 (fixed scale): absolute orientation of 3 points
# ---------------------------------------------------------------------------------------------
def test_sim3_three_point_alignment_matches_svd():
    rng = np.random.default_rng(7)
    checked = 0
    for _ in range(40):
        pair = synth.make_sim3_pair(rng, 200, 160)
        o = ol.OracleSim3(pair, 1)
        p = o.prepared()
        X1, X2 = p["X1c"].astype(np.float64), p["X2c"].astype(np.float64)
        for _ in range(10):
            idx = rng.choice(len(X1), size=3, replace=False).astype(np.int32)
            A, B = X1[idx], X2[idx]
            H = (B - B.mean(0)).T @ (A - A.mean(0))
            sv = np.linalg.svd(H, compute_uv=False)
            if sv[1] < 1e-2 * sv[0]:  # near-collinear triplet: orientation ill-posed
                continue
            R, t = _procrustes(B, A)  # maps frame-2 points onto frame 1
            Ro, to = o.compute(idx)
            checked += 1
            assert np.abs(Ro - R).max() < 1e-4, np.abs(Ro - R).max()
            assert np.abs(to - t).max() < 1e-4 * max(1.0, np.abs(t).max()), np.abs(to - t).max()
    assert checked > 200


# ---------------------------------------------------------------------------------------------
# MLPnP residual Jacobian
# ---------------------------------------------------------------------------------------------
def _rodrigues(w):
    th = np.linalg.norm(w)
    S = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-11:
        return np.eye(3)
    return np.eye(3) + np.sin(th) / th * S + (1 - np.cos(th)) / th ** 2 * (S @ S)


def _residual(x, X, nr, ns):
    y = _rodrigues(x[:3]) @ X + x[3:]
    u = y / np.linalg.norm(y)
    return np.array([nr @ u, ns @ u])


def _nullspace(b):
    U, _, _ = np.linalg.svd(b.reshape(3, 1))
    return U[:, 1], U[:, 2]


def _oracle_jac(X, nr, ns, x):
    J = np.zeros(12)
    ol.lib().ora_mlpnp_jac(np.ascontiguousarray(X, np.float64), np.ascontiguousarray(nr, np.float64),
                           np.ascontiguousarray(ns, np.float64), np.ascontiguousarray(x, np.float64), J)
    return J.reshape(2, 6)


def _fd_jac(X, nr, ns, x, h=1e-6):
    J = np.zeros((2, 6))
    for k in range(6):
        e = np.zeros(6)
        e[k] = h
        J[:, k] = (_residual(x + e, X, nr, ns) - _residual(x - e, X, nr, ns)) / (2 * h)
    return J


def test_mlpnp_jacobian_is_the_residual_derivative():
    rng = np.random.default_rng(11)
    worst = 0.0
    for _ in range(2000):
        w = synth.random_rotation(rng)  # a rotation -> its axis-angle vector
        th = np.arccos(np.clip((np.trace(w) - 1) / 2, -1, 1))
        axis = rng.normal(size=3)
        x = np.concatenate([axis / np.linalg.norm(axis) * max(th, 1e-3), rng.uniform(-2, 2, 3)])
        X = rng.uniform(-3, 3, 3) + np.array([0, 0, 6.0])
        b = _rodrigues(x[:3]) @ X + x[3:]
        b = b / np.linalg.norm(b) + rng.normal(size=3) * 1e-3
        nr, ns = _nullspace(b / np.linalg.norm(b))
        Ja = _oracle_jac(X, nr, ns, x)
        Jf = _fd_jac(X, nr, ns, x)
        scale = np.abs(Jf).max() + 1e-12
        worst = max(worst, np.abs(Ja - Jf).max() / scale)
    assert worst < 1e-6, worst


def _gn(x, X, NR, NS, jac):
    """mlpnp_gn's iteration (5 steps, LDLT normal equations -> lstsq here, x -= dx)."""
    x = x.copy()
    for _ in range(5):
        r = np.concatenate([_residual(x, X[i], NR[i], NS[i]) for i in range(len(X))])
        J = np.vstack([jac(X[i], NR[i], NS[i], x) for i in range(len(X))])
        dx = np.linalg.solve(J.T @ J, J.T @ r)
        x = x - dx
        if np.abs(J @ dx).max() < 1e-5:
            break
    return x


@pytest.mark.parametrize("n", [6, 20, 100])
def test_mlpnp_gauss_newton_poses_agree_with_finite_difference_jacobian(n):
    rng = np.random.default_rng(20 + n)
    for _ in range(10):
        R = synth.random_rotation(rng, 0.8)
        t = rng.uniform(-1, 1, 3)
        X = rng.uniform(-3, 3, (n, 3)) + np.array([0, 0, 7.0])
        B = (X @ R.T + t)
        B = B / np.linalg.norm(B, axis=1, keepdims=True) + rng.normal(size=(n, 3)) * 5e-4
        B = B / np.linalg.norm(B, axis=1, keepdims=True)
        NR, NS = zip(*[_nullspace(b) for b in B])
        th = np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))
        w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) * th / (2 * np.sin(th))
        x0 = np.concatenate([w, t]) + rng.normal(size=6) * 1e-2
        xa = _gn(x0, X, NR, NS, _oracle_jac)
        xf = _gn(x0, X, NR, NS, _fd_jac)
        Ra, Rf = _rodrigues(xa[:3]), _rodrigues(xf[:3])
        assert np.abs(Ra - Rf).max() < 1e-4 and np.abs(xa[3:] - xf[3:]).max() < 1e-4
        assert np.abs(Ra - R).max() < 5e-2
