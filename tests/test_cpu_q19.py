"""Q19 — the eta of PnPsolver::qr_solve (PnPsolver.cpp:714-720).

The reference scans column k with a pointer that is dereferenced BEFORE it advances:

    double * ppAik = ppAkk, eta = fabs(*ppAik);
    for(int i = k + 1; i < nr; i++) { double elt = fabs(*ppAik); if (eta < elt) eta = elt; ppAik += nc; }

so iteration i reads row i-1: eta = max |A[k..nr-2][k]| (row k twice, row nr-1 = 5 never).  The
oracle (and the kernels, checked on the GPU in tests/test_gpu_pnp.py) must scale the Householder
column by THAT eta, and take the singular bail-out (:722-726) when rows k..4 are zero even if row 5
is not.  The checker here is a literal transcription of the pointer walk over the row-major buffer
(A.data() of the RowMajor 6x4 matrix), evaluated in IEEE double in the reference's operation order.
"""
import math

import numpy as np

import oracle_lib as ol


def pointer_walk_qr_solve(A, b, X):
    """PnPsolver.cpp:693-796 transcribed with the flat row-major buffer and pointer offsets."""
    pA = [float(v) for v in np.asarray(A, np.float64).reshape(24)]
    pb = [float(v) for v in np.asarray(b, np.float64).reshape(6)]
    pX = [float(v) for v in np.asarray(X, np.float64).reshape(4)]
    nr, nc = 6, 4
    A1 = [0.0] * nr
    A2 = [0.0] * nr
    ppAkk = 0
    for k in range(nc):
        ppAik = ppAkk
        eta = abs(pA[ppAik])
        for _i in range(k + 1, nr):
            elt = abs(pA[ppAik])
            if eta < elt:
                eta = elt
            ppAik += nc
        if eta == 0:
            A1[k] = A2[k] = 0.0
            return pX, False
        ppAik = ppAkk
        s = 0.0
        inv_eta = 1.0 / eta
        for _i in range(k, nr):
            pA[ppAik] *= inv_eta
            s += pA[ppAik] * pA[ppAik]
            ppAik += nc
        sigma = math.sqrt(s)
        if pA[ppAkk] < 0:
            sigma = -sigma
        pA[ppAkk] += sigma
        A1[k] = sigma * pA[ppAkk]
        A2[k] = -eta * sigma
        for j in range(k + 1, nc):
            ppAik = ppAkk
            s = 0.0
            for _i in range(k, nr):
                s += pA[ppAik] * pA[ppAik + j - k]
                ppAik += nc
            tau = s / A1[k]
            ppAik = ppAkk
            for _i in range(k, nr):
                pA[ppAik + j - k] -= tau * pA[ppAik]
                ppAik += nc
        ppAkk += nc + 1
    ppAjj = 0
    for j in range(nc):
        ppAij = ppAjj
        tau = 0.0
        for i in range(j, nr):
            tau += pA[ppAij] * pb[i]
            ppAij += nc
        tau /= A1[j]
        ppAij = ppAjj
        for i in range(j, nr):
            pb[i] -= tau * pA[ppAij]
            ppAij += nc
        ppAjj += nc + 1
    pX[nc - 1] = pb[nc - 1] / A2[nc - 1]
    for i in range(nc - 2, -1, -1):
        ppAij = i * nc + (i + 1)
        s = 0.0
        for j in range(i + 1, nc):
            s += pA[ppAij] * pX[j]
            ppAij += 1
        pX[i] = (pb[i] - s) / A2[i]
    return pX, True


def q19_cases(seed=19, n_random=400):
    """(A, b, X0) systems: row 5 the column maximum in every column, only row 5 non-zero in a
    column (singular in the reference, regular with an eta over all six rows), and random ones."""
    rng = np.random.default_rng(seed)
    cases = []
    for _ in range(64):  # |A[5][k]| the column maximum for every k
        A = rng.uniform(-1, 1, (6, 4))
        A[5] = np.sign(rng.uniform(-1, 1, 4)) * rng.uniform(3, 50, 4)
        cases.append((A, rng.uniform(-2, 2, 6), rng.uniform(-1, 1, 4)))
    for k in range(4):  # column k zero in rows k..4, row 5 non-zero (singular at k = 0)
        for _ in range(4):
            A = rng.uniform(-1, 1, (6, 4))
            A[k:5, k] = 0.0
            A[5, k] = rng.uniform(0.5, 2.0)
            cases.append((A, rng.uniform(-2, 2, 6), rng.uniform(-1, 1, 4)))
    for _ in range(n_random):
        A = rng.normal(size=(6, 4)) * 10.0 ** rng.uniform(-3, 3)
        cases.append((A, rng.normal(size=6), np.zeros(4)))
    # an exactly singular column and an all-zero system
    A = rng.uniform(-1, 1, (6, 4)); A[:, 2] = 0.0
    cases.append((A, rng.normal(size=6), np.array([0.25, -0.5, 1.0, 2.0])))
    cases.append((np.zeros((6, 4)), rng.normal(size=6), np.array([1.0, 2.0, 3.0, 4.0])))
    return cases


def test_q19_oracle_equals_pointer_walk_bit_for_bit():
    for n, (A, b, X0) in enumerate(q19_cases()):
        want, ok_want = pointer_walk_qr_solve(A, b, X0)
        got, ok = ol.qr_solve(A, b, X0)
        assert ok == ok_want, n
        assert np.array_equal(np.array(want).view(np.uint64), got.view(np.uint64)), (n, want, got)


def test_q19_row5_never_scanned():
    """Row 5 the column maximum: the reference's eta (rows k..4) changes the rounding of X against an
    eta over all six rows; only row 5 non-zero: the reference bails out (X kept), a six-row scan
    would not."""
    rng = np.random.default_rng(7)
    differs = 0
    for _ in range(64):
        A = rng.uniform(-1, 1, (6, 4))
        A[5] = rng.uniform(3, 50, 4)
        b = rng.uniform(-2, 2, 6)
        X, ok = ol.qr_solve(A, b, np.zeros(4))
        assert ok
        # the six-row variant, for contrast: scale row 5 into the eta by putting the max into row 4
        # is NOT equivalent, so emulate it by transcribing with the true column maximum.
        six = _six_row_eta_solve(A, b)
        differs += not np.array_equal(X.view(np.uint64), np.array(six).view(np.uint64))
        # both are solutions of the same least-squares problem
        ref = np.linalg.lstsq(A[:, :4], b, rcond=None)[0]
        assert np.allclose(X, ref, rtol=1e-9, atol=1e-9)
    assert differs > 0
    # column 0 is examined on the untransformed A: rows 0..4 zero, row 5 not -> bail-out
    for _ in range(8):
        A = rng.uniform(-1, 1, (6, 4))
        A[0:5, 0] = 0.0
        A[5, 0] = rng.uniform(0.5, 2.0)
        X0 = np.array([0.5, -0.25, 0.125, 4.0])
        X, ok = ol.qr_solve(A, rng.uniform(-1, 1, 6), X0)
        assert not ok
        assert np.array_equal(X, X0)
        assert _six_row_eta_solve(A, rng.uniform(-1, 1, 6)) is not None  # regular for a six-row scan


def _six_row_eta_solve(A, b):
    """The textbook form (eta over rows k..5) — what rounds 1-3 restated; used only for contrast."""
    A = np.array(A, np.float64).copy()
    b = [float(v) for v in b]
    A1 = [0.0] * 4
    A2 = [0.0] * 4
    for k in range(4):
        eta = max(abs(float(A[i, k])) for i in range(k, 6))
        inv_eta = 1.0 / eta
        s = 0.0
        for i in range(k, 6):
            A[i, k] = float(A[i, k]) * inv_eta
            s += float(A[i, k]) * float(A[i, k])
        sigma = math.sqrt(s)
        if A[k, k] < 0:
            sigma = -sigma
        A[k, k] = float(A[k, k]) + sigma
        A1[k] = sigma * float(A[k, k])
        A2[k] = -eta * sigma
        for j in range(k + 1, 4):
            s = 0.0
            for i in range(k, 6):
                s += float(A[i, k]) * float(A[i, j])
            tau = s / A1[k]
            for i in range(k, 6):
                A[i, j] = float(A[i, j]) - tau * float(A[i, k])
    for j in range(4):
        tau = 0.0
        for i in range(j, 6):
            tau += float(A[i, j]) * b[i]
        tau /= A1[j]
        for i in range(j, 6):
            b[i] -= tau * float(A[i, j])
    X = [0.0] * 4
    X[3] = b[3] / A2[3]
    for i in range(2, -1, -1):
        s = 0.0
        for j in range(i + 1, 4):
            s += float(A[i, j]) * X[j]
        X[i] = (b[i] - s) / A2[i]
    return X
