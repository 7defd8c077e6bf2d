"""CPU: the event form and the split chase (QrChase12 + QrRowApply: one lane chases and logs the
rotations, any lanes replay them on rows of Q, in chunks) of the 12x12 implicit symmetric QR (rsc_core.h tridiag_qr_events12, used by
the hypothesis eigen-stage kernel) is bit-identical to the sweep form tridiag_qr (the restated
SelfAdjointEigenSolver) — eigenvalues, sort permutation, eigenvector matrix and the converged flag —
on EPnP-like spectra (four near-null eigenvalues), wide dynamic ranges, repeated and exactly zero
eigenvalues, diagonal and already-tridiagonal inputs."""
import numpy as np
import pytest

import hostemu_lib as hl


def run(A):
    A = np.ascontiguousarray(A, np.float64).reshape(144)
    out = [np.zeros(12), np.zeros(12, np.int32), np.zeros(144), np.zeros(1, np.int32),
           np.zeros(12), np.zeros(12, np.int32), np.zeros(144), np.zeros(1, np.int32)]
    hl.lib().he_qr_compare(A, *out)
    return out


def split(A, cap):
    A = np.ascontiguousarray(A, np.float64).reshape(144)
    out = [np.zeros(12), np.zeros(12, np.int32), np.zeros(144), np.zeros(1, np.int32)]
    hl.lib().he_qr_split(A, cap, *out)
    return out


def same(a, b):
    d1, p1, q1, o1 = a
    d2, p2, q2, o2 = b
    assert o1[0] == o2[0]
    assert np.array_equal(p1, p2)
    assert np.array_equal(d1.view(np.uint64), d2.view(np.uint64))
    assert np.array_equal(q1.view(np.uint64), q2.view(np.uint64))


def check(A):
    r = run(A)
    same(r[:4], r[4:])
    for cap in (1, 7, 32):
        same(r[:4], split(A, cap))


def spd(rng, lams):
    V, _ = np.linalg.qr(rng.normal(size=(12, 12)))
    return (V * lams) @ V.T


@pytest.mark.parametrize("seed", range(4))
def test_epnp_like_spectra(seed):
    rng = np.random.default_rng(seed)
    for _ in range(250):
        null = 10.0 ** rng.uniform(-14, -3, 4)
        rest = 10.0 ** rng.uniform(-2, 7, 8)
        A = spd(rng, rng.permutation(np.concatenate([null, rest])))
        check(A)


def test_from_epnp_rows():
    """M^T M of random 2n x 12 EPnP-shaped systems (n = 4..40)."""
    rng = np.random.default_rng(9)
    for _ in range(300):
        n = int(rng.integers(4, 41))
        M = rng.normal(size=(2 * n, 12)) * 10.0 ** rng.uniform(-1, 3, 12)
        check(M.T @ M)


def test_degenerate_inputs():
    rng = np.random.default_rng(10)
    check(np.zeros((12, 12)))
    check(np.eye(12))
    check(np.diag(rng.normal(size=12)))
    check(np.diag(np.repeat([1.0, 2.0, 3.0], 4)))
    T = np.diag(rng.normal(size=12)) + np.diag(rng.normal(size=11), 1) + np.diag(rng.normal(size=11), -1)
    check(T)
    T[5, 6] = T[6, 5] = 0.0
    check(T)
    for _ in range(50):
        lam = rng.choice([0.0, 1.0, 1e-9, 5.0], size=12)
        check(spd(rng, lam))
