"""GPU: the device libm restatement (rsc_math.h — fdlibm-style sin/cos/acos/cbrt/log and the
correctly rounded pow(x, 1/3) / pow(x, 3/2) used by the Sim3 angles, MLPnP and MapPoint::PredictScale in SearchBySim3) evaluated ON THE GPU through
rsc_selftest_math, checked (a) bit-for-bit against the same functions compiled for the host (the
oracle's ora_dm_*: device code generation changes nothing) and (b) within 1 ulp of glibc (Python's
math module), the CPU test's bar (tests/test_cpu_mlpnp.py), on the ranges the kernels feed them."""
import math

import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import ctx as gpu_ctx

pytestmark = pytest.mark.gpu


def _inputs(rng):
    xs = np.concatenate([rng.uniform(-1, 1, 20000) * s for s in (1e-8, 1e-3, 1.0, 3.2, 50.0, 1e4)])
    edge = np.array([0.0, -0.0, math.pi / 4, -math.pi / 4, math.pi / 2, math.pi, 2 * math.pi, 1e-300, 5e-324])
    return np.concatenate([xs, edge])


def _ulp_close(a, b, k):
    return abs(a - b) <= k * math.ulp(b) + 1e-300


@pytest.mark.parametrize("name", ["sin", "cos", "acos", "cbrt", "log", "logf", "pow_1_3", "pow_3_2"])
def test_device_libm_matches_host_restatement_and_glibc(name):
    rng = np.random.default_rng(42)
    if name == "acos":
        x = np.concatenate([rng.uniform(-1, 1, 60000), [-1.0, 1.0, 0.0, 0.5, -0.5, 1 - 2**-52, -1 + 2**-52]])
    elif name in ("cbrt", "pow_1_3", "pow_3_2"):
        x = np.abs(_inputs(rng)) + 1e-300
        if name != "cbrt":  # MLPnP's ranges: the scale's |s| and the Jacobian's squared norms
            x = np.concatenate([x, 10.0 ** rng.uniform(-12, 12, 40000), [0.0, 1.0, 4.0, 8.0, 27.0]])
    elif name in ("log", "logf"):
        # SearchBySim3's PredictScale ratios and a wide sweep
        x = np.concatenate([rng.uniform(0.5, 3.0, 30000), 10.0 ** rng.uniform(-30, 30, 30000), [1.0, 2.0, 1.2]])
    else:
        x = _inputs(rng)
    dev = gpu_ctx().selftest_math(name, x)
    L = ol.lib()
    host_fn = {"sin": L.ora_dm_sin, "cos": L.ora_dm_cos, "acos": L.ora_dm_acos, "cbrt": L.ora_dm_cbrt,
               "log": L.ora_dm_log, "logf": L.ora_dm_log, "pow_1_3": L.ora_dm_pow13, "pow_3_2": L.ora_dm_pow32}[name]
    if name == "logf":
        host = np.array([float(np.float32(host_fn(float(np.float32(v))))) for v in x])
    else:
        host = np.array([host_fn(float(v)) for v in x])
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64)), name
    glibc = {"sin": math.sin, "cos": math.cos, "acos": math.acos,
             "cbrt": lambda v: float(np.cbrt(v)), "log": math.log,
             "pow_1_3": lambda v: math.pow(v, 1.0 / 3.0), "pow_3_2": lambda v: math.pow(v, 3.0 / 2.0),
             "logf": lambda v: float(np.float32(math.log(float(np.float32(v)))))}[name]
    k = 1
    for xi, di in zip(x, dev):
        gi = glibc(float(xi))
        if name == "logf":
            assert abs(di - gi) <= math.ulp(np.float32(gi)) + 1e-300, (name, xi, di, gi)
        else:
            assert _ulp_close(di, gi, k), (name, xi, di, gi)


# ---- the QR chase's short-chain forms (rsc_core.h sqrt_unit / recip_unit, and make_givens built
# from them) against IEEE numpy, bit for bit ----

def _givens_ieee(p, q):
    """JacobiRotation::makeGivens (real case) with IEEE operations (numpy), as rsc_core.h."""
    with np.errstate(all="ignore"):
        big = np.abs(p) > np.abs(q)
        t = np.where(big, q, p) / np.where(big, p, q)
        u = np.sqrt(1.0 + t * t)
        u = np.where(np.where(big, p, q) < 0, -u, u)
        r = 1.0 / u
        sb = -r
        c = np.where(big, r, (-t) * sb)
        s = np.where(big, (-t) * r, sb)
        c = np.where(p == 0, 0.0, c)
        s = np.where(p == 0, np.where(q < 0, 1.0, -1.0), s)
        c = np.where(q == 0, np.where(p < 0, -1.0, 1.0), c)
        s = np.where(q == 0, 0.0, s)
    return c, s


def _same_bits(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("name", ["sqrt_unit", "recip_unit", "givens_c", "givens_s"])
def test_chase_arithmetic_is_ieee(name):
    rng = np.random.default_rng(11)
    if name == "sqrt_unit":
        x = np.concatenate([rng.uniform(1.0, 4.0, 300000), 1.0 + rng.uniform(0, 1, 100000) ** 2,
                            [1.0, 2.0, 3.0, np.nextafter(4.0, 0), np.nextafter(1.0, 2), 2.0 - 2**-52]])
        want = np.sqrt(x)
    elif name == "recip_unit":
        x = rng.uniform(1.0, 2.0, 300000) * rng.choice([-1.0, 1.0], 300000)
        x = np.concatenate([x, [1.0, -1.0, np.nextafter(2.0, 0), -np.nextafter(2.0, 0), 2.0**0.5, -(2.0**0.5),
                                np.nextafter(1.0, 2)]])
        want = 1.0 / x
    else:
        n = 200000
        mags = 10.0 ** rng.uniform(-300, 300, n) * rng.choice([-1.0, 1.0], n)
        mid = rng.standard_normal(n) * 10.0 ** rng.integers(-20, 3, n)
        special = np.array([0.0, -0.0, 1.0, -1.0, 5e-324, -5e-324, np.inf, -np.inf, np.nan, 1e-300, -1e-300] * 10)
        x = np.concatenate([mags, mid, special])
        x = x[rng.permutation(x.size)]
        c, s = _givens_ieee(x, x[(np.arange(x.size) + x.size // 2) % x.size])
        want = c if name == "givens_c" else s
    dev = gpu_ctx().selftest_math(name, x)
    bad = np.flatnonzero(~_same_bits(dev, want))
    assert bad.size == 0, [(float(x[i]), float(dev[i]), float(want[i])) for i in bad[:8]]


def test_device_qr_solve_q19_matches_oracle():
    """Q19 (PnPsolver.cpp:714-720): the kernels' qr_solve_6x4 on the GPU — eta over rows k..4,
    the singular bail-out keeping X — bit-for-bit equal to the oracle (itself equal to a literal
    pointer-walk transcription, tests/test_cpu_q19.py)."""
    from test_cpu_q19 import q19_cases
    cases = q19_cases(seed=1919, n_random=2000)
    A = np.stack([c[0] for c in cases])
    b = np.stack([c[1] for c in cases])
    X0 = np.stack([c[2] for c in cases])
    X, ok = gpu_ctx().qr_solve(A, b, X0)
    n_singular = 0
    for i, (Ai, bi, Xi) in enumerate(cases):
        want, ok_want = ol.qr_solve(Ai, bi, Xi)
        assert ok[i] == ok_want, i
        assert np.array_equal(X[i].view(np.uint64), want.view(np.uint64)), (i, X[i], want)
        n_singular += not ok_want
    assert n_singular >= 4


def test_scan_reciprocal_is_ieee_in_its_range():
    """The PnP scan's invZc = 1/Zc (PnPsolver.cpp:251) is v_rcp_f32 + one FMA Newton step
    (kernels.hip pnp_inlier2), used only for 2^-126 <= |z| <= 2^125 (the scan redoes a hypothesis
    with the IEEE division when a depth falls outside).  Here: every significand of one binade in
    both signs, both ends of the range, and random floats across the range, against IEEE float32
    1/z (numpy) bit for bit.  The whole 2^32 sweep is tools/rcp_exhaustive.hip
    (profiles/r05/rcp_exhaustive_r5f.txt: 0 mismatches for exponent fields 1..252)."""
    rng = np.random.default_rng(5)
    mant = np.arange(1 << 23, dtype=np.uint32)
    pats = [mant | np.uint32(127 << 23), mant[::7] | np.uint32(1 << 23), mant[::7] | np.uint32(252 << 23),
            rng.integers(1 << 23, 253 << 23, 2_000_000, dtype=np.uint32)]
    bits = np.concatenate(pats)
    bits = np.concatenate([bits, bits[: 1 << 23] | np.uint32(0x80000000)])
    z = bits.view(np.float32)
    dev = gpu_ctx().selftest_math("rcp_scan", z.astype(np.float64)).astype(np.float32)
    ref = np.float32(1.0) / z
    bad = np.flatnonzero(dev.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, (bad.size, z[bad[:5]], dev[bad[:5]], ref[bad[:5]])


def test_ldlt_row_per_lane_matches_scalar():
    """The LM steps' LDLT (rsc_poseopt.h): the row-per-lane form the PoseOptimization / OptimizeSim3
    kernels run equals the scalar restatement bit for bit — solution and isPositive() — on SPD systems
    like H + lambda I, on matrices whose pivoting exchanges rows, with ties on the diagonal, indefinite
    and singular ones (zero first pivot: Eigen's early stop) and non-finite entries."""
    rng = np.random.default_rng(1616)
    recs = []
    for t in range(3000):
        kind = t % 6
        if kind == 0:      # SPD, LM-like scales
            J = rng.standard_normal((12, 6)) * 10.0 ** rng.uniform(-3, 3, 6)
            A = J.T @ J + np.eye(6) * 10.0 ** rng.uniform(-6, 2)
        elif kind == 1:    # random symmetric (indefinite)
            M = rng.standard_normal((6, 6))
            A = M + M.T
        elif kind == 2:    # diagonal ties
            M = rng.standard_normal((6, 6)) * 0.1
            A = M + M.T + np.diag(np.repeat(rng.uniform(1, 3), 6))
        elif kind == 3:    # singular / zero pivot
            M = rng.standard_normal((6, 3))
            A = M @ M.T
            A[:, rng.integers(6)] = 0.0
            A[rng.integers(6), :] = 0.0
            A = 0.5 * (A + A.T)
            if t % 12 == 3:
                A[:] = 0.0
        elif kind == 4:    # large dynamic range
            d = 10.0 ** rng.uniform(-150, 150, 6)
            A = np.diag(d) + np.outer(d, d) ** 0.5 * 1e-3
        else:              # non-finite entries
            M = rng.standard_normal((6, 6))
            A = M + M.T
            i, j = rng.integers(6, size=2)
            A[i, j] = A[j, i] = [np.inf, np.nan, -np.inf][t % 3]
        b = rng.standard_normal(6) * 10.0 ** rng.uniform(-3, 3)
        recs.append(np.concatenate([A.reshape(-1), b]))
    x = np.concatenate(recs)
    out = gpu_ctx().selftest_math("ldlt_lanes", x).reshape(-1, 42)
    assert np.array_equal(out[:, 6], out[:, 13])
    ok = out[:, 6] == 1.0
    assert ok.sum() > 1000 and (~ok).sum() > 100
    same = _same_bits(out[ok, 0:6], out[ok, 7:13]).all(axis=1)
    assert same.all(), np.flatnonzero(ok)[~same][:8]
