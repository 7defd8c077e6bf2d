"""CPU: the Optimizer::OptimizeSim3 oracle (oracle/sim3opt_oracle.cpp) on known answers and the
reference's control-flow rules (Optimizer.cpp:1054-1250), and the host build of the device
orchestration (rsc_sim3opt.h via tests/hostemu) against it, bit for bit.  Parity against the
reference binary is unpinned (g2o and Eigen cannot be built here)."""
import numpy as np
import pytest

import hostemu_lib as hl
import oracle_lib as ol
from rsc import synth


def q2R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def prob(seed, n, **kw):
    return synth.make_sim3opt_problem(np.random.default_rng(seed), n, **kw)


def test_noise_free_recovers_relative_pose_and_rejects_outliers():
    """Known answer: exact observations, planted outliers, a perturbed start -> the true S12
    (scale stays 1: _fix_scale) and exactly the planted outliers set to NULL."""
    for seed, n in [(1, 300), (2, 800), (3, 60)]:
        p = prob(seed, n, noise=False, outlier_frac=0.2, pose_noise=0.02)
        r, S, keep, st = ol.optimize_sim3(p)
        corr = p.valid == 1
        assert r == int((corr & p.inlier_true).sum())
        assert (keep[corr & ~p.inlier_true] == 0).all() and (keep[corr & p.inlier_true] == 1).all()
        assert (keep[~corr] == 1).all()
        assert np.abs(q2R(S[:4]) - p.R12_true).max() < 1e-6
        assert np.abs(S[4:7] - p.t12_true).max() < 1e-6
        assert S[7] == 1.0
        assert st[0] == int(corr.sum()) and st[1] == int((corr & ~p.inlier_true).sum())


def test_fewer_than_ten_inliers_returns_zero_and_keeps_the_estimate():
    """`if(nCorrespondences-nBad<10) return 0;` (Optimizer.cpp:1201-1202): g2oS12 untouched, the
    outliers of the first pass already set to NULL."""
    p = prob(4, 40, noise=False, outlier_frac=0.9, valid_frac=1.0)
    r, S, keep, st = ol.optimize_sim3(p)
    assert r == 0 and np.array_equal(S, p.S0)
    assert st[0] - st[1] < 10 and int((keep == 0).sum()) == st[1]


def test_no_correspondence():
    p = prob(5, 20, valid_frac=0.0)
    r, S, keep, st = ol.optimize_sim3(p)
    assert r == 0 and np.array_equal(S, p.S0) and (keep == 1).all() and st[2] == 0


def test_second_pass_iterations_rule():
    """nMoreIterations = 10 after removals, 5 otherwise (Optimizer.cpp:1196-1199): with no outlier the
    whole run is at most 5 + 5 LM iterations."""
    p = prob(6, 300, noise=False, outlier_frac=0.0, pose_noise=0.01)
    r, S, keep, st = ol.optimize_sim3(p)
    assert st[1] == 0 and st[2] <= 10 and r == int(p.valid.sum())


@pytest.mark.parametrize("block", range(3))
def test_device_numerics_match_oracle_bitwise(block):
    """rsc_sim3opt.h (compiled for the host) in the kernel's orchestration == the oracle, bit for bit:
    nIn, the Sim3 (q, t, s), the NULLed matches and the iteration/trial counts."""
    rng = np.random.default_rng(700 + block)
    for _ in range(15):
        p = synth.make_sim3opt_problem(rng, int(rng.integers(5, 700)), valid_frac=float(rng.uniform(0.4, 1.0)),
                                       outlier_frac=float(rng.uniform(0.0, 0.6)), noise=bool(rng.random() < 0.8),
                                       pose_noise=float(rng.uniform(0.0, 0.08)))
        a = ol.optimize_sim3(p)
        b = hl.optimize_sim3(p)
        assert a[0] == b[0]
        assert np.array_equal(a[1].view(np.uint64), b[1].view(np.uint64))
        assert np.array_equal(a[2], b[2])
        assert list(a[3][1:]) == list(b[3][1:])
