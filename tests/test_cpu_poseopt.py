"""CPU: the Optimizer::PoseOptimization oracle (oracle/poseopt_oracle.cpp) on known answers and the
reference's control-flow rules, and the host build of the device orchestration (rsc_poseopt.h via
tests/hostemu) against it, bit for bit.  Parity against the reference binary is unpinned (g2o and
Eigen cannot be built here); these tests pin the restatement."""
import numpy as np
import pytest

import hostemu_lib as hl
import oracle_lib as ol
from rsc import synth


def frame(seed, n, ratio=0.8, **kw):
    return synth.make_poseopt_frame(np.random.default_rng(seed), n, ratio, **kw)


def test_noise_free_recovers_pose():
    """Known answer: exact observations, perturbed start -> the true pose (float output)."""
    for seed, n in [(1, 300), (2, 60), (3, 2000)]:
        f = frame(seed, n, 1.0, noise=False, rot_noise=0.05, trans_noise=0.1)
        r, T, out, st = ol.pose_optimization(f)
        assert r == n and not out.any()
        assert np.abs(T[:3, :3] - f.R_true).max() < 1e-5
        assert np.abs(T[:3, 3] - f.t_true).max() < 1e-5
        assert st[0] == 4  # all four rounds run with >= 10 edges


def test_gross_outliers_flagged():
    f = frame(4, 800, 0.7)
    r, T, out, st = ol.pose_optimization(f)
    assert (out[~f.inlier_true] == 1).all()          # every uniform-pixel outlier rejected
    assert r == int((out == 0).sum())                 # nGood = nInitial - nBad
    assert np.abs(T[:3, 3] - f.t_true).max() < 0.01


def test_fewer_than_three_edges_returns_zero_untouched():
    f = frame(5, 6, 1.0)
    f.has_mp[:] = 0
    f.has_mp[:2] = 1
    r, T, out, st = ol.pose_optimization(f)
    assert r == 0 and st[0] == 0
    assert np.array_equal(T, f.Tcw)
    assert list(out[:2]) == [0, 0] and (out[2:] == 255).all()  # mvbOutlier set false, others untouched


def test_fewer_than_ten_edges_single_round():
    """`if(optimizer.edges().size()<10) break;` (Optimizer.cpp:407-408) counts all edges."""
    r, T, out, st = ol.pose_optimization(frame(6, 9, 1.0))
    assert st[0] == 1
    r, T, out, st = ol.pose_optimization(frame(6, 10, 1.0))
    assert st[0] == 4


def test_slots_without_map_point_untouched():
    f = frame(7, 400, 0.8, no_mp_frac=0.3)
    r, T, out, st = ol.pose_optimization(f)
    assert (out[f.has_mp == 0] == 255).all()
    assert set(np.unique(out[f.has_mp == 1])) <= {0, 1}
    assert r == int((out[f.has_mp == 1] == 0).sum())


@pytest.mark.parametrize("block", range(4))
def test_device_numerics_match_oracle_bitwise(block):
    """rsc_poseopt.h (compiled for the host) in the kernel's orchestration == the oracle, bit for bit:
    pose bits, nGood, outlier flags and the LM iteration/trial counts."""
    rng = np.random.default_rng(900 + block)
    for _ in range(25):
        n = int(rng.integers(3, 700))
        f = synth.make_poseopt_frame(rng, n, float(rng.uniform(0.3, 1.0)), rot_noise=float(rng.uniform(0, 0.15)),
                                     trans_noise=float(rng.uniform(0, 0.4)),
                                     no_mp_frac=float(rng.choice([0.0, 0.2])))
        if int(f.has_mp.sum()) < 3:
            continue
        r, T, out, st = ol.pose_optimization(f)
        r2, T2, out2, st2 = hl.pose_optimization(f)
        sel = np.nonzero(f.has_mp)[0]
        assert r == r2
        assert np.array_equal(T.view(np.uint32), T2.view(np.uint32))
        assert np.array_equal(out[sel], out2)
        assert np.array_equal(st, st2)


def test_stereo_noise_free_recovers_pose():
    """Known answer with EdgeStereoSE3ProjectXYZOnlyPose edges (mvuRight >= 0): exact (u, v, u_right)
    observations, perturbed start -> the true pose, no outliers (Optimizer.cpp:290-323)."""
    for seed, n, sf in [(11, 300, 1.0), (12, 800, 0.7), (13, 60, 0.5)]:
        f = frame(seed, n, 1.0, noise=False, rot_noise=0.05, trans_noise=0.1, stereo_frac=sf)
        assert (f.u_right >= 0).sum() > 0
        r, T, out, st = ol.pose_optimization(f)
        assert r == n and not out.any()
        assert np.abs(T[:3, :3] - f.R_true).max() < 1e-5
        assert np.abs(T[:3, 3] - f.t_true).max() < 1e-5


def test_stereo_outliers_use_7815_threshold():
    """Stereo edges are classified against chi2 > 7.815 (chi2Stereo), mono edges against 5.991: a
    stereo edge whose only error is a right-image offset with chi2 between the two thresholds stays an
    inlier; the same offset on u (mono) is an outlier."""
    f = frame(14, 200, 1.0, noise=False, rot_noise=0.0, trans_noise=0.0, stereo_frac=1.0)
    f.Tcw[:3, :3] = f.R_true.astype(np.float32)
    f.Tcw[:3, 3] = f.t_true.astype(np.float32)
    k = 5
    off = np.float32(np.sqrt(6.9 / f.inv_sigma2[k]))  # chi2 = inv * off^2 = 6.9 in (5.991, 7.815]
    f.u_right[k] += off
    r, T, out, st = ol.pose_optimization(f)
    assert out[k] == 0
    g = frame(14, 200, 1.0, noise=False, rot_noise=0.0, trans_noise=0.0)
    g.Tcw[:3, :3] = g.R_true.astype(np.float32)
    g.Tcw[:3, 3] = g.t_true.astype(np.float32)
    g.uv[k, 0] += off
    r, T, out, st = ol.pose_optimization(g)
    assert out[k] == 1


def test_stereo_gross_outliers_flagged():
    f = frame(15, 900, 0.7, stereo_frac=0.8)
    r, T, out, st = ol.pose_optimization(f)
    assert (out[~f.inlier_true] == 1).all()
    assert r == int((out == 0).sum())
    assert np.abs(T[:3, 3] - f.t_true).max() < 0.01


@pytest.mark.parametrize("block", range(3))
def test_device_numerics_stereo_match_oracle_bitwise(block):
    """Mixed mono/stereo Frames (stereo share 0..100 %): rsc_poseopt.h host build == the oracle."""
    rng = np.random.default_rng(950 + block)
    for _ in range(20):
        n = int(rng.integers(3, 700))
        f = synth.make_poseopt_frame(rng, n, float(rng.uniform(0.3, 1.0)), rot_noise=float(rng.uniform(0, 0.15)),
                                     trans_noise=float(rng.uniform(0, 0.4)),
                                     no_mp_frac=float(rng.choice([0.0, 0.2])),
                                     stereo_frac=float(rng.choice([0.3, 0.6, 0.9, 1.0])))
        if int(f.has_mp.sum()) < 3:
            continue
        r, T, out, st = ol.pose_optimization(f)
        r2, T2, out2, st2 = hl.pose_optimization(f)
        sel = np.nonzero(f.has_mp)[0]
        assert r == r2
        assert np.array_equal(T.view(np.uint32), T2.view(np.uint32))
        assert np.array_equal(out[sel], out2)
        assert np.array_equal(st, st2)


def test_golden_regression():
    """Committed outputs of the oracle (tests/golden/poseopt_traces.npz, make_golden.py)."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "poseopt_traces.npz")
    g = np.load(path)
    for k in range(len(g["seeds"])):
        f = synth.make_poseopt_frame(np.random.default_rng(int(g["seeds"][k])), int(g["ns"][k]), float(g["ratios"][k]),
                                     no_mp_frac=float(g["no_mp"][k]))
        r, T, out, st = ol.pose_optimization(f)
        assert r == g["n_good"][k]
        assert np.array_equal(T.reshape(16).view(np.uint32), g["T"][k].view(np.uint32))
        assert np.array_equal(st, g["stats"][k])


def test_zero_product_free_terms_fold_identically():
    """The kernel's per-edge terms skip the products by the information matrix's zero entries
    (po_quad_terms_finite): the folded H / b must equal the full form's bit for bit, on edges chosen to
    make signed zeros (coordinates and errors of exactly +-0, points on the optical axis), on edges
    whose Jacobian overflows or is not finite (those take the full form), and on ordinary edges."""
    rng = np.random.default_rng(4242)
    K5 = np.array([458.654, 457.296, 367.215, 248.375, 47.9], np.float64)
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    pose = np.concatenate([q, rng.normal(size=3) * 0.3])
    ident = np.array([0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
    n = 600
    X = rng.normal(size=(n, 3)) * [2.0, 1.5, 1.0] + [0.0, 0.0, 5.0]
    e = rng.normal(size=(n, 3)) * 3.0
    inv = rng.choice([1.0, 0.694, 0.482, 0.335], n)
    flags = rng.integers(0, 4, n).astype(np.int32)
    zero = rng.random(n) < 0.3          # signed zeros in the inputs
    X[zero, 0] = np.where(rng.random(int(zero.sum())) < 0.5, 0.0, -0.0)
    X[zero[::-1], 1] = -0.0
    e[rng.random(n) < 0.2, 0] = -0.0
    e[rng.random(n) < 0.2, 1] = 0.0
    e[rng.random(n) < 0.2, 2] = -0.0
    for pz in (pose, ident):
        a, b, full = hl.po_fold_compare(X, e, inv, flags, pz, K5)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), np.nonzero(a.view(np.uint64) != b.view(np.uint64))
        assert full == 0
    # an axis point of the identity pose (x = y = 0: exact zero Jacobian entries everywhere)
    Xa = np.array([[0.0, 0.0, 4.0], [-0.0, 0.0, 3.0], [0.0, -0.0, 2.0]])
    ea = np.array([[0.0, -0.0, 0.0], [-0.0, -0.0, -0.0], [1.0, -0.0, 0.0]])
    a, b, full = hl.po_fold_compare(Xa, ea, np.ones(3), np.array([3, 1, 0], np.int32), ident, K5)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) and full == 0
    # non-finite and overflowing edges: full form, same bits (NaN payloads included)
    Xb = np.array([[1.0, 2.0, 0.0], [1e200, 1e200, 1e-200], [1.0, 1.0, 3.0], [1.0, 1.0, 3.0]])
    eb = np.array([[1.0, 1.0, 1.0], [1.0, 1.0, 1.0], [np.inf, 0.0, 0.0], [np.nan, 1.0, 0.0]])
    a, b, full = hl.po_fold_compare(Xb, eb, np.ones(4), np.array([3, 3, 3, 1], np.int32), ident, K5)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) and full == 4
