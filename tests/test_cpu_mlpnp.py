"""MLPnPsolver (config 4): oracle known answers, deterministic libm, and the host-compiled device
numerics (rsc_mlpnp.h) against the oracle restatement — bit-exact per hypothesis.

Parity with the reference itself is UNPINNED: MLPnPsolver.cpp is never compiled by the reference
(CMakeLists.txt:75) and has no tests.
"""
import math

import numpy as np
import pytest

import hostemu_lib as he
import oracle_lib as ol
from rsc import synth

RELOC6 = (0.99, 10, 300, 6, 0.5, 5.991)  # commented call Tracking.cpp:1227-1228


def test_libm_within_one_ulp_of_glibc():
    L = ol.lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-1, 1, 3000) * s for s in (1e-3, 1.0, 3.2, 50.0, 1e4)])
    for name, ref, dom in (("sin", math.sin, xs), ("cos", math.cos, xs),
                           ("acos", math.acos, rng.uniform(-1, 1, 5000)),
                           ("cbrt", lambda v: math.copysign(abs(v) ** (1.0 / 3.0), v), np.abs(xs) + 1e-300)):
        f = getattr(L, "ora_dm_" + name)
        for x in dom:
            a, b = f(float(x)), ref(float(x))
            tol = (4 if name == "cbrt" else 1) * math.ulp(b) + 1e-300
            assert abs(a - b) <= tol, (name, x, a, b)
    assert L.ora_dm_acos(1.0) == 0.0 and L.ora_dm_acos(-1.0) == math.pi
    assert math.isnan(L.ora_dm_acos(1.5))


def test_known_answer_noise_free():
    rng = np.random.default_rng(3)
    for _ in range(10):
        sc = synth.make_pnp_scene(rng, 60, 1.0, noise=False)
        o = ol.OracleMLPnP(sc, 1)
        for n in (6, 12, 60):
            R, t = o.compute_pose(np.arange(n))
            assert np.abs(R - sc.R_true).max() < 2e-6 and np.abs(t - sc.t_true).max() < 2e-5, n


def test_ransac_recovers_pose_and_iterate_contract():
    rng = np.random.default_rng(4)
    sc = synth.make_pnp_scene(rng, 800, 0.6)
    o = ol.OracleMLPnP(sc, 1)
    o.set_ransac_parameters(*RELOC6)
    r = o.iterate(5)
    assert r["ok"] and r["n_inliers"] > o.info()["min_inliers"]
    assert np.abs(r["T"][:3, :3] - sc.R_true).max() < 2e-2
    # failure: identity T and empty inliers (Q10)
    sc2 = synth.make_pnp_scene(rng, 800, 0.3)
    o2 = ol.OracleMLPnP(sc2, 1)
    o2.set_ransac_parameters(*RELOC6)
    r2 = o2.iterate(5)
    assert not r2["ok"] and len(r2["inliers"]) == 0
    assert np.array_equal(r2["T"], np.eye(4, dtype=np.float32))


@pytest.mark.parametrize("ns", [6, 7, 8])
def test_device_numerics_bitexact_vs_oracle(ns):
    rng = np.random.default_rng(10 + ns)
    sc = synth.make_pnp_scene(rng, 500, 0.5)
    o = ol.OracleMLPnP(sc, 7)
    o.set_ransac_parameters(0.99, 10, 300, ns, 0.5, 5.991)
    o.enable_trace()
    o.iterate(60)
    ints, dbl = o.trace()
    assert len(ints) == 60
    for h in range(60):
        idx, R, t = he.mlpnp_hypothesis(sc, 7, h, ns)
        assert idx.tolist() == ints[h, :ns].tolist(), h
        assert np.array_equal(R.ravel().view(np.uint64), dbl[h, :9].view(np.uint64)), h
        assert np.array_equal(t.view(np.uint64), dbl[h, 9:].view(np.uint64)), h
        c, _ = he.mlpnp_count(sc, R, t)
        assert c == ints[h, 8], h


def test_device_numerics_planar_bitexact():
    """Points on a plane through the world origin take the planar branch (FullPivHouseholderQR rank 2)."""
    rng = np.random.default_rng(21)
    R = synth.random_rotation(rng)
    t = np.array([0.2, -0.1, 4.0])
    n = 200
    Xw = np.c_[rng.uniform(-1.5, 1.5, (n, 2)), np.zeros(n)]
    Xc = Xw @ R.T + t
    uv = np.c_[synth.FX * Xc[:, 0] / Xc[:, 2] + synth.CX, synth.FY * Xc[:, 1] / Xc[:, 2] + synth.CY]
    uv += rng.normal(size=uv.shape) * 0.5
    sc = synth.PnPScene(p2d=uv.astype(np.float32), p3dw=Xw.astype(np.float32), sigma2=np.ones(n, np.float32),
                        kp_index=np.arange(n, dtype=np.int32), n_points=n, R_true=R, t_true=t,
                        inlier_true=np.ones(n, bool))
    o = ol.OracleMLPnP(sc, 3)
    o.set_ransac_parameters(*RELOC6)
    o.enable_trace()
    o.iterate(20)
    ints, dbl = o.trace()
    for h in range(len(ints)):
        idx, Rh, th = he.mlpnp_hypothesis(sc, 3, h, 6)
        assert idx.tolist() == ints[h, :6].tolist()
        assert np.array_equal(Rh.ravel().view(np.uint64), dbl[h, :9].view(np.uint64)), h
        assert np.array_equal(th.view(np.uint64), dbl[h, 9:].view(np.uint64)), h


def bearing_covariances(sc, extra=1e-9):
    """computePose covMats for the config-4 'with covariances' case: the keypoint's isotropic pixel
    variance (mvLevelSigma2) pushed through the bearing map ((u - cx) / fx, (v - cy) / fy, 1), plus
    a tiny isotropic term; [n, 3, 3]."""
    s2 = np.asarray(sc.sigma2, np.float64)
    cov = np.zeros((sc.n, 3, 3))
    cov[:, 0, 0] = s2 / float(sc.fx) ** 2
    cov[:, 1, 1] = s2 / float(sc.fy) ** 2
    cov += np.eye(3) * extra
    return cov


@pytest.mark.parametrize("ns", [6, 7, 8])
def test_covariance_branch_bitexact_vs_oracle(ns):
    """computePose's covMats branch (MLPnPsolver.cpp:375-388, :483-484, :694-695; dead in the
    reference's own calls, parity unpinned): the device numerics (host-compiled) against the
    oracle's restatement, per hypothesis."""
    rng = np.random.default_rng(40 + ns)
    sc = synth.make_pnp_scene(rng, 400, 0.6)
    cov = bearing_covariances(sc)
    o = ol.OracleMLPnP(sc, 5)
    o.set_covariances(cov)
    o.set_ransac_parameters(0.99, 10, 300, ns, 0.5, 5.991)
    o.enable_trace()
    o.iterate(40)
    ints, dbl = o.trace()
    assert len(ints) >= 10  # iterate returns early once a hypothesis refines
    for h in range(len(ints)):
        idx, R, t = he.mlpnp_hypothesis(sc, 5, h, ns, cov=cov)
        assert idx.tolist() == ints[h, :ns].tolist(), h
        assert np.array_equal(R.ravel().view(np.uint64), dbl[h, :9].view(np.uint64)), h
        assert np.array_equal(t.view(np.uint64), dbl[h, 9:].view(np.uint64)), h


def test_covariance_branch_known_answer_and_difference():
    """Noise-free correspondences: the weighted solution is exact; on noisy ones it differs from the
    unweighted one (the branch is live), and both recover the pose."""
    rng = np.random.default_rng(44)
    sc = synth.make_pnp_scene(rng, 80, 1.0, noise=False)
    o = ol.OracleMLPnP(sc, 1)
    o.set_covariances(bearing_covariances(sc))
    for n in (6, 12, 80):
        R, t = o.compute_pose(np.arange(n))
        assert np.abs(R - sc.R_true).max() < 2e-6 and np.abs(t - sc.t_true).max() < 2e-5, n
    sc2 = synth.make_pnp_scene(rng, 80, 1.0)
    a, b = ol.OracleMLPnP(sc2, 1), ol.OracleMLPnP(sc2, 1)
    b.set_covariances(bearing_covariances(sc2))
    Ra, ta = a.compute_pose(np.arange(80))
    Rb, tb = b.compute_pose(np.arange(80))
    assert not np.array_equal(Ra, Rb)
    for R in (Ra, Rb):
        assert np.abs(R - sc2.R_true).max() < 2e-2
