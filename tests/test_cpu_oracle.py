"""The oracle (CPU restatement of PnPsolver / Sim3Solver / DUtils::Random) pinned by everything this
container can check: glibc rand() via ctypes, numpy linear algebra, noise-free known answers, the
reference's quirk ledger and committed golden traces.  No GPU."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_lib as ol
from rsc import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def glibc_fixture():
    with open(os.path.join(GOLD, "glibc_rand.json")) as f:
        return json.load(f)


def test_glibc_rand_matches_fixture_and_libc(glibc_fixture):
    for seed, ref in glibc_fixture["rand"].items():
        assert np.array_equal(ol.glibc_rand(int(seed), len(ref)), np.array(ref, np.int32)), seed
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(31337))
    live = [libc.rand() for _ in range(5000)]
    assert np.array_equal(ol.glibc_rand(31337, 5000), np.array(live, np.int32))


def test_seed_zero_is_seed_one():
    assert np.array_equal(ol.glibc_rand(0, 100), ol.glibc_rand(1, 100))


def test_swap_remove_sample_stream(glibc_fixture):
    for case in glibc_fixture["samples"]:
        got = ol.sample_stream(case["seed"], case["N"], case["min_set"], case["hyps"])
        assert np.array_equal(got, np.array(case["idx"], np.int32)), case["N"]
        # a hypothesis never repeats an index (swap-remove)
        assert all(len(set(r)) == len(r) for r in got.tolist())


def test_random_int_formula():
    r = ol.glibc_rand(5, 1000)
    maxes = np.random.default_rng(0).integers(0, 5000, size=1000).astype(np.int32)
    got = ol.random_int(5, maxes)
    want = [int((x / 2147483648.0) * (m + 1)) for x, m in zip(r.tolist(), maxes.tolist())]
    assert got.tolist() == want


@pytest.mark.parametrize("n", [3, 4, 12])
def test_sym_eig_vs_numpy(n):
    rng = np.random.default_rng(n)
    for _ in range(20):
        A = rng.normal(size=(n, n))
        A = A + A.T
        w, V, ok = ol.sym_eig(A)
        assert ok
        assert np.all(np.diff(w) >= 0)  # ascending (Q4)
        assert np.allclose(w, np.linalg.eigvalsh(A), atol=1e-12 * np.abs(A).max() * n)
        assert np.abs(A @ V - V * w).max() < 1e-11 * np.abs(A).max() * n
        assert np.abs(V.T @ V - np.eye(n)).max() < 1e-12


def test_sym_eig_float4_vs_numpy():
    rng = np.random.default_rng(4)
    for _ in range(20):
        A = rng.normal(size=(4, 4)).astype(np.float32)
        A = A + A.T
        w, V, ok = ol.sym_eig4f(A)
        assert ok and np.all(np.diff(w) >= 0)
        assert np.allclose(w, np.linalg.eigvalsh(A.astype(np.float64)), atol=1e-5)


def test_sym_eig_rank_deficient_nullspace():
    """EPnP's MtM for 4 points has a 4-dim null space; the restated solver must find it."""
    rng = np.random.default_rng(1)
    M = rng.normal(size=(8, 12))
    A = M.T @ M
    w, V, ok = ol.sym_eig(A)
    assert ok
    assert np.abs(w[:4]).max() < 1e-12 * np.abs(A).max()
    assert np.abs(M @ V[:, :4]).max() < 1e-10


@pytest.mark.parametrize("k", [3, 4, 5])
def test_svd_solve_vs_numpy(k):
    rng = np.random.default_rng(k)
    for _ in range(20):
        A = rng.normal(size=(6, k))
        b = rng.normal(size=6)
        assert np.allclose(ol.svd_solve(A, b), np.linalg.lstsq(A, b, rcond=None)[0], atol=1e-12)
    A = rng.normal(size=(6, k))
    A[:, -1] = A[:, 0]  # rank deficient: minimum-norm solution, as JacobiSVD::solve
    b = rng.normal(size=6)
    assert np.allclose(ol.svd_solve(A, b), np.linalg.pinv(A) @ b, atol=1e-10)


def test_epnp_known_answer_minimal_is_basis_dependent():
    """n = 4 (the RANSAC sample): M is 8 x 12, so MtM has an exact 4-dimensional null space whose
    eigenvector basis is fixed by rounding alone, and find_betas_approx_1/2/3 keep only
    some of the 10 beta products — whether Gauss-Newton then reaches the true pose depends on that
    basis.  Over 200 noise-free scenes the restatement recovers it about 45 % of the time (the rounds
    1-3 left-to-right order: about 42 %), so the known answer is a rate, not a per-sample property;
    n >= 5 recovers it always (test_epnp_known_answer)."""
    ok = 0
    for k in range(200):
        rng = np.random.default_rng(4000 + k)
        sc = synth.make_pnp_scene(rng, 60, 1.0, noise=False)
        o = ol.OraclePnP(sc, 1)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        idx = np.sort(rng.choice(sc.n, 4, replace=False)).astype(np.int32)
        R, t, err = o.compute_pose(idx)
        good = np.abs(R - sc.R_true).max() < 2e-5 and np.abs(t - sc.t_true).max() < 2e-4
        ok += good
        if good:
            assert err < 0.05  # pixels; float-rounded inputs
    assert 0.3 < ok / 200 < 0.7


@pytest.mark.parametrize("n", [5, 6, 10, 50, 500])
def test_epnp_known_answer(n):
    """Noise-free correspondences: EPnP (compute_pose, PnPsolver.cpp:359-415) recovers Tcw."""
    rng = np.random.default_rng(100 + n)
    sc = synth.make_pnp_scene(rng, max(n, 60), 1.0, noise=False)
    o = ol.OraclePnP(sc, 1)
    o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    idx = np.sort(rng.choice(sc.n, n, replace=False)).astype(np.int32)
    R, t, err = o.compute_pose(idx)
    assert np.abs(R - sc.R_true).max() < 2e-5
    assert np.abs(t - sc.t_true).max() < 2e-4
    assert err < 1e-3


def test_horn_known_answer():
    """Noise-free 3-point Horn (Sim3Solver::ComputeSim3, scale 1) maps X2c onto X1c."""
    rng = np.random.default_rng(3)
    pair = synth.make_sim3_pair(rng, 200, 200, noise3d=0.0)
    o = ol.OracleSim3(pair, 1)
    p = o.prepared()
    for trial in range(20):
        idx = rng.choice(o.N, 3, replace=False).astype(np.int32)
        R, t = o.compute(idx)
        assert np.abs(p["X2c"] @ R.T + t - p["X1c"]).max() < 1e-4
        assert np.abs(R @ R.T - np.eye(3)).max() < 1e-5


def test_q2_iteration_formula():
    """Q2/Q17/Q18: minInliers = max(N*eps, minInliers, minSet), maxIts from log(1-p)/log(1-eps^3)."""
    rng = np.random.default_rng(0)
    sc = synth.make_pnp_scene(rng, 2000, 0.4)
    o = ol.OraclePnP(sc, 1)
    for eps, want_its in [(0.5, 35), (0.4, 70), (0.2, 300)]:
        o.set_ransac_parameters(0.99, 10, 300, 4, eps, 5.991)
        info = o.info()
        assert info["max_iterations"] == want_its
        assert info["min_inliers"] == int(2000 * np.float32(eps))
    pair = synth.make_sim3_pair(rng, 1000, 100)
    s = ol.OracleSim3(pair, 1)
    s.set_ransac_parameters(0.99, 20, 300)
    assert s.info()["max_iterations"] == 300


def test_q1_loop_conditions():
    """Q1: PnP '||' runs maxIts on the first iterate(5); Sim3 '&&' runs exactly 5."""
    rng = np.random.default_rng(1)
    sc = synth.make_pnp_scene(rng, 1000, 0.3)
    o = ol.OraclePnP(sc, 1)
    o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    r = o.iterate(5)
    assert o.info()["iterations"] == 35 and r["no_more"] and not r["ok"]
    assert len(r["inliers"]) == 0  # Q10: vbInliers cleared on failure
    r = o.iterate(5)
    assert o.info()["iterations"] == 40
    pair = synth.make_sim3_pair(rng, 1000, 10)
    s = ol.OracleSim3(pair, 1)
    s.set_ransac_parameters(0.99, 20, 300)
    r = s.iterate(5)
    assert s.info()["iterations"] == 5 and not r["no_more"]
    assert len(r["inliers"]) == pair.n1  # Q10: Sim3 vbInliers always sized mN1


def test_q11_sim3_thresholds_truncated():
    s2 = synth.level_sigma2()
    assert [int(9.210 * float(x)) for x in s2] == [9, 13, 19, 27, 39, 57, 82, 118]
    rng = np.random.default_rng(2)
    pair = synth.make_sim3_pair(rng, 100, 50)
    o = ol.OracleSim3(pair, 1)
    p = o.prepared()
    valid = pair.valid.astype(bool)
    assert np.array_equal(p["maxerr1"], (9.210 * pair.sigma2_1[valid].astype(np.float64)).astype(np.uint64))


def test_q6_stale_rows_change_later_hypotheses():
    """Q6: after an EPnP over many rows, a 4-point pose sees the stale rows in its centroids."""
    rng = np.random.default_rng(5)
    sc = synth.make_pnp_scene(rng, 300, 0.6)
    small = np.array([3, 17, 150, 211], np.int32)
    fresh = ol.OraclePnP(sc, 1)
    fresh.set_ransac_parameters()
    Rf, tf, _ = fresh.compute_pose(small)
    o = ol.OraclePnP(sc, 1)
    o.set_ransac_parameters()
    o.compute_pose(np.arange(120, dtype=np.int32))
    Rs, ts, _ = o.compute_pose(small)
    assert o.info()["max_rows"] == 120
    assert not (np.array_equal(Rf, Rs) and np.array_equal(tf, ts))


def test_q8_refine_strictness_and_q12_first_success():
    rng = np.random.default_rng(6)
    for k in range(4):
        sc = synth.make_pnp_scene(rng, 400, 0.65)
        o = ol.OraclePnP(sc, 10 + k)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        o.enable_trace()
        r = o.iterate(300)
        ints, _ = o.trace()
        mi = o.info()["min_inliers"]
        for row in ints:
            if row[9]:  # refine called iff count >= minInliers (Q8)
                assert row[8] >= mi and row[11] == (row[10] > mi)
            else:
                assert row[8] < mi
        if r["ok"] and ints[-1, 11] == 1:  # returned by a successful Refine (:159-166)
            assert r["n_inliers"] == ints[-1, 10]
        elif r["ok"]:  # budget exhausted, best >= minInliers returned (:173-188)
            assert r["no_more"] and len(ints) == o.info()["max_iterations"] or len(ints) == 300
            assert r["n_inliers"] == o.info()["best_inliers"] >= mi
    pair = synth.make_sim3_pair(rng, 500, 200)
    s = ol.OracleSim3(pair, 3)
    s.set_ransac_parameters(0.99, 20, 300)
    s.enable_trace()
    r = s.iterate(300)
    ints, _ = s.trace()
    assert r["ok"]
    first = int(np.argmax(ints[:, 3] > 20))
    assert first == len(ints) - 1 and r["n_inliers"] == ints[first, 3]


def test_golden_traces_reproduced():
    g = np.load(os.path.join(GOLD, "pnp_traces.npz"))
    for k in range(3):
        n, seed, sseed = g[f"s{k}_meta"].tolist()
        ratio = float(g[f"s{k}_ratio"][0])
        sc = synth.make_pnp_scene(np.random.default_rng(sseed), n, ratio)
        o = ol.OraclePnP(sc, seed)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        o.enable_trace()
        r = o.iterate(80)
        ints, fl = o.trace()
        assert np.array_equal(ints, g[f"s{k}_ints"])
        assert np.array_equal(fl.view(np.uint32), g[f"s{k}_poses"].view(np.uint32))
        assert [r["ok"], r["no_more"], r["n_inliers"]] == g[f"s{k}_result"].tolist()
    g = np.load(os.path.join(GOLD, "sim3_traces.npz"))
    for k in range(2):
        n1, ninl, seed, sseed = g[f"s{k}_meta"].tolist()
        pair = synth.make_sim3_pair(np.random.default_rng(sseed), n1, ninl, invalid_frac=0.1)
        o = ol.OracleSim3(pair, seed)
        o.set_ransac_parameters(0.99, 20, 300)
        o.enable_trace()
        r = o.iterate(60)
        ints, fl = o.trace()
        assert np.array_equal(ints, g[f"s{k}_ints"])
        assert np.array_equal(fl.view(np.uint32), g[f"s{k}_poses"].view(np.uint32))
