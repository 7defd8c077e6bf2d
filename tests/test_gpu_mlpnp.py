"""GPU parity of the MLPnPsolver path (config 4) against the oracle restatement — bit-exact
per-hypothesis double poses, counts, masks and iterate() results.  (Parity with the reference
itself is unpinned: the reference never compiles MLPnPsolver.cpp)"""
import numpy as np
import pytest

from gpu_common import ctx, bits
import oracle_lib as ol
from rsc import synth

pytestmark = pytest.mark.gpu


def make(scene, seed, params):
    from rsc import engine
    g = engine.MLPnPSolver(ctx(), scene, seed)
    g.set_ransac_parameters(*params)
    o = ol.OracleMLPnP(scene, seed)
    o.set_ransac_parameters(*params)
    return g, o


def assert_ml_equal(g, o, where):
    assert g["ok"] == o["ok"], f"{where} ok"
    assert g["no_more"] == o["no_more"], f"{where} no_more"
    assert g["n_inliers"] == o["n_inliers"], f"{where} n_inliers {g['n_inliers']} vs {o['n_inliers']}"
    assert g["iterations"] == o["iterations"], f"{where} iterations"
    assert np.array_equal(bits(g["T"]), bits(o["T"])), f"{where} T\n{g['T']}\n{o['T']}"
    if o["ok"]:
        assert np.array_equal(g["inliers"], o["inliers"]), f"{where} inliers"


@pytest.mark.parametrize("ns", [6, 7, 8])
def test_hypotheses_bitexact(ns):
    rng = np.random.default_rng(40 + ns)
    sc = synth.make_pnp_scene(rng, 900, 0.4)
    params = (0.99, 10, 300, ns, 0.5, 5.991)
    g, o = make(sc, 11, params)
    o.enable_trace()
    rg = g.iterate(70)
    ro = o.iterate(70)
    assert_ml_equal(rg, ro, "exhaustive")
    smp, pos = g.last_hypotheses()
    ints, dbl = o.trace()
    assert len(smp) == len(ints) == 70
    assert np.array_equal(smp[:, :ns], ints[:, :ns])
    assert np.array_equal(pos.view(np.uint64), dbl.view(np.uint64))


@pytest.mark.parametrize("ratio,seed", [(0.55, 1), (0.7, 2), (0.5, 3), (0.45, 4)])
def test_iterate_round_robin(ratio, seed):
    rng = np.random.default_rng(100 + seed)
    sc = synth.make_pnp_scene(rng, 600, ratio, n_points=700)
    g, o = make(sc, seed, (0.99, 10, 300, 6, 0.5, 5.991))
    for k in range(8):
        assert_ml_equal(g.iterate(5), o.iterate(5), f"call {k}")


def test_iterate_many_equals_sequential_and_batch():
    from rsc import engine
    rng = np.random.default_rng(77)
    scenes = [synth.make_pnp_scene(rng, 500, r) for r in (0.4, 0.6, 0.5, 0.65, 0.45)]
    params = (0.99, 10, 300, 6, 0.5, 5.991)
    pairs = [make(sc, 20 + i, params) for i, sc in enumerate(scenes)]
    many = engine.mlpnp_iterate_many([p[0] for p in pairs], 40)
    for i, (g, o) in enumerate(pairs):
        assert_ml_equal(many[i], o.iterate(40), f"cand {i}")
    b = engine.SolverBatch([make(sc, 20 + i, params)[0] for i, sc in enumerate(scenes)])
    raw = b.iterate_raw(40)
    for i in range(len(scenes)):
        assert raw["n_inliers"][i] == many[i]["n_inliers"] and raw["ok"][i] == many[i]["ok"]


def test_min_set_out_of_range_is_rejected():
    from rsc import engine
    rng = np.random.default_rng(5)
    g = engine.MLPnPSolver(ctx(), synth.make_pnp_scene(rng, 100, 0.5), 1)
    with pytest.raises(RuntimeError):
        g.set_ransac_parameters(0.99, 10, 300, 5, 0.5, 5.991)


@pytest.mark.parametrize("ns", [6, 8])
def test_covariance_branch_bitexact(ns):
    """computePose's covMats branch (config 4 'with bearing-vector covariances'; never reached by
    the reference's own calls, parity against the reference unpinned): per-hypothesis double poses
    and iterate() results bit-exact against the oracle's restatement, and switching the
    covariances off restores the reference path."""
    from test_cpu_mlpnp import bearing_covariances
    rng = np.random.default_rng(60 + ns)
    sc = synth.make_pnp_scene(rng, 700, 0.4)
    params = (0.99, 10, 300, ns, 0.5, 5.991)
    g, o = make(sc, 13, params)
    cov = bearing_covariances(sc)
    g.set_covariances(cov)
    o.set_covariances(cov)
    o.enable_trace()
    assert_ml_equal(g.iterate(60), o.iterate(60), "cov exhaustive")
    smp, pos = g.last_hypotheses()
    ints, dbl = o.trace()
    assert len(smp) == len(ints) == 60
    assert np.array_equal(smp[:, :ns], ints[:, :ns])
    assert np.array_equal(pos.view(np.uint64), dbl.view(np.uint64))
    sc2 = synth.make_pnp_scene(rng, 600, 0.65)
    g2, o2 = make(sc2, 14, params)
    cov2 = bearing_covariances(sc2)
    g2.set_covariances(cov2)
    o2.set_covariances(cov2)
    for k in range(4):
        assert_ml_equal(g2.iterate(5), o2.iterate(5), f"cov call {k}")
    g2.set_covariances(None)
    o2.set_covariances(None)
    for k in range(3):
        assert_ml_equal(g2.iterate(5), o2.iterate(5), f"no-cov call {k}")
