"""GPU parity of the PnPsolver path (librsc.so on cuda:0) against the oracle restatement.

Bar: bit-exact — identical sample indices, inlier counts and masks, and bitwise-identical
float poses (the north-star tolerance is 1e-4; the shared arithmetic contract makes it exact).
"""
import numpy as np
import pytest

from gpu_common import assert_pnp_equal, ctx, bits
import oracle_lib as ol
from rsc import synth

pytestmark = pytest.mark.gpu

RELOC = (0.99, 10, 300, 4, 0.5, 5.991)  # Tracking.cpp:1226


def make(scene, seed, params=RELOC):
    from rsc import engine
    g = engine.PnPSolver(ctx(), scene, seed)
    g.set_ransac_parameters(*params)
    o = ol.OraclePnP(scene, seed)
    o.set_ransac_parameters(*params)
    return g, o


def test_rand_stream_matches_libc():
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    for seed in (0, 1, 42, 1234, 987654321):
        libc.srand(seed)
        ref = np.array([libc.rand() for _ in range(20000)], np.int32)
        assert np.array_equal(ctx().rand_stream(seed, 20000), ref)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_hypotheses_bitexact(seed):
    """Per-hypothesis samples / poses / counts of one long iterate() (exhaustive: no refine)."""
    rng = np.random.default_rng(100 + seed)
    sc = synth.make_pnp_scene(rng, 400, 0.4)
    g, o = make(sc, seed)
    o.enable_trace()
    rg = g.iterate(300)
    ro = o.iterate(300)
    assert_pnp_equal(rg, ro)
    ints, fl = o.trace()
    samp = g.last_samples()
    assert samp.shape[0] == 300 and len(ints) == 300
    assert np.array_equal(samp[:, :4], ints[:, :4])
    assert g.state()["iterations"] == o.info()["iterations"] == 300


@pytest.mark.parametrize("n,ratio,seed", [(300, 0.6, 1), (500, 0.7, 5), (1200, 0.6, 9), (2000, 0.65, 4)])
def test_parity_mode_refine(n, ratio, seed):
    """Reachable minInliers: best update + Refine + early exit (Q8) must match exactly."""
    rng = np.random.default_rng(n + seed)
    sc = synth.make_pnp_scene(rng, n, ratio, n_points=n + 37)
    g, o = make(sc, seed)
    rg = g.iterate(300)
    ro = o.iterate(300)
    assert_pnp_equal(rg, ro)
    sg, so = g.state(), o.info()
    assert sg["iterations"] == so["iterations"] and sg["best_inliers"] == so["best_inliers"]
    assert sg["max_rows"] == so["max_rows"]


@pytest.mark.parametrize("seed", [11, 12])
def test_round_robin_iterate5(seed):
    """Relocalization driver shape: repeated iterate(5) calls on several candidates (Tracking.cpp:1239-1262),
    including hypotheses evaluated after a Refine (stale EPnP rows, Q6)."""
    from rsc import engine
    rng = np.random.default_rng(seed)
    scenes = [synth.make_pnp_scene(rng, int(rng.integers(60, 600)), float(rng.uniform(0.3, 0.8))) for _ in range(5)]
    pairs = [make(sc, seed * 10 + i) for i, sc in enumerate(scenes)]
    for rnd in range(10):
        outs_g = engine.pnp_iterate_many([p[0] for p in pairs], 5)
        for i, (g, o) in enumerate(pairs):
            ro = o.iterate(5)
            assert_pnp_equal(outs_g[i], ro, f"round {rnd} cand {i}")
            assert g.state()["max_rows"] == o.info()["max_rows"]


def test_find_and_small_problems():
    from rsc import engine
    rng = np.random.default_rng(7)
    # N < minInliers -> bNoMore immediately (PnPsolver.cpp:110-114)
    sc = synth.make_pnp_scene(rng, 8, 1.0)
    g, o = make(sc, 3, (0.99, 10, 300, 4, 0.5, 5.991))
    assert_pnp_equal(g.iterate(5), o.iterate(5))
    # minimal N with all inliers, find()
    sc = synth.make_pnp_scene(rng, 30, 1.0, noise=False)
    g, o = make(sc, 4)
    rg = g.find()
    bNoMore = None
    ro = o.iterate(o.info()["max_iterations"])
    assert_pnp_equal(rg, ro)
    assert rg["ok"]
    assert np.abs(rg["T"][:3, :3] - sc.R_true).max() < 1e-4
    assert np.abs(rg["T"][:3, 3] - sc.t_true).max() < 1e-4


@pytest.mark.parametrize("ms", [5, 6])
def test_min_set_variants(ms):
    rng = np.random.default_rng(ms)
    sc = synth.make_pnp_scene(rng, 500, 0.6)
    params = (0.99, 10, 300, ms, 0.5, 5.991)
    g, o = make(sc, 21, params)
    assert_pnp_equal(g.iterate(40), o.iterate(40))


def test_iterate_many_equals_sequential():
    from rsc import engine
    rng = np.random.default_rng(33)
    scenes = [synth.make_pnp_scene(rng, 800, 0.4) for _ in range(6)]
    a = [make(sc, 40 + i)[0] for i, sc in enumerate(scenes)]
    b = [make(sc, 40 + i)[0] for i, sc in enumerate(scenes)]
    many = engine.pnp_iterate_many(a, 120)
    for i in range(6):
        one = b[i].iterate(120)
        assert_pnp_equal(many[i], one, f"cand {i}")


@pytest.mark.parametrize("case", [1, 4, 17, 43, 66, 72, 74, 83, 95, 98])
def test_refine_failure_respeculation(case):
    """Failed Refine -> stale EPnP rows -> later hypotheses recomputed on the GPU (Q6, Q8)."""
    from gpu_common import refine_fail_scene
    sc, seed = refine_fail_scene(case)
    g, o = make(sc, seed)
    for rnd in range(20):
        assert_pnp_equal(g.iterate(5), o.iterate(5), f"round {rnd}")
        assert g.state()["max_rows"] == o.info()["max_rows"]


def test_min_sets_bitexact():
    """The hypothesis kernels for every supported sample size against the oracle (samples, counts,
    poses), min_set 4..6."""
    from rsc import engine
    rng = np.random.default_rng(7)
    c = engine.Context(0)
    for ms in (4, 5, 6):
        sc = synth.make_pnp_scene(rng, 700, 0.5)
        params = (0.99, 10, 300, ms, 0.5, 5.991)
        g = engine.PnPSolver(c, sc, 100 + ms)
        g.set_ransac_parameters(*params)
        o = ol.OraclePnP(sc, 100 + ms)
        o.set_ransac_parameters(*params)
        for k in range(3):
            assert_pnp_equal(g.iterate(37), o.iterate(37), f"ms={ms} call {k}")


def test_batch_iterate_raw_matches_dicts():
    from rsc import engine
    rng = np.random.default_rng(8)
    scenes = [synth.make_pnp_scene(rng, 600, 0.4) for _ in range(5)]
    a = engine.SolverBatch([make(sc, 60 + i)[0] for i, sc in enumerate(scenes)])
    b = engine.SolverBatch([make(sc, 60 + i)[0] for i, sc in enumerate(scenes)])
    raw = a.iterate_raw(90)
    outs = b.iterate(90)
    for i, o in enumerate(outs):
        assert raw["ok"][i] == o["ok"] and raw["n_inliers"][i] == o["n_inliers"]
        assert raw["iterations"][i] == o["iterations"] and raw["no_more"][i] == o["no_more"]
        if o["ok"]:
            assert bits(raw["T"][i].reshape(4, 4)).tolist() == bits(o["T"]).tolist()


@pytest.mark.parametrize("mode", ["fused", "large_round", "unfused"])
def test_iterate_many_mixed_n_refines(mode, monkeypatch):
    """Solvers of very different N whose Refines land in the same launch: the device-side
    selection + Refine (rounds <= 4,096 hypotheses, `fused`), the two-launch form for a larger round
    (`large_round`: 16 solvers x 300) and with RSC_FUSED_REFINE=0 (`unfused`).  Every solver's
    result, mask and EPnP row count must equal its own sequential oracle run: a Refine writing past a
    shorter solver's bitsets, or one the host did not ask for, shows up as a neighbour's mask."""
    from rsc import engine
    if mode == "unfused":
        monkeypatch.setenv("RSC_FUSED_REFINE", "0")
    c = engine.Context(0)
    sizes = [100, 3000, 240, 1800, 64, 2500, 130, 900]
    if mode == "large_round":
        sizes = sizes * 2
    rng = np.random.default_rng({"fused": 5, "large_round": 6, "unfused": 7}[mode])
    scenes = [synth.make_pnp_scene(rng, n, float(rng.uniform(0.55, 0.8)), n_points=n + 11) for n in sizes]
    gs, os_ = [], []
    for i, sc in enumerate(scenes):
        g = engine.PnPSolver(c, sc, 500 + i)
        g.set_ransac_parameters(*RELOC)
        o = ol.OraclePnP(sc, 500 + i)
        o.set_ransac_parameters(*RELOC)
        gs.append(g)
        os_.append(o)
    its = 300 if mode == "large_round" else 5
    n_ok = 0
    for rnd in range(4):
        outs = engine.pnp_iterate_many(gs, its)
        for i, (g, o) in enumerate(zip(gs, os_)):
            ro = o.iterate(its)
            assert_pnp_equal(outs[i], ro, f"{mode} round {rnd} solver {i} (N={sizes[i]})")
            assert g.state()["max_rows"] == o.info()["max_rows"]
            n_ok += ro["ok"]
    assert n_ok >= len(sizes) // 2
