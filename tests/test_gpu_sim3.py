"""GPU parity of the Sim3Solver path against the oracle restatement (bit-exact)."""
import numpy as np
import pytest

from gpu_common import assert_sim3_equal, ctx
import oracle_lib as ol
from rsc import synth

pytestmark = pytest.mark.gpu

LOOP = (0.99, 20, 300)  # LoopClosing.cpp:261


def make(pair, seed, params=LOOP):
    from rsc import engine
    g = engine.Sim3Solver(ctx(), pair, seed)
    g.set_ransac_parameters(*params)
    o = ol.OracleSim3(pair, seed)
    o.set_ransac_parameters(*params)
    return g, o


def test_constructor_prepared_arrays_bitexact():
    from rsc import engine
    rng = np.random.default_rng(1)
    pair = synth.make_sim3_pair(rng, 700, 300, invalid_frac=0.15)
    g = engine.Sim3Solver(ctx(), pair, 1)
    o = ol.OracleSim3(pair, 1)
    pg, po = g.prepared(), o.prepared()
    for k in ("X1c", "X2c", "P1im1", "P2im2", "maxerr1", "maxerr2", "indices"):
        assert np.array_equal(pg[k], po[k]), k


@pytest.mark.parametrize("n1,ninl,seed", [(300, 120, 1), (1000, 300, 2), (1000, 15, 3), (600, 400, 4)])
def test_iterate_parity(n1, ninl, seed):
    rng = np.random.default_rng(seed)
    pair = synth.make_sim3_pair(rng, n1, ninl, invalid_frac=0.05)
    g, o = make(pair, seed)
    assert_sim3_equal(g.iterate(300), o.iterate(300))
    assert g.state()["iterations"] == o.info()["iterations"]


@pytest.mark.parametrize("seed", [7, 8])
def test_round_robin_iterate5(seed):
    """LoopClosing::ComputeSim3 shape (LoopClosing.cpp:271-327): iterate(5) rounds, including
    calls after a success (best >= previous count needed, Q12)."""
    from rsc import engine
    rng = np.random.default_rng(seed)
    pairs_in = [synth.make_sim3_pair(rng, int(rng.integers(40, 800)), int(rng.integers(10, 300)))
                for _ in range(4)]
    pairs = [make(p, seed * 10 + i) for i, p in enumerate(pairs_in)]
    for rnd in range(15):
        outs = engine.sim3_iterate_many([p[0] for p in pairs], 5)
        for i, (g, o) in enumerate(pairs):
            assert_sim3_equal(outs[i], o.iterate(5), f"round {rnd} pair {i}")


def test_small_and_find():
    rng = np.random.default_rng(9)
    pair = synth.make_sim3_pair(rng, 15, 15)
    g, o = make(pair, 3)  # N < 20 -> bNoMore
    assert_sim3_equal(g.iterate(5), o.iterate(5))
    pair = synth.make_sim3_pair(rng, 200, 200, noise3d=0.0)
    g, o = make(pair, 4, (0.99, 6, 300))
    rg = g.find()
    ro = o.iterate(o.info()["max_iterations"])
    assert_sim3_equal(rg, ro)
    assert rg["ok"]
