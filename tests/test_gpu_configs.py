"""GPU parity at the BASELINE.json configurations' bench shapes (the exact inputs bench.py times,
rsc/workloads.py), bit-exact against the oracle restatement:

* config 2 — 64 candidates x 2000 correspondences, iterate(300), exhaustive batch (every
  hypothesis' sample, inlier count and float pose) and a parity-mode batch with Refine;
* config 3 — 32 KeyFrame pairs x 1000 matches, iterate(300), exhaustive and parity mode;
* config 4 — 32 candidates x 4096 correspondences of MLPnP (the per-GPU share of 128 over 4 GPUs):
  the 16-points-per-thread scan and the 4096-row solve slab;
* config 5 — the full 150 relocalization + 20 loop-closure event stream.
"""
import numpy as np
import pytest

from gpu_common import assert_pnp_equal, assert_sim3_equal, bits, ctx
import events_oracle as eo
import oracle_lib as ol
from rsc import events as rev
from rsc import workloads as wl

pytestmark = pytest.mark.gpu


def _pnp_batch(scenes, seeds, params):
    from rsc import engine
    gs = [engine.PnPSolver(ctx(), sc, int(s)) for sc, s in zip(scenes, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*params)
    return gs, b


def test_config2_exhaustive_batch_every_hypothesis():
    """64 x 2000 x iterate(300), 19,200 hypotheses in one rsc_pnp_iterate_many (bench step 0)."""
    scenes = wl.config2_scenes()
    seeds = wl.config2_seeds(0)
    gs, b = _pnp_batch(scenes, seeds, wl.RELOC)
    outs = b.iterate(300, with_masks=True)
    hyp = [g.last_hypotheses(400) for g in gs]
    smp = [g.last_samples(400) for g in gs]
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OraclePnP(sc, int(s))
        o.set_ransac_parameters(*wl.RELOC)
        o.enable_trace()
        ro = o.iterate(300)
        assert_pnp_equal(outs[i], ro, f"cand {i}")
        assert not ro["ok"] and ro["iterations"] == 300 and outs[i]["iterations"] == 300
        ints, fl = o.trace()
        cnt, pos = hyp[i]
        assert len(cnt) == len(ints) == 300
        assert np.array_equal(smp[i][:, :4], ints[:, :4]), f"cand {i} samples"
        assert np.array_equal(cnt, ints[:, 8]), f"cand {i} counts"
        assert np.array_equal(bits(pos), bits(fl)), f"cand {i} poses"


def test_config2_parity_batch_with_refine():
    """Same shape, 60 % inliers: qualifying hypotheses, Refine and early exit for every candidate."""
    scenes = wl.config2_scenes(ratio=0.6, seed=20300)
    seeds = wl.config2_seeds(0)
    gs, b = _pnp_batch(scenes, seeds, wl.RELOC)
    outs = b.iterate(300, with_masks=True)
    n_ok = 0
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OraclePnP(sc, int(s))
        o.set_ransac_parameters(*wl.RELOC)
        ro = o.iterate(300)
        assert_pnp_equal(outs[i], ro, f"cand {i}")
        assert outs[i]["iterations"] == ro["iterations"]
        assert gs[i].state()["max_rows"] == o.info()["max_rows"]
        n_ok += ro["ok"]
    assert 32 <= n_ok < 64  # both outcomes (Refine success, budget exhausted) exercised


def _sim3_batch(pairs, seeds):
    from rsc import engine
    gs = [engine.Sim3Solver(ctx(), p, int(s)) for p, s in zip(pairs, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.LOOP)
    return gs, b


def test_config3_exhaustive_batch_every_hypothesis():
    pairs = wl.config3_pairs()
    seeds = wl.step_seeds(0, len(pairs))
    gs, b = _sim3_batch(pairs, seeds)
    outs = b.iterate(300, with_masks=True)
    hyp = [g.last_hypotheses(400) for g in gs]
    for i, (p, s) in enumerate(zip(pairs, seeds)):
        o = ol.OracleSim3(p, int(s))
        o.set_ransac_parameters(*wl.LOOP)
        o.enable_trace()
        ro = o.iterate(300)
        assert_sim3_equal(outs[i], ro, f"pair {i}")
        assert not ro["ok"] and outs[i]["iterations"] == ro["iterations"] == 300
        ints, fl = o.trace()
        cnt, pos = hyp[i]
        assert len(cnt) == len(ints) == 300
        assert np.array_equal(cnt, ints[:, 3]), f"pair {i} counts"
        assert np.array_equal(bits(pos), bits(fl)), f"pair {i} poses"


def test_config3_parity_batch_first_success():
    pairs = wl.config3_pairs(n_inliers=300, seed=177)
    seeds = wl.step_seeds(0, len(pairs))
    gs, b = _sim3_batch(pairs, seeds)
    outs = b.iterate(300, with_masks=True)
    n_ok = 0
    for i, (p, s) in enumerate(zip(pairs, seeds)):
        o = ol.OracleSim3(p, int(s))
        o.set_ransac_parameters(*wl.LOOP)
        ro = o.iterate(300)
        assert_sim3_equal(outs[i], ro, f"pair {i}")
        assert outs[i]["iterations"] == ro["iterations"]
        n_ok += ro["ok"]
    assert n_ok >= 24


@pytest.mark.parametrize("candidates", [32, 128])
def test_config4_mlpnp_4096_batch_every_hypothesis(candidates):
    """MLPnP at N = 4096: mlpnp_scan_kernel<16> and the 4096-row LDS slab of the solve, at the per-GPU
    share of 4 GPUs (32 candidates) and at the bench's single-GPU launch shape (all 128 candidates of
    config 4 in one launch: 38,400 hypotheses, bench.py's mlpnp section at N = 1)."""
    from rsc import engine
    scenes = wl.config4_scenes(candidates=candidates)
    seeds = wl.step_seeds(0, len(scenes))
    gs = [engine.MLPnPSolver(ctx(), sc, int(s)) for sc, s in zip(scenes, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.MLPNP)
    outs = b.iterate(300, with_masks=True)
    hyp = [g.last_hypotheses(400) for g in gs]
    cnts = [g.last_counts(400) for g in gs]
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OracleMLPnP(sc, int(s))
        o.set_ransac_parameters(*wl.MLPNP)
        o.enable_trace()
        ro = o.iterate(300)
        assert outs[i]["ok"] == ro["ok"] and outs[i]["n_inliers"] == ro["n_inliers"], f"cand {i}"
        assert outs[i]["iterations"] == ro["iterations"] == 300
        assert np.array_equal(bits(outs[i]["T"]), bits(ro["T"])), f"cand {i} T"
        ints, dbl = o.trace()
        smp, pos = hyp[i]
        assert len(smp) == len(ints) == 300
        assert np.array_equal(smp[:, :6], ints[:, :6]), f"cand {i} samples"
        assert np.array_equal(cnts[i], ints[:, 8]), f"cand {i} counts"
        assert np.array_equal(pos.view(np.uint64), dbl.view(np.uint64)), f"cand {i} poses"


def test_config4_mlpnp_4096_covariances_every_hypothesis():
    """Config 4 "with bearing-vector covariances" at the per-GPU share (32 candidates x 4096, the
    bench's covariance section): computePose's covMats branch (MLPnPsolver.cpp:375-388, 483-484,
    694-695; mlpnp_quad_kernel<6, MlIndexedCov>) — samples, counts, double poses bit-exact against the
    oracle's restatement (parity with the reference unpinned: it never reaches this branch, Q15)."""
    from rsc import engine
    scenes = wl.config4_scenes()
    seeds = wl.step_seeds(0, len(scenes))
    gs = [engine.MLPnPSolver(ctx(), sc, int(s)) for sc, s in zip(scenes, seeds)]
    for g, sc in zip(gs, scenes):
        g.set_covariances(wl.config4_covariances(sc))
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.MLPNP)
    outs = b.iterate(300, with_masks=True)
    hyp = [g.last_hypotheses(400) for g in gs]
    cnts = [g.last_counts(400) for g in gs]
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OracleMLPnP(sc, int(s))
        o.set_covariances(wl.config4_covariances(sc))
        o.set_ransac_parameters(*wl.MLPNP)
        o.enable_trace()
        ro = o.iterate(300)
        assert outs[i]["ok"] == ro["ok"] and outs[i]["n_inliers"] == ro["n_inliers"], f"cand {i}"
        assert outs[i]["iterations"] == ro["iterations"] == 300
        assert np.array_equal(bits(outs[i]["T"]), bits(ro["T"])), f"cand {i} T"
        ints, dbl = o.trace()
        smp, pos = hyp[i]
        assert len(smp) == len(ints) == 300
        assert np.array_equal(smp[:, :6], ints[:, :6]), f"cand {i} samples"
        assert np.array_equal(cnts[i], ints[:, 8]), f"cand {i} counts"
        assert np.array_equal(pos.view(np.uint64), dbl.view(np.uint64)), f"cand {i} poses"


def test_config4_mlpnp_4096_parity_mode_refine():
    """Config 4's shape (32 candidates x 4096, the per-GPU share) in parity mode: 60 % inliers, so
    hypotheses reach minInliers (floor(0.5 N) = 2048) and MLPnP's Refine runs at N = 4096
    (MLPnPsolver.cpp:257-318: its computePose result is discarded and the current hypothesis
    re-counted, Q15) and iterate returns at the first success.  Outcome, iterations, pose and
    vbInliers bit-exact against the oracle; most candidates succeed."""
    from rsc import engine
    scenes = wl.config4_scenes(ratio=0.6, seed=79)
    seeds = wl.step_seeds(0, len(scenes))
    gs = [engine.MLPnPSolver(ctx(), sc, int(s)) for sc, s in zip(scenes, seeds)]
    b = engine.SolverBatch(gs)
    b.set_ransac_parameters(*wl.MLPNP)
    outs = b.iterate(300, with_masks=True)
    n_ok = 0
    for i, (sc, s) in enumerate(zip(scenes, seeds)):
        o = ol.OracleMLPnP(sc, int(s))
        o.set_ransac_parameters(*wl.MLPNP)
        ro = o.iterate(300)
        g = outs[i]
        assert (g["ok"], g["no_more"], g["n_inliers"], g["iterations"]) == \
            (ro["ok"], ro["no_more"], ro["n_inliers"], ro["iterations"]), f"cand {i}"
        assert np.array_equal(bits(g["T"]), bits(ro["T"])), f"cand {i} T"
        assert np.array_equal(g["inliers"], ro["inliers"]), f"cand {i} inliers"
        n_ok += ro["ok"]
    assert n_ok >= 20


def test_config5_full_event_stream():
    """The bench's 150 + 20 event stream (rsc.events.make_event_stream() defaults) through
    rsc_reloc_events / rsc_loop_events against the sequential round-robin replay."""
    from test_gpu_events import _gpu_records
    evs = rev.make_event_stream()
    assert sum(ev.kind == "reloc" for ev in evs) == 150 and sum(ev.kind == "loop" for ev in evs) == 20
    g = _gpu_records(evs)
    o = eo.run_events(evs)
    assert np.array_equal(g[:, :5], o[:, :5])
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32))
