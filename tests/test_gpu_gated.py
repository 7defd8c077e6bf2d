"""Gated events on the device: the reference's post-RANSAC acceptance test inside
the relocalization / loop-closure round-robin, bit-exact against an oracle replay of the same gate.

* rsc_reloc_events_gated — Tracking::Relocalization (Tracking.cpp:1239-1335): PoseOptimization on
  every success in the reference's order; nGood < 10 continues with the next candidate, >= 50 is a
  match, 10..49 hands off to SearchByProjection.  Candidates with wrong stereo matches on their slots
  (synth.make_reloc_gate_event `poisoned`) return a RANSAC pose that PoseOptimization rejects, so
  the event's first winner is rejected and the next success (same round or later) is the answer.
* rsc_loop_events_gated — LoopClosing::ComputeSim3 (LoopClosing.cpp:268-329): SearchBySim3(7.5) +
  OptimizeSim3(10) on every success in (round, candidate) order, accepted when nInliers >= 20;
  candidates whose keypoints disagree with their MapPoints (`poisoned`) pass the Sim3 RANSAC (which
  never reads keypoints) and fail OptimizeSim3.

Checked per event: status, winner, round, hypothesis, RANSAC inliers, the gate's outputs (nGood / pose
/ outlier flags / vbInliers; nfound / nInliers / g2oS12 / matches) and the number of rejected
successes — all equal to the oracle's sequential replay, floats bit for bit."""
import numpy as np
import pytest

from gpu_common import bits, ctx
import events_oracle as eo
from rsc import events as rev
from rsc import synth

pytestmark = pytest.mark.gpu


def _reloc_events():
    rng = np.random.default_rng(606)
    specs = [
        ([(500, 0.9), (400, 0.85)], (0,), 0.0),                           # first winner rejected, same round
        ([(300, 0.05), (450, 0.9), (250, 0.04), (220, 0.9)], (1,), 0.0),   # rejected, then a later candidate
        ([(50, 0.8)], (), 0.0),                                           # 10 <= nGood < 50: handoff
        ([(300, 0.05), (200, 0.05)], (), 0.0),                            # nothing: bMatch false
        ([(600, 0.75), (350, 0.6)], (), 0.5),                             # stereo edges on the winner
        ([(420, 0.9), (380, 0.88), (500, 0.85)], (0, 1), 0.3),            # two rejected candidates
    ]
    evs = []
    for cands, poisoned, stereo in specs:
        scenes, ur, bf = synth.make_reloc_gate_event(rng, 900, cands, poisoned, stereo)
        seeds = [int(x) for x in rng.integers(1, 1 << 30, len(scenes))]
        mono = stereo == 0.0 and not poisoned
        evs.append((scenes, seeds, None if mono else ur, bf))
    return evs


def test_reloc_events_gated_match_oracle():
    from rsc import engine
    evs = _reloc_events()
    eb = engine.EventBatch([[engine.PnPSolver(ctx(), sc, s) for sc, s in zip(scs, sds)] for scs, sds, _, _ in evs])
    eb.batch.reset(np.array([s for _, sds, _, _ in evs for s in sds], np.uint32))
    eb.batch.set_ransac_parameters(*rev.RELOC_PARAMS)
    res, outl, inl = eb.run_reloc_gated([(ur, bf) for _, _, ur, bf in evs])
    seen = set()
    for e, (scs, sds, ur, bf) in enumerate(evs):
        o = eo.run_reloc_gated(scs, sds, ur, bf)
        g = res[e]
        got = tuple(int(g[k]) for k in ("status", "winner", "round", "hypothesis", "n_inliers", "n_good", "rejected",
                                        "gates"))
        want = tuple(int(o[k]) for k in ("status", "winner", "round", "hypothesis", "n_inliers", "n_good", "rejected",
                                         "gates"))
        assert got == want, f"event {e}: {got} vs {want}"
        seen.add(o["status"])
        if o["status"] != eo.GATE_NONE:
            assert np.array_equal(bits(np.asarray(g["Tcw"])), bits(o["Tcw"])), f"event {e} Tcw"
            assert np.array_equal(outl[e], o["outlier"]), f"event {e} mvbOutlier"
            assert np.array_equal(inl[e], o["inliers"]), f"event {e} vbInliers"
    assert seen == {eo.GATE_NONE, eo.GATE_MATCH, eo.GATE_HANDOFF}
    assert int(res["rejected"][0]) >= 1 and int(res["status"][0]) == eo.GATE_MATCH and int(res["winner"][0]) == 1
    assert int(res["rejected"][5]) >= 2


def _loop_events():
    rng = np.random.default_rng(707)
    specs = [
        ([0.9, 0.85], (0,)),           # the round-0 winner rejected, the next candidate accepted
        ([0.02, 0.9], ()),             # a candidate whose RANSAC never succeeds, then a match
        ([0.02, 0.8, 0.9], (1,)),      # rejected in the middle, accepted after it
        ([0.85], ()),
    ]
    evs = []
    for goods, poisoned in specs:
        kf1, cands = synth.make_loop_gate_event(rng, goods, poisoned=poisoned)
        seeds = [int(x) for x in rng.integers(1, 1 << 30, len(cands))]
        evs.append((kf1, cands, seeds))
    return evs


def test_loop_events_gated_match_oracle():
    from rsc import engine
    evs = _loop_events()
    views, solvers, cand_in = [], [], []
    for kf1, cands, seeds in evs:
        v1 = engine.KFView(ctx(), kf1)
        views.append(v1)
        row_s, row_c = [], []
        for (kf2, m12, pair), s in zip(cands, seeds):
            v2 = engine.KFView(ctx(), kf2)
            views.append(v2)
            row_s.append(engine.Sim3Solver(ctx(), pair, s))
            row_c.append((v1, v2, m12))
        solvers.append(row_s)
        cand_in.append(row_c)
    eb = engine.EventBatch(solvers)
    eb.batch.reset(np.array([s for _, _, sds in evs for s in sds], np.uint32))
    eb.batch.set_ransac_parameters(*rev.LOOP_PARAMS)
    res, matches = eb.run_loop_gated(cand_in)
    n_rej = 0
    for e, (kf1, cands, seeds) in enumerate(evs):
        o = eo.run_loop_gated(kf1, cands, seeds)
        g = res[e]
        keys = ("status", "winner", "round", "hypothesis", "n_inliers", "n_found", "n_opt_inliers", "rejected")
        got = tuple(int(g[k]) for k in keys)
        want = tuple(int(o[k]) for k in keys)
        assert got == want, f"event {e}: {got} vs {want}"
        n_rej += want[-1]
        if o["status"] == eo.GATE_MATCH:
            assert np.array_equal(np.asarray(g["S"]).view(np.uint64), np.asarray(o["S"]).view(np.uint64)), f"event {e} S"
            assert np.array_equal(matches[e], o["matches"]), f"event {e} matches"
    assert (res["status"] == eo.GATE_MATCH).all()
    assert int(res["rejected"][0]) >= 1 and int(res["winner"][0]) == 1
    assert n_rej >= 2
