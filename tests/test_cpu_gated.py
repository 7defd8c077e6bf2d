"""The gated-event oracle replays (tests/events_oracle.py run_reloc_gated / run_loop_gated) on the
scenes of tests/test_gpu_gated.py: the reference's post-RANSAC gates (Tracking.cpp:1284-1331,
LoopClosing.cpp:296-325) produce every outcome the GPU test relies on — a rejected first winner
(wrong stereo matches / displaced keypoints), a handoff (10 <= nGood < 50), no match — so the device
comparison exercises the continue-after-rejection path.  Also: the gate scenes' generators build
solver inputs consistent with the KeyFrame views (synth.sim3_pair_from_kfs)."""
import numpy as np

import events_oracle as eo
import test_gpu_gated as tg


def test_reloc_gate_replay_outcomes():
    recs = [eo.run_reloc_gated(*ev) for ev in tg._reloc_events()]
    assert {r["status"] for r in recs} == {eo.GATE_NONE, eo.GATE_MATCH, eo.GATE_HANDOFF}
    assert recs[0]["rejected"] >= 1 and recs[0]["winner"] == 1 and recs[0]["status"] == eo.GATE_MATCH
    assert recs[5]["rejected"] >= 2
    for r in recs:
        if r["status"] == eo.GATE_MATCH:
            assert r["n_good"] >= 50
        elif r["status"] == eo.GATE_HANDOFF:
            assert 10 <= r["n_good"] < 50
        assert r["gates"] == r["rejected"] + (r["status"] != eo.GATE_NONE)


def test_loop_gate_replay_outcomes():
    evs = tg._loop_events()
    recs = [eo.run_loop_gated(*ev) for ev in evs]
    assert all(r["status"] == eo.GATE_MATCH and r["n_opt_inliers"] >= 20 for r in recs)
    assert recs[0]["rejected"] >= 1 and recs[0]["winner"] == 1
    assert sum(r["rejected"] for r in recs) >= 2
    for (kf1, cands, _), r in zip(evs, recs):
        kf2, m12, pair = cands[r["winner"]]
        m = r["matches"]
        # every kept match is a KF2 keypoint whose MapPoint exists; RANSAC inliers stay unless culled
        assert ((m == -1) | ((m >= 0) & (m < kf2.n))).all()
        assert (kf2.mp_state[m[m >= 0]] >= 1).all()
        assert pair.valid.sum() > 0 and pair.n1 == kf1.n
