"""GPU parity of ORBmatcher::SearchBySim3 (ORBmatcher.cpp:948-1170) through the C ABI
(rsc_search_by_sim3_many) against the oracle: new-match vectors and counts bit-exact on the golden
fixtures, batched loop-closure-shaped pairs (a shared current KeyFrame), and edge cases."""
import os

import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import ctx
from rsc import engine, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check(problems, th=7.5):
    outs, nf = engine.search_by_sim3_many(ctx(), problems, th)
    for (kf1, kf2, R12, t12, m12), o, n in zip(problems, outs, nf):
        on, oo = ol.search_by_sim3(kf1, kf2, R12, t12, m12, th)
        assert n == on and np.array_equal(o, oo)
    return nf


def test_golden_fixtures():
    from test_cpu_sim3match import synth as _s  # noqa: F401
    g = np.load(os.path.join(ROOT, "tests", "golden", "sim3match_traces.npz"))
    probs = []
    for k in range(int(g["cases"])):
        kfs = []
        for side in ("A", "B"):
            f = {x: g[f"c{k}_{side}_{x}"] for x in ("kp", "octave", "desc", "cell_begin", "cell_feat", "Rcw", "tcw",
                                                    "mp_state", "mp_pos", "mp_dmax", "mp_dmin", "mp_desc")}
            kfs.append(synth.Sim3KF(len(f["kp"]), mp_id=np.zeros(len(f["kp"]), np.int64), **f))
        probs.append((kfs[0], kfs[1], g[f"c{k}_R12"], g[f"c{k}_t12"], g[f"c{k}_m12"]))
    outs, nf = engine.search_by_sim3_many(ctx(), probs)
    for k in range(int(g["cases"])):
        assert nf[k] == int(g[f"c{k}_n"]) and np.array_equal(outs[k], g[f"c{k}_out"]), k


def test_batched_pairs_parity():
    rng = np.random.default_rng(201)
    probs = [synth.make_sim3match_pair(rng, int(rng.integers(200, 1200)), int(rng.integers(0, 400)),
                                       float(rng.uniform(0, 0.6))) for _ in range(12)]
    nf = check(probs)
    assert nf.max() > 20


def test_shared_current_keyframe():
    """LoopClosing shape: the current KeyFrame against several candidates (one upload)."""
    rng = np.random.default_rng(202)
    base = synth.make_sim3match_pair(rng, 800, 200, 0.3)
    probs = [base]
    for _ in range(5):
        other = synth.make_sim3match_pair(rng, 800, 200, 0.3)
        probs.append((base[0], other[1], other[2], other[3], np.full(base[0].n, -1, np.int32)))
    check(probs)


@pytest.mark.parametrize("th", [3.0, 7.5, 15.0])
def test_thresholds(th):
    rng = np.random.default_rng(203)
    check([synth.make_sim3match_pair(rng, 600, 150, 0.2) for _ in range(3)], th)


def test_edge_cases():
    rng = np.random.default_rng(204)
    kf1, kf2, R12, t12, m12 = synth.make_sim3match_pair(rng, 300, 50, 0.0)
    all_matched = np.where(kf1.mp_state > 0, -2, -1).astype(np.int32)
    far = (R12, (t12 + np.float32(100.0)).astype(np.float32))  # everything projects out of the image
    empty = synth.Sim3KF(0, np.zeros((0, 2), np.float32), np.zeros(0, np.int32), np.zeros((0, 32), np.uint8),
                         np.zeros(64 * 48 + 1, np.int32), np.zeros(0, np.int32), kf2.Rcw, kf2.tcw,
                         np.zeros(0, np.uint8), np.zeros((0, 3), np.float32), np.zeros(0, np.float32),
                         np.zeros(0, np.float32), np.zeros((0, 32), np.uint8), np.zeros(0, np.int64))
    nf = check([(kf1, kf2, R12, t12, all_matched), (kf1, kf2, far[0], far[1], m12), (kf1, empty, R12, t12, m12)])
    assert (nf == 0).all()
