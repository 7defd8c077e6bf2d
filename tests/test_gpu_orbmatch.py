"""GPU parity of ORBmatcher::SearchByBoW (ORBmatcher.cpp:110-240 Frame overload, :354-488 KeyFrame
overload) through the C ABI (rsc_bow_create / rsc_search_by_bow_*_many) against the oracle: match
vectors and counts bit-exact, on the golden fixtures, relocalization- and loop-closure-shaped
batches, and the edge cases (empty views, no common nodes, nodes wider than a wavefront, maximum
view size, descriptor ties, invalid map points, refreshed validity)."""
import os

import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import ctx
from rsc import engine, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check_batch(shared, others, frame_overload, nnratio=0.75, check=True):
    c = ctx()
    gs = engine.BowView(c, shared)
    go = [engine.BowView(c, o) for o in others]
    g_out, g_nm = engine.BowSearch(c, gs, go, frame_overload, nnratio, check).run()
    o_out, o_nm = ol.search_by_bow_many(frame_overload, [ol.OracleBow(o) for o in others], ol.OracleBow(shared),
                                        nnratio, check)
    assert np.array_equal(g_nm, o_nm), (g_nm, o_nm)
    assert np.array_equal(g_out, o_out)
    return g_out, g_nm


def test_golden_fixtures():
    from test_cpu_orbmatch import golden_views
    g = np.load(os.path.join(ROOT, "tests", "golden", "bow_traces.npz"))
    c = ctx()
    for k in range(int(g["cases"])):
        A, B, fv, ratio, check = golden_views(g, k)
        ga, gb = engine.BowView(c, A), engine.BowView(c, B)
        if fv:
            out, nm = engine.BowSearch(c, gb, [ga], True, ratio, check).run()
        else:
            out, nm = engine.BowSearch(c, ga, [gb], False, ratio, check).run()
        assert int(nm[0]) == int(g[f"c{k}_n"]), k
        assert np.array_equal(out[0], g[f"c{k}_out"]), k


def test_relocalization_batch():
    """Tracking::Relocalization shape: 64 candidate KeyFrames x the current Frame (2000 features)."""
    rng = np.random.default_rng(101)
    F = synth.make_bow_view(rng, 2000)
    kfs = [synth.make_bow_related(rng, F, int(rng.integers(800, 2000)), float(rng.uniform(0.1, 0.7)),
                                  float(rng.uniform(0, 360)), mean_flips=float(rng.uniform(8, 30)))
           for _ in range(64)]
    _, nm = check_batch(F, kfs, True)
    assert nm.max() > 100


def test_loop_closure_batch():
    """LoopClosing::ComputeSim3 shape: the current KeyFrame x 32 loop candidates."""
    rng = np.random.default_rng(102)
    K = synth.make_bow_view(rng, 1500, valid_frac=0.8)
    cands = [synth.make_bow_related(rng, K, int(rng.integers(300, 1500)), float(rng.uniform(0.05, 0.6)),
                                    float(rng.uniform(0, 360)), valid_frac=0.8) for _ in range(32)]
    _, nm = check_batch(K, cands, False)
    assert nm.max() > 50


@pytest.mark.parametrize("nnratio", [0.6, 0.9, 1.0])
@pytest.mark.parametrize("check", [True, False])
def test_ratio_and_orientation_flags(nnratio, check):
    rng = np.random.default_rng(103)
    F = synth.make_bow_view(rng, 700)
    kfs = [synth.make_bow_related(rng, F, 600, 0.5, float(rng.uniform(0, 360))) for _ in range(6)]
    check_batch(F, kfs, True, nnratio, check)
    check_batch(F, kfs, False, nnratio, check)


def test_wide_nodes_and_maximum_size():
    """Nodes holding hundreds to thousands of features (several 64-lane chunks per node) and the
    8192-keypoint limit."""
    rng = np.random.default_rng(104)
    F = synth.make_bow_view(rng, 8192, skew=3.0)  # one node holds most features
    assert np.diff(F.node_begin).max() > 4096
    kfs = [synth.make_bow_related(rng, F, 8192, 0.5, 10.0, skew=3.0),
           synth.make_bow_related(rng, F, 3000, 0.3, 200.0, skew=2.0)]
    check_batch(F, kfs, True)
    check_batch(F, kfs, False)


def test_ties_and_duplicate_descriptors():
    rng = np.random.default_rng(105)
    F = synth.make_bow_view(rng, 500, skew=1.5)
    F.desc[:] = F.desc[rng.integers(0, 20, 500)]  # only 20 distinct descriptors: many equal distances
    kfs = [synth.make_bow_related(rng, F, 400, 0.7, 5.0, mean_flips=3.0, skew=1.5) for _ in range(4)]
    for k in kfs:
        k.desc[::3] = F.desc[rng.integers(0, 500, len(k.desc[::3]))]
    check_batch(F, kfs, True, 1.0)
    check_batch(F, kfs, False, 1.0)


def test_empty_and_disjoint_views():
    rng = np.random.default_rng(106)
    F = synth.make_bow_view(rng, 300)
    empty = synth.BowFeatures(0, np.zeros((0, 32), np.uint8), np.zeros(0, np.float32), np.zeros(0, np.uint8),
                              np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.uint32))
    disjoint = synth.make_bow_view(rng, 200, nodes=np.full(200, 5000, np.uint32))
    all_invalid = synth.make_bow_related(rng, F, 300, 0.8, 0.0, valid_frac=0.0)
    check_batch(F, [empty, disjoint, all_invalid, F], True)
    check_batch(F, [empty, disjoint, all_invalid, F], False)
    c = ctx()
    ge = engine.BowView(c, empty)
    out, nm = engine.BowSearch(c, ge, [engine.BowView(c, F)], True).run()
    assert out.shape == (1, 0) and nm[0] == 0


def test_set_valid_refresh():
    rng = np.random.default_rng(107)
    F = synth.make_bow_view(rng, 1000)
    K = synth.make_bow_related(rng, F, 1000, 0.6, 40.0)
    c = ctx()
    gF, gK = engine.BowView(c, F), engine.BowView(c, K)
    for frac in (1.0, 0.5, 0.1):
        K.valid = (rng.random(1000) < frac).astype(np.uint8)
        gK.set_valid(K.valid)
        out, nm = engine.BowSearch(c, gF, [gK], True).run()
        o_nm, o_out = ol.search_by_bow(True, ol.OracleBow(K), ol.OracleBow(F))
        assert nm[0] == o_nm and np.array_equal(out[0], o_out)


def test_invalid_feature_vectors_rejected():
    rng = np.random.default_rng(108)
    v = synth.make_bow_view(rng, 100)
    v.feat = v.feat.copy()
    v.feat[1] = v.feat[0]  # a feature in the FeatureVector twice
    with pytest.raises(RuntimeError):
        engine.BowView(ctx(), v)
    big = synth.make_bow_view(rng, 8193)
    with pytest.raises(RuntimeError):
        engine.BowView(ctx(), big)
