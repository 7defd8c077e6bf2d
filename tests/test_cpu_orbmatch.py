"""ORBmatcher::SearchByBoW oracle (oracle/orbmatch_oracle.cpp) pinned on CPU:

* DescriptorDistance (ORBmatcher.cpp:1492-1508) against numpy popcount;
* ComputeThreeMaxima (:1446-1487) on hand-made histograms with the reference's tie and 10 % rules;
* hand-built known-answer searches exercising every branch of both overloads (ORBmatcher.cpp:110-240,
  :354-488): inclusive vs strict TH_LOW, the ratio test, first-minimum ties, the greedy "already
  matched" exclusion, invalid map points, the rotation filter (and its 1/HISTO_LENGTH bin factor);
* an independent pure-Python restatement (dict FeatureVector + the reference's merge walk) against the
  C oracle on random views;
* the committed golden fixtures tests/golden/bow_traces.npz (made by tests/golden/make_golden.py).

The reference ships no tests or fixtures for this path: the known answers below are
derived by hand from the reference text.
"""
import math
import os

import numpy as np
import pytest

import oracle_lib as ol
from rsc import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---- independent restatement (pure Python, small cases only) -----------------------------------
def py_dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def py_bin(a, b):
    factor = np.float32(1.0) / np.float32(30)
    rot = np.float32(np.float32(a) - np.float32(b))
    if rot < 0.0:
        rot = np.float32(rot + np.float32(360.0))
    x = float(np.float32(rot * factor))
    b = int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))
    return 0 if b == 30 else b


def py_three_maxima(sizes):
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(sizes):
        if s > max1:
            max3, max2, max1 = max2, max1, s
            i3, i2, i1 = i2, i1, i
        elif s > max2:
            max3, max2 = max2, s
            i3, i2 = i2, i
        elif s > max3:
            max3, i3 = s, i
    if max2 < np.float32(0.1) * np.float32(max1):
        i2 = i3 = -1
    elif max3 < np.float32(0.1) * np.float32(max1):
        i3 = -1
    return i1, i2, i3


def fv_dict(v):
    return {int(v.node_id[k]): [int(x) for x in v.feat[v.node_begin[k]:v.node_begin[k + 1]]]
            for k in range(len(v.node_id))}


def py_search(frame_variant, A, B, nnratio=0.75, check=True):
    """SearchByBoW restated with Python dicts; frame_variant: (pKF=A, F=B) else (pKF1=A, pKF2=B)."""
    fa, fb = fv_dict(A), fv_dict(B)
    out = [-1] * (B.n if frame_variant else A.n)
    matched_b = [False] * B.n
    hist = [[] for _ in range(30)]
    nm = 0
    ratio = np.float32(nnratio)
    for node in sorted(set(fa) & set(fb)):
        for a in fa[node]:
            if A.valid is not None and not A.valid[a]:
                continue
            b1, bi, b2 = 256, -1, 256
            for b in fb[node]:
                if frame_variant:
                    if out[b] >= 0:
                        continue
                else:
                    if matched_b[b] or (B.valid is not None and not B.valid[b]):
                        continue
                d = py_dist(A.desc[a], B.desc[b])
                if d < b1:
                    b2, b1, bi = b1, d, b
                elif d < b2:
                    b2 = d
            ok = b1 <= 50 if frame_variant else b1 < 50
            if ok and np.float32(b1) < ratio * np.float32(b2):
                if frame_variant:
                    out[bi] = a
                    key = bi
                else:
                    out[a] = bi
                    matched_b[bi] = True
                    key = a
                if check:
                    hist[py_bin(A.angle[a], B.angle[bi])].append(key)
                nm += 1
    if check:
        keep = py_three_maxima([len(h) for h in hist])
        for i, h in enumerate(hist):
            if i in keep:
                continue
            for key in h:
                out[key] = -1
                nm -= 1
    return nm, np.array(out, np.int32)


# ---- hand-built views --------------------------------------------------------------------------
def view(desc_bits, angles, nodes, valid=None):
    """desc_bits: list of sets of bit positions set in each descriptor (rest zero)."""
    n = len(desc_bits)
    desc = np.zeros((n, 32), np.uint8)
    for i, bits in enumerate(desc_bits):
        for b in bits:
            desc[i, b // 8] |= np.uint8(1 << (b % 8))
    node_id, begin, feat = synth._feature_vector(np.asarray(nodes, np.uint32))
    return synth.BowFeatures(n, desc, np.asarray(angles, np.float32),
                             None if valid is None else np.asarray(valid, np.uint8), node_id, begin, feat)


def bits(k, start=0):
    return set(range(start, start + k))


def run_both(frame_variant, A, B, nnratio=0.75, check=True):
    nm, out = ol.search_by_bow(frame_variant, ol.OracleBow(A), ol.OracleBow(B), nnratio, check)
    pnm, pout = py_search(frame_variant, A, B, nnratio, check)
    assert nm == pnm and np.array_equal(out, pout), (nm, out, pnm, pout)
    return nm, out


def test_descriptor_distance_is_popcount():
    rng = np.random.default_rng(5)
    for _ in range(200):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert ol.descriptor_distance(a, b) == py_dist(a, b)
    z = np.zeros(32, np.uint8)
    assert ol.descriptor_distance(z, np.full(32, 255, np.uint8)) == 256
    assert ol.descriptor_distance(z, z) == 0


@pytest.mark.parametrize("sizes,expect", [
    ([0] * 30, (-1, -1, -1)),
    ([5] + [0] * 29, (0, -1, -1)),                 # max2 = 0 < 0.5 -> ind2 = ind3 = -1
    ([10, 1, 1] + [0] * 27, (0, 1, 2)),            # 1 < 0.1f * 10 = 1.0 is false: all kept
    ([20, 3, 1] + [0] * 27, (0, 1, -1)),           # 1 < 2.0 -> ind3 dropped
    ([3, 9, 9, 2] + [0] * 26, (1, 2, 0)),          # ties keep the earlier bin (strict >)
    ([4, 4, 4, 4] + [0] * 26, (0, 1, 2)),
    ([100, 10, 9] + [0] * 27, (0, 1, -1)),         # 9 < 10.0 -> ind3 dropped
    ([100, 9, 50] + [0] * 27, (0, 2, -1)),         # max2=50, max3=9 < 10 -> ind3 dropped
])
def test_three_maxima(sizes, expect):
    got = ol.compute_three_maxima(sizes)
    assert got == py_three_maxima(sizes) == expect


def test_bin_factor_quirk():
    """factor = 1/HISTO_LENGTH (ORBmatcher.cpp:123,189): a rotation of 359 degrees lands in bin 12."""
    assert py_bin(359.0, 0.0) == 12 and py_bin(0.0, 1.0) == 12 and py_bin(10.0, 10.0) == 0
    assert py_bin(44.9, 0.0) == 1 and py_bin(45.1, 0.0) == 2


def test_frame_overload_known_answer():
    # one node; KF features 0,1,2 ; Frame features 0,1,2
    A = view([bits(0), bits(0), bits(0, 100)], [0, 0, 0], [11, 11, 11])
    # F0 at distance 10 from A0, F1 at distance 30, F2 at distance 50 (exactly TH_LOW)
    B = view([bits(10), bits(30), bits(50, 150)], [0, 0, 0], [11, 11, 11])
    nm, out = run_both(True, A, B)
    # A0: best F0 (10), second F1 (30): 10 < 0.75*30 -> match F0 <- A0
    # A1: F0 taken; best F1 (30), second F2 (50+0 vs zero desc = 50): 30 < 37.5 -> F1 <- A1
    # A2 (bits 100..199 != F2 bits 150..199 -> distance 50): only F2 left -> 50 <= 50 and 50 < 0.75*256
    assert out.tolist() == [0, 1, 2] and nm == 3


def test_kf_overload_threshold_is_strict():
    A = view([bits(0, 100)], [0], [11])
    B = view([bits(50, 150)], [0], [11])  # distance exactly 50
    nm, out = run_both(False, A, B)
    assert nm == 0 and out.tolist() == [-1]
    nm, out = run_both(True, A, B)  # the Frame overload accepts <= TH_LOW
    assert nm == 1 and out.tolist() == [0]


def test_ratio_test_and_first_min_ties():
    A = view([bits(0)], [0], [11])
    B = view([bits(20), bits(20, 100), bits(22)], [0, 0, 0], [11, 11, 11])  # F0 and F1 tie at 20
    nm, out = run_both(True, A, B)
    # best = F0 (first), second = 20 -> 20 < 15 false: no match
    assert nm == 0 and out.tolist() == [-1, -1, -1]
    nm, out = run_both(True, A, B, nnratio=1.01)
    assert nm == 1 and out.tolist() == [0, -1, -1]


def test_invalid_map_points_and_no_common_nodes():
    A = view([bits(0), bits(0)], [0, 0], [11, 12], valid=[0, 1])
    B = view([bits(1), bits(1), bits(2)], [0, 0, 0], [11, 12, 13], valid=[1, 0, 1])
    nm, out = run_both(True, A, B)  # A0 invalid; A1 -> B1 (the Frame side's validity is not checked)
    assert out.tolist() == [-1, 1, -1] and nm == 1
    nm, out = run_both(False, A, B)  # KF overload: B1 invalid -> A1 has no candidate in node 12
    assert out.tolist() == [-1, -1] and nm == 0
    C = view([bits(0)], [0], [99])
    assert run_both(True, A, C)[0] == 0 and run_both(False, C, B)[0] == 0


def test_rotation_filter_removes_minor_bins():
    # 12 matches with a rotation of 0 degrees and 1 match at 90 degrees (bin 3): 1 < 0.1 * 12 -> removed
    n = 13
    A = view([bits(i % 4, 8 * i) for i in range(n)], [0.0] * 12 + [90.0], [11 + i for i in range(n)])
    B = view([bits(i % 4, 8 * i) for i in range(n)], [0.0] * n, [11 + i for i in range(n)])
    nm, out = run_both(True, A, B)
    assert nm == 12 and out[12] == -1 and (out[:12] == np.arange(12)).all()
    nm, out = run_both(True, A, B, check=False)
    assert nm == 13


def test_random_views_match_python_restatement():
    rng = np.random.default_rng(11)
    for trial in range(12):
        n1, n2 = rng.integers(5, 160, 2)
        A = synth.make_bow_view(rng, int(n1), valid_frac=0.8, skew=1.2)
        B = synth.make_bow_related(rng, A, int(n2), overlap=0.6, rot_deg=rng.uniform(0, 360), valid_frac=0.8,
                                   mean_flips=float(rng.uniform(5, 40)), skew=1.2)
        for fv in (True, False):
            for check in (True, False):
                run_both(fv, A, B, nnratio=float(rng.choice([0.6, 0.75, 0.9])), check=check)


def golden_views(g, k):
    def side(s):
        f = {x: g[f"c{k}_{s}_{x}"] for x in ("desc", "angle", "valid", "node_id", "node_begin", "feat")}
        return synth.BowFeatures(len(f["angle"]), **f)
    fv, check = (bool(x) for x in g[f"c{k}_cfg"])
    return side("A"), side("B"), fv, float(g[f"c{k}_ratio"]), check


def test_golden_bow_traces():
    g = np.load(os.path.join(ROOT, "tests", "golden", "bow_traces.npz"))
    for k in range(int(g["cases"])):
        A, B, fv, ratio, check = golden_views(g, k)
        nm, out = ol.search_by_bow(fv, ol.OracleBow(A), ol.OracleBow(B), ratio, check)
        assert nm == int(g[f"c{k}_n"]) and nm > 0, k
        assert np.array_equal(out, g[f"c{k}_out"]), k
        if A.n <= 400 and B.n <= 400:
            pnm, pout = py_search(fv, A, B, ratio, check)
            assert pnm == nm and np.array_equal(pout, out), k
