"""ORBmatcher::SearchBySim3 oracle (oracle/sim3match_oracle.cpp) pinned on CPU:

* the fdlibm log restatement used for MapPoint::PredictScale (rsc_math.h) against numpy / glibc;
* PredictScale (MapPoint.cpp:367-381) on hand-made ratios, including both clamps;
* hand-built known answers (ORBmatcher.cpp:948-1170): the mutual-agreement rule, already-matched
  (with and without an index in KF2) and bad MapPoints, the octave window [level-1, level],
  TH_HIGH inclusive;
* an independent pure-Python restatement (numpy float32 scalars) against the C oracle on random
  pairs — the branches not hand-built above (depth, IsInImage, scale-invariance window, grid-order
  first minimum, pKF1's intrinsics in both directions) are exercised there;
* the committed golden fixture tests/golden/sim3match_traces.npz.

The reference ships no tests for this path; the known answers follow its text.
"""
import math
import os

import numpy as np
import pytest

import oracle_lib as ol
from rsc import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f32 = np.float32


def test_log_restatement_within_one_ulp():
    rng = np.random.default_rng(3)
    x = np.exp(rng.uniform(-40, 40, 20000))
    L = ol.lib()
    got = np.array([L.ora_dm_log(float(v)) for v in x])
    ref = np.log(x)
    ulp = np.abs(np.spacing(ref))
    assert (np.abs(got - ref) <= ulp).all()
    # logf as the float rounding: equal to float32(log) except within an ulp of a rounding boundary
    xf = x.astype(np.float32)
    lf = np.array([np.float32(L.ora_dm_log(float(v))) for v in xf])
    assert (lf == np.log(xf.astype(np.float64)).astype(np.float32)).mean() > 0.999


@pytest.mark.parametrize("dmax,dist,expect", [
    (1.0, 1.0, 0),             # log(1) = 0 -> ceil(0) = 0
    (1.0, 2.0, 0),             # negative -> clamped to 0
    (10.0, 1.0, 7),            # ceil(log(10)/log(1.2)) = 13 -> clamped to levels - 1
    (1.44, 1.0, 2),            # 1.2^2 in float: log ratio / log 1.2 rounds to just above or at 2
    (1.3, 1.0, 2),             # between 1.2 and 1.44 -> 2
    (1.1, 1.0, 1),
])
def test_predict_scale(dmax, dist, expect):
    got = ol.lib().ora_predict_scale(dmax, dist, float(synth.LOG_SCALE_FACTOR), 8)
    if dmax == 1.44:
        r = f32(f32(dmax) / f32(dist))
        q = f32(np.float32(ol.lib().ora_dm_log(float(r))) / synth.LOG_SCALE_FACTOR)
        expect = int(math.ceil(q))
    assert got == expect


# ---- independent restatement (pure Python + numpy float32 scalars) ----------------------------
def py_search(kf1, kf2, R12, t12, m12, th=7.5):
    L = ol.lib()
    sf = synth.scale_factors()
    R12 = np.asarray(R12, f32).reshape(3, 3)
    t12 = np.asarray(t12, f32).reshape(3)
    R21 = R12.T.copy()
    t21 = np.array([-f32(f32(f32(R21[r, 0] * t12[0]) + f32(R21[r, 1] * t12[1])) + f32(R21[r, 2] * t12[2]))
                    for r in range(3)], f32)

    def rot_add(R, x, t):
        R = np.asarray(R, f32).reshape(3, 3)
        return np.array([f32(f32(f32(f32(R[r, 0] * x[0]) + f32(R[r, 1] * x[1])) + f32(R[r, 2] * x[2])) + t[r])
                         for r in range(3)], f32)

    def direction(src, dst, Rsd, tsd, already):
        out = [-1] * src.n
        for i in range(src.n):
            if src.mp_state[i] != 1 or already[i]:
                continue
            pc = rot_add(src.Rcw, src.mp_pos[i], np.asarray(src.tcw, f32))
            pd = rot_add(Rsd, pc, tsd)
            if pd[2] < 0:
                continue
            invz = f32(1.0 / np.float64(pd[2]))
            x, y = f32(pd[0] * invz), f32(pd[1] * invz)
            u = f32(f32(f32(kf1.fx) * x) + f32(kf1.cx))
            v = f32(f32(f32(kf1.fy) * y) + f32(kf1.cy))
            if not (u >= dst.min_x and u < dst.max_x and v >= dst.min_y and v < dst.max_y):
                continue
            mx, mn = f32(f32(1.2) * src.mp_dmax[i]), f32(f32(0.8) * src.mp_dmin[i])
            d3 = np.sqrt(f32(f32(f32(pd[0] * pd[0]) + f32(pd[1] * pd[1])) + f32(pd[2] * pd[2])))
            if d3 < mn or d3 > mx:
                continue
            ratio = f32(src.mp_dmax[i] / d3)
            lvl = int(math.ceil(f32(np.float32(L.ora_dm_log(float(ratio))) / synth.LOG_SCALE_FACTOR)))
            lvl = min(max(lvl, 0), len(sf) - 1)
            r = f32(f32(th) * sf[lvl])
            gx, gy = synth.GRID_W_INV, synth.GRID_H_INV
            x0 = max(0, math.floor(f32(f32(f32(u - f32(dst.min_x)) - r) * gx)))
            x1 = min(63, math.ceil(f32(f32(f32(u - f32(dst.min_x)) + r) * gx)))
            y0 = max(0, math.floor(f32(f32(f32(v - f32(dst.min_y)) - r) * gy)))
            y1 = min(47, math.ceil(f32(f32(f32(v - f32(dst.min_y)) + r) * gy)))
            if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
                continue
            best, bi = 1 << 31, -1
            for ix in range(x0, x1 + 1):
                for iy in range(y0, y1 + 1):
                    c = ix * 48 + iy
                    for e in range(dst.cell_begin[c], dst.cell_begin[c + 1]):
                        j = int(dst.cell_feat[e])
                        if not (abs(f32(dst.kp[j, 0] - u)) < r and abs(f32(dst.kp[j, 1] - v)) < r):
                            continue
                        if dst.octave[j] < lvl - 1 or dst.octave[j] > lvl:
                            continue
                        d = int(np.unpackbits(np.bitwise_xor(src.mp_desc[i], dst.desc[j])).sum())
                        if d < best:
                            best, bi = d, j
            if best <= 100:
                out[i] = bi
        return out

    a1 = [m != -1 for m in m12]
    a2 = [False] * kf2.n
    for m in m12:
        if m >= 0:
            a2[m] = True
    m1 = direction(kf1, kf2, R21, t21, a1)
    m2 = direction(kf2, kf1, R12, t12, a2)
    out = np.full(kf1.n, -1, np.int32)
    for i in range(kf1.n):
        if m1[i] >= 0 and m2[m1[i]] == i:
            out[i] = m1[i]
    return int((out >= 0).sum()), out


def test_random_pairs_match_python_restatement():
    for seed in range(3):
        kf1, kf2, R12, t12, m12 = synth.make_sim3match_pair(np.random.default_rng(100 + seed), n_points=150,
                                                            n_extra=60)
        nf, out = ol.search_by_sim3(kf1, kf2, R12, t12, m12)
        pnf, pout = py_search(kf1, kf2, R12, t12, m12)
        assert nf == pnf and np.array_equal(out, pout), seed
        assert nf > 5


# ---- known answers --------------------------------------------------------------------------
def tiny_pair(n=1):
    """KF1 and KF2 with identity poses looking at points straight ahead; R12 = I, t12 = 0."""
    rng = np.random.default_rng(7)
    P = np.array([[0.1 * i, 0.05 * i, 4.0] for i in range(n)], np.float32)

    def kf(extra_kp=None):
        uv = np.stack([synth.FX * P[:, 0] / P[:, 2] + synth.CX, synth.FY * P[:, 1] / P[:, 2] + synth.CY], 1)
        kp = uv.astype(np.float32)
        if extra_kp is not None:
            kp = np.concatenate([kp, np.asarray(extra_kp, np.float32)])
        m = len(kp)
        begin, feat = synth.build_grid(kp)
        desc = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        state = np.zeros(m, np.uint8)
        state[:n] = 1
        pos = np.zeros((m, 3), np.float32)
        pos[:n] = P
        dmax = np.zeros(m, np.float32)
        dmax[:n] = 4.0
        dmin = (dmax / synth.scale_factors()[-1]).astype(np.float32)
        mdesc = desc.copy()
        return synth.Sim3KF(m, kp, np.zeros(m, np.int32), desc, begin, feat, np.eye(3, dtype=np.float32),
                            np.zeros(3, np.float32), state, pos, dmax, dmin, mdesc, np.arange(m))
    return kf, P


def run_tiny(kf1, kf2, m12=None):
    if m12 is None:
        m12 = np.full(kf1.n, -1, np.int32)
    I, z = np.eye(3, dtype=np.float32), np.zeros(3, np.float32)
    nf, out = ol.search_by_sim3(kf1, kf2, I, z, m12)
    pnf, pout = py_search(kf1, kf2, I, z, m12)
    assert nf == pnf and np.array_equal(out, pout)
    return nf, out


def matched_tiny(kf):
    a, b = kf(), kf()
    b.desc[0] = a.mp_desc[0]  # KF2's keypoint carries KF1's MapPoint descriptor and vice versa
    a.desc[0] = b.mp_desc[0]
    return a, b


def test_mutual_match_and_rejections():
    kf, P = tiny_pair(1)
    k1, k2 = matched_tiny(kf)
    nf, out = run_tiny(k1, k2)
    assert nf == 1 and out.tolist() == [0]
    # already matched (a MapPoint in vpMatches12 with or without an index in KF2) -> not searched
    assert run_tiny(k1, k2, np.array([0], np.int32))[0] == 0
    assert run_tiny(k1, k2, np.array([-2], np.int32))[0] == 0
    # bad MapPoint in KF1
    a, b = matched_tiny(kf)
    a.mp_state[0] = 2
    assert run_tiny(a, b)[0] == 0
    # octave outside [level-1, level]: predicted level 0 (dist == dmax), KF2's keypoint at octave 3
    a, b = matched_tiny(kf)
    b.octave[0] = 3
    assert run_tiny(a, b)[0] == 0
    # one direction only (KF2's MapPoint descriptor far from KF1's keypoint): no agreement
    a, b = matched_tiny(kf)
    a.desc[0] = np.bitwise_not(b.mp_desc[0])
    assert run_tiny(a, b)[0] == 0


def test_th_high_inclusive():
    kf, P = tiny_pair(1)
    k1, k2 = matched_tiny(kf)
    # KF2 keypoint at Hamming distance exactly 100 from KF1's MapPoint descriptor
    d = k1.mp_desc[0].copy()
    bits = np.arange(100)
    np.bitwise_xor.at(d, bits // 8, (1 << (bits % 8)).astype(np.uint8))
    k2.desc[0] = d
    assert run_tiny(k1, k2)[0] == 1
    np.bitwise_xor.at(d, np.array([100 // 8]), np.array([1 << (100 % 8)], np.uint8))
    k2.desc[0] = d
    assert run_tiny(k1, k2)[0] == 0


def test_golden_sim3match_traces():
    g = np.load(os.path.join(ROOT, "tests", "golden", "sim3match_traces.npz"))
    for k in range(int(g["cases"])):
        kfs = []
        for side in ("A", "B"):
            f = {x: g[f"c{k}_{side}_{x}"] for x in ("kp", "octave", "desc", "cell_begin", "cell_feat", "Rcw", "tcw",
                                                    "mp_state", "mp_pos", "mp_dmax", "mp_dmin", "mp_desc")}
            kfs.append(synth.Sim3KF(len(f["kp"]), mp_id=np.zeros(len(f["kp"]), np.int64), **f))
        nf, out = ol.search_by_sim3(kfs[0], kfs[1], g[f"c{k}_R12"], g[f"c{k}_t12"], g[f"c{k}_m12"])
        assert nf == int(g[f"c{k}_n"]) and nf > 0, k
        assert np.array_equal(out, g[f"c{k}_out"]), k
