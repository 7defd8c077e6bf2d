"""The C++ drop-in facade (rsc_orb::PnPsolver / Sim3Solver templates, csrc/facade/) driven through
mock ORB-SLAM types — null matches, bad MapPoints, invalid keyframe indices — against the oracle.
The binary (orb-slam2-optimized_amd/lib/facade_test) is built by __graft_entry__.build()."""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as ol
from gpu_common import bits
from rsc import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "orb-slam2-optimized_amd", "lib", "facade_test")


def run(inp: bytes) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        open(a, "wb").write(inp)
        subprocess.run([BIN, a, b], check=True, timeout=120)
        return open(b, "rb").read()


def test_pnp_facade_matches_oracle():
    rng = np.random.default_rng(3)
    n_frame = 700
    s2 = synth.level_sigma2()
    sc = synth.make_pnp_scene(rng, 560, 0.62)
    # frame with 700 keypoints: 560 matched (some bad), 140 without MapPoint
    slots = np.sort(rng.choice(n_frame, sc.n, replace=False))
    bad = rng.random(sc.n) < 0.05
    octaves = np.array([int(np.where(s2 == v)[0][0]) for v in sc.sigma2])
    buf = struct.pack("<i", 1) + struct.pack("<i4f", n_frame, sc.fx, sc.fy, sc.cx, sc.cy)
    buf += struct.pack("<i", len(s2)) + s2.astype("<f4").tobytes()
    present = np.zeros(n_frame, np.int32)
    kp = np.zeros((n_frame, 2), np.float32)
    oc = np.zeros(n_frame, np.int32)
    X = np.zeros((n_frame, 3), np.float32)
    present[slots] = np.where(bad, 2, 1)
    kp[slots] = sc.p2d
    oc[slots] = octaves
    X[slots] = sc.p3dw
    for i in range(n_frame):
        buf += struct.pack("<i2fi3f", present[i], kp[i, 0], kp[i, 1], oc[i], *X[i])
    calls = [5, 5, 5, 5, 300, -1]
    buf += struct.pack("<I", 9) + struct.pack("<d", 0.99) + struct.pack("<iii", 10, 300, 4)
    buf += struct.pack("<ff", 0.5, 5.991) + struct.pack("<i", len(calls)) + struct.pack(f"<{len(calls)}i", *calls)
    out = run(buf)
    # oracle on the compacted arrays (PnPsolver.cpp:22-44: skip null and bad)
    keep = ~bad
    comp = synth.PnPScene(p2d=sc.p2d[keep], p3dw=sc.p3dw[keep], sigma2=sc.sigma2[keep],
                          kp_index=slots[keep].astype(np.int32), n_points=n_frame, R_true=sc.R_true,
                          t_true=sc.t_true, inlier_true=sc.inlier_true[keep])
    o = ol.OraclePnP(comp, 9)
    o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    off = 0
    for c in calls:
        ok, nm, ni = struct.unpack_from("<3i", out, off); off += 12
        T = np.frombuffer(out, "<f4", 16, off).reshape(4, 4); off += 64
        (ml,) = struct.unpack_from("<i", out, off); off += 4
        mask = np.frombuffer(out, np.uint8, ml, off).astype(bool); off += ml
        r = o.iterate(o.info()["max_iterations"] if c < 0 else c)
        assert (bool(ok), bool(nm) if c >= 0 else r["no_more"], ni) == (r["ok"], r["no_more"], r["n_inliers"])
        if r["ok"]:
            assert np.array_equal(bits(T), bits(r["T"])) and np.array_equal(mask, r["inliers"])
        else:
            assert ml == 0


def test_sim3_facade_matches_oracle():
    rng = np.random.default_rng(4)
    pair = synth.make_sim3_pair(rng, 500, 200)
    n1 = pair.n1
    s2 = synth.level_sigma2()
    oc1 = np.array([int(np.where(s2 == v)[0][0]) for v in pair.sigma2_1], np.int32)
    oc2 = np.array([int(np.where(s2 == v)[0][0]) for v in pair.sigma2_2], np.int32)
    flags = np.full(n1, 1 | 2, np.int32)
    r = rng.random(n1)
    flags[r < 0.04] = 2          # no match
    flags[(r >= 0.04) & (r < 0.07)] = 1  # match but KF1 has no MapPoint in that slot
    flags[(r >= 0.07) & (r < 0.09)] |= 4   # pMP1 bad
    flags[(r >= 0.09) & (r < 0.11)] |= 8   # pMP2 bad
    flags[(r >= 0.11) & (r < 0.13)] |= 16  # pMP1 not in KF1
    flags[(r >= 0.13) & (r < 0.15)] |= 32  # pMP2 not in KF2
    buf = struct.pack("<i", 2) + struct.pack("<i", n1)
    for R, t, K in ((pair.R1, pair.t1, pair.K1), (pair.R2, pair.t2, pair.K2)):
        buf += np.asarray(R, "<f4").tobytes() + np.asarray(t, "<f4").tobytes() + np.asarray(K, "<f4").tobytes()
        buf += struct.pack("<i", len(s2)) + s2.astype("<f4").tobytes()
    for i in range(n1):
        buf += struct.pack("<i3f3fii", flags[i], *pair.Xw1[i], *pair.Xw2[i], oc1[i], oc2[i])
    calls = [5] * 8 + [300]
    buf += struct.pack("<I", 5) + struct.pack("<d", 0.99) + struct.pack("<ii", 20, 300)
    buf += struct.pack("<i", len(calls)) + struct.pack(f"<{len(calls)}i", *calls)
    out = run(buf)
    valid = ((flags & 1) > 0) & ((flags & 2) > 0) & ((flags & (4 | 8 | 16 | 32)) == 0)
    p2 = synth.Sim3Pair(valid=valid.astype(np.uint8), Xw1=pair.Xw1, Xw2=pair.Xw2, sigma2_1=pair.sigma2_1,
                        sigma2_2=pair.sigma2_2, R1=pair.R1, t1=pair.t1, R2=pair.R2, t2=pair.t2, K1=pair.K1,
                        K2=pair.K2, inlier_true=pair.inlier_true)
    o = ol.OracleSim3(p2, 5)
    o.set_ransac_parameters(0.99, 20, 300)
    off = 0
    for c in calls:
        ok, nm, ni = struct.unpack_from("<3i", out, off); off += 12
        R = np.frombuffer(out, "<f4", 9, off).reshape(3, 3); off += 36
        t = np.frombuffer(out, "<f4", 3, off); off += 12
        (ml,) = struct.unpack_from("<i", out, off); off += 4
        mask = np.frombuffer(out, np.uint8, ml, off).astype(bool); off += ml
        r = o.iterate(c)
        assert (bool(ok), bool(nm), ni) == (r["ok"], r["no_more"], r["n_inliers"])
        assert np.array_equal(bits(R), bits(r["R"])) and np.array_equal(bits(t), bits(r["t"]))
        assert np.array_equal(mask, r["inliers"])


def test_mlpnp_facade_matches_oracle():
    rng = np.random.default_rng(8)
    n_frame = 600
    s2 = synth.level_sigma2()
    sc = synth.make_pnp_scene(rng, 480, 0.58)
    slots = np.sort(rng.choice(n_frame, sc.n, replace=False))
    bad = rng.random(sc.n) < 0.05
    octaves = np.array([int(np.where(s2 == v)[0][0]) for v in sc.sigma2])
    buf = struct.pack("<i", 3) + struct.pack("<i4f", n_frame, sc.fx, sc.fy, sc.cx, sc.cy)
    buf += struct.pack("<i", len(s2)) + s2.astype("<f4").tobytes()
    present = np.zeros(n_frame, np.int32)
    kp = np.zeros((n_frame, 2), np.float32)
    oc = np.zeros(n_frame, np.int32)
    X = np.zeros((n_frame, 3), np.float32)
    present[slots] = np.where(bad, 2, 1)
    kp[slots] = sc.p2d
    oc[slots] = octaves
    X[slots] = sc.p3dw
    for i in range(n_frame):
        buf += struct.pack("<i2fi3f", present[i], kp[i, 0], kp[i, 1], oc[i], *X[i])
    calls = [5, 5, 5, 40]
    buf += struct.pack("<I", 4) + struct.pack("<d", 0.99) + struct.pack("<iii", 10, 300, 6)
    buf += struct.pack("<ff", 0.5, 5.991) + struct.pack("<i", len(calls)) + struct.pack(f"<{len(calls)}i", *calls)
    out = run(buf)
    keep = ~bad
    comp = synth.PnPScene(p2d=sc.p2d[keep], p3dw=sc.p3dw[keep], sigma2=sc.sigma2[keep],
                          kp_index=slots[keep].astype(np.int32), n_points=n_frame, R_true=sc.R_true,
                          t_true=sc.t_true, inlier_true=sc.inlier_true[keep])
    o = ol.OracleMLPnP(comp, 4)
    o.set_ransac_parameters(0.99, 10, 300, 6, 0.5, 5.991)
    off = 0
    for c in calls:
        ok, nm, ni = struct.unpack_from("<3i", out, off); off += 12
        T = np.frombuffer(out, "<f4", 16, off).reshape(4, 4); off += 64
        (ml,) = struct.unpack_from("<i", out, off); off += 4
        mask = np.frombuffer(out, np.uint8, ml, off).astype(bool); off += ml
        r = o.iterate(c)
        assert (bool(ok), bool(nm), ni) == (r["ok"], r["no_more"], r["n_inliers"])
        assert np.array_equal(bits(T), bits(r["T"]))
        if r["ok"]:
            assert np.array_equal(mask, r["inliers"])
        else:
            assert ml == 0


@pytest.mark.parametrize("stereo", [0.0, 0.75])
def test_pose_optimization_facade_matches_oracle(stereo):
    """rsc_orb::PoseOptimization(Frame*) (Optimizer.cpp:205-424) on a mock Frame (monocular, or with
    75 % stereo slots mvuRight >= 0): slots without a MapPoint keep mvbOutlier, SetPose is called once,
    nGood / pose / flags equal the oracle."""
    rng = np.random.default_rng(31)
    f = synth.make_poseopt_frame(rng, 900, 0.75, no_mp_frac=0.2, stereo_frac=stereo)
    ur = f.u_right if f.u_right is not None else np.full(f.n, -1.0, np.float32)
    inv_levels = (np.float32(1.0) / synth.level_sigma2()).astype(np.float32)
    oc = np.array([int(np.where(inv_levels == v)[0][0]) for v in f.inv_sigma2])
    buf = struct.pack("<i", 4) + struct.pack("<i5f", f.n, f.fx, f.fy, f.cx, f.cy, f.bf)
    buf += f.Tcw.astype("<f4").tobytes() + struct.pack("<i", len(inv_levels)) + inv_levels.astype("<f4").tobytes()
    for i in range(f.n):
        buf += struct.pack("<i2fi3ff", int(f.has_mp[i]), f.uv[i, 0], f.uv[i, 1], oc[i], *f.Xw[i], ur[i])
    out = run(buf)
    n_good, calls = struct.unpack_from("<ii", out, 0)
    T = np.frombuffer(out, "<f4", 16, 8).reshape(4, 4)
    flags = np.frombuffer(out, np.uint8, f.n, 8 + 64)
    r, To, outl, st = ol.pose_optimization(f)
    assert n_good == r and calls == 1
    assert np.array_equal(bits(T), bits(To))
    sel = f.has_mp == 1
    assert np.array_equal(flags[sel], outl[sel])
    assert (flags[~sel] == 1).all()  # untouched (the mock starts them at true)


def _view_bytes(v, mp_state):
    """facade_test view record; mp_state[i]: 0 no map point, 1 good, 2 bad."""
    b = struct.pack("<i", v.n) + np.ascontiguousarray(v.desc, np.uint8).tobytes()
    b += np.ascontiguousarray(v.angle, "<f4").tobytes() + np.asarray(mp_state, np.uint8).tobytes()
    b += struct.pack("<i", len(v.node_id))
    for k in range(len(v.node_id)):
        f = v.feat[v.node_begin[k]:v.node_begin[k + 1]]
        b += struct.pack("<II", int(v.node_id[k]), len(f)) + np.asarray(f, "<u4").tobytes()
    return b


@pytest.mark.parametrize("frame_overload", [True, False])
def test_orbmatcher_facade_matches_oracle(frame_overload):
    """rsc_orb::ORBmatcher::SearchByBoW (ORBmatcher.cpp:110-240 / :354-488) on mock KeyFrames /
    Frame (cv::Mat-like descriptor rows, std::map FeatureVector, null and bad MapPoints): per-call
    and batched results equal the oracle, MapPoint by MapPoint."""
    rng = np.random.default_rng(41 + frame_overload)
    S = synth.make_bow_view(rng, 900)
    views = [synth.make_bow_related(rng, S, int(rng.integers(300, 900)), float(rng.uniform(0.2, 0.7)),
                                    float(rng.uniform(0, 360))) for _ in range(5)]
    states = []
    for v in [S] + views:
        st = rng.choice([0, 1, 2], size=v.n, p=[0.1, 0.8, 0.1]).astype(np.uint8)
        states.append(st)
        v.valid = (st == 1).astype(np.uint8)
    buf = struct.pack("<iifii", 5, int(frame_overload), 0.75, 1, len(views))
    buf += _view_bytes(S, states[0])
    for v, st in zip(views, states[1:]):
        buf += _view_bytes(v, st)
    out = np.frombuffer(run(buf), "<i4")
    oS = ol.OracleBow(S)
    pos = 0
    expect = []
    for v in views:
        ov = ol.OracleBow(v)
        nm, m = ol.search_by_bow(frame_overload, ov, oS) if frame_overload else ol.search_by_bow(False, oS, ov)
        expect.append((nm, m))
    for nm, m in expect:
        assert out[pos] == nm and out[pos + 1] == len(m)
        assert np.array_equal(out[pos + 2:pos + 2 + len(m)], m)
        pos += 2 + len(m)
    for nm, m in expect:  # batched form
        assert out[pos] == nm
        assert np.array_equal(out[pos + 1:pos + 1 + len(m)], m)
        pos += 1 + len(m)
    assert pos == len(out)


def _bow_bytes(ids, vals):
    return struct.pack("<i", len(ids)) + np.asarray(ids, "<u4").tobytes() + np.asarray(vals, "<f8").tobytes()


@pytest.mark.parametrize("seed", [3, 8])
def test_keyframe_database_facade_matches_oracle(seed):
    """rsc_orb::KeyFrameDatabase (KeyFrameDatabase.cpp) on mock KeyFrames / Frames (std::map
    BowVectors, GetBestCovisibilityKeyFrames, GetConnectedKeyFrames): an operation script's
    candidates equal the oracle's, KeyFrame by KeyFrame and in order."""
    import kfdb_script as ks
    ops = ks.make_script(seed, n_kfs=50, n_queries=30, words=250)
    K = 50
    bows, covis = [None] * K, [np.zeros(0, np.int32)] * K
    for op in ops:
        if op[0] == "add" and bows[op[1]] is None:
            bows[op[1]] = (op[2], op[3])
        elif op[0] == "covis":
            covis[op[1]] = op[2]
    buf = struct.pack("<iIi", 6, 10 ** 6, K)
    for k in range(K):
        buf += _bow_bytes(*bows[k]) + struct.pack("<i", len(covis[k])) + np.asarray(covis[k], "<i4").tobytes()
    body, nops = b"", 0
    for op in ops:
        kind = ks.OPS[op[0]]
        if op[0] == "covis":
            continue
        nops += 1
        body += struct.pack("<i", kind)
        if op[0] in ("add", "erase"):
            body += struct.pack("<i", op[1])
        elif op[0] == "reloc":
            body += struct.pack("<Q", op[1]) + _bow_bytes(op[2], op[3])
        elif op[0] == "loop":
            body += struct.pack("<Q", op[1]) + _bow_bytes(op[2], op[3])
            body += struct.pack("<i", len(op[4])) + np.asarray(op[4], "<i4").tobytes() + struct.pack("<f", op[5])
    out = np.frombuffer(run(buf + struct.pack("<i", nops) + body), "<i4")
    want = ks.run_script(ol.OracleKFDB(K), ops)
    pos = 0
    for w in want:
        n = out[pos]
        assert list(out[pos + 1:pos + 1 + n]) == list(w)
        pos += 1 + n
    assert pos == len(out)


def _s3kf_bytes(kf):
    from rsc import synth
    b = struct.pack("<i", kf.n) + np.ascontiguousarray(kf.kp, "<f4").tobytes()
    b += np.ascontiguousarray(kf.octave, "<i4").tobytes() + np.ascontiguousarray(kf.desc, np.uint8).tobytes()
    b += np.ascontiguousarray(kf.cell_begin, "<i4").tobytes() + np.ascontiguousarray(kf.cell_feat, "<i4").tobytes()
    b += struct.pack("<4i", int(kf.min_x), int(kf.max_x), int(kf.min_y), int(kf.max_y))
    b += struct.pack("<6f", synth.GRID_W_INV, synth.GRID_H_INV, kf.fx, kf.fy, kf.cx, kf.cy)
    sf = synth.scale_factors()
    b += struct.pack("<i", len(sf)) + sf.astype("<f4").tobytes() + struct.pack("<f", synth.LOG_SCALE_FACTOR)
    b += np.asarray(kf.Rcw, "<f4").tobytes() + np.asarray(kf.tcw, "<f4").tobytes()
    for i in range(kf.n):
        b += struct.pack("<B3f2f", int(kf.mp_state[i]), *kf.mp_pos[i], kf.mp_dmax[i], kf.mp_dmin[i])
        b += np.ascontiguousarray(kf.mp_desc[i], np.uint8).tobytes()
    return b


@pytest.mark.parametrize("seed", [51, 52])
def test_search_by_sim3_facade_matches_oracle(seed):
    """rsc_orb::ORBmatcher::SearchBySim3 (ORBmatcher.cpp:948-1170, LoopClosing.cpp:309) on mock
    KeyFrames / MapPoints (null, bad, already-matched and foreign MapPoints): nfound and vpMatches12
    after the call equal the oracle."""
    rng = np.random.default_rng(seed)
    kf1, kf2, R12, t12, m12 = synth.make_sim3match_pair(rng, 700, 200, 0.3)
    m12[rng.random(kf1.n) < 0.02] = -2
    buf = struct.pack("<i", 7) + _s3kf_bytes(kf1) + _s3kf_bytes(kf2)
    buf += np.asarray(R12, "<f4").tobytes() + np.asarray(t12, "<f4").tobytes() + struct.pack("<f", 7.5)
    buf += np.asarray(m12, "<i4").tobytes()
    out = run(buf)
    nf = struct.unpack_from("<i", out, 0)[0]
    got = np.frombuffer(out, "<i4", kf1.n, 4)
    onf, o12 = ol.search_by_sim3(kf1, kf2, R12, t12, m12, 7.5)
    o12 = o12[:kf1.n]
    exp = np.where(o12 >= 0, o12, m12)
    assert nf == onf and nf > 20
    assert np.array_equal(got, exp)


def test_optimize_sim3_facade_matches_oracle():
    """rsc_orb::OptimizeSim3 (Optimizer.cpp:1054-1250, LoopClosing.cpp:311) on mock KeyFrames /
    MapPoints / g2o::Sim3: every reason a slot is not a correspondence (NULL match, NULL or bad
    MapPoint 1, bad MapPoint 2, not in KF2), KF2 keypoints in another order; nIn, g2oS12 and the NULLed
    vpMatches1 entries equal the oracle."""
    rng = np.random.default_rng(61)
    p = synth.make_sim3opt_problem(rng, 600, valid_frac=0.8, outlier_frac=0.2)
    n1, n2 = p.n, p.n + 50
    inv_levels = (np.float32(1.0) / synth.level_sigma2()).astype(np.float32)
    oc1 = np.array([int(np.where(inv_levels == v)[0][0]) for v in p.inv1])
    oc2 = np.array([int(np.where(inv_levels == v)[0][0]) for v in p.inv2])
    i2 = rng.permutation(n2)[:n1]
    kind = np.where(p.valid == 1, 5, rng.integers(0, 5, n1))
    kp2 = np.zeros((n2, 2), np.float32)
    o2 = np.zeros(n2, np.int32)
    kp2[i2] = p.uv2
    o2[i2] = oc2
    buf = struct.pack("<iii", 8, n1, n2)
    for R, t, K in ((p.R1w, p.t1w, p.K1), (p.R2w, p.t2w, p.K2)):
        buf += np.asarray(R, "<f4").tobytes() + np.asarray(t, "<f4").tobytes() + np.asarray(K, "<f4").tobytes()
        buf += struct.pack("<i", len(inv_levels)) + inv_levels.astype("<f4").tobytes()
    for j in range(n2):
        buf += struct.pack("<2fi", kp2[j, 0], kp2[j, 1], int(o2[j]))
    for i in range(n1):
        buf += struct.pack("<2fii3f3fi", p.uv1[i, 0], p.uv1[i, 1], int(oc1[i]), int(kind[i]), *p.X1w[i], *p.X2w[i],
                           int(i2[i]))
    buf += np.asarray(p.S0, "<f8").tobytes() + struct.pack("<f", p.th2)
    out = run(buf)
    nIn = struct.unpack_from("<i", out, 0)[0]
    S = np.frombuffer(out, "<f8", 8, 4)
    still = np.frombuffer(out, np.uint8, n1, 4 + 64)
    r, So, keep, st = ol.optimize_sim3(p)
    assert nIn == r and r > 100
    assert np.array_equal(S.view(np.uint64), So.view(np.uint64))
    expect = (kind != 0) & (keep == 1)
    assert np.array_equal(still.astype(bool), expect)


def test_relocalization_loop_on_the_reference_rand_stream():
    """The facade in reference_rand mode (csrc/facade/rsc_context.hpp, Q3): Tracking::Relocalization's
    round-robin (Tracking.cpp:1239-1262) over several candidate Frames, every solver drawing from the
    thread's one srand(1) stream in call order — every call equals the oracle's call on libc's real
    rand(), and the stream ends at the oracle's position."""
    rng = np.random.default_rng(12)
    s2 = synth.level_sigma2()
    scenes = [synth.make_pnp_scene(rng, int(rng.integers(150, 600)), r) for r in (0.2, 0.3, 0.05, 0.62, 0.7)]
    params = (0.99, 10, 300, 4, 0.5, 5.991)
    buf = struct.pack("<i", 9) + struct.pack("<i", len(scenes)) + struct.pack("<d", params[0])
    buf += struct.pack("<iii", *params[1:4]) + struct.pack("<ff", *params[4:])
    for sc in scenes:
        octaves = np.array([int(np.where(s2 == v)[0][0]) for v in sc.sigma2])
        buf += struct.pack("<i4f", sc.n, sc.fx, sc.fy, sc.cx, sc.cy) + struct.pack("<i", len(s2))
        buf += s2.astype("<f4").tobytes()
        for i in range(sc.n):
            buf += struct.pack("<i2fi3f", 1, sc.p2d[i, 0], sc.p2d[i, 1], octaves[i], *sc.p3dw[i])
    out = run(buf)
    os_ = [ol.OraclePnP(sc, 1) for sc in scenes]
    for o in os_:
        o.set_ransac_parameters(*params)
        o.use_libc_rand()
    ol.libc_srand(1)
    off, calls, used = 0, 0, 0
    while True:
        (i,) = struct.unpack_from("<i", out, off); off += 4
        if i < 0:
            break
        ok, nm, ni = struct.unpack_from("<3i", out, off); off += 12
        T = np.frombuffer(out, "<f4", 16, off).reshape(4, 4); off += 64
        before = os_[i].info()["iterations"]
        r = os_[i].iterate(5)
        used += 4 * (os_[i].info()["iterations"] - before)
        assert (bool(ok), bool(nm), ni) == (r["ok"], r["no_more"], r["n_inliers"]), f"call {calls} cand {i}"
        if r["ok"]:
            assert np.array_equal(bits(T), bits(r["T"]))
        calls += 1
    (pos,) = struct.unpack_from("<q", out, off)
    assert calls >= 4 and pos == used
