#!/usr/bin/env python3
"""Generates the committed fixtures under tests/golden/.

* glibc_rand.json — rand() after srand(seed) from THIS container's glibc (2.35) through ctypes,
  plus DUtils::Random::RandomInt swap-remove sample streams computed in pure Python from those
  libc outputs (Random.cpp:47-50, PnPsolver.cpp:125-138).  Independent of the oracle.
* poseopt_traces.npz — Optimizer::PoseOptimization oracle outputs (pose bits, nGood, round / LM
  iteration / trial counts) on seeded synthetic Frames (regression pins, parity unpinned).
* bow_traces.npz — ORBmatcher::SearchByBoW (both overloads) inputs and oracle outputs on seeded
  synthetic views (the views themselves are stored, so the fixture does not depend on the generator).
* sim3match_traces.npz — ORBmatcher::SearchBySim3 inputs (both KeyFrames, R12/t12, matched12) and
  oracle outputs on seeded synthetic pairs.
* pnp_traces.npz / sim3_traces.npz — per-hypothesis sample indices, inlier counts and poses of the
  oracle restatement on small seeded scenes (regression pins of the oracle; the reference itself
  cannot be built here, see DESIGN.md "Oracle").

Run from the repo root:  python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))

SEEDS = [0, 1, 42, 1234, 987654321]


def libc_rand(seed, n):
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    return [libc.rand() for _ in range(n)]


def python_sample_stream(rands, N, min_set, hyps):
    it = iter(rands)
    out = []
    for _ in range(hyps):
        av = list(range(N))
        s = []
        for _ in range(min_set):
            d = len(av)
            randi = int((next(it) / (2147483647 + 1.0)) * d)
            s.append(av[randi])
            av[randi] = av[-1]
            av.pop()
        out.append(s)
    return out


def main():
    poseopt()
    g = {"glibc": "2.35 (ctypes libc.so.6)", "rand": {}, "samples": []}
    for s in SEEDS:
        g["rand"][str(s)] = libc_rand(s, 2000)
    for (seed, N, ms, hyps) in [(1, 4, 4, 5), (1, 7, 4, 20), (42, 500, 4, 50), (1234, 2000, 4, 50), (7, 1000, 3, 60),
                                (9, 600, 6, 30)]:
        r = libc_rand(seed, ms * hyps)
        g["samples"].append({"seed": seed, "N": N, "min_set": ms, "hyps": hyps,
                             "idx": python_sample_stream(r, N, ms, hyps)})
    with open(os.path.join(HERE, "glibc_rand.json"), "w") as f:
        json.dump(g, f)

    import oracle_lib as ol
    from rsc import synth
    out = {}
    for k, (n, ratio, seed) in enumerate([(64, 0.5, 1), (120, 0.7, 2), (300, 0.4, 3)]):
        sc = synth.make_pnp_scene(np.random.default_rng(900 + k), n, ratio)
        o = ol.OraclePnP(sc, seed)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        o.enable_trace()
        r = o.iterate(80)
        ints, fl = o.trace()
        out[f"s{k}_ints"] = ints
        out[f"s{k}_poses"] = fl
        out[f"s{k}_result"] = np.array([r["ok"], r["no_more"], r["n_inliers"]], np.int32)
        out[f"s{k}_T"] = r["T"]
        out[f"s{k}_mask"] = r["inliers"].astype(np.uint8)
        out[f"s{k}_meta"] = np.array([n, seed, 900 + k], np.int64)
        out[f"s{k}_ratio"] = np.array([ratio])
    np.savez_compressed(os.path.join(HERE, "pnp_traces.npz"), **out)
    out = {}
    for k, (n1, ninl, seed) in enumerate([(80, 40, 1), (300, 90, 2)]):
        pair = synth.make_sim3_pair(np.random.default_rng(950 + k), n1, ninl, invalid_frac=0.1)
        o = ol.OracleSim3(pair, seed)
        o.set_ransac_parameters(0.99, 20, 300)
        o.enable_trace()
        r = o.iterate(60)
        ints, fl = o.trace()
        out[f"s{k}_ints"] = ints
        out[f"s{k}_poses"] = fl
        out[f"s{k}_result"] = np.array([r["ok"], r["no_more"], r["n_inliers"]], np.int32)
        out[f"s{k}_meta"] = np.array([n1, ninl, seed, 950 + k], np.int64)
    np.savez_compressed(os.path.join(HERE, "sim3_traces.npz"), **out)
    print("golden fixtures written")


def poseopt():
    import oracle_lib as ol
    from rsc import synth
    cases = [(11, 300, 0.8, 0.0), (12, 50, 0.6, 0.2), (13, 9, 1.0, 0.0), (14, 1500, 0.5, 0.1), (15, 120, 0.95, 0.0)]
    out = {"seeds": [], "ns": [], "ratios": [], "no_mp": [], "n_good": [], "T": [], "stats": []}
    for seed, n, ratio, nomp in cases:
        f = synth.make_poseopt_frame(np.random.default_rng(seed), n, ratio, no_mp_frac=nomp)
        r, T, o, st = ol.pose_optimization(f)
        for k, v in zip(["seeds", "ns", "ratios", "no_mp", "n_good", "T", "stats"],
                        [seed, n, ratio, nomp, r, T.reshape(16), st]):
            out[k].append(v)
    np.savez_compressed(os.path.join(HERE, "poseopt_traces.npz"), **{k: np.array(v) for k, v in out.items()})


BOW_FIELDS = ("desc", "angle", "valid", "node_id", "node_begin", "feat")


def bow():
    import oracle_lib as ol
    from rsc import synth
    # (seed, nA, nB, overlap, flips, frame overload, nnratio, check orientation)
    cases = [(21, 300, 400, 0.6, 15.0, True, 0.75, True), (22, 400, 300, 0.5, 25.0, False, 0.75, True),
             (23, 1200, 1000, 0.4, 20.0, True, 0.7, True), (24, 200, 200, 0.8, 10.0, False, 0.9, False),
             (25, 60, 900, 0.9, 30.0, True, 0.6, False), (26, 900, 60, 0.3, 12.0, False, 0.6, True)]
    out = {}
    for k, (seed, na, nb, ov, fl, fv, ratio, check) in enumerate(cases):
        rng = np.random.default_rng(seed)
        A = synth.make_bow_view(rng, na, valid_frac=0.85)
        B = synth.make_bow_related(rng, A, nb, ov, rng.uniform(0, 360), mean_flips=fl)
        nm, res = ol.search_by_bow(fv, ol.OracleBow(A), ol.OracleBow(B), ratio, check)
        key = f"c{k}"
        for side, v in (("A", A), ("B", B)):
            for f in BOW_FIELDS:
                out[f"{key}_{side}_{f}"] = getattr(v, f)
        out[f"{key}_cfg"] = np.array([int(fv), int(check)], np.int32)
        out[f"{key}_ratio"] = np.float32(ratio)
        out[f"{key}_n"] = np.int32(nm)
        out[f"{key}_out"] = res
        print(key, "nmatches", nm)
    out["cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(HERE, "bow_traces.npz"), **out)


S3_FIELDS = ("kp", "octave", "desc", "cell_begin", "cell_feat", "Rcw", "tcw", "mp_state", "mp_pos", "mp_dmax",
             "mp_dmin", "mp_desc")


def sim3match():
    import oracle_lib as ol
    from rsc import synth
    out = {}
    cases = [(31, 300, 80, 0.3), (32, 600, 150, 0.5), (33, 150, 40, 0.0)]
    for k, (seed, n, extra, mf) in enumerate(cases):
        kf1, kf2, R12, t12, m12 = synth.make_sim3match_pair(np.random.default_rng(seed), n, extra, mf)
        nf, res = ol.search_by_sim3(kf1, kf2, R12, t12, m12)
        for side, v in (("A", kf1), ("B", kf2)):
            for f in S3_FIELDS:
                out[f"c{k}_{side}_{f}"] = getattr(v, f)
        out[f"c{k}_R12"], out[f"c{k}_t12"], out[f"c{k}_m12"] = R12, t12, m12
        out[f"c{k}_n"] = np.int32(nf)
        out[f"c{k}_out"] = res
        print(f"c{k} nfound", nf)
    out["cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(HERE, "sim3match_traces.npz"), **out)


def kfdb():
    import oracle_lib as ol
    import kfdb_script as ks
    out = {}
    cases = [(11, 60, 40, 300), (12, 30, 25, 150)]
    for c, (seed, n_kfs, nq, words) in enumerate(cases):
        ops = ks.make_script(seed, n_kfs=n_kfs, n_queries=nq, words=words)
        res = ks.run_script(ol.OracleKFDB(n_kfs), ops)
        ks.save_script(f"c{c}", ops, out)
        out[f"c{c}_cap"] = np.int32(n_kfs)
        out[f"c{c}_nr"] = np.int32(len(res))
        for i, r in enumerate(res):
            out[f"c{c}_r{i}"] = r
        print(f"c{c}: {len(res)} queries, candidates per query", [len(r) for r in res])
    out["cases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(HERE, "kfdb_traces.npz"), **out)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "kfdb":
        kfdb()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "sim3match":
        sim3match()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "poseopt":
        poseopt()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "bow":
        bow()
        sys.exit(0)
    main()
