"""A/B of two builds of the oracle restatement on the BASELINE workloads (test infrastructure).

    python tools/oracle_ab.py dump OUT.npz [--lib PATH]      # run the workloads on one build
    python tools/oracle_ab.py compare A.npz B.npz [--json F]  # outcome agreement of two dumps

Workloads (rsc/workloads.py, rsc/events.py):
  c2x  config 2 exhaustive: 64 candidates x 2000, iterate(300) -> every hypothesis' sample, inlier
       count and float pose (19,200 hypotheses);
  c2p  config 2 parity mode (60 % inliers, Refine + early exit): the iterate(300) outcome per candidate;
  c3x  config 3 exhaustive Sim3 (32 x 1000, iterate(300)): every hypothesis' count and pose;
  c3p  config 3 parity (300 true inliers): the outcome per pair;
  c4x  config 4 MLPnP exhaustive (32 x 4096, iterate(300)): every hypothesis' count and double pose;
  c5   config 5 event stream (150 relocalization + 20 loop-closure events): winner records.

Used for: the Q19 qr_solve change (round-3 oracle vs round-4 oracle) and the arithmetic-order choice
of the 3-term fixed-size Eigen products (profiles/r04/order_choice.json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(lib):
    if lib:
        os.environ["RSC_ORACLE_LIB"] = os.path.abspath(lib)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))


def dump(out, lib=None, quick=False):
    _setup(lib)
    import oracle_lib as ol
    import events_oracle as eo
    from rsc import workloads as W, events as rev
    res = {}
    nc = 8 if quick else 64
    # c2x
    scenes = W.config2_scenes(candidates=nc)
    seeds = W.config2_seeds(0, candidates=nc)
    ints, fls, outs = [], [], []
    for sc, s in zip(scenes, seeds):
        o = ol.OraclePnP(sc, int(s))
        o.set_ransac_parameters(*W.RELOC)
        o.enable_trace()
        o.iterate(300)
        i, f = o.trace()
        ints.append(i[:, [0, 1, 2, 3, 8]])
        fls.append(f)
    res["c2x_ints"] = np.stack(ints)
    res["c2x_poses"] = np.stack(fls)
    # c2p
    scenes = W.config2_scenes(candidates=nc, ratio=W.CONFIG2["parity_ratio"], seed=20241)
    rec, Ts, masks = [], [], []
    for sc, s in zip(scenes, seeds):
        o = ol.OraclePnP(sc, int(s))
        o.set_ransac_parameters(*W.RELOC)
        r = o.iterate(300)
        rec.append([r["ok"], r["no_more"], r["n_inliers"], r["iterations"]])
        Ts.append(np.asarray(r["T"], np.float32).ravel())
        m = np.zeros(sc.n_points, np.uint8)
        m[:len(r["inliers"])] = r["inliers"]
        masks.append(m)
    res["c2p_rec"] = np.array(rec, np.int32)
    res["c2p_T"] = np.stack(Ts)
    res["c2p_masks"] = np.stack(masks)
    # c3x / c3p
    for tag, ninl in (("c3x", W.CONFIG3["exhaustive_inliers"]), ("c3p", W.CONFIG3["parity_inliers"])):
        pairs = W.config3_pairs(n_inliers=ninl, pairs=8 if quick else 32)
        seeds3 = W.step_seeds(0, len(pairs))
        ints, fls, rec, masks = [], [], [], []
        for p, s in zip(pairs, seeds3):
            o = ol.OracleSim3(p, int(s))
            o.set_ransac_parameters(*W.LOOP)
            o.enable_trace()
            r = o.iterate(300)
            i, f = o.trace()
            pad = lambda a, n: np.concatenate([a, np.zeros((n - len(a),) + a.shape[1:], a.dtype)])
            ints.append(pad(i, 300))
            fls.append(pad(f, 300))
            rec.append([r["ok"], r["no_more"], r["n_inliers"], len(i)])
            masks.append(np.asarray(r["inliers"], np.uint8))
        res[tag + "_ints"] = np.stack(ints)
        res[tag + "_poses"] = np.stack(fls)
        res[tag + "_rec"] = np.array(rec, np.int32)
        res[tag + "_masks"] = np.stack(masks)
    # c4x: config 4 MLPnP exhaustive (per GPU share 32 x 4096): every hypothesis' count and double pose
    ints, dbls = [], []
    scenes4 = W.config4_scenes(candidates=4 if quick else W.CONFIG4["candidates_per_gpu"])
    for sc, s in zip(scenes4, W.step_seeds(0, len(scenes4))):
        o = ol.OracleMLPnP(sc, int(s))
        o.set_ransac_parameters(*W.MLPNP)
        o.enable_trace()
        o.iterate(300)
        i, d = o.trace()
        ints.append(i)
        dbls.append(d)
    res["c4x_ints"] = np.stack(ints)
    res["c4x_poses"] = np.stack(dbls)
    # c5
    evs = rev.make_event_stream(n_reloc=30 if quick else 150, n_loop=6 if quick else 20)
    recs = []
    for kind in ("reloc", "loop"):
        sub = [ev for ev in evs if ev.kind == kind]
        recs.append(eo.PackedEvents(sub).run(nthreads=os.cpu_count() or 1).records())
    res["c5_records"] = np.concatenate(recs)
    np.savez_compressed(out, **res)


def _agree(a, b):
    return float(np.mean(np.all(a.reshape(len(a), -1) == b.reshape(len(b), -1), axis=1)))


def compare(a_path, b_path):
    A, B = np.load(a_path), np.load(b_path)
    rep = {}
    # per-hypothesis (exhaustive workloads)
    for tag in ("c2x", "c3x"):
        ia, ib = A[tag + "_ints"], B[tag + "_ints"]
        pa, pb = A[tag + "_poses"], B[tag + "_poses"]
        same_bits = np.all(pa.view(np.uint32) == pb.view(np.uint32), axis=-1)
        same_count = ia[..., -1] == ib[..., -1] if tag == "c2x" else ia[..., 3] == ib[..., 3]
        finite = np.isfinite(pa).all(-1) & np.isfinite(pb).all(-1)
        dpose = np.abs(pa.astype(np.float64) - pb.astype(np.float64)).max(-1)
        cc = np.argwhere(~same_count)
        rep[tag] = dict(hypotheses=int(same_bits.size), pose_bits_changed=int((~same_bits).sum()),
                        count_changed=int((~same_count).sum()),
                        count_changed_first50=[[int(a), int(b)] for a, b in cc[:50]],  # (problem, hypothesis)
                        max_abs_count_diff=int(np.abs(ia[..., -1 if tag == "c2x" else 3].astype(np.int64)
                                                      - ib[..., -1 if tag == "c2x" else 3]).max()),
                        max_abs_pose_diff=float(dpose[finite].max()) if finite.any() else 0.0,
                        pose_within_1em4=float(np.mean(dpose[finite] <= 1e-4)) if finite.any() else 1.0,
                        count_agreement=float(np.mean(same_count)))
    for tag in ("c2p", "c3p"):
        ra, rb = A[tag + "_rec"], B[tag + "_rec"]
        ma, mb = A[tag + "_masks"], B[tag + "_masks"]
        d = dict(problems=int(len(ra)), outcome_agreement=_agree(ra, rb), mask_agreement=_agree(ma, mb))
        bad = ~np.all(ra == rb, axis=1) | ~np.all(ma.reshape(len(ma), -1) == mb.reshape(len(mb), -1), axis=1)
        d["mismatching_problems"] = [int(i) for i in np.flatnonzero(bad)]
        d["records_a_b"] = {int(i): [ra[i].tolist(), rb[i].tolist()] for i in np.flatnonzero(bad)}
        if tag == "c2p":
            Ta, Tb = A["c2p_T"], B["c2p_T"]
            dT = np.abs(Ta.astype(np.float64) - Tb).max(-1)
            d["pose_bits_agreement"] = _agree(Ta.view(np.uint32), Tb.view(np.uint32))
            d["pose_within_1em4"] = float(np.mean(dT <= 1e-4))
            d["max_abs_pose_diff"] = float(dT.max())
            d["median_abs_pose_diff_of_mismatches"] = float(np.median(dT[bad])) if bad.any() else 0.0
        rep[tag] = d
    if "c4x_ints" in A and "c4x_ints" in B:
        ia, ib = A["c4x_ints"], B["c4x_ints"]
        pa, pb = A["c4x_poses"], B["c4x_poses"]
        same_bits = np.all(pa.view(np.uint64) == pb.view(np.uint64), axis=-1)
        same_count = ia[..., 8] == ib[..., 8]
        finite = np.isfinite(pa).all(-1) & np.isfinite(pb).all(-1)
        dpose = np.abs(pa - pb).max(-1)
        rep["c4x"] = dict(hypotheses=int(same_bits.size), pose_bits_changed=int((~same_bits).sum()),
                          count_changed=int((~same_count).sum()), count_agreement=float(np.mean(same_count)),
                          max_abs_count_diff=int(np.abs(ia[..., 8].astype(np.int64) - ib[..., 8]).max()),
                          max_abs_pose_diff=float(dpose[finite].max()) if finite.any() else 0.0,
                          pose_within_1em4=float(np.mean(dpose[finite] <= 1e-4)) if finite.any() else 1.0)
    ea, eb = A["c5_records"], B["c5_records"]
    same = np.all(ea[:, :5] == eb[:, :5], axis=1)
    rep["c5"] = dict(events=int(len(ea)), winner_record_agreement=float(same.mean()),
                     pose_within_1em4=float(np.mean(np.abs(ea[:, 5:] - eb[:, 5:]).max(-1) <= 1e-4)),
                     pose_bits_agreement=_agree(ea[:, 5:].view(np.uint32), eb[:, 5:].view(np.uint32)),
                     mismatching_events=[int(e) for e in ea[~same, 0]])
    return rep


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["dump", "compare"])
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--lib")
    ap.add_argument("--json")
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    if a.mode == "dump":
        dump(a.paths[0], a.lib, a.quick)
    else:
        rep = compare(a.paths[0], a.paths[1])
        txt = json.dumps(rep, indent=1)
        print(txt)
        if a.json:
            open(a.json, "w").write(txt + "\n")
