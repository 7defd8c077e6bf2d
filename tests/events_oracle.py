"""Reference-order event replay on the oracle solvers (test infrastructure): the sequential
round-robin of iterate(5) calls of Tracking::Relocalization (Tracking.cpp:1239-1262) and
LoopClosing::ComputeSim3 (LoopClosing.cpp:271-286), stopping at the first candidate that returns
a pose.  Returns the per-event record of rsc.events.pack_events."""
import numpy as np

import oracle_lib as ol
from rsc import events as rev


def run_event(ev, inputs=None):
    inputs = inputs if inputs is not None else rev.event_inputs(ev)
    if ev.kind == "reloc":
        solvers = [ol.OraclePnP(sc, s) for sc, s in zip(inputs, ev.seeds)]
        for o in solvers:
            o.set_ransac_parameters(*rev.RELOC_PARAMS)
    else:
        solvers = [ol.OracleSim3(p, s) for p, s in zip(inputs, ev.seeds)]
        for o in solvers:
            o.set_ransac_parameters(*rev.LOOP_PARAMS)
    active = list(range(len(solvers)))
    rnd = 0
    while active:
        nxt = []
        for i in active:
            r = solvers[i].iterate(5)
            if r["ok"]:
                pose = np.asarray(r["T"], np.float32).ravel() if ev.kind == "reloc" else rev.sim3_pose16(r["R"], r["t"])
                return dict(winner=i, round=rnd, hypothesis=r["iterations"] - 1, n_inliers=r["n_inliers"]), pose
            if not r["no_more"]:
                nxt.append(i)
        active = nxt
        rnd += 1
    return dict(winner=-1, round=-1, hypothesis=-1, n_inliers=0), np.zeros(16, np.float32)


def run_event_shared(ev, seed: int = 1, inputs=None):
    """The event on the reference's ONE process-global rand() stream (Q3, Random.cpp:47-50): srand(seed)
    (1 = the reference's unseeded state), then the round-robin's iterate(5) calls in order, every
    candidate drawing from libc's rand() where the previous call stopped.  Returns (record, pose,
    rand() calls consumed)."""
    inputs = inputs if inputs is not None else rev.event_inputs(ev)
    if ev.kind == "reloc":
        solvers = [ol.OraclePnP(sc, 1) for sc in inputs]
        for o in solvers:
            o.set_ransac_parameters(*rev.RELOC_PARAMS)
    else:
        solvers = [ol.OracleSim3(p, 1) for p in inputs]
        for o in solvers:
            o.set_ransac_parameters(*rev.LOOP_PARAMS)
    per = (rev.RELOC_PARAMS[3] if ev.kind == "reloc" else 3)
    for o in solvers:
        o.use_libc_rand()
    ol.libc_srand(seed)
    active = list(range(len(solvers)))
    rnd, used = 0, 0
    while active:
        nxt = []
        for i in active:
            before = solvers[i].info()["iterations"]
            r = solvers[i].iterate(5)
            used += (solvers[i].info()["iterations"] - before) * per
            if r["ok"]:
                pose = np.asarray(r["T"], np.float32).ravel() if ev.kind == "reloc" else rev.sim3_pose16(r["R"], r["t"])
                return dict(winner=i, round=rnd, hypothesis=r["iterations"] - 1, n_inliers=r["n_inliers"]), pose, used
            if not r["no_more"]:
                nxt.append(i)
        active = nxt
        rnd += 1
    return dict(winner=-1, round=-1, hypothesis=-1, n_inliers=0), np.zeros(16, np.float32), used


def run_events(evs):
    recs, poses = [], []
    for ev in evs:
        r, p = run_event(ev)
        recs.append(r)
        poses.append(p)
    return rev.pack_events([ev.eid for ev in evs], recs, poses)


class PackedEvents:
    """The inputs of a list of same-kind events packed once for the oracle's C event runners
    (ora_reloc_events_batch / ora_loop_events_batch): the CPU baseline of config 5 and a second,
    C-level replay of the reference order."""

    def __init__(self, evs, inputs=None):
        assert len({ev.kind for ev in evs}) == 1
        self.kind = evs[0].kind
        self.eids = [ev.eid for ev in evs]
        inputs = inputs if inputs is not None else [rev.event_inputs(ev) for ev in evs]
        flat = [x for xs in inputs for x in xs]
        self.ev_begin = np.concatenate([[0], np.cumsum([len(ev.sizes) for ev in evs])]).astype(np.int32)
        self.seeds = np.array([s for ev in evs for s in ev.seeds], np.uint32)
        if self.kind == "reloc":
            self.n = np.array([sc.n for sc in flat], np.int32)
            self.p2d = np.ascontiguousarray(np.concatenate([sc.p2d for sc in flat]), np.float32)
            self.p3d = np.ascontiguousarray(np.concatenate([sc.p3dw for sc in flat]), np.float32)
            self.s2 = np.ascontiguousarray(np.concatenate([sc.sigma2 for sc in flat]), np.float32)
            self.K = (flat[0].fx, flat[0].fy, flat[0].cx, flat[0].cy)
        else:
            self.n = np.array([p.n1 for p in flat], np.int32)
            cat = lambda f, dt: np.ascontiguousarray(np.concatenate([f(p) for p in flat]), dt)
            self.valid = cat(lambda p: p.valid.astype(np.uint8), np.uint8)
            self.Xw1 = cat(lambda p: p.Xw1, np.float32)
            self.Xw2 = cat(lambda p: p.Xw2, np.float32)
            self.s1 = cat(lambda p: p.sigma2_1, np.float32)
            self.s2 = cat(lambda p: p.sigma2_2, np.float32)
            self.poses = np.ascontiguousarray(np.stack([np.concatenate([
                np.asarray(p.R1, np.float32).ravel(), np.asarray(p.t1, np.float32),
                np.asarray(p.R2, np.float32).ravel(), np.asarray(p.t2, np.float32),
                np.asarray(p.K1, np.float32), np.asarray(p.K2, np.float32)]) for p in flat]), np.float32)
        self.off = np.concatenate([[0], np.cumsum(self.n)[:-1]]).astype(np.int64)
        self.rec = np.zeros((len(evs), 4), np.int32)
        self.T = np.zeros((len(evs), 16), np.float32)

    def run(self, nthreads: int = 1):
        L = ol.lib()
        ne = len(self.eids)
        if self.kind == "reloc":
            L.ora_reloc_events_batch(ne, self.ev_begin, self.n, self.off, self.p2d, self.p3d, self.s2, *self.K,
                                     self.seeds, *rev.RELOC_PARAMS, nthreads, self.rec.reshape(-1),
                                     self.T.reshape(-1))
        else:
            L.ora_loop_events_batch(ne, self.ev_begin, self.n, self.off, self.valid, self.Xw1, self.Xw2, self.s1,
                                    self.s2, self.poses.reshape(-1), self.seeds, *rev.LOOP_PARAMS, nthreads,
                                    self.rec.reshape(-1), self.T.reshape(-1))
        return self

    def records(self) -> np.ndarray:
        per = [dict(winner=r[0], round=r[1], hypothesis=r[2], n_inliers=r[3]) for r in self.rec]
        return rev.pack_events(self.eids, per, self.T)


# ---- Gated events: the reference's post-RANSAC acceptance test (rsc_*_events_gated) -------------
GATE_NONE, GATE_MATCH, GATE_HANDOFF = 0, 1, 2


def _frame_for(sc, inliers, T, u_right, bf):
    """mCurrentFrame as PoseOptimization sees it after a candidate's success (Tracking.cpp:1268-1284):
    mvpMapPoints[j] = the candidate's match where vbInliers[j], else NULL; mTcw = the RANSAC pose."""
    import types
    nf = sc.n_points
    has = np.zeros(nf, np.uint8)
    uv = np.zeros((nf, 2), np.float32)
    Xw = np.zeros((nf, 3), np.float32)
    inv = np.zeros(nf, np.float32)
    sel = np.asarray(inliers, bool)[sc.kp_index]
    j = sc.kp_index[sel]
    has[j] = 1
    uv[j] = sc.p2d[sel]
    Xw[j] = sc.p3dw[sel]
    inv[j] = (np.float32(1.0) / sc.sigma2[sel]).astype(np.float32)
    return types.SimpleNamespace(n=nf, has_mp=has, uv=uv, Xw=Xw, inv_sigma2=inv, fx=sc.fx, fy=sc.fy, cx=sc.cx,
                                 cy=sc.cy, Tcw=np.asarray(T, np.float32).reshape(4, 4), u_right=u_right,
                                 bf=np.float32(bf))


def run_reloc_gated(scenes, seeds, u_right, bf, params=rev.RELOC_PARAMS):
    """Tracking::Relocalization's round-robin (Tracking.cpp:1239-1335) on the oracle: iterate(5) per live
    candidate, and on a pose PoseOptimization on the Frame; nGood < 10 continues with the next
    candidate, >= 50 matches, in between hands off to SearchByProjection.  Returns the record of
    rsc_reloc_gate_result (status, winner, round, hypothesis, n_inliers, n_good, rejected, gates, Tcw,
    outlier mask, vbInliers)."""
    solvers = [ol.OraclePnP(sc, int(s)) for sc, s in zip(scenes, seeds)]
    for o in solvers:
        o.set_ransac_parameters(*params)
    rec = dict(status=GATE_NONE, winner=-1, round=-1, hypothesis=-1, n_inliers=0, n_good=0, rejected=0, gates=0,
               Tcw=np.zeros(16, np.float32), outlier=None, inliers=None)
    active = list(range(len(solvers)))
    rnd = 0
    while active:
        nxt = []
        for i in active:
            r = solvers[i].iterate(5)
            if not r["no_more"]:
                nxt.append(i)
            if not r["ok"]:
                continue
            f = _frame_for(scenes[i], r["inliers"], r["T"], u_right, bf)
            n_good, T, outl, _ = ol.pose_optimization(f)
            rec["gates"] += 1
            if n_good < 10:
                rec["rejected"] += 1
                continue
            rec.update(status=GATE_MATCH if n_good >= 50 else GATE_HANDOFF, winner=i, round=rnd,
                       hypothesis=r["iterations"] - 1, n_inliers=r["n_inliers"], n_good=n_good,
                       Tcw=np.asarray(T, np.float32).ravel(), outlier=np.where(f.has_mp == 1, outl, 0).astype(np.uint8),
                       inliers=np.asarray(r["inliers"], np.uint8))
            return rec
        active = nxt
        rnd += 1
    return rec


def inv_level_sigma2():
    """mvInvLevelSigma2 = 1.0f / (scale * scale) in float (ORBextractor)."""
    from rsc import synth
    s = synth.scale_factors()
    return (np.float32(1.0) / (s * s)).astype(np.float32)


def sim3opt_problem_from_kfs(kf1, kf2, m12, R, t):
    """Optimizer::OptimizeSim3(pKF1, pKF2, vpMatches1, gScm, 10) inputs (Optimizer.cpp:1108-1171) from the
    KeyFrame views and vpMatches1 as KF2 indices; gScm = g2o::Sim3(R.cast<double>(), t.cast<double>(), 1)."""
    import types
    from rsc import synth
    inv = inv_level_sigma2()
    m = np.asarray(m12)
    y = np.maximum(m, 0)
    valid = (m >= 0) & (kf1.mp_state == 1) & (kf2.mp_state[y] == 1)
    S0 = np.concatenate([synth.quat_from_R(np.asarray(R, np.float32).astype(np.float64)),
                         np.asarray(t, np.float32).astype(np.float64), [1.0]])
    K = np.array([kf1.fx, kf1.fy, kf1.cx, kf1.cy], np.float32)
    p = synth.Sim3OptProblem(valid=valid.astype(np.uint8), X1w=np.ascontiguousarray(kf1.mp_pos, np.float32),
                             X2w=np.ascontiguousarray(kf2.mp_pos[y], np.float32),
                             uv1=np.ascontiguousarray(kf1.kp, np.float32), uv2=np.ascontiguousarray(kf2.kp[y], np.float32),
                             inv1=inv[kf1.octave], inv2=inv[kf2.octave[y]], R1w=kf1.Rcw, t1w=kf1.tcw, R2w=kf2.Rcw,
                             t2w=kf2.tcw, S0=S0, R12_true=None, t12_true=None, inlier_true=None, K1=K, K2=K.copy(),
                             th2=10.0)
    return p


def run_loop_gated(kf1, cands, seeds, params=rev.LOOP_PARAMS):
    """LoopClosing::ComputeSim3's round-robin (LoopClosing.cpp:268-329) on the oracle: iterate(5) per live
    candidate; on a Sim3, SearchBySim3(7.5) over the RANSAC inliers, OptimizeSim3(10), accepted when
    nInliers >= 20.  cands = [(kf2, matches12, Sim3Pair)].  Returns the record of rsc_loop_gate_result
    (+ the accepted candidate's matches as KF2 indices)."""
    solvers = [ol.OracleSim3(p, int(s)) for (_, _, p), s in zip(cands, seeds)]
    for o in solvers:
        o.set_ransac_parameters(*params)
    rec = dict(status=GATE_NONE, winner=-1, round=-1, hypothesis=-1, n_inliers=0, n_found=0, n_opt_inliers=0,
               rejected=0, S=np.zeros(8), matches=None)
    active = list(range(len(solvers)))
    rnd = 0
    while active:
        nxt = []
        for i in active:
            r = solvers[i].iterate(5)
            if r["no_more"]:
                pass
            else:
                nxt.append(i)
            if not r["ok"]:
                continue
            kf2, m12, _ = cands[i]
            matched = np.where(np.asarray(r["inliers"], bool), m12, -1).astype(np.int32)
            nf, out12 = ol.search_by_sim3(kf1, kf2, r["R"], r["t"], matched, 7.5)
            vp = np.where(out12 >= 0, out12, matched).astype(np.int32)
            p = sim3opt_problem_from_kfs(kf1, kf2, vp, r["R"], r["t"])
            n_in, S, keep, _ = ol.optimize_sim3(p)
            if n_in < 20:
                rec["rejected"] += 1
                continue
            rec.update(status=GATE_MATCH, winner=i, round=rnd, hypothesis=r["iterations"] - 1,
                       n_inliers=r["n_inliers"], n_found=nf, n_opt_inliers=n_in, S=S,
                       matches=np.where(keep == 1, vp, -1).astype(np.int32))
            return rec
        active = nxt
        rnd += 1
    return rec
