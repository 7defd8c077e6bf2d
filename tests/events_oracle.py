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
