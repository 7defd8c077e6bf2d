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


def run_events(evs):
    recs, poses = [], []
    for ev in evs:
        r, p = run_event(ev)
        recs.append(r)
        poses.append(p)
    return rev.pack_events([ev.eid for ev in evs], recs, poses)
