"""Config-5 event stream: EuRoC-MH01-shaped relocalization and
loop-closure events, cost-balanced sharding of whole events across ranks, and the fixed-size
per-event winner record that the ranks all-gather (RCCL over xGMI; gloo in the CPU tests).

* A relocalization event (Tracking::Relocalization, Tracking.cpp:1198-1334) is C~U[1,30]
  candidates x N~U[15,1200] correspondences (>= 15 per Tracking.cpp:1215), PnPsolver parameters
  (0.99,10,300,4,0.5,5.991) (:1226), then iterate(5) round-robin over the non-discarded
  candidates until one returns a pose (:1239-1262).
* A loop event (LoopClosing::ComputeSim3, LoopClosing.cpp:196-327) is C~U[1,4] pairs x
  N~U[20,600] matches (>= 20 per :253), Sim3Solver parameters (0.99,20,300) (:258), the same
  iterate(5) round-robin (:271-286).

Winner semantics: an event ends at the FIRST candidate whose RANSAC iterate() returns a pose.  The
reference keeps the round-robin going when that pose then fails its later gates —
PoseOptimization + SearchByProjection reaching nGood >= 50 (Tracking.cpp:1278-1330) for
relocalization, OptimizeSim3 keeping >= 20 inliers (LoopClosing.cpp:296-312) for loops — so the
records (and the throughput) equal the reference's only where the first RANSAC success also passes
those gates.  The stream measures the RANSAC stage the north star names; a caller that needs the
full gate drives the round-robin with the per-solver iterate calls and the device
PoseOptimization / OptimizeSim3 (after the event entry points).

Events are independent, so a rank processes whole events (no data-path collective); the only
exchange is one all-gather of the per-event records at the end.  Every candidate owns its rand()
stream (seed fixed by its global id), so the gathered records equal a one-rank run.
"""
from __future__ import annotations

import dataclasses

import numpy as np

RELOC_PARAMS = (0.99, 10, 300, 4, 0.5, 5.991)
LOOP_PARAMS = (0.99, 20, 300)
# record (float32): [event, winner, round, hypothesis, n_inliers, pose[16]]
EVENT_RECORD = 21


@dataclasses.dataclass
class Event:
    kind: str            # "reloc" | "loop"
    eid: int             # global event id (reloc events first, then loop events)
    sizes: list          # correspondences per candidate
    ratios: list         # true inlier fraction per candidate
    seeds: list          # srand() seed per candidate

    @property
    def cost(self) -> float:
        """Work estimate: N x (hypotheses a candidate can run)."""
        return float(sum(self.sizes)) * 300.0


def make_event_stream(seed: int = 5, n_reloc: int = 150, n_loop: int = 20) -> list:
    """Seed-fixed event sizes.  Most relocalization candidates are wrong
    keyframes (few true inliers); some are right."""
    rng = np.random.default_rng(seed)
    events = []
    for e in range(n_reloc):
        C = int(rng.integers(1, 31))
        sizes = [int(x) for x in rng.integers(15, 1201, size=C)]
        ratios = [float(x) for x in rng.choice([0.05, 0.2, 0.6, 0.8], size=C, p=[0.5, 0.2, 0.15, 0.15])]
        events.append(Event("reloc", e, sizes, ratios, [1 + 1000 * e + c for c in range(C)]))
    for e in range(n_loop):
        C = int(rng.integers(1, 5))
        sizes = [int(x) for x in rng.integers(20, 601, size=C)]
        ratios = [float(x) for x in rng.choice([0.02, 0.1, 0.3, 0.6], size=C)]
        events.append(Event("loop", n_reloc + e, sizes, ratios, [1 + 1000 * (n_reloc + e) + c for c in range(C)]))
    return events


def event_inputs(ev: Event):
    """Deterministic synthetic inputs of one event (scenes for reloc, pairs for loop)."""
    from . import synth
    rng = np.random.default_rng(1_000_003 * (ev.eid + 1))
    if ev.kind == "reloc":
        return [synth.make_pnp_scene(rng, n, r) for n, r in zip(ev.sizes, ev.ratios)]
    return [synth.make_sim3_pair(rng, n, int(round(r * n))) for n, r in zip(ev.sizes, ev.ratios)]


def shard_events(costs, world: int) -> list:
    """Longest-processing-time assignment of whole events to ranks; returns per-rank sorted id lists."""
    costs = np.asarray(costs, np.float64)
    load = np.zeros(world)
    out = [[] for _ in range(world)]
    for i in np.argsort(-costs, kind="stable"):
        r = int(np.argmin(load))
        out[r].append(int(i))
        load[r] += costs[i]
    return [sorted(x) for x in out]


def pack_events(event_ids, per_event, poses) -> np.ndarray:
    """per_event: structured records (winner, round, hypothesis, n_inliers); poses: [n, 16] float32
    (PnP Tcw, or Sim3 [R|t] rows padded) of the winning candidate (zeros when none)."""
    out = np.zeros((len(event_ids), EVENT_RECORD), np.float32)
    for i, e in enumerate(event_ids):
        out[i, 0] = e
        out[i, 1:5] = [per_event[i]["winner"], per_event[i]["round"], per_event[i]["hypothesis"],
                       per_event[i]["n_inliers"]]
        out[i, 5:21] = np.asarray(poses[i], np.float32).ravel()
    return out


def all_gather_events(dist, records: np.ndarray, max_per_rank: int, device=None) -> np.ndarray:
    """One fixed-size all-gather of padded per-event record blocks; rows sorted by event id."""
    import torch
    world = dist.get_world_size()
    pad = np.full((max_per_rank, EVENT_RECORD), -1.0, np.float32)
    pad[:len(records)] = records
    t = torch.from_numpy(pad)
    if device is not None:
        t = t.to(device)
    out = torch.empty((world * max_per_rank, EVENT_RECORD), dtype=torch.float32, device=t.device)
    dist.all_gather_into_tensor(out, t)
    allr = out.cpu().numpy()
    allr = allr[allr[:, 0] >= 0]
    return allr[np.argsort(allr[:, 0], kind="stable")]


def sim3_pose16(R, t) -> np.ndarray:
    T = np.zeros(16, np.float32)
    T[0:3], T[4:7], T[8:11] = R[0], R[1], R[2]
    T[3], T[7], T[11], T[15] = t[0], t[1], t[2], 1.0
    return T
