"""Multi-GPU layer: candidates shard across ranks, one process per GPU; the only
exchange is an all-gather of fixed-size per-candidate result records (RCCL over xGMI on MI355X,
gloo in the CPU tests), after which every rank replays the reference's selection order:

* relocalization (Tracking.cpp:1239-1334): candidates are visited in index order, so the winner of
  a round is the lowest candidate index whose iterate() succeeded;
* loop closure (LoopClosing.cpp:271-327): candidate c succeeding at hypothesis h_c is observed at
  round floor(h_c / 5); the winner is the lexicographically smallest (round, c).

Sharding changes no arithmetic: every solver owns its rand() stream (H4), so gathered records are
identical to a single-GPU run.
"""
from __future__ import annotations

import numpy as np

# record layout (float32): [candidate, ok, no_more, n_inliers, iterations, T[16] (PnP) | R[9] t[3] pad]
RECORD = 21


def shard_range(n_items: int, world: int, rank: int, cost=None) -> tuple[int, int]:
    """Contiguous block of candidates for `rank`, balanced by cost (N*H) when given."""
    if cost is None:
        base, rem = divmod(n_items, world)
        lo = rank * base + min(rank, rem)
        return lo, lo + base + (1 if rank < rem else 0)
    c = np.cumsum(np.asarray(cost, np.float64))
    total = c[-1] if len(c) else 0.0
    bounds = [0] + [int(np.searchsorted(c, total * r / world, side="right")) for r in range(1, world)] + [n_items]
    return bounds[rank], bounds[rank + 1]


def _fields(results, names):
    """Columns of per-candidate results: a numpy structured array (SolverBatch.iterate_raw, read
    without a Python loop) or a list of result dicts."""
    if isinstance(results, np.ndarray) and results.dtype.names:
        return [np.asarray(results[n]) for n in names]
    return [np.asarray([r[n] for r in results]) for n in names]


def _pack(cand_ids, results, pose_cols):
    n = len(results)
    out = np.zeros((n, RECORD), np.float32)
    if n == 0:
        return out
    ok, nm, ni, it = _fields(results, ("ok", "no_more", "n_inliers", "iterations"))
    out[:, 0] = np.asarray(cand_ids, np.float32)
    out[:, 1], out[:, 2], out[:, 3], out[:, 4] = ok, nm, ni, it
    col = 5
    for name, width in pose_cols:
        (v,) = _fields(results, (name,))
        out[:, col:col + width] = v.reshape(n, width)
        col += width
    return out


def pack_pnp(cand_ids, results) -> np.ndarray:
    """PnP / MLPnP records: [candidate, ok, no_more, n_inliers, iterations, T[16]]."""
    return _pack(cand_ids, results, (("T", 16),))


def pack_sim3(cand_ids, results) -> np.ndarray:
    """Sim3 records: [candidate, ok, no_more, n_inliers, iterations, R[9], t[3], 0 0 0 0]."""
    return _pack(cand_ids, results, (("R", 9), ("t", 3)))


def all_gather_records(dist, records: np.ndarray, max_per_rank: int, device=None) -> np.ndarray:
    """All-gather padded record blocks (one collective, fixed size) and drop the padding rows.

    `dist` is torch.distributed (backend nccl = RCCL on ROCm, or gloo); `device` is the tensor
    device for the collective (cuda for RCCL, cpu for gloo)."""
    import torch
    world = dist.get_world_size()
    pad = np.full((max_per_rank, RECORD), -1.0, np.float32)
    pad[:len(records)] = records
    t = torch.from_numpy(pad)
    if device is not None:
        t = t.to(device)
    out = torch.empty((world * max_per_rank, RECORD), dtype=torch.float32, device=t.device)
    dist.all_gather_into_tensor(out, t)
    allr = out.cpu().numpy()
    allr = allr[allr[:, 0] >= 0]
    return allr[np.argsort(allr[:, 0], kind="stable")]


def reloc_winner(records: np.ndarray) -> int:
    """Lowest candidate index whose iterate() returned true (Tracking.cpp:1241-1265), or -1."""
    ok = records[records[:, 1] > 0]
    return int(ok[0, 0]) if len(ok) else -1


def loop_winner(success_hyp: dict) -> int:
    """success_hyp: candidate -> hypothesis index of its first success (-1 if none).  The round-robin
    iterate(5) schedule observes candidate c at round h_c // 5; winner = min (round, c)."""
    best = None
    for c, h in success_hyp.items():
        if h < 0:
            continue
        key = (h // 5, c)
        if best is None or key < best:
            best = key
    return -1 if best is None else best[1]
