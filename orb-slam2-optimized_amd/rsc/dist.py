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


def local_reloc_candidate(records: np.ndarray) -> int:
    """The candidate of this rank's contiguous block that can be the relocalization winner of the
    RANSAC stage: its lowest-index successful one (Tracking.cpp:1241-1265), or -1.

    Limitation: the reference moves on to the next successful candidate when PoseOptimization of
    the winner keeps fewer than 50 inliers (Tracking.cpp:1284-1331).  Only the winner's vbInliers is
    exchanged, so a caller that needs that fallback gathers the next candidate's mask with
    successful_candidates() / a second all_gather_records_and_mask."""
    ok = records[records[:, 1] > 0] if len(records) else records
    return int(ok[0, 0]) if len(ok) else -1


def local_loop_candidate(records: np.ndarray, exclude=()) -> int:
    """The loop-closure winner among this rank's candidates: smallest (round, c) with round =
    (hypothesis of the first success) // 5 (LoopClosing.cpp:271-327), or -1.  ``exclude`` drops
    candidates already rejected by the OptimizeSim3 gate (< 20 inliers, LoopClosing.cpp:311-324), so
    a second exchange finds the next one the reference's loop would reach."""
    ok = records[records[:, 1] > 0] if len(records) else records
    hyp = {int(r[0]): int(r[4]) - 1 for r in ok if int(r[0]) not in exclude}
    return loop_winner(hyp) if hyp else -1


def successful_candidates(records: np.ndarray, kind: str = "reloc") -> list:
    """Every successful candidate of a record block in the order the reference's event loop visits
    them: index order for relocalization (Tracking.cpp:1241-1331), (round, c) for loop closure
    (LoopClosing.cpp:271-327).  The fallback order after a rejected winner."""
    ok = records[records[:, 1] > 0] if len(records) else records
    if kind == "reloc":
        return [int(r[0]) for r in ok]
    return [c for _, c in sorted(((int(r[4]) - 1) // 5, int(r[0])) for r in ok)]


def all_gather_records_and_mask(dist, records: np.ndarray, max_per_rank: int, local_cand: int, local_mask,
                                mask_len: int, device=None):
    """The records all-gather of all_gather_records plus the winner's inlier vector in the SAME
    collective (the winner's bitset as the optional second payload).

    Every rank appends the vbInliers of its own candidate that can win (local_reloc_candidate /
    local_loop_candidate; -1 for none) as a bitset of mask_len bits — the length is common to all
    candidates of an event: F.N for relocalization (PnPsolver vbInliers, PnPsolver.hpp:31), mN1 for
    loop closure (Sim3Solver.cpp:116).  After the gather every rank holds the global winner's
    vbInliers and can run PoseOptimization (Tracking.cpp:1271-1284) or SearchBySim3
    (LoopClosing.cpp:300-309) itself.  One fixed-size int32 payload per rank:
    [max_per_rank x RECORD float32 bit patterns | candidate | words of the bitset].

    Returns (records sorted by candidate, {candidate: bool[mask_len]} for every rank's entry)."""
    import torch
    world = dist.get_world_size()
    words = (mask_len + 31) // 32
    per = max_per_rank * RECORD + 1 + words
    buf = np.full(per, -1, np.int32)
    pad = np.full((max_per_rank, RECORD), -1.0, np.float32)
    pad[:len(records)] = records
    buf[:max_per_rank * RECORD] = pad.view(np.int32).ravel()
    buf[max_per_rank * RECORD] = local_cand
    bits = np.zeros(words * 32, np.uint8)
    if local_cand >= 0:
        m = np.asarray(local_mask, bool)
        assert len(m) == mask_len
        bits[:mask_len] = m
    buf[max_per_rank * RECORD + 1:] = np.packbits(bits, bitorder="little").view(np.int32)
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * per, dtype=torch.int32, device=t.device)
    dist.all_gather_into_tensor(out, t)
    allb = out.cpu().numpy().reshape(world, per)
    recs = allb[:, :max_per_rank * RECORD].copy().view(np.float32).reshape(-1, RECORD)
    recs = recs[recs[:, 0] >= 0]
    recs = recs[np.argsort(recs[:, 0], kind="stable")]
    masks = {}
    for r in range(world):
        c = int(allb[r, max_per_rank * RECORD])
        if c >= 0:
            w = allb[r, max_per_rank * RECORD + 1:].copy().view(np.uint8)
            masks[c] = np.unpackbits(w, bitorder="little")[:mask_len].astype(bool)
    return recs, masks


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
