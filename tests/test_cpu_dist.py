"""N>1 path on CPU: world_size-2 gloo ranks shard relocalization candidates, run their solvers
(here: the oracle, since there is no GPU), all-gather the fixed-size records and pick the winner;
the result must equal the single-process run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rsc import dist as rdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scenes():
    from rsc import synth
    rng = np.random.default_rng(123)
    return [synth.make_pnp_scene(rng, int(rng.integers(60, 400)), float(rng.uniform(0.3, 0.8))) for _ in range(7)]


def _solve(idx, scenes):
    import oracle_lib as ol
    out = []
    for c in idx:
        o = ol.OraclePnP(scenes[c], 1 + c)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        out.append(o.iterate(300))
    return out


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist
    from rsc import dist as rd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scenes = _scenes()
    lo, hi = rd.shard_range(len(scenes), world, rank, cost=[s.n for s in scenes])
    res = _solve(range(lo, hi), scenes)
    rec = rd.pack_pnp(list(range(lo, hi)), res)
    allr = rd.all_gather_records(dist, rec, max_per_rank=len(scenes))
    if rank == 0:
        q.put((allr, rd.reloc_winner(allr)))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers():
    for world in (1, 2, 3, 8):
        for n in (0, 1, 5, 64):
            cover = []
            for r in range(world):
                lo, hi = rdist.shard_range(n, world, r)
                cover += list(range(lo, hi))
            assert cover == list(range(n))
            cost = np.arange(1, n + 1)
            cover = []
            for r in range(world):
                lo, hi = rdist.shard_range(n, world, r, cost=cost if n else None)
                cover += list(range(lo, hi))
            assert cover == list(range(n))


def test_loop_winner_round_robin_order():
    # candidate 2 succeeds at h=3 (round 0) beats candidate 0 at h=7 (round 1)
    assert rdist.loop_winner({0: 7, 1: -1, 2: 3}) == 2
    assert rdist.loop_winner({0: 4, 2: 3}) == 0
    assert rdist.loop_winner({0: -1}) == -1


def test_gloo_world2_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    allr, win = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    scenes = _scenes()
    single = rdist.pack_pnp(list(range(len(scenes))), _solve(range(len(scenes)), scenes))
    assert np.array_equal(allr, single)
    assert win == rdist.reloc_winner(single)


def _events_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist
    import events_oracle as eo
    from rsc import events as rev
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    evs = rev.make_event_stream(seed=13, n_reloc=8, n_loop=3)
    mine = rev.shard_events([ev.cost for ev in evs], world)[rank]
    rec = eo.run_events([evs[i] for i in mine])
    allr = rev.all_gather_events(dist, rec, max_per_rank=len(evs))
    if rank == 0:
        q.put((allr, mine))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_events_partition_and_balance():
    from rsc import events as rev
    evs = rev.make_event_stream()
    assert len(evs) == 170 and sum(ev.kind == "loop" for ev in evs) == 20
    costs = [ev.cost for ev in evs]
    for world in (1, 2, 4, 8):
        parts = rev.shard_events(costs, world)
        assert sorted(i for p in parts for i in p) == list(range(len(evs)))
        loads = [sum(costs[i] for i in p) for p in parts]
        assert max(loads) <= sum(costs) / world + max(costs)  # LPT bound


def test_gloo_world2_events_match_single_process():
    import events_oracle as eo
    from rsc import events as rev
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_events_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    allr, mine = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    evs = rev.make_event_stream(seed=13, n_reloc=8, n_loop=3)
    assert 0 < len(mine) < len(evs)
    single = eo.run_events(evs)
    assert np.array_equal(allr.view(np.uint32), single.view(np.uint32))


F_N = 1300  # keypoints of the current Frame: the common length of every candidate's vbInliers


def _mask_scenes():
    from rsc import synth
    rng = np.random.default_rng(77)
    # parity mode (>= 60 % inliers): several candidates succeed, with Refine
    return [synth.make_pnp_scene(rng, int(rng.integers(300, 1200)), float(rng.uniform(0.65, 0.85)), n_points=F_N)
            for _ in range(7)]


def _mask_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist
    from rsc import dist as rd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scenes = _mask_scenes()
    lo, hi = rd.shard_range(len(scenes), world, rank, cost=[s.n for s in scenes])
    res = _solve(range(lo, hi), scenes)
    rec = rd.pack_pnp(list(range(lo, hi)), res)
    c = rd.local_reloc_candidate(rec)
    mask = res[c - lo]["inliers"] if c >= 0 else None
    allr, masks = rd.all_gather_records_and_mask(dist, rec, len(scenes), c, mask, F_N)
    q.put((rank, c, allr, masks))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_winner_mask_in_the_exchange():
    """The winner's vbInliers travels in the records all-gather: after it, EVERY rank
    holds the relocalization winner's mask, equal to the single-process run's (Tracking.cpp:1271-1284
    can run on any rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mask_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=120) for _ in range(2)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    scenes = _mask_scenes()
    res = _solve(range(len(scenes)), scenes)
    single = rdist.pack_pnp(list(range(len(scenes))), res)
    win = rdist.reloc_winner(single)
    assert win >= 0
    for rank, c, allr, masks in got:
        assert np.array_equal(allr, single)
        assert rdist.reloc_winner(allr) == win
        assert win in masks and np.array_equal(masks[win], res[win]["inliers"])
        assert masks[win].sum() == res[win]["n_inliers"]
    assert sum(g[1] >= 0 for g in got) >= 1


def test_mask_exchange_packing_round_trip():
    """Single process, world 1 gloo: odd mask lengths, no local candidate, all-ones masks."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(3)
        for n in (1, 31, 32, 33, 1999, 2000):
            rec = np.zeros((3, rdist.RECORD), np.float32)
            rec[:, 0] = [4, 5, 6]
            rec[1, 1] = 1
            m = rng.random(n) < 0.5
            allr, masks = rdist.all_gather_records_and_mask(dist, rec, 5, 5, m, n)
            assert np.array_equal(allr, rec) and np.array_equal(masks[5], m)
            allr, masks = rdist.all_gather_records_and_mask(dist, rec, 5, -1, None, n)
            assert masks == {}
            allr, masks = rdist.all_gather_records_and_mask(dist, rec, 5, 6, np.ones(n, bool), n)
            assert masks[6].all() and len(masks[6]) == n
        assert rdist.local_reloc_candidate(rec) == 5
        rec2 = rec.copy()
        rec2[:, 1] = 1
        rec2[:, 4] = [12, 4, 9]  # first successes at hypotheses 11, 3, 8 -> rounds 2, 0, 1
        assert rdist.local_loop_candidate(rec2) == 5
        # the fallback order after a rejected winner (LoopClosing.cpp:311-324, Tracking.cpp:1284-1331)
        assert rdist.successful_candidates(rec2, "loop") == [5, 6, 4]
        assert rdist.local_loop_candidate(rec2, exclude={5}) == 6
        assert rdist.successful_candidates(rec2, "reloc") == [4, 5, 6]
    finally:
        dist.destroy_process_group()


N1 = 600  # matches of the current KeyFrame: the common length of every loop candidate's vbInliers


def _loop_pairs():
    from rsc import synth
    rng = np.random.default_rng(78)
    return [synth.make_sim3_pair(rng, N1, int(rng.integers(60, 250))) for _ in range(6)]


def _solve_sim3(idx, pairs):
    import oracle_lib as ol
    out = []
    for c in idx:
        o = ol.OracleSim3(pairs[c], 1 + c)
        o.set_ransac_parameters(0.99, 20, 300)
        out.append(o.iterate(300))
    return out


def _loop_mask_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist
    from rsc import dist as rd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pairs = _loop_pairs()
    lo, hi = rd.shard_range(len(pairs), world, rank)
    res = _solve_sim3(range(lo, hi), pairs)
    rec = rd.pack_sim3(list(range(lo, hi)), res)
    c = rd.local_loop_candidate(rec)
    allr, masks = rd.all_gather_records_and_mask(dist, rec, len(pairs), c, res[c - lo]["inliers"] if c >= 0 else None,
                                                 N1)
    q.put((rank, c, allr, masks))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_loop_winner_mask_in_the_exchange():
    """Loop closure (LoopClosing.cpp:271-309): every rank gets the records and the Sim3 winner's
    vbInliers (mN1 entries) in one all-gather; the global winner by (round, candidate) is one rank's
    local winner, and its mask equals the single-process run's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loop_mask_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=120) for _ in range(2)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pairs = _loop_pairs()
    res = _solve_sim3(range(len(pairs)), pairs)
    single = rdist.pack_sim3(list(range(len(pairs))), res)
    win = rdist.local_loop_candidate(single)
    # every pair succeeds; candidate 1 wins at round 2 ahead of candidate 0 (round 5)
    assert win == 1 and all(r["ok"] for r in res)
    for rank, c, allr, masks in got:
        assert np.array_equal(allr, single)
        assert rdist.local_loop_candidate(allr) == win
        assert win in masks and np.array_equal(masks[win], res[win]["inliers"])
        assert masks[win].sum() == res[win]["n_inliers"]
    assert all(g[1] >= 0 for g in got)  # both ranks hold a successful pair
