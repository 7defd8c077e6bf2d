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
