"""The N > 1 product path on the GPU: two fresh rank processes (world size 2, both driving device 0,
gloo collectives — the one-GPU stand-in for RCCL over xGMI) each run their shard THROUGH librsc
(relocalization candidates, config-3 Sim3 pairs and config-4 MLPnP candidates by cost-balanced
contiguous blocks; config-5 events whole, LPT), then all-gather the fixed-size records.  A world-1
process group with the nccl backend (RCCL) runs the same all-gather on device tensors.  The gathered records must equal a single-process librsc run and
the oracle bit for bit (sharding changes no arithmetic)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rsc import dist as rdist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scenes():
    from rsc import synth
    rng = np.random.default_rng(321)
    return [synth.make_pnp_scene(rng, int(rng.integers(200, 1500)), float(rng.uniform(0.35, 0.75)))
            for _ in range(12)]


def _pairs():
    from rsc import synth
    rng = np.random.default_rng(654)
    return [synth.make_sim3_pair(rng, int(rng.integers(150, 700)), int(rng.integers(10, 200))) for _ in range(6)]


def _ml_scenes():
    from rsc import synth
    rng = np.random.default_rng(987)
    return [synth.make_pnp_scene(rng, int(rng.integers(100, 900)), float(rng.uniform(0.3, 0.8))) for _ in range(6)]


def _run_sim3(ctx, pairs, idx, with_masks=False):
    from rsc import engine
    solvers = [engine.Sim3Solver(ctx, pairs[c], 1 + c) for c in idx]
    if not solvers:
        return []
    b = engine.SolverBatch(solvers)
    b.set_ransac_parameters(0.99, 20, 300)
    return b.iterate(300, with_masks=with_masks)


def _run_mlpnp(ctx, scenes, idx):
    from rsc import engine
    solvers = [engine.MLPnPSolver(ctx, scenes[c], 1 + c) for c in idx]
    if not solvers:
        return []
    b = engine.SolverBatch(solvers)
    b.set_ransac_parameters(0.99, 10, 300, 6, 0.5, 5.991)
    return b.iterate(300)


def _events():
    from rsc import events as rev
    return rev.make_event_stream(seed=17, n_reloc=10, n_loop=4)


F_N, N1 = 1300, 600  # common vbInliers lengths: the Frame's keypoints / the KeyFrame's matches


def _mask_scenes():
    from rsc import synth
    rng = np.random.default_rng(77)
    return [synth.make_pnp_scene(rng, int(rng.integers(300, 1200)), float(rng.uniform(0.65, 0.85)), n_points=F_N)
            for _ in range(7)]


def _mask_pairs():
    from rsc import synth
    rng = np.random.default_rng(78)
    return [synth.make_sim3_pair(rng, N1, int(rng.integers(60, 250))) for _ in range(6)]


def _run_pnp(ctx, scenes, idx):
    from rsc import engine
    solvers = [engine.PnPSolver(ctx, scenes[c], 1 + c) for c in idx]
    if not solvers:
        return []
    b = engine.SolverBatch(solvers)
    b.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    return b.iterate(300)


def _run_events(ctx, evs):
    from rsc import engine, events as rev
    out = []
    for kind in ("reloc", "loop"):
        sub = [ev for ev in evs if ev.kind == kind]
        if not sub:
            continue
        cls = engine.PnPSolver if kind == "reloc" else engine.Sim3Solver
        eb = engine.EventBatch([[cls(ctx, x, s) for x, s in zip(rev.event_inputs(ev), ev.seeds)] for ev in sub])
        eb.batch.set_ransac_parameters(*(rev.RELOC_PARAMS if kind == "reloc" else rev.LOOP_PARAMS))
        eb.run()
        out.append(rev.pack_events([ev.eid for ev in sub], eb.per_event, eb.winner_poses()))
    return np.concatenate(out) if out else np.zeros((0, rev.EVENT_RECORD), np.float32)


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist
    from rsc import dist as rd, engine, events as rev
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = engine.Context(0)
    scenes = _scenes()
    lo, hi = rd.shard_range(len(scenes), world, rank, cost=[s.n for s in scenes])
    rec = rd.pack_pnp(list(range(lo, hi)), _run_pnp(ctx, scenes, range(lo, hi)))
    allr = rd.all_gather_records(dist, rec, max_per_rank=len(scenes))
    evs = _events()
    mine = rev.shard_events([ev.cost for ev in evs], world)[rank]
    erec = _run_events(ctx, [evs[i] for i in mine])
    alle = rev.all_gather_events(dist, erec, max_per_rank=len(evs))
    # configs 3 and 4 (bench.py run_sim3 / run_mlpnp): contiguous blocks by N, one all-gather each
    pairs = _pairs()
    lo3, hi3 = rd.shard_range(len(pairs), world, rank, cost=[p.n1 for p in pairs])
    s3 = rd.all_gather_records(dist, rd.pack_sim3(list(range(lo3, hi3)), _run_sim3(ctx, pairs, range(lo3, hi3))),
                               max_per_rank=len(pairs))
    mls = _ml_scenes()
    lo4, hi4 = rd.shard_range(len(mls), world, rank, cost=[m.n for m in mls])
    m4 = rd.all_gather_records(dist, rd.pack_pnp(list(range(lo4, hi4)), _run_mlpnp(ctx, mls, range(lo4, hi4))),
                               max_per_rank=len(mls))
    # the winner's vbInliers in the same all-gather: relocalization candidates in
    # parity mode (Refine successes) — the mask of the rank's local candidate fetched after a raw
    # iterate with rsc_pnp_last_inliers — and loop-closure pairs (masks from iterate)
    ps = _mask_scenes()
    lo5, hi5 = rd.shard_range(len(ps), world, rank, cost=[s.n for s in ps])
    sol = [engine.PnPSolver(ctx, ps[c], 1 + c) for c in range(lo5, hi5)]
    b = engine.SolverBatch(sol)
    b.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    rec5 = rd.pack_pnp(list(range(lo5, hi5)), b.iterate_raw(300))
    c5 = rd.local_reloc_candidate(rec5)
    r5, k5 = rd.all_gather_records_and_mask(dist, rec5, len(ps), c5,
                                            sol[c5 - lo5].last_inliers() if c5 >= 0 else None, F_N)
    pp = _mask_pairs()
    lo6, hi6 = rd.shard_range(len(pp), world, rank)
    res6 = _run_sim3(ctx, pp, range(lo6, hi6), with_masks=True)
    rec6 = rd.pack_sim3(list(range(lo6, hi6)), res6)
    c6 = rd.local_loop_candidate(rec6)
    r6, k6 = rd.all_gather_records_and_mask(dist, rec6, len(pp), c6,
                                            res6[c6 - lo6]["inliers"] if c6 >= 0 else None, N1)
    q.put((rank, hi - lo, len(mine), allr, alle, hi3 - lo3, s3, hi4 - lo4, m4, r5, k5, r6, k6))
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


def test_world2_librsc_shards_match_single_process_and_oracle():
    from gpu_common import ctx
    import events_oracle as eo
    import oracle_lib as ol
    sp = mp.get_context("spawn")
    q = sp.Queue()
    port = _free_port()
    procs = [sp.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    scenes, evs = _scenes(), _events()
    assert all(g[1] > 0 and g[2] > 0 for g in got)  # both ranks had work
    single = rdist.pack_pnp(list(range(len(scenes))), _run_pnp(ctx(), scenes, range(len(scenes))))
    single_ev = _run_events(ctx(), evs)
    for g in got:  # every rank holds the full gathered result
        allr, alle = g[3], g[4]
        assert np.array_equal(allr.view(np.uint32), single.view(np.uint32))
        assert np.array_equal(alle.view(np.uint32), single_ev.view(np.uint32))
    # and the single-process run is the oracle's
    ora = []
    for c, sc in enumerate(scenes):
        o = ol.OraclePnP(sc, 1 + c)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        ora.append(o.iterate(300))
    assert np.array_equal(single.view(np.uint32), rdist.pack_pnp(list(range(len(scenes))), ora).view(np.uint32))
    assert np.array_equal(single_ev.view(np.uint32), eo.run_events(evs).view(np.uint32))
    assert rdist.reloc_winner(single) == rdist.reloc_winner(got[0][3])
    # configs 3 / 4: both ranks ran a block, every rank holds all records, equal to one process and
    # to the oracle
    pairs, mls = _pairs(), _ml_scenes()
    assert all(g[5] > 0 and g[7] > 0 for g in got)
    s3_single = rdist.pack_sim3(list(range(len(pairs))), _run_sim3(ctx(), pairs, range(len(pairs))))
    m4_single = rdist.pack_pnp(list(range(len(mls))), _run_mlpnp(ctx(), mls, range(len(mls))))
    for g in got:
        assert np.array_equal(g[6].view(np.uint32), s3_single.view(np.uint32))
        assert np.array_equal(g[8].view(np.uint32), m4_single.view(np.uint32))
    o3, o4 = [], []
    for c, p in enumerate(pairs):
        o = ol.OracleSim3(p, 1 + c)
        o.set_ransac_parameters(0.99, 20, 300)
        o3.append(o.iterate(300))
    for c, sc in enumerate(mls):
        o = ol.OracleMLPnP(sc, 1 + c)
        o.set_ransac_parameters(0.99, 10, 300, 6, 0.5, 5.991)
        o4.append(o.iterate(300))
    assert np.array_equal(s3_single.view(np.uint32), rdist.pack_sim3(list(range(len(pairs))), o3).view(np.uint32))
    assert np.array_equal(m4_single.view(np.uint32), rdist.pack_pnp(list(range(len(mls))), o4).view(np.uint32))
    # the winner's mask in the exchange: every rank holds it, equal to one process and the oracle
    ps, pp = _mask_scenes(), _mask_pairs()
    ora5 = []
    for c, sc in enumerate(ps):
        o = ol.OraclePnP(sc, 1 + c)
        o.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
        ora5.append(o.iterate(300))
    w5 = rdist.reloc_winner(rdist.pack_pnp(list(range(len(ps))), ora5))
    ora6 = []
    for c, p in enumerate(pp):
        o = ol.OracleSim3(p, 1 + c)
        o.set_ransac_parameters(0.99, 20, 300)
        ora6.append(o.iterate(300))
    rec6_ora = rdist.pack_sim3(list(range(len(pp))), ora6)
    w6 = rdist.local_loop_candidate(rec6_ora)
    assert w5 >= 0 and w6 >= 0
    from rsc import engine
    b5 = engine.SolverBatch([engine.PnPSolver(ctx(), sc, 1 + c) for c, sc in enumerate(ps)])
    b5.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    single5 = b5.iterate(300, with_masks=True)
    for g in got:
        r5, k5, r6, k6 = g[9], g[10], g[11], g[12]
        assert np.array_equal(r5.view(np.uint32), rdist.pack_pnp(list(range(len(ps))), ora5).view(np.uint32))
        assert rdist.reloc_winner(r5) == w5
        assert np.array_equal(k5[w5], ora5[w5]["inliers"]) and np.array_equal(k5[w5], single5[w5]["inliers"])
        assert np.array_equal(r6.view(np.uint32), rec6_ora.view(np.uint32))
        assert rdist.local_loop_candidate(r6) == w6
        assert w6 in k6 and k6[w6].sum() == ora6[w6]["n_inliers"] > 0
        assert np.array_equal(k6[w6], ora6[w6]["inliers"])


def _rccl_worker(port, q):
    """World-1 RCCL (backend "nccl"): the config-2 result records through all_gather_into_tensor on
    device tensors, as bench.py's N > 1 step does over xGMI."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "orb-slam2-optimized_amd"))
    import torch
    import torch.distributed as dist
    from rsc import dist as rd, engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ctx = engine.Context(0)
    scenes = _scenes()
    rec = rd.pack_pnp(list(range(len(scenes))), _run_pnp(ctx, scenes, range(len(scenes))))
    allr = rd.all_gather_records(dist, rec, max_per_rank=len(scenes) + 3, device="cuda")
    q.put((dist.get_backend(), allr, rec))
    dist.destroy_process_group()
    ctx.close()


def test_world1_rccl_all_gather_of_records():
    sp = mp.get_context("spawn")
    q = sp.Queue()
    p = sp.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    backend, allr, rec = q.get(timeout=240)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert backend == "nccl"
    assert np.array_equal(allr.view(np.uint32), rec.view(np.uint32))
