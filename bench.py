#!/usr/bin/env python3
"""Headline benchmark: RANSAC hypotheses/s (+ poses/s) of the relocalization EPnP batch.

Workload (BASELINE.json configs[1]): per GPU, 64 relocalization
candidates x 2000 correspondences, SetRansacParameters(0.99,10,300,4,0.5,5.991) (Tracking.cpp:1226)
then iterate(300) on every candidate — 300 hypotheses each (Q1: '||' loop) in exhaustive mode
(40% inliers, minInliers=1000 unreachable), i.e. 19,200 hypotheses per step, all candidates in one
rsc_pnp_iterate_many call.  A "step" = reset every solver with a fresh rand() seed + the call above
(sampling, EPnP solves, inlier scans, selection replay, result records).  With N GPUs (one process
per GPU, torchrun) every rank runs its own 64-candidate batch (weak scaling) and the per-candidate
result records are all-gathered over RCCL at the end of each step.

The Sim3 loop-closure batch (config 3: 32 pairs x 1000 matches, iterate(300)) is measured in the
same run and reported under "sim3".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

RELOC = (0.99, 10, 300, 4, 0.5, 5.991)
LOOP = (0.99, 20, 300)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X vector FP64 (spec)
PROFILE_DIR = "profiles/r01"


def _profile_json(name):
    """Committed measurement side files (op-count, PMC traffic) of this round, or None."""
    path = os.path.join(ROOT, PROFILE_DIR, name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--candidates", type=int, default=64)
    p.add_argument("--corrs", type=int, default=2000)
    p.add_argument("--iters", type=int, default=300)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-sim3", action="store_true")
    p.add_argument("--no-mlpnp", action="store_true")
    p.add_argument("--no-events", action="store_true")
    p.add_argument("--no-poseopt", action="store_true")
    p.add_argument("--no-bow", action="store_true")
    p.add_argument("--no-sim3match", action="store_true")
    p.add_argument("--no-kfdb", action="store_true")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local, dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def pnp_batch(rng, C, N, ratio):
    from rsc import synth
    return [synth.make_pnp_scene(rng, N, ratio) for _ in range(C)]


def run_pnp(engine, ctx, scenes, args, dist, rank, world):
    solvers = [engine.PnPSolver(ctx, sc, 1) for sc in scenes]
    batch = engine.SolverBatch(solvers)
    C = len(solvers)
    gather = None
    if dist is not None:
        import torch
        rec = torch.zeros(C, 20, dtype=torch.float32, device="cuda")
        gather = (torch, rec, torch.zeros(world * C, 20, dtype=torch.float32, device="cuda"))

    seeds = np.zeros(C, np.uint32)
    h = np.zeros((C, 20), np.float32)

    def step(s):
        seeds[:] = 1 + np.arange(C) + C * (s + 1000 * rank)
        batch.reset(seeds)
        batch.set_ransac_parameters(*RELOC)
        outs = batch.iterate_raw(args.iters)
        if gather is not None:
            torch, rec, allrec = gather
            h[:, 0], h[:, 1], h[:, 2], h[:, 3] = outs["ok"], outs["no_more"], outs["n_inliers"], outs["iterations"]
            h[:, 4:20] = outs["T"].reshape(C, 16)
            rec.copy_(torch.from_numpy(h))
            dist.all_gather_into_tensor(allrec, rec)  # RCCL over xGMI: winner records of all ranks
            torch.cuda.synchronize()
        return int(outs["iterations"].sum()), outs

    for s in range(args.warmup):
        step(s)
    # Timed region 1 (the metric): K steps, no instrumentation in the queue.
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    hyps = 0
    for s in range(args.steps):
        n, outs = step(args.warmup + s)
        hyps += n
    ctx.synchronize()
    barrier(dist)
    dt = time.perf_counter() - t0
    # Timed region 2 (roofline): the same K steps with HIP events around the kernels on the
    # context stream (eigen stage, betas, scan); events add gaps, so this pass is not the metric.
    ctx.enable_timing(True)
    solve_ms = scan_ms = eig_ms = 0.0
    launches = 0
    barrier(dist)
    ctx.synchronize()
    t1 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + args.steps + s)
        tm = ctx.last_timing()
        solve_ms += tm["solve_ms"]
        scan_ms += tm["scan_ms"]
        eig_ms += tm["eig_ms"]
        launches += tm["solve_launches"]
    ctx.synchronize()
    barrier(dist)
    dt_inst = time.perf_counter() - t1
    ctx.enable_timing(False)
    return dict(seconds=dt, seconds_instrumented=dt_inst, hyps=hyps, problems=C * args.steps,
                solve_ms=solve_ms / max(launches, 1),
                scan_ms=scan_ms / max(launches, 1), eig_ms=eig_ms / max(launches, 1), launches=launches, last=outs)


def run_sim3(engine, ctx, rng, args):
    from rsc import synth
    pairs = [synth.make_sim3_pair(rng, 1000, 15) for _ in range(32)]
    solvers = [engine.Sim3Solver(ctx, p, 1) for p in pairs]
    batch = engine.SolverBatch(solvers)

    def step(s):
        batch.reset(1 + np.arange(32) + 32 * s)
        batch.set_ransac_parameters(*LOOP)
        return int(batch.iterate_raw(args.iters)["iterations"].sum())

    for s in range(args.warmup):
        step(s)
    ctx.synchronize()
    t0 = time.perf_counter()
    h = 0
    for s in range(args.steps):
        h += step(args.warmup + s)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    return dict(hyp_per_s=h / dt, ms_per_step=1e3 * dt / args.steps, hypotheses_per_step=h // args.steps,
                pairs=32, correspondences=1000)


def run_mlpnp(engine, ctx, rng, args):
    """Config 4 on one GPU: 32 candidates x 4096 correspondences, MLPnP SetRansacParameters
    (0.99,10,300,6,0.5,5.991) (commented call Tracking.cpp:1227-1228), iterate(300), exhaustive."""
    from rsc import synth
    scenes = [synth.make_pnp_scene(rng, 4096, 0.4) for _ in range(32)]
    batch = engine.SolverBatch([engine.MLPnPSolver(ctx, sc, 1) for sc in scenes])

    def step(s):
        batch.reset(1 + np.arange(32) + 32 * s)
        batch.set_ransac_parameters(0.99, 10, 300, 6, 0.5, 5.991)
        return int(batch.iterate_raw(args.iters)["iterations"].sum())

    for s in range(args.warmup):
        step(s)
    ctx.synchronize()
    steps = max(1, args.steps // 4)
    t0 = time.perf_counter()
    h = 0
    for s in range(steps):
        h += step(args.warmup + s)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    return dict(hyp_per_s=h / dt, ms_per_step=1e3 * dt / steps, hypotheses_per_step=h // steps, candidates=32,
                correspondences=4096, steps=steps)


def run_events(engine, ctx, args, dist, rank, world):
    """Config 5: the EuRoC-MH01-shaped event stream (150 relocalization + 20 loop events, seed-fixed
    sizes), whole events sharded across ranks by cost (LPT), each event run with the reference's
    iterate(5) round-robin (rsc_reloc_events / rsc_loop_events: all candidates of all local events in
    the same launches), then ONE all-gather of the per-event winner records (RCCL over xGMI).
    A step = reset + SetRansacParameters of every candidate + both drivers + the all-gather."""
    from rsc import events as rev
    evs = rev.make_event_stream()
    mine = rev.shard_events([ev.cost for ev in evs], world)[rank]
    groups = {"reloc": [], "loop": []}
    for i in mine:
        ev = evs[i]
        cls = engine.PnPSolver if ev.kind == "reloc" else engine.Sim3Solver
        groups[ev.kind].append((ev, [cls(ctx, x, s) for x, s in zip(rev.event_inputs(ev), ev.seeds)]))
    drivers = []
    for kind, params in (("reloc", rev.RELOC_PARAMS), ("loop", rev.LOOP_PARAMS)):
        if groups[kind]:
            eb = engine.EventBatch([g[1] for g in groups[kind]])
            seeds = np.array([s for ev, _ in groups[kind] for s in ev.seeds], np.uint32)
            drivers.append((eb, params, seeds, [ev.eid for ev, _ in groups[kind]]))
    max_per_rank = max(len(p) for p in rev.shard_events([ev.cost for ev in evs], world))

    def step():
        recs, hyps = [], 0
        for eb, params, seeds, eids in drivers:
            eb.batch.reset(seeds)
            eb.batch.set_ransac_parameters(*params)
            eb.run()
            hyps += int(eb.cand["iterations"].sum())
            recs.append(rev.pack_events(eids, eb.per_event, eb.winner_poses()))
        rec = np.concatenate(recs) if recs else np.zeros((0, rev.EVENT_RECORD), np.float32)
        if dist is not None:
            rec = rev.all_gather_events(dist, rec, max_per_rank, device="cuda")
        return hyps, rec

    for _ in range(args.warmup):
        step()
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    hyps = 0
    for _ in range(args.steps):
        h, rec = step()
        hyps += h
    ctx.synchronize()
    barrier(dist)
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt, float(hyps)], dtype=torch.float64, device="cuda")
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, hyps = float(t[0]), int(t[1])
    n_ev = len(evs) * args.steps
    return dict(events_per_s=n_ev / dt, ms_per_stream=1e3 * dt / args.steps, hyp_per_s=hyps / dt,
                events=len(evs), candidates=sum(len(ev.sizes) for ev in evs),
                resolved=int((rec[:, 1] >= 0).sum()),
                sharding=f"{world} rank(s), LPT by N*300, RCCL all-gather of {rev.EVENT_RECORD}-float records")


def poseopt_frames(rng, F=64, N=2000, ratio=0.8):
    from rsc import synth
    return [synth.make_poseopt_frame(rng, N, ratio) for _ in range(F)]


def run_poseopt(engine, ctx, frames, args):
    """Optimizer::PoseOptimization (Optimizer.cpp:205-424) on a batch of Frames
    (64 x 2000 map-point matches, 80 % inliers, start pose perturbed like a RANSAC estimate), one
    rsc_pose_optimization_many call per step; kernel time from HIP events in a second pass."""
    batch = engine.PoseOptBatch(ctx, frames)

    def step():
        batch.run()

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    steps = max(1, args.steps // 2)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    dt = time.perf_counter() - t0
    res = batch.results()
    ctx.enable_timing(True)
    kms = 0.0
    for _ in range(steps):
        step()
        kms += ctx.last_timing()["refine_ms"]
    ctx.enable_timing(False)
    its = sum(r["lm_iterations"] for r in res)
    trials = sum(r["lm_trials"] for r in res)
    F = len(frames)
    return dict(poses_per_s=F * steps / dt, ms_per_step=1e3 * dt / steps, kernel_ms=kms / steps, frames=F,
                edges_per_frame=frames[0].n, lm_iterations_per_frame=its / F, lm_trials_per_frame=trials / F,
                steps=steps)


def bow_views(rng, C=64, N=2000):
    """Relocalization-shaped SearchByBoW input: the current Frame (N features) and C candidate
    KeyFrames sharing 10-70 % of its features (Tracking.cpp:1207-1214)."""
    from rsc import synth
    F = synth.make_bow_view(rng, N)
    kfs = [synth.make_bow_related(rng, F, N, float(rng.uniform(0.1, 0.7)), float(rng.uniform(0, 360)),
                                  mean_flips=float(rng.uniform(8, 30))) for _ in range(C)]
    return F, kfs


def bow_comparisons(F, kfs):
    """Descriptor comparisons the reference's SearchByBoW(pKF, F) walk can make: sum over common
    nodes of (#valid KF features) x (#Frame features) — an upper bound (matched Frame features are
    skipped)."""
    fsz = dict(zip(F.node_id.tolist(), np.diff(F.node_begin).tolist()))
    tot = 0
    for k in kfs:
        for j, nid in enumerate(k.node_id.tolist()):
            if nid in fsz:
                tot += int(k.valid[k.feat[k.node_begin[j]:k.node_begin[j + 1]]].sum()) * fsz[nid]
    return tot


def run_bow(engine, ctx, F, kfs, args):
    """ORBmatcher::SearchByBoW(pKF, F) of 64 candidate KeyFrames against the
    current Frame (2000 features each, ORBmatcher(0.75, true) as in Tracking.cpp:1212), views
    resident in HBM; one rsc_search_by_bow_frame_many per step."""
    gF = engine.BowView(ctx, F)
    gK = [engine.BowView(ctx, k) for k in kfs]
    batch = engine.BowSearch(ctx, gF, gK, True, 0.75, True)
    for _ in range(args.warmup):
        batch.run()
    ctx.synchronize()
    steps = max(1, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, nm = batch.run()
    ctx.synchronize()
    dt = time.perf_counter() - t0
    ctx.enable_timing(True)
    kms = 0.0
    for _ in range(steps):
        batch.run()
        kms += ctx.last_timing()["refine_ms"]
    ctx.enable_timing(False)
    kms /= steps
    cmp = bow_comparisons(F, kfs)
    C = len(kfs)
    # algorithmic bytes per launch: every descriptor row of both views once (32 B) + angle (4 B) +
    # FeatureVector index (4 B) + validity (1 B) per feature, + the int32 output vector
    algo = C * (F.n + kfs[0].n) * 41 + C * F.n * 4
    return dict(pairs_per_s=C * steps / dt, ms_per_step=1e3 * dt / steps, kernel_ms=kms, pairs=C,
                features=F.n, comparisons_per_pair=cmp / C, comparisons_per_s=cmp / (kms * 1e-3) if kms else None,
                mean_matches=float(np.mean(nm)), algorithmic_bytes_per_launch=algo,
                hbm_frac=(algo / (kms * 1e-3) / 1e9) / HBM_PEAK_GBS if kms else None, steps=steps)


def cpu_baseline_bow(F, kfs, seconds):
    """The SearchByBoW oracle (std::map FeatureVector walk, as the reference) on ONE host core."""
    import ctypes
    import oracle_lib as ol
    L = ol.lib()
    oF = ol.OracleBow(F)
    oK = [ol.OracleBow(k) for k in kfs]
    C = len(kfs)
    hs = (ctypes.c_void_p * C)(*[o.h for o in oK])
    out = np.zeros((C, F.n), np.int32)
    nm = np.zeros(C, np.int32)
    done = 0
    t0 = time.perf_counter()
    while True:
        L.ora_search_by_bow_many(1, C, hs, oF.h, 0.75, 1, out.reshape(-1), F.n, nm)
        done += C
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=round(done / dt, 2), unit="pairs/s", cores=1, kind="port",
                sample=f"{done // C} batches of {C} KeyFrame x Frame searches ({F.n} features) in {dt:.1f} s, "
                       "oracle restatement, 1 thread")


def run_sim3match(engine, ctx, probs, args):
    """SURVEY §8(f) rank 3 (first half): ORBmatcher::SearchBySim3 (ORBmatcher.cpp:948-1170) on 32
    loop-closure pairs (config-3 shape: ~1000 MapPoints per KeyFrame, 30 % already matched by the
    Sim3 RANSAC), th = 7.5 as LoopClosing.cpp:309; one rsc_search_by_sim3_many per step (inputs
    packed and uploaded in the call)."""
    batch = engine.Sim3Search(ctx, probs, 7.5)
    for _ in range(args.warmup):
        batch.run()
    steps = max(1, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, nf = batch.run()
    dt = time.perf_counter() - t0
    ctx.enable_timing(True)
    kms = 0.0
    for _ in range(steps):
        batch.run()
        kms += ctx.last_timing()["refine_ms"]
    ctx.enable_timing(False)
    C = len(probs)
    pts = sum(p[0].n + p[1].n for p in probs)
    return dict(pairs_per_s=C * steps / dt, ms_per_step=1e3 * dt / steps, kernel_ms=kms / steps, pairs=C,
                points_per_pair=pts / C, mean_new_matches=float(np.mean(nf)), steps=steps)


def cpu_baseline_sim3match(probs, seconds):
    """The SearchBySim3 oracle on ONE host core over the same pairs (inputs marshalled once)."""
    import ctypes
    import oracle_lib as ol
    from rsc import engine
    L = ol.lib()
    prepared = []
    for kf1, kf2, R12, t12, m12 in probs:
        k1, keep1 = engine.sim3_kf_struct(kf1)
        k2, keep2 = engine.sim3_kf_struct(kf2)
        prepared.append((k1, k2, keep1, keep2, np.ascontiguousarray(m12, np.int32),
                         np.ascontiguousarray(np.asarray(R12, np.float32).reshape(9)),
                         np.ascontiguousarray(np.asarray(t12, np.float32).reshape(3)),
                         np.zeros(max(kf1.n, 1), np.int32)))
    done = 0
    t0 = time.perf_counter()
    while True:
        for k1, k2, _, _, m12, R, t, out in prepared:
            L.ora_search_by_sim3(ctypes.addressof(k1), ctypes.addressof(k2), m12, R, t, 7.5, out)
        done += len(probs)
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=round(done / dt, 2), unit="pairs/s", cores=1, kind="port",
                sample=f"{done // len(probs)} batches of {len(probs)} KeyFrame pairs in {dt:.1f} s, oracle "
                       "restatement, 1 thread")


def kfdb_scene(seed=82, n_kfs=2000, n_queries=64):
    """a 2000-KeyFrame database (600-word BowVectors, a long EuRoC/KITTI map)
    and 64 relocalization queries (Frame BowVectors observed along the trajectory)."""
    from rsc import synth
    rng = np.random.default_rng(seed)
    sc = synth.make_kfdb_scene(rng, n_kfs, words_per_kf=600)
    queries = [synth.make_kfdb_query(rng, sc, rng.uniform(0, n_kfs - 1)) for _ in range(n_queries)]
    return sc, queries


def run_kfdb(engine, ctx, sc, queries, args):
    """KeyFrameDatabase::DetectRelocalizationCandidates (KeyFrameDatabase.cpp:174-283) over the
    resident database: one rsc_kfdb_detect_relocalization per query (query upload, four kernels,
    candidates back), fresh Frame ids every step so every query walks the full path."""
    n = len(sc.bows)
    db = engine.KeyFrameDatabase(ctx, n)
    for k in range(n):
        db.add(k, *sc.bows[k])
        db.set_covisibility(k, sc.covis[k])
    fid = [1]

    def step():
        nc = 0
        for ids, vals in queries:
            nc += len(db.detect_relocalization(fid[0], ids, vals))
            fid[0] += 1
        return nc
    for _ in range(args.warmup):
        step()
    steps = max(1, args.steps)
    t0 = time.perf_counter()
    nc = 0
    for _ in range(steps):
        nc += step()
    dt = time.perf_counter() - t0
    ctx.enable_timing(True)
    kms = 0.0
    for ids, vals in queries:
        db.detect_relocalization(fid[0], ids, vals)
        fid[0] += 1
        kms += ctx.last_timing()["refine_ms"]
    ctx.enable_timing(False)
    Q = len(queries)
    words = sum(len(b[0]) for b in sc.bows)
    return dict(queries_per_s=Q * steps / dt, ms_per_query=1e3 * dt / (Q * steps), kernel_ms_per_query=kms / Q,
                keyframes=n, words_per_keyframe=words / n, mean_candidates=nc / (Q * steps),
                count_kernel_bytes=4 * words, steps=steps)


def cpu_baseline_kfdb(sc, queries, seconds):
    """The KeyFrameDatabase oracle on ONE host core, same database and queries."""
    import oracle_lib as ol
    n = len(sc.bows)
    db = ol.OracleKFDB(n)
    for k in range(n):
        db.add(k, *sc.bows[k])
        db.set_covisibility(k, sc.covis[k])
    prepared = [(np.ascontiguousarray(i, np.uint32), np.ascontiguousarray(v, np.float64)) for i, v in queries]
    done, fid = 0, 1
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for ids, vals in prepared:
            db.detect_relocalization(fid, ids, vals)
            fid += 1
        done += len(prepared)
    dt = time.perf_counter() - t0
    return dict(value=round(done / dt, 2), unit="queries/s", cores=1, kind="port",
                sample=f"{done} DetectRelocalizationCandidates queries on a {n}-KeyFrame database in {dt:.1f} s, "
                       "oracle restatement, 1 thread")


def cpu_baseline_poseopt(frames, seconds):
    """The PoseOptimization oracle on ONE host core over the same frames."""
    import oracle_lib as ol
    L = ol.lib()
    F = len(frames)
    n = np.array([f.n for f in frames], np.int64)
    off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    uv = np.ascontiguousarray(np.concatenate([f.uv for f in frames]), np.float32)
    Xw = np.ascontiguousarray(np.concatenate([f.Xw for f in frames]), np.float32)
    inv = np.ascontiguousarray(np.concatenate([f.inv_sigma2 for f in frames]), np.float32)
    T = np.ascontiguousarray(np.stack([f.Tcw.reshape(16) for f in frames]), np.float32).reshape(-1)
    To = np.zeros(16 * F, np.float32)
    outl = np.zeros(int(off[-1]), np.uint8)
    good = np.zeros(F, np.int32)
    f0 = frames[0]
    done = 0
    t0 = time.perf_counter()
    while True:
        L.ora_pose_optimization_batch(F, off, uv, Xw, inv, f0.fx, f0.fy, f0.cx, f0.cy, T, To, outl, good)
        done += F
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=round(done / dt, 2), unit="poses/s", cores=1, kind="port",
                sample=f"{done // F} batches of {F} Frames x {f0.n} edges in {dt:.1f} s, oracle restatement, 1 thread")


def cpu_baseline(scenes, args):
    """Oracle restatement (test infrastructure) of the same workload on ONE host core."""
    import oracle_lib as ol
    L = ol.lib()
    C = len(scenes)
    n = np.array([sc.n for sc in scenes], np.int32)
    off = np.concatenate([[0], np.cumsum(n)[:-1]]).astype(np.int64)
    p2d = np.ascontiguousarray(np.concatenate([sc.p2d for sc in scenes]), np.float32)
    p3d = np.ascontiguousarray(np.concatenate([sc.p3dw for sc in scenes]), np.float32)
    s2 = np.ascontiguousarray(np.concatenate([sc.sigma2 for sc in scenes]), np.float32)
    out_i4 = np.zeros(4 * C, np.int32)
    out_T = np.zeros(16 * C, np.float32)
    sc0 = scenes[0]
    hyps = 0
    batches = 0
    t0 = time.perf_counter()
    while True:
        seeds = (1 + np.arange(C) + C * batches).astype(np.uint32)
        L.ora_pnp_run_batch(C, n, off, p2d, p3d, s2, sc0.fx, sc0.fy, sc0.cx, sc0.cy, seeds, *RELOC, args.iters,
                            1, out_i4, out_T, None)
        hyps += int(out_i4.reshape(C, 4)[:, 3].sum())
        batches += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return dict(value=hyps / dt, unit="hypotheses/s", cores=1, kind="port",
                sample=f"{batches} full batches ({C} candidates x {sc0.n} corrs x iterate({args.iters})) "
                       f"= {hyps} hypotheses in {dt:.1f} s, oracle restatement, 1 thread")


def main():
    args = parse()
    world, rank, local, dist = dist_setup(args)
    from rsc import engine
    ctx = engine.Context(local)
    rng = np.random.default_rng(20240 + rank)
    scenes = pnp_batch(rng, args.candidates, args.corrs, 0.4)
    r = run_pnp(engine, ctx, scenes, args, dist, rank, world)
    # max over ranks of the timed region
    dt = r["seconds"]
    hyps_total = r["hyps"]
    if dist is not None:
        import torch
        t = torch.tensor([dt, float(r["hyps"])], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt = float(mx[0])
        hyps_total = int(t[1])
    events = None if args.no_events else run_events(engine, ctx, args, dist, rank, world)
    sim3 = mlpnp = None
    if rank == 0 and not args.no_sim3:
        sim3 = run_sim3(engine, ctx, np.random.default_rng(77), args)
    if rank == 0 and not args.no_mlpnp:
        mlpnp = run_mlpnp(engine, ctx, np.random.default_rng(78), args)
    poseopt = po_frames = None
    if rank == 0 and not args.no_poseopt:
        po_frames = poseopt_frames(np.random.default_rng(79))
        poseopt = run_poseopt(engine, ctx, po_frames, args)
    s3m = s3m_probs = None
    if rank == 0 and not args.no_sim3match:
        from rsc import synth
        r3 = np.random.default_rng(81)
        s3m_probs = [synth.make_sim3match_pair(r3, 1000, 250, 0.3) for _ in range(32)]
        s3m = run_sim3match(engine, ctx, s3m_probs, args)
    kfdb = kfdb_sc = kfdb_q = None
    if rank == 0 and not args.no_kfdb:
        kfdb_sc, kfdb_q = kfdb_scene()
        kfdb = run_kfdb(engine, ctx, kfdb_sc, kfdb_q, args)
    bow = bow_F = bow_K = None
    if rank == 0 and not args.no_bow:
        bow_F, bow_K = bow_views(np.random.default_rng(80))
        bow = run_bow(engine, ctx, bow_F, bow_K, args)
    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    value = hyps_total / dt
    per_launch_hyps = args.candidates * args.iters
    B_h = 24 * args.corrs  # PnP scan bytes per hypothesis (p3D 12 + p2D 8 + maxErr 4)
    algo_bytes = per_launch_hyps * B_h
    eig_ms, solve_ms, scan_ms = r["eig_ms"], r["solve_ms"], r["scan_ms"]
    set_ms = solve_ms + scan_ms
    achieved = algo_bytes / (set_ms * 1e-3) / 1e9 if set_ms > 0 else 0.0
    opc = _profile_json("opcount.json")
    traffic = _profile_json("pmc_traffic.json")
    S_h = opc["fp64_flops_mean"] if opc else None
    fp64 = None
    if S_h and solve_ms > 0:
        tf = per_launch_hyps * S_h / (solve_ms * 1e-3) / 1e12
        fp64 = {"kernel": "pnp_eig_quad_kernel<4> + pnp_betas_kernel<4> (hypothesis solve)",
                "achieved": round(tf, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / FP64_PEAK_TFLOPS, 5), "S_h_fp64_flops_per_hypothesis": S_h,
                "S_h_source": "tools/opcount.cpp (op-counter build of the oracle EPnP), " + PROFILE_DIR}
    out = {
        "metric": "RANSAC hypotheses/sec (EPnP relocalization batch, 2k corrs x 64 candidates per GPU)",
        "value": round(value, 1),
        "unit": "hypotheses/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded EuRoC-shaped scenes; no dataset)",
        "config": {"workload": "reloc_pnp: candidates x correspondences, iterate(300), exhaustive (40% inliers)",
                   "candidates_per_gpu": args.candidates, "correspondences": args.corrs,
                   "hypotheses_per_candidate": args.iters, "params": "SetRansacParameters(0.99,10,300,4,0.5,5.991)",
                   "parallelism": f"candidates sharded, {world} rank(s), RCCL all-gather of result records"},
        "poses_per_s": round(world * r["problems"] / dt, 2),
        # achieved = effective scan bandwidth of one EPnP launch set
        # (C*H hypotheses x B_h algorithmic bytes) / (HIP-event time of eig + betas + scan kernels).
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": round(traffic["epnp_launch_set_bytes"]) if traffic else None,
                     "kernel": "EPnP launch set: pnp_eig_quad_kernel<4> + pnp_betas_kernel<4> + pnp_scan_kernel<8>",
                     "ms_per_launch": {"eig": round(eig_ms, 4), "betas": round(solve_ms - eig_ms, 4),
                                       "scan": round(scan_ms, 4), "set": round(set_ms, 4)},
                     "launches": r["launches"], "algorithmic_bytes_per_launch": algo_bytes,
                     "timing": "HIP events on the context stream, second pass of the same K steps "
                               f"({1e3 * r['seconds_instrumented'] / args.steps:.4f} ms/step with events)",
                     "traffic_source": (PROFILE_DIR + "/pmc_traffic.json (2 x FETCH_SIZE + WRITE_SIZE)")
                     if traffic else None},
    }
    if fp64 is not None:
        out["roofline_fp64"] = fp64
    if sim3 is not None:
        out["sim3"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in sim3.items()}
    if events is not None:
        out["events"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in events.items()}
    if mlpnp is not None:
        out["mlpnp"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in mlpnp.items()}
    if poseopt is not None:
        out["poseopt"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in poseopt.items()}
        if not args.no_cpu and world == 1:
            cb = cpu_baseline_poseopt(po_frames, min(3.0, args.cpu_seconds))
            out["poseopt"]["cpu_baseline"] = cb
            out["poseopt"]["speedup_vs_cpu_1core"] = round(poseopt["poses_per_s"] / cb["value"], 1)
    if bow is not None:
        out["search_by_bow"] = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in bow.items()}
        if not args.no_cpu and world == 1:
            cb = cpu_baseline_bow(bow_F, bow_K, min(3.0, args.cpu_seconds))
            out["search_by_bow"]["cpu_baseline"] = cb
            out["search_by_bow"]["speedup_vs_cpu_1core"] = round(bow["pairs_per_s"] / cb["value"], 1)
    if s3m is not None:
        out["search_by_sim3"] = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in s3m.items()}
        if not args.no_cpu and world == 1:
            cb = cpu_baseline_sim3match(s3m_probs, min(2.0, args.cpu_seconds))
            out["search_by_sim3"]["cpu_baseline"] = cb
            out["search_by_sim3"]["speedup_vs_cpu_1core"] = round(s3m["pairs_per_s"] / cb["value"], 1)
    if kfdb is not None:
        out["kfdb_relocalization"] = {k: (round(v, 5) if isinstance(v, float) else v) for k, v in kfdb.items()}
        if not args.no_cpu and world == 1:
            cb = cpu_baseline_kfdb(kfdb_sc, kfdb_q, min(2.0, args.cpu_seconds))
            out["kfdb_relocalization"]["cpu_baseline"] = cb
            out["kfdb_relocalization"]["speedup_vs_cpu_1core"] = round(kfdb["queries_per_s"] / cb["value"], 1)
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(scenes, args)
        out["cpu_baseline"]["value"] = round(out["cpu_baseline"]["value"], 1)
        out["speedup_vs_cpu_1core"] = round(value / out["cpu_baseline"]["value"], 1)
    print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
