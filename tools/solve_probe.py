#!/usr/bin/env python3
"""Diagnostic: per-phase wall clock of the config-2 hypothesis solve across all workgroups, from
rsc_diag_solve_phase_stamps (a library built with RSC_SOLVE_STAMPS=1: make -C tools solve_stamps_lib,
RSC_LIBRSC=tools/bin/librsc_solvestamps.so).  Eigen stage: per workgroup (20 hypotheses) the
phases sample + MtM / tridiagonal / Q / chase + store; betas stage: per wave (64 hypotheses, one
approximation) L + rho / find_betas / Gauss-Newton / row loads / R and t / hand-off, by
approximation.  Times in us (10 ns ticks), median / 90th percentile / max over workgroups, and
the spread of the workgroups' start and end times within the launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
from rsc import engine, workloads as wl  # noqa: E402

ctx = engine.Context(0)
if len(sys.argv) > 1 and sys.argv[1] == "event":
    # the bench's single relocalization event (bench.py latency_event: C = 15, N ~ U[300, 900]): its
    # first round is the launch whose stamps remain (rows-form eigen stage)
    from rsc import events as rev
    rng = np.random.default_rng(4242)
    C = 15
    sizes = [int(x) for x in rng.integers(300, 901, size=C)]
    ratios = [float(x) for x in rng.choice([0.05, 0.2, 0.6, 0.8], size=C, p=[0.5, 0.2, 0.15, 0.15])]
    ev = rev.Event("reloc", 100000, sizes, ratios, [7 + c for c in range(C)])
    eb = engine.EventBatch([[engine.PnPSolver(ctx, x, s) for x, s in zip(rev.event_inputs(ev), ev.seeds)]])
    for _ in range(3):
        eb.batch.reset(np.array(ev.seeds, np.uint32))
        eb.batch.set_ransac_parameters(*rev.RELOC_PARAMS)
        eb.batch.iterate_raw(5)  # round 0 of the event: every candidate's first iterate(5)
    print("single relocalization event, round 0 (rows-form eigen stage)")
else:
    scenes = wl.config2_scenes()
    batch = engine.SolverBatch([engine.PnPSolver(ctx, sc, 1) for sc in scenes])
    for s in range(3):
        batch.reset(wl.config2_seeds(s))
        batch.set_ransac_parameters(*wl.RELOC)
        batch.iterate_raw(300)
st = np.zeros(3 * 4096 * 8, np.uint64)
engine._check(engine.load_library().rsc_diag_solve_phase_stamps(ctx.h, st, st.size), "solve stamps")
st = st.reshape(3, 4096, 8).astype(np.int64)


def stats(x):
    return f"med {np.median(x):7.2f}  p90 {np.percentile(x, 90):7.2f}  max {x.max():7.2f}"


e = st[0][st[0][:, 0] > 0]
t0 = min(e[:, 0].min(), st[1][st[1][:, 0] > 0][:, 0].min() if (st[1][:, 0] > 0).any() else e[:, 0].min())
print(f"eigen stage: {len(e)} workgroups; start spread {(e[:, 0].max() - e[:, 0].min()) / 100:.2f} us, "
      f"launch span {(e[:, 4].max() - e[:, 0].min()) / 100:.2f} us")
for k, name in enumerate(["sample + MtM", "tridiagonal", "Q accumulate", "chase + store"]):
    print(f"  {name:14s} {stats(np.diff(e[:, k:k + 2], axis=1)[:, 0] / 100)}")
print(f"  {'total':14s} {stats((e[:, 4] - e[:, 0]) / 100)}")
b = st[1][st[1][:, 0] > 0]
apx = b[:, 7] & 255
print(f"betas stage: {len(b)} waves; start spread {(b[:, 0].max() - b[:, 0].min()) / 100:.2f} us, "
      f"launch span {(b[:, 6].max() - b[:, 0].min()) / 100:.2f} us (first eig start -> last betas hand-off "
      f"{(b[:, 6].max() - t0) / 100:.2f} us)")
for a in range(3):
    ba = b[apx == a]
    print(f" approximation {a + 1}: {len(ba)} waves")
    for k, name in enumerate(["L + rho", "find_betas", "Gauss-Newton", "row loads", "R and t", "hand-off"]):
        print(f"  {name:14s} {stats(np.diff(ba[:, k:k + 2], axis=1)[:, 0] / 100)}")
    print(f"  {'total':14s} {stats((ba[:, 6] - ba[:, 0]) / 100)}")
j = st[2][st[2][:, 0] > 0]
if len(j):
    print("find_betas' Jacobi SVD (from the L + rho stamp of the same wave):")
    for k in (4, 3, 5):
        jj = j[j[:, 3] == k]
        if not len(jj):
            continue
        idx = np.flatnonzero((st[2][:, 0] > 0) & (st[2][:, 3] == k))
        fb0 = st[1][idx, 1]  # find_betas entry
        print(f" k = {k}: {len(jj)} waves")
        for name, x in [("QR precond.", jj[:, 0] - fb0), ("U formed", jj[:, 1] - jj[:, 0]),
                        ("Jacobi sweeps", jj[:, 2] - jj[:, 1]), ("solve + betas", st[1][idx, 2] - jj[:, 2])]:
            print(f"  {name:14s} {stats(x / 100)}")

