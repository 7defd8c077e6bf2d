#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock of the PnP refine kernel in the config-5 event stream (the
launch with the most refine jobs), from rsc_diag_refine_phase_stamps (a library built with
RSC_REFINE_STAMPS=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
from rsc import engine, events as rev  # noqa: E402

ctx = engine.Context(0)
evs = [ev for ev in rev.make_event_stream() if ev.kind == "reloc"]
solvers = [[engine.PnPSolver(ctx, x, s) for x, s in zip(rev.event_inputs(ev), ev.seeds)] for ev in evs]
eb = engine.EventBatch(solvers)
seeds = np.array([s for ev in evs for s in ev.seeds], np.uint32)
names = ["compaction", "ctrl pts", "MtM", "eigen", "betas", "check", "exit"]
for rep in range(2):
    eb.batch.reset(seeds)
    eb.batch.set_ransac_parameters(*rev.RELOC_PARAMS)
    eb.run()
st = np.zeros(64 * 24, np.uint64)
engine._check(engine.load_library().rsc_diag_refine_phase_stamps(ctx.h, st, st.size), "refine stamps")
st = st.reshape(64, 24).astype(np.int64)
ok = st[:, 0] > 0
d = np.diff(st[ok][:, :8], axis=1) / 100.0
print(f"jobs stamped: {ok.sum()}  total us: mean {((st[ok, 6] - st[ok, 0]) / 100.0).mean():.1f} "
      f"max {((st[ok, 6] - st[ok, 0]) / 100.0).max():.1f}")
for i, n in enumerate(names[:6]):
    print(f"  {n:10s} mean {d[:, i].mean():8.1f} us  max {d[:, i].max():8.1f} us")
if (st[ok, 8] > 0).all():  # eigen sub-phases (RSC_REFINE_STAMPS builds)
    e = np.diff(np.concatenate([st[ok][:, 3:4], st[ok][:, 8:12], st[ok][:, 4:5]], axis=1), axis=1) / 100.0
    for i, n in enumerate(["tridiag", "accumulate", "QR chase", "eigvecs", "L + rho"]):
        print(f"    eigen/{n:10s} mean {e[:, i].mean():8.1f} us  max {e[:, i].max():8.1f} us")
