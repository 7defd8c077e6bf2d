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
if len(sys.argv) > 1 and sys.argv[1] == "event":
    # the bench's single relocalization event (bench.py latency_event: C = 15, N ~ U[300, 900]): the
    # Refine jobs of ONE Tracking::Relocalization call, the latency case
    rng = np.random.default_rng(4242)
    C = 15
    sizes = [int(x) for x in rng.integers(300, 901, size=C)]
    ratios = [float(x) for x in rng.choice([0.05, 0.2, 0.6, 0.8], size=C, p=[0.5, 0.2, 0.15, 0.15])]
    evs = [rev.Event("reloc", 100000, sizes, ratios, [7 + c for c in range(C)])]
    print("single relocalization event (bench latency_event)")
else:
    evs = [ev for ev in rev.make_event_stream() if ev.kind == "reloc"]
    print("config-5 stream, the launch with the most Refine jobs")
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
if (st[ok, 12] > 0).all():  # beta-approximation waves (refine_wave_stamp: slots 12 + 4 * wave + j)
    for w in range(3):
        b = st[ok][:, 12 + 4 * w: 16 + 4 * w]
        seg = np.diff(np.concatenate([st[ok][:, 4:5], b], axis=1), axis=1) / 100.0
        print(f"  betas wave {w}: betas+GN+ccs {seg[:, 0].mean():6.1f}  pc0 {seg[:, 1].mean():5.1f}  "
              f"M+Horn {seg[:, 2].mean():5.1f}  err {seg[:, 3].mean():5.1f} us")
