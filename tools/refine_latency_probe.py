#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock of the PnP refine kernel in the single-event latency case
(bench.py's `single_event_latency` relocalization event: C = 15, N ~ 570), from
rsc_diag_refine_phase_stamps after one rsc_reloc_events call (a library built with RSC_REFINE_STAMPS=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

# a stamped build (make -C tools stamps_lib) when given, else the product library
if len(sys.argv) > 1:
    engine.load_library(sys.argv[1])
ctx = engine.Context(0)
ev = bench.latency_event("reloc")
(eb, params, seeds, _), = bench.build_event_drivers(engine, ctx, [ev], [0])
names = ["compaction", "ctrl pts", "MtM", "eigen", "betas", "check", "exit"]
for rep in range(5):
    eb.batch.reset(seeds)
    eb.batch.set_ransac_parameters(*params)
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
eg = np.diff(np.concatenate([st[ok][:, 3:4], st[ok][:, 8:12]], axis=1), axis=1) / 100.0
for i, n in enumerate(["tridiag", "accumulate", "QR chase", "extract"]):
    print(f"  eigen/{n:10s} mean {eg[:, i].mean():8.1f} us")
for w in range(3):
    b = np.diff(np.concatenate([st[ok][:, 4:5], st[ok][:, 12 + 4 * w:16 + 4 * w]], axis=1), axis=1) / 100.0
    print(f"  betas wave {w}: " + "  ".join(f"{n} {b[:, i].mean():6.1f}" for i, n in
                                          enumerate(["betas+GN+ccs", "pc0", "M+Horn", "err"])) + " us")
if (st[ok, 8] > 0).all():  # eigen sub-phases (RSC_REFINE_STAMPS builds)
    e = np.diff(np.concatenate([st[ok][:, 3:4], st[ok][:, 8:12], st[ok][:, 4:5]], axis=1), axis=1) / 100.0
    for i, n in enumerate(["tridiag", "accumulate", "QR chase", "eigvecs", "L + rho"]):
        print(f"    eigen/{n:10s} mean {e[:, i].mean():8.1f} us  max {e[:, i].max():8.1f} us")
