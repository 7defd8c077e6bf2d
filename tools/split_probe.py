#!/usr/bin/env python3
"""Diagnostic: phase clocks of the split-form eigen stage (RSC_EIG_SPLIT=1) on config 2, from the
stamped library (make -C tools solve_stamps_lib).  Per workgroup: A (wave 0 pairs), B and C (quads
over both waves), the chase (wave 0 reaching its final barrier), the final barrier, and the row wave
leaving its loop; plus the number of QR steps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
from rsc import engine, workloads as wl  # noqa: E402

ctx = engine.Context(0)
batch = engine.SolverBatch([engine.PnPSolver(ctx, sc, 1) for sc in wl.config2_scenes()])
for s in range(3):
    batch.reset(wl.config2_seeds(s))
    batch.set_ransac_parameters(*wl.RELOC)
    batch.iterate_raw(300)
st = np.zeros(3 * 4096 * 8, np.uint64)
engine._check(engine.load_library().rsc_diag_solve_phase_stamps(ctx.h, st, st.size), "solve stamps")
e = st.reshape(3, 4096, 8)[0].astype(np.int64)
e = e[e[:, 0] > 0]


def stats(x):
    return f"med {np.median(x):7.2f}  p90 {np.percentile(x, 90):7.2f}  max {x.max():7.2f}"


print(f"split eigen stage: {len(e)} workgroups of 4 units, launch span {(e[:, 4].max() - e[:, 0].min()) / 100:.2f} us")
for name, a, b in [("A (pairs)", 0, 1), ("B (quads)", 1, 2), ("C (quads)", 2, 3), ("chase", 3, 6),
                   ("final barrier", 6, 4), ("rows leave", 3, 5), ("total", 0, 4)]:
    print(f"  {name:14s} {stats((e[:, b] - e[:, a]) / 100)}")
print(f"  QR steps       {stats(e[:, 7].astype(float) - 1)}")
