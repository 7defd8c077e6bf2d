#!/usr/bin/env python3
"""Diagnostic: where OptimizeSim3's kernel time goes (bench.py's optimize_sim3 section, 32 pairs x
~900 correspondences): per-pair wall clocks of the fused passes, the perturbed-estimate builds, the
LM solves, wave 1's edge evaluation per slab and wave 0's folds (rsc_diag_sim3opt_phases, compiled in
with -DRSC_SO_PHASES=1: make -C tools variant NAME=so0 SRC=sim3opt DEFS=-DRSC_SO_PHASES=1), averaged
over the pairs of the last launch; the batch kernel time (HIP events) always."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

ctx = engine.Context(0)
probs = bench.sim3opt_problems()
b = engine.Sim3OptBatch(ctx, probs)
for _ in range(5):
    b.run()
ph = np.zeros(64 * 8, np.uint64)
engine._check(engine.load_library().rsc_diag_sim3opt_phases(ctx.h, ph, ph.size), "sim3opt phases")
ph = ph.reshape(64, 8)[: len(probs)].astype(np.float64)
ctx.enable_timing(True)
kms = []
for _ in range(5):
    b.run()
    kms.append(ctx.last_timing()["refine_ms"])
ctx.enable_timing(False)
res = b.results()
its = np.mean([r["lm_iterations"] for r in res])
if not ph[:, 7].any():
    print(f"batch kernel {np.median(kms):.3f} ms; LM iterations {its:.1f} (phase clocks not compiled in)")
    sys.exit(0)
us = ph / 100.0
ok = ph[:, 1] > 0
npass, nsl = ph[ok, 1], ph[ok, 5]
print(f"batch kernel {np.median(kms):.3f} ms; kernel/pair {us[ok, 7].mean():.1f} us (max {us[ok, 7].max():.1f}); "
      f"passes {us[ok, 0].mean():.1f} us = {npass.mean():.1f} x {(us[ok, 0] / npass).mean():.2f}; LM iterations {its:.1f}")
print(f"    per pass: perturbed estimates {(us[ok, 2] / npass).mean():.2f} us, folds {(us[ok, 6] / npass).mean():.2f} us; "
      f"LM solves {us[ok, 3].mean():.1f} us per pair; wave-1 edge evaluation {(us[ok, 4] / nsl).mean() * 1e3:.0f} ns "
      f"per slab ({nsl.mean():.0f} slabs per pair); rest {(us[ok, 7] - us[ok, 0] - us[ok, 3]).mean():.1f} us")
