#!/usr/bin/env python3
"""Diagnostic: where the cooperative OptimizeSim3 form's time goes (bench.py's optimize_sim3 section,
32 pairs x ~900 correspondences), from the phase clocks of a -DRSC_SO_PHASES=1 build
(make -C tools variant NAME=soc SRC=sim3opt DEFS=-DRSC_SO_PHASES=1; RSC_LIBRSC=tools/bin/librsc_soc.so):
per pass the perturbed-estimate build + publication, publication -> first chunk in the master's
ring, publication -> last fold; the LM solves; chunks the master's wave 1 evaluated itself.  Argument:
helper workgroups per pair (default: automatic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

ctx = engine.Context(0)
if len(sys.argv) > 1:
    ctx.set_sim3opt_helpers(int(sys.argv[1]))
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
us = ph / 100.0
ok = ph[:, 1] > 0
n = ph[ok, 1]
slow = int(np.argmax(us[:, 7]))
print(f"helpers {sys.argv[1] if len(sys.argv) > 1 else 'auto'}: batch kernel {np.median(kms):.3f} ms; kernel/pair "
      f"{us[ok, 7].mean():.1f} us (max {us[ok, 7].max():.1f}, pair {slow}); passes {us[ok, 0].mean():.1f} us = "
      f"{n.mean():.1f} x {(us[ok, 0] / n).mean():.2f}; LM solves {us[ok, 3].mean():.1f} us per pair")
print(f"    per pass: build + publish {(us[ok, 2] / n).mean():.2f} us, publish -> first chunk {(us[ok, 4] / n).mean():.2f} us, "
      f"publish -> last fold {(us[ok, 6] / n).mean():.2f} us; chunks evaluated by master wave 1 {(ph[ok, 5] / n).mean():.2f} per pass")
print(f"    slowest pair {slow}: passes {us[slow, 0]:.1f} us = {ph[slow, 1]:.0f} x {us[slow, 0] / max(ph[slow, 1], 1):.2f}, "
      f"LM {us[slow, 3]:.1f} us, kernel {us[slow, 7]:.1f} us")
