#!/usr/bin/env python3
"""A/B timing of OptimizeSim3 (bench.py's optimize_sim3 workload): median HIP-event kernel time of
20 launches for the library in RSC_LIBRSC (or the in-tree one) at the helper count given (-1 auto,
0 one workgroup per pair)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

h = int(sys.argv[1]) if len(sys.argv) > 1 else -1
ctx = engine.Context(0)
ctx.set_sim3opt_helpers(h)
b = engine.Sim3OptBatch(ctx, bench.sim3opt_problems())
for _ in range(5):
    b.run()
ctx.enable_timing(True)
kms = []
for _ in range(20):
    b.run()
    kms.append(ctx.last_timing()["refine_ms"])
print(f"{os.path.basename(os.environ.get('RSC_LIBRSC', 'librsc.so'))} helpers {h}: median {np.median(kms):.4f} ms "
      f"(min {min(kms):.4f}, max {max(kms):.4f})")
