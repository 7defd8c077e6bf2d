#!/usr/bin/env python3
"""Host-side cost of one config-2 step, split by API call (run on the GPU box):
reset_many, set_ransac_parameters_many, iterate_many (GPU kernels + host replay)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))
import numpy as np  # noqa: E402
from rsc import engine, synth  # noqa: E402

ctx = engine.Context(0)
rng = np.random.default_rng(20240)
scenes = [synth.make_pnp_scene(rng, 2000, 0.4) for _ in range(64)]
batch = engine.SolverBatch([engine.PnPSolver(ctx, sc, 1) for sc in scenes])
seeds = np.zeros(64, np.uint32)
acc = np.zeros(4)
hacc = np.zeros(4)
ctx.enable_timing(os.environ.get("TIMING", "1") == "1")
gpu = 0.0
for s in range(60):
    seeds[:] = 1 + np.arange(64) + 64 * s
    t0 = time.perf_counter()
    batch.reset(seeds)
    t1 = time.perf_counter()
    batch.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    t2 = time.perf_counter()
    batch.iterate_raw(300)
    t3 = time.perf_counter()
    if s >= 10:
        acc += [t1 - t0, t2 - t1, t3 - t2, t3 - t0]
        tm = ctx.last_timing()
        gpu += tm["solve_ms"] + tm["scan_ms"]
        hacc += ctx.host_timing()
n = 50
print(f"reset {1e6*acc[0]/n:.1f} us  params {1e6*acc[1]/n:.1f} us  iterate {1e6*acc[2]/n:.1f} us  "
      f"step {1e6*acc[3]/n:.1f} us  gpu(kernels) {1e3*gpu/n:.1f} us")
print("inside iterate_many (us from entry): first launch %.1f, enqueued %.1f, synced %.1f, return %.1f" % tuple(hacc / n))
