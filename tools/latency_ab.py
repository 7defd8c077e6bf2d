#!/usr/bin/env python3
"""Diagnostic A/B of the single-event latency (bench.py's relocalization event) across engine
variants set through the environment at context creation (e.g. RSC_FUSED_REFINE; the round-3
RSC_EIG_SHAPE / RSC_BETAS_HB shapes were measured with it and removed): one context + solver set per variant in ONE process, the GPU first kept busy for
~1 s with the config-2 batch, then the variants measured in rotation (clock state shared).
    python3 tools/latency_ab.py "base:" "eig1:RSC_EIG_SHAPE=1" "hb64:RSC_BETAS_HB=64" ...
Each argument is name:VAR=val,VAR=val.  Prints the median per variant."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine, workloads as wl  # noqa: E402

specs = []
for arg in sys.argv[1:] or ["base:"]:
    name, _, spec = arg.partition(":")
    specs.append((name, dict(kv.split("=") for kv in spec.split(",") if kv)))
KEYS = sorted({k for _, env in specs for k in env})
variants = []
for name, env in specs:
    for k in KEYS:
        os.environ.pop(k, None)
    os.environ.update(env)
    ctx = engine.Context(0)
    ev = bench.latency_event("reloc")
    (eb, params, seeds, _), = bench.build_event_drivers(engine, ctx, [ev], [0])
    variants.append((name, ctx, eb, params, seeds))
for k in KEYS:
    os.environ.pop(k, None)
warm_ctx = variants[0][1]
warm = engine.SolverBatch([engine.PnPSolver(warm_ctx, sc, 1) for sc in wl.config2_scenes(0, 64, 2000)])


def heat(seconds):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        warm.reset(wl.config2_seeds(0, 0, 64))
        warm.set_ransac_parameters(*wl.RELOC)
        warm.iterate_raw(300)


heat(1.0)
times = {v[0]: [] for v in variants}
results = {}
for rot in range(8):
    for name, ctx, eb, params, seeds in variants:
        for r in range(12):
            t0 = time.perf_counter()
            eb.batch.reset(seeds)
            eb.batch.set_ransac_parameters(*params)
            eb.run()
            if r >= 2:
                times[name].append(time.perf_counter() - t0)
        pe = eb.per_event[0]
        results[name] = (int(pe["winner"]), int(pe["round"]), int(pe["n_inliers"]), int(eb.cand["iterations"].sum()))
    heat(0.1)
ref = results[variants[0][0]]
for name, *_ in variants:
    print(f"{name:12s} median {1e3 * np.median(times[name]):.4f} ms  p10 {1e3 * np.percentile(times[name], 10):.4f}  "
          f"result {results[name]} {'==' if results[name] == ref else 'DIFFERS'}")
