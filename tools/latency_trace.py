#!/usr/bin/env python3
"""Diagnostic: the single-event latency case of bench.py (one relocalization event, C = 15, N ~ 570,
or one loop event) run `reps` times with nothing else in the process, so a rocprofv3 kernel trace of
this command holds only that event's kernels:
    rocprofv3 --kernel-trace --stats -d OUT -o lat --output-format csv -- python3 tools/latency_trace.py
Prints the median wall time per event call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "reloc"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ctx = engine.Context(0)
ev = bench.latency_event(kind)
(eb, params, seeds, _), = bench.build_event_drivers(engine, ctx, [ev], [0])
times = []
for r in range(reps + 5):
    t0 = time.perf_counter()
    eb.batch.reset(seeds)
    eb.batch.set_ransac_parameters(*params)
    eb.run()
    if r >= 5:
        times.append(time.perf_counter() - t0)
pe = eb.per_event[0]
print(f"{kind}: median {1e3 * np.median(times):.4f} ms over {reps} calls; winner {pe['winner']} round {pe['round']} "
      f"hypotheses {int(eb.cand['iterations'].sum())}")
