#!/usr/bin/env python3
"""Diagnostic: per-phase wall clock of mlpnp_quad_kernel<6> on the config-4 launch (bench.py's mlpnp
section: candidates x 4096 correspondences, iterate(300) exhaustive), from rsc_diag_mlpnp_phase_stamps
of a library built with RSC_ML_STAMPS=1 (make -C tools mlstamps_lib; RSC_LIBRSC=tools/bin/librsc_mlstamps.so).
Usage: mlpnp_probe.py [candidates] [stamps|run] [steps]
  stamps: one launch, per-phase medians over the stamped workgroups (16 hypotheses each)
  run:    `steps` launches and nothing else (a rocprofv3 / PMC target)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT]
import numpy as np  # noqa: E402
from rsc import engine  # noqa: E402
from rsc import workloads as wl  # noqa: E402

cands = int(sys.argv[1]) if len(sys.argv) > 1 else 128
mode = sys.argv[2] if len(sys.argv) > 2 else "stamps"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = engine.Context(0)
scenes = wl.config4_scenes(candidates=cands)
gs = [engine.MLPnPSolver(ctx, sc, 1) for sc in scenes]
b = engine.SolverBatch(gs)
for rep in range(steps if mode == "run" else 2):
    b.reset(wl.step_seeds(rep, len(gs)))
    b.set_ransac_parameters(*wl.MLPNP)
    t0 = time.perf_counter()
    b.iterate_raw(300)
    print(f"step {rep}: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
if mode == "stamps":
    st = np.zeros(8192 * 8, np.uint64)
    engine._check(engine.load_library().rsc_diag_mlpnp_phase_stamps(ctx.h, st, st.size), "ml stamps")
    st = st.reshape(8192, 8).astype(np.int64)
    ok = (st[:, 0] > 0) & (st[:, 5] > 0)
    d = np.diff(st[ok][:, :6], axis=1) / 100.0  # 100 MHz wall clock
    names = ["sample", "A + normal matrix", "JacobiSVD", "pose recovery", "Gauss-Newton"]
    tot = (st[ok, 5] - st[ok, 0]) / 100.0
    span = (st[ok, 5].max() - st[ok, 0].min()) / 100.0
    print(f"mlpnp_quad_kernel<6>: {ok.sum()} workgroups stamped (16 hypotheses each), launch span {span:.1f} us, "
          f"per-workgroup total med {np.median(tot):.1f} p90 {np.percentile(tot, 90):.1f} max {tot.max():.1f} us")
    for i, n in enumerate(names):
        print(f"  {n:18s} med {np.median(d[:, i]):8.2f}  p90 {np.percentile(d[:, i], 90):8.2f}  "
              f"max {d[:, i].max():8.2f} us  share {d[:, i].sum() / tot.sum():.3f}")
