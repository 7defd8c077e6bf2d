#!/usr/bin/env python3
"""Diagnostic: in-kernel s_memtime stamps at the EPnP phase boundaries of pnp_solve_kernel<4>
(a separate STAMP=true instantiation; the production kernel executes no stamp).  Prints the mean
cycles per phase for the bench workload.  Read shares, not absolute time (stamps serialize)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))
import numpy as np  # noqa: E402
from rsc import engine, synth  # noqa: E402

PHASES = ["rng+sample+load", "control pts+alphas", "MtM", "eig12", "L6x10+rho+svd1", "gn1", "R,t 1",
          "approx2 (svd+gn+R,t)", "approx3 (svd+gn+R,t)", "finish"]


def main():
    ctx = engine.Context(0)
    rng = np.random.default_rng(1)
    C = int(os.environ.get("C", "64"))
    sols = [engine.PnPSolver(ctx, synth.make_pnp_scene(rng, 2000, 0.4), 1 + i) for i in range(C)]
    b = engine.SolverBatch(sols)
    b.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    st = b.phase_stamps(300).astype(np.int64)
    d = np.diff(st, axis=2)
    tot = st[:, :, 9] - st[:, :, 0]
    print(f"total cycles per hypothesis: mean {tot.mean():.0f}  max {tot.max():.0f}")
    for k, name in enumerate(PHASES[:9]):
        print(f"{name:26s} {d[:, :, k].mean():10.0f}  ({100 * d[:, :, k].mean() / tot.mean():5.1f}%)")


if __name__ == "__main__":
    main()
