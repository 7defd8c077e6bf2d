"""Planar-content variant of config 2 (VERDICT r3 "Next round" 2): 64 candidates x 2000
correspondences on an exactly planar floor (rsc.synth.make_planar_pnp_scene, Q4 NaN hypotheses),
iterate(300) exhaustive, beside the regular config-2 batch — eigen-stage / solve / scan kernel times
(HIP events on the context stream) and ms per step, for the library in RSC_LIBRSC (default the
product).  Run once with the product and once with tools/bin/librsc_nonanexit.so (make -C tools
nonan_lib: the QR sweep without the non-finite-block exit) to get the before / after:

    python tools/planar_ab.py OUT.json [label]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))

from rsc import engine, synth, workloads as wl  # noqa: E402


def measure(ctx, scenes, steps=10, warmup=3):
    gs = [engine.PnPSolver(ctx, sc, 1 + i) for i, sc in enumerate(scenes)]
    b = engine.SolverBatch(gs)
    res = {}
    for timing in (False, True):
        ctx.enable_timing(timing)
        acc = dict(solve_ms=0.0, scan_ms=0.0, eig_ms=0.0, launches=0)
        t0 = None
        for s in range(warmup + steps):
            if s == warmup:
                ctx.synchronize()
                t0 = time.perf_counter()
            b.reset(wl.config2_seeds(s, candidates=len(gs)))
            b.set_ransac_parameters(*wl.RELOC)
            out = b.iterate_raw(300)
            if timing and s >= warmup:
                tm = ctx.last_timing()
                for k in ("solve_ms", "scan_ms", "eig_ms"):
                    acc[k] += tm[k]
                acc["launches"] += tm["solve_launches"]
        ctx.synchronize()
        dt = time.perf_counter() - t0
        if timing:
            n = max(acc["launches"], 1)
            res.update(eig_us=1e3 * acc["eig_ms"] / n, solve_us=1e3 * acc["solve_ms"] / n,
                       betas_us=1e3 * (acc["solve_ms"] - acc["eig_ms"]) / n, scan_us=1e3 * acc["scan_ms"] / n)
        else:
            res["ms_per_step"] = 1e3 * dt / steps
            res["hypotheses_per_step"] = int(np.sum(out["iterations"]))
    ctx.enable_timing(False)
    return res


def main(out, label="product"):
    ctx = engine.Context(0)
    rep = dict(library=engine._lib_path_loaded if hasattr(engine, "_lib_path_loaded") else None, label=label)
    rep["config2"] = measure(ctx, wl.config2_scenes())
    floor = [synth.make_planar_pnp_scene(np.random.default_rng(20500 + i), 2000, 0.4, "floor") for i in range(64)]
    rep["config2_planar_floor"] = measure(ctx, floor)
    tilted = [synth.make_planar_pnp_scene(np.random.default_rng(20600 + i), 2000, 0.4, "tilted") for i in range(64)]
    rep["config2_planar_tilted"] = measure(ctx, tilted)
    rep["library"] = engine._lib_path_loaded
    print(json.dumps(rep, indent=1))
    with open(out, "w") as f:
        json.dump(rep, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main(*sys.argv[1:3])
