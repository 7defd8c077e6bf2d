#!/usr/bin/env python3
"""Diagnostic: where PoseOptimization's kernel time goes (bench.py's poseopt section, 64 stereo Frames x
2000 edges): per-frame wall-clock of the build passes, chi2 passes and re-classification
(rsc_diag_poseopt_phases, compiled in with -DRSC_POSE_PHASES=1), averaged over the 64 Frames of the
last launch; the batch kernel time (HIP events) always."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
from rsc import engine  # noqa: E402

ctx = engine.Context(0)
for sf in (0.8, 0.0):
    frames = bench.poseopt_frames(np.random.default_rng(79), stereo_frac=sf)
    b = engine.PoseOptBatch(ctx, frames)
    for _ in range(5):
        b.run()
    ph = np.zeros(64 * 24, np.uint64)
    engine._check(engine.load_library().rsc_diag_poseopt_phases(ctx.h, ph, ph.size), "poseopt phases")
    hw = ph.reshape(64, 24)[:, 8:16].astype(np.int64)
    fold = ph.reshape(64, 24)[:, 16:22].astype(np.float64)
    ph = ph.reshape(64, 24)[:, :8].astype(np.float64)
    npass = (ph[:, 1].astype(np.uint64) & np.uint64(0xFFFFFF)).astype(np.float64)
    summ = (ph[:, 1].astype(np.uint64) >> np.uint64(24)).astype(np.float64)
    ph /= 100.0  # us
    res = b.results()
    its = np.mean([r["lm_iterations"] for r in res])
    trials = np.mean([r["lm_trials"] for r in res])
    ctx.enable_timing(True)
    kms = []
    for _ in range(5):
        b.run()
        kms.append(ctx.last_timing()["refine_ms"])
    ctx.enable_timing(False)
    if not ph[:, 3].any():
        print(f"stereo_frac {sf}: batch kernel {np.median(kms):.3f} ms; LM iterations {its:.1f}, trials {trials:.1f} "
              "(phase clocks not compiled in: build poseopt.hip with -DRSC_POSE_PHASES=1)")
        continue
    print(f"stereo_frac {sf}: batch kernel {np.median(kms):.3f} ms; kernel/frame {ph[:, 3].mean():.1f} us "
          f"(max {ph[:, 3].max():.1f}); passes {ph[:, 0].mean():.1f} us = {npass.mean():.1f} x "
          f"{(ph[:, 0] / npass).mean():.2f} (active edges per pass {(summ / npass).mean():.0f}: "
          f"{(ph[:, 0] / summ).mean() * 1e3:.2f} ns per edge); LM iterations {its:.1f}, trials {trials:.1f}; re-classification "
          f"{ph[:, 2].mean():.1f}; LM solves {ph[:, 4].mean():.1f}; rest {(ph[:, 3] - ph[:, 0] - ph[:, 2] - ph[:, 4]).mean():.1f}")
    if hw.any():
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        print("    SIMD of waves 0..7, frames 0-3: " + "; ".join(" ".join(str(int(v)) for v in simd[f]) for f in range(4))
              + f"  (CU ids {sorted(set(cu[:4, 0].tolist()))})")
    if fold[:, 1].any():
        print(f"    wave-0 folds: {(fold[:, 0] / fold[:, 1]).mean() * 10:.0f} ns per fold of a slab, "
              f"{fold[:, 0].mean() / 100:.1f} us per frame ({fold[:, 1].mean():.0f} folds); LDLT part of the LM "
              f"solves {fold[:, 2].mean() / 100:.1f} us per frame")
        if fold[:, 3].any() or fold[:, 5].any():
            print(f"    streamed pass: fold waits {fold[:, 3].mean() / 100:.1f} us per frame, wave-1 slot waits "
                  f"{fold[:, 4].mean() / 100:.1f} us, pass start -> first slab in {fold[:, 5].mean() / 100:.1f} us")
    nsl = ph[:, 7] * 100.0  # slab count (undo the us scaling)
    if nsl.any():
        print(f"    wave-1 slab phases: to the errors {(ph[:, 5] / nsl).mean() * 1e3:.0f} ns, errors -> terms stored "
              f"{(ph[:, 6] / nsl).mean() * 1e3:.0f} ns per slab ({nsl.mean():.0f} slabs per frame)")
