#!/usr/bin/env python3
"""Diagnostic: SearchByBoW kernel time (HIP events around the launch) under input / flag variants,
to locate what bounds the three kernels.  Prints one line per variant."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), os.path.join(ROOT, "tests"), ROOT]
import numpy as np  # noqa: E402
from rsc import engine, synth  # noqa: E402


def views(seed, C=64, N=2000, skew=0.8, flips=(8, 30), overlap=(0.1, 0.7)):
    rng = np.random.default_rng(seed)
    F = synth.make_bow_view(rng, N, skew=skew)
    kfs = [synth.make_bow_related(rng, F, N, float(rng.uniform(*overlap)), float(rng.uniform(0, 360)),
                                  mean_flips=float(rng.uniform(*flips)), skew=skew) for _ in range(C)]
    return F, kfs


def timeit(ctx, F, kfs, ratio=0.75, check=True, frame=True, reps=20):
    gF = engine.BowView(ctx, F)
    gK = [engine.BowView(ctx, k) for k in kfs]
    b = engine.BowSearch(ctx, gF, gK, frame, ratio, check) if frame else engine.BowSearch(ctx, gF, gK, False, ratio, check)
    b.run()
    ctx.enable_timing(True)
    ms = []
    for _ in range(reps):
        _, nm = b.run()
        ms.append(ctx.last_timing()["refine_ms"])
    ctx.enable_timing(False)
    return float(np.median(ms)), float(np.mean(nm))


def phases(ctx, F, kfs):
    """Per-phase wall-clock (us) of the last launch, from rsc_diag_bow_phase_stamps."""
    from rsc.engine import load_library
    st = np.zeros(64 * 96 + 32 * 8 * 4, np.uint64)
    load_library().rsc_diag_bow_phase_stamps(ctx.h, st, st.size)
    ts = st[64 * 96:].reshape(32, 8, 4).copy()
    st = st[:64 * 96].reshape(64, 96).astype(np.int64)
    nbs = (ts[:, :, 3] >> np.uint64(48)).astype(np.int64)
    ts = (ts & np.uint64((1 << 48) - 1)).astype(np.int64)
    base = st[0, 21:85].reshape(32, 2)[:, 0].min()
    for v in range(0, 32, 8):
        row = []
        for i in range(8):
            if ts[v, i, 0] == 0 or ts[v, i, 0] < base:
                break
            e = (ts[v, i] - base) / 100.0
            row.append(f"[{e[0]:.1f} load {e[1] - e[0]:.1f} stage {e[2] - e[1]:.1f} comp {e[3] - e[2]:.1f} nb {nbs[v, i]}]")
        print(f"  topk wave {v}: " + " ".join(row))
    C = min(64, len(kfs))
    for p in range(min(C, 4)):
        r = st[p]
        t0 = r[0]
        walk = (r[2:18] - t0) / 100.0
        tk = r[21:85].reshape(32, 2)
        tk0 = tk[:, 0].min()
        print(f"  pair {p}: topk waves {((tk[:, 1] - tk0) / 100.0).max():.1f} us (start spread "
              f"{((tk[:, 0] - tk0) / 100.0).max():.1f}); resolve: init {(r[1] - t0) / 100.0:.1f} walk max "
              f"{walk.max():.1f} min {walk.min():.1f} res {(r[18] - t0) / 100.0:.1f} hist {(r[19] - t0) / 100.0:.1f} "
              f"end {(r[20] - t0) / 100.0:.1f}; topk end -> resolve start {(t0 - tk[:, 1].max()) / 100.0:.1f}",
              flush=True)


def main():
    ctx = engine.Context(0)
    base = views(80)
    only = sys.argv[1:]
    for name, kw, v in [("base", {}, base), ("no_ori", {"check": False}, base), ("ratio0", {"ratio": 0.0}, base),
                        ("kf_overload", {"frame": False}, base),
                        ("C=1", {}, (base[0], base[1][:1])), ("C=8", {}, (base[0], base[1][:8])),
                        ("skew0", {}, views(81, skew=0.0)), ("skew2", {}, views(82, skew=2.0)),
                        ("nocand", {}, views(83, flips=(90, 100))), ("N500", {}, views(84, N=500))]:
        if only and name not in only:
            continue
        ms, nm = timeit(ctx, v[0], v[1], **kw)
        sizes = np.diff(v[0].node_begin)
        if name in ("base", "C=1", "skew0"):
            phases(ctx, v[0], v[1])
        print(f"{name:12s} C={len(v[1]):3d} N={v[0].n} kernel_ms={ms:.4f} mean_matches={nm:.1f} "
              f"max_node={sizes.max()} nodes={len(sizes)}", flush=True)


if __name__ == "__main__":
    main()
