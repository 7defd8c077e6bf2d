#!/usr/bin/env python3
"""Algorithmic FP64 work per unit of the solver kernels (SURVEY.md §8(d) "Solve FLOPs S_h: measure
it by an op-counter build of the CPU restatement and report mean ± σ per config"), on the bench's
own inputs: the oracle restatements compiled with a counting scalar (tools/opc_*.cpp ->
tools/build/libopcount.so: +, -, *, /, sqrt and fma count as flops, transcendental calls one each).

    make -C tools opcount_lib && python3 tools/opcount_report.py [OUT]   # default profiles/r05/opcount.json

Units: EPnP / MLPnP — one compute_pose on a minimal sample (4 / 6 points); PoseOptimization — one
Frame's whole call (4 rounds of LM); OptimizeSim3 — one KeyFrame pair's whole call.  Sim3 (config 3)
is float arithmetic and scan-dominated: its unit figures are SURVEY §8(d)'s F_h = 62 N FP32 flops and
B_h = 48 N bytes per hypothesis (no counter build)."""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from rsc import workloads as wl  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "tools", "build", "libopcount.so"))
f32 = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
f64 = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i32 = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
u8 = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
for pre in ("pnp", "mlpnp"):
    getattr(L, f"opc_{pre}_create").restype = C.c_void_p
    getattr(L, f"opc_{pre}_create").argtypes = [C.c_int, f32, f32, f32, C.c_float, C.c_float, C.c_float, C.c_float]
    getattr(L, f"opc_{pre}_destroy").argtypes = [C.c_void_p]
    getattr(L, f"opc_{pre}_compute_pose").restype = C.c_double
    getattr(L, f"opc_{pre}_compute_pose").argtypes = [C.c_void_p, i32, C.c_int]
L.opc_pose_optimization.restype = C.c_double
L.opc_pose_optimization.argtypes = [C.c_int, f32, f32, f32, C.c_float, C.c_float, C.c_float, C.c_float, f32,
                                    C.c_void_p, C.c_float, i32]
L.opc_optimize_sim3.restype = C.c_double
L.opc_optimize_sim3.argtypes = [C.c_int, u8, f32, f32, f32, f32, f32, f32, f32, f32, C.c_float, f64, i32]


def stats(v, **extra):
    v = np.asarray(v, np.float64)
    return dict(fp64_flops_mean=round(float(v.mean()), 1), std=round(float(v.std()), 1), min=float(v.min()),
                max=float(v.max()), samples=int(v.size), **extra)


def minimal_samples(pre, scenes, k, per_scene, seed):
    rng = np.random.default_rng(seed)
    out = []
    for sc in scenes:
        h = getattr(L, f"opc_{pre}_create")(sc.n, np.ascontiguousarray(sc.p2d, np.float32),
                                             np.ascontiguousarray(sc.p3dw, np.float32),
                                             np.ascontiguousarray(sc.sigma2, np.float32), sc.fx, sc.fy, sc.cx, sc.cy)
        for _ in range(per_scene):
            idx = rng.choice(sc.n, k, replace=False).astype(np.int32)
            out.append(getattr(L, f"opc_{pre}_compute_pose")(h, idx, k))
        getattr(L, f"opc_{pre}_destroy")(h)
    return out


def main():
    import bench
    rep = {}
    rep["pnp"] = stats(minimal_samples("pnp", wl.config2_scenes(0, 8, 2000), 4, 2500, 1),
                       unit="EPnP compute_pose, 4-point sample (config 2 scenes)")
    rep["mlpnp"] = stats(minimal_samples("mlpnp", wl.config4_scenes(8), 6, 600, 2),
                         unit="MLPnP computePose, 6-point sample (config 4 scenes)")
    for name, sf in (("poseopt", 0.8), ("poseopt_mono", 0.0)):
        frames = bench.poseopt_frames(np.random.default_rng(79), stereo_frac=sf)
        fl, its = [], []
        for f in frames:
            st = np.zeros(3, np.int32)
            ur = np.ascontiguousarray(f.u_right, np.float32) if sf > 0 else None
            fl.append(L.opc_pose_optimization(f.n, np.ascontiguousarray(f.uv, np.float32),
                                              np.ascontiguousarray(f.Xw, np.float32),
                                              np.ascontiguousarray(f.inv_sigma2, np.float32), f.fx, f.fy, f.cx, f.cy,
                                              np.ascontiguousarray(f.Tcw, np.float32).reshape(16),
                                              None if ur is None else ur.ctypes.data, float(getattr(f, "bf", 0.0)),
                                              st))
            its.append(st[1])
        rep[name] = stats(fl, unit=f"one PoseOptimization call: Frame x {frames[0].n} edges (bench section {name})",
                          lm_iterations_mean=float(np.mean(its)))
    fl, its = [], []
    for p in bench.sim3opt_problems():
        st = np.zeros(4, np.int32)
        S = np.ascontiguousarray(p.S0, np.float64).copy()
        fl.append(L.opc_optimize_sim3(p.n, np.ascontiguousarray(p.valid, np.uint8), np.ascontiguousarray(p.X1w, np.float32),
                                      np.ascontiguousarray(p.X2w, np.float32), np.ascontiguousarray(p.uv1, np.float32),
                                      np.ascontiguousarray(p.uv2, np.float32), np.ascontiguousarray(p.inv1, np.float32),
                                      np.ascontiguousarray(p.inv2, np.float32), p.poses24(), p.K8(), float(p.th2), S, st))
        its.append(st[2])
    rep["optimize_sim3"] = stats(fl, unit="one OptimizeSim3 call: KeyFrame pair (bench section optimize_sim3)",
                                 lm_iterations_mean=float(np.mean(its)))
    rep["sim3"] = dict(unit="one hypothesis scan at N correspondences (SURVEY §8(d))", fp32_flops_per_corr=62,
                       bytes_per_corr=48)
    rep["commit"] = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True,
                                   text=True).stdout.strip()
    rep["counting"] = ("op-counter builds of the oracle restatements (tools/opc_*.cpp): +, -, *, /, sqrt = 1 flop, "
                       "fma = 2, sin/cos/acos/pow/log/exp calls = 1; comparisons and fabs not counted")
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05", "opcount.json")
    with open(out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
