"""TEST HELPER (run as a subprocess by tests/test_cpu_libm_choice.py): the libm-dependent oracle
paths — MLPnPsolver::iterate (Rodrigues sin/cos, acos, pow(x, 1/3)), Optimizer::PoseOptimization
(SE3 exp map sin/cos), ORBmatcher::SearchBySim3 (MapPoint::PredictScale logf) and
Optimizer::OptimizeSim3 (Sim3 exp map sin/cos) — on seed-fixed workloads, through whichever oracle
build oracle_lib loads (RSC_ORACLE_LIBM=glibc: host glibc, as the reference; default: the fdlibm
restatement the kernels compile).  Writes the outcomes to the .npz path given as argv[1]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orb-slam2-optimized_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import oracle_lib as ol  # noqa: E402
from rsc import synth  # noqa: E402

SIZES = dict(mlpnp=40, poseopt=96, sim3match=48, sim3opt=32)


def mlpnp():
    rng = np.random.default_rng(1101)
    out = []
    for c in range(SIZES["mlpnp"]):
        sc = synth.make_pnp_scene(rng, int(rng.integers(150, 1200)), float(rng.uniform(0.45, 0.85)))
        o = ol.OracleMLPnP(sc, 1 + c)
        o.set_ransac_parameters(0.99, 10, 300, 6, 0.5, 5.991)
        r = o.iterate(300)
        out.append((np.array([r["ok"], r["no_more"], r["n_inliers"], r["iterations"]], np.int64),
                    np.asarray(r["T"], np.float64).ravel(), np.packbits(np.asarray(r["inliers"], np.uint8))))
    return out


def poseopt():
    rng = np.random.default_rng(1102)
    out = []
    for c in range(SIZES["poseopt"]):
        f = synth.make_poseopt_frame(rng, int(rng.integers(100, 800)), float(rng.uniform(0.6, 0.9)),
                                     stereo_frac=0.5 if c % 2 else 0.0)
        n, T, flags, st = ol.pose_optimization(f)
        out.append((np.array([n], np.int64), np.asarray(T, np.float64).ravel(), flags.astype(np.uint8)))
    return out


def sim3match():
    rng = np.random.default_rng(1103)
    out = []
    for _ in range(SIZES["sim3match"]):
        kf1, kf2, R12, t12, m12 = synth.make_sim3match_pair(rng, int(rng.integers(300, 900)), 150, 0.3)
        nf, o12 = ol.search_by_sim3(kf1, kf2, R12, t12, m12, 7.5)
        out.append((np.array([nf], np.int64), np.zeros(0), o12.astype(np.int32).view(np.uint8)))
    return out


def sim3opt():
    rng = np.random.default_rng(1104)
    out = []
    for _ in range(SIZES["sim3opt"]):
        p = synth.make_sim3opt_problem(rng, int(rng.integers(60, 700)), outlier_frac=0.25)
        n, S, keep, st = ol.optimize_sim3(p)
        out.append((np.array([n], np.int64), np.asarray(S, np.float64).ravel(), keep.astype(np.uint8)))
    return out


def main(path):
    arrays = {}
    for name, fn in (("mlpnp", mlpnp), ("poseopt", poseopt), ("sim3match", sim3match), ("sim3opt", sim3opt)):
        for i, (disc, pose, bits) in enumerate(fn()):
            arrays[f"{name}_{i}_d"] = disc
            arrays[f"{name}_{i}_p"] = pose
            arrays[f"{name}_{i}_b"] = bits
    np.savez(path, **arrays)


if __name__ == "__main__":
    main(sys.argv[1])
