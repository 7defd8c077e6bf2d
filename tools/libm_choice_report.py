#!/usr/bin/env python3
"""Writes profiles/r03/libm_choice.json: (1) how often the fdlibm restatement (csrc/rsc_math.h, what
the kernels compile) returns a different double than host glibc on random arguments of each
function's working range, and (2) the outcome comparison of tests/test_cpu_libm_choice.py (the oracle
built with each libm on the MLPnP / PoseOptimization / SearchBySim3 / OptimizeSim3 workloads)."""
import ctypes
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "orb-slam2-optimized_amd")]
import numpy as np  # noqa: E402
import oracle_lib as ol  # noqa: E402
import test_cpu_libm_choice as t  # noqa: E402

L = ol.lib()
libm = ctypes.CDLL("libm.so.6")
for name in ("sin", "cos", "acos", "cbrt", "log"):
    f = getattr(L, "ora_dm_" + name)
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
for name in ("sin", "cos", "acos", "pow", "log"):
    getattr(libm, name).restype = ctypes.c_double
libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]
for name in ("sin", "cos", "acos", "log"):
    getattr(libm, name).argtypes = [ctypes.c_double]
libm.logf.restype, libm.logf.argtypes = ctypes.c_float, [ctypes.c_float]
rng = np.random.default_rng(5)
n = 200000
cases = {
    "sin (|x| <= pi)": (L.ora_dm_sin, libm.sin, rng.uniform(-np.pi, np.pi, n)),
    "cos (|x| <= pi)": (L.ora_dm_cos, libm.cos, rng.uniform(-np.pi, np.pi, n)),
    "acos ([-1, 1])": (L.ora_dm_acos, libm.acos, rng.uniform(-1, 1, n)),
    "cbrt vs pow(x, 1/3) ([1e-6, 1e3])": (L.ora_dm_cbrt, lambda x: libm.pow(x, 1.0 / 3.0), 10 ** rng.uniform(-6, 3, n)),
}
funcs = {}
for k, (f, g, xs) in cases.items():
    d = sum(1 for v in xs if f(float(v)) != g(float(v)))
    funcs[k] = dict(samples=n, differing=d, frac=round(d / n, 5))
xs = rng.uniform(0.2, 5.0, n).astype(np.float32)
d = sum(1 for v in xs if np.float32(L.ora_dm_log(float(v))) != np.float32(libm.logf(float(v))))
funcs["logf ([0.2, 5], PredictScale ratios)"] = dict(samples=n, differing=d, frac=round(d / n, 5))
with tempfile.TemporaryDirectory() as td:
    import pathlib
    a = t._run(pathlib.Path(td), "fdlibm")
    b = t._run(pathlib.Path(td), "glibc")
    stats, bad = t.compare(a, b)
head = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
out = dict(commit=head, function_differences=funcs, outcomes=stats, mismatching_problems=[list(map(str, x)) for x in bad],
           note="outcome = discrete results (ok / counts / iterations, inlier, outlier, match and keep decisions) "
                "identical and pose within 1e-4; the GPU is bit-exact to the fdlibm build")
os.makedirs(os.path.join(ROOT, "profiles", "r03"), exist_ok=True)
with open(os.path.join(ROOT, "profiles", "r03", "libm_choice.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
