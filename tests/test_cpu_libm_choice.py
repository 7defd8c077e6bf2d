"""How much the restatement's libm choice matters (VERDICT r2 "What's weak" 1 / "Next round" 7).

The kernels and the checker oracle evaluate sin / cos / acos / pow(x, 1/3) / logf with the fdlibm
restatement of csrc/rsc_math.h; the reference links host glibc.  The oracle is built twice from the
same sources (oracle/ora_libm.h): the checker, and librsc_oracle_glibc.so calling glibc exactly where
the reference does (MLPnPsolver.cpp:567,636-653; g2o's SE3 / Sim3 exp maps under PoseOptimization and
OptimizeSim3; MapPoint::PredictScale's log(float), MapPoint.cpp:375).  The GPU is bit-exact to the
checker (tests/test_gpu_*.py), so the checker-vs-glibc comparison below is the GPU-vs-glibc one.

Over seed-fixed MLPnP / PoseOptimization / SearchBySim3 / OptimizeSim3 workloads
(tests/libm_workload.py) every problem's outcome must be within north_star's tolerance of the glibc
build — 1e-4 on the pose, identical inlier / outlier / match / keep decisions — in >= 99.9 % of the
problems; the mismatching problems, if any, are listed in the assertion message."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLIBC = os.path.join(ROOT, "oracle", "build", "librsc_oracle_glibc.so")


def _run(tmp_path, variant):
    path = str(tmp_path / f"libm_{variant}.npz")
    env = dict(os.environ)
    env.pop("RSC_ORACLE_LIBM", None)
    if variant == "glibc":
        env["RSC_ORACLE_LIBM"] = "glibc"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "libm_workload.py"), path], env=env, check=True,
                   timeout=300)
    return np.load(path)


def compare(a, b, tol=1e-4):
    """Per workload: problems, problems within tolerance, bit-equal problems, decisions compared,
    max pose difference; and the list of mismatching problems."""
    out, bad = {}, []
    for k in sorted(a.files):
        if not k.endswith("_d"):
            continue
        base = k[:-2]
        name = base.split("_")[0]
        d_eq = np.array_equal(a[base + "_d"], b[base + "_d"])
        b_eq = np.array_equal(a[base + "_b"], b[base + "_b"])
        pa, pb = a[base + "_p"], b[base + "_p"]
        pd = float(np.max(np.abs(pa - pb))) if pa.size else 0.0
        bit = d_eq and b_eq and np.array_equal(pa.view(np.uint64), pb.view(np.uint64))
        s = out.setdefault(name, dict(problems=0, within_tol=0, bit_equal=0, decision_bytes=0, max_pose_diff=0.0))
        s["problems"] += 1
        s["decision_bytes"] += int(a[base + "_b"].size)
        ok = d_eq and b_eq and pd <= tol
        s["within_tol"] += int(ok)
        s["bit_equal"] += int(bit)
        s["max_pose_diff"] = max(s["max_pose_diff"], pd)
        if not ok:
            bad.append((base, d_eq, b_eq, pd))
    return out, bad


@pytest.mark.skipif(not os.path.exists(GLIBC), reason="oracle glibc build missing (make -C oracle all)")
def test_fdlibm_restatement_vs_glibc_outcomes(tmp_path):
    a, b = _run(tmp_path, "fdlibm"), _run(tmp_path, "glibc")
    stats, bad = compare(a, b)
    total = sum(s["problems"] for s in stats.values())
    within = sum(s["within_tol"] for s in stats.values())
    assert set(stats) == {"mlpnp", "poseopt", "sim3match", "sim3opt"}
    assert within / total >= 0.999, (stats, bad)
    for name, s in stats.items():
        assert s["problems"] >= 32, (name, s)
