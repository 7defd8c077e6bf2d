"""profiles/r05/order_choice.json (r04 + the MLPnP sites, config 4) — how much the association order of the 3-term fixed-size Eigen
reductions matters (VERDICT r3 "Next round" 8).

Two builds of the same oracle sources: librsc_oracle_ltr.so (-DORA_LTR_ORDER: every sum left to
right, the rounds 1-3 restatement) and librsc_oracle.so (Eigen 3.3's order on the reference's x86-64
SSE2 build: `ered3` / `emv3d_row`, oracle/ora_linalg.h), run on the config 2 / 3 / 5 workloads by
tools/oracle_ab.py (config 4 MLPnP since round 5).  "full" = the bench shapes, "quick" = the reduced shapes that
tests/test_cpu_order_choice.py recomputes and compares with this file.

    python tools/order_choice.py profiles/r05/order_choice.json
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "oracle", "build")
SITES = {
    "PnPsolver.cpp:250": "CheckInliers mRi*p3Dw + mti (Matrix3f*Vector3f, all rows ered3)",
    "PnPsolver.cpp:338": "compute_barycentric_coordinates CC_inv.row(j).dot(...) (ered3)",
    "PnPsolver.cpp:423": "reprojection_error R*pws.row(i)^T + t (Matrix3d*Vector3d: rows 0-1 packet chain, row 2 ered3)",
    "PnPsolver.cpp:492": "estimate_R_and_t t = pc0 - R*pw0 (as :423)",
    "PnPsolver.cpp:626-635": "compute_L_6x10 dv rows dot (ered3)",
    "PnPsolver.cpp:640-645": "compute_rho squaredNorm of cws rows (ered3)",
    "Sim3Solver.cpp:58,62": "ctor Rcw*X3Dw + tcw (Matrix3f*Vector3f, ered3)",
    "Sim3Solver.cpp:188": "ComputeCentroid P.rowwise().sum() (ered3)",
    "Sim3Solver.cpp:212": "M = Pr2*Pr1^T (ered3)",
    "Sim3Solver.cpp:253": "t12 = O1 - R12*O2 (ered3)",
    "Sim3Solver.cpp:264": "T21 = T12.inverse(): -(R21*t12) (ered3)",
    "Sim3Solver.cpp:320": "Project Rcw*P3Dw + tcw (ered3)",
    "MLPnPsolver.cpp:363": "planar branch eigenRot*points3.col(i) (Matrix3d*Vector3d: emv3d_row)",
    "MLPnPsolver.cpp:548": "planar sign test Ts[i].block<3,3>*points3v[p] + t (emv3d_row)",
    "MLPnPsolver.cpp:576": "tout = Rout*(scale*t) (emv3d_row)",
    "MLPnPsolver.cpp:591": "direction test Ts[s].block<3,3>*points3v[p] + t (emv3d_row)",
    "MLPnPsolver.cpp:738": "mlpnp_residuals_and_jacs R*pts[i] + T (emv3d_row)",
}


def run(quick):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import oracle_ab
    with tempfile.TemporaryDirectory() as d:
        paths = {}
        for name, lib in (("ltr", "librsc_oracle_ltr.so"), ("eigen", "librsc_oracle.so")):
            paths[name] = os.path.join(d, name + ".npz")
            cmd = [sys.executable, os.path.join(ROOT, "tools", "oracle_ab.py"), "dump", paths[name],
                   "--lib", os.path.join(BUILD, lib)] + (["--quick"] if quick else [])
            subprocess.run(cmd, check=True, timeout=600)
        return oracle_ab.compare(paths["ltr"], paths["eigen"])


if __name__ == "__main__":
    rep = dict(a="left to right (rounds 1-3)", b="Eigen 3.3 SSE2 order (round 4, kernels + oracle)", sites=SITES,
               full=run(False), quick=run(True))
    rep["decision"] = ("outcome agreement < 100 % (config 2 parity-mode outcomes, config 5 winners): the kernels "
                       "and the checker oracle follow the Eigen order")
    with open(sys.argv[1], "w") as f:
        json.dump(rep, f, indent=1)
        f.write("\n")
    print(json.dumps({k: {a: b for a, b in v.items() if not isinstance(b, (list, dict))}
                      for k, v in rep["full"].items()}, indent=1))
