"""Q19 (qr_solve eta over rows k..4, PnPsolver.cpp:714-720): how often it matters on the bench
workloads.  Builds an instrumented oracle (-DORA_QR_STATS) into /tmp, counts the qr_solve column
scans in which row 5 is the strict column maximum (there the reference's eta differs from a six-row
eta, so the Gauss-Newton iterates round differently), and, given two tools/oracle_ab.py dumps of the
round-3 and round-4 oracles, how many float poses / counts / outcomes changed.

    python tools/q19_stats.py R3.npz R4.npz OUT.json
"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_SO = "/tmp/rsc_oracle_qrstats.so"


def main(r3, r4, out):
    src = os.path.join(ROOT, "oracle")
    cpp = [os.path.join(src, f) for f in os.listdir(src) if f.endswith(".cpp")]
    subprocess.check_call(["g++", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
                           "-DORA_QR_STATS", "-shared", "-o", OUT_SO] + cpp + ["-lpthread"])
    os.environ["RSC_ORACLE_LIB"] = OUT_SO
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "orb-slam2-optimized_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import oracle_lib as ol
    from rsc import workloads as W
    import oracle_ab
    L = ol.lib()
    L.ora_qr_stats.argtypes = [ctypes.POINTER(ctypes.c_long)]
    rep = {}
    from rsc import synth
    import numpy as np
    prev = [0] * 6
    work = [("config2_exhaustive", lambda: W.config2_scenes(ratio=0.4)),
            ("config2_parity", lambda: W.config2_scenes(ratio=0.6))]
    for plane in ("floor", "wall", "tilted", "duplicates"):
        work.append((f"planar_{plane}_16x2000", lambda p=plane: [
            synth.make_planar_pnp_scene(np.random.default_rng(300 + i), 2000, 0.6, p) for i in range(16)]))
    for name, make in work:
        scenes = make()
        for sc, s in zip(scenes, W.config2_seeds(0, candidates=len(scenes))):
            o = ol.OraclePnP(sc, int(s))
            o.set_ransac_parameters(*W.RELOC)
            o.iterate(300)
        c = (ctypes.c_long * 6)()
        L.ora_qr_stats(c)
        cur = list(c)
        d = [a - b for a, b in zip(cur, prev)]
        prev = cur
        rep[name] = dict(qr_solve_calls=d[0], column_scans=4 * d[0],
                         scans_row5_strict_max=sum(d[1:5]), by_column=d[1:5],
                         fraction_of_scans=sum(d[1:5]) / max(1, 4 * d[0]),
                         singular_bailouts=d[5])
    rep["round3_vs_round4_oracle"] = oracle_ab.compare(r3, r4)
    rep["note"] = ("Q19 changes the double-precision Gauss-Newton iterates whenever row 5 is a column's "
                   "strict maximum; the float poses returned by compute_pose (cast at PnPsolver.cpp:411-412) "
                   "are what the counts, masks and outcomes depend on")
    txt = json.dumps(rep, indent=1)
    print(txt)
    open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:4])
