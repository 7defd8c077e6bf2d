"""ctypes binding of tests/hostemu (TEST-ONLY host build of the product's per-lane numerics)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "hostemu", "build", "libhostemu.so")
_lib = None
f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "hostemu")])
        L = C.CDLL(LIB)
        L.he_rng_window.argtypes = [C.c_uint32, u32p, C.POINTER(C.c_int32)]
        L.he_rand_stream.argtypes = [C.c_uint32, C.c_int, i32p]
        L.he_pnp_hypothesis.argtypes = [C.c_int, u32p, C.c_int, C.c_int, C.c_int, f32p, f32p, f32p, C.c_int,
                                        C.c_void_p, C.c_void_p, i32p, f32p, f32p]
        L.he_pnp_count.argtypes = [f32p, f32p, f32p, C.c_float, C.c_int, f32p, f32p, u8p]
        L.he_pnp_rows.restype = C.c_double
        L.he_pnp_rows.argtypes = [C.c_int, C.c_int, f64p, f64p, f64p, f32p, f32p, f32p]
        L.he_mlpnp_hypothesis.argtypes = [C.c_int, u32p, C.c_int, C.c_int, C.c_int, f32p, f32p, i32p, f64p, f64p]
        L.he_mlpnp_hypothesis_cov.argtypes = [C.c_int, u32p, C.c_int, C.c_int, C.c_int, f32p, f32p, f64p, i32p,
                                              f64p, f64p]
        L.he_mlpnp_count.argtypes = [f64p, f64p, f32p, C.c_float, C.c_int, f32p, f32p, u8p]
        L.he_sim3_hypothesis.argtypes = [u32p, C.c_int, C.c_int, C.c_int, f32p, f32p, i32p, f32p]
        L.he_sim3_count.argtypes = [f32p, f32p, f32p, C.c_int, f32p, f32p, f32p, f32p, u64p, u64p, u8p]
        L.he_pose_optimization.argtypes = [C.c_int, f32p, f32p, f32p, f32p, f32p, u8p, C.c_void_p, C.c_float]
        L.he_qr_compare.argtypes = [f64p, f64p, i32p, f64p, i32p, f64p, i32p, f64p, i32p]
        L.he_qr_split.argtypes = [f64p, C.c_int, f64p, i32p, f64p, i32p]
        L.he_optimize_sim3.argtypes = [C.c_int, f32p, f32p, f32p, f32p, C.c_float, f64p, u8p, i32p]
        L.he_poll_until.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.he_po_fold_compare.argtypes = [C.c_int, f64p, f64p, f64p, i32p, f64p, f64p, f64p]
        _lib = L
    return _lib


def poll_until(limit, ready_after):
    """(held, loads, pauses) of rsc_core.h poll_until on a flag ready at load `ready_after`."""
    n, p = C.c_int(), C.c_int()
    ok = lib().he_poll_until(limit, ready_after, C.byref(n), C.byref(p))
    return bool(ok), n.value, p.value


def rand_stream(seed, n):
    out = np.zeros(n, np.int32)
    lib().he_rand_stream(seed, n, out)
    return out


def window(seed):
    w = np.zeros(31, np.uint32)
    g = C.c_int32()
    lib().he_rng_window(seed, w, C.byref(g))
    return w, g.value


def pack_pts(scene):
    pts4 = np.concatenate([scene.p3dw, scene.sigma2[:, None]], 1).astype(np.float32).copy()
    return pts4, np.ascontiguousarray(scene.p2d, np.float32)


def pnp_hypothesis(scene, seed, h, ns=4, rows=None, spw=None, sal=None):
    w, g0 = window(seed)
    pts4, uv = pack_pts(scene)
    K = np.array([scene.fx, scene.fy, scene.cx, scene.cy], np.float32)
    idx = np.zeros(8, np.int32)
    R = np.zeros(9, np.float32)
    t = np.zeros(3, np.float32)
    rows = ns if rows is None else rows
    lib().he_pnp_hypothesis(ns, w, g0, h, scene.n, pts4, uv, K, rows,
                            None if spw is None else spw.ctypes.data, None if sal is None else sal.ctypes.data,
                            idx, R, t)
    return idx[:ns], R.reshape(3, 3), t


def pnp_count(scene, R, t, th2=5.991):
    pts4, uv = pack_pts(scene)
    K = np.array([scene.fx, scene.fy, scene.cx, scene.cy], np.float32)
    m = np.zeros(scene.n, np.uint8)
    c = lib().he_pnp_count(np.ascontiguousarray(R, np.float32).ravel(), np.ascontiguousarray(t, np.float32), K,
                           th2, scene.n, pts4, uv, m)
    return c, m.astype(bool)


def bearings(scene):
    """MLPnPsolver bearing (x, y) per correspondence, float arithmetic (MLPnPsolver.cpp:32-33)."""
    fx, fy, cx, cy = (np.float32(v) for v in (scene.fx, scene.fy, scene.cx, scene.cy))
    p = np.asarray(scene.p2d, np.float32)
    return np.ascontiguousarray(np.stack([(p[:, 0] - cx) / fx, (p[:, 1] - cy) / fy], 1).astype(np.float32))


def mlpnp_hypothesis(scene, seed, h, ns=6, cov=None):
    w, g0 = window(seed)
    pts4, _ = pack_pts(scene)
    idx = np.zeros(8, np.int32)
    R = np.zeros(9)
    t = np.zeros(3)
    if cov is None:
        lib().he_mlpnp_hypothesis(ns, w, g0, h, scene.n, pts4, bearings(scene), idx, R, t)
    else:
        c = np.ascontiguousarray(np.asarray(cov, np.float64).reshape(-1, 9))
        lib().he_mlpnp_hypothesis_cov(ns, w, g0, h, scene.n, pts4, bearings(scene), c, idx, R, t)
    return idx[:ns], R.reshape(3, 3), t


def mlpnp_count(scene, R, t, th2=5.991):
    pts4, uv = pack_pts(scene)
    K = np.array([scene.fx, scene.fy, scene.cx, scene.cy], np.float32)
    m = np.zeros(scene.n, np.uint8)
    c = lib().he_mlpnp_count(np.ascontiguousarray(R, np.float64).ravel(), np.ascontiguousarray(t, np.float64), K,
                             th2, scene.n, pts4, uv, m)
    return c, m.astype(bool)


class EmuPnP:
    """Full PnPsolver::iterate emulation on the CPU: product replay logic (rsc_engine.h) + the
    host-compiled per-lane device numerics.  TEST-ONLY."""

    def __init__(self, scene, seed=1):
        L = lib()
        L.he_pnp_create.restype = C.c_void_p
        L.he_pnp_create.argtypes = [C.c_int, C.c_int, f32p, f32p, f32p, i32p, C.c_float, C.c_float, C.c_float,
                                    C.c_float, C.c_uint32]
        L.he_pnp_destroy.argtypes = [C.c_void_p]
        L.he_pnp_set_params.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
        L.he_pnp_iterate_many.argtypes = [C.POINTER(C.c_void_p), C.c_int, i32p, i32p, f32p, C.POINTER(C.c_void_p)]
        L.he_pnp_state.argtypes = [C.c_void_p, i32p]
        self._keep = (np.ascontiguousarray(scene.p2d, np.float32), np.ascontiguousarray(scene.p3dw, np.float32),
                      np.ascontiguousarray(scene.sigma2, np.float32), np.ascontiguousarray(scene.kp_index, np.int32))
        self.n_points = int(scene.n_points)
        self.h = L.he_pnp_create(scene.n, self.n_points, *self._keep, scene.fx, scene.fy, scene.cx, scene.cy, seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().he_pnp_destroy(self.h)
            self.h = None

    def set_ransac_parameters(self, *p):
        lib().he_pnp_set_params(self.h, *p)

    def state(self):
        out = np.zeros(5, np.int32)
        lib().he_pnp_state(self.h, out)
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]), max_rows=int(out[4]))

    def iterate(self, n):
        return iterate_many([self], n)[0]


def iterate_many(emus, n):
    k = len(emus)
    hs = (C.c_void_p * k)(*[e.h for e in emus])
    its = np.ascontiguousarray(np.broadcast_to(np.asarray(n, np.int32), (k,)))
    i4 = np.zeros(4 * k, np.int32)
    T = np.zeros(16 * k, np.float32)
    masks = [np.zeros(max(e.n_points, 1), np.uint8) for e in emus]
    mp = (C.c_void_p * k)(*[m.ctypes.data for m in masks])
    st = lib().he_pnp_iterate_many(hs, k, its, i4, T, mp)
    assert st == 0
    out = []
    for i in range(k):
        ok = bool(i4[4 * i])
        out.append(dict(ok=ok, no_more=bool(i4[4 * i + 1]), n_inliers=int(i4[4 * i + 2]),
                        iterations=int(i4[4 * i + 3]), T=T[16 * i:16 * i + 16].reshape(4, 4),
                        inliers=(masks[i][:emus[i].n_points].astype(bool) if ok else np.zeros(0, bool))))
    return out


def pose_optimization(frame):
    """Host build of the device PoseOptimization orchestration: (n_good, Tcw[4,4], outlier over the
    edges (slots with a map point, in slot order), stats[3])."""
    sel = np.nonzero(frame.has_mp)[0]
    n = len(sel)
    xw4 = np.zeros((n, 4), np.float32)
    xw4[:, :3] = frame.Xw[sel]
    xw4[:, 3] = frame.inv_sigma2[sel]
    uv = np.ascontiguousarray(frame.uv[sel], np.float32)
    K = np.array([frame.fx, frame.fy, frame.cx, frame.cy], np.float32)
    T12 = np.ascontiguousarray(frame.Tcw[:3], np.float32).reshape(12)
    out = np.zeros(16, np.float32)
    outl = np.zeros(max(n, 1), np.uint8)
    ur = getattr(frame, "u_right", None)
    ur = None if ur is None else np.ascontiguousarray(np.asarray(ur, np.float32)[sel])
    lib().he_pose_optimization(n, xw4.reshape(-1) if n else np.zeros(4, np.float32), uv.reshape(-1) if n else
                               np.zeros(2, np.float32), K, T12, out, outl,
                               None if ur is None else ur.ctypes.data, float(getattr(frame, "bf", 0.0)))
    ints = out[12:].view(np.int32)
    T = np.eye(4, dtype=np.float32)
    T[:3] = out[:12].reshape(3, 4)
    return int(ints[0]), T, outl[:n], ints[1:].copy()


def sim3opt_compact(p):
    """Host compaction of a rsc.synth.Sim3OptProblem as rsc_optimize_sim3_many does it: per
    correspondence (P3D2c, inv1), (P3D1c, inv2), (uv1, uv2) with the float camera-frame transforms."""
    sel = np.nonzero(p.valid)[0]
    f = np.float32
    R1, t1, R2, t2 = (np.asarray(a, f) for a in (p.R1w, p.t1w, p.R2w, p.t2w))
    def cam(R, t, X):  # ((R0*x + R1*y) + R2*z) + t in float
        out = np.zeros((len(X), 3), f)
        for r in range(3):
            out[:, r] = ((R[r, 0] * X[:, 0] + R[r, 1] * X[:, 1]) + R[r, 2] * X[:, 2]) + t[r]
        return out
    X1 = np.asarray(p.X1w, f)[sel]
    X2 = np.asarray(p.X2w, f)[sel]
    e12 = np.concatenate([cam(R2, t2, X2), np.asarray(p.inv1, f)[sel, None]], 1)
    e21 = np.concatenate([cam(R1, t1, X1), np.asarray(p.inv2, f)[sel, None]], 1)
    uv = np.concatenate([np.asarray(p.uv1, f)[sel], np.asarray(p.uv2, f)[sel]], 1)
    return sel, np.ascontiguousarray(e12, f), np.ascontiguousarray(e21, f), np.ascontiguousarray(uv, f)


def optimize_sim3(p):
    """Host build of the device OptimizeSim3 orchestration: (nIn, S[8], keep over the slots, stats[4])."""
    sel, e12, e21, uv = sim3opt_compact(p)
    m = len(sel)
    S = np.ascontiguousarray(p.S0, np.float64).copy()
    keep_c = np.zeros(max(m, 1), np.uint8)
    st = np.zeros(4, np.int32)
    if m:
        lib().he_optimize_sim3(m, e12.reshape(-1), e21.reshape(-1), uv.reshape(-1), p.K8(), float(p.th2), S, keep_c, st)
    keep = np.ones(p.n, np.uint8)
    keep[sel] = keep_c[:m]
    return int(st[0]), S, keep, st


def po_fold_compare(X, e, inv, flags, pose7, K5):
    """PoseOptimization folds over the edges with the full and with the kernel's term form
    (hostemu he_po_fold_compare): returns (full [28], kernel [28], edges that took the full form)."""
    n = len(inv)
    out = np.zeros(56, np.float64)
    full = lib().he_po_fold_compare(n, np.ascontiguousarray(X, np.float64).reshape(-1),
                                    np.ascontiguousarray(e, np.float64).reshape(-1),
                                    np.ascontiguousarray(inv, np.float64), np.ascontiguousarray(flags, np.int32),
                                    np.ascontiguousarray(pose7, np.float64), np.ascontiguousarray(K5, np.float64), out)
    return out[:28], out[28:], full
