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
        L.he_sim3_hypothesis.argtypes = [u32p, C.c_int, C.c_int, C.c_int, f32p, f32p, i32p, f32p]
        L.he_sim3_count.argtypes = [f32p, f32p, f32p, C.c_int, f32p, f32p, f32p, f32p, u64p, u64p, u8p]
        _lib = L
    return _lib


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
