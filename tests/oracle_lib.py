"""ctypes binding of the parity oracle (oracle/build/librsc_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The oracle is the checker, never the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RSC_ORACLE_LIBM=glibc selects the build whose transcendental functions are host glibc's (the
# reference's), for tests/test_cpu_libm_choice.py; the default build is the checker.
LIB_PATH = os.path.join(ROOT, "oracle", "build",
                        "librsc_oracle_glibc.so" if os.environ.get("RSC_ORACLE_LIBM") == "glibc"
                        else "librsc_oracle.so")
# RSC_ORACLE_LIB=<path>: another build of the restatement (tools/oracle_ab.py compares two builds,
# e.g. an arithmetic-order variant or the previous round's oracle).
LIB_PATH = os.environ.get("RSC_ORACLE_LIB", LIB_PATH)

_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build_oracle() -> str:
    if "RSC_ORACLE_LIB" in os.environ:
        return LIB_PATH
    if not os.path.exists(LIB_PATH) or _stale():
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
    return LIB_PATH


def _stale() -> bool:
    src_dir = os.path.join(ROOT, "oracle")
    t = os.path.getmtime(LIB_PATH)
    for f in os.listdir(src_dir):
        if f.endswith((".cpp", ".h")) and os.path.getmtime(os.path.join(src_dir, f)) > t:
            return True
    return False


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build_oracle()
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.ora_pose_optimization.argtypes = [C.c_int, u8p, f32p, f32p, f32p, C.c_float, C.c_float, C.c_float,
                                        C.c_float, f32p, f32p, u8p, i32p, C.c_void_p, C.c_float]
    L.ora_pose_optimization.restype = C.c_int
    L.ora_pose_optimization_batch.argtypes = [C.c_int, i64p, f32p, f32p, f32p, C.c_float, C.c_float, C.c_float,
                                              C.c_float, f32p, f32p, u8p, i32p, C.c_void_p, C.c_float]
    L.ora_optimize_sim3.argtypes = [C.c_int, u8p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, C.c_float,
                                    np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS"), u8p, i32p]
    L.ora_glibc_rand.argtypes = [C.c_uint32, C.c_int, i32p]
    L.ora_sample_stream.argtypes = [C.c_uint32, C.c_int, C.c_int, C.c_int, i32p]
    L.ora_pnp_create.restype = vp
    L.ora_pnp_create.argtypes = [C.c_int, C.c_int, f32p, f32p, f32p, i32p, C.c_float, C.c_float, C.c_float,
                                 C.c_float, C.c_uint32]
    L.ora_pnp_destroy.argtypes = [vp]
    for f in ("ora_pnp_use_libc_rand", "ora_sim3_use_libc_rand", "ora_mlpnp_use_libc_rand"):
        getattr(L, f).argtypes = [vp, C.c_int]
    L.ora_libc_srand.argtypes = [C.c_uint32]
    L.ora_libc_rand.restype = C.c_int
    L.ora_pnp_set_params.argtypes = [vp, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
    L.ora_pnp_iterate.argtypes = [vp, C.c_int, C.POINTER(C.c_int), u8p, C.POINTER(C.c_int), C.POINTER(C.c_int), f32p]
    L.ora_pnp_info.argtypes = [vp, i32p]
    L.ora_pnp_max_error.argtypes = [vp, f32p]
    L.ora_pnp_compute_pose.restype = C.c_double
    L.ora_pnp_compute_pose.argtypes = [vp, i32p, C.c_int, f32p, f32p]
    L.ora_pnp_check_inliers.argtypes = [vp, f32p, f32p, u8p]
    L.ora_pnp_trace_enable.argtypes = [vp]
    L.ora_pnp_trace_get.argtypes = [vp, C.c_int, i32p, f32p]
    L.ora_pnp_run_batch.argtypes = [C.c_int, i32p, i64p, f32p, f32p, f32p, C.c_float, C.c_float, C.c_float,
                                    C.c_float, u32p, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                    C.c_int, C.c_int, i32p, f32p, C.c_void_p]
    L.ora_sim3_create.restype = vp
    L.ora_sim3_create.argtypes = [C.c_int, u8p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p, f32p,
                                  C.c_uint32]
    L.ora_sim3_destroy.argtypes = [vp]
    L.ora_sim3_set_params.argtypes = [vp, C.c_double, C.c_int, C.c_int]
    L.ora_sim3_n.argtypes = [vp]
    L.ora_sim3_prepared.argtypes = [vp, f32p, f32p, f32p, f32p, u64p, u64p, i32p]
    L.ora_sim3_iterate.argtypes = [vp, C.c_int, C.POINTER(C.c_int), u8p, C.POINTER(C.c_int)]
    L.ora_sim3_estimate.argtypes = [vp, f32p, f32p]
    L.ora_sim3_info.argtypes = [vp, i32p]
    L.ora_sim3_compute.argtypes = [vp, i32p, f32p, f32p]
    L.ora_sim3_check_inliers.argtypes = [vp, f32p, f32p, u8p]
    L.ora_sim3_trace_enable.argtypes = [vp]
    L.ora_sim3_trace_get.argtypes = [vp, C.c_int, i32p, f32p]
    L.ora_sim3_run_prepared_batch.argtypes = [C.c_int, i32p, i64p, f32p, f32p, f32p, f32p, u64p, u64p, f32p, f32p,
                                              u32p, C.c_double, C.c_int, C.c_int, C.c_int, C.c_int, i32p, f32p]
    f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    L.ora_mlpnp_create.restype = vp
    L.ora_mlpnp_create.argtypes = [C.c_int, C.c_int, f32p, f32p, f32p, i32p, C.c_float, C.c_float, C.c_float,
                                   C.c_float, C.c_uint32]
    L.ora_mlpnp_destroy.argtypes = [vp]
    L.ora_mlpnp_set_cov.argtypes = [vp, C.c_void_p]
    L.ora_mlpnp_set_params.argtypes = [vp, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
    L.ora_mlpnp_iterate.argtypes = [vp, C.c_int, C.POINTER(C.c_int), u8p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    f32p]
    L.ora_mlpnp_info.argtypes = [vp, i32p]
    L.ora_mlpnp_compute_pose.argtypes = [vp, i32p, C.c_int, f64p, f64p]
    L.ora_mlpnp_trace_enable.argtypes = [vp]
    L.ora_mlpnp_trace_get.argtypes = [vp, C.c_int, i32p, f64p]
    L.ora_mlpnp_trace_planar.argtypes = [vp, C.c_int, i32p]
    L.ora_mlpnp_run_batch.argtypes = [C.c_int, i32p, i64p, f32p, f32p, f32p, C.c_float, C.c_float, C.c_float,
                                      C.c_float, u32p, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                      C.c_int, C.c_int, i32p, f32p]
    L.ora_reloc_events_batch.argtypes = [C.c_int, i32p, i32p, i64p, f32p, f32p, f32p, C.c_float, C.c_float,
                                         C.c_float, C.c_float, u32p, C.c_double, C.c_int, C.c_int, C.c_int,
                                         C.c_float, C.c_float, C.c_int, i32p, f32p]
    L.ora_loop_events_batch.argtypes = [C.c_int, i32p, i32p, i64p, u8p, f32p, f32p, f32p, f32p, f32p, u32p,
                                        C.c_double, C.c_int, C.c_int, C.c_int, i32p, f32p]
    for fn in ("ora_dm_sin", "ora_dm_cos", "ora_dm_acos", "ora_dm_cbrt") + \
            tuple(f for f in ("ora_dm_pow13", "ora_dm_pow32") if hasattr(L, f)):
        getattr(L, fn).restype = C.c_double
        getattr(L, fn).argtypes = [C.c_double]
    L.ora_mlpnp_jac.argtypes = [f64p, f64p, f64p, f64p, f64p]
    if hasattr(L, "ora_qr_solve"):  # absent from round-3 builds compared by tools/oracle_ab.py
        L.ora_qr_solve.argtypes = [f64p, f64p, f64p]
        L.ora_qr_solve.restype = C.c_int
    L.ora_sym_eig.argtypes = [C.c_int, f64p, f64p, f64p]
    L.ora_sym_eig4f.argtypes = [f32p, f32p, f32p]
    L.ora_svd_solve.argtypes = [C.c_int, f64p, f64p, f64p]
    L.ora_random_int.argtypes = [C.c_uint32, C.c_int, i32p, i32p]
    L.ora_bow_create.restype = vp
    L.ora_bow_create.argtypes = [C.c_int, u8p, f32p, C.c_void_p, C.c_int, u32p, i32p, u32p]
    L.ora_bow_destroy.argtypes = [vp]
    L.ora_search_by_bow.argtypes = [C.c_int, vp, vp, C.c_float, C.c_int, i32p]
    L.ora_search_by_bow_many.restype = C.c_int64
    L.ora_search_by_bow_many.argtypes = [C.c_int, C.c_int, C.POINTER(vp), vp, C.c_float, C.c_int, i32p,
                                         C.c_int64, i32p]
    L.ora_descriptor_distance.argtypes = [u8p, u8p]
    L.ora_search_by_sim3.argtypes = [vp, vp, i32p, f32p, f32p, C.c_float, i32p]
    L.ora_predict_scale.argtypes = [C.c_float, C.c_float, C.c_float, C.c_int]
    u32p_ = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
    f64p_ = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    u64p_ = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
    L.ora_kfdb_create.restype = vp
    L.ora_kfdb_create.argtypes = [C.c_int]
    L.ora_kfdb_destroy.argtypes = [vp]
    L.ora_kfdb_add.argtypes = [vp, C.c_int, C.c_int, u32p_, f64p_]
    L.ora_kfdb_erase.argtypes = [vp, C.c_int]
    L.ora_kfdb_clear.argtypes = [vp]
    L.ora_kfdb_set_covisibility.argtypes = [vp, C.c_int, C.c_int, i32p]
    L.ora_kfdb_detect_relocalization.argtypes = [vp, C.c_uint64, C.c_int, u32p_, f64p_, i32p]
    L.ora_kfdb_detect_loop.argtypes = [vp, C.c_uint64, C.c_int, u32p_, f64p_, C.c_int, i32p, C.c_float, i32p]
    L.ora_kfdb_state.argtypes = [vp, C.c_int, u64p_, i32p, f32p]
    L.ora_l1_score.restype = C.c_double
    L.ora_l1_score.argtypes = [C.c_int, u32p_, f64p_, C.c_int, u32p_, f64p_]
    L.ora_dm_log.restype = C.c_double
    L.ora_dm_log.argtypes = [C.c_double]
    L.ora_compute_three_maxima.argtypes = [i32p, C.c_int, i32p]
    _lib = L
    return L


def sym_eig(A):
    A = np.ascontiguousarray(A, np.float64)
    n = A.shape[0]
    V = np.zeros((n, n)); w = np.zeros(n)
    st = lib().ora_sym_eig(n, A.ravel(), V.reshape(-1), w)
    return w, V, st == 0


def sym_eig4f(A):
    A = np.ascontiguousarray(A, np.float32)
    V = np.zeros((4, 4), np.float32); w = np.zeros(4, np.float32)
    st = lib().ora_sym_eig4f(A.ravel(), V.reshape(-1), w)
    return w, V, st == 0


def svd_solve(A, b):
    A = np.ascontiguousarray(A, np.float64)
    k = A.shape[1]
    x = np.zeros(k)
    lib().ora_svd_solve(k, A.ravel(), np.ascontiguousarray(b, np.float64), x)
    return x


def qr_solve(A, b, X0):
    """PnPsolver::qr_solve (PnPsolver.cpp:693-796) as restated: (X, ok)."""
    A = np.array(A, np.float64).reshape(24)
    b = np.array(b, np.float64).reshape(6)
    X = np.array(X0, np.float64).reshape(4)
    ok = lib().ora_qr_solve(A, b, X)
    return X, bool(ok)


def random_int(seed, maxes):
    maxes = np.ascontiguousarray(maxes, np.int32)
    out = np.zeros(len(maxes), np.int32)
    lib().ora_random_int(seed, len(maxes), maxes, out)
    return out


def glibc_rand(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.int32)
    lib().ora_glibc_rand(seed, n, out)
    return out


def sample_stream(seed: int, N: int, min_set: int, hyps: int) -> np.ndarray:
    out = np.zeros(hyps * min_set, dtype=np.int32)
    lib().ora_sample_stream(seed, N, min_set, hyps, out)
    return out.reshape(hyps, min_set)


class OraclePnP:
    """PnPsolver restatement: same ctor/SetRansacParameters/iterate/find semantics."""

    def __init__(self, scene, seed: int = 1):
        self._keep = (np.ascontiguousarray(scene.p2d, np.float32), np.ascontiguousarray(scene.p3dw, np.float32),
                      np.ascontiguousarray(scene.sigma2, np.float32), np.ascontiguousarray(scene.kp_index, np.int32))
        self.n_points = int(scene.n_points)
        self.h = lib().ora_pnp_create(scene.n, self.n_points, *self._keep, scene.fx, scene.fy, scene.cx,
                                      scene.cy, seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_pnp_destroy(self.h)
            self.h = None

    def use_libc_rand(self, on=True):
        """Draw samples from the process-global libc rand() (the reference's RandomInt source, Q3);
        seed it with libc_srand.  on=False: back to the own srand(seed) stream where it stopped."""
        lib().ora_pnp_use_libc_rand(self.h, int(on))

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=4,
                              epsilon=0.4, th2=5.991):
        lib().ora_pnp_set_params(self.h, probability, min_inliers, max_iterations, min_set, epsilon, th2)

    def iterate(self, n_iterations: int):
        nm, ml, ni = C.c_int(), C.c_int(), C.c_int()
        mask = np.zeros(max(self.n_points, 1), dtype=np.uint8)
        T = np.zeros(16, dtype=np.float32)
        ok = lib().ora_pnp_iterate(self.h, n_iterations, C.byref(nm), mask, C.byref(ml), C.byref(ni), T)
        return dict(ok=bool(ok), no_more=bool(nm.value), n_inliers=ni.value,
                    inliers=mask[:ml.value].astype(bool), T=T.reshape(4, 4), iterations=self.info()["iterations"])

    def info(self):
        out = np.zeros(5, dtype=np.int32)
        lib().ora_pnp_info(self.h, out)
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]), max_rows=int(out[4]))

    def max_error(self, n):
        out = np.zeros(n, dtype=np.float32)
        lib().ora_pnp_max_error(self.h, out)
        return out

    def compute_pose(self, idx):
        idx = np.ascontiguousarray(idx, np.int32)
        R = np.zeros(9, np.float32)
        t = np.zeros(3, np.float32)
        e = lib().ora_pnp_compute_pose(self.h, idx, len(idx), R, t)
        return R.reshape(3, 3), t, e

    def check_inliers(self, R, t, n):
        inl = np.zeros(n, np.uint8)
        c = lib().ora_pnp_check_inliers(self.h, np.ascontiguousarray(R, np.float32).ravel(),
                                        np.ascontiguousarray(t, np.float32), inl)
        return c, inl.astype(bool)

    def enable_trace(self):
        lib().ora_pnp_trace_enable(self.h)

    def trace(self, cap=100000):
        ints = np.zeros((cap, 12), np.int32)
        fl = np.zeros((cap, 12), np.float32)
        n = lib().ora_pnp_trace_get(self.h, cap, ints, fl)
        return ints[:n], fl[:n]


class OracleSim3:
    def __init__(self, pair, seed: int = 1):
        self._keep = [np.ascontiguousarray(a) for a in (
            pair.valid.astype(np.uint8), pair.Xw1.astype(np.float32), pair.Xw2.astype(np.float32),
            pair.sigma2_1.astype(np.float32), pair.sigma2_2.astype(np.float32),
            pair.R1.astype(np.float32).ravel(), pair.t1.astype(np.float32), pair.R2.astype(np.float32).ravel(),
            pair.t2.astype(np.float32), pair.K1.astype(np.float32), pair.K2.astype(np.float32))]
        self.n1 = pair.n1
        self.h = lib().ora_sim3_create(self.n1, *self._keep, seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_sim3_destroy(self.h)
            self.h = None

    def use_libc_rand(self, on=True):
        """Draw samples from the process-global libc rand() (the reference's RandomInt source, Q3);
        seed it with libc_srand.  on=False: back to the own srand(seed) stream where it stopped."""
        lib().ora_sim3_use_libc_rand(self.h, int(on))

    @property
    def N(self):
        return lib().ora_sim3_n(self.h)

    def prepared(self):
        N = self.N
        X1 = np.zeros((N, 3), np.float32); X2 = np.zeros((N, 3), np.float32)
        P1 = np.zeros((N, 2), np.float32); P2 = np.zeros((N, 2), np.float32)
        e1 = np.zeros(N, np.uint64); e2 = np.zeros(N, np.uint64); idx = np.zeros(N, np.int32)
        lib().ora_sim3_prepared(self.h, X1, X2, P1, P2, e1, e2, idx)
        return dict(X1c=X1, X2c=X2, P1im1=P1, P2im2=P2, maxerr1=e1, maxerr2=e2, indices=idx)

    def set_ransac_parameters(self, probability=0.99, min_inliers=6, max_iterations=300):
        lib().ora_sim3_set_params(self.h, probability, min_inliers, max_iterations)

    def iterate(self, n_iterations: int):
        nm, ni = C.c_int(), C.c_int()
        mask = np.zeros(max(self.n1, 1), np.uint8)
        ok = lib().ora_sim3_iterate(self.h, n_iterations, C.byref(nm), mask, C.byref(ni))
        R = np.zeros(9, np.float32); t = np.zeros(3, np.float32)
        lib().ora_sim3_estimate(self.h, R, t)
        return dict(ok=bool(ok), no_more=bool(nm.value), n_inliers=ni.value, inliers=mask[:self.n1].astype(bool),
                    R=R.reshape(3, 3), t=t, iterations=self.info()["iterations"])

    def info(self):
        out = np.zeros(3, np.int32)
        lib().ora_sim3_info(self.h, out)
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), N=int(out[2]))

    def compute(self, idx):
        R = np.zeros(9, np.float32); t = np.zeros(3, np.float32)
        lib().ora_sim3_compute(self.h, np.ascontiguousarray(idx, np.int32), R, t)
        return R.reshape(3, 3), t

    def enable_trace(self):
        lib().ora_sim3_trace_enable(self.h)

    def trace(self, cap=100000):
        ints = np.zeros((cap, 4), np.int32)
        fl = np.zeros((cap, 12), np.float32)
        n = lib().ora_sim3_trace_get(self.h, cap, ints, fl)
        return ints[:n], fl[:n]


class OracleMLPnP:
    """MLPnPsolver restatement (parity unpinned, see oracle/mlpnp_oracle.h)."""

    def __init__(self, scene, seed: int = 1):
        self._keep = (np.ascontiguousarray(scene.p2d, np.float32), np.ascontiguousarray(scene.p3dw, np.float32),
                      np.ascontiguousarray(scene.sigma2, np.float32), np.ascontiguousarray(scene.kp_index, np.int32))
        self.n_points = int(scene.n_points)
        self.h = lib().ora_mlpnp_create(scene.n, self.n_points, *self._keep, scene.fx, scene.fy, scene.cx,
                                        scene.cy, seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_mlpnp_destroy(self.h)
            self.h = None

    def use_libc_rand(self, on=True):
        """Draw samples from the process-global libc rand() (the reference's RandomInt source, Q3);
        seed it with libc_srand.  on=False: back to the own srand(seed) stream where it stopped."""
        lib().ora_mlpnp_use_libc_rand(self.h, int(on))

    def set_covariances(self, cov):
        """computePose's covMats ([n, 3, 3]) or None."""
        if cov is None:
            lib().ora_mlpnp_set_cov(self.h, None)
            return
        self._cov = np.ascontiguousarray(np.asarray(cov, np.float64).reshape(-1, 9))
        lib().ora_mlpnp_set_cov(self.h, self._cov.ctypes.data)

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=6, epsilon=0.4,
                              th2=5.991):
        lib().ora_mlpnp_set_params(self.h, probability, min_inliers, max_iterations, min_set, epsilon, th2)

    def iterate(self, n_iterations: int):
        nm, ml, ni = C.c_int(), C.c_int(), C.c_int()
        mask = np.zeros(max(self.n_points, 1), np.uint8)
        T = np.zeros(16, np.float32)
        ok = lib().ora_mlpnp_iterate(self.h, n_iterations, C.byref(nm), mask, C.byref(ml), C.byref(ni), T)
        return dict(ok=bool(ok), no_more=bool(nm.value), n_inliers=ni.value,
                    inliers=mask[:ml.value].astype(bool), T=T.reshape(4, 4), iterations=self.info()["iterations"])

    def info(self):
        out = np.zeros(4, np.int32)
        lib().ora_mlpnp_info(self.h, out)
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]))

    def compute_pose(self, idx):
        idx = np.ascontiguousarray(idx, np.int32)
        R = np.zeros(9)
        t = np.zeros(3)
        lib().ora_mlpnp_compute_pose(self.h, idx, len(idx), R, t)
        return R.reshape(3, 3), t

    def enable_trace(self):
        lib().ora_mlpnp_trace_enable(self.h)

    def trace(self, cap=100000):
        ints = np.zeros((cap, 9), np.int32)
        dbl = np.zeros((cap, 12))
        n = lib().ora_mlpnp_trace_get(self.h, cap, ints, dbl)
        return ints[:n], dbl[:n]

    def trace_planar(self, cap=100000):
        """bool per traced hypothesis: computePose took the planar branch (rank(PP^T) == 2)."""
        out = np.zeros(cap, np.int32)
        n = lib().ora_mlpnp_trace_planar(self.h, cap, out)
        return out[:n].astype(bool)


def pose_optimization(frame):
    """Optimizer::PoseOptimization on the oracle: (nGood, Tcw float32[4,4], outlier uint8[n], stats[3]).
    outlier slots without a map point are 255 (untouched)."""
    L = lib()
    n = frame.n
    T = np.zeros(16, np.float32)
    out = np.full(n, 255, np.uint8)
    st = np.zeros(3, np.int32)
    ur = getattr(frame, "u_right", None)
    ur = None if ur is None else np.ascontiguousarray(ur, np.float32)
    r = L.ora_pose_optimization(n, np.ascontiguousarray(frame.has_mp, np.uint8),
                                np.ascontiguousarray(frame.uv, np.float32),
                                np.ascontiguousarray(frame.Xw, np.float32),
                                np.ascontiguousarray(frame.inv_sigma2, np.float32), frame.fx, frame.fy, frame.cx,
                                frame.cy, np.ascontiguousarray(frame.Tcw, np.float32).reshape(16), T, out, st,
                                None if ur is None else ur.ctypes.data, float(getattr(frame, "bf", 0.0)))
    if r == 0 and not T.any():
        T = np.ascontiguousarray(frame.Tcw, np.float32).reshape(16).copy()
    return r, T.reshape(4, 4), out, st


class OracleBow:
    """A view (rsc.synth.BowFeatures) held by the oracle with its FeatureVector as a std::map."""

    def __init__(self, view):
        self.n = int(view.n)
        self._keep = [np.ascontiguousarray(view.desc, np.uint8).reshape(-1),
                      np.ascontiguousarray(view.angle, np.float32),
                      None if view.valid is None else np.ascontiguousarray(view.valid, np.uint8),
                      np.ascontiguousarray(view.node_id, np.uint32), np.ascontiguousarray(view.node_begin, np.int32),
                      np.ascontiguousarray(view.feat, np.uint32)]
        d, a, v, ids, beg, feat = self._keep
        if feat.size == 0:
            feat = np.zeros(1, np.uint32)
            self._keep[5] = feat
        if d.size == 0:
            d = np.zeros(32, np.uint8)
            a = np.zeros(1, np.float32)
            self._keep[0], self._keep[1] = d, a
        if ids.size == 0:
            ids = np.zeros(1, np.uint32)
            self._keep[3] = ids
        self.h = lib().ora_bow_create(self.n, d, a, None if v is None else v.ctypes.data,
                                      len(view.node_id), ids, beg, feat)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_bow_destroy(self.h)
            self.h = None


def search_by_bow(frame_variant: bool, a: OracleBow, b: OracleBow, nnratio=0.75, check_ori=True):
    """frame_variant: SearchByBoW(pKF = a, F = b) -> (nmatches, int32[b.n]); else
    SearchByBoW(pKF1 = a, pKF2 = b) -> (nmatches, int32[a.n])."""
    out = np.full(max(b.n if frame_variant else a.n, 1), -7, np.int32)
    nm = lib().ora_search_by_bow(int(frame_variant), a.h, b.h, nnratio, int(check_ori), out)
    return nm, out[:(b.n if frame_variant else a.n)]


def search_by_bow_many(frame_variant: bool, others, shared, nnratio=0.75, check_ori=True):
    """Frame variant: SearchByBoW(others[c], shared); KF variant: SearchByBoW(shared, others[c]).
    Returns (matches int32[count, shared.n], nmatches int32[count])."""
    L = lib()
    out = np.full((max(len(others), 1), max(shared.n, 1)), -7, np.int32)
    nm = np.zeros(max(len(others), 1), np.int32)
    for c, o in enumerate(others):
        a, b = (o, shared) if frame_variant else (shared, o)
        nm[c] = L.ora_search_by_bow(int(frame_variant), a.h, b.h, nnratio, int(check_ori), out[c])
    return out[:len(others), :shared.n], nm[:len(others)]


def descriptor_distance(a, b) -> int:
    return lib().ora_descriptor_distance(np.ascontiguousarray(a, np.uint8), np.ascontiguousarray(b, np.uint8))


def compute_three_maxima(sizes):
    ind = np.zeros(3, np.int32)
    lib().ora_compute_three_maxima(np.ascontiguousarray(sizes, np.int32), len(sizes), ind)
    return tuple(int(x) for x in ind)


def search_by_sim3(kf1, kf2, R12, t12, matched12, th=7.5):
    """ORBmatcher::SearchBySim3 on the oracle: (nfound, out12 int32[kf1.n])."""
    from rsc import engine
    k1, keep1 = engine.sim3_kf_struct(kf1)
    k2, keep2 = engine.sim3_kf_struct(kf2)
    out = np.full(max(kf1.n, 1), -7, np.int32)
    nf = lib().ora_search_by_sim3(C.addressof(k1), C.addressof(k2), np.ascontiguousarray(matched12, np.int32),
                                  np.ascontiguousarray(np.asarray(R12, np.float32).reshape(9)),
                                  np.ascontiguousarray(np.asarray(t12, np.float32).reshape(3)), th, out)
    return nf, out[:kf1.n]


class OracleKFDB:
    """KeyFrameDatabase on the oracle (oracle/kfdb_oracle.h); same interface as
    rsc.engine.KeyFrameDatabase."""

    def __init__(self, capacity: int):
        self.capacity = int(capacity)
        self.h = lib().ora_kfdb_create(self.capacity)
        self._cand = np.zeros(max(self.capacity, 1), np.int32)

    @staticmethod
    def _bow(ids, vals):
        return np.ascontiguousarray(ids, np.uint32), np.ascontiguousarray(vals, np.float64)

    def add(self, kf, ids, vals):
        i, v = self._bow(ids, vals)
        lib().ora_kfdb_add(self.h, int(kf), len(i), i, v)

    def erase(self, kf):
        lib().ora_kfdb_erase(self.h, int(kf))

    def clear(self):
        lib().ora_kfdb_clear(self.h)

    def set_covisibility(self, kf, best):
        b = np.ascontiguousarray(best, np.int32)
        lib().ora_kfdb_set_covisibility(self.h, int(kf), len(b), b)

    def detect_relocalization(self, frame_id, ids, vals):
        i, v = self._bow(ids, vals)
        n = lib().ora_kfdb_detect_relocalization(self.h, int(frame_id), len(i), i, v, self._cand)
        return self._cand[:n].copy()

    def detect_loop(self, kf_id, ids, vals, connected, min_score):
        i, v = self._bow(ids, vals)
        c = np.ascontiguousarray(connected, np.int32)
        n = lib().ora_kfdb_detect_loop(self.h, int(kf_id), len(i), i, v, len(c), c, float(min_score), self._cand)
        return self._cand[:n].copy()

    def state(self, kf):
        q = np.zeros(2, np.uint64)
        w = np.zeros(2, np.int32)
        s = np.zeros(2, np.float32)
        lib().ora_kfdb_state(self.h, int(kf), q, w, s)
        return tuple(int(x) for x in q), tuple(int(x) for x in w), tuple(float(x) for x in s)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_kfdb_destroy(self.h)
            self.h = None


def l1_score(ids1, v1, ids2, v2) -> float:
    a, b = np.ascontiguousarray(ids1, np.uint32), np.ascontiguousarray(ids2, np.uint32)
    return lib().ora_l1_score(len(a), a, np.ascontiguousarray(v1, np.float64), len(b), b,
                              np.ascontiguousarray(v2, np.float64))


def optimize_sim3(p):
    """Optimizer::OptimizeSim3 on the oracle for a rsc.synth.Sim3OptProblem: (nIn, S float64[8] = q (x, y,
    z, w), t, s after the call, keep uint8[n] (0 where vpMatches1[i] is set to NULL), stats[4])."""
    n = p.n
    S = np.ascontiguousarray(p.S0, np.float64).copy()
    keep = np.zeros(max(n, 1), np.uint8)
    st = np.zeros(4, np.int32)
    r = lib().ora_optimize_sim3(n, np.ascontiguousarray(p.valid, np.uint8), np.ascontiguousarray(p.X1w, np.float32),
                                np.ascontiguousarray(p.X2w, np.float32), np.ascontiguousarray(p.uv1, np.float32),
                                np.ascontiguousarray(p.uv2, np.float32), np.ascontiguousarray(p.inv1, np.float32),
                                np.ascontiguousarray(p.inv2, np.float32), p.poses24(), p.K8(), float(p.th2), S, keep, st)
    return r, S, keep[:n], st


def libc_srand(seed: int):
    """srand(seed) of the process-global libc stream the use_libc_rand solvers draw from."""
    lib().ora_libc_srand(seed)


def libc_rand() -> int:
    return int(lib().ora_libc_rand())
