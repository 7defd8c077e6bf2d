"""ctypes binding of librsc.so (include/rsc.h) with the reference's solver API.

``PnPSolver`` / ``Sim3Solver`` mirror ORB_SLAM_CUSTOM::PnPsolver / Sim3Solver
(include/PnPsolver.hpp:24-31, include/Sim3Solver.hpp:21-30): same constructor inputs (already
reduced to plain arrays), ``set_ransac_parameters`` / ``iterate`` / ``find`` with the same argument
meaning and results.  Every call runs on the MI355X; there is no CPU fallback — if librsc.so is
missing or no HIP device is present the calls raise ``RuntimeError``.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RSC_LIBRSC: another build of the same library (A/B kernel comparisons in tools/); the default is
# the in-tree build.
LIB_PATH = os.environ.get("RSC_LIBRSC") or os.path.join(PKG_DIR, "lib", "librsc.so")

RSC_OK = 0

_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")

# Every symbol declared in include/rsc.h (checked by tests/test_cpu_abi.py).
EXPORTED = [
    "rsc_version", "rsc_status_string", "rsc_context_create", "rsc_context_destroy", "rsc_context_set_stream",
    "rsc_context_synchronize", "rsc_context_last_timing", "rsc_context_last_kernel_timing", "rsc_diag_host_timing", "rsc_context_enable_timing", "rsc_selftest_math",
    "rsc_context_set_eig_rows", "rsc_context_set_eig_split", "rsc_context_set_sim3opt_helpers",
    "rsc_pnp_create", "rsc_pnp_destroy", "rsc_pnp_set_ransac_parameters", "rsc_pnp_iterate", "rsc_pnp_find",
    "rsc_pnp_last_inliers",
    "rsc_pnp_iterate_many", "rsc_pnp_reset", "rsc_pnp_get_state", "rsc_pnp_last_samples", "rsc_pnp_last_hypotheses",
    "rsc_sim3_last_hypotheses", "rsc_mlpnp_last_counts",
    "rsc_sim3_create", "rsc_sim3_destroy", "rsc_sim3_set_ransac_parameters", "rsc_sim3_iterate", "rsc_sim3_find",
    "rsc_sim3_iterate_many", "rsc_sim3_reset", "rsc_sim3_get_state", "rsc_sim3_prepared", "rsc_rand_stream",
    "rsc_pnp_reset_many", "rsc_pnp_set_ransac_parameters_many", "rsc_sim3_reset_many",
    "rsc_sim3_set_ransac_parameters_many",
    "rsc_mlpnp_create", "rsc_mlpnp_destroy", "rsc_mlpnp_set_covariances", "rsc_mlpnp_set_ransac_parameters",
    "rsc_mlpnp_set_ransac_parameters_many", "rsc_mlpnp_iterate", "rsc_mlpnp_iterate_many", "rsc_mlpnp_reset",
    "rsc_mlpnp_reset_many", "rsc_mlpnp_get_state", "rsc_mlpnp_last_poses", "rsc_mlpnp_last_samples",
    "rsc_reloc_events", "rsc_loop_events", "rsc_pose_optimization_many",
    "rsc_bow_create", "rsc_bow_destroy", "rsc_bow_set_valid", "rsc_search_by_bow_frame_many",
    "rsc_search_by_bow_kf_many", "rsc_diag_bow_phase_stamps", "rsc_diag_refine_phase_stamps", "rsc_diag_solve_phase_stamps", "rsc_diag_poseopt_phases", "rsc_diag_sim3opt_phases", "rsc_diag_kfdb_stamps",
    "rsc_search_by_sim3_many", "rsc_kfview_create", "rsc_kfview_destroy",
    "rsc_optimize_sim3_many",
    "rsc_kfdb_create", "rsc_kfdb_destroy", "rsc_kfdb_add", "rsc_kfdb_erase", "rsc_kfdb_release", "rsc_kfdb_clear",
    "rsc_kfdb_set_covisibility", "rsc_kfdb_set_covisibility_many", "rsc_kfdb_detect_relocalization", "rsc_kfdb_detect_loop", "rsc_kfdb_state",
    "rsc_stream_create", "rsc_stream_destroy", "rsc_stream_skip", "rsc_stream_position", "rsc_stream_peek",
    "rsc_pnp_bind_stream", "rsc_sim3_bind_stream", "rsc_mlpnp_bind_stream", "rsc_reloc_events_shared",
    "rsc_loop_events_shared", "rsc_reloc_events_gated", "rsc_loop_events_gated",
    "rsc_diag_mlpnp_phase_stamps",
]

# include/rsc.h RSC_GATE_*
GATE_NONE, GATE_MATCH, GATE_HANDOFF = 0, 1, 2


class EventResult(C.Structure):
    _fields_ = [("winner", C.c_int32), ("round", C.c_int32), ("hypothesis", C.c_int32), ("n_inliers", C.c_int32)]


class RelocFrame(C.Structure):
    _fields_ = [("u_right", C.c_void_p), ("bf", C.c_float)]


class RelocGateResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("winner", C.c_int32), ("round", C.c_int32), ("hypothesis", C.c_int32),
                ("n_inliers", C.c_int32), ("n_good", C.c_int32), ("rejected", C.c_int32), ("gates", C.c_int32),
                ("Tcw", C.c_float * 16)]


class LoopCandidate(C.Structure):
    _fields_ = [("kf1", C.c_void_p), ("kf2", C.c_void_p), ("matches12", C.c_void_p)]


class LoopGateResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("winner", C.c_int32), ("round", C.c_int32), ("hypothesis", C.c_int32),
                ("n_inliers", C.c_int32), ("n_found", C.c_int32), ("n_opt_inliers", C.c_int32),
                ("rejected", C.c_int32), ("S", C.c_double * 8)]


class PnPProblem(C.Structure):
    _fields_ = [("n", C.c_int32), ("n_points", C.c_int32), ("p2d", C.c_void_p), ("p3dw", C.c_void_p),
                ("sigma2", C.c_void_p), ("kp_index", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float)]


class PnPResult(C.Structure):
    _fields_ = [("ok", C.c_int32), ("no_more", C.c_int32), ("n_inliers", C.c_int32), ("iterations", C.c_int32),
                ("T", C.c_float * 16)]


class Sim3Input(C.Structure):
    _fields_ = [("n1", C.c_int32), ("valid", C.c_void_p), ("Xw1", C.c_void_p), ("Xw2", C.c_void_p),
                ("sigma2_1", C.c_void_p), ("sigma2_2", C.c_void_p), ("R1", C.c_float * 9), ("t1", C.c_float * 3),
                ("R2", C.c_float * 9), ("t2", C.c_float * 3), ("K1", C.c_float * 4), ("K2", C.c_float * 4)]


class Sim3Result(C.Structure):
    _fields_ = [("ok", C.c_int32), ("no_more", C.c_int32), ("n_inliers", C.c_int32), ("iterations", C.c_int32),
                ("R", C.c_float * 9), ("t", C.c_float * 3)]


class PoseOptProblem(C.Structure):
    _fields_ = [("n", C.c_int32), ("has_mp", C.c_void_p), ("uv", C.c_void_p), ("Xw", C.c_void_p),
                ("inv_sigma2", C.c_void_p), ("u_right", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("Tcw", C.c_float * 16), ("bf", C.c_float)]


class Sim3OptProblem(C.Structure):
    _fields_ = [("n", C.c_int32), ("valid", C.c_void_p), ("X1w", C.c_void_p), ("X2w", C.c_void_p),
                ("uv1", C.c_void_p), ("uv2", C.c_void_p), ("inv1", C.c_void_p), ("inv2", C.c_void_p),
                ("R1w", C.c_float * 9), ("t1w", C.c_float * 3), ("R2w", C.c_float * 9), ("t2w", C.c_float * 3),
                ("K1", C.c_float * 4), ("K2", C.c_float * 4), ("S", C.c_double * 8), ("th2", C.c_float)]


class Sim3OptResult(C.Structure):
    _fields_ = [("n_inliers", C.c_int32), ("n_correspondences", C.c_int32), ("n_bad", C.c_int32),
                ("lm_iterations", C.c_int32), ("lm_trials", C.c_int32), ("S", C.c_double * 8)]


class BowFeatures(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("angle", C.c_void_p), ("valid", C.c_void_p),
                ("n_nodes", C.c_int32), ("node_id", C.c_void_p), ("node_begin", C.c_void_p), ("feat", C.c_void_p)]


class Sim3KFStruct(C.Structure):
    """rsc_sim3_kf (include/rsc.h)."""
    _fields_ = [("n", C.c_int32), ("kp", C.c_void_p), ("octave", C.c_void_p), ("desc", C.c_void_p),
                ("cell_begin", C.c_void_p), ("cell_feat", C.c_void_p), ("min_x", C.c_float), ("max_x", C.c_float),
                ("min_y", C.c_float), ("max_y", C.c_float), ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("scale_factors", C.c_void_p), ("n_levels", C.c_int32), ("log_scale_factor", C.c_float),
                ("Rcw", C.c_float * 9), ("tcw", C.c_float * 3), ("mp_state", C.c_void_p), ("mp_pos", C.c_void_p),
                ("mp_dmax", C.c_void_p), ("mp_dmin", C.c_void_p), ("mp_desc", C.c_void_p)]


def sim3_kf_struct(kf):
    """(ctypes rsc_sim3_kf, keep-alive arrays) for a rsc.synth.Sim3KF-like object."""
    from rsc import synth
    keep = [np.ascontiguousarray(kf.kp, np.float32), np.ascontiguousarray(kf.octave, np.int32),
            np.ascontiguousarray(kf.desc, np.uint8), np.ascontiguousarray(kf.cell_begin, np.int32),
            np.ascontiguousarray(kf.cell_feat, np.int32), synth.scale_factors(),
            np.ascontiguousarray(kf.mp_state, np.uint8), np.ascontiguousarray(kf.mp_pos, np.float32),
            np.ascontiguousarray(kf.mp_dmax, np.float32), np.ascontiguousarray(kf.mp_dmin, np.float32),
            np.ascontiguousarray(kf.mp_desc, np.uint8)]
    if keep[4].size == 0:
        keep[4] = np.zeros(1, np.int32)
    k = Sim3KFStruct()
    k.n = int(kf.n)
    (k.kp, k.octave, k.desc, k.cell_begin, k.cell_feat, k.scale_factors, k.mp_state, k.mp_pos, k.mp_dmax,
     k.mp_dmin, k.mp_desc) = (a.ctypes.data for a in keep)
    k.min_x, k.max_x, k.min_y, k.max_y = kf.min_x, kf.max_x, kf.min_y, kf.max_y
    k.grid_w_inv, k.grid_h_inv = float(synth.GRID_W_INV), float(synth.GRID_H_INV)
    k.fx, k.fy, k.cx, k.cy = kf.fx, kf.fy, kf.cx, kf.cy
    k.n_levels = len(keep[5])
    k.log_scale_factor = float(synth.LOG_SCALE_FACTOR)
    k.Rcw[:] = [float(v) for v in np.asarray(kf.Rcw, np.float32).reshape(9)]
    k.tcw[:] = [float(v) for v in np.asarray(kf.tcw, np.float32).reshape(3)]
    return k, keep


class KFView:
    """A KeyFrame's SearchBySim3 inputs resident in HBM (rsc_kfview_create)."""

    def __init__(self, ctx: Context, kf):
        self.ctx, self.n = ctx, int(kf.n)
        k, keep = sim3_kf_struct(kf)
        h = C.c_void_p()
        _check(load_library().rsc_kfview_create(ctx.h, C.byref(k), C.byref(h)), "rsc_kfview_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_kfview_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Sim3Search:
    """Prepared ORBmatcher::SearchBySim3 batch (ORBmatcher.cpp:948-1170): count (kf1, kf2, R12, t12,
    matched12) problems in one launch over resident KeyFrame views, threshold th (7.5 in
    LoopClosing.cpp:309).  The same KeyFrame object is uploaded once."""

    def __init__(self, ctx: Context, problems, th: float = 7.5):
        self.ctx, self.th = ctx, float(th)
        c = len(problems)
        self.count = c
        self.views = {}
        for p in problems:
            for kf in (p[0], p[1]):
                if id(kf) not in self.views:
                    self.views[id(kf)] = KFView(ctx, kf)
        self.h1 = (C.c_void_p * max(c, 1))(*[self.views[id(p[0])].h.value for p in problems])
        self.h2 = (C.c_void_p * max(c, 1))(*[self.views[id(p[1])].h.value for p in problems])
        self.R = np.ascontiguousarray(np.stack([np.asarray(p[2], np.float32).reshape(9) for p in problems]))
        self.t = np.ascontiguousarray(np.stack([np.asarray(p[3], np.float32).reshape(3) for p in problems]))
        self.m_in = [np.ascontiguousarray(p[4], np.int32) for p in problems]
        self.out = [np.full(max(p[0].n, 1), -7, np.int32) for p in problems]
        self.pin = (C.c_void_p * max(c, 1))(*[a.ctypes.data for a in self.m_in])
        self.pout = (C.c_void_p * max(c, 1))(*[a.ctypes.data for a in self.out])
        self.nfound = np.zeros(max(c, 1), np.int32)
        self.n1 = [p[0].n for p in problems]

    def run(self):
        _check(load_library().rsc_search_by_sim3_many(self.ctx.h, self.h1, self.h2, self.count, self.R, self.t,
                                                      self.th, self.pin, self.pout, self.nfound),
               "rsc_search_by_sim3_many")
        return [o[:n] for o, n in zip(self.out, self.n1)], self.nfound[:self.count]


def search_by_sim3_many(ctx: Context, problems, th: float = 7.5):
    """SearchBySim3 for each (kf1, kf2, R12, t12, matched12): returns (list of out12 int32 arrays =
    new match's KF2 keypoint or -1, nfound int32[count])."""
    return Sim3Search(ctx, problems, th).run()


class KeyFrameDatabase:
    """Device-resident KeyFrameDatabase (src/KeyFrameDatabase.cpp, rsc_kfdb_*): KeyFrames are slots
    in [0, capacity); each BowVector is (word ids ascending uint32, values float64).  The per-
    KeyFrame query state (mnLoopQuery/Words/Score, mnRelocQuery/Words/Score) persists across
    queries as in the reference."""

    def __init__(self, ctx: Context, capacity: int, max_words: int = 4096, vocab_words: int = 10 ** 6):
        self.ctx, self.capacity = ctx, int(capacity)
        h = C.c_void_p()
        _check(load_library().rsc_kfdb_create(ctx.h, int(vocab_words), self.capacity, int(max_words), C.byref(h)),
               "rsc_kfdb_create")
        self.h = h
        self._cand = np.zeros(max(self.capacity, 1), np.int32)
        self._n = np.zeros(1, np.int32)

    @staticmethod
    def _bow(ids, vals):
        return np.ascontiguousarray(ids, np.uint32), np.ascontiguousarray(vals, np.float64)

    def add(self, kf: int, ids, vals):
        i, v = self._bow(ids, vals)
        _check(load_library().rsc_kfdb_add(self.h, int(kf), len(i), i, v), "rsc_kfdb_add")

    def erase(self, kf: int):
        _check(load_library().rsc_kfdb_erase(self.h, int(kf)), "rsc_kfdb_erase")

    def release(self, kf: int):
        """Free slot kf for reuse (erase + fresh query state and covisibility row)."""
        _check(load_library().rsc_kfdb_release(self.h, int(kf)), "rsc_kfdb_release")

    def clear(self):
        _check(load_library().rsc_kfdb_clear(self.h), "rsc_kfdb_clear")

    def set_covisibility(self, kf: int, best):
        b = np.ascontiguousarray(best, np.int32)
        _check(load_library().rsc_kfdb_set_covisibility(self.h, int(kf), len(b), b), "rsc_kfdb_set_covisibility")

    def set_covisibility_many(self, kfs, bests):
        """set_covisibility for many slots in one upload (bests: sequences of <= 10 slots)."""
        k = np.ascontiguousarray(kfs, np.int32)
        n = np.array([len(b) for b in bests], np.int32)
        tab = np.zeros((max(len(k), 1), 10), np.int32)
        for i, b in enumerate(bests):
            tab[i, :len(b)] = b
        _check(load_library().rsc_kfdb_set_covisibility_many(self.h, len(k), k, n, tab), "set_covisibility_many")

    def set_covisibility_table(self, kfs, counts, table):
        """set_covisibility_many with the rows already packed: kfs int32 [c], counts int32 [c],
        table int32 [c, 10] (what a C++ caller passes; no per-row Python work)."""
        _check(load_library().rsc_kfdb_set_covisibility_many(self.h, len(kfs), kfs, counts, table),
               "set_covisibility_many")

    def detect_relocalization(self, frame_id: int, ids, vals) -> np.ndarray:
        """DetectRelocalizationCandidates(F) (:174-283): candidate slots in the reference's order."""
        i, v = self._bow(ids, vals)
        _check(load_library().rsc_kfdb_detect_relocalization(self.h, int(frame_id), len(i), i, v, self._cand,
                                                              self._n), "rsc_kfdb_detect_relocalization")
        return self._cand[:self._n[0]].copy()

    def detect_loop(self, kf_id: int, ids, vals, connected, min_score: float) -> np.ndarray:
        """DetectLoopCandidates(pKF, minScore) (:52-172)."""
        i, v = self._bow(ids, vals)
        c = np.ascontiguousarray(connected, np.int32)
        _check(load_library().rsc_kfdb_detect_loop(self.h, int(kf_id), len(i), i, v, len(c), c, float(min_score),
                                                   self._cand, self._n), "rsc_kfdb_detect_loop")
        return self._cand[:self._n[0]].copy()

    def state(self, kf: int):
        """((mnLoopQuery, mnRelocQuery), (mnLoopWords, mnRelocWords), (mLoopScore, mRelocScore))"""
        q = np.zeros(2, np.uint64)
        w = np.zeros(2, np.int32)
        s = np.zeros(2, np.float32)
        _check(load_library().rsc_kfdb_state(self.h, int(kf), q, w, s), "rsc_kfdb_state")
        return tuple(int(x) for x in q), tuple(int(x) for x in w), tuple(float(x) for x in s)

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_kfdb_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class PoseOptResult(C.Structure):
    _fields_ = [("n_good", C.c_int32), ("n_initial", C.c_int32), ("rounds", C.c_int32),
                ("lm_iterations", C.c_int32), ("lm_trials", C.c_int32), ("Tcw", C.c_float * 16)]


_fast = None


def _fast_library():
    """Second handle of librsc.so whose batched reset / iterate prototypes take raw addresses
    (c_void_p) instead of checked ndarrays; used only by SolverBatch with buffers it owns."""
    global _fast
    if _fast is None:
        F = C.CDLL(_lib_path_loaded)
        vp = C.c_void_p
        for kind, rec in (("pnp", PnPResult), ("mlpnp", PnPResult), ("sim3", Sim3Result)):
            f = getattr(F, f"rsc_{kind}_reset_many")
            f.argtypes = [C.POINTER(vp), C.c_int, vp]
            f.restype = C.c_int
            f = getattr(F, f"rsc_{kind}_iterate_many")
            f.argtypes = [C.POINTER(vp), C.c_int, vp, C.POINTER(rec), C.POINTER(vp)]
            f.restype = C.c_int
        _fast = F
    return _fast


_lib_path_loaded = LIB_PATH


def load_library(path: str = LIB_PATH):
    """Load librsc.so (raises if it was not built: no fallback)."""
    global _lib, _lib_path_loaded
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"librsc.so not found at {path}: run __graft_entry__.build() / make")
    L = C.CDLL(path)
    _lib_path_loaded = path
    vp = C.c_void_p
    L.rsc_version.restype = C.c_int
    L.rsc_status_string.restype = C.c_char_p
    L.rsc_status_string.argtypes = [C.c_int]
    L.rsc_context_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.rsc_context_destroy.argtypes = [vp]
    L.rsc_selftest_math.argtypes = [vp, C.c_int, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    L.rsc_context_set_stream.argtypes = [vp, vp]
    L.rsc_context_synchronize.argtypes = [vp]
    L.rsc_context_last_timing.argtypes = [vp, C.POINTER(C.c_double)]
    L.rsc_context_last_kernel_timing.argtypes = [vp, C.POINTER(C.c_double)]
    L.rsc_diag_host_timing.argtypes = [vp, C.POINTER(C.c_double)]
    L.rsc_context_enable_timing.argtypes = [vp, C.c_int]
    L.rsc_context_set_eig_rows.argtypes = [vp, C.c_int]
    L.rsc_context_set_eig_split.argtypes = [vp, C.c_int]
    L.rsc_context_set_sim3opt_helpers.argtypes = [vp, C.c_int]
    L.rsc_pnp_create.argtypes = [vp, C.POINTER(PnPProblem), C.c_uint32, C.POINTER(vp)]
    L.rsc_pnp_destroy.argtypes = [vp]
    L.rsc_pnp_set_ransac_parameters.argtypes = [vp, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
    L.rsc_pnp_iterate.argtypes = [vp, C.c_int, C.POINTER(PnPResult), C.c_void_p]
    L.rsc_pnp_find.argtypes = [vp, C.POINTER(PnPResult), C.c_void_p]
    L.rsc_pnp_last_inliers.argtypes = [vp, C.c_void_p]
    L.rsc_pnp_last_inliers.restype = C.c_int
    L.rsc_pnp_iterate_many.argtypes = [C.POINTER(vp), C.c_int, i32p, C.POINTER(PnPResult), C.POINTER(C.c_void_p)]
    L.rsc_pnp_reset.argtypes = [vp, C.c_uint32]
    L.rsc_pnp_get_state.argtypes = [vp, i32p]
    L.rsc_pnp_last_samples.argtypes = [vp, i32p, C.c_int]
    L.rsc_pnp_last_hypotheses.argtypes = [vp, i32p, f32p, C.c_int]
    L.rsc_sim3_last_hypotheses.argtypes = [vp, i32p, f32p, C.c_int]
    L.rsc_mlpnp_last_counts.argtypes = [vp, i32p, C.c_int]
    L.rsc_sim3_create.argtypes = [vp, C.POINTER(Sim3Input), C.c_uint32, C.POINTER(vp)]
    L.rsc_sim3_destroy.argtypes = [vp]
    L.rsc_sim3_set_ransac_parameters.argtypes = [vp, C.c_double, C.c_int, C.c_int]
    L.rsc_sim3_iterate.argtypes = [vp, C.c_int, C.POINTER(Sim3Result), C.c_void_p]
    L.rsc_sim3_find.argtypes = [vp, C.POINTER(Sim3Result), C.c_void_p]
    L.rsc_sim3_iterate_many.argtypes = [C.POINTER(vp), C.c_int, i32p, C.POINTER(Sim3Result), C.POINTER(C.c_void_p)]
    L.rsc_sim3_reset.argtypes = [vp, C.c_uint32]
    L.rsc_sim3_get_state.argtypes = [vp, i32p]
    L.rsc_sim3_prepared.argtypes = [vp, f32p, f32p, f32p, f32p, u64p, u64p, i32p]
    L.rsc_rand_stream.argtypes = [vp, C.c_uint32, C.c_int, i32p]
    u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
    L.rsc_pnp_reset_many.argtypes = [C.POINTER(vp), C.c_int, u32p]
    L.rsc_pnp_set_ransac_parameters_many.argtypes = [C.POINTER(vp), C.c_int, C.c_double, C.c_int, C.c_int, C.c_int,
                                                     C.c_float, C.c_float]
    L.rsc_sim3_reset_many.argtypes = [C.POINTER(vp), C.c_int, u32p]
    L.rsc_sim3_set_ransac_parameters_many.argtypes = [C.POINTER(vp), C.c_int, C.c_double, C.c_int, C.c_int]
    f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    L.rsc_mlpnp_create.argtypes = [vp, C.POINTER(PnPProblem), C.c_uint32, C.POINTER(vp)]
    L.rsc_mlpnp_destroy.argtypes = [vp]
    L.rsc_mlpnp_set_covariances.argtypes = [vp, C.POINTER(C.c_double)]
    L.rsc_mlpnp_set_ransac_parameters.argtypes = [vp, C.c_double, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
    L.rsc_mlpnp_set_ransac_parameters_many.argtypes = [C.POINTER(vp), C.c_int, C.c_double, C.c_int, C.c_int,
                                                       C.c_int, C.c_float, C.c_float]
    L.rsc_mlpnp_iterate.argtypes = [vp, C.c_int, C.POINTER(PnPResult), C.c_void_p]
    L.rsc_mlpnp_iterate_many.argtypes = [C.POINTER(vp), C.c_int, i32p, C.POINTER(PnPResult), C.POINTER(C.c_void_p)]
    L.rsc_mlpnp_reset.argtypes = [vp, C.c_uint32]
    L.rsc_mlpnp_reset_many.argtypes = [C.POINTER(vp), C.c_int, u32p]
    L.rsc_mlpnp_get_state.argtypes = [vp, i32p]
    L.rsc_mlpnp_last_poses.argtypes = [vp, f64p, C.c_int]
    L.rsc_mlpnp_last_samples.argtypes = [vp, i32p, C.c_int]
    L.rsc_reloc_events.argtypes = [C.POINTER(vp), i32p, C.c_int, C.POINTER(PnPResult), C.POINTER(EventResult)]
    L.rsc_stream_create.argtypes = [vp, C.c_uint32, C.POINTER(vp)]
    L.rsc_stream_destroy.argtypes = [vp]
    L.rsc_stream_destroy.restype = None
    L.rsc_stream_skip.argtypes = [vp, C.c_int64]
    L.rsc_stream_position.argtypes = [vp, C.POINTER(C.c_int64)]
    L.rsc_stream_peek.argtypes = [vp, C.c_int, i32p]
    for f in ("rsc_pnp_bind_stream", "rsc_sim3_bind_stream", "rsc_mlpnp_bind_stream"):
        getattr(L, f).argtypes = [vp, vp]
    L.rsc_reloc_events_shared.argtypes = [C.POINTER(vp), i32p, C.c_int, C.POINTER(vp), C.POINTER(PnPResult),
                                          C.POINTER(EventResult)]
    L.rsc_loop_events_shared.argtypes = [C.POINTER(vp), i32p, C.c_int, C.POINTER(vp), C.POINTER(Sim3Result),
                                         C.POINTER(EventResult)]
    L.rsc_pose_optimization_many.argtypes = [vp, C.POINTER(PoseOptProblem), C.c_int, C.POINTER(PoseOptResult),
                                             C.POINTER(C.c_void_p)]
    L.rsc_optimize_sim3_many.argtypes = [vp, C.POINTER(Sim3OptProblem), C.c_int, C.POINTER(Sim3OptResult),
                                         C.POINTER(C.c_void_p)]
    L.rsc_bow_create.argtypes = [vp, C.POINTER(BowFeatures), C.POINTER(vp)]
    L.rsc_bow_destroy.argtypes = [vp]
    L.rsc_bow_set_valid.argtypes = [vp, u8p]
    L.rsc_search_by_bow_frame_many.argtypes = [vp, C.POINTER(vp), C.c_int, vp, C.c_float, C.c_int,
                                               C.POINTER(C.c_void_p), i32p]
    L.rsc_search_by_bow_kf_many.argtypes = [vp, vp, C.POINTER(vp), C.c_int, C.c_float, C.c_int,
                                            C.POINTER(C.c_void_p), i32p]
    L.rsc_diag_bow_phase_stamps.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"),
                                            C.c_int]
    L.rsc_diag_refine_phase_stamps.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"),
                                               C.c_int]
    L.rsc_diag_solve_phase_stamps.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"),
                                              C.c_int]
    L.rsc_diag_mlpnp_phase_stamps.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"),
                                              C.c_int]
    L.rsc_diag_poseopt_phases.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"), C.c_int]
    L.rsc_diag_sim3opt_phases.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"), C.c_int]
    L.rsc_diag_kfdb_stamps.argtypes = [vp, np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS"), C.c_int]
    f32p_ = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
    L.rsc_kfview_create.argtypes = [vp, C.POINTER(Sim3KFStruct), C.POINTER(vp)]
    L.rsc_kfview_destroy.argtypes = [vp]
    L.rsc_search_by_sim3_many.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.c_int, f32p_, f32p_, C.c_float,
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), i32p]
    u32p_ = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
    f64p_ = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
    u64p_ = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
    L.rsc_kfdb_create.argtypes = [vp, C.c_uint32, C.c_int, C.c_int, C.POINTER(vp)]
    L.rsc_kfdb_destroy.argtypes = [vp]
    L.rsc_kfdb_add.argtypes = [vp, C.c_int, C.c_int, u32p_, f64p_]
    L.rsc_kfdb_erase.argtypes = [vp, C.c_int]
    L.rsc_kfdb_release.argtypes = [vp, C.c_int]
    L.rsc_kfdb_clear.argtypes = [vp]
    L.rsc_kfdb_set_covisibility.argtypes = [vp, C.c_int, C.c_int, i32p]
    L.rsc_kfdb_set_covisibility_many.argtypes = [vp, C.c_int, i32p, i32p, i32p]
    L.rsc_kfdb_detect_relocalization.argtypes = [vp, C.c_uint64, C.c_int, u32p_, f64p_, i32p, i32p]
    L.rsc_kfdb_detect_loop.argtypes = [vp, C.c_uint64, C.c_int, u32p_, f64p_, C.c_int, i32p, C.c_float, i32p, i32p]
    L.rsc_kfdb_state.argtypes = [vp, C.c_int, u64p_, i32p, f32p_]
    L.rsc_loop_events.argtypes = [C.POINTER(vp), i32p, C.c_int, C.POINTER(Sim3Result), C.POINTER(EventResult)]
    L.rsc_reloc_events_gated.argtypes = [C.POINTER(vp), i32p, C.c_int, C.POINTER(RelocFrame), C.POINTER(PnPResult),
                                         C.POINTER(RelocGateResult), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
    L.rsc_loop_events_gated.argtypes = [C.POINTER(vp), C.POINTER(LoopCandidate), i32p, C.c_int,
                                        C.POINTER(Sim3Result), C.POINTER(LoopGateResult), C.POINTER(C.c_void_p)]
    _lib = L
    return L


def _check(st: int, what: str):
    if st != RSC_OK:
        raise RuntimeError(f"rsc: {what}: {load_library().rsc_status_string(st).decode()} ({st})")


class Context:
    """One engine context (HIP stream + work buffers + rand() jump table) on one device."""

    def __init__(self, device: int = 0):
        L = load_library()
        h = C.c_void_p()
        _check(L.rsc_context_create(device, C.byref(h)), "rsc_context_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_context_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_stream(self, stream_ptr: int):
        _check(load_library().rsc_context_set_stream(self.h, C.c_void_p(stream_ptr)), "set_stream")

    def synchronize(self):
        _check(load_library().rsc_context_synchronize(self.h), "synchronize")

    def enable_timing(self, on: bool = True):
        _check(load_library().rsc_context_enable_timing(self.h, int(on)), "enable_timing")

    def set_eig_rows(self, max_workgroups: int):
        """Eigen stage in the rows form for launches of <= max_workgroups workgroups (0: off)."""
        _check(load_library().rsc_context_set_eig_rows(self.h, int(max_workgroups)), "set_eig_rows")

    def set_eig_split(self, on: bool):
        """Split-form eigen stage (chase and Q rotations on two waves) for the launches the rows form
        does not take (default on); off: the lane-pair form."""
        _check(load_library().rsc_context_set_eig_split(self.h, int(bool(on))), "set_eig_split")

    def set_sim3opt_helpers(self, helpers: int):
        """OptimizeSim3's form: helper workgroups per pair (the cooperative form), 0 = one workgroup
        per pair, -1 = automatic (default)."""
        _check(load_library().rsc_context_set_sim3opt_helpers(self.h, int(helpers)), "set_sim3opt_helpers")

    MATH_FNS = {"sin": 0, "cos": 1, "acos": 2, "cbrt": 3, "log": 4, "logf": 5, "sqrt_unit": 6, "recip_unit": 7,
                "givens_c": 8, "givens_s": 9, "qr_solve": 10, "pow_1_3": 11, "pow_3_2": 12, "rcp_scan": 13,
                "ldlt_lanes": 16}

    def selftest_math(self, fn: str, x):
        """rsc_math.h evaluated on the GPU (f64 array in, f64 array out; logf: float in/out)."""
        x = np.ascontiguousarray(x, np.float64)
        out = np.empty_like(x)
        dp = C.POINTER(C.c_double)
        _check(load_library().rsc_selftest_math(self.h, self.MATH_FNS[fn], x.ctypes.data_as(dp), int(x.size),
                                                out.ctypes.data_as(dp)), "selftest_math")
        return out

    def qr_solve(self, A, b, X0):
        """PnPsolver::qr_solve (the kernels' qr_solve_6x4) ON THE GPU for a batch of 6x4 systems:
        A [k,6,4], b [k,6], X0 [k,4] (kept on the singular bail-out) -> (X [k,4], ok [k] bool)."""
        A = np.asarray(A, np.float64).reshape(-1, 24)
        k = A.shape[0]
        rec = np.zeros((k, 34))
        rec[:, :24] = A
        rec[:, 24:30] = np.asarray(b, np.float64).reshape(k, 6)
        rec[:, 30:34] = np.asarray(X0, np.float64).reshape(k, 4)
        out = self.selftest_math("qr_solve", rec.ravel()).reshape(k, 34)
        return out[:, :4].copy(), out[:, 4] == 1.0

    def last_timing(self):
        out = (C.c_double * 6)()
        _check(load_library().rsc_context_last_kernel_timing(self.h, out), "last_timing")
        return dict(solve_ms=out[0], scan_ms=out[1], refine_ms=out[2], solve_launches=int(out[3]),
                    hypotheses=int(out[4]), eig_ms=out[5])

    def host_timing(self):
        """Diagnostic host clock (us) of the last PnP iterate_many: first launch, enqueued, synced, return."""
        out = (C.c_double * 4)()
        _check(load_library().rsc_diag_host_timing(self.h, out), "host_timing")
        return list(out)

    def rand_stream(self, seed: int, n: int) -> np.ndarray:
        out = np.zeros(n, np.int32)
        _check(load_library().rsc_rand_stream(self.h, seed, n, out), "rand_stream")
        return out


class Stream:
    """The reference's process-global rand() stream (Q3): srand(seed) and a position.  Solvers bound
    to it (``solver.bind_stream(stream)``) draw their samples from it in call order; an event batch
    run with one stream per event (``EventBatch.run(streams=...)``) draws each event's calls from its
    stream in the round-robin's order."""

    def __init__(self, ctx: "Context", seed: int = 1):
        h = C.c_void_p()
        _check(load_library().rsc_stream_create(ctx.h, seed, C.byref(h)), "rsc_stream_create")
        self.h = h
        self.ctx = ctx

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_stream_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def skip(self, n: int):
        _check(load_library().rsc_stream_skip(self.h, int(n)), "rsc_stream_skip")

    @property
    def position(self) -> int:
        v = C.c_int64()
        _check(load_library().rsc_stream_position(self.h, C.byref(v)), "rsc_stream_position")
        return int(v.value)

    def peek(self, n: int) -> np.ndarray:
        out = np.zeros(max(n, 1), np.int32)
        _check(load_library().rsc_stream_peek(self.h, n, out), "rsc_stream_peek")
        return out[:n]


def _bind(fn, solver, stream):
    _check(fn(solver.h, stream.h if stream is not None else None), "bind_stream")
    solver._stream = stream  # keep the stream alive while bound


def _pnp_out(r: PnPResult, mask) -> dict:
    """Result dict of one PnP / MLPnP iterate().  ``mask`` None = the caller asked for no vbInliers:
    ``inliers`` is then None (never a zero array that reads like a result)."""
    T = np.array(r.T, dtype=np.float32).reshape(4, 4)
    inl = None if mask is None else (mask.astype(bool) if r.ok else np.zeros(0, bool))
    return dict(ok=bool(r.ok), no_more=bool(r.no_more), n_inliers=int(r.n_inliers), iterations=int(r.iterations),
                T=T, inliers=inl)


class PnPSolver:
    """PnPsolver (PnPsolver.cpp) on the GPU.  ``scene`` carries the compacted constructor arrays."""

    def __init__(self, ctx: Context, scene, seed: int = 1):
        L = load_library()
        self.ctx = ctx
        self._keep = [np.ascontiguousarray(scene.p2d, np.float32), np.ascontiguousarray(scene.p3dw, np.float32),
                      np.ascontiguousarray(scene.sigma2, np.float32), np.ascontiguousarray(scene.kp_index, np.int32)]
        pb = PnPProblem(int(scene.n), int(scene.n_points), self._keep[0].ctypes.data, self._keep[1].ctypes.data,
                        self._keep[2].ctypes.data, self._keep[3].ctypes.data, float(scene.fx), float(scene.fy),
                        float(scene.cx), float(scene.cy))
        h = C.c_void_p()
        _check(L.rsc_pnp_create(ctx.h, C.byref(pb), seed, C.byref(h)), "rsc_pnp_create")
        self.h = h
        self.n_points = int(scene.n_points)
        self.n = int(scene.n)

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_pnp_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=4, epsilon=0.4,
                              th2=5.991):
        _check(load_library().rsc_pnp_set_ransac_parameters(self.h, probability, min_inliers, max_iterations,
                                                            min_set, epsilon, th2), "SetRansacParameters")

    def iterate(self, n_iterations: int) -> dict:
        r = PnPResult()
        mask = np.zeros(max(self.n_points, 1), np.uint8)
        _check(load_library().rsc_pnp_iterate(self.h, n_iterations, C.byref(r), mask.ctypes.data), "iterate")
        return _pnp_out(r, mask[:self.n_points])

    def find(self) -> dict:
        r = PnPResult()
        mask = np.zeros(max(self.n_points, 1), np.uint8)
        _check(load_library().rsc_pnp_find(self.h, C.byref(r), mask.ctypes.data), "find")
        return _pnp_out(r, mask[:self.n_points])

    def last_inliers(self):
        """vbInliers of the last iterate()/find() (bool[n_points]; None when it returned false),
        fetched after the call (rsc_pnp_last_inliers) — e.g. after SolverBatch.iterate_raw."""
        mask = np.zeros(max(self.n_points, 1), np.uint8)
        st = load_library().rsc_pnp_last_inliers(self.h, mask.ctypes.data)
        if st < 0:
            _check(st, "last_inliers")
        return mask[:self.n_points].astype(bool) if st == 1 else None

    def reset(self, seed: int):
        _check(load_library().rsc_pnp_reset(self.h, seed), "reset")

    def bind_stream(self, stream):
        """Draw from a shared Stream (None: back to the own stream) — rsc_pnp_bind_stream."""
        _bind(load_library().rsc_pnp_bind_stream, self, stream)

    def state(self) -> dict:
        out = np.zeros(8, np.int32)
        _check(load_library().rsc_pnp_get_state(self.h, out), "get_state")
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]), max_rows=int(out[4]), N=int(out[5]), n_points=int(out[6]),
                    min_set=int(out[7]))

    def last_samples(self, cap: int = 100000) -> np.ndarray:
        out = np.zeros((cap, 8), np.int32)
        n = load_library().rsc_pnp_last_samples(self.h, out.reshape(-1), cap)
        return out[:max(n, 0)]

    def last_hypotheses(self, cap: int = 4096):
        """(counts [H], float poses [H, 12] = R row-major + t) of the last launch (parity hook)."""
        cnt = np.zeros(cap, np.int32)
        pos = np.zeros((cap, 12), np.float32)
        n = load_library().rsc_pnp_last_hypotheses(self.h, cnt, pos.reshape(-1), cap)
        if n < 0:
            _check(n, "last_hypotheses")
        return cnt[:n], pos[:n]


def pnp_iterate_many(solvers, n_iterations, with_masks: bool = True):
    """rsc_pnp_iterate_many: iterate() of every solver in one set of launches."""
    L = load_library()
    n = len(solvers)
    hs = (C.c_void_p * n)(*[s.h.value for s in solvers])
    its = np.ascontiguousarray(np.broadcast_to(np.asarray(n_iterations, np.int32), (n,)))
    res = (PnPResult * n)()
    masks = [np.zeros(max(s.n_points, 1), np.uint8) if with_masks else None for s in solvers]
    mp = (C.c_void_p * n)(*[(m.ctypes.data if m is not None else None) for m in masks])
    _check(L.rsc_pnp_iterate_many(hs, n, its, res, mp), "iterate_many")
    return [_pnp_out(res[i], None if masks[i] is None else masks[i][:solvers[i].n_points]) for i in range(n)]


def mlpnp_iterate_many(solvers, n_iterations, with_masks: bool = True):
    """rsc_mlpnp_iterate_many: iterate() of every MLPnP solver in one set of launches."""
    L = load_library()
    n = len(solvers)
    hs = (C.c_void_p * n)(*[s.h.value for s in solvers])
    its = np.ascontiguousarray(np.broadcast_to(np.asarray(n_iterations, np.int32), (n,)))
    res = (PnPResult * n)()
    masks = [np.zeros(max(s.n_points, 1), np.uint8) if with_masks else None for s in solvers]
    mp = (C.c_void_p * n)(*[(m.ctypes.data if m is not None else None) for m in masks])
    _check(L.rsc_mlpnp_iterate_many(hs, n, its, res, mp), "mlpnp_iterate_many")
    return [_pnp_out(res[i], None if masks[i] is None else masks[i][:solvers[i].n_points]) for i in range(n)]


def _sim3_out(r: Sim3Result, mask) -> dict:
    """Result dict of one Sim3 iterate(); ``inliers`` None when no vbInliers were requested."""
    return dict(ok=bool(r.ok), no_more=bool(r.no_more), n_inliers=int(r.n_inliers), iterations=int(r.iterations),
                R=np.array(r.R, np.float32).reshape(3, 3), t=np.array(r.t, np.float32),
                inliers=None if mask is None else mask.astype(bool))


class Sim3Solver:
    """Sim3Solver (Sim3Solver.cpp) on the GPU, built from the raw keyframe-pair inputs."""

    def __init__(self, ctx: Context, pair, seed: int = 1):
        L = load_library()
        self.ctx = ctx
        self._keep = [np.ascontiguousarray(a) for a in (
            pair.valid.astype(np.uint8), pair.Xw1.astype(np.float32), pair.Xw2.astype(np.float32),
            pair.sigma2_1.astype(np.float32), pair.sigma2_2.astype(np.float32))]
        inp = Sim3Input()
        inp.n1 = int(pair.n1)
        inp.valid, inp.Xw1, inp.Xw2, inp.sigma2_1, inp.sigma2_2 = [a.ctypes.data for a in self._keep]
        inp.R1[:] = [float(x) for x in np.asarray(pair.R1, np.float32).ravel()]
        inp.t1[:] = [float(x) for x in np.asarray(pair.t1, np.float32)]
        inp.R2[:] = [float(x) for x in np.asarray(pair.R2, np.float32).ravel()]
        inp.t2[:] = [float(x) for x in np.asarray(pair.t2, np.float32)]
        inp.K1[:] = [float(x) for x in np.asarray(pair.K1, np.float32)]
        inp.K2[:] = [float(x) for x in np.asarray(pair.K2, np.float32)]
        h = C.c_void_p()
        _check(L.rsc_sim3_create(ctx.h, C.byref(inp), seed, C.byref(h)), "rsc_sim3_create")
        self.h = h
        self.n1 = int(pair.n1)

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_sim3_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_ransac_parameters(self, probability=0.99, min_inliers=6, max_iterations=300):
        _check(load_library().rsc_sim3_set_ransac_parameters(self.h, probability, min_inliers, max_iterations),
               "SetRansacParameters")

    def iterate(self, n_iterations: int) -> dict:
        r = Sim3Result()
        mask = np.zeros(max(self.n1, 1), np.uint8)
        _check(load_library().rsc_sim3_iterate(self.h, n_iterations, C.byref(r), mask.ctypes.data), "iterate")
        return _sim3_out(r, mask[:self.n1])

    def find(self) -> dict:
        r = Sim3Result()
        mask = np.zeros(max(self.n1, 1), np.uint8)
        _check(load_library().rsc_sim3_find(self.h, C.byref(r), mask.ctypes.data), "find")
        return _sim3_out(r, mask[:self.n1])

    def reset(self, seed: int):
        _check(load_library().rsc_sim3_reset(self.h, seed), "reset")

    def bind_stream(self, stream):
        _bind(load_library().rsc_sim3_bind_stream, self, stream)

    def state(self) -> dict:
        out = np.zeros(6, np.int32)
        _check(load_library().rsc_sim3_get_state(self.h, out), "get_state")
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]), N=int(out[4]), n1=int(out[5]))

    def prepared(self) -> dict:
        N = self.state()["N"]
        X1 = np.zeros((N, 3), np.float32); X2 = np.zeros((N, 3), np.float32)
        P1 = np.zeros((N, 2), np.float32); P2 = np.zeros((N, 2), np.float32)
        e1 = np.zeros(N, np.uint64); e2 = np.zeros(N, np.uint64); idx = np.zeros(N, np.int32)
        _check(load_library().rsc_sim3_prepared(self.h, X1, X2, P1, P2, e1, e2, idx), "prepared")
        return dict(X1c=X1, X2c=X2, P1im1=P1, P2im2=P2, maxerr1=e1, maxerr2=e2, indices=idx)

    def last_hypotheses(self, cap: int = 4096):
        """(counts [H], float (R12, t12) [H, 12]) of the last launch (parity hook)."""
        cnt = np.zeros(cap, np.int32)
        pos = np.zeros((cap, 12), np.float32)
        n = load_library().rsc_sim3_last_hypotheses(self.h, cnt, pos.reshape(-1), cap)
        if n < 0:
            _check(n, "last_hypotheses")
        return cnt[:n], pos[:n]


def sim3_iterate_many(solvers, n_iterations, with_masks: bool = True):
    L = load_library()
    n = len(solvers)
    hs = (C.c_void_p * n)(*[s.h.value for s in solvers])
    its = np.ascontiguousarray(np.broadcast_to(np.asarray(n_iterations, np.int32), (n,)))
    res = (Sim3Result * n)()
    masks = [np.zeros(max(s.n1, 1), np.uint8) if with_masks else None for s in solvers]
    mp = (C.c_void_p * n)(*[(m.ctypes.data if m is not None else None) for m in masks])
    _check(L.rsc_sim3_iterate_many(hs, n, its, res, mp), "iterate_many")
    return [_sim3_out(res[i], None if masks[i] is None else masks[i][:solvers[i].n1]) for i in range(n)]


class MLPnPSolver:
    """MLPnPsolver (MLPnPsolver.cpp) on the GPU; same constructor arrays as PnPSolver."""

    def __init__(self, ctx: Context, scene, seed: int = 1):
        L = load_library()
        self.ctx = ctx
        self._keep = [np.ascontiguousarray(scene.p2d, np.float32), np.ascontiguousarray(scene.p3dw, np.float32),
                      np.ascontiguousarray(scene.sigma2, np.float32), np.ascontiguousarray(scene.kp_index, np.int32)]
        pb = PnPProblem(int(scene.n), int(scene.n_points), self._keep[0].ctypes.data, self._keep[1].ctypes.data,
                        self._keep[2].ctypes.data, self._keep[3].ctypes.data, float(scene.fx), float(scene.fy),
                        float(scene.cx), float(scene.cy))
        h = C.c_void_p()
        _check(L.rsc_mlpnp_create(ctx.h, C.byref(pb), seed, C.byref(h)), "rsc_mlpnp_create")
        self.h = h
        self.n_points = int(scene.n_points)
        self.n = int(scene.n)

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_mlpnp_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_covariances(self, cov):
        """computePose's covMats: [n, 3, 3] bearing-vector covariances (None: the reference's path)."""
        if cov is None:
            _check(load_library().rsc_mlpnp_set_covariances(self.h, None), "rsc_mlpnp_set_covariances")
            return
        self._cov = np.ascontiguousarray(np.asarray(cov, np.float64).reshape(self.n, 9))
        _check(load_library().rsc_mlpnp_set_covariances(self.h, self._cov.ctypes.data_as(C.POINTER(C.c_double))),
               "rsc_mlpnp_set_covariances")

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=6, epsilon=0.4,
                              th2=5.991):
        _check(load_library().rsc_mlpnp_set_ransac_parameters(self.h, probability, min_inliers, max_iterations,
                                                              min_set, epsilon, th2), "SetRansacParameters")

    def iterate(self, n_iterations: int) -> dict:
        r = PnPResult()
        mask = np.zeros(max(self.n_points, 1), np.uint8)
        _check(load_library().rsc_mlpnp_iterate(self.h, n_iterations, C.byref(r), mask.ctypes.data), "iterate")
        return _pnp_out(r, mask[:self.n_points])

    def reset(self, seed: int):
        _check(load_library().rsc_mlpnp_reset(self.h, seed), "reset")

    def bind_stream(self, stream):
        _bind(load_library().rsc_mlpnp_bind_stream, self, stream)

    def state(self) -> dict:
        out = np.zeros(6, np.int32)
        _check(load_library().rsc_mlpnp_get_state(self.h, out), "get_state")
        return dict(iterations=int(out[0]), max_iterations=int(out[1]), min_inliers=int(out[2]),
                    best_inliers=int(out[3]), n=int(out[4]), min_set=int(out[5]))

    def last_hypotheses(self, cap=4096):
        """(samples [H, 8], double poses [H, 12]) of the last launch (parity hook)."""
        smp = np.zeros((cap, 8), np.int32)
        pos = np.zeros((cap, 12))
        L = load_library()
        n = L.rsc_mlpnp_last_samples(self.h, smp.reshape(-1), cap)
        m = L.rsc_mlpnp_last_poses(self.h, pos.reshape(-1), cap)
        if n < 0 or m < 0:
            _check(min(n, m), "last_hypotheses")
        if n != m:
            raise RuntimeError(f"last_hypotheses: {n} samples vs {m} poses")
        return smp[:n], pos[:n]

    def last_counts(self, cap=4096):
        cnt = np.zeros(cap, np.int32)
        n = load_library().rsc_mlpnp_last_counts(self.h, cnt, cap)
        if n < 0:
            _check(n, "last_counts")
        return cnt[:n]


class SolverBatch:
    """A fixed list of solvers (one context) with batched reset / SetRansacParameters / iterate —
    the relocalization (PnP) or loop-closure (Sim3) candidate set of one event."""

    def __init__(self, solvers):
        self.solvers = list(solvers)
        first = self.solvers[0]
        self.kind = "pnp" if isinstance(first, PnPSolver) else ("mlpnp" if isinstance(first, MLPnPSolver) else "sim3")
        self._h = (C.c_void_p * len(self.solvers))(*[s.h.value for s in self.solvers])
        n = len(self.solvers)
        # hot-path prototypes with raw addresses (the ndpointer checks cost ~4 us per call): a
        # second handle of the same library keeps the checked prototypes of load_library() intact
        load_library()
        F = _fast_library()
        self._reset_f = {"pnp": F.rsc_pnp_reset_many, "mlpnp": F.rsc_mlpnp_reset_many,
                         "sim3": F.rsc_sim3_reset_many}[self.kind]
        self._iter_f = {"pnp": F.rsc_pnp_iterate_many, "mlpnp": F.rsc_mlpnp_iterate_many,
                        "sim3": F.rsc_sim3_iterate_many}[self.kind]
        self._seeds = np.zeros(n, np.uint32)
        self._seeds_p = self._seeds.ctypes.data
        rec = Sim3Result if self.kind == "sim3" else PnPResult
        self._raw = (rec * n)()
        self._its = np.zeros(n, np.int32)
        self._its_p = self._its.ctypes.data
        self._nomask = (C.c_void_p * n)()
        self._view = np.ctypeslib.as_array(self._raw)

    def reset(self, seeds):
        self._seeds[:] = seeds
        _check(self._reset_f(self._h, len(self.solvers), self._seeds_p), "reset_many")

    def set_ransac_parameters(self, *params):
        L = load_library()
        if self.kind == "pnp":
            _check(L.rsc_pnp_set_ransac_parameters_many(self._h, len(self.solvers), *params), "params_many")
        elif self.kind == "mlpnp":
            _check(L.rsc_mlpnp_set_ransac_parameters_many(self._h, len(self.solvers), *params), "params_many")
        else:
            _check(L.rsc_sim3_set_ransac_parameters_many(self._h, len(self.solvers), *params), "params_many")

    def iterate(self, n_iterations, with_masks=False):
        """iterate() of every solver; ``inliers`` of each result is None unless with_masks."""
        if self.kind == "pnp":
            return pnp_iterate_many(self.solvers, n_iterations, with_masks)
        if self.kind == "mlpnp":
            return mlpnp_iterate_many(self.solvers, n_iterations, with_masks)
        return sim3_iterate_many(self.solvers, n_iterations, with_masks)

    def iterate_raw(self, n_iterations):
        """iterate() of every solver without inlier vectors; returns the C result records as a
        numpy structured array (fields ok, no_more, n_inliers, iterations, T | R, t) without
        per-solver Python objects (the hot loop of bench.py)."""
        self._its[:] = n_iterations
        _check(self._iter_f(self._h, len(self.solvers), self._its_p, self._raw, self._nomask), "iterate_many")
        return self._view


class EventBatch:
    """Config-5 style event driver: many relocalization (PnP) or loop-closure (Sim3) events, each a
    contiguous group of candidate solvers; all candidates of all events run in the same launches
    (rsc_reloc_events / rsc_loop_events)."""

    def __init__(self, events):
        self.events = [list(ev) for ev in events]
        flat = [s for ev in self.events for s in ev]
        self.kind = "sim3" if isinstance(flat[0], Sim3Solver) else "pnp"
        self.batch = SolverBatch(flat)
        self.begin = np.zeros(len(self.events) + 1, np.int32)
        self.begin[1:] = np.cumsum([len(ev) for ev in self.events])
        rec = Sim3Result if self.kind == "sim3" else PnPResult
        self._cand = (rec * len(flat))()
        self._ev = (EventResult * len(self.events))()
        self.cand = np.ctypeslib.as_array(self._cand)
        self.per_event = np.ctypeslib.as_array(self._ev)

    def run(self, streams=None):
        """Run every event.  ``streams``: one Stream per event = the reference's shared rand() stream
        at that event's call (rsc_reloc_events_shared / rsc_loop_events_shared); None = every
        candidate on its own stream (H4)."""
        L = load_library()
        if streams is None:
            f = L.rsc_loop_events if self.kind == "sim3" else L.rsc_reloc_events
            _check(f(self.batch._h, self.begin, len(self.events), self._cand, self._ev), "events")
            return self.per_event
        if len(streams) != len(self.events) or any(st is None for st in streams):
            raise ValueError(f"one Stream per event: {len(self.events)} events, {len(streams)} streams")
        hs = (C.c_void_p * len(streams))(*[st.h.value for st in streams])
        f = L.rsc_loop_events_shared if self.kind == "sim3" else L.rsc_reloc_events_shared
        _check(f(self.batch._h, self.begin, len(self.events), hs, self._cand, self._ev), "events_shared")
        return self.per_event

    def run_reloc_gated(self, frames):
        """Relocalization events with the reference's PoseOptimization gate (rsc_reloc_events_gated,
        Tracking.cpp:1239-1335).  frames[e] = (u_right [n_points] float32 or None, bf).  Returns
        (per-event RelocGateResult records, winner outlier masks, winner vbInliers) — the masks are
        [n_points] uint8 arrays per event (zeros without a winner)."""
        assert self.kind == "pnp"
        if len(frames) != len(self.events):
            raise ValueError(f"one frame per event: {len(self.events)} events, {len(frames)} frames")
        L = load_library()
        fr = (RelocFrame * len(self.events))()
        keep = []
        for e, (ur, bf) in enumerate(frames):
            if ur is not None:
                a = np.ascontiguousarray(ur, np.float32)
                keep.append(a)
                fr[e].u_right = a.ctypes.data
            fr[e].bf = float(bf)
        res = (RelocGateResult * len(self.events))()
        npts = [ev[0].n_points if ev else 0 for ev in self.events]
        outl = [np.zeros(max(n, 1), np.uint8) for n in npts]
        inl = [np.zeros(max(n, 1), np.uint8) for n in npts]
        po = (C.c_void_p * len(self.events))(*[a.ctypes.data for a in outl])
        pi = (C.c_void_p * len(self.events))(*[a.ctypes.data for a in inl])
        _check(L.rsc_reloc_events_gated(self.batch._h, self.begin, len(self.events), fr, self._cand, res, po, pi),
               "reloc_events_gated")
        return np.ctypeslib.as_array(res).copy(), [o[:n] for o, n in zip(outl, npts)], \
            [m[:n] for m, n in zip(inl, npts)]

    def run_loop_gated(self, candidates):
        """Loop-closure events with the reference's SearchBySim3 + OptimizeSim3 gate
        (rsc_loop_events_gated, LoopClosing.cpp:268-329).  candidates[e][c] = (KFView of mpCurrentKF,
        KFView of the candidate, matches12 int32 [kf1 n]).  Returns (per-event LoopGateResult records,
        the accepted candidate's mvpCurrentMatchedPoints per event as KF2 indices)."""
        assert self.kind == "sim3"
        if len(candidates) != len(self.events) or any(len(c) != len(ev) for c, ev in zip(candidates, self.events)):
            raise ValueError("one (kf1, kf2, matches12) per candidate of every event")
        L = load_library()
        flat = [c for cs in candidates for c in cs]
        lc = (LoopCandidate * max(len(flat), 1))()
        keep = []
        for k, (v1, v2, m) in enumerate(flat):
            a = np.ascontiguousarray(m, np.int32)
            keep.append(a)
            lc[k].kf1, lc[k].kf2, lc[k].matches12 = v1.h.value, v2.h.value, a.ctypes.data
        res = (LoopGateResult * len(self.events))()
        n1 = [cs[0][0].n if cs else 0 for cs in candidates]
        mo = [np.full(max(n, 1), -1, np.int32) for n in n1]
        pm = (C.c_void_p * len(self.events))(*[a.ctypes.data for a in mo])
        _check(L.rsc_loop_events_gated(self.batch._h, lc, self.begin, len(self.events), self._cand, res, pm),
               "loop_events_gated")
        return np.ctypeslib.as_array(res).copy(), [m[:n] for m, n in zip(mo, n1)]

    def winner_poses(self) -> np.ndarray:
        """[n_events, 16] float32 pose of each event's winning candidate (PnP Tcw row-major, Sim3
        [R|t; 0 0 0 1]); zeros for events without a winner."""
        out = np.zeros((len(self.events), 16), np.float32)
        for e in range(len(self.events)):
            w = int(self.per_event["winner"][e])
            if w < 0:
                continue
            r = self.cand[self.begin[e] + w]
            if self.kind == "pnp":
                out[e] = np.asarray(r["T"], np.float32).ravel()
            else:
                R = np.asarray(r["R"], np.float32).reshape(3, 3)
                out[e, 0:3], out[e, 4:7], out[e, 8:11] = R[0], R[1], R[2]
                out[e, 3], out[e, 7], out[e, 11], out[e, 15] = r["t"][0], r["t"][1], r["t"][2], 1.0
        return out


class PoseOptBatch:
    """Frames prepared once for repeated rsc_pose_optimization_many calls (the ctypes problem
    records and contiguous arrays are built here, so a call is one C entry)."""

    def __init__(self, ctx: Context, frames, with_outliers: bool = True):
        self.ctx = ctx
        self.frames = list(frames)
        n = len(self.frames)
        self.probs = (PoseOptProblem * max(n, 1))()
        self.res = (PoseOptResult * max(n, 1))()
        self.ptrs = (C.c_void_p * max(n, 1))()
        self.keep, self.outs = [], []
        for i, f in enumerate(self.frames):
            arrs = [np.ascontiguousarray(f.has_mp, np.uint8), np.ascontiguousarray(f.uv, np.float32).reshape(-1),
                    np.ascontiguousarray(f.Xw, np.float32).reshape(-1),
                    np.ascontiguousarray(f.inv_sigma2, np.float32)]
            ur = getattr(f, "u_right", None)
            if ur is not None:
                arrs.append(np.ascontiguousarray(ur, np.float32))
            self.keep.append(arrs)
            p = self.probs[i]
            p.n = f.n
            p.has_mp, p.uv, p.Xw, p.inv_sigma2 = (a.ctypes.data for a in arrs[:4])
            p.u_right = arrs[4].ctypes.data if ur is not None else None
            p.bf = float(getattr(f, "bf", 0.0))
            p.fx, p.fy, p.cx, p.cy = float(f.fx), float(f.fy), float(f.cx), float(f.cy)
            p.Tcw[:] = [float(v) for v in np.asarray(f.Tcw, np.float32).reshape(16)]
            o = np.full(max(f.n, 1), 255, np.uint8)
            self.outs.append(o)
            self.ptrs[i] = o.ctypes.data if with_outliers else None

    def run(self):
        _check(load_library().rsc_pose_optimization_many(self.ctx.h, self.probs, len(self.frames), self.res,
                                                         self.ptrs), "rsc_pose_optimization_many")

    def results(self):
        out = []
        for i, f in enumerate(self.frames):
            r = self.res[i]
            out.append({"n_good": r.n_good, "n_initial": r.n_initial, "rounds": r.rounds,
                        "lm_iterations": r.lm_iterations, "lm_trials": r.lm_trials,
                        "Tcw": np.array(r.Tcw[:], np.float32).reshape(4, 4), "outlier": self.outs[i][:f.n].copy()})
        return out


class Sim3OptBatch:
    """Loop-closure pairs prepared once for repeated rsc_optimize_sim3_many calls
    (Optimizer::OptimizeSim3, Optimizer.cpp:1054-1250).  problems: rsc.synth.Sim3OptProblem-likes."""

    def __init__(self, ctx: Context, problems):
        self.ctx = ctx
        self.problems = list(problems)
        n = len(self.problems)
        self.probs = (Sim3OptProblem * max(n, 1))()
        self.res = (Sim3OptResult * max(n, 1))()
        self.ptrs = (C.c_void_p * max(n, 1))()
        self.keep, self.keeps = [], []
        for i, p in enumerate(self.problems):
            arrs = [np.ascontiguousarray(p.valid, np.uint8)] + [np.ascontiguousarray(a, np.float32).reshape(-1) for a in
                                                                (p.X1w, p.X2w, p.uv1, p.uv2, p.inv1, p.inv2)]
            self.keep.append(arrs)
            q = self.probs[i]
            q.n = p.n
            q.valid, q.X1w, q.X2w, q.uv1, q.uv2, q.inv1, q.inv2 = (a.ctypes.data for a in arrs)
            q.R1w[:] = [float(v) for v in np.asarray(p.R1w, np.float32).ravel()]
            q.t1w[:] = [float(v) for v in np.asarray(p.t1w, np.float32)]
            q.R2w[:] = [float(v) for v in np.asarray(p.R2w, np.float32).ravel()]
            q.t2w[:] = [float(v) for v in np.asarray(p.t2w, np.float32)]
            q.K1[:] = [float(v) for v in np.asarray(p.K1, np.float32)]
            q.K2[:] = [float(v) for v in np.asarray(p.K2, np.float32)]
            q.S[:] = [float(v) for v in np.asarray(p.S0, np.float64)]
            q.th2 = float(p.th2)
            k = np.full(max(p.n, 1), 7, np.uint8)
            self.keeps.append(k)
            self.ptrs[i] = k.ctypes.data

    def run(self):
        _check(load_library().rsc_optimize_sim3_many(self.ctx.h, self.probs, len(self.problems), self.res, self.ptrs),
               "rsc_optimize_sim3_many")

    def results(self):
        out = []
        for i, p in enumerate(self.problems):
            r = self.res[i]
            out.append({"n_inliers": r.n_inliers, "n_correspondences": r.n_correspondences, "n_bad": r.n_bad,
                        "lm_iterations": r.lm_iterations, "lm_trials": r.lm_trials,
                        "S": np.array(r.S[:], np.float64), "keep": self.keeps[i][:p.n].copy()})
        return out


def optimize_sim3_many(ctx: Context, problems):
    """Optimizer::OptimizeSim3 on every loop-closure pair in one launch.  Returns per pair a dict:
    n_inliers (the reference's return value), n_correspondences, n_bad, lm_iterations, lm_trials,
    S float64[8] (g2oS12 after the call: q x, y, z, w, t, s), keep uint8[n] (0 where vpMatches1[i]
    is set to NULL)."""
    b = Sim3OptBatch(ctx, problems)
    b.run()
    return b.results()


def pose_optimization_many(ctx: Context, frames, with_outliers: bool = True):
    """Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) on every frame in one launch.

    frames: objects with has_mp, uv, Xw, inv_sigma2, Tcw, fx..cy and optionally u_right (mvuRight,
    >= 0 on stereo slots) + bf (rsc.synth.PoseOptFrame).  Returns
    per frame a dict: n_good (the reference's return value), n_initial, rounds, lm_iterations,
    lm_trials, Tcw float32[4,4] (pFrame->mTcw after the call), outlier uint8[n] (mvbOutlier; 255 on
    slots without a map point)."""
    b = PoseOptBatch(ctx, frames, with_outliers)
    b.run()
    return b.results()


class BowView:
    """A KeyFrame's / Frame's ORB features resident in HBM for ORBmatcher::SearchByBoW: descriptors
    (mDescriptors), keypoint angles, map-point validity and the DBoW2 FeatureVector (mFeatVec) as
    CSR (rsc_bow_features, include/rsc.h).  `view` is an object with n, desc uint8[n,32],
    angle float32[n], valid uint8[n] (or None), node_id uint32[], node_begin int32[], feat uint32[]
    (rsc.synth.BowFeatures)."""

    def __init__(self, ctx: Context, view):
        self.ctx = ctx
        self.n = int(view.n)
        arrs = [np.ascontiguousarray(view.desc, np.uint8).reshape(-1), np.ascontiguousarray(view.angle, np.float32),
                None if view.valid is None else np.ascontiguousarray(view.valid, np.uint8),
                np.ascontiguousarray(view.node_id, np.uint32), np.ascontiguousarray(view.node_begin, np.int32),
                np.ascontiguousarray(view.feat, np.uint32)]
        f = BowFeatures()
        f.n = self.n
        f.desc, f.angle = arrs[0].ctypes.data, arrs[1].ctypes.data
        f.valid = None if arrs[2] is None else arrs[2].ctypes.data
        f.n_nodes = len(arrs[3])
        f.node_id, f.node_begin, f.feat = arrs[3].ctypes.data, arrs[4].ctypes.data, arrs[5].ctypes.data
        h = C.c_void_p()
        _check(load_library().rsc_bow_create(ctx.h, C.byref(f), C.byref(h)), "rsc_bow_create")
        self.h = h

    def set_valid(self, valid):
        _check(load_library().rsc_bow_set_valid(self.h, np.ascontiguousarray(valid, np.uint8)), "rsc_bow_set_valid")

    def close(self):
        if getattr(self, "h", None):
            load_library().rsc_bow_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class BowSearch:
    """Prepared SearchByBoW batch (ORBmatcher.cpp:110-240 / :354-488): `count` searches in one launch.

    frame_overload=True: SearchByBoW(pKF = others[c], F = shared) -> rows of shared.n (KeyFrame index
    per Frame feature).  False: SearchByBoW(pKF1 = shared, pKF2 = others[c]) -> rows of shared.n
    (KF2 index per KF1 feature)."""

    def __init__(self, ctx: Context, shared: BowView, others, frame_overload: bool, nnratio: float = 0.75,
                 check_orientation: bool = True):
        self.ctx, self.shared, self.others = ctx, shared, list(others)
        self.frame_overload = frame_overload
        self.nnratio, self.check = float(nnratio), int(bool(check_orientation))
        c = len(self.others)
        self.handles = (C.c_void_p * max(c, 1))(*[o.h for o in self.others])
        self.out = np.zeros((max(c, 1), max(shared.n, 1)), np.int32)
        self.ptrs = (C.c_void_p * max(c, 1))(*[self.out[i].ctypes.data for i in range(c)])
        self.nmatches = np.zeros(max(c, 1), np.int32)

    def run(self):
        L = load_library()
        c = len(self.others)
        if self.frame_overload:
            st = L.rsc_search_by_bow_frame_many(self.ctx.h, self.handles, c, self.shared.h, self.nnratio, self.check,
                                                self.ptrs, self.nmatches)
        else:
            st = L.rsc_search_by_bow_kf_many(self.ctx.h, self.shared.h, self.handles, c, self.nnratio, self.check,
                                             self.ptrs, self.nmatches)
        _check(st, "rsc_search_by_bow")
        c = len(self.others)
        return self.out[:c, :self.shared.n], self.nmatches[:c]


def search_by_bow_frame_many(ctx: Context, kfs, frame, nnratio=0.75, check_orientation=True):
    """SearchByBoW(pKF, F, vpMapPointMatches) for every KeyFrame view against one Frame view
    (Tracking::Relocalization, Tracking.cpp:1207-1214: ORBmatcher(0.75, true)).  Returns
    (matches int32[count, F.n] = KeyFrame feature index or -1, nmatches int32[count])."""
    return BowSearch(ctx, frame, kfs, True, nnratio, check_orientation).run()


def search_by_bow_kf_many(ctx: Context, kf1, kf2s, nnratio=0.75, check_orientation=True):
    """SearchByBoW(pKF1, pKF2, vpMatches12) of one KeyFrame view against each candidate
    (LoopClosing::ComputeSim3, LoopClosing.cpp:238-251).  Returns (matches12 int32[count, kf1.n],
    nmatches int32[count])."""
    return BowSearch(ctx, kf1, kf2s, False, nnratio, check_orientation).run()
