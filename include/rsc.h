/*
 * rsc.h — C ABI of the MI355X RANSAC pose engine (librsc.so).
 *
 * Drop-in boundary for the hot path of Luigi940260/orb-slam2-optimized: the geometric RANSAC
 * solvers called by Tracking::Relocalization() and LoopClosing::ComputeSim3().  Every entry point
 * below replaces one member of the reference classes (file:line of the reference cited per
 * function); the C++ facade in orb-slam2-optimized_amd/csrc/facade/ re-exposes them with the
 * reference's exact class signatures.  Plain pointers and sizes only; no torch / HIP types.
 *
 * Semantics are the reference's, including its quirks.  rand(): by default
 * every solver owns a glibc stream seeded with `seed` (H4: identical to srand(seed) right before that
 * solver runs alone); solvers bound to an rsc_stream (rsc_*_bind_stream) instead draw from ONE shared
 * stream in call order, the reference's process-global rand() (Q3, Random.cpp:47-50).
 *
 * Status codes: 0 = ok, < 0 = error (see rsc_status_string).  The library fails loudly: when no
 * HIP device is present, rsc_context_create returns RSC_ERR_NODEVICE; there is no CPU fallback.
 */
#ifndef RSC_H_
#define RSC_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSC_OK 0
#define RSC_ERR_ARG (-1)
#define RSC_ERR_HIP (-2)
#define RSC_ERR_OOM (-3)
#define RSC_ERR_UNSUPPORTED (-4)
#define RSC_ERR_NODEVICE (-5)
#define RSC_ERR_INTERNAL (-6) /* an engine invariant failed (a bug; rsc_status_string says which) */

typedef struct rsc_context rsc_context;
typedef struct rsc_pnp rsc_pnp;
typedef struct rsc_sim3 rsc_sim3;
typedef struct rsc_mlpnp rsc_mlpnp;
typedef struct rsc_stream rsc_stream;

/* ---- library / context ------------------------------------------------------------------ */
int rsc_version(void);
const char* rsc_status_string(int status);
/* One context per host thread (reference: the Tracking and LoopClosing threads each own their
 * solvers, System.cpp:58-69).  Owns a HIP stream, the rand() jump table and work buffers. */
int rsc_context_create(int device, rsc_context** out);
void rsc_context_destroy(rsc_context* ctx);
/* Use a caller-owned hipStream_t (e.g. torch's current stream) instead of the private one. */
int rsc_context_set_stream(rsc_context* ctx, void* hip_stream);
int rsc_context_synchronize(rsc_context* ctx);
/* Per-kernel timing of the last iterate call, in milliseconds (HIP events on the context stream):
 * out[0] = hypothesis-solve kernels, out[1] = inlier-scan kernels, out[2] = refine kernels,
 * out[3] = number of solve launches, out[4] = hypotheses solved. */
int rsc_context_last_timing(rsc_context* ctx, double out[5]);
/* As above plus out[5] = eigen-stage kernel (pnp_eig_group/lane_kernel) alone, split solve modes. */
int rsc_context_last_kernel_timing(rsc_context* ctx, double out[6]);
/* Diagnostic: host clock of the last rsc_pnp_iterate_many in microseconds from entry to
 * [0] first launch, [1] kernels enqueued, [2] results back on the host, [3] return. */
int rsc_diag_host_timing(rsc_context* ctx, double out[4]);
int rsc_context_enable_timing(rsc_context* ctx, int enable);
/* Eigen-stage form of the EPnP hypothesis solve (no effect on results): launches whose eigen stage
 * has at most max_workgroups workgroups of 20 hypotheses run it in the Refine's rows form (a 12-lane
 * group per hypothesis, Q rows in VGPRs: lower latency for small, latency-bound launches such as one
 * relocalization event); larger launches use the split form (below).  Default 64 (env RSC_EIG_ROWS
 * overrides); 0 = never the rows form. */
int rsc_context_set_eig_rows(rsc_context* ctx, int max_workgroups);
/* Eigen-stage form of the launches the rows form does not take: 1 (default; env RSC_EIG_SPLIT) the
 * split form — the QR chase and the Q rotations on two waves of one SIMD (pnp_eig_split_kernel) — or
 * 0 the lane-pair form (pnp_eig_group_kernel).  Both are bit-identical. */
int rsc_context_set_eig_split(rsc_context* ctx, int on);
/* Form of rsc_optimize_sim3_many (no effect on results): helpers > 0 runs each pair on one master
 * workgroup plus that many helper workgroups that evaluate the edges' numeric Jacobians in chunks
 * (the cooperative form); 0 one workgroup per pair; -1 (default; env RSC_SO_HELPERS) as many helpers
 * as fit one workgroup per CU, at most 7 per pair.  Bit-identical results. */
int rsc_context_set_sim3opt_helpers(rsc_context* ctx, int helpers);
/* Self-test of the device libm restatement (rsc_math.h, used by Sim3 angles, MLPnP, SearchBySim3):
 * out[i] = f(x[i]) computed ON THE GPU, f = 0 sin, 1 cos, 2 acos, 3 cbrt, 4 log, 5 logf
 * ((float)x[i] in, float result widened); and the eigen-solver chase's short-chain forms
 * (rsc_core.h): 6 sqrt for x in [1,4), 7 1/x for |x| in [1,2), 8 / 9 make_givens(x[i],
 * x[(i+n/2)%n]) c / s; 10 qr_solve_6x4 (PnPsolver.cpp:693-796) on records of 34 doubles
 * (A[6][4] row-major, b[6], previous X[4]) -> X in out[0..3], 1/0 success in out[4] of each record
 * (n a multiple of 34); 11 pow(x, 1.0/3.0), 12 pow(x, 3.0/2.0) as MLPnP computes them (x >= 0;
 * MLPnPsolver.cpp:567, :839, :901); 13 the PnP scan's float reciprocal of (float)x (v_rcp_f32 + one
 * Newton step, PnPsolver.cpp:251); (14, 15 unused); 16 the LM steps' 6 x 6 LDLT solve in its scalar and row-per-lane forms
 * (records of 42: matrix row-major + b in, x / ok of each form out; n a multiple of 42).  Host
 * pointers, n >= 0.  Tests compare with glibc / IEEE numpy / the oracle. */
int rsc_selftest_math(rsc_context* ctx, int fn, const double* x, int n, double* out);

/* ---- PnPsolver (include/PnPsolver.hpp:21-138, src/PnPsolver.cpp) ------------------------------ */
typedef struct {
    int32_t n;               /* compacted valid matches N (PnPsolver.cpp:22-44) */
    int32_t n_points;        /* vpMapPointMatches.size(): length of the returned inlier vector */
    const float* p2d;        /* [n][2] mvP2D = mvKeysUn[i].pt                       (:33) */
    const float* p3dw;       /* [n][3] mvP3Dw = MapPoint::GetWorldPos()             (:36) */
    const float* sigma2;     /* [n] mvSigma2 = mvLevelSigma2[kp.octave]             (:34) */
    const int32_t* kp_index; /* [n] mvKeyPointIndices; NULL = identity               (:38) */
    float fx, fy, cx, cy;    /* Frame::fx,fy,cx,cy (static float members, :47-50)       */
} rsc_pnp_problem;

typedef struct {
    int32_t ok;         /* iterate()/find() return value */
    int32_t no_more;    /* bNoMore */
    int32_t n_inliers;  /* nInliers */
    int32_t iterations; /* mnIterations after the call */
    float T[16];        /* row-major Tcw; written only when ok (PnPsolver.cpp:166,185) */
} rsc_pnp_result;

/* PnPsolver::PnPsolver (PnPsolver.cpp:11-55).  Copies the arrays to HBM. */
int rsc_pnp_create(rsc_context* ctx, const rsc_pnp_problem* problem, uint32_t seed, rsc_pnp** out);
void rsc_pnp_destroy(rsc_pnp* s);
/* PnPsolver::SetRansacParameters (PnPsolver.cpp:58-94; defaults 0.99, 8, 300, 4, 0.4, 5.991). */
int rsc_pnp_set_ransac_parameters(rsc_pnp* s, double probability, int min_inliers, int max_iterations,
                                  int min_set, float epsilon, float th2);
/* PnPsolver::iterate (PnPsolver.cpp:102-191).  `inliers` receives n_points bytes (vbInliers) or
 * is left untouched when the reference returns an empty vector (:105); may be NULL. */
int rsc_pnp_iterate(rsc_pnp* s, int n_iterations, rsc_pnp_result* out, uint8_t* inliers);
/* PnPsolver::find (PnPsolver.cpp:96-100). */
int rsc_pnp_find(rsc_pnp* s, rsc_pnp_result* out, uint8_t* inliers);
/* vbInliers of the last iterate() / find() of this solver (n_points bytes; mvbRefinedInliers or
 * mvbBestInliers scattered through the keypoint indices, PnPsolver.cpp:159-166, :176-186), fetched
 * after the call — e.g. for the candidate a rank contributes to the multi-GPU winner exchange.
 * Returns 1, or 0 with all-zero bytes when that call returned false (vbInliers empty, :105). */
int rsc_pnp_last_inliers(rsc_pnp* s, uint8_t* out);
/* iterate() on `count` solvers of ONE context at once (the relocalization candidates of
 * Tracking.cpp:1239-1334); all hypotheses of all solvers run in the same kernel launches.
 * Results are identical to calling rsc_pnp_iterate on each solver in order. */
int rsc_pnp_iterate_many(rsc_pnp* const* solvers, int count, const int32_t* n_iterations, rsc_pnp_result* out,
                         uint8_t* const* inliers);
/* Back to the freshly constructed state with a new rand() stream (reuse HBM-resident data). */
int rsc_pnp_reset(rsc_pnp* s, uint32_t seed);
/* rsc_pnp_reset / rsc_pnp_set_ransac_parameters over `count` solvers in one call. */
int rsc_pnp_reset_many(rsc_pnp* const* solvers, int count, const uint32_t* seeds);
int rsc_pnp_set_ransac_parameters_many(rsc_pnp* const* solvers, int count, double probability, int min_inliers,
                                       int max_iterations, int min_set, float epsilon, float th2);
/* out: [0] mnIterations [1] mRansacMaxIts [2] mRansacMinInliers [3] mnBestInliers
 *      [4] maximum_number_of_correspondences [5] N [6] N_points [7] mRansacMinSet */
int rsc_pnp_get_state(const rsc_pnp* s, int32_t out[8]);
/* Debug/parity hook: sample indices (8 per hypothesis) of the last launch for this solver. */
int rsc_pnp_last_samples(rsc_pnp* s, int32_t* out, int cap);
/* Parity hook: inlier counts and float poses (R row-major 9 + t 3) of every hypothesis of the last
 * launch for this solver (PnPsolver.cpp:139-146 mnInliersi / mRi, mti per hypothesis).  Valid until
 * the context's next launch. */
int rsc_pnp_last_hypotheses(rsc_pnp* s, int32_t* counts, float* poses, int cap);

/* ---- Sim3Solver (include/Sim3Solver.hpp:16-103, src/Sim3Solver.cpp) --------------------------- */
/* Raw constructor inputs for one keyframe pair (Sim3Solver.cpp:6-85), per match slot i1 < n1. */
typedef struct {
    int32_t n1;              /* vpMatched12.size() */
    const uint8_t* valid;    /* slot usable: match, pMP1, not bad, both indices >= 0 (:28-43) */
    const float* Xw1;        /* [n1][3] pMP1->GetWorldPos() */
    const float* Xw2;        /* [n1][3] pMP2->GetWorldPos() */
    const float* sigma2_1;   /* [n1] pKF1->mvLevelSigma2[kp1.octave] */
    const float* sigma2_2;   /* [n1] pKF2->mvLevelSigma2[kp2.octave] */
    float R1[9], t1[3];      /* pKF1->GetRotation()/GetTranslation(), row-major */
    float R2[9], t2[3];
    float K1[4], K2[4];      /* fx, fy, cx, cy of KeyFrame::mK */
} rsc_sim3_input;

/* Sim3Solver::Sim3Solver (Sim3Solver.cpp:6-85, includes its SetRansacParameters() call). */
int rsc_sim3_create(rsc_context* ctx, const rsc_sim3_input* in, uint32_t seed, rsc_sim3** out);
void rsc_sim3_destroy(rsc_sim3* s);
/* Sim3Solver::SetRansacParameters (Sim3Solver.cpp:87-111; defaults 0.99, 6, 300). */
int rsc_sim3_set_ransac_parameters(rsc_sim3* s, double probability, int min_inliers, int max_iterations);
typedef struct {
    int32_t ok, no_more, n_inliers, iterations;
    float R[9], t[3];    /* GetEstimatedRotation()/GetEstimatedTranslation() after the call */
} rsc_sim3_result;
/* Sim3Solver::iterate (Sim3Solver.cpp:113-178); `inliers` receives n1 bytes (always sized). */
int rsc_sim3_iterate(rsc_sim3* s, int n_iterations, rsc_sim3_result* out, uint8_t* inliers);
int rsc_sim3_find(rsc_sim3* s, rsc_sim3_result* out, uint8_t* inliers);
int rsc_sim3_iterate_many(rsc_sim3* const* solvers, int count, const int32_t* n_iterations, rsc_sim3_result* out,
                          uint8_t* const* inliers);
int rsc_sim3_reset(rsc_sim3* s, uint32_t seed);
int rsc_sim3_reset_many(rsc_sim3* const* solvers, int count, const uint32_t* seeds);
int rsc_sim3_set_ransac_parameters_many(rsc_sim3* const* solvers, int count, double probability, int min_inliers,
                                        int max_iterations);
/* out: [0] mnIterations [1] mRansacMaxIts [2] mRansacMinInliers [3] mnBestInliers [4] N [5] mN1 */
int rsc_sim3_get_state(const rsc_sim3* s, int32_t out[6]);
/* Prepared per-correspondence arrays built by the constructor (for parity tests):
 * X1c/X2c [N][3], P1im1/P2im2 [N][2], max_err1/2 [N] (size_t thresholds), indices1 [N]. */
/* Parity hook: inlier counts and float (R12 9 + t12 3) of every hypothesis of the last launch
 * (Sim3Solver.cpp:150-153 mnInliersi / mR12i, mt12i). */
int rsc_sim3_last_hypotheses(rsc_sim3* s, int32_t* counts, float* poses, int cap);
int rsc_sim3_prepared(const rsc_sim3* s, float* X1c, float* X2c, float* P1im1, float* P2im2, uint64_t* max_err1,
                      uint64_t* max_err2, int32_t* indices1);

/* ---- MLPnPsolver (include/MLPnPsolver.hpp:10-199, src/MLPnPsolver.cpp) ----------------------------
 * Dormant in the reference (not compiled, call sites commented out, Tracking.cpp:1222,1227-1228);
 * exported for BASELINE config 4.  Same problem struct and result record as PnP.  Parity of this
 * solver against the reference is unpinned. */
/* MLPnPsolver::MLPnPsolver (MLPnPsolver.cpp:5-53, includes its SetRansacParameters() call). */
int rsc_mlpnp_create(rsc_context* ctx, const rsc_pnp_problem* problem, uint32_t seed, rsc_mlpnp** out);
void rsc_mlpnp_destroy(rsc_mlpnp* s);
/* computePose's covMats (MLPnPsolver.cpp:321, :375-388, :483-484, :694-695): cov = [n][9] row-major
 * 3x3 bearing-vector covariance per correspondence (the problem's compacted order), or NULL for the
 * reference's own configuration (it passes a single-element covMats, so use_cov is false).  With
 * covariances the hypotheses solve A^T P A and the Gauss-Newton runs on J^T Kll J, P = Kll the
 * block-diagonal (N^T Sigma N)^-1.  Not reachable from the reference's callers: parity unpinned
 * (SURVEY.md Q15); checked against the oracle's restatement. */
int rsc_mlpnp_set_covariances(rsc_mlpnp* s, const double* cov);
/* MLPnPsolver::SetRansacParameters (MLPnPsolver.cpp:185-220; defaults 0.99, 8, 300, 6, 0.4, 5.991).
 * min_set must be in [6, 8] (computePose asserts n > 5, :324) -> RSC_ERR_UNSUPPORTED otherwise. */
int rsc_mlpnp_set_ransac_parameters(rsc_mlpnp* s, double probability, int min_inliers, int max_iterations,
                                    int min_set, float epsilon, float th2);
int rsc_mlpnp_set_ransac_parameters_many(rsc_mlpnp* const* solvers, int count, double probability, int min_inliers,
                                         int max_iterations, int min_set, float epsilon, float th2);
/* MLPnPsolver::iterate (MLPnPsolver.cpp:56-183): T is identity unless ok (Tout.setIdentity(), :57). */
int rsc_mlpnp_iterate(rsc_mlpnp* s, int n_iterations, rsc_pnp_result* out, uint8_t* inliers);
int rsc_mlpnp_iterate_many(rsc_mlpnp* const* solvers, int count, const int32_t* n_iterations, rsc_pnp_result* out,
                           uint8_t* const* inliers);
int rsc_mlpnp_reset(rsc_mlpnp* s, uint32_t seed);
int rsc_mlpnp_reset_many(rsc_mlpnp* const* solvers, int count, const uint32_t* seeds);
/* out: [0] mnIterations [1] mRansacMaxIts [2] mRansacMinInliers [3] mnBestInliers [4] N [5] mRansacMinSet */
int rsc_mlpnp_get_state(const rsc_mlpnp* s, int32_t out[6]);
/* Parity hooks: double poses (R 9 + t 3) and sample indices (8 per hypothesis) of the last launch. */
int rsc_mlpnp_last_poses(rsc_mlpnp* s, double* out, int cap);
int rsc_mlpnp_last_samples(rsc_mlpnp* s, int32_t* out, int cap);
int rsc_mlpnp_last_counts(rsc_mlpnp* s, int32_t* counts, int cap);

/* ---- The reference's shared rand() stream (Q3) ---------------------------------------------------
 * DUtils::Random::RandomInt (Thirdparty/DBoW2/DUtils/Random.cpp:47-50) draws from glibc's process-
 * global rand(), which the reference never seeds (= srand(1)); every candidate's iterate() of a
 * relocalization (Tracking.cpp:1239-1262) or loop closure (LoopClosing.cpp:271-286) continues that one
 * stream where the previous call stopped.  An rsc_stream is that stream: srand(seed) and a position. */
int rsc_stream_create(rsc_context* ctx, uint32_t seed, rsc_stream** out);
void rsc_stream_destroy(rsc_stream* s);
/* Consume n draws (rand() calls made elsewhere in the process between two solver calls). */
int rsc_stream_skip(rsc_stream* s, int64_t n);
/* Draws consumed since srand(seed). */
int rsc_stream_position(const rsc_stream* s, int64_t* out);
/* The next n rand() outputs, without consuming them (parity hook; computed on the device). */
int rsc_stream_peek(rsc_stream* s, int n, int32_t* out);
/* Bind a solver to a shared stream (NULL: back to its own stream, which resumes where it stopped).
 * Every later iterate()/find() of a bound solver draws its samples from the stream's current position
 * and advances it by the draws it made (mRansacMinSet per PnP / MLPnP hypothesis, 3 per Sim3
 * hypothesis), exactly as the reference's call does.  *_iterate_many over bound solvers runs the
 * calls one after the other in list order (the reference's call order). */
int rsc_pnp_bind_stream(rsc_pnp* s, rsc_stream* stream);
int rsc_sim3_bind_stream(rsc_sim3* s, rsc_stream* stream);
int rsc_mlpnp_bind_stream(rsc_mlpnp* s, rsc_stream* stream);

/* ---- Event drivers (BASELINE config 5) -----------------------------------------------------------
 * One relocalization or loop-closure event = the candidate solvers one Tracking::Relocalization() /
 * LoopClosing::ComputeSim3() call builds (Tracking.cpp:1207-1232, LoopClosing.cpp:238-265), stored
 * contiguously: event e owns solvers[event_begin[e] .. event_begin[e+1]).  Every candidate of every
 * event runs in the same launches. */
typedef struct {
    int32_t winner;      /* first candidate (in the reference's round-robin order) whose iterate()
                            returns a pose, -1 if none: the pose the reference hands to
                            PoseOptimization / SearchBySim3 first */
    int32_t round;       /* round of iterate(5) calls in which it returns */
    int32_t hypothesis;  /* index of the returning hypothesis in that candidate's stream */
    int32_t n_inliers;
} rsc_event_result;
/* Relocalization (Tracking.cpp:1239-1262): rounds of iterate(5) over the non-discarded candidates
 * (bNoMore discards) until a candidate returns a pose; per_candidate receives each candidate's last
 * iterate() result (candidates after the winner in the winning round are iterated as well — the
 * reference reaches them only if the downstream check rejects the winner, with identical results). */
int rsc_reloc_events(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events, rsc_pnp_result* per_candidate,
                     rsc_event_result* per_event);
/* Loop closure (LoopClosing.cpp:271-286): each candidate's stream is run to its first success or
 * to mRansacMaxIts in one call; the winner is the lexicographically smallest (round, candidate) with
 * round = hypothesis / 5 — identical to the reference's round-robin of iterate(5) calls. */
int rsc_loop_events(rsc_sim3* const* solvers, const int32_t* event_begin, int n_events,
                    rsc_sim3_result* per_candidate, rsc_event_result* per_event);
/* The same events on the reference's shared rand() stream: event e's calls draw from streams[e]
 * (one distinct stream per event; its position at the Relocalization / ComputeSim3 call) in the
 * round-robin's call order — round by round, candidate by candidate, iterate(5) each — and advance it.
 * All events' rounds still run in the same launches: each call is positioned assuming every earlier
 * call of its round ran its whole loop, which holds up to the first success (the only early return),
 * and that success ends the event.  Candidates after the winner in the winning round are calls the
 * reference never makes: their per_candidate records are left as they were and their solver state
 * is unspecified.  Solvers must not be bound to a stream (RSC_ERR_ARG). */
int rsc_reloc_events_shared(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events,
                            rsc_stream* const* streams, rsc_pnp_result* per_candidate, rsc_event_result* per_event);
int rsc_loop_events_shared(rsc_sim3* const* solvers, const int32_t* event_begin, int n_events,
                           rsc_stream* const* streams, rsc_sim3_result* per_candidate, rsc_event_result* per_event);

/* ---- Gated events (round 6): the reference's post-RANSAC acceptance test inside the event loop ----
 * The drivers above end an event at the first candidate whose iterate() returns a pose.  The
 * reference then checks that pose with the next stages and, on rejection, continues the round-robin
 * (the next candidate of the same round, then later rounds, the rejected candidate included).  The
 * gated drivers run those stages on the device (PoseOptimization / SearchBySim3 + OptimizeSim3, the
 * kernels of rsc_pose_optimization_many / rsc_search_by_sim3_many / rsc_optimize_sim3_many) for every
 * success in the reference's order, batched across events, until a success passes.  Solvers draw
 * from their own streams (bound solvers: RSC_ERR_UNSUPPORTED).  per_candidate: each candidate's last
 * iterate() record. */
#define RSC_GATE_NONE 0    /* every candidate discarded without an accepted pose (bMatch false) */
#define RSC_GATE_MATCH 1   /* a success passed the gate (bMatch = true) */
#define RSC_GATE_HANDOFF 2 /* relocalization: 10 <= nGood < 50 after PoseOptimization; the reference runs
                              SearchByProjection next (Tracking.cpp:1294-1323, outside this engine) —
                              the event stops here and the host continues it (the records of the
                              candidates after the winner in its round are already those calls' results) */
/* Tracking::Relocalization (Tracking.cpp:1239-1335).  The current Frame's data PoseOptimization reads
 * beyond what the solvers hold (their compacted p2d / p3dw / sigma2 are Frame::mvKeysUn, the MapPoint
 * positions and mvLevelSigma2; mvInvLevelSigma2 = 1.0f / mvLevelSigma2 as ORBextractor sets it). */
typedef struct {
    const float* u_right;  /* [n_points] Frame::mvuRight (>= 0: stereo edge), NULL for a monocular Frame */
    float bf;              /* Frame::mbf */
} rsc_reloc_frame;
typedef struct {
    int32_t status;       /* RSC_GATE_* */
    int32_t winner;       /* candidate of the accepted (MATCH) or handed-off success, -1 for NONE */
    int32_t round;        /* its round of iterate(5) calls */
    int32_t hypothesis;   /* index of the returning hypothesis in that candidate's stream */
    int32_t n_inliers;    /* RANSAC nInliers of that success */
    int32_t n_good;       /* PoseOptimization's return value on it (Tracking.cpp:1284) */
    int32_t rejected;     /* successes rejected before it (nGood < 10, Tracking.cpp:1286-1287) */
    int32_t gates;        /* PoseOptimization runs of the event */
    float Tcw[16];        /* row-major pose after PoseOptimization (mCurrentFrame.mTcw) */
} rsc_reloc_gate_result;
/* frames[e]: event e's current Frame (its solvers' n_points = Frame::N).  outlier[e] (may be NULL, or
 * NULL entries): [n_points] mvbOutlier of the winner's PoseOptimization for the slots with a map point
 * (others 0); inliers[e] (may be NULL / NULL entries): [n_points] the winner's vbInliers. */
int rsc_reloc_events_gated(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events,
                           const rsc_reloc_frame* frames, rsc_pnp_result* per_candidate,
                           rsc_reloc_gate_result* per_event, uint8_t* const* outlier, uint8_t* const* inliers);

/* LoopClosing::ComputeSim3 (LoopClosing.cpp:268-329).  A candidate's Sim3 solver was built from
 * (kf1 = mpCurrentKF, kf2 = the candidate KeyFrame, vvpMapPointMatches[i]); the gate needs those
 * views and matches: SearchBySim3(kf1, kf2, vpMapPointMatches = the RANSAC inliers of matches12, R,
 * t, 7.5) then OptimizeSim3(kf1, kf2, vpMapPointMatches, gScm = Sim3(R, t, 1), 10) with
 * mvInvLevelSigma2 = 1 / (scale_factors[l]^2) (float, as ORBextractor); accepted when nInliers >= 20. */
struct rsc_kfview;
typedef struct {
    struct rsc_kfview* kf1;    /* mpCurrentKF's view (rsc_kfview_create) */
    struct rsc_kfview* kf2;    /* the candidate KeyFrame's view */
    const int32_t* matches12;  /* [kf1 n] vvpMapPointMatches[i]: KF2 keypoint index of the matched
                                  MapPoint, -1 NULL, -2 a MapPoint not in KF2 (the solver's input) */
} rsc_loop_candidate;
typedef struct {
    int32_t status;         /* RSC_GATE_NONE or RSC_GATE_MATCH */
    int32_t winner, round, hypothesis, n_inliers;  /* the accepted success (as rsc_event_result) */
    int32_t n_found;        /* SearchBySim3's return value on it */
    int32_t n_opt_inliers;  /* OptimizeSim3's return value (>= 20 on MATCH) */
    int32_t rejected;       /* successes rejected before it (nInliers < 20) */
    double S[8];            /* gScm after OptimizeSim3: q (x, y, z, w), t, s */
} rsc_loop_gate_result;
/* matches_out[e] (may be NULL / NULL entries): [kf1 n] mvpCurrentMatchedPoints of the accepted
 * candidate as KF2 keypoint indices (-1 NULL, -2 a MapPoint not in KF2). */
int rsc_loop_events_gated(rsc_sim3* const* solvers, const rsc_loop_candidate* candidates,
                          const int32_t* event_begin, int n_events, rsc_sim3_result* per_candidate,
                          rsc_loop_gate_result* per_event, int32_t* const* matches_out);

/* ---- Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) ------------------------------------
 * The pose-only g2o optimisation every tracking step and Tracking::Relocalization()
 * (Tracking.cpp:1284,1300,1315) run on the RANSAC pose: Levenberg-Marquardt of one VertexSE3Expmap
 * over EdgeSE3ProjectXYZOnlyPose (mvuRight < 0) and EdgeStereoSE3ProjectXYZOnlyPose (mvuRight >= 0,
 * Optimizer.cpp:252-323) edges with Huber kernels (delta sqrt(5.991) / sqrt(7.815)), 4 rounds of 10
 * iterations, each restarted from the entry pose, with chi2 > 5.991 / 7.815 outlier re-classification.
 * Parity against the reference is unpinned (g2o/Eigen cannot be built here). */
typedef struct {
    int32_t n;                /* pFrame->N keypoint slots */
    const uint8_t* has_mp;    /* [n] mvpMapPoints[i] != NULL (an edge is built); NULL = every slot */
    const float* uv;          /* [n][2] mvKeysUn[i].pt */
    const float* Xw;          /* [n][3] MapPoint::GetWorldPos() */
    const float* inv_sigma2;  /* [n] mvInvLevelSigma2[kpUn.octave] (information = I * invSigma2) */
    const float* u_right;     /* [n] mvuRight (>= 0: stereo observation), or NULL for a monocular Frame */
    float fx, fy, cx, cy;     /* Frame::fx,fy,cx,cy */
    float Tcw[16];            /* row-major pFrame->mTcw on entry */
    float bf;                 /* Frame::mbf (stereo baseline * fx; unused without stereo slots) */
} rsc_poseopt_problem;

typedef struct {
    int32_t n_good;        /* return value: nInitialCorrespondences - nBad (0 if < 3 edges) */
    int32_t n_initial;     /* nInitialCorrespondences */
    int32_t rounds;        /* outer rounds run (breaks after one when fewer than 10 edges) */
    int32_t lm_iterations; /* OptimizationAlgorithmLevenberg::solve calls */
    int32_t lm_trials;     /* linear solves (Levenberg trials) */
    float Tcw[16];         /* row-major pose after the call (pFrame->SetPose, Optimizer.cpp:420-421);
                              the entry pose when fewer than 3 edges (the reference returns early) */
} rsc_poseopt_result;

/* Optimizer::PoseOptimization on `count` Frames in one launch (one workgroup per Frame).
 * outlier[c] receives mvbOutlier for the slots with a map point (others untouched); may be NULL. */
int rsc_pose_optimization_many(rsc_context* ctx, const rsc_poseopt_problem* problems, int count,
                               rsc_poseopt_result* out, uint8_t* const* outlier);

/* ---- Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) ----------------------------------------
 * The loop-closure refinement LoopClosing::ComputeSim3 runs on every candidate whose Sim3 RANSAC
 * succeeded, right after SearchBySim3 (LoopClosing.cpp:309-311): g2o Levenberg-Marquardt of one
 * VertexSim3Expmap (_fix_scale) over EdgeSim3ProjectXYZ / EdgeInverseSim3ProjectXYZ pairs (numeric
 * Jacobians) with Huber kernels (delta = sqrt(th2)), optimize(5), outlier removal (chi2 > th2),
 * optimize(5 or 10).  Parity against the reference is unpinned (g2o/Eigen cannot be built here). */
typedef struct {
    int32_t n;               /* vpMatches1.size() = pKF1->N (KeyFrame 1 keypoint slots) */
    const uint8_t* valid;    /* [n] slot i is a correspondence: vpMatches1[i] and vpMapPoints1[i] set, neither
                                isBad(), vpMatches1[i]->GetIndexInKeyFrame(pKF2) >= 0 (Optimizer.cpp:1112-1143) */
    const float* X1w;        /* [n][3] vpMapPoints1[i]->GetWorldPos() */
    const float* X2w;        /* [n][3] vpMatches1[i]->GetWorldPos() */
    const float* uv1;        /* [n][2] pKF1->mvKeysUn[i].pt */
    const float* uv2;        /* [n][2] pKF2->mvKeysUn[i2].pt, i2 = GetIndexInKeyFrame(pKF2) */
    const float* inv1;       /* [n] pKF1->mvInvLevelSigma2[octave of i] */
    const float* inv2;       /* [n] pKF2->mvInvLevelSigma2[octave of i2] */
    float R1w[9], t1w[3];    /* pKF1->GetRotation(), GetTranslation() (row-major) */
    float R2w[9], t2w[3];    /* pKF2 */
    float K1[4], K2[4];      /* mK: fx, fy, cx, cy */
    double S[8];             /* g2oS12 on entry: quaternion (x, y, z, w), t, s */
    float th2;               /* 10 in LoopClosing.cpp:311 */
} rsc_sim3opt_problem;

typedef struct {
    int32_t n_inliers;          /* return value nIn (0 when nCorrespondences - nBad < 10) */
    int32_t n_correspondences;
    int32_t n_bad;              /* correspondences removed after the first optimize(5) */
    int32_t lm_iterations;      /* OptimizationAlgorithmLevenberg::solve calls */
    int32_t lm_trials;
    double S[8];                /* g2oS12 after the call (the entry value when n_inliers == 0) */
} rsc_sim3opt_result;

/* OptimizeSim3 on `count` KeyFrame pairs in one launch (one workgroup per pair).  keep[c] (may be
 * NULL) receives per slot 0 where vpMatches1[i] is set to NULL (an outlier), 1 elsewhere. */
int rsc_optimize_sim3_many(rsc_context* ctx, const rsc_sim3opt_problem* problems, int count,
                           rsc_sim3opt_result* out, uint8_t* const* keep);

/* ---- ORBmatcher::SearchByBoW (src/ORBmatcher.cpp:110-240, :354-488) -----------------------------
 * The producer of every RANSAC correspondence set: Hamming-256 matching of ORB descriptors that
 * share a DBoW2 FeatureVector node, with the nearest-neighbour ratio test and the rotation-histogram
 * consistency check.  Views (KeyFrames, the current Frame) are uploaded once and stay resident in
 * HBM; searches name them by handle.  Integer work: results are bit-exact with the reference. */
typedef struct {
    int32_t n;                 /* keypoints (KeyFrame::N / Frame::N), <= 8192 */
    const uint8_t* desc;       /* [n][32] mDescriptors rows (CV_8U, 32 columns) */
    const float* angle;        /* [n] keypoint angle: mvKeysUn[i].angle for a KeyFrame, mvKeys[i].angle for
                                  the Frame (the angles the two overloads read, ORBmatcher.cpp:185,435) */
    const uint8_t* valid;      /* [n] GetMapPointMatches()[i] != NULL && !isBad(); NULL = all.
                                  Unused for the Frame side of the Frame overload. */
    int32_t n_nodes;           /* mFeatVec.size() */
    const uint32_t* node_id;   /* [n_nodes] mFeatVec keys, strictly ascending (std::map order) */
    const int32_t* node_begin; /* [n_nodes + 1] CSR offsets into feat */
    const uint32_t* feat;      /* [node_begin[n_nodes]] each node's vector<unsigned int>, in order; every
                                  feature index < n and at most once overall (DBoW2 transform) */
} rsc_bow_features;

typedef struct rsc_bow rsc_bow;

/* Upload a view's descriptors, angles, map-point validity and FeatureVector (KeyFrame::mFeatVec /
 * Frame::mFeatVec after ComputeBoW) to HBM. */
int rsc_bow_create(rsc_context* ctx, const rsc_bow_features* features, rsc_bow** out);
void rsc_bow_destroy(rsc_bow* view);
/* Refresh the map-point validity of a resident view (map points culled or replaced since upload). */
int rsc_bow_set_valid(rsc_bow* view, const uint8_t* valid);

/* SearchByBoW(pKF = kfs[c], F = frame, vpMapPointMatches) for c < count in one launch (the
 * relocalization candidate loop, Tracking.cpp:1207-1232).  matches[c][i] (i < frame->n) = the
 * KeyFrame feature whose map point matched Frame feature i (vpMapPointMatches[i] =
 * kf.GetMapPointMatches()[matches[c][i]]), or -1; nmatches[c] = the return value. */
int rsc_search_by_bow_frame_many(rsc_context* ctx, rsc_bow* const* kfs, int count, const rsc_bow* frame,
                                 float nnratio, int check_orientation, int32_t* const* matches, int32_t* nmatches);
/* SearchByBoW(pKF1 = kf1, pKF2 = kf2s[c], vpMatches12) for c < count in one launch (the loop
 * candidate loop, LoopClosing.cpp:238-265).  matches12[c][i] (i < kf1->n) = the KF2 feature whose
 * map point vpMatches12[i] is, or -1; nmatches[c] = the return value. */
int rsc_search_by_bow_kf_many(rsc_context* ctx, const rsc_bow* kf1, rsc_bow* const* kf2s, int count,
                              float nnratio, int check_orientation, int32_t* const* matches12, int32_t* nmatches);

/* ---- ORBmatcher::SearchBySim3 (src/ORBmatcher.cpp:948-1170) ---------------------------------
 * The loop-closure matcher run after a Sim3 RANSAC success (LoopClosing.cpp:296-309): unmatched
 * MapPoints of each KeyFrame are projected into the other with (R12, t12), matched to the best
 * descriptor among the keypoints of the predicted pyramid levels inside th * scale of the projection
 * (KeyFrame::GetFeaturesInArea), and kept when both directions agree. */
typedef struct {
    int32_t n;                  /* KeyFrame::N */
    const float* kp;            /* [n][2] mvKeysUn[i].pt */
    const int32_t* octave;      /* [n] mvKeysUn[i].octave */
    const uint8_t* desc;        /* [n][32] mDescriptors */
    const int32_t* cell_begin;  /* [64*48 + 1] CSR over mGrid[ix][iy] (cell = ix * 48 + iy) */
    const int32_t* cell_feat;   /* mGrid contents, each cell's vector<size_t> in order */
    float min_x, max_x, min_y, max_y;  /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    float grid_w_inv, grid_h_inv;      /* mfGridElementWidthInv, mfGridElementHeightInv */
    float fx, fy, cx, cy;
    const float* scale_factors; /* [n_levels] mvScaleFactors */
    int32_t n_levels;           /* mnScaleLevels */
    float log_scale_factor;     /* mfLogScaleFactor */
    float Rcw[9], tcw[3];       /* GetRotation(), GetTranslation(), row-major */
    const uint8_t* mp_state;    /* [n] GetMapPointMatches()[i]: 0 = NULL, 1 = good, 2 = isBad() */
    const float* mp_pos;        /* [n][3] GetWorldPos() */
    const float* mp_dmax;       /* [n] mfMaxDistance */
    const float* mp_dmin;       /* [n] mfMinDistance */
    const uint8_t* mp_desc;     /* [n][32] MapPoint::GetDescriptor() */
} rsc_sim3_kf;

typedef struct rsc_kfview rsc_kfview;
/* Upload a KeyFrame's SearchBySim3 inputs (keypoints, grid, descriptors, pose, MapPoints) to HBM. */
int rsc_kfview_create(rsc_context* ctx, const rsc_sim3_kf* kf, rsc_kfview** out);
void rsc_kfview_destroy(rsc_kfview* view);

/* SearchBySim3(pKF1 = kf1[c], pKF2 = kf2[c], vpMatches12, R12[c], t12[c], th) for c < count in one
 * launch over resident views.  matched12[c][i1] (in, kf1[c] n entries): the KF2 keypoint index of
 * the MapPoint already in vpMatches12[i1] (GetIndexInKeyFrame(pKF2)), -1 for NULL, -2 for a
 * MapPoint not in KF2.  out12[c][i1]: the KF2 keypoint index of each new match
 * (vpMatches12[i1] = vpMapPoints2[idx2]), else -1; nfound[c] = the return value.
 * R12 [count][9] row-major, t12 [count][3]. */
int rsc_search_by_sim3_many(rsc_context* ctx, rsc_kfview* const* kf1, rsc_kfview* const* kf2, int count,
                            const float* R12, const float* t12, float th, const int32_t* const* matched12,
                            int32_t* const* out12, int32_t* nfound);

/* ---- KeyFrameDatabase: BoW candidate scoring (src/KeyFrameDatabase.cpp) ---------------------- */
/* A device-resident keyframe database: each KeyFrame is a slot in [0, capacity) holding its
 * BowVector (word ids ascending, TF-IDF values, DBoW2 L1_NORM scoring), its
 * GetBestCovisibilityKeyFrames(10) list and the per-KeyFrame query state of the reference
 * (mnLoopQuery/mnLoopWords/mLoopScore, mnRelocQuery/mnRelocWords/mRelocScore, KeyFrame.hpp:129-134),
 * which persists across queries exactly as the KeyFrame members do.  Replaces
 * KeyFrameDatabase (include/KeyFrameDatabase.hpp). */
typedef struct rsc_kfdb rsc_kfdb;
/* KeyFrameDatabase(voc) (KeyFrameDatabase.cpp:8-13): vocab_words = voc->size() (word ids are below
 * it; 10^6 for ORBvoc.txt), capacity slots, max_words (<= 4096) bounds one BowVector. */
int rsc_kfdb_create(rsc_context* ctx, uint32_t vocab_words, int capacity, int max_words, rsc_kfdb** out);
void rsc_kfdb_destroy(rsc_kfdb* db);
/* add(pKF) (:15-21): ids strictly ascending (a std::map BowVector) and below vocab_words; a slot
 * already present ->
 * RSC_ERR_UNSUPPORTED (the reference would list it twice per word). */
int rsc_kfdb_add(rsc_kfdb* db, int kf, int n_words, const uint32_t* word_id, const double* word_value);
/* erase(pKF) (:23-43); erasing an absent slot is a no-op as in the reference. */
int rsc_kfdb_erase(rsc_kfdb* db, int kf);
/* Frees slot kf for reuse by another KeyFrame (not a reference operation): erase + the slot's
 * query state and covisibility row reset to the fresh-KeyFrame values (KeyFrame.cpp:15).  The
 * facade calls it when a KeyFrame leaves the database. */
int rsc_kfdb_release(rsc_kfdb* db, int kf);
/* clear() (:45-49): empties the inverted file; the per-KeyFrame query state is kept. */
int rsc_kfdb_clear(rsc_kfdb* db);
/* pKF->GetBestCovisibilityKeyFrames(10) of slot kf (n <= 10 slots, in order). */
int rsc_kfdb_set_covisibility(rsc_kfdb* db, int kf, int n, const int32_t* best);
/* The same for count slots at once (kf[c], n[c] <= 10, best[c][10] row-major); only the span of
 * rows whose content changed is uploaded. */
int rsc_kfdb_set_covisibility_many(rsc_kfdb* db, int count, const int32_t* kf, const int32_t* n,
                                   const int32_t* best);
/* DetectRelocalizationCandidates(F) (:174-283): frame_id = F->mnId, (word_id, word_value) =
 * F->mBowVec.  candidates (room for 1 + the highest slot added or referenced so far; capacity
 * always suffices): the returned vector's slots in order.  Queries sweep only the slots in use. */
int rsc_kfdb_detect_relocalization(rsc_kfdb* db, uint64_t frame_id, int n_words, const uint32_t* word_id,
                                   const double* word_value, int32_t* candidates, int32_t* n_candidates);
/* DetectLoopCandidates(pKF, minScore) (:52-172): kf_id = pKF->mnId, connected =
 * pKF->GetConnectedKeyFrames() (slots). */
int rsc_kfdb_detect_loop(rsc_kfdb* db, uint64_t kf_id, int n_words, const uint32_t* word_id,
                         const double* word_value, int n_connected, const int32_t* connected, float min_score,
                         int32_t* candidates, int32_t* n_candidates);
/* Per-slot query state (parity hook): q[2] = {mnLoopQuery, mnRelocQuery}, w[2] = {mnLoopWords,
 * mnRelocWords}, s[2] = {mLoopScore, mRelocScore}. */
int rsc_kfdb_state(rsc_kfdb* db, int kf, uint64_t* q, int32_t* w, float* s);

/* Diagnostics below: `cap` = number of uint64 slots at `out`; RSC_ERR_ARG when it is smaller than
 * the layout (64*24, 64*8, 4096*4 and at most 64*96 words).
 * Diagnostic: wall-clock (100 MHz) phase stamps of the last PnP refine launch, [job < 64][24]:
 * entry, compaction, control points, MtM, eigen, betas, check, exit, then inside the eigen phase:
 * tridiagonal, Q accumulated, QR chase, eigenvectors, then [12 + 4w + j] inside the betas phase of
 * wave w: betas + Gauss-Newton, pc0 sum, M sum + Horn, error sum (zeros unless built with
 * RSC_REFINE_STAMPS=1). */
int rsc_diag_refine_phase_stamps(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic: wall-clock (100 MHz) phase stamps of the last PnP hypothesis solve, [3][wg < 4096][8]:
 * [0] eigen stage per workgroup (entry, sample + MtM, tridiagonal, Q, chase + store), [1] betas stage
 * per wave (entry, L + rho, find_betas, Gauss-Newton, row loads, R and t, hand-off; [7] = the
 * approximation | 256 * group), [2] inside find_betas' Jacobi SVD per betas wave (QR preconditioner,
 * U formed, sweeps done, then k = the SVD's columns) (zeros unless built with RSC_SOLVE_STAMPS=1;
 * cap >= 98304). */
int rsc_diag_solve_phase_stamps(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic wall-clock (100 MHz) stamps of mlpnp_quad_kernel's phases, [8192 workgroups][8]: entry,
 * sample, design + normal matrix, JacobiSVD, pose recovery, Gauss-Newton (zeros unless the library is
 * built with RSC_ML_STAMPS=1; tools/mlpnp_probe.py). cap >= 8192 * 8. */
int rsc_diag_mlpnp_phase_stamps(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic: wall-clock (100 MHz) ticks of the last PoseOptimization launch (built with
 * RSC_POSE_PHASES=1), [frame < 64][8]: fused passes (ticks), number of passes + (their active edges
 * << 24), re-classification, whole kernel, the LM solves, wave 1's slab phases (to the errors, to the
 * terms) and its slab count.  cap >= 64 * 24 returns [frame][24]: columns 8..15 = the HW_ID register
 * of waves 0..7 (SIMD in bits 5:4, CU in 11:8), 16 / 17 = wave 0's folding ticks and fold count. */
int rsc_diag_poseopt_phases(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic: wall-clock (100 MHz) ticks of the last OptimizeSim3 launch (built with RSC_SO_PHASES=1),
 * [pair < 64][8]: passes, pass count, perturbed-estimate builds, LM solves, wave 1's edge evaluation
 * and its slab count, wave 0's folds, whole kernel.  cap >= 64 * 8. */
int rsc_diag_sim3opt_phases(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic: wall clock (100 MHz) of KeyFrameDatabase slots 0..4095 in the last count launch,
 * [slot][4] = entry, staged, counted, exit (zeros unless built with RSC_KFDB_STAMPS=1). */
int rsc_diag_kfdb_stamps(rsc_context* ctx, uint64_t* out, int cap);
/* Diagnostic: wall-clock (100 MHz) phase stamps of the last SearchByBoW launch, [pair < 64][96]. */
int rsc_diag_bow_phase_stamps(rsc_context* ctx, uint64_t* out, int cap);

/* ---- glibc rand() helpers (Thirdparty/DBoW2/DUtils/Random.cpp:33-50) -------------------------- */
/* First n rand() outputs after srand(seed), produced with the device jump table (parity hook). */
int rsc_rand_stream(rsc_context* ctx, uint32_t seed, int n, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* RSC_H_ */
