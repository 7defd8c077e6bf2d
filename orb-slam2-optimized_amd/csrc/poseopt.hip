// poseopt.hip — Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) kernel: one 256-thread
// workgroup per Frame.  See rsc_poseopt.h for the mapping and the arithmetic contract.
//
// Where the time goes: every g2o reduction is a sequential sum over the active edges, and its
// dependent FP64 additions (~8 ns each) are the floor of a pass.  A pass is pipelined over slabs of
// kPoseSlab active edges: waves 1..3 compute the per-edge terms of slab k (error, robust chi2, the
// 27 H/b terms) into one of two LDS buffers while lanes 0..27 of wave 0 fold slab k-1 out of the
// other — all 28 columns on one wave instruction stream (b's terms are stored negated, so every lane
// runs the same additions: a - t == a + (-t) in IEEE arithmetic).  Only the active (level-0) edges
// are listed, in edge order, so the folds add exactly the reference's terms.
//
// The per-edge _error of a pass is not stored: re-classification needs only the last pass's errors
// of the level-0 edges, and recomputes them at that pass's estimate (po_error is a pure function of
// the estimate and the edge, so the values are the ones the pass computed).  Global stores in the
// slab loop would count in vmcnt with the next slab's prefetch loads and be waited for at every slab.
//
// Every pass is the fused computeActiveErrors + activeRobustChi2 + buildSystem at one estimate: the
// LM trial's chi2 pass (optimization_algorithm_levenberg.cpp:108-112) also builds the system at the
// trial estimate, which is the next iteration's buildSystem when the trial is accepted
// (solve() starts with computeActiveErrors/activeRobustChi2/buildSystem at that same estimate,
// lines 63-75); a rejected trial's system is dropped and the current one kept.  The chi2 that
// solve() recomputes at its start is therefore the chi2 of the pass that built the current system.
#include <hip/hip_runtime.h>
#include <atomic>
#include <cfloat>
#include "rsc_poseopt.h"
#include "rsc_kernels.h"
#include "rsc_fold.h"
#include "rsc_quad.h"  // split_wait (bounded hand-off waits, fault word)

namespace rsc {

namespace {

// Diagnostic phase clocks (rsc_diag_poseopt_phases) are compiled in only with RSC_POSE_PHASES=1:
// an outstanding s_memrealtime makes every LDS wait of the folds a full lgkmcnt(0).
#ifndef RSC_POSE_PHASES
#define RSC_POSE_PHASES 0
#endif
constexpr bool kPosePhases = RSC_POSE_PHASES;
// Timing diagnostics only (wrong results): 1 = the edge waves store placeholder terms instead of
// evaluating the edges (the pass is then the folds + barriers), 2 = wave 0 skips the folds (the pass
// is then the edge evaluation + barriers).  tools/Makefile povariant.
#ifndef RSC_PO_DIAG
#define RSC_PO_DIAG 0
#endif

// Pass form.
// RSC_PO_STREAM = 1: a streamed pass.  Wave 0 folds; RSC_PO_STREAM_WAVES edge waves take
// 64-edge chunks from an LDS counter (the next chunk's inputs loaded while the current one is
// evaluated), write a chunk's terms into its slab's slot of a two-slot ring (256 edges per slab) once
// the fold has released that slot, and count it in; the fold wave folds a slab as soon as its four
// chunks are in and releases the slot.  No workgroup barrier per slab: an edge wave that is ahead
// keeps evaluating, a slower one (the one beside the fold on SIMD 0) takes fewer chunks, and the
// fold never waits on the slowest wave of a tick.  Every wait is bounded (split_wait: on give-up
// the launch's fault word is raised and the host returns an error).  Measured no faster
// (profiles/r06/poseopt_probe_s6n/s6o/s6p.txt: 12.9-13.7 us per pass of 1,494 edges against 13.0 for
// the ticked form): the fold waits 4.7 us per pass, 2 of them for the first slab, while the edge
// waves wait 3 us for free slots — a two-slot ring behind per-wave queues of three chunks blocks at
// the head of the line; kept as an option (its parity tests pass, gpu_tests_lm_s6n.txt).
// RSC_PO_STREAM = 0 (default): barrier-ticked slabs — RSC_PO_WIDE = 0: RSC_PO_EDGE_WAVES (3 or 4) edge waves,
// double-buffered slabs of 64 x that; RSC_PO_WIDE = 1: 512 threads, seven edge waves (RSC_PO_IDLE = w
// leaves wave w out), slabs of 448 into a single buffer, a slab's terms held in VGPRs until the
// previous slab's fold is done.  Measured (profiles/r06/poseopt_probe_s6l.txt, s6m): the edge
// evaluation is issue-bound (about 380 VALU instructions per edge); per pass of 1,494 edges 13.7 us
// with 3 edge waves, 12.9 with 4, 14.1 wide (448), 14.4 wide with an idle wave.
#ifndef RSC_PO_STREAM
#define RSC_PO_STREAM 0
#endif
#ifndef RSC_PO_STREAM_WAVES
#define RSC_PO_STREAM_WAVES 7
#endif
#ifndef RSC_PO_WIDE
#define RSC_PO_WIDE 0
#endif
#ifndef RSC_PO_EDGE_WAVES
#define RSC_PO_EDGE_WAVES 4
#endif
constexpr bool kPoseStream = RSC_PO_STREAM != 0;
// the LM trials' LDLT with one matrix row per lane (rsc_poseopt.h po_ldlt_solve_lanes): measured
// slower than the scalar form (profiles/r06/poseopt_probe_s6t.txt: 118 vs 107 us of LDLT per stereo
// Frame; sim3opt_probe_s6t.txt: 47.8 vs 42.7 us of LM solves per pair) — the factorization is a
// latency chain and the lane form adds a v_readlane round trip to every link; off
#ifndef RSC_LM_LDLT_LANES
#define RSC_LM_LDLT_LANES 0
#endif
constexpr bool kLdltLanes = RSC_LM_LDLT_LANES != 0;
constexpr bool kPoseWide = !kPoseStream && RSC_PO_WIDE != 0;
// the wide form's idle wave (0: none): waves w and w + 4 of a workgroup land on one SIMD
// (profiles/r06/poseopt_probe_s6j.txt), so wave 4 shares the fold wave's SIMD
#ifndef RSC_PO_IDLE
#define RSC_PO_IDLE 0
#endif
static_assert(RSC_PO_IDLE >= 0 && RSC_PO_IDLE <= 7, "idle wave");
static_assert(RSC_PO_EDGE_WAVES == 3 || RSC_PO_EDGE_WAVES == 4, "edge waves of the ticked form");
static_assert(RSC_PO_STREAM_WAVES >= 1 && RSC_PO_STREAM_WAVES <= 7, "edge waves of the streamed form");
constexpr int kPoseEdgeWaves =
    kPoseStream ? RSC_PO_STREAM_WAVES : (kPoseWide ? (RSC_PO_IDLE ? 6 : 7) : RSC_PO_EDGE_WAVES);
constexpr int kPoseThreads = kPoseWide ? 512 : 64 * (1 + kPoseEdgeWaves);
constexpr int kPoseChunks = 4;  // 64-edge chunks per slab of the streamed form
constexpr int kPoseFoldLanes = 64;                // wave 0 folds
constexpr int kPoseSlab = kPoseStream ? 64 * kPoseChunks : 64 * kPoseEdgeWaves;  // active edges per slab
constexpr int kPoseBufs = kPoseWide ? 1 : 2;
constexpr int kPoseCol = kPoseSlab + 2;           // padded column stride (doubles): 16 B bank shift per column
constexpr int kPoseCols = kPoseTerms + 1;         // 27 H/b columns + the chi2 column
constexpr int kPoseBuf = kPoseCols * kPoseCol;    // one slab buffer
constexpr size_t kPoseLds =
    sizeof(double) * kPoseBufs * kPoseBuf + sizeof(uint16_t) * kPoseMaxEdges + kPoseMaxEdges;
static_assert(kPoseCol % 2 == 0, "fold_run reads 16-byte aligned columns");
static_assert(kPoseSlab % 16 == 0, "fold_fixed folds whole 16-term groups");
static_assert(kPoseMaxEdges <= 65536, "active list is uint16");
static_assert(kPoseLds <= 160 * 1024 - 1024, "LDS");

// Slab position of this thread's edge (-1: the fold wave, and the idle wave of the wide form).
__device__ __forceinline__ int po_slot(int tid) {
    const int w = tid >> 6, lane = tid & 63;
    if constexpr (kPoseWide && RSC_PO_IDLE != 0)
        return (w == 0 || w == RSC_PO_IDLE) ? -1 : (w - (w > RSC_PO_IDLE ? 2 : 1)) * 64 + lane;
    else if constexpr (kPoseWide) return w == 0 ? -1 : (w - 1) * 64 + lane;
    else return tid - kPoseFoldLanes;
}

struct PoseLds {
    double* terms;   // [kPoseBufs][kPoseCols][kPoseCol] slab buffers
    uint16_t* list;  // [kPoseMaxEdges] active edges of the round, in edge order
    uint8_t* lvl;    // [kPoseMaxEdges] edge level: 0 active, 1 outlier (g2o setLevel)
    double* red;     // [32] a pass's folded sums (H lower triangle row-major, b, chi2)
    double* cur;     // [32] the LM's current system (a copy of an adopted pass's red)
    int* scan;       // [kPoseThreads / 64] wave totals
    int* nbad;
    int* ctl;        // streamed pass: [0] next chunk, [1 + s] chunks stored in slot s, [3] slabs folded,
                     // [4] a wait gave up
};

// The problem's arrays as global-address-space pointers: accessed through them the compiler issues
// global (not flat) loads and stores, and a pending flat access would make every LDS wait of the
// folds a full lgkmcnt(0) (flat may complete out of order with the LDS reads).
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* po_g(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
// HIP's vector structs do not copy out of address space 1: the vector accesses go through the
// native vector types
__device__ __forceinline__ float4 po_ld(const float4* p, int e) {
    using V = float __attribute__((ext_vector_type(4)));
    const V v = po_g(reinterpret_cast<const V*>(p))[e];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 po_ld(const float2* p, int e) {
    using V = float __attribute__((ext_vector_type(2)));
    const V v = po_g(reinterpret_cast<const V*>(p))[e];
    return make_float2(v.x, v.y);
}
__device__ __forceinline__ double2 po_ld(const double2* p, int e) {
    using V = double __attribute__((ext_vector_type(2)));
    const V v = po_g(reinterpret_cast<const V*>(p))[e];
    return make_double2(v.x, v.y);
}

// An estimate in LDS (quaternion x, y, z, w, then t).
__device__ __forceinline__ void po_put(double* d, const PoSE3& e) {
    d[0] = e.r.x; d[1] = e.r.y; d[2] = e.r.z; d[3] = e.r.w;
    d[4] = e.t[0]; d[5] = e.t[1]; d[6] = e.t[2];
}
__device__ __forceinline__ PoSE3 po_get(const double* d) {
    PoSE3 e;
    e.r.x = d[0]; e.r.y = d[1]; e.r.z = d[2]; e.r.w = d[3];
    e.t[0] = d[4]; e.t[1] = d[5]; e.t[2] = d[6];
    return e;
}

// Huber kernels of the two edge types (Optimizer.cpp:240-241: float deltas, setDelta(double)).
struct PoKernels {
    double dm, dm2, ds, ds2;
};

__device__ __forceinline__ bool po_is_stereo(const DevPoseProb& P, int e) { return P.ur && po_g(P.ur)[e] >= 0.0f; }

// Error of edge e at `est` (computeError of its edge type).
__device__ __forceinline__ double3 po_edge_error(const DevPoseProb& P, int e, const PoSE3& est, const PoCam& K) {
    const float4 xw = po_ld(P.xw, e);
    const float2 uv = po_ld(P.uv, e);
    const bool st = po_is_stereo(P, e);
    const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
    double e0, e1, e2;
    po_error(est, K, X, (double)uv.x, (double)uv.y, st ? (double)po_g(P.ur)[e] : 0.0, st, e0, e1, e2);
    return make_double3(e0, e1, e2);
}

// Inputs of one edge, loaded a slab ahead of their use in a pass.
struct PoEdgeIn {
    float4 xw;
    float2 uv;
    float ur;  // mvuRight, < 0 for a monocular edge
    int e;
};

__device__ __forceinline__ PoEdgeIn po_load(const DevPoseProb& P, int e) {
    PoEdgeIn in;
    in.e = e;
    in.xw = po_ld(P.xw, e);
    in.uv = po_ld(P.uv, e);
    in.ur = P.ur ? po_g(P.ur)[e] : -1.0f;
    return in;
}

// The level-0 edges in edge order (SparseOptimizer::initializeOptimization(0) keeps the edges of
// level 0 in the order they were added, sparse_optimizer.cpp:174-182); returns their count.
__device__ int po_list_active(const PoseLds& S, int n) {
    // tid laundered: the scan's shuffle addresses are recomputed per call instead of being hoisted
    // out of the round loop and held (spilled) across the passes
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6;
    const int per = (n + kPoseThreads - 1) / kPoseThreads;
    const int lo = min(n, tid * per), hi = min(n, lo + per);
    int c = 0;
    for (int e = lo; e < hi; ++e) c += (S.lvl[e] == 0);
    int inc = c;  // inclusive wave scan
    RSC_UNROLL for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) S.scan[w] = inc;
    __syncthreads();
    int pos = inc - c, total = 0;
    RSC_UNROLL for (int q = 0; q < kPoseThreads / 64; ++q) {
        const int t = S.scan[q];
        if (q < w) pos += t;
        total += t;
    }
    for (int e = lo; e < hi; ++e)
        if (S.lvl[e] == 0) S.list[pos++] = (uint16_t)e;
    __syncthreads();
    return total;
}

// The first slab's inputs of this lane (edge list position po_slot), kept in registers
// for the round's passes: a pass then starts on its first slab without a load round trip.
__device__ __forceinline__ PoEdgeIn po_first(const DevPoseProb& P, const PoseLds& S, int m) {
    const int j = po_slot(threadIdx.x);
    PoEdgeIn f{};
    if (j >= 0 && j < m) f = po_load(P, S.list[j]);
    return f;
}

// The streamed pass's first two chunks of edge wave w (chunks w - 1 and w - 1 + E, E edge waves),
// loaded once per round and kept in VGPRs: a pass starts evaluating at once instead of after a
// global-load round trip (measured 3.1 us from pass start to the first slab when they were loaded
// per pass, profiles/r06/poseopt_probe_s6o.txt).
struct PoFirst2 {
    PoEdgeIn a, b;
};
__device__ __forceinline__ PoEdgeIn po_chunk_load(const DevPoseProb& P, const PoseLds& S, int m, int c) {
    const int lane = threadIdx.x & 63;
    const int pos = (c / kPoseChunks) * kPoseSlab + (c % kPoseChunks) * 64 + lane;
    PoEdgeIn in{};
    if (pos < m) in = po_load(P, S.list[pos]);
    return in;
}
__device__ __forceinline__ PoFirst2 po_first_stream(const DevPoseProb& P, const PoseLds& S, int m) {
    const int w = threadIdx.x >> 6;
    PoFirst2 f{};
    if (w > 0) {
        f.a = po_chunk_load(P, S, m, w - 1);
        f.b = po_chunk_load(P, S, m, w - 1 + kPoseEdgeWaves);
    }
    return f;
}

// One pass at `est` over the m active edges: computeActiveErrors, activeRobustChi2
// (sparse_optimizer.cpp:61-114) and BlockSolver::buildSystem (block_solver.hpp:502-560: H lower
// triangle added, b subtracted, both from 0.0), every sum folded in edge order; the folded sums are
// left in S.red (returns chi2).  `first` = the inputs of the lane's edge in the first slab, loaded
// once per round (po_first).
__device__ double po_pass(const DevPoseProb& P, const PoseLds& S, int m, const PoEdgeIn& first, const PoSE3& est,
                          const PoCam& K, bool robust, const PoKernels& hk, uint64_t (&ps)[9]) {
    const int tid = threadIdx.x;
    const int nslab = (m + kPoseSlab - 1) / kPoseSlab;
    const int j = po_slot(tid);
    PoEdgeIn nx = first;
    double acc = 0.0;
    for (int k = 0; k <= nslab; ++k) {
        double t[kPoseTerms], tc = 0.0;
        const int pos = k * kPoseSlab + j;
        if (j >= 0 && k < nslab) {
            if (pos < m) {
                // phase clocks of wave 1 (lane 0): [0] slab start -> error, [1] error -> terms
                const bool pclk = kPosePhases && tid == kPoseFoldLanes;
                uint64_t c0 = pclk ? wall_clock64() : 0;
                const PoEdgeIn in = nx;
                if (pos + kPoseSlab < m) nx = po_load(P, S.list[pos + kPoseSlab]);
                const bool st = in.ur >= 0.0f;
                const double X[3] = {(double)in.xw.x, (double)in.xw.y, (double)in.xw.z};
                if constexpr (RSC_PO_DIAG == 1) {
                    RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) t[q] = X[q % 3] * 1e-30;
                    tc = X[0] * 1e-30;
                } else {
                    double e0, e1, e2;
                    po_error(est, K, X, (double)in.uv.x, (double)in.uv.y, st ? (double)in.ur : 0.0, st, e0, e1, e2);
                    if (pclk) {
                        __builtin_amdgcn_sched_barrier(0);
                        const uint64_t c1 = wall_clock64() + (uint64_t)(e0 != e0) + (uint64_t)(e2 != e2);
                        ps[0] += c1 - c0;
                        c0 = c1;
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    const double delta = st ? hk.ds : hk.dm, dsqr = st ? hk.ds2 : hk.dm2;
                    // the zero-product-free form, and the full one for an edge outside its precondition
                    if (!po_quad_terms_finite(est, K, X, (double)in.xw.w, e0, e1, e2, st, robust, delta, dsqr, t))
                        po_quad_terms(est, K, X, (double)in.xw.w, e0, e1, e2, st, robust, delta, dsqr, t);
                    tc = po_chi_term(robust, st, (double)in.xw.w, e0, e1, e2, delta, dsqr);
                }
                RSC_UNROLL for (int q = 21; q < kPoseTerms; ++q) t[q] = -t[q];
                if (pclk) {
                    __builtin_amdgcn_sched_barrier(0);
                    ps[1] += wall_clock64() - c0 + (uint64_t)(t[0] != t[0]);
                    ps[2] += 1;
                }
            } else {
                // padding of the last slab: +0.0 terms are exact identities of these folds (an
                // accumulator that starts at +0.0 never becomes -0.0 under round-to-nearest)
                RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) t[q] = 0.0;
            }
            if constexpr (!kPoseWide) {
                double* buf = S.terms + (k & 1) * kPoseBuf + j;
                RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) buf[q * kPoseCol] = t[q];
                buf[kPoseTerms * kPoseCol] = tc;
            }
        } else if (tid < kPoseCols && k > 0) {
            // fold clocks of lane 0: [3] folding, [4] folds
            const bool fclk = kPosePhases && tid == 0;
            const uint64_t f0 = fclk ? wall_clock64() : 0;
            if constexpr (RSC_PO_DIAG != 2)
                acc = fold_fixed<kPoseSlab>(acc, S.terms + (kPoseWide ? 0 : ((k - 1) & 1) * kPoseBuf) + tid * kPoseCol);
            if (fclk) {
                __builtin_amdgcn_sched_barrier(0);
                ps[3] += wall_clock64() - f0 + (uint64_t)(acc != acc);
                ps[4] += 1;
            }
        }
        __syncthreads();
        if constexpr (kPoseWide) {
            // the fold of slab k - 1 is done: slab k's terms go into the buffer
            if (k < nslab) {
                if (j >= 0) {
                    double* buf = S.terms + j;
                    RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) buf[q * kPoseCol] = t[q];
                    buf[kPoseTerms * kPoseCol] = tc;
                }
                __syncthreads();
            }
        }
    }
    if (tid < kPoseCols) S.red[tid] = acc;
    __syncthreads();
    return S.red[kPoseTerms];
    // S.red is next written after the next pass's slab barriers, by which time every thread has read it
}

// The streamed pass (RSC_PO_STREAM): the same sums as po_pass, folded in the same edge order (a
// slab's chunks land at their edge positions, so fold_fixed reads exactly po_pass's columns).
__device__ double po_pass_stream(const DevPoseProb& P, const PoseLds& S, int m, const PoFirst2& first,
                                 const PoSE3& est, const PoCam& K, bool robust, const PoKernels& hk, unsigned* fault,
                                 uint64_t (&ps)[9]) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nslab = (m + kPoseSlab - 1) / kPoseSlab;
    const int nchunks = nslab * kPoseChunks;
    int* const ctl = S.ctl;
    if (tid < 5) ctl[tid] = tid == 0 ? 2 * kPoseEdgeWaves : 0;  // chunks 0 .. 2E - 1 are dealt statically
    __syncthreads();
    // a wait that gives up raises the fault word and ctl[4]: every later wait of the launch's
    // workgroup returns at once, so a broken hand-off ends the kernel after one time-out per wave
    auto wait_for = [ctl, fault](int* flag, int need) {
        if (__hip_atomic_load(ctl + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return;
        const int v = split_wait(flag, fault, [need](int x) { return x >= need; });
        if (v < need) __hip_atomic_store(ctl + 4, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    double acc = 0.0;
    if (w == 0) {
        const bool fclk = kPosePhases && tid == 0;
        const uint64_t p0 = fclk ? wall_clock64() : 0;
        for (int k = 0; k < nslab; ++k) {
            const uint64_t wt0 = fclk ? wall_clock64() : 0;
            wait_for(ctl + 1 + (k & 1), kPoseChunks * ((k >> 1) + 1));  // slot k & 1 holds slab k
            const uint64_t f0 = fclk ? wall_clock64() : 0;
            if (fclk) {  // [5] the fold's waits, [7] pass start -> first slab in
                ps[5] += f0 - wt0;
                if (k == 0) ps[7] += f0 - p0;
            }
            if (lane < kPoseCols) {
                if constexpr (RSC_PO_DIAG != 2) acc = fold_fixed<kPoseSlab>(acc, S.terms + (k & 1) * kPoseBuf + lane * kPoseCol);
            }
            if (fclk) {
                __builtin_amdgcn_sched_barrier(0);
                ps[3] += wall_clock64() - f0 + (uint64_t)(acc != acc);
                ps[4] += 1;
            }
            // the slot's reads are complete (release): slab k + 2 may overwrite it
            if (lane == 0) __hip_atomic_store(ctl + 3, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
        auto grab = [&]() {
            int c = 0;
            if (lane == 0) c = __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return __builtin_amdgcn_readfirstlane(c);
        };
        auto edge_pos = [&](int c) { return (c / kPoseChunks) * kPoseSlab + (c % kPoseChunks) * 64 + lane; };
        // the wave's chunks in increasing order: two dealt statically (inputs in VGPRs since the round
        // began), then grabbed ones, each loaded two chunks ahead of its evaluation
        int c = w - 1, cn = w - 1 + kPoseEdgeWaves;
        PoEdgeIn in_c = first.a, in_n = first.b;
        while (c < nchunks) {
            const int cnn = grab();
            PoEdgeIn in_nn{};
            if (cnn < nchunks) in_nn = po_chunk_load(P, S, m, cnn);
            const PoEdgeIn in = in_c;
            in_c = in_n;
            in_n = in_nn;
            const int k = c / kPoseChunks, pos = edge_pos(c);
            // phase clocks of wave 1 (lane 0): [0] chunk start -> error, [1] error -> terms
            const bool pclk = kPosePhases && tid == kPoseFoldLanes;
            uint64_t c0 = pclk ? wall_clock64() : 0;
            double t[kPoseTerms], tc = 0.0;
            if (pos < m) {
                const bool st = in.ur >= 0.0f;
                const double X[3] = {(double)in.xw.x, (double)in.xw.y, (double)in.xw.z};
                if constexpr (RSC_PO_DIAG == 1) {
                    RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) t[q] = X[q % 3] * 1e-30;
                    tc = X[0] * 1e-30;
                } else {
                    double e0, e1, e2;
                    po_error(est, K, X, (double)in.uv.x, (double)in.uv.y, st ? (double)in.ur : 0.0, st, e0, e1, e2);
                    if (pclk) {
                        __builtin_amdgcn_sched_barrier(0);
                        const uint64_t c1 = wall_clock64() + (uint64_t)(e0 != e0) + (uint64_t)(e2 != e2);
                        ps[0] += c1 - c0;
                        c0 = c1;
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    const double delta = st ? hk.ds : hk.dm, dsqr = st ? hk.ds2 : hk.dm2;
                    if (!po_quad_terms_finite(est, K, X, (double)in.xw.w, e0, e1, e2, st, robust, delta, dsqr, t))
                        po_quad_terms(est, K, X, (double)in.xw.w, e0, e1, e2, st, robust, delta, dsqr, t);
                    tc = po_chi_term(robust, st, (double)in.xw.w, e0, e1, e2, delta, dsqr);
                }
                RSC_UNROLL for (int q = 21; q < kPoseTerms; ++q) t[q] = -t[q];
            } else {
                // padding of the last slab: +0.0 terms are exact identities of these folds
                RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) t[q] = 0.0;
            }
            if (pclk) {
                __builtin_amdgcn_sched_barrier(0);
                ps[1] += wall_clock64() - c0 + (uint64_t)(t[0] != t[0]);
                ps[2] += 1;
            }
            // slot k & 1 held slab k - 2: it is free once the fold has passed slab k - 2
            const uint64_t ws = pclk ? wall_clock64() : 0;
            wait_for(ctl + 3, k - 1);
            if (pclk) ps[6] += wall_clock64() - ws;  // [6] wave 1's slot waits
            double* buf = S.terms + (k & 1) * kPoseBuf + (c % kPoseChunks) * 64 + lane;
            RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) buf[q * kPoseCol] = t[q];
            buf[kPoseTerms * kPoseCol] = tc;
            // count the chunk in (release: the wave's stores above complete first)
            if (lane == 0) __hip_atomic_fetch_add(ctl + 1 + (k & 1), 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            c = cn;
            cn = cnn;
        }
    }
    if (tid < kPoseCols) S.red[tid] = acc;
    __syncthreads();
    return S.red[kPoseTerms];
}

// S.cur = S.red (the LM adopts the last pass's system); every thread reads S.cur after the barrier.
__device__ __forceinline__ void po_adopt(const PoseLds& S) {
    if (threadIdx.x < kPoseCols) S.cur[threadIdx.x] = S.red[threadIdx.x];
    __syncthreads();
}

}  // namespace

// Diagnostic phase clock (wall clock, 100 MHz ticks) of the last launch, frames 0..63: [0] passes,
// [1] number of passes + (sum of their active edges << 24), [2] re-classification, [3] whole kernel
// (thread 0); [4] the LM trials' solve (LDLT + exp + product, thread 0); [5] / [6] wave 1's slab time
// up to the edges' errors / from there to the terms stored, [7] its slab count; [8 + w] the HW_ID
// register of wave w (which SIMD each wave of the workgroup landed on); [16] / [17] wave 0's folding
// time and fold count; [18] the LDLT part of [4]; streamed pass: [19] the fold wave's waits for
// chunks, [20] wave 1's waits for a free slot, [21] pass start to the first slab in.
__device__ uint64_t g_po_phase[64][24];

__global__ __launch_bounds__(kPoseThreads) void poseopt_kernel(const DevPoseProb* __restrict__ probs, unsigned* fault) {
    extern __shared__ __attribute__((aligned(16))) double po_lds[];
    __shared__ double red_sh[32], cur_sh[32];
    __shared__ int scan_sh[kPoseThreads / 64];
    __shared__ int nbad_sh;
    __shared__ int ctl_sh[5];
    const PoseLds S{po_lds, reinterpret_cast<uint16_t*>(po_lds + kPoseBufs * kPoseBuf),
                    reinterpret_cast<uint8_t*>(po_lds + kPoseBufs * kPoseBuf) + sizeof(uint16_t) * kPoseMaxEdges,
                    red_sh, cur_sh, scan_sh, &nbad_sh, ctl_sh};
    const DevPoseProb& P = probs[blockIdx.x];
    const int tid = threadIdx.x, n = P.n;
    const PoCam K{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy, (double)P.bf};
    const float deltaMono = sqrt(5.991);    // Optimizer.cpp:240
    const float deltaStereo = sqrt(7.815);  // Optimizer.cpp:241
    PoKernels hk;                           // RobustKernelHuber::setDelta
    hk.dm = deltaMono;
    hk.dm2 = hk.dm * hk.dm;
    hk.ds = deltaStereo;
    hk.ds2 = hk.ds * hk.ds;
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    double R0[3][3], t0[3];
    RSC_UNROLL for (int r = 0; r < 3; ++r) {
        RSC_UNROLL for (int c = 0; c < 3; ++c) R0[r][c] = (double)P.T[4 * r + c];
        t0[r] = (double)P.T[4 * r + 3];
    }
    // Converter::toSE3Quat (rotation() = linear(), Q14), parked in LDS and read back per round rather
    // than held in VGPRs across the passes (read after the barrier below)
    __shared__ double init_sh[8];
    if (tid == 0) po_put(init_sh, po_from_Rt(R0, t0));
    auto init = [&]() { return po_get(init_sh); };
    const bool clk = kPosePhases && blockIdx.x < 64 && tid == 0;
    uint64_t ph_pass = 0, n_pass = 0, ph_cls = 0, ph_solve = 0, ph_ldlt = 0, t_start = clk ? wall_clock64() : 0;
    uint64_t ps[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // wave 1's slab and wave 0's fold clocks (po_pass)
    for (int e = tid; e < n; e += kPoseThreads) {
        S.lvl[e] = 0;
        po_g(P.outlier)[e] = 0;
    }
    if (tid == 0) *S.nbad = 0;
    if (kPosePhases && blockIdx.x < 64 && (tid & 63) == 0) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        g_po_phase[blockIdx.x][8 + (tid >> 6)] = hw;
    }
    __syncthreads();

    double x[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // BlockSolver::_x persists across rounds
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, rounds = 0, lm_its = 0, lm_trials = 0, nBad = 0;
    bool robust = true;
    PoSE3 est = init();
    // the estimate of the round's last pass (the level-0 edges' _error is evaluated there), in LDS
    __shared__ double last_sh[8];
    for (int it = 0; it < 4; ++it) {
        rounds++;
        est = init();
        if (tid == 0) po_put(last_sh, est);  // read after the round's barriers
        const int m = po_list_active(S, n);
        if (m > 0) {
            const PoEdgeIn first = kPoseStream ? PoEdgeIn{} : po_first(P, S, m);
            const PoFirst2 first2 = kPoseStream ? po_first_stream(P, S, m) : PoFirst2{};
            // the system at est (S.cur) and the chi2 solve() computes there
            uint64_t tp = clk ? wall_clock64() : 0;
            double chiEst = kPoseStream ? po_pass_stream(P, S, m, first2, est, K, robust, hk, fault, ps)
                                        : po_pass(P, S, m, first, est, K, robust, hk, ps);
            if (clk) { ph_pass += wall_clock64() - tp; n_pass += 1 + ((uint64_t)m << 24); }
            po_adopt(S);
            bool ok = true;
            for (int i = 0; i < 10 && ok; ++i) {
                lm_its++;
                double currentChi = chiEst;
                const double iniChi = currentChi;
                if (i == 0) {
                    double maxDiagonal = 0.;
                    RSC_UNROLL for (int j = 0; j < 6; ++j) {  // std::max(fabs(H(j,j)), maxDiagonal)
                        const double a = rabs(S.cur[j * (j + 1) / 2 + j]);
                        maxDiagonal = (a < maxDiagonal) ? maxDiagonal : a;
                    }
                    lambda = 1e-5 * maxDiagonal;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    lm_trials++;
                    const uint64_t ts = clk ? wall_clock64() : 0;
                    double b[6], xs[6];
                    RSC_UNROLL for (int r = 0; r < 6; ++r) b[r] = S.cur[21 + r];
                    bool ok2;
                    if constexpr (kLdltLanes) {
                        // this lane's row of H + lambda I (rows 0..5 on lanes 0..5)
                        const int lr = min((int)(tid & 63), 5);
                        double row[6];
                        RSC_UNROLL for (int c = 0; c < 6; ++c)
                            row[c] = lr >= c ? S.cur[lr * (lr + 1) / 2 + c] : S.cur[c * (c + 1) / 2 + lr];
                        RSC_UNROLL for (int c = 0; c < 6; ++c) row[c] = (c == lr) ? row[c] + lambda : row[c];
                        ok2 = po_ldlt_solve_lanes<6>(row, b, xs);
                    } else {
                        double Hd[6][6];
                        RSC_UNROLL for (int r = 0; r < 6; ++r)
                            RSC_UNROLL for (int c = 0; c < 6; ++c)
                                Hd[r][c] = r >= c ? S.cur[r * (r + 1) / 2 + c] : S.cur[c * (c + 1) / 2 + r];
                        RSC_UNROLL for (int r = 0; r < 6; ++r) Hd[r][r] += lambda;
                        ok2 = po_ldlt_solve6(Hd, b, xs);
                    }
                    if (ok2) RSC_UNROLL for (int j = 0; j < 6; ++j) x[j] = xs[j];
                    if (clk) {
                        __builtin_amdgcn_sched_barrier(0);
                        ph_ldlt += wall_clock64() - ts + (uint64_t)(x[0] != x[0]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    const PoSE3 trial = po_mul(po_exp(x), est);
                    tp = clk ? wall_clock64() + (uint64_t)(trial.t[0] != trial.t[0]) : 0;
                    if (clk) ph_solve += tp - ts;
                    const double chiT = kPoseStream ? po_pass_stream(P, S, m, first2, trial, K, robust, hk, fault, ps)
                                                    : po_pass(P, S, m, first, trial, K, robust, hk, ps);
                    if (tid == 0) po_put(last_sh, trial);  // read after this pass's barriers
                    if (clk) { ph_pass += wall_clock64() - tp; n_pass += 1 + ((uint64_t)m << 24); }
                    const double tempChi = ok2 ? chiT : DBL_MAX;
                    rho = (currentChi - tempChi);
                    double scale = 0.;
                    RSC_UNROLL for (int j = 0; j < 6; ++j) scale += x[j] * (lambda * x[j] + b[j]);
                    scale += 1e-3;
                    rho /= scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - po_cube(2 * rho - 1);
                        alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;              // std::min(alpha, 2/3)
                        const double scaleFactor = (1. / 3. < alpha) ? alpha : 1. / 3.;  // std::max(1/3, alpha)
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                        est = trial;
                        po_adopt(S);  // the trial's system (a uniform branch: every thread decides alike)
                        chiEst = chiT;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                if (qmax == 10 || rho == 0) {
                    ok = false;
                } else {
                    if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                    else nBadLM = 0;
                    ok = nBadLM < 3;
                }
            }
        }
        // re-classification (Optimizer.cpp:347-398; mono and stereo loops are per-edge decisions);
        // the level-0 edges keep the _error of the last pass (g2o's last computeActiveErrors)
        const uint64_t tr0 = clk ? wall_clock64() : 0;
        int cnt = 0;
        for (int e = tid; e < n; e += kPoseThreads) {
            const double3 er = po_edge_error(P, e, S.lvl[e] ? est : po_get(last_sh), K);
            const bool st = po_is_stereo(P, e);
            const float c2 = (float)po_chi2((double)po_ld(P.xw, e).w, st, er.x, er.y, er.z);
            const bool bad = c2 > (st ? chi2Stereo : chi2Mono);
            S.lvl[e] = bad ? 1 : 0;
            po_g(P.outlier)[e] = bad ? 1 : 0;
            cnt += bad;
        }
        if (cnt) atomicAdd(S.nbad, cnt);
        __syncthreads();
        nBad = *S.nbad;
        __syncthreads();
        if (tid == 0) *S.nbad = 0;
        if (clk) ph_cls += wall_clock64() - tr0;
        if (it == 2) robust = false;
        if (n < 10) break;
    }
    if (tid == 0) {
        double R[3][3];
        po_quat_to_R(est.r, R);
        RSC_UNROLL for (int r = 0; r < 3; ++r) {
            RSC_UNROLL for (int c = 0; c < 3; ++c) po_g(P.out)[4 * r + c] = (float)R[r][c];
            po_g(P.out)[4 * r + 3] = (float)est.t[r];
        }
        po_g(P.out)[12] = __int_as_float(n - nBad);
        po_g(P.out)[13] = __int_as_float(rounds);
        po_g(P.out)[14] = __int_as_float(lm_its);
        po_g(P.out)[15] = __int_as_float(lm_trials);
    }
    if (clk) {
        g_po_phase[blockIdx.x][0] = ph_pass;
        g_po_phase[blockIdx.x][1] = n_pass;
        g_po_phase[blockIdx.x][2] = ph_cls;
        g_po_phase[blockIdx.x][3] = wall_clock64() - t_start;
        g_po_phase[blockIdx.x][4] = ph_solve;
        g_po_phase[blockIdx.x][16] = ps[3];
        g_po_phase[blockIdx.x][17] = ps[4];
        g_po_phase[blockIdx.x][18] = ph_ldlt;
        g_po_phase[blockIdx.x][19] = ps[5];
        g_po_phase[blockIdx.x][21] = ps[7];
    }
    if (kPosePhases && blockIdx.x < 64 && tid == kPoseFoldLanes) {
        g_po_phase[blockIdx.x][5] = ps[0];
        g_po_phase[blockIdx.x][6] = ps[1];
        g_po_phase[blockIdx.x][7] = ps[2];
        g_po_phase[blockIdx.x][20] = ps[6];
    }
}

hipError_t read_poseopt_phases(uint64_t* out, bool wide) {
    uint64_t all[64][24];
    if (hipError_t e = hipMemcpyFromSymbol(all, HIP_SYMBOL(g_po_phase), sizeof(all), 0, hipMemcpyDeviceToHost)) return e;
    const int w = wide ? 24 : 8;
    for (int f = 0; f < 64; ++f)
        for (int k = 0; k < w; ++k) out[f * w + k] = all[f][k];
    return hipSuccess;
}

__global__ __launch_bounds__(64) void selftest_ldlt_kernel(const double* __restrict__ x, double* __restrict__ out) {
    const double* rec = x + 42 * (size_t)blockIdx.x;
    double* o = out + 42 * (size_t)blockIdx.x;
    const int lane = threadIdx.x, r = lane < 6 ? lane : 5;
    double A[6][6], b[6], xs[6] = {0, 0, 0, 0, 0, 0}, xl[6] = {0, 0, 0, 0, 0, 0}, row[6];
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        RSC_UNROLL for (int j = 0; j < 6; ++j) A[i][j] = rec[6 * i + j];
        b[i] = rec[36 + i];
    }
    RSC_UNROLL for (int c = 0; c < 6; ++c) row[c] = rec[6 * r + c];
    const bool oks = po_ldlt_solve<6>(A, b, xs);
    const bool okl = po_ldlt_solve_lanes<6>(row, b, xl);
    if (lane == 0) {
        RSC_UNROLL for (int i = 0; i < 6; ++i) {
            o[i] = xs[i];
            o[7 + i] = xl[i];
        }
        o[6] = oks ? 1.0 : 0.0;
        o[13] = okl ? 1.0 : 0.0;
        for (int i = 14; i < 42; ++i) o[i] = 0.0;
    }
}

hipError_t launch_selftest_ldlt(const double* x, int nrec, double* out, hipStream_t st) {
    if (nrec > 0) selftest_ldlt_kernel<<<nrec, 64, 0, st>>>(x, out);
    return hipGetLastError();
}

hipError_t launch_poseopt(int count, const DevPoseProb* probs, unsigned* fault, hipStream_t st) {
    // the dynamic-LDS size above 64 KB needs the per-device function attribute: raised lazily at
    // this kernel's first launch on each device, so only callers of this path depend on it
    static std::atomic<unsigned long long> raised{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (!((raised.load(std::memory_order_acquire) >> dev) & 1ull)) {
        if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&poseopt_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPoseLds))
            return e;
        raised.fetch_or(1ull << dev, std::memory_order_acq_rel);
    }
    poseopt_kernel<<<count, kPoseThreads, kPoseLds, st>>>(probs, fault);
    return hipGetLastError();
}

}  // namespace rsc
