// sim3opt.hip — Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) kernel: one 256-thread
// workgroup per KeyFrame pair.  See rsc_sim3opt.h for the arithmetic contract.
//
// The pass structure is PoseOptimization's (poseopt.hip): every pass is the fused
// computeActiveErrors + activeRobustChi2 + buildSystem at one estimate — the LM trial's chi2 pass
// builds the system at the trial estimate, which is the next iteration's system when the trial is
// accepted (optimization_algorithm_levenberg.cpp:63-75,108-112) — over the active edges in g2o's
// order (e12_c, e21_c of every kept correspondence c, ascending), in slabs of 192 edges: waves 1..3
// evaluate one edge per lane (error, robust chi2 term, the 14-estimate numeric Jacobian and its 35
// H/b terms) into one of two LDS slab buffers while lanes 0..35 of wave 0 fold the previous slab.
// The 14 perturbed estimates of a pass (and their inverses) are built once, one per lane, into LDS
// and read from there by every edge.  The 7x7 LDLT and the LM control run redundantly in every lane.
// The edges' _error is not stored by the passes: the inlier checks recompute it at the estimate of the
// last pass (SoLM::last), which is what g2o's edges hold then (a pure function of the estimate and the
// edge, so the same bits); global stores in the slab loop would be waited for at every slab.
#include <hip/hip_runtime.h>
#include <atomic>
#include <cfloat>
#include "rsc_sim3opt.h"
#include "rsc_fold.h"

namespace rsc {

namespace {

// Diagnostic phase clocks (rsc_diag_sim3opt_phases) only with RSC_SO_PHASES=1 (an outstanding
// s_memrealtime turns the folds' LDS waits into full lgkmcnt(0) waits).
#ifndef RSC_SO_PHASES
#define RSC_SO_PHASES 0
#endif
constexpr bool kSoPhases = RSC_SO_PHASES;
// the LM trials' LDLT with one matrix row per lane (rsc_poseopt.h po_ldlt_solve_lanes; measured
// slower, poseopt.hip): off
#ifndef RSC_LM_LDLT_LANES
#define RSC_LM_LDLT_LANES 0
#endif


// Pass form, as poseopt.hip's: 1 (wide) = 512 threads, wave 0 folds, the wave sharing its SIMD
// (RSC_SO_IDLE) idles in the passes, six waves evaluate 384 edges per slab into a single buffer;
// 0 = 256 threads, three edge waves, double-buffered slabs of 192.
#ifndef RSC_SO_WIDE
#define RSC_SO_WIDE 0
#endif
#ifndef RSC_SO_IDLE
#define RSC_SO_IDLE 4
#endif
constexpr bool kSoWide = RSC_SO_WIDE != 0;
constexpr int kSoThreads = kSoWide ? 512 : 256;
constexpr int kSoFoldLanes = 64;                 // wave 0 folds
constexpr int kSoSlab = kSoWide ? 384 : 192;     // active edges per slab
constexpr int kSoBufs = kSoWide ? 1 : 2;
constexpr int kSoCol = kSoSlab + 2;              // padded column stride (doubles)
constexpr int kSoCols = kSim3OptTerms + 1;       // 35 H/b columns + the chi2 column
constexpr int kSoBuf = kSoCols * kSoCol;         // one slab buffer
constexpr size_t kSoPt = sizeof(SoPerturbed);
constexpr size_t kSoLds = sizeof(double) * kSoBufs * kSoBuf + kSoPt + sizeof(uint16_t) * kSim3OptMaxCorr;
static_assert(kSoCol % 2 == 0, "fold_fixed reads 16-byte aligned columns");
static_assert(kSoLds <= 160 * 1024 - 1024, "LDS");
static_assert(RSC_SO_IDLE >= 1 && RSC_SO_IDLE <= 7, "idle wave");

// Slab position of this thread's edge (-1: the fold wave, and the idle wave of the wide form).
__device__ __forceinline__ int so_slot(int tid) {
    const int w = tid >> 6, lane = tid & 63;
    if constexpr (kSoWide) return (w == 0 || w == RSC_SO_IDLE) ? -1 : (w - (w > RSC_SO_IDLE ? 2 : 1)) * 64 + lane;
    else return tid - kSoFoldLanes;
}
static_assert(kSoPt % 16 == 0, "the active list follows the perturbed estimates");
static_assert(kSim3OptMaxCorr <= 65536, "active list is uint16");

// The problem's arrays as global-address-space pointers (global, not flat, accesses: a pending
// flat access would turn every LDS wait of the folds into a full lgkmcnt(0)).
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* so_g(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}
__device__ __forceinline__ float4 so_ld(const float4* p, int e) {
    using V = float __attribute__((ext_vector_type(4)));
    const V v = so_g(reinterpret_cast<const V*>(p))[e];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ double2 so_ld(const double2* p, int e) {
    using V = double __attribute__((ext_vector_type(2)));
    const V v = so_g(reinterpret_cast<const V*>(p))[e];
    return make_double2(v.x, v.y);
}

struct SoCtx {
    const DevSim3OptProb& P;
    double* terms;       // [kSoBufs][kSoCols][kSoCol] slab buffers
    SoPerturbed* pt;     // the pass's perturbed estimates
    uint16_t* list;      // kept correspondences in order
    double* red;         // [36] a pass's folded sums
    double* cur;         // [35] the current system (H lower triangle, b), kept in LDS across passes
    int* cnt;            // scan / count scratch
    SoCam K1, K2;
    double delta, dsqr, th2;
    uint64_t* clk;       // [8] phase clocks (RSC_SO_PHASES): written by threads 0 and 64 only
    // the cooperative form (so_pass_coop)
    double* ring = nullptr;     // [kSoRing][kSoCols][kSoRCol] the fold's chunk ring
    int* rf = nullptr;          // [kSoRing] chunk index + 1 whose terms fill the slot
    int* rd = nullptr;          // [kSoRing] chunk index + 1 the fold consumed last from the slot
    unsigned* pid = nullptr;    // the last pass id published (every lane's copy)
    unsigned* fault = nullptr;  // the launch's fault word
    int* cflt = nullptr;        // LDS: a wait of this workgroup gave up (later waits return at once)
};

// Inputs of one edge (side 0: e12 of correspondence c, side 1: e21), loaded a slab ahead.
struct SoEdgeIn {
    float4 a;  // point (camera of the other KeyFrame), w = invSigma2
    float4 o;  // observations (kpUn1, kpUn2)
    int c, side;
};

__device__ __forceinline__ SoEdgeIn so_load_edge(const SoCtx& C, int pos) {
    SoEdgeIn in;
    in.c = C.list[pos >> 1];
    in.side = pos & 1;
    in.a = so_ld(in.side ? C.P.e21 : C.P.e12, in.c);
    in.o = so_ld(C.P.uv, in.c);
    return in;
}

// The kept correspondences in order (the edges initializeOptimization() keeps, in the order
// Optimizer.cpp:1106-1160 added them); returns their count.
__device__ int so_list_kept(const SoCtx& C) {
    const int m = C.P.m, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (m + kSoThreads - 1) / kSoThreads;
    const int lo = min(m, tid * per), hi = min(m, lo + per);
    int c = 0;
    for (int i = lo; i < hi; ++i) c += so_g(C.P.keep)[i] != 0;
    int inc = c;
    RSC_UNROLL for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) C.cnt[w] = inc;
    __syncthreads();
    int pos = inc - c, total = 0;
    RSC_UNROLL for (int q = 0; q < kSoThreads / 64; ++q) {
        const int t = C.cnt[q];
        if (q < w) pos += t;
        total += t;
    }
    for (int i = lo; i < hi; ++i)
        if (so_g(C.P.keep)[i]) C.list[pos++] = (uint16_t)i;
    __syncthreads();
    return total;
}

// BaseBinaryEdge::linearizeOplus's 14 perturbed estimates of S and their inverses (so_perturb),
// one per lane of wave 1, into LDS.
__device__ void so_build_perturbed(const SoCtx& C, const SoSim3& S) {
    const int tid = threadIdx.x - kSoFoldLanes;
    if (tid >= 0 && tid < 14) {
        const int d = tid % 7;
        double u[7];
        RSC_UNROLL for (int i = 0; i < 7; ++i) u[i] = (i == d) ? (tid < 7 ? 1e-9 : -1e-9) : 0.0;  // static indices
        const SoSim3 e = so_oplus(u, S);
        const SoSim3 ei = so_inverse(e);
        SoSim3* dst = tid < 7 ? C.pt->p : C.pt->m;
        SoSim3* dsti = tid < 7 ? C.pt->pi : C.pt->mi;
        dst[d] = e;
        dsti[d] = ei;
    }
    __syncthreads();
}

// One pass at S over the 2 mk active edges: computeActiveErrors,
// activeRobustChi2 (sparse_optimizer.cpp:61-114) and BlockSolverX::buildSystem
// (block_solver.hpp:502-560: H lower triangle and b added from 0.0), every sum folded in edge order.
// The folded sums are left in C.red (H lower triangle row-major, b, chi2); C.red is next written at
// the end of the next pass, so they can be read until then.
__device__ double so_pass(const SoCtx& C, int mk, const SoSim3& S) {
    const int tid = threadIdx.x, me = 2 * mk;
    const int nslab = (me + kSoSlab - 1) / kSoSlab;
    const int j = so_slot(tid);
    // the first slab's inputs are loaded before the perturbed estimates are built, so their global
    // round trip overlaps that build instead of delaying the first slab
    SoEdgeIn nx{};
    if (j >= 0 && j < me) nx = so_load_edge(C, j);
    const bool clk0 = kSoPhases && blockIdx.x < 64 && tid == 0, clk1 = kSoPhases && blockIdx.x < 64 && tid == 64;
    const uint64_t tp0 = clk0 ? wall_clock64() : 0;
    so_build_perturbed(C, S);
    if (clk0) C.clk[2] += wall_clock64() - tp0;  // [2] perturbed estimates (incl. the barrier)
    const SoSim3 Si = so_inverse(S);
    double acc = 0.0;
    for (int k = 0; k <= nslab; ++k) {
        double t[kSim3OptTerms], tc = 0.0;
        if (j >= 0 && k < nslab) {
            const int pos = k * kSoSlab + j;
            if (pos < me) {
                const uint64_t c0 = clk1 ? wall_clock64() : 0;
                const SoEdgeIn in = nx;
                if (pos + kSoSlab < me) nx = so_load_edge(C, pos + kSoSlab);
                const bool inv_edge = in.side == 1;
                const double X[3] = {(double)in.a.x, (double)in.a.y, (double)in.a.z};
                const double inv = in.a.w;
                const double u = inv_edge ? in.o.z : in.o.x, v = inv_edge ? in.o.w : in.o.y;
                const SoCam& K = inv_edge ? C.K2 : C.K1;
                double e0, e1;
                so_edge_error(inv_edge ? Si : S, K, X, u, v, e0, e1);
                double r1;
                po_huber(po_chi2(inv, false, e0, e1, 0.0), C.delta, C.dsqr, tc, r1);
                // the perturbed estimates are read from LDS per edge: laundering the pointer keeps the
                // compiler from hoisting all 28 of them out of the slab loop into VGPRs
                int z = 0;
                asm volatile("" : "+v"(z));
                const SoPerturbed* pt = C.pt + z;
                so_quad_terms(*pt, inv_edge, K, X, u, v, inv, e0, e1, C.delta, C.dsqr, t);
                if (clk1) {  // [4] / [5] wave 1's edge evaluation per slab
                    __builtin_amdgcn_sched_barrier(0);
                    C.clk[4] += wall_clock64() - c0 + (uint64_t)(t[0] != t[0]);
                    C.clk[5] += 1;
                }
            } else {
                // padding of the last slab: +0.0 terms are exact identities of these folds (an
                // accumulator that starts at +0.0 never becomes -0.0 under round-to-nearest)
                RSC_UNROLL for (int q = 0; q < kSim3OptTerms; ++q) t[q] = 0.0;
            }
            if constexpr (!kSoWide) {
                double* buf = C.terms + (k & 1) * kSoBuf + j;
                RSC_UNROLL for (int q = 0; q < kSim3OptTerms; ++q) buf[q * kSoCol] = t[q];
                buf[kSim3OptTerms * kSoCol] = tc;
            }
        } else if (k > 0 && tid < kSoCols) {
            const uint64_t f0 = clk0 ? wall_clock64() : 0;
            acc = fold_fixed<kSoSlab>(acc, C.terms + (kSoWide ? 0 : ((k - 1) & 1) * kSoBuf) + tid * kSoCol);
            if (clk0) {  // [6] wave 0's folds
                __builtin_amdgcn_sched_barrier(0);
                C.clk[6] += wall_clock64() - f0 + (uint64_t)(acc != acc);
            }
        }
        __syncthreads();
        if constexpr (kSoWide) {
            // the fold of slab k - 1 is done: slab k's terms go into the buffer
            if (k < nslab) {
                if (j >= 0) {
                    double* buf = C.terms + j;
                    RSC_UNROLL for (int q = 0; q < kSim3OptTerms; ++q) buf[q * kSoCol] = t[q];
                    buf[kSim3OptTerms * kSoCol] = tc;
                }
                __syncthreads();
            }
        }
    }
    if (tid < kSoCols) C.red[tid] = acc;
    __syncthreads();
    if (clk0) {  // [0] / [1] whole passes
        C.clk[0] += wall_clock64() - tp0;
        C.clk[1] += 1;
    }
    return C.red[kSim3OptTerms];
}

// Diagnostic phase clocks of the last launch (RSC_SO_PHASES=1; wall clock, 100 MHz ticks), pairs
// 0..63: [0] passes, [1] pass count, [2] perturbed-estimate builds, [3] LM solves (LDLT + oplus),
// [4] / [5] wave 1's edge evaluation time / slabs, [6] wave 0's folds, [7] whole kernel.
__device__ uint64_t g_so_phase[64][8];

// ---- The cooperative form (RSC_SO_COOP; rsc_sim3opt.h) ----
// A pass of the one-workgroup form spends two thirds of its time evaluating the numeric Jacobians
// (14 projections per edge) on three waves; the ordered folds need one.  Here the master workgroup
// of a pair publishes each pass's estimate (S, S^-1 and the 14 perturbed estimates) and the helper
// workgroups of the pair claim chunks of 64 active edges with a pass-tagged compare-and-swap (an
// atomic add could take a chunk of the next pass), evaluate J and the error per edge and hand the 17
// doubles per edge to the master: write-through (sc1) stores, drained (vmcnt(0)), then the chunk's
// ready word = the pass id (sc1).  The master's waves 1..3 load the chunks in edge order (sc1 loads,
// no stale L1), expand them into the 35 H/b terms and the chi2 term (so_quad_tail: the same
// operations as so_quad_terms, so the same bits) into an LDS ring, and wave 0 folds the ring in
// chunk order exactly as so_pass folds its slabs.  Progress never depends on the helpers being
// resident: a master wave waiting for a chunk nobody claimed claims and evaluates it itself, and a
// helper that sees no new pass within its bound just ends.  Every master wait is bounded: on give-up
// the fault word is raised (an error status), never a silently wrong sum.
#ifndef RSC_SO_RING
#define RSC_SO_RING 6
#endif
constexpr int kSoRing = RSC_SO_RING;            // LDS ring slots (chunks)
constexpr int kSoRCol = kSoCoopChunk + 2;       // padded column stride (doubles)
constexpr int kSoRBuf = kSoCols * kSoRCol;      // one slot
constexpr size_t kSoCoopLds = sizeof(double) * kSoRing * kSoRBuf + kSoPt + sizeof(uint16_t) * kSim3OptMaxCorr;
constexpr int kSoSpin = 1 << 22;                // polls before a master wait gives up
constexpr int kSoHelperSpin = 1 << 20;          // polls before an idle helper ends
static_assert(kSoRing >= 3, "one slot per loader wave at least");
static_assert((kSoRBuf * 8) % 16 == 0 && (kSoRCol * 8) % 16 == 0, "fold_fixed reads 16-byte aligned columns");
static_assert(kSoCoopLds <= 160 * 1024 - 1024, "LDS");
static_assert(16 + 224 + 1 <= kSoCoopPub && sizeof(SoPerturbed) == 224 * sizeof(double), "publication layout");

using so_gu32 = __attribute__((address_space(1))) unsigned;
using so_gu64 = __attribute__((address_space(1))) unsigned long long;
using so_gi32 = __attribute__((address_space(1))) int;
using so_gf64 = __attribute__((address_space(1))) double;

__device__ __forceinline__ unsigned co_ld(const unsigned* p) {
    return __hip_atomic_load((so_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double co_ldd(const double* p) {
    return __hip_atomic_load((so_gf64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void co_std(double* p, double v) {
    __hip_atomic_store((so_gf64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void co_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// S's components in so_write's order (r.x, r.y, r.z, r.w, t, s), to the publication and back.
__device__ __forceinline__ void so_put(double* p, const SoSim3& a) {
    co_std(p + 0, a.r.x); co_std(p + 1, a.r.y); co_std(p + 2, a.r.z); co_std(p + 3, a.r.w);
    co_std(p + 4, a.t[0]); co_std(p + 5, a.t[1]); co_std(p + 6, a.t[2]);
    co_std(p + 7, a.s);
}
__device__ __forceinline__ SoSim3 so_from(const double* p) {
    SoSim3 a;
    a.r.x = p[0]; a.r.y = p[1]; a.r.z = p[2]; a.r.w = p[3];
    a.t[0] = p[4]; a.t[1] = p[5]; a.t[2] = p[6];
    a.s = p[7];
    return a;
}

__device__ __forceinline__ unsigned long long co_first(unsigned long long v) {
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
}

// Chunk claims of a pass: the claim word is (pass << 32) | (front << 16) | back — the master's waves
// take chunks 0, 1, ... from the front (evaluated straight into its fold ring), the helpers take
// nch - 1, nch - 2, ... from the back (handed off through global memory; the fold reaches them
// last, so their hand-off latency is covered).  Returns the claimed chunk or -1 when front and back
// have met (*boundary = the first back chunk then) or the pass is over.  The loop is wave-uniform
// (lane 0's atomics broadcast after each step): a lane-0-only retry loop lets the compiler give the
// lanes separate loop exits, and the chunk loops around it then diverge.
template <bool Front>
__device__ __forceinline__ int co_claim(SoCoopFlags* cf, unsigned pid, int nch, int* boundary) {
    so_gu64* cw = (so_gu64*)&cf->claim;
    const bool l0 = (threadIdx.x & 63) == 0;
    unsigned long long v = 0;
    if (l0) v = __hip_atomic_load(cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = co_first(v);
    for (;;) {
        const int front = (int)((v >> 16) & 0xffff), back = (int)(v & 0xffff);
        if ((unsigned)(v >> 32) != pid || front + back >= nch) {
            if (boundary) *boundary = front;
            return -1;
        }
        unsigned long long e = v;
        if (l0)
            __hip_atomic_compare_exchange_strong(cw, &e, v + (Front ? 0x10000ull : 1ull), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        e = co_first(e);
        if (e == v) return Front ? front : nch - 1 - back;
        v = e;
    }
}

// The hand-off of edge j * 64 + lane (< me): J (14), e0, e1, inv.
__device__ __forceinline__ void co_eval(const DevSim3OptProb& P, const SoPerturbed* pt, const SoSim3& S,
                                        const SoSim3& Si, const SoCam& K1, const SoCam& K2, int pos,
                                        double (&h)[kSoCoopJd]) {
    const int c = __hip_atomic_load((so_gi32*)(P.clist + (pos >> 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool inv_edge = (pos & 1) != 0;
    const float4 a = so_ld(inv_edge ? P.e21 : P.e12, c), o = so_ld(P.uv, c);
    const double X[3] = {(double)a.x, (double)a.y, (double)a.z};
    const double u = inv_edge ? o.z : o.x, v = inv_edge ? o.w : o.y;
    const SoCam& K = inv_edge ? K2 : K1;
    double e0, e1, J[2][7];
    so_edge_error(inv_edge ? Si : S, K, X, u, v, e0, e1);
    int z = 0;  // the perturbed estimates stay in LDS (as so_pass)
    asm volatile("" : "+v"(z));
    so_jacobian(*(pt + z), inv_edge, K, X, u, v, J);
    RSC_UNROLL for (int k = 0; k < 14; ++k) h[k] = J[k / 7][k % 7];
    h[14] = e0;
    h[15] = e1;
    h[16] = a.w;
}

// One wave evaluates chunk j of pass pid (edge j * 64 + lane of the kept list) and hands it off.
__device__ __forceinline__ void co_chunk(const DevSim3OptProb& P, const SoPerturbed* pt, const SoSim3& S,
                                         const SoSim3& Si, const SoCam& K1, const SoCam& K2, int me, int j,
                                         unsigned pid) {
    const int lane = threadIdx.x & 63, pos = j * kSoCoopChunk + lane;
    if (pos < me) {
        double h[kSoCoopJd];
        co_eval(P, pt, S, Si, K1, K2, pos, h);
        double* dst = P.cstore + (size_t)j * kSoCoopJd * kSoCoopChunk + lane;
        RSC_UNROLL for (int k = 0; k < kSoCoopJd; ++k) co_std(dst + k * kSoCoopChunk, h[k]);
    }
    co_drain();
    if (lane == 0) __hip_atomic_store((so_gu32*)&P.cf->ready[j], pid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void co_fail(const SoCtx& C) {
    __hip_atomic_store(C.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(C.cflt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Bounded wait for an LDS ring word to reach `need` (returns at once after a give-up of this
// workgroup).
__device__ __forceinline__ void co_wait_lds(const SoCtx& C, int* f, int need) {
    int v = 0;
    const bool ok = poll_until(
        kSoSpin,
        [&]() {
            if (__hip_atomic_load(C.cflt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return need;
            return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        },
        []() { __builtin_amdgcn_s_sleep(1); }, [need](int x) { return x >= need; }, v);
    if (!ok) co_fail(C);
}

// One pass at S (so_pass's contract, the cooperative form).
__device__ double so_pass_coop(const SoCtx& C, int mk, const SoSim3& S) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, me = 2 * mk;
    const int nch = (me + kSoCoopChunk - 1) / kSoCoopChunk;
    SoCoopFlags* cf = C.P.cf;
    const bool clk0 = kSoPhases && blockIdx.x < 64 && tid == 0, clk1 = kSoPhases && blockIdx.x < 64 && tid == 64;
    const uint64_t tp0 = clk0 ? wall_clock64() : 0;
    so_build_perturbed(C, S);
    const SoSim3 Si = so_inverse(S);
    const unsigned pid = ++*C.pid;
    // publish the pass: S, S^-1, the perturbed estimates, me and the claim word; then the pass id
    if (tid == 0) {
        so_put(C.P.cpub, S);
        so_put(C.P.cpub + 8, Si);
        // the claim word before the barrier: the master's waves claim right after it
        __hip_atomic_store((so_gu64*)&cf->claim, (unsigned long long)pid << 32, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else if (tid >= 16 && tid < 16 + 224 + 1) {
        co_std(C.P.cpub + tid, tid < 240 ? reinterpret_cast<const double*>(C.pt)[tid - 16] : (double)me);
    }
    if (tid < kSoRing) {
        C.rf[tid] = 0;
        C.rd[tid] = 0;
    }
    co_drain();
    __syncthreads();
    if (tid == 0) __hip_atomic_store((so_gu32*)&cf->pass, pid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tp1 = clk0 ? wall_clock64() : 0;
    if (clk0) C.clk[2] += tp1 - tp0;  // [2] perturbed estimates + publication
    double acc = 0.0;
    if (w == 0) {
        // the folds, chunk by chunk in edge order (lanes 0..35: one accumulator each)
        if (lane < kSoCols) {
            for (int i = 0; i < nch; ++i) {
                const int sl = i % kSoRing;
                co_wait_lds(C, C.rf + sl, i + 1);
                if (clk0 && i == 0) C.clk[4] += wall_clock64() - tp1;  // [4] publication -> first chunk in the ring
                acc = fold_fixed<kSoCoopChunk>(acc, C.ring + sl * kSoRBuf + lane * kSoRCol);
                // every lane's reads of the slot are done before it is handed back
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(C.rd + sl, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (clk0) C.clk[6] += wall_clock64() - tp1;  // [6] publication -> last fold done
        }
    } else {
        // waves 1..3: front chunks, evaluated here straight into the ring, until front and back meet;
        // then the helpers' chunks [b, nch), chunk c = b + w - 1 (mod 3), from the store into the
        // ring, the hand-off of the wave's next chunk loaded (when it is ready) before this one is
        // expanded
        auto put = [&](int c, const double (&h)[kSoCoopJd]) {
            const int pos = c * kSoCoopChunk + lane;
            double t[kSim3OptTerms], tc = 0.0;
            if (pos < me) {
                double J[2][7];
                RSC_UNROLL for (int k = 0; k < 14; ++k) J[k / 7][k % 7] = h[k];
                const double e0 = h[14], e1 = h[15], inv = h[16];
                double r1;
                po_huber(po_chi2(inv, false, e0, e1, 0.0), C.delta, C.dsqr, tc, r1);
                so_quad_tail(J, inv, e0, e1, C.delta, C.dsqr, t);
            } else {
                // padding of the last chunk: +0.0 terms (so_pass's argument)
                RSC_UNROLL for (int q = 0; q < kSim3OptTerms; ++q) t[q] = 0.0;
            }
            const int sl = c % kSoRing;
            if (c >= kSoRing) co_wait_lds(C, C.rd + sl, c - kSoRing + 1);
            double* slot = C.ring + sl * kSoRBuf + lane;
            RSC_UNROLL for (int q = 0; q < kSim3OptTerms; ++q) slot[q * kSoRCol] = t[q];
            slot[kSim3OptTerms * kSoRCol] = tc;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(C.rf + sl, c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        int b = nch;
        for (;;) {
            const int j = co_claim<true>(cf, pid, nch, &b);
            if (j < 0) break;
            double h[kSoCoopJd];
            const int pos = j * kSoCoopChunk + lane;
            if (pos < me) co_eval(C.P, C.pt, S, Si, C.K1, C.K2, pos, h);
            put(j, h);
            if (clk1) C.clk[5] += 1;  // [5] front chunks of wave 1
        }
        auto ready = [&](int c) { return __builtin_amdgcn_readfirstlane(co_ld(&cf->ready[c])) == pid; };
        auto wait_ready = [&](int c) {  // the helper that claimed it is running: a bounded wait
            int v = 0;
            if (!poll_until(
                    kSoSpin,
                    [&]() {
                        if (__hip_atomic_load(C.cflt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return 1;
                        return ready(c) ? 1 : 0;
                    },
                    []() { __builtin_amdgcn_s_sleep(1); }, [](int x) { return x != 0; }, v))
                co_fail(C);
        };
        auto load = [&](int c, double (&h)[kSoCoopJd]) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // the loads stay after the poll
            const double* src = C.P.cstore + (size_t)c * kSoCoopJd * kSoCoopChunk + lane;
            RSC_UNROLL for (int k = 0; k < kSoCoopJd; ++k) h[k] = co_ldd(src + k * kSoCoopChunk);
        };
        double hc[kSoCoopJd];
        bool have = false;
        for (int i = b + w - 1; i < nch; i += 3) {
            if (!have) {
                wait_ready(i);
                load(i, hc);
            }
            const int n = i + 3;
            have = n < nch && ready(n);
            double hn[kSoCoopJd];
            load(have ? n : i, hn);  // issued either way (straight-line waits); used when have
            put(i, hc);
            RSC_UNROLL for (int k = 0; k < kSoCoopJd; ++k) hc[k] = hn[k];
        }
    }
    __syncthreads();
    if (tid < kSoCols) C.red[tid] = acc;
    __syncthreads();
    if (clk0) {  // [0] / [1] whole passes
        C.clk[0] += wall_clock64() - tp0;
        C.clk[1] += 1;
    }
    return C.red[kSim3OptTerms];
}

// A helper workgroup of pair P: every pass the master publishes, claim and evaluate chunks until
// none is left; end at kSoCoopDone (or when no new pass comes within the bound).
__device__ __forceinline__ void so_helper(const DevSim3OptProb& P, double* pub, unsigned* pid_sh) {
    const int tid = threadIdx.x;
    const SoCam K1{(double)P.K1[0], (double)P.K1[1], (double)P.K1[2], (double)P.K1[3]};
    const SoCam K2{(double)P.K2[0], (double)P.K2[1], (double)P.K2[2], (double)P.K2[3]};
    const SoPerturbed* pt = reinterpret_cast<const SoPerturbed*>(pub + 16);
    unsigned last = 0;
    for (;;) {
        if (tid == 0) {
            int v = 0;
            const bool ok = poll_until(
                kSoHelperSpin, [&]() { return (int)co_ld(&P.cf->pass); }, []() { __builtin_amdgcn_s_sleep(2); },
                [last](int x) { return (unsigned)x != last; }, v);
            *pid_sh = ok ? (unsigned)v : kSoCoopDone;
        }
        __syncthreads();
        const unsigned pid = *pid_sh;
        if (pid == kSoCoopDone) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (tid < 16 + 224 + 1) pub[tid] = co_ldd(P.cpub + tid);
        __syncthreads();
        const SoSim3 S = so_from(pub), Si = so_from(pub + 8);
        const int me = (int)pub[240];
        const int nch = (me + kSoCoopChunk - 1) / kSoCoopChunk;
        for (;;) {
            const int j = co_claim<false>(P.cf, pid, nch, nullptr);
            if (j < 0) break;
            co_chunk(P, pt, S, Si, K1, K2, me, j, pid);
        }
        __syncthreads();  // every wave is done with this pass's publication in LDS
        last = pid;
    }
}

struct SoLM {
    double x[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // BlockSolver::_x persists across optimize() calls
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, its = 0, trials = 0;
    SoSim3 last;  // estimate of the last pass (the edges' _error is evaluated there)
};

// initializeOptimization() + optimize(iterations) (sparse_optimizer.cpp:354-414) with
// OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:59-151).
template <bool Coop>
__device__ __forceinline__ double so_pass_any(const SoCtx& C, int mk, const SoSim3& S) {
    if constexpr (Coop) return so_pass_coop(C, mk, S);
    else return so_pass(C, mk, S);
}

template <bool Coop>
__device__ void so_optimize(const SoCtx& C, SoLM& L, SoSim3& S, int iterations) {
    const int mk = so_list_kept(C);
    if (mk == 0) return;
    if constexpr (Coop) {  // the helpers read the kept list from global memory
        for (int i = threadIdx.x; i < mk; i += kSoThreads)
            __hip_atomic_store((so_gi32*)(C.P.clist + i), (int)C.list[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the system at S (C.cur: lower triangle row-major, then b) and the chi2 solve() computes there
    double chiS = so_pass_any<Coop>(C, mk, S);
    L.last = S;
    auto adopt = [&]() {  // C.cur = the last pass's system
        if (threadIdx.x < kSim3OptTerms) C.cur[threadIdx.x] = C.red[threadIdx.x];
        __syncthreads();
    };
    adopt();
    bool ok = true;
    for (int i = 0; i < iterations && ok; ++i) {
        L.its++;
        double currentChi = chiS;
        const double iniChi = currentChi;
        if (i == 0) {
            double maxDiagonal = 0.;
            RSC_UNROLL for (int j = 0; j < 7; ++j) {  // std::max(fabs(H(j,j)), maxDiagonal)
                const double a = rabs(C.cur[j * (j + 1) / 2 + j]);
                maxDiagonal = (a < maxDiagonal) ? maxDiagonal : a;
            }
            L.lambda = 1e-5 * maxDiagonal;
            L.ni = 2;
            L.nBadLM = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            L.trials++;
            const bool sclk = kSoPhases && blockIdx.x < 64 && threadIdx.x == 0;
            const uint64_t ts = sclk ? wall_clock64() : 0;
            double b[7], xs[7];
            RSC_UNROLL for (int r = 0; r < 7; ++r) b[r] = C.cur[28 + r];
            bool ok2;
            if constexpr (RSC_LM_LDLT_LANES) {
                // this lane's row of H + lambda I (rows 0..6 on lanes 0..6; rsc_poseopt.h)
                const int lr = min((int)(threadIdx.x & 63), 6);
                double row[7];
                RSC_UNROLL for (int c = 0; c < 7; ++c)
                    row[c] = lr >= c ? C.cur[lr * (lr + 1) / 2 + c] : C.cur[c * (c + 1) / 2 + lr];
                RSC_UNROLL for (int c = 0; c < 7; ++c) row[c] = (c == lr) ? row[c] + L.lambda : row[c];
                ok2 = po_ldlt_solve_lanes<7>(row, b, xs);
            } else {
                double Hd[7][7];
                RSC_UNROLL for (int r = 0; r < 7; ++r)
                    RSC_UNROLL for (int c = 0; c < 7; ++c)
                        Hd[r][c] = r >= c ? C.cur[r * (r + 1) / 2 + c] : C.cur[c * (c + 1) / 2 + r];
                RSC_UNROLL for (int r = 0; r < 7; ++r) Hd[r][r] += L.lambda;
                ok2 = po_ldlt_solve<7>(Hd, b, xs);
            }
            if (ok2) RSC_UNROLL for (int j = 0; j < 7; ++j) L.x[j] = xs[j];
            const SoSim3 trial = so_oplus(L.x, S);
            if (sclk) C.clk[3] += wall_clock64() - ts + (uint64_t)(trial.t[0] != trial.t[0]);  // [3] LM solves
            const double chiT = so_pass_any<Coop>(C, mk, trial);
            L.last = trial;
            const double tempChi = ok2 ? chiT : DBL_MAX;
            rho = (currentChi - tempChi);
            double scale = 0.;
            RSC_UNROLL for (int j = 0; j < 7; ++j) scale += L.x[j] * (L.lambda * L.x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1. - po_cube(2 * rho - 1);
                alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;                   // std::min(alpha, 2/3)
                const double scaleFactor = (1. / 3. < alpha) ? alpha : 1. / 3.;  // std::max(1/3, alpha)
                L.lambda *= scaleFactor;
                L.ni = 2;
                currentChi = tempChi;
                S = trial;
                adopt();  // the trial's system
                chiS = chiT;
            } else {
                // pop: the edges keep the rejected trial's errors (no recompute in g2o)
                L.lambda *= L.ni;
                L.ni *= 2;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) {
            ok = false;
        } else {
            if ((iniChi - currentChi) * 1e3 < iniChi) L.nBadLM++;
            else L.nBadLM = 0;
            ok = L.nBadLM < 3;
        }
    }
}

// chi2 > th2 test of correspondence c (Optimizer.cpp:1184, :1216) on the errors of the last pass:
// e12 at S, e21 at S^-1 (Sl, Sli), as so_pass evaluated them.
__device__ __forceinline__ bool so_outlier(const SoCtx& C, int c, const SoSim3& Sl, const SoSim3& Sli) {
    const float4 p = so_ld(C.P.e12, c), q = so_ld(C.P.e21, c), o = so_ld(C.P.uv, c);
    double a0, a1, b0, b1;
    so_edge_error(Sl, C.K1, {(double)p.x, (double)p.y, (double)p.z}, o.x, o.y, a0, a1);
    so_edge_error(Sli, C.K2, {(double)q.x, (double)q.y, (double)q.z}, o.z, o.w, b0, b1);
    return po_chi2((double)p.w, false, a0, a1, 0.0) > C.th2 || po_chi2((double)q.w, false, b0, b1, 0.0) > C.th2;
}

__device__ void so_write(const DevSim3OptProb& P, const SoSim3& S, int nIn, int nBad, const SoLM& L) {
    auto out = so_g(P.out);
    out[0] = S.r.x; out[1] = S.r.y; out[2] = S.r.z; out[3] = S.r.w;
    out[4] = S.t[0]; out[5] = S.t[1]; out[6] = S.t[2];
    out[7] = S.s;
    auto o = so_g(reinterpret_cast<int*>(P.out + 8));
    o[0] = nIn; o[1] = nBad; o[2] = L.its; o[3] = L.trials;
}

}  // namespace



// One pair (master workgroup) or, in the cooperative form, one helper workgroup: blocks [0, npairs)
// are the masters, blocks rpad + h * rpad + p (p < npairs) the helpers of pair p — the same block index
// modulo 8 as the master, so the dispatch order puts them on its XCD (a speed matter only: the
// hand-off is write-through and read past L1).
template <bool Coop>
__global__ __launch_bounds__(kSoThreads) void sim3opt_kernel(const DevSim3OptProb* __restrict__ probs, int npairs,
                                                            int rpad, unsigned* fault) {
    extern __shared__ __attribute__((aligned(16))) double so_lds[];
    __shared__ double red_sh[kSoCols];
    __shared__ double cur_sh[kSim3OptTerms];
    __shared__ int cnt_sh[kSoThreads / 64];
    __shared__ int tot_sh;
    __shared__ uint64_t clk_sh[8];
    __shared__ int rf_sh[Coop ? kSoRing : 1], rd_sh[Coop ? kSoRing : 1], cflt_sh;
    __shared__ unsigned hpid_sh;
    const int tid = threadIdx.x;
    if (Coop && (int)blockIdx.x >= rpad) {
        const int p = ((int)blockIdx.x - rpad) % rpad;
        if (p < npairs) so_helper(probs[p], so_lds, &hpid_sh);
        return;
    }
    if ((int)blockIdx.x >= npairs) return;
    const DevSim3OptProb& P = probs[blockIdx.x];
    constexpr size_t kTermBytes = Coop ? sizeof(double) * kSoRing * kSoRBuf : sizeof(double) * kSoBufs * kSoBuf;
    SoPerturbed* pt = reinterpret_cast<SoPerturbed*>(reinterpret_cast<unsigned char*>(so_lds) + kTermBytes);
    uint16_t* list = reinterpret_cast<uint16_t*>(reinterpret_cast<unsigned char*>(pt) + kSoPt);
    unsigned pid = 0;
    SoCtx C{P, so_lds, pt, list, red_sh, cur_sh, cnt_sh, {}, {}, 0.0, 0.0, (double)P.th2, clk_sh};
    if constexpr (Coop) {
        C.ring = so_lds;
        C.rf = rf_sh;
        C.rd = rd_sh;
        C.pid = &pid;
        C.fault = fault;
        C.cflt = &cflt_sh;
        if (tid == 0) cflt_sh = 0;
    }
    if (kSoPhases && tid < 8) clk_sh[tid] = 0;
    const uint64_t t_start = kSoPhases ? wall_clock64() : 0;
    C.K1 = SoCam{(double)P.K1[0], (double)P.K1[1], (double)P.K1[2], (double)P.K1[3]};
    C.K2 = SoCam{(double)P.K2[0], (double)P.K2[1], (double)P.K2[2], (double)P.K2[3]};
    C.delta = P.delta;
    C.dsqr = C.delta * C.delta;
    SoSim3 S;
    S.r.x = P.S0[0]; S.r.y = P.S0[1]; S.r.z = P.S0[2]; S.r.w = P.S0[3];
    S.t[0] = P.S0[4]; S.t[1] = P.S0[5]; S.t[2] = P.S0[6];
    S.s = P.S0[7];
    const SoSim3 S_in = S;
    for (int c = tid; c < P.m; c += kSoThreads) so_g(P.keep)[c] = 1;
    if (tid == 0) tot_sh = 0;
    __syncthreads();
    SoLM L;
    L.last = S;
    // the helpers end when this workgroup does, whichever way it returns
    auto done = [&]() {
        if constexpr (Coop) {
            if (tid == 0) __hip_atomic_store((so_gu32*)&P.cf->pass, kSoCoopDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    so_optimize<Coop>(C, L, S, 5);
    // Check inliers (Optimizer.cpp:1176-1194): remove both edges of a failing correspondence
    int bad = 0;
    SoSim3 Sli = so_inverse(L.last);
    for (int c = tid; c < P.m; c += kSoThreads) {
        if (so_outlier(C, c, L.last, Sli)) {
            so_g(P.keep)[c] = 0;
            ++bad;
        }
    }
    if (bad) atomicAdd(&tot_sh, bad);
    __syncthreads();
    const int nBad = tot_sh;
    __syncthreads();
    if (P.m - nBad < 10) {  // return 0, g2oS12 untouched (:1201-1202)
        if (tid == 0) so_write(P, S_in, 0, nBad, L);
        done();
        return;
    }
    if (tid == 0) tot_sh = 0;
    so_optimize<Coop>(C, L, S, nBad > 0 ? 10 : 5);
    done();
    int in = 0;
    Sli = so_inverse(L.last);
    for (int c = tid; c < P.m; c += kSoThreads) {
        if (!so_g(P.keep)[c]) continue;
        if (so_outlier(C, c, L.last, Sli)) so_g(P.keep)[c] = 0;
        else ++in;
    }
    if (in) atomicAdd(&tot_sh, in);
    __syncthreads();
    if (tid == 0) so_write(P, S, tot_sh, nBad, L);
    if (kSoPhases && blockIdx.x < 64) {
        __syncthreads();
        if (tid == 0) clk_sh[7] = wall_clock64() - t_start;  // [7] whole kernel
        __syncthreads();
        if (tid < 8) g_so_phase[blockIdx.x][tid] = clk_sh[tid];
    }
}

hipError_t read_sim3opt_phases(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_so_phase), sizeof(uint64_t) * 64 * 8, 0, hipMemcpyDeviceToHost);
}

hipError_t launch_sim3opt(int count, const DevSim3OptProb* probs, int helpers, unsigned* fault, hipStream_t st) {
    // the dynamic-LDS size above 64 KB needs the per-device function attribute: raised lazily at
    // this kernel's first launch on each device, so only callers of this path depend on it
    static std::atomic<unsigned long long> raised{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (helpers < 0 || (helpers > 0 && !fault)) return hipErrorInvalidValue;
    if (!((raised.load(std::memory_order_acquire) >> dev) & 1ull)) {
        if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sim3opt_kernel<false>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSoLds))
            return e;
        if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sim3opt_kernel<true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSoCoopLds))
            return e;
        raised.fetch_or(1ull << dev, std::memory_order_acq_rel);
    }
    if (helpers == 0) {
        sim3opt_kernel<false><<<count, kSoThreads, kSoLds, st>>>(probs, count, count, fault);
    } else {
        const int rpad = (count + 7) / 8 * 8;  // helpers share their master's block index modulo 8
        sim3opt_kernel<true><<<rpad * (1 + helpers), kSoThreads, kSoCoopLds, st>>>(probs, count, rpad, fault);
    }
    return hipGetLastError();
}

}  // namespace rsc
