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

constexpr int kPoseThreads = 256;                 // one wave per SIMD of a CU
constexpr int kPoseFoldLanes = 64;                // wave 0 folds
constexpr int kPoseSlab = kPoseThreads - kPoseFoldLanes;  // active edges per slab (waves 1..3)
constexpr int kPoseCol = kPoseSlab + 2;           // padded column stride (doubles): 16 B bank shift per column
constexpr int kPoseCols = kPoseTerms + 1;         // 27 H/b columns + the chi2 column
constexpr int kPoseBuf = kPoseCols * kPoseCol;    // one slab buffer
constexpr size_t kPoseLds = sizeof(double) * 2 * kPoseBuf + sizeof(uint16_t) * kPoseMaxEdges + kPoseMaxEdges;
static_assert(kPoseCol % 2 == 0, "fold_run reads 16-byte aligned columns");
static_assert(kPoseMaxEdges <= 65536, "active list is uint16");

struct PoseLds {
    double* terms;   // [2][kPoseCols][kPoseCol] slab buffers
    uint16_t* list;  // [kPoseMaxEdges] active edges of the round, in edge order
    uint8_t* lvl;    // [kPoseMaxEdges] edge level: 0 active, 1 outlier (g2o setLevel)
    double* red;     // [32] folded sums
    int* scan;       // [kPoseThreads / 64] wave totals
    int* nbad;
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
__device__ __forceinline__ void po_st(double2* p, int e, double a, double b) {
    using V = double __attribute__((ext_vector_type(2)));
    V v;
    v.x = a;
    v.y = b;
    po_g(reinterpret_cast<V*>(p))[e] = v;
}

// Huber kernels of the two edge types (Optimizer.cpp:240-241: float deltas, setDelta(double)).
struct PoKernels {
    double dm, dm2, ds, ds2;
};

__device__ __forceinline__ bool po_is_stereo(const DevPoseProb& P, int e) { return P.ur && po_g(P.ur)[e] >= 0.0f; }

// Error of edge e at `est` (computeError of its edge type), stored as _error.
__device__ __forceinline__ double3 po_edge_error(const DevPoseProb& P, int e, const PoSE3& est, const PoCam& K) {
    const float4 xw = po_ld(P.xw, e);
    const float2 uv = po_ld(P.uv, e);
    const bool st = po_is_stereo(P, e);
    const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
    double e0, e1, e2;
    po_error(est, K, X, (double)uv.x, (double)uv.y, st ? (double)po_g(P.ur)[e] : 0.0, st, e0, e1, e2);
    po_st(P.err, e, e0, e1);
    if (st) po_g(P.err_r)[e] = e2;
    return make_double3(e0, e1, e2);
}

__device__ __forceinline__ double3 po_stored_error(const DevPoseProb& P, int e) {
    const double2 er = po_ld(P.err, e);
    return make_double3(er.x, er.y, po_is_stereo(P, e) ? po_g(P.err_r)[e] : 0.0);
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
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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

// One pass at `est` over the m active edges: computeActiveErrors (errors stored),
// activeRobustChi2 (sparse_optimizer.cpp:61-114) and BlockSolver::buildSystem
// (block_solver.hpp:502-560: H lower triangle added, b subtracted, both from 0.0), every sum
// folded in edge order.
__device__ void po_pass(const DevPoseProb& P, const PoseLds& S, int m, const PoSE3& est, const PoCam& K, bool robust,
                        const PoKernels& hk, double (&H)[6][6], double (&b)[6], double& chi) {
    const int tid = threadIdx.x;
    const int nslab = (m + kPoseSlab - 1) / kPoseSlab;
    const int j = tid - kPoseFoldLanes;
    PoEdgeIn nx{};
    if (j >= 0 && j < m) nx = po_load(P, S.list[j]);
    double acc = 0.0;
    for (int k = 0; k <= nslab; ++k) {
        if (j >= 0) {
            const int pos = k * kPoseSlab + j;
            if (k < nslab && pos < m) {
                const PoEdgeIn in = nx;
                if (pos + kPoseSlab < m) nx = po_load(P, S.list[pos + kPoseSlab]);
                const bool st = in.ur >= 0.0f;
                const double X[3] = {(double)in.xw.x, (double)in.xw.y, (double)in.xw.z};
                double t[kPoseTerms], tc;
                if constexpr (RSC_PO_DIAG == 1) {
                    RSC_UNROLL for (int q = 0; q < kPoseTerms; ++q) t[q] = X[q % 3] * 1e-30;
                    tc = X[0] * 1e-30;
                } else {
                    double e0, e1, e2;
                    po_error(est, K, X, (double)in.uv.x, (double)in.uv.y, st ? (double)in.ur : 0.0, st, e0, e1, e2);
                    po_st(P.err, in.e, e0, e1);
                    if (st) po_g(P.err_r)[in.e] = e2;
                    const double delta = st ? hk.ds : hk.dm, dsqr = st ? hk.ds2 : hk.dm2;
                    po_quad_terms(est, K, X, (double)in.xw.w, e0, e1, e2, st, robust, delta, dsqr, t);
                    tc = po_chi_term(robust, st, (double)in.xw.w, e0, e1, e2, delta, dsqr);
                }
                double* buf = S.terms + (k & 1) * kPoseBuf + j;
                RSC_UNROLL for (int q = 0; q < 21; ++q) buf[q * kPoseCol] = t[q];
                RSC_UNROLL for (int q = 21; q < kPoseTerms; ++q) buf[q * kPoseCol] = -t[q];
                buf[kPoseTerms * kPoseCol] = tc;
            } else if (k < nslab) {
                // padding of the last slab: +0.0 terms are exact identities of these folds (an
                // accumulator that starts at +0.0 never becomes -0.0 under round-to-nearest)
                double* buf = S.terms + (k & 1) * kPoseBuf + j;
                RSC_UNROLL for (int q = 0; q < kPoseCols; ++q) buf[q * kPoseCol] = 0.0;
            }
        } else if (k > 0 && tid < kPoseCols) {
            if constexpr (RSC_PO_DIAG != 2) acc = fold_fixed<kPoseSlab>(acc, S.terms + ((k - 1) & 1) * kPoseBuf + tid * kPoseCol);
        }
        __syncthreads();
    }
    if (tid < kPoseCols) S.red[tid] = acc;
    __syncthreads();
    int q = 0;
    RSC_UNROLL for (int i = 0; i < 6; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            H[i][j] = S.red[q++];
            H[j][i] = H[i][j];
        }
    RSC_UNROLL for (int i = 0; i < 6; ++i) b[i] = S.red[21 + i];
    chi = S.red[kPoseTerms];
    // S.red is next written after the next pass's slab barriers, by which time every thread has read it
}

}  // namespace

// Diagnostic phase clock (wall clock, 100 MHz ticks) of the last launch, frames 0..63: [0] passes,
// [1] number of passes + (sum of their active edges << 24), [2] re-classification, [3] whole kernel
// (thread 0); [4..7] unused.
__device__ uint64_t g_po_phase[64][8];

__global__ __launch_bounds__(kPoseThreads) void poseopt_kernel(const DevPoseProb* __restrict__ probs) {
    extern __shared__ __attribute__((aligned(16))) double po_lds[];
    __shared__ double red_sh[32];
    __shared__ int scan_sh[kPoseThreads / 64];
    __shared__ int nbad_sh;
    const PoseLds S{po_lds, reinterpret_cast<uint16_t*>(po_lds + 2 * kPoseBuf),
                    reinterpret_cast<uint8_t*>(po_lds + 2 * kPoseBuf) + sizeof(uint16_t) * kPoseMaxEdges, red_sh,
                    scan_sh, &nbad_sh};
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
    const PoSE3 init = po_from_Rt(R0, t0);  // Converter::toSE3Quat (rotation() = linear(), Q14)
    const bool clk = kPosePhases && blockIdx.x < 64 && tid == 0;
    uint64_t ph_pass = 0, n_pass = 0, ph_cls = 0, t_start = clk ? wall_clock64() : 0;
    for (int e = tid; e < n; e += kPoseThreads) {
        S.lvl[e] = 0;
        po_g(P.outlier)[e] = 0;
    }
    if (tid == 0) *S.nbad = 0;
    __syncthreads();

    double x[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // BlockSolver::_x persists across rounds
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, rounds = 0, lm_its = 0, lm_trials = 0, nBad = 0;
    bool robust = true;
    PoSE3 est = init;
    for (int it = 0; it < 4; ++it) {
        rounds++;
        est = init;
        const int m = po_list_active(S, n);
        if (m > 0) {
            // the system at est and the chi2 solve() computes there
            double H[6][6], b[6], chiEst;
            uint64_t tp = clk ? wall_clock64() : 0;
            po_pass(P, S, m, est, K, robust, hk, H, b, chiEst);
            if (clk) { ph_pass += wall_clock64() - tp; n_pass += 1 + ((uint64_t)m << 24); }
            bool ok = true;
            for (int i = 0; i < 10 && ok; ++i) {
                lm_its++;
                double currentChi = chiEst;
                const double iniChi = currentChi;
                if (i == 0) {
                    double maxDiagonal = 0.;
                    RSC_UNROLL for (int j = 0; j < 6; ++j) {  // std::max(fabs(H(j,j)), maxDiagonal)
                        const double a = rabs(H[j][j]);
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
                    double Hd[6][6];
                    RSC_UNROLL for (int r = 0; r < 6; ++r)
                        RSC_UNROLL for (int c = 0; c < 6; ++c) Hd[r][c] = H[r][c];
                    RSC_UNROLL for (int r = 0; r < 6; ++r) Hd[r][r] += lambda;
                    double xs[6];
                    const bool ok2 = po_ldlt_solve6(Hd, b, xs);
                    if (ok2) RSC_UNROLL for (int j = 0; j < 6; ++j) x[j] = xs[j];
                    const PoSE3 trial = po_mul(po_exp(x), est);
                    double Ht[6][6], bt[6], chiT;
                    tp = clk ? wall_clock64() : 0;
                    po_pass(P, S, m, trial, K, robust, hk, Ht, bt, chiT);
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
                        RSC_UNROLL for (int r = 0; r < 6; ++r) {
                            RSC_UNROLL for (int c = 0; c < 6; ++c) H[r][c] = Ht[r][c];
                            b[r] = bt[r];
                        }
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
            const double3 er = S.lvl[e] ? po_edge_error(P, e, est, K) : po_stored_error(P, e);
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
    }
}

hipError_t read_poseopt_phases(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_po_phase), sizeof(uint64_t) * 64 * 8, 0, hipMemcpyDeviceToHost);
}

hipError_t launch_poseopt(int count, const DevPoseProb* probs, hipStream_t st) {
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
    poseopt_kernel<<<count, kPoseThreads, kPoseLds, st>>>(probs);
    return hipGetLastError();
}

}  // namespace rsc
