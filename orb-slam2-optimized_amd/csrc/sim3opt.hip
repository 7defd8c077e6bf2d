// sim3opt.hip — Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) kernel: one 256-thread
// workgroup per KeyFrame pair.  See rsc_sim3opt.h for the mapping and the arithmetic contract.
//
// A pass computes the per-edge terms of all correspondences in parallel (thread = correspondence,
// both of its edges) into LDS columns in g2o's edge order, then folds every column in that order on
// its own lane: H lower triangle (28) and b (7) on lanes 0..34 of wave 0, the robust chi2 column on
// wave 1.  The LM control, the 7x7 LDLT and the 14 perturbed estimates of the numeric Jacobian run
// redundantly in every lane (bit-identical values, no broadcast).
#include <hip/hip_runtime.h>
#include <atomic>
#include <cfloat>
#include "rsc_sim3opt.h"
#include "rsc_fold.h"

namespace rsc {

namespace {

constexpr int kSoThreads = 256;                  // correspondences per chunk
constexpr int kSoChunkEdges = 2 * kSoThreads;    // 512 edge terms per chunk
constexpr int kSoCol = kSoChunkEdges + 2;        // padded column stride (doubles)
constexpr int kSoCols = kSim3OptTerms + 1;       // 35 H/b columns + the chi2 column
constexpr int kSoTermDoubles = kSoCols * kSoCol;
static_assert(kSoTermDoubles >= 2 * kSim3OptMaxCorr, "chi2 terms of a whole pass must fit the term buffer");
constexpr size_t kSoLds = sizeof(double) * kSoTermDoubles;

struct SoCtx {
    const DevSim3OptProb& P;
    double* terms;
    double* red;  // [36]
    SoCam K1, K2;
    double delta, dsqr, th2;
};

__device__ __forceinline__ void so_load(const SoCtx& C, int c, bool inverse, double (&X)[3], double& u, double& v,
                                        double& inv) {
    const float4 a = inverse ? C.P.e21[c] : C.P.e12[c];
    const float4 o = C.P.uv[c];
    X[0] = a.x; X[1] = a.y; X[2] = a.z;
    inv = a.w;
    u = inverse ? o.z : o.x;
    v = inverse ? o.w : o.y;
}

// computeActiveErrors at S + activeRobustChi2 (sparse_optimizer.cpp:61-114): errors of the active
// edges stored as _error, robust chi2 terms (0.0 for inactive edges: an exact identity of a sum that
// starts at +0.0) folded in edge order by one lane.
__device__ double so_chi_pass(const SoCtx& C, const SoSim3& S) {
    const DevSim3OptProb& P = C.P;
    const int tid = threadIdx.x;
    const SoSim3 Si = so_inverse(S);
    for (int c = tid; c < P.m; c += kSoThreads) {
        double t0 = 0.0, t1 = 0.0;
        if (P.keep[c]) {
            double X[3], u, v, inv, e0, e1;
            so_load(C, c, false, X, u, v, inv);
            so_edge_error(S, C.K1, X, u, v, e0, e1);
            P.err[2 * c] = make_double2(e0, e1);
            double r1;
            po_huber(po_chi2(inv, false, e0, e1, 0.0), C.delta, C.dsqr, t0, r1);
            so_load(C, c, true, X, u, v, inv);
            so_edge_error(Si, C.K2, X, u, v, e0, e1);
            P.err[2 * c + 1] = make_double2(e0, e1);
            po_huber(po_chi2(inv, false, e0, e1, 0.0), C.delta, C.dsqr, t1, r1);
        }
        C.terms[2 * c] = t0;
        C.terms[2 * c + 1] = t1;
    }
    __syncthreads();
    if (tid == 0) C.red[0] = fold_run<false>(0.0, C.terms, 2 * P.m);
    __syncthreads();
    const double chi = C.red[0];
    __syncthreads();
    return chi;
}

// BlockSolverX::buildSystem (block_solver.hpp:502-560) with the stored errors at S.
__device__ void so_build_pass(const SoCtx& C, const SoSim3& S, double (&H)[7][7], double (&b)[7]) {
    const DevSim3OptProb& P = C.P;
    const int tid = threadIdx.x;
    SoPerturbed Pt;
    so_perturb(S, Pt);
    double acc = 0.0;
    for (int base = 0; base < P.m; base += kSoThreads) {
        const int c = base + tid;
        RSC_UNROLL for (int side = 0; side < 2; ++side) {
            double t[kSim3OptTerms];
            RSC_UNROLL for (int k = 0; k < kSim3OptTerms; ++k) t[k] = 0.0;
            if (c < P.m && P.keep[c]) {
                double X[3], u, v, inv;
                so_load(C, c, side == 1, X, u, v, inv);
                const double2 er = P.err[2 * c + side];
                so_quad_terms(Pt, side == 1, side == 1 ? C.K2 : C.K1, X, u, v, inv, er.x, er.y, C.delta, C.dsqr, t);
            }
            RSC_UNROLL for (int k = 0; k < kSim3OptTerms; ++k) C.terms[k * kSoCol + 2 * tid + side] = t[k];
        }
        __syncthreads();
        const int m = 2 * min(kSoThreads, P.m - base);
        if (tid < kSim3OptTerms) acc = fold_run<false>(acc, C.terms + tid * kSoCol, m);
        __syncthreads();
    }
    if (tid < kSim3OptTerms) C.red[tid] = acc;
    __syncthreads();
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 7; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            H[i][j] = C.red[k++];
            H[j][i] = H[i][j];
        }
    RSC_UNROLL for (int i = 0; i < 7; ++i) b[i] = C.red[28 + i];
    __syncthreads();
}

struct SoLM {
    double x[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // BlockSolver::_x persists across optimize() calls
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, its = 0, trials = 0;
};

// initializeOptimization() + optimize(iterations) (sparse_optimizer.cpp:354-414) with
// OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:59-151).
__device__ void so_optimize(const SoCtx& C, SoLM& L, SoSim3& S, int iterations) {
    bool ok = true;
    for (int i = 0; i < iterations && ok; ++i) {
        L.its++;
        double currentChi = so_chi_pass(C, S);
        const double iniChi = currentChi;
        double H[7][7], b[7];
        so_build_pass(C, S, H, b);
        if (i == 0) {
            double maxDiagonal = 0.;
            RSC_UNROLL for (int j = 0; j < 7; ++j) {  // std::max(fabs(H(j,j)), maxDiagonal)
                const double a = rabs(H[j][j]);
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
            const SoSim3 saved = S;
            double Hd[7][7];
            RSC_UNROLL for (int r = 0; r < 7; ++r)
                RSC_UNROLL for (int c = 0; c < 7; ++c) Hd[r][c] = H[r][c];
            RSC_UNROLL for (int r = 0; r < 7; ++r) Hd[r][r] += L.lambda;
            double xs[7];
            const bool ok2 = po_ldlt_solve<7>(Hd, b, xs);
            if (ok2) RSC_UNROLL for (int j = 0; j < 7; ++j) L.x[j] = xs[j];
            S = so_oplus(L.x, S);
            double tempChi = so_chi_pass(C, S);
            if (!ok2) tempChi = DBL_MAX;
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
            } else {
                L.lambda *= L.ni;
                L.ni *= 2;
                S = saved;  // pop: the edges keep the rejected trial's errors (no recompute in g2o)
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

// chi2 > th2 test of correspondence c on its stored errors (Optimizer.cpp:1184, :1216).
__device__ __forceinline__ bool so_outlier(const SoCtx& C, int c) {
    const double2 a = C.P.err[2 * c], b = C.P.err[2 * c + 1];
    const float4 p = C.P.e12[c], q = C.P.e21[c];
    return po_chi2((double)p.w, false, a.x, a.y, 0.0) > C.th2 || po_chi2((double)q.w, false, b.x, b.y, 0.0) > C.th2;
}

__device__ void so_write(const DevSim3OptProb& P, const SoSim3& S, int nIn, int nBad, const SoLM& L) {
    P.out[0] = S.r.x; P.out[1] = S.r.y; P.out[2] = S.r.z; P.out[3] = S.r.w;
    P.out[4] = S.t[0]; P.out[5] = S.t[1]; P.out[6] = S.t[2];
    P.out[7] = S.s;
    int* o = reinterpret_cast<int*>(P.out + 8);
    o[0] = nIn; o[1] = nBad; o[2] = L.its; o[3] = L.trials;
}

}  // namespace

__global__ __launch_bounds__(kSoThreads) void sim3opt_kernel(const DevSim3OptProb* __restrict__ probs) {
    extern __shared__ __attribute__((aligned(16))) double so_lds[];
    __shared__ double red_sh[kSoCols];
    __shared__ int cnt_sh;
    const DevSim3OptProb& P = probs[blockIdx.x];
    const int tid = threadIdx.x;
    SoCtx C{P, so_lds, red_sh, {}, {}, 0.0, 0.0, (double)P.th2};
    C.K1 = SoCam{(double)P.K1[0], (double)P.K1[1], (double)P.K1[2], (double)P.K1[3]};
    C.K2 = SoCam{(double)P.K2[0], (double)P.K2[1], (double)P.K2[2], (double)P.K2[3]};
    C.delta = P.delta;
    C.dsqr = C.delta * C.delta;
    SoSim3 S;
    S.r.x = P.S0[0]; S.r.y = P.S0[1]; S.r.z = P.S0[2]; S.r.w = P.S0[3];
    S.t[0] = P.S0[4]; S.t[1] = P.S0[5]; S.t[2] = P.S0[6];
    S.s = P.S0[7];
    const SoSim3 S_in = S;
    for (int c = tid; c < P.m; c += kSoThreads) P.keep[c] = 1;
    if (tid == 0) cnt_sh = 0;
    __syncthreads();
    SoLM L;
    so_optimize(C, L, S, 5);
    // Check inliers (Optimizer.cpp:1176-1194): remove both edges of a failing correspondence
    int bad = 0;
    for (int c = tid; c < P.m; c += kSoThreads) {
        if (so_outlier(C, c)) {
            P.keep[c] = 0;
            ++bad;
        }
    }
    if (bad) atomicAdd(&cnt_sh, bad);
    __syncthreads();
    const int nBad = cnt_sh;
    __syncthreads();
    if (P.m - nBad < 10) {  // return 0, g2oS12 untouched (:1201-1202)
        if (tid == 0) so_write(P, S_in, 0, nBad, L);
        return;
    }
    if (tid == 0) cnt_sh = 0;
    so_optimize(C, L, S, nBad > 0 ? 10 : 5);
    int in = 0;
    for (int c = tid; c < P.m; c += kSoThreads) {
        if (!P.keep[c]) continue;
        if (so_outlier(C, c)) P.keep[c] = 0;
        else ++in;
    }
    if (in) atomicAdd(&cnt_sh, in);
    __syncthreads();
    if (tid == 0) so_write(P, S, cnt_sh, nBad, L);
}

hipError_t launch_sim3opt(int count, const DevSim3OptProb* probs, hipStream_t st) {
    // the dynamic-LDS size above 64 KB needs the per-device function attribute: raised lazily at
    // this kernel's first launch on each device, so only callers of this path depend on it
    static std::atomic<unsigned long long> raised{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (!((raised.load(std::memory_order_acquire) >> dev) & 1ull)) {
        if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sim3opt_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSoLds))
            return e;
        raised.fetch_or(1ull << dev, std::memory_order_acq_rel);
    }
    sim3opt_kernel<<<count, kSoThreads, kSoLds, st>>>(probs);
    return hipGetLastError();
}

}  // namespace rsc
