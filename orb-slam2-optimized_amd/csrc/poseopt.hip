// poseopt.hip — Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) kernel: one 256-thread
// workgroup per Frame.  See rsc_poseopt.h for the mapping and the arithmetic contract.
//
// Where the time goes: every g2o reduction is a sequential sum over the edges, and only its
// dependent FP64 additions are serial here.  A pass computes all per-edge terms in parallel, then
// folds them in edge order out of LDS; the build pass folds the 27 H/b columns on lanes of wave 0
// while the chi2 column (when needed) folds on wave 1, and chunk columns are padded so the 27
// lanes read different banks.  The fold reads run 32 terms ahead of the additions.
// OptimizationAlgorithmLevenberg::solve recomputes activeRobustChi2 at its start; that value is the
// previous solve's currentChi at the same estimate (accepted trial -> the trial's chi2, rejected ->
// popped to the state currentChi belongs to), so it is reused bit for bit instead of refolded, and
// the per-edge errors are recomputed only when the last trial was rejected.
#include <hip/hip_runtime.h>
#include <atomic>
#include <cfloat>
#include "rsc_poseopt.h"
#include "rsc_kernels.h"
#include "rsc_fold.h"

namespace rsc {

namespace {

// Edges per build chunk = threads per workgroup.  256 (one wave per SIMD of a CU): the per-thread
// LM control state and an edge's 27 H/b terms fit the 512-VGPR budget of a 4-wave workgroup without
// scratch (512 threads capped a wave at 256 VGPRs and spilled 35 of them, round 2).
#ifndef RSC_POSE_CHUNK
#define RSC_POSE_CHUNK 256
#endif
constexpr int kPoseChunk = RSC_POSE_CHUNK;
constexpr int kPoseCol = kPoseChunk + 2;        // padded column stride (doubles): 16 B bank shift per column
constexpr int kPoseCols = kPoseTerms + 1;       // 27 H/b columns + the chi2 column
// term buffer: the build pass's columns, or the chi2 terms of a whole pass (n <= kPoseMaxEdges)
constexpr int kPoseTermDoubles = (kPoseCols * kPoseCol > kPoseMaxEdges) ? kPoseCols * kPoseCol : kPoseMaxEdges;
constexpr size_t kPoseLds = sizeof(double) * kPoseTermDoubles + kPoseMaxEdges;

struct PoseLds {
    double* terms;
    double* red;   // [32] folded sums
    uint8_t* lvl;  // [kPoseMaxEdges] edge level: 0 active, 1 outlier (g2o setLevel)
    int* nbad;
};

// Huber kernels of the two edge types (Optimizer.cpp:240-241: float deltas, setDelta(double)).
struct PoKernels {
    double dm, dm2, ds, ds2;
};

__device__ __forceinline__ bool po_is_stereo(const DevPoseProb& P, int e) { return P.ur && P.ur[e] >= 0.0f; }

// Error of edge e at `est` (computeError of its edge type), stored as _error.
__device__ __forceinline__ double3 po_edge_error(const DevPoseProb& P, int e, const PoSE3& est, const PoCam& K) {
    const float4 xw = P.xw[e];
    const float2 uv = P.uv[e];
    const bool st = po_is_stereo(P, e);
    const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
    double e0, e1, e2;
    po_error(est, K, X, (double)uv.x, (double)uv.y, st ? (double)P.ur[e] : 0.0, st, e0, e1, e2);
    P.err[e] = make_double2(e0, e1);
    if (st) P.err_r[e] = e2;
    return make_double3(e0, e1, e2);
}

__device__ __forceinline__ double3 po_stored_error(const DevPoseProb& P, int e) {
    const double2 er = P.err[e];
    return make_double3(er.x, er.y, po_is_stereo(P, e) ? P.err_r[e] : 0.0);
}

// activeRobustChi2 after computeActiveErrors at `est` (sparse_optimizer.cpp:61-114): errors of the
// level-0 edges recomputed and stored, their robust chi2 terms (0.0 for inactive edges — an exact
// identity for a sum that starts at +0.0) folded in edge order by one lane.
__device__ double po_chi_pass(const DevPoseProb& P, const PoseLds& S, const PoSE3& est, const PoCam& K, bool robust,
                              const PoKernels& hk) {
    const int tid = threadIdx.x;
    for (int e = tid; e < P.n; e += kPoseChunk) {
        double t = 0.0;
        if (S.lvl[e] == 0) {
            const double3 er = po_edge_error(P, e, est, K);
            const bool st = po_is_stereo(P, e);
            t = po_chi_term(robust, st, (double)P.xw[e].w, er.x, er.y, er.z, st ? hk.ds : hk.dm, st ? hk.ds2 : hk.dm2);
        }
        S.terms[e] = t;
    }
    __syncthreads();
    if (tid == 0) S.red[0] = fold_run<false>(0.0, S.terms, P.n);
    __syncthreads();
    const double chi = S.red[0];
    __syncthreads();
    return chi;
}

// computeActiveErrors (if `errors`) + activeRobustChi2 (if `chi`) + BlockSolver::buildSystem
// (block_solver.hpp:502-560) in one pass over kPoseChunk-edge chunks: H lower triangle folded on
// lanes 0..26 of wave 0 (added) and b (subtracted), both from 0.0; the chi2 column on wave 1.
__device__ void po_build_pass(const DevPoseProb& P, const PoseLds& S, const PoSE3& est, const PoCam& K, bool robust,
                              const PoKernels& hk, bool errors, bool chi, double (&H)[6][6], double (&b)[6],
                              double& chi_out) {
    const int tid = threadIdx.x;
    double acc = 0.0;
    for (int base = 0; base < P.n; base += kPoseChunk) {
        const int e = base + tid;
        double t[kPoseTerms];
        RSC_UNROLL for (int k = 0; k < kPoseTerms; ++k) t[k] = 0.0;
        double tc = 0.0;
        if (e < P.n && S.lvl[e] == 0) {
            const double3 er = errors ? po_edge_error(P, e, est, K) : po_stored_error(P, e);
            const float4 xw = P.xw[e];
            const bool st = po_is_stereo(P, e);
            const double delta = st ? hk.ds : hk.dm, dsqr = st ? hk.ds2 : hk.dm2;
            const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
            po_quad_terms(est, K, X, (double)xw.w, er.x, er.y, er.z, st, robust, delta, dsqr, t);
            if (chi) tc = po_chi_term(robust, st, (double)xw.w, er.x, er.y, er.z, delta, dsqr);
        }
        RSC_UNROLL for (int k = 0; k < kPoseTerms; ++k) S.terms[k * kPoseCol + tid] = t[k];
        if (chi) S.terms[kPoseTerms * kPoseCol + tid] = tc;
        __syncthreads();
        const int m = min(kPoseChunk, P.n - base);
        if (tid < kPoseTerms) {
            const double* c = S.terms + tid * kPoseCol;
            acc = (tid >= 21) ? fold_run<true>(acc, c, m) : fold_run<false>(acc, c, m);
        } else if (chi && tid == 64) {
            acc = fold_run<false>(acc, S.terms + kPoseTerms * kPoseCol, m);
        }
        __syncthreads();
    }
    if (tid < kPoseTerms) S.red[tid] = acc;
    if (chi && tid == 64) S.red[kPoseTerms] = acc;
    __syncthreads();
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 6; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            H[i][j] = S.red[k++];
            H[j][i] = H[i][j];
        }
    RSC_UNROLL for (int i = 0; i < 6; ++i) b[i] = S.red[21 + i];
    if (chi) chi_out = S.red[kPoseTerms];
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(kPoseChunk) void poseopt_kernel(const DevPoseProb* __restrict__ probs) {
    extern __shared__ __attribute__((aligned(16))) double po_lds[];
    __shared__ double red_sh[32];
    __shared__ int nbad_sh;
    const PoseLds S{po_lds, red_sh, reinterpret_cast<uint8_t*>(po_lds + kPoseTermDoubles), &nbad_sh};
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
    for (int e = tid; e < n; e += kPoseChunk) {
        S.lvl[e] = 0;
        P.outlier[e] = 0;
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
        int mine = 0;
        for (int e = tid; e < n; e += kPoseChunk) mine |= (S.lvl[e] == 0);
        const bool any = __syncthreads_or(mine) != 0;
        if (any) {
            bool ok = true;
            double chiNow = 0.0;       // activeRobustChi2 at est, when chiKnown
            bool chiKnown = false;     // (the previous solve's currentChi, computed at this est)
            bool errorsAtEst = false;  // the stored _error values belong to est
            for (int i = 0; i < 10 && ok; ++i) {
                lm_its++;
                double H[6][6], b[6];
                double chiFold = 0.0;
                po_build_pass(P, S, est, K, robust, hk, !errorsAtEst, !chiKnown, H, b, chiFold);
                double currentChi = chiKnown ? chiNow : chiFold;
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
                bool chiReal = true;  // currentChi is a computed chi2 (not the DBL_MAX of a failed solve)
                do {
                    lm_trials++;
                    const PoSE3 saved = est;
                    double Hd[6][6];
                    RSC_UNROLL for (int r = 0; r < 6; ++r)
                        RSC_UNROLL for (int c = 0; c < 6; ++c) Hd[r][c] = H[r][c];
                    RSC_UNROLL for (int r = 0; r < 6; ++r) Hd[r][r] += lambda;
                    double xs[6];
                    const bool ok2 = po_ldlt_solve6(Hd, b, xs);
                    if (ok2) RSC_UNROLL for (int j = 0; j < 6; ++j) x[j] = xs[j];
                    est = po_mul(po_exp(x), est);
                    double tempChi = po_chi_pass(P, S, est, K, robust, hk);
                    if (!ok2) tempChi = DBL_MAX;
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
                        chiReal = ok2;
                        errorsAtEst = true;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        est = saved;
                        errorsAtEst = false;
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                chiNow = currentChi;
                chiKnown = chiReal;
                if (qmax == 10 || rho == 0) {
                    ok = false;
                } else {
                    if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                    else nBadLM = 0;
                    ok = nBadLM < 3;
                }
            }
        }
        // re-classification (Optimizer.cpp:347-398; mono and stereo loops are per-edge decisions)
        int cnt = 0;
        for (int e = tid; e < n; e += kPoseChunk) {
            const double3 er = S.lvl[e] ? po_edge_error(P, e, est, K) : po_stored_error(P, e);
            const bool st = po_is_stereo(P, e);
            const float c2 = (float)po_chi2((double)P.xw[e].w, st, er.x, er.y, er.z);
            const bool bad = c2 > (st ? chi2Stereo : chi2Mono);
            S.lvl[e] = bad ? 1 : 0;
            P.outlier[e] = bad ? 1 : 0;
            cnt += bad;
        }
        if (cnt) atomicAdd(S.nbad, cnt);
        __syncthreads();
        nBad = *S.nbad;
        __syncthreads();
        if (tid == 0) *S.nbad = 0;
        if (it == 2) robust = false;
        if (n < 10) break;
    }
    if (tid == 0) {
        double R[3][3];
        po_quat_to_R(est.r, R);
        RSC_UNROLL for (int r = 0; r < 3; ++r) {
            RSC_UNROLL for (int c = 0; c < 3; ++c) P.out[4 * r + c] = (float)R[r][c];
            P.out[4 * r + 3] = (float)est.t[r];
        }
        P.out[12] = __int_as_float(n - nBad);
        P.out[13] = __int_as_float(rounds);
        P.out[14] = __int_as_float(lm_its);
        P.out[15] = __int_as_float(lm_trials);
    }
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
    poseopt_kernel<<<count, kPoseChunk, kPoseLds, st>>>(probs);
    return hipGetLastError();
}

}  // namespace rsc
