// poseopt.hip — Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) kernel: one 256-thread
// workgroup per Frame.  See rsc_poseopt.h for the mapping and the arithmetic contract.
#include <hip/hip_runtime.h>
#include <cfloat>
#include "rsc_poseopt.h"
#include "rsc_kernels.h"

namespace rsc {

namespace {

struct PoseShared {
    double terms[kPoseTerms * kPoseThreads];  // per-chunk edge terms, column k at [k * 256]
    double red[kPoseTerms];                   // folded sums
    uint8_t lvl[kPoseMaxEdges];               // edge level: 0 active, 1 outlier (g2o setLevel)
    int nbad;
};

// activeRobustChi2 after computeActiveErrors at `est` (sparse_optimizer.cpp:61-114): errors of the
// level-0 edges are recomputed and stored, their robust chi2 terms folded in edge order.
__device__ double po_chi_pass(const DevPoseProb& P, PoseShared& S, const PoSE3& est, const PoCam& K, bool robust,
                              double delta, double dsqr) {
    const int tid = threadIdx.x;
    double acc = 0.0;
    for (int base = 0; base < P.n; base += kPoseThreads) {
        const int e = base + tid;
        double t = 0.0;
        if (e < P.n && S.lvl[e] == 0) {
            const float4 xw = P.xw[e];
            const float2 uv = P.uv[e];
            const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
            double e0, e1;
            po_error(est, K, X, (double)uv.x, (double)uv.y, e0, e1);
            P.err[e] = make_double2(e0, e1);
            t = po_chi_term(robust, (double)xw.w, e0, e1, delta, dsqr);
        }
        S.terms[tid] = t;
        __syncthreads();
        if (tid == 0) {
            const int m = min(kPoseThreads, P.n - base);
            const double* c = S.terms;
            int r = 0;
            for (; r + 4 <= m; r += 4) {
                const double a = c[r], b = c[r + 1], d = c[r + 2], f = c[r + 3];
                acc = acc + a;
                acc = acc + b;
                acc = acc + d;
                acc = acc + f;
            }
            for (; r < m; ++r) acc = acc + c[r];
        }
        __syncthreads();
    }
    if (tid == 0) S.red[0] = acc;
    __syncthreads();
    const double chi = S.red[0];
    __syncthreads();
    return chi;
}

// BlockSolver::buildSystem (block_solver.hpp:502-560): H (lower triangle) and b, folded in edge
// order on lanes 0..26 (H entries added, b entries subtracted, both from 0.0).
__device__ void po_build_pass(const DevPoseProb& P, PoseShared& S, const PoSE3& est, const PoCam& K, bool robust,
                              double delta, double dsqr, double (&H)[6][6], double (&b)[6]) {
    const int tid = threadIdx.x;
    double acc = 0.0;
    for (int base = 0; base < P.n; base += kPoseThreads) {
        const int e = base + tid;
        double t[kPoseTerms];
        RSC_UNROLL for (int k = 0; k < kPoseTerms; ++k) t[k] = 0.0;
        if (e < P.n && S.lvl[e] == 0) {
            const float4 xw = P.xw[e];
            const double2 er = P.err[e];
            const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
            po_quad_terms(est, K, X, (double)xw.w, er.x, er.y, robust, delta, dsqr, t);
        }
        RSC_UNROLL for (int k = 0; k < kPoseTerms; ++k) S.terms[k * kPoseThreads + tid] = t[k];
        __syncthreads();
        if (tid < kPoseTerms) {
            const int m = min(kPoseThreads, P.n - base);
            const double* c = S.terms + tid * kPoseThreads;
            const bool sub = tid >= 21;
            int r = 0;
            for (; r + 4 <= m; r += 4) {
                const double a = c[r], bb = c[r + 1], d = c[r + 2], f = c[r + 3];
                acc = sub ? acc - a : acc + a;
                acc = sub ? acc - bb : acc + bb;
                acc = sub ? acc - d : acc + d;
                acc = sub ? acc - f : acc + f;
            }
            for (; r < m; ++r) acc = sub ? acc - c[r] : acc + c[r];
        }
        __syncthreads();
    }
    if (tid < kPoseTerms) S.red[tid] = acc;
    __syncthreads();
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 6; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            H[i][j] = S.red[k++];
            H[j][i] = H[i][j];
        }
    RSC_UNROLL for (int i = 0; i < 6; ++i) b[i] = S.red[21 + i];
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(kPoseThreads) void poseopt_kernel(const DevPoseProb* __restrict__ probs) {
    __shared__ PoseShared S;
    const DevPoseProb& P = probs[blockIdx.x];
    const int tid = threadIdx.x, n = P.n;
    const PoCam K{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy};
    const float deltaMono = sqrt(5.991);  // Optimizer.cpp:240
    const double delta = deltaMono, dsqr = delta * delta;  // RobustKernelHuber::setDelta
    const float chi2Mono = 5.991f;
    double R0[3][3], t0[3];
    RSC_UNROLL for (int r = 0; r < 3; ++r) {
        RSC_UNROLL for (int c = 0; c < 3; ++c) R0[r][c] = (double)P.T[4 * r + c];
        t0[r] = (double)P.T[4 * r + 3];
    }
    const PoSE3 init = po_from_Rt(R0, t0);  // Converter::toSE3Quat (rotation() = linear(), Q14)
    for (int e = tid; e < n; e += kPoseThreads) {
        S.lvl[e] = 0;
        P.outlier[e] = 0;
    }
    if (tid == 0) S.nbad = 0;
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
        for (int e = tid; e < n; e += kPoseThreads) mine |= (S.lvl[e] == 0);
        const bool any = __syncthreads_or(mine) != 0;
        if (any) {
            bool ok = true;
            for (int i = 0; i < 10 && ok; ++i) {
                lm_its++;
                double currentChi = po_chi_pass(P, S, est, K, robust, delta, dsqr);
                const double iniChi = currentChi;
                double H[6][6], b[6];
                po_build_pass(P, S, est, K, robust, delta, dsqr, H, b);
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
                    const PoSE3 saved = est;
                    double Hd[6][6];
                    RSC_UNROLL for (int r = 0; r < 6; ++r)
                        RSC_UNROLL for (int c = 0; c < 6; ++c) Hd[r][c] = H[r][c];
                    RSC_UNROLL for (int r = 0; r < 6; ++r) Hd[r][r] += lambda;
                    double xs[6];
                    const bool ok2 = po_ldlt_solve6(Hd, b, xs);
                    if (ok2) RSC_UNROLL for (int j = 0; j < 6; ++j) x[j] = xs[j];
                    est = po_mul(po_exp(x), est);
                    double tempChi = po_chi_pass(P, S, est, K, robust, delta, dsqr);
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
                    } else {
                        lambda *= ni;
                        ni *= 2;
                        est = saved;
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
        // re-classification (Optimizer.cpp:347-376)
        int cnt = 0;
        for (int e = tid; e < n; e += kPoseThreads) {
            double2 er;
            if (S.lvl[e]) {
                const float4 xw = P.xw[e];
                const float2 uv = P.uv[e];
                const double X[3] = {(double)xw.x, (double)xw.y, (double)xw.z};
                po_error(est, K, X, (double)uv.x, (double)uv.y, er.x, er.y);
                P.err[e] = er;
            } else {
                er = P.err[e];
            }
            const float c2 = (float)po_chi2((double)P.xw[e].w, er.x, er.y);
            const bool bad = c2 > chi2Mono;
            S.lvl[e] = bad ? 1 : 0;
            P.outlier[e] = bad ? 1 : 0;
            cnt += bad;
        }
        if (cnt) atomicAdd(&S.nbad, cnt);
        __syncthreads();
        nBad = S.nbad;
        __syncthreads();
        if (tid == 0) S.nbad = 0;
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
    poseopt_kernel<<<count, kPoseThreads, 0, st>>>(probs);
    return hipGetLastError();
}

}  // namespace rsc
