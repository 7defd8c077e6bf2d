// mlpnp.hip — gfx950 kernels of MLPnPsolver (src/MLPnPsolver.cpp):
//   mlpnp_quad_kernel<NS, Cov>  one quad (4 lanes) per hypothesis: sample, computePose with the
//                               12x12 JacobiSVD in the quad's VGPRs (rsc_mlpnp_quad.h), pose record;
//                               Cov = MlIndexedCov: the covMats branch (bearing covariances given)
//   mlpnp_scan_kernel<PPT>      MLPnPsolver::CheckInliers, points-stationary, double pose broadcast.
#include <hip/hip_runtime.h>
#include <cstdint>
// Diagnostic phase stamps of mlpnp_quad_kernel (rsc_diag_mlpnp_phase_stamps, tools/mlpnp_probe.py),
// compiled in only with RSC_ML_STAMPS=1 (a stamp is a wall-clock read and a store per phase):
// [workgroup][k] = 0 entry, 1 sample drawn, 2 design matrix + normal matrix, 3 JacobiSVD, 4 pose
// recovery (sign tests), 5 Gauss-Newton done; first 8192 workgroups.
#ifndef RSC_ML_STAMPS
#define RSC_ML_STAMPS 0
#endif
namespace rsc {
__device__ uint64_t g_ml_stamps[8192][8];
}
#if RSC_ML_STAMPS
#define RSC_ML_STAMP(k)                                                                       \
    do {                                                                                      \
        if (blockIdx.x < 8192 && threadIdx.x == 0) ::rsc::g_ml_stamps[blockIdx.x][k] = wall_clock64(); \
    } while (0)
#endif
#include "rsc_core.h"
#include "rsc_math.h"
#include "rsc_mlpnp.h"
#include "rsc_mlpnp_quad.h"
#include "rsc_kernels.h"

namespace rsc {

// ------------------------------------------------------------------------------------------------
// MLPnP hypotheses (one quad each, W / V of the 12x12 JacobiSVD in the quad's VGPRs,
// rsc_mlpnp_quad.h) and the MLPnP CheckInliers scan.
// ------------------------------------------------------------------------------------------------
template <int NS, class Cov>
__global__ __launch_bounds__(64) void mlpnp_quad_kernel(const DevML* __restrict__ probs,
                                                        const LaunchProb* __restrict__ lps,
                                                        const int2* __restrict__ wg_table,
                                                        const uint32_t* __restrict__ rng_T,
                                                        double* __restrict__ poses, int32_t* __restrict__ samples) {
    constexpr int kRegion = ml_quad_region<NS, Cov>();
    __shared__ __attribute__((aligned(16))) double smem[kMlQuadHyps * kRegion];
    const int lane = threadIdx.x, g = lane >> 2, q = lane & 3;
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const bool active = wt.y + g < lp.H;
    const int h = active ? wt.y + g : lp.H - 1;  // idle quads repeat the last hypothesis (no writes)
    const DevML& P = probs[lp.prob];
    RSC_ML_STAMP(0);
    int idx[NS];
    {
        uint32_t w[31];
        RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
        uint32_t words[NS];
        RSC_UNROLL for (int d = 0; d < NS; ++d) words[d] = rng_word(rng_T, w, lp.g0 + h * NS + d);
        swap_remove_sample<NS>(words, NS, P.n, idx);
    }
    RSC_ML_STAMP(1);
    double R[3][3], t[3];
    double* region = smem + g * kRegion;
    if constexpr (Cov::on) {  // covariances supplied: the covMats branch of computePose
        mlpnp_quad_hypothesis<NS>(P, idx, MlIndexedCov{P.cov, idx}, q, region, R, t);
    } else {
        mlpnp_quad_hypothesis<NS>(P, idx, MlNoCov{}, q, region, R, t);
    }
    RSC_ML_STAMP(5);
    if (active && q == 0) {
        const size_t rec = (size_t)(lp.out0 + h);
        double* out = poses + rec * 12;
        RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) out[3 * r + c] = R[r][c];
        RSC_UNROLL for (int r = 0; r < 3; ++r) out[9 + r] = t[r];
        if (samples) RSC_UNROLL for (int i = 0; i < NS; ++i) samples[rec * 8 + i] = idx[i];
    }
}

template <int PPT>
__global__ __launch_bounds__(256) void mlpnp_scan_kernel(const DevML* __restrict__ probs,
                                                         const LaunchProb* __restrict__ lps,
                                                         const int4* __restrict__ wg_table,
                                                         const double* __restrict__ poses,
                                                         int32_t* __restrict__ counts,
                                                         uint64_t* __restrict__ masks, int mask_words) {
    __shared__ int wave_cnt[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int4 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const DevML& P = probs[lp.prob];
    float X[PPT], Y[PPT], Z[PPT], U[PPT], V[PPT], E[PPT];
    RSC_UNROLL for (int s = 0; s < PPT; ++s) {
        const int i = s * 256 + tid;
        if (i < P.n) {
            const float4 p = P.pts[i];
            const float2 q = P.uv[i];
            X[s] = p.x; Y[s] = p.y; Z[s] = p.z; E[s] = p.w * P.th2; U[s] = q.x; V[s] = q.y;
        } else {
            X[s] = 0.f; Y[s] = 0.f; Z[s] = 1.f; E[s] = -1.f; U[s] = 0.f; V[s] = 0.f;
        }
    }
    for (int j = 0; j < wt.z; ++j) {
        const int h = wt.y + j;
        const double* pp = poses + (size_t)(lp.out0 + h) * 12;
        double R[9], t[3];
        RSC_UNROLL for (int k = 0; k < 9; ++k) R[k] = pp[k];
        RSC_UNROLL for (int k = 0; k < 3; ++k) t[k] = pp[9 + k];
        // all PPT ballots first, then one predicated store by lanes 0..PPT-1 (as the PnP scan)
        uint64_t b[PPT];
        RSC_UNROLL for (int s = 0; s < PPT; ++s)
            b[s] = __ballot(mlpnp_inlier(R, t, P.fx, P.fy, P.cx, P.cy, X[s], Y[s], Z[s], U[s], V[s], E[s]));
        int cnt = 0;
        uint64_t mine = 0;
        RSC_UNROLL for (int s = 0; s < PPT; ++s) {
            cnt += __popcll(b[s]);
            mine = (lane == s) ? b[s] : mine;
        }
        if (masks && lane < PPT) masks[(size_t)(lp.out0 + h) * mask_words + lane * 4 + wave] = mine;
        if (lane == 0) wave_cnt[wave][j & 63] = cnt;
        if ((j & 63) == 63 || j == wt.z - 1) {
            __syncthreads();
            const int base = j & ~63;
            if (tid <= (j & 63)) {
                const int c = wave_cnt[0][tid] + wave_cnt[1][tid] + wave_cnt[2][tid] + wave_cnt[3][tid];
                counts[lp.out0 + wt.y + base + tid] = c;
            }
            __syncthreads();
        }
    }
}

hipError_t launch_mlpnp_solve(int ns, bool cov, int nwg, const DevML* probs, const LaunchProb* lps, const int2* wgt,
                              const uint32_t* T, double* poses, int32_t* samples, hipStream_t st) {
    if (nwg <= 0) return hipSuccess;
    switch (ns * 2 + (cov ? 1 : 0)) {
#define RSC_CASE(N)                                                                                        \
    case 2 * N: mlpnp_quad_kernel<N, MlNoCov><<<nwg, 64, 0, st>>>(probs, lps, wgt, T, poses, samples); break; \
    case 2 * N + 1: mlpnp_quad_kernel<N, MlIndexedCov><<<nwg, 64, 0, st>>>(probs, lps, wgt, T, poses, samples); break;
        RSC_CASE(6) RSC_CASE(7) RSC_CASE(8)
#undef RSC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t read_ml_stamps(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ml_stamps), sizeof(uint64_t) * 8192 * 8, 0, hipMemcpyDeviceToHost);
}

hipError_t launch_mlpnp_scan(int ppt, int nwg, const DevML* probs, const LaunchProb* lps, const int4* wgt,
                             const double* poses, int32_t* counts, uint64_t* masks, int mask_words, hipStream_t st) {
    switch (ppt) {
#define RSC_CASE(P) case P: mlpnp_scan_kernel<P><<<nwg, 256, 0, st>>>(probs, lps, wgt, poses, counts, masks, mask_words); break;
        RSC_CASE(1) RSC_CASE(2) RSC_CASE(4) RSC_CASE(8) RSC_CASE(16) RSC_CASE(32)
#undef RSC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rsc
