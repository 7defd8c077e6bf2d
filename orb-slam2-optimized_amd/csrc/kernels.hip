// kernels.hip — gfx950 kernels of the RANSAC pose engine.
//
//   pnp_eig_group_kernel<NS> / pnp_betas_kernel<NS>   EPnP hypotheses (sample -> compute_pose)
//                          in two stages: lane pairs per hypothesis for the 12x12 eigenvectors,
//                          then one wave per (beta approximation, 64 hypotheses) (rsc_quad.h).
//   pnp_scan_kernel<PPT>   PnPsolver::CheckInliers for a chunk of hypotheses of one problem:
//                          256 threads hold the problem's correspondences in VGPRs (PPT per
//                          thread); per hypothesis every lane tests its points, __ballot gives the
//                          64-bit inlier words, popcount gives the count.
//   pnp_refine_kernel      PnPsolver::Refine: compaction of the best inlier set into the grow-only
//                          EPnP buffers, EPnP over n_r rows (MtM built block-parallel), then the
//                          block-parallel CheckInliers of the refined pose.
//   sim3_solve_kernel / sim3_scan_kernel   the same split for Sim3Solver (Horn, float).
//   (MLPnPsolver's kernels are in mlpnp.hip.)
//
// Reference: src/PnPsolver.cpp, src/Sim3Solver.cpp (see rsc_core.h for the arithmetic contract).
#include <hip/hip_runtime.h>
#include <climits>

// Diagnostic phase stamps of the refine kernel (rsc_diag_refine_phase_stamps), compiled in only with
// RSC_REFINE_STAMPS=1: [job][0..7] = entry, compaction, control points, MtM, eigen, betas, check,
// exit; [8..11] inside the eigen phase = scaled + tridiagonal, Q accumulated, QR chase, eigenvectors;
// [12 + 4w + j] inside the betas phase, wave w (approximation w + 1): j = 0 betas + Gauss-Newton + ccs,
// 1 pc0 sum, 2 M sum + Horn, 3 reprojection-error sum.
#ifndef RSC_REFINE_STAMPS
#define RSC_REFINE_STAMPS 0
#endif
namespace rsc {
__device__ uint64_t g_refine_stamps[64][24];
}
// Diagnostic phase stamps of the hypothesis solve (rsc_diag_solve_phase_stamps), compiled in only
// with RSC_SOLVE_STAMPS=1: [0][wg][k] eigen stage (entry, sample + MtM, tridiagonal, Q, chase + store),
// [1][wg][k] betas stage (entry, L + rho, find_betas, Gauss-Newton, row loads, R and t, hand-off,
// exit); slot 7 = the approximation (betas) | 256 * launch-table index.
#ifndef RSC_SOLVE_STAMPS
#define RSC_SOLVE_STAMPS 0
#endif
namespace rsc {
__device__ uint64_t g_solve_stamps[3][4096][8];
}
#if RSC_SOLVE_STAMPS
// inside jacobi_svd_solve_6xk (find_betas): plane 2, [wave][j], j = QR done, U formed, sweeps done,
// [wave][3] = k (only the betas kernel's single-wave workgroups, blockIdx.x < 4096)
#define RSC_JSVD_STAMP(k, j)                                                                           \
    do {                                                                                               \
        if (blockIdx.x < 4096 && (threadIdx.x & 63) == 0 && blockDim.x == 64) {                       \
            ::rsc::g_solve_stamps[2][blockIdx.x][j] = wall_clock64();                                  \
            ::rsc::g_solve_stamps[2][blockIdx.x][3] = (k);                                             \
        }                                                                                              \
    } while (0)
#define RSC_SOLVE_STAMP(st, k)                                                                         \
    do {                                                                                               \
        if (blockIdx.x < 4096 && (threadIdx.x & 63) == 0) ::rsc::g_solve_stamps[st][blockIdx.x][k] = wall_clock64(); \
    } while (0)
#endif
// (the stamp macros above are defined before the headers that expand them)
#include "rsc_core.h"
#include "rsc_epnp.h"
#include "rsc_sim3.h"
#if RSC_REFINE_STAMPS
#define RSC_EIG_PHASE(k)                                                                               \
    do {                                                                                               \
        if (blockIdx.x < 64 && threadIdx.x == 0) ::rsc::g_refine_stamps[blockIdx.x][8 + (k)] = wall_clock64(); \
    } while (0)
#endif
#include "rsc_quad.h"
#include "rsc_math.h"
#include "rsc_kernels.h"

namespace rsc {

// ------------------------------------------------------------------------------------------------
// PnP hypotheses
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// PnP hypotheses, two-kernel form (rsc_quad.h): lane-group eigenvectors (kEigLanes lanes per
// hypothesis, kEigHyps per workgroup, one wave per SIMD), then one wave per beta approximation.
// ------------------------------------------------------------------------------------------------
template <int NS>
__global__ __launch_bounds__(64) void pnp_eig_group_kernel(const DevPnP* __restrict__ probs,
                                                          const LaunchProb* __restrict__ lps,
                                                          const int2* __restrict__ wg_table,
                                                          const uint32_t* __restrict__ rng_T,
                                                          double* __restrict__ stage, int32_t* __restrict__ samples) {
    __shared__ __attribute__((aligned(16))) double smem[kEigHyps * kQuadRegion];
    pnp_eig_group_body<NS, 99, kEigLanes, kEigHyps>(probs, lps, wg_table, rng_T, stage, samples, smem);
}

// split form (rsc_quad.h pnp_eig_split_body): wave 0 chases, wave 1 rotates Q
// (<= 256 registers: two waves per SIMD, so a SIMD holds a chase wave and its row wave)
template <int NS>
__global__ __launch_bounds__(128 * kSplitUnits) __attribute__((amdgpu_waves_per_eu(2))) void pnp_eig_split_kernel(
    const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps, const int2* __restrict__ wg_table,
    int nwg_table, const uint32_t* __restrict__ rng_T, double* __restrict__ stage, int32_t* __restrict__ samples,
    unsigned* fault) {
    __shared__ __attribute__((aligned(16))) double smem[kSplitHyps * kQuadRegion];
    __shared__ __attribute__((aligned(16))) double dsub[kSplitHyps * kSplitDsub];
    __shared__ int pub[kSplitUnits], ack[kSplitUnits];
    pnp_eig_split_body<NS>(probs, lps, wg_table, nwg_table, rng_T, stage, samples, smem, dsub, pub, ack, fault);
}

template <int NS>
__global__ __launch_bounds__(64) void pnp_betas_kernel(const DevPnP* __restrict__ probs,
                                                       const LaunchProb* __restrict__ lps,
                                                       const int2* __restrict__ wg_table, int ngroups,
                                                       const double* __restrict__ stage,
                                                       const int32_t* __restrict__ samples,
                                                       float* __restrict__ poses, double* __restrict__ berr,
                                                       float* __restrict__ bpose, unsigned* __restrict__ bctr,
                                                       size_t hcap, int hb) {
    __shared__ __attribute__((aligned(16))) double smem[kBetasWaveSmemDoubles];
    pnp_betas_wave_body<NS>(probs, lps, wg_table, ngroups, hb, stage, samples, poses, berr, bpose, bctr, hcap, smem);
}

// ------------------------------------------------------------------------------------------------
// PnP inlier scan (CheckInliers) — points-stationary, pose broadcast.
// ------------------------------------------------------------------------------------------------
// pnp_inlier (rsc_core.h) for two correspondences at once, in the scan's fast form:
//   * the float rotation, the error and its squared norm run as packed FP32 (v_pk_mul_f32 /
//     v_pk_add_f32: two IEEE operations per instruction, the same roundings as two scalar ones;
//     no contraction, -ffp-contract=off);
//   * invZc = 1/Zc is v_rcp_f32 + one FMA Newton step, which is the correctly rounded reciprocal
//     for every float with 2^-126 <= |z| <= 2^125 (all 2^32 patterns against IEEE 1.0f / z:
//     tools/rcp_exhaustive.hip); the compiler's IEEE division is the same core wrapped in range
//     scaling and special-value fix-ups (10 instructions per point instead of 2).  `ok` is cleared
//     for a point outside that range (0, denormals, huge, inf, NaN), and the caller then redoes the
//     hypothesis with pnp_inlier.
// The projection stays scalar double as the reference's (:253).
typedef float rsc_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pnp_inlier2(const float (&R)[9], const float (&t)[3], double fx, double fy, double cx,
                                            double cy, rsc_f2 X, rsc_f2 Y, rsc_f2 Z, rsc_f2 u, rsc_f2 v, rsc_f2 maxErr,
                                            bool& in0, bool& in1, bool& ok) {
    const rsc_f2 Xc = (R[0] * X + (R[1] * Y + R[2] * Z)) + t[0];  // ered3, then + mti
    const rsc_f2 Yc = (R[3] * X + (R[4] * Y + R[5] * Z)) + t[1];
    const rsc_f2 Zc = (R[6] * X + (R[7] * Y + R[8] * Z)) + t[2];
    const rsc_f2 r0 = {__builtin_amdgcn_rcpf(Zc.x), __builtin_amdgcn_rcpf(Zc.y)};
    const rsc_f2 e = __builtin_elementwise_fma(-Zc, r0, (rsc_f2){1.0f, 1.0f});
    const rsc_f2 iz = __builtin_elementwise_fma(e, r0, r0);
    const float a0 = fabsf(Zc.x), a1 = fabsf(Zc.y);
    ok = ok & (a0 >= 0x1p-126f) & (a0 <= 0x1p125f) & (a1 >= 0x1p-126f) & (a1 <= 0x1p125f);
    const rsc_f2 ue = {(float)(cx + fx * (double)Xc.x * (double)iz.x), (float)(cx + fx * (double)Xc.y * (double)iz.y)};
    const rsc_f2 ve = {(float)(cy + fy * (double)Yc.x * (double)iz.x), (float)(cy + fy * (double)Yc.y * (double)iz.y)};
    const rsc_f2 du = ue - u, dv = ve - v;
    const rsc_f2 e2 = du * du + dv * dv;
    in0 = e2.x < maxErr.x;
    in1 = e2.y < maxErr.y;
}

template <int PPT>
__global__ __launch_bounds__(256) void pnp_scan_kernel(const DevPnP* __restrict__ probs,
                                                       const LaunchProb* __restrict__ lps,
                                                       const int4* __restrict__ wg_table,  // lp, hyp0, count
                                                       const float* __restrict__ poses,
                                                       int32_t* __restrict__ counts,
                                                       int32_t* __restrict__ counts_dev,
                                                       uint64_t* __restrict__ masks, int mask_words,
                                                       int32_t* __restrict__ qual) {
    // Hypotheses per flush: the 4 waves' mask words of a batch wait in LDS (16 KB) until the batch's
    // counts are summed; only hypotheses reaching mRansacMinInliers — the only ones whose inlier
    // mask the host ever adopts (PnPsolver.cpp:176-195) — are stored.  In exhaustive
    // relocalization batches almost none qualify, so the 4.8 MB of mask writes per config-2
    // launch become a few KB.
    constexpr int B = PPT <= 8 ? 64 : 512 / PPT;
    __shared__ int wave_cnt[4][B];
    __shared__ uint64_t mbuf[B][4][PPT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int4 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const DevPnP& P = probs[lp.prob];
    const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy;
    float X[PPT], Y[PPT], Z[PPT], U[PPT], V[PPT], E[PPT];
    RSC_UNROLL for (int s = 0; s < PPT; ++s) {
        const int i = s * 256 + tid;
        if (i < P.n) {
            const float4 p = P.pts[i];
            const float2 q = P.uv[i];
            X[s] = p.x; Y[s] = p.y; Z[s] = p.z; E[s] = p.w * P.th2; U[s] = q.x; V[s] = q.y;  // mvMaxError (:91-93)
        } else {
            X[s] = 0.f; Y[s] = 0.f; Z[s] = 1.f; E[s] = -1.f; U[s] = 0.f; V[s] = 0.f;  // never an inlier
        }
    }
    // The PPT points of a lane are independent: all ballots are taken first and the mask words
    // are kept by lanes 0..PPT-1 in one predicated store, so the compiler can interleave the
    // points' arithmetic (a lane-0 branch per point would serialise them).  The next pose is
    // loaded before the current one is used.
    const float* pp = poses + (size_t)(lp.out0 + wt.y) * 12;
    float Rn[9], tn[3];
    RSC_UNROLL for (int k = 0; k < 9; ++k) Rn[k] = pp[k];
    RSC_UNROLL for (int k = 0; k < 3; ++k) tn[k] = pp[9 + k];
    for (int j = 0; j < wt.z; ++j) {
        float R[9], t[3];
        RSC_UNROLL for (int k = 0; k < 9; ++k) R[k] = Rn[k];
        RSC_UNROLL for (int k = 0; k < 3; ++k) t[k] = tn[k];
        if (j + 1 < wt.z) {
            pp += 12;
            RSC_UNROLL for (int k = 0; k < 9; ++k) Rn[k] = pp[k];
            RSC_UNROLL for (int k = 0; k < 3; ++k) tn[k] = pp[9 + k];
        }
        uint64_t b[PPT];
        if constexpr (PPT >= 2) {
            bool ok = true;
            RSC_UNROLL for (int s = 0; s < PPT; s += 2) {
                bool i0, i1;
                pnp_inlier2(R, t, fx, fy, cx, cy, (rsc_f2){X[s], X[s + 1]}, (rsc_f2){Y[s], Y[s + 1]},
                            (rsc_f2){Z[s], Z[s + 1]}, (rsc_f2){U[s], U[s + 1]}, (rsc_f2){V[s], V[s + 1]},
                            (rsc_f2){E[s], E[s + 1]}, i0, i1, ok);
                b[s] = __ballot(i0);
                b[s + 1] = __ballot(i1);
            }
            // a depth outside the fast reciprocal's range on any lane (a point on the camera
            // plane, a degenerate pose): the whole hypothesis again with the IEEE division
            if (__builtin_expect(__any(!ok), 0)) {
                RSC_UNROLL for (int s = 0; s < PPT; ++s)
                    b[s] = __ballot(pnp_inlier(R, t, fx, fy, cx, cy, X[s], Y[s], Z[s], U[s], V[s], E[s]));
            }
        } else {
            RSC_UNROLL for (int s = 0; s < PPT; ++s)
                b[s] = __ballot(pnp_inlier(R, t, fx, fy, cx, cy, X[s], Y[s], Z[s], U[s], V[s], E[s]));
        }
        int cnt = 0;
        uint64_t mine = 0;
        RSC_UNROLL for (int s = 0; s < PPT; ++s) {
            cnt += __popcll(b[s]);
            mine = (lane == s) ? b[s] : mine;
        }
        const int jb = j % B;
        if (lane < PPT) mbuf[jb][wave][lane] = mine;
        if (lane == 0) wave_cnt[wave][jb] = cnt;
        if (jb == B - 1 || j == wt.z - 1) {
            __syncthreads();
            const int base = j - jb;
            if (tid <= jb) {
                const int c = wave_cnt[0][tid] + wave_cnt[1][tid] + wave_cnt[2][tid] + wave_cnt[3][tid];
                counts[lp.out0 + wt.y + base + tid] = c;
                if (counts_dev) counts_dev[lp.out0 + wt.y + base + tid] = c;  // pnp_select_refine_kernel
                // the problem has a hypothesis reaching mRansacMinInliers: the host replay reads its
                // counts (it skips the counts of a problem without one, rsc_engine.h)
                if (c >= lp.min_inliers) qual[wt.x] = 1;
                wave_cnt[0][tid] = c;  // the batch's totals, for the mask stores below
            }
            __syncthreads();
            if (masks) {
                for (int w = tid; w < (jb + 1) * 4 * PPT; w += 256) {
                    const int hb = w / (4 * PPT), r = w - hb * (4 * PPT), s = r >> 2, wv = r & 3;
                    if (wave_cnt[0][hb] >= lp.min_inliers)
                        masks[(size_t)(lp.out0 + wt.y + base + hb) * mask_words + r] = mbuf[hb][wv][s];
                }
            }
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// PnP Refine: one 256-thread workgroup (4 waves) per refining problem.
//
// EPnP over the n_r best inliers is a chain of left-to-right sums over the rows (arithmetic
// contract: same association as the reference).  The per-row TERMS of every sum are independent,
// so a wave evaluates 64 rows' terms at once into LDS and then K lanes fold the K columns in row
// order (wave_ordered_sum); only the additions stay serial.  The three beta approximations, each
// with its compute_R_and_t over all rows, run on waves 0..2 in parallel.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// s + col[r] + col[r+1] + ... + col[m-1], left to right.  The LDS loads of 16 rows are issued
// before their additions, so the fold runs at the FP64 add latency instead of one LDS round trip
// per row (the refine's folds were LDS-latency-bound: tools/refine_latency_probe.py).
__device__ __forceinline__ double fold_col(double s, const double* col, int r, int m) {
    for (; r + 16 <= m; r += 16) {
        double v[16];
        RSC_UNROLL for (int k = 0; k < 16; ++k) v[k] = col[r + k];
        RSC_UNROLL for (int k = 0; k < 16; ++k) s = s + v[k];
    }
    for (; r < m; ++r) s = s + col[r];
    return s;
}

// Column stride of the fold buffer: 65 doubles, so the K folding lanes read different LDS banks.
constexpr int kFoldStride = 65;

// Lanes of the Refine's 12x12 eigen-solve group (4: a quad; 2: a pair, as the hypothesis eigen
// stage).  Both are bit-identical; for the single solve the quad is faster (single-event refine
// eigen phase 110 us vs 124 us with a pair, tools/refine_latency_probe.py).  RSC_REFINE_EIG_LANES
// overrides at build time for A/B runs.
#ifndef RSC_REFINE_EIG_LANES
#define RSC_REFINE_EIG_LANES 4
#endif
constexpr int kRefineEigLanes = RSC_REFINE_EIG_LANES;
// Refine 12x12 eigen phase in the split form (chase wave + row wave, rsc_quad.h refine_eig12_*)
#ifndef RSC_REFINE_SPLIT
#define RSC_REFINE_SPLIT 0
#endif
// Refine beta waves: the Jacobi SVD's U / V rows distributed over the (uniform) wave's lanes
#ifndef RSC_REFINE_LANE_ROWS
#define RSC_REFINE_LANE_ROWS 1
#endif
constexpr bool kRefineLaneRows = RSC_REFINE_LANE_ROWS != 0;
// Refine ordered sums (control points, pc0, M, error) pipelined over double-buffered blocks
// (profiles/r06/refine_probe_foldstamps_s6f.txt: control points 13.9 -> 12.4 us, pc0 + M/Horn + error
// 24.9 -> 22.6 us on the approximation-3 wave; single event 0.385-0.390 -> 0.382-0.383 ms)
#ifndef RSC_FOLD_PIPE
#define RSC_FOLD_PIPE 1
#endif
// Refine MtM fold with the LDS reads of the next 8 rows issued ahead of the current 8 rows' adds
#ifndef RSC_MTM_PIPELINE
#define RSC_MTM_PIPELINE 1
#endif
static_assert(kRefineEigLanes == 2 || kRefineEigLanes == 4, "refine eigen group: pair or quad");

// Eigen stage in the Refine's rows form for small launches (rsc_quad.h pnp_eig_rows_body; A/B
// variant behind RSC_EIG_ROWS): same workgroup table and stage records as pnp_eig_group_kernel.
template <int NS>
__global__ __launch_bounds__(256) void pnp_eig_rows_kernel(const DevPnP* __restrict__ probs,
                                                           const LaunchProb* __restrict__ lps,
                                                           const int2* __restrict__ wg_table,
                                                           const uint32_t* __restrict__ rng_T,
                                                           double* __restrict__ stage, int32_t* __restrict__ samples) {
    __shared__ __attribute__((aligned(16))) double smem[kEigHyps * kRowsRegion];
    pnp_eig_rows_body<NS, kRefineEigLanes>(probs, lps, wg_table, rng_T, stage, samples, smem, [] { wave_lds_sync(); });
}

#if RSC_FOLD_PIPE
// Ordered sums of K columns of per-row terms over rows [0, count), by one wave: row i's operands are
// v = load(i) (global loads only), its terms term(i, v, t[K]).  Software-pipelined over blocks of 64
// rows with two LDS buffers: while lanes 0..K-1 add block b's terms in order, the wave evaluates block
// b + 1's terms into the other buffer (in the same straight-line block for full blocks, so the term
// arithmetic fills the dependent additions' latency) and block b + 2's loads are in flight; one wave
// barrier per block.  Lanes >= K fold a copy of column K - 1 (discarded), so no exec-mask region
// splits the block.  from_zero: s = ((0.0 + t0) + t1) + ..., else s = (t0 + t1) + ...
// Returns column k's sum in lane k (k < K); buf holds 2 * K * kFoldStride2 doubles of this wave.
constexpr int kFoldStride2 = 66;  // even (16-byte column starts), 132 words: K <= 16 columns on distinct banks
template <int K, class Load, class Term>
__device__ __forceinline__ double wave_ordered_sum(int count, double* buf, bool from_zero, Load&& load, Term&& term) {
    constexpr int CS = kFoldStride2;
    const int lane = threadIdx.x & 63;
    const int colk = lane < K ? lane : K - 1;
    double s = 0.0;
    if (count <= 0) return s;
    const int nb = (count + 63) / 64;
    auto put = [&](int b, const auto& v) {
        double t[K];
        term(min(b * 64 + lane, count - 1), v, t);
        double* dst = buf + (b & 1) * (K * CS) + lane;
        RSC_UNROLL for (int k = 0; k < K; ++k) dst[k * CS] = t[k];
    };
    auto v = load(min(lane, count - 1));
    put(0, v);
    v = load(min(64 + lane, count - 1));  // clamped: a block past the end reloads the last row
    wave_lds_sync();
    for (int b = 0; b < nb; ++b) {
        const double* c = buf + (b & 1) * (K * CS) + colk * CS;
        const bool steady = (b + 1 < nb) & (b * 64 + 64 <= count) & ((b > 0) | from_zero);
        if (steady) {
            // block b + 1's terms and block b's 64 ordered additions in one basic block
            const auto vn = v;
            v = load(min((b + 2) * 64 + lane, count - 1));
            put(b + 1, vn);
            const double2* c2 = reinterpret_cast<const double2*>(c);
            RSC_UNROLL for (int g = 0; g < 4; ++g) {
                double2 x[8];
                RSC_UNROLL for (int q = 0; q < 8; ++q) x[q] = c2[8 * g + q];
                RSC_UNROLL for (int q = 0; q < 8; ++q) {
                    s = s + x[q].x;
                    s = s + x[q].y;
                }
            }
        } else {
            if (b + 1 < nb) {
                const auto vn = v;
                v = load(min((b + 2) * 64 + lane, count - 1));
                put(b + 1, vn);
            }
            const int m = min(64, count - b * 64);
            int r = 0;
            if (b == 0 && !from_zero) {
                s = c[0];
                r = 1;
            }
            s = fold_col(s, c, r, m);
        }
        wave_lds_sync();
    }
    return s;
}
#else
// Ordered sums of K columns of per-row terms over rows [0, count), by one wave: row i's operands are
// v = load(i) (global loads only), its terms term(i, v, t[K]).  The next block's loads are issued
// before the current block is folded, so their latency overlaps the fold's dependent additions.
// from_zero: s = ((0.0 + t0) + t1) + ... (loops starting from 0.0), else s = (t0 + t1) + ...
// Returns column k's sum in lane k (k < K); buf holds kFoldStride*K doubles of this wave.
template <int K, class Load, class Term>
__device__ __forceinline__ double wave_ordered_sum(int count, double* buf, bool from_zero, Load&& load, Term&& term) {
    const int lane = threadIdx.x & 63;
    double s = 0.0;
    auto next = load(min(lane, max(count - 1, 0)));
    for (int base = 0; base < count; base += 64) {
        const int i = base + lane;
        const auto v = next;
        if (i < count) {
            double t[K];
            term(i, v, t);
            RSC_UNROLL for (int k = 0; k < K; ++k) buf[k * kFoldStride + lane] = t[k];
        }
        if (base + 64 < count) next = load(min(i + 64, count - 1));  // in flight during the fold
        wave_lds_sync();
        if (lane < K) {
            const int m = min(64, count - base);
            const double* col = buf + lane * kFoldStride;
            int r = 0;
            if (base == 0 && !from_zero) { s = col[0]; r = 1; }
            s = fold_col(s, col, r, m);
        }
        wave_lds_sync();
    }
    return s;
}

#endif

// Operands of one EPnP row for the Refine's ordered sums (global loads; the unused ones are dead).
struct RefRow {
    double a[4], p[3], u[2];
};

__device__ __forceinline__ void refine_stamp(int slot) {
    if (RSC_REFINE_STAMPS && blockIdx.x < 64 && threadIdx.x == 0) g_refine_stamps[blockIdx.x][slot] = wall_clock64();
}
__device__ __forceinline__ void refine_wave_stamp(int wave, int j) {
    if (RSC_REFINE_STAMPS && blockIdx.x < 64 && (threadIdx.x & 63) == 0)
        g_refine_stamps[blockIdx.x][12 + 4 * wave + j] = wall_clock64();
}

__device__ __forceinline__ void pnp_refine_body(const DevPnP* __restrict__ probs, const RefineJob& J, unsigned* fault) {
    __shared__ __attribute__((aligned(16))) double slab[kSlabDoubles];
#if RSC_FOLD_PIPE
    __shared__ __attribute__((aligned(16))) double wbuf[4][2 * 9 * kFoldStride2];
#else
    __shared__ __attribute__((aligned(16))) double wbuf[4][kFoldStride * 9];
#endif
    __shared__ int prefix[129];
    __shared__ double cen_sh[3], cws_sh[12], cci_sh[9];
    __shared__ double res_sh[3][13];  // per approximation: R[9], t[3], error
    __shared__ float pose_sh[12];
    __shared__ int cnt_sh[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const DevPnP& P = probs[J.prob];
    const int n = P.n;
    const int nwords = (n + 63) / 64;
    double* buf = wbuf[wave];

    refine_stamp(0);
    // 0. new-best bookkeeping (PnPsolver.cpp:147-156) fused here: mvbBestInliers, mBestTcw.
    if (J.adopt_mask)
        for (int wd = tid; wd < nwords; wd += 256) J.adopt_mask[wd] = J.best_mask[wd];
    if (J.adopt_pose && tid < 12) J.out_best_pose[tid] = J.adopt_pose[tid];
    // 1. compaction of the best-inlier set (PnPsolver.cpp:195-214), in index order.  Bits at or
    // above n in the last word are cleared, so the popcount prefix and the scatter agree by
    // construction whatever the mask's padding holds.
    const uint64_t tail = (n & 63) ? (1ull << (n & 63)) - 1ull : ~0ull;
    auto best_word = [&](int wd) {
        const uint64_t m = J.best_mask[wd];
        return wd == nwords - 1 ? (m & tail) : m;
    };
    // exclusive prefix of the mask words' popcounts by wave 0 (one word per lane, wave scan;
    // integer sums, so the order is free)
    if (tid < 64) {
        int carry = 0;
        for (int w0 = 0; w0 < nwords; w0 += 64) {
            const int wd = w0 + lane;
            const int c = wd < nwords ? __popcll(best_word(wd)) : 0;
            int x = c;
            RSC_UNROLL for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            if (wd < nwords) prefix[wd] = carry + x - c;
            carry += __shfl(x, 63);
        }
        if (lane == 0) prefix[nwords] = carry;
    }
    __syncthreads();
    const int nr = prefix[nwords];
    // one thread per correspondence: its row is the word's prefix + the set bits below it
    for (int i = tid; i < n; i += 256) {
        const int wd = i >> 6, b = i & 63;
        const uint64_t m = best_word(wd);
        if ((m >> b) & 1ull) {
            const int r = prefix[wd] + __popcll(m & ((1ull << b) - 1ull));
            const float4 p = P.pts[i];
            const float2 q = P.uv[i];
            P.pws[3 * r + 0] = p.x; P.pws[3 * r + 1] = p.y; P.pws[3 * r + 2] = p.z;
            P.us[2 * r + 0] = q.x; P.us[2 * r + 1] = q.y;
        }
    }
    // set_maximum_number_of_correspondences(nr): growth zero-fills (the rows beyond nr do not
    // exist after growth; rows = nr).  Without growth the rows beyond nr stay stale (Q6).
    const int rows = J.rows_after;
    __syncthreads();
    refine_stamp(1);

    const double* __restrict__ pws = P.pws;
    const double* __restrict__ us = P.us;
    double* __restrict__ als = P.als;
    RowStore st{nr, rows, P.pws, P.us, P.als};
    const Intrinsics K{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy};
    LaneMat S{slab, 1};
    // 2. choose_control_points + barycentric coordinates (PnPsolver.cpp:296-343), wave 0
    if (wave == 0) {
        auto ld_p = [&](int i) { return RefRow{{0, 0, 0, 0}, {pws[3 * i], pws[3 * i + 1], pws[3 * i + 2]}, {0, 0}}; };
        const double cs = wave_ordered_sum<3>(rows, buf, false, ld_p, [&](int, const RefRow& v, double (&t)[3]) {
            t[0] = v.p[0]; t[1] = v.p[1]; t[2] = v.p[2];
        });
        if (lane < 3) cen_sh[lane] = cs / nr;
        wave_lds_sync();
        const double c0 = cen_sh[0], c1 = cen_sh[1], c2 = cen_sh[2];
        // A[a][b], (a,b) in (00 01 02 11 12 22); A[b][a] is the same sum of the same products
        const double as = wave_ordered_sum<6>(nr, buf, false, ld_p, [&](int, const RefRow& v, double (&t)[6]) {
            const double d0 = v.p[0] - c0, d1 = v.p[1] - c1, d2 = v.p[2] - c2;
            t[0] = d0 * d0; t[1] = d0 * d1; t[2] = d0 * d2; t[3] = d1 * d1; t[4] = d1 * d2; t[5] = d2 * d2;
        });
        if (lane < 6) buf[lane] = as;
        wave_lds_sync();
        // the 3x3 eigensolver, control points and C^-1 on every lane of the wave (identical values
        // and writes): a uniform chain runs with scalar branches, about twice as fast as the same
        // chain on one lane under an exec mask (tools/eig_probe.hip refine_betas_like)
        {
            double cws[4][3];
            cws[0][0] = c0; cws[0][1] = c1; cws[0][2] = c2;
            const double A[3][3] = {{buf[0], buf[1], buf[2]}, {buf[1], buf[3], buf[4]}, {buf[2], buf[4], buf[5]}};
            double V[3][3], w[3];
            sym_eig_reg<double, 3>(A, V, w);
            RSC_UNROLL for (int i = 0; i < 3; ++i) {
                double k = sqrt(w[i] / nr);
                RSC_UNROLL for (int c = 0; c < 3; ++c) cws[i + 1][c] = cws[0][c] + k * V[c][i];
            }
            double CC[3][3], CCi[3][3];
            RSC_UNROLL for (int i = 0; i < 3; ++i)
                RSC_UNROLL for (int j = 1; j < 4; ++j) CC[i][j - 1] = cws[j][i] - cws[0][i];
            inverse3(CC, CCi);
            RSC_UNROLL for (int i = 0; i < 4; ++i)
                RSC_UNROLL for (int c = 0; c < 3; ++c) cws_sh[3 * i + c] = cws[i][c];
            RSC_UNROLL for (int i = 0; i < 3; ++i)
                RSC_UNROLL for (int c = 0; c < 3; ++c) cci_sh[3 * i + c] = CCi[i][c];
        }
    }
    __syncthreads();
    for (int i = tid; i < nr; i += 256) {
        const double d0 = pws[3 * i] - cws_sh[0], d1 = pws[3 * i + 1] - cws_sh[1], d2 = pws[3 * i + 2] - cws_sh[2];
        const double a1 = ered3(cci_sh[0] * d0, cci_sh[1] * d1, cci_sh[2] * d2);  // :338, ered3
        const double a2 = ered3(cci_sh[3] * d0, cci_sh[4] * d1, cci_sh[5] * d2);
        const double a3 = ered3(cci_sh[6] * d0, cci_sh[7] * d1, cci_sh[8] * d2);
        als[4 * i + 1] = a1;
        als[4 * i + 2] = a2;
        als[4 * i + 3] = a3;
        als[4 * i + 0] = 1.0 - a1 - a2 - a3;
    }
    __threadfence_block();
    __syncthreads();
    refine_stamp(2);
    // 3. MtM lower triangle, one entry per folding thread, each folded over the 2*nr rows in order.
#if RSC_MTM_PIPELINE
    // The rows of M are staged through LDS in chunks of 128 correspondences (256 rows), column-major
    // (column j of the chunk at j * kMtmRS, rows contiguous; kMtmRS = 258 doubles puts the 12 columns
    // on different LDS banks) and double-buffered: lanes 0..38 of waves 0 and 1 fold chunk c (the 78
    // entries) while waves 2 and 3 stage chunk c + 1, one correspondence (its two rows of M,
    // PnPsolver.cpp:365-377, the values of M_entry) per thread, one 16-byte store per column.  A
    // folder reads two rows of each of its columns per 16-byte load and issues the next 8 rows' loads
    // before adding the current 8 products, so the LDS round trip stays off the ordered add chain.
    {
        constexpr int kPairs = 128, kMtmRS = 2 * kPairs + 2;
        __shared__ __attribute__((aligned(16))) double mtm_buf[2][12 * kMtmRS];
        const bool folder = wave < 2 && lane < 39;
        int a = 0, b = wave * 39 + lane;
        while (b > a) { b -= a + 1; ++a; }  // fold id -> (a,b) with b <= a, row-major lower triangle
        const int nchunks = (nr + kPairs - 1) / kPairs;
        auto stage = [&](int c, int t0, int nt) {
            const int i0 = c * kPairs, m = min(kPairs, nr - i0);
            double* dst = mtm_buf[c & 1];
            for (int t = t0; t < m; t += nt) {
                const int i = i0 + t;
                const double al4[4] = {als[4 * i], als[4 * i + 1], als[4 * i + 2], als[4 * i + 3]};
                const double u0 = us[2 * i], u1 = us[2 * i + 1];
                RSC_UNROLL for (int j = 0; j < 4; ++j) {  // (row 2i, row 2i + 1) of columns 3j .. 3j + 2
                    *reinterpret_cast<double2*>(dst + (3 * j) * kMtmRS + 2 * t) = double2{al4[j] * K.fx, 0.0};
                    *reinterpret_cast<double2*>(dst + (3 * j + 1) * kMtmRS + 2 * t) = double2{0.0, al4[j] * K.fy};
                    *reinterpret_cast<double2*>(dst + (3 * j + 2) * kMtmRS + 2 * t) =
                        double2{al4[j] * (K.cx - u0), al4[j] * (K.cy - u1)};
                }
            }
        };
        if (nchunks > 0) stage(0, tid, 256);
        __syncthreads();
        double s = 0.0;
        for (int c = 0; c < nchunks; ++c) {
            if (wave >= 2 && c + 1 < nchunks) stage(c + 1, tid - 128, 128);
            if (folder) {
                const double* Ma = mtm_buf[c & 1] + a * kMtmRS;
                const double* Mb = mtm_buf[c & 1] + b * kMtmRS;
                const int m = 2 * min(kPairs, nr - c * kPairs);  // even, >= 2
                int r = 0;
                if (c == 0) {
                    s = Ma[0] * Mb[0];
                    s = s + Ma[1] * Mb[1];
                    r = 2;
                }
                if (r + 8 <= m) {
                    double p[8];
                    RSC_UNROLL for (int k = 0; k < 4; ++k) {
                        const double2 x = *reinterpret_cast<const double2*>(Ma + r + 2 * k);
                        const double2 y = *reinterpret_cast<const double2*>(Mb + r + 2 * k);
                        p[2 * k] = x.x * y.x;
                        p[2 * k + 1] = x.y * y.y;
                    }
                    for (r += 8; r + 8 <= m; r += 8) {
                        double2 x[4], y[4];
                        RSC_UNROLL for (int k = 0; k < 4; ++k) {
                            x[k] = *reinterpret_cast<const double2*>(Ma + r + 2 * k);
                            y[k] = *reinterpret_cast<const double2*>(Mb + r + 2 * k);
                        }
                        RSC_UNROLL for (int k = 0; k < 8; ++k) s = s + p[k];
                        RSC_UNROLL for (int k = 0; k < 4; ++k) {
                            p[2 * k] = x[k].x * y[k].x;
                            p[2 * k + 1] = x[k].y * y[k].y;
                        }
                    }
                    RSC_UNROLL for (int k = 0; k < 8; ++k) s = s + p[k];
                }
                for (; r < m; ++r) s = s + Ma[r] * Mb[r];
            }
            __syncthreads();  // chunk c folded, chunk c + 1 staged
        }
        if (folder) S.at(a, b) = s;
    }
#else
    // The rows of M are staged through LDS in chunks of 97 correspondences (194 rows x 12),
    // double-buffered: lanes 0..38 of waves 0 and 1 fold chunk c (the 78 entries) while waves 2 and 3
    // stage chunk c + 1, one correspondence (its two rows of M, PnPsolver.cpp:365-377, the values of
    // M_entry) per thread, so the chunk's operand loads are one round trip (one barrier per chunk).
    {
        constexpr int kPairs = (4 * kFoldStride * 9) / 24;  // 97 correspondences per chunk
        __shared__ __attribute__((aligned(16))) double mtm_stage2[kPairs * 24];
        auto chunk_buf = [&](int c) { return (c & 1) ? mtm_stage2 : &wbuf[0][0]; };
        const bool folder = wave < 2 && lane < 39;
        int a = 0, b = wave * 39 + lane;
        while (b > a) { b -= a + 1; ++a; }  // fold id -> (a,b) with b <= a, row-major lower triangle
        const int nchunks = (nr + kPairs - 1) / kPairs;
        auto stage = [&](int c, int t0, int nt) {
            const int i0 = c * kPairs, m = min(kPairs, nr - i0);
            double* dst = chunk_buf(c);
            for (int t = t0; t < m; t += nt) {
                const int i = i0 + t;
                const double al4[4] = {als[4 * i], als[4 * i + 1], als[4 * i + 2], als[4 * i + 3]};
                const double u0 = us[2 * i], u1 = us[2 * i + 1];
                double* ev = dst + 24 * t;  // row 2i
                double* od = ev + 12;       // row 2i + 1
                RSC_UNROLL for (int j = 0; j < 4; ++j) {
                    ev[3 * j] = al4[j] * K.fx;
                    ev[3 * j + 1] = 0.0;
                    ev[3 * j + 2] = al4[j] * (K.cx - u0);
                    od[3 * j] = 0.0;
                    od[3 * j + 1] = al4[j] * K.fy;
                    od[3 * j + 2] = al4[j] * (K.cy - u1);
                }
            }
        };
        if (nchunks > 0) stage(0, tid, 256);
        __syncthreads();
        double s = 0.0;
        for (int c = 0; c < nchunks; ++c) {
            if (wave >= 2 && c + 1 < nchunks) stage(c + 1, tid - 128, 128);
            if (folder) {
                const double* M = chunk_buf(c);
                const int m = 2 * min(kPairs, nr - c * kPairs);
                int r = 0;
                if (c == 0) {
                    s = M[a] * M[b];
                    r = 1;
                }
                // 8 rows' operands loaded before their products and ordered additions
                for (; r + 8 <= m; r += 8) {
                    double x[8], y[8];
                    RSC_UNROLL for (int k = 0; k < 8; ++k) { x[k] = M[(r + k) * 12 + a]; y[k] = M[(r + k) * 12 + b]; }
                    RSC_UNROLL for (int k = 0; k < 8; ++k) s = s + x[k] * y[k];
                }
                for (; r < m; ++r) s = s + M[r * 12 + a] * M[r * 12 + b];
            }
            __syncthreads();  // chunk c folded, chunk c + 1 staged
        }
        if (folder) S.at(a, b) = s;
    }
#endif
    __syncthreads();
    refine_stamp(3);
    // 4. 12x12 eigenvectors (rows_eig12_ev4: Householder phases on lanes 0..kRefineEigLanes-1 of
    // wave 0 as one lane group, the QR chase on lanes 0..11 with one row of Q in each lane's VGPRs),
    // then L_6x10 and rho (single lane).  The MtM lower triangle in the slab is the group's T region;
    // wbuf the E scratch.  The eigenvector columns 0..3 go back to slab columns 0..3 (SlabView::ev).
#if RSC_REFINE_SPLIT
    // split form (rsc_quad.h refine_eig12_*): phases B-C on wave 0, then the chase on lane 0 of wave 0
    // and the Q rows on lanes 0..11 of wave 1, hand-off through a SplitRing in wbuf[1]
    {
        __shared__ int rpub, rack;
        if (tid == 0) { rpub = 0; rack = 0; }
        if (wave == 0) refine_eig12_bc<kRefineEigLanes>(slab, &wbuf[0][0], lane, [] { wave_lds_sync(); });
        __syncthreads();
        if (RSC_REFINE_STAMPS && blockIdx.x < 64 && tid == 0)
            g_refine_stamps[blockIdx.x][8] = g_refine_stamps[blockIdx.x][9] = wall_clock64();
        if (wave == 0) {
            if (lane == 0) refine_eig12_chase(&wbuf[0][0], &wbuf[1][0], &rpub, &rack, fault);
            if (RSC_REFINE_STAMPS && blockIdx.x < 64 && tid == 0) g_refine_stamps[blockIdx.x][10] = wall_clock64();
        } else if (wave == 1 && lane < 12) {
            double ev[4];
            refine_eig12_rows(slab, &wbuf[1][0], &rpub, &rack, fault, lane, ev);
            RSC_UNROLL for (int c = 0; c < 4; ++c) slab[lane * 12 + c] = ev[c];
        }
        __syncthreads();
        if (RSC_REFINE_STAMPS && blockIdx.x < 64 && tid == 0) g_refine_stamps[blockIdx.x][11] = wall_clock64();
    }
#else
    if (wave == 0) {
        double ev[4];
        rows_eig12_ev4<kRefineEigLanes>(slab, &wbuf[0][0], lane, [] { wave_lds_sync(); }, ev);
        if (lane < 12) RSC_UNROLL for (int c = 0; c < 4; ++c) slab[lane * 12 + c] = ev[c];
    }
    __syncthreads();
#endif
    if (wave == 0) {  // every lane of wave 0, identical values and writes
        compute_L_6x10(SlabView{S});
        auto d2 = [&](int a, int b) {
            double x = cws_sh[3 * a] - cws_sh[3 * b], y = cws_sh[3 * a + 1] - cws_sh[3 * b + 1],
                   z = cws_sh[3 * a + 2] - cws_sh[3 * b + 2];
            return ered3(x * x, y * y, z * z);  // squaredNorm of a row of cws (:640-645)
        };
        const SlabView SV{S};
        SV.rho(0) = d2(0, 1); SV.rho(1) = d2(0, 2); SV.rho(2) = d2(0, 3);
        SV.rho(3) = d2(1, 2); SV.rho(4) = d2(1, 3); SV.rho(5) = d2(2, 3);
    }
    __syncthreads();
    refine_stamp(4);
    // 5. beta approximation (wave + 1), Gauss-Newton, compute_R_and_t over all rows
    if (wave < 3) {
        const SlabView SV{S};
        __shared__ double ccs_sh[3][12];
        {  // every lane of the wave (identical values and writes; see the control points above)
            double betas[4] = {0.0, 0.0, 0.0, 0.0};
            if (wave == 0) find_betas<1, SlabView, kRefineLaneRows>(SV, betas);
            else if (wave == 1) find_betas<2, SlabView, kRefineLaneRows>(SV, betas);
            else find_betas<3, SlabView, kRefineLaneRows>(SV, betas);
            gauss_newton(SV, betas);
            double ccs[4][3];
            ccs_with_sign(st, SV, betas, ccs);
            RSC_UNROLL for (int i = 0; i < 4; ++i)
                RSC_UNROLL for (int c = 0; c < 3; ++c) ccs_sh[wave][3 * i + c] = ccs[i][c];
        }
        wave_lds_sync();
        refine_wave_stamp(wave, 0);
        double ccs[4][3];
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) ccs[i][c] = ccs_sh[wave][3 * i + c];
        const double pw0[3] = {cws_sh[0], cws_sh[1], cws_sh[2]};
        // pc0 over all allocated rows (stale rows use their stale alphas, Q6)
        auto ld_a = [&](int i) {
            return RefRow{{als[4 * i], als[4 * i + 1], als[4 * i + 2], als[4 * i + 3]}, {0, 0, 0}, {0, 0}};
        };
        const double ps = wave_ordered_sum<3>(rows, buf, false, ld_a, [&](int, const RefRow& v, double (&t)[3]) {
            RSC_UNROLL for (int c = 0; c < 3; ++c) t[c] = pcs_of(v.a, ccs, c);
        });
        __shared__ double pc0_sh[3][3];
        if (lane < 3) pc0_sh[wave][lane] = ps / nr;
        wave_lds_sync();
        refine_wave_stamp(wave, 1);
        const double pc0[3] = {pc0_sh[wave][0], pc0_sh[wave][1], pc0_sh[wave][2]};
        auto ld_ap = [&](int i) {
            return RefRow{{als[4 * i], als[4 * i + 1], als[4 * i + 2], als[4 * i + 3]},
                          {pws[3 * i], pws[3 * i + 1], pws[3 * i + 2]}, {0, 0}};
        };
        const double ms = wave_ordered_sum<9>(nr, buf, true, ld_ap, [&](int, const RefRow& v, double (&t)[9]) {
            double a[3], b[3];
            RSC_UNROLL for (int c = 0; c < 3; ++c) { a[c] = pcs_of(v.a, ccs, c) - pc0[c]; b[c] = v.p[c] - pw0[c]; }
            RSC_UNROLL for (int r = 0; r < 3; ++r)
                RSC_UNROLL for (int c = 0; c < 3; ++c) t[3 * r + c] = a[r] * b[c];
        });
        __shared__ double m_sh[3][9];
        if (lane < 9) m_sh[wave][lane] = ms;
        wave_lds_sync();
        __shared__ double rt_sh[3][12];
        {  // every lane of the wave, as above
            double M[3][3], R[3][3], t[3];
            RSC_UNROLL for (int r = 0; r < 3; ++r)
                RSC_UNROLL for (int c = 0; c < 3; ++c) M[r][c] = m_sh[wave][3 * r + c];
            horn_from_M(M, pc0, pw0, R, t);
            RSC_UNROLL for (int k = 0; k < 9; ++k) rt_sh[wave][k] = R[k / 3][k % 3];
            RSC_UNROLL for (int k = 0; k < 3; ++k) rt_sh[wave][9 + k] = t[k];
        }
        wave_lds_sync();
        refine_wave_stamp(wave, 2);
        double R[3][3], t[3];
        RSC_UNROLL for (int k = 0; k < 9; ++k) R[k / 3][k % 3] = rt_sh[wave][k];
        RSC_UNROLL for (int k = 0; k < 3; ++k) t[k] = rt_sh[wave][9 + k];
        auto ld_pu = [&](int i) {
            return RefRow{{0, 0, 0, 0}, {pws[3 * i], pws[3 * i + 1], pws[3 * i + 2]}, {us[2 * i], us[2 * i + 1]}};
        };
        const double es = wave_ordered_sum<1>(nr, buf, true, ld_pu, [&](int, const RefRow& v, double (&tt)[1]) {
            tt[0] = reproj_term(R, t, K, v.p[0], v.p[1], v.p[2], v.u[0], v.u[1]);
        });
        if (lane == 0) {
            RSC_UNROLL for (int k = 0; k < 12; ++k) res_sh[wave][k] = rt_sh[wave][k];
            res_sh[wave][12] = es / nr;
        }
        refine_wave_stamp(wave, 3);
    }
    __syncthreads();
    refine_stamp(5);
    // smallest reprojection error, approximations in order 1, 2, 3 (strict <, PnPsolver.cpp:405-411)
    if (tid == 0) {
        int b = 0;
        if (res_sh[1][12] < res_sh[b][12]) b = 1;
        if (res_sh[2][12] < res_sh[b][12]) b = 2;
        RSC_UNROLL for (int k = 0; k < 12; ++k) pose_sh[k] = (float)res_sh[b][k];
    }
    __syncthreads();
    // 6. CheckInliers of the refined pose
    float R[9], t[3];
    RSC_UNROLL for (int k = 0; k < 9; ++k) R[k] = pose_sh[k];
    RSC_UNROLL for (int k = 0; k < 3; ++k) t[k] = pose_sh[9 + k];
    int cnt = 0;
    const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy;
    // the solver's own mask words only (a launch can hold solvers of different N)
    const int mask_words_out = J.out_words;
    for (int base = 0; base < mask_words_out * 64; base += 256) {
        const int i = base + tid;
        bool inl = false;
        if (i < n) {
            const float4 p = P.pts[i];
            const float2 q = P.uv[i];
            inl = pnp_inlier(R, t, fx, fy, cx, cy, p.x, p.y, p.z, q.x, q.y, p.w * P.th2);
        }
        const uint64_t b = __ballot(inl);
        cnt += __popcll(b);
        if (lane == 0 && (base / 64 + wave) < mask_words_out) J.out_mask[base / 64 + wave] = b;
    }
    if (lane == 0) cnt_sh[wave] = cnt;
    __syncthreads();
    refine_stamp(6);
    if (tid == 0) {
        *J.out_count = cnt_sh[0] + cnt_sh[1] + cnt_sh[2] + cnt_sh[3];
        RSC_UNROLL for (int k = 0; k < 12; ++k) J.out_pose[k] = pose_sh[k];
    }
}

__global__ __launch_bounds__(256) void pnp_refine_kernel(const DevPnP* __restrict__ probs,
                                                         const RefineJob* __restrict__ jobs, unsigned* fault) {
    const RefineJob J = jobs[blockIdx.x];
    pnp_refine_body(probs, J, fault);
}

// The host replay's first pause of a speculation round, evaluated on the device right after the scan
// (one workgroup per solver of the round), and its Refine() run at once — no host round trip between
// the scan and the Refine.  PnPsolver.cpp:139-157 for the round's hypotheses [0, H): the first k with
// nInliers >= mRansacMinInliers pauses the loop; it becomes the new best when nInliers > mnBestInliers
// (best0: the value when the round was launched), and Refine() runs on mvbBestInliers with
// set_maximum_number_of_correspondences(max(rows0, mnBestInliers)).  The host replay applies the
// same rules to the same counts and takes these results (RefineSelOut) instead of launching the
// refine itself; a solver without a qualifying hypothesis leaves k = -1 and touches nothing.
__global__ __launch_bounds__(256) void pnp_select_refine_kernel(const DevPnP* __restrict__ probs,
                                                                const RefineSel* __restrict__ sels,
                                                                const int32_t* __restrict__ counts,
                                                                uint64_t* __restrict__ masks, int mask_words,
                                                                const float* __restrict__ poses,
                                                                RefineSelOut* __restrict__ out, unsigned* fault) {
    __shared__ int k_sh;
    const RefineSel S = sels[blockIdx.x];
    const int tid = threadIdx.x;
    if (tid < 64) {
        int k = -1;
        for (int base = 0; base < S.H && k < 0; base += 64) {  // wave-uniform loop
            const int idx = base + tid;
            const bool q = idx < S.H && counts[S.out0 + idx] >= S.min_inliers;
            const uint64_t b = __ballot(q);
            if (b) k = base + __ffsll((unsigned long long)b) - 1;
        }
        if (tid == 0) k_sh = k;
    }
    __syncthreads();
    const int k = k_sh;
    RefineSelOut& o = out[blockIdx.x];
    if (k < 0) {
        if (tid == 0) o.k = -1;
        return;
    }
    const size_t rec = (size_t)(S.out0 + k);
    const int c = counts[rec];
    const bool adopt = c > S.best0;
    const int nr = adopt ? c : S.best0;
    RefineJob J;
    J.prob = S.prob;
    J.rows_after = max(S.rows0, nr);
    J.best_mask = adopt ? masks + rec * mask_words : S.best;
    J.adopt_mask = adopt ? S.best : nullptr;
    J.adopt_pose = adopt ? poses + rec * 12 : nullptr;
    J.out_best_pose = o.best_pose;
    J.out_pose = o.pose;
    J.out_count = &o.count;
    J.out_mask = S.refined;
    J.out_words = S.words;
    if (tid == 0) {
        o.k = k;
        o.adopt = adopt ? 1 : 0;
        o.rows_after = J.rows_after;
    }
    pnp_refine_body(probs, J, fault);
}

// ------------------------------------------------------------------------------------------------
// Sim3 hypotheses + scan
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void sim3_solve_kernel(const DevSim3* __restrict__ probs,
                                                        const LaunchProb* __restrict__ lps,
                                                        const int2* __restrict__ wg_table,
                                                        const uint32_t* __restrict__ rng_T,
                                                        float* __restrict__ poses, int32_t* __restrict__ samples) {
    const int lane = threadIdx.x;
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const int h = wt.y + lane;
    if (h >= lp.H) return;
    const DevSim3& P = probs[lp.prob];
    uint32_t w[31];
    RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
    uint32_t words[3];
    RSC_UNROLL for (int d = 0; d < 3; ++d) words[d] = rng_word(rng_T, w, lp.g0 + h * 3 + d);
    int idx[3];
    swap_remove_sample<3>(words, 3, P.n, idx);
    float P1[3][3], P2[3][3];
    RSC_UNROLL for (int i = 0; i < 3; ++i) {
        const float4 a = P.x1[idx[i]];
        const float4 b = P.x2[idx[i]];
        P1[0][i] = a.x; P1[1][i] = a.y; P1[2][i] = a.z;
        P2[0][i] = b.x; P2[1][i] = b.y; P2[2][i] = b.z;
    }
    Sim3Pose T;
    sim3_compute(P1, P2, T);
    float* out = poses + (size_t)(lp.out0 + h) * 24;
    RSC_UNROLL for (int k = 0; k < 9; ++k) out[k] = T.R12[k];
    RSC_UNROLL for (int k = 0; k < 3; ++k) out[9 + k] = T.t12[k];
    RSC_UNROLL for (int k = 0; k < 9; ++k) out[12 + k] = T.R21[k];
    RSC_UNROLL for (int k = 0; k < 3; ++k) out[21 + k] = T.t21[k];
    if (samples) {
        RSC_UNROLL for (int i = 0; i < 3; ++i) samples[(size_t)(lp.out0 + h) * 8 + i] = idx[i];
    }
}

template <int PPT>
__global__ __launch_bounds__(256) void sim3_scan_kernel(const DevSim3* __restrict__ probs,
                                                        const LaunchProb* __restrict__ lps,
                                                        const int4* __restrict__ wg_table,
                                                        const float* __restrict__ poses,
                                                        int32_t* __restrict__ counts,
                                                        int32_t* __restrict__ counts_dev,
                                                        uint64_t* __restrict__ masks, int mask_words) {
    __shared__ int wave_cnt[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int4 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const DevSim3& P = probs[lp.prob];
    const float K1[4] = {P.K1[0], P.K1[1], P.K1[2], P.K1[3]};
    const float K2[4] = {P.K2[0], P.K2[1], P.K2[2], P.K2[3]};
    float A[PPT][3], B[PPT][3], p1u[PPT], p1v[PPT], p2u[PPT], p2v[PPT], e1[PPT], e2[PPT];
    RSC_UNROLL for (int s = 0; s < PPT; ++s) {
        const int i = s * 256 + tid;
        if (i < P.n) {
            const float4 a = P.x1[i], b = P.x2[i], pp = P.pim[i];
            A[s][0] = a.x; A[s][1] = a.y; A[s][2] = a.z; e1[s] = a.w;
            B[s][0] = b.x; B[s][1] = b.y; B[s][2] = b.z; e2[s] = b.w;
            p1u[s] = pp.x; p1v[s] = pp.y; p2u[s] = pp.z; p2v[s] = pp.w;
        } else {
            A[s][0] = A[s][1] = 0.f; A[s][2] = 1.f; B[s][0] = B[s][1] = 0.f; B[s][2] = 1.f;
            e1[s] = e2[s] = -1.f; p1u[s] = p1v[s] = p2u[s] = p2v[s] = 0.f;
        }
    }
    for (int j = 0; j < wt.z; ++j) {
        const int h = wt.y + j;
        const float* pp = poses + (size_t)(lp.out0 + h) * 24;
        Sim3Pose T;
        RSC_UNROLL for (int k = 0; k < 9; ++k) { T.R12[k] = pp[k]; T.R21[k] = pp[12 + k]; }
        RSC_UNROLL for (int k = 0; k < 3; ++k) { T.t12[k] = pp[9 + k]; T.t21[k] = pp[21 + k]; }
        // all PPT ballots first, then one predicated store by lanes 0..PPT-1 (as the PnP scan)
        uint64_t b[PPT];
        RSC_UNROLL for (int s = 0; s < PPT; ++s)
            b[s] = __ballot(sim3_inlier(T, K1, K2, A[s], B[s], p1u[s], p1v[s], p2u[s], p2v[s], e1[s], e2[s]));
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
                if (counts_dev) counts_dev[lp.out0 + wt.y + base + tid] = c;  // for sim3_pick_kernel
            }
            __syncthreads();
        }
    }
}

// Gather `take` floats of records idx[q] (record stride `stride` floats) into dst[q][take].
__global__ void gather_records_kernel(const float* __restrict__ src, int stride, int take,
                                      const int32_t* __restrict__ idx, int n, float* __restrict__ dst) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * take) return;
    const int q = t / take, e = t - q * take;
    dst[t] = src[(size_t)idx[q] * stride + e];
}

// Sim3Solver::iterate (Sim3Solver.cpp:155-166) keeps the hypothesis with nInliers >= mnBestInliers
// (later ties win) and returns at the first one with nInliers > mRansacMinInliers.  Evaluated after
// the scan, one workgroup per solver, so the kept pose comes back with the counts instead of in a
// second round trip after the host replay (which still decides; the backend serves the pose from
// here when the replay kept the same index).  In parallel: hypothesis k updates the best iff
// c_k >= max(best0, c_0..c_k-1) (a prefix maximum over per-thread chunks); the return index r is
// the first update with c_k > minInliers; the kept index is the last update <= r.
__global__ __launch_bounds__(256) void sim3_pick_kernel(const LaunchProb* __restrict__ lps,
                                                        const int32_t* __restrict__ counts,
                                                        const float* __restrict__ poses, float* __restrict__ pick) {
    constexpr int T = 256, PER = kPickMaxH / T;
    __shared__ int pre[T];
    __shared__ int ret_k, keep_k;
    const int tid = threadIdx.x;
    const LaunchProb& lp = lps[blockIdx.x];
    const int H = lp.H;
    const int per = (H + T - 1) / T;  // <= PER: contiguous chunk [tid*per, tid*per + per)
    int c[PER];
    int mx = INT_MIN;
    RSC_UNROLL for (int u = 0; u < PER; ++u) {
        const int k = tid * per + u;
        c[u] = (u < per && k < H) ? counts[lp.out0 + k] : INT_MIN;
        mx = max(mx, c[u]);
    }
    pre[tid] = mx;
    if (tid == 0) { ret_k = INT_MAX; keep_k = -1; }
    __syncthreads();
    for (int d = 1; d < T; d <<= 1) {  // inclusive prefix maximum of the chunk maxima
        const int v = (tid >= d) ? pre[tid - d] : INT_MIN;
        __syncthreads();
        pre[tid] = max(pre[tid], v);
        __syncthreads();
    }
    int run = max(lp.best0, tid > 0 ? pre[tid - 1] : INT_MIN);  // best before this chunk
    int my_ret = INT_MAX;
    RSC_UNROLL for (int u = 0; u < PER; ++u) {
        const int k = tid * per + u;
        if (u < per && k < H && c[u] >= run) {
            run = c[u];
            if (c[u] > lp.min_inliers) my_ret = min(my_ret, k);
        }
    }
    atomicMin(&ret_k, my_ret);  // LDS atomics
    __syncthreads();
    const int r = ret_k;
    run = max(lp.best0, tid > 0 ? pre[tid - 1] : INT_MIN);
    int my_keep = -1;
    RSC_UNROLL for (int u = 0; u < PER; ++u) {
        const int k = tid * per + u;
        if (u < per && k < H && k <= r && c[u] >= run) {
            run = c[u];
            my_keep = k;
        }
    }
    atomicMax(&keep_k, my_keep);
    __syncthreads();
    const int k = keep_k;
    float* o = pick + (size_t)blockIdx.x * 16;
    if (tid == 0) reinterpret_cast<int32_t*>(o)[0] = k;
    if (k >= 0 && tid < 12) o[1 + tid] = poses[(size_t)(lp.out0 + k) * 24 + tid];
}

hipError_t launch_sim3_pick(int count, const LaunchProb* lps, const int32_t* counts, const float* poses,
                            float* pick, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    sim3_pick_kernel<<<count, 256, 0, st>>>(lps, counts, poses, pick);
    return hipGetLastError();
}

hipError_t launch_gather_records(const float* src, int stride, int take, const int32_t* idx, int n, float* dst,
                                 hipStream_t st) {
    if (n <= 0) return hipSuccess;
    gather_records_kernel<<<(n * take + 255) / 256, 256, 0, st>>>(src, stride, take, idx, n, dst);
    return hipGetLastError();
}

// rand() outputs straight from the jump table (parity hook for the RNG contract).
__global__ void rng_stream_kernel(const uint32_t* __restrict__ T, Window31 w, int g0, int n, int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t ww[31];
    RSC_UNROLL for (int j = 0; j < 31; ++j) ww[j] = w.w[j];
    out[i] = (int32_t)(rng_word(T, ww, g0 + i) >> 1);
}

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
// The rows-form eigen stage exists only for the 20-hypothesis workgroup (4 waves x 5 twelve-lane
// groups); builds with another RSC_EIG_HYPS compile without it and refuse the variant.
template <int N>
static hipError_t launch_eig_rows(int nwgE, const int2* wgtE, const DevPnP* probs, const LaunchProb* lps,
                                  const uint32_t* T, double* stage, int32_t* samples, hipStream_t st) {
    if constexpr (kEigHyps == 4 * kRowsGroups) {
        pnp_eig_rows_kernel<N><<<nwgE, 256, 0, st>>>(probs, lps, wgtE, T, stage, samples);
        return hipSuccess;
    } else {
        return hipErrorInvalidValue;
    }
}

hipError_t launch_pnp_solve_split(int ns, int nwgE, const int2* wgtE, int nwgB, const int2* wgtB,
                                  const DevPnP* probs, const LaunchProb* lps, const uint32_t* T, double* stage,
                                  float* poses, int32_t* samples, const BetasScratch& bs, hipStream_t st,
                                  hipEvent_t eig_begin, hipEvent_t eig_end, bool eig_rows, bool eig_split,
                                  unsigned* fault, int betas_hb) {
    if (ns < 4 || ns > 6 || betas_hb < 1 || betas_hb > kBetasHyps) return hipErrorInvalidValue;
    if (eig_split && !eig_rows && !fault) return hipErrorInvalidValue;
    if (eig_begin) (void)hipEventRecord(eig_begin, st);
    switch (ns) {
#define RSC_CASE(N)                                                                                   \
    case N:                                                                                           \
        if (eig_rows) {                                                                               \
            const hipError_t e = launch_eig_rows<N>(nwgE, wgtE, probs, lps, T, stage, samples, st);   \
            if (e != hipSuccess) return e;                                                            \
        } else if (eig_split)                                                                         \
            pnp_eig_split_kernel<N><<<(nwgE + kSplitUnits - 1) / kSplitUnits, 128 * kSplitUnits, 0, st>>>( \
                probs, lps, wgtE, nwgE, T, stage, samples, fault);                                    \
        else                                                                                          \
            pnp_eig_group_kernel<N><<<nwgE, 64, 0, st>>>(probs, lps, wgtE, T, stage, samples);        \
        if (eig_end) (void)hipEventRecord(eig_end, st);                                               \
        pnp_betas_kernel<N><<<3 * nwgB, 64, 0, st>>>(probs, lps, wgtB, nwgB, stage, samples, poses,   \
                                                     bs.err, bs.pose, bs.ctr, bs.hcap, betas_hb);     \
        break;
        RSC_CASE(4) RSC_CASE(5) RSC_CASE(6)
#undef RSC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Device libm restatement self-test (rsc_selftest_math): the functions as the kernels compile them.
__global__ __launch_bounds__(256) void selftest_math_kernel(int fn, const double* __restrict__ x, int n,
                                                            double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r;
    switch (fn) {
        case 0: r = dm::sin(v); break;
        case 1: r = dm::cos(v); break;
        case 2: r = dm::acos(v); break;
        case 3: r = dm::cbrt(v); break;
        case 4: r = dm::log(v); break;
        case 5: r = (double)dm::logf((float)v); break;
        // the chase's short-chain IEEE forms (rsc_core.h) and make_givens built from them;
        // make_givens pairs x[i] with x[(i + n/2) % n]
        case 6: r = sqrt_unit(v); break;
        case 7: r = recip_unit(v); break;
        // MLPnP's pow(x, 1.0/3.0) and pow(t, 3.0/2.0) restatements (rsc_math.h)
        case 11: r = dm::pow_1_3(v); break;
        case 12: r = dm::pow_3_2(v); break;
        // the PnP scan's reciprocal (pnp_inlier2, one element) of (float)v; rcp_fast_ok is not
        // applied, so the caller sees the fast form on every argument
        case 13: {
            const float z = (float)v;
            const float r0 = __builtin_amdgcn_rcpf(z);
            r = (double)__builtin_fmaf(__builtin_fmaf(-z, r0, 1.0f), r0, r0);
            break;
        }

        default: {
            double c, s;
            make_givens(v, x[(i + n / 2) % n], c, s);
            r = fn == 8 ? c : s;
            break;
        }
    }
    out[i] = r;
}

// qr_solve_6x4 self-test (rsc_selftest_math fn 10): record r = x[34 r ..] holds A[6][4] row-major,
// b[6] and the previous X[4]; out[34 r + 0..3] = X after the solve, out[34 r + 4] = 1 on success,
// 0 on the singular bail-out (Q9 / Q19).
__global__ __launch_bounds__(256) void selftest_qr_kernel(const double* __restrict__ x, int nrec,
                                                          double* __restrict__ out) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrec) return;
    const double* in = x + 34 * (size_t)r;
    double A[6][4], b[6], X[4];
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        RSC_UNROLL for (int j = 0; j < 4; ++j) A[i][j] = in[4 * i + j];
        b[i] = in[24 + i];
    }
    RSC_UNROLL for (int j = 0; j < 4; ++j) X[j] = in[30 + j];
    const bool ok = qr_solve_6x4(A, b, X);
    double* o = out + 34 * (size_t)r;
    RSC_UNROLL for (int j = 0; j < 4; ++j) o[j] = X[j];
    o[4] = ok ? 1.0 : 0.0;
    for (int j = 5; j < 34; ++j) o[j] = 0.0;
}

__global__ __launch_bounds__(256) void upload16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

// Byte copy between pinned host memory and HBM (either direction) by one kernel: thread i moves
// bytes [16 i, 16 i + 16) as one 16-B word, four 4-B words or single bytes (`unit`, by alignment).
__global__ __launch_bounds__(256) void copy_bytes_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         size_t n, int unit) {
    const size_t b = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (b >= n) return;
    if (b + 16 <= n && unit == 16) {
        *reinterpret_cast<uint4*>(dst + b) = *reinterpret_cast<const uint4*>(src + b);
    } else if (b + 16 <= n && unit == 4) {
        RSC_UNROLL for (int k = 0; k < 16; k += 4)
            *reinterpret_cast<uint32_t*>(dst + b + k) = *reinterpret_cast<const uint32_t*>(src + b + k);
    } else {
        const size_t e = (b + 16 < n) ? b + 16 : n;
        for (size_t k = b; k < e; ++k) dst[k] = src[k];
    }
}

hipError_t launch_copy_bytes(const void* src, void* dst, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uintptr_t a = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst);
    const int unit = (a % 16 == 0) ? 16 : (a % 4 == 0 ? 4 : 1);
    const unsigned blocks = (unsigned)((n + 16 * 256 - 1) / (16 * 256));
    copy_bytes_kernel<<<blocks, 256, 0, st>>>(static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst), n, unit);
    return hipGetLastError();
}

// Completion flag of a speculation round for the host's spin wait (rsc_api.cpp stream_wait): one
// lane stores the round's sequence number to pinned host memory with a system-scope release once
// every earlier operation of the stream has finished (a vector store; no scalar-cache writes).
__global__ __launch_bounds__(64) void signal_kernel(uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_signal(uint32_t* host_flag, uint32_t value, hipStream_t st) {
    signal_kernel<<<1, 64, 0, st>>>(host_flag, value);
    return hipGetLastError();
}

hipError_t launch_upload16(const void* host_src, void* dev_dst, size_t n16, hipStream_t st) {
    if (n16 == 0) return hipSuccess;
    const unsigned blocks = (unsigned)((n16 + 255) / 256);
    upload16_kernel<<<blocks, 256, 0, st>>>(static_cast<const uint4*>(host_src), static_cast<uint4*>(dev_dst), n16);
    return hipGetLastError();
}

hipError_t launch_selftest_math(int fn, const double* x, int n, double* out, hipStream_t st) {
    if (fn < 0 || fn > 13 || n <= 0) return hipErrorInvalidValue;
    if (fn == 10) {
        if (n % 34) return hipErrorInvalidValue;
        const int nrec = n / 34;
        selftest_qr_kernel<<<(nrec + 255) / 256, 256, 0, st>>>(x, nrec, out);
        return hipGetLastError();
    }
    selftest_math_kernel<<<(n + 255) / 256, 256, 0, st>>>(fn, x, n, out);
    return hipGetLastError();
}

hipError_t launch_pnp_scan(int ppt, int nwg, const DevPnP* probs, const LaunchProb* lps, const int4* wgt,
                           const float* poses, int32_t* counts, int32_t* counts_dev, uint64_t* masks, int mask_words,
                           int32_t* qual, hipStream_t st) {
    switch (ppt) {
#define RSC_CASE(P) case P: pnp_scan_kernel<P><<<nwg, 256, 0, st>>>(probs, lps, wgt, poses, counts, counts_dev, masks, mask_words, qual); break;
        RSC_CASE(1) RSC_CASE(2) RSC_CASE(4) RSC_CASE(8) RSC_CASE(16) RSC_CASE(32)
#undef RSC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t read_solve_stamps(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solve_stamps), sizeof(uint64_t) * 3 * 4096 * 8, 0, hipMemcpyDeviceToHost);
}

hipError_t read_refine_stamps(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_refine_stamps), sizeof(uint64_t) * 64 * 24, 0, hipMemcpyDeviceToHost);
}

hipError_t launch_pnp_refine(int njobs, const DevPnP* probs, const RefineJob* jobs, unsigned* fault, hipStream_t st) {
    if (!fault) return hipErrorInvalidValue;
    pnp_refine_kernel<<<njobs, 256, 0, st>>>(probs, jobs, fault);
    return hipGetLastError();
}

hipError_t launch_pnp_select_refine(int nsel, const DevPnP* probs, const RefineSel* sels, const int32_t* counts,
                                    uint64_t* masks, int mask_words, const float* poses, RefineSelOut* out,
                                    unsigned* fault, hipStream_t st) {
    if (nsel <= 0) return hipSuccess;
    if (!fault) return hipErrorInvalidValue;
    pnp_select_refine_kernel<<<nsel, 256, 0, st>>>(probs, sels, counts, masks, mask_words, poses, out, fault);
    return hipGetLastError();
}

hipError_t launch_sim3_solve(int nwg, const DevSim3* probs, const LaunchProb* lps, const int2* wgt, const uint32_t* T,
                             float* poses, int32_t* samples, hipStream_t st) {
    sim3_solve_kernel<<<nwg, 64, 0, st>>>(probs, lps, wgt, T, poses, samples);
    return hipGetLastError();
}

hipError_t launch_sim3_scan(int ppt, int nwg, const DevSim3* probs, const LaunchProb* lps, const int4* wgt,
                            const float* poses, int32_t* counts, int32_t* counts_dev, uint64_t* masks, int mask_words,
                            hipStream_t st) {
    switch (ppt) {
#define RSC_CASE(P) case P: sim3_scan_kernel<P><<<nwg, 256, 0, st>>>(probs, lps, wgt, poses, counts, counts_dev, masks, mask_words); break;
        RSC_CASE(1) RSC_CASE(2) RSC_CASE(4) RSC_CASE(8) RSC_CASE(16) RSC_CASE(32)
#undef RSC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rng_stream(const uint32_t* T, const uint32_t* window, int g0, int n, int32_t* out, hipStream_t st) {
    Window31 w;
    for (int j = 0; j < 31; ++j) w.w[j] = window[j];
    rng_stream_kernel<<<(n + 255) / 256, 256, 0, st>>>(T, w, g0, n, out);
    return hipGetLastError();
}

}  // namespace rsc
