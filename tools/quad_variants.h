// quad_variants.h — DIAGNOSTIC forms of the EPnP hypothesis stages (not part of the product),
// kept for tools/quad_bench.hip: the lane-per-hypothesis eigen stage, the three-wave betas stage
// (round-1 form) and the event-form QR sink.  Every form is bit-identical to the product's
// (rsc_quad.h); all were measured slower on gfx950.
#pragma once
#include "../orb-slam2-optimized_amd/csrc/rsc_quad.h"
#include "qr_events.h"

namespace rsc {

// pnp_betas_body LDS (three-wave form): eigenvectors [48][64], L+rho [66][64], errors [3][64],
// poses [3][12][64] f32.
constexpr int kBetasSmemDoubles = (48 + 66) * 64 + 3 * 64 + 3 * 12 * 64 / 2;

// The quad's own three rows of Q as the rotation sink of tridiag_qr_events12 (diagnostic variant).
struct QuadRowsEv {
    double* T;
    int q;
    RSC_HD double load(int r, int col) const { return T[(4 * r + q) * 12 + col]; }
    RSC_HD void store(int r, int col, double v) { T[(4 * r + q) * 12 + col] = v; }
};

// Kernel 1, lane form: one lane per hypothesis (sample, control points, alphas, MtM, 12x12
// eigenvectors in the per-lane LDS slab), same stage record as the quad form.
template <int NS>
__device__ __forceinline__ void pnp_eig_lane_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                  const int2* __restrict__ wg_table, const uint32_t* __restrict__ rng_T,
                                                  double* __restrict__ stage, int32_t* __restrict__ samples,
                                                  double* slab) {
    const int lane = threadIdx.x;
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const int h = wt.y + lane;
    if (h >= lp.H) return;
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    double* out = stage + rec * kStageDoubles;
    int idx[NS];
    {
        uint32_t w[31];
        RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
        uint32_t words[NS];
        RSC_UNROLL for (int d = 0; d < NS; ++d) words[d] = rng_word(rng_T, w, lp.g0 + h * NS + d);
        swap_remove_sample<NS>(words, NS, P.n, idx);
    }
    RSC_UNROLL for (int i = 0; i < NS; ++i) samples[rec * 8 + i] = idx[i];
    const LaneMat S{slab + lane, 64};
    {
        HypStore<NS> st;
        RSC_UNROLL for (int i = 0; i < NS; ++i) {
            const float4 p = P.pts[idx[i]];
            const float2 uv = P.uv[idx[i]];
            st.pw_[i][0] = p.x; st.pw_[i][1] = p.y; st.pw_[i][2] = p.z;
            st.u_[i][0] = uv.x; st.u_[i][1] = uv.y;
        }
        st.rows_ = P.rows;
        st.spw = P.pws;
        st.sal = P.als;
        const Intrinsics K{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy};
        double cws[4][3];
        control_points_and_alphas(st, cws);
        RSC_UNROLL for (int i = 0; i < NS; ++i)
            RSC_UNROLL for (int j = 0; j < 4; ++j) out[kStAl + i * 4 + j] = st.al(i, j);
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) out[kStCws + i * 3 + c] = cws[i][c];
        build_MtM(st, K, S);
    }
    sym_eig12(S);
    RSC_UNROLL for (int r = 0; r < 12; ++r)
        RSC_UNROLL for (int c = 0; c < 4; ++c) out[kStEv + r * 4 + c] = S.at(r, c);
}

// Kernel 2: 192 threads = 3 waves over the same 64 hypotheses; wave w runs find_betas_approx_{w+1}
// + gauss_newton + compute_R_and_t (PnPsolver.cpp:383-408), wave 0 keeps the smallest error in the
// reference's order (:393-414) and writes the float pose.  FORCE >= 0 (diagnostics only,
// tools/quad_bench) makes every wave run approximation FORCE + 1.
template <int NS, int FORCE = -1>
__device__ __forceinline__ void pnp_betas_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                               const int2* __restrict__ wg_table, const double* __restrict__ stage,
                                               const int32_t* __restrict__ samples, float* __restrict__ poses,
                                               double* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int apx = FORCE >= 0 ? FORCE : wave;
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const bool active = wt.y + lane < lp.H;
    const int h = active ? wt.y + lane : lp.H - 1;
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    const double* in = stage + rec * kStageDoubles;
    double* EV = smem;
    double* LR = EV + 48 * 64;
    double* ERR = LR + 66 * 64;
    float* PZ = reinterpret_cast<float*>(ERR + 3 * 64);
    RSC_UNROLL for (int e = 0; e < 16; ++e) EV[(16 * wave + e) * 64 + lane] = in[kStEv + 16 * wave + e];
    __syncthreads();
    const SplitView V{EV + lane, LR + lane, 64};
    if (wave == 0) {
        compute_L_6x10(V);
        double cws[4][3];
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) cws[i][c] = in[kStCws + i * 3 + c];
        auto d2 = [&](int a, int b) {
            double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
            return x * x + y * y + z * z;
        };
        V.rho(0) = d2(0, 1); V.rho(1) = d2(0, 2); V.rho(2) = d2(0, 3);
        V.rho(3) = d2(1, 2); V.rho(4) = d2(1, 3); V.rho(5) = d2(2, 3);
    }
    __syncthreads();
    double betas[4] = {0.0, 0.0, 0.0, 0.0};
    if (apx == 0) find_betas<1>(V, betas);
    else if (apx == 1) find_betas<2>(V, betas);
    else find_betas<3>(V, betas);
    gauss_newton(V, betas);
    // the hypothesis' points and alphas are read only now: live across the solves above they
    // pushed the wave past 256 VGPRs (scratch spills, round 1)
    HypStore<NS> st;
    RSC_UNROLL for (int i = 0; i < NS; ++i) {
        const int id = samples[rec * 8 + i];
        const float4 p = P.pts[id];
        const float2 uv = P.uv[id];
        st.pw_[i][0] = p.x; st.pw_[i][1] = p.y; st.pw_[i][2] = p.z;
        st.u_[i][0] = uv.x; st.u_[i][1] = uv.y;
        RSC_UNROLL for (int j = 0; j < 4; ++j) st.al_[i][j] = in[kStAl + i * 4 + j];
    }
    st.rows_ = P.rows;
    st.spw = P.pws;
    st.sal = P.als;
    const Intrinsics K{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy};
    const double pw0[3] = {in[kStCws + 0], in[kStCws + 1], in[kStCws + 2]};
    double R[3][3], t[3];
    ERR[wave * 64 + lane] = compute_R_and_t(st, K, V, betas, pw0, R, t);
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) PZ[(wave * 12 + 3 * r + c) * 64 + lane] = (float)R[r][c];
    RSC_UNROLL for (int r = 0; r < 3; ++r) PZ[(wave * 12 + 9 + r) * 64 + lane] = (float)t[r];
    __syncthreads();
    if (wave == 0 && active) {
        int best = 0;
        double be = ERR[lane];
        if (ERR[64 + lane] < be) { be = ERR[64 + lane]; best = 1; }
        if (ERR[128 + lane] < be) { be = ERR[128 + lane]; best = 2; }
        float* o = poses + rec * 12;
        RSC_UNROLL for (int k = 0; k < 12; ++k) o[k] = PZ[(best * 12 + k) * 64 + lane];
    }
}

}  // namespace rsc
