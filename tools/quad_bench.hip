// quad_bench.hip — diagnostic: time the two-kernel (quad-cooperative eig + per-branch betas)
// hypothesis solve, truncated after each phase, on a config-2 shaped launch (64 problems x 300
// hypotheses of 4 points by default).  Not part of the product; build: make -C tools quad_bench.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "quad_variants.h"

using namespace rsc;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// L lanes per hypothesis, HPW hypotheses per workgroup
template <int STOP, int L, int HPW>
__global__ __launch_bounds__(64) void eig_g(const DevPnP* probs, const LaunchProb* lps, const int2* wgt, const uint32_t* T,
                                            double* stage, int32_t* samples) {
    __shared__ __attribute__((aligned(16))) double smem[HPW * kQuadRegion];
    pnp_eig_group_body<4, STOP, L, HPW>(probs, lps, wgt, T, stage, samples, smem);
}
template <int STOP>
__global__ __launch_bounds__(64, 2) void eig_k2(const DevPnP* probs, const LaunchProb* lps, const int2* wgt,
                                                const uint32_t* T, double* stage, int32_t* samples) {
    __shared__ __attribute__((aligned(16))) double smem[16 * kQuadRegion];
    pnp_eig_group_body<4, STOP, 4, 16>(probs, lps, wgt, T, stage, samples, smem);
}
__global__ __launch_bounds__(64) void eig_lane_k(const DevPnP* probs, const LaunchProb* lps, const int2* wgt,
                                                  const uint32_t* T, double* stage, int32_t* samples) {
    __shared__ __attribute__((aligned(16))) double slab[144 * 64];
    pnp_eig_lane_body<4>(probs, lps, wgt, T, stage, samples, slab);
}
// variants of pnp_eig_lane_body: CR = constant rows (no stale rows), HS = host-drawn samples
template <bool CR, bool HS, bool SUM = false>
__global__ __launch_bounds__(64) void eig_lane_v(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                 const int2* __restrict__ wg_table, const uint32_t* __restrict__ rng_T,
                                                 double* __restrict__ stage, int32_t* __restrict__ samples,
                                                 const int4* __restrict__ hs) {
    __shared__ __attribute__((aligned(16))) double slab[144 * 64];
    constexpr int NS = 4;
    const int lane = threadIdx.x;
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const int h = wt.y + lane;
    if (h >= lp.H) return;
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    double* out = stage + rec * kStageDoubles;
    int idx[NS];
    if (HS) {
        const int4 v = hs[rec];
        idx[0] = v.x; idx[1] = v.y; idx[2] = v.z; idx[3] = v.w;
    } else {
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
        st.rows_ = CR ? NS : P.rows;
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
    if (SUM) {
        double acc = 0.0;
        RSC_UNROLL for (int e = 0; e < 144; ++e) acc += S(e);
        out[0] = acc;
        return;
    }
    RSC_UNROLL for (int r = 0; r < 12; ++r)
        RSC_UNROLL for (int c = 0; c < 4; ++c) out[kStEv + r * 4 + c] = S.at(r, c);
}
// phase_bench's phase_kernel<4> structure with switches: V=1 runtime K, V=2 slab 144, V=3 al/cws
// writes, V=4 sym_eig12(S)
template <int V>
__global__ __launch_bounds__(64) void pb4(const float4* __restrict__ pts, const float2* __restrict__ uv,
                                          const int4* __restrict__ samples, int H, double* __restrict__ out, int N,
                                          const DevPnP* __restrict__ probs) {
    __shared__ __attribute__((aligned(16))) double slab[(V == 2 ? 144 : kSlabDoubles) * 64];
    const int lane = threadIdx.x;
    const int h = blockIdx.x * 64 + lane;
    if (h >= H) return;
    const int4 s = samples[h];
    const int idx[4] = {s.x, s.y, s.z, s.w};
    const int prob = h / 300;
    HypStore<4> st;
    RSC_UNROLL for (int i = 0; i < 4; ++i) {
        const float4 p = pts[(size_t)prob * N + idx[i]];
        const float2 q = uv[(size_t)prob * N + idx[i]];
        st.pw_[i][0] = p.x; st.pw_[i][1] = p.y; st.pw_[i][2] = p.z;
        st.u_[i][0] = q.x; st.u_[i][1] = q.y;
    }
    st.rows_ = 4;
    st.spw = nullptr;
    st.sal = nullptr;
    const DevPnP& P = probs[prob];
    const Intrinsics K = (V == 1) ? Intrinsics{(double)P.fx, (double)P.fy, (double)P.cx, (double)P.cy}
                                  : Intrinsics{435.20468, 435.20468, 367.45172, 252.20085};
    LaneMat S{slab + lane, 64};
    double cws[4][3];
    control_points_and_alphas(st, cws);
    if (V == 3) {
        double* o = out + (size_t)h * kStageDoubles;
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int j = 0; j < 4; ++j) o[kStAl + i * 4 + j] = st.al(i, j);
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) o[kStCws + i * 3 + c] = cws[i][c];
    }
    build_MtM(st, K, S);
    if (V == 4) {
        sym_eig12(S);
    } else {
        double diag[12], sub[11];
        sym_eig12_tridiag(S, diag, sub);
        sym_eig12_qr(S, diag, sub);
    }
    double acc = 0.0;
    RSC_UNROLL for (int e = 0; e < 144; ++e) acc += S(e);
    out[(size_t)h * kStageDoubles] = acc;
}
template <int FORCE = -1>
__global__ __launch_bounds__(192) void betas_k1(const DevPnP* probs, const LaunchProb* lps, const int2* wgt,
                                               const double* stage, const int32_t* samples, float* poses) {
    __shared__ __attribute__((aligned(16))) double smem[kBetasSmemDoubles];
    pnp_betas_body<4, FORCE>(probs, lps, wgt, stage, samples, poses, smem);
}
template <int FORCE = -1>
__global__ __launch_bounds__(192, 2) void betas_k(const DevPnP* probs, const LaunchProb* lps, const int2* wgt,
                                               const double* stage, const int32_t* samples, float* poses) {
    __shared__ __attribute__((aligned(16))) double smem[kBetasSmemDoubles];
    pnp_betas_body<4, FORCE>(probs, lps, wgt, stage, samples, poses, smem);
}

int main(int argc, char** argv) {
    const int NP = 64, N = 2000;
    const int Hp = (argc > 1) ? atoi(argv[1]) : 300;
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(s >> 11) / 9007199254740992.0; };
    // problem data: tools/data/scenes.bin (64 x 2000, written by tools/dump_scenes.py) when given,
    // else one random scene shared by all problems
    std::vector<float4> pts((size_t)NP * N);
    std::vector<float2> uv((size_t)NP * N);
    const bool from_file = argc > 2;
    if (from_file) {
        FILE* f = fopen(argv[2], "rb");
        int hdr[2];
        if (!f || fread(hdr, 4, 2, f) != 2 || hdr[0] != NP || hdr[1] != N) { printf("bad scenes file\n"); return 1; }
        if (fread(pts.data(), 16, pts.size(), f) != pts.size() || fread(uv.data(), 8, uv.size(), f) != uv.size()) return 1;
        fclose(f);
    } else {
        for (int i = 0; i < N; ++i) {
            double X = rnd() * 8 - 4, Y = rnd() * 6 - 3, Z = 2 + rnd() * 10;
            double u = 367.215 + 458.654 * X / Z, v = 248.375 + 457.296 * Y / Z;
            if (rnd() < 0.6) { u = rnd() * 752; v = rnd() * 480; }
            for (int c = 0; c < NP; ++c) {
                pts[(size_t)c * N + i] = make_float4((float)X, (float)Y, (float)Z, 1.0f);
                uv[(size_t)c * N + i] = make_float2((float)u, (float)v);
            }
        }
    }
    const int G = Hp * 4 + 64;
    std::vector<uint32_t> T((size_t)G * 32);
    for (auto& x : T) x = (uint32_t)(rnd() * 4294967296.0);
    float4* dp; float2* du; uint32_t* dT; double* dst; int32_t* dsm; float* dpo;
    CK(hipMalloc(&dp, pts.size() * sizeof(float4)));
    CK(hipMalloc(&du, uv.size() * sizeof(float2)));
    CK(hipMalloc(&dT, T.size() * 4));
    CK(hipMemcpy(dp, pts.data(), pts.size() * sizeof(float4), hipMemcpyHostToDevice));
    CK(hipMemcpy(du, uv.data(), uv.size() * sizeof(float2), hipMemcpyHostToDevice));
    CK(hipMemcpy(dT, T.data(), T.size() * 4, hipMemcpyHostToDevice));
    const int total = NP * Hp;
    CK(hipMalloc(&dst, (size_t)total * kStageDoubles * 8));
    CK(hipMalloc(&dsm, (size_t)total * 8 * 4));
    CK(hipMalloc(&dpo, (size_t)total * 12 * 4));
    std::vector<DevPnP> probs(NP);
    std::vector<LaunchProb> lps(NP);
    std::vector<int2> w16, w64, w32, w20;
    for (int i = 0; i < NP; ++i) {
        DevPnP& d = probs[i];
        d.pts = dp + (size_t)i * N; d.uv = du + (size_t)i * N; d.n = N;
        d.fx = 435.20468f; d.fy = 435.20468f; d.cx = 367.45172f; d.cy = 252.20085f;
        d.th2 = 5.991f; d.rows = 4; d.pws = nullptr; d.us = nullptr; d.als = nullptr;
        LaunchProb& l = lps[i];
        l.prob = i; l.H = Hp; l.out0 = i * Hp; l.g0 = 0; l.min_inliers = 0;
        for (int j = 0; j < 31; ++j) l.window[j] = (uint32_t)(rnd() * 4294967296.0);
        for (int h0 = 0; h0 < Hp; h0 += 16) w16.push_back(make_int2(i, h0));
        for (int h0 = 0; h0 < Hp; h0 += 32) w32.push_back(make_int2(i, h0));
        for (int h0 = 0; h0 < Hp; h0 += 20) w20.push_back(make_int2(i, h0));
        for (int h0 = 0; h0 < Hp; h0 += 64) w64.push_back(make_int2(i, h0));
    }
    DevPnP* dprobs; LaunchProb* dlps; int2 *dw16, *dw64, *dw32, *dw20;
    CK(hipMalloc(&dw32, w32.size() * sizeof(int2)));
    CK(hipMalloc(&dw20, w20.size() * sizeof(int2)));
    CK(hipMemcpy(dw32, w32.data(), w32.size() * sizeof(int2), hipMemcpyHostToDevice));
    CK(hipMemcpy(dw20, w20.data(), w20.size() * sizeof(int2), hipMemcpyHostToDevice));
    CK(hipMalloc(&dprobs, NP * sizeof(DevPnP)));
    CK(hipMalloc(&dlps, NP * sizeof(LaunchProb)));
    CK(hipMalloc(&dw16, w16.size() * sizeof(int2)));
    CK(hipMalloc(&dw64, w64.size() * sizeof(int2)));
    CK(hipMemcpy(dprobs, probs.data(), NP * sizeof(DevPnP), hipMemcpyHostToDevice));
    CK(hipMemcpy(dlps, lps.data(), NP * sizeof(LaunchProb), hipMemcpyHostToDevice));
    CK(hipMemcpy(dw16, w16.data(), w16.size() * sizeof(int2), hipMemcpyHostToDevice));
    CK(hipMemcpy(dw64, w64.data(), w64.size() * sizeof(int2), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 20;
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return 1e3f * ms / reps;
    };
    const int n16 = (int)w16.size(), n64 = (int)w64.size();
    printf("hyps=%d eig WGs=%d betas WGs=%d\n", total, n16, n64);
    const int n32 = (int)w32.size(), n20 = (int)w20.size();
    // reference stage records: the quad sweep form (the round-1/2 product kernel)
    const size_t nst = (size_t)total * kStageDoubles;
    std::vector<double> ref(nst), got(nst);
    std::vector<int32_t> refs((size_t)total * 8), gots((size_t)total * 8);
    auto snap = [&](std::vector<double>& d, std::vector<int32_t>& sm) {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(d.data(), dst, nst * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sm.data(), dsm, sm.size() * 4, hipMemcpyDeviceToHost));
    };
    CK(hipMemset(dst, 0, nst * 8));
    eig_k2<99><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm);
    snap(ref, refs);
    auto cmp = [&](const char* name, auto launch) {
        CK(hipMemset(dst, 0, nst * 8));
        CK(hipMemset(dsm, 0, gots.size() * 4));
        launch();
        snap(got, gots);
        const bool ok = !memcmp(got.data(), ref.data(), nst * 8) && !memcmp(gots.data(), refs.data(), gots.size() * 4);
        printf("%-22s %8.1f us  %s\n", name, timeit(launch), ok ? "bit-exact" : "MISMATCH");
        fflush(stdout);
    };
    printf("eig2 A (sample..MtM)  %8.1f us\n", timeit([&] { eig_k2<1><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm); }));
    printf("eig2 A+tridiag        %8.1f us\n", timeit([&] { eig_k2<2><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm); }));
    printf("eig2 A+tri+accum      %8.1f us\n", timeit([&] { eig_k2<3><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm); }));
    cmp("eig2 quad sweep-QR", [&] { eig_k2<99><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm); });
    printf("pair32 A              %8.1f us\n", timeit([&] { eig_g<1, 2, 32><<<n32, 64>>>(dprobs, dlps, dw32, dT, dst, dsm); }));
    printf("pair32 A+tridiag      %8.1f us\n", timeit([&] { eig_g<2, 2, 32><<<n32, 64>>>(dprobs, dlps, dw32, dT, dst, dsm); }));
    printf("pair32 A+tri+accum    %8.1f us\n", timeit([&] { eig_g<3, 2, 32><<<n32, 64>>>(dprobs, dlps, dw32, dT, dst, dsm); }));
    cmp("pair32 full", [&] { eig_g<99, 2, 32><<<n32, 64>>>(dprobs, dlps, dw32, dT, dst, dsm); });
    cmp("pair20 full", [&] { eig_g<99, 2, 20><<<n20, 64>>>(dprobs, dlps, dw20, dT, dst, dsm); });
    cmp("quad16 (lb64) full", [&] { eig_g<99, 4, 16><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm); });
    printf("WGs: quad16 %d pair32 %d pair20 %d\n", n16, n32, n20);
    {  // eig -> betas back to back (as the product stream): betas time after each eig form
        hipEvent_t t0, t1, t2;
        CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1)); CK(hipEventCreate(&t2));
        for (int form = 0; form < 2; ++form) {
            float se = 0, sb = 0;
            for (int r = 0; r < 21; ++r) {
                CK(hipEventRecord(t0));
                if (form == 0) eig_k2<99><<<n16, 64>>>(dprobs, dlps, dw16, dT, dst, dsm);
                else eig_g<99, 2, 20><<<n20, 64>>>(dprobs, dlps, dw20, dT, dst, dsm);
                CK(hipEventRecord(t1));
                betas_k<<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo);
                CK(hipEventRecord(t2));
                CK(hipEventSynchronize(t2));
                float a, b2;
                CK(hipEventElapsedTime(&a, t0, t1));
                CK(hipEventElapsedTime(&b2, t1, t2));
                if (r) { se += a; sb += b2; }
            }
            printf("%s eig %8.1f us -> betas %8.1f us\n", form ? "pair20" : "quad16", se * 50, sb * 50);
        }
        // fresh sample streams per step (as bench.py's reset(seeds) per step)
        for (int st = 0; st < 6; ++st) {
            for (auto& l : lps)
                for (int j = 0; j < 31; ++j) l.window[j] = (uint32_t)(rnd() * 4294967296.0);
            CK(hipMemcpy(dlps, lps.data(), NP * sizeof(LaunchProb), hipMemcpyHostToDevice));
            CK(hipEventRecord(t0));
            eig_g<99, 2, 20><<<n20, 64>>>(dprobs, dlps, dw20, dT, dst, dsm);
            CK(hipEventRecord(t1));
            betas_k<<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo);
            CK(hipEventRecord(t2));
            CK(hipEventSynchronize(t2));
            float a, b2;
            CK(hipEventElapsedTime(&a, t0, t1));
            CK(hipEventElapsedTime(&b2, t1, t2));
            printf("step %d: pair20 eig %8.1f us -> betas %8.1f us\n", st, a * 1e3f, b2 * 1e3f);
        }
    }
    if (argc > 3) return 0;  // eig only
    printf("eig lane              %8.1f us\n", timeit([&] { eig_lane_k<<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm); }));
    std::vector<int4> hsv(total);
    for (int i = 0; i < total; ++i) {
        int a[4];
        for (int k = 0; k < 4; ++k) {
            bool dup;
            do { a[k] = (int)(rnd() * N); dup = false; for (int j = 0; j < k; ++j) dup |= a[j] == a[k]; } while (dup);
        }
        hsv[i] = make_int4(a[0], a[1], a[2], a[3]);
    }
    int4* dhs;
    CK(hipMalloc(&dhs, total * sizeof(int4)));
    CK(hipMemcpy(dhs, hsv.data(), total * sizeof(int4), hipMemcpyHostToDevice));
    printf("eig lane v00          %8.1f us\n", timeit([&] { eig_lane_v<false, false><<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm, dhs); }));
    printf("eig lane v10 (rows)   %8.1f us\n", timeit([&] { eig_lane_v<true, false><<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm, dhs); }));
    printf("eig lane v01 (hs)     %8.1f us\n", timeit([&] { eig_lane_v<false, true><<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm, dhs); }));
    printf("eig lane v11 sum      %8.1f us\n", timeit([&] { eig_lane_v<true, true, true><<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm, dhs); }));
    printf("eig lane v11          %8.1f us\n", timeit([&] { eig_lane_v<true, true><<<n64, 64>>>(dprobs, dlps, dw64, dT, dst, dsm, dhs); }));
    for (int v = 0; v <= 4; ++v) {
        float us = 0;
        switch (v) {
            case 0: us = timeit([&] { pb4<0><<<(total + 63) / 64, 64>>>(dp, du, dhs, total, dst, N, dprobs); }); break;
            case 1: us = timeit([&] { pb4<1><<<(total + 63) / 64, 64>>>(dp, du, dhs, total, dst, N, dprobs); }); break;
            case 2: us = timeit([&] { pb4<2><<<(total + 63) / 64, 64>>>(dp, du, dhs, total, dst, N, dprobs); }); break;
            case 3: us = timeit([&] { pb4<3><<<(total + 63) / 64, 64>>>(dp, du, dhs, total, dst, N, dprobs); }); break;
            case 4: us = timeit([&] { pb4<4><<<(total + 63) / 64, 64>>>(dp, du, dhs, total, dst, N, dprobs); }); break;
        }
        printf("pb4 variant %d         %8.1f us\n", v, us);
    }
    printf("betas                 %8.1f us\n", timeit([&] { betas_k<<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo); }));
    printf("betas lb(192)         %8.1f us\n", timeit([&] { betas_k1<<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo); }));
    printf("betas all approx1     %8.1f us\n", timeit([&] { betas_k<0><<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo); }));
    printf("betas all approx2     %8.1f us\n", timeit([&] { betas_k<1><<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo); }));
    printf("betas all approx3     %8.1f us\n", timeit([&] { betas_k<2><<<n64, 192>>>(dprobs, dlps, dw64, dst, dsm, dpo); }));
    return 0;
}
