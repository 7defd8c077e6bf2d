// phase_bench.hip — diagnostic: time the per-lane EPnP hypothesis pipeline truncated after each
// phase (config-2 shape: 19,200 hypotheses of 4 points, one lane per hypothesis, 64-lane WGs).
// Every truncation writes a checksum of its live state so no phase is dead-code eliminated.
// Not part of the product; build: make -C tools phase_bench.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../orb-slam2-optimized_amd/csrc/rsc_core.h"
#include "../orb-slam2-optimized_amd/csrc/rsc_epnp.h"

using namespace rsc;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int STOP>
__global__ __launch_bounds__(64) void phase_kernel(const float4* __restrict__ pts, const float2* __restrict__ uv,
                                                   const int4* __restrict__ samples, int H, double* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) double slab[kSlabDoubles * 64];
    const int lane = threadIdx.x;
    const int h = blockIdx.x * 64 + lane;
    if (h >= H) return;
    const int4 s = samples[h];
    const int idx[4] = {s.x, s.y, s.z, s.w};
    HypStore<4> st;
    RSC_UNROLL for (int i = 0; i < 4; ++i) {
        const float4 p = pts[idx[i]];
        const float2 q = uv[idx[i]];
        st.pw_[i][0] = p.x; st.pw_[i][1] = p.y; st.pw_[i][2] = p.z;
        st.u_[i][0] = q.x; st.u_[i][1] = q.y;
    }
    st.rows_ = 4;
    st.spw = nullptr;
    st.sal = nullptr;
    const Intrinsics K{458.654, 457.296, 367.215, 248.375};
    LaneMat S{slab + lane, 64};
    double cws[4][3];
    control_points_and_alphas(st, cws);
    double acc = 0.0;
    if (STOP == 1) {
        RSC_UNROLL for (int i = 0; i < 4; ++i) RSC_UNROLL for (int j = 0; j < 4; ++j) acc += st.al(i, j);
        RSC_UNROLL for (int i = 0; i < 4; ++i) RSC_UNROLL for (int j = 0; j < 3; ++j) acc += cws[i][j];
        out[h] = acc;
        return;
    }
    build_MtM(st, K, S);
    if (STOP == 2) {
        RSC_UNROLL for (int e = 0; e < 144; ++e) acc += S(e);
        out[h] = acc;
        return;
    }
    double diag[12], sub[11];
    sym_eig12_tridiag(S, diag, sub);
    if (STOP == 3) {
        RSC_UNROLL for (int e = 0; e < 144; ++e) acc += S(e);
        RSC_UNROLL for (int e = 0; e < 12; ++e) acc += diag[e];
        RSC_UNROLL for (int e = 0; e < 11; ++e) acc += sub[e];
        out[h] = acc;
        return;
    }
    if (STOP == 50) {  // QR chase with the rotations only logged (no Q update)
        int m = 0;
        auto qlog = [&](int k, double c, double s2, bool) {
            S(144 + (m & 7)) = c;
            S(152 + (m & 7)) = s2 + (double)k;
            ++m;
        };
        int perm[12];
        tridiag_qr<double, 12>(diag, sub, qlog, perm);
        RSC_UNROLL for (int e = 0; e < 12; ++e) acc += diag[e] + (double)perm[e];
        out[h] = acc + S(144) + S(152) + m;
        return;
    }
    sym_eig12_qr(S, diag, sub);
    if (STOP == 4) {
        RSC_UNROLL for (int e = 0; e < 144; ++e) acc += S(e);
        out[h] = acc;
        return;
    }
    // STOP 5..7: 1..3 beta branches (5 = branch 1 only, 6 = branches 1+2, 7 = full stage C)
    // STOP 11/12/13: only branch 1 / 2 / 3 (after L, rho)
    compute_L_6x10(SlabView{S});
    {
        auto d2 = [&](int a, int b) {
            double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
            return x * x + y * y + z * z;
        };
        rhoref(S, 0) = d2(0, 1); rhoref(S, 1) = d2(0, 2); rhoref(S, 2) = d2(0, 3);
        rhoref(S, 3) = d2(1, 2); rhoref(S, 4) = d2(1, 3); rhoref(S, 5) = d2(2, 3);
    }
    const double pw0[3] = {cws[0][0], cws[0][1], cws[0][2]};
    double R[3][3], t[3];
    if (STOP >= 5 && STOP <= 7 || STOP == 11) {
        double betas[4] = {0, 0, 0, 0};
        find_betas<1>(SlabView{S}, betas);
        gauss_newton(SlabView{S}, betas);
        acc += compute_R_and_t(st, K, SlabView{S}, betas, pw0, R, t);
    }
    if (STOP >= 6 && STOP <= 7 || STOP == 12) {
        double betas[4] = {0, 0, 0, 0};
        find_betas<2>(SlabView{S}, betas);
        gauss_newton(SlabView{S}, betas);
        acc += compute_R_and_t(st, K, SlabView{S}, betas, pw0, R, t);
    }
    if (STOP == 7 || STOP == 13) {
        double betas[4] = {0, 0, 0, 0};
        find_betas<3>(SlabView{S}, betas);
        gauss_newton(SlabView{S}, betas);
        acc += compute_R_and_t(st, K, SlabView{S}, betas, pw0, R, t);
    }
    if (STOP == 21 || STOP == 22 || STOP == 23) {  // SVD only
        double betas[4] = {0, 0, 0, 0};
        if (STOP == 21) find_betas<1>(SlabView{S}, betas);
        if (STOP == 22) find_betas<2>(SlabView{S}, betas);
        if (STOP == 23) find_betas<3>(SlabView{S}, betas);
        acc += betas[0] + betas[1] + betas[2] + betas[3];
    }
    if (STOP == 31) {  // GN only (betas from L)
        double betas[4] = {S(slab_free(0)), S(slab_free(1)), S(slab_free(2)), S(slab_free(3))};
        gauss_newton(SlabView{S}, betas);
        acc += betas[0] + betas[1] + betas[2] + betas[3];
    }
    if (STOP == 41) {  // R and t only
        double betas[4] = {S(slab_free(0)), S(slab_free(1)), S(slab_free(2)), S(slab_free(3))};
        acc += compute_R_and_t(st, K, SlabView{S}, betas, pw0, R, t);
    }
    out[h] = acc + R[0][0] + t[2];
}

template <int STOP>
static float time_kernel(int nwg, const float4* pts, const float2* uv, const int4* smp, int H, double* out, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    phase_kernel<STOP><<<nwg, 64>>>(pts, uv, smp, H, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) phase_kernel<STOP><<<nwg, 64>>>(pts, uv, smp, H, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int N = 2000, H = (argc > 1) ? atoi(argv[1]) : 19200;
    std::vector<float4> pts(N);
    std::vector<float2> uv(N);
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(s >> 11) / 9007199254740992.0; };
    for (int i = 0; i < N; ++i) {
        double X = rnd() * 8 - 4, Y = rnd() * 6 - 3, Z = 2 + rnd() * 10;
        pts[i] = make_float4((float)X, (float)Y, (float)Z, 1.0f);
        double u = 367.215 + 458.654 * X / Z, v = 248.375 + 457.296 * Y / Z;
        if (rnd() < 0.6) { u = rnd() * 752; v = rnd() * 480; }
        uv[i] = make_float2((float)u, (float)v);
    }
    std::vector<int4> smp(H);
    for (int h = 0; h < H; ++h) {
        int a[4];
        for (int k = 0; k < 4; ++k) {
            bool dup;
            do {
                a[k] = (int)(rnd() * N);
                dup = false;
                for (int j = 0; j < k; ++j) dup |= a[j] == a[k];
            } while (dup);
        }
        smp[h] = make_int4(a[0], a[1], a[2], a[3]);
    }
    float4* dp; float2* du; int4* ds; double* dout;
    CK(hipMalloc(&dp, N * sizeof(float4)));
    CK(hipMalloc(&du, N * sizeof(float2)));
    CK(hipMalloc(&ds, H * sizeof(int4)));
    CK(hipMalloc(&dout, H * sizeof(double)));
    CK(hipMemcpy(dp, pts.data(), N * sizeof(float4), hipMemcpyHostToDevice));
    CK(hipMemcpy(du, uv.data(), N * sizeof(float2), hipMemcpyHostToDevice));
    CK(hipMemcpy(ds, smp.data(), H * sizeof(int4), hipMemcpyHostToDevice));
    const int nwg = (H + 63) / 64, reps = 20;
    printf("H=%d nwg=%d\n", H, nwg);
    printf("1 cp+alphas       %8.1f us\n", 1e3 * time_kernel<1>(nwg, dp, du, ds, H, dout, reps));
    printf("2 +MtM            %8.1f us\n", 1e3 * time_kernel<2>(nwg, dp, du, ds, H, dout, reps));
    printf("3 +tridiag        %8.1f us\n", 1e3 * time_kernel<3>(nwg, dp, du, ds, H, dout, reps));
    printf("50 +QR no-Q       %8.1f us\n", 1e3 * time_kernel<50>(nwg, dp, du, ds, H, dout, reps));
    printf("4 +QR             %8.1f us\n", 1e3 * time_kernel<4>(nwg, dp, du, ds, H, dout, reps));
    printf("5 +branch1        %8.1f us\n", 1e3 * time_kernel<5>(nwg, dp, du, ds, H, dout, reps));
    printf("6 +branch2        %8.1f us\n", 1e3 * time_kernel<6>(nwg, dp, du, ds, H, dout, reps));
    printf("7 +branch3 (full) %8.1f us\n", 1e3 * time_kernel<7>(nwg, dp, du, ds, H, dout, reps));
    printf("11 eig+branch1    %8.1f us\n", 1e3 * time_kernel<11>(nwg, dp, du, ds, H, dout, reps));
    printf("12 eig+branch2    %8.1f us\n", 1e3 * time_kernel<12>(nwg, dp, du, ds, H, dout, reps));
    printf("13 eig+branch3    %8.1f us\n", 1e3 * time_kernel<13>(nwg, dp, du, ds, H, dout, reps));
    printf("21 eig+svd4       %8.1f us\n", 1e3 * time_kernel<21>(nwg, dp, du, ds, H, dout, reps));
    printf("22 eig+svd3       %8.1f us\n", 1e3 * time_kernel<22>(nwg, dp, du, ds, H, dout, reps));
    printf("23 eig+svd5       %8.1f us\n", 1e3 * time_kernel<23>(nwg, dp, du, ds, H, dout, reps));
    printf("31 eig+GN         %8.1f us\n", 1e3 * time_kernel<31>(nwg, dp, du, ds, H, dout, reps));
    printf("41 eig+R_and_t    %8.1f us\n", 1e3 * time_kernel<41>(nwg, dp, du, ds, H, dout, reps));
    return 0;
}
