// eig_probe.hip — diagnostic: where the single-event latency of the EPnP stages goes.  One wave (or
// a few) on an idle GPU, phase stamps from s_memrealtime (100 MHz) and the shader clock, on
// realistic inputs built on the host with the product's own RSC_HD routines:
//   refine  rows_eig12_ev4<4> on the MtM of a 500-row Refine (phases: Householder / accumulate /
//           chase / sort), plus the number of rotations the chase applies (host count);
//   hyp1    group_eig12_ev4<2> on one 4-point hypothesis (one pair active);
//   hyp20   the same on 20 hypotheses in one wave (the product's pair wave);
//   betas   compute_L_6x10 / find_betas<a> / gauss_newton / compute_R_and_t of one hypothesis,
//           a = 1, 2, 3 on three single-wave workgroups.
// Not part of the product.  Build: make -C tools eig_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <random>
#include <cstring>

__device__ unsigned long long g_st[8][16];
__device__ unsigned long long g_clk[8][16];
#define RSC_EIG_PHASE(k)                                                       \
    do {                                                                       \
        if (threadIdx.x == 0) {                                                \
            g_st[blockIdx.x][1 + (k)] = wall_clock64();                        \
            g_clk[blockIdx.x][1 + (k)] = clock64();                            \
        }                                                                      \
    } while (0)
#include "../orb-slam2-optimized_amd/csrc/rsc_quad.h"

using namespace rsc;

// Instrumented copy of the product chase (per-sweep bookkeeping vs slot time).
namespace rsc {
template <typename S, int n, typename QApply>
__device__ bool tridiag_qr_st(S (&diag)[n], S (&sub)[n - 1], QApply&& qapply, int (&perm)[n], unsigned long long (&acc)[4]) {
    const int maxIterations = 30;
    int end = n - 1, start = 0, iter = 0;
    const S considerAsZero = lim<S>::min();
    const S precision_inv = S(1) / lim<S>::eps();
    // Branch-free sweep bookkeeping.  Each `if` of Eigen's loop (deflation test, end/start
    // searches, shift cases, the chase's edge updates) compiled to a branch — a scalar branch when
    // the group's values are uniform, an exec-mask region otherwise — and the sweep's ~100 branches
    // cost more than its rotations (one 12x12 Refine chase: 156 rotations, 23 sweeps, 221 k shader
    // clocks, 3x the make_givens chains; tools/eig_probe.hip).  Here every test is a value select on
    // the same operands (same results, bit for bit); the only branches left are the loop exit and
    // the chase's per-slot range guard, which skips slots outside [start, end).  Conditions are
    // combined with the non-short-circuit & and | (a short-circuit || is a branch again).
    // Single-exit loop (Eigen's two `break`s folded into `run`): with several exits the CFG
    // structurizer nests the loop and every lane pays for the extra control flow.
    bool run = true;
    while (run) {
        const unsigned long long t0 = clock64();
        // for (i = start; i < end; ++i): |sub| < considerAsZero, or (sub/eps)^2 <= |d_i| + |d_i+1|
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
            const S scaled = precision_inv * sub[i];
            const bool z = (rabs(sub[i]) < considerAsZero) | (scaled * scaled <= (rabs(diag[i]) + rabs(diag[i + 1])));
            sub[i] = (z & (i >= start) & (i < end)) ? S(0) : sub[i];
        }
        // The two searches on a bit mask of the nonzero sub-diagonal entries (a find-last-set instead
        // of an 11-step select chain each):
        // while (end > 0 && sub[end-1] == 0) end--;  ->  end = 1 + last nonzero index below end, or 0
        unsigned nz = 0u;
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) nz |= (sub[i] != S(0)) ? (1u << i) : 0u;
        const unsigned live = nz & ((1u << end) - 1u);
        end = live ? 32 - __builtin_clz(live) : 0;
        run = end > 0;
        iter = run ? iter + 1 : iter;
        run = run & (iter <= maxIterations * n);
        if (!run) continue;
        // start = end - 1; while (start > 0 && sub[start-1] != 0) start--;
        //   ->  start = 1 + last zero index below end - 1, or 0
        const unsigned zero = ~nz & ((1u << (end - 1)) - 1u);
        start = zero ? 32 - __builtin_clz(zero) : 0;
        // ---- tridiagonal_qr_step(diag, sub, start, end) ----
        S dEm1 = S(0), dE = S(0), eE = S(0), dS = S(0), zS = S(0);
        RSC_UNROLL for (int j = 1; j < n; ++j) {
            const bool m = j == end;
            dEm1 = m ? diag[j - 1] : dEm1;
            dE = m ? diag[j] : dE;
            eE = m ? sub[j - 1] : eE;
        }
        RSC_UNROLL for (int j = 0; j < n - 1; ++j) {
            const bool m = j == start;
            dS = m ? diag[j] : dS;
            zS = m ? sub[j] : zS;
        }
        // Wilkinson shift; the three cases of Eigen are evaluated side by side and selected
        // (td == 0: mu - |e|; e^2 underflows: the two-quotient form; otherwise e^2/(td +- h))
        const S td = (dEm1 - dE) * S(0.5);
        const S e = eE;
        const S e2 = eE * eE;
        const S h = eig_hypot(td, e);
        const S mu_z = dE - rabs(e);
        const S mu_u = dE - (e / (td + (td > S(0) ? S(1) : S(-1)))) * (e / h);
        const S mu_n = dE - e2 / (td + (td > S(0) ? h : -h));
        const S mu = (td == S(0)) ? mu_z : ((e2 == S(0)) ? mu_u : mu_n);
        S x = dS - mu;
        const unsigned long long t1 = clock64();
        acc[0] += t1 - t0;
        S z = zS;
        RSC_UNROLL for (int k = 0; k < n - 1; ++k) {
            if (k >= start && k < end) {
                if constexpr (qr_has_prefetch<QApply>::value) qapply.prefetch(k);
                S c, s;
                make_givens(x, z, c, s);
                S sdk = s * diag[k] + c * sub[k];
                S dkp1 = s * sub[k] + c * diag[k + 1];
                diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
                diag[k + 1] = s * sdk + c * dkp1;
                sub[k] = c * sdk - s * dkp1;
                if (k > 0) sub[k - 1] = (k > start) ? c * sub[k - 1] - s * z : sub[k - 1];
                x = sub[k];
                if (k < n - 2) {
                    const bool m = k < end - 1;
                    z = m ? -s * sub[k + 1] : z;
                    sub[k + 1] = m ? c * sub[k + 1] : sub[k + 1];
                }
                // Eigen skips identity rotations; qapply receives the flag and selects (a
                // conditional call here gets tail-duplicated into the loop latch, which turns
                // the QR loop into a nested loop that serialises the lanes of a wave)
                qapply(k, c, s, !(c == S(1) && s == S(0)));
            }
        }
        acc[1] += clock64() - t1;
        acc[2] += 1;
        RSC_LOOP_FENCE();
    }
    const bool ok = (iter <= maxIterations * n);
    RSC_UNROLL for (int i = 0; i < n; ++i) perm[i] = i;
    if (ok) eig_sort<S, n>(diag, perm);
    return ok;
}

}  // namespace rsc

// The round-3 (branchy) chase, for the A/B in chase_only<3>.
namespace rsc {
template <typename S, int n, typename QApply>
RSC_HD bool tridiag_qr_old(S (&diag)[n], S (&sub)[n - 1], QApply&& qapply, int (&perm)[n]) {
    const int maxIterations = 30;
    int end = n - 1, start = 0, iter = 0;
    const S considerAsZero = lim<S>::min();
    const S precision_inv = S(1) / lim<S>::eps();
    // Single-exit loop (Eigen's two `break`s folded into `run`): with several exits the CFG
    // structurizer nests the loop and every lane pays for the extra control flow.
    bool run = true;
    while (run) {
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
            if (i >= start && i < end) {
                if (rabs(sub[i]) < considerAsZero) {
                    sub[i] = S(0);
                } else {
                    const S scaled = precision_inv * sub[i];
                    if (scaled * scaled <= (rabs(diag[i]) + rabs(diag[i + 1]))) sub[i] = S(0);
                }
            }
        }
        RSC_UNROLL for (int i = n - 2; i >= 0; --i)
            if (i == end - 1 && sub[i] == S(0)) end--;
        run = end > 0;
        if (run) {
            iter++;
            run = iter <= maxIterations * n;
        }
        if (!run) continue;
        start = end - 1;
        RSC_UNROLL for (int i = n - 2; i >= 0; --i)
            if (i == start - 1 && sub[i] != S(0)) start--;
        // ---- tridiagonal_qr_step(diag, sub, start, end) ----
        S dEm1 = S(0), dE = S(0), eE = S(0), dS = S(0), zS = S(0);
        RSC_UNROLL for (int j = 1; j < n; ++j)
            if (j == end) { dEm1 = diag[j - 1]; dE = diag[j]; eE = sub[j - 1]; }
        RSC_UNROLL for (int j = 0; j < n - 1; ++j)
            if (j == start) { dS = diag[j]; zS = sub[j]; }
        S td = (dEm1 - dE) * S(0.5);
        S e = eE;
        S mu = dE;
        if (td == S(0)) {
            mu -= rabs(e);
        } else {
            S e2 = eE * eE;
            S h = eig_hypot(td, e);
            if (e2 == S(0))
                mu -= (e / (td + (td > S(0) ? S(1) : S(-1)))) * (e / h);
            else
                mu -= e2 / (td + (td > S(0) ? h : -h));
        }
        S x = dS - mu;
        S z = zS;
        RSC_UNROLL for (int k = 0; k < n - 1; ++k) {
            if (k >= start && k < end) {
                if constexpr (qr_has_prefetch<QApply>::value) qapply.prefetch(k);
                S c, s;
                make_givens(x, z, c, s);
                S sdk = s * diag[k] + c * sub[k];
                S dkp1 = s * sub[k] + c * diag[k + 1];
                diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
                diag[k + 1] = s * sdk + c * dkp1;
                sub[k] = c * sdk - s * dkp1;
                if (k > 0 && k > start) sub[k - 1] = c * sub[k - 1] - s * z;
                x = sub[k];
                if (k < n - 2 && k < end - 1) {
                    z = -s * sub[k + 1];
                    sub[k + 1] = c * sub[k + 1];
                }
                // Eigen skips identity rotations; qapply receives the flag and selects (a
                // conditional call here gets tail-duplicated into the loop latch, which turns
                // the QR loop into a nested loop that serialises the lanes of a wave)
                qapply(k, c, s, !(c == S(1) && s == S(0)));
            }
        }
        RSC_LOOP_FENCE();
    }
    const bool ok = (iter <= maxIterations * n);
    RSC_UNROLL for (int i = 0; i < n; ++i) perm[i] = i;
    if (ok) eig_sort<S, n>(diag, perm);
    return ok;
}

}  // namespace rsc
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void stamp(int k) {
    if (threadIdx.x == 0) { g_st[blockIdx.x][k] = wall_clock64(); g_clk[blockIdx.x][k] = clock64(); }
}
__device__ __forceinline__ void wstamp(int b, int k) {
    if ((threadIdx.x & 63) == 0) { g_st[b][k] = wall_clock64(); g_clk[b][k] = clock64(); }
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Refine form: MtM (lower triangle, row-major [144]) of one problem.
__global__ __launch_bounds__(64) void refine_eig(const double* __restrict__ mtm, double* __restrict__ out) {
    __shared__ double T[144];
    __shared__ double E[128];
    const int lane = threadIdx.x;
    for (int e = lane; e < 144; e += 64) T[e] = mtm[e];
    wsync();
    stamp(0);
    double ev[4];
    rows_eig12_ev4<4>(T, E, lane, [] { wsync(); }, ev);
    stamp(5);
    if (lane < 12) for (int c = 0; c < 4; ++c) out[lane * 4 + c] = ev[c];
}

// Hypothesis form: HPW pairs, each on its own MtM.
template <int HPW>
__global__ __launch_bounds__(64) void hyp_eig(const double* __restrict__ mtm, double* __restrict__ out) {
    __shared__ double R[20 * kQuadRegion];
    const int lane = threadIdx.x, g = lane / 2, q = lane % 2;
    if (g >= HPW) return;
    double* T = R + g * kQuadRegion;
    double* E = T + kQuadT;
    for (int e = q; e < 144; e += 2) T[e] = mtm[g * 144 + e];
    wsync();
    stamp(0);
    double ev[6][4];
    group_eig12_ev4<2>(T, E, q, [] { wsync(); }, ev);
    stamp(5);
    for (int j = 0; j < 6; ++j)
        for (int c = 0; c < 4; ++c) out[(g * 12 + 2 * j + q) * 4 + c] = ev[j][c];
}

// Betas: block a = approximation; every lane computes the same hypothesis (lane-private L in LDS).
struct ProbeHyp {
    double ev[48], cws[12], al[16], pw[12], u[8];
    double fx, fy, cx, cy;
};
template <int MODE>
__global__ __launch_bounds__(192) void betas_probe(const ProbeHyp* __restrict__ hp, int H_n, double* __restrict__ out) {
    __shared__ double Lsh[3][66 * 64];
    const int lane = threadIdx.x & 63, apx = MODE == 1 ? threadIdx.x / 64 : blockIdx.x;
    const int blk = MODE == 1 ? apx : blockIdx.x;
    const ProbeHyp& H = hp[MODE == 2 ? lane % H_n : 0];
    const SplitView V{H.ev, Lsh[apx] + lane, 64};
    wstamp(blk, 0);
    compute_L_6x10(V);
    {
        auto d2 = [&](int a, int b) {
            double x = H.cws[3 * a] - H.cws[3 * b], y = H.cws[3 * a + 1] - H.cws[3 * b + 1], z = H.cws[3 * a + 2] - H.cws[3 * b + 2];
            return x * x + y * y + z * z;
        };
        V.rho(0) = d2(0, 1); V.rho(1) = d2(0, 2); V.rho(2) = d2(0, 3);
        V.rho(3) = d2(1, 2); V.rho(4) = d2(1, 3); V.rho(5) = d2(2, 3);
    }
    double betas[4] = {0.0, 0.0, 0.0, 0.0};
    wstamp(blk, 1);
    if (apx == 0) find_betas<1>(V, betas);
    else if (apx == 1) find_betas<2>(V, betas);
    else find_betas<3>(V, betas);
    wstamp(blk, 2);
    gauss_newton(V, betas);
    wstamp(blk, 3);
    HypStore<4> st;
    for (int i = 0; i < 4; ++i) {
        for (int c = 0; c < 3; ++c) st.pw_[i][c] = H.pw[3 * i + c];
        for (int c = 0; c < 2; ++c) st.u_[i][c] = H.u[2 * i + c];
        for (int j = 0; j < 4; ++j) st.al_[i][j] = H.al[4 * i + j];
    }
    st.rows_ = 4; st.spw = nullptr; st.sal = nullptr;
    const Intrinsics K{H.fx, H.fy, H.cx, H.cy};
    const double pw0[3] = {H.cws[0], H.cws[1], H.cws[2]};
    double R[3][3], t[3];
    wstamp(blk, 4);
    const double err = compute_R_and_t(st, K, V, betas, pw0, R, t);
    wstamp(blk, 5);
    if (lane == 0 || MODE == 2) {
        out[apx * 16] = err;
        for (int k = 0; k < 9; ++k) out[apx * 16 + 1 + k] = R[k / 3][k % 3];
        for (int k = 0; k < 3; ++k) out[apx * 16 + 10 + k] = t[k];
    }
}

// Bare make_givens chain on one wave (clock reference).
__global__ __launch_bounds__(64) void givens_chain(double* out, int iters) {
    double x = 1.5 + threadIdx.x * 1e-3, z = 0.75;
    stamp(0);
    for (int i = 0; i < iters; ++i) {
        double c, s;
        make_givens(x, z, c, s);
        x = c * 3.0 + s;
        z = s * 0.5 + 0.25;
    }
    stamp(1);
    out[threadIdx.x] = x + z;
}

// The QR chase alone on one tridiagonal problem (diag/sub prepared by tridiag_of), lanes 0..11 with
// identical values (the Refine's form): MODE 0 without a rotation sink, 1 with one row of Q in each
// lane's VGPRs (RegRowQ), 2 with Q rows in LDS (the pair kernel's GroupLdsRows<4>).
__global__ void tridiag_of(double* mtm, double* ds) {
    if (threadIdx.x != 0) return;
    double W[160];
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < 12; ++c) W[r * 12 + c] = (c <= r) ? mtm[r * 12 + c] : 0.0;
    double diag[12], sub[11];
    sym_eig12_tridiag(LaneMat{W, 1}, diag, sub);
    for (int i = 0; i < 12; ++i) ds[i] = diag[i];
    for (int i = 0; i < 11; ++i) ds[12 + i] = sub[i];
    int rot = 0, it = 0;
    auto qa = [&](int, double, double, bool apply) { rot += apply ? 1 : 0; };
    int perm[12];
    double d2[12], s2[11];
    for (int i = 0; i < 12; ++i) d2[i] = diag[i];
    for (int i = 0; i < 11; ++i) s2[i] = sub[i];
    tridiag_qr<double, 12>(d2, s2, qa, perm);
    ds[23] = rot;
}
struct NoSink {
    RSC_HD void operator()(int, double, double, bool) const {}
};
template <int MODE>
__global__ __launch_bounds__(64) void chase_only(const double* __restrict__ ds, double* __restrict__ out) {
    __shared__ double T[144];
    const int lane = threadIdx.x;
    if (lane >= 12) return;
    double diag[12], sub[11], row[12];
    for (int i = 0; i < 12; ++i) diag[i] = ds[i];
    for (int i = 0; i < 11; ++i) sub[i] = ds[12 + i];
    for (int c = 0; c < 12; ++c) row[c] = (c == lane) ? 1.0 : 0.0;
    for (int c = 0; c < 12; ++c) T[lane * 12 + c] = row[c];
    wsync();
    int perm[12];
    stamp(0);
    if (MODE == 0) {
        tridiag_qr<double, 12>(diag, sub, NoSink{}, perm);
    } else if (MODE == 1) {
        RegRowQ qa{row};
        tridiag_qr<double, 12>(diag, sub, qa, perm);
    } else if (MODE == 2) {
        GroupLdsRows<4> qa{T, lane & 3};
        tridiag_qr<double, 12>(diag, sub, qa, perm);
    } else {
        RegRowQ qa{row};
        tridiag_qr_old<double, 12>(diag, sub, qa, perm);
    }
    stamp(1);
    double acc = 0;
    for (int i = 0; i < 12; ++i) acc += diag[i] + row[i] + T[lane * 12 + i];
    out[lane] = acc + perm[0];
}


__device__ unsigned long long g_acc[4];
__global__ __launch_bounds__(64) void chase_stamped(const double* __restrict__ ds, double* __restrict__ out) {
    const int lane = threadIdx.x;
    if (lane >= 12) return;
    double diag[12], sub[11], row[12];
    for (int i = 0; i < 12; ++i) diag[i] = ds[i];
    for (int i = 0; i < 11; ++i) sub[i] = ds[12 + i];
    for (int c = 0; c < 12; ++c) row[c] = (c == lane) ? 1.0 : 0.0;
    int perm[12];
    unsigned long long acc[4] = {0, 0, 0, 0};
    stamp(0);
    RegRowQ qa{row};
    tridiag_qr_st<double, 12>(diag, sub, qa, perm, acc);
    stamp(1);
    if (lane == 0) for (int i = 0; i < 4; ++i) g_acc[i] = acc[i];
    double a = 0;
    for (int i = 0; i < 12; ++i) a += diag[i] + row[i];
    out[lane] = a + perm[0];
}


// The Refine kernel's betas structure: 256 threads, the slab (eigenvectors, L, rho) in LDS read
// through SlabView, lane 0 of waves 0..2 running find_betas<w+1> + gauss_newton (MODE 0) — or all 64
// lanes of the wave running it redundantly (MODE 1).
template <int MODE>
__global__ __launch_bounds__(256) void refine_betas_like(const double* __restrict__ slab_in, double* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) double slab[kSlabDoubles];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int e = tid; e < kSlabDoubles; e += 256) slab[e] = slab_in[e];
    __syncthreads();
    wstamp(wave, 0);
    if (wave < 3) {
        // MODE 2: the same slab through a base the compiler sees as lane-varying (an inline-asm VGPR
        // zero), so the values read are divergent and data-dependent ifs stay selects / exec masks
        int z = 0;
        if (MODE == 2) asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        const SlabView SV{LaneMat{slab + z, 1}};
        if (MODE >= 1 || lane == 0) {
            double betas[4] = {0.0, 0.0, 0.0, 0.0};
            if (wave == 0) find_betas<1>(SV, betas);
            else if (wave == 1) find_betas<2>(SV, betas);
            else find_betas<3>(SV, betas);
            wstamp(wave, 1);
            gauss_newton(SV, betas);
            wstamp(wave, 2);
            if (lane == 0) for (int k = 0; k < 4; ++k) out[wave * 4 + k] = betas[k];
        }
    }
    __syncthreads();
}


// Which factor makes the Refine-shaped betas slow: (a) 64-thread workgroups, SlabView over a
// shared slab (wave = blockIdx); (b) 256-thread workgroup, SplitView per lane (stride 64).
__global__ __launch_bounds__(64) void slab_betas_64(const double* __restrict__ slab_in, double* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) double slab[kSlabDoubles];
    const int lane = threadIdx.x, wave = blockIdx.x;
    for (int e = lane; e < kSlabDoubles; e += 64) slab[e] = slab_in[e];
    __syncthreads();
    wstamp(wave, 0);
    const SlabView SV{LaneMat{slab, 1}};
    double betas[4] = {0.0, 0.0, 0.0, 0.0};
    if (wave == 0) find_betas<1>(SV, betas);
    else if (wave == 1) find_betas<2>(SV, betas);
    else find_betas<3>(SV, betas);
    wstamp(wave, 1);
    gauss_newton(SV, betas);
    wstamp(wave, 2);
    if (lane == 0) for (int k = 0; k < 4; ++k) out[wave * 4 + k] = betas[k];
}
__global__ __launch_bounds__(256) void split_betas_256(const double* __restrict__ slab_in, double* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) double Lsh[3][66 * 64];
    __shared__ double ev[48];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 48) ev[tid] = slab_in[(tid / 4) * 12 + tid % 4];
    if (wave < 3) {
        for (int q = 0; q < 66; ++q) Lsh[wave][q * 64 + lane] = slab_in[slab_free(q)];
    }
    __syncthreads();
    wstamp(wave, 0);
    if (wave < 3) {
        const SplitView V{ev, Lsh[wave] + lane, 64};
        double betas[4] = {0.0, 0.0, 0.0, 0.0};
        if (wave == 0) find_betas<1>(V, betas);
        else if (wave == 1) find_betas<2>(V, betas);
        else find_betas<3>(V, betas);
        wstamp(wave, 1);
        gauss_newton(V, betas);
        wstamp(wave, 2);
        if (lane == 0) for (int k = 0; k < 4; ++k) out[wave * 4 + k] = betas[k];
    }
    __syncthreads();
}

// The betas kernel's cross-workgroup hand-off (stores, agent release, atomic, agent acquire, loads).
__global__ __launch_bounds__(64) void fence_probe(double* buf, unsigned* ctr) {
    const int lane = threadIdx.x;
    stamp(0);
    buf[blockIdx.x * 64 + lane] = lane * 1.5;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(1);
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __builtin_amdgcn_readlane(prev, 0);
    stamp(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(3);
    const double v = buf[((blockIdx.x + 1) % gridDim.x) * 64 + lane];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(4);
    buf[4096 + blockIdx.x * 64 + lane] = v + prev;
}

// ---- host inputs ----
struct Scene {
    std::vector<double> pw, u;
    double fx = 458.654, fy = 457.296, cx = 367.215, cy = 248.375;
};
static Scene make_scene(std::mt19937& g, int n) {
    std::uniform_real_distribution<double> U(-1, 1);
    Scene s;
    for (int i = 0; i < n; ++i) {
        double X = 3 * U(g), Y = 2 * U(g), Z = 5 + 3 * U(g);
        s.pw.push_back((float)X); s.pw.push_back((float)Y); s.pw.push_back((float)Z);
        double u = s.cx + s.fx * X / Z + 0.5 * U(g), v = s.cy + s.fy * Y / Z + 0.5 * U(g);
        s.u.push_back((float)u); s.u.push_back((float)v);
    }
    return s;
}

// Inputs are built on the device with the product's routines (an -O3 host build of the unrolled
// 12x12 code takes minutes).
__global__ void setup_hyp(const double* __restrict__ pw, const double* __restrict__ u, const int* __restrict__ idx,
                          int H, double fx, double fy, double cx, double cy, double* __restrict__ mtm,
                          ProbeHyp* __restrict__ hp) {
    const int h = threadIdx.x;
    if (h >= H) return;
    HypStore<4> st;
    for (int i = 0; i < 4; ++i) {
        const int k = idx[4 * h + i];
        for (int c = 0; c < 3; ++c) st.pw_[i][c] = pw[3 * k + c];
        for (int c = 0; c < 2; ++c) st.u_[i][c] = u[2 * k + c];
    }
    st.rows_ = 4; st.spw = nullptr; st.sal = nullptr;
    double cws[4][3];
    control_points_and_alphas(st, cws);
    const Intrinsics K{fx, fy, cx, cy};
    double* S = mtm + h * 160;
    build_MtM(st, K, LaneMat{S, 1});
    if (hp) {
        double M[160];
        for (int e = 0; e < 160; ++e) M[e] = S[e];
        sym_eig12(LaneMat{M, 1});
        for (int r = 0; r < 12; ++r)
            for (int c = 0; c < 4; ++c) hp[h].ev[r * 4 + c] = M[r * 12 + c];
        for (int i = 0; i < 4; ++i)
            for (int c = 0; c < 3; ++c) hp[h].cws[3 * i + c] = cws[i][c];
        for (int i = 0; i < 4; ++i) {
            for (int c = 0; c < 3; ++c) hp[h].pw[3 * i + c] = st.pw_[i][c];
            for (int c = 0; c < 2; ++c) hp[h].u[2 * i + c] = st.u_[i][c];
            for (int j = 0; j < 4; ++j) hp[h].al[4 * i + j] = st.al_[i][j];
        }
        hp[h].fx = fx; hp[h].fy = fy; hp[h].cx = cx; hp[h].cy = cy;
    }
}

__global__ void setup_refine(double* pws, const double* us, double* als, int n, double fx, double fy, double cx,
                             double cy, double* __restrict__ mtm) {
    if (threadIdx.x != 0) return;
    RowStore st{n, n, pws, us, als};
    double cws[4][3];
    control_points_and_alphas(st, cws);
    const Intrinsics K{fx, fy, cx, cy};
    build_MtM(st, K, LaneMat{mtm, 1});
}


// ProbeHyp from a Refine problem (500 rows): its eigenvectors and control points (the betas
// chain on a least-squares L_6x10); pw/u/al of its first four rows.
__global__ void setup_refine_hyp(double* pws, const double* us, double* als, int n, double fx, double fy, double cx,
                                 double cy, double* __restrict__ M, ProbeHyp* __restrict__ hp) {
    if (threadIdx.x != 0) return;
    RowStore st{n, n, pws, us, als};
    double cws[4][3];
    control_points_and_alphas(st, cws);
    const Intrinsics K{fx, fy, cx, cy};
    for (int e = 0; e < 160; ++e) M[e] = 0.0;
    build_MtM(st, K, LaneMat{M, 1});
    sym_eig12(LaneMat{M, 1});
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < 4; ++c) hp->ev[r * 4 + c] = M[r * 12 + c];
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 3; ++c) hp->cws[3 * i + c] = cws[i][c];
    {
        const SlabView SV{LaneMat{M, 1}};
        compute_L_6x10(SV);
        auto d2 = [&](int a, int b) {
            double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
            return x * x + y * y + z * z;
        };
        SV.rho(0) = d2(0, 1); SV.rho(1) = d2(0, 2); SV.rho(2) = d2(0, 3);
        SV.rho(3) = d2(1, 2); SV.rho(4) = d2(1, 3); SV.rho(5) = d2(2, 3);
    }
    for (int i = 0; i < 4; ++i) {
        for (int c = 0; c < 3; ++c) hp->pw[3 * i + c] = pws[3 * i + c];
        for (int c = 0; c < 2; ++c) hp->u[2 * i + c] = us[2 * i + c];
        for (int j = 0; j < 4; ++j) hp->al[4 * i + j] = als[4 * i + j];
    }
    hp->fx = fx; hp->fy = fy; hp->cx = cx; hp->cy = cy;
}

// rotations applied by the chase of MtM p (stride 160), one lane per problem
__global__ void count_rot(double* mtm, int P, int* out) {
    const int p = threadIdx.x;
    if (p >= P) return;
    double* M = mtm + p * 160;
    double W[144];
    for (int r = 0; r < 12; ++r)
        for (int c = 0; c < 12; ++c) W[r * 12 + c] = (c <= r) ? M[r * 12 + c] : 0.0;
    double diag[12], sub[11];
    sym_eig12_tridiag(LaneMat{W, 1}, diag, sub);
    int rot = 0;
    auto qa = [&](int, double, double, bool apply) { rot += apply ? 1 : 0; };
    int perm[12];
    tridiag_qr<double, 12>(diag, sub, qa, perm);
    out[p] = rot;
}

static void report(const char* name, int blk, int nph, const char* const* names) {
    unsigned long long st[8][16], ck[8][16];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_st), sizeof(st)));
    CK(hipMemcpyFromSymbol(ck, HIP_SYMBOL(g_clk), sizeof(ck)));
    const double tot_us = (st[blk][nph] - st[blk][0]) / 100.0;
    const double ghz = (double)(ck[blk][nph] - ck[blk][0]) / (tot_us * 1e3);
    printf("%-22s total %8.2f us  (shader clock %.2f GHz)\n", name, tot_us, ghz);
    for (int k = 0; k < nph; ++k)
        printf("    %-18s %8.2f us  %9llu clk\n", names[k], (st[blk][k + 1] - st[blk][k]) / 100.0,
               ck[blk][k + 1] - ck[blk][k]);
}

int main() {
    std::mt19937 g(7);
    Scene s = make_scene(g, 600);
    const int n = 600;
    double *d_pw, *d_u, *d_als, *d_mtm, *d_out;
    int *d_idx, *d_rot;
    CK(hipMalloc(&d_pw, 3 * n * 8)); CK(hipMalloc(&d_u, 2 * n * 8)); CK(hipMalloc(&d_als, 4 * n * 8));
    CK(hipMalloc(&d_mtm, 22 * 160 * 8)); CK(hipMalloc(&d_out, 8192 * 8));
    CK(hipMalloc(&d_idx, 80 * 4)); CK(hipMalloc(&d_rot, 32 * 4));
    CK(hipMemcpy(d_pw, s.pw.data(), 3 * n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_u, s.u.data(), 2 * n * 8, hipMemcpyHostToDevice));
    const char* eigph[] = {"householder", "accumulate", "chase", "sort/extract", "exit"};
    double* d_ds_g = nullptr;
    int rot[32];
    // Refine (500 rows)
    {
        setup_refine<<<1, 64>>>(d_pw, d_u, d_als, 500, s.fx, s.fy, s.cx, s.cy, d_mtm + 21 * 160);
        count_rot<<<1, 64>>>(d_mtm + 21 * 160, 1, d_rot);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(rot, d_rot, 4, hipMemcpyDeviceToHost));
        printf("refine MtM (n=500): chase applies %d rotations\n", rot[0]);
        // compact to [144] for the kernel
        double m[160];
        CK(hipMemcpy(m, d_mtm + 21 * 160, 160 * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(d_out, m, 144 * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_out + 4096, m, 144 * 8, hipMemcpyHostToDevice));
        for (int rep = 0; rep < 3; ++rep) {
            refine_eig<<<1, 64>>>(d_out, d_out + 512);
            CK(hipDeviceSynchronize());
        }
        report("refine rows_eig12<4>", 0, 5, eigph);
        CK(hipMalloc(&d_ds_g, 32 * 8));
        double* d_ds = d_ds_g;
        tridiag_of<<<1, 64>>>(d_out, d_ds);
        CK(hipDeviceSynchronize());
        double ds[24];
        CK(hipMemcpy(ds, d_ds, sizeof(ds), hipMemcpyDeviceToHost));
        printf("refine tridiagonal: %d rotations\n", (int)ds[23]);
        const char* cph[] = {"chase"};
        for (int rep = 0; rep < 3; ++rep) { chase_only<0><<<1, 64>>>(d_ds, d_out + 1024); CK(hipDeviceSynchronize()); }
        report("chase, no sink", 0, 1, cph);
        for (int rep = 0; rep < 3; ++rep) { chase_only<1><<<1, 64>>>(d_ds, d_out + 1024); CK(hipDeviceSynchronize()); }
        report("chase, VGPR rows", 0, 1, cph);
        for (int rep = 0; rep < 3; ++rep) { chase_only<2><<<1, 64>>>(d_ds, d_out + 1024); CK(hipDeviceSynchronize()); }
        report("chase, LDS rows (quad)", 0, 1, cph);
        for (int rep = 0; rep < 3; ++rep) { chase_only<3><<<1, 64>>>(d_ds, d_out + 1024); CK(hipDeviceSynchronize()); }
        report("chase, VGPR rows, old", 0, 1, cph);
        for (int rep = 0; rep < 3; ++rep) { chase_stamped<<<1, 64>>>(d_ds, d_out + 1024); CK(hipDeviceSynchronize()); }
        report("chase, stamped", 0, 1, cph);
        unsigned long long acc[4];
        CK(hipMemcpyFromSymbol(acc, HIP_SYMBOL(g_acc), sizeof(acc)));
        printf("    sweeps %llu: bookkeeping+shift %llu clk (%.0f/sweep), slots %llu clk (%.0f/sweep, %.0f/rotation)\n",
               acc[2], acc[0], (double)acc[0] / acc[2], acc[1], (double)acc[1] / acc[2], (double)acc[1] / 156.0);
    }
    // hypotheses
    std::uniform_int_distribution<int> D(0, n - 1);
    int idx[80];
    for (int k = 0; k < 80; ++k) idx[k] = D(g);
    CK(hipMemcpy(d_idx, idx, sizeof(idx), hipMemcpyHostToDevice));
    ProbeHyp* d_hp;
    CK(hipMalloc(&d_hp, 20 * sizeof(ProbeHyp)));
    setup_hyp<<<1, 64>>>(d_pw, d_u, d_idx, 20, s.fx, s.fy, s.cx, s.cy, d_mtm, d_hp);
    ProbeHyp* d_hp64;
    CK(hipMalloc(&d_hp64, 64 * sizeof(ProbeHyp)));
    double* d_m64;
    CK(hipMalloc(&d_m64, 64 * 160 * 8));
    int* d_idx64;
    {
        int idx64[256];
        for (int k = 0; k < 256; ++k) idx64[k] = D(g);
        CK(hipMalloc(&d_idx64, sizeof(idx64)));
        CK(hipMemcpy(d_idx64, idx64, sizeof(idx64), hipMemcpyHostToDevice));
    }
    setup_hyp<<<1, 64>>>(d_pw, d_u, d_idx64, 64, s.fx, s.fy, s.cx, s.cy, d_m64, d_hp64);
    count_rot<<<1, 64>>>(d_mtm, 20, d_rot);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(rot, d_rot, 20 * 4, hipMemcpyDeviceToHost));
    int mx = 0, sum = 0;
    for (int h = 0; h < 20; ++h) { mx = rot[h] > mx ? rot[h] : mx; sum += rot[h]; }
    printf("20 hypotheses: rotations mean %.1f max %d (hyp 0: %d)\n", sum / 20.0, mx, rot[0]);
    {
        std::vector<double> m(20 * 160), c(20 * 144);
        CK(hipMemcpy(m.data(), d_mtm, 20 * 160 * 8, hipMemcpyDeviceToHost));
        for (int h = 0; h < 20; ++h)
            for (int e = 0; e < 144; ++e) c[h * 144 + e] = m[h * 160 + e];
        CK(hipMemcpy(d_mtm, c.data(), 20 * 144 * 8, hipMemcpyHostToDevice));
    }
    for (int rep = 0; rep < 3; ++rep) { hyp_eig<1><<<1, 64>>>(d_mtm, d_out); CK(hipDeviceSynchronize()); }
    report("hyp pair x1", 0, 5, eigph);
    for (int rep = 0; rep < 3; ++rep) { hyp_eig<20><<<1, 64>>>(d_mtm, d_out); CK(hipDeviceSynchronize()); }
    report("hyp pairs x20", 0, 5, eigph);
    // betas
    const char* bph[] = {"L_6x10 + rho", "find_betas", "gauss_newton", "store setup", "compute_R_and_t"};
    for (int rep = 0; rep < 3; ++rep) { betas_probe<0><<<3, 64>>>(d_hp, 1, d_out); CK(hipDeviceSynchronize()); }
    report("betas apx 1", 0, 5, bph);
    report("betas apx 2", 1, 5, bph);
    report("betas apx 3", 2, 5, bph);
    {
        ProbeHyp* d_rh;
        CK(hipMalloc(&d_rh, sizeof(ProbeHyp)));
        setup_refine_hyp<<<1, 64>>>(d_pw, d_u, d_als, 500, s.fx, s.fy, s.cx, s.cy, d_mtm + 21 * 160, d_rh);
        CK(hipDeviceSynchronize());
        for (int rep = 0; rep < 3; ++rep) { betas_probe<0><<<3, 64>>>(d_rh, 1, d_out + 2048); CK(hipDeviceSynchronize()); }
        report("refine-data betas apx 1", 0, 5, bph);
        report("refine-data betas apx 2", 1, 5, bph);
        report("refine-data betas apx 3", 2, 5, bph);
        for (int rep = 0; rep < 3; ++rep) { betas_probe<1><<<1, 192>>>(d_rh, 1, d_out + 2048); CK(hipDeviceSynchronize()); }
        report("one 3-wave WG, apx 1", 0, 5, bph);
        report("one 3-wave WG, apx 2", 1, 5, bph);
        report("one 3-wave WG, apx 3", 2, 5, bph);
        {
            const char* rph[] = {"find_betas", "gauss_newton"};
            double* slab_g = d_mtm + 21 * 160;
            for (int rep = 0; rep < 3; ++rep) { refine_betas_like<0><<<1, 256>>>(slab_g, d_out + 3000); CK(hipDeviceSynchronize()); }
            report("refine-like lane 0, w0", 0, 2, rph);
            report("refine-like lane 0, w1", 1, 2, rph);
            report("refine-like lane 0, w2", 2, 2, rph);
            for (int rep = 0; rep < 3; ++rep) { refine_betas_like<1><<<1, 256>>>(slab_g, d_out + 3000); CK(hipDeviceSynchronize()); }
            report("refine-like 64 lanes, w0", 0, 2, rph);
            report("refine-like 64 lanes, w1", 1, 2, rph);
            report("refine-like 64 lanes, w2", 2, 2, rph);
            for (int rep = 0; rep < 3; ++rep) { refine_betas_like<2><<<1, 256>>>(slab_g, d_out + 3000); CK(hipDeviceSynchronize()); }
            report("refine-like divergent, w0", 0, 2, rph);
            report("refine-like divergent, w1", 1, 2, rph);
            report("refine-like divergent, w2", 2, 2, rph);
            for (int rep = 0; rep < 3; ++rep) { slab_betas_64<<<3, 64>>>(slab_g, d_out + 3000); CK(hipDeviceSynchronize()); }
            report("slab view, 64-thread WGs, w0", 0, 2, rph);
            report("slab view, 64-thread WGs, w2", 2, 2, rph);
            for (int rep = 0; rep < 3; ++rep) { split_betas_256<<<1, 256>>>(slab_g, d_out + 3000); CK(hipDeviceSynchronize()); }
            report("split view, 256-thread WG, w0", 0, 2, rph);
            report("split view, 256-thread WG, w2", 2, 2, rph);
            double bo[12], bo2[12];
            CK(hipMemcpy(bo, d_out + 3000, sizeof(bo), hipMemcpyDeviceToHost));
            refine_betas_like<0><<<1, 256>>>(slab_g, d_out + 3000);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(bo2, d_out + 3000, sizeof(bo2), hipMemcpyDeviceToHost));
            printf("    divergent-form betas bit-equal to lane-0 form: %s\n", memcmp(bo, bo2, sizeof(bo)) == 0 ? "yes" : "NO");
        }
        // instruction-cache effect: the same launch right after other large kernels (cold) and
        // then again (warm)
        for (int rep = 0; rep < 2; ++rep) {
            hyp_eig<20><<<1, 64>>>(d_mtm, d_out);
            chase_only<3><<<1, 64>>>(d_ds_g, d_out + 1024);
            refine_eig<<<1, 64>>>(d_out + 4096, d_out + 512);
            CK(hipDeviceSynchronize());
            betas_probe<0><<<3, 64>>>(d_rh, 1, d_out + 2048);
            CK(hipDeviceSynchronize());
            report(rep == 0 ? "COLD refine-data apx 3" : "COLD2 refine-data apx 3", 2, 5, bph);
            betas_probe<0><<<3, 64>>>(d_rh, 1, d_out + 2048);
            CK(hipDeviceSynchronize());
            report("WARM refine-data apx 3", 2, 5, bph);
        }
        for (int rep = 0; rep < 2; ++rep) {
            betas_probe<0><<<3, 64>>>(d_rh, 1, d_out + 2048);
            hyp_eig<20><<<1, 64>>>(d_mtm, d_out);
            CK(hipDeviceSynchronize());
            refine_eig<<<1, 64>>>(d_out + 4096, d_out + 512);
            CK(hipDeviceSynchronize());
            report("COLD refine_eig", 0, 5, eigph);
            refine_eig<<<1, 64>>>(d_out + 4096, d_out + 512);
            CK(hipDeviceSynchronize());
            report("WARM refine_eig", 0, 5, eigph);
        }
        for (int H : {4, 16, 64}) {
            for (int rep = 0; rep < 3; ++rep) { betas_probe<2><<<3, 64>>>(d_hp64, H, d_out + 2048); CK(hipDeviceSynchronize()); }
            char nm[64];
            snprintf(nm, sizeof nm, "%d hyps/wave, apx 1", H); report(nm, 0, 5, bph);
            snprintf(nm, sizeof nm, "%d hyps/wave, apx 2", H); report(nm, 1, 5, bph);
            snprintf(nm, sizeof nm, "%d hyps/wave, apx 3", H); report(nm, 2, 5, bph);
        }
    }
    double o[48];
    CK(hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost));
    printf("errors: %.6g %.6g %.6g\n", o[0], o[16], o[32]);
    const char* gph[] = {"1000 make_givens"};
    for (int rep = 0; rep < 3; ++rep) { givens_chain<<<1, 64>>>(d_out, 1000); CK(hipDeviceSynchronize()); }
    report("make_givens chain", 0, 1, gph);
    {
        double* buf;
        unsigned* ctr;
        CK(hipMalloc(&buf, 8192 * 8));
        CK(hipMalloc(&ctr, 64));
        CK(hipMemset(ctr, 0, 64));
        const char* fph[] = {"stores+release", "atomic add", "acquire", "dependent load"};
        for (int rep = 0; rep < 3; ++rep) { fence_probe<<<3, 64>>>(buf, ctr); CK(hipDeviceSynchronize()); }
        report("hand-off wave 0", 0, 4, fph);
        report("hand-off wave 2", 2, 4, fph);
    }
    return 0;
}
