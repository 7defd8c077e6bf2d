// rsc_quad.h — lane-group EPnP hypothesis solve (2 or 4 lanes of a wave per hypothesis).
//
// Why: one lane per hypothesis runs PnPsolver::compute_pose as one long dependent FP64 chain, and a
// relocalization batch (19,200 hypotheses) fills only 300 of the 1,024 SIMDs with one wave each, so
// the solve is latency-bound.  A group of L lanes per hypothesis splits the row work of the chain:
//   * 12x12 Householder tridiagonalisation: member q owns rows L*j+q of the full symmetric matrix in
//     VGPRs; the Householder vector and A*v are exchanged with DPP quad_perm broadcasts;
//   * accumulation of the Householder sequence: member q owns columns L*j+q of Q;
//   * implicit QR: the Givens chase is computed redundantly by the group (bitwise identical), each
//     member applying the rotations to its own rows of Q;
//   * the three beta approximations of PnPsolver.cpp:383-414 (+ Gauss-Newton + compute_R_and_t)
//     run in a second kernel, one single-wave workgroup per (approximation, 64 hypotheses), and
//     the smallest error wins in the reference's order.
// The product runs pairs (L = 2, 20 hypotheses per wave: 960 waves for the 1,024 SIMDs on config
// 2); the Refine kernel's single eigenproblem uses one quad.
// Every scalar is produced by the same operations on the same operands as the sequential
// restatement (rsc_core.h / oracle), so results are bitwise identical; the only reorderings are of
// independent scalars (and of max(), which is order-free for the non-NaN case handled below).
#pragma once
#include "rsc_core.h"
#include "rsc_epnp.h"
#include "rsc_kernels.h"

#ifndef RSC_EIG_PHASE
#define RSC_EIG_PHASE(k) \
    do {                 \
    } while (0)
#endif
#ifndef RSC_SOLVE_STAMP
#define RSC_SOLVE_STAMP(st, k) \
    do {                       \
    } while (0)
#endif

namespace rsc {

constexpr int kQuadT = 144;  // MtM lower triangle, then the Q transpose
constexpr int kQuadE = 55;   // Householder essential vectors
constexpr int kQuadRegion = kQuadT + kQuadE + 1;  // 200 doubles per hypothesis
// stage record offsets (rsc_kernels.h kStageDoubles)
constexpr int kStEv = 0, kStAl = 48, kStCws = 72;
// pnp_betas_wave_body LDS: L + rho [66][kBetasHyps].
constexpr int kBetasWaveSmemDoubles = 66 * kBetasHyps;

// Offset of step i's essential Householder vector (entries v[1..10-i]) in the E region.
RSC_HD constexpr int quad_eoff(int i) { return 10 * i - (i * (i - 1)) / 2; }

// Value of x in member SRC of this lane's group of L lanes (L = 4: the quad; L = 2: the pair,
// lanes {0,1} and {2,3} of each quad) — one DPP quad_perm move per 32-bit half.
template <int L, int SRC>
__device__ __forceinline__ double gb_(double x) {
    static_assert(L == 2 || L == 4, "lane groups of 2 or 4");
    constexpr int ctrl = (L == 4) ? SRC * 0x55 : (SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6));
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// src is a compile-time constant after unrolling.
template <int L>
__device__ __forceinline__ double gb(double x, int src) {
    switch (src % L) {
        case 0: return gb_<L, 0>(x);
        case 1: return gb_<L, 1>(x);
        case 2: return gb_<L, (L == 4 ? 2 : 0)>(x);
        default: return gb_<L, (L == 4 ? 3 : 1)>(x);
    }
}
template <int SRC>
__device__ __forceinline__ double qb_(double x) { return gb_<4, SRC>(x); }

// x[base + q] of a register array (static base), 0 outside [0, n).
template <int L, int n>
__device__ __forceinline__ double seln(const double (&x)[n], int base, int q) {
    double r = 0.0;
    RSC_UNROLL for (int t = 0; t < L; ++t) {
        const int i = base + t;
        if (i >= 0 && i < n && q == t) r = x[i];
    }
    return r;
}

// Tridiagonalisation of the scaled 12x12 (sym_eig12_tridiag, Householder part) by a group of L
// lanes, member q owning rows L*j + q.  A: own rows, full symmetric.  E: this hypothesis'
// essential-vector region (written by member 0).
template <int L>
__device__ __forceinline__ void group_tridiag(double (&A)[12 / L][12], int q, double* E, double (&diag)[12],
                                              double (&sub)[11], double (&hC)[11]) {
    constexpr int n = 12, NN = 11, RJ = 12 / L;
    RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
        const int rs = n - i - 1;
        double v[NN], w2[NN], hcv[NN];
        RSC_UNROLL for (int k = 0; k < NN; ++k) {
            v[k] = 0.0;
            hcv[k] = 0.0;
            if (k < rs) v[k] = gb<L>(A[(i + 1 + k) / L][i], (i + 1 + k) % L);
        }
        double tail = 0.0;
        if (rs > 1) {
            tail = v[1] * v[1];
            RSC_UNROLL for (int k = 2; k < NN; ++k) if (k < rs) tail = tail + v[k] * v[k];
        }
        const double c0 = v[0];
        double h, beta;
        if (tail <= lim<double>::min()) {
            h = 0.0;
            beta = c0;
            RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) v[k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double den = c0 - beta;
            RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) v[k] = v[k] / den;
            h = (beta - c0) / beta;
        }
        v[0] = 1.0;
        if (q == 0) {
            RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) E[quad_eoff(i) + k - 1] = v[k];
        }
        RSC_UNROLL for (int k = 0; k < NN; ++k) w2[k] = h * v[k];
        // own rows of hc = A_sub * (h v)
        double hco[RJ];
        RSC_UNROLL for (int j = 0; j < RJ; ++j) {
            hco[j] = 0.0;
            if (L * j + L - 1 >= i + 1) {
                double acc = A[j][i + 1] * w2[0];
                RSC_UNROLL for (int m = 1; m < NN; ++m) if (m < rs) acc = acc + A[j][i + 1 + m] * w2[m];
                hco[j] = acc;
            }
        }
        RSC_UNROLL for (int k = 0; k < NN; ++k) if (k < rs) hcv[k] = gb<L>(hco[(i + 1 + k) / L], (i + 1 + k) % L);
        double dot = hcv[0] * v[0];
        RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) dot = dot + hcv[k] * v[k];
        const double alpha = (h * -0.5) * dot;
        RSC_UNROLL for (int k = 0; k < NN; ++k) if (k < rs) hcv[k] = hcv[k] + alpha * v[k];
        // rank-2 update of the own rows (both triangles: the mirrored element gets the same bits,
        // the two products are the same and IEEE addition commutes)
        RSC_UNROLL for (int j = 0; j < RJ; ++j) {
            if (L * j + L - 1 >= i + 1) {
                const int kr = L * j + q - (i + 1);
                const double vo = seln<L>(v, L * j - (i + 1), q);
                const double ho = seln<L>(hcv, L * j - (i + 1), q);
                if (kr >= 0) {
                    RSC_UNROLL for (int c = 0; c < NN; ++c)
                        if (c < rs) A[j][i + 1 + c] = A[j][i + 1 + c] + ((-v[c]) * ho + (-hcv[c]) * vo);
                }
            }
        }
        if (q == (i + 1) % L) A[(i + 1) / L][i] = beta;
        hC[i] = h;
    }
    RSC_UNROLL for (int k = 0; k < n; ++k) diag[k] = gb<L>(A[k / L][k], k % L);
    RSC_UNROLL for (int k = 0; k < n - 1; ++k) sub[k] = gb<L>(A[(k + 1) / L][k], (k + 1) % L);
}

// Householder sequence evalTo (sym_eig12_tridiag, accumulation part), own columns L*j + q of Q.
template <int L>
__device__ __forceinline__ void group_accumulate(double (&Qc)[12 / L][12], int q, const double* E,
                                                 const double (&hC)[11]) {
    constexpr int RJ = 12 / L;
    RSC_UNROLL for (int j = 0; j < RJ; ++j)
        RSC_UNROLL for (int r = 0; r < 12; ++r) Qc[j][r] = (r == L * j + q) ? 1.0 : 0.0;
    RSC_UNROLL for (int k = 10; k >= 0; --k) {
        const int cs = 11 - k, b0 = k + 1;
        const double tau = hC[k];
        if (cs == 1) {
            if (q == 11 % L) Qc[11 / L][11] = Qc[11 / L][11] * (1.0 - tau);
        } else if (tau != 0.0) {
            double ev[10];
            RSC_UNROLL for (int r = 0; r < 10; ++r) ev[r] = (r < cs - 1) ? E[quad_eoff(k) + r] : 0.0;
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                if (L * j + L - 1 >= b0 && L * j + q >= b0) {
                    double acc = ev[0] * Qc[j][b0 + 1];
                    RSC_UNROLL for (int r = 1; r < 10; ++r) if (r < cs - 1) acc = acc + ev[r] * Qc[j][b0 + 1 + r];
                    const double tmp = acc + Qc[j][b0];
                    Qc[j][b0] = Qc[j][b0] - tau * tmp;
                    RSC_UNROLL for (int r = 0; r < 10; ++r) {
                        if (r < cs - 1) {
                            const double te = tau * ev[r];
                            Qc[j][b0 + 1 + r] = Qc[j][b0 + 1 + r] - tmp * te;
                        }
                    }
                }
            }
        }
    }
}

// The group's own rows of Q (rows L*j + q of the row-major 12x12 in T) as the QR's rotation sink:
// prefetch(k) loads columns k, k+1 at the top of the chase slot so the LDS round trip overlaps the
// Givens computation; operator() rotates and stores them (tridiag_qr's qapply contract:
// bit-identical values when !apply).
template <int L>
struct GroupLdsRows {
    static constexpr int RJ = 12 / L;
    double* T;
    int q;
    double x[RJ], y[RJ];
    RSC_HD void prefetch(int k) {
        RSC_UNROLL for (int j = 0; j < RJ; ++j) {
            const double* row = T + (L * j + q) * 12;
            x[j] = row[k];
            y[j] = row[k + 1];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the rotation's chain
    }
    // Eigen skips identity rotations (c == 1, s == 0); the chase only produces one when an entry
    // underflows, so the selects that keep the rows bit-identical then run behind a wave-uniform
    // branch instead of on every rotation (4 fewer VALU instructions per row, tools/qr_bench).
    RSC_HD void operator()(int k, double c, double s, bool apply) {
        if (__builtin_expect(__any(!apply), 0)) {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                double* row = T + (L * j + q) * 12;
                row[k] = apply ? c * x[j] - s * y[j] : x[j];
                row[k + 1] = apply ? s * x[j] + c * y[j] : y[j];
            }
        } else {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                double* row = T + (L * j + q) * 12;
                row[k] = c * x[j] - s * y[j];
                row[k + 1] = s * x[j] + c * y[j];
            }
        }
    }
};

// The group's own rows of Q held in VGPRs (Qr[j] = row L*j + q): the same rotation as
// GroupLdsRows without the LDS round trip (the hypothesis eigen stage's sink since round 5;
// tools/qr_bench sink 2).
template <int L>
struct GroupRegRows {
    static constexpr int RJ = 12 / L;
    double (&Q)[RJ][12];
    RSC_HD void operator()(int k, double c, double s, bool apply) {
        if (__builtin_expect(__any(!apply), 0)) {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                const double x = Q[j][k], y = Q[j][k + 1];
                Q[j][k] = apply ? c * x - s * y : x;
                Q[j][k + 1] = apply ? s * x + c * y : y;
            }
        } else {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                const double x = Q[j][k], y = Q[j][k + 1];
                Q[j][k] = c * x - s * y;
                Q[j][k + 1] = s * x + c * y;
            }
        }
    }
};

// Scale of SelfAdjointEigenSolver = max |lower triangle| over the group's own rows (A: full
// symmetric own rows, R = L*j + q); a NaN M(0,0) poisons it, as there.
template <int L>
__device__ __forceinline__ double group_scale(const double (&A)[12 / L][12], int q) {
    double m = 0.0;
    RSC_UNROLL for (int j = 0; j < 12 / L; ++j) {
        const int R = L * j + q;
        RSC_UNROLL for (int c = 0; c < 12; ++c) {
            const double a = fabs(A[j][c]);
            if (c <= R && a > m) m = a;
        }
    }
    double scale = gb_<L, 0>(m);
    const double m1 = gb_<L, 1>(m);
    if (m1 > scale) scale = m1;
    if (L == 4) {
        const double m2 = gb_<L, (L == 4 ? 2 : 0)>(m), m3 = gb_<L, (L == 4 ? 3 : 1)>(m);
        if (m2 > scale) scale = m2;
        if (m3 > scale) scale = m3;
    }
    const double a00 = fabs(gb_<L, 0>(A[0][0]));
    if (a00 != a00) scale = a00;
    if (scale == 0.0) scale = 1.0;
    return scale;
}

// Eigenvectors of the four smallest eigenvalues of a symmetric 12x12 (SelfAdjointEigenSolver on
// MtM, PnPsolver.cpp:379-382) by the L lanes of one lane group (q = lane index in the group, L = 2:
// a pair, L = 4: a quad): phases B-D of pnp_eig_group_body below as a standalone routine (used by
// the Refine kernel, where one group of wave 0 serves the workgroup).  T: the group's 144-double
// LDS region holding the lower triangle row-major (T[R*12+c], c <= R) on entry; E: 55 doubles of
// LDS scratch; sync(): an LDS visibility point for the group.  ev[j][c] = eigenvector column c of
// row L*j+q, bit-identical to sym_eig12 (rsc_core.h) and to the hypothesis path.
template <int L, class Sync>
__device__ __forceinline__ void group_eig12_ev4(double* T, double* E, int q, Sync sync, double (&ev)[12 / L][4]) {
    constexpr int RJ = 12 / L;
    double diag[12], sub[11], hC[11];
    {
        double A[RJ][12];
        RSC_UNROLL for (int j = 0; j < RJ; ++j) {
            const int R = L * j + q;
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = T[(R >= c) ? R * 12 + c : c * 12 + R];
        }
        const double scale = group_scale<L>(A, q);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = A[j][c] / scale;
        sync();  // every lane has read T before phase C overwrites it
        group_tridiag<L>(A, q, E, diag, sub, hC);
    }
    sync();
    RSC_EIG_PHASE(0);
    {
        double Qc[RJ][12];
        group_accumulate<L>(Qc, q, E, hC);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int r = 0; r < 12; ++r) T[r * 12 + L * j + q] = Qc[j][r];
    }
    sync();
    RSC_EIG_PHASE(1);
    GroupLdsRows<L> qapply{T, q};
    int perm[12];
    tridiag_qr<double, 12>(diag, sub, qapply, perm);
    RSC_EIG_PHASE(2);
    RSC_UNROLL for (int j = 0; j < RJ; ++j) {
        const double* row = T + (L * j + q) * 12;
        double Qr[12];
        RSC_UNROLL for (int p = 0; p < 12; ++p) Qr[p] = row[p];
        RSC_UNROLL for (int c = 0; c < 4; ++c) {
            double x = Qr[0];
            RSC_UNROLL for (int p = 1; p < 12; ++p) x = (perm[c] == p) ? Qr[p] : x;
            ev[j][c] = x;
        }
    }
    RSC_EIG_PHASE(3);
}

// Q = Q * G on columns k, k+1 of one row held in VGPRs (tridiag_qr's qapply contract).
struct RegRowQ {
    double (&row)[12];
    RSC_HD void operator()(int k, double c, double s, bool apply) {
        const double x = row[k], y = row[k + 1];
        row[k] = apply ? c * x - s * y : x;
        row[k + 1] = apply ? s * x + c * y : y;
    }
};

// The Refine's 12x12 eigenvectors (one problem per workgroup): phases B-C (scale, Householder
// tridiagonalisation, Q accumulation) on lanes 0..L-1 of the calling wave exactly as
// group_eig12_ev4, then the implicit-QR chase on lanes 0..11, lane r holding row r of Q in VGPRs: the
// chase is computed redundantly (identical values) and each lane rotates its own row — no LDS round
// trip and no Q-row traffic in the rotation chain, which is what bounds one lone problem.  T: the
// 144-double LDS region (MtM lower triangle on entry, Q after phase C); E: LDS scratch of at least
// 90 doubles; sync(): an LDS visibility point of the wave.  Lanes 0..11 return the four eigenvector
// entries of their row, bit-identical to group_eig12_ev4.
template <int L, class Sync>
__device__ __forceinline__ void rows_eig12_ev4(double* T, double* E, int lane, Sync sync, double (&ev)[4]) {
    constexpr int RJ = 12 / L;
    constexpr int kDiag = 64, kSub = 76;  // diag / sub hand-off in E, after the Householder vectors
    if (lane < L) {
        double diag[12], sub[11], hC[11];
        {
            double A[RJ][12];
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                const int R = L * j + lane;
                RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = T[(R >= c) ? R * 12 + c : c * 12 + R];
            }
            const double scale = group_scale<L>(A, lane);
            RSC_UNROLL for (int j = 0; j < RJ; ++j)
                RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = A[j][c] / scale;
            sync();  // every lane has read T before phase C overwrites it
            group_tridiag<L>(A, lane, E, diag, sub, hC);
        }
        sync();
        RSC_EIG_PHASE(0);
        double Qc[RJ][12];
        group_accumulate<L>(Qc, lane, E, hC);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int r = 0; r < 12; ++r) T[r * 12 + L * j + lane] = Qc[j][r];
        if (lane == 0) {
            RSC_UNROLL for (int i = 0; i < 12; ++i) E[kDiag + i] = diag[i];
            RSC_UNROLL for (int i = 0; i < 11; ++i) E[kSub + i] = sub[i];
        }
    }
    sync();
    RSC_EIG_PHASE(1);
    if (lane < 12) {
        double diag[12], sub[11], row[12];
        RSC_UNROLL for (int i = 0; i < 12; ++i) diag[i] = E[kDiag + i];
        RSC_UNROLL for (int i = 0; i < 11; ++i) sub[i] = E[kSub + i];
        RSC_UNROLL for (int c = 0; c < 12; ++c) row[c] = T[lane * 12 + c];
        RegRowQ qapply{row};
        int perm[12];
        tridiag_qr<double, 12>(diag, sub, qapply, perm);
        RSC_EIG_PHASE(2);
        RSC_UNROLL for (int c = 0; c < 4; ++c) {
            double x = row[0];
            RSC_UNROLL for (int p = 1; p < 12; ++p) x = (perm[c] == p) ? row[p] : x;
            ev[c] = x;
        }
    }
    RSC_EIG_PHASE(3);
}

// Kernel 1 of the two-kernel hypothesis solve: sample, control points, alphas, MtM, and the 12x12
// eigenvectors, L lanes per hypothesis (a lane group), HPW hypotheses per 64-lane workgroup
// (HPW * L <= 64; lanes beyond leave at once).  Writes the stage record (eigenvectors, alphas, cws)
// and the sample indices.  STOP < 99 truncates (diagnostics only, tools/quad_bench).
//
// Why pairs (L = 2, the product's choice): the implicit-QR chase is a serial FP64 chain that every
// lane of a group computes redundantly, so the wave's instruction stream costs the same whether it
// serves 16 hypotheses (quads) or 32 (pairs); a group only shares the row work (the rotations on
// Q, the Householder updates).  A config-2 batch (19,200 hypotheses) is 1,200 quad waves for the
// 1,024 SIMDs — the last 176 SIMDs run two waves back to back — but 960 pair waves of 20
// hypotheses (kEigHyps), one per SIMD; 32 per pair wave (600 waves) leaves SIMDs idle at the same
// per-wave latency (tools/qr_bench).
template <int NS, int STOP, int L, int HPW>
__device__ __forceinline__ void pnp_eig_group_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                   const int2* __restrict__ wg_table, const uint32_t* __restrict__ rng_T,
                                                   double* __restrict__ stage, int32_t* __restrict__ samples,
                                                   double* smem) {
    static_assert(HPW * L <= 64 && (L == 2 || L == 4), "lane groups of 2 or 4 within one wave");
    constexpr int RJ = 12 / L;
    const int lane = threadIdx.x, g = lane / L, q = lane % L;
    if (g >= HPW) return;  // whole groups only: the DPP broadcasts never read a departed lane
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const bool active = wt.y + g < lp.H;
    const int h = active ? wt.y + g : lp.H - 1;  // idle groups repeat the last hypothesis (no writes)
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    double* out = stage + rec * kStageDoubles;
    double* T = smem + g * kQuadRegion;
    double* E = T + kQuadT;
    RSC_SOLVE_STAMP(0, 0);

    // ---- A: sample, control points, alphas, MtM (every lane of the group, identical values) ----
    {
        int idx[NS];
        uint32_t w[31];
        RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
        uint32_t words[NS];
        RSC_UNROLL for (int d = 0; d < NS; ++d) words[d] = rng_word(rng_T, w, lp.g0 + h * NS + d);
        swap_remove_sample<NS>(words, NS, P.n, idx);
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
        if (q == 0) {
            build_MtM(st, K, LaneMat{T, 1});
            if (active) {
                RSC_UNROLL for (int i = 0; i < NS; ++i)
                    RSC_UNROLL for (int j = 0; j < 4; ++j) out[kStAl + i * 4 + j] = st.al(i, j);
                RSC_UNROLL for (int i = 0; i < 4; ++i)
                    RSC_UNROLL for (int c = 0; c < 3; ++c) out[kStCws + i * 3 + c] = cws[i][c];
                RSC_UNROLL for (int i = 0; i < NS; ++i) samples[rec * 8 + i] = idx[i];
            }
        }
    }
    __syncthreads();
    RSC_SOLVE_STAMP(0, 1);
    if (STOP == 1) {
        if (active && q == 0) out[0] = T[0] + T[143];
        return;
    }

    // ---- B: scale + tridiagonalise (own rows) ----
    double diag[12], sub[11], hC[11];
    {
        double A[RJ][12];
        RSC_UNROLL for (int j = 0; j < RJ; ++j) {
            const int R = L * j + q;
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = T[(R >= c) ? R * 12 + c : c * 12 + R];
        }
        const double scale = group_scale<L>(A, q);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = A[j][c] / scale;
        group_tridiag<L>(A, q, E, diag, sub, hC);
    }
    __syncthreads();
    RSC_SOLVE_STAMP(0, 2);
    if (STOP == 2) {
        if (active && q == 0) {
            double acc = 0.0;
            RSC_UNROLL for (int k = 0; k < 12; ++k) acc += diag[k];
            RSC_UNROLL for (int k = 0; k < 11; ++k) acc += sub[k] + hC[k];
            out[0] = acc;
        }
        return;
    }

    // ---- C: accumulate Q (own columns), transpose to row-major Q in this hypothesis' T region ----
    {
        double Qc[RJ][12];
        group_accumulate<L>(Qc, q, E, hC);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int r = 0; r < 12; ++r) T[r * 12 + L * j + q] = Qc[j][r];
    }
    __syncthreads();
    RSC_SOLVE_STAMP(0, 3);
    if (STOP == 3) {
        if (active) {
            double acc = 0.0;
            RSC_UNROLL for (int j = 0; j < RJ; ++j)
                RSC_UNROLL for (int c = 0; c < 12; ++c) acc += T[(L * j + q) * 12 + c];
            out[q] = acc + diag[0] + sub[0];
        }
        return;
    }

    // ---- D: implicit symmetric QR, rotations applied to the own rows ----
    // Sweep form with the own rows of Q in VGPRs (round 5: eigen stage 132 -> 119-122 us per config-2
    // launch against the rows in LDS, profiles/r05/regrows_ab_r5c.json; 256 VGPRs + AGPRs, no
    // scratch).  RSC_EIG_LDSROWS builds the LDS-row form for A/B (tools/Makefile ldsrows_lib).  (The
    // event and split-chase forms of the QR, tools/qr_events.h, are bit-identical and measured slower
    // on gfx950)
#ifndef RSC_EIG_LDSROWS
    {
        int perm[12];
        double Qr[RJ][12];
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int c = 0; c < 12; ++c) Qr[j][c] = T[(L * j + q) * 12 + c];
#ifndef RSC_EIG_NULLSINK
        GroupRegRows<L> qapply{Qr};
#else
        // timing diagnostic only (tools/Makefile nullsink_lib): the chase without the Q rotations
        struct {
            RSC_HD void operator()(int, double, double, bool) {}
        } qapply;
#endif
        tridiag_qr<double, 12>(diag, sub, qapply, perm);
        if (active) {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                RSC_UNROLL for (int c = 0; c < 4; ++c) {
                    double x = Qr[j][0];
                    RSC_UNROLL for (int p = 1; p < 12; ++p) x = (perm[c] == p) ? Qr[j][p] : x;
                    out[kStEv + (L * j + q) * 4 + c] = x;
                }
            }
        }
        RSC_SOLVE_STAMP(0, 4);
    }
#else
    {
        int perm[12];
        GroupLdsRows<L> qapply{T, q};
        tridiag_qr<double, 12>(diag, sub, qapply, perm);
        // sorted eigenvector columns 0..3 (the four smallest eigenvalues) of the own rows
        if (active) {
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                const double* row = T + (L * j + q) * 12;
                double Qr[12];
                RSC_UNROLL for (int p = 0; p < 12; ++p) Qr[p] = row[p];
                RSC_UNROLL for (int c = 0; c < 4; ++c) {
                    double x = Qr[0];
                    RSC_UNROLL for (int p = 1; p < 12; ++p) x = (perm[c] == p) ? Qr[p] : x;
                    out[kStEv + (L * j + q) * 4 + c] = x;
                }
            }
        }
    }
#endif
}

// The eigen stage in the Refine's form, for small (latency-bound) launches (A/B variant, selected
// by RSC_EIG_ROWS, rsc_api.cpp): a 12-lane group per hypothesis, 5 groups per wave, 4 waves per
// workgroup of kEigHyps = 20 hypotheses (the pair form's workgroup table).  Phase A as
// pnp_eig_group_body; phases B-D by rows_eig12_ev4 — Householder phases on the group's first L
// lanes, then the chase with lane r holding row r of Q in VGPRs, which runs a rotation slot in the
// Refine's ~685 clocks instead of the pair form's ~1,500.  Bit-identical to the pair
// form (rows_eig12_ev4 is group_eig12_ev4's arithmetic).  Needs kEigHyps * kRowsRegion doubles.
constexpr int kRowsGroups = 5;                    // 12-lane groups per wave
constexpr int kRowsRegion = kQuadT + 90 + 1;      // T, E (rows_eig12_ev4: >= 90 doubles), odd pad
template <int NS, int L, class Sync>
__device__ __forceinline__ void pnp_eig_rows_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                  const int2* __restrict__ wg_table, const uint32_t* __restrict__ rng_T,
                                                  double* __restrict__ stage, int32_t* __restrict__ samples,
                                                  double* smem, Sync sync) {
    static_assert(kEigHyps == 4 * kRowsGroups, "4 waves of 5 twelve-lane groups per workgroup");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane / 12, r = lane - 12 * g;
    if (g >= kRowsGroups) return;  // lanes 60..63: whole groups only
    const int2 wt = wg_table[blockIdx.x];
    const LaunchProb& lp = lps[wt.x];
    const int slot = kRowsGroups * wave + g;
    if (wt.y + kRowsGroups * wave >= lp.H) return;  // a wave without hypotheses (no cross-wave sync below)
    const bool active = wt.y + slot < lp.H;
    const int h = active ? wt.y + slot : lp.H - 1;  // idle groups repeat the last hypothesis (no writes)
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    double* out = stage + rec * kStageDoubles;
    double* T = smem + slot * kRowsRegion;
    double* E = T + kQuadT;
#if RSC_SOLVE_STAMPS
    // per wave (its 5 hypotheses run independently of the other waves): [0][4 * block + wave][k],
    // k = 0 entry, 1-3 phase A done, 4 eigenvectors stored (tools/solve_probe.py event)
    const int stamp_row = 4 * (int)blockIdx.x + wave;
#define RSC_ROWS_STAMP(k0, k1)                                                   \
    do {                                                                         \
        if (lane == 0 && stamp_row < 4096) {                                     \
            const uint64_t t_ = wall_clock64();                                  \
            for (int k_ = (k0); k_ <= (k1); ++k_) g_solve_stamps[0][stamp_row][k_] = t_; \
        }                                                                        \
    } while (0)
#else
#define RSC_ROWS_STAMP(k0, k1) do {} while (0)
#endif
    RSC_ROWS_STAMP(0, 0);

    // ---- A: sample, control points, alphas, MtM (every lane of the group, identical values) ----
    {
        int idx[NS];
        uint32_t w[31];
        RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
        uint32_t words[NS];
        RSC_UNROLL for (int d = 0; d < NS; ++d) words[d] = rng_word(rng_T, w, lp.g0 + h * NS + d);
        swap_remove_sample<NS>(words, NS, P.n, idx);
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
        if (r == 0) {
            build_MtM(st, K, LaneMat{T, 1});
            if (active) {
                RSC_UNROLL for (int i = 0; i < NS; ++i)
                    RSC_UNROLL for (int j = 0; j < 4; ++j) out[kStAl + i * 4 + j] = st.al(i, j);
                RSC_UNROLL for (int i = 0; i < 4; ++i)
                    RSC_UNROLL for (int c = 0; c < 3; ++c) out[kStCws + i * 3 + c] = cws[i][c];
                RSC_UNROLL for (int i = 0; i < NS; ++i) samples[rec * 8 + i] = idx[i];
            }
        }
    }
    sync();
    RSC_ROWS_STAMP(1, 3);
    // ---- B-D: 12x12 eigenvectors, row r of the four smallest eigenvalues' columns in lane r ----
    double ev[4];
    rows_eig12_ev4<L>(T, E, r, sync, ev);
    if (active) RSC_UNROLL for (int c = 0; c < 4; ++c) out[kStEv + r * 4 + c] = ev[c];
    RSC_ROWS_STAMP(4, 4);
#undef RSC_ROWS_STAMP
}

// ---- The eigen stage with the QR chase and the Q rotations on different waves (split form) ----
// A workgroup of 2 * kSplitUnits waves serves kSplitUnits units of kEigHyps = 20 hypotheses (one
// entry of the eigen-stage work table each); unit c owns chase wave c and row wave kSplitUnits + c,
// which the dispatcher places on the same SIMD (waves go round-robin over the CU's four SIMDs):
//   A    chase wave c, lane pairs as pnp_eig_group_body: sample, control points, alphas, MtM into T;
//   B-C  lane quads over the unit's two waves (hypotheses 0-15 in the chase wave, 16-19 in the row
//        wave): scale, Householder tridiagonalisation and Q accumulation exactly as group_eig12_ev4
//        (the Refine's quad form, bit-identical to the pair form), Q row-major into T, (diag, sub)
//        into a slab of their own;
//   D    the chase wave, one lane per hypothesis, runs the implicit-QR chase on (diag, sub) alone:
//        each QR step's rotations — (c, s) per slot and a bit per slot that rotated — go into the
//        hypothesis' E region (two parities; E is free after phase C) and the step number into the
//        unit's `pub` word (tridiag_qr's sweep_end hook); the row wave holds Q in VGPRs, lane 3h + m
//        owning rows m, m+3, m+6, m+9 of hypothesis h, waits for each step on `pub`, applies it,
//        slots in order — GroupRegRows' operations in its order, so the eigenvectors are
//        bit-identical — and acknowledges it in `ack`; before step s + 1 overwrites the parity of
//        step s - 1 the chase wave waits for that acknowledgement.
// The chase wave issues only the scalar chain (no Q rows in its registers), the row updates issue
// from the other wave of the SIMD (<= 256 registers: two waves per SIMD), and the units run
// independently (LDS flags, not workgroup barriers, between a chase wave and its row wave).  A step
// is valid for a hypothesis when its step number matches (a converged hypothesis publishes nothing
// and keeps an older number in its ring slot); the chase wave's last `pub` carries kSplitDone.
// Traffic diagnostics of the split eigen stage (wrong results; tools/Makefile variants, the PMC
// FETCH_SIZE / WRITE_SIZE attribution of DESIGN.md section 9): no stage-record stores, samples from a
// hash instead of the rand() jump table.
#ifndef RSC_DIAG_NO_STAGE
#define RSC_DIAG_NO_STAGE 0
#endif
#ifndef RSC_DIAG_NO_RNG
#define RSC_DIAG_NO_RNG 0
#endif
constexpr int kSplitUnits = 4;     // chase / row wave pairs per workgroup (one per SIMD)
constexpr int kSplitRowLanes = 3;  // row-wave lanes per hypothesis (4 rows of Q each)
constexpr int kRingPar = 24;       // doubles per parity in E: (c, s) of slots 0..10, then the step word
constexpr int kRingPerm = 48;      // E[48..49]: the four sorted column indices (int32)
constexpr int kSplitDsub = 24;     // doubles per hypothesis of the (diag, sub) slab
constexpr int kSplitHyps = kSplitUnits * 20;

// s_sleep argument between polls of a pub / ack flag (0: poll back to back)
#ifndef RSC_SPLIT_SLEEP
#define RSC_SPLIT_SLEEP 1
#endif
constexpr int kSplitDone = 1 << 30;    // `pub` flag: the chase has ended (low bits: its steps)
// polls before a wait gives up (a stall of seconds: never reached by a working hand-off); giving up
// raises the launch's fault word, which the host returns as RSC_ERR_INTERNAL
#ifndef RSC_SPLIT_SPIN_LIMIT
#define RSC_SPLIT_SPIN_LIMIT (1 << 24)
#endif
constexpr int kSplitSpinLimit = RSC_SPLIT_SPIN_LIMIT;

// Wait (wave-uniformly) until pred(value of *flag) holds; returns the value seen.  On give-up the
// fault word (pinned host memory, rsc_context::h_flag) is set.
template <class Pred>
__device__ __forceinline__ int split_wait(int* flag, unsigned* fault, Pred pred) {
    int v = 0;
    const bool ok = poll_until(
        kSplitSpinLimit, [flag]() { return __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); },
        []() {
#if RSC_SPLIT_SLEEP
            __builtin_amdgcn_s_sleep(RSC_SPLIT_SLEEP);
#endif
        },
        pred, v);
    if (!ok) __hip_atomic_store(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return v;
}

struct SplitRing {
    double* E;          // this hypothesis' E region (55 doubles)
    int* pub;           // this unit's published step count
    int* ack;           // this unit's applied step count (row wave)
    unsigned* fault;    // the launch's fault word (split_wait)
    uint32_t mask = 0;  // slots of the step being built that rotated
    uint32_t seq = 0;   // steps published
    RSC_HD void operator()(int k, double c, double s, bool apply) {
        double* r = E + kRingPar * ((seq + 1) & 1) + 2 * k;
        r[0] = c;
        r[1] = s;
        mask |= apply ? (1u << k) : 0u;
    }
    RSC_HD void sweep_end() {
        ++seq;
        *reinterpret_cast<uint64_t*>(E + kRingPar * (seq & 1) + 22) = (uint64_t)seq | ((uint64_t)mask << 32);
        mask = 0;
        // every lane still iterating is at the same step: the ring stores above, then the count
        __hip_atomic_store(pub, (int)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        // step seq + 1 overwrites the parity of step seq - 1: it must have been applied
        const int need = (int)seq - 1;
        split_wait(ack, fault, [need](int v) { return v >= need; });
    }
};

// ---- The Refine's 12x12 eigenvectors in the split form (one problem, two waves) ----
// Phases B-C as rows_eig12_ev4 on lanes 0..L-1 of the chase wave (Q row-major into T, (diag, sub)
// into E[64..87]); after a workgroup barrier, lane 0 of the chase wave runs the implicit-QR chase on
// (diag, sub) alone and publishes every step's rotations through the SplitRing in `ring` (two
// parities, then the sorted column indices at kRingPerm), while lanes 0..11 of the row wave hold the
// rows of Q in VGPRs, apply each published step in slot order (RegRowQ's operations, so the
// eigenvectors are bit-identical) and acknowledge it.  The chase wave issues the scalar chain alone.
template <int L, class Sync>
__device__ __forceinline__ void refine_eig12_bc(double* T, double* E, int lane, Sync sync) {
    constexpr int RJ = 12 / L;
    constexpr int kDiag = 64, kSub = 76;
    if (lane < L) {
        double diag[12], sub[11], hC[11];
        {
            double A[RJ][12];
            RSC_UNROLL for (int j = 0; j < RJ; ++j) {
                const int R = L * j + lane;
                RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = T[(R >= c) ? R * 12 + c : c * 12 + R];
            }
            const double scale = group_scale<L>(A, lane);
            RSC_UNROLL for (int j = 0; j < RJ; ++j)
                RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = A[j][c] / scale;
            sync();
            group_tridiag<L>(A, lane, E, diag, sub, hC);
        }
        sync();
        double Qc[RJ][12];
        group_accumulate<L>(Qc, lane, E, hC);
        RSC_UNROLL for (int j = 0; j < RJ; ++j)
            RSC_UNROLL for (int r = 0; r < 12; ++r) T[r * 12 + L * j + lane] = Qc[j][r];
        if (lane == 0) {
            RSC_UNROLL for (int i = 0; i < 12; ++i) E[kDiag + i] = diag[i];
            RSC_UNROLL for (int i = 0; i < 11; ++i) E[kSub + i] = sub[i];
        }
    }
}

// Chase wave, lane 0 (after refine_eig12_bc and a workgroup barrier; pub / ack zeroed before it).
__device__ __forceinline__ void refine_eig12_chase(const double* E, double* ring, int* pub, int* ack, unsigned* fault) {
    constexpr int kDiag = 64, kSub = 76;
    *reinterpret_cast<uint64_t*>(ring + 22) = 0;
    *reinterpret_cast<uint64_t*>(ring + kRingPar + 22) = 0;
    double diag[12], sub[11];
    RSC_UNROLL for (int i = 0; i < 12; ++i) diag[i] = E[kDiag + i];
    RSC_UNROLL for (int i = 0; i < 11; ++i) sub[i] = E[kSub + i];
    int perm[12];
    SplitRing rg{ring, pub, ack, fault};
    tridiag_qr<double, 12>(diag, sub, rg, perm);
    int32_t* pm = reinterpret_cast<int32_t*>(ring + kRingPerm);
    RSC_UNROLL for (int c = 0; c < 4; ++c) pm[c] = perm[c];
    const int steps = __hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(pub, steps | kSplitDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Row wave, lanes 0..11: row `lane` of Q from T, the published steps applied in order; returns the
// row's entries of the four sorted eigenvector columns.
__device__ __forceinline__ void refine_eig12_rows(const double* T, const double* ring, int* pub, int* ack,
                                                  unsigned* fault, int lane, double (&ev)[4]) {
    double row[12];
    RSC_UNROLL for (int c = 0; c < 12; ++c) row[c] = T[lane * 12 + c];
    for (int s = 1;; ++s) {
        const int v = split_wait(pub, fault, [s](int x) { return (x & (kSplitDone - 1)) >= s || (x & kSplitDone); });
        if ((v & (kSplitDone - 1)) < s) break;
        const double* r = ring + kRingPar * (s & 1);
        const uint64_t word = *reinterpret_cast<const uint64_t*>(r + 22);
        const uint32_t bits = ((uint32_t)word == (uint32_t)s) ? (uint32_t)(word >> 32) : 0u;
        RSC_UNROLL for (int k = 0; k < 11; ++k) {
            if ((bits >> k) & 1u) {
                const double c = r[2 * k], sn = r[2 * k + 1];
                const double x = row[k], y = row[k + 1];
                row[k] = c * x - sn * y;
                row[k + 1] = sn * x + c * y;
            }
        }
        __hip_atomic_store(ack, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const int32_t* pm = reinterpret_cast<const int32_t*>(ring + kRingPerm);
    RSC_UNROLL for (int c = 0; c < 4; ++c) {
        const int pc = pm[c];
        double x = row[0];
        RSC_UNROLL for (int p = 1; p < 12; ++p) x = (pc == p) ? row[p] : x;
        ev[c] = x;
    }
}

template <int NS>
__device__ __forceinline__ void pnp_eig_split_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                   const int2* __restrict__ wg_table, int nwg_table,
                                                   const uint32_t* __restrict__ rng_T, double* __restrict__ stage,
                                                   int32_t* __restrict__ samples, double* smem, double* dsub,
                                                   int* pub, int* ack, unsigned* fault) {
    constexpr int HPW = kEigHyps, U = kSplitUnits;
    static_assert(HPW == 20 && 2 * HPW <= 64 && 4 * HPW <= 128 && HPW * kSplitRowLanes <= 64, "unit layout");
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int unit = wave % U;
    const bool row_wave = wave >= U;
    const int entry = blockIdx.x * U + unit;
    const bool unit_ok = entry < nwg_table;  // the last workgroup may hold fewer units
    const int2 wt = wg_table[unit_ok ? entry : 0];
    const LaunchProb& lp = lps[wt.x];
    const DevPnP& P = probs[lp.prob];
    double* Tu = smem + unit * HPW * kQuadRegion;  // the unit's 20 regions
    double* Du = dsub + unit * HPW * kSplitDsub;
#if RSC_SOLVE_STAMPS
#define RSC_SPLIT_STAMP(k) \
    do { if (tid == 0 && blockIdx.x < 4096) g_solve_stamps[0][blockIdx.x][k] = wall_clock64(); } while (0)
#else
#define RSC_SPLIT_STAMP(k) do {} while (0)
#endif
    RSC_SPLIT_STAMP(0);
    if (tid < U) {
        pub[tid] = 0;
        ack[tid] = 0;
    }
    // ---- A: chase waves, lane pairs ----
    if (!row_wave && unit_ok && lane < 2 * HPW) {
        const int g = lane >> 1, q = lane & 1;
        const bool active = wt.y + g < lp.H;
        const int h = active ? wt.y + g : lp.H - 1;
        const size_t rec = (size_t)(lp.out0 + h);
        double* out = stage + rec * kStageDoubles;
        double* T = Tu + g * kQuadRegion;
        int idx[NS];
        uint32_t w[31];
        RSC_UNROLL for (int j = 0; j < 31; ++j) w[j] = lp.window[j];
        uint32_t words[NS];
        RSC_UNROLL for (int d = 0; d < NS; ++d) words[d] = RSC_DIAG_NO_RNG ? (uint32_t)(2654435761u * (uint32_t)(h * NS + d + 1)) : rng_word(rng_T, w, lp.g0 + h * NS + d);
        swap_remove_sample<NS>(words, NS, P.n, idx);
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
        if (q == 0) {
            build_MtM(st, K, LaneMat{T, 1});
            if (active && !RSC_DIAG_NO_STAGE) {
                RSC_UNROLL for (int i = 0; i < NS; ++i)
                    RSC_UNROLL for (int j = 0; j < 4; ++j) out[kStAl + i * 4 + j] = st.al(i, j);
                RSC_UNROLL for (int i = 0; i < 4; ++i)
                    RSC_UNROLL for (int c = 0; c < 3; ++c) out[kStCws + i * 3 + c] = cws[i][c];
                RSC_UNROLL for (int i = 0; i < NS; ++i) samples[rec * 8 + i] = idx[i];
            }
        }
    }
    __syncthreads();  // A: MtM (lower triangle) in T
    RSC_SPLIT_STAMP(1);
    // ---- B-C: scale, Householder tridiagonalisation, Q accumulation ----
    // RSC_SPLIT_BC_LANES 4: lane quads over the unit's two waves (hypotheses 0-15 in the chase wave,
    // 16-19 in the row wave); 2: lane pairs in the chase wave alone (lanes 0-39; the row wave only
    // passes the barriers, so the chase wave has the SIMD's issue to itself).  Same values either way
    // (group_eig12_ev4's forms are bit-identical).
#ifndef RSC_SPLIT_BC_LANES
#define RSC_SPLIT_BC_LANES 4
#endif
    constexpr int LB = RSC_SPLIT_BC_LANES, RB = 12 / LB;
    static_assert(LB == 2 || LB == 4, "B-C in lane pairs or quads");
    const int gB = (LB == 4) ? (row_wave ? 16 : 0) + (lane >> 2) : (row_wave ? HPW : lane >> 1);
    const int qB = lane & (LB - 1);
    const bool grp = unit_ok && gB < HPW;
    double* TB = Tu + (grp ? gB : 0) * kQuadRegion;
    double* EB = TB + kQuadT;
    double hC[11];
    if (grp) {
        double diag[12], sub[11];
        double A[RB][12];
        RSC_UNROLL for (int j = 0; j < RB; ++j) {
            const int R = LB * j + qB;
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = TB[(R >= c) ? R * 12 + c : c * 12 + R];
        }
        const double scale = group_scale<LB>(A, qB);
        RSC_UNROLL for (int j = 0; j < RB; ++j)
            RSC_UNROLL for (int c = 0; c < 12; ++c) A[j][c] = A[j][c] / scale;
        __builtin_amdgcn_wave_barrier();
        group_tridiag<LB>(A, qB, EB, diag, sub, hC);
        if (qB == 0) {
            double* ds = Du + gB * kSplitDsub;
            RSC_UNROLL for (int i = 0; i < 12; ++i) ds[i] = diag[i];
            RSC_UNROLL for (int i = 0; i < 11; ++i) ds[12 + i] = sub[i];
        }
    }
    __syncthreads();  // B: every lane of a group has read T; E holds the Householder vectors
    RSC_SPLIT_STAMP(2);
    if (grp) {
        double Qc[RB][12];
        group_accumulate<LB>(Qc, qB, EB, hC);
        RSC_UNROLL for (int j = 0; j < RB; ++j)
            RSC_UNROLL for (int r = 0; r < 12; ++r) TB[r * 12 + LB * j + qB] = Qc[j][r];
    }
    __syncthreads();  // C: Q row-major in T, (diag, sub) in the slab; E is read by no one any more
    RSC_SPLIT_STAMP(3);
    // (no workgroup barrier below: a unit's two waves synchronise through pub / ack)
    if (row_wave) {
        // ---- D, row wave: Q rows ----
        const int g = lane / kSplitRowLanes, m = lane - kSplitRowLanes * g;
        const bool lane_ok = unit_ok && g < HPW;
        const bool active = lane_ok && wt.y + g < lp.H;
        const int h = active ? wt.y + g : lp.H - 1;
        const double* T = Tu + (lane_ok ? g : 0) * kQuadRegion;
        const double* E = T + kQuadT;
        double Q[4][12];
        RSC_UNROLL for (int j = 0; j < 4; ++j)
            RSC_UNROLL for (int c = 0; c < 12; ++c) Q[j][c] = T[(kSplitRowLanes * j + m) * 12 + c];
        for (int s = 1;; ++s) {
            // step s published, or the chase ended before it
            const int v = split_wait(pub + unit, fault, [s](int x) { return (x & (kSplitDone - 1)) >= s || (x & kSplitDone); });
            if ((v & (kSplitDone - 1)) < s) break;
            const double* ring = E + kRingPar * (s & 1);
            const uint64_t word = *reinterpret_cast<const uint64_t*>(ring + 22);
            const uint32_t bits = (lane_ok && (uint32_t)word == (uint32_t)s) ? (uint32_t)(word >> 32) : 0u;
            RSC_UNROLL for (int k = 0; k < 11; ++k) {
                if ((bits >> k) & 1u) {
                    const double c = ring[2 * k], sn = ring[2 * k + 1];
                    RSC_UNROLL for (int j = 0; j < 4; ++j) {
                        const double x = Q[j][k], y = Q[j][k + 1];
                        Q[j][k] = c * x - sn * y;
                        Q[j][k + 1] = sn * x + c * y;
                    }
                }
            }
            __hip_atomic_store(ack + unit, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (active && !RSC_DIAG_NO_STAGE) {
            const int32_t* pm = reinterpret_cast<const int32_t*>(E + kRingPerm);
            int perm4[4];
            RSC_UNROLL for (int c = 0; c < 4; ++c) perm4[c] = pm[c];
            double* out = stage + (size_t)(lp.out0 + h) * kStageDoubles;
            RSC_UNROLL for (int j = 0; j < 4; ++j) {
                RSC_UNROLL for (int c = 0; c < 4; ++c) {
                    double x = Q[j][0];
                    RSC_UNROLL for (int p = 1; p < 12; ++p) x = (perm4[c] == p) ? Q[j][p] : x;
                    out[kStEv + (kSplitRowLanes * j + m) * 4 + c] = x;
                }
            }
        }
        return;
    }
    // ---- D, chase wave: one lane per hypothesis ----
    // the chain's instructions win the SIMD's issue arbitration against the row wave's
#ifndef RSC_SPLIT_PRIO
#define RSC_SPLIT_PRIO 3
#endif
    __builtin_amdgcn_s_setprio(RSC_SPLIT_PRIO);
    if (unit_ok && lane < HPW) {
        double* E = Tu + lane * kQuadRegion + kQuadT;
        // the ring's step words start below step 1 (E held the Householder vectors)
        *reinterpret_cast<uint64_t*>(E + 22) = 0;
        *reinterpret_cast<uint64_t*>(E + kRingPar + 22) = 0;
        double diag[12], sub[11];
        const double* ds = Du + lane * kSplitDsub;
        RSC_UNROLL for (int i = 0; i < 12; ++i) diag[i] = ds[i];
        RSC_UNROLL for (int i = 0; i < 11; ++i) sub[i] = ds[12 + i];
        int perm[12];
        SplitRing ring{E, pub + unit, ack + unit, fault};
        tridiag_qr<double, 12>(diag, sub, ring, perm);
        int32_t* pm = reinterpret_cast<int32_t*>(E + kRingPerm);
        RSC_UNROLL for (int c = 0; c < 4; ++c) pm[c] = perm[c];
    }
    RSC_SPLIT_STAMP(6);
    // the chase has ended (the permutation above, then the flag; a unit without hypotheses publishes
    // zero steps)
    if (lane == 0) {
        const int steps = __hip_atomic_load(pub + unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(pub + unit, steps | kSplitDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    RSC_SPLIT_STAMP(4);
#undef RSC_SPLIT_STAMP
}

// Eigenvectors read from the stage record in global memory (stride 1), L + rho in LDS
// (element-major across the wave).
struct StageEvView {
    const double* evp;
    double* Lp;
    RSC_HD double ev(int r, int c) const { return evp[r * 4 + c]; }
    RSC_HD double& L(int i, int j) const { return Lp[(i * 10 + j) * kBetasHyps]; }
    RSC_HD double& rho(int i) const { return Lp[(60 + i) * kBetasHyps]; }
};

// Block -> (64-hypothesis group, approximation) of pnp_betas_kernel: the three waves of a group are
// blocks b, b+8, b+16 of a run of 24 (one L2: blocks b and b+8 share an XCD), so the group keeps
// the XCD its wg_table slot was ordered for; the last (ngroups % 8) groups are dealt plainly.
RSC_HD void betas_block(int b, int ngroups, int& g, int& apx) {
    const int q = ngroups / 8;
    if (b < 24 * q) {
        g = (b % 8) + 8 * (b / 24);
        apx = (b / 8) % 3;
    } else {
        const int r = ngroups - 8 * q, rem = b - 24 * q;
        g = 8 * q + rem % r;
        apx = rem / r;
    }
}

// Kernel 2 (product form): ONE wave per (64 hypotheses, beta approximation), so config 2's 960
// waves sit one per SIMD instead of 320 three-wave workgroups doubling up on 64 of the 256 CUs.
// Wave apx runs compute_L_6x10 + find_betas_approx_{apx+1} + gauss_newton + compute_R_and_t
// (PnPsolver.cpp:383-408) and leaves (error, float pose) in `berr` / `bpose`; the group's last wave
// to finish (agent-scope counter) keeps the smallest error in the reference's order (:393-414) and
// writes the pose.  Hand-off: producer stores -> vmcnt(0) -> agent release -> vmcnt(0) -> relaxed
// agent add; the last adder: agent acquire -> vmcnt(0) -> loads (MI355X_MICROARCH.md, inter-
// workgroup visibility).  It resets the counter, so every launch starts from zero.
// hb: hypotheses per wave (64 for large rounds; fewer for small ones, so a wave carries the union
// of fewer data-dependent chains): lanes >= hb mirror lane % hb (same control flow, no writes).
template <int NS>
__device__ __forceinline__ void pnp_betas_wave_body(const DevPnP* __restrict__ probs, const LaunchProb* __restrict__ lps,
                                                    const int2* __restrict__ wg_table, int ngroups, int hb,
                                                    const double* __restrict__ stage,
                                                    const int32_t* __restrict__ samples, float* __restrict__ poses,
                                                    double* __restrict__ berr, float* __restrict__ bpose,
                                                    unsigned* __restrict__ bctr, size_t hcap, double* smem) {
    const int lane = threadIdx.x;
    int g, apx;
    betas_block(blockIdx.x, ngroups, g, apx);
    const int2 wt = wg_table[g];
    const LaunchProb& lp = lps[wt.x];
    const bool active = lane < hb && wt.y + lane < lp.H;
    const int hm = wt.y + lane % hb;
    const int h = active ? wt.y + lane : (hm < lp.H ? hm : wt.y);
    const DevPnP& P = probs[lp.prob];
    const size_t rec = (size_t)(lp.out0 + h);
    const double* in = stage + rec * kStageDoubles;
    // lanes >= kBetasHyps (a build with fewer hypotheses per wave) mirror lane % kBetasHyps and
    // write the same values into the same LDS column
    const StageEvView V{in + kStEv, smem + lane % kBetasHyps};
    RSC_SOLVE_STAMP(1, 0);
    compute_L_6x10(V);
    {
        double cws[4][3];
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) cws[i][c] = in[kStCws + i * 3 + c];
        auto d2 = [&](int a, int b) {
            double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
            return ered3(x * x, y * y, z * z);  // squaredNorm of a row of cws (:640-645)
        };
        V.rho(0) = d2(0, 1); V.rho(1) = d2(0, 2); V.rho(2) = d2(0, 3);
        V.rho(3) = d2(1, 2); V.rho(4) = d2(1, 3); V.rho(5) = d2(2, 3);
    }
    double betas[4] = {0.0, 0.0, 0.0, 0.0};
    RSC_SOLVE_STAMP(1, 1);
    if (apx == 0) find_betas<1>(V, betas);
    else if (apx == 1) find_betas<2>(V, betas);
    else find_betas<3>(V, betas);
    RSC_SOLVE_STAMP(1, 2);
    gauss_newton(V, betas);
    RSC_SOLVE_STAMP(1, 3);
    // the hypothesis' points and alphas are read only now (live across the solves above they pushed
    // the wave past 256 VGPRs: scratch spills, round 1)
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
    RSC_SOLVE_STAMP(1, 4);
    const double err = compute_R_and_t(st, K, V, betas, pw0, R, t);
    RSC_SOLVE_STAMP(1, 5);
    float pz[12];
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) pz[3 * r + c] = (float)R[r][c];
    RSC_UNROLL for (int r = 0; r < 3; ++r) pz[9 + r] = (float)t[r];
    if (active) {
        berr[apx * hcap + rec] = err;
        RSC_UNROLL for (int k = 0; k < 12; ++k) bpose[(apx * 12 + k) * hcap + rec] = pz[k];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(bctr + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __builtin_amdgcn_readlane(prev, 0);
    RSC_SOLVE_STAMP(1, 6);
#if RSC_SOLVE_STAMPS
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_solve_stamps[1][blockIdx.x][7] = (uint64_t)apx | ((uint64_t)g << 8);
#endif
    if (prev != 2) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(bctr + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!active) return;
    double e[3];
    RSC_UNROLL for (int a = 0; a < 3; ++a) e[a] = (a == apx) ? err : berr[a * hcap + rec];
    int best = 0;
    double be = e[0];
    if (e[1] < be) { be = e[1]; best = 1; }
    if (e[2] < be) { be = e[2]; best = 2; }
    float* o = poses + rec * 12;
    if (best == apx) {
        RSC_UNROLL for (int k = 0; k < 12; ++k) o[k] = pz[k];
    } else {
        RSC_UNROLL for (int k = 0; k < 12; ++k) o[k] = bpose[(best * 12 + k) * hcap + rec];
    }
}

}  // namespace rsc
