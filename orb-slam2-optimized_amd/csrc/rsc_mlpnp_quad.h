// rsc_mlpnp_quad.h — MLPnP hypothesis solve with four lanes (a quad) per hypothesis.
//
// Why: the lane-per-hypothesis form kept the 12x12 JacobiSVD work matrices (W, V) in a 288-double
// LDS slab per lane — 147 KB per 64-lane workgroup, so one wave per CU: a config-4 round of 9,600
// hypotheses ran on 150 of the 1,024 SIMDs, each wave bound by its lanes' LDS round trips inside
// the sweeps, and the rest of the kernel spilled 167 VGPRs.  Here the quad holds W and V in VGPRs,
// lane q owning columns 4j + q (Wc[j][r] = W(r, 4j + q)): the left rotation of a Jacobi step (rows
// p, s) is lane-local, the right one (columns p, s of W and V) swaps one column between two lanes
// with a DPP quad_perm; the 2x2 SVD is computed redundantly by the four lanes.  16 hypotheses per
// wave: 600 waves for a 32-candidate config-4 round, 2,400 for the 128-candidate one.
// Phases 1 and 3 of computePose (mlpnp_prepare / mlpnp_finish_pose, rsc_mlpnp.h) run redundantly in
// the quad, with their state parked in LDS across the SVD (so it does not hold VGPRs there).
// Every scalar is produced by the same operations on the same operands as the sequential form
// (ml_jacobi_svd_lds): bit-identical results.
#pragma once
#include "rsc_kernels.h"
#include "rsc_mlpnp.h"
#include "rsc_quad.h"

namespace rsc {

// Per-hypothesis LDS region: a slab shared by the phase-1 design matrix A (2 NS x 12) and the
// Gauss-Newton system (ml_gn_slab), then the parked phase-1 state of the variant; rounded up to an
// odd number of doubles so the quads of a wave start on different LDS banks.  The common variant
// (NS = 6, no covariances) takes 239 doubles, 30 KB per 16-hypothesis workgroup: LDS no longer caps
// the CU at three workgroups (it did at 361 doubles), one wave per SIMD is the VGPR bound.
template <int NS>
constexpr int ml_quad_slab() {
    return (24 * NS > ml_gn_slab<NS>()) ? 24 * NS : ml_gn_slab<NS>();
}
template <int NS, class Cov>
constexpr int ml_quad_parked() {
    return 3 * NS + 3 * NS + 6 * NS + (Cov::on ? 4 * NS : 0) + 9 + 1;
}
template <int NS, class Cov>
constexpr int ml_quad_region() {
    return (ml_quad_slab<NS>() + ml_quad_parked<NS, Cov>()) | 1;
}

// DPP quad_perm control that swaps lanes a and b of every quad (others read themselves).
__host__ __device__ constexpr int quad_swap_ctrl(int a, int b) {
    int ctrl = 0;
    for (int k = 0; k < 4; ++k) {
        const int src = (k == a) ? b : ((k == b) ? a : k);
        ctrl |= src << (2 * k);
    }
    return ctrl;
}
template <int CTRL>
__device__ __forceinline__ double quad_perm_d(double x) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// W(r, c) of a quad-distributed matrix in every lane of the quad (r, c static after unrolling).
template <int r, int c>
__device__ __forceinline__ double qm_get(const double (&M)[3][12]) {
    return gb_<4, c % 4>(M[c / 4][r]);
}

// Jacobi rotation of columns P, S (P > S) of a quad-distributed matrix:
// M(r, P) = cr * M(r, P) - sr * M(r, S), M(r, S) = sr * M(r, P) + cr * M(r, S), rows r < n.
// The owner of column P (lane P % 4) receives column S by a DPP swap and vice versa; each lane
// evaluates its own column's expression (cr*mine + (-sr)*other == cr*x - sr*y and
// cr*mine + sr*other == sr*x + cr*y bit for bit: negation is exact, IEEE addition commutes).
template <int n, int P, int S>
__device__ __forceinline__ void qm_rotate_cols(double (&M)[3][12], int q, double cr, double sr) {
    constexpr int lp = P % 4, ls = S % 4, jp = P / 4, js = S / 4;
    const bool ownp = (q == lp), owns = (q == ls);
    const double b = ownp ? -sr : sr;
    RSC_UNROLL for (int r = 0; r < n; ++r) {
        double mine, other;
        if constexpr (lp == ls) {
            // both columns in one lane
            mine = M[jp][r];
            other = M[js][r];
            const double np = cr * mine + (-sr) * other;
            const double ns = cr * other + sr * mine;
            M[jp][r] = ownp ? np : M[jp][r];
            M[js][r] = owns ? ns : M[js][r];
        } else {
            mine = ownp ? M[jp][r] : M[js][r];
            other = quad_perm_d<quad_swap_ctrl(lp, ls)>(mine);
            const double nv = cr * mine + b * other;
            M[jp][r] = ownp ? nv : M[jp][r];
            M[js][r] = owns ? nv : M[js][r];
        }
    }
}

// One (P, S) step of a JacobiSVD sweep (ml_jacobi_svd_lds's inner body) on the quad.
template <int n, int P, int S>
__device__ __forceinline__ void ml_quad_jacobi_step(double (&Wc)[3][12], double (&Vc)[3][12], int q, double& maxDiag,
                                                    bool& finished) {
    const double precision = 2.0 * lim<double>::eps();
    const double considerAsZero = lim<double>::min();
    const double pt = precision * maxDiag;
    const double threshold = (considerAsZero < pt) ? pt : considerAsZero;
    const double wps = qm_get<P, S>(Wc), wsp = qm_get<S, P>(Wc);
    if (rabs(wps) > threshold || rabs(wsp) > threshold) {
        finished = false;
        double cl, sl, cr, sr;
        ml_jacobi_2x2(qm_get<P, P>(Wc), wps, wsp, qm_get<S, S>(Wc), cl, sl, cr, sr);
        const bool lrot = !((int)(cl == 1.0) & (int)(sl == 0.0));  // a select: 6 products per lane
        RSC_UNROLL for (int j = 0; j < 3; ++j) {  // rows P, S over the own columns
            const double xi = Wc[j][P], yi = Wc[j][S];
            Wc[j][P] = lrot ? cl * xi + sl * yi : xi;
            Wc[j][S] = lrot ? -sl * xi + cl * yi : yi;
        }
        if (!(cr == 1.0 && sr == 0.0)) {
            qm_rotate_cols<n, P, S>(Wc, q, cr, sr);
            qm_rotate_cols<n, P, S>(Vc, q, cr, sr);
        }
        const double a = rabs(qm_get<P, P>(Wc)), b = rabs(qm_get<S, S>(Wc));
        const double mm = (a < b) ? b : a;
        maxDiag = (maxDiag < mm) ? mm : maxDiag;
    }
}

template <int n, int P, int S>
__device__ __forceinline__ void ml_quad_sweep(double (&Wc)[3][12], double (&Vc)[3][12], int q, double& maxDiag,
                                              bool& finished) {
    if constexpr (P < n) {
        ml_quad_jacobi_step<n, P, S>(Wc, Vc, q, maxDiag, finished);
        if constexpr (S + 1 < P) ml_quad_sweep<n, P, S + 1>(Wc, Vc, q, maxDiag, finished);
        else ml_quad_sweep<n, P + 1, 0>(Wc, Vc, q, maxDiag, finished);
    }
}

// JacobiSVD<MatrixXd>(W, ComputeFullV) of the n x n (n = 9 or 12) quad-distributed matrix; r1 = the
// V column of the smallest singular value after Eigen's descending sort (every lane of the quad).
template <int n>
__device__ __forceinline__ void ml_quad_jacobi_svd(double (&Wc)[3][12], double (&Vc)[3][12], int q, double (&r1)[12]) {
    // scale = |W(0,0)| then every other entry in turn (`>`): the maximum, except that a NaN W(0,0)
    // poisons it and other NaN entries are skipped, as in the sequential loop
    double m = 0.0;
    RSC_UNROLL for (int j = 0; j < 3; ++j)
        RSC_UNROLL for (int r = 0; r < n; ++r) {
            const int c = 4 * j + q;
            const double a = rabs(Wc[j][r]);
            if (c < n && !(r == 0 && c == 0) && a > m) m = a;
        }
    double mq = m;
    {
        const double m1 = gb_<4, 1>(m), m2 = gb_<4, 2>(m), m3 = gb_<4, 3>(m), m0 = gb_<4, 0>(m);
        mq = m0;
        if (m1 > mq) mq = m1;
        if (m2 > mq) mq = m2;
        if (m3 > mq) mq = m3;
    }
    double scale = rabs(qm_get<0, 0>(Wc));
    if (mq > scale) scale = mq;
    if (scale == 0.0) scale = 1.0;
    RSC_UNROLL for (int j = 0; j < 3; ++j)
        RSC_UNROLL for (int r = 0; r < 12; ++r) {
            Wc[j][r] = (r < n) ? Wc[j][r] / scale : 0.0;
            Vc[j][r] = (r == 4 * j + q) ? 1.0 : 0.0;
        }
    double maxDiag = rabs(qm_get<0, 0>(Wc));
    RSC_UNROLL for (int i = 1; i < n; ++i) {
        double d = 0.0;
        if (i % 4 == 0) d = gb_<4, 0>(Wc[i / 4][i]);
        else if (i % 4 == 1) d = gb_<4, 1>(Wc[i / 4][i]);
        else if (i % 4 == 2) d = gb_<4, 2>(Wc[i / 4][i]);
        else d = gb_<4, 3>(Wc[i / 4][i]);
        if (rabs(d) > maxDiag) maxDiag = rabs(d);
    }
    bool finished = false;
    while (!finished) {
        finished = true;
        ml_quad_sweep<n, 1, 0>(Wc, Vc, q, maxDiag, finished);
        RSC_LOOP_FENCE();
    }
    // singular values, descending selection sort (first maximum), stop at a zero maximum
    double sv[12];
    int perm[12];
    RSC_UNROLL for (int i = 0; i < 12; ++i) {
        double d = 0.0;
        if (i % 4 == 0) d = gb_<4, 0>(Wc[i / 4][i]);
        else if (i % 4 == 1) d = gb_<4, 1>(Wc[i / 4][i]);
        else if (i % 4 == 2) d = gb_<4, 2>(Wc[i / 4][i]);
        else d = gb_<4, 3>(Wc[i / 4][i]);
        sv[i] = (i < n) ? rabs(d) * scale : 0.0;
        perm[i] = i;
    }
    bool stopped = false;
    RSC_UNROLL for (int i = 0; i < 12; ++i) {
        if (i < n && !stopped) {
            int pos = 0;
            double mv = sv[i];
            RSC_UNROLL for (int j = 1; j < 12; ++j) {
                const bool gt = (i + j < n) && sv[(i + j) < 12 ? i + j : 11] > mv;
                mv = gt ? sv[(i + j) < 12 ? i + j : 11] : mv;
                pos = gt ? j : pos;
            }
            if (mv == 0.0) {
                stopped = true;
            } else {
                RSC_UNROLL for (int j = 1; j < 12; ++j) {
                    if (i + j < 12) {
                        const bool sw = (j == pos);
                        const double a = sv[i], b = sv[i + j];
                        sv[i] = sw ? b : a;
                        sv[i + j] = sw ? a : b;
                        const int pa = perm[i], pb = perm[i + j];
                        perm[i] = sw ? pb : pa;
                        perm[i + j] = sw ? pa : pb;
                    }
                }
            }
        }
    }
    int last = perm[11];
    RSC_UNROLL for (int i = 0; i < 12; ++i) last = (i == n - 1) ? perm[i] : last;
    // V column `last`: slot last / 4 of lane last % 4
    const int lj = last >> 2, ll = last & 3;
    RSC_UNROLL for (int r = 0; r < 12; ++r) {
        const double v = (lj == 0) ? Vc[0][r] : ((lj == 1) ? Vc[1][r] : Vc[2][r]);
        const double b0 = gb_<4, 0>(v), b1 = gb_<4, 1>(v), b2 = gb_<4, 2>(v), b3 = gb_<4, 3>(v);
        r1[r] = (ll == 0) ? b0 : ((ll == 1) ? b1 : ((ll == 2) ? b2 : b3));
    }
}

// Park the phase-1 state (and the hypothesis' points and bearings) in the hypothesis' LDS
// region while the SVD holds W and V in VGPRs.  All four lanes write the same values.
template <int NS, class Cov>
__device__ __forceinline__ void ml_park(double* st, const double (&pw)[NS][3], const double (&f)[NS][3],
                                        const MlPrep<NS, Cov>& m) {
    int k = 0;
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int c = 0; c < 3; ++c) st[k++] = pw[i][c];
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int c = 0; c < 3; ++c) st[k++] = f[i][c];
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int s = 0; s < 2; ++s)
        st[k++] = m.Ns[i][r][s];
    if constexpr (Cov::on) RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int e = 0; e < 4; ++e) st[k++] = m.Pw[i][e];
    RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) st[k++] = m.eigenRot[r][c];
    st[k++] = m.planar ? 1.0 : 0.0;
}
template <int NS, class Cov>
__device__ __forceinline__ void ml_unpark(const double* st, double (&pw)[NS][3], double (&f)[NS][3], MlPrep<NS, Cov>& m) {
    int k = 0;
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int c = 0; c < 3; ++c) pw[i][c] = st[k++];
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int c = 0; c < 3; ++c) f[i][c] = st[k++];
    RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int s = 0; s < 2; ++s)
        m.Ns[i][r][s] = st[k++];
    if constexpr (Cov::on) RSC_UNROLL for (int i = 0; i < NS; ++i) RSC_UNROLL for (int e = 0; e < 4; ++e) m.Pw[i][e] = st[k++];
    RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) m.eigenRot[r][c] = st[k++];
    m.planar = st[k++] != 0.0;
}
static_assert(ml_quad_region<8, MlIndexedCov>() * kMlQuadHyps * 8 <= 48 * 1024, "the largest region");

// The parked state (ml_park layout) read in place by mlpnp_finish_pose.
template <int NS, class Cov>
struct MlParked {
    const double* st;
    static constexpr int kF = 3 * NS, kNs = 6 * NS, kPw = 12 * NS, kEig = 12 * NS + (Cov::on ? 4 * NS : 0);
    __device__ double pw(int i, int c) const { return st[3 * i + c]; }
    __device__ double f(int i, int c) const { return st[kF + 3 * i + c]; }
    __device__ double ns(int i, int r, int s) const { return st[kNs + 6 * i + 2 * r + s]; }
    __device__ double pwgt(int i, int e) const { return st[kPw + 4 * i + e]; }
    __device__ double eig(int r, int c) const { return st[kEig + 3 * r + c]; }
    __device__ bool planar() const { return st[kEig + 9] != 0.0; }
};

// One MLPnP hypothesis per quad: sample, computePose (MLPnPsolver.cpp:321-623), pose record.
template <int NS, class Cov>
__device__ __forceinline__ void mlpnp_quad_hypothesis(const DevML& P, const int (&idx)[NS], const Cov& cov, int q,
                                                      double* region, double (&Rout)[3][3], double (&tout)[3]) {
    double* stash = region + ml_quad_slab<NS>();
    double Wc[3][12], Vc[3][12];
    bool planar;
    {
        double pw[NS][3], f[NS][3];
        RSC_UNROLL for (int i = 0; i < NS; ++i) {
            const float4 p = P.pts[idx[i]];
            const float2 b = P.brg[idx[i]];
            pw[i][0] = p.x; pw[i][1] = p.y; pw[i][2] = p.z;
            f[i][0] = b.x; f[i][1] = b.y; f[i][2] = 1.0;
        }
        // the design matrix A (2 NS x 12, columns beyond colsA zero) through the GN slab: every lane
        // writes all of it (identical values, static indices), then reads its own columns back
        double* At = region;
        constexpr bool kParkAsYouGo = Cov::on || NS > 6;
        // phase-1 state: in registers (NS = 6 without covariances), or — where the nullspaces, the
        // covariance weights and the points do not fit beside each other (19 NS + 9 doubles) —
        // parked correspondence by correspondence as it is produced (ml_park's layout) and read back
        MlPrep<NS, Cov> m;
        if constexpr (!kParkAsYouGo) {
            mlpnp_prepare<NS, Cov>(pw, f, cov, m);
            planar = m.planar;
            ml_park<NS, Cov>(stash, pw, f, m);
        } else {
            using PV = MlParked<NS, Cov>;
            RSC_UNROLL for (int i = 0; i < NS; ++i) {
                double Ns[3][2];
                ml_bearing_nullspace(f[i], Ns);
                RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int s = 0; s < 2; ++s) stash[PV::kNs + 6 * i + 2 * r + s] = Ns[r][s];
                if constexpr (Cov::on) {
                    double Pw4[4];
                    ml_cov_weight(Ns, cov, i, Pw4);
                    RSC_UNROLL for (int e = 0; e < 4; ++e) stash[PV::kPw + 4 * i + e] = Pw4[e];
                }
                RSC_UNROLL for (int c = 0; c < 3; ++c) { stash[3 * i + c] = pw[i][c]; stash[PV::kF + 3 * i + c] = f[i][c]; }
            }
            double eigenRot[3][3];
            planar = ml_planarity<NS>(pw, eigenRot);
            RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) stash[PV::kEig + 3 * r + c] = eigenRot[r][c];
            stash[PV::kEig + 9] = planar ? 1.0 : 0.0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            RSC_UNROLL for (int i = 0; i < NS; ++i) {
                double Pi[3];
                ml_design_point(planar, eigenRot, pw[i], Pi);
                RSC_UNROLL for (int s = 0; s < 2; ++s) {
                    const double n0 = stash[PV::kNs + 6 * i + s], n1 = stash[PV::kNs + 6 * i + 2 + s],
                                 n2 = stash[PV::kNs + 6 * i + 4 + s];
                    RSC_UNROLL for (int c = 0; c < 12; ++c)
                        At[(2 * i + s) * 12 + c] = (c < (planar ? 9 : 12)) ? mlpnp_A_entry(planar, n0, n1, n2, Pi, c) : 0.0;
                }
            }
        }
        const int colsA = planar ? 9 : 12;
        if constexpr (!kParkAsYouGo) {
            RSC_UNROLL for (int i = 0; i < NS; ++i)
                RSC_UNROLL for (int s = 0; s < 2; ++s)
                    RSC_UNROLL for (int c = 0; c < 12; ++c)
                        At[(2 * i + s) * 12 + c] = (c < colsA) ? mlpnp_A<NS, Cov>(m, i, s, c) : 0.0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double rb[3][NS][2];  // own columns c = 4j + q
        RSC_UNROLL for (int j = 0; j < 3; ++j)
            RSC_UNROLL for (int i = 0; i < NS; ++i)
                RSC_UNROLL for (int s = 0; s < 2; ++s) rb[j][i][s] = At[(2 * i + s) * 12 + 4 * j + q];
        // normal matrix entries (r, own c) (entries outside colsA x colsA stay 0)
        RSC_UNROLL for (int r = 0; r < 12; ++r) {
            double ra[NS][2];
            RSC_UNROLL for (int i = 0; i < NS; ++i)
                RSC_UNROLL for (int s = 0; s < 2; ++s) ra[i][s] = At[(2 * i + s) * 12 + r];
            RSC_UNROLL for (int j = 0; j < 3; ++j) {
                double v;
                if constexpr (Cov::on || NS > 6) v = mlpnp_normal_entry<NS, Cov>(MlParked<NS, Cov>{stash}, ra, rb[j]);
                else v = mlpnp_normal_entry<NS, Cov>(m, ra, rb[j]);
                Wc[j][r] = (r < colsA && 4 * j + q < colsA) ? v : 0.0;
            }
        }
    }
    RSC_ML_STAMP(2);
    double r1[12];
    if (planar) ml_quad_jacobi_svd<9>(Wc, Vc, q, r1);
    else ml_quad_jacobi_svd<12>(Wc, Vc, q, r1);
    RSC_ML_STAMP(3);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (!Cov::on && NS == 6) {
        // the common case fits the registers: the state back in VGPRs for the Gauss-Newton loop
        // (fewer LDS round trips in its dependent chain; measured 2.86 vs 3.42 ms per 128-candidate step)
        double pw[NS][3], f[NS][3];
        MlPrep<NS, Cov> m;
        ml_unpark<NS, Cov>(stash, pw, f, m);
        mlpnp_finish_pose<NS, Cov>(MlRegs<NS, Cov>{pw, f, m}, MlParked<NS, Cov>{stash}, r1, LaneMat{region, 1}, Rout,
                                   tout);
    } else {
        mlpnp_finish_pose<NS, Cov>(MlParked<NS, Cov>{stash}, MlParked<NS, Cov>{stash}, r1, LaneMat{region, 1}, Rout,
                                   tout);
    }
}

}  // namespace rsc
