// rsc_epnp.h — per-lane EPnP pose (PnPsolver::compute_pose, src/PnPsolver.cpp:359-415) and the
// helpers it calls, written for one hypothesis per lane.
//
// Row storage is abstracted by a Store:
//   HypStore<NS>: the NS sampled correspondences of a RANSAC hypothesis in VGPRs (static indices);
//   RowStore:     all rows in global memory (Refine over the best inlier set, n up to N).
// Both expose the reference's grow-only EPnP buffers (Q6): rows [n, rows) are the stale rows left
// by earlier Refine() calls; every column sum over "all allocated rows" (PnPsolver.cpp:301, :356,
// :435-436) reads them, exactly as the reference does.
#pragma once
#include "rsc_core.h"

namespace rsc {

struct Intrinsics {
    double fx, fy, cx, cy;
};

// Free slots of the per-lane slab once the 12x12 eigenvectors are formed: columns 4..11 of every
// row (96 doubles) plus 16 extra doubles after the matrix.  L_6x10 and rho live there.
RSC_HD int slab_free(int q) { return q < 96 ? (q >> 3) * 12 + 4 + (q & 7) : 144 + (q - 96); }
constexpr int kSlabDoubles = 160;  // per lane: 64 lanes x 160 x 8 B = 80 KiB per workgroup

template <int NS>
struct HypStore {
    double pw_[NS][3], u_[NS][2], al_[NS][4];
    int rows_;                      // maximum_number_of_correspondences
    const double* __restrict__ spw;  // stale pws  [rows][3]   (global, rows >= NS read)
    const double* __restrict__ sal;  // stale alphas [rows][4]
    RSC_HD static constexpr int n() { return NS; }
    RSC_HD int rows() const { return rows_; }
    RSC_HD double pw(int i, int c) const { return pw_[i][c]; }
    RSC_HD double u(int i, int c) const { return u_[i][c]; }
    RSC_HD double al(int i, int j) const { return al_[i][j]; }
    RSC_HD void set_al(int i, int j, double v) { al_[i][j] = v; }
#if defined(__HIP_DEVICE_COMPILE__)
    // The stale tail is the same for every lane of a workgroup (all its hypotheses belong to one
    // problem) and read-only within the kernel: read through the constant address space it is
    // fetched with scalar loads, one broadcast per row, instead of a vector load round trip per
    // row inside the dependent chain (hundreds of rows after a Refine).
    RSC_HD double stale_pw(int i, int c) const {
        return ((const __attribute__((address_space(4))) double*)spw)[3 * i + c];
    }
    RSC_HD double stale_al(int i, int j) const {
        return ((const __attribute__((address_space(4))) double*)sal)[4 * i + j];
    }
#else
    RSC_HD double stale_pw(int i, int c) const { return spw[3 * i + c]; }
    RSC_HD double stale_al(int i, int j) const { return sal[4 * i + j]; }
#endif
};

struct RowStore {
    int n_, rows_;
    double* __restrict__ pws;     // [rows][3]
    const double* __restrict__ us; // [n][2]
    double* __restrict__ als;     // [rows][4]
    RSC_HD int n() const { return n_; }
    RSC_HD int rows() const { return rows_; }
    RSC_HD double pw(int i, int c) const { return pws[3 * i + c]; }
    RSC_HD double u(int i, int c) const { return us[2 * i + c]; }
    RSC_HD double al(int i, int j) const { return als[4 * i + j]; }
    RSC_HD void set_al(int i, int j, double v) { als[4 * i + j] = v; }
    RSC_HD double stale_pw(int i, int c) const { return pws[3 * i + c]; }
    RSC_HD double stale_al(int i, int j) const { return als[4 * i + j]; }
};

// Column sums of pws over ALL allocated rows (current rows first, then stale rows), each column's
// additions in row order; the three columns share one pass over the stale tail (Q6: after a
// Refine the tail holds hundreds of rows, read from global memory).
template <class St>
RSC_HD void sum_pw_cols(const St& st, double (&s)[3]) {
    RSC_UNROLL for (int c = 0; c < 3; ++c) {
        s[c] = st.pw(0, c);
        RSC_UNROLL for (int i = 1; i < st.n(); ++i) s[c] = s[c] + st.pw(i, c);
    }
#pragma unroll 4
    for (int i = st.n(); i < st.rows(); ++i) {
        const double a = st.stale_pw(i, 0), b = st.stale_pw(i, 1), d = st.stale_pw(i, 2);
        s[0] = s[0] + a;
        s[1] = s[1] + b;
        s[2] = s[2] + d;
    }
}

// choose_control_points + compute_barycentric_coordinates (PnPsolver.cpp:296-343).
// Returns cws (4x3).
template <class St>
RSC_HD void control_points_and_alphas(St& st, double (&cws)[4][3]) {
    const int n = st.n();
    sum_pw_cols(st, cws[0]);
    RSC_UNROLL for (int c = 0; c < 3; ++c) cws[0][c] = cws[0][c] / n;
    double A[3][3];
    RSC_UNROLL for (int a = 0; a < 3; ++a)
        RSC_UNROLL for (int b = 0; b < 3; ++b) {
            double s = (st.pw(0, a) - cws[0][a]) * (st.pw(0, b) - cws[0][b]);
            RSC_UNROLL for (int i = 1; i < n; ++i) s = s + (st.pw(i, a) - cws[0][a]) * (st.pw(i, b) - cws[0][b]);
            A[a][b] = s;
        }
    double V[3][3], w[3];
    sym_eig_reg<double, 3>(A, V, w);
    RSC_UNROLL for (int i = 0; i < 3; ++i) {
        double k = sqrt(w[i] / n);
        RSC_UNROLL for (int c = 0; c < 3; ++c) cws[i + 1][c] = cws[0][c] + k * V[c][i];
    }
    double CC[3][3], CCi[3][3];
    RSC_UNROLL for (int i = 0; i < 3; ++i)
        RSC_UNROLL for (int j = 1; j < 4; ++j) CC[i][j - 1] = cws[j][i] - cws[0][i];
    inverse3(CC, CCi);
    RSC_UNROLL for (int i = 0; i < n; ++i) {
        double d0 = st.pw(i, 0) - cws[0][0];
        double d1 = st.pw(i, 1) - cws[0][1];
        double d2 = st.pw(i, 2) - cws[0][2];
        // CC_inv.row(j).dot(pws.row(i) - cws.row(0)) (:338): rows of column-major matrices, ered3
        double a1 = ered3(CCi[0][0] * d0, CCi[0][1] * d1, CCi[0][2] * d2);
        double a2 = ered3(CCi[1][0] * d0, CCi[1][1] * d1, CCi[1][2] * d2);
        double a3 = ered3(CCi[2][0] * d0, CCi[2][1] * d1, CCi[2][2] * d2);
        st.set_al(i, 1, a1);
        st.set_al(i, 2, a2);
        st.set_al(i, 3, a3);
        st.set_al(i, 0, 1.0 - a1 - a2 - a3);
    }
}

// Entry (r, col) of the 2n x 12 matrix M (PnPsolver.cpp:365-377).
template <class St>
RSC_HD double M_entry(const St& st, const Intrinsics& K, int r, int col) {
    const int i = r >> 1, j = col / 3, s = col % 3;
    const double a = st.al(i, j);
    if ((r & 1) == 0) {
        if (s == 0) return a * K.fx;
        if (s == 1) return 0.0;
        return a * (K.cx - st.u(i, 0));
    } else {
        if (s == 0) return 0.0;
        if (s == 1) return a * K.fy;
        return a * (K.cy - st.u(i, 1));
    }
}

// Lower triangle of MtM = M^T M into the slab (sum over the 2n rows, first term first).
template <class St>
RSC_HD void build_MtM(const St& st, const Intrinsics& K, const LaneMat& S) {
    const int rows2 = 2 * st.n();
    RSC_UNROLL for (int a = 0; a < 12; ++a)
        RSC_UNROLL for (int b = 0; b <= a; ++b) {
            double s = M_entry(st, K, 0, a) * M_entry(st, K, 0, b);
            RSC_UNROLL for (int r = 1; r < rows2; ++r) s = s + M_entry(st, K, r, a) * M_entry(st, K, r, b);
            S.at(a, b) = s;
        }
}

RSC_HD double& Lref(const LaneMat& S, int i, int j) { return S(slab_free(i * 10 + j)); }
RSC_HD double& rhoref(const LaneMat& S, int i) { return S(slab_free(60 + i)); }

// Stage-C storage views: eigenvector columns 0..3 (ev), L_6x10 and rho.
// SlabView: everything inside one per-lane slab (the lane-per-hypothesis kernels and Refine).
struct SlabView {
    LaneMat S;
    RSC_HD double ev(int r, int c) const { return S.at(r, c); }
    RSC_HD double& L(int i, int j) const { return Lref(S, i, j); }
    RSC_HD double& rho(int i) const { return rhoref(S, i); }
};
// SplitView: eigenvectors [12][4], L [6][10] + rho [6] in separate (LDS) arrays, element stride
// `stride` (1 = contiguous per hypothesis, 64 = element-major across a wave).
struct SplitView {
    const double* evp;
    double* Lp;
    int stride;
    RSC_HD double ev(int r, int c) const { return evp[(r * 4 + c) * stride]; }
    RSC_HD double& L(int i, int j) const { return Lp[(i * 10 + j) * stride]; }
    RSC_HD double& rho(int i) const { return Lp[(60 + i) * stride]; }
};

// compute_L_6x10 (PnPsolver.cpp:604-637) from the eigenvector columns 0..3 held in the slab.
template <class SV>
RSC_HD void compute_L_6x10(const SV& S) {
    RSC_UNROLL for (int j = 0; j < 6; ++j) {
        const int a = (j < 3) ? 0 : (j < 5 ? 1 : 2);
        const int b = (j < 3) ? j + 1 : (j < 5 ? j - 1 : 3);
        double dv[4][3];
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) dv[i][c] = S.ev(3 * a + c, i) - S.ev(3 * b + c, i);
        // dv[i].row(j).dot(...) (:626-635): rows of Matrix<double,6,3>, ered3
        auto dot = [&](int x, int y) { return ered3(dv[x][0] * dv[y][0], dv[x][1] * dv[y][1], dv[x][2] * dv[y][2]); };
        S.L(j, 0) = dot(0, 0);
        S.L(j, 1) = 2.0 * dot(0, 1);
        S.L(j, 2) = dot(1, 1);
        S.L(j, 3) = 2.0 * dot(0, 2);
        S.L(j, 4) = 2.0 * dot(1, 2);
        S.L(j, 5) = dot(2, 2);
        S.L(j, 6) = 2.0 * dot(0, 3);
        S.L(j, 7) = 2.0 * dot(1, 3);
        S.L(j, 8) = 2.0 * dot(2, 3);
        S.L(j, 9) = dot(3, 3);
    }
}

// qr_solve (PnPsolver.cpp:693-796).  Returns false on the singular bail-out (X left unchanged):
// rows k..4 of column k all zero (Q19: row 5 is not looked at, :714-726).
RSC_HD bool qr_solve_6x4(double (&A)[6][4], double (&b)[6], double (&X)[4]) {
    double A1[4], A2[4];
    bool singular = false;
    RSC_UNROLL for (int k = 0; k < 4; k++) {
        if (!singular) {
            // Q19: the reference's pointer loop (:714-720) reads *ppAik before advancing it, so
            // eta is the largest |A[i][k]| over rows k..4 (row k twice, row 5 never).
            double eta = rabs(A[k][k]);
            RSC_UNROLL for (int i = k + 1; i < 6; i++) {
                double elt = rabs(A[i - 1][k]);
                if (eta < elt) eta = elt;
            }
            if (eta == 0) {
                singular = true;
            } else {
                double sum = 0.0, inv_eta = 1. / eta;
                RSC_UNROLL for (int i = k; i < 6; i++) {
                    A[i][k] *= inv_eta;
                    sum += A[i][k] * A[i][k];
                }
                double sigma = sqrt(sum);
                if (A[k][k] < 0) sigma = -sigma;
                A[k][k] += sigma;
                A1[k] = sigma * A[k][k];
                A2[k] = -eta * sigma;
                RSC_UNROLL for (int j = k + 1; j < 4; j++) {
                    double s = 0;
                    RSC_UNROLL for (int i = k; i < 6; i++) s += A[i][k] * A[i][j];
                    double tau = s / A1[k];
                    RSC_UNROLL for (int i = k; i < 6; i++) A[i][j] -= tau * A[i][k];
                }
            }
        }
    }
    if (singular) return false;
    RSC_UNROLL for (int j = 0; j < 4; j++) {
        double tau = 0;
        RSC_UNROLL for (int i = j; i < 6; i++) tau += A[i][j] * b[i];
        tau /= A1[j];
        RSC_UNROLL for (int i = j; i < 6; i++) b[i] -= tau * A[i][j];
    }
    X[3] = b[3] / A2[3];
    RSC_UNROLL for (int i = 2; i >= 0; i--) {
        double s = 0;
        RSC_UNROLL for (int j = i + 1; j < 4; j++) s += A[i][j] * X[j];
        X[i] = (b[i] - s) / A2[i];
    }
    return true;
}

// gauss_newton (PnPsolver.cpp:649-691); X persists across the 5 iterations (Q9).
template <class SV>
RSC_HD void gauss_newton(const SV& S, double (&betas)[4]) {
    double X[4] = {0.0, 0.0, 0.0, 0.0};
    // Rolled, with a compiler-only memory fence per iteration: unrolled (or with the L reads
    // hoisted out of the loop) the 60 L entries stay live in VGPRs across all five solves and the
    // betas kernel spills to scratch; re-read from the view (LDS) they cost 60 loads per iteration.
#pragma unroll 1
    for (int it = 0; it < 5; it++) {
        asm volatile("" ::: "memory");
        double A[6][4], B[6];
        RSC_UNROLL for (int i = 0; i < 6; i++) {
            double l[10];
            RSC_UNROLL for (int j = 0; j < 10; ++j) l[j] = S.L(i, j);
            const double Lt[4][4] = {{2 * l[0], l[1], l[3], l[6]},
                                     {l[1], 2 * l[2], l[4], l[7]},
                                     {l[3], l[4], 2 * l[5], l[8]},
                                     {l[6], l[7], l[8], 2 * l[9]}};
            RSC_UNROLL for (int r = 0; r < 4; ++r)
                A[i][r] = Lt[r][0] * betas[0] + Lt[r][1] * betas[1] + Lt[r][2] * betas[2] + Lt[r][3] * betas[3];
            const double* b = betas;
            B[i] = S.rho(i) - (l[0] * b[0] * b[0] + l[1] * b[0] * b[1] + l[2] * b[1] * b[1] +
                                   l[3] * b[0] * b[2] + l[4] * b[1] * b[2] + l[5] * b[2] * b[2] +
                                   l[6] * b[0] * b[3] + l[7] * b[1] * b[3] + l[8] * b[2] * b[3] +
                                   l[9] * b[3] * b[3]);
        }
        qr_solve_6x4(A, B, X);
        RSC_UNROLL for (int c = 0; c < 4; ++c) betas[c] = betas[c] + X[c];
    }
}

// find_betas_approx_{1,2,3} (PnPsolver.cpp:520-602).
// LaneRows: the wave's lanes hold the same problem (jacobi_svd_solve_6xk's lane-row form).
template <int which, class SV, bool LaneRows = false>
RSC_HD void find_betas(const SV& S, double (&betas)[4]) {
    double rho[6];
    RSC_UNROLL for (int r = 0; r < 6; ++r) rho[r] = S.rho(r);
    if (which == 1) {
        double A[6][4], b4[4];
        RSC_UNROLL for (int r = 0; r < 6; ++r) {
            A[r][0] = S.L(r, 0); A[r][1] = S.L(r, 1); A[r][2] = S.L(r, 3); A[r][3] = S.L(r, 6);
        }
        jacobi_svd_solve_6xk<4, LaneRows>(A, rho, b4);
        if (b4[0] < 0) {
            betas[0] = sqrt(-b4[0]);
            betas[1] = -b4[1] / betas[0];
            betas[2] = -b4[2] / betas[0];
            betas[3] = -b4[3] / betas[0];
        } else {
            betas[0] = sqrt(b4[0]);
            betas[1] = b4[1] / betas[0];
            betas[2] = b4[2] / betas[0];
            betas[3] = b4[3] / betas[0];
        }
    } else if (which == 2) {
        double A[6][3], b3[3];
        RSC_UNROLL for (int r = 0; r < 6; ++r) { A[r][0] = S.L(r, 0); A[r][1] = S.L(r, 1); A[r][2] = S.L(r, 2); }
        jacobi_svd_solve_6xk<3, LaneRows>(A, rho, b3);
        if (b3[0] < 0) {
            betas[0] = sqrt(-b3[0]);
            betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
        } else {
            betas[0] = sqrt(b3[0]);
            betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) betas[0] = -betas[0];
        betas[2] = 0.0;
        betas[3] = 0.0;
    } else {
        double A[6][5], b5[5];
        RSC_UNROLL for (int r = 0; r < 6; ++r)
            RSC_UNROLL for (int c = 0; c < 5; ++c) A[r][c] = S.L(r, c);
        jacobi_svd_solve_6xk<5, LaneRows>(A, rho, b5);
        if (b5[0] < 0) {
            betas[0] = sqrt(-b5[0]);
            betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
        } else {
            betas[0] = sqrt(b5[0]);
            betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) betas[0] = -betas[0];
        betas[2] = b5[3] / betas[0];
        betas[3] = 0.0;
    }
}

// compute_ccs (PnPsolver.cpp:285-294) + the sign test of solve_for_sign (:445-456): pcs(0,2) of
// the unflipped ccs decides whether every ccs is negated.
template <class St, class SV>
RSC_HD void ccs_with_sign(const St& st, const SV& S, const double (&betas)[4], double (&ccs)[4][3]) {
    RSC_UNROLL for (int i = 0; i < 4; i++)
        RSC_UNROLL for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            RSC_UNROLL for (int j = 0; j < 4; j++) s = s + betas[j] * S.ev(3 * i + c, j);
            ccs[i][c] = s;
        }
    const double pcs02 = st.al(0, 0) * ccs[0][2] + st.al(0, 1) * ccs[1][2] + st.al(0, 2) * ccs[2][2] +
                         st.al(0, 3) * ccs[3][2];
    if (pcs02 < 0.0) {
        RSC_UNROLL for (int i = 0; i < 4; ++i)
            RSC_UNROLL for (int c = 0; c < 3; ++c) ccs[i][c] = -ccs[i][c];
    }
}

// pcs row i (compute_pcs, :296-305) from alphas a[4] and ccs.
RSC_HD double pcs_of(const double (&a)[4], const double (&ccs)[4][3], int c) {
    return a[0] * ccs[0][c] + a[1] * ccs[1][c] + a[2] * ccs[2][c] + a[3] * ccs[3][c];
}

// Horn step of estimate_R_and_t (:474-493) from the accumulated M: float N entries, 4x4
// eigenvectors, conjugated quaternion, det fix, t = pc0 - R pw0.
RSC_HD void horn_from_M(const double (&M)[3][3], const double (&pc0)[3], const double (&pw0)[3], double (&R)[3][3],
                        double (&t)[3]) {
    const float N11 = M[0][0] + M[1][1] + M[2][2];
    const float N12 = M[1][2] - M[2][1];
    const float N13 = M[2][0] - M[0][2];
    const float N14 = M[0][1] - M[1][0];
    const float N22 = M[0][0] - M[1][1] - M[2][2];
    const float N23 = M[0][1] + M[1][0];
    const float N24 = M[2][0] + M[0][2];
    const float N33 = -M[0][0] + M[1][1] - M[2][2];
    const float N34 = M[1][2] + M[2][1];
    const float N44 = -M[0][0] - M[1][1] + M[2][2];
    const double Nm[4][4] = {{N11, N12, N13, N14}, {N12, N22, N23, N24}, {N13, N23, N33, N34}, {N14, N24, N34, N44}};
    double V[4][4], w[4];
    sym_eig_reg<double, 4>(Nm, V, w);
    quat_to_R<double>(V[0][3], -V[1][3], -V[2][3], -V[3][3], R);
    if (det3(R) < 0) {
        RSC_UNROLL for (int c = 0; c < 3; ++c) R[2][c] = -R[2][c];
    }
    // t = pc0 - R*pw0 (:492) into a Vector3d: emv3d_row
    RSC_UNROLL for (int r = 0; r < 3; ++r) t[r] = pc0[r] - emv3d_row(r, R[r][0] * pw0[0], R[r][1] * pw0[1], R[r][2] * pw0[2]);
}

// One term of reprojection_error (:417-431).
RSC_HD double reproj_term(const double (&R)[3][3], const double (&t)[3], const Intrinsics& K, double P0, double P1,
                          double P2, double u0, double u1) {
    // R*pws.row(i).transpose() + t (:423) into a Vector3d: emv3d_row
    double X = emv3d_row(0, R[0][0] * P0, R[0][1] * P1, R[0][2] * P2) + t[0];
    double Y = emv3d_row(1, R[1][0] * P0, R[1][1] * P1, R[1][2] * P2) + t[1];
    double Z = emv3d_row(2, R[2][0] * P0, R[2][1] * P1, R[2][2] * P2) + t[2];
    double inv_Zc = 1.0 / Z;
    double u = K.cx + K.fx * X * inv_Zc;
    double v = K.cy + K.fy * Y * inv_Zc;
    double du = u0 - u, dv = u1 - v;
    return sqrt(du * du + dv * dv);
}

// compute_R_and_t (PnPsolver.cpp:504-515) = compute_ccs + compute_pcs + solve_for_sign +
// estimate_R_and_t (:433-493, Horn with float N entries, conjugated quaternion) +
// reprojection_error (:417-431).  pw0 equals the centroid cws[0] (same sum, same division).
template <class St, class SV>
RSC_HD double compute_R_and_t(const St& st, const Intrinsics& K, const SV& S, const double (&betas)[4],
                              const double (&pw0)[3], double (&R)[3][3], double (&t)[3]) {
    const int n = st.n();
    double ccs[4][3];
    ccs_with_sign(st, S, betas, ccs);
    auto pcs = [&](int i, int c) {
        return st.al(i, 0) * ccs[0][c] + st.al(i, 1) * ccs[1][c] + st.al(i, 2) * ccs[2][c] + st.al(i, 3) * ccs[3][c];
    };
    double pc0[3];
    RSC_UNROLL for (int c = 0; c < 3; ++c) {
        double s = pcs(0, c);
        RSC_UNROLL for (int i = 1; i < n; ++i) s = s + pcs(i, c);
        pc0[c] = s;
    }
    // stale rows (Q6): one pass, the row's alphas loaded once for the three columns
#pragma unroll 4
    for (int i = n; i < st.rows(); ++i) {
        const double a0 = st.stale_al(i, 0), a1 = st.stale_al(i, 1), a2 = st.stale_al(i, 2), a3 = st.stale_al(i, 3);
        RSC_UNROLL for (int c = 0; c < 3; ++c)
            pc0[c] = pc0[c] + (a0 * ccs[0][c] + a1 * ccs[1][c] + a2 * ccs[2][c] + a3 * ccs[3][c]);
    }
    RSC_UNROLL for (int c = 0; c < 3; ++c) pc0[c] = pc0[c] / n;
    double M[3][3];
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) M[r][c] = 0.0;
    RSC_UNROLL for (int i = 0; i < n; ++i) {
        double a[3], b[3];
        RSC_UNROLL for (int c = 0; c < 3; ++c) { a[c] = pcs(i, c) - pc0[c]; b[c] = st.pw(i, c) - pw0[c]; }
        RSC_UNROLL for (int r = 0; r < 3; ++r)
            RSC_UNROLL for (int c = 0; c < 3; ++c) M[r][c] = M[r][c] + a[r] * b[c];
    }
    horn_from_M(M, pc0, pw0, R, t);
    double sum2 = 0.0;
    RSC_UNROLL for (int i = 0; i < n; i++)
        sum2 += reproj_term(R, t, K, st.pw(i, 0), st.pw(i, 1), st.pw(i, 2), st.u(i, 0), st.u(i, 1));
    return sum2 / n;
}

// Second half of compute_pose: with the lower triangle of MtM already in the slab, run the 12x12
// eigensolver, L_6x10/rho, the three beta approximations + Gauss-Newton + compute_R_and_t, and
// keep the smallest reprojection error (PnPsolver.cpp:379-414).
struct NoStamp {
    RSC_HD void operator()(int) const {}
};

template <class St, class Stamp = NoStamp>
RSC_HD double epnp_stage_c(const St& st, const Intrinsics& K, const LaneMat& S, const double (&cws)[4][3],
                           float (&Rf)[9], float (&tf)[3], Stamp stamp = Stamp()) {
    sym_eig12(S);
    stamp(3);
    return epnp_betas_and_pose(st, K, SlabView{S}, cws, Rf, tf, stamp);
}

// L_6x10, rho, the three beta approximations + Gauss-Newton + compute_R_and_t, smallest
// reprojection error wins (PnPsolver.cpp:383-414), given the eigenvectors in the view.
template <class St, class SV, class Stamp = NoStamp>
RSC_HD double epnp_betas_and_pose(const St& st, const Intrinsics& K, const SV& S, const double (&cws)[4][3],
                                  float (&Rf)[9], float (&tf)[3], Stamp stamp = Stamp()) {
    compute_L_6x10(S);
    {
        auto d2 = [&](int a, int b) {
            double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
            return ered3(x * x, y * y, z * z);  // squaredNorm of a row of cws (:640-645)
        };
        S.rho(0) = d2(0, 1); S.rho(1) = d2(0, 2); S.rho(2) = d2(0, 3);
        S.rho(3) = d2(1, 2); S.rho(4) = d2(1, 3); S.rho(5) = d2(2, 3);
    }
    const double pw0[3] = {cws[0][0], cws[0][1], cws[0][2]};
    double bestR[3][3], bestt[3], best_err;
    {
        double betas[4] = {0.0, 0.0, 0.0, 0.0};
        find_betas<1>(S, betas);
        stamp(4);
        gauss_newton(S, betas);
        stamp(5);
        best_err = compute_R_and_t(st, K, S, betas, pw0, bestR, bestt);
        stamp(6);
    }
    {
        double betas[4] = {0.0, 0.0, 0.0, 0.0}, R[3][3], t[3];
        find_betas<2>(S, betas);
        gauss_newton(S, betas);
        double e = compute_R_and_t(st, K, S, betas, pw0, R, t);
        stamp(7);
        if (e < best_err) {
            best_err = e;
            RSC_UNROLL for (int r = 0; r < 3; ++r) {
                bestt[r] = t[r];
                RSC_UNROLL for (int c = 0; c < 3; ++c) bestR[r][c] = R[r][c];
            }
        }
    }
    {
        double betas[4] = {0.0, 0.0, 0.0, 0.0}, R[3][3], t[3];
        find_betas<3>(S, betas);
        gauss_newton(S, betas);
        double e = compute_R_and_t(st, K, S, betas, pw0, R, t);
        stamp(8);
        if (e < best_err) {
            best_err = e;
            RSC_UNROLL for (int r = 0; r < 3; ++r) {
                bestt[r] = t[r];
                RSC_UNROLL for (int c = 0; c < 3; ++c) bestR[r][c] = R[r][c];
            }
        }
    }
    RSC_UNROLL for (int r = 0; r < 3; ++r) {
        tf[r] = (float)bestt[r];
        RSC_UNROLL for (int c = 0; c < 3; ++c) Rf[3 * r + c] = (float)bestR[r][c];
    }
    return best_err;
}

// PnPsolver::compute_pose (PnPsolver.cpp:359-415) for one lane.  Outputs float R (row-major) and t.
template <class St, class Stamp = NoStamp>
RSC_HD double epnp_compute_pose(St& st, const Intrinsics& K, const LaneMat& S, float (&Rf)[9], float (&tf)[3],
                                Stamp stamp = Stamp()) {
    double cws[4][3];
    control_points_and_alphas(st, cws);
    stamp(1);
    build_MtM(st, K, S);
    stamp(2);
    return epnp_stage_c(st, K, S, cws, Rf, tf, stamp);
}

}  // namespace rsc
