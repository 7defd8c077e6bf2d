// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
// Restatement of src/PnPsolver.cpp (reference) — see pnp_oracle.h.  Line numbers cite the reference.
#include "pnp_oracle.h"
#include "ora_linalg.h"
#include <cmath>
#include <algorithm>

namespace rsc_oracle {

static void set_identity4(float T[16]) {
    for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.f : 0.f;
}

// PnPsolver.cpp:11-55
PnPOracle::PnPOracle(int n, int n_points, const float* p2d, const float* p3dw, const float* sigma2,
                     const int32_t* kp_index, float fx_, float fy_, float cx_, float cy_, uint32_t seed)
    : rng(seed) {
    N_points = n_points;
    mvP2D.assign(p2d, p2d + 2 * n);
    mvSigma2.assign(sigma2, sigma2 + n);
    mvP3Dw.assign(p3dw, p3dw + 3 * n);
    mvKeyPointIndices.assign(kp_index, kp_index + n);
    mvAllIndices.resize(n);
    for (int i = 0; i < n; ++i) mvAllIndices[i] = i;
    fx = fx_; fy = fy_; cx = cx_; cy = cy_;
    set_identity4(mRefinedTcw);
    set_identity4(mBestTcw);
    for (int i = 0; i < 4; ++i) qr_X[i] = 0.0;
    for (int i = 0; i < 3; ++i) { mti[i] = 0.f; for (int j = 0; j < 3; ++j) mRi[i][j] = 0.f; }
}

// PnPsolver.cpp:58-94
void PnPOracle::SetRansacParameters(double probability, int minInliers, int maxIterations, int minSet,
                                    float epsilon, float th2) {
    mRansacProb = probability;
    mRansacMinInliers = minInliers;
    mRansacMaxIts = maxIterations;
    mRansacEpsilon = epsilon;
    mRansacMinSet = minSet;
    N = (int)(mvP2D.size() / 2);
    mvbInliersi.assign(N, 0);
    int nMinInliers = N * mRansacEpsilon;  // float product truncated (Q2)
    if (nMinInliers < mRansacMinInliers) nMinInliers = mRansacMinInliers;
    if (nMinInliers < minSet) nMinInliers = minSet;
    mRansacMinInliers = nMinInliers;
    if (mRansacEpsilon < (float)mRansacMinInliers / N) mRansacEpsilon = (float)mRansacMinInliers / N;
    int nIterations;
    if (mRansacMinInliers == N)
        nIterations = 1;
    else
        nIterations = (int)std::ceil(std::log(1 - mRansacProb) / std::log(1 - std::pow((double)mRansacEpsilon, 3.0)));
    mRansacMaxIts = std::max(1, std::min(nIterations, mRansacMaxIts));
    mvMaxError.resize(mvSigma2.size());
    for (size_t i = 0; i < mvSigma2.size(); i++) mvMaxError[i] = mvSigma2[i] * th2;
}

// PnPsolver.cpp:96-100
bool PnPOracle::find(std::vector<uint8_t>& vbInliers, int& nInliers, float T[16]) {
    bool bFlag;
    return iterate(mRansacMaxIts, bFlag, vbInliers, nInliers, T);
}

// PnPsolver.cpp:102-191
bool PnPOracle::iterate(int nIterations, bool& bNoMore, std::vector<uint8_t>& vbInliers, int& nInliers,
                        float T[16]) {
    bNoMore = false;
    vbInliers.clear();
    nInliers = 0;
    set_maximum_number_of_correspondences(mRansacMinSet);
    if (N < mRansacMinInliers) {
        bNoMore = true;
        return false;
    }
    int nCurrentIterations = 0;
    while (mnIterations < mRansacMaxIts || nCurrentIterations < nIterations) {  // Q1: '||'
        nCurrentIterations++;
        mnIterations++;
        reset_correspondences();
        // Swap-remove sampling over a fresh copy of mvAllIndices (:125-138).  Only the touched
        // slots are materialised; the result is identical to copying the whole vector.
        std::vector<int32_t> vAvailableIndices = mvAllIndices;
        PnPTrace tr{};
        for (short i = 0; i < mRansacMinSet; ++i) {
            int randi = rng.random_int(0, (int)vAvailableIndices.size() - 1);
            int idx = vAvailableIndices[randi];
            if (i < 8) tr.sample[i] = idx;
            add_correspondence(&mvP3Dw[3 * idx], &mvP2D[2 * idx]);
            vAvailableIndices[randi] = vAvailableIndices.back();
            vAvailableIndices.pop_back();
        }
        compute_pose(mRi, mti);
        CheckInliers();
        tr.n_inliers = mnInliersi;
        for (int r = 0; r < 3; ++r) { tr.t[r] = mti[r]; for (int c = 0; c < 3; ++c) tr.R[3 * r + c] = mRi[r][c]; }
        if (mnInliersi >= mRansacMinInliers) {
            if (mnInliersi > mnBestInliers) {
                mvbBestInliers = mvbInliersi;
                mnBestInliers = mnInliersi;
                for (int r = 0; r < 3; ++r) {
                    for (int c = 0; c < 3; ++c) mBestTcw[4 * r + c] = mRi[r][c];
                    mBestTcw[4 * r + 3] = mti[r];
                }
            }
            tr.refine_called = 1;
            bool ok = Refine();
            tr.refine_inliers = mnRefinedInliers;
            tr.refine_ok = ok;
            if (trace) trace->push_back(tr);
            if (ok) {
                nInliers = mnRefinedInliers;
                vbInliers.assign(N_points, 0);
                for (int i = 0; i < N; i++)
                    if (mvbRefinedInliers[i]) vbInliers[mvKeyPointIndices[i]] = 1;
                for (int i = 0; i < 16; ++i) T[i] = mRefinedTcw[i];
                return true;
            }
        } else if (trace) {
            trace->push_back(tr);
        }
    }
    if (mnIterations >= mRansacMaxIts) {
        bNoMore = true;
        if (mnBestInliers >= mRansacMinInliers) {
            nInliers = mnBestInliers;
            vbInliers.assign(N_points, 0);
            for (int i = 0; i < N; i++)
                if (mvbBestInliers[i]) vbInliers[mvKeyPointIndices[i]] = 1;
            for (int i = 0; i < 16; ++i) T[i] = mBestTcw[i];
            return true;
        }
    }
    return false;
}

// PnPsolver.cpp:193-238
bool PnPOracle::Refine() {
    std::vector<int> vIndices;
    vIndices.reserve(mvbBestInliers.size());
    for (size_t i = 0; i < mvbBestInliers.size(); i++)
        if (mvbBestInliers[i]) vIndices.push_back((int)i);
    set_maximum_number_of_correspondences((int)vIndices.size());
    reset_correspondences();
    for (size_t i = 0; i < vIndices.size(); i++) {
        int idx = vIndices[i];
        add_correspondence(&mvP3Dw[3 * idx], &mvP2D[2 * idx]);
    }
    compute_pose(mRi, mti);
    CheckInliers();
    mnRefinedInliers = mnInliersi;
    mvbRefinedInliers = mvbInliersi;
    if (mnInliersi > mRansacMinInliers) {  // Q8: strict
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) mRefinedTcw[4 * r + c] = mRi[r][c];
            mRefinedTcw[4 * r + 3] = mti[r];
        }
        return true;
    }
    return false;
}

// PnPsolver.cpp:241-268 — float rotation/translation, float reciprocal, projection evaluated in
// double (cx,fx are double members) and rounded to float, float squared error (Q7).
void PnPOracle::CheckInliers() {
    mnInliersi = 0;
    for (int i = 0; i < N; i++) {
        const float* P = &mvP3Dw[3 * i];
        const float* p = &mvP2D[2 * i];
        // :250 Matrix3f * Vector3f: three coefficient-path reductions (ered3), then + mti
        float Xc = ered3(mRi[0][0] * P[0], mRi[0][1] * P[1], mRi[0][2] * P[2]) + mti[0];
        float Yc = ered3(mRi[1][0] * P[0], mRi[1][1] * P[1], mRi[1][2] * P[2]) + mti[1];
        float Zc = ered3(mRi[2][0] * P[0], mRi[2][1] * P[1], mRi[2][2] * P[2]) + mti[2];
        float invZc = 1 / Zc;
        float ue = (float)(cx + fx * Xc * invZc);
        float ve = (float)(cy + fy * Yc * invZc);
        float du = ue - p[0], dv = ve - p[1];
        float error2 = du * du + dv * dv;
        if (error2 < mvMaxError[i]) {
            mvbInliersi[i] = 1;
            mnInliersi++;
        } else {
            mvbInliersi[i] = 0;
        }
    }
}

// PnPsolver.cpp:271-281 — grow-only, zero-filled on growth (Q6).
void PnPOracle::set_maximum_number_of_correspondences(int n) {
    if (maximum_number_of_correspondences < n) {
        maximum_number_of_correspondences = n;
        pws.assign(3 * n, 0.0);
        us.assign(2 * n, 0.0);
        alphas.assign(4 * n, 0.0);
        pcs.assign(3 * n, 0.0);
    }
}

// PnPsolver.cpp:288-294
void PnPOracle::add_correspondence(const float* p3D, const float* p2D) {
    const int r = number_of_correspondences;
    pws[3 * r + 0] = p3D[0]; pws[3 * r + 1] = p3D[1]; pws[3 * r + 2] = p3D[2];
    us[2 * r + 0] = p2D[0]; us[2 * r + 1] = p2D[1];
    number_of_correspondences++;
}

// PnPsolver.cpp:296-321 — centroid over ALL allocated rows (stale rows included, Q6), divided by n;
// PCA axes in ASCENDING eigenvalue order (Q4).
void PnPOracle::choose_control_points() {
    const int n = number_of_correspondences, rows = maximum_number_of_correspondences;
    for (int i = 0; i < 4; ++i) for (int c = 0; c < 3; ++c) cws[i][c] = 0.0;
    for (int c = 0; c < 3; ++c) {
        double s = pws[c];
        for (int i = 1; i < rows; ++i) s = s + pws[3 * i + c];
        cws[0][c] = s;
    }
    for (int c = 0; c < 3; ++c) cws[0][c] = cws[0][c] / n;
    std::vector<double> PW0(3 * n);
    for (int i = 0; i < n; i++)
        for (int c = 0; c < 3; ++c) PW0[3 * i + c] = pws[3 * i + c] - cws[0][c];
    double A[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double s = PW0[a] * PW0[b];
            for (int i = 1; i < n; ++i) s = s + PW0[3 * i + a] * PW0[3 * i + b];
            A[a][b] = s;
        }
    SymEig<double, 3> es = sym_eig<double, 3>(A);
    for (int i = 0; i < 3; i++) {
        double k = std::sqrt(es.w[i] / n);
        for (int c = 0; c < 3; ++c) cws[i + 1][c] = cws[0][c] + k * es.V[c][i];
    }
}

// PnPsolver.cpp:323-343
void PnPOracle::compute_barycentric_coordinates() {
    double CC[3][3], CC_inv[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) CC[i][j - 1] = cws[j][i] - cws[0][i];
    inverse3(CC, CC_inv);
    for (int i = 0; i < number_of_correspondences; i++) {
        double d0 = pws[3 * i + 0] - cws[0][0];
        double d1 = pws[3 * i + 1] - cws[0][1];
        double d2 = pws[3 * i + 2] - cws[0][2];
        // :338 row(j).dot(...) over rows of column-major 3x3 / dynamic matrices: halving redux
        for (int j = 0; j < 3; j++) alphas[4 * i + j + 1] = ered3(CC_inv[j][0] * d0, CC_inv[j][1] * d1, CC_inv[j][2] * d2);
        alphas[4 * i + 0] = 1.0 - alphas[4 * i + 1] - alphas[4 * i + 2] - alphas[4 * i + 3];
    }
}

// PnPsolver.cpp:345-352 (ccs.setZero() then +=, so the sum starts from 0.0)
void PnPOracle::compute_ccs(const double betas[4], const double (*U)[12]) {
    for (int i = 0; i < 4; i++)
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int j = 0; j < 4; j++) s = s + betas[j] * U[3 * i + c][j];
            ccs[i][c] = s;
        }
}

// PnPsolver.cpp:354-357 — over ALL allocated rows (Q6).
void PnPOracle::compute_pcs() {
    const int rows = maximum_number_of_correspondences;
    for (int i = 0; i < rows; ++i)
        for (int c = 0; c < 3; ++c)
            pcs[3 * i + c] = alphas[4 * i + 0] * ccs[0][c] + alphas[4 * i + 1] * ccs[1][c] +
                             alphas[4 * i + 2] * ccs[2][c] + alphas[4 * i + 3] * ccs[3][c];
}

// PnPsolver.cpp:359-415
double PnPOracle::compute_pose(float R[3][3], float t[3]) {
    choose_control_points();
    compute_barycentric_coordinates();
    const int n = number_of_correspondences;
    // MtM = M^T M with M (2n x 12) as built at :365-377.
    std::vector<double> M(2 * n * 12);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 4; j++) {
            const double a = alphas[4 * i + j];
            double* r0 = &M[(2 * i) * 12];
            double* r1 = &M[(2 * i + 1) * 12];
            r0[3 * j] = a * fx;
            r0[3 * j + 1] = 0.0;
            r0[3 * j + 2] = a * (cx - us[2 * i + 0]);
            r1[3 * j] = 0.0;
            r1[3 * j + 1] = a * fy;
            r1[3 * j + 2] = a * (cy - us[2 * i + 1]);
        }
    double MtM[12][12];
    for (int a = 0; a < 12; ++a)
        for (int b = 0; b < 12; ++b) {
            double s = M[a] * M[b];
            for (int r = 1; r < 2 * n; ++r) s = s + M[r * 12 + a] * M[r * 12 + b];
            MtM[a][b] = s;
        }
    SymEig<double, 12> es = sym_eig<double, 12>(MtM);
    const double (*U)[12] = es.V;

    double L_6x10[6][10], rho[6];
    compute_L_6x10(U, L_6x10);
    compute_rho(rho);

    double Betas[4][4] = {};
    double rep_errors[4];
    double Rs[4][3][3], ts[4][3];

    find_betas_approx_1(L_6x10, rho, Betas[1]);
    gauss_newton(L_6x10, rho, Betas[1]);
    rep_errors[1] = compute_R_and_t(U, Betas[1], Rs[1], ts[1]);

    find_betas_approx_2(L_6x10, rho, Betas[2]);
    gauss_newton(L_6x10, rho, Betas[2]);
    rep_errors[2] = compute_R_and_t(U, Betas[2], Rs[2], ts[2]);

    find_betas_approx_3(L_6x10, rho, Betas[3]);
    gauss_newton(L_6x10, rho, Betas[3]);
    rep_errors[3] = compute_R_and_t(U, Betas[3], Rs[3], ts[3]);

    int Nb = 1;
    if (rep_errors[2] < rep_errors[1]) Nb = 2;
    if (rep_errors[3] < rep_errors[Nb]) Nb = 3;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) R[r][c] = (float)Rs[Nb][r][c];
        t[r] = (float)ts[Nb][r];
    }
    return rep_errors[Nb];
}

// PnPsolver.cpp:417-431
double PnPOracle::reprojection_error(const double R[3][3], const double t[3]) {
    double sum2 = 0.0;
    for (int i = 0; i < number_of_correspondences; i++) {
        const double* P = &pws[3 * i];
        // :423 Matrix3d * Vector3d + t into a Vector3d (emv3d_row)
        double X = emv3d_row(0, R[0][0] * P[0], R[0][1] * P[1], R[0][2] * P[2]) + t[0];
        double Y = emv3d_row(1, R[1][0] * P[0], R[1][1] * P[1], R[1][2] * P[2]) + t[1];
        double Z = emv3d_row(2, R[2][0] * P[0], R[2][1] * P[1], R[2][2] * P[2]) + t[2];
        double inv_Zc = 1.0 / Z;
        double u = cx + fx * X * inv_Zc;
        double v = cy + fy * Y * inv_Zc;
        double du = us[2 * i + 0] - u, dv = us[2 * i + 1] - v;
        sum2 += std::sqrt(du * du + dv * dv);
    }
    return sum2 / number_of_correspondences;
}

// PnPsolver.cpp:433-493 — Horn quaternion with the N entries truncated to float (Q5); the
// quaternion is conjugated (:473-476).
void PnPOracle::estimate_R_and_t(double R[3][3], double t[3]) {
    const int n = number_of_correspondences, rows = maximum_number_of_correspondences;
    double pc0[3], pw0[3];
    for (int c = 0; c < 3; ++c) {
        double s = pcs[c];
        for (int i = 1; i < rows; ++i) s = s + pcs[3 * i + c];
        pc0[c] = s;
        double w = pws[c];
        for (int i = 1; i < rows; ++i) w = w + pws[3 * i + c];
        pw0[c] = w;
    }
    for (int c = 0; c < 3; ++c) { pc0[c] = pc0[c] / n; pw0[c] = pw0[c] / n; }
    double M[3][3] = {};
    for (int i = 0; i < n; i++) {
        double a[3], b[3];
        for (int c = 0; c < 3; ++c) { a[c] = pcs[3 * i + c] - pc0[c]; b[c] = pws[3 * i + c] - pw0[c]; }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) M[r][c] = M[r][c] + a[r] * b[c];
    }
    float N11, N12, N13, N14, N22, N23, N24, N33, N34, N44;
    N11 = (float)(M[0][0] + M[1][1] + M[2][2]);
    N12 = (float)(M[1][2] - M[2][1]);
    N13 = (float)(M[2][0] - M[0][2]);
    N14 = (float)(M[0][1] - M[1][0]);
    N22 = (float)(M[0][0] - M[1][1] - M[2][2]);
    N23 = (float)(M[0][1] + M[1][0]);
    N24 = (float)(M[2][0] + M[0][2]);
    N33 = (float)(-M[0][0] + M[1][1] - M[2][2]);
    N34 = (float)(M[1][2] + M[2][1]);
    N44 = (float)(-M[0][0] - M[1][1] + M[2][2]);
    double Nm[4][4] = {{N11, N12, N13, N14}, {N12, N22, N23, N24}, {N13, N23, N33, N34}, {N14, N24, N34, N44}};
    SymEig<double, 4> es = sym_eig<double, 4>(Nm);
    double qw = es.V[0][3], qx = -es.V[1][3], qy = -es.V[2][3], qz = -es.V[3][3];
    quat_to_R(qw, qx, qy, qz, R);
    if (det3(R) < 0)
        for (int c = 0; c < 3; ++c) R[2][c] = -R[2][c];
    // :492 pc0 - Matrix3d * pw0 into a Vector3d (emv3d_row)
    for (int r = 0; r < 3; ++r) t[r] = pc0[r] - emv3d_row(r, R[r][0] * pw0[0], R[r][1] * pw0[1], R[r][2] * pw0[2]);
}

// PnPsolver.cpp:495-502 — negates ALL allocated rows of pcs.
void PnPOracle::solve_for_sign() {
    if (pcs[2] < 0.0) {
        for (int i = 0; i < 4; ++i) for (int c = 0; c < 3; ++c) ccs[i][c] = -ccs[i][c];
        for (size_t i = 0; i < 3 * (size_t)maximum_number_of_correspondences; ++i) pcs[i] = -pcs[i];
    }
}

// PnPsolver.cpp:504-515
double PnPOracle::compute_R_and_t(const double (*U)[12], const double betas[4], double R[3][3], double t[3]) {
    compute_ccs(betas, U);
    compute_pcs();
    solve_for_sign();
    estimate_R_and_t(R, t);
    return reprojection_error(R, t);
}

// PnPsolver.cpp:520-544
void PnPOracle::find_betas_approx_1(const double L[6][10], const double rho[6], double betas[4]) {
    double A[6][4];
    for (int r = 0; r < 6; ++r) { A[r][0] = L[r][0]; A[r][1] = L[r][1]; A[r][2] = L[r][3]; A[r][3] = L[r][6]; }
    double b4[4];
    jacobi_svd_solve_6xk<4>(A, rho, b4);
    if (b4[0] < 0) {
        betas[0] = std::sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0];
        betas[2] = -b4[2] / betas[0];
        betas[3] = -b4[3] / betas[0];
    } else {
        betas[0] = std::sqrt(b4[0]);
        betas[1] = b4[1] / betas[0];
        betas[2] = b4[2] / betas[0];
        betas[3] = b4[3] / betas[0];
    }
}

// PnPsolver.cpp:549-573
void PnPOracle::find_betas_approx_2(const double L[6][10], const double rho[6], double betas[4]) {
    double A[6][3];
    for (int r = 0; r < 6; ++r) { A[r][0] = L[r][0]; A[r][1] = L[r][1]; A[r][2] = L[r][2]; }
    double b3[3];
    jacobi_svd_solve_6xk<3>(A, rho, b3);
    if (b3[0] < 0) {
        betas[0] = std::sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? std::sqrt(-b3[2]) : 0.0;
    } else {
        betas[0] = std::sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? std::sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
}

// PnPsolver.cpp:578-602
void PnPOracle::find_betas_approx_3(const double L[6][10], const double rho[6], double betas[4]) {
    double A[6][5];
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 5; ++c) A[r][c] = L[r][c];
    double b5[5];
    jacobi_svd_solve_6xk<5>(A, rho, b5);
    if (b5[0] < 0) {
        betas[0] = std::sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? std::sqrt(-b5[2]) : 0.0;
    } else {
        betas[0] = std::sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? std::sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
}

// PnPsolver.cpp:604-637
void PnPOracle::compute_L_6x10(const double (*U)[12], double l[6][10]) {
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
        int a = 0, b = 1;
        for (int j = 0; j < 6; j++) {
            for (int c = 0; c < 3; ++c) dv[i][j][c] = U[3 * a + c][i] - U[3 * b + c][i];
            b++;
            if (b > 3) { a++; b = a + 1; }
        }
    }
    // rows of column-major Matrix<double,6,3>: halving redux (ered3)
    auto dot = [](const double* x, const double* y) { return ered3(x[0] * y[0], x[1] * y[1], x[2] * y[2]); };
    for (int i = 0; i < 6; i++) {
        l[i][0] = dot(dv[0][i], dv[0][i]);
        l[i][1] = 2.0 * dot(dv[0][i], dv[1][i]);
        l[i][2] = dot(dv[1][i], dv[1][i]);
        l[i][3] = 2.0 * dot(dv[0][i], dv[2][i]);
        l[i][4] = 2.0 * dot(dv[1][i], dv[2][i]);
        l[i][5] = dot(dv[2][i], dv[2][i]);
        l[i][6] = 2.0 * dot(dv[0][i], dv[3][i]);
        l[i][7] = 2.0 * dot(dv[1][i], dv[3][i]);
        l[i][8] = 2.0 * dot(dv[2][i], dv[3][i]);
        l[i][9] = dot(dv[3][i], dv[3][i]);
    }
}

// PnPsolver.cpp:639-647
void PnPOracle::compute_rho(double rho[6]) {
    auto d2 = [&](int a, int b) {
        double x = cws[a][0] - cws[b][0], y = cws[a][1] - cws[b][1], z = cws[a][2] - cws[b][2];
        return ered3(x * x, y * y, z * z);  // squaredNorm of a row of Matrix<double,4,3>
    };
    rho[0] = d2(0, 1); rho[1] = d2(0, 2); rho[2] = d2(0, 3);
    rho[3] = d2(1, 2); rho[4] = d2(1, 3); rho[5] = d2(2, 3);
}

// PnPsolver.cpp:649-673
void PnPOracle::compute_A_and_b_gauss_newton(const double l[6][10], const double rho[6], const double b[4],
                                             double A[6][4], double B[6]) {
    for (int i = 0; i < 6; i++) {
        const double Lt[4][4] = {{2 * l[i][0], l[i][1], l[i][3], l[i][6]},
                                 {l[i][1], 2 * l[i][2], l[i][4], l[i][7]},
                                 {l[i][3], l[i][4], 2 * l[i][5], l[i][8]},
                                 {l[i][6], l[i][7], l[i][8], 2 * l[i][9]}};
        for (int r = 0; r < 4; ++r) A[i][r] = Lt[r][0] * b[0] + Lt[r][1] * b[1] + Lt[r][2] * b[2] + Lt[r][3] * b[3];
        B[i] = rho[i] - (l[i][0] * b[0] * b[0] + l[i][1] * b[0] * b[1] + l[i][2] * b[1] * b[1] +
                         l[i][3] * b[0] * b[2] + l[i][4] * b[1] * b[2] + l[i][5] * b[2] * b[2] +
                         l[i][6] * b[0] * b[3] + l[i][7] * b[1] * b[3] + l[i][8] * b[2] * b[3] +
                         l[i][9] * b[3] * b[3]);
    }
}

// PnPsolver.cpp:675-691 — X persists across iterations; when qr_solve bails on a singular A (Q9)
// the reference leaves X uninitialised/stale; the restatement keeps the previous X (0 at first).
void PnPOracle::gauss_newton(const double L[6][10], const double rho[6], double betas[4]) {
    double A[6][4], B[6];
    double* X = qr_X;
    X[0] = X[1] = X[2] = X[3] = 0.0;
    for (int k = 0; k < 5; k++) {
        compute_A_and_b_gauss_newton(L, rho, betas, A, B);
        qr_solve(A, B, X);
        for (int c = 0; c < 4; ++c) betas[c] = betas[c] + X[c];
    }
}

// PnPsolver.cpp:693-796 — Householder QR solve of the 6x4 system, verbatim structure.
#ifdef ORA_QR_STATS
// tools/q19_stats.py: how often the last row is a column's strict maximum (the scans where Q19's eta
// differs from a six-row eta).  Only in the instrumented build (-DORA_QR_STATS).
static long g_qr_calls = 0, g_qr_row5[4] = {0, 0, 0, 0}, g_qr_singular = 0;
extern "C" void ora_qr_stats(long* o) {
    o[0] = g_qr_calls;
    for (int k = 0; k < 4; ++k) o[1 + k] = g_qr_row5[k];
    o[5] = g_qr_singular;
}
#endif
bool PnPOracle::qr_solve(double A[6][4], double b[6], double X[4]) {
    const int nr = 6, nc = 4;
#ifdef ORA_QR_STATS
    ++g_qr_calls;
#endif
    double A1[4], A2[4];
    for (int k = 0; k < nc; k++) {
        // :714-720 — `elt = fabs(*ppAik)` is read BEFORE `ppAik += nc`, so iteration i reads row
        // i-1: eta = max |A[k..nr-2][k]| (row k twice, the last row never) (Q19).
#ifdef ORA_QR_STATS
        {
            double m = 0.0;
            for (int i = k; i < nr - 1; ++i) m = std::max(m, ab(A[i][k]));
            if (ab(A[nr - 1][k]) > m) ++g_qr_row5[k];
        }
#endif
        double eta = ab(A[k][k]);
        for (int i = k + 1; i < nr; i++) {
            double elt = ab(A[i - 1][k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
#ifdef ORA_QR_STATS
            ++g_qr_singular;
#endif
            return false;  // "A is singular" (:722-726)
        }
        double sum = 0.0, inv_eta = 1. / eta;
        for (int i = k; i < nr; i++) {
            A[i][k] *= inv_eta;
            sum += A[i][k] * A[i][k];
        }
        double sigma = std::sqrt(sum);
        if (A[k][k] < 0) sigma = -sigma;
        A[k][k] += sigma;
        A1[k] = sigma * A[k][k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double s = 0;
            for (int i = k; i < nr; i++) s += A[i][k] * A[i][j];
            double tau = s / A1[k];
            for (int i = k; i < nr; i++) A[i][j] -= tau * A[i][k];
        }
    }
    for (int j = 0; j < nc; j++) {
        double tau = 0;
        for (int i = j; i < nr; i++) tau += A[i][j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; i++) b[i] -= tau * A[i][j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double s = 0;
        for (int j = i + 1; j < nc; j++) s += A[i][j] * X[j];
        X[i] = (b[i] - s) / A2[i];
    }
    return true;
}

// ---- test hooks ----
double PnPOracle::compute_pose_public(const int* idx, int n, float R[9], float t[3]) {
    set_maximum_number_of_correspondences(n);
    reset_correspondences();
    for (int i = 0; i < n; ++i) add_correspondence(&mvP3Dw[3 * idx[i]], &mvP2D[2 * idx[i]]);
    float Rm[3][3], tm[3];
    double e = compute_pose(Rm, tm);
    for (int r = 0; r < 3; ++r) { t[r] = tm[r]; for (int c = 0; c < 3; ++c) R[3 * r + c] = Rm[r][c]; }
    return e;
}

void PnPOracle::check_inliers_public(const float R[9], const float t[3], std::vector<uint8_t>& inl, int& count) {
    for (int r = 0; r < 3; ++r) { mti[r] = t[r]; for (int c = 0; c < 3; ++c) mRi[r][c] = R[3 * r + c]; }
    if ((int)mvbInliersi.size() != N) mvbInliersi.assign(N, 0);
    CheckInliers();
    inl = mvbInliersi;
    count = mnInliersi;
}

}  // namespace rsc_oracle
