// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
// Restatement of src/Sim3Solver.cpp (reference) — see sim3_oracle.h.  Line numbers cite the reference.
#include "sim3_oracle.h"
#include "ora_linalg.h"
#include <cmath>
#include <algorithm>

namespace rsc_oracle {

// X3Dc = Rcw * Xw + tcw (:58, :62; Matrix3f * Vector3f: coefficient-path reductions, ered3)
static inline void xform(const float R[9], const float t[3], const float* X, float* out) {
    for (int r = 0; r < 3; ++r) out[r] = ered3(R[3 * r + 0] * X[0], R[3 * r + 1] * X[1], R[3 * r + 2] * X[2]) + t[r];
}

// Sim3Solver.cpp:6-85
Sim3Oracle::Sim3Oracle(const Sim3Input& in, uint32_t seed) : rng(seed) {
    mN1 = in.n1;
    int idx = 0;
    for (int i1 = 0; i1 < mN1; i1++) {
        if (!in.valid[i1]) continue;
        const float sigmaSquare1 = in.sigma2_1[i1];
        const float sigmaSquare2 = in.sigma2_2[i1];
        mvnMaxError1.push_back((uint64_t)(9.210 * sigmaSquare1));  // stored as size_t (Q11)
        mvnMaxError2.push_back((uint64_t)(9.210 * sigmaSquare2));
        mvnIndices1.push_back(i1);
        float c1[3], c2[3];
        xform(in.R1, in.t1, &in.Xw1[3 * i1], c1);
        xform(in.R2, in.t2, &in.Xw2[3 * i1], c2);
        mvX3Dc1.insert(mvX3Dc1.end(), c1, c1 + 3);
        mvX3Dc2.insert(mvX3Dc2.end(), c2, c2 + 3);
        mvAllIndices.push_back(idx);
        idx++;
    }
    N = idx;
    for (int r = 0; r < 3; ++r) {
        mt12i[r] = 0.f; mt21i[r] = 0.f; mBestTranslation[r] = 0.f;
        for (int c = 0; c < 3; ++c) {
            mR12i[r][c] = (r == c) ? 1.f : 0.f;
            mR21i[r][c] = mR12i[r][c];
            mBestRotation[r][c] = mR12i[r][c];
        }
    }
    for (int k = 0; k < 4; ++k) { mK1[k] = in.K1[k]; mK2[k] = in.K2[k]; }
    // FromCameraToImage (:329-347)
    auto to_image = [](const std::vector<float>& X, std::vector<float>& P, const float K[4]) {
        const size_t n = X.size() / 3;
        P.resize(2 * n);
        for (size_t i = 0; i < n; ++i) {
            const float invz = 1 / X[3 * i + 2];
            const float x = X[3 * i + 0] * invz;
            const float y = X[3 * i + 1] * invz;
            P[2 * i + 0] = K[0] * x + K[2];
            P[2 * i + 1] = K[1] * y + K[3];
        }
    };
    to_image(mvX3Dc1, mvP1im1, mK1);
    to_image(mvX3Dc2, mvP2im2, mK2);
    SetRansacParameters();
}

// Sim3Solver.cpp:87-111
void Sim3Oracle::SetRansacParameters(double probability, int minInliers, int maxIterations) {
    mRansacProb = probability;
    mRansacMinInliers = minInliers;
    mRansacMaxIts = maxIterations;
    mvbInliersi.assign(N, 0);
    float epsilon = (float)mRansacMinInliers / N;
    int nIterations;
    if (mRansacMinInliers == N)
        nIterations = 1;
    else
        nIterations = (int)std::ceil(std::log(1 - mRansacProb) / std::log(1 - std::pow((double)epsilon, 3.0)));
    mRansacMaxIts = std::max(1, std::min(nIterations, mRansacMaxIts));
    mnIterations = 0;
}

// Sim3Solver.cpp:113-178
bool Sim3Oracle::iterate(int nIterations, bool& bNoMore, std::vector<uint8_t>& vbInliers, int& nInliers) {
    bNoMore = false;
    vbInliers.assign(mN1, 0);
    nInliers = 0;
    if (N < mRansacMinInliers) {
        bNoMore = true;
        return false;
    }
    float P3Dc1i[3][3], P3Dc2i[3][3];  // columns = points
    int nCurrentIterations = 0;
    while (mnIterations < mRansacMaxIts && nCurrentIterations < nIterations) {  // Q1: '&&'
        nCurrentIterations++;
        mnIterations++;
        std::vector<int32_t> vAvailableIndices = mvAllIndices;
        Sim3Trace tr{};
        for (short i = 0; i < 3; ++i) {
            int randi = rng.random_int(0, (int)vAvailableIndices.size() - 1);
            int idx = vAvailableIndices[randi];
            tr.sample[i] = idx;
            for (int r = 0; r < 3; ++r) {
                P3Dc1i[r][i] = mvX3Dc1[3 * idx + r];
                P3Dc2i[r][i] = mvX3Dc2[3 * idx + r];
            }
            vAvailableIndices[randi] = vAvailableIndices.back();
            vAvailableIndices.pop_back();
        }
        ComputeSim3(P3Dc1i, P3Dc2i);
        CheckInliers();
        tr.n_inliers = mnInliersi;
        for (int r = 0; r < 3; ++r) { tr.t[r] = mt12i[r]; for (int c = 0; c < 3; ++c) tr.R[3 * r + c] = mR12i[r][c]; }
        if (trace) trace->push_back(tr);
        if (mnInliersi >= mnBestInliers) {  // Q12: ties -> later wins
            mvbBestInliers = mvbInliersi;
            mnBestInliers = mnInliersi;
            for (int r = 0; r < 3; ++r) {
                mBestTranslation[r] = mt12i[r];
                for (int c = 0; c < 3; ++c) mBestRotation[r][c] = mR12i[r][c];
            }
            if (mnInliersi > mRansacMinInliers) {
                nInliers = mnInliersi;
                for (int i = 0; i < N; i++)
                    if (mvbInliersi[i]) vbInliers[mvnIndices1[i]] = 1;
                return true;
            }
        }
    }
    if (mnIterations >= mRansacMaxIts) bNoMore = true;
    return false;
}

// Sim3Solver.cpp:180-184
bool Sim3Oracle::find(std::vector<uint8_t>& vbInliers12, int& nInliers) {
    bool bFlag;
    return iterate(mRansacMaxIts, bFlag, vbInliers12, nInliers);
}

// Sim3Solver.cpp:186-266 (ComputeCentroid + ComputeSim3), all float.
void Sim3Oracle::ComputeSim3(const float P1[3][3], const float P2[3][3]) {
    float O1[3], O2[3], Pr1[3][3], Pr2[3][3];
    for (int r = 0; r < 3; ++r) {
        O1[r] = ered3(P1[r][0], P1[r][1], P1[r][2]);  // P.rowwise().sum() (:188)
        O2[r] = ered3(P2[r][0], P2[r][1], P2[r][2]);
    }
    for (int r = 0; r < 3; ++r) { O1[r] = O1[r] / 3.f; O2[r] = O2[r] / 3.f; }
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) { Pr1[r][i] = P1[r][i] - O1[r]; Pr2[r][i] = P2[r][i] - O2[r]; }
    // M = Pr2 * Pr1^T
    float M[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) M[a][b] = ered3(Pr2[a][0] * Pr1[b][0], Pr2[a][1] * Pr1[b][1], Pr2[a][2] * Pr1[b][2]);
    float N11 = M[0][0] + M[1][1] + M[2][2];
    float N12 = M[1][2] - M[2][1];
    float N13 = M[2][0] - M[0][2];
    float N14 = M[0][1] - M[1][0];
    float N22 = M[0][0] - M[1][1] - M[2][2];
    float N23 = M[0][1] + M[1][0];
    float N24 = M[2][0] + M[0][2];
    float N33 = -M[0][0] + M[1][1] - M[2][2];
    float N34 = M[1][2] + M[2][1];
    float N44 = -M[0][0] - M[1][1] + M[2][2];
    float Nm[4][4] = {{N11, N12, N13, N14}, {N12, N22, N23, N24}, {N13, N23, N33, N34}, {N14, N24, N34, N44}};
    SymEig<float, 4> es = sym_eig<float, 4>(Nm);
    // q = (w,x,y,z) = eigenvector of the largest eigenvalue, NOT conjugated (:243-246)
    quat_to_R(es.V[0][3], es.V[1][3], es.V[2][3], es.V[3][3], mR12i);
    // scale fixed to 1 (:250); t12 = O1 - R12*O2 (:253)
    for (int r = 0; r < 3; ++r) mt12i[r] = O1[r] - ered3(mR12i[r][0] * O2[0], mR12i[r][1] * O2[1], mR12i[r][2] * O2[2]);
    // T21 = T12.inverse() for an Isometry: R^T, -(R^T t)
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) mR21i[r][c] = mR12i[c][r];
    for (int r = 0; r < 3; ++r) mt21i[r] = -ered3(mR21i[r][0] * mt12i[0], mR21i[r][1] * mt12i[1], mR21i[r][2] * mt12i[2]);
}

// Sim3Solver.cpp:306-327 (rotation() taken as linear(), Q14)
void Sim3Oracle::Project(const std::vector<float>& X, std::vector<float>& P2D, const float R[3][3], const float t[3],
                         const float K[4]) {
    const size_t n = X.size() / 3;
    P2D.resize(2 * n);
    for (size_t i = 0; i < n; ++i) {
        const float* p = &X[3 * i];
        float x3 = ered3(R[0][0] * p[0], R[0][1] * p[1], R[0][2] * p[2]) + t[0];  // :320
        float y3 = ered3(R[1][0] * p[0], R[1][1] * p[1], R[1][2] * p[2]) + t[1];
        float z3 = ered3(R[2][0] * p[0], R[2][1] * p[1], R[2][2] * p[2]) + t[2];
        const float invz = 1 / z3;
        const float x = x3 * invz;
        const float y = y3 * invz;
        P2D[2 * i + 0] = K[0] * x + K[2];
        P2D[2 * i + 1] = K[1] * y + K[3];
    }
}

// Sim3Solver.cpp:269-293
void Sim3Oracle::CheckInliers() {
    std::vector<float> vP1im2, vP2im1;
    Project(mvX3Dc2, vP2im1, mR12i, mt12i, mK1);
    Project(mvX3Dc1, vP1im2, mR21i, mt21i, mK2);
    mnInliersi = 0;
    for (int i = 0; i < N; i++) {
        float d1x = mvP1im1[2 * i] - vP2im1[2 * i], d1y = mvP1im1[2 * i + 1] - vP2im1[2 * i + 1];
        float d2x = vP1im2[2 * i] - mvP2im2[2 * i], d2y = vP1im2[2 * i + 1] - mvP2im2[2 * i + 1];
        const float err1 = d1x * d1x + d1y * d1y;
        const float err2 = d2x * d2x + d2y * d2y;
        if (err1 < (float)mvnMaxError1[i] && err2 < (float)mvnMaxError2[i]) {
            mvbInliersi[i] = 1;
            mnInliersi++;
        } else {
            mvbInliersi[i] = 0;
        }
    }
}

void Sim3Oracle::GetEstimatedRotation(float R[9]) const {
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R[3 * r + c] = mBestRotation[r][c];
}
void Sim3Oracle::GetEstimatedTranslation(float t[3]) const {
    for (int r = 0; r < 3; ++r) t[r] = mBestTranslation[r];
}

void Sim3Oracle::compute_sim3_public(const int idx[3], float R[9], float t[3]) {
    float P1[3][3], P2[3][3];
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) { P1[r][i] = mvX3Dc1[3 * idx[i] + r]; P2[r][i] = mvX3Dc2[3 * idx[i] + r]; }
    ComputeSim3(P1, P2);
    for (int r = 0; r < 3; ++r) { t[r] = mt12i[r]; for (int c = 0; c < 3; ++c) R[3 * r + c] = mR12i[r][c]; }
}

int Sim3Oracle::check_inliers_public(const float R[9], const float t[3], std::vector<uint8_t>& inl) {
    for (int r = 0; r < 3; ++r) { mt12i[r] = t[r]; for (int c = 0; c < 3; ++c) mR12i[r][c] = R[3 * r + c]; }
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) mR21i[r][c] = mR12i[c][r];
    for (int r = 0; r < 3; ++r) mt21i[r] = -ered3(mR21i[r][0] * mt12i[0], mR21i[r][1] * mt12i[1], mR21i[r][2] * mt12i[2]);
    CheckInliers();
    inl = mvbInliersi;
    return mnInliersi;
}

}  // namespace rsc_oracle
