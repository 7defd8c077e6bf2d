// rsc_sim3.h — per-lane Horn closed form of Sim3Solver (scale fixed to 1) and its two-way
// reprojection inlier test (reference: src/Sim3Solver.cpp:186-293, :306-327).  All float.
#pragma once
#include "rsc_core.h"

namespace rsc {

struct Sim3Pose {
    float R12[9], t12[3];  // T12 (row-major R)
    float R21[9], t21[3];  // T21 = T12.inverse() (Isometry: R^T, -(R^T t))
};

// ComputeCentroid + ComputeSim3 (Sim3Solver.cpp:186-266).  P1/P2: columns = the 3 sampled points
// (P[r][i] = coordinate r of point i), as P3Dc1i / P3Dc2i.
RSC_HD void sim3_compute(const float (&P1)[3][3], const float (&P2)[3][3], Sim3Pose& T) {
    float O1[3], O2[3], Pr1[3][3], Pr2[3][3];
    RSC_UNROLL for (int r = 0; r < 3; ++r) {
        O1[r] = ered3(P1[r][0], P1[r][1], P1[r][2]);  // P.rowwise().sum() (:188)
        O2[r] = ered3(P2[r][0], P2[r][1], P2[r][2]);
    }
    RSC_UNROLL for (int r = 0; r < 3; ++r) { O1[r] = O1[r] / 3.f; O2[r] = O2[r] / 3.f; }
    RSC_UNROLL for (int i = 0; i < 3; ++i)
        RSC_UNROLL for (int r = 0; r < 3; ++r) { Pr1[r][i] = P1[r][i] - O1[r]; Pr2[r][i] = P2[r][i] - O2[r]; }
    float M[3][3];
    RSC_UNROLL for (int a = 0; a < 3; ++a)
        RSC_UNROLL for (int b = 0; b < 3; ++b) M[a][b] = ered3(Pr2[a][0] * Pr1[b][0], Pr2[a][1] * Pr1[b][1], Pr2[a][2] * Pr1[b][2]);
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
    const float Nm[4][4] = {{N11, N12, N13, N14}, {N12, N22, N23, N24}, {N13, N23, N33, N34}, {N14, N24, N34, N44}};
    float V[4][4], w[4];
    sym_eig_reg<float, 4>(Nm, V, w);
    float R[3][3];
    quat_to_R<float>(V[0][3], V[1][3], V[2][3], V[3][3], R);  // not conjugated (:243-246)
    RSC_UNROLL for (int r = 0; r < 3; ++r) {
        T.t12[r] = O1[r] - ered3(R[r][0] * O2[0], R[r][1] * O2[1], R[r][2] * O2[2]);
        RSC_UNROLL for (int c = 0; c < 3; ++c) { T.R12[3 * r + c] = R[r][c]; T.R21[3 * c + r] = R[r][c]; }
    }
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        T.t21[r] = -ered3(T.R21[3 * r + 0] * T.t12[0], T.R21[3 * r + 1] * T.t12[1], T.R21[3 * r + 2] * T.t12[2]);
}

// Sim3Solver::Project of one point (Rcw = Tcw.rotation() taken as linear(), Q14).
RSC_HD void sim3_project(const float (&R)[9], const float (&t)[3], float fx, float fy, float cx, float cy,
                         float X, float Y, float Z, float& u, float& v) {
    float x3 = ered3(R[0] * X, R[1] * Y, R[2] * Z) + t[0];  // Rcw*P3Dw + tcw (:320)
    float y3 = ered3(R[3] * X, R[4] * Y, R[5] * Z) + t[1];
    float z3 = ered3(R[6] * X, R[7] * Y, R[8] * Z) + t[2];
    const float invz = 1.0f / z3;
    const float x = x3 * invz;
    const float y = y3 * invz;
    u = fx * x + cx;
    v = fy * y + cy;
}

// Sim3Solver::CheckInliers for one correspondence (Sim3Solver.cpp:277-292); e1/e2 are the size_t
// thresholds already converted to float (the comparison float < size_t converts the size_t).
RSC_HD bool sim3_inlier(const Sim3Pose& T, const float (&K1)[4], const float (&K2)[4],
                        const float (&X1)[3], const float (&X2)[3], float p1u, float p1v, float p2u, float p2v,
                        float e1, float e2) {
    float u21, v21, u12, v12;
    sim3_project(T.R12, T.t12, K1[0], K1[1], K1[2], K1[3], X2[0], X2[1], X2[2], u21, v21);  // vP2im1
    sim3_project(T.R21, T.t21, K2[0], K2[1], K2[2], K2[3], X1[0], X1[1], X1[2], u12, v12);  // vP1im2
    float d1x = p1u - u21, d1y = p1v - v21;
    float d2x = u12 - p2u, d2y = v12 - p2v;
    const float err1 = d1x * d1x + d1y * d1y;
    const float err2 = d2x * d2x + d2y * d2y;
    return err1 < e1 && err2 < e2;
}

}  // namespace rsc
