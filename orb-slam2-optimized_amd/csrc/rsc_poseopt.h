// rsc_poseopt.h — Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) on the GPU: the g2o
// Levenberg-Marquardt of one VertexSE3Expmap over EdgeSE3ProjectXYZOnlyPose (mono) and
// EdgeStereoSE3ProjectXYZOnlyPose (stereo) edges with Huber kernels (delta sqrt(5.991) / sqrt(7.815)),
// 4 rounds of 10 iterations with inlier/outlier re-classification (chi2 > 5.991 / 7.815).
//
// Mapping: one 256-thread workgroup per Frame (problem).  A pass (computeActiveErrors +
// activeRobustChi2 + buildSystem at one estimate) walks the round's active edges in slabs of 192:
// waves 1..3 evaluate one edge per lane (error, robust chi2 term, Jacobian and its 27 Hessian /
// gradient terms) into an LDS slab buffer while wave 0 folds the previous slab, one lane per
// accumulator, so every sum g2o performs as a sequential loop over the active edges has the
// reference's evaluation order.  The LM control (6x6 LDLT, exp map, lambda schedule, stop rules) is
// tiny and runs redundantly in every lane from the folded values in LDS, so no further broadcast is
// needed.
//
// g2o source followed (Thirdparty/g2o/g2o): optimization_algorithm_levenberg.cpp:59-172,
// sparse_optimizer.cpp:61-114,354-414, block_solver.hpp:502-604, solvers/linear_solver_dense.h,
// base_unary_edge.hpp:43-71, robust_kernel_impl.cpp:65-91, types/types_six_dof_expmap.{h,cpp}
// (EdgeSE3ProjectXYZOnlyPose, VertexSE3Expmap::oplusImpl), types/se3quat.h.  Eigen arithmetic is
// restated with every sum left to right; the oracle (oracle/poseopt_oracle.cpp) is
// an independent sequential restatement and the two agree bit for bit.
#pragma once
#include "rsc_core.h"
#include "rsc_math.h"

namespace rsc {

constexpr int kPoseMaxEdges = 8192;  // LDS level flags per problem
constexpr int kPoseTerms = 27;       // 21 lower-triangle H entries + 6 b entries

#if defined(__HIPCC__)
struct DevPoseProb {
    const float4* xw;    // [n] Xw (x, y, z), w = invSigma2 (information = I * invSigma2)
    const float2* uv;    // [n] observation mvKeysUn[i].pt
    const float* ur;     // [n] mvuRight (>= 0: stereo edge), or nullptr: every edge monocular
    uint8_t* outlier;    // [n] out: mvbOutlier of each edge
    float* out;          // out: [0..11] Tcw rows 0..2 (float), [12] nGood (as float bits of int), [13..15] stats
    int n;               // edges (slots with a map point), >= 3
    float fx, fy, cx, cy, bf;
    float T[12];         // initial pFrame->mTcw rows 0..2
};
#endif

// ---- g2o::SE3Quat / Eigen::Quaterniond ------------------------------------------------------------
struct PoQuat {
    double x, y, z, w;
};
struct PoSE3 {
    PoQuat r;
    double t[3];
};

RSC_HD PoQuat po_quat_from_R(const double (&m)[3][3]) {
    PoQuat q;
    const double tr = m[0][0] + m[1][1] + m[2][2];
    if (tr > 0.0) {
        double t = sqrt(tr + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
        return q;
    }
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > (i == 1 ? m[1][1] : m[0][0])) i = 2;
    // static-index form of Eigen's (i, j, k) cyclic branch
    double c[3];
    double w;
    if (i == 0) {
        double t = sqrt(m[0][0] - m[1][1] - m[2][2] + 1.0);
        c[0] = 0.5 * t;
        t = 0.5 / t;
        w = (m[2][1] - m[1][2]) * t;
        c[1] = (m[1][0] + m[0][1]) * t;
        c[2] = (m[2][0] + m[0][2]) * t;
    } else if (i == 1) {
        double t = sqrt(m[1][1] - m[2][2] - m[0][0] + 1.0);
        c[1] = 0.5 * t;
        t = 0.5 / t;
        w = (m[0][2] - m[2][0]) * t;
        c[2] = (m[2][1] + m[1][2]) * t;
        c[0] = (m[0][1] + m[1][0]) * t;
    } else {
        double t = sqrt(m[2][2] - m[0][0] - m[1][1] + 1.0);
        c[2] = 0.5 * t;
        t = 0.5 / t;
        w = (m[1][0] - m[0][1]) * t;
        c[0] = (m[0][2] + m[2][0]) * t;
        c[1] = (m[1][2] + m[2][1]) * t;
    }
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
    q.w = w;
    return q;
}

RSC_HD void po_quat_to_R(const PoQuat& q, double (&R)[3][3]) { quat_to_R<double>(q.w, q.x, q.y, q.z, R); }

RSC_HD PoQuat po_quat_mul(const PoQuat& a, const PoQuat& b) {
    PoQuat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

// Quaternion * Vector3 (_transformVector): uv = 2 (q.vec x v); v + w uv + q.vec x uv.
RSC_HD void po_rotate(const PoQuat& q, const double (&v)[3], double (&o)[3]) {
    double uv0 = q.y * v[2] - q.z * v[1];
    double uv1 = q.z * v[0] - q.x * v[2];
    double uv2 = q.x * v[1] - q.y * v[0];
    uv0 = uv0 + uv0;
    uv1 = uv1 + uv1;
    uv2 = uv2 + uv2;
    const double c0 = q.y * uv2 - q.z * uv1;
    const double c1 = q.z * uv0 - q.x * uv2;
    const double c2 = q.x * uv1 - q.y * uv0;
    o[0] = v[0] + q.w * uv0 + c0;
    o[1] = v[1] + q.w * uv1 + c1;
    o[2] = v[2] + q.w * uv2 + c2;
}

RSC_HD void po_normalize(PoQuat& q) {
    if (q.w < 0.0) {
        q.x *= -1.0; q.y *= -1.0; q.z *= -1.0; q.w *= -1.0;
    }
    const double z = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    if (z > 0.0) {
        const double s = sqrt(z);
        q.x /= s; q.y /= s; q.z /= s; q.w /= s;
    }
}

RSC_HD PoSE3 po_from_Rt(const double (&R)[3][3], const double (&t)[3]) {
    PoSE3 s;
    s.r = po_quat_from_R(R);
    RSC_UNROLL for (int i = 0; i < 3; ++i) s.t[i] = t[i];
    po_normalize(s.r);
    return s;
}

RSC_HD PoSE3 po_mul(const PoSE3& a, const PoSE3& b) {
    PoSE3 r = a;
    double rb[3];
    po_rotate(a.r, b.t, rb);
    RSC_UNROLL for (int i = 0; i < 3; ++i) r.t[i] = r.t[i] + rb[i];
    r.r = po_quat_mul(a.r, b.r);
    po_normalize(r.r);
    return r;
}

RSC_HD void po_map(const PoSE3& s, const double (&p)[3], double (&o)[3]) {
    double rp[3];
    po_rotate(s.r, p, rp);
    RSC_UNROLL for (int i = 0; i < 3; ++i) o[i] = rp[i] + s.t[i];
}

// pow(x, 3) as the correctly rounded cube (same formula as the oracle).
RSC_HD double po_cube(double x) {
    const double p = x * x;
    const double e1 = fma(x, x, -p);
    const double c = p * x;
    const double e2 = fma(p, x, -c);
    return c + (e2 + e1 * x);
}

// SE3Quat::exp(update), update = (omega, upsilon).
RSC_HD PoSE3 po_exp(const double (&u)[6]) {
    const double o0 = u[0], o1 = u[1], o2 = u[2];
    const double theta = sqrt(o0 * o0 + o1 * o1 + o2 * o2);
    const double Om[3][3] = {{0.0, -o2, o1}, {o2, 0.0, -o0}, {-o1, o0, 0.0}};
    double Om2[3][3];
    RSC_UNROLL for (int i = 0; i < 3; ++i)
        RSC_UNROLL for (int j = 0; j < 3; ++j) Om2[i][j] = Om[i][0] * Om[0][j] + Om[i][1] * Om[1][j] + Om[i][2] * Om[2][j];
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        RSC_UNROLL for (int i = 0; i < 3; ++i)
            RSC_UNROLL for (int j = 0; j < 3; ++j) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + Om[i][j]) + Om2[i][j];
                V[i][j] = R[i][j];
            }
    } else {
        const double st = dm::sin(theta), ct = dm::cos(theta);
        const double a = st / theta;
        const double b = (1.0 - ct) / (theta * theta);
        const double c = (theta - st) / po_cube(theta);
        RSC_UNROLL for (int i = 0; i < 3; ++i)
            RSC_UNROLL for (int j = 0; j < 3; ++j) {
                const double I = (i == j) ? 1.0 : 0.0;
                R[i][j] = (I + a * Om[i][j]) + b * Om2[i][j];
                V[i][j] = (I + b * Om[i][j]) + c * Om2[i][j];
            }
    }
    double t[3];
    RSC_UNROLL for (int i = 0; i < 3; ++i) t[i] = V[i][0] * u[3] + V[i][1] * u[4] + V[i][2] * u[5];
    return po_from_Rt(R, t);
}

// ---- edges ---------------------------------------------------------------------------------------
// EdgeSE3ProjectXYZOnlyPose (mono, 2-D error) and EdgeStereoSE3ProjectXYZOnlyPose (stereo, 3-D error
// (u, v, u_right)); a Frame slot is stereo iff mvuRight[i] >= 0 (Optimizer.cpp:252,290-323).  The
// stereo forms below reduce to the mono ones' exact operations when `stereo` is false.
struct PoCam {
    double fx, fy, cx, cy, bf;
};

// computeError: obs - cam_project(est.map(Xw)).  Mono: project2d = (x/z, y/z) in double.  Stereo
// (types_six_dof_expmap.cpp:299-306): `const float invz = 1.0f/z` — a double division rounded to
// float — then res0 = x*invz*fx + cx, res1 = y*invz*fy + cy, res2 = res0 - bf*invz.
RSC_HD void po_error(const PoSE3& est, const PoCam& K, const double (&Xw)[3], double u, double v, double ur,
                     bool stereo, double& e0, double& e1, double& e2) {
    double p[3];
    po_map(est, Xw, p);
    double r0, r1, r2 = 0.0;
    if (stereo) {
        const double invz = (double)(float)(1.0 / p[2]);
        r0 = p[0] * invz * K.fx + K.cx;
        r1 = p[1] * invz * K.fy + K.cy;
        r2 = r0 - K.bf * invz;
    } else {
        const double pr0 = p[0] / p[2], pr1 = p[1] / p[2];
        r0 = pr0 * K.fx + K.cx;
        r1 = pr1 * K.fy + K.cy;
    }
    e0 = u - r0;
    e1 = v - r1;
    e2 = stereo ? ur - r2 : 0.0;
}

// _error.dot(information() * _error), information = I * inv, Eigen sums left to right.
RSC_HD double po_chi2(double inv, bool stereo, double e0, double e1, double e2) {
    if (!stereo) {
        const double w0 = inv * e0 + 0.0 * e1;
        const double w1 = 0.0 * e0 + inv * e1;
        return e0 * w0 + e1 * w1;
    }
    const double w0 = (inv * e0 + 0.0 * e1) + 0.0 * e2;
    const double w1 = (0.0 * e0 + inv * e1) + 0.0 * e2;
    const double w2 = (0.0 * e0 + 0.0 * e1) + inv * e2;
    return (e0 * w0 + e1 * w1) + e2 * w2;
}

// RobustKernelHuber::robustify (rho[0], rho[1]; rho[2] is unused by g2o's robustInformation).
RSC_HD void po_huber(double e, double delta, double dsqr, double& rho0, double& rho1) {
    if (e <= dsqr) {
        rho0 = e;
        rho1 = 1.0;
    } else {
        const double sqrte = sqrt(e);
        rho0 = 2 * sqrte * delta - dsqr;
        rho1 = delta / sqrte;
    }
}

// Term of activeRobustChi2 for one edge (delta / dsqr of the edge's own kernel).
RSC_HD double po_chi_term(bool robust, bool stereo, double inv, double e0, double e1, double e2, double delta,
                          double dsqr) {
    const double c = po_chi2(inv, stereo, e0, e1, e2);
    if (!robust) return c;
    double r0, r1;
    po_huber(c, delta, dsqr, r0, r1);
    return r0;
}

// linearizeOplus + constructQuadraticForm terms of one edge: t[0..20] = lower triangle of
// J^T W J (row-major i >= j), t[21..26] = the gradient term subtracted from b.  Stereo adds the third
// Jacobian row (types_six_dof_expmap.cpp:359-364) and a third term to every row/column sum.
RSC_HD void po_quad_terms(const PoSE3& est, const PoCam& K, const double (&Xw)[3], double inv, double e0, double e1,
                          double e2, bool stereo, bool robust, double delta, double dsqr, double (&t)[kPoseTerms]) {
    double p[3];
    po_map(est, Xw, p);
    const double x = p[0], y = p[1];
    const double invz = 1.0 / p[2];
    const double invz_2 = invz * invz;
    double A[3][6];
    A[0][0] = x * y * invz_2 * K.fx;
    A[0][1] = -(1 + (x * x * invz_2)) * K.fx;
    A[0][2] = y * invz * K.fx;
    A[0][3] = -invz * K.fx;
    A[0][4] = 0;
    A[0][5] = x * invz_2 * K.fx;
    A[1][0] = (1 + y * y * invz_2) * K.fy;
    A[1][1] = -x * y * invz_2 * K.fy;
    A[1][2] = -x * invz * K.fy;
    A[1][3] = 0;
    A[1][4] = -invz * K.fy;
    A[1][5] = y * invz_2 * K.fy;
    A[2][0] = A[0][0] - K.bf * y * invz_2;
    A[2][1] = A[0][1] + K.bf * x * invz_2;
    A[2][2] = A[0][2];
    A[2][3] = A[0][3];
    A[2][4] = 0;
    A[2][5] = A[0][5] - K.bf * invz_2;
    double Wd = inv, Wo = 0.0, rho1 = 1.0;
    if (robust) {
        double r0;
        po_huber(po_chi2(inv, stereo, e0, e1, e2), delta, dsqr, r0, rho1);
        Wd = rho1 * inv;
        Wo = rho1 * 0.0;
    }
    double tm[6][3];  // A^T W
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        const double a0 = A[0][i] * Wd + A[1][i] * Wo;
        const double a1 = A[0][i] * Wo + A[1][i] * Wd;
        tm[i][0] = stereo ? a0 + A[2][i] * Wo : a0;
        tm[i][1] = stereo ? a1 + A[2][i] * Wo : a1;
        tm[i][2] = (A[0][i] * Wo + A[1][i] * Wo) + A[2][i] * Wd;
    }
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 6; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            const double h = tm[i][0] * A[0][j] + tm[i][1] * A[1][j];
            t[k++] = stereo ? h + tm[i][2] * A[2][j] : h;
        }
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        double a0 = A[0][i], a1 = A[1][i], a2 = A[2][i];
        if (robust) {
            a0 = rho1 * a0;
            a1 = rho1 * a1;
            a2 = rho1 * a2;
        }
        double g0 = a0 * inv + a1 * 0.0;
        double g1 = a0 * 0.0 + a1 * inv;
        const double g2 = (a0 * 0.0 + a1 * 0.0) + a2 * inv;
        if (stereo) {
            g0 = g0 + a2 * 0.0;
            g1 = g1 + a2 * 0.0;
        }
        const double gb = g0 * e0 + g1 * e1;
        t[21 + i] = stereo ? gb + g2 * e2 : gb;
    }
}

// po_quad_terms without its multiplications by the information matrix's zero off-diagonal entries
// (Wo = rho1 * 0.0, the 0.0 of omega): when every Jacobian entry, rho1 and inv are finite, each such
// product is a signed zero, and x + (+-0) is x for x != 0 and a zero otherwise — so every term equals
// po_quad_terms' up to the sign of a zero term.  The folds cannot tell those apart: every H / b / chi2
// accumulator starts at +0.0 and adds (b: subtracts) the terms, and under round-to-nearest a sum is
// -0 only when both operands are -0, so an accumulator that starts at +0.0 never holds -0 and
// acc + (+0) == acc + (-0) for every acc it can hold.  The errors are in the precondition too (a zero
// term times an infinite error would be a NaN whose bits the folds carry).  Returns false (t
// unspecified) when the finite precondition fails; the caller then evaluates po_quad_terms.  Products
// by zero make up about a third of po_quad_terms' multiply-adds.
RSC_HD bool po_quad_terms_finite(const PoSE3& est, const PoCam& K, const double (&Xw)[3], double inv, double e0,
                                 double e1, double e2, bool stereo, bool robust, double delta, double dsqr,
                                 double (&t)[kPoseTerms]) {
    double p[3];
    po_map(est, Xw, p);
    const double x = p[0], y = p[1];
    const double invz = 1.0 / p[2];
    const double invz_2 = invz * invz;
    double A[3][6];
    A[0][0] = x * y * invz_2 * K.fx;
    A[0][1] = -(1 + (x * x * invz_2)) * K.fx;
    A[0][2] = y * invz * K.fx;
    A[0][3] = -invz * K.fx;
    A[0][4] = 0;
    A[0][5] = x * invz_2 * K.fx;
    A[1][0] = (1 + y * y * invz_2) * K.fy;
    A[1][1] = -x * y * invz_2 * K.fy;
    A[1][2] = -x * invz * K.fy;
    A[1][3] = 0;
    A[1][4] = -invz * K.fy;
    A[1][5] = y * invz_2 * K.fy;
    A[2][0] = A[0][0] - K.bf * y * invz_2;
    A[2][1] = A[0][1] + K.bf * x * invz_2;
    A[2][2] = A[0][2];
    A[2][3] = A[0][3];
    A[2][4] = 0;
    A[2][5] = A[0][5] - K.bf * invz_2;
    double Wd = inv, rho1 = 1.0;
    if (robust) {
        double r0;
        po_huber(po_chi2(inv, stereo, e0, e1, e2), delta, dsqr, r0, rho1);
        Wd = rho1 * inv;
    }
    // finite precondition (a sum of magnitudes: an overflow only sends the edge to the full form)
    double mag = ((rabs(rho1) + rabs(inv)) + (rabs(e0) + rabs(e1))) + rabs(e2);
    RSC_UNROLL for (int i = 0; i < 6; ++i) mag = mag + ((rabs(A[0][i]) + rabs(A[1][i])) + rabs(A[2][i]));
    // The Jacobian's constant zeros A[0][4] = A[1][3] = A[2][4] = 0 make every product through them a
    // signed zero too (finite precondition), so those products are dropped from the sums the same way
    // (z0 / z1 / z2 below: static after unrolling).
    double tm[6][3];  // A^T W
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        tm[i][0] = A[0][i] * Wd;
        tm[i][1] = A[1][i] * Wd;
        tm[i][2] = A[2][i] * Wd;
    }
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 6; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) {
            const bool z0 = (i == 4) | (j == 4), z1 = (i == 3) | (j == 3), z2 = (i == 4) | (j == 4);
            double h;
            if (!z0 && !z1) h = tm[i][0] * A[0][j] + tm[i][1] * A[1][j];
            else if (!z0) h = tm[i][0] * A[0][j];
            else if (!z1) h = tm[i][1] * A[1][j];
            else h = 0.0;
            t[k++] = (stereo && !z2) ? h + tm[i][2] * A[2][j] : h;
        }
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        double a0 = A[0][i], a1 = A[1][i], a2 = A[2][i];
        if (robust) {
            a0 = rho1 * a0;
            a1 = rho1 * a1;
            a2 = rho1 * a2;
        }
        double gb;
        if (i == 3) gb = (a0 * inv) * e0;       // a1 = rho1 A[1][3] = 0
        else if (i == 4) gb = (a1 * inv) * e1;  // a0 = a2 = 0
        else gb = (a0 * inv) * e0 + (a1 * inv) * e1;
        t[21 + i] = (stereo && i != 4) ? gb + (a2 * inv) * e2 : gb;
    }
    return mag <= 1.7976931348623157e308;  // finite (a NaN compares false)
}

// A pivot index every lane of the wave holds (device: read from the first lane into an SGPR, so the
// branches on it are scalar and only the taken transposition runs; host: itself).
RSC_HD int po_uniform(int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(v);
#else
    return v;
#endif
}

// Eigen::LDLT<MatrixXd> on the lower triangle of the n x n (ldlt_inplace<Lower>::unblocked) and
// _solve_impl; returns isPositive() (x untouched otherwise, as LinearSolverDense::solve).
// Register arrays with static indices only: the diagonal pivot search is a select chain, the pivot
// it finds is made wave-uniform (po_uniform) and the symmetric transposition and the solve's
// permutation steps branch on it.  Precondition: every lane of the wave solves the same system (the
// callers' LM steps run redundantly on identical data).  n = 6 (PoseOptimization), 7 (OptimizeSim3).
template <int n>
RSC_HD bool po_ldlt_solve(double (&A)[n][n], const double (&b)[n], double (&x)[n]) {
    int sign = 0;  // 0 zero, 1 positive semidef, 2 negative semidef, 3 indefinite
    int tr[n];
    bool stop = false;
    RSC_UNROLL for (int k = 0; k < n; ++k) {
        tr[k] = k;
        if (!stop) {
            int big = k;
            double bv = rabs(A[k][k]);
            RSC_UNROLL for (int i = k + 1; i < n; ++i)
                if (rabs(A[i][i]) > bv) { bv = rabs(A[i][i]); big = i; }
            big = po_uniform(big);
            tr[k] = big;
            // symmetric swap of k and big on the lower triangle (Eigen's four-step exchange)
            RSC_UNROLL for (int bb = k + 1; bb < n; ++bb) {
                if (bb == big) {
                    RSC_UNROLL for (int j = 0; j < k; ++j) { const double t = A[k][j]; A[k][j] = A[bb][j]; A[bb][j] = t; }
                    RSC_UNROLL for (int i = bb + 1; i < n; ++i) { const double t = A[i][k]; A[i][k] = A[i][bb]; A[i][bb] = t; }
                    { const double t = A[k][k]; A[k][k] = A[bb][bb]; A[bb][bb] = t; }
                    RSC_UNROLL for (int i = k + 1; i < bb; ++i) { const double t = A[i][k]; A[i][k] = A[bb][i]; A[bb][i] = t; }
                }
            }
            if (k > 0) {
                double temp[n];
                RSC_UNROLL for (int j = 0; j < k; ++j) temp[j] = A[j][j] * A[k][j];
                double acc = A[k][0] * temp[0];
                RSC_UNROLL for (int j = 1; j < k; ++j) acc = acc + A[k][j] * temp[j];
                A[k][k] -= acc;
                RSC_UNROLL for (int r = k + 1; r < n; ++r) {
                    double a = A[r][0] * temp[0];
                    RSC_UNROLL for (int j = 1; j < k; ++j) a = a + A[r][j] * temp[j];
                    A[r][k] -= a;
                }
            }
            const double akk = A[k][k];
            const bool valid = po_uniform(rabs(akk) > 0.0);
            if (k == 0 && !valid) {
                sign = 0;
                stop = true;
                tr[0] = 0;
            } else {
                if (valid) RSC_UNROLL for (int r = k + 1; r < n; ++r) A[r][k] /= akk;
                if (sign == 1) {
                    if (akk < 0.0) sign = 3;
                } else if (sign == 2) {
                    if (akk > 0.0) sign = 3;
                } else if (sign == 0) {
                    if (akk > 0.0) sign = 1;
                    else if (akk < 0.0) sign = 2;
                }
            }
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[n];
    RSC_UNROLL for (int i = 0; i < n; ++i) y[i] = b[i];
    RSC_UNROLL for (int k = 0; k < n; ++k)
        RSC_UNROLL for (int j = k + 1; j < n; ++j)
            if (tr[k] == j) rswap(y[k], y[j]);
    RSC_UNROLL for (int i = 1; i < n; ++i) {
        double acc = A[i][0] * y[0];
        RSC_UNROLL for (int j = 1; j < i; ++j) acc = acc + A[i][j] * y[j];
        y[i] -= acc;
    }
    const double tol = lim<double>::min();
    RSC_UNROLL for (int i = 0; i < n; ++i) y[i] = (rabs(A[i][i]) > tol) ? y[i] / A[i][i] : 0.0;
    RSC_UNROLL for (int i = n - 2; i >= 0; --i) {
        double acc = A[i + 1][i] * y[i + 1];
        RSC_UNROLL for (int j = i + 2; j < n; ++j) acc = acc + A[j][i] * y[j];
        y[i] -= acc;
    }
    RSC_UNROLL for (int k = n - 1; k >= 0; --k)
        RSC_UNROLL for (int j = k + 1; j < n; ++j)
            if (tr[k] == j) rswap(y[k], y[j]);
    RSC_UNROLL for (int i = 0; i < n; ++i) x[i] = y[i];
    return true;
}

RSC_HD bool po_ldlt_solve6(double (&A)[6][6], const double (&b)[6], double (&x)[6]) { return po_ldlt_solve<6>(A, b, x); }

#if defined(__HIP_DEVICE_COMPILE__)
// po_ldlt_solve with the matrix distributed one ROW PER LANE (lane r < n holds row r of the full
// symmetric matrix in VGPRs; lanes >= n mirror row n - 1 and are never read).  Same operations on
// the same operands, so the same bits: the pivot search reads the diagonal with v_readlane; the
// symmetric transposition of k and big is the permutation P A P of the full storage — rows k and big
// exchanged across lanes, columns k and big inside every lane — which equals Eigen's four-step
// lower-triangle exchange because the trailing block (rows and columns >= k) is never written before
// its own step and so is still symmetric; a step's column update and division run on the n - k
// lanes at once (one IEEE division per lane instead of n - k in sequence).  The solve reads L and D
// back with v_readlane and runs wave-uniformly as po_ldlt_solve's.  `row` = this lane's row of
// H (lambda added to its diagonal by the caller), `b` wave-uniform.  Every lane of the wave must
// call it (wave-uniform control).
template <int n>
__device__ bool po_ldlt_solve_lanes(const double (&row)[n], const double (&b)[n], double (&x)[n]) {
    const int lane = (int)(threadIdx.x & 63);
    double a[n];
    RSC_UNROLL for (int c = 0; c < n; ++c) a[c] = row[c];
    int sign = 0;
    int tr[n];
    bool stop = false;
    RSC_UNROLL for (int k = 0; k < n; ++k) {
        tr[k] = k;
        if (!stop) {
            int big = k;
            double bv = rabs(lane_read(a[k], k));
            RSC_UNROLL for (int i = k + 1; i < n; ++i) {
                const double d = rabs(lane_read(a[i], i));
                if (d > bv) { bv = d; big = i; }
            }
            big = po_uniform(big);
            tr[k] = big;
            if (big != k) {
                RSC_UNROLL for (int c = 0; c < n; ++c) {  // rows k and big
                    const double vb = lane_read(a[c], big), vk = lane_read(a[c], k);
                    a[c] = (lane == k) ? vb : ((lane == big) ? vk : a[c]);
                }
                RSC_UNROLL for (int c = k + 1; c < n; ++c)  // columns k and big
                    if (c == big) rswap(a[k], a[c]);
            }
            if (k > 0) {
                double temp[n];
                RSC_UNROLL for (int j = 0; j < k; ++j) temp[j] = lane_read(a[j], j) * lane_read(a[j], k);
                double acc = a[0] * temp[0];
                RSC_UNROLL for (int j = 1; j < k; ++j) acc = acc + a[j] * temp[j];
                if (lane >= k) a[k] -= acc;  // A[k][k] on lane k, A[r][k] on lanes r > k
            }
            const double akk = lane_read(a[k], k);
            const bool valid = po_uniform(rabs(akk) > 0.0);
            if (k == 0 && !valid) {
                sign = 0;
                stop = true;
                tr[0] = 0;
            } else {
                if (valid && lane > k) a[k] /= akk;
                if (sign == 1) {
                    if (akk < 0.0) sign = 3;
                } else if (sign == 2) {
                    if (akk > 0.0) sign = 3;
                } else if (sign == 0) {
                    if (akk > 0.0) sign = 1;
                    else if (akk < 0.0) sign = 2;
                }
            }
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double L[n][n];  // the factor read back, wave-uniform (lower triangle and diagonal)
    RSC_UNROLL for (int i = 0; i < n; ++i)
        RSC_UNROLL for (int j = 0; j <= i; ++j) L[i][j] = lane_read(a[j], i);
    double y[n];
    RSC_UNROLL for (int i = 0; i < n; ++i) y[i] = b[i];
    RSC_UNROLL for (int k = 0; k < n; ++k)
        RSC_UNROLL for (int j = k + 1; j < n; ++j)
            if (tr[k] == j) rswap(y[k], y[j]);
    RSC_UNROLL for (int i = 1; i < n; ++i) {
        double acc = L[i][0] * y[0];
        RSC_UNROLL for (int j = 1; j < i; ++j) acc = acc + L[i][j] * y[j];
        y[i] -= acc;
    }
    const double tol = lim<double>::min();
    RSC_UNROLL for (int i = 0; i < n; ++i) y[i] = (rabs(L[i][i]) > tol) ? y[i] / L[i][i] : 0.0;
    RSC_UNROLL for (int i = n - 2; i >= 0; --i) {
        double acc = L[i + 1][i] * y[i + 1];
        RSC_UNROLL for (int j = i + 2; j < n; ++j) acc = acc + L[j][i] * y[j];
        y[i] -= acc;
    }
    RSC_UNROLL for (int k = n - 1; k >= 0; --k)
        RSC_UNROLL for (int j = k + 1; j < n; ++j)
            if (tr[k] == j) rswap(y[k], y[j]);
    RSC_UNROLL for (int i = 0; i < n; ++i) x[i] = y[i];
    return true;
}
#elif defined(__HIPCC__)
// host pass of a .hip file: declared for the kernels' parse, defined for the device only
template <int n>
__device__ bool po_ldlt_solve_lanes(const double (&row)[n], const double (&b)[n], double (&x)[n]);
#endif

#if defined(__HIPCC__)
hipError_t read_poseopt_phases(uint64_t* out, bool wide);  // diagnostic, [64][8] or [64][24] (poseopt.hip)
// rsc_selftest_math fn 16: record r = x[42 r ..] holds a 6 x 6 matrix (row-major, symmetric) and b[6];
// out[42 r + 0..5] / [6] = po_ldlt_solve's x / ok, [7..12] / [13] = po_ldlt_solve_lanes' (one wave per record)
hipError_t launch_selftest_ldlt(const double* x, int nrec, double* out, hipStream_t st);
// fault: the launch's fault word (pinned host memory; raised when a streamed pass's hand-off wait gives up)
hipError_t launch_poseopt(int count, const DevPoseProb* probs, unsigned* fault, hipStream_t st);
#endif

}  // namespace rsc
