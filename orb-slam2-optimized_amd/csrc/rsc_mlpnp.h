// rsc_mlpnp.h — per-lane MLPnP hypothesis (MLPnPsolver::computePose, src/MLPnPsolver.cpp:321-623)
// for one hypothesis per lane.  Same arithmetic as the oracle restatement (oracle/mlpnp_oracle.cpp):
// every sum left to right, fdlibm transcendentals (rsc_math.h), correctly rounded restatements of
// glibc's pow(x, 1.0/3.0) and pow(x, 3.0/2.0) (rsc_math.h), the reference's own generated residual
// Jacobian mlpnpJacs operation for operation (rsc_mlpnp_jac.h), generic cofactor 4x4 inverse.
//
// Storage: small matrices in VGPRs with static indices; the 12x12 (or 9x9) JacobiSVD work matrix W
// and its V accumulate in a per-lane LDS slab (LaneMat, element-major across the wave, 288 doubles
// per lane); during Gauss-Newton the W region holds the 2n x 6 Jacobian and the LDLT factor.
#pragma once
// phase stamp hook (mlpnp.hip defines it for its RSC_ML_STAMPS=1 diagnostic build)
#ifndef RSC_ML_STAMP
#define RSC_ML_STAMP(k) \
    do {                \
    } while (0)
#endif
#include "rsc_core.h"
#include "rsc_math.h"
#include "rsc_mlpnp_jac.h"

namespace rsc {

constexpr int kMlSlabDoubles = 288;  // W [12][12] + V [12][12] per lane

struct MlView {  // row-major 12-stride matrix inside the lane slab, at element offset `off`
    double* base;
    int stride, off;
    RSC_HD double& at(int r, int c) const { return base[(off + r * 12 + c) * stride]; }
    RSC_HD double& e(int i) const { return base[(off + i) * stride]; }
};

RSC_HD double ml_dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
RSC_HD double ml_norm3(const double* a) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }
RSC_HD void ml_cross3(const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
RSC_HD double ml_det3(const double (&m)[3][3]) {
    return m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[1][0] * (m[0][1] * m[2][2] - m[0][2] * m[2][1]) +
           m[2][0] * (m[0][1] * m[1][2] - m[0][2] * m[1][1]);
}

// Nullspace of the bearing f (JacobiSVD<.., HouseholderQRPreconditioner>(f^T, FullV), V cols 1..2).
RSC_HD void ml_bearing_nullspace(const double (&f)[3], double (&Ns)[3][2]) {
    double scale = rabs(f[0]);
    if (rabs(f[1]) > scale) scale = rabs(f[1]);
    if (rabs(f[2]) > scale) scale = rabs(f[2]);
    if (scale == 0.0) scale = 1.0;
    double v[3] = {f[0] / scale, f[1] / scale, f[2] / scale};
    double tau, beta;
    make_householder<double, 3>(v, tau, beta);
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    if (tau != 0.0) {
        double tmp[3];
        RSC_UNROLL for (int c = 0; c < 3; ++c) tmp[c] = (v[1] * V[1][c] + v[2] * V[2][c]) + V[0][c];
        RSC_UNROLL for (int c = 0; c < 3; ++c) V[0][c] = V[0][c] - tau * tmp[c];
        RSC_UNROLL for (int r = 0; r < 2; ++r) {
            const double te = tau * v[1 + r];
            RSC_UNROLL for (int c = 0; c < 3; ++c) V[1 + r][c] = V[1 + r][c] - te * tmp[c];
        }
    }
    RSC_UNROLL for (int r = 0; r < 3; ++r) { Ns[r][0] = V[r][1]; Ns[r][1] = V[r][2]; }
}

// FullPivHouseholderQR<Matrix3d>(A).rank(), registers, select-based pivoting.
RSC_HD int ml_fullpiv_rank3(const double (&A)[3][3]) {
    double m[3][3];
    RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) m[r][c] = A[r][c];
    const double precision = lim<double>::eps() * 3.0;
    double biggest = 0.0, maxpivot = 0.0;
    int nonzero = 3;
    bool stopped = false;
    RSC_UNROLL for (int k = 0; k < 3; ++k) {
        if (!stopped) {
            int br = k, bc = k;
            double bv = rabs(m[k][k]);
            RSC_UNROLL for (int c = k; c < 3; ++c)
                RSC_UNROLL for (int r = k; r < 3; ++r) {
                    if (r == k && c == k) continue;
                    const double a = rabs(m[r][c]);
                    const bool gt = a > bv;
                    bv = gt ? a : bv;
                    br = gt ? r : br;
                    bc = gt ? c : bc;
                }
            if (k == 0) biggest = bv;
            if (bv <= biggest * precision) {
                nonzero = k;
                stopped = true;
            } else {
                RSC_UNROLL for (int r = k + 1; r < 3; ++r) {
                    const bool sw = (r == br);
                    RSC_UNROLL for (int c = k; c < 3; ++c) {
                        const double a = m[k][c], b = m[r][c];
                        m[k][c] = sw ? b : a;
                        m[r][c] = sw ? a : b;
                    }
                }
                RSC_UNROLL for (int c = k + 1; c < 3; ++c) {
                    const bool sw = (c == bc);
                    RSC_UNROLL for (int r = 0; r < 3; ++r) {
                        const double a = m[r][k], b = m[r][c];
                        m[r][k] = sw ? b : a;
                        m[r][c] = sw ? a : b;
                    }
                }
                double col[3] = {0.0, 0.0, 0.0};
                RSC_UNROLL for (int r = k; r < 3; ++r) col[r - k] = m[r][k];
                double tau, beta;
                if (k == 0) { make_householder<double, 3>(col, tau, beta); }
                else if (k == 1) { double c2[2] = {col[0], col[1]}; make_householder<double, 2>(c2, tau, beta); col[1] = c2[1]; }
                else { double c1[1] = {col[0]}; make_householder<double, 1>(c1, tau, beta); }
                RSC_UNROLL for (int r = k + 1; r < 3; ++r) m[r][k] = col[r - k];
                m[k][k] = beta;
                if (rabs(beta) > maxpivot) maxpivot = rabs(beta);
                const int rows = 3 - k, cols = 3 - k - 1;
                if (cols > 0 && rows > 1 && tau != 0.0) {
                    double tmp[3];
                    RSC_UNROLL for (int c = 0; c < cols; ++c) {
                        double acc = col[1] * m[k + 1][k + 1 + c];
                        RSC_UNROLL for (int r = 1; r < rows - 1; ++r) acc = acc + col[1 + r] * m[k + 1 + r][k + 1 + c];
                        tmp[c] = acc + m[k][k + 1 + c];
                    }
                    RSC_UNROLL for (int c = 0; c < cols; ++c) m[k][k + 1 + c] = m[k][k + 1 + c] - tau * tmp[c];
                    RSC_UNROLL for (int r = 0; r < rows - 1; ++r) {
                        const double te = tau * col[1 + r];
                        RSC_UNROLL for (int c = 0; c < cols; ++c)
                            m[k + 1 + r][k + 1 + c] = m[k + 1 + r][k + 1 + c] - te * tmp[c];
                    }
                }
            }
        }
    }
    const double thr = rabs(maxpivot) * precision;
    int rank = 0;
    RSC_UNROLL for (int i = 0; i < 3; ++i) rank += (i < nonzero && rabs(m[i][i]) > thr) ? 1 : 0;
    return rank;
}

// One two-sided Jacobi step of JacobiSVD on the 2x2 (p,q) block: rotations (cl, sl) on the left,
// (cr, sr) on the right (real_2x2_jacobi_svd).  Returns false when W(p,q), W(q,p) are below
// threshold (no rotation).
RSC_HD void ml_jacobi_2x2(double m00, double m01, double m10, double m11, double& cl, double& sl, double& cr,
                          double& sr) {
    // real_2x2_jacobi_svd with its ifs as value selects on the same operands (a divergent if is an
    // exec-mask region; the selects keep the 16 hypotheses of a wave on one instruction stream), and
    // 1 / sqrt(tt^2 + 1) in the short-chain unit forms: |tt| <= 1 (|tau +- w| >= 1), so tt^2 + 1 is
    // in [1, 2] and its root in [1, sqrt 2] (rsc_core.h sqrt_unit / recip_unit, correctly rounded).
    const double considerAsZero = lim<double>::min();
    const double t = m00 + m11;
    const double d = m10 - m01;
    const bool dz = rabs(d) < considerAsZero;
    const double u = t / d;
    const double tmp = sqrt(1.0 + u * u);
    const double s1 = dz ? 0.0 : 1.0 / tmp;
    const double c1 = dz ? 1.0 : u / tmp;
    {
        const bool rot = !((int)(c1 == 1.0) & (int)(s1 == 0.0));
        const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
        m00 = rot ? c1 * x0 + s1 * y0 : x0;
        m10 = rot ? -s1 * x0 + c1 * y0 : y0;
        m01 = rot ? c1 * x1 + s1 * y1 : x1;
        m11 = rot ? -s1 * x1 + c1 * y1 : y1;
    }
    const double deno = 2.0 * rabs(m01);
    const bool nz = deno < considerAsZero;
    const double tau = (m00 - m11) / deno;
    const double w = sqrt(tau * tau + 1.0);
    const double tt = 1.0 / (tau > 0.0 ? tau + w : tau - w);
    const double sign_t = tt > 0.0 ? 1.0 : -1.0;
    const double nn = recip_unit(sqrt_unit(tt * tt + 1.0));
    sr = nz ? 0.0 : -sign_t * (m01 / rabs(m01)) * rabs(tt) * nn;
    cr = nz ? 1.0 : nn;
    const double crt = cr, srt = -sr;
    cl = c1 * crt - s1 * srt;
    sl = c1 * srt + s1 * crt;
}

// JacobiSVD<MatrixXd>(A, ComputeFullV) of the n x n (n = 9 or 12) matrix in W (LDS); returns the V
// column of the smallest singular value after Eigen's descending sort, in r1[0..n).
RSC_HD void ml_jacobi_svd_lds(const MlView& W, const MlView& V, int n, double (&r1)[12]) {
    const double precision = 2.0 * lim<double>::eps();
    const double considerAsZero = lim<double>::min();
    double scale = rabs(W.at(0, 0));
    for (int c = 0; c < n; ++c)
        for (int r = 0; r < n; ++r) {
            if (r == 0 && c == 0) continue;
            const double a = rabs(W.at(r, c));
            if (a > scale) scale = a;
        }
    if (scale == 0.0) scale = 1.0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            W.at(r, c) = W.at(r, c) / scale;
            V.at(r, c) = (r == c) ? 1.0 : 0.0;
        }
    double maxDiag = rabs(W.at(0, 0));
    for (int i = 1; i < n; ++i)
        if (rabs(W.at(i, i)) > maxDiag) maxDiag = rabs(W.at(i, i));
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < n; ++p) {
            for (int q = 0; q < p; ++q) {
                const double pt = precision * maxDiag;
                const double threshold = (considerAsZero < pt) ? pt : considerAsZero;
                const double wpq = W.at(p, q), wqp = W.at(q, p);
                if (rabs(wpq) > threshold || rabs(wqp) > threshold) {
                    finished = false;
                    double cl, sl, cr, sr;
                    ml_jacobi_2x2(W.at(p, p), wpq, wqp, W.at(q, q), cl, sl, cr, sr);
                    if (!(cl == 1.0 && sl == 0.0)) {
                        for (int c = 0; c < n; ++c) {
                            const double xi = W.at(p, c), yi = W.at(q, c);
                            W.at(p, c) = cl * xi + sl * yi;
                            W.at(q, c) = -sl * xi + cl * yi;
                        }
                    }
                    if (!(cr == 1.0 && sr == 0.0)) {
                        for (int r = 0; r < n; ++r) {
                            const double xi = W.at(r, p), yi = W.at(r, q);
                            W.at(r, p) = cr * xi - sr * yi;
                            W.at(r, q) = sr * xi + cr * yi;
                        }
                        for (int r = 0; r < n; ++r) {
                            const double xi = V.at(r, p), yi = V.at(r, q);
                            V.at(r, p) = cr * xi - sr * yi;
                            V.at(r, q) = sr * xi + cr * yi;
                        }
                    }
                    const double a = rabs(W.at(p, p)), b = rabs(W.at(q, q));
                    const double mm = (a < b) ? b : a;
                    maxDiag = (maxDiag < mm) ? mm : maxDiag;
                }
            }
        }
        RSC_LOOP_FENCE();
    }
    // singular values, descending selection sort (first maximum), stop at a zero maximum
    double sv[12];
    int perm[12];
    RSC_UNROLL for (int i = 0; i < 12; ++i) {
        sv[i] = (i < n) ? rabs(W.at(i, i)) * scale : 0.0;
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
    for (int r = 0; r < n; ++r) r1[r] = V.at(r, last);
}

// JacobiSVD<MatrixXd>(3x3, ComputeFullU|ComputeFullV) in registers; returns U * V^T (sorted).
RSC_HD void ml_nearest_rotation(const double (&A)[3][3], double (&Rout)[3][3]) {
    const double precision = 2.0 * lim<double>::eps();
    const double considerAsZero = lim<double>::min();
    double scale = rabs(A[0][0]);
    RSC_UNROLL for (int c = 0; c < 3; ++c)
        RSC_UNROLL for (int r = 0; r < 3; ++r) {
            if (r == 0 && c == 0) continue;
            if (rabs(A[r][c]) > scale) scale = rabs(A[r][c]);
        }
    if (scale == 0.0) scale = 1.0;
    double W[3][3], U[3][3], V[3][3];
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) {
            W[r][c] = A[r][c] / scale;
            U[r][c] = (r == c) ? 1.0 : 0.0;
            V[r][c] = (r == c) ? 1.0 : 0.0;
        }
    double maxDiag = rabs(W[0][0]);
    RSC_UNROLL for (int i = 1; i < 3; ++i) if (rabs(W[i][i]) > maxDiag) maxDiag = rabs(W[i][i]);
    bool finished = false;
    while (!finished) {
        finished = true;
        RSC_UNROLL for (int p = 1; p < 3; ++p) {
            RSC_UNROLL for (int q = 0; q < p; ++q) {
                const double pt = precision * maxDiag;
                const double threshold = (considerAsZero < pt) ? pt : considerAsZero;
                if (rabs(W[p][q]) > threshold || rabs(W[q][p]) > threshold) {
                    finished = false;
                    double cl, sl, cr, sr;
                    ml_jacobi_2x2(W[p][p], W[p][q], W[q][p], W[q][q], cl, sl, cr, sr);
                    const bool left = !(cl == 1.0 && sl == 0.0);
                    RSC_UNROLL for (int c = 0; c < 3; ++c) {
                        const double xi = W[p][c], yi = W[q][c];
                        W[p][c] = left ? cl * xi + sl * yi : xi;
                        W[q][c] = left ? -sl * xi + cl * yi : yi;
                    }
                    RSC_UNROLL for (int r = 0; r < 3; ++r) {
                        const double xi = U[r][p], yi = U[r][q];
                        U[r][p] = left ? cl * xi + sl * yi : xi;
                        U[r][q] = left ? -sl * xi + cl * yi : yi;
                    }
                    const bool right = !(cr == 1.0 && sr == 0.0);
                    RSC_UNROLL for (int r = 0; r < 3; ++r) {
                        const double xi = W[r][p], yi = W[r][q];
                        W[r][p] = right ? cr * xi - sr * yi : xi;
                        W[r][q] = right ? sr * xi + cr * yi : yi;
                    }
                    RSC_UNROLL for (int r = 0; r < 3; ++r) {
                        const double xi = V[r][p], yi = V[r][q];
                        V[r][p] = right ? cr * xi - sr * yi : xi;
                        V[r][q] = right ? sr * xi + cr * yi : yi;
                    }
                    const double a = rabs(W[p][p]), b = rabs(W[q][q]);
                    const double mm = (a < b) ? b : a;
                    maxDiag = (maxDiag < mm) ? mm : maxDiag;
                }
            }
        }
        RSC_LOOP_FENCE();
    }
    double sv[3];
    RSC_UNROLL for (int i = 0; i < 3; ++i) {
        const double a = W[i][i];
        sv[i] = rabs(a);
        const bool neg = a < 0.0;
        RSC_UNROLL for (int r = 0; r < 3; ++r) U[r][i] = neg ? -U[r][i] : U[r][i];
    }
    RSC_UNROLL for (int i = 0; i < 3; ++i) sv[i] = sv[i] * scale;
    bool stopped = false;
    RSC_UNROLL for (int i = 0; i < 3; ++i) {
        if (!stopped) {
            int pos = 0;
            double mv = sv[i];
            RSC_UNROLL for (int j = 1; j < 3 - i; ++j) {
                const bool gt = sv[i + j] > mv;
                mv = gt ? sv[i + j] : mv;
                pos = gt ? j : pos;
            }
            if (mv == 0.0) {
                stopped = true;
            } else {
                RSC_UNROLL for (int j = 1; j < 3 - i; ++j) {
                    const bool sw = (j == pos);
                    const double a = sv[i], b = sv[i + j];
                    sv[i] = sw ? b : a;
                    sv[i + j] = sw ? a : b;
                    RSC_UNROLL for (int r = 0; r < 3; ++r) {
                        const double ua = U[r][i], ub = U[r][i + j];
                        U[r][i] = sw ? ub : ua;
                        U[r][i + j] = sw ? ua : ub;
                        const double va = V[r][i], vb = V[r][i + j];
                        V[r][i] = sw ? vb : va;
                        V[r][i + j] = sw ? va : vb;
                    }
                }
            }
        }
    }
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) Rout[r][c] = U[r][0] * V[c][0] + U[r][1] * V[c][1] + U[r][2] * V[c][2];
}

// Matrix4d::inverse, generic cofactor expansion (see oracle/mlpnp_oracle.cpp inverse4).
RSC_HD void ml_inverse4(const double (&m)[4][4], double (&out)[4][4]) {
    RSC_UNROLL for (int i = 0; i < 4; ++i)
        RSC_UNROLL for (int j = 0; j < 4; ++j) {
            const int i1 = (i + 1) % 4, i2 = (i + 2) % 4, i3 = (i + 3) % 4;
            const int j1 = (j + 1) % 4, j2 = (j + 2) % 4, j3 = (j + 3) % 4;
            auto h = [&](int a1, int a2, int a3) {
                return m[a1][j1] * (m[a2][j2] * m[a3][j3] - m[a2][j3] * m[a3][j2]);
            };
            const double c = h(i1, i2, i3) + h(i2, i3, i1) + h(i3, i1, i2);
            out[j][i] = ((i + j) & 1) ? -c : c;
        }
    const double det = ((m[0][0] * out[0][0] + m[1][0] * out[0][1]) + m[2][0] * out[0][2]) + m[3][0] * out[0][3];
    RSC_UNROLL for (int r = 0; r < 4; ++r) RSC_UNROLL for (int c = 0; c < 4; ++c) out[r][c] = out[r][c] / det;
}

RSC_HD void ml_rodrigues2rot(const double (&w)[3], double (&R)[3][3]) {
    const double S[3][3] = {{0.0, -w[2], w[1]}, {w[2], 0.0, -w[0]}, {-w[1], w[0], 0.0}};
    const double nrm = ml_norm3(w);
    RSC_UNROLL for (int i = 0; i < 3; ++i) RSC_UNROLL for (int j = 0; j < 3; ++j) R[i][j] = (i == j) ? 1.0 : 0.0;
    if (nrm > lim<double>::eps()) {
        const double a = dm::sin(nrm) / nrm;
        const double b = (1.0 - dm::cos(nrm)) / (nrm * nrm);
        RSC_UNROLL for (int i = 0; i < 3; ++i)
            RSC_UNROLL for (int j = 0; j < 3; ++j) {
                const double ss = S[i][0] * S[0][j] + S[i][1] * S[1][j] + S[i][2] * S[2][j];
                R[i][j] = (R[i][j] + a * S[i][j]) + b * ss;
            }
    }
}

RSC_HD void ml_rot2rodrigues(const double (&R)[3][3], double (&w)[3]) {
    w[0] = w[1] = w[2] = 0.0;
    const double trace = ((R[0][0] + R[1][1]) + R[2][2]) - 1.0;
    const double wnorm = dm::acos(trace / 2.0);
    if (wnorm > lim<double>::eps()) {
        w[0] = R[2][1] - R[1][2];
        w[1] = R[0][2] - R[2][0];
        w[2] = R[1][0] - R[0][1];
        const double sc = wnorm / (2.0 * dm::sin(wnorm));
        RSC_UNROLL for (int k = 0; k < 3; ++k) w[k] *= sc;
    }
}

// LDLT<MatrixXd>(A).solve(g), 6x6, A in LDS view L (rows/cols 0..5), pivoted as Eigen.
RSC_HD void ml_ldlt_solve6(const MlView& L, const double (&g)[6], double (&x)[6]) {
    const int n = 6;
    int transp[6];
    RSC_UNROLL for (int k = 0; k < 6; ++k) transp[k] = k;
    bool dead = false;
    for (int k = 0; k < n && !dead; ++k) {
        int big = k;
        double bv = rabs(L.at(k, k));
        for (int i = k + 1; i < n; ++i)
            if (rabs(L.at(i, i)) > bv) { bv = rabs(L.at(i, i)); big = i; }
        RSC_UNROLL for (int q = 0; q < 6; ++q) transp[q] = (q == k) ? big : transp[q];
        if (k != big) {
            const int s = n - big - 1;
            for (int j = 0; j < k; ++j) { const double t = L.at(k, j); L.at(k, j) = L.at(big, j); L.at(big, j) = t; }
            for (int j = 0; j < s; ++j) {
                const double t = L.at(big + 1 + j, k);
                L.at(big + 1 + j, k) = L.at(big + 1 + j, big);
                L.at(big + 1 + j, big) = t;
            }
            { const double t = L.at(k, k); L.at(k, k) = L.at(big, big); L.at(big, big) = t; }
            for (int i = k + 1; i < big; ++i) {
                const double t = L.at(i, k);
                L.at(i, k) = L.at(big, i);
                L.at(big, i) = t;
            }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            // temp (diagonal * A10) lives in row 6 of the view
            for (int j = 0; j < k; ++j) L.at(6, j) = L.at(j, j) * L.at(k, j);
            double acc = L.at(k, 0) * L.at(6, 0);
            for (int j = 1; j < k; ++j) acc = acc + L.at(k, j) * L.at(6, j);
            L.at(k, k) -= acc;
            for (int r = 0; r < rs; ++r) {
                double a = L.at(k + 1 + r, 0) * L.at(6, 0);
                for (int j = 1; j < k; ++j) a = a + L.at(k + 1 + r, j) * L.at(6, j);
                L.at(k + 1 + r, k) -= a;
            }
        }
        const double akk = L.at(k, k);
        const bool valid = rabs(akk) > 0.0;
        if (k == 0 && !valid) {
            RSC_UNROLL for (int q = 0; q < 6; ++q) transp[q] = q;
            dead = true;
        } else if (rs > 0 && valid) {
            for (int r = 0; r < rs; ++r) L.at(k + 1 + r, k) /= akk;
        }
    }
    double y[6];
    RSC_UNROLL for (int i = 0; i < 6; ++i) y[i] = g[i];
    RSC_UNROLL for (int k = 0; k < 6; ++k) {  // P b
        RSC_UNROLL for (int j = k + 1; j < 6; ++j) {
            const bool sw = (transp[k] == j);
            const double a = y[k], b = y[j];
            y[k] = sw ? b : a;
            y[j] = sw ? a : b;
        }
    }
    RSC_UNROLL for (int i = 1; i < 6; ++i) {
        double acc = L.at(i, 0) * y[0];
        RSC_UNROLL for (int j = 1; j < i; ++j) acc = acc + L.at(i, j) * y[j];
        y[i] -= acc;
    }
    const double tol = lim<double>::min();
    RSC_UNROLL for (int i = 0; i < 6; ++i) {
        const double d = L.at(i, i);
        y[i] = (rabs(d) > tol) ? y[i] / d : 0.0;
    }
    RSC_UNROLL for (int i = 4; i >= 0; --i) {
        double acc = L.at(i + 1, i) * y[i + 1];
        RSC_UNROLL for (int j = i + 2; j < 6; ++j) acc = acc + L.at(j, i) * y[j];
        y[i] -= acc;
    }
    RSC_UNROLL for (int k = 5; k >= 0; --k) {  // P^T
        RSC_UNROLL for (int j = k + 1; j < 6; ++j) {
            const bool sw = (transp[k] == j);
            const double a = y[k], b = y[j];
            y[k] = sw ? b : a;
            y[j] = sw ? a : b;
        }
    }
    RSC_UNROLL for (int i = 0; i < 6; ++i) x[i] = y[i];
}

// Bearing-vector covariances of computePose's covMats argument (MLPnPsolver.cpp:321, :375-388):
// cov(i, k) = entry k (row-major) of correspondence i's 3x3 covariance.  MlNoCov: the reference's
// call (covMats of size 1 != n, so use_cov = false).
struct MlNoCov {
    static constexpr bool on = false;
    RSC_HD double operator()(int, int) const { return 0.0; }
};

// Covariances of the sampled correspondences idx[i] in a [n][9] table.
struct MlIndexedCov {
    static constexpr bool on = true;
    const double* c;
    const int* idx;
    RSC_HD double operator()(int i, int k) const { return c[(size_t)idx[i] * 9 + k]; }
};

// The 2x2 weight of correspondence i: (N^T Sigma N)^-1 (:380-386; Matrix2d::inverse =
// adjugate / determinant).  P[0] = P(0,0), P[1] = P(0,1), P[2] = P(1,0), P[3] = P(1,1).
template <class Cov>
RSC_HD void ml_cov_weight(const double (&N)[3][2], const Cov& cov, int i, double (&P)[4]) {
    double NtS[2][3];
    RSC_UNROLL for (int s = 0; s < 2; ++s)
        RSC_UNROLL for (int c = 0; c < 3; ++c)
            NtS[s][c] = (N[0][s] * cov(i, c) + N[1][s] * cov(i, 3 + c)) + N[2][s] * cov(i, 6 + c);
    double T[2][2];
    RSC_UNROLL for (int s = 0; s < 2; ++s)
        RSC_UNROLL for (int q = 0; q < 2; ++q) T[s][q] = (NtS[s][0] * N[0][q] + NtS[s][1] * N[1][q]) + NtS[s][2] * N[2][q];
    const double invdet = 1.0 / (T[0][0] * T[1][1] - T[1][0] * T[0][1]);
    P[0] = T[1][1] * invdet;
    P[1] = -T[0][1] * invdet;
    P[2] = -T[1][0] * invdet;
    P[3] = T[0][0] * invdet;
}

// Phase 1 of MLPnPsolver::computePose (:321-416): bearing nullspaces, covariance weights (covMats),
// the planarity test (FullPivHouseholderQR rank of P P^T) and the points P (rotated into the plane's
// eigenbasis when planar).  Shared by the lane form (mlpnp_compute_pose) and the quad kernel.
template <int NS, class Cov>
struct MlPrep {
    double Ns[NS][3][2];
    double Pw[Cov::on ? NS : 1][4];
    double eigenRot[3][3];
    double P[NS][3];
    bool planar;
    RSC_HD double pwgt(int i, int e) const { return Pw[Cov::on ? i : 0][e]; }
};

// The planarity test (:346-364): rank of P P^T == 2, and the plane's eigenbasis (identity otherwise).
template <int NS>
RSC_HD bool ml_planarity(const double (&pw)[NS][3], double (&eigenRot)[3][3]) {
    double PPt[3][3];
    RSC_UNROLL for (int a = 0; a < 3; ++a)
        RSC_UNROLL for (int b = 0; b < 3; ++b) {
            double s = pw[0][a] * pw[0][b];
            RSC_UNROLL for (int i = 1; i < NS; ++i) s = s + pw[i][a] * pw[i][b];
            PPt[a][b] = s;
        }
    const bool planar = ml_fullpiv_rank3(PPt) == 2;
    RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) eigenRot[r][c] = (r == c) ? 1.0 : 0.0;
    if (planar) {
        double Ve[3][3], we[3];
        sym_eig_reg<double, 3>(PPt, Ve, we);
        RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) eigenRot[r][c] = Ve[c][r];
    }
    return planar;
}

// Point i of the design matrix: pw (general) or eigenRot * pw (planar).
RSC_HD void ml_design_point(bool planar, const double (&eigenRot)[3][3], const double* pw, double (&P)[3]) {
    double q[3];
    RSC_UNROLL for (int r = 0; r < 3; ++r)  // Matrix3d * Vector3d (MLPnPsolver.cpp:363): Eigen's row order
        q[r] = emv3d_row(r, eigenRot[r][0] * pw[0], eigenRot[r][1] * pw[1], eigenRot[r][2] * pw[2]);
    RSC_UNROLL for (int r = 0; r < 3; ++r) P[r] = planar ? q[r] : pw[r];
}

template <int NS, class Cov>
RSC_HD void mlpnp_prepare(const double (&pw)[NS][3], const double (&f)[NS][3], const Cov& cov, MlPrep<NS, Cov>& m) {
    RSC_UNROLL for (int i = 0; i < NS; ++i) ml_bearing_nullspace(f[i], m.Ns[i]);
    if constexpr (Cov::on) RSC_UNROLL for (int i = 0; i < NS; ++i) ml_cov_weight(m.Ns[i], cov, i, m.Pw[i]);
    m.planar = ml_planarity<NS>(pw, m.eigenRot);
    RSC_UNROLL for (int i = 0; i < NS; ++i) ml_design_point(m.planar, m.eigenRot, pw[i], m.P[i]);
}

// Row (2i + s) of the design matrix A (:418-470), column col (< 9 planar, < 12 general).
RSC_HD double mlpnp_A_entry(bool planar, double n0, double n1, double n2, const double (&P)[3], int col) {
    if (planar) {
        switch (col) {
            case 0: return n0 * P[1]; case 1: return n0 * P[2];
            case 2: return n1 * P[1]; case 3: return n1 * P[2];
            case 4: return n2 * P[1]; case 5: return n2 * P[2];
            case 6: return n0; case 7: return n1; default: return n2;
        }
    }
    switch (col) {
        case 0: return n0 * P[0]; case 1: return n0 * P[1]; case 2: return n0 * P[2];
        case 3: return n1 * P[0]; case 4: return n1 * P[1]; case 5: return n1 * P[2];
        case 6: return n2 * P[0]; case 7: return n2 * P[1]; case 8: return n2 * P[2];
        case 9: return n0; case 10: return n1; default: return n2;
    }
}
template <int NS, class Cov>
RSC_HD double mlpnp_A(const MlPrep<NS, Cov>& m, int i, int s, int col) {
    return mlpnp_A_entry(m.planar, m.Ns[i][0][s], m.Ns[i][1][s], m.Ns[i][2][s], m.P[i], col);
}

// Entry (a, b) of the normal matrix A^T A (:471-478), or A^T P A with covariances (:483-484,
// evaluated as (A^T P) then the row sums in order).  ra[i][s] / rb[i][s]: A(2i + s, a) / A(2i + s, b).
// Without covariances the value is symmetric bit for bit (the products commute).
template <int NS, class Cov, class M>
RSC_HD double mlpnp_normal_entry(const M& m, const double (&ra)[NS][2], const double (&rb)[NS][2]) {
    if constexpr (Cov::on) {
        auto AtP = [&](int i, int q) { return ra[i][0] * m.pwgt(i, q) + ra[i][1] * m.pwgt(i, 2 + q); };
        double s = AtP(0, 0) * rb[0][0];
        s = s + AtP(0, 1) * rb[0][1];
        RSC_UNROLL for (int i = 1; i < NS; ++i) {
            s = s + AtP(i, 0) * rb[i][0];
            s = s + AtP(i, 1) * rb[i][1];
        }
        return s;
    } else {
        double s = ra[0][0] * rb[0][0];
        s = s + ra[0][1] * rb[0][1];
        RSC_UNROLL for (int i = 1; i < NS; ++i) {
            s = s + ra[i][0] * rb[i][0];
            s = s + ra[i][1] * rb[i][1];
        }
        return s;
    }
}

// Read access to a hypothesis' correspondences and phase-1 state for mlpnp_finish_pose: from
// registers (MlRegs, the sequential form) or from the quad kernel's parked LDS copy (MlParked in
// rsc_mlpnp_quad.h), so that kernel does not hold them in VGPRs through the Gauss-Newton loop.
template <int NS, class Cov>
struct MlRegs {
    const double (&pw_)[NS][3];
    const double (&f_)[NS][3];
    const MlPrep<NS, Cov>& m;
    RSC_HD double pw(int i, int c) const { return pw_[i][c]; }
    RSC_HD double f(int i, int c) const { return f_[i][c]; }
    RSC_HD double ns(int i, int r, int s) const { return m.Ns[i][r][s]; }
    RSC_HD double pwgt(int i, int e) const { return m.Pw[Cov::on ? i : 0][e]; }
    RSC_HD double eig(int r, int c) const { return m.eigenRot[r][c]; }
    RSC_HD bool planar() const { return m.planar; }
};

// Doubles of the Gauss-Newton slab: J (2 NS x 6), g (6), the 6x6 system + its temp row (stride 12).
// While the Jacobian rows are evaluated, mlpnpJacs' stored w-only temporaries (kMlJacStored doubles)
// occupy the space of g and the system, which are written only after the last row.
template <int NS>
constexpr int ml_gn_slab() {
    return 12 * NS + 6 + 6 * 12 + 6;
}
static_assert(12 * 6 + kMlJacStored <= ml_gn_slab<6>(), "mlpnpJacs temporaries do not fit the system's space");

// Phase 3 of computePose (:480-623): pose recovery from the null vector r1 (the V column of the
// smallest singular value of the normal matrix) and the Gauss-Newton refinement (mlpnp_gn,
// :659-723).  slab: kMlSlabDoubles doubles (element stride slab.stride) for J and the LDLT system.
// jin: the correspondences again, read with a run-time index by the Jacobian loop (the parked LDS
// copy in the quad kernel, so no register array is indexed dynamically).
template <int NS, class Cov, class View, class JView>
RSC_HD void mlpnp_finish_pose(const View& in, const JView& jin, const double (&r1)[12], const LaneMat& slab,
                              double (&Rout)[3][3], double (&tout)[3]) {
    const bool planar = in.planar();
    double R[3][3], t[3];
    if (planar) {
        double tmp[3][3] = {{0.0, r1[0], r1[1]}, {0.0, r1[2], r1[3]}, {0.0, r1[4], r1[5]}};
        {
            const double c1[3] = {tmp[0][1], tmp[1][1], tmp[2][1]}, c2[3] = {tmp[0][2], tmp[1][2], tmp[2][2]};
            double c0[3];
            ml_cross3(c1, c2, c0);
            RSC_UNROLL for (int r = 0; r < 3; ++r) tmp[r][0] = c0[r];
        }
        double tt[3][3];
        RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) tt[r][c] = tmp[c][r];
        const double cn1[3] = {tt[0][1], tt[1][1], tt[2][1]}, cn2[3] = {tt[0][2], tt[1][2], tt[2][2]};
        const double scale = 1.0 / sqrt(rabs(ml_norm3(cn1) * ml_norm3(cn2)));
        double R1[3][3];
        ml_nearest_rotation(tt, R1);
        if (ml_det3(R1) < 0) RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) R1[r][c] *= -1.0;
        double R2[3][3];
        RSC_UNROLL for (int r = 0; r < 3; ++r)
            RSC_UNROLL for (int c = 0; c < 3; ++c)
                R2[r][c] = in.eig(0, r) * R1[0][c] + in.eig(1, r) * R1[1][c] + in.eig(2, r) * R1[2][c];
        const double tv[3] = {scale * r1[6], scale * r1[7], scale * r1[8]};
        double Ro[3][3];
        RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) Ro[r][c] = -R2[c][r];
        if (ml_det3(Ro) < 0.0) RSC_UNROLL for (int r = 0; r < 3; ++r) Ro[r][2] = -Ro[r][2];
        double best_val = 0.0;
        int best = 0;
        RSC_UNROLL for (int k = 0; k < 4; ++k) {
            const bool flipR = k >= 2, flipT = (k & 1) != 0;
            double Rc[3][3], Tc[3];
            RSC_UNROLL for (int r = 0; r < 3; ++r) {
                RSC_UNROLL for (int c = 0; c < 3; ++c) Rc[r][c] = (flipR && c < 2) ? -Ro[r][c] : Ro[r][c];
                Tc[r] = flipT ? -tv[r] : tv[r];
            }
            double norms = 0.0;
            RSC_UNROLL for (int p = 0; p < 6; ++p) {
                double v[3];
                RSC_UNROLL for (int r = 0; r < 3; ++r)
                    v[r] = emv3d_row(r, Rc[r][0] * in.pw(p, 0), Rc[r][1] * in.pw(p, 1), Rc[r][2] * in.pw(p, 2)) + Tc[r];
                const double nv = ml_norm3(v);
                RSC_UNROLL for (int r = 0; r < 3; ++r) v[r] = v[r] / nv;
                { const double fp[3] = {in.f(p, 0), in.f(p, 1), in.f(p, 2)}; norms += (1.0 - ml_dot3(v, fp)); }
            }
            const bool take = (k == 0) || (norms < best_val);
            best_val = take ? norms : best_val;
            best = take ? k : best;
        }
        RSC_UNROLL for (int r = 0; r < 3; ++r) {
            RSC_UNROLL for (int c = 0; c < 3; ++c) R[r][c] = ((best >= 2) && c < 2) ? -Ro[r][c] : Ro[r][c];
            t[r] = (best & 1) ? -tv[r] : tv[r];
        }
    } else {
        const double tmp[3][3] = {{r1[0], r1[3], r1[6]}, {r1[1], r1[4], r1[7]}, {r1[2], r1[5], r1[8]}};
        const double c0[3] = {r1[0], r1[1], r1[2]}, c1[3] = {r1[3], r1[4], r1[5]}, c2[3] = {r1[6], r1[7], r1[8]};
        const double scale = 1.0 / dm::pow_1_3(rabs(ml_norm3(c0) * ml_norm3(c1) * ml_norm3(c2)));  // :567
        ml_nearest_rotation(tmp, R);
        if (ml_det3(R) < 0) RSC_UNROLL for (int r = 0; r < 3; ++r) RSC_UNROLL for (int c = 0; c < 3; ++c) R[r][c] *= -1.0;
        const double ts[3] = {scale * r1[9], scale * r1[10], scale * r1[11]};
        double tv[3];
        RSC_UNROLL for (int r = 0; r < 3; ++r) tv[r] = emv3d_row(r, R[r][0] * ts[0], R[r][1] * ts[1], R[r][2] * ts[2]);
        double err[2], Ti[2][4][4];
        RSC_UNROLL for (int s = 0; s < 2; ++s) {
            const double T4[4][4] = {{R[0][0], R[0][1], R[0][2], s ? -tv[0] : tv[0]},
                                     {R[1][0], R[1][1], R[1][2], s ? -tv[1] : tv[1]},
                                     {R[2][0], R[2][1], R[2][2], s ? -tv[2] : tv[2]},
                                     {0.0, 0.0, 0.0, 1.0}};
            ml_inverse4(T4, Ti[s]);
            err[s] = 0.0;
            RSC_UNROLL for (int p = 0; p < 6; ++p) {
                double v[3];
                RSC_UNROLL for (int r = 0; r < 3; ++r)
                    v[r] = emv3d_row(r, Ti[s][r][0] * in.pw(p, 0), Ti[s][r][1] * in.pw(p, 1), Ti[s][r][2] * in.pw(p, 2)) +
                           Ti[s][r][3];
                const double nv = ml_norm3(v);
                RSC_UNROLL for (int r = 0; r < 3; ++r) v[r] = v[r] / nv;
                { const double fp[3] = {in.f(p, 0), in.f(p, 1), in.f(p, 2)}; err[s] += (1.0 - ml_dot3(v, fp)); }
            }
        }
        const bool k0 = err[0] < err[1];
        RSC_UNROLL for (int r = 0; r < 3; ++r) {
            t[r] = k0 ? Ti[0][r][3] : Ti[1][r][3];
            RSC_UNROLL for (int c = 0; c < 3; ++c) R[r][c] = Ti[0][r][c];
        }
    }
    RSC_ML_STAMP(4);
    // Gauss-Newton (mlpnp_gn); J rows in the W region, A = J^T J (or J^T Kll J) in the V region
    double x[6];
    {
        double w3[3];
        ml_rot2rodrigues(R, w3);
        x[0] = w3[0]; x[1] = w3[1]; x[2] = w3[2];
        x[3] = t[0]; x[4] = t[1]; x[5] = t[2];
    }
    // J(r, k) = e(r*6 + k), r < 2*NS; g right after J; the 6x6 system (+ temp row 6) after g: the
    // Gauss-Newton slab is ml_gn_slab<NS>() doubles
    const MlView Jv{slab.base, slab.stride, 0};
    const MlView Av{slab.base, slab.stride, 12 * NS + 6};
    int it = 0;
    bool stop = false;
    while (it < 5 && !stop) {
        double Rg[3][3];
        const double w3[3] = {x[0], x[1], x[2]};
        ml_rodrigues2rot(w3, Rg);
        // mlpnpJacs' w-only temporaries, once per iteration, parked after the system (rsc_mlpnp_jac.h)
        const MlJacWStrided JW{{slab.base + 12 * NS * slab.stride, slab.stride}};
        {
            MlJacWStrided JWw = JW;
            mlpnp_jac_w<MlJacDeviceLibm>(x, JWw);
        }
        double rr[2 * NS];
        RSC_UNROLL for (int i = 0; i < NS; ++i) {
            double pc[3];
            RSC_UNROLL for (int k = 0; k < 3; ++k)
                pc[k] = emv3d_row(k, Rg[k][0] * jin.pw(i, 0), Rg[k][1] * jin.pw(i, 1), Rg[k][2] * jin.pw(i, 2)) + x[3 + k];
            const double nrm = ml_norm3(pc);
            RSC_UNROLL for (int k = 0; k < 3; ++k) pc[k] = pc[k] / nrm;
            const double nr[3] = {jin.ns(i, 0, 0), jin.ns(i, 1, 0), jin.ns(i, 2, 0)};
            const double ns[3] = {jin.ns(i, 0, 1), jin.ns(i, 1, 1), jin.ns(i, 2, 1)};
            rr[2 * i] = ml_dot3(nr, pc);
            rr[2 * i + 1] = ml_dot3(ns, pc);
        }
        // the Jacobian rows (mlpnpJacs, MLPnPsolver.cpp:749-767), one correspondence at a time: its
        // ~200 temporaries are live for that correspondence only
#pragma unroll 1
        for (int i = 0; i < NS; ++i) {
            const double nr[3] = {jin.ns(i, 0, 0), jin.ns(i, 1, 0), jin.ns(i, 2, 0)};
            const double ns[3] = {jin.ns(i, 0, 1), jin.ns(i, 1, 1), jin.ns(i, 2, 1)};
            const double pwi[3] = {jin.pw(i, 0), jin.pw(i, 1), jin.pw(i, 2)};
            double J[2][6];
            mlpnp_jac_pt<MlJacDeviceLibm>(JW, pwi, nr, ns, x + 3, x, J);
            RSC_UNROLL for (int k = 0; k < 6; ++k) {
                Jv.e((2 * i) * 6 + k) = J[0][k];
                Jv.e((2 * i + 1) * 6 + k) = J[1][k];
            }
            RSC_LOOP_FENCE();
        }
        // J^T J (or J^T Kll J) and J^T r one row a at a time; where registers are short (covariances,
        // NS > 6) the row loop stays rolled, so J stays in the slab instead of 2 NS x 6 doubles of
        // VGPRs; g[a] waits in the J region's spare rows (e >= 2 NS * 6)
        constexpr int kG = 12 * NS;
        auto row = [&](int a) {
            if constexpr (Cov::on) {
                // JacTSKll = J^T Kll: (k, 2i + q) = J(2i, k) P_i(0, q) + J(2i + 1, k) P_i(1, q)
                double jk[2 * NS];
                RSC_UNROLL for (int i = 0; i < NS; ++i)
                    RSC_UNROLL for (int q = 0; q < 2; ++q)
                        jk[2 * i + q] = Jv.e((2 * i) * 6 + a) * in.pwgt(i, q) + Jv.e((2 * i + 1) * 6 + a) * in.pwgt(i, 2 + q);
                RSC_UNROLL for (int b = 0; b < 6; ++b) {
                    double s = jk[0] * Jv.e(b);
                    RSC_UNROLL for (int q = 1; q < 2 * NS; ++q) s = s + jk[q] * Jv.e(q * 6 + b);
                    Av.at(a, b) = s;
                }
                double s = jk[0] * rr[0];
                RSC_UNROLL for (int q = 1; q < 2 * NS; ++q) s = s + jk[q] * rr[q];
                Jv.e(kG + a) = s;
            } else {
                RSC_UNROLL for (int b = 0; b < 6; ++b) {
                    double s = Jv.e(a) * Jv.e(b);
                    RSC_UNROLL for (int q = 1; q < 2 * NS; ++q) s = s + Jv.e(q * 6 + a) * Jv.e(q * 6 + b);
                    Av.at(a, b) = s;
                }
                double s = Jv.e(a) * rr[0];
                RSC_UNROLL for (int q = 1; q < 2 * NS; ++q) s = s + Jv.e(q * 6 + a) * rr[q];
                Jv.e(kG + a) = s;
            }
        };
        if constexpr (Cov::on || NS > 6) {
#pragma unroll 1
            for (int a = 0; a < 6; ++a) row(a);
        } else {
            RSC_UNROLL for (int a = 0; a < 6; ++a) row(a);
        }
        double g[6];
        RSC_UNROLL for (int a = 0; a < 6; ++a) g[a] = Jv.e(kG + a);
        double dx[6];
        ml_ldlt_solve6(Av, g, dx);
        double mx = rabs(dx[0]), mn = rabs(dx[0]);
        RSC_UNROLL for (int k = 1; k < 6; ++k) {
            const double v = rabs(dx[k]);
            mx = (mx < v) ? v : mx;
            mn = (v < mn) ? v : mn;
        }
        if (mx > 5.0 || mn > 1.0) {
            stop = true;
        } else {
            double dlm = 0.0;
            RSC_UNROLL for (int q = 0; q < 2 * NS; ++q) {
                double s = Jv.e(q * 6) * dx[0];
                RSC_UNROLL for (int k = 1; k < 6; ++k) s = s + Jv.e(q * 6 + k) * dx[k];
                const double v = rabs(s);
                dlm = (q == 0) ? v : ((dlm < v) ? v : dlm);
            }
            RSC_UNROLL for (int k = 0; k < 6; ++k) x[k] = x[k] - dx[k];
            if (dlm < 1e-5) stop = true;
            ++it;
        }
        RSC_LOOP_FENCE();
    }
    const double wf[3] = {x[0], x[1], x[2]};
    ml_rodrigues2rot(wf, Rout);
    tout[0] = x[3];
    tout[1] = x[4];
    tout[2] = x[5];
}

// MLPnPsolver::computePose for NS correspondences (pts world, f bearings), result R (row-major), t,
// one lane (the sequential composition; the host emulation tests it and the quad kernel runs the same
// phases with the 12x12 SVD spread over four lanes).  S: the lane slab (kMlSlabDoubles doubles,
// element stride S.stride): the normal matrix and V of the JacobiSVD, then J and the LDLT system.
template <int NS, class Cov = MlNoCov>
RSC_HD void mlpnp_compute_pose(const double (&pw)[NS][3], const double (&f)[NS][3], const LaneMat& slab,
                               double (&Rout)[3][3], double (&tout)[3], const Cov& cov = Cov()) {
    MlPrep<NS, Cov> m;
    mlpnp_prepare<NS, Cov>(pw, f, cov, m);
    const int colsA = m.planar ? 9 : 12;
    const MlView W{slab.base, slab.stride, 0}, V{slab.base, slab.stride, 144};
    RSC_UNROLL for (int a = 0; a < 12; ++a)
        RSC_UNROLL for (int b = 0; b < 12; ++b) {
            if (a < colsA && b < colsA) {
                double ra[NS][2], rb[NS][2];
                RSC_UNROLL for (int i = 0; i < NS; ++i)
                    RSC_UNROLL for (int s2 = 0; s2 < 2; ++s2) {
                        ra[i][s2] = mlpnp_A<NS, Cov>(m, i, s2, a);
                        rb[i][s2] = mlpnp_A<NS, Cov>(m, i, s2, b);
                    }
                W.at(a, b) = mlpnp_normal_entry<NS, Cov>(m, ra, rb);
            }
        }
    double r1[12];
    ml_jacobi_svd_lds(W, V, colsA, r1);
    const MlRegs<NS, Cov> in{pw, f, m};
    mlpnp_finish_pose<NS, Cov>(in, in, r1, slab, Rout, tout);
}

// MLPnPsolver::CheckInliers for one correspondence (MLPnPsolver.cpp:222-255).
RSC_HD bool mlpnp_inlier(const double (&R)[9], const double (&t)[3], float fx, float fy, float cx, float cy,
                         float X, float Y, float Z, float u, float v, float maxErr) {
    const float xc = (float)(R[0] * X + R[1] * Y + R[2] * Z + t[0]);
    const float yc = (float)(R[3] * X + R[4] * Y + R[5] * Z + t[1]);
    const float zc = (float)(R[6] * X + R[7] * Y + R[8] * Z + t[2]);
    const float ue = fx * xc / zc + cx;
    const float ve = fy * yc / zc + cy;
    const float dX = u - ue, dY = v - ve;
    return dX * dX + dY * dY < maxErr;
}

}  // namespace rsc
