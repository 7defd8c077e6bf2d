// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Restatement of the Eigen dense algorithms the reference solvers call.  Eigen is NOT vendored in
// the reference and is absent from this container; the version inferred from the
// reference's build (Ubuntu 20.04: Eigen 3.3.7) is restated from its published algorithms:
//   * SelfAdjointEigenSolver::compute  — scale to [-1,1], Householder tridiagonalisation (closed
//     form for 3x3), implicit symmetric QR with Wilkinson shift, ascending selection sort.
//     Used at PnPsolver.cpp:311 (3x3 double), :380 (12x12 double), :469 (4x4 double) and
//     Sim3Solver.cpp:238-239 (4x4 float).
//   * JacobiSVD (what MatrixXd::bdcSvd() falls back to below 16 columns) with the default
//     ColPivHouseholderQR preconditioner, ThinU|ThinV, and SVDBase::solve — PnPsolver.cpp:531,559,590.
//   * Matrix3d::inverse (cofactors) — PnPsolver.cpp:331.
//   * Quaternion::toRotationMatrix — PnPsolver.cpp:478, Sim3Solver.cpp:248.
//
// ARITHMETIC CONTRACT (shared with the HIP kernels; see DESIGN.md §"Arithmetic contract"):
// Sums are evaluated left to right in index order, starting from the first term (or from 0.0
// where the reference itself starts from setZero()) — EXCEPT the 3-term reductions of fixed-size
// Eigen expressions, which follow Eigen 3.3's evaluation on the reference's x86-64 SSE2 build
// (round 4, profiles/r04/order_choice.json): a reduction that cannot use packets (a dot / squared
// norm / product coefficient over a row of a column-major matrix, or any float 3-vector: 3 < 4
// lanes) is redux_novec_unroller's halving tree a0 + (a1 + a2) (`ered3`); a Matrix3d * Vector3d
// assigned to a Vector3d evaluates rows 0-1 as one Packet2d multiply-add chain in index order and
// row 2 by the coefficient path (halving).  Dynamic-size reductions (column sums, M^T M) stay left
// to right: their order depends on the run-time alignment and GEMM blocking.
// -DORA_LTR_ORDER restores the rounds 1-3 left-to-right order everywhere (tools/oracle_ab.py A/B).
// No FMA contraction (-ffp-contract=off), IEEE division and sqrt.
#pragma once
#include <cmath>
#include <cfloat>
#include <cstring>
#include <limits>
#include <algorithm>

namespace rsc_oracle {

template <typename S> struct Lim;
template <> struct Lim<double> { static double eps() { return DBL_EPSILON; } static double min() { return DBL_MIN; } };
template <> struct Lim<float>  { static float eps() { return FLT_EPSILON; }  static float min() { return FLT_MIN; } };

template <typename S> static inline S ab(S x) { return std::fabs(x); }

// 3-term reduction of a non-vectorisable fixed-size Eigen expression (see the contract above).
#ifndef ORA_LTR_ORDER
template <typename S> static inline S ered3(S a0, S a1, S a2) { return a0 + (a1 + a2); }
#else
template <typename S> static inline S ered3(S a0, S a1, S a2) { return a0 + a1 + a2; }
#endif
// Row r of Matrix3d * Vector3d into a Vector3d: rows 0-1 one Packet2d chain, row 2 coefficient-wise.
template <typename S> static inline S emv3d_row(int r, S a0, S a1, S a2) { return r < 2 ? (a0 + a1) + a2 : ered3(a0, a1, a2); }
template <typename S> static inline S sq(S x) { return x * x; }

// Eigen numext::hypot (MathFunctions.h, hypot_impl) for real scalars.
template <typename S> static inline S eig_hypot(S x, S y) {
    S ax = ab(x), ay = ab(y), p, qp;
    if (ax > ay) { p = ax; qp = ay / p; } else { p = ay; qp = ax / p; }
    if (p == S(0)) return S(0);
    return p * std::sqrt(S(1) + qp * qp);
}

// JacobiRotation::makeGivens (Jacobi.h) for real scalars.
template <typename S> static inline void make_givens(S p, S q, S& c, S& s) {
    if (q == S(0)) {
        c = p < S(0) ? S(-1) : S(1);
        s = S(0);
    } else if (p == S(0)) {
        c = S(0);
        s = q < S(0) ? S(1) : S(-1);
    } else if (ab(p) > ab(q)) {
        S t = q / p;
        S u = std::sqrt(S(1) + t * t);
        if (p < S(0)) u = -u;
        c = S(1) / u;
        s = -t * c;
    } else {
        S t = p / q;
        S u = std::sqrt(S(1) + t * t);
        if (q < S(0)) u = -u;
        s = -S(1) / u;
        c = -t * s;
    }
}

// ---------------------------------------------------------------------------------------------
// SelfAdjointEigenSolver<Matrix<S,n,n>>::compute(A) — eigenvalues ascending in w[], eigenvector of
// w[j] in column j of V (V[i][j]).  Only the lower triangle of A is read.  Returns true on
// "Success" (the sort is skipped otherwise, as in Eigen).
// ---------------------------------------------------------------------------------------------
template <typename S, int n>
struct SymEig {
    S V[n][n];
    S w[n];
    bool ok;
};

// Householder reflector of v[0..len-1] (MatrixBase::makeHouseholder): returns tau, beta and the
// essential part written back into v[1..].
template <typename S>
static inline void make_householder(S* v, int stride, int len, S& tau, S& beta) {
    S tailSqNorm = S(0);
    if (len > 1) {
        tailSqNorm = sq(v[stride]);
        for (int k = 2; k < len; ++k) tailSqNorm = tailSqNorm + sq(v[k * stride]);
    }
    S c0 = v[0];
    const S tol = Lim<S>::min();
    if (tailSqNorm <= tol) {
        tau = S(0);
        beta = c0;
        for (int k = 1; k < len; ++k) v[k * stride] = S(0);
    } else {
        beta = std::sqrt(c0 * c0 + tailSqNorm);
        if (c0 >= S(0)) beta = -beta;
        S den = c0 - beta;
        for (int k = 1; k < len; ++k) v[k * stride] = v[k * stride] / den;
        tau = (beta - c0) / beta;
    }
}

// tridiagonal_qr_step (SelfAdjointEigenSolver.h) on diag/subdiag with Q (n x n, row-major) updated
// by Q = Q * G on columns k,k+1.
template <typename S, int n>
static inline void tridiagonal_qr_step(S* diag, S* subdiag, int start, int end, S (*Q)[n]) {
    S td = (diag[end - 1] - diag[end]) * S(0.5);
    S e = subdiag[end - 1];
    S mu = diag[end];
    if (td == S(0)) {
        mu -= ab(e);
    } else {
        S e2 = sq(subdiag[end - 1]);
        S h = eig_hypot(td, e);
        if (e2 == S(0))
            mu -= (e / (td + (td > S(0) ? S(1) : S(-1)))) * (e / h);
        else
            mu -= e2 / (td + (td > S(0) ? h : -h));
    }
    S x = diag[start] - mu;
    S z = subdiag[start];
    for (int k = start; k < end; ++k) {
        S c, s;
        make_givens(x, z, c, s);
        S sdk = s * diag[k] + c * subdiag[k];
        S dkp1 = s * subdiag[k] + c * diag[k + 1];
        diag[k] = c * (c * diag[k] - s * subdiag[k]) - s * (c * subdiag[k] - s * diag[k + 1]);
        diag[k + 1] = s * sdk + c * dkp1;
        subdiag[k] = c * sdk - s * dkp1;
        if (k > start) subdiag[k - 1] = c * subdiag[k - 1] - s * z;
        x = subdiag[k];
        if (k < end - 1) {
            z = -s * subdiag[k + 1];
            subdiag[k + 1] = c * subdiag[k + 1];
        }
        // q.applyOnTheRight(k,k+1,rot): x' = c*x - s*y, y' = s*x + c*y
        if (!(c == S(1) && s == S(0))) {
            for (int i = 0; i < n; ++i) {
                S xi = Q[i][k], yi = Q[i][k + 1];
                Q[i][k] = c * xi - s * yi;
                Q[i][k + 1] = s * xi + c * yi;
            }
        }
    }
}

template <typename S, int n>
static SymEig<S, n> sym_eig(const S (*A)[n]) {
    SymEig<S, n> out;
    S (*mat)[n] = out.V;
    // mat = A.triangularView<Lower>()
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) mat[i][j] = (i >= j) ? A[i][j] : S(0);
    // scale = mat.cwiseAbs().maxCoeff()  (column-major visit order, strict '>')
    S scale = ab(mat[0][0]);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            if (i == 0 && j == 0) continue;
            S v = ab(mat[i][j]);
            if (v > scale) scale = v;
        }
    if (scale == S(0)) scale = S(1);
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) mat[i][j] = mat[i][j] / scale;

    S diag[n], subdiag[n > 1 ? n - 1 : 1];
    if (n == 3) {
        // tridiagonalization_inplace_selector<MatrixType,3,false>
        const S tol = Lim<S>::min();
        diag[0] = mat[0][0];
        S v1norm2 = sq(mat[2][0]);
        if (v1norm2 <= tol) {
            diag[1] = mat[1][1];
            diag[2] = mat[2][2];
            subdiag[0] = mat[1][0];
            subdiag[1] = mat[2][1];
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < n; ++j) mat[i][j] = (i == j) ? S(1) : S(0);
        } else {
            S beta = std::sqrt(sq(mat[1][0]) + v1norm2);
            S invBeta = S(1) / beta;
            S m01 = mat[1][0] * invBeta;
            S m02 = mat[2][0] * invBeta;
            S q = S(2) * m01 * mat[2][1] + m02 * (mat[2][2] - mat[1][1]);
            diag[1] = mat[1][1] + m02 * q;
            diag[2] = mat[2][2] - m02 * q;
            subdiag[0] = beta;
            subdiag[1] = mat[2][1] - m01 * q;
            S Q3[3][3] = {{S(1), S(0), S(0)}, {S(0), m01, m02}, {S(0), m02, -m01}};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) mat[i][j] = Q3[i][j];
        }
    } else {
        // tridiagonalization_inplace(matA, hCoeffs) (Tridiagonalization.h)
        S hC[n];
        for (int i = 0; i < n - 1; ++i) {
            const int rs = n - i - 1;
            S h, beta;
            make_householder(&mat[i + 1][i], n, rs, h, beta);
            mat[i + 1][i] = S(1);
            S v[n], w[n], hc[n];
            for (int k = 0; k < rs; ++k) v[k] = mat[i + 1 + k][i];
            for (int k = 0; k < rs; ++k) w[k] = h * v[k];
            // hCoeffs.tail = bottomRightCorner.selfadjointView<Lower>() * (h * v)
            for (int k = 0; k < rs; ++k) {
                S acc = S(0);
                for (int m = 0; m < rs; ++m) {
                    const int r = i + 1 + k, c = i + 1 + m;
                    S a = (r >= c) ? mat[r][c] : mat[c][r];
                    acc = (m == 0) ? a * w[m] : acc + a * w[m];
                }
                hc[k] = acc;
            }
            // hCoeffs.tail += (h * -0.5 * dot(hCoeffs.tail, v)) * v
            S dot = hc[0] * v[0];
            for (int k = 1; k < rs; ++k) dot = dot + hc[k] * v[k];
            S alpha = (h * S(-0.5)) * dot;
            for (int k = 0; k < rs; ++k) hc[k] = hc[k] + alpha * v[k];
            // selfadjointView<Lower>().rankUpdate(v, hc, -1): A += -v hc^T - hc v^T (lower)
            for (int c = 0; c < rs; ++c) {
                S s1 = -v[c];   // conj(alpha) * conj(u(c)), alpha = -1
                S s2 = -hc[c];  // alpha * conj(v(c))
                for (int r = c; r < rs; ++r)
                    mat[i + 1 + r][i + 1 + c] = mat[i + 1 + r][i + 1 + c] + (s1 * hc[r] + s2 * v[r]);
            }
            mat[i + 1][i] = beta;
            hC[i] = h;
        }
        for (int k = 0; k < n; ++k) diag[k] = mat[k][k];
        for (int k = 0; k < n - 1; ++k) subdiag[k] = mat[k + 1][k];
        // mat = HouseholderSequence(mat, hCoeffs).setLength(n-1).setShift(1)  (in-place evalTo)
        for (int i = 0; i < n; ++i) {
            mat[i][i] = S(1);
            for (int j = i + 1; j < n; ++j) mat[i][j] = S(0);
        }
        for (int k = n - 2; k >= 0; --k) {
            const int cs = n - k - 1;  // corner rows/cols k+1..n-1
            const int b0 = k + 1;
            const S tau = hC[k];
            if (cs == 1) {
                mat[b0][b0] = mat[b0][b0] * (S(1) - tau);
            } else if (tau != S(0)) {
                // essential = mat[k+2..n-1][k]
                S tmp[n];
                for (int c = 0; c < cs; ++c) {
                    S acc = mat[k + 2][k] * mat[b0 + 1][b0 + c];
                    for (int r = 1; r < cs - 1; ++r) acc = acc + mat[k + 2 + r][k] * mat[b0 + 1 + r][b0 + c];
                    tmp[c] = acc + mat[b0][b0 + c];
                }
                for (int c = 0; c < cs; ++c) mat[b0][b0 + c] = mat[b0][b0 + c] - tau * tmp[c];
                for (int r = 0; r < cs - 1; ++r) {
                    S te = tau * mat[k + 2 + r][k];
                    for (int c = 0; c < cs; ++c) mat[b0 + 1 + r][b0 + c] = mat[b0 + 1 + r][b0 + c] - tmp[c] * te;
                }
            }
            for (int r = k + 1; r < n; ++r) mat[r][k] = S(0);
        }
    }

    // computeFromTridiagonal_impl
    const int maxIterations = 30;
    int end = n - 1, start = 0, iter = 0;
    const S considerAsZero = Lim<S>::min();
    const S precision_inv = S(1) / Lim<S>::eps();
    while (end > 0) {
        for (int i = start; i < end; ++i) {
            if (ab(subdiag[i]) < considerAsZero) {
                subdiag[i] = S(0);
            } else {
                const S scaled = precision_inv * subdiag[i];
                if (scaled * scaled <= (ab(diag[i]) + ab(diag[i + 1]))) subdiag[i] = S(0);
            }
        }
        while (end > 0 && subdiag[end - 1] == S(0)) end--;
        if (end <= 0) break;
        iter++;
        if (iter > maxIterations * n) break;
        start = end - 1;
        while (start > 0 && subdiag[start - 1] != S(0)) start--;
        tridiagonal_qr_step<S, n>(diag, subdiag, start, end, mat);
    }
    out.ok = (iter <= maxIterations * n);
    if (out.ok) {
        for (int i = 0; i < n - 1; ++i) {
            int k = 0;
            S mn = diag[i];
            for (int j = 1; j < n - i; ++j)
                if (diag[i + j] < mn) { mn = diag[i + j]; k = j; }
            if (k > 0) {
                std::swap(diag[i], diag[k + i]);
                for (int r = 0; r < n; ++r) std::swap(mat[r][i], mat[r][k + i]);
            }
        }
    }
    for (int i = 0; i < n; ++i) out.w[i] = diag[i] * scale;
    return out;
}

// ---------------------------------------------------------------------------------------------
// JacobiSVD<MatrixXd>(A, ComputeThinU|ComputeThinV).solve(b) for a 6 x k matrix, k < 6.
// (BDCSVD::compute delegates to JacobiSVD when cols < 16; the default QR preconditioner is
// ColPivHouseholderQRPreconditioner, which runs because rows > cols.)
// A is row-major A[r][c], r < 6, c < k.  x receives k values.
// ---------------------------------------------------------------------------------------------
template <int k>
static void jacobi_svd_solve_6xk(const double (*Ain)[k], const double* b, double* x) {
    const int rows = 6;
    const double eps = DBL_EPSILON;
    const double precision = 2.0 * eps;
    const double considerAsZero = DBL_MIN;
    // scale = matrix.cwiseAbs().maxCoeff() (column-major order, strict '>')
    double scale = ab(Ain[0][0]);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < rows; ++r) {
            if (r == 0 && c == 0) continue;
            double v = ab(Ain[r][c]);
            if (v > scale) scale = v;
        }
    if (scale == 0.0) scale = 1.0;
    double qr[6][k];
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < k; ++c) qr[r][c] = Ain[r][c] / scale;

    // --- ColPivHouseholderQR::computeInPlace ---
    double hCoeffs[k], normsUpd[k], normsDir[k];
    int transp[k];
    for (int c = 0; c < k; ++c) {
        double s = sq(qr[0][c]);
        for (int r = 1; r < rows; ++r) s = s + sq(qr[r][c]);
        normsDir[c] = std::sqrt(s);
        normsUpd[c] = normsDir[c];
    }
    double mx = normsUpd[0];
    for (int c = 1; c < k; ++c) if (normsUpd[c] > mx) mx = normsUpd[c];
    (void)mx;  // threshold_helper only feeds m_nonzero_pivots, which solve() does not use
    const double norm_downdate_threshold = std::sqrt(eps);
    for (int kk = 0; kk < k; ++kk) {
        int big = kk;
        double bv = normsUpd[kk];
        for (int c = kk + 1; c < k; ++c)
            if (normsUpd[c] > bv) { bv = normsUpd[c]; big = c; }
        transp[kk] = big;
        if (kk != big) {
            for (int r = 0; r < rows; ++r) std::swap(qr[r][kk], qr[r][big]);
            std::swap(normsUpd[kk], normsUpd[big]);
            std::swap(normsDir[kk], normsDir[big]);
        }
        double beta;
        make_householder(&qr[kk][kk], k, rows - kk, hCoeffs[kk], beta);
        qr[kk][kk] = beta;
        // bottomRightCorner(rows-kk, k-kk-1).applyHouseholderOnTheLeft(essential, tau)
        const double tau = hCoeffs[kk];
        const int bc = k - kk - 1;
        if (bc > 0 && tau != 0.0) {
            double tmp[k];
            for (int c = 0; c < bc; ++c) {
                double acc = qr[kk + 1][kk] * qr[kk + 1][kk + 1 + c];
                for (int r = 2; r < rows - kk; ++r) acc = acc + qr[kk + r][kk] * qr[kk + r][kk + 1 + c];
                tmp[c] = acc + qr[kk][kk + 1 + c];
            }
            for (int c = 0; c < bc; ++c) qr[kk][kk + 1 + c] = qr[kk][kk + 1 + c] - tau * tmp[c];
            for (int r = 1; r < rows - kk; ++r) {
                double te = tau * qr[kk + r][kk];
                for (int c = 0; c < bc; ++c) qr[kk + r][kk + 1 + c] = qr[kk + r][kk + 1 + c] - tmp[c] * te;
            }
        }
        for (int j = kk + 1; j < k; ++j) {
            if (normsUpd[j] != 0.0) {
                double temp = ab(qr[kk][j]) / normsUpd[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                double temp2 = temp * sq(normsUpd[j] / normsDir[j]);
                if (temp2 <= norm_downdate_threshold) {
                    double s = 0.0;
                    if (kk + 1 < rows) {
                        s = sq(qr[kk + 1][j]);
                        for (int r = kk + 2; r < rows; ++r) s = s + sq(qr[r][j]);
                    }
                    normsDir[j] = std::sqrt(s);
                    normsUpd[j] = normsDir[j];
                } else {
                    normsUpd[j] *= std::sqrt(temp);
                }
            }
        }
    }
    int perm[k];
    for (int c = 0; c < k; ++c) perm[c] = c;
    for (int kk = 0; kk < k; ++kk) std::swap(perm[kk], perm[transp[kk]]);

    // workMatrix = R (upper triangle), U = Q.leftCols(k), V = P
    double W[k][k], U[6][k], V[k][k];
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) W[r][c] = (c >= r) ? qr[r][c] : 0.0;
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < k; ++c) U[r][c] = (r == c) ? 1.0 : 0.0;
    for (int kk = k - 1; kk >= 0; --kk) {
        // U.bottomRows(rows-kk).applyHouseholderOnTheLeft(qr[kk+1..][kk], hCoeffs[kk])
        const double tau = hCoeffs[kk];
        if (tau != 0.0) {
            double tmp[k];
            for (int c = 0; c < k; ++c) {
                double acc = qr[kk + 1][kk] * U[kk + 1][c];
                for (int r = 2; r < rows - kk; ++r) acc = acc + qr[kk + r][kk] * U[kk + r][c];
                tmp[c] = acc + U[kk][c];
            }
            for (int c = 0; c < k; ++c) U[kk][c] = U[kk][c] - tau * tmp[c];
            for (int r = 1; r < rows - kk; ++r) {
                double te = tau * qr[kk + r][kk];
                for (int c = 0; c < k; ++c) U[kk + r][c] = U[kk + r][c] - tmp[c] * te;
            }
        }
    }
    for (int r = 0; r < k; ++r)
        for (int c = 0; c < k; ++c) V[r][c] = 0.0;
    for (int c = 0; c < k; ++c) V[perm[c]][c] = 1.0;

    // --- two-sided Jacobi sweeps ---
    double maxDiag = ab(W[0][0]);
    for (int i = 1; i < k; ++i) if (ab(W[i][i]) > maxDiag) maxDiag = ab(W[i][i]);
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < k; ++p) {
            for (int q = 0; q < p; ++q) {
                double pt = precision * maxDiag;
                double threshold = (considerAsZero < pt) ? pt : considerAsZero;
                if (ab(W[p][q]) > threshold || ab(W[q][p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd
                    double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                    double c1, s1;
                    double t = m00 + m11;
                    double d = m10 - m01;
                    if (ab(d) < DBL_MIN) {
                        s1 = 0.0; c1 = 1.0;
                    } else {
                        double u = t / d;
                        double tmp = std::sqrt(1.0 + u * u);
                        s1 = 1.0 / tmp;
                        c1 = u / tmp;
                    }
                    if (!(c1 == 1.0 && s1 == 0.0)) {
                        double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
                        m00 = c1 * x0 + s1 * y0; m10 = -s1 * x0 + c1 * y0;
                        m01 = c1 * x1 + s1 * y1; m11 = -s1 * x1 + c1 * y1;
                    }
                    // j_right.makeJacobi(m, 0, 1)
                    double cr, sr;
                    {
                        double xx = m00, yy = m01, zz = m11;
                        double deno = 2.0 * ab(yy);
                        if (deno < DBL_MIN) {
                            cr = 1.0; sr = 0.0;
                        } else {
                            double tau = (xx - zz) / deno;
                            double w = std::sqrt(tau * tau + 1.0);
                            double tt;
                            if (tau > 0.0) tt = 1.0 / (tau + w); else tt = 1.0 / (tau - w);
                            double sign_t = tt > 0.0 ? 1.0 : -1.0;
                            double nn = 1.0 / std::sqrt(tt * tt + 1.0);
                            sr = -sign_t * (yy / ab(yy)) * ab(tt) * nn;
                            cr = nn;
                        }
                    }
                    // j_left = rot1 * j_right.transpose()
                    double crt = cr, srt = -sr;
                    double cl = c1 * crt - s1 * srt;
                    double sl = c1 * srt + s1 * crt;
                    // W.applyOnTheLeft(p,q,j_left)
                    if (!(cl == 1.0 && sl == 0.0)) {
                        for (int c = 0; c < k; ++c) {
                            double xi = W[p][c], yi = W[q][c];
                            W[p][c] = cl * xi + sl * yi;
                            W[q][c] = -sl * xi + cl * yi;
                        }
                    }
                    // U.applyOnTheRight(p,q,j_left.transpose()) -> rotation j_left on columns
                    if (!(cl == 1.0 && sl == 0.0)) {
                        for (int r = 0; r < rows; ++r) {
                            double xi = U[r][p], yi = U[r][q];
                            U[r][p] = cl * xi + sl * yi;
                            U[r][q] = -sl * xi + cl * yi;
                        }
                    }
                    // W.applyOnTheRight(p,q,j_right), V.applyOnTheRight(p,q,j_right)
                    if (!(cr == 1.0 && sr == 0.0)) {
                        for (int r = 0; r < k; ++r) {
                            double xi = W[r][p], yi = W[r][q];
                            W[r][p] = cr * xi - sr * yi;
                            W[r][q] = sr * xi + cr * yi;
                        }
                        for (int r = 0; r < k; ++r) {
                            double xi = V[r][p], yi = V[r][q];
                            V[r][p] = cr * xi - sr * yi;
                            V[r][q] = sr * xi + cr * yi;
                        }
                    }
                    double a = ab(W[p][p]), bq = ab(W[q][q]);
                    double mm = (a < bq) ? bq : a;
                    maxDiag = (maxDiag < mm) ? mm : maxDiag;
                }
            }
        }
    }
    double sv[k];
    for (int i = 0; i < k; ++i) {
        double a = W[i][i];
        sv[i] = ab(a);
        if (a < 0.0)
            for (int r = 0; r < rows; ++r) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < k; ++i) sv[i] = sv[i] * scale;
    int nonzero = k;
    for (int i = 0; i < k; ++i) {
        int pos = 0;
        double mv = sv[i];
        for (int j = 1; j < k - i; ++j)
            if (sv[i + j] > mv) { mv = sv[i + j]; pos = j; }
        if (mv == 0.0) { nonzero = i; break; }
        if (pos) {
            pos += i;
            std::swap(sv[i], sv[pos]);
            for (int r = 0; r < rows; ++r) std::swap(U[r][pos], U[r][i]);
            for (int r = 0; r < k; ++r) std::swap(V[r][pos], V[r][i]);
        }
    }
    // SVDBase::rank() with the default threshold diagSize*epsilon
    double thr = sv[0] * ((double)k * eps);
    double premult = (thr < DBL_MIN) ? DBL_MIN : thr;
    int i = nonzero - 1;
    while (i >= 0 && sv[i] < premult) --i;
    const int rank = i + 1;
    double tmp[k];
    for (int j = 0; j < rank; ++j) {
        double acc = U[0][j] * b[0];
        for (int r = 1; r < rows; ++r) acc = acc + U[r][j] * b[r];
        tmp[j] = (1.0 / sv[j]) * acc;
    }
    for (int r = 0; r < k; ++r) {
        if (rank == 0) { x[r] = 0.0; continue; }
        double acc = V[r][0] * tmp[0];
        for (int j = 1; j < rank; ++j) acc = acc + V[r][j] * tmp[j];
        x[r] = acc;
    }
}

// Matrix3d::inverse() (InverseImpl.h, compute_inverse<...,3>): result(r,c) = cofactor(c,r) / det.
static inline void inverse3(const double m[3][3], double out[3][3]) {
    auto cof = [&](int i, int j) {
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
    };
    double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    double det = c0 * m[0][0] + c1 * m[1][0] + c2 * m[2][0];
    double invdet = 1.0 / det;
    out[0][0] = c0 * invdet; out[0][1] = c1 * invdet; out[0][2] = c2 * invdet;
    out[1][0] = cof(0, 1) * invdet; out[1][1] = cof(1, 1) * invdet; out[1][2] = cof(2, 1) * invdet;
    out[2][0] = cof(0, 2) * invdet; out[2][1] = cof(1, 2) * invdet; out[2][2] = cof(2, 2) * invdet;
}

// Quaternion<S>::toRotationMatrix (Quaternion.h).
template <typename S>
static inline void quat_to_R(S w, S x, S y, S z, S R[3][3]) {
    const S tx = S(2) * x, ty = S(2) * y, tz = S(2) * z;
    const S twx = tx * w, twy = ty * w, twz = tz * w;
    const S txx = tx * x, txy = ty * x, txz = tz * x;
    const S tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0][0] = S(1) - (tyy + tzz); R[0][1] = txy - twz;          R[0][2] = txz + twy;
    R[1][0] = txy + twz;          R[1][1] = S(1) - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy;          R[2][1] = tyz + twx;          R[2][2] = S(1) - (txx + tyy);
}

// MatrixBase::determinant for 3x3 (Determinant.h, bruteforce_det3_helper).
static inline double det3(const double m[3][3]) {
    auto h = [&](int a, int b, int c) { return m[0][a] * (m[1][b] * m[2][c] - m[1][c] * m[2][b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

}  // namespace rsc_oracle
