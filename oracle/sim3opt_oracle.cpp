// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
// Sequential restatement of Optimizer::OptimizeSim3 + the g2o code it runs (see the header).
#include "sim3opt_oracle.h"
#include "ora_libm.h"

#include <cfloat>
#include <cmath>
#include <limits>
#include <utility>
#include <vector>
#include "../orb-slam2-optimized_amd/csrc/rsc_math.h"

namespace rsc_oracle {
namespace {

struct Quat {
    double x, y, z, w;
};

// Quaterniond(const Matrix3d&) (Eigen quaternionbase_assign_impl<Matrix3>).
Quat quat_from_R(const double m[3][3]) {
    Quat q;
    double t = m[0][0] + m[1][1] + m[2][2];
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
        return q;
    }
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m[k][j] - m[j][k]) * t;
    c[j] = (m[j][i] + m[i][j]) * t;
    c[k] = (m[k][i] + m[i][k]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
    return q;
}

// Generic quat_product (Eigen Geometry/Quaternion.h).
Quat quat_mul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

void cross(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// Quaternion * Vector3 (QuaternionBase::_transformVector).
void quat_rotate(const Quat& q, const double v[3], double o[3]) {
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], c[3];
    cross(qv, v, uv);
    for (int i = 0; i < 3; ++i) uv[i] = uv[i] + uv[i];
    cross(qv, uv, c);
    for (int i = 0; i < 3; ++i) o[i] = v[i] + q.w * uv[i] + c[i];
}

// ---- g2o::Sim3 (types/sim3.h) --------------------------------------------------------------------
struct Sim3 {
    Quat r;
    double t[3];
    double s;
};

Sim3 sim3_mul(const Sim3& a, const Sim3& b) {  // operator*
    Sim3 r;
    r.r = quat_mul(a.r, b.r);
    double rb[3];
    quat_rotate(a.r, b.t, rb);
    for (int i = 0; i < 3; ++i) r.t[i] = a.s * rb[i] + a.t[i];
    r.s = a.s * b.s;
    return r;
}

Sim3 sim3_inverse(const Sim3& a) {  // Sim3(r.conjugate(), r.conjugate()*((-1./s)*t), 1./s)
    Sim3 r;
    r.r = {-a.r.x, -a.r.y, -a.r.z, a.r.w};
    const double f = -1. / a.s;
    const double mt[3] = {f * a.t[0], f * a.t[1], f * a.t[2]};
    quat_rotate(r.r, mt, r.t);
    r.s = 1. / a.s;
    return r;
}

void sim3_map(const Sim3& a, const double p[3], double o[3]) {  // s*(r*xyz) + t
    double rp[3];
    quat_rotate(a.r, p, rp);
    for (int i = 0; i < 3; ++i) o[i] = a.s * rp[i] + a.t[i];
}

void mat3_mul(const double A[3][3], const double B[3][3], double C[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}

// Sim3(const Vector7d& update): the exponential map (sim3.h constructor).
Sim3 sim3_exp(const double u[7]) {
    const double omega[3] = {u[0], u[1], u[2]};
    const double ups[3] = {u[3], u[4], u[5]};
    const double sigma = u[6];
    const double theta = std::sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
    const double Om[3][3] = {{0.0, -omega[2], omega[1]}, {omega[2], 0.0, -omega[0]}, {-omega[1], omega[0], 0.0}};
    Sim3 S;
    S.s = std::exp(sigma);
    double Om2[3][3];
    mat3_mul(Om, Om, Om2);
    double R[3][3];
    const double eps = 0.00001;
    double A, B, C;
    if (std::fabs(sigma) < eps) {
        C = 1;
        if (theta < eps) {
            A = 1. / 2.;
            B = 1. / 6.;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + Om[i][j]) + Om2[i][j];
        } else {
            const double st = ora_libm::sin(theta), ct = ora_libm::cos(theta);
            const double theta2 = theta * theta;
            A = (1 - ct) / (theta2);
            B = (theta - st) / (theta2 * theta);
            const double a = st / theta, b = (1 - ct) / (theta * theta);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + a * Om[i][j]) + b * Om2[i][j];
        }
    } else {
        C = (S.s - 1) / sigma;
        if (theta < eps) {
            const double sigma2 = sigma * sigma;
            A = ((sigma - 1) * S.s + 1) / sigma2;
            B = ((0.5 * sigma2 - sigma + 1) * S.s) / (sigma2 * sigma);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + Om[i][j]) + Om2[i][j];
        } else {
            const double st = ora_libm::sin(theta), ct = ora_libm::cos(theta);
            const double ra = st / theta, rb = (1 - ct) / (theta * theta);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + ra * Om[i][j]) + rb * Om2[i][j];
            const double a = S.s * st, b = S.s * ct;
            const double theta2 = theta * theta, sigma2 = sigma * sigma;
            const double c = theta2 + sigma2;
            A = (a * sigma + (1 - b) * theta) / (theta * c);
            B = (C - ((b - 1) * sigma + a * theta) / (c)) * 1. / (theta2);
        }
    }
    S.r = quat_from_R(R);
    double W[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) W[i][j] = (A * Om[i][j] + B * Om2[i][j]) + C * (i == j ? 1.0 : 0.0);
    for (int i = 0; i < 3; ++i) S.t[i] = W[i][0] * ups[0] + W[i][1] * ups[1] + W[i][2] * ups[2];
    return S;
}

// VertexSim3Expmap::oplusImpl with _fix_scale: update[6] = 0 (written into the caller's vector),
// estimate = Sim3(update) * estimate.
Sim3 oplus(double u[7], const Sim3& est) {
    u[6] = 0;
    return sim3_mul(sim3_exp(u), est);
}

// ---- Eigen::LDLT<MatrixXd> (ldlt_inplace<Lower>::unblocked + _solve_impl), n x n -------------------
template <int n>
bool ldlt_solve(double A[n][n], const double b[n], double x[n]) {
    enum { Zero, Pos, Neg, Indef } sign = Zero;
    int tr[n];
    double temp[n];
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = std::fabs(A[k][k]);
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(A[i][i]) > bv) { bv = std::fabs(A[i][i]); big = i; }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) std::swap(A[k][j], A[big][j]);
            for (int i = big + 1; i < n; ++i) std::swap(A[i][k], A[i][big]);
            std::swap(A[k][k], A[big][big]);
            for (int i = k + 1; i < big; ++i) {
                const double t = A[i][k];
                A[i][k] = A[big][i];
                A[big][i] = t;
            }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = A[j][j] * A[k][j];
            double acc = A[k][0] * temp[0];
            for (int j = 1; j < k; ++j) acc = acc + A[k][j] * temp[j];
            A[k][k] -= acc;
            for (int r = k + 1; r < n; ++r) {
                double a = A[r][0] * temp[0];
                for (int j = 1; j < k; ++j) a = a + A[r][j] * temp[j];
                A[r][k] -= a;
            }
        }
        const double akk = A[k][k];
        const bool valid = std::fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            sign = Zero;
            for (int j = 0; j < n; ++j) tr[j] = j;
            break;
        }
        if (rs > 0 && valid)
            for (int r = k + 1; r < n; ++r) A[r][k] /= akk;
        if (sign == Pos) {
            if (akk < 0.0) sign = Indef;
        } else if (sign == Neg) {
            if (akk > 0.0) sign = Indef;
        } else if (sign == Zero) {
            if (akk > 0.0) sign = Pos;
            else if (akk < 0.0) sign = Neg;
        }
    }
    if (!(sign == Pos || sign == Zero)) return false;  // isPositive()
    double y[n];
    for (int i = 0; i < n; ++i) y[i] = b[i];
    for (int k = 0; k < n; ++k) std::swap(y[k], y[tr[k]]);
    for (int i = 1; i < n; ++i) {
        double acc = A[i][0] * y[0];
        for (int j = 1; j < i; ++j) acc = acc + A[i][j] * y[j];
        y[i] -= acc;
    }
    const double tol = DBL_MIN;
    for (int i = 0; i < n; ++i) y[i] = (std::fabs(A[i][i]) > tol) ? y[i] / A[i][i] : 0.0;
    for (int i = n - 2; i >= 0; --i) {
        double acc = A[i + 1][i] * y[i + 1];
        for (int j = i + 2; j < n; ++j) acc = acc + A[j][i] * y[j];
        y[i] -= acc;
    }
    for (int k = n - 1; k >= 0; --k) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; ++i) x[i] = y[i];
    return true;
}

// ---- EdgeSim3ProjectXYZ (e12) / EdgeInverseSim3ProjectXYZ (e21) ----------------------------------
struct Edge {
    double X[3];    // the fixed point vertex (P3D2c for e12, P3D1c for e21)
    double obs[2];
    double inv;     // information = I * invSigmaSquare
    bool inverse;   // e21: uses the inverse Sim3 and camera 2
    double err[2];  // _error of the last computeError
    bool active;
};

struct Cam {
    double f[2], pp[2];  // VertexSim3Expmap::_focal_length, _principle_point (float K -> double)
};

// computeError at estimate S (Sinv = S.inverse(), precomputed for the e21 edges).
void edge_error(const Edge& e, const Sim3& S, const Sim3& Sinv, const Cam& K1, const Cam& K2, double out[2]) {
    double p[3];
    sim3_map(e.inverse ? Sinv : S, e.X, p);
    const double pr0 = p[0] / p[2], pr1 = p[1] / p[2];  // project()
    const Cam& K = e.inverse ? K2 : K1;
    const double r0 = pr0 * K.f[0] + K.pp[0], r1 = pr1 * K.f[1] + K.pp[1];  // cam_map1 / cam_map2
    out[0] = e.obs[0] - r0;
    out[1] = e.obs[1] - r1;
}

double chi2(const Edge& e) {  // _error.dot(information() * _error)
    const double w0 = e.inv * e.err[0] + 0.0 * e.err[1];
    const double w1 = 0.0 * e.err[0] + e.inv * e.err[1];
    return e.err[0] * w0 + e.err[1] * w1;
}

struct Huber {
    double delta, dsqr;
    void robustify(double e, double rho[3]) const {
        if (e <= dsqr) {
            rho[0] = e; rho[1] = 1.0; rho[2] = 0.0;
        } else {
            const double sqrte = std::sqrt(e);
            rho[0] = 2 * sqrte * delta - dsqr;
            rho[1] = delta / sqrte;
            rho[2] = -0.5 * rho[1] / e;
        }
    }
};

// pow(x, 3) as the correctly rounded cube (as oracle/poseopt_oracle.cpp).
double cube(double x) {
    const double p = x * x;
    const double e1 = std::fma(x, x, -p);
    const double c = p * x;
    const double e2 = std::fma(p, x, -c);
    return c + (e2 + e1 * x);
}

struct Problem {
    std::vector<Edge> edges;
    Cam K1, K2;
    Huber huber;
    double x[7] = {0, 0, 0, 0, 0, 0, 0};  // BlockSolver::_x: persists across iterations and optimize() calls
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0;
    Sim3OptStats st = {0, 0, 0, 0};

    void compute_active_errors(const Sim3& S) {
        const Sim3 Si = sim3_inverse(S);
        for (Edge& e : edges)
            if (e.active) edge_error(e, S, Si, K1, K2, e.err);
    }
    double active_robust_chi2() const {
        double chi = 0.0;
        for (const Edge& e : edges) {
            if (!e.active) continue;
            double rho[3];
            huber.robustify(chi2(e), rho);  // every edge carries a Huber kernel (Optimizer.cpp:1149,1165)
            chi += rho[0];
        }
        return chi;
    }
    // BlockSolverX::buildSystem: per active edge, the numeric Jacobian of the Sim3 vertex
    // (BaseBinaryEdge::linearizeOplus; the point vertex is fixed) and the robust quadratic form.
    void build_system(const Sim3& S, double H[7][7], double b[7]) const {
        for (int i = 0; i < 7; ++i) {
            b[i] = 0.0;
            for (int j = 0; j < 7; ++j) H[i][j] = 0.0;
        }
        const double delta = 1e-9;
        const double scalar = 1.0 / (2 * delta);
        // vj->push(); oplus(+-delta e_d); ...; pop(): the perturbed estimates are the same for every edge
        Sim3 Sp[7], Sm[7], Spi[7], Smi[7];
        for (int d = 0; d < 7; ++d) {
            double u[7] = {0, 0, 0, 0, 0, 0, 0};
            u[d] = delta;
            Sp[d] = oplus(u, S);
            u[d] = -delta;
            Sm[d] = oplus(u, S);
            Spi[d] = sim3_inverse(Sp[d]);
            Smi[d] = sim3_inverse(Sm[d]);
        }
        for (const Edge& e : edges) {
            if (!e.active) continue;
            double J[2][7];
            for (int d = 0; d < 7; ++d) {
                double ep[2], em[2];
                edge_error(e, Sp[d], Spi[d], K1, K2, ep);
                edge_error(e, Sm[d], Smi[d], K1, K2, em);
                J[0][d] = scalar * (ep[0] - em[0]);
                J[1][d] = scalar * (ep[1] - em[1]);
            }
            double rho[3];
            huber.robustify(chi2(e), rho);
            // omega_r = -omega * _error, *= rho[1]
            double omr0 = (-e.inv) * e.err[0] + (-0.0) * e.err[1];
            double omr1 = (-0.0) * e.err[0] + (-e.inv) * e.err[1];
            omr0 *= rho[1];
            omr1 *= rho[1];
            const double W[2][2] = {{rho[1] * e.inv, rho[1] * 0.0}, {rho[1] * 0.0, rho[1] * e.inv}};
            for (int i = 0; i < 7; ++i) b[i] += J[0][i] * omr0 + J[1][i] * omr1;
            for (int i = 0; i < 7; ++i) {
                const double t0 = J[0][i] * W[0][0] + J[1][i] * W[1][0];
                const double t1 = J[0][i] * W[0][1] + J[1][i] * W[1][1];
                for (int j = 0; j < 7; ++j) H[i][j] += t0 * J[0][j] + t1 * J[1][j];
            }
        }
    }

    enum Result { OK, Terminate };

    // OptimizationAlgorithmLevenberg::solve(iteration, online = false).
    Result lm_solve(int iteration, Sim3& S) {
        st.lm_iterations++;
        compute_active_errors(S);
        double currentChi = active_robust_chi2();
        double tempChi = currentChi;
        const double iniChi = currentChi;
        double H[7][7], b[7];
        build_system(S, H, b);
        if (iteration == 0) {
            double maxDiagonal = 0.;
            for (int j = 0; j < 7; ++j) maxDiagonal = std::max(std::fabs(H[j][j]), maxDiagonal);
            lambda = 1e-5 * maxDiagonal;
            ni = 2;
            nBadLM = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            st.lm_trials++;
            const Sim3 saved = S;  // push
            double Hd[7][7];
            for (int i = 0; i < 7; ++i)
                for (int j = 0; j < 7; ++j) Hd[i][j] = H[i][j];
            for (int i = 0; i < 7; ++i) Hd[i][i] += lambda;  // setLambda
            double xs[7];
            const bool ok2 = ldlt_solve<7>(Hd, b, xs);
            if (ok2)
                for (int i = 0; i < 7; ++i) x[i] = xs[i];
            S = oplus(x, S);  // _optimizer->update(x): zeroes x[6] in place
            compute_active_errors(S);
            tempChi = active_robust_chi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = (currentChi - tempChi);
            double scale = 0.;
            for (int j = 0; j < 7; ++j) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - cube(2 * rho - 1);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                S = saved;  // pop (the edges keep the errors of the rejected trial)
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) return Terminate;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
        else nBadLM = 0;
        if (nBadLM >= 3) return Terminate;
        return OK;
    }

    // initializeOptimization() + optimize(iterations).
    void optimize(int iterations, Sim3& S) {
        bool any = false;
        for (const Edge& e : edges) any |= e.active;
        if (!any) return;  // "0 vertices to optimize": returns -1
        bool ok = true;
        for (int i = 0; i < iterations && ok; i++) ok = (lm_solve(i, S) == OK);
    }
};

}  // namespace

int optimize_sim3(const Sim3OptInput& in, Sim3Est& S_io, uint8_t* keep, Sim3OptStats* stats) {
    Problem P;
    P.K1 = {{(double)in.K1[0], (double)in.K1[1]}, {(double)in.K1[2], (double)in.K1[3]}};
    P.K2 = {{(double)in.K2[0], (double)in.K2[1]}, {(double)in.K2[2], (double)in.K2[3]}};
    const float deltaHuber = std::sqrt(in.th2);  // float sqrt (Optimizer.cpp:1104)
    P.huber.delta = deltaHuber;
    P.huber.dsqr = P.huber.delta * P.huber.delta;
    std::vector<int> slot;
    for (int i = 0; i < in.n; ++i) {
        keep[i] = 1;
        if (!in.valid[i]) continue;
        // P3D1c = R1w*P3D1w + t1w, P3D2c = R2w*P3D2w + t2w in float, then cast<double>()
        float c1[3], c2[3];
        const float* a = in.X1w + 3 * (size_t)i;
        const float* b = in.X2w + 3 * (size_t)i;
        for (int r = 0; r < 3; ++r) {
            c1[r] = in.R1w[3 * r] * a[0] + in.R1w[3 * r + 1] * a[1] + in.R1w[3 * r + 2] * a[2] + in.t1w[r];
            c2[r] = in.R2w[3 * r] * b[0] + in.R2w[3 * r + 1] * b[1] + in.R2w[3 * r + 2] * b[2] + in.t2w[r];
        }
        Edge e12{{c2[0], c2[1], c2[2]}, {in.uv1[2 * i], in.uv1[2 * i + 1]}, (double)in.inv1[i], false, {0, 0}, true};
        Edge e21{{c1[0], c1[1], c1[2]}, {in.uv2[2 * i], in.uv2[2 * i + 1]}, (double)in.inv2[i], true, {0, 0}, true};
        P.edges.push_back(e12);
        P.edges.push_back(e21);
        slot.push_back(i);
    }
    const int nCorrespondences = (int)slot.size();
    P.st.n_correspondences = nCorrespondences;
    Sim3 S;
    S.r = {S_io.q[0], S_io.q[1], S_io.q[2], S_io.q[3]};
    for (int i = 0; i < 3; ++i) S.t[i] = S_io.t[i];
    S.s = S_io.s;
    P.optimize(5, S);
    int nBad = 0;
    for (int c = 0; c < nCorrespondences; ++c) {
        Edge& e12 = P.edges[2 * c];
        Edge& e21 = P.edges[2 * c + 1];
        if (chi2(e12) > in.th2 || chi2(e21) > in.th2) {
            keep[slot[c]] = 0;
            e12.active = e21.active = false;  // optimizer.removeEdge
            nBad++;
        }
    }
    P.st.n_bad = nBad;
    const int nMoreIterations = nBad > 0 ? 10 : 5;
    if (nCorrespondences - nBad < 10) {
        if (stats) *stats = P.st;
        return 0;
    }
    P.optimize(nMoreIterations, S);
    int nIn = 0;
    for (int c = 0; c < nCorrespondences; ++c) {
        const Edge& e12 = P.edges[2 * c];
        const Edge& e21 = P.edges[2 * c + 1];
        if (!e12.active) continue;
        if (chi2(e12) > in.th2 || chi2(e21) > in.th2) keep[slot[c]] = 0;
        else nIn++;
    }
    S_io.q[0] = S.r.x; S_io.q[1] = S.r.y; S_io.q[2] = S.r.z; S_io.q[3] = S.r.w;
    for (int i = 0; i < 3; ++i) S_io.t[i] = S.t[i];
    S_io.s = S.s;
    if (stats) *stats = P.st;
    return nIn;
}

}  // namespace rsc_oracle
