// rsc_sim3opt.h — Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) on the GPU: the g2o
// Levenberg-Marquardt of one VertexSim3Expmap (_fix_scale) over the EdgeSim3ProjectXYZ (x1 = S12 X2)
// and EdgeInverseSim3ProjectXYZ (x2 = S12^-1 X1) edges of the loop-closure correspondences, with
// Huber kernels (delta = sqrt(th2)): optimize(5), drop the correspondences with chi2 > th2, then
// optimize(5 or 10) again over the rest (LoopClosing.cpp:311 runs it after SearchBySim3).
//
// The vendored g2o declares no analytic Jacobian for these edges (types_seven_dof_expmap.h), so
// BaseBinaryEdge::linearizeOplus differentiates numerically: central differences with delta = 1e-9
// through VertexSim3Expmap::oplusImpl (Sim3(update) * estimate, update[6] forced to 0).  The 14
// perturbed estimates depend only on the current estimate, so they are built once per build pass
// (every lane redundantly, bit-identical) and every edge evaluates its error at all of them.
//
// Mapping (sim3opt.hip): one 256-thread workgroup per KeyFrame pair; thread t owns correspondence c
// (its two edges, terms 2c and 2c+1 of the g2o edge order e12_0, e21_0, e12_1, ...); every g2o sum
// over the active edges (activeRobustChi2, buildSystem's H/b) is folded in edge order on one lane
// per accumulator; the 7x7 LDLT and the LM control run redundantly in every lane.  g2o source
// followed: types/sim3.h, types/types_seven_dof_expmap.h, core/base_binary_edge.hpp,
// core/block_solver.hpp, solvers/linear_solver_dense.h, core/optimization_algorithm_levenberg.cpp,
// core/sparse_optimizer.cpp, core/robust_kernel_impl.cpp.  The oracle (oracle/sim3opt_oracle.cpp) is
// an independent sequential restatement; the two agree bit for bit.
#pragma once
#include "rsc_core.h"
#include "rsc_math.h"
#include "rsc_poseopt.h"

namespace rsc {

constexpr int kSim3OptMaxCorr = 8192;  // correspondences per pair
constexpr int kSim3OptTerms = 35;      // 28 lower-triangle H entries + 7 b entries

// The cooperative form (sim3opt.hip, RSC_SO_COOP): per pair one master workgroup (the LM control and
// the ordered folds) and helper workgroups that evaluate the edges' numeric Jacobians in chunks of 64
// active edges and hand them to the master through global memory (write-through, drained, flagged).
constexpr int kSoCoopChunk = 64;                                   // active edges per chunk
constexpr int kSoCoopJd = 17;                                      // doubles per edge: J (14), e0, e1, inv
constexpr int kSoCoopMaxChunks = 2 * kSim3OptMaxCorr / kSoCoopChunk;
constexpr int kSoCoopPub = 256;                                    // doubles per pair: S, S^-1, perturbed, me

// The polled words of one pair (zeroed before every launch).  Pass ids count from 1 within a launch;
// kSoCoopDone ends the helpers.
struct SoCoopFlags {
    unsigned long long claim;          // (pass << 32) | next unclaimed chunk
    unsigned pass;                     // the pass the master published last
    unsigned pad[13];
    unsigned ready[kSoCoopMaxChunks];  // pass id once chunk k of that pass is in the store
};
static_assert(sizeof(SoCoopFlags) % 16 == 0, "memset block");
constexpr unsigned kSoCoopDone = 0xffffffffu;

#if defined(__HIPCC__)
struct DevSim3OptProb {
    const float4* e12;   // [m] (P3D2c, invSigma2 of KF1's keypoint)   — edge x1 = S12 * X2
    const float4* e21;   // [m] (P3D1c, invSigma2 of KF2's keypoint)   — edge x2 = S21 * X1
    const float4* uv;    // [m] (kpUn1.pt, kpUn2.pt)
    uint8_t* keep;       // [m] in/out: 1 while the correspondence's edges are in the graph / inliers
    double* out;         // out [16]: q (x, y, z, w), t, s of g2oS12; then nIn, nBad, LM its, LM trials (int bits)
    int m;               // correspondences (>= 1)
    float th2;
    double delta;        // Huber delta: (double) of the float sqrt(th2) (Optimizer.cpp:1104)
    float K1[4], K2[4];  // fx, fy, cx, cy
    double S0[8];        // g2oS12 on entry
    // the cooperative form's per-pair hand-off (unused by the one-workgroup form)
    SoCoopFlags* cf;     // polled words
    double* cpub;        // [kSoCoopPub] the pass's estimate, its inverse, the perturbed estimates, me
    int* clist;          // [m] the kept correspondences of the current optimize()
    double* cstore;      // [ceil(2m / 64)][kSoCoopJd][64] the chunks' edge hand-offs
};
#endif

// ---- g2o::Sim3 (types/sim3.h) --------------------------------------------------------------------
struct SoSim3 {
    PoQuat r;
    double t[3];
    double s;
};

// operator*: r = r * other.r (generic quaternion product, not normalised), t = s*(r*other.t) + t.
RSC_HD SoSim3 so_mul(const SoSim3& a, const SoSim3& b) {
    SoSim3 o;
    o.r = po_quat_mul(a.r, b.r);
    double rb[3];
    po_rotate(a.r, b.t, rb);
    RSC_UNROLL for (int i = 0; i < 3; ++i) o.t[i] = a.s * rb[i] + a.t[i];
    o.s = a.s * b.s;
    return o;
}

// inverse(): Sim3(r.conjugate(), r.conjugate()*((-1./s)*t), 1./s).
RSC_HD SoSim3 so_inverse(const SoSim3& a) {
    SoSim3 o;
    o.r.x = -a.r.x;
    o.r.y = -a.r.y;
    o.r.z = -a.r.z;
    o.r.w = a.r.w;
    const double f = -1. / a.s;
    const double mt[3] = {f * a.t[0], f * a.t[1], f * a.t[2]};
    po_rotate(o.r, mt, o.t);
    o.s = 1. / a.s;
    return o;
}

// map(xyz) = s*(r*xyz) + t.
RSC_HD void so_map(const SoSim3& a, const double (&p)[3], double (&o)[3]) {
    double rp[3];
    po_rotate(a.r, p, rp);
    RSC_UNROLL for (int i = 0; i < 3; ++i) o[i] = a.s * rp[i] + a.t[i];
}

// Sim3(const Vector7d& update) for update[6] = 0 (sigma = 0: s = exp(0) = 1, C = 1) — the only form
// oplusImpl builds under _fix_scale.
RSC_HD SoSim3 so_exp_fixed_scale(const double (&u)[7]) {
    const double o0 = u[0], o1 = u[1], o2 = u[2];
    const double theta = sqrt(o0 * o0 + o1 * o1 + o2 * o2);
    const double Om[3][3] = {{0.0, -o2, o1}, {o2, 0.0, -o0}, {-o1, o0, 0.0}};
    double Om2[3][3];
    RSC_UNROLL for (int i = 0; i < 3; ++i)
        RSC_UNROLL for (int j = 0; j < 3; ++j) Om2[i][j] = Om[i][0] * Om[0][j] + Om[i][1] * Om[1][j] + Om[i][2] * Om[2][j];
    double R[3][3], A, B;
    const double C = 1;
    if (theta < 0.00001) {
        A = 1. / 2.;
        B = 1. / 6.;
        RSC_UNROLL for (int i = 0; i < 3; ++i)
            RSC_UNROLL for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + Om[i][j]) + Om2[i][j];
    } else {
        const double st = dm::sin(theta), ct = dm::cos(theta);
        const double theta2 = theta * theta;
        A = (1 - ct) / (theta2);
        B = (theta - st) / (theta2 * theta);
        const double a = st / theta, b = (1 - ct) / (theta * theta);
        RSC_UNROLL for (int i = 0; i < 3; ++i)
            RSC_UNROLL for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + a * Om[i][j]) + b * Om2[i][j];
    }
    SoSim3 S;
    S.r = po_quat_from_R(R);
    S.s = 1.0;
    RSC_UNROLL for (int i = 0; i < 3; ++i) {
        double W[3];
        RSC_UNROLL for (int j = 0; j < 3; ++j) W[j] = (A * Om[i][j] + B * Om2[i][j]) + C * (i == j ? 1.0 : 0.0);
        S.t[i] = W[0] * u[3] + W[1] * u[4] + W[2] * u[5];
    }
    return S;
}

// VertexSim3Expmap::oplusImpl (_fix_scale): update[6] = 0 in the caller's vector (the solver's x),
// estimate = Sim3(update) * estimate.
RSC_HD SoSim3 so_oplus(double (&u)[7], const SoSim3& est) {
    u[6] = 0;
    return so_mul(so_exp_fixed_scale(u), est);
}

struct SoCam {
    double f0, f1, p0, p1;  // _focal_length, _principle_point (mK entries, float -> double)
};

// computeError of EdgeSim3ProjectXYZ (S = the estimate, camera 1) or EdgeInverseSim3ProjectXYZ
// (S = estimate.inverse(), camera 2): obs - cam_map(project(S.map(X))).
RSC_HD void so_edge_error(const SoSim3& S, const SoCam& K, const double (&X)[3], double u, double v, double& e0,
                          double& e1) {
    double p[3];
    so_map(S, X, p);
    const double pr0 = p[0] / p[2], pr1 = p[1] / p[2];
    e0 = u - (pr0 * K.f0 + K.p0);
    e1 = v - (pr1 * K.f1 + K.p1);
}

// The 14 perturbed estimates of BaseBinaryEdge::linearizeOplus (d = 0..6, +delta then -delta) and
// their inverses (the e21 edges map with the inverse).
struct SoPerturbed {
    SoSim3 p[7], m[7], pi[7], mi[7];
};

RSC_HD void so_perturb(const SoSim3& S, SoPerturbed& P) {
    const double delta = 1e-9;
    RSC_UNROLL for (int d = 0; d < 7; ++d) {
        double u[7] = {0, 0, 0, 0, 0, 0, 0};
        u[d] = delta;
        P.p[d] = so_oplus(u, S);
        u[d] = -delta;
        P.m[d] = so_oplus(u, S);
        P.pi[d] = so_inverse(P.p[d]);
        P.mi[d] = so_inverse(P.m[d]);
    }
}

// linearizeOplus (numeric, the point vertex fixed): central differences of the edge error over the
// 14 perturbed estimates.
RSC_HD void so_jacobian(const SoPerturbed& P, bool inverse, const SoCam& K, const double (&X)[3], double u, double v,
                        double (&J)[2][7]) {
    const double scalar = 1.0 / (2 * 1e-9);
    RSC_UNROLL for (int d = 0; d < 7; ++d) {
        double a0, a1, b0, b1;
        so_edge_error(inverse ? P.pi[d] : P.p[d], K, X, u, v, a0, a1);
        so_edge_error(inverse ? P.mi[d] : P.m[d], K, X, u, v, b0, b1);
        J[0][d] = scalar * (a0 - b0);
        J[1][d] = scalar * (a1 - b1);
    }
}

// constructQuadraticForm (robust branch) of an edge with Jacobian J and _error (e0, e1):
// t[0..27] = lower triangle of B^T (rho1 omega) B (row-major i >= j), t[28..34] = B^T omega_r added to
// b (omega_r = -omega * error * rho1).
RSC_HD void so_quad_tail(const double (&J)[2][7], double inv, double e0, double e1, double delta, double dsqr,
                         double (&t)[kSim3OptTerms]) {
    double r0, rho1;
    po_huber(po_chi2(inv, false, e0, e1, 0.0), delta, dsqr, r0, rho1);
    double omr0 = (-inv) * e0 + (-0.0) * e1;
    double omr1 = (-0.0) * e0 + (-inv) * e1;
    omr0 *= rho1;
    omr1 *= rho1;
    const double Wd = rho1 * inv, Wo = rho1 * 0.0;
    int k = 0;
    RSC_UNROLL for (int i = 0; i < 7; ++i) {
        const double t0 = J[0][i] * Wd + J[1][i] * Wo;
        const double t1 = J[0][i] * Wo + J[1][i] * Wd;
        RSC_UNROLL for (int j = 0; j <= i; ++j) t[k++] = t0 * J[0][j] + t1 * J[1][j];
    }
    RSC_UNROLL for (int i = 0; i < 7; ++i) t[28 + i] = J[0][i] * omr0 + J[1][i] * omr1;
}

// Both: linearizeOplus + constructQuadraticForm of one edge.
RSC_HD void so_quad_terms(const SoPerturbed& P, bool inverse, const SoCam& K, const double (&X)[3], double u,
                          double v, double inv, double e0, double e1, double delta, double dsqr,
                          double (&t)[kSim3OptTerms]) {
    double J[2][7];
    so_jacobian(P, inverse, K, X, u, v, J);
    so_quad_tail(J, inv, e0, e1, delta, dsqr, t);
}

#if defined(__HIPCC__)
// helpers = 0: one workgroup per pair; helpers > 0: the cooperative form with that many helper
// workgroups per pair (fault: the launch's fault word, raised when a bounded hand-off wait gives up).
hipError_t launch_sim3opt(int count, const DevSim3OptProb* probs, int helpers, unsigned* fault, hipStream_t st);
hipError_t read_sim3opt_phases(uint64_t* out);  // diagnostic, [64][8] (sim3opt.hip)
#endif

}  // namespace rsc
