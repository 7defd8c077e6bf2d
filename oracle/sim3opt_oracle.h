// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) — the 7-DoF
// loop-closure refinement LoopClosing::ComputeSim3 runs after SearchBySim3 (LoopClosing.cpp:309-311)
// — with the parts of the vendored g2o it runs:
//   SparseOptimizer::initializeOptimization/optimize/computeActiveErrors/activeRobustChi2
//     (Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:61-114,199-267,354-414): the Sim3 vertex is the
//     only non-fixed vertex (the point vertices are fixed), active edges in insertion (id) order
//     e12_0, e21_0, e12_1, e21_1, ...;
//   OptimizationAlgorithmLevenberg::solve / computeLambdaInit / computeScale
//     (core/optimization_algorithm_levenberg.cpp:59-172, ORB-SLAM2's nBad stop rule);
//   BlockSolverX::buildSystem (core/block_solver.hpp:502-560) + the Schur path with no landmarks,
//     LinearSolverDense (solvers/linear_solver_dense.h:64-107: the full 7x7 block, LDLT on its lower
//     triangle), BlockSolver::_x persisting across iterations and both optimize() calls;
//   BaseBinaryEdge::linearizeOplus — NUMERIC Jacobian, delta 1e-9, central differences through
//     VertexSim3Expmap::oplusImpl (core/base_binary_edge.hpp; EdgeSim3ProjectXYZ /
//     EdgeInverseSim3ProjectXYZ declare no analytic linearizeOplus, types_seven_dof_expmap.h) —
//     and BaseBinaryEdge::constructQuadraticForm (robust branch: omega_r = -omega*error*rho1,
//     b += B^T omega_r, H += B^T (rho1 omega) B);
//   VertexSim3Expmap::oplusImpl with _fix_scale (update[6] = 0 written into the solver's x),
//   g2o::Sim3 (types/sim3.h: exp-map constructor, operator*, inverse, map), project, cam_map1/2,
//   RobustKernelHuber (core/robust_kernel_impl.cpp:65-91).
//
// PARITY UNPINNED against the reference binary: g2o and Eigen need Eigen headers, which this image
// lacks, and the reference has no tests or fixtures for this path.  Restatement choices where the
// reference leaves the arithmetic to Eigen/glibc internals (as oracle/poseopt_oracle.h): every Eigen
// sum and small product left to right, the generic quaternion product and _transformVector,
// Quaterniond(Matrix3d) as Eigen's trace/largest-diagonal algorithm, sin/cos from fdlibm
// (rsc_math.h), exp(0) = 1.
#pragma once
#include <cstdint>

namespace rsc_oracle {

struct Sim3OptInput {
    int n;                   // vpMatches1.size() (= pKF1->N)
    const uint8_t* valid;    // [n] the slot forms a correspondence (Optimizer.cpp:1112-1143 tests)
    const float* X1w;        // [n][3] vpMapPoints1[i]->GetWorldPos()
    const float* X2w;        // [n][3] vpMatches1[i]->GetWorldPos()
    const float* uv1;        // [n][2] pKF1->mvKeysUn[i].pt
    const float* uv2;        // [n][2] pKF2->mvKeysUn[i2].pt
    const float* inv1;       // [n] pKF1->mvInvLevelSigma2[kpUn1.octave]
    const float* inv2;       // [n] pKF2->mvInvLevelSigma2[kpUn2.octave]
    float R1w[9], t1w[3], R2w[9], t2w[3];  // GetRotation()/GetTranslation() (row-major)
    float K1[4], K2[4];      // mK: fx, fy, cx, cy
    float th2;               // chi2 threshold (10 in LoopClosing.cpp:311)
};

struct Sim3Est {
    double q[4];  // Quaterniond coefficients x, y, z, w
    double t[3];
    double s;
};

struct Sim3OptStats {
    int n_correspondences;
    int n_bad;        // removed after the first optimize(5)
    int lm_iterations;
    int lm_trials;
};

// Returns nIn (0 when nCorrespondences - nBad < 10; g2oS12 is then left unchanged).  keep[i] = 0
// where vpMatches1[i] is set to NULL (outliers), 1 elsewhere.  S: g2oS12 in / out.
int optimize_sim3(const Sim3OptInput& in, Sim3Est& S, uint8_t* keep, Sim3OptStats* stats);

}  // namespace rsc_oracle
