// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of Optimizer::PoseOptimization (src/Optimizer.cpp:205-424), monocular
// (mvuRight < 0) and stereo (mvuRight >= 0) edges, with the parts of the vendored g2o it runs:
//   SparseOptimizer::initializeOptimization/optimize/computeActiveErrors/activeRobustChi2
//     (Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:61-114,199-267,354-414),
//   OptimizationAlgorithmLevenberg::solve/computeLambdaInit/computeScale
//     (core/optimization_algorithm_levenberg.cpp:59-172, incl. ORB-SLAM2's "Raul" stop rule),
//   BlockSolver::buildSystem/setLambda/restoreDiagonal (core/block_solver.hpp:502-604),
//   LinearSolverDense::solve = Eigen::LDLT (solvers/linear_solver_dense.h:66-114),
//   BaseUnaryEdge::constructQuadraticForm (core/base_unary_edge.hpp:43-71),
//   RobustKernelHuber (core/robust_kernel_impl.cpp:65-91),
//   EdgeSE3ProjectXYZOnlyPose::computeError/linearizeOplus (types/types_six_dof_expmap.h:153-157,
//     types/types_six_dof_expmap.cpp:266-296), EdgeStereoSE3ProjectXYZOnlyPose::computeError/
//     cam_project/linearizeOplus (types_six_dof_expmap.h:184-188, .cpp:299-306,335-366),
//     VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:73),
//   SE3Quat (types/se3quat.h: ctor, operator*, map, exp, normalizeRotation),
//   Converter::toSE3Quat / toIso (src/Converter.cpp:16-29).
//
// PARITY UNPINNED against the reference binary: g2o and Eigen need Eigen headers, which this
// image lacks, so neither can be built here, and the reference has no tests or fixtures for this
// path.  Restatement choices where the reference leaves arithmetic to Eigen/glibc internals:
// every Eigen sum and small product left to right (Eigen's generic, non-SIMD kernels), the
// generic quaternion product, sin/cos from fdlibm (rsc_math.h, as MLPnP), pow(x, 3) as a
// correctly rounded cube, Isometry3f::rotation() as linear().
#pragma once
#include <cstdint>

namespace rsc_oracle {

struct PoseOptInput {
    int n;                    // keypoint slots (pFrame->N)
    const uint8_t* has_mp;    // [n] mvpMapPoints[i] != NULL; NULL = every slot has a map point
    const float* uv;          // [n][2] mvKeysUn[i].pt
    const float* Xw;          // [n][3] MapPoint::GetWorldPos()
    const float* inv_sigma2;  // [n] mvInvLevelSigma2[kpUn.octave]
    float fx, fy, cx, cy;     // Frame::fx..cy
    float Tcw[16];            // row-major pFrame->mTcw
    const float* u_right = nullptr;  // [n] mvuRight (>= 0: stereo edge, Optimizer.cpp:252,290-323); NULL = mono
    float bf = 0.0f;                 // Frame::mbf (stereo baseline x fx)
};

struct PoseOptStats {
    int rounds;          // outer rounds run (<= 4)
    int lm_iterations;   // solve() calls over all rounds
    int lm_trials;       // Levenberg trials (linear solves) over all rounds
};

// Returns nInitialCorrespondences - nBad (0 without touching Tcw_out when fewer than 3 edges).
// outlier[i] is written for slots with a map point (mvbOutlier), left untouched otherwise.
int pose_optimization(const PoseOptInput& in, float Tcw_out[16], uint8_t* outlier, PoseOptStats* stats);

}  // namespace rsc_oracle
