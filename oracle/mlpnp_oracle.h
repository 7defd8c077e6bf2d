// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of ORB_SLAM_CUSTOM::MLPnPsolver (reference: include/MLPnPsolver.hpp:10-199,
// src/MLPnPsolver.cpp:5-1020): MLPnP (Urban et al.) inside the PnP-style RANSAC loop.
//
// PARITY UNPINNED: the reference never compiles this file (CMakeLists.txt:75 leaves it out, the call
// sites Tracking.cpp:1222,1227-1228 are commented out) and it has no tests, so there is nothing to
// pin against.  Choices this restatement makes where the reference leaves the
// arithmetic to Eigen/glibc internals (documented in DESIGN.md):
//   * every dot product / matrix product is summed left to right in index order;
//   * sin, cos, acos are the fdlibm algorithms of csrc/rsc_math.h (glibc differs by <= 1 ulp);
//     pow(x, 1/3) is cbrt(x), pow(x, 3/2) is x*sqrt(x);
//   * Matrix4d::inverse is the generic cofactor expansion (Eigen's SSE kernel is not restated);
//   * mlpnpJacs (MLPnPsolver.cpp:773-1020, machine-generated) is replaced by the analytic
//     Jacobian of the same residual (Gallego & Yezzi's Rodrigues derivative), NaN at w = 0 like
//     the reference;
//   * Refine() (MLPnPsolver.cpp:257-318) discards its computePose result and re-counts the current
//     hypothesis, so it is restated as that re-count (no solve).
#pragma once
#include <cstdint>
#include <vector>
#include "glibc_rand.h"

namespace rsc_oracle {

class MLPnPOracle {
public:
    // MLPnPsolver::MLPnPsolver (MLPnPsolver.cpp:5-53) on compacted arrays; calls SetRansacParameters().
    MLPnPOracle(int n, int n_points, const float* p2d, const float* p3dw, const float* sigma2,
                const int32_t* kp_index, float fx, float fy, float cx, float cy, uint32_t seed);

    // MLPnPsolver.cpp:185-220 (defaults hpp:16-17: 0.99, 8, 300, 6, 0.4, 5.991)
    void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300,
                             int minSet = 6, float epsilon = 0.4f, float th2 = 5.991f);
    // MLPnPsolver.cpp:56-183.  T is set to identity on entry (Q10).
    bool iterate(int nIterations, bool& bNoMore, std::vector<uint8_t>& vbInliers, int& nInliers, float T[16]);

    int iterations() const { return mnIterations; }
    int max_iterations() const { return mRansacMaxIts; }
    int min_inliers() const { return mRansacMinInliers; }
    int best_inliers() const { return mnBestInliers; }

    // computePose's covMats (MLPnPsolver.cpp:321): cov [N][9] row-major 3x3 per correspondence
    // (compacted order), or null for the reference's own call (no covariance: use_cov = false).
    void set_covariances(const double* cov);
    // computePose on correspondences idx[0..n) (hypothesis or any subset); R row-major, t.
    void compute_pose_public(const int* idx, int n, double R[9], double t[3]);
    // Per-hypothesis trace: sample indices, count, double pose.
    struct Trace {
        int sample[8];
        int n_inliers;
        double R[9], t[3];
        int planar;  // computePose took the planar branch (MLPnPsolver.cpp:354-364: rank(PP^T) == 2)
    };
    std::vector<Trace>* trace = nullptr;

    // Draw from the process-global libc rand() instead of the own stream: the reference's actual
    // RandomInt (Random.cpp:47-50), for event replays on one shared stream (Q3).
    void use_libc_rand(bool on = true) { rng.use_libc = on; }  // off: the own stream resumes
private:
    void CheckInliers();
    void computePose(const int* idx, int n, double R[3][3], double t[3]);

    float fx, fy, cx, cy;
    int N_points;
    std::vector<float> mvP2D;      // [N][2]
    std::vector<float> mvSigma2;   // [N]
    std::vector<double> mvBearing; // [N][3]  ((u-cx)/fx, (v-cy)/fy, 1) in float, then double
    std::vector<double> mvP3Dw;    // [N][3]  float positions widened to double
    std::vector<int32_t> mvKeyPointIndices;
    std::vector<double> mvCov;     // [N][9] or empty

    double mRi[3][3], mti[3];
    bool mLastPlanar = false;  // branch taken by the last computePose (trace only)
    std::vector<uint8_t> mvbInliersi;
    int mnInliersi = 0;
    int mnIterations = 0;
    std::vector<uint8_t> mvbBestInliers;
    int mnBestInliers = 0;
    float mBestTcw[16];

    int N = 0;
    std::vector<int32_t> mvAllIndices;
    double mRansacProb;
    int mRansacMinInliers;
    int mRansacMaxIts;
    float mRansacEpsilon;
    int mRansacMinSet;
    std::vector<float> mvMaxError;

    GlibcRand rng;
};

// Residual Jacobian d(r_r, r_s)/d(w, t) of one correspondence at x = (w, t) (test hook).
void mlpnp_jacobian_public(const double X[3], const double nr[3], const double ns[3], const double x[6],
                           double J[12]);

}  // namespace rsc_oracle
