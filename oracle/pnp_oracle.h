// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of ORB_SLAM_CUSTOM::PnPsolver (reference: include/PnPsolver.hpp:21-138,
// src/PnPsolver.cpp:11-796): EPnP + RANSAC with every quirk of SURVEY.md §8(a) (Q1-Q10, Q16, Q17).
// Inputs are the plain arrays the reference constructor builds from Frame/MapPoint
// (PnPsolver.cpp:22-44), i.e. the already-compacted correspondences.
#pragma once
#include <cstdint>
#include <vector>
#include "glibc_rand.h"

namespace rsc_oracle {

struct PnPTrace {  // one entry per hypothesis (debug/golden-vector hook)
    int sample[8];
    int n_inliers;
    float R[9], t[3];
    int refine_called, refine_inliers, refine_ok;
};

class PnPOracle {
public:
    // PnPsolver::PnPsolver (PnPsolver.cpp:11-55) on compacted arrays.
    //   p2d[n][2] = kp.pt, p3dw[n][3] = MapPoint::GetWorldPos(), sigma2[n] = mvLevelSigma2[octave],
    //   kp_index[n] = keypoint index in the Frame, n_points = vpMapPointMatches.size().
    //   fx..cy are Frame's static float intrinsics, stored as double members (PnPsolver.hpp:71).
    PnPOracle(int n, int n_points, const float* p2d, const float* p3dw, const float* sigma2,
              const int32_t* kp_index, float fx, float fy, float cx, float cy, uint32_t seed);

    void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300,
                             int minSet = 4, float epsilon = 0.4f, float th2 = 5.991f);
    bool find(std::vector<uint8_t>& vbInliers, int& nInliers, float T[16]);
    bool iterate(int nIterations, bool& bNoMore, std::vector<uint8_t>& vbInliers, int& nInliers, float T[16]);

    // Accessors for tests.
    int iterations() const { return mnIterations; }
    int max_iterations() const { return mRansacMaxIts; }
    int min_inliers() const { return mRansacMinInliers; }
    int best_inliers() const { return mnBestInliers; }
    int max_rows() const { return maximum_number_of_correspondences; }
    const std::vector<float>& max_error() const { return mvMaxError; }
    std::vector<PnPTrace>* trace = nullptr;

    // Exposed pieces for known-answer tests.
    double compute_pose_public(const int* idx, int n, float R[9], float t[3]);
    void check_inliers_public(const float R[9], const float t[3], std::vector<uint8_t>& inl, int& count);
    // qr_solve (PnPsolver.cpp:693-796); false on the singular bail-out (X untouched).
    static bool qr_solve(double A[6][4], double b[6], double X[4]);

    // Draw from the process-global libc rand() instead of the own stream: the reference's actual
    // RandomInt (Random.cpp:47-50), for event replays on one shared stream (Q3).
    void use_libc_rand(bool on = true) { rng.use_libc = on; }  // off: the own stream resumes
private:
    void CheckInliers();
    bool Refine();
    void set_maximum_number_of_correspondences(int n);
    void reset_correspondences() { number_of_correspondences = 0; }
    void add_correspondence(const float* p3D, const float* p2D);
    double compute_pose(float R[3][3], float t[3]);
    double reprojection_error(const double R[3][3], const double t[3]);
    void choose_control_points();
    void compute_barycentric_coordinates();
    void compute_ccs(const double betas[4], const double (*U)[12]);
    void compute_pcs();
    void solve_for_sign();
    void find_betas_approx_1(const double L[6][10], const double rho[6], double betas[4]);
    void find_betas_approx_2(const double L[6][10], const double rho[6], double betas[4]);
    void find_betas_approx_3(const double L[6][10], const double rho[6], double betas[4]);
    void compute_rho(double rho[6]);
    void compute_L_6x10(const double (*U)[12], double L[6][10]);
    void gauss_newton(const double L[6][10], const double rho[6], double betas[4]);
    void compute_A_and_b_gauss_newton(const double L[6][10], const double rho[6], const double cb[4],
                                      double A[6][4], double b[6]);
    double compute_R_and_t(const double (*U)[12], const double betas[4], double R[3][3], double t[3]);
    void estimate_R_and_t(double R[3][3], double t[3]);

    double cx, cy, fx, fy;
    double cws[4][3], ccs[4][3];
    // Dynamic-row EPnP buffers: only grow (set_maximum_number_of_correspondences), never shrink.
    std::vector<double> pws, pcs, alphas, us;  // rows x {3,3,4,2}
    int maximum_number_of_correspondences = 0;
    int number_of_correspondences = 0;
    int N_points;

    std::vector<float> mvP2D;    // [N][2]
    std::vector<float> mvSigma2; // [N]
    std::vector<float> mvP3Dw;   // [N][3]
    std::vector<int32_t> mvKeyPointIndices;

    float mRi[3][3], mti[3];
    std::vector<uint8_t> mvbInliersi;
    int mnInliersi = 0;

    int mnIterations = 0;
    std::vector<uint8_t> mvbBestInliers;
    int mnBestInliers = 0;
    float mBestTcw[16];

    float mRefinedTcw[16];
    std::vector<uint8_t> mvbRefinedInliers;
    int mnRefinedInliers = 0;

    int N = 0;
    std::vector<int32_t> mvAllIndices;
    double mRansacProb;
    int mRansacMinInliers;
    int mRansacMaxIts;
    float mRansacEpsilon;
    int mRansacMinSet;
    std::vector<float> mvMaxError;
    double qr_X[4];  // X of gauss_newton: holds its previous value when qr_solve bails (Q9)

    GlibcRand rng;
};

}  // namespace rsc_oracle
