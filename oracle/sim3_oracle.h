// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of ORB_SLAM_CUSTOM::Sim3Solver (reference: include/Sim3Solver.hpp:16-103,
// src/Sim3Solver.cpp:6-347): Horn closed form with scale fixed to 1 (SE3, Q13), two-way reprojection
// inlier test, '&&' loop condition (Q1), size_t thresholds (Q11), '>=' best update then '>' return
// (Q12).  Isometry3f::rotation() is taken as linear() (Q14, Eigen 3.4 behaviour; documented).
#pragma once
#include <cstdint>
#include <vector>
#include "glibc_rand.h"

namespace rsc_oracle {

// Raw inputs of the Sim3Solver constructor (Sim3Solver.cpp:6-85) for ONE keyframe pair, already
// reduced to plain arrays:  for every match slot i1 < n1 (vpMatched12.size()):
//   valid[i1]   — vpMatched12[i1] && pMP1 && !bad && both GetIndexInKeyFrame >= 0 (:28-43)
//   Xw1/Xw2     — world positions of pMP1 / pMP2 (float[3])
//   sigma2_1/2  — mvLevelSigma2[kp.octave] of the two keypoints
// plus the keyframe poses (Rcw row-major float[9], tcw float[3]) and the intrinsics K (fx,fy,cx,cy).
struct Sim3Input {
    int n1;
    const uint8_t* valid;
    const float* Xw1;
    const float* Xw2;
    const float* sigma2_1;
    const float* sigma2_2;
    float R1[9], t1[3], R2[9], t2[3];
    float K1[4], K2[4];  // fx, fy, cx, cy
};

struct Sim3Trace {
    int sample[3];
    int n_inliers;
    float R[9], t[3];
};

class Sim3Oracle {
public:
    Sim3Oracle(const Sim3Input& in, uint32_t seed);
    void SetRansacParameters(double probability = 0.99, int minInliers = 6, int maxIterations = 300);
    bool find(std::vector<uint8_t>& vbInliers12, int& nInliers);
    bool iterate(int nIterations, bool& bNoMore, std::vector<uint8_t>& vbInliers, int& nInliers);
    void GetEstimatedRotation(float R[9]) const;
    void GetEstimatedTranslation(float t[3]) const;

    // Prepared per-correspondence arrays (what the ctor builds), for tests.
    int N = 0;
    int mN1 = 0;
    std::vector<float> mvX3Dc1, mvX3Dc2, mvP1im1, mvP2im2;  // [N][3],[N][3],[N][2],[N][2]
    std::vector<uint64_t> mvnMaxError1, mvnMaxError2;        // size_t thresholds (Q11)
    std::vector<int32_t> mvnIndices1;
    int iterations() const { return mnIterations; }
    int max_iterations() const { return mRansacMaxIts; }
    std::vector<Sim3Trace>* trace = nullptr;

    void compute_sim3_public(const int idx[3], float R[9], float t[3]);
    int check_inliers_public(const float R[9], const float t[3], std::vector<uint8_t>& inl);

    // Draw from the process-global libc rand() instead of the own stream: the reference's actual
    // RandomInt (Random.cpp:47-50), for event replays on one shared stream (Q3).
    void use_libc_rand(bool on = true) { rng.use_libc = on; }  // off: the own stream resumes
private:
    void ComputeSim3(const float P1[3][3], const float P2[3][3]);
    void CheckInliers();
    void Project(const std::vector<float>& X, std::vector<float>& P2D, const float R[3][3], const float t[3],
                 const float K[4]);

    float mR12i[3][3], mt12i[3];
    float mR21i[3][3], mt21i[3];  // mT21i = mT12i.inverse()
    std::vector<uint8_t> mvbInliersi;
    int mnInliersi = 0;
    int mnIterations = 0;
    std::vector<uint8_t> mvbBestInliers;
    int mnBestInliers = 0;
    float mBestRotation[3][3], mBestTranslation[3];
    std::vector<int32_t> mvAllIndices;
    double mRansacProb;
    int mRansacMinInliers;
    int mRansacMaxIts;
    float mK1[4], mK2[4];
    GlibcRand rng;
};

}  // namespace rsc_oracle
