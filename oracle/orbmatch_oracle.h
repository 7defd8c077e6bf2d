// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of the two ORBmatcher::SearchByBoW overloads that produce the
// correspondences of the RANSAC solvers:
//   * SearchByBoW(KeyFrame, Frame, ...)  (src/ORBmatcher.cpp:110-240) — Tracking::Relocalization
//     (Tracking.cpp:1214) and TrackReferenceKeyFrame (Tracking.cpp:611) feed PnPsolver with it;
//   * SearchByBoW(KeyFrame, KeyFrame, ...) (src/ORBmatcher.cpp:354-488) — LoopClosing::ComputeSim3
//     (LoopClosing.cpp:251) feeds Sim3Solver with it;
// plus ORBmatcher::DescriptorDistance (:1492-1508) and ComputeThreeMaxima (:1446-1487).
// DBoW2::FeatureVector is a std::map<NodeId, std::vector<unsigned int>> (node -> feature indices,
// ascending node ids); it is restated as exactly that so the reference's merge walk with
// lower_bound (:204-211, :452-460) is followed literally.
//
// Pure integer/byte work plus the float orientation bin: the restatement is exact arithmetic; the
// reference ships no tests or fixtures for this path, so parity is pinned by the
// known-answer cases of tests/test_cpu_orbmatch.py and the golden traces in tests/golden/.
#pragma once
#include <cstdint>
#include <map>
#include <vector>

namespace rsc_oracle {

using FeatureVector = std::map<uint32_t, std::vector<uint32_t>>;

struct BowView {
    int n;                    // keypoints
    const uint8_t* desc;      // [n][32] descriptor rows
    const float* angle;       // [n] keypoint angle (degrees)
    const uint8_t* valid;     // [n] map point present and not bad (NULL = all)
    FeatureVector fv;
};

// ORBmatcher::DescriptorDistance (ORBmatcher.cpp:1492-1508): popcount of a XOR b over 8 int32 words
int descriptor_distance(const uint8_t* a, const uint8_t* b);

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cpp:1446-1487) over bin sizes
void compute_three_maxima(const int* sizes, int L, int& ind1, int& ind2, int& ind3);

// SearchByBoW(pKF, F, vpMapPointMatches): match[F.n] = KeyFrame feature index matched to each Frame
// feature (the MapPoint vpMapPointsKF[idx]) or -1.  Returns nmatches.
int search_by_bow_frame(const BowView& kf, const BowView& frame, float nnratio, bool check_ori,
                        int32_t* match);

// SearchByBoW(pKF1, pKF2, vpMatches12): match12[kf1.n] = KF2 feature index (the MapPoint
// vpMapPoints2[idx2]) or -1.  Returns nmatches.
int search_by_bow_kf(const BowView& kf1, const BowView& kf2, float nnratio, bool check_ori, int32_t* match12);

}  // namespace rsc_oracle
