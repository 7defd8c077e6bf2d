// rsc_sim3match.h — ORBmatcher::SearchBySim3 (src/ORBmatcher.cpp:948-1170) on the GPU: device layout.
//
// Mapping: one lane per MapPoint of the source KeyFrame, both directions of every pair in one
// launch (grid (points / 256, 2, pairs)); a lane projects its point with the pair's (R, t), walks
// the destination grid cells of GetFeaturesInArea in the reference's order (ix, iy, cell order) and
// keeps the first minimum descriptor distance over the keypoints of the predicted levels — the
// same candidates in the same order as the reference's vIndices loop, so bestIdx is identical.  A
// second kernel (one workgroup per pair) keeps the mutual matches (:1152-1167) and counts them.
// Float arithmetic is the reference's (oracle/sim3match_oracle.h lists the choices); the work per
// point is a few dozen flops plus ~10-50 candidate descriptor comparisons: latency-bound, no MFMA.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace rsc {

constexpr int kSim3GridCols = 64, kSim3GridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.hpp:20-21)
constexpr int kSim3ThHigh = 100;                       // ORBmatcher::TH_HIGH (ORBmatcher.cpp:8)

struct DevSim3KF {
    const float2* kp;        // [n] mvKeysUn[i].pt
    const int32_t* octave;   // [n]
    const uint4* desc;       // [n][2]
    const int32_t* cell_begin;  // [64*48 + 1]
    const int32_t* cell_feat;
    const float* scale;      // [n_levels] mvScaleFactors
    const uint8_t* mp_state; // [n] 0 NULL, 1 good, 2 bad
    const float* mp_pos;     // [n][3]
    const float* mp_dmax;    // [n]
    const float* mp_dmin;    // [n]
    const uint4* mp_desc;    // [n][2]
    float min_x, max_x, min_y, max_y, gw_inv, gh_inv, fx, fy, cx, cy, log_sf;
    float R[9], t[3];
    int n, n_levels;
};

struct Sim3MatchPair {
    const DevSim3KF* k1;
    const DevSim3KF* k2;
    float R12[9], t12[3];
    const uint8_t* already1;  // [k1.n] vbAlreadyMatched1
    const uint8_t* already2;  // [k2.n] vbAlreadyMatched2
    int32_t* m1;              // [k1.n] vnMatch1
    int32_t* m2;              // [k2.n] vnMatch2
    int32_t* out;             // [k1.n] new match (KF2 keypoint) or -1
    int32_t* nfound;          // [1]
};

hipError_t launch_search_by_sim3(int count, int max_points, const Sim3MatchPair* pairs, float th, hipStream_t st);

}  // namespace rsc
