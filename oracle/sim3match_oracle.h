// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of ORBmatcher::SearchBySim3 (src/ORBmatcher.cpp:948-1170): the
// loop-closure matcher that, after Sim3Solver::iterate returned a transformation
// (LoopClosing.cpp:296-309), projects each unmatched MapPoint of one KeyFrame into the other with
// (R12, t12), searches the keypoints of the predicted pyramid levels inside a radius
// (KeyFrame::GetFeaturesInArea, KeyFrame.cpp:560-599; IsInImage :601-604; MapPoint::PredictScale,
// GetMin/MaxDistanceInvariance, MapPoint.cpp:355-381) for the best descriptor distance
// (ORBmatcher::DescriptorDistance), in both directions, and keeps the mutual matches.
//
// Float arithmetic follows the reference's expressions and types: Eigen 3x3 products summed left to
// right (the repository-wide convention), `1.0/z` in double rounded to float
// (:1011, :1091), norm = sqrt((x*x + y*y) + z*z), floor/ceil of the float grid coordinates.
// PredictScale's `log(ratio)` (float overload -> glibc logf) is restated as the float rounding of
// the fdlibm double log (rsc_math.h): it differs from glibc's logf in ~0.04 % of arguments, which
// can change ceil() only for ratios within an ulp of a power of the scale factor — parity with the
// reference binary is unpinned at that level.
#pragma once
#include <cstdint>

namespace rsc_oracle {

// One KeyFrame as SearchBySim3 reads it.
struct Sim3KF {
    int n;                    // N
    const float* kp;          // [n][2] mvKeysUn[i].pt
    const int32_t* octave;    // [n] mvKeysUn[i].octave
    const uint8_t* desc;      // [n][32] mDescriptors
    const int32_t* cell_begin;  // [64*48 + 1] CSR of mGrid[ix][iy], cell = ix * 48 + iy
    const int32_t* cell_feat;   // mGrid contents (vector<size_t> order)
    float min_x, max_x, min_y, max_y;  // mnMinX, mnMaxX, mnMinY, mnMaxY
    float grid_w_inv, grid_h_inv;      // mfGridElementWidthInv, mfGridElementHeightInv
    float fx, fy, cx, cy;
    const float* scale_factors;  // [n_levels] mvScaleFactors
    int n_levels;                // mnScaleLevels
    float log_scale_factor;      // mfLogScaleFactor
    float Rcw[9], tcw[3];        // GetRotation(), GetTranslation() (row-major)
    // GetMapPointMatches(): per keypoint slot
    const uint8_t* mp_state;  // [n] 0 = NULL, 1 = good, 2 = isBad()
    const float* mp_pos;      // [n][3] GetWorldPos()
    const float* mp_dmax;     // [n] mfMaxDistance
    const float* mp_dmin;     // [n] mfMinDistance
    const uint8_t* mp_desc;   // [n][32] GetDescriptor()
};

constexpr int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS (Frame.hpp:20-21)

// SearchBySim3(pKF1, pKF2, vpMatches12, R12, t12, th).  matched12[i1] (in): the keypoint index in
// KF2 of the MapPoint already in vpMatches12[i1] (GetIndexInKeyFrame(pKF2)), -1 for NULL, or -2
// for a MapPoint not observed in KF2.  out12[i1]: KF2 keypoint index of each NEW match (the
// reference sets vpMatches12[i1] = vpMapPoints2[idx2]), else -1.  Returns nFound.
int search_by_sim3(const Sim3KF& kf1, const Sim3KF& kf2, const int32_t* matched12, const float* R12,
                   const float* t12, float th, int32_t* out12);

// MapPoint::PredictScale (MapPoint.cpp:367-381)
int predict_scale(float dmax, float current_dist, float log_scale_factor, int n_levels);

}  // namespace rsc_oracle
