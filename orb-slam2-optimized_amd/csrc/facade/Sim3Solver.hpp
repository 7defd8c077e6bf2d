// Sim3Solver.hpp — drop-in facade of ORB_SLAM_CUSTOM::Sim3Solver (reference include/Sim3Solver.hpp:16-30)
// over the rsc C ABI.  KeyFrameT needs GetMapPointMatches(), GetRotation(), GetTranslation(),
// mvKeysUn, mvLevelSigma2 and a static/instance mK with (r,c) access (KeyFrame.hpp:149-174);
// MapPointT needs isBad(), GetWorldPos() and GetIndexInKeyFrame(pKF) (MapPoint.cpp:297-304).
// Rotation/translation types need (r,c) / (i) access and a default constructor.
//
// GetEstimatedRotation() / GetEstimatedTranslation() return Mat3 / Vec3, by default the types of
// KeyFrameT::GetRotation() / GetTranslation() — Eigen::Matrix3f / Eigen::Vector3f for the reference's
// KeyFrame (KeyFrame.hpp:42-43), the types include/Sim3Solver.hpp:29-30 declares — so the call sites
// `Eigen::Matrix3f R = vpSim3Solvers[i]->GetEstimatedRotation();` (LoopClosing.cpp:307-308) compile
// unchanged.
#pragma once
#include <cstring>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

template <class KeyFrameT>
using kf_rotation_t = typename std::decay<decltype(std::declval<KeyFrameT&>().GetRotation())>::type;
template <class KeyFrameT>
using kf_translation_t = typename std::decay<decltype(std::declval<KeyFrameT&>().GetTranslation())>::type;

template <class KeyFrameT, class MapPointT, class Mat3 = kf_rotation_t<KeyFrameT>,
          class Vec3 = kf_translation_t<KeyFrameT>>
class Sim3Solver {
public:
    // Sim3Solver::Sim3Solver (Sim3Solver.cpp:6-85): the match validity / keypoint lookup is done
    // here on the host (it walks the map objects); the arithmetic runs in librsc.
    Sim3Solver(std::shared_ptr<KeyFrameT> pKF1, std::shared_ptr<KeyFrameT> pKF2,
               const std::vector<std::shared_ptr<MapPointT>>& vpMatched12, uint32_t seed = 1) {
        std::vector<std::shared_ptr<MapPointT>> vpKeyFrameMP1 = pKF1->GetMapPointMatches();
        const int n1 = (int)vpMatched12.size();
        std::vector<uint8_t> valid(n1, 0);
        std::vector<float> Xw1(3 * n1, 0.f), Xw2(3 * n1, 0.f), s1(n1, 0.f), s2(n1, 0.f);
        for (int i1 = 0; i1 < n1; i1++) {
            if (!vpMatched12[i1]) continue;
            std::shared_ptr<MapPointT> pMP1 = vpKeyFrameMP1[i1];
            std::shared_ptr<MapPointT> pMP2 = vpMatched12[i1];
            if (!pMP1) continue;
            if (pMP1->isBad() || pMP2->isBad()) continue;
            const int indexKF1 = pMP1->GetIndexInKeyFrame(pKF1);
            const int indexKF2 = pMP2->GetIndexInKeyFrame(pKF2);
            if (indexKF1 < 0 || indexKF2 < 0) continue;
            valid[i1] = 1;
            s1[i1] = pKF1->mvLevelSigma2[pKF1->mvKeysUn[indexKF1].octave];
            s2[i1] = pKF2->mvLevelSigma2[pKF2->mvKeysUn[indexKF2].octave];
            const auto a = pMP1->GetWorldPos();
            const auto b = pMP2->GetWorldPos();
            for (int r = 0; r < 3; ++r) { Xw1[3 * i1 + r] = a(r); Xw2[3 * i1 + r] = b(r); }
        }
        rsc_sim3_input in;
        in.n1 = n1;
        in.valid = valid.data();
        in.Xw1 = Xw1.data(); in.Xw2 = Xw2.data();
        in.sigma2_1 = s1.data(); in.sigma2_2 = s2.data();
        const auto R1 = pKF1->GetRotation();
        const auto t1 = pKF1->GetTranslation();
        const auto R2 = pKF2->GetRotation();
        const auto t2 = pKF2->GetTranslation();
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) { in.R1[3 * r + c] = R1(r, c); in.R2[3 * r + c] = R2(r, c); }
            in.t1[r] = t1(r);
            in.t2[r] = t2(r);
        }
        const auto& K1 = pKF1->mK;
        const auto& K2 = pKF2->mK;
        in.K1[0] = K1(0, 0); in.K1[1] = K1(1, 1); in.K1[2] = K1(0, 2); in.K1[3] = K1(1, 2);
        in.K2[0] = K2(0, 0); in.K2[1] = K2(1, 1); in.K2[2] = K2(0, 2); in.K2[3] = K2(1, 2);
        check(rsc_sim3_create(thread_context(), &in, seed, &s_), "rsc_sim3_create");
        if (rsc_stream* st = construction_stream()) check(rsc_sim3_bind_stream(s_, st), "rsc_sim3_bind_stream");
        n1_ = n1;
    }
    ~Sim3Solver() { rsc_sim3_destroy(s_); }
    Sim3Solver(const Sim3Solver&) = delete;
    Sim3Solver& operator=(const Sim3Solver&) = delete;

    void SetRansacParameters(double probability = 0.99, int minInliers = 6, int maxIterations = 300) {
        check(rsc_sim3_set_ransac_parameters(s_, probability, minInliers, maxIterations), "SetRansacParameters");
    }

    bool find(std::vector<bool>& vbInliers12, int& nInliers) {
        int32_t st[6];
        check(rsc_sim3_get_state(s_, st), "get_state");
        bool bFlag;
        return iterate(st[1], bFlag, vbInliers12, nInliers);
    }

    bool iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers) {
        rsc_sim3_result r;
        std::vector<uint8_t> mask(n1_ > 0 ? n1_ : 1, 0);
        check(rsc_sim3_iterate(s_, nIterations, &r, mask.data()), "iterate");
        bNoMore = r.no_more != 0;
        nInliers = r.n_inliers;
        vbInliers.assign(n1_, false);  // Sim3Solver.cpp:116
        for (int i = 0; i < n1_; ++i) vbInliers[i] = mask[i] != 0;
        std::memcpy(R_, r.R, sizeof(R_));
        std::memcpy(t_, r.t, sizeof(t_));
        return r.ok != 0;
    }

    // GetEstimatedRotation / GetEstimatedTranslation (Sim3Solver.hpp:29-30, Sim3Solver.cpp:296-304):
    // the reference signatures, returning the best hypothesis' R12 / t12 of the last iterate().
    Mat3 GetEstimatedRotation() const { return GetEstimatedRotation<Mat3>(); }
    Vec3 GetEstimatedTranslation() const { return GetEstimatedTranslation<Vec3>(); }

    // The same into any type with (r,c) / (i) access.
    template <class M3>
    M3 GetEstimatedRotation() const {
        M3 R;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) R(r, c) = R_[3 * r + c];
        return R;
    }
    template <class V3>
    V3 GetEstimatedTranslation() const {
        V3 t;
        for (int r = 0; r < 3; ++r) t(r) = t_[r];
        return t;
    }

    rsc_sim3* handle() { return s_; }

private:
    rsc_sim3* s_ = nullptr;
    int n1_ = 0;
    float R_[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    float t_[3] = {0, 0, 0};
};

}  // namespace rsc_orb
