// Optimizer.hpp — drop-in facade of ORB_SLAM_CUSTOM::Optimizer::PoseOptimization
// (reference include/Optimizer.hpp, src/Optimizer.cpp:205-424) and Optimizer::OptimizeSim3
// (:1054-1250) over the rsc C ABI: the g2o Levenberg-Marquardt runs on the MI355X (librsc.so), one
// workgroup per Frame / KeyFrame pair.
//
// FrameT needs (include/Frame.hpp): mvpMapPoints (pointer-likes, tested for null), mvuRight,
// mvKeysUn[i].pt.{x,y} and .octave, mvInvLevelSigma2[], fx, fy, cx, cy, mbf, mTcw with operator()(r,c)
// (Eigen::Isometry3f), SetPose(const decltype(mTcw)&), and mvbOutlier (std::vector<bool>).
// MapPoint::GetWorldPos() must return something indexable with (i).  In the reference tree:
//     int nGood = rsc_orb::PoseOptimization(&mCurrentFrame);       // Tracking.cpp:621,745,787,1284
// Slots with mvuRight >= 0 become EdgeStereoSE3ProjectXYZOnlyPose edges (Optimizer.cpp:290-323), the
// others monocular edges, exactly as the reference's stereo_euroc / stereo_kitti builds run it.
#pragma once
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

namespace detail {
template <class FrameT>
struct PoseOptInputs {
    std::vector<uint8_t> has_mp;
    std::vector<float> uv, Xw, inv, ur;
    std::vector<uint8_t> outlier;
    rsc_poseopt_problem pb;

    explicit PoseOptInputs(const FrameT& F) {
        const int N = (int)F.mvpMapPoints.size();
        has_mp.assign(N, 0);
        uv.assign(2 * (size_t)N, 0.0f);
        Xw.assign(3 * (size_t)N, 0.0f);
        inv.assign(N, 0.0f);
        ur.assign(N, -1.0f);
        outlier.assign(N > 0 ? N : 1, 0);
        for (int i = 0; i < N; ++i) {  // Optimizer.cpp:247-325 (under MapPoint::mGlobalMutex there)
            const auto& pMP = F.mvpMapPoints[i];
            if (!pMP) continue;
            has_mp[i] = 1;
            const auto& kp = F.mvKeysUn[i];
            uv[2 * i] = kp.pt.x;
            uv[2 * i + 1] = kp.pt.y;
            inv[i] = F.mvInvLevelSigma2[kp.octave];
            if ((size_t)i < F.mvuRight.size()) ur[i] = F.mvuRight[i];
            const auto X = pMP->GetWorldPos();
            Xw[3 * i] = X(0);
            Xw[3 * i + 1] = X(1);
            Xw[3 * i + 2] = X(2);
        }
        pb.n = N;
        pb.has_mp = has_mp.data();
        pb.uv = uv.data();
        pb.Xw = Xw.data();
        pb.inv_sigma2 = inv.data();
        pb.u_right = ur.data();
        pb.fx = F.fx; pb.fy = F.fy; pb.cx = F.cx; pb.cy = F.cy;
        pb.bf = F.mbf;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) pb.Tcw[4 * r + c] = F.mTcw(r, c);
    }

    // mvbOutlier and SetPose (Optimizer.cpp:255,347-376,420-421); returns nGood.
    int apply(FrameT& F, const rsc_poseopt_result& r) const {
        if ((int)F.mvbOutlier.size() < pb.n) F.mvbOutlier.resize(pb.n, false);
        for (int i = 0; i < pb.n; ++i)
            if (has_mp[i]) F.mvbOutlier[i] = outlier[i] != 0;
        if (r.n_initial >= 3) {
            auto T = F.mTcw;
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) T(a, b) = r.Tcw[4 * a + b];
            F.SetPose(T);
        }
        return r.n_good;
    }
};
}  // namespace detail

// Optimizer::PoseOptimization(Frame*) (Optimizer.cpp:205-424).
template <class FrameT>
int PoseOptimization(FrameT* pFrame) {
    detail::PoseOptInputs<FrameT> in(*pFrame);
    rsc_poseopt_result r;
    uint8_t* o = in.outlier.data();
    check(rsc_pose_optimization_many(thread_context(), &in.pb, 1, &r, &o), "PoseOptimization");
    return in.apply(*pFrame, r);
}

// PoseOptimization of several Frames in one launch (e.g. the relocalization candidates that
// returned a pose in the same round); results identical to calling PoseOptimization on each.
template <class FrameT>
std::vector<int> PoseOptimizationMany(const std::vector<FrameT*>& frames) {
    const int n = (int)frames.size();
    std::vector<detail::PoseOptInputs<FrameT>> in;
    in.reserve(n);
    for (FrameT* f : frames) in.emplace_back(*f);
    std::vector<rsc_poseopt_problem> pb(n);
    std::vector<uint8_t*> o(n);
    for (int i = 0; i < n; ++i) {
        pb[i] = in[i].pb;
        o[i] = in[i].outlier.data();
    }
    std::vector<rsc_poseopt_result> r(n);
    check(rsc_pose_optimization_many(thread_context(), pb.data(), n, r.data(), o.data()), "PoseOptimizationMany");
    std::vector<int> good(n);
    for (int i = 0; i < n; ++i) good[i] = in[i].apply(*frames[i], r[i]);
    return good;
}

// ---- Optimizer::OptimizeSim3 (Optimizer.cpp:1054-1250; LoopClosing.cpp:311) -----------------------
// KeyFrameT needs GetMapPointMatches(), GetRotation(), GetTranslation(), mvKeysUn[i].pt/.octave,
// mvInvLevelSigma2, mK (operator()(r, c)); MapPoint isBad(), GetWorldPos(), GetIndexInKeyFrame(pKF).
// Sim3T is g2o::Sim3 (or alike): rotation().coeffs()[0..3] = (x, y, z, w), translation()[0..2],
// scale(), all writable references — read on entry, written on return as the reference's
// `g2oS12 = vSim3_recov->estimate()` does (unchanged when the < 10 rule returns 0).
namespace detail {
template <class KFPtr, class MPPtr, class Sim3T>
struct Sim3OptInputs {
    std::vector<uint8_t> valid, keep;
    std::vector<float> X1w, X2w, uv1, uv2, inv1, inv2;
    rsc_sim3opt_problem pb;

    Sim3OptInputs(const KFPtr& pKF1, const KFPtr& pKF2, const std::vector<MPPtr>& vpMatches1, Sim3T& S,
                  float th2) {
        const int N = (int)vpMatches1.size();
        const auto vpMapPoints1 = pKF1->GetMapPointMatches();
        valid.assign(N > 0 ? N : 1, 0);
        keep.assign(N > 0 ? N : 1, 1);
        X1w.assign(3 * (size_t)N, 0.f);
        X2w.assign(3 * (size_t)N, 0.f);
        uv1.assign(2 * (size_t)N, 0.f);
        uv2.assign(2 * (size_t)N, 0.f);
        inv1.assign(N, 0.f);
        inv2.assign(N, 0.f);
        for (int i = 0; i < N; ++i) {  // Optimizer.cpp:1108-1143
            if (!vpMatches1[i]) continue;
            const auto& pMP1 = (size_t)i < vpMapPoints1.size() ? vpMapPoints1[i] : MPPtr();
            const auto& pMP2 = vpMatches1[i];
            const int i2 = pMP2->GetIndexInKeyFrame(pKF2);
            if (!pMP1 || pMP1->isBad() || pMP2->isBad() || i2 < 0) continue;
            valid[i] = 1;
            const auto a = pMP1->GetWorldPos();
            const auto b = pMP2->GetWorldPos();
            for (int c = 0; c < 3; ++c) {
                X1w[3 * i + c] = a(c);
                X2w[3 * i + c] = b(c);
            }
            const auto& k1 = pKF1->mvKeysUn[i];
            const auto& k2 = pKF2->mvKeysUn[i2];
            uv1[2 * i] = k1.pt.x;
            uv1[2 * i + 1] = k1.pt.y;
            uv2[2 * i] = k2.pt.x;
            uv2[2 * i + 1] = k2.pt.y;
            inv1[i] = pKF1->mvInvLevelSigma2[k1.octave];
            inv2[i] = pKF2->mvInvLevelSigma2[k2.octave];
        }
        pb.n = N;
        pb.valid = valid.data();
        pb.X1w = X1w.data(); pb.X2w = X2w.data();
        pb.uv1 = uv1.data(); pb.uv2 = uv2.data();
        pb.inv1 = inv1.data(); pb.inv2 = inv2.data();
        const auto R1 = pKF1->GetRotation();
        const auto t1 = pKF1->GetTranslation();
        const auto R2 = pKF2->GetRotation();
        const auto t2 = pKF2->GetTranslation();
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) {
                pb.R1w[3 * r + c] = R1(r, c);
                pb.R2w[3 * r + c] = R2(r, c);
            }
            pb.t1w[r] = t1(r);
            pb.t2w[r] = t2(r);
        }
        const auto& K1 = pKF1->mK;
        const auto& K2 = pKF2->mK;
        pb.K1[0] = K1(0, 0); pb.K1[1] = K1(1, 1); pb.K1[2] = K1(0, 2); pb.K1[3] = K1(1, 2);
        pb.K2[0] = K2(0, 0); pb.K2[1] = K2(1, 1); pb.K2[2] = K2(0, 2); pb.K2[3] = K2(1, 2);
        for (int k = 0; k < 4; ++k) pb.S[k] = S.rotation().coeffs()[k];
        for (int k = 0; k < 3; ++k) pb.S[4 + k] = S.translation()[k];
        pb.S[7] = S.scale();
        pb.th2 = th2;
    }

    int apply(std::vector<MPPtr>& vpMatches1, Sim3T& S, const rsc_sim3opt_result& r) const {
        for (size_t i = 0; i < vpMatches1.size(); ++i)
            if (!keep[i]) vpMatches1[i] = nullptr;  // vpMatches1[idx] = NULL (:1186, :1219)
        for (int k = 0; k < 4; ++k) S.rotation().coeffs()[k] = r.S[k];
        for (int k = 0; k < 3; ++k) S.translation()[k] = r.S[4 + k];
        S.scale() = r.S[7];
        return r.n_inliers;
    }
};
}  // namespace detail

// Optimizer::OptimizeSim3(pKF1, pKF2, vpMatches1, g2oS12, th2).
template <class KFPtr, class MPPtr, class Sim3T>
int OptimizeSim3(KFPtr pKF1, KFPtr pKF2, std::vector<MPPtr>& vpMatches1, Sim3T& g2oS12, const float th2) {
    detail::Sim3OptInputs<KFPtr, MPPtr, Sim3T> in(pKF1, pKF2, vpMatches1, g2oS12, th2);
    rsc_sim3opt_result r;
    uint8_t* k = in.keep.data();
    check(rsc_optimize_sim3_many(thread_context(), &in.pb, 1, &r, &k), "OptimizeSim3");
    return in.apply(vpMatches1, g2oS12, r);
}

}  // namespace rsc_orb
