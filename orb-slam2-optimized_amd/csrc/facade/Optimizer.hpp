// Optimizer.hpp — drop-in facade of ORB_SLAM_CUSTOM::Optimizer::PoseOptimization
// (reference include/Optimizer.hpp, src/Optimizer.cpp:205-424) over the rsc C ABI: the g2o
// pose-only Levenberg-Marquardt runs on the MI355X (librsc.so), one workgroup per Frame.
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

}  // namespace rsc_orb
