// PnPsolver.hpp — drop-in facade of ORB_SLAM_CUSTOM::PnPsolver (reference include/PnPsolver.hpp:21-31)
// over the rsc C ABI.  Same constructor, SetRansacParameters, find and iterate signatures and
// semantics; the EPnP RANSAC itself runs on the MI355X (librsc.so).
//
// Template parameters are the caller's types: FrameT needs mvKeysUn[i].pt.{x,y}, mvKeysUn[i].octave,
// mvLevelSigma2[], fx, fy, cx, cy (include/Frame.hpp:102-105,127,168); MapPointT needs isBad() and
// GetWorldPos() returning something indexable with (i) (MapPoint.cpp:58-62,199-204); the pose type
// of find/iterate needs operator()(r,c) (Eigen::Matrix4f).  In the reference tree:
//     using PnPsolver = rsc_orb::PnPsolver<Frame, MapPoint>;
#pragma once
#include <memory>
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

template <class FrameT, class MapPointT>
class PnPsolver {
public:
    // PnPsolver::PnPsolver (PnPsolver.cpp:11-55).  By default the solver draws from its thread's one
    // rand() stream (the reference's, rsc_context.hpp); `seed` is the per-solver stream srand(seed)
    // after the opt-in reference_rand(false) (H4).
    PnPsolver(const FrameT& F, const std::vector<std::shared_ptr<MapPointT>>& vpMapPointMatches, uint32_t seed = 1) {
        std::vector<float> p2d, p3d, s2;
        std::vector<int32_t> kp;
        for (size_t i = 0, iend = vpMapPointMatches.size(); i < iend; i++) {
            const std::shared_ptr<MapPointT>& pMP = vpMapPointMatches[i];
            if (pMP && !pMP->isBad()) {
                const auto& k = F.mvKeysUn[i];
                p2d.push_back(k.pt.x);
                p2d.push_back(k.pt.y);
                s2.push_back(F.mvLevelSigma2[k.octave]);
                const auto X = pMP->GetWorldPos();
                p3d.push_back(X(0));
                p3d.push_back(X(1));
                p3d.push_back(X(2));
                kp.push_back((int32_t)i);
            }
        }
        rsc_pnp_problem pb;
        pb.n = (int32_t)kp.size();
        pb.n_points = (int32_t)vpMapPointMatches.size();
        pb.p2d = p2d.data();
        pb.p3dw = p3d.data();
        pb.sigma2 = s2.data();
        pb.kp_index = kp.data();
        pb.fx = F.fx; pb.fy = F.fy; pb.cx = F.cx; pb.cy = F.cy;
        check(rsc_pnp_create(thread_context(), &pb, seed, &s_), "rsc_pnp_create");
        if (rsc_stream* st = construction_stream()) check(rsc_pnp_bind_stream(s_, st), "rsc_pnp_bind_stream");
        n_points_ = pb.n_points;
    }
    ~PnPsolver() { rsc_pnp_destroy(s_); }
    PnPsolver(const PnPsolver&) = delete;
    PnPsolver& operator=(const PnPsolver&) = delete;

    void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300, int minSet = 4,
                             float epsilon = 0.4, float th2 = 5.991) {
        check(rsc_pnp_set_ransac_parameters(s_, probability, minInliers, maxIterations, minSet, epsilon, th2),
              "SetRansacParameters");
    }

    template <class Mat4>
    bool find(std::vector<bool>& vbInliers, int& nInliers, Mat4& T) {
        int32_t st[8];
        check(rsc_pnp_get_state(s_, st), "get_state");
        bool bFlag;
        return iterate(st[1], bFlag, vbInliers, nInliers, T);
    }

    template <class Mat4>
    bool iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers, Mat4& T) {
        rsc_pnp_result r;
        std::vector<uint8_t> mask(n_points_ > 0 ? n_points_ : 1, 0);
        check(rsc_pnp_iterate(s_, nIterations, &r, mask.data()), "iterate");
        return unpack(r, mask, bNoMore, vbInliers, nInliers, T);
    }

    rsc_pnp* handle() { return s_; }

    template <class Mat4>
    static bool unpack(const rsc_pnp_result& r, const std::vector<uint8_t>& mask, bool& bNoMore,
                       std::vector<bool>& vbInliers, int& nInliers, Mat4& T) {
        bNoMore = r.no_more != 0;
        nInliers = r.n_inliers;
        vbInliers.clear();  // PnPsolver.cpp:105
        if (r.ok) {
            vbInliers.assign(mask.size(), false);
            for (size_t i = 0; i < mask.size(); ++i) vbInliers[i] = mask[i] != 0;
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 4; ++b) T(a, b) = r.T[4 * a + b];
        }
        return r.ok != 0;
    }

private:
    rsc_pnp* s_ = nullptr;
    int n_points_ = 0;
};

// All relocalization candidates' iterate() calls of one round in one launch (Tracking.cpp:1241-1255).
template <class Solver, class Mat4>
void iterate_round(std::vector<Solver*>& solvers, int nIterations, std::vector<char>& ok, std::vector<char>& noMore,
                   std::vector<std::vector<bool>>& inliers, std::vector<int>& nInliers, std::vector<Mat4>& T,
                   const std::vector<int>& n_points) {
    const int n = (int)solvers.size();
    std::vector<rsc_pnp*> h(n);
    std::vector<int32_t> its(n, nIterations);
    std::vector<rsc_pnp_result> r(n);
    std::vector<std::vector<uint8_t>> masks(n);
    std::vector<uint8_t*> mp(n);
    for (int i = 0; i < n; ++i) {
        h[i] = solvers[i]->handle();
        masks[i].assign(n_points[i] > 0 ? n_points[i] : 1, 0);
        mp[i] = masks[i].data();
    }
    check(rsc_pnp_iterate_many(h.data(), n, its.data(), r.data(), mp.data()), "iterate_many");
    ok.resize(n); noMore.resize(n); inliers.resize(n); nInliers.resize(n); T.resize(n);
    for (int i = 0; i < n; ++i) {
        bool nm;
        ok[i] = Solver::unpack(r[i], masks[i], nm, inliers[i], nInliers[i], T[i]);
        noMore[i] = nm;
    }
}

}  // namespace rsc_orb
