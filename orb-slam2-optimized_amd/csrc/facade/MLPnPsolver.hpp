// MLPnPsolver.hpp — drop-in facade of ORB_SLAM_CUSTOM::MLPnPsolver (reference
// include/MLPnPsolver.hpp:10-21) over the rsc C ABI: same constructor, SetRansacParameters and
// iterate signatures and semantics (Tout = identity unless a pose is returned, MLPnPsolver.cpp:57).
// The reference never compiles this class (CMakeLists.txt:75); the facade exists for BASELINE
// config 4.  Type requirements as in PnPsolver.hpp.  In the reference tree:
//     using MLPnPsolver = rsc_orb::MLPnPsolver<Frame, MapPoint>;
#pragma once
#include <memory>
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

template <class FrameT, class MapPointT>
class MLPnPsolver {
public:
    // MLPnPsolver::MLPnPsolver (MLPnPsolver.cpp:5-53); calls SetRansacParameters() with the defaults.
    MLPnPsolver(const FrameT& F, const std::vector<std::shared_ptr<MapPointT>>& vpMapPointMatches, uint32_t seed = 1) {
        std::vector<float> p2d, p3d, s2;
        std::vector<int32_t> kp;
        for (size_t i = 0, iend = vpMapPointMatches.size(); i < iend; i++) {
            const std::shared_ptr<MapPointT>& pMP = vpMapPointMatches[i];
            if (!pMP || pMP->isBad()) continue;
            if (i >= F.mvKeysUn.size()) continue;  // (:25)
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
        rsc_pnp_problem pb;
        pb.n = (int32_t)kp.size();
        pb.n_points = (int32_t)vpMapPointMatches.size();
        pb.p2d = p2d.data();
        pb.p3dw = p3d.data();
        pb.sigma2 = s2.data();
        pb.kp_index = kp.data();
        pb.fx = F.fx; pb.fy = F.fy; pb.cx = F.cx; pb.cy = F.cy;
        check(rsc_mlpnp_create(thread_context(), &pb, seed, &s_), "rsc_mlpnp_create");
        if (rsc_stream* st = construction_stream()) check(rsc_mlpnp_bind_stream(s_, st), "rsc_mlpnp_bind_stream");
        n_points_ = pb.n_points;
    }
    ~MLPnPsolver() { rsc_mlpnp_destroy(s_); }
    MLPnPsolver(const MLPnPsolver&) = delete;
    MLPnPsolver& operator=(const MLPnPsolver&) = delete;

    void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300, int minSet = 6,
                             float epsilon = 0.4, float th2 = 5.991) {
        check(rsc_mlpnp_set_ransac_parameters(s_, probability, minInliers, maxIterations, minSet, epsilon, th2),
              "SetRansacParameters");
    }

    template <class Mat4>
    bool iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers, Mat4& Tout) {
        rsc_pnp_result r;
        std::vector<uint8_t> mask(n_points_ > 0 ? n_points_ : 1, 0);
        check(rsc_mlpnp_iterate(s_, nIterations, &r, mask.data()), "iterate");
        bNoMore = r.no_more != 0;
        nInliers = r.n_inliers;
        vbInliers.clear();
        if (r.ok) {
            vbInliers.assign(mask.size(), false);
            for (size_t i = 0; i < mask.size(); ++i) vbInliers[i] = mask[i] != 0;
        }
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) Tout(a, b) = r.T[4 * a + b];
        return r.ok != 0;
    }

    rsc_mlpnp* handle() { return s_; }

private:
    rsc_mlpnp* s_ = nullptr;
    int n_points_ = 0;
};

}  // namespace rsc_orb
