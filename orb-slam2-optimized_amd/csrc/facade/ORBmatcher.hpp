// ORBmatcher.hpp — drop-in facade of ORB_SLAM_CUSTOM::ORBmatcher::SearchByBoW (reference
// include/ORBmatcher.hpp:35-60, src/ORBmatcher.cpp:110-240 and :354-488) over the rsc C ABI: the
// Hamming-256 node-restricted matching, ratio test and rotation-histogram filter run on the MI355X
// (librsc.so); results are bit-identical to the reference's sequential walk.
//
// KeyFrameT needs (include/KeyFrame.hpp): N, mDescriptors with template ptr<uint8_t>(row) (cv::Mat,
// 32 CV_8U columns), mvKeysUn[i].angle, mFeatVec (DBoW2::FeatureVector: std::map<NodeId,
// std::vector<unsigned int>>) and GetMapPointMatches() (pointer-likes with isBad()).  FrameT needs
// N, mDescriptors, mvKeys[i].angle and mFeatVec.  In the reference tree:
//     rsc_orb::ORBmatcher matcher(0.75, true);                               // Tracking.cpp:1199
//     int nmatches = matcher.SearchByBoW(pKF, mCurrentFrame, vvpMapPointMatches[i]);  // :1214
//     int nmatches = matcher.SearchByBoW(mpCurrentKF, pKF, vvpMapPointMatches[i]);   // LoopClosing.cpp:251
// and the batched forms run a whole candidate loop (Tracking.cpp:1207-1232,
// LoopClosing.cpp:238-265) in one launch with the shared view uploaded once.
#pragma once
#include <algorithm>
#include <memory>
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

namespace detail {

// A KeyFrame's or Frame's SearchByBoW inputs uploaded to HBM (rsc_bow_create).
struct BowUpload {
    rsc_bow* h = nullptr;
    int n = 0;
    BowUpload() = default;
    BowUpload(const BowUpload&) = delete;
    BowUpload& operator=(const BowUpload&) = delete;
    BowUpload(BowUpload&& o) noexcept : h(o.h), n(o.n) { o.h = nullptr; }
    ~BowUpload() { rsc_bow_destroy(h); }

    // angles(i) gives the keypoint angle the overload reads; valid(i) the map-point test (or true)
    template <class ViewT, class AngleF, class ValidF>
    void build(const ViewT& v, AngleF angles, ValidF valid) {
        n = (int)v.N;
        std::vector<uint8_t> desc(32 * (size_t)n), ok((size_t)n);
        std::vector<float> ang((size_t)n);
        for (int i = 0; i < n; ++i) {
            const uint8_t* row = v.mDescriptors.template ptr<uint8_t>(i);
            std::copy(row, row + 32, desc.begin() + 32 * (size_t)i);
            ang[i] = angles(i);
            ok[i] = valid(i) ? 1 : 0;
        }
        std::vector<uint32_t> ids, feat;
        std::vector<int32_t> begin(1, 0);
        for (const auto& node : v.mFeatVec) {  // std::map order = ascending node ids
            ids.push_back((uint32_t)node.first);
            for (auto f : node.second) feat.push_back((uint32_t)f);
            begin.push_back((int32_t)feat.size());
        }
        rsc_bow_features f;
        f.n = n;
        f.desc = desc.data();
        f.angle = ang.data();
        f.valid = ok.data();
        f.n_nodes = (int32_t)ids.size();
        f.node_id = ids.data();
        f.node_begin = begin.data();
        f.feat = feat.data();
        check(rsc_bow_create(thread_context(), &f, &h), "rsc_bow_create");
    }
};

// pKF side: mvKeysUn angles (ORBmatcher.cpp:185, :435), valid = map point present and not bad
template <class KFPtr>
BowUpload upload_keyframe(const KFPtr& pKF) {
    const auto mps = pKF->GetMapPointMatches();
    BowUpload u;
    u.build(*pKF, [&](int i) { return (float)pKF->mvKeysUn[i].angle; },
            [&](int i) { return (size_t)i < mps.size() && mps[i] && !mps[i]->isBad(); });
    return u;
}

// Frame side of the Frame overload: mvKeys angles (:185), no map-point test
template <class FrameT>
BowUpload upload_frame(const FrameT& F) {
    BowUpload u;
    u.build(F, [&](int i) { return (float)F.mvKeys[i].angle; }, [](int) { return true; });
    return u;
}

}  // namespace detail

class ORBmatcher {
public:
    // ORBmatcher::ORBmatcher (ORBmatcher.cpp:12; defaults include/ORBmatcher.hpp:35)
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    // SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cpp:110-240)
    template <class KFPtr, class FrameT, class MPPtr>
    int SearchByBoW(KFPtr pKF, FrameT& F, std::vector<MPPtr>& vpMapPointMatches) {
        std::vector<KFPtr> kfs(1, pKF);
        std::vector<std::vector<MPPtr>> out;
        const int n = SearchByBoWMany(kfs, F, out)[0];
        vpMapPointMatches.swap(out[0]);
        return n;
    }

    // SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.cpp:354-488)
    template <class KFPtr, class MPPtr>
    int SearchByBoW(KFPtr pKF1, KFPtr pKF2, std::vector<MPPtr>& vpMatches12) {
        std::vector<KFPtr> kf2s(1, pKF2);
        std::vector<std::vector<MPPtr>> out;
        const int n = SearchByBoWMany(pKF1, kf2s, out)[0];
        vpMatches12.swap(out[0]);
        return n;
    }

    // SearchByBoW(vpKFs[c], F, out[c]) for every candidate in one launch (Tracking.cpp:1207-1232).
    template <class KFPtr, class FrameT, class MPPtr>
    std::vector<int> SearchByBoWMany(const std::vector<KFPtr>& vpKFs, FrameT& F,
                                     std::vector<std::vector<MPPtr>>& out) {
        const int C = (int)vpKFs.size();
        detail::BowUpload frame = detail::upload_frame(F);
        std::vector<detail::BowUpload> kfs;
        std::vector<rsc_bow*> hs;
        std::vector<std::vector<MPPtr>> mps;
        kfs.reserve(C);
        for (const auto& k : vpKFs) {
            kfs.push_back(detail::upload_keyframe(k));
            hs.push_back(kfs.back().h);
            mps.push_back(k->GetMapPointMatches());
        }
        std::vector<std::vector<int32_t>> idx(C, std::vector<int32_t>(frame.n > 0 ? frame.n : 1));
        std::vector<int32_t*> ptr(C);
        for (int c = 0; c < C; ++c) ptr[c] = idx[c].data();
        std::vector<int32_t> nm(C > 0 ? C : 1, 0);
        check(rsc_search_by_bow_frame_many(thread_context(), hs.data(), C, frame.h, mfNNratio,
                                           mbCheckOrientation ? 1 : 0, ptr.data(), nm.data()),
              "SearchByBoW(KeyFrame, Frame)");
        out.assign(C, std::vector<MPPtr>(frame.n, nullptr));  // vector<MapPoint*>(F.N, NULL) (:114)
        for (int c = 0; c < C; ++c)
            for (int i = 0; i < frame.n; ++i)
                if (idx[c][i] >= 0) out[c][i] = mps[c][idx[c][i]];
        return std::vector<int>(nm.begin(), nm.begin() + C);
    }

    // SearchByBoW(pKF1, vpKF2[c], out[c]) for every loop candidate in one launch
    // (LoopClosing.cpp:238-265).
    template <class KFPtr, class MPPtr>
    std::vector<int> SearchByBoWMany(KFPtr pKF1, const std::vector<KFPtr>& vpKF2,
                                     std::vector<std::vector<MPPtr>>& out) {
        const int C = (int)vpKF2.size();
        detail::BowUpload kf1 = detail::upload_keyframe(pKF1);
        std::vector<detail::BowUpload> kf2;
        std::vector<rsc_bow*> hs;
        std::vector<std::vector<MPPtr>> mps;
        kf2.reserve(C);
        for (const auto& k : vpKF2) {
            kf2.push_back(detail::upload_keyframe(k));
            hs.push_back(kf2.back().h);
            mps.push_back(k->GetMapPointMatches());
        }
        const int n1 = (int)pKF1->GetMapPointMatches().size();
        std::vector<std::vector<int32_t>> idx(C, std::vector<int32_t>(kf1.n > 0 ? kf1.n : 1));
        std::vector<int32_t*> ptr(C);
        for (int c = 0; c < C; ++c) ptr[c] = idx[c].data();
        std::vector<int32_t> nm(C > 0 ? C : 1, 0);
        check(rsc_search_by_bow_kf_many(thread_context(), kf1.h, hs.data(), C, mfNNratio, mbCheckOrientation ? 1 : 0,
                                        ptr.data(), nm.data()),
              "SearchByBoW(KeyFrame, KeyFrame)");
        out.assign(C, std::vector<MPPtr>(n1, nullptr));  // vpMatches12 sized vpMapPoints1 (:366)
        for (int c = 0; c < C; ++c)
            for (int i = 0; i < kf1.n && i < n1; ++i)
                if (idx[c][i] >= 0) out[c][i] = mps[c][idx[c][i]];
        return std::vector<int>(nm.begin(), nm.begin() + C);
    }

private:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace rsc_orb
