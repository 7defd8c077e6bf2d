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
//
// SearchBySim3 (ORBmatcher.cpp:948-1170, LoopClosing.cpp:309) additionally needs, per KeyFrame,
// mvKeysUn[i].pt/.octave, mDescriptors, fx..cy, mnMinX..mnMaxY, mfGridElementWidth/HeightInv,
// mvScaleFactors, mnScaleLevels, mfLogScaleFactor, GetRotation(), GetTranslation(),
// GetMapPointMatches(); per MapPoint isBad(), GetWorldPos(), GetDescriptor() (one cv::Mat row),
// GetIndexInKeyFrame(pKF).  Three members the reference keeps protected are read through the
// customization points below, whose defaults call one-line getters INTEGRATION.md §2 adds to the
// reference: KeyFrame::GetGrid() (mGrid: the grid cannot be rebuilt from the KeyFrame's integer
// image bounds, Frame assigned it with float bounds) and MapPoint::GetMaxDistance()/GetMinDistance()
// (mfMaxDistance/mfMinDistance: GetMaxDistanceInvariance() returns 1.2f*mfMaxDistance, which does
// not round-trip in float).
#pragma once
#include <algorithm>
#include <memory>
#include <stdexcept>
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

// ---- SearchBySim3 ----------------------------------------------------------------------------------
// Customization points (specialise for types with other accessors).
template <class KF>
const auto& kf_grid(const KF& kf) { return kf.GetGrid(); }                   // KeyFrame::mGrid
template <class MP>
float mp_max_distance(MP& mp) { return mp.GetMaxDistance(); }                // MapPoint::mfMaxDistance
template <class MP>
float mp_min_distance(MP& mp) { return mp.GetMinDistance(); }                // MapPoint::mfMinDistance

// A KeyFrame's SearchBySim3 inputs uploaded to HBM (rsc_kfview_create).
struct KFViewUpload {
    rsc_kfview* h = nullptr;
    int n = 0;
    KFViewUpload() = default;
    KFViewUpload(const KFViewUpload&) = delete;
    KFViewUpload& operator=(const KFViewUpload&) = delete;
    KFViewUpload(KFViewUpload&& o) noexcept : h(o.h), n(o.n) { o.h = nullptr; }
    ~KFViewUpload() { rsc_kfview_destroy(h); }
};

template <class KFPtr, class MPPtr>
KFViewUpload upload_kfview(const KFPtr& pKF, const std::vector<MPPtr>& mps) {
    const auto& K = *pKF;
    const int n = (int)K.N;
    std::vector<float> kp(2 * (size_t)n), pos(3 * (size_t)n, 0.f), dmax((size_t)n, 0.f), dmin((size_t)n, 0.f);
    std::vector<int32_t> oct((size_t)n);
    std::vector<uint8_t> desc(32 * (size_t)n), state((size_t)n, 0), mdesc(32 * (size_t)n, 0);
    for (int i = 0; i < n; ++i) {
        kp[2 * i] = K.mvKeysUn[i].pt.x;
        kp[2 * i + 1] = K.mvKeysUn[i].pt.y;
        oct[i] = K.mvKeysUn[i].octave;
        const uint8_t* row = K.mDescriptors.template ptr<uint8_t>(i);
        std::copy(row, row + 32, desc.begin() + 32 * (size_t)i);
        if ((size_t)i >= mps.size() || !mps[i]) continue;  // vpMapPoints[i] NULL
        auto& mp = *mps[i];
        if (mp.isBad()) { state[i] = 2; continue; }
        state[i] = 1;
        const auto X = mp.GetWorldPos();
        for (int c = 0; c < 3; ++c) pos[3 * i + c] = X(c);
        dmax[i] = mp_max_distance(mp);
        dmin[i] = mp_min_distance(mp);
        const auto d = mp.GetDescriptor();
        const uint8_t* dr = d.template ptr<uint8_t>(0);
        std::copy(dr, dr + 32, mdesc.begin() + 32 * (size_t)i);
    }
    const auto& grid = kf_grid(K);  // mGrid[ix][iy] -> CSR over cell = ix * 48 + iy
    if (grid.size() != 64) throw std::runtime_error("rsc: SearchBySim3: FRAME_GRID_COLS must be 64");
    std::vector<int32_t> begin(1, 0), feat;
    for (int ix = 0; ix < 64; ++ix) {
        if (grid[ix].size() != 48) throw std::runtime_error("rsc: SearchBySim3: FRAME_GRID_ROWS must be 48");
        for (int iy = 0; iy < 48; ++iy) {
            for (auto f : grid[ix][iy]) feat.push_back((int32_t)f);
            begin.push_back((int32_t)feat.size());
        }
    }
    if (feat.empty()) feat.push_back(0);
    rsc_sim3_kf k;
    k.n = n;
    k.kp = kp.data();
    k.octave = oct.data();
    k.desc = desc.data();
    k.cell_begin = begin.data();
    k.cell_feat = feat.data();
    k.min_x = (float)K.mnMinX; k.max_x = (float)K.mnMaxX; k.min_y = (float)K.mnMinY; k.max_y = (float)K.mnMaxY;
    k.grid_w_inv = K.mfGridElementWidthInv;
    k.grid_h_inv = K.mfGridElementHeightInv;
    k.fx = K.fx; k.fy = K.fy; k.cx = K.cx; k.cy = K.cy;
    k.scale_factors = K.mvScaleFactors.data();
    k.n_levels = (int32_t)K.mnScaleLevels;
    k.log_scale_factor = K.mfLogScaleFactor;
    const auto R = pKF->GetRotation();
    const auto t = pKF->GetTranslation();
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) k.Rcw[3 * r + c] = R(r, c);
        k.tcw[r] = t(r);
    }
    k.mp_state = state.data();
    k.mp_pos = pos.data();
    k.mp_dmax = dmax.data();
    k.mp_dmin = dmin.data();
    k.mp_desc = mdesc.data();
    KFViewUpload u;
    u.n = n;
    check(rsc_kfview_create(thread_context(), &k, &u.h), "rsc_kfview_create");
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

    // SearchBySim3(pKF1, pKF2, vpMatches12, R12, t12, th) (ORBmatcher.cpp:948-1170;
    // LoopClosing.cpp:309 after a Sim3Solver success): new mutual matches are written into
    // vpMatches12 (entries already set are kept), returns their number.
    template <class KFPtr, class MPPtr, class Mat3, class Vec3>
    int SearchBySim3(KFPtr pKF1, KFPtr pKF2, std::vector<MPPtr>& vpMatches12, const Mat3& R12, const Vec3& t12,
                     const float th) {
        std::vector<std::vector<MPPtr>*> m(1, &vpMatches12);
        std::vector<KFPtr> a(1, pKF1), b(1, pKF2);
        float R[9], t[3];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) R[3 * r + c] = R12(r, c);
            t[r] = t12(r);
        }
        return SearchBySim3Many(a, b, m, R, t, th)[0];
    }

    // SearchBySim3 of several (pKF1[c], pKF2[c]) pairs in one launch; R12 [count][9] row-major,
    // t12 [count][3].  Each KeyFrame object is uploaded once.
    template <class KFPtr, class MPPtr>
    std::vector<int> SearchBySim3Many(const std::vector<KFPtr>& pKF1, const std::vector<KFPtr>& pKF2,
                                      const std::vector<std::vector<MPPtr>*>& vpMatches12, const float* R12,
                                      const float* t12, const float th) {
        const int C = (int)pKF1.size();
        std::vector<const void*> keys;
        std::vector<detail::KFViewUpload> views;
        std::vector<std::vector<MPPtr>> mps;
        auto view_of = [&](const KFPtr& k) {
            for (size_t j = 0; j < keys.size(); ++j)
                if (keys[j] == (const void*)&*k) return (int)j;
            keys.push_back((const void*)&*k);
            mps.push_back(k->GetMapPointMatches());
            views.push_back(detail::upload_kfview(k, mps.back()));
            return (int)keys.size() - 1;
        };
        std::vector<int> v1(C), v2(C);
        for (int c = 0; c < C; ++c) {
            v1[c] = view_of(pKF1[c]);
            v2[c] = view_of(pKF2[c]);
        }
        std::vector<rsc_kfview*> h1(C), h2(C);
        std::vector<std::vector<int32_t>> in(C), out(C);
        std::vector<const int32_t*> pin(C);
        std::vector<int32_t*> pout(C);
        for (int c = 0; c < C; ++c) {
            h1[c] = views[v1[c]].h;
            h2[c] = views[v2[c]].h;
            const int n1 = views[v1[c]].n;
            const std::vector<MPPtr>& m = *vpMatches12[c];
            in[c].assign(n1 > 0 ? n1 : 1, -1);
            out[c].assign(n1 > 0 ? n1 : 1, -1);
            for (int i = 0; i < n1 && (size_t)i < m.size(); ++i) {  // vbAlreadyMatched1/2 (:980-990)
                if (!m[i]) continue;
                const int idx2 = m[i]->GetIndexInKeyFrame(pKF2[c]);
                in[c][i] = (idx2 >= 0 && idx2 < views[v2[c]].n) ? idx2 : -2;
            }
            pin[c] = in[c].data();
            pout[c] = out[c].data();
        }
        std::vector<int32_t> nfound(C > 0 ? C : 1, 0);
        check(rsc_search_by_sim3_many(thread_context(), h1.data(), h2.data(), C, R12, t12, th, pin.data(), pout.data(),
                                      nfound.data()),
              "SearchBySim3");
        for (int c = 0; c < C; ++c) {  // vpMatches12[i1] = vpMapPoints2[idx2] (:1160-1166)
            std::vector<MPPtr>& m = *vpMatches12[c];
            const std::vector<MPPtr>& mp2 = mps[v2[c]];
            for (int i = 0; i < views[v1[c]].n && (size_t)i < m.size(); ++i)
                if (out[c][i] >= 0) m[i] = mp2[out[c][i]];
        }
        return std::vector<int>(nfound.begin(), nfound.begin() + C);
    }

private:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace rsc_orb
