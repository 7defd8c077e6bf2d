// KeyFrameDatabase.hpp — drop-in facade of ORB_SLAM_CUSTOM::KeyFrameDatabase (reference
// include/KeyFrameDatabase.hpp, src/KeyFrameDatabase.cpp) over the rsc C ABI: the inverted-file
// walk, DBoW2 L1 scoring, covisibility accumulation and retain run on the MI355X against a
// device-resident database (rsc_kfdb_*); candidates are the reference's vectors, in its order.
//
// KeyFramePtr needs (include/KeyFrame.hpp): mnId, mBowVec (DBoW2::BowVector: std::map<WordId,
// WordValue>), GetBestCovisibilityKeyFrames(10) and GetConnectedKeyFrames(); FrameT needs mnId and
// mBowVec.  VocT needs size() (mvInvertedFile.resize(voc->size()), KeyFrameDatabase.cpp:11).
// The per-KeyFrame query state (mnLoopQuery, mnLoopWords, mLoopScore, mnRelocQuery, mnRelocWords,
// mRelocScore) lives on the device, one slot per KeyFrame seen by this database, so callers must not
// rely on those KeyFrame members.  The covisibility of every known KeyFrame is refreshed (one
// upload) before each query, as the reference reads GetBestCovisibilityKeyFrames at query time.
// One mutex serialises the calls, as the reference's mMutex does (Tracking, LocalMapping and
// LoopClosing threads share the database).  In the reference tree:
//     mpKeyFrameDatabase = new rsc_orb::KeyFrameDatabase<std::shared_ptr<KeyFrame>>(mpVocabulary);
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>
#include "rsc_context.hpp"

namespace rsc_orb {

template <class KeyFramePtr>
class KeyFrameDatabase {
public:
    // KeyFrameDatabase(voc) (:8-13); capacity = the most KeyFrames the map will hold
    template <class VocPtr>
    explicit KeyFrameDatabase(const VocPtr& voc, int capacity = 1 << 16, int max_words = 4096) {
        check(rsc_context_create(device(), &ctx_), "rsc_context_create");
        check(rsc_kfdb_create(ctx_, (uint32_t)voc->size(), capacity, max_words, &db_), "rsc_kfdb_create");
    }
    KeyFrameDatabase(const KeyFrameDatabase&) = delete;
    KeyFrameDatabase& operator=(const KeyFrameDatabase&) = delete;
    ~KeyFrameDatabase() {
        rsc_kfdb_destroy(db_);
        rsc_context_destroy(ctx_);
    }

    // add(pKF) (:15-21)
    void add(KeyFramePtr pKF) {
        std::lock_guard<std::mutex> lock(mutex_);
        std::vector<uint32_t> ids;
        std::vector<double> vals;
        bow(pKF->mBowVec, ids, vals);
        check(rsc_kfdb_add(db_, slot(pKF), (int)ids.size(), ids.data(), vals.data()), "KeyFrameDatabase::add");
    }

    // erase(pKF) (:23-43)
    void erase(KeyFramePtr pKF) {
        std::lock_guard<std::mutex> lock(mutex_);
        auto it = slots_.find(pKF.get());
        if (it != slots_.end()) check(rsc_kfdb_erase(db_, it->second), "KeyFrameDatabase::erase");
    }

    // clear() (:45-49)
    void clear() {
        std::lock_guard<std::mutex> lock(mutex_);
        check(rsc_kfdb_clear(db_), "KeyFrameDatabase::clear");
    }

    // DetectLoopCandidates(pKF, minScore) (:52-172)
    std::vector<KeyFramePtr> DetectLoopCandidates(KeyFramePtr pKF, float minScore) {
        std::lock_guard<std::mutex> lock(mutex_);
        std::vector<int32_t> conn;
        for (const auto& k : pKF->GetConnectedKeyFrames()) conn.push_back(slot(k));
        std::vector<uint32_t> ids;
        std::vector<double> vals;
        bow(pKF->mBowVec, ids, vals);
        refresh_covisibility();
        std::vector<int32_t> cand(kfs_.size() + 1);
        int32_t n = 0;
        check(rsc_kfdb_detect_loop(db_, (uint64_t)pKF->mnId, (int)ids.size(), ids.data(), vals.data(),
                                   (int)conn.size(), conn.data(), minScore, cand.data(), &n),
              "DetectLoopCandidates");
        return resolve(cand, n);
    }

    // DetectRelocalizationCandidates(F) (:174-283)
    template <class FrameT>
    std::vector<KeyFramePtr> DetectRelocalizationCandidates(FrameT* F) {
        std::lock_guard<std::mutex> lock(mutex_);
        std::vector<uint32_t> ids;
        std::vector<double> vals;
        bow(F->mBowVec, ids, vals);
        refresh_covisibility();
        std::vector<int32_t> cand(kfs_.size() + 1);
        int32_t n = 0;
        check(rsc_kfdb_detect_relocalization(db_, (uint64_t)F->mnId, (int)ids.size(), ids.data(), vals.data(),
                                             cand.data(), &n),
              "DetectRelocalizationCandidates");
        return resolve(cand, n);
    }

private:
    static int device() {
        const char* d = std::getenv("RSC_DEVICE");
        return d ? std::atoi(d) : 0;
    }

    template <class BowVec>
    static void bow(const BowVec& v, std::vector<uint32_t>& ids, std::vector<double>& vals) {
        for (const auto& w : v) {  // std::map: ascending word ids
            ids.push_back((uint32_t)w.first);
            vals.push_back((double)w.second);
        }
    }

    // the KeyFrame's slot (its query state lives there), assigned on first sight
    int slot(const KeyFramePtr& k) {
        auto it = slots_.find(k.get());
        if (it != slots_.end()) return it->second;
        const int s = (int)kfs_.size();
        slots_.emplace(k.get(), s);
        kfs_.push_back(k);
        return s;
    }

    // GetBestCovisibilityKeyFrames(10) of every known KeyFrame, one upload
    void refresh_covisibility() {
        const int n = (int)kfs_.size();
        std::vector<int32_t> kf(n), cnt(n), best((size_t)n * 10, 0);
        for (int i = 0; i < n; ++i) {
            kf[i] = i;
            const auto nb = kfs_[i]->GetBestCovisibilityKeyFrames(10);
            cnt[i] = (int32_t)nb.size();
            for (int j = 0; j < cnt[i]; ++j) best[(size_t)i * 10 + j] = slot(nb[j]);
        }
        check(rsc_kfdb_set_covisibility_many(db_, n, kf.data(), cnt.data(), best.data()), "covisibility");
    }

    std::vector<KeyFramePtr> resolve(const std::vector<int32_t>& cand, int n) const {
        std::vector<KeyFramePtr> out;
        out.reserve(n);
        for (int i = 0; i < n; ++i) out.push_back(kfs_[cand[i]]);
        return out;
    }

    rsc_context* ctx_ = nullptr;
    rsc_kfdb* db_ = nullptr;
    std::mutex mutex_;
    std::unordered_map<const void*, int> slots_;
    std::vector<KeyFramePtr> kfs_;
};

}  // namespace rsc_orb
