// KeyFrameDatabase.hpp — drop-in facade of ORB_SLAM_CUSTOM::KeyFrameDatabase (reference
// include/KeyFrameDatabase.hpp, src/KeyFrameDatabase.cpp) over the rsc C ABI: the inverted-file
// walk, DBoW2 L1 scoring, covisibility accumulation and retain run on the MI355X against a
// device-resident database (rsc_kfdb_*); candidates are the reference's vectors, in its order.
//
// KeyFramePtr needs (include/KeyFrame.hpp): mnId, mBowVec (DBoW2::BowVector: std::map<WordId,
// WordValue>), GetBestCovisibilityKeyFrames(10) and GetConnectedKeyFrames(); FrameT needs mnId and
// mBowVec.  VocT needs size() (mvInvertedFile.resize(voc->size()), KeyFrameDatabase.cpp:11).
// The per-KeyFrame query state (mnLoopQuery, mnLoopWords, mLoopScore, mnRelocQuery, mnRelocWords,
// mRelocScore) lives on the device, one slot per KeyFrame in the database, so callers must not
// rely on those KeyFrame members.  Slots (slot 0 is reserved, see kNone) are taken on add() and given
// back on erase(), with their state reset: a KeyFrame outside the database is never in the inverted
// file, so its query state can never match a query, and every such KeyFrame met through
// covisibility or connections is represented by the one never-added slot kNone (same outcome).
// The covisibility of every KeyFrame in the database is refreshed before each query, as the
// reference reads GetBestCovisibilityKeyFrames at query time; only rows that changed are uploaded.
// One mutex serialises the calls, as the reference's mMutex does (Tracking, LocalMapping and
// LoopClosing threads share the database).  In the reference tree:
//     mpKeyFrameDatabase = new rsc_orb::KeyFrameDatabase<std::shared_ptr<KeyFrame>>(mpVocabulary);
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
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
        capacity_ = capacity + 1;  // + the kNone slot
        check(rsc_kfdb_create(ctx_, (uint32_t)voc->size(), capacity_, max_words, &db_), "rsc_kfdb_create");
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
        const bool fresh = slots_.find(pKF.get()) == slots_.end();
        const int s = take_slot(pKF);
        const int st = rsc_kfdb_add(db_, s, (int)ids.size(), ids.data(), vals.data());
        if (st != RSC_OK && fresh) give_back(s);
        check(st, "KeyFrameDatabase::add");
    }

    // erase(pKF) (:23-43): the KeyFrame leaves the inverted file; its slot is reused
    void erase(KeyFramePtr pKF) {
        std::lock_guard<std::mutex> lock(mutex_);
        auto it = slots_.find(pKF.get());
        if (it == slots_.end()) return;
        const int s = it->second;
        check(rsc_kfdb_release(db_, s), "KeyFrameDatabase::erase");
        give_back(s);
    }

    // clear() (:45-49): empties the inverted file (the KeyFrames keep their query state and slots)
    void clear() {
        std::lock_guard<std::mutex> lock(mutex_);
        check(rsc_kfdb_clear(db_), "KeyFrameDatabase::clear");
    }

    // DetectLoopCandidates(pKF, minScore) (:52-172)
    std::vector<KeyFramePtr> DetectLoopCandidates(KeyFramePtr pKF, float minScore) {
        std::lock_guard<std::mutex> lock(mutex_);
        std::vector<int32_t> conn;  // only KeyFrames in the database can be excluded from the walk
        for (const auto& k : pKF->GetConnectedKeyFrames()) {
            const int s = slot_of(k);
            if (s != kNone) conn.push_back(s);
        }
        std::vector<uint32_t> ids;
        std::vector<double> vals;
        bow(pKF->mBowVec, ids, vals);
        refresh_covisibility();
        std::vector<int32_t> cand(kfs_.size() + 1);  // one more than the slots in use
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

    static constexpr int kNone = 0;  // never added: stands for every KeyFrame outside the database

    int slot_of(const KeyFramePtr& k) const {
        auto it = slots_.find(k.get());
        return it == slots_.end() ? kNone : it->second;
    }

    // the KeyFrame's slot (its query state lives there), taken when it joins the database
    int take_slot(const KeyFramePtr& k) {
        auto it = slots_.find(k.get());
        if (it != slots_.end()) return it->second;
        int s;
        if (!free_.empty()) {
            s = free_.back();
            free_.pop_back();
        } else {
            if ((int)kfs_.size() >= capacity_)
                throw std::runtime_error("rsc_orb::KeyFrameDatabase: " + std::to_string(capacity_ - 1) +
                                         " KeyFrames are in the database (its capacity); erase some or "
                                         "construct it with a larger capacity");
            s = (int)kfs_.size();
            kfs_.push_back(nullptr);
        }
        slots_.emplace(k.get(), s);
        kfs_[s] = k;
        return s;
    }

    void give_back(int s) {
        slots_.erase(kfs_[s].get());
        kfs_[s] = nullptr;  // the database no longer holds the KeyFrame alive
        free_.push_back(s);
    }

    // GetBestCovisibilityKeyFrames(10) of every KeyFrame in the database; the C ABI uploads only
    // the rows that changed since the last query
    void refresh_covisibility() {
        std::vector<int32_t> kf, cnt, best;
        for (int i = 1; i < (int)kfs_.size(); ++i) {
            if (!kfs_[i]) continue;
            const auto nb = kfs_[i]->GetBestCovisibilityKeyFrames(10);
            kf.push_back(i);
            cnt.push_back((int32_t)nb.size());
            for (int j = 0; j < 10; ++j) best.push_back(j < (int)nb.size() ? slot_of(nb[j]) : 0);
        }
        check(rsc_kfdb_set_covisibility_many(db_, (int)kf.size(), kf.data(), cnt.data(), best.data()),
              "covisibility");
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
    int capacity_ = 0;
    std::unordered_map<const void*, int> slots_;
    std::vector<KeyFramePtr> kfs_{KeyFramePtr()};  // [slot]; slot 0 = kNone
    std::vector<int> free_;
};

}  // namespace rsc_orb
