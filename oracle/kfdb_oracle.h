// TEST INFRASTRUCTURE — parity oracle, never linked into the product library.
//
// Sequential CPU restatement of KeyFrameDatabase (src/KeyFrameDatabase.cpp): the inverted file
// (add :15-21, erase :23-43, clear :45-49) and the two BoW candidate queries,
// DetectLoopCandidates (:52-172) and DetectRelocalizationCandidates (:174-283), with DBoW2's
// L1 score (Thirdparty/DBoW2/DBoW2/ScoringObject.cpp:23-67; the ORB vocabulary's scoring type,
// ORBvoc.txt header "10 6 0 0" = L1_NORM, TF_IDF).
//
// KeyFrames are slots 0..capacity-1.  The per-KeyFrame query state the reference keeps in
// KeyFrame members (mnLoopQuery, mnLoopWords, mLoopScore, mnRelocQuery, mnRelocWords,
// mRelocScore; include/KeyFrame.hpp:129-134, KeyFrame.cpp:15 zero-initialises the ids and word
// counts) lives here per slot and persists across queries, so the reference's cross-query quirks
// are reproduced: a covisible neighbour that shares words but was not scored in this query
// contributes its previous mRelocScore (:245-252).  mLoopScore / mRelocScore are uninitialised in
// the reference (undefined on a first read); this restatement defines them as 0.
// GetBestCovisibilityKeyFrames(10) (KeyFrame.cpp:161-169) is the per-slot neighbour list the
// caller sets.
#pragma once
#include <cstdint>
#include <list>
#include <map>
#include <vector>

namespace rsc_oracle {

class KFDatabase {
public:
    explicit KFDatabase(int capacity);
    // KeyFrameDatabase::add: pKF->mBowVec = (ids ascending, values)
    void add(int kf, int n, const uint32_t* ids, const double* vals);
    void erase(int kf);
    void clear();
    void set_covisibility(int kf, int n, const int32_t* best);
    // returns the candidate slots in the reference's vector order
    std::vector<int> detect_relocalization(uint64_t frame_id, int n, const uint32_t* ids, const double* vals);
    std::vector<int> detect_loop(uint64_t kf_id, int n, const uint32_t* ids, const double* vals,
                                 int n_connected, const int32_t* connected, float min_score);
    // per-slot state (for tests)
    struct State {
        uint64_t loop_query = 0, reloc_query = 0;
        int loop_words = 0, reloc_words = 0;
        float loop_score = 0.f, reloc_score = 0.f;
    };
    const State& state(int kf) const { return st_[kf]; }

private:
    int cap_;
    std::map<uint32_t, std::list<int>> inv_;  // mvInvertedFile (only non-empty words materialised)
    std::vector<std::map<uint32_t, double>> bow_;  // mBowVec of each slot (as last added)
    std::vector<std::vector<int>> covis_;
    std::vector<State> st_;
};

// L1Scoring::score(v1, v2) (ScoringObject.cpp:23-67), v1/v2 sorted by word id
double l1_score(int n1, const uint32_t* id1, const double* v1, int n2, const uint32_t* id2, const double* v2);

}  // namespace rsc_oracle
