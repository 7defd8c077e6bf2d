// rsc_kfdb.h — KeyFrameDatabase BoW candidate scoring (src/KeyFrameDatabase.cpp:52-283) on the GPU:
// device layout.
//
// The database lives in HBM as fixed-stride slots: slot k holds its BowVector (word ids ascending,
// TF-IDF values) at [k * max_words, k * max_words + len[k]), its add order seq[k] (the position
// the reference's inverted-file lists give it: add() appends to every word's list, erase() removes
// without reordering, so each list is in ascending seq), its best-10 covisibility list and the
// per-KeyFrame query state (KeyFrame.hpp:129-134).  A query runs two kernels:
//   count:      one wave per slot, the query BowVector staged in each workgroup's LDS as a hash —
//               a probe per slot word gives the common-word count (the number of times the
//               reference's inverted-file walk meets the slot) and the first query word it meets
//               (the list position); the state update reproduces the
//               walk's per-occurrence rules exactly; a slot that enters lKFsSharingWords also gets
//               its DBoW2 L1 score here (terms in parallel, summed in ascending word order through
//               the wave's shuffles), while its words are in cache and off the finish kernel's
//               single-workgroup critical path (kept only for the slots finish scores).
//   finish:     one workgroup — maxCommonWords, minCommonWords = int(max * 0.8f), the scored slots
//               in lKFsSharingWords order (rank by (first query word, seq)) and their scores;
//               covisibility accumulation, 0.75 * best retain,
//               first-occurrence de-duplication; candidates in the reference's vector order.
// Integer/latency-bound work (a few bytes per BowVector entry, no MFMA); the HBM stream is the
// slots' word ids (4 B per word) in `count`, plus the values of the common words.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace rsc {

constexpr int kKfdbMaxWords = 4096;  // BowVector bound (words per KeyFrame / Frame)
constexpr int kKfdbCovis = 10;       // GetBestCovisibilityKeyFrames(10)

struct DevKFDB {
    int cap, max_words;
    uint32_t vocab;          // word ids < vocab (KeyFrameDatabase(voc): mvInvertedFile sized voc->size())
    const uint32_t* ids;     // [cap][max_words]
    const double* vals;      // [cap][max_words]
    const int32_t* len;      // [cap] 0 = not in the inverted file
    const uint32_t* seq;     // [cap] add order
    const int32_t* covis;    // [cap][10]
    const int32_t* covis_n;  // [cap]
    // per-KeyFrame query state (persistent): [0] loop, [1] reloc
    unsigned long long* query[2];
    int32_t* words[2];
    float* score[2];
    // per-query scratch
    float* tscore;           // [cap] L1 score of every listed slot (count kernel), kept for the scored ones
    int32_t* list;           // [cap] 1 = in lKFsSharingWords this query
    unsigned long long* key; // [cap] (first query word << 32) | seq
    int32_t* scored;         // [cap] scored slots in list order
    float* sc;               // [cap] their scores
    float* acc;              // [cap]
    int32_t* best;           // [cap]
    int32_t* tmp;            // [cap]
    int32_t* counters;       // [0] n_list, [1] n_scored, [2] min_common, [3] n_tmp
    int32_t* out;            // [1 + cap]: n_candidates, candidates
    const uint32_t* qids;    // [max_words] query BowVector (ids strictly ascending)
    const double* qvals;
    const uint8_t* conn;     // [cap] connected-KeyFrame mask (loop query)
};

struct KfdbQuery {
    unsigned long long id;  // F->mnId / pKF->mnId
    int n;                  // query words
    int loop;               // 1 = DetectLoopCandidates, 0 = DetectRelocalizationCandidates
    float min_score;
};

hipError_t launch_kfdb_query(const DevKFDB& db, const KfdbQuery& q, hipStream_t st);
hipError_t read_kfdb_stamps(uint64_t* out);  // diagnostic, [4096][4] (kfdb.hip, RSC_KFDB_STAMPS=1 builds)

}  // namespace rsc
