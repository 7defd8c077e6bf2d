// TEST INFRASTRUCTURE — parity oracle (see kfdb_oracle.h).  KeyFrameDatabase restated over slots.
#include "kfdb_oracle.h"

#include <cmath>
#include <set>
#include <utility>

namespace rsc_oracle {

double l1_score(int n1, const uint32_t* id1, const double* v1, int n2, const uint32_t* id2, const double* v2) {
    // ScoringObject.cpp:23-67: walk both sorted vectors; only common words contribute, in
    // ascending word order (the lower_bound jumps skip non-common words without arithmetic)
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        if (id1[i] == id2[j]) {
            const double vi = v1[i], wi = v2[j];
            score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
            ++i;
            ++j;
        } else if (id1[i] < id2[j]) {
            ++i;
        } else {
            ++j;
        }
    }
    score = -score / 2.0;
    return score;
}

KFDatabase::KFDatabase(int capacity) : cap_(capacity), bow_(capacity), covis_(capacity), st_(capacity) {}

void KFDatabase::add(int kf, int n, const uint32_t* ids, const double* vals) {
    bow_[kf].clear();
    for (int i = 0; i < n; ++i) bow_[kf][ids[i]] = vals[i];
    for (const auto& w : bow_[kf]) inv_[w.first].push_back(kf);  // :19-20
}

void KFDatabase::erase(int kf) {
    for (const auto& w : bow_[kf]) {  // :28-42: first occurrence in each word's list
        auto it = inv_.find(w.first);
        if (it == inv_.end()) continue;
        for (auto lit = it->second.begin(); lit != it->second.end(); ++lit)
            if (*lit == kf) {
                it->second.erase(lit);
                break;
            }
    }
}

void KFDatabase::clear() { inv_.clear(); }

void KFDatabase::set_covisibility(int kf, int n, const int32_t* best) { covis_[kf].assign(best, best + n); }

namespace {
struct QueryVec {
    std::vector<uint32_t> ids;
    std::vector<double> vals;
};
double score_against(const QueryVec& q, const std::map<uint32_t, double>& b) {
    std::vector<uint32_t> ids;
    std::vector<double> vals;
    for (const auto& w : b) {
        ids.push_back(w.first);
        vals.push_back(w.second);
    }
    return l1_score((int)q.ids.size(), q.ids.data(), q.vals.data(), (int)ids.size(), ids.data(), vals.data());
}
}  // namespace

std::vector<int> KFDatabase::detect_relocalization(uint64_t frame_id, int n, const uint32_t* ids, const double* vals) {
    QueryVec q{std::vector<uint32_t>(ids, ids + n), std::vector<double>(vals, vals + n)};
    std::list<int> sharing;
    for (int i = 0; i < n; ++i) {  // :181-196
        auto it = inv_.find(ids[i]);
        if (it == inv_.end()) continue;
        for (int kfi : it->second) {
            State& s = st_[kfi];
            if (s.reloc_query != frame_id) {
                s.reloc_words = 0;
                s.reloc_query = frame_id;
                sharing.push_back(kfi);
            }
            s.reloc_words++;
        }
    }
    if (sharing.empty()) return {};
    int maxCommon = 0;  // :201-207
    for (int kfi : sharing)
        if (st_[kfi].reloc_words > maxCommon) maxCommon = st_[kfi].reloc_words;
    const int minCommon = (int)(maxCommon * 0.8f);
    std::list<std::pair<float, int>> scored;  // :216-228
    for (int kfi : sharing) {
        if (st_[kfi].reloc_words > minCommon) {
            const float si = (float)score_against(q, bow_[kfi]);
            st_[kfi].reloc_score = si;
            scored.push_back({si, kfi});
        }
    }
    if (scored.empty()) return {};
    std::list<std::pair<float, int>> acc;  // :233-259
    float bestAcc = 0;
    for (const auto& e : scored) {
        float bestScore = e.first;
        float accScore = bestScore;
        int bestKF = e.second;
        for (int kf2 : covis_[e.second]) {
            if (st_[kf2].reloc_query != frame_id) continue;
            accScore += st_[kf2].reloc_score;
            if (st_[kf2].reloc_score > bestScore) {
                bestKF = kf2;
                bestScore = st_[kf2].reloc_score;
            }
        }
        acc.push_back({accScore, bestKF});
        if (accScore > bestAcc) bestAcc = accScore;
    }
    const float minRetain = 0.75f * bestAcc;  // :262-279
    std::set<int> added;
    std::vector<int> out;
    for (const auto& e : acc)
        if (e.first > minRetain && !added.count(e.second)) {
            out.push_back(e.second);
            added.insert(e.second);
        }
    return out;
}

std::vector<int> KFDatabase::detect_loop(uint64_t kf_id, int n, const uint32_t* ids, const double* vals,
                                         int n_connected, const int32_t* connected, float min_score) {
    QueryVec q{std::vector<uint32_t>(ids, ids + n), std::vector<double>(vals, vals + n)};
    const std::set<int> conn(connected, connected + n_connected);
    std::list<int> sharing;
    for (int i = 0; i < n; ++i) {  // :60-78
        auto it = inv_.find(ids[i]);
        if (it == inv_.end()) continue;
        for (int kfi : it->second) {
            State& s = st_[kfi];
            if (s.loop_query != kf_id) {
                s.loop_words = 0;
                if (!conn.count(kfi)) {
                    s.loop_query = kf_id;
                    sharing.push_back(kfi);
                }
            }
            s.loop_words++;
        }
    }
    if (sharing.empty()) return {};
    int maxCommon = 0;  // :86-93
    for (int kfi : sharing)
        if (st_[kfi].loop_words > maxCommon) maxCommon = st_[kfi].loop_words;
    const int minCommon = (int)(maxCommon * 0.8f);
    std::list<std::pair<float, int>> scored;  // :98-113
    for (int kfi : sharing) {
        if (st_[kfi].loop_words > minCommon) {
            const float si = (float)score_against(q, bow_[kfi]);
            st_[kfi].loop_score = si;
            if (si >= min_score) scored.push_back({si, kfi});
        }
    }
    if (scored.empty()) return {};
    std::list<std::pair<float, int>> acc;  // :118-147
    float bestAcc = min_score;
    for (const auto& e : scored) {
        float bestScore = e.first;
        float accScore = e.first;
        int bestKF = e.second;
        for (int kf2 : covis_[e.second]) {
            if (st_[kf2].loop_query == kf_id && st_[kf2].loop_words > minCommon) {
                accScore += st_[kf2].loop_score;
                if (st_[kf2].loop_score > bestScore) {
                    bestKF = kf2;
                    bestScore = st_[kf2].loop_score;
                }
            }
        }
        acc.push_back({accScore, bestKF});
        if (accScore > bestAcc) bestAcc = accScore;
    }
    const float minRetain = 0.75f * bestAcc;  // :150-168
    std::set<int> added;
    std::vector<int> out;
    for (const auto& e : acc)
        if (e.first > minRetain && !added.count(e.second)) {
            out.push_back(e.second);
            added.insert(e.second);
        }
    return out;
}

}  // namespace rsc_oracle
