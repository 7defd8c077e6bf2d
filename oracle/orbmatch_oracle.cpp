// TEST INFRASTRUCTURE — parity oracle (see orbmatch_oracle.h).
#include "orbmatch_oracle.h"

#include <cmath>
#include <cstring>

namespace rsc_oracle {

namespace {
constexpr int kThLow = 50;        // ORBmatcher::TH_LOW (ORBmatcher.cpp:9)
constexpr int kHistoLength = 30;  // ORBmatcher::HISTO_LENGTH (ORBmatcher.cpp:10)

// the orientation bin of a match (ORBmatcher.cpp:187-195 / :437-445); the reference's factor is
// 1/HISTO_LENGTH, so bins 0..12 are the only ones reached
int rot_bin(float angle_a, float angle_b) {
    const float factor = 1.0f / kHistoLength;
    float rot = angle_a - angle_b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == kHistoLength) bin = 0;
    return bin;
}

// the histogram filter shared by both overloads (ORBmatcher.cpp:218-237 / :466-485): entries are
// the indices the reference pushes; removal clears them in `match` and decrements nmatches
int orientation_filter(const std::vector<int> (&hist)[kHistoLength], int32_t* match, int nmatches) {
    int sizes[kHistoLength];
    for (int i = 0; i < kHistoLength; ++i) sizes[i] = (int)hist[i].size();
    int ind1 = -1, ind2 = -1, ind3 = -1;
    compute_three_maxima(sizes, kHistoLength, ind1, ind2, ind3);
    for (int i = 0; i < kHistoLength; ++i) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (int idx : hist[i]) {
            match[idx] = -1;
            --nmatches;
        }
    }
    return nmatches;
}
}  // namespace

int descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        int32_t wa, wb;
        std::memcpy(&wa, a + 4 * i, 4);
        std::memcpy(&wb, b + 4 * i, 4);
        unsigned int v = (unsigned int)(wa ^ wb);
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

void compute_three_maxima(const int* sizes, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; ++i) {
        const int s = sizes[i];
        if (s > max1) {
            max3 = max2;
            max2 = max1;
            max1 = s;
            ind3 = ind2;
            ind2 = ind1;
            ind1 = i;
        } else if (s > max2) {
            max3 = max2;
            max2 = s;
            ind3 = ind2;
            ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

// ORBmatcher.cpp:110-240
int search_by_bow_frame(const BowView& kf, const BowView& F, float nnratio, bool check_ori, int32_t* match) {
    for (int i = 0; i < F.n; ++i) match[i] = -1;  // vpMapPointMatches = vector(F.N, nullptr) (:114)
    std::vector<int> hist[kHistoLength];
    int nmatches = 0;
    auto KFit = kf.fv.begin();
    auto Fit = F.fv.begin();
    while (KFit != kf.fv.end() && Fit != F.fv.end()) {
        if (KFit->first == Fit->first) {
            const std::vector<uint32_t>& vKF = KFit->second;
            const std::vector<uint32_t>& vF = Fit->second;
            for (size_t iKF = 0; iKF < vKF.size(); ++iKF) {
                const uint32_t realIdxKF = vKF[iKF];
                if (kf.valid && !kf.valid[realIdxKF]) continue;  // !pMP || pMP->isBad() (:144-148)
                const uint8_t* dKF = kf.desc + 32 * (size_t)realIdxKF;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (size_t iF = 0; iF < vF.size(); ++iF) {
                    const uint32_t realIdxF = vF[iF];
                    if (match[realIdxF] >= 0) continue;  // already matched (:160-161)
                    const int dist = descriptor_distance(dKF, F.desc + 32 * (size_t)realIdxF);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdxF = (int)realIdxF;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 <= kThLow) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        match[bestIdxF] = (int32_t)realIdxKF;
                        if (check_ori) hist[rot_bin(kf.angle[realIdxKF], F.angle[bestIdxF])].push_back(bestIdxF);
                        ++nmatches;
                    }
                }
            }
            ++KFit;
            ++Fit;
        } else if (KFit->first < Fit->first) {
            KFit = kf.fv.lower_bound(Fit->first);
        } else {
            Fit = F.fv.lower_bound(KFit->first);
        }
    }
    if (check_ori) nmatches = orientation_filter(hist, match, nmatches);
    return nmatches;
}

// ORBmatcher.cpp:354-488
int search_by_bow_kf(const BowView& k1, const BowView& k2, float nnratio, bool check_ori, int32_t* match12) {
    for (int i = 0; i < k1.n; ++i) match12[i] = -1;  // vpMatches12 (:366)
    std::vector<uint8_t> matched2(k2.n, 0);          // vbMatched2 (:367)
    std::vector<int> hist[kHistoLength];
    int nmatches = 0;
    auto f1 = k1.fv.begin();
    auto f2 = k2.fv.begin();
    while (f1 != k1.fv.end() && f2 != k2.fv.end()) {
        if (f1->first == f2->first) {
            for (size_t i1 = 0; i1 < f1->second.size(); ++i1) {
                const uint32_t idx1 = f1->second[i1];
                if (k1.valid && !k1.valid[idx1]) continue;  // (:388-392)
                const uint8_t* d1 = k1.desc + 32 * (size_t)idx1;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (size_t i2 = 0; i2 < f2->second.size(); ++i2) {
                    const uint32_t idx2 = f2->second[i2];
                    if (matched2[idx2] || (k2.valid && !k2.valid[idx2])) continue;  // (:404-410)
                    const int dist = descriptor_distance(d1, k2.desc + 32 * (size_t)idx2);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdx2 = (int)idx2;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 < kThLow) {  // strict here (:430), <= in the Frame overload (:179)
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        match12[idx1] = bestIdx2;
                        matched2[bestIdx2] = 1;
                        if (check_ori) hist[rot_bin(k1.angle[idx1], k2.angle[bestIdx2])].push_back((int)idx1);
                        ++nmatches;
                    }
                }
            }
            ++f1;
            ++f2;
        } else if (f1->first < f2->first) {
            f1 = k1.fv.lower_bound(f2->first);
        } else {
            f2 = k2.fv.lower_bound(f1->first);
        }
    }
    if (check_ori) nmatches = orientation_filter(hist, match12, nmatches);
    return nmatches;
}

}  // namespace rsc_oracle
