// rsc_engine.h — host side of the RANSAC engine: solver state, SetRansacParameters, and the
// sequential selection replay of iterate() over speculatively evaluated hypotheses.
//
// How iterate() is executed (DESIGN.md "Selection replay"):
//   1. speculate: all hypotheses the reference loop could run in this call are sampled, solved and
//      scored on the GPU in two launches (counts come back to the host, poses/masks stay in HBM);
//   2. replay: the host walks the counts in hypothesis order and applies the reference's control
//      flow exactly (PnPsolver.cpp:119-190 / Sim3Solver.cpp:131-177);
//   3. a qualifying PnP hypothesis triggers Refine() on the GPU.  A failed Refine mutates the
//      grow-only EPnP buffers (Q6), so the hypotheses after it are re-speculated with the new
//      buffer state; a successful one ends the call.
// The backend interface is implemented by the HIP backend (rsc_api.cpp).
#pragma once
#include <cstdint>
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>

namespace rsc {

// ------------------------------------------------------------------------------------------------
// glibc TYPE_3 rand() stream as (31-word window, draw offset) — Random.cpp:47-50 + glibc random_r.
// ------------------------------------------------------------------------------------------------
constexpr int kRngTableRows = 16384 + 320;  // draws addressable from one window

struct RngTable {
    std::vector<uint32_t> T;  // [kRngTableRows][32]
    void build() {
        T.assign((size_t)kRngTableRows * 32, 0u);
        auto unit = [](uint32_t* row, int j) { for (int k = 0; k < 32; ++k) row[k] = (k == j) ? 1u : 0u; };
        uint32_t a[32], b[32];
        for (int k = 0; k < kRngTableRows; ++k) {
            uint32_t* row = &T[(size_t)k * 32];
            const uint32_t* p31;
            const uint32_t* p3;
            if (k - 31 < 0) { unit(a, k); p31 = a; } else p31 = &T[(size_t)(k - 31) * 32];
            if (k - 3 < 0) { unit(b, k + 28); p3 = b; } else p3 = &T[(size_t)(k - 3) * 32];
            for (int j = 0; j < 31; ++j) row[j] = p31[j] + p3[j];
            row[31] = 0;
        }
    }
    uint32_t word(const uint32_t* w, int g) const {
        const uint32_t* t = &T[(size_t)g * 32];
        uint32_t acc = 0;
        for (int j = 0; j < 31; ++j) acc += t[j] * w[j];
        return acc;
    }
};

struct RngStream {
    uint32_t window[31];
    int g;  // draws already consumed, relative to the window
    // srand(seed): r[0..30] by Schrage, r[31..33] = r[0..2]; window = r[3..33] (m = 34) and the
    // first output r[344] is draw g = 310.
    void seed(uint32_t s) {
        int32_t r[34];
        r[0] = (s == 0) ? 1 : (int32_t)s;
        for (int i = 1; i < 31; ++i) {
            int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
            int32_t word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            r[i] = word;
        }
        for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
        for (int j = 0; j < 31; ++j) window[j] = (uint32_t)r[3 + j];
        g = 310;
    }
    // Move the window forward so that `need` more draws stay addressable by the table:
    // new window = r[m+g-31 .. m+g-1], new m = m+g, next draw 0.
    void ensure(const RngTable& tab, int need) {
        if (g + need <= kRngTableRows) return;
        rebase(tab);
    }
    void rebase(const RngTable& tab) {  // requires g <= kRngTableRows
        uint32_t nw[31];
        for (int j = 0; j < 31; ++j) {
            const int x = g - 31 + j;
            nw[j] = (x >= 0) ? tab.word(window, x) : window[31 + x];
        }
        std::memcpy(window, nw, sizeof(nw));
        g = 0;
    }
    // Skip n draws of the stream (any n >= 0): the window is re-based once per table reach, so a
    // position millions of draws ahead costs O(n / 16704) re-bases of 31 table rows each.
    void advance(const RngTable& tab, int64_t n) {
        while (n > 0) {
            const int64_t room = (int64_t)kRngTableRows - g;
            if (n <= room) { g += (int)n; return; }
            n -= room;
            g = kRngTableRows;
            rebase(tab);
        }
    }
};

constexpr int kMaxSpeculate = 4000;  // hypotheses per solver per launch round

// ------------------------------------------------------------------------------------------------
// PnPsolver state (include/PnPsolver.hpp:71-136)
// ------------------------------------------------------------------------------------------------
struct PnPParams {
    double probability = 0.99;
    int min_inliers = 8, max_iterations = 300, min_set = 4;
    float epsilon = 0.4f, th2 = 5.991f;
};

struct PnPState {
    int N = 0, N_points = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    std::vector<int32_t> kp_index;  // mvKeyPointIndices
    std::vector<float> sigma2;      // mvSigma2 (host copy; the device copy sits in pts.w)
    // SetRansacParameters outputs
    double mRansacProb = 0.99;
    int mRansacMinInliers = 0, mRansacMaxIts = 0, mRansacMinSet = 4;
    float mRansacEpsilon = 0.4f, th2 = 5.991f;
    bool params_set = false;
    // RANSAC state
    int mnIterations = 0;
    int mnBestInliers = 0;
    float mBestTcw[16];
    int max_rows = 0;  // maximum_number_of_correspondences
    float mRefinedTcw[16];
    int mnRefinedInliers = 0;
    RngStream rng;
    uint32_t seed = 1;
    void reset(uint32_t s) {
        mnIterations = 0;
        mnBestInliers = 0;
        max_rows = 0;
        mnRefinedInliers = 0;
        for (int i = 0; i < 16; ++i) mBestTcw[i] = mRefinedTcw[i] = (i % 5 == 0) ? 1.f : 0.f;
        seed = s;
        rng.seed(s);
    }
};

// PnPsolver::SetRansacParameters (PnPsolver.cpp:58-94) — host arithmetic, same types as the reference.
inline void pnp_set_params(PnPState& S, double probability, int minInliers, int maxIterations, int minSet,
                           float epsilon, float th2) {
    S.mRansacProb = probability;
    S.mRansacMinInliers = minInliers;
    S.mRansacMaxIts = maxIterations;
    S.mRansacEpsilon = epsilon;
    S.mRansacMinSet = minSet;
    const int N = S.N;
    int nMinInliers = N * S.mRansacEpsilon;
    if (nMinInliers < S.mRansacMinInliers) nMinInliers = S.mRansacMinInliers;
    if (nMinInliers < minSet) nMinInliers = minSet;
    S.mRansacMinInliers = nMinInliers;
    if (S.mRansacEpsilon < (float)S.mRansacMinInliers / N) S.mRansacEpsilon = (float)S.mRansacMinInliers / N;
    int nIterations;
    if (S.mRansacMinInliers == N)
        nIterations = 1;
    else
        nIterations = (int)std::ceil(std::log(1 - S.mRansacProb) / std::log(1 - std::pow((double)S.mRansacEpsilon, 3.0)));
    S.mRansacMaxIts = std::max(1, std::min(nIterations, S.mRansacMaxIts));
    S.th2 = th2;
    S.params_set = true;
}

struct PnPResult {
    int ok = 0, no_more = 0, n_inliers = 0, iterations = 0;
    float T[16];
    int mask_kind = 0;  // 0: empty vector, 1: refined inliers, 2: best inliers
};

// Backend contract for the PnP replay.
struct PnPBackend {
    // Speculate hypotheses [0, H[i]) for solver states[i] (from their current rng position and
    // EPnP buffer rows).  Fills counts[i][0..H[i]), or leaves counts[i] empty when none of those
    // counts reaches states[i]->mRansacMinInliers (the replay then only advances the counters).
    virtual int speculate(PnPState* const* states, int count, const int* H, std::vector<std::vector<int32_t>>& counts) = 0;
    // Refine() for each listed solver, paused at hypothesis pause_k[q] of speculation slot
    // spec_j[q], preceded (adopt_k[q] >= 0) by the new-best bookkeeping of PnPsolver.cpp:147-156:
    // mvbBestInliers/mBestTcw := that hypothesis (the backend writes states[q]->mBestTcw).  Uses the
    // best mask and rows_after; writes the refined count and pose (the caller decides success) into
    // the out arrays.  A backend may have run exactly this Refine already on the device with the
    // round (the first pause of each solver); it then only hands back the results.  Called after
    // every speculation, with count == 0 when no solver paused.
    virtual int refine(PnPState* const* states, int count, const int* spec_j, const int* pause_k,
                       const int* adopt_k, const int* rows_after, int* refined_count,
                       float (*refined_pose)[12]) = 0;
    // vbInliers: scatter best (kind 2) or refined (kind 1) mask through kp_index into n_points bytes.
    virtual int fetch_mask(PnPState* const* states, int count, const int* kind, uint8_t* const* out) = 0;
    virtual ~PnPBackend() {}
};

static inline void pose12_to_T(const float* p, float* T) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T[4 * r + c] = p[3 * r + c];
        T[4 * r + 3] = p[9 + r];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

// PnPsolver::iterate (PnPsolver.cpp:102-191) for `count` solvers.  `best_pose(i,k)` must return the
// 12-float pose of hypothesis k of solver i of the last speculation (the backend provides it via
// adopt_best's side effect in s->mBestTcw).
inline int pnp_iterate_many(PnPBackend& be, PnPState* const* S, int count, const int* n_its, PnPResult* res,
                            uint8_t* const* inliers) {
    std::vector<int> remaining(count, 0), ncur(count, 0), active;
    for (int i = 0; i < count; ++i) {
        PnPResult& R = res[i];
        R = PnPResult();
        PnPState& s = *S[i];
        // set_maximum_number_of_correspondences(mRansacMinSet) (:108): grow-only
        if (s.max_rows < s.mRansacMinSet) s.max_rows = s.mRansacMinSet;
        if (s.N < s.mRansacMinInliers) {
            R.no_more = 1;
            R.iterations = s.mnIterations;
            continue;
        }
        active.push_back(i);
    }
    // The loop `while (mnIterations < maxIts || nCur < nIts)` (Q1) runs exactly
    // max(nIts - nCur, maxIts - mnIterations) more times unless Refine() succeeds.
    auto loop_len = [&](int i) {
        const PnPState& s = *S[i];
        int a = n_its[i] - ncur[i];
        int b = s.mRansacMaxIts - s.mnIterations;
        return std::max(0, std::max(a, b));
    };
    std::vector<char> done(count, 0);
    while (!active.empty()) {
        std::vector<PnPState*> spec;
        std::vector<int> H, who;
        for (int i : active) {
            int h = std::min(loop_len(i), kMaxSpeculate);
            if (h > 0) { spec.push_back(S[i]); H.push_back(h); who.push_back(i); }
        }
        thread_local std::vector<std::vector<int32_t>> counts;  // capacity kept across rounds
        if (!spec.empty()) {
            int st = be.speculate(spec.data(), (int)spec.size(), H.data(), counts);
            if (st) return st;
        }
        // replay, pausing at qualifying hypotheses (they need Refine)
        std::vector<int> pause_k(spec.size(), -1), adopt_k(spec.size(), -1);
        for (size_t j = 0; j < spec.size(); ++j) {
            PnPState& s = *spec[j];
            const int i = who[j];
            // hypotheses [0, k) are below minInliers: they only advance the counters
            // (a backend may hand back no counts for a slot none of whose hypotheses reaches mi)
            const int32_t* cj = counts[j].data();
            const int hj = H[j], mi = s.mRansacMinInliers;
            int k = counts[j].empty() ? hj : 0;
            while (k < hj && cj[k] < mi) ++k;
            const int ran = (k < hj) ? k + 1 : hj;
            ncur[i] += ran;
            s.mnIterations += ran;
            s.rng.g += ran * s.mRansacMinSet;
            if (k < hj) {
                const int c = cj[k];
                if (c > s.mnBestInliers) {
                    s.mnBestInliers = c;
                    adopt_k[j] = k;  // applied by the backend together with Refine()
                }
                pause_k[j] = k;
            }
        }
        // Refine() for every paused solver
        std::vector<PnPState*> rs;
        std::vector<int> rows_after, rj, rk, rp;
        for (size_t j = 0; j < spec.size(); ++j)
            if (pause_k[j] >= 0) {
                PnPState& s = *spec[j];
                const int nr = s.mnBestInliers;
                const int ra = std::max(s.max_rows, nr);
                rs.push_back(&s);
                rows_after.push_back(ra);
                rj.push_back((int)j);
                rp.push_back(pause_k[j]);
                rk.push_back(adopt_k[j]);
            }
        std::vector<int> rcount(rs.size());
        std::vector<float> rpose(rs.size() * 12);
        // called after every speculation, with an empty list when no solver paused, so that a
        // backend that selected Refines on the device checks it selected none
        if (!spec.empty()) {
            int st = be.refine(rs.data(), (int)rs.size(), rj.data(), rp.data(), rk.data(), rows_after.data(),
                               rcount.data(), reinterpret_cast<float(*)[12]>(rpose.data()));
            if (st) return st;
        }
        for (size_t q = 0; q < rs.size(); ++q) {
            PnPState& s = *rs[q];
            s.max_rows = rows_after[q];
            s.mnRefinedInliers = rcount[q];
            const int i = who[rj[q]];
            if (rcount[q] > s.mRansacMinInliers) {  // Refine success (Q8: strict)
                pose12_to_T(&rpose[12 * q], s.mRefinedTcw);
                PnPResult& R = res[i];
                R.ok = 1;
                R.n_inliers = rcount[q];
                std::memcpy(R.T, s.mRefinedTcw, sizeof(R.T));
                R.mask_kind = 1;
                done[i] = 1;
            }
        }
        // next round: solvers that failed Refine (or hit the per-launch cap) continue the loop
        std::vector<int> next;
        for (size_t j = 0; j < spec.size(); ++j) {
            const int i = who[j];
            if (done[i]) continue;
            if (loop_len(i) > 0) next.push_back(i);
        }
        active.swap(next);
    }
    // epilogue (:173-190)
    for (int i = 0; i < count; ++i) {
        PnPResult& R = res[i];
        PnPState& s = *S[i];
        if (R.ok || R.no_more) { R.iterations = s.mnIterations; continue; }
        if (s.N < s.mRansacMinInliers) continue;
        if (s.mnIterations >= s.mRansacMaxIts) {
            R.no_more = 1;
            if (s.mnBestInliers >= s.mRansacMinInliers) {
                R.ok = 1;
                R.n_inliers = s.mnBestInliers;
                std::memcpy(R.T, s.mBestTcw, sizeof(R.T));
                R.mask_kind = 2;
            }
        }
        R.iterations = s.mnIterations;
    }
    // vbInliers
    std::vector<PnPState*> ms;
    std::vector<int> kinds;
    std::vector<uint8_t*> outs;
    for (int i = 0; i < count; ++i)
        if (res[i].mask_kind && inliers && inliers[i]) {
            ms.push_back(S[i]);
            kinds.push_back(res[i].mask_kind);
            outs.push_back(inliers[i]);
        }
    if (!ms.empty()) {
        int st = be.fetch_mask(ms.data(), (int)ms.size(), kinds.data(), outs.data());
        if (st) return st;
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
// Sim3Solver state (include/Sim3Solver.hpp:45-101)
// ------------------------------------------------------------------------------------------------
struct Sim3State {
    int N = 0, mN1 = 0;
    std::vector<int32_t> indices1;  // mvnIndices1
    double mRansacProb = 0.99;
    int mRansacMinInliers = 6, mRansacMaxIts = 300;
    int mnIterations = 0, mnBestInliers = 0;
    float mBestRotation[9], mBestTranslation[3];
    RngStream rng;
    uint32_t seed = 1;
    void reset(uint32_t s) {
        mnIterations = 0;
        mnBestInliers = 0;
        for (int i = 0; i < 9; ++i) mBestRotation[i] = (i % 4 == 0) ? 1.f : 0.f;
        for (int i = 0; i < 3; ++i) mBestTranslation[i] = 0.f;
        seed = s;
        rng.seed(s);
    }
};

// Sim3Solver::SetRansacParameters (Sim3Solver.cpp:87-111)
inline void sim3_set_params(Sim3State& S, double probability, int minInliers, int maxIterations) {
    S.mRansacProb = probability;
    S.mRansacMinInliers = minInliers;
    S.mRansacMaxIts = maxIterations;
    const int N = S.N;
    float epsilon = (float)S.mRansacMinInliers / N;
    int nIterations;
    if (S.mRansacMinInliers == N)
        nIterations = 1;
    else
        nIterations = (int)std::ceil(std::log(1 - S.mRansacProb) / std::log(1 - std::pow((double)epsilon, 3.0)));
    S.mRansacMaxIts = std::max(1, std::min(nIterations, S.mRansacMaxIts));
    S.mnIterations = 0;
}

struct Sim3Result {
    int ok = 0, no_more = 0, n_inliers = 0, iterations = 0;
    float R[9], t[3];
    int mask_k = -1;  // hypothesis index (last speculation) whose mask is vbInliers
};

struct Sim3Backend {
    virtual int speculate(Sim3State* const* states, int count, const int* H, std::vector<std::vector<int32_t>>& counts) = 0;
    // poses (R12 9 + t12 3) of hypotheses k[q] of solvers i[q] of the last speculation, q < n
    virtual int fetch_poses(const int* i, const int* k, int n, float (*pose12)[12]) = 0;
    virtual int fetch_mask(const int* which_i, const int* which_k, Sim3State* const* states, int count,
                           uint8_t* const* out) = 0;
    virtual ~Sim3Backend() {}
};

// Sim3Solver::iterate (Sim3Solver.cpp:113-178) for `count` solvers.  '&&' loop (Q1), '>=' best
// update with later ties winning, return at the first hypothesis with count > minInliers (Q12).
inline int sim3_iterate_many(Sim3Backend& be, Sim3State* const* S, int count, const int* n_its, Sim3Result* res,
                             uint8_t* const* inliers) {
    std::vector<Sim3State*> spec;
    std::vector<int> H, who;
    for (int i = 0; i < count; ++i) {
        res[i] = Sim3Result();
        Sim3State& s = *S[i];
        if (s.N < s.mRansacMinInliers) {
            res[i].no_more = 1;
            continue;
        }
        const int h = std::max(0, std::min(n_its[i], s.mRansacMaxIts - s.mnIterations));
        if (h > 0) { spec.push_back(&s); H.push_back(h); who.push_back(i); }
    }
    thread_local std::vector<std::vector<int32_t>> counts;  // capacity kept across calls
    if (!spec.empty()) {
        int st = be.speculate(spec.data(), (int)spec.size(), H.data(), counts);
        if (st) return st;
    }
    std::vector<int> mi, mk, pj, pk;
    std::vector<Sim3State*> ms;
    std::vector<uint8_t*> mo;
    for (size_t j = 0; j < spec.size(); ++j) {
        Sim3State& s = *spec[j];
        const int i = who[j];
        int best_k = -1;
        const int32_t* cj = counts[j].data();
        const int hj = H[j], mi_ = s.mRansacMinInliers;
        int best = s.mnBestInliers, k = 0;
        for (; k < hj; ++k) {
            const int c = cj[k];
            if (c >= best) {
                best = c;
                best_k = k;
                if (c > mi_) break;
            }
        }
        const int ran = (k < hj) ? k + 1 : hj;
        s.mnIterations += ran;
        s.rng.g += 3 * ran;
        s.mnBestInliers = best;
        if (k < hj) {
            res[i].ok = 1;
            res[i].n_inliers = cj[k];
            res[i].mask_k = k;
        }
        if (best_k >= 0) {
            pj.push_back((int)j);
            pk.push_back(best_k);
        }
        if (res[i].ok && inliers && inliers[i]) {
            mi.push_back((int)j);
            mk.push_back(res[i].mask_k);
            ms.push_back(&s);
            mo.push_back(inliers[i]);
        }
    }
    if (!pj.empty()) {  // mBestRotation / mBestTranslation of every solver that improved, one fetch
        std::vector<float> p(pj.size() * 12);
        int st = be.fetch_poses(pj.data(), pk.data(), (int)pj.size(), reinterpret_cast<float(*)[12]>(p.data()));
        if (st) return st;
        for (size_t q = 0; q < pj.size(); ++q) {
            Sim3State& s = *spec[pj[q]];
            std::memcpy(s.mBestRotation, &p[q * 12], 9 * sizeof(float));
            std::memcpy(s.mBestTranslation, &p[q * 12 + 9], 3 * sizeof(float));
        }
    }
    for (int i = 0; i < count; ++i) {
        Sim3State& s = *S[i];
        if (!res[i].ok && !(s.N < s.mRansacMinInliers) && s.mnIterations >= s.mRansacMaxIts) res[i].no_more = 1;
        res[i].iterations = s.mnIterations;
        std::memcpy(res[i].R, s.mBestRotation, sizeof(res[i].R));
        std::memcpy(res[i].t, s.mBestTranslation, sizeof(res[i].t));
        if (!res[i].ok && inliers && inliers[i]) std::memset(inliers[i], 0, s.mN1);
    }
    if (!ms.empty()) {
        int st = be.fetch_mask(mi.data(), mk.data(), ms.data(), (int)ms.size(), mo.data());
        if (st) return st;
    }
    return 0;
}


// ------------------------------------------------------------------------------------------------
// MLPnPsolver state (include/MLPnPsolver.hpp:10-199) and iterate() replay (MLPnPsolver.cpp:56-183)
// ------------------------------------------------------------------------------------------------
struct MLState {
    int N = 0, N_points = 0;
    std::vector<int32_t> kp_index;
    double mRansacProb = 0.99;
    int mRansacMinInliers = 0, mRansacMaxIts = 0, mRansacMinSet = 6;
    float mRansacEpsilon = 0.4f, th2 = 5.991f;
    int mnIterations = 0;
    int mnBestInliers = 0;
    float mBestTcw[16];
    RngStream rng;
    uint32_t seed = 1;
    void reset(uint32_t s) {
        mnIterations = 0;
        mnBestInliers = 0;
        for (int i = 0; i < 16; ++i) mBestTcw[i] = (i % 5 == 0) ? 1.f : 0.f;
        seed = s;
        rng.seed(s);
    }
};

// MLPnPsolver::SetRansacParameters (MLPnPsolver.cpp:185-220): the PnPsolver formula (Q2).
inline void mlpnp_set_params(MLState& S, double probability, int minInliers, int maxIterations, int minSet,
                             float epsilon, float th2) {
    S.mRansacProb = probability;
    S.mRansacMinInliers = minInliers;
    S.mRansacMaxIts = maxIterations;
    S.mRansacEpsilon = epsilon;
    S.mRansacMinSet = minSet;
    const int N = S.N;
    int nMinInliers = N * S.mRansacEpsilon;
    if (nMinInliers < S.mRansacMinInliers) nMinInliers = S.mRansacMinInliers;
    if (nMinInliers < minSet) nMinInliers = minSet;
    S.mRansacMinInliers = nMinInliers;
    if (S.mRansacEpsilon < (float)S.mRansacMinInliers / N) S.mRansacEpsilon = (float)S.mRansacMinInliers / N;
    int nIterations;
    if (S.mRansacMinInliers == N)
        nIterations = 1;
    else
        nIterations = (int)std::ceil(std::log(1 - S.mRansacProb) / std::log(1 - std::pow((double)S.mRansacEpsilon, 3.0)));
    S.mRansacMaxIts = std::max(1, std::min(nIterations, S.mRansacMaxIts));
    S.th2 = th2;
}

struct MLResult {
    int ok = 0, no_more = 0, n_inliers = 0, iterations = 0;
    float T[16];
    int mask_kind = 0;  // 0: empty, 1: the returning hypothesis (= Refine's re-count), 2: best
    int mask_j = -1, mask_k = -1;
    MLResult() {
        for (int i = 0; i < 16; ++i) T[i] = (i % 5 == 0) ? 1.f : 0.f;  // Tout.setIdentity() (Q10)
    }
};

struct MLBackend {
    virtual int speculate(MLState* const* states, int count, const int* H, std::vector<std::vector<int32_t>>& counts) = 0;
    // mvbBestInliers / mBestTcw := hypothesis k of slot j of the last speculation
    virtual int adopt_best(MLState* s, int j, int k) = 0;
    // float poses (R 9 + t 3) of hypotheses (j[q], k[q]) of the last speculation
    virtual int fetch_poses(const int* j, const int* k, int n, float (*pose12)[12]) = 0;
    // masks: kind 1 = hypothesis (j, k) of the last speculation, kind 2 = the solver's best mask
    virtual int fetch_mask(MLState* const* states, int count, const int* kind, const int* j, const int* k,
                           uint8_t* const* out) = 0;
    virtual ~MLBackend() {}
};

// MLPnPsolver::iterate for `count` solvers.  Refine() re-counts the current hypothesis (its
// computePose result is discarded, MLPnPsolver.cpp:290), so the call returns at the first
// hypothesis whose count is > minInliers; the best is updated on '>' among counts >= minInliers.
inline int mlpnp_iterate_many(MLBackend& be, MLState* const* S, int count, const int* n_its, MLResult* res,
                              uint8_t* const* inliers) {
    std::vector<int> ncur(count, 0), active;
    for (int i = 0; i < count; ++i) {
        res[i] = MLResult();
        MLState& s = *S[i];
        if (s.N < s.mRansacMinInliers) {
            res[i].no_more = 1;
            res[i].iterations = s.mnIterations;
            continue;
        }
        active.push_back(i);
    }
    auto loop_len = [&](int i) {
        const MLState& s = *S[i];
        return std::max(0, std::max(n_its[i] - ncur[i], s.mRansacMaxIts - s.mnIterations));
    };
    std::vector<char> done(count, 0);
    std::vector<int> succ_i, succ_j, succ_k;
    while (!active.empty()) {
        std::vector<MLState*> spec;
        std::vector<int> H, who;
        for (int i : active) {
            const int h = std::min(loop_len(i), kMaxSpeculate);
            if (h > 0) { spec.push_back(S[i]); H.push_back(h); who.push_back(i); }
        }
        if (spec.empty()) break;
        thread_local std::vector<std::vector<int32_t>> counts;  // capacity kept across rounds
        if (int st = be.speculate(spec.data(), (int)spec.size(), H.data(), counts)) return st;
        std::vector<int> pj, pk, pi;
        for (size_t j = 0; j < spec.size(); ++j) {
            MLState& s = *spec[j];
            const int i = who[j];
            for (int k = 0; k < H[j]; ++k) {
                ncur[i]++;
                s.mnIterations++;
                s.rng.g += s.mRansacMinSet;
                const int c = counts[j][k];
                if (c >= s.mRansacMinInliers) {
                    if (c > s.mnBestInliers) {
                        s.mnBestInliers = c;
                        if (int st = be.adopt_best(&s, (int)j, k)) return st;
                    }
                    if (c > s.mRansacMinInliers) {
                        res[i].ok = 1;
                        res[i].n_inliers = c;
                        res[i].mask_kind = 1;
                        res[i].mask_j = (int)j;
                        res[i].mask_k = k;
                        pj.push_back((int)j);
                        pk.push_back(k);
                        pi.push_back(i);
                        done[i] = 1;
                        break;
                    }
                }
            }
        }
        if (!pj.empty()) {
            std::vector<float> p(pj.size() * 12);
            if (int st = be.fetch_poses(pj.data(), pk.data(), (int)pj.size(), reinterpret_cast<float(*)[12]>(p.data())))
                return st;
            for (size_t q = 0; q < pj.size(); ++q) pose12_to_T(&p[12 * q], res[pi[q]].T);
            // the masks of returning hypotheses must be read before the next speculation reuses
            // the record buffers
            std::vector<MLState*> ms;
            std::vector<int> kinds, mj, mk;
            std::vector<uint8_t*> outs;
            for (size_t q = 0; q < pj.size(); ++q)
                if (inliers && inliers[pi[q]]) {
                    ms.push_back(S[pi[q]]);
                    kinds.push_back(1);
                    mj.push_back(pj[q]);
                    mk.push_back(pk[q]);
                    outs.push_back(inliers[pi[q]]);
                }
            if (!ms.empty())
                if (int st = be.fetch_mask(ms.data(), (int)ms.size(), kinds.data(), mj.data(), mk.data(), outs.data()))
                    return st;
        }
        std::vector<int> next;
        for (size_t j = 0; j < spec.size(); ++j) {
            const int i = who[j];
            if (!done[i] && loop_len(i) > 0) next.push_back(i);
        }
        active.swap(next);
    }
    std::vector<MLState*> ms;
    std::vector<int> kinds, mj, mk;
    std::vector<uint8_t*> outs;
    for (int i = 0; i < count; ++i) {
        MLResult& R = res[i];
        MLState& s = *S[i];
        if (R.ok || R.no_more) { R.iterations = s.mnIterations; continue; }
        if (s.mnIterations >= s.mRansacMaxIts) {
            R.no_more = 1;
            if (s.mnBestInliers >= s.mRansacMinInliers) {
                R.ok = 1;
                R.n_inliers = s.mnBestInliers;
                std::memcpy(R.T, s.mBestTcw, sizeof(R.T));
                R.mask_kind = 2;
                if (inliers && inliers[i]) {
                    ms.push_back(&s);
                    kinds.push_back(2);
                    mj.push_back(-1);
                    mk.push_back(-1);
                    outs.push_back(inliers[i]);
                }
            }
        }
        R.iterations = s.mnIterations;
    }
    if (!ms.empty())
        if (int st = be.fetch_mask(ms.data(), (int)ms.size(), kinds.data(), mj.data(), mk.data(), outs.data())) return st;
    return 0;
}

}  // namespace rsc
