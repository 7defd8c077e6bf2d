// kfdb.hip — KeyFrameDatabase candidate queries (src/KeyFrameDatabase.cpp:52-283); see rsc_kfdb.h.
#include <hip/hip_runtime.h>
#include <climits>
#include "rsc_kfdb.h"

namespace rsc {

namespace {

constexpr int kBatch = 8;        // words per lane per batch of loads (score phase)
constexpr int kCountBatch = 16;  // words per lane per batch in the count kernel (1024 per wave)
constexpr int kRankLds = 1024;  // scored slots ranked from LDS (beyond: from global memory)

// The query's word -> position table (wpos[word] = index in F->mBowVec, -1 elsewhere): scattered
// before the count kernel, cleared by the finish kernel, so a lookup is one gather.
__global__ __launch_bounds__(256) void kfdb_scatter_kernel(DevKFDB db, KfdbQuery q) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < q.n) db.wpos[db.qids[i]] = i;
}

// The inverted-file walk (:60-78 loop, :181-196 reloc) seen from one slot: the walk meets slot k
// once per common word, first at the query word `first`, in list order (ascending seq) within a
// word.  One wave per slot; lane 0 applies the walk's per-occurrence state rules in closed form.
__global__ __launch_bounds__(256) void kfdb_count_kernel(DevKFDB db, KfdbQuery q) {
    const int lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (slot >= db.cap) return;
    if (lane == 0) db.list[slot] = 0;  // in lKFsSharingWords (a flag per slot: no shared counter)
    const int t = q.loop ? 0 : 1;
    // independent loads issued together: the slot length, its state, and the first
    // 64 * kCountBatch word ids (the slot stride is max_words, so the window is in bounds whatever
    // the length); the table gathers follow, masked by the length
    const int len = db.len[slot];
    const unsigned long long qb0 = db.query[t][slot];
    const int w0 = db.words[t][slot];
    const uint32_t* ids = db.ids + (size_t)slot * db.max_words;
    int c = 0, first = INT_MAX;
    for (int base = 0; base == 0 || base < len; base += 64 * kCountBatch) {
        uint32_t w[kCountBatch];
        int p[kCountBatch];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) w[b] = ids[min(base + b * 64 + lane, db.max_words - 1)];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) p[b] = db.wpos[base + b * 64 + lane < len ? w[b] : 0u];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b)
            if (base + b * 64 + lane < len && p[b] >= 0) {
                c++;
                first = min(first, p[b]);
            }
    }
    if (len == 0) return;  // not in any list: the walk never touches its state
    for (int off = 32; off > 0; off >>= 1) {
        c += __shfl_xor(c, off);
        first = min(first, __shfl_xor(first, off));
    }
    if (c == 0) return;
    // the walk's state rules (every lane: the inputs are wave-uniform)
    unsigned long long qb = qb0;
    int w = w0;
    bool in_list = false;
    if (qb != q.id) {
        if (q.loop && db.conn[slot]) {
            w = 1;  // connected: mnLoopWords = 0 then ++ at every occurrence, query id untouched
        } else {
            w = c;  // reset at the first occurrence, then one increment per occurrence
            qb = q.id;
            in_list = true;
        }
    } else {
        w += c;  // already met by an earlier query with the same id: counts accumulate, not listed
    }
    if (lane == 0) {
        db.query[t][slot] = qb;
        db.words[t][slot] = w;
        if (in_list) {
            db.list[slot] = 1;
            db.key[slot] = ((unsigned long long)first << 32) | db.seq[slot];
        }
    }
    if (!in_list) return;
    // L1Scoring::score(F->mBowVec, pKFi->mBowVec) (ScoringObject.cpp:23-67): per-word terms in
    // parallel, the sum in ascending word order on the wave's scalar path; finish keeps it only if
    // the slot is scored (mLoopScore / mRelocScore are written there)
    const double* vals = db.vals + (size_t)slot * db.max_words;
    double score = 0;
    for (int base = 0; base < len; base += 64 * kBatch) {
        uint32_t wd[kBatch];
        double wv[kBatch], vv[kBatch];
        int p[kBatch];
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
            const int j = min(base + b * 64 + lane, db.max_words - 1);
            wd[b] = ids[j];
            wv[b] = vals[j];
        }
#pragma unroll
        for (int b = 0; b < kBatch; ++b) p[b] = db.wpos[base + b * 64 + lane < len ? wd[b] : 0u];
#pragma unroll
        for (int b = 0; b < kBatch; ++b) p[b] = base + b * 64 + lane < len ? p[b] : -1;
#pragma unroll
        for (int b = 0; b < kBatch; ++b) vv[b] = db.qvals[max(p[b], 0)];
#pragma unroll
        for (int b = 0; b < kBatch; ++b) {
            const double vi = vv[b], wi = wv[b];
            const double term = fabs(vi - wi) - fabs(vi) - fabs(wi);
            const long long tb = __double_as_longlong(term);
            const int lo = (int)(tb & 0xffffffff), hi = (int)(tb >> 32);
            unsigned long long m = __ballot(p[b] >= 0);
            while (m) {  // ascending word order: batch b, then lane (uniform lane index)
                const int src = __builtin_amdgcn_readfirstlane(__ffsll((long long)m) - 1);
                const unsigned long long v = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane(hi, src) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane(lo, src);
                score += __longlong_as_double((long long)v);
                m &= m - 1;
            }
        }
    }
    score = -score / 2.0;
    if (lane == 0) db.tscore[slot] = (float)score;  // float si = mpVoc->score(...)
}

template <typename T, typename Op>
__device__ T block_reduce(T v, T* s_red, Op op) {
    for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off));
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[wave] = v;
    __syncthreads();
    T r = s_red[0];
    for (int i = 1; i < nw; ++i) r = op(r, s_red[i]);
    return r;
}

// The rest of the query in one workgroup (16 waves), phases separated by barriers:
//   select:     maxCommonWords / minCommonWords (:86-93, :201-207) and the scored slots in
//               lKFsSharingWords order (rank by the walk's first meeting);
//   scores:     the scored slots' L1 scores from the count kernel (ScoringObject.cpp:23-67), stored
//               as mLoopScore / mRelocScore;
//   accumulate: covisibility accumulation (:118-147, :233-259), retain (> 0.75 * best) and
//               first-occurrence de-duplication (:150-168, :262-279);
//   and the word-position table is cleared for the next query.
__global__ __launch_bounds__(1024) void kfdb_finish_kernel(DevKFDB db, KfdbQuery q) {
    __shared__ int s_red[16];
    __shared__ float s_redf[16];
    __shared__ int s_wcnt[16];
    __shared__ int s_cnt;
    __shared__ unsigned long long s_key[kRankLds];
    // per-query lists of the scored slots: in LDS when they fit (the usual case: a handful), else
    // in the global scratch (flat pointers address either)
    __shared__ int s_tmp[kRankLds], s_scored[kRankLds], s_best[kRankLds];
    __shared__ float s_sc[kRankLds], s_acc[kRankLds];
    const int t = q.loop ? 0 : 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    // the query words, held for the final table clear (no reload at the end)
    uint32_t qw[kKfdbMaxWords / 1024];
#pragma unroll
    for (int k = 0; k < kKfdbMaxWords / 1024; ++k) {
        const int i = threadIdx.x + k * 1024;
        qw[k] = i < q.n ? db.qids[i] : 0u;
    }
    // ---- select ----
    const int n = db.cap;
    constexpr int kHeld = 4;  // list entries per thread kept in registers between the two passes
    int held[kHeld];
    int mx = 0;
#pragma unroll
    for (int k = 0; k < kHeld; ++k) {
        const int i = threadIdx.x + k * 1024;
        held[k] = (i < n && db.list[i]) ? db.words[t][i] : -1;
        mx = max(mx, held[k]);
    }
    for (int i = threadIdx.x + kHeld * 1024; i < n; i += blockDim.x)
        if (db.list[i]) mx = max(mx, db.words[t][i]);
    const int maxc = block_reduce(mx, s_red, [](int a, int b) { return max(a, b); });
    const int minc = (int)((float)maxc * 0.8f);  // int minCommonWords = maxCommonWords*0.8f
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    auto keep = [&](int i) {
        const int c = atomicAdd(&s_cnt, 1);
        if (c < kRankLds) s_tmp[c] = i;
        db.tmp[c] = i;
    };
#pragma unroll
    for (int k = 0; k < kHeld; ++k)
        if (held[k] > minc) keep(threadIdx.x + k * 1024);
    for (int i = threadIdx.x + kHeld * 1024; i < n; i += blockDim.x)
        if (db.list[i] && db.words[t][i] > minc) keep(i);
    __syncthreads();
    const int S = s_cnt;
    const bool small = S <= kRankLds;
    int* scored = small ? s_scored : db.scored;
    float* sc = small ? s_sc : db.sc;
    float* accs = small ? s_acc : db.acc;
    int* bests = small ? s_best : db.best;
    if (small) {
        for (int i = threadIdx.x; i < S; i += blockDim.x) s_key[i] = db.key[s_tmp[i]];
        __syncthreads();
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            const unsigned long long k = s_key[i];
            int r = 0;
            for (int j = 0; j < S; ++j) r += s_key[j] < k;
            s_scored[r] = s_tmp[i];
        }
    } else {
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            const int kf = db.tmp[i];
            const unsigned long long k = db.key[kf];
            int r = 0;
            for (int j = 0; j < S; ++j) r += db.key[db.tmp[j]] < k;
            db.scored[r] = kf;
        }
    }
    __syncthreads();
    // ---- scores (computed by the count kernel for every listed slot) ----
    for (int e = threadIdx.x; e < S; e += blockDim.x) {
        const int kf = scored[e];
        const float si = db.tscore[kf];
        sc[e] = si;
        db.score[t][kf] = si;  // mLoopScore / mRelocScore
    }
    __syncthreads();
    // ---- accumulate ----
    float m = q.loop ? q.min_score : 0.0f;  // bestAccScore's initial value
    for (int i = threadIdx.x; i < S; i += blockDim.x) {
        const int kf = scored[i];
        const float si = sc[i];
        if (q.loop && !(si >= q.min_score)) {  // not in lScoreAndMatch
            bests[i] = -1;
            continue;
        }
        float bestScore = si, accScore = si;
        int bk = kf;
        const int nn = db.covis_n[kf];
        int k2[kKfdbCovis], w2[kKfdbCovis];
        unsigned long long q2[kKfdbCovis];
        float s2[kKfdbCovis];
#pragma unroll
        for (int k = 0; k < kKfdbCovis; ++k) k2[k] = db.covis[kf * kKfdbCovis + k];  // rows zero-padded
#pragma unroll
        for (int k = 0; k < kKfdbCovis; ++k) {
            q2[k] = db.query[t][k2[k]];
            w2[k] = db.words[t][k2[k]];
            s2[k] = db.score[t][k2[k]];
        }
#pragma unroll
        for (int k = 0; k < kKfdbCovis; ++k) {
            if (k >= nn || q2[k] != q.id) continue;
            if (q.loop && !(w2[k] > minc)) continue;
            accScore += s2[k];
            if (s2[k] > bestScore) {
                bk = k2[k];
                bestScore = s2[k];
            }
        }
        accs[i] = accScore;
        bests[i] = bk;
        if (accScore > m) m = accScore;
    }
    const float bestAcc = block_reduce(m, s_redf, [](float a, float b) { return a > b ? a : b; });
    const float minRetain = 0.75f * bestAcc;
    __syncthreads();
    int total = 0;
    for (int base = 0; base < S; base += blockDim.x) {
        const int i = base + threadIdx.x;
        bool kept = false;
        if (i < S && bests[i] >= 0 && accs[i] > minRetain) {
            kept = true;
            const int b = bests[i];
            for (int j = 0; j < i && kept; ++j)
                if (bests[j] == b && accs[j] > minRetain) kept = false;  // already added
        }
        const unsigned long long bal = __ballot(kept);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        __syncthreads();
        if (lane == 0) s_wcnt[wave] = __popcll(bal);
        __syncthreads();
        int off = total;
        for (int w = 0; w < wave; ++w) off += s_wcnt[w];
        if (kept) db.out[1 + off + before] = bests[i];
        for (int w = 0; w < nw; ++w) total += s_wcnt[w];
    }
    if (threadIdx.x == 0) db.out[0] = total;
    // ---- clear the word-position table ----
#pragma unroll
    for (int k = 0; k < kKfdbMaxWords / 1024; ++k)
        if (threadIdx.x + k * 1024 < q.n) db.wpos[qw[k]] = -1;
}

}  // namespace

hipError_t launch_kfdb_query(const DevKFDB& db, const KfdbQuery& q, hipStream_t st) {
    if (q.n < 0 || q.n > kKfdbMaxWords || db.cap <= 0) return hipErrorInvalidValue;
    if (q.n > 0) kfdb_scatter_kernel<<<(q.n + 255) / 256, 256, 0, st>>>(db, q);
    kfdb_count_kernel<<<(db.cap + 3) / 4, 256, 0, st>>>(db, q);
    kfdb_finish_kernel<<<1, 1024, 0, st>>>(db, q);
    return hipGetLastError();
}

}  // namespace rsc
