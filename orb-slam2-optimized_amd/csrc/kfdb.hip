// kfdb.hip — KeyFrameDatabase candidate queries (src/KeyFrameDatabase.cpp:52-283); see rsc_kfdb.h.
#include <hip/hip_runtime.h>
#include <atomic>
#include <climits>
#include "rsc_kfdb.h"
#include "rsc_fold.h"

namespace rsc {

namespace {

constexpr int kCountBatch = 16;  // words per lane per batch in the count kernel (1024 per wave)
constexpr int kRankLds = 1024;  // scored slots ranked from LDS (beyond: from global memory)

constexpr uint64_t kKfEmpty = ~0ull;

// log2 of the query hash size: the power of two >= 2 n (at least 64)
__host__ __device__ inline int kf_hash_bits(int n) {
    int b = 6;
    while ((1 << b) < 2 * n) ++b;
    return b;
}  // empty hash entry (word ids are below 2^30)

// The query BowVector as an open-addressing hash in LDS: entry = (position in F->mBowVec << 32) |
// word id, linear probing, 2^bits >= 2 * n entries.
__device__ __forceinline__ uint32_t kf_hash(uint32_t w, int bits) { return (w * 0x9E3779B1u) >> (32 - bits); }

// Positions of B words per lane (-1: not a query word).  Probe rounds are wave-uniform: every round
// reads one entry per word (reads unconditional, so a round's B reads issue together) until every
// word has met its key or an empty entry.
template <int B>
__device__ __forceinline__ void kf_find(const uint64_t* tab, int bits, const uint32_t (&x)[B], const bool (&valid)[B],
                                        int (&p)[B]) {
    const uint32_t mask = (1u << bits) - 1u;
    uint32_t h[B];
    bool done[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        h[b] = kf_hash(x[b], bits);
        done[b] = !valid[b];
        p[b] = -1;
    }
    while (true) {
        uint64_t e[B];
#pragma unroll
        for (int b = 0; b < B; ++b) e[b] = tab[h[b]];
        bool more = false;
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint32_t k = (uint32_t)e[b];
            const bool hit = !done[b] && k == x[b];
            const bool miss = !done[b] && k == (uint32_t)kKfEmpty;
            p[b] = hit ? (int)(e[b] >> 32) : p[b];
            done[b] = done[b] || hit || miss;
            h[b] = (h[b] + 1u) & mask;
            more = more || !done[b];
        }
        if (__ballot(more) == 0) break;
    }
}

// The inverted-file walk (:60-78 loop, :181-196 reloc) seen from one slot: the walk meets slot k
// once per common word, first at the query word `first`, in list order (ascending seq) within a
// word.  One wave per slot, four slots per workgroup; the query BowVector is staged in the
// workgroup's LDS as a hash, so a slot word's position in F->mBowVec is one or two LDS probes (no
// vocabulary-sized table to scatter and clear per query).  Every lane applies the walk's
// per-occurrence state rules in closed form (the inputs are wave-uniform); lane 0 stores them.
#ifndef RSC_KFDB_STAMPS
#define RSC_KFDB_STAMPS 0
#endif
// Diagnostic (built with RSC_KFDB_STAMPS=1): wall clock of slots 0..4095 of the last count launch at
// entry, after the staging barrier, after the common-word count, at exit.
__device__ uint64_t g_kf_stamps[4096][4];
#define KF_STAMP(k) \
    do { \
        if (RSC_KFDB_STAMPS && lane == 0 && slot < 4096) g_kf_stamps[slot][k] = wall_clock64(); \
    } while (0)

__global__ __launch_bounds__(256) void kfdb_count_kernel(DevKFDB db, KfdbQuery q) {
    extern __shared__ __attribute__((aligned(16))) unsigned char kf_lds[];
    // [4 waves][64 * kCountBatch] compacted score terms, the query values, the query hash
    double* s_terms = reinterpret_cast<double*>(kf_lds) + (threadIdx.x >> 6) * (64 * kCountBatch);
    double* s_qv = reinterpret_cast<double*>(kf_lds) + 4 * 64 * kCountBatch;
    uint64_t* s_tab = reinterpret_cast<uint64_t*>(s_qv + q.n);
    const int bits = kf_hash_bits(q.n);
    const int lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool live = slot < db.cap;
    const int t = q.loop ? 0 : 1;
    KF_STAMP(0);
    // the slot's loads issued before the staging: its length, state and first 64 * kCountBatch
    // word ids (the slot stride is max_words, so the window is in bounds whatever the length); the
    // values are gathered later for the common words only (a few percent of a BowVector)
    const size_t row = (size_t)(live ? slot : 0) * db.max_words;
    const uint32_t* ids = db.ids + row;
    const double* vals = db.vals + row;
    int len = 0, w0 = 0;
    unsigned long long qb0 = 0;
    uint32_t w[kCountBatch];
    if (live) {
        len = db.len[slot];
        qb0 = db.query[t][slot];
        w0 = db.words[t][slot];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) w[b] = ids[min(b * 64 + lane, db.max_words - 1)];
    }
    // the query staged with all of a thread's loads in flight at once (up to kKfdbMaxWords words),
    // its hash built while they arrive
    {
        uint32_t qi[kKfdbMaxWords / 256];
        double qv[kKfdbMaxWords / 256];
#pragma unroll
        for (int k = 0; k < kKfdbMaxWords / 256; ++k) {
            const int i = threadIdx.x + 256 * k;
            if (i < q.n) {
                qi[k] = db.qids[i];
                qv[k] = db.qvals[i];
            }
        }
        for (int i = threadIdx.x; i < (1 << bits); i += 256) s_tab[i] = kKfEmpty;
        __syncthreads();
        const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
        for (int k = 0; k < kKfdbMaxWords / 256; ++k) {
            const int i = threadIdx.x + 256 * k;
            if (i < q.n) {
                s_qv[i] = qv[k];
                const uint64_t ent = ((uint64_t)i << 32) | qi[k];
                uint32_t h = kf_hash(qi[k], bits);
                while (atomicCAS((unsigned long long*)&s_tab[h], (unsigned long long)kKfEmpty, (unsigned long long)ent) !=
                       (unsigned long long)kKfEmpty)
                    h = (h + 1u) & mask;
            }
        }
    }
    __syncthreads();
    if (!live) return;
    KF_STAMP(1);
    if (lane == 0) db.list[slot] = 0;  // in lKFsSharingWords (a flag per slot: no shared counter)
    if (len == 0 || q.n == 0) return;  // the walk never touches this slot's state
    int c = 0, first = INT_MAX;
    int p0[kCountBatch];  // positions of the first batch, kept for the score
    for (int base = 0; base < len; base += 64 * kCountBatch) {
        if (base > 0) {
#pragma unroll
            for (int b = 0; b < kCountBatch; ++b) w[b] = ids[min(base + b * 64 + lane, db.max_words - 1)];
        }
        bool valid[kCountBatch];
        int p[kCountBatch];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) valid[b] = base + b * 64 + lane < len;
        kf_find<kCountBatch>(s_tab, bits, w, valid, p);
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) {
            if (p[b] >= 0) {
                c++;
                first = min(first, p[b]);
            }
            if (base == 0) p0[b] = p[b];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        c += __shfl_xor(c, off);
        first = min(first, __shfl_xor(first, off));
    }
    KF_STAMP(2);
    if (c == 0) return;
    unsigned long long qb = qb0;
    int wc = w0;
    bool in_list = false;
    if (qb != q.id) {
        if (q.loop && db.conn[slot]) {
            wc = 1;  // connected: mnLoopWords = 0 then ++ at every occurrence, query id untouched
        } else {
            wc = c;  // reset at the first occurrence, then one increment per occurrence
            qb = q.id;
            in_list = true;
        }
    } else {
        wc += c;  // already met by an earlier query with the same id: counts accumulate, not listed
    }
    if (lane == 0) {
        db.query[t][slot] = qb;
        db.words[t][slot] = wc;
        if (in_list) {
            db.list[slot] = 1;
            db.key[slot] = ((unsigned long long)first << 32) | db.seq[slot];
        }
    }
    if (!in_list) return;
    // L1Scoring::score(F->mBowVec, pKFi->mBowVec) (ScoringObject.cpp:23-67): per-word terms in
    // parallel, compacted into the wave's LDS run in ascending word order (batch, then lane), then
    // summed in that order by lane 0 (the dependent additions are the whole serial part); finish
    // keeps the score only if the slot is scored (mLoopScore / mRelocScore are written there)
    double score = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    auto add_batch = [&](int base, const int (&p)[kCountBatch]) {
        double wv[kCountBatch];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) wv[b] = p[b] >= 0 ? vals[base + b * 64 + lane] : 0.0;
        int off = 0;
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) {
            const double vi = s_qv[max(p[b], 0)], wi = wv[b];
            const double term = fabs(vi - wi) - fabs(vi) - fabs(wi);
            const unsigned long long m = __ballot(p[b] >= 0);
            if (p[b] >= 0) s_terms[off + __popcll(m & below)] = term;
            off += __popcll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) score = fold_run<false>(score, s_terms, off);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    add_batch(0, p0);
    for (int base = 64 * kCountBatch; base < len; base += 64 * kCountBatch) {  // BowVectors over 1024 words
        bool valid[kCountBatch];
        int p[kCountBatch];
#pragma unroll
        for (int b = 0; b < kCountBatch; ++b) {
            w[b] = ids[min(base + b * 64 + lane, db.max_words - 1)];
            valid[b] = base + b * 64 + lane < len;
        }
        kf_find<kCountBatch>(s_tab, bits, w, valid, p);
        add_batch(base, p);
    }
    score = -score / 2.0;
    if (lane == 0) db.tscore[slot] = (float)score;  // float si = mpVoc->score(...)
    KF_STAMP(3);
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
//   select:     maxCommonWords / minCommonWords (:86-93, :201-207); each thread's slots are read
//               once (list flag, word count, rank key, L1 score: independent loads in flight
//               together);
//   keep:       the scored slots (words > minCommonWords);
//   accumulate: one kept slot per thread: covisibility accumulation (:118-147, :233-259) — a
//               neighbour's score is the L1 score the count kernel computed when the neighbour is
//               scored in this query too (the reference writes every scored KeyFrame's score before
//               it accumulates), its stored mLoopScore / mRelocScore otherwise, so the accumulation
//               needs no ranking first;
//   rank:       the scored slots in lKFsSharingWords order (rank by the walk's first meeting); their
//               scores stored as mLoopScore / mRelocScore;
//   retain:     0.75 * best retain and first-occurrence de-duplication (:150-168, :262-279) in that
//               order, candidates written in the reference's vector order.
__global__ __launch_bounds__(1024) void kfdb_finish_kernel(DevKFDB db, KfdbQuery q) {
    __shared__ int s_red[16];
    __shared__ float s_redf[16];
    __shared__ int s_wcnt[16];
    __shared__ int s_cnt;
    // per kept slot (keep order): slot, rank key, score, accumulated score, best KeyFrame; and per
    // rank the retained best KeyFrame (s_rank).  In LDS when they fit (the usual case: a handful),
    // else in the global scratch (flat pointers address either)
    __shared__ unsigned long long s_key[kRankLds];
    __shared__ int s_tmp[kRankLds], s_rank[kRankLds], s_best[kRankLds];
    __shared__ float s_sc[kRankLds], s_acc[kRankLds];
    const int t = q.loop ? 0 : 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    // ---- select ----
    const int n = db.cap;
    constexpr int kHeld = 4;  // slots per thread kept in registers between the passes
    int held[kHeld];
    unsigned long long hkey[kHeld];
    float hsc[kHeld];
    int mx = 0;
#pragma unroll
    for (int k = 0; k < kHeld; ++k) {
        const int i = threadIdx.x + k * 1024;
        const int ii = i < n ? i : 0;
        const int listed = db.list[ii], words = db.words[t][ii];
        hkey[k] = db.key[ii];
        hsc[k] = db.tscore[ii];
        held[k] = (i < n && listed) ? words : -1;
        mx = max(mx, held[k]);
    }
    for (int i = threadIdx.x + kHeld * 1024; i < n; i += blockDim.x)
        if (db.list[i]) mx = max(mx, db.words[t][i]);
    const int maxc = block_reduce(mx, s_red, [](int a, int b) { return max(a, b); });
    const int minc = (int)((float)maxc * 0.8f);  // int minCommonWords = maxCommonWords*0.8f
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    // ---- keep ----
    auto keep = [&](int kf, unsigned long long key, float si) {
        const int c = atomicAdd(&s_cnt, 1);
        db.tmp[c] = kf;
        db.sc[c] = si;
        if (c < kRankLds) {
            s_tmp[c] = kf;
            s_key[c] = key;
            s_sc[c] = si;
        }
    };
#pragma unroll
    for (int k = 0; k < kHeld; ++k)
        if (held[k] > minc) keep(threadIdx.x + k * 1024, hkey[k], hsc[k]);
    for (int i = threadIdx.x + kHeld * 1024; i < n; i += blockDim.x)
        if (db.list[i] && db.words[t][i] > minc) keep(i, db.key[i], db.tscore[i]);
    __syncthreads();
    const int S = s_cnt;
    const bool small = S <= kRankLds;
    // ---- accumulate, one kept slot per thread (keep order) ----
    float m = q.loop ? q.min_score : 0.0f;  // bestAccScore's initial value
    for (int c = threadIdx.x; c < S; c += blockDim.x) {
        const int kf = small ? s_tmp[c] : db.tmp[c];
        const float si = small ? s_sc[c] : db.sc[c];
        float accScore = si, bestScore = si;
        int bk = kf;
        if (q.loop && !(si >= q.min_score)) {  // not in lScoreAndMatch
            bk = -1;
        } else {
            const int nn = db.covis_n[kf];
            int k2[kKfdbCovis], w2[kKfdbCovis], l2[kKfdbCovis];
            unsigned long long q2[kKfdbCovis];
            float s2[kKfdbCovis], t2[kKfdbCovis];
#pragma unroll
            for (int k = 0; k < kKfdbCovis; ++k) k2[k] = db.covis[kf * kKfdbCovis + k];  // rows zero-padded
#pragma unroll
            for (int k = 0; k < kKfdbCovis; ++k) {
                q2[k] = db.query[t][k2[k]];
                w2[k] = db.words[t][k2[k]];
                s2[k] = db.score[t][k2[k]];
                t2[k] = db.tscore[k2[k]];
                l2[k] = db.list[k2[k]];
            }
#pragma unroll
            for (int k = 0; k < kKfdbCovis; ++k) {
                if (k >= nn || q2[k] != q.id) continue;
                if (q.loop && !(w2[k] > minc)) continue;
                // a neighbour scored in this query too carries its new score (the reference writes
                // every scored KeyFrame's score before it accumulates), any other its stored one
                const float sk = (l2[k] && w2[k] > minc) ? t2[k] : s2[k];
                accScore += sk;
                if (sk > bestScore) {
                    bk = k2[k];
                    bestScore = sk;
                }
            }
            if (accScore > m) m = accScore;
        }
        if (small) {
            s_acc[c] = accScore;
            s_best[c] = bk;
        } else {
            db.acc[c] = accScore;
            db.best[c] = bk;
        }
    }
    const float bestAcc = block_reduce(m, s_redf, [](float a, float b) { return a > b ? a : b; });
    const float minRetain = 0.75f * bestAcc;
    const float* sc = small ? s_sc : db.sc;
    const float* accs = small ? s_acc : db.acc;
    const int* bests = small ? s_best : db.best;
    // the retained best KeyFrame of every rank (-1: not retained), in lKFsSharingWords order
    int* rb = small ? s_rank : db.scored;
    // ---- rank + store the scores ----
    for (int c = threadIdx.x; c < S; c += blockDim.x) {
        const int kf = small ? s_tmp[c] : db.tmp[c];
        const unsigned long long k = small ? s_key[c] : db.key[kf];
        int r = 0;
        if (small) {
#pragma unroll 8
            for (int j = 0; j < S; ++j) r += s_key[j] < k;
        } else {
            for (int j = 0; j < S; ++j) r += db.key[db.tmp[j]] < k;
        }
        const int b = bests[c];
        rb[r] = (b >= 0 && accs[c] > minRetain) ? b : -1;
        db.score[t][kf] = sc[c];  // mLoopScore / mRelocScore
    }
    __syncthreads();
    // ---- retain + de-duplicate, in lKFsSharingWords order ----
    int total = 0;
    for (int base = 0; base < S; base += blockDim.x) {
        const int i = base + threadIdx.x;
        bool kept = false;
        int b = -1;
        if (i < S) {
            b = rb[i];
            kept = b >= 0;
            int dup = 0;
#pragma unroll 8
            for (int j = 0; j < i; ++j) dup |= rb[j] == b;  // already added
            kept = kept && !dup;
        }
        const unsigned long long bal = __ballot(kept);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        __syncthreads();
        if (lane == 0) s_wcnt[wave] = __popcll(bal);
        __syncthreads();
        int off = total;
        for (int w = 0; w < wave; ++w) off += s_wcnt[w];
        if (kept) db.out[1 + off + before] = b;
        for (int w = 0; w < nw; ++w) total += s_wcnt[w];
    }
    if (threadIdx.x == 0) db.out[0] = total;
}

}  // namespace

hipError_t read_kfdb_stamps(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kf_stamps), sizeof(g_kf_stamps), 0, hipMemcpyDeviceToHost);
}

hipError_t launch_kfdb_query(const DevKFDB& db, const KfdbQuery& q, hipStream_t st) {
    if (q.n < 0 || q.n > kKfdbMaxWords || db.cap <= 0) return hipErrorInvalidValue;
    // dynamic LDS: the four waves' term runs + the query values and hash (up to 128 KB, above the
    // default 64 KB: the attribute is raised lazily at the first launch on each device)
    const size_t lds = sizeof(double) * (4 * 64 * kCountBatch + (size_t)q.n + ((size_t)1 << kf_hash_bits(q.n)));
    static std::atomic<unsigned long long> raised{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (!((raised.load(std::memory_order_acquire) >> dev) & 1ull)) {
        if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&kfdb_count_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(sizeof(double) * (4 * 64 * kCountBatch + kKfdbMaxWords +
                                                                       (1 << kf_hash_bits(kKfdbMaxWords))))))
            return e;
        raised.fetch_or(1ull << dev, std::memory_order_acq_rel);
    }
    kfdb_count_kernel<<<(db.cap + 3) / 4, 256, lds, st>>>(db, q);
    kfdb_finish_kernel<<<1, 1024, 0, st>>>(db, q);
    return hipGetLastError();
}

}  // namespace rsc
