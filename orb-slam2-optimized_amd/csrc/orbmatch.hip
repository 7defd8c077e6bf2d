// orbmatch.hip — ORBmatcher::SearchByBoW kernels (src/ORBmatcher.cpp:110-240 and :354-488).
// See rsc_orbmatch.h for the mapping: bow_topk_kernel (distance work, parallel over outer
// features) then bow_resolve_kernel (greedy walk per node, orientation filter, output).
#include <hip/hip_runtime.h>
#include "rsc_orbmatch.h"

namespace rsc {

// Diagnostic phase stamps (wall clock, 100 MHz) of the first 64 pairs of the last launch:
// [pair][0] resolve entry, [1] after LDS init, [2 + w] wave w's walk end (16), [18] matches
// written, [19] histogram done, [20] exit, [21 + 2*v], [22 + 2*v] topk wave v (32) entry / exit.
__device__ uint64_t g_bow_stamps[64][96];
__device__ uint64_t g_bow_task_stamps[32][8][4];  // pair 0, wave v, task i: entry, task loaded, staged, done

namespace {

__device__ __forceinline__ void stamp(int pair, int slot) {
    if (pair < 64 && (threadIdx.x & 63) == 0) g_bow_stamps[pair][slot] = wall_clock64();
}

constexpr uint32_t kIdx = ~kBowInvalid;

// ORBmatcher::DescriptorDistance (ORBmatcher.cpp:1492-1508): the bit-parallel count of each XOR
// word is exactly its popcount
__device__ __forceinline__ uint32_t desc_dist(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// TH_LOW is inclusive in the Frame overload (:179), strict in the KeyFrame one (:430)
template <bool kFrame>
__device__ __forceinline__ bool close_enough(uint32_t d) {
    return kFrame ? d <= (uint32_t)kBowThLow : d < (uint32_t)kBowThLow;
}

// Exclusive prefix sum over a 256-thread workgroup (4 waves): returns this thread's offset and
// writes the total to *sum.
__device__ int block_scan256(int v, int* wsum, int* sum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int before = 0;
    for (int i = 0; i < w; ++i) before += wsum[i];
    if (threadIdx.x == 0) *sum = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return before + x - v;
}

// ------------------------------------------------------------------------------------------------
// Kernel 0: common nodes and their 64-feature chunks (one 256-thread workgroup per pair).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBowTopkThreads) void bow_join_kernel(const BowPair* __restrict__ pairs) {
    __shared__ int wsum[4];
    __shared__ int tot[2];
    const BowPair P = pairs[blockIdx.x];
    const DevBow& A = P.outer;
    const DevBow& B = P.inner;
    const int tid = threadIdx.x;
    const int nn = A.n_nodes;
    const int per = (nn + kBowTopkThreads - 1) / kBowTopkThreads;
    const int k0 = min(nn, tid * per), k1 = min(nn, k0 + per);
    // two classes, each listed in node order: "wide" nodes (>= 64 outer features: the long greedy
    // walks of kernel 2) and tasks over >= 128 inner features (the long scans of kernel 1) first
    for (int i = tid; i < A.node_begin[nn]; i += kBowTopkThreads) P.mcp[i] = -1;
    int tw = 0, tn = 0, cw = 0, cn = 0;
    for (int pass = 0; pass < 2; ++pass) {
        int tb_w = 0, tb_n = 0, nb_w = 0, nb_n = 0;
        if (pass == 1) {
            tb_w = block_scan256(tw, wsum, &tot[0]);
            tb_n = tot[0] + block_scan256(tn, wsum, &tot[1]);
            const int tasks_total = tot[0] + tot[1];
            nb_w = block_scan256(cw, wsum, &tot[0]);
            nb_n = tot[0] + block_scan256(cn, wsum, &tot[1]);
            const int nodes_total = tot[0] + tot[1];
            __syncthreads();
            if (tid == 0) {
                P.ntasks[0] = tasks_total;
                P.ntasks[1] = nodes_total;
            }
        }
        for (int k = k0; k < k1; ++k) {
            const uint32_t id = A.node_id[k];
            int lo = 0, hi = B.n_nodes;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (B.node_id[mid] < id) lo = mid + 1;
                else hi = mid;
            }
            if (lo >= B.n_nodes || B.node_id[lo] != id) continue;
            const int a0 = A.node_begin[k], a1 = A.node_begin[k + 1];
            const int b0 = B.node_begin[lo], nb = B.node_begin[lo + 1] - b0;
            const int nsg = bow_segments(nb);
            const int nt = ((a1 - a0 + 63) >> 6) * nsg;
            const bool wide_node = a1 - a0 >= 64, wide_scan = nb >= 128;
            if (pass == 0) {
                if (wide_node) ++cw; else ++cn;
                if (wide_scan) tw += nt; else tn += nt;
            } else {
                P.nodes[wide_node ? nb_w++ : nb_n++] = make_int4(a0, a1, b0, nb);
                const int L = (nb + nsg - 1) / nsg;
                for (int c = a0; c < a1; c += 64)
                    for (int g = 0; g < nsg; ++g) {
                        const int sb = g * L, sl = max(0, min(nb, sb + L) - sb);
                        P.tasks[wide_scan ? tb_w++ : tb_n++] =
                            make_int4(c | (min(64, a1 - c) << 16), b0 | (g << 16), nb, sb | (sl << 16));
                    }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Kernel 1: top-4 (distance, position) keys of every valid outer feature of every common node.
// grid (kBowTopkGroups, pairs); the pair's 4 * kBowTopkGroups waves take its chunk tasks
// round-robin.
// ------------------------------------------------------------------------------------------------
template <bool kFrame>
__global__ __launch_bounds__(kBowTopkThreads) void bow_topk_kernel(const BowPair* __restrict__ pairs) {
    __shared__ uint4 seg_desc[kBowTopkThreads / 64][2 * kBowSeg];  // per-wave inner-node segment
    __shared__ uint32_t seg_key[kBowTopkThreads / 64][kBowSeg];
    const BowPair P = pairs[blockIdx.y];
    const DevBow& A = P.outer;
    const DevBow& B = P.inner;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint4* sd = seg_desc[w];
    uint32_t* sk = seg_key[w];
    const int total = P.ntasks[0];
    const int W = kBowTopkGroups * (kBowTopkThreads / 64);
    const int vw = blockIdx.x * (kBowTopkThreads / 64) + w;
    stamp(blockIdx.y, 21 + 2 * vw);
    int ti = 0;
    for (int t = blockIdx.x * (kBowTopkThreads / 64) + w; t < total; t += W, ++ti) {
        const bool tsv = blockIdx.y == 0 && ti < 8 && lane == 0;
        if (tsv) g_bow_task_stamps[vw][ti][0] = wall_clock64();
        const int4 task = P.tasks[t];
        const int c0 = task.x & 0xFFFF, cnt = task.x >> 16;
        const int b0 = task.y & 0xFFFF, seg = task.y >> 16;
        const int sb = task.w & 0xFFFF, se = sb + (task.w >> 16);  // this task's inner positions
        const bool active = lane < cnt;
        const uint32_t fa = active ? A.feat[c0 + lane] : kBowInvalid;
        const int ea = active ? c0 + lane : c0;
        (void)task.z;
        const uint4 ad0 = A.desc_fv[2 * ea], ad1 = A.desc_fv[2 * ea + 1];
        if (tsv) g_bow_task_stamps[vw][ti][1] = wall_clock64() + (ad0.x & 0);
        uint32_t t0 = kBowNoKey, t1 = kBowNoKey, t2 = kBowNoKey, t3 = kBowNoKey;
        for (int s0 = sb; s0 < se; s0 += kBowSeg) {
            const int m = min(kBowSeg, se - s0);
            // stage this segment of the inner node (rows in FeatureVector order + position keys) in
            // the wave's LDS slot: all loads of the segment issued before the first store
            __builtin_amdgcn_wave_barrier();
            // (descriptor words as plain uint32 arrays: arrays of uint4 were not promoted to
            // registers and went through scratch)
            uint32_t r[kBowSeg / 64][8];
            uint32_t fb[kBowSeg / 64];
#pragma unroll
            for (int u = 0; u < kBowSeg / 64; ++u) {
                // clamped, unconditional loads (see walk_node)
                const int x = min(lane + 64 * u, m - 1);
                const uint4 a = B.desc_fv[2 * (b0 + s0 + x)], b = B.desc_fv[2 * (b0 + s0 + x) + 1];
                r[u][0] = a.x; r[u][1] = a.y; r[u][2] = a.z; r[u][3] = a.w;
                r[u][4] = b.x; r[u][5] = b.y; r[u][6] = b.z; r[u][7] = b.w;
                fb[u] = kFrame ? 0u : B.feat[b0 + s0 + x];
            }
            // every slot entry is stored, without a branch (entries past m hold copies of row m - 1
            // and are never read: the insertion below stops at m)
#pragma unroll
            for (int u = 0; u < kBowSeg / 64; ++u) {
                const int x = lane + 64 * u;
                sd[2 * x] = make_uint4(r[u][0], r[u][1], r[u][2], r[u][3]);
                sd[2 * x + 1] = make_uint4(r[u][4], r[u][5], r[u][6], r[u][7]);
                // invalid inner features (KeyFrame overload, :404-410) get the empty key, which
                // the insertion below leaves out
                sk[x] = (kFrame || !(fb[u] & kBowInvalid)) ? (uint32_t)(s0 + x) : kBowNoKey;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (tsv && s0 == sb) g_bow_task_stamps[vw][ti][2] = wall_clock64() + (sk[0] & 0);
#pragma unroll 4
            for (int q = 0; q < m; ++q) {
                const uint32_t d = desc_dist(ad0, ad1, sd[2 * q], sd[2 * q + 1]);
                const uint32_t kq = sk[q];
                // keys arrive in increasing position, so (distance, position) order is the
                // reference's strict first minimum (:168-177); a 4-deep insertion network
                uint32_t key = kq == kBowNoKey ? kBowNoKey : ((d << 16) | kq);
                uint32_t mn = min(t0, key); key = max(t0, key); t0 = mn;
                mn = min(t1, key); key = max(t1, key); t1 = mn;
                mn = min(t2, key); key = max(t2, key); t2 = mn;
                t3 = min(t3, key);
            }
        }
        // records of invalid outer features stay empty, so kernel 2 never takes them as candidates
        if (active) {
            const uint4 r = (fa & kBowInvalid) ? make_uint4(kBowNoKey, kBowNoKey, kBowNoKey, kBowNoKey)
                                               : make_uint4(t0, t1, t2, t3);
            P.rec[seg * A.node_begin[A.n_nodes] + c0 + lane] = r;
        }
        if (tsv) g_bow_task_stamps[vw][ti][3] = wall_clock64() + (t0 & 0);
    }
    stamp(blockIdx.y, 22 + 2 * vw);
}

// ------------------------------------------------------------------------------------------------
// Kernel 2: greedy walk per common node (one wave each), orientation filter, output.
// ------------------------------------------------------------------------------------------------

// Fold one (distance, position) candidate into a lane's running (first-min key, second-min distance).
__device__ __forceinline__ void fold(uint32_t key, uint32_t& k1, uint32_t& d2) {
    if (key < k1) {
        d2 = min(d2, k1 >> 16);
        k1 = key;
    } else {
        d2 = min(d2, key >> 16);
    }
}

// Matched inner positions of the node being walked (the reference's vpMapPointMatches[realIdxF] /
// vbMatched2 restricted to the node).  Nodes of up to 64 / 256 positions keep them in one / four
// wave-uniform 64-bit words (scalar registers); larger nodes spread them over the lanes: lane
// pos % 64, bit pos / 64 (read with v_readlane, pos is wave-uniform).  test4 returns the matched
// flags of the four record slots whose positions are packed 16 bits each in `pk`.
struct Set64 {
    uint64_t w = 0;
    __device__ bool test(uint32_t pos) const { return (w >> (pos & 63)) & 1ull; }
    __device__ uint32_t test4(uint64_t pk) const {
        return (uint32_t)(((w >> (pk & 63)) & 1ull) | (((w >> ((pk >> 16) & 63)) & 1ull) << 1) |
                          (((w >> ((pk >> 32) & 63)) & 1ull) << 2) | (((w >> ((pk >> 48) & 63)) & 1ull) << 3));
    }
    __device__ bool lane_test(uint32_t, int lane) const { return (w >> lane) & 1ull; }
    __device__ void set(uint32_t pos, int) { w |= 1ull << (pos & 63); }
};

struct Set256 {
    uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __device__ uint64_t word(uint32_t c) const { return c == 0 ? w0 : c == 1 ? w1 : c == 2 ? w2 : w3; }
    __device__ bool test(uint32_t pos) const { return (word((pos >> 6) & 3) >> (pos & 63)) & 1ull; }
    __device__ uint32_t test4(uint64_t pk) const {
        return (uint32_t)test((uint32_t)pk & 0xFFFFu) | ((uint32_t)test((uint32_t)(pk >> 16) & 0xFFFFu) << 1) |
               ((uint32_t)test((uint32_t)(pk >> 32) & 0xFFFFu) << 2) | ((uint32_t)test((uint32_t)(pk >> 48)) << 3);
    }
    __device__ bool lane_test(uint32_t c, int lane) const { return (word(c) >> lane) & 1ull; }
    __device__ void set(uint32_t pos, int) {
        const uint64_t b = 1ull << (pos & 63);
        const uint32_t c = pos >> 6;
        if (c == 0) w0 |= b;
        else if (c == 1) w1 |= b;
        else if (c == 2) w2 |= b;
        else w3 |= b;
    }
};

struct LaneSet {
    uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;  // this lane's positions, bit = chunk
    __device__ uint32_t word(uint32_t c) const { return c < 32 ? m0 : c < 64 ? m1 : c < 96 ? m2 : m3; }
    __device__ bool test(uint32_t pos) const {
        if (pos >= (uint32_t)kBowMaxFeatures) return false;
        const uint32_t c = pos >> 6;
        return ((uint32_t)__builtin_amdgcn_readlane(word(c), pos & 63) >> (c & 31)) & 1u;
    }
    __device__ uint32_t test4(uint64_t pk) const {
        return (uint32_t)test((uint32_t)pk & 0xFFFFu) | ((uint32_t)test((uint32_t)(pk >> 16) & 0xFFFFu) << 1) |
               ((uint32_t)test((uint32_t)(pk >> 32) & 0xFFFFu) << 2) | ((uint32_t)test((uint32_t)(pk >> 48)) << 3);
    }
    __device__ bool lane_test(uint32_t c, int) const { return (word(c) >> (c & 31)) & 1u; }
    __device__ void set(uint32_t pos, int lane) {
        const uint32_t c = pos >> 6;
        if (lane == (int)(pos & 63)) {
            const uint32_t bit = 1u << (c & 31);
            if (c < 32) m0 |= bit;
            else if (c < 64) m1 |= bit;
            else if (c < 96) m2 |= bit;
            else m3 |= bit;
        }
    }
};

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32);
}

// insert `key` into the ascending 4-list t (the kernel-1 network; merges the segment records)
__device__ __forceinline__ void insert4(uint32_t (&t)[4], uint32_t key) {
    uint32_t mn = min(t[0], key); key = max(t[0], key); t[0] = mn;
    mn = min(t[1], key); key = max(t[1], key); t[1] = mn;
    mn = min(t[2], key); key = max(t[2], key); t[2] = mn;
    t[3] = min(t[3], key);
}

// The greedy walk of one common node (:152-200 / :384-449) over its outer features in order.
// Lane-parallel part (per chunk of 64 outer features): merge the node's segment records into the
// top-4 keys, and tabulate for each of the 16 matched-subsets of the 4 slots the reference's
// outcome (best slot, reject, or "rescan" when fewer than two slots are unmatched in a full
// record).  Serial part: the candidates in order, each a table lookup indexed by the matched flags
// of its slots, and an update of the matched set.
template <bool kFrame, class M>
__device__ void walk_node(const BowPair& P, const DevBow& A, const DevBow& B, int a0, int a1, int b0, int nb,
                          int nseg, int rec_stride, float nnratio, int16_t* mcp, int lane) {
    M matched;
    for (int c0 = a0; c0 < a1; c0 += 64) {
        const bool act = c0 + lane < a1;
        // all segment records loaded unconditionally (clamped indices) before any use: a per-load
        // condition makes hipcc branch around each load and wait for it
        const int ea = act ? c0 + lane : c0;
        uint4 sr[kBowMaxSegs];
#pragma unroll
        for (int g = 0; g < kBowMaxSegs; ++g) sr[g] = P.rec[min(g, nseg - 1) * rec_stride + ea];
        uint32_t t[4] = {sr[0].x, sr[0].y, sr[0].z, sr[0].w};
#pragma unroll
        for (int g = 1; g < kBowMaxSegs; ++g) {
            const bool use = g < nseg;
            insert4(t, use ? sr[g].x : kBowNoKey);
            insert4(t, use ? sr[g].y : kBowNoKey);
            insert4(t, use ? sr[g].z : kBowNoKey);
            insert4(t, use ? sr[g].w : kBowNoKey);
        }
        if (!act) t[0] = t[1] = t[2] = t[3] = kBowNoKey;
        // outer features that can match at all: valid map point (:144-148, :388-392; kernel 1 writes
        // empty records for invalid ones) and a first key within TH_LOW (bestDist1 only grows when
        // keys are excluded)
        uint64_t cand = __ballot(act && close_enough<kFrame>(t[0] >> 16));
        if (!cand) continue;
        uint32_t real = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) real |= (t[q] != kBowNoKey ? 1u : 0u) << q;
        const bool complete = real != 0xFu;  // real keys are a prefix; an empty slot = complete list
        uint64_t tab = 0;
#pragma unroll
        for (uint32_t mm = 0; mm < 16; ++mm) {
            const uint32_t um = real & ~mm;
            const int found = __builtin_popcount(um);
            uint32_t out = 4;  // reject
            if (found < 2 && !complete) {
                out = 5;  // rescan the node
            } else if (found >= 1) {
                const int i1 = __builtin_ctz(um);
                const uint32_t best1 = (i1 == 0 ? t[0] : i1 == 1 ? t[1] : i1 == 2 ? t[2] : t[3]) >> 16;
                uint32_t d2 = 256;
                if (found >= 2) {
                    const int i2 = __builtin_ctz(um & (um - 1));
                    d2 = (i2 == 1 ? t[1] : i2 == 2 ? t[2] : t[3]) >> 16;
                }
                if (close_enough<kFrame>(best1) && (float)best1 < nnratio * (float)d2) out = (uint32_t)i1;
            }
            tab |= (uint64_t)out << (3 * mm);
        }
        const uint64_t pk = (uint64_t)(t[0] & 0xFFFFu) | ((uint64_t)(t[1] & 0xFFFFu) << 16) |
                            ((uint64_t)(t[2] & 0xFFFFu) << 32) | ((uint64_t)(t[3] & 0xFFFFu) << 48);
        int mine = -1;  // this lane's matched inner FeatureVector entry
        while (cand) {
            const int l = __builtin_ctzll(cand);
            cand &= cand - 1;
            const uint64_t pkl = readlane64(pk, l);
            const uint32_t mm = matched.test4(pkl);
            const uint32_t out = (uint32_t)(readlane64(tab, l) >> (3 * mm)) & 7u;
            uint32_t pos = 0xFFFFu;
            if (out < 4) {
                pos = (uint32_t)(pkl >> (16 * out)) & 0xFFFFu;
            } else if (out == 5) {
                // three or four of the record's keys already matched: rescan the node with the
                // inner positions on the lanes (:155-178 / :398-428)
                uint32_t k1 = kBowNoKey, dd = 256;
                const int ea = c0 + l;
                const uint4 ad0 = A.desc_fv[2 * ea], ad1 = A.desc_fv[2 * ea + 1];
                for (int c = 0; c < (nb + 63) >> 6; ++c) {
                    const int q = (c << 6) + lane;
                    if (q >= nb) continue;
                    const uint32_t fb = kFrame ? 0u : B.feat[b0 + q];
                    const int eb = b0 + q;
                    if ((kFrame || !(fb & kBowInvalid)) && !matched.lane_test((uint32_t)c, lane))
                        fold((desc_dist(ad0, ad1, B.desc_fv[2 * eb], B.desc_fv[2 * eb + 1]) << 16) | (uint32_t)q, k1,
                             dd);
                }
                // butterfly merge: the multiset second minimum of a union is min(second of the
                // side holding the minimum, first of the other)
                for (int off = 32; off >= 1; off >>= 1) {
                    const uint32_t o1 = __shfl_xor(k1, off);
                    const uint32_t od = __shfl_xor(dd, off);
                    if (o1 < k1) {
                        dd = min(od, k1 >> 16);
                        k1 = o1;
                    } else {
                        dd = min(dd, o1 >> 16);
                    }
                }
                k1 = uniform(k1);
                dd = uniform(dd);
                const uint32_t best1 = k1 >> 16;
                if (close_enough<kFrame>(best1) && (float)best1 < nnratio * (float)dd) pos = k1 & 0xFFFFu;
            }
            if (pos != 0xFFFFu) {
                matched.set(pos, lane);
                mine = lane == l ? b0 + (int)pos : mine;
            }
        }
        if (act) mcp[c0 + lane] = (int16_t)mine;
    }
}

// ------------------------------------------------------------------------------------------------
// Kernel 2: the greedy walk, one wave per common node (grid (nodes / 4, pairs)); matches go to the
// pair's mcp vector (matched inner FeatureVector entry per outer entry, -1 from kernel 0).
// ------------------------------------------------------------------------------------------------
template <bool kFrame>
__global__ __launch_bounds__(kBowTopkThreads) void bow_walk_kernel(const BowPair* __restrict__ pairs, float nnratio) {
    const BowPair P = pairs[blockIdx.y];
    const int lane = threadIdx.x & 63;
    const int k = blockIdx.x * (kBowTopkThreads / 64) + (threadIdx.x >> 6);
    if (k >= P.ntasks[1]) return;
    const DevBow& A = P.outer;
    const DevBow& B = P.inner;
    const int nfA = A.node_begin[A.n_nodes];
    const int4 node = P.nodes[k];
    const int nseg = bow_segments(node.w);
    if (node.w <= 64)
        walk_node<kFrame, Set64>(P, A, B, node.x, node.y, node.z, node.w, nseg, nfA, nnratio, P.mcp, lane);
    else if (node.w <= 256)
        walk_node<kFrame, Set256>(P, A, B, node.x, node.y, node.z, node.w, nseg, nfA, nnratio, P.mcp, lane);
    else
        walk_node<kFrame, LaneSet>(P, A, B, node.x, node.y, node.z, node.w, nseg, nfA, nnratio, P.mcp, lane);
}

// ------------------------------------------------------------------------------------------------
// Kernel 3: matches -> the reference's vector, orientation filter, output (one workgroup per pair).
// ------------------------------------------------------------------------------------------------
template <bool kFrame>
__global__ __launch_bounds__(kBowResolveThreads) void bow_resolve_kernel(const BowPair* __restrict__ pairs,
                                                                         float nnratio, int check_ori) {
    __shared__ int16_t res[kBowMaxFeatures];  // the output vector in the reference's indexing
    __shared__ int hist[kBowHistoLength];
    __shared__ int keep[3];
    __shared__ int total;
    const BowPair P = pairs[blockIdx.x];
    const DevBow& A = P.outer;
    const DevBow& B = P.inner;
    const int outN = kFrame ? B.n : A.n;
    const int nfA = A.node_begin[A.n_nodes];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) stamp(blockIdx.x, 0);
    for (int i = tid; i < outN; i += kBowResolveThreads) res[i] = -1;
    if (tid < kBowHistoLength) hist[tid] = 0;
    if (tid == 0) total = 0;
    __syncthreads();

    if (tid == 0) stamp(blockIdx.x, 1);
    // matches -> the reference's vector: vpMapPointMatches[bestIdxF] = pMP (:183) /
    // vpMatches12[idx1] = vpMapPoints2[bestIdx2] (:434)
    for (int i = tid; i < nfA; i += kBowResolveThreads) {
        const int cp = P.mcp[i];
        if (cp < 0) continue;
        const int ai = (int)(A.feat[i] & kIdx), bi = (int)(B.feat[cp] & kIdx);
        if (kFrame) res[bi] = (int16_t)ai;
        else res[ai] = (int16_t)bi;
    }
    __syncthreads();
    if (tid == 0) stamp(blockIdx.x, 18);

    // rotation consistency (:218-237, :466-485): histogram of the matches' bins, three maxima,
    // every match outside the kept bins removed
    if (check_ori) {
        // per-wave bin counts by ballot, one LDS add per (wave, bin present)
        for (int i0 = tid - lane; i0 < outN; i0 += kBowResolveThreads) {
            const int i = i0 + lane;
            const int v = i < outN ? res[i] : -1;
            int bin = -1;
            if (v >= 0) {
                const int a = kFrame ? v : i, b = kFrame ? i : v;
                bin = bow_rot_bin(A.angle[a], B.angle[b]);
            }
            uint64_t any = __ballot(bin >= 0);
            while (any) {
                const int bb = __builtin_amdgcn_readlane(bin, __builtin_ctzll(any));
                const uint64_t same = __ballot(bin == bb);
                if (lane == 0) atomicAdd(&hist[bb], (int)__popcll(same));
                any &= ~same;
            }
        }
        __syncthreads();
        if (tid == 0) {
            // ComputeThreeMaxima (ORBmatcher.cpp:1446-1487)
            int hs[kBowHistoLength];  // all bin reads issued before the serial scan
#pragma unroll
            for (int i = 0; i < kBowHistoLength; ++i) hs[i] = hist[i];
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
#pragma unroll
            for (int i = 0; i < kBowHistoLength; ++i) {
                const int s = hs[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s; ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1;
                ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
            keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
        }
        __syncthreads();
    }
    if (tid == 0) stamp(blockIdx.x, 19);
    int cnt = 0;
    for (int i = tid; i < outN; i += kBowResolveThreads) {
        int v = res[i];
        if (v >= 0 && check_ori) {
            const int a = kFrame ? v : i, b = kFrame ? i : v;
            const int bin = bow_rot_bin(A.angle[a], B.angle[b]);
            if (bin != keep[0] && bin != keep[1] && bin != keep[2]) v = -1;
        }
        P.out[i] = v;
        cnt += v >= 0;
    }
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0 && cnt) atomicAdd(&total, cnt);
    __syncthreads();
    if (tid == 0) {
        *P.nmatches = total;
        stamp(blockIdx.x, 20);
    }
}

}  // namespace

hipError_t read_bow_stamps(uint64_t* out, int cap) {
    const int n = cap < 64 * 96 ? cap : 64 * 96;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bow_stamps), sizeof(uint64_t) * n, 0, hipMemcpyDeviceToHost);
    if (e != hipSuccess || cap < 64 * 96 + 32 * 8 * 4) return e;
    return hipMemcpyFromSymbol(out + 64 * 96, HIP_SYMBOL(g_bow_task_stamps), sizeof(uint64_t) * 32 * 8 * 4, 0,
                               hipMemcpyDeviceToHost);
}

hipError_t launch_bow_search(bool frame_overload, int count, int max_outer_nodes, const BowPair* pairs, float nnratio,
                             int check_ori, hipStream_t st) {
    const dim3 g1(kBowTopkGroups, count);
    const dim3 g2((max_outer_nodes + 3) / 4 > 0 ? (max_outer_nodes + 3) / 4 : 1, count);
    bow_join_kernel<<<count, kBowTopkThreads, 0, st>>>(pairs);
    if (frame_overload) {
        bow_topk_kernel<true><<<g1, kBowTopkThreads, 0, st>>>(pairs);
        bow_walk_kernel<true><<<g2, kBowTopkThreads, 0, st>>>(pairs, nnratio);
        bow_resolve_kernel<true><<<count, kBowResolveThreads, 0, st>>>(pairs, nnratio, check_ori);
    } else {
        bow_topk_kernel<false><<<g1, kBowTopkThreads, 0, st>>>(pairs);
        bow_walk_kernel<false><<<g2, kBowTopkThreads, 0, st>>>(pairs, nnratio);
        bow_resolve_kernel<false><<<count, kBowResolveThreads, 0, st>>>(pairs, nnratio, check_ori);
    }
    return hipGetLastError();
}

}  // namespace rsc
