// orbmatch.hip — ORBmatcher::SearchByBoW kernels (src/ORBmatcher.cpp:110-240 and :354-488).
// See rsc_orbmatch.h for the mapping: bow_topk_kernel (distance work, parallel over outer
// features) then bow_resolve_kernel (greedy walk per node, orientation filter, output).
#include <hip/hip_runtime.h>
#include "rsc_orbmatch.h"

namespace rsc {

namespace {

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
    const DevBow A = *P.outer;
    const DevBow B = *P.inner;
    const int tid = threadIdx.x;
    const int nn = A.n_nodes;
    const int per = (nn + kBowTopkThreads - 1) / kBowTopkThreads;
    const int k0 = min(nn, tid * per), k1 = min(nn, k0 + per);
    int tasks = 0, common = 0;
    for (int k = k0; k < k1; ++k) {
        const uint32_t id = A.node_id[k];
        int lo = 0, hi = B.n_nodes;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.node_id[mid] < id) lo = mid + 1;
            else hi = mid;
        }
        if (lo < B.n_nodes && B.node_id[lo] == id) {
            ++common;
            tasks += (A.node_begin[k + 1] - A.node_begin[k] + 63) >> 6;
        }
    }
    int tbase = block_scan256(tasks, wsum, &tot[0]);
    int nbase = block_scan256(common, wsum, &tot[1]);
    for (int k = k0; k < k1; ++k) {
        const uint32_t id = A.node_id[k];
        int lo = 0, hi = B.n_nodes;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.node_id[mid] < id) lo = mid + 1;
            else hi = mid;
        }
        if (lo < B.n_nodes && B.node_id[lo] == id) {
            const int a0 = A.node_begin[k], a1 = A.node_begin[k + 1];
            const int b0 = B.node_begin[lo], nb = B.node_begin[lo + 1] - b0;
            P.nodes[nbase++] = make_int4(a0, a1, b0, nb);
            for (int c = a0; c < a1; c += 64) P.tasks[tbase++] = make_int4(c, min(64, a1 - c), b0, nb);
        }
    }
    if (tid == 0) {
        P.ntasks[0] = tot[0];
        P.ntasks[1] = tot[1];
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
    const DevBow A = *P.outer;
    const DevBow B = *P.inner;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint4* sd = seg_desc[w];
    uint32_t* sk = seg_key[w];
    const int total = P.ntasks[0];
    const int W = kBowTopkGroups * (kBowTopkThreads / 64);
    for (int t = blockIdx.x * (kBowTopkThreads / 64) + w; t < total; t += W) {
        const int4 task = P.tasks[t];
        const int c0 = task.x, b0 = task.z, nb = task.w;
        const bool active = lane < task.y;
        const uint32_t fa = active ? A.feat[c0 + lane] : kBowInvalid;
        const uint32_t ai = fa & kIdx;
        const uint4 ad0 = A.desc[2 * ai], ad1 = A.desc[2 * ai + 1];
        uint32_t t0 = kBowNoKey, t1 = kBowNoKey, t2 = kBowNoKey, t3 = kBowNoKey;
        for (int s0 = 0; s0 < nb; s0 += kBowSeg) {
            const int m = min(kBowSeg, nb - s0);
            // stage this segment of the inner node (descriptors + position keys) in the wave's
            // LDS slot: coalesced index loads, then one 32-B row per lane
            __builtin_amdgcn_wave_barrier();
            for (int x = lane; x < m; x += 64) {
                const uint32_t fb = B.feat[b0 + s0 + x];
                const uint32_t bi = fb & kIdx;
                sd[2 * x] = B.desc[2 * bi];
                sd[2 * x + 1] = B.desc[2 * bi + 1];
                // invalid inner features (KeyFrame overload, :404-410) get the empty key, which the
                // insertion below leaves out
                sk[x] = (kFrame || !(fb & kBowInvalid)) ? (uint32_t)(s0 + x) : kBowNoKey;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
        if (active && !(fa & kBowInvalid)) P.rec[c0 + lane] = make_uint4(t0, t1, t2, t3);
    }
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

// matched flag of inner position `pos` of the node being walked: lane pos % 64, bit pos / 64 of the
// lane's 128-bit mask (read with v_readlane, pos is wave-uniform)
__device__ __forceinline__ bool is_matched(uint32_t pos, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
    const uint32_t c = pos >> 6;
    const uint32_t v = c < 32 ? m0 : c < 64 ? m1 : c < 96 ? m2 : m3;
    return ((uint32_t)__builtin_amdgcn_readlane(v, pos & 63) >> (c & 31)) & 1u;
}

template <bool kFrame>
__global__ __launch_bounds__(kBowResolveThreads) void bow_resolve_kernel(const BowPair* __restrict__ pairs,
                                                                         float nnratio, int check_ori) {
    __shared__ int16_t res[kBowMaxFeatures];  // the output vector in the reference's indexing
    __shared__ int16_t mcp[kBowMaxFeatures];  // per outer FeatureVector entry: matched inner entry or -1
    __shared__ int hist[kBowHistoLength];
    __shared__ int keep[3];
    __shared__ int total;
    const BowPair P = pairs[blockIdx.x];
    const DevBow A = *P.outer;
    const DevBow B = *P.inner;
    const int outN = kFrame ? B.n : A.n;
    const int nfA = A.node_begin[A.n_nodes];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < outN; i += kBowResolveThreads) res[i] = -1;
    for (int i = tid; i < nfA; i += kBowResolveThreads) mcp[i] = -1;
    if (tid < kBowHistoLength) hist[tid] = 0;
    if (tid == 0) total = 0;
    __syncthreads();

    const int ncommon = P.ntasks[1];
    for (int k = wave; k < ncommon; k += kBowResolveThreads / 64) {
        const int4 node = P.nodes[k];
        const int a0 = node.x, a1 = node.y, b0 = node.z, nb = node.w;
        uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;  // matched inner positions of this lane, bit = chunk
        uint32_t fa_n = kBowInvalid;
        uint4 rec_n = make_uint4(kBowNoKey, kBowNoKey, kBowNoKey, kBowNoKey);
        if (a0 + lane < a1) {  // records of invalid features are never written; read and ignored
            fa_n = A.feat[a0 + lane];
            rec_n = P.rec[a0 + lane];
        }
        for (int c0 = a0; c0 < a1; c0 += 64) {
            // this chunk of 64 outer features on the lanes; the next chunk's loads go out now
            const uint32_t fa = fa_n;
            const uint4 rec = rec_n;
            fa_n = kBowInvalid;
            if (c0 + 64 + lane < a1) {
                fa_n = A.feat[c0 + 64 + lane];
                rec_n = P.rec[c0 + 64 + lane];
            }
            // outer features that can match at all: valid map point (:144-148, :388-392) and a first
            // key within TH_LOW (bestDist1 can only grow when keys are excluded)
            uint64_t cand = __ballot(c0 + lane < a1 && !(fa & kBowInvalid) && close_enough<kFrame>(rec.x >> 16));
            while (cand) {
                const int l = __builtin_ctzll(cand);
                cand &= cand - 1;
                const uint32_t r[4] = {(uint32_t)__builtin_amdgcn_readlane(rec.x, l),
                                       (uint32_t)__builtin_amdgcn_readlane(rec.y, l),
                                       (uint32_t)__builtin_amdgcn_readlane(rec.z, l),
                                       (uint32_t)__builtin_amdgcn_readlane(rec.w, l)};
                // first two unmatched keys of the record
                uint32_t u1 = kBowNoKey, d2 = 256;
                int found = 0;
                bool complete = false;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if (found == 2 || complete) continue;
                    if (r[s] == kBowNoKey) {
                        complete = true;
                        continue;
                    }
                    if (is_matched(r[s] & 0xFFFFu, m0, m1, m2, m3)) continue;
                    if (found == 0) u1 = r[s];
                    else d2 = r[s] >> 16;
                    ++found;
                }
                if (found < 2 && !complete) {
                    // three or four of the record's keys already matched: rescan the node with the
                    // inner positions on the lanes (:155-178 / :398-428)
                    uint32_t k1 = kBowNoKey, dd = 256;
                    const uint32_t ai = (uint32_t)__builtin_amdgcn_readlane(fa, l) & kIdx;
                    const uint4 ad0 = A.desc[2 * ai], ad1 = A.desc[2 * ai + 1];
                    for (int c = 0; c < (nb + 63) >> 6; ++c) {
                        const int pos = (c << 6) + lane;
                        if (pos >= nb) continue;
                        const uint32_t mw = c < 32 ? m0 : c < 64 ? m1 : c < 96 ? m2 : m3;
                        const uint32_t fb = B.feat[b0 + pos];
                        const uint32_t bi = fb & kIdx;
                        if ((kFrame || !(fb & kBowInvalid)) && !((mw >> (c & 31)) & 1u))
                            fold((desc_dist(ad0, ad1, B.desc[2 * bi], B.desc[2 * bi + 1]) << 16) | (uint32_t)pos, k1, dd);
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
                    u1 = uniform(k1);
                    d2 = uniform(dd);
                }
                const uint32_t best1 = u1 >> 16;
                if (close_enough<kFrame>(best1) && (float)best1 < nnratio * (float)d2) {
                    const uint32_t pos = u1 & 0xFFFFu;
                    const uint32_t c = pos >> 6;
                    if (lane == (int)(pos & 63)) {
                        const uint32_t bit = 1u << (c & 31);
                        if (c < 32) m0 |= bit;
                        else if (c < 64) m1 |= bit;
                        else if (c < 96) m2 |= bit;
                        else m3 |= bit;
                    }
                    if (lane == 0) mcp[c0 + l] = (int16_t)(b0 + pos);
                }
            }
        }
    }
    __syncthreads();
    // matches -> the reference's vector: vpMapPointMatches[bestIdxF] = pMP (:183) /
    // vpMatches12[idx1] = vpMapPoints2[bestIdx2] (:434)
    for (int i = tid; i < nfA; i += kBowResolveThreads) {
        const int cp = mcp[i];
        if (cp < 0) continue;
        const int ai = (int)(A.feat[i] & kIdx), bi = (int)(B.feat[cp] & kIdx);
        if (kFrame) res[bi] = (int16_t)ai;
        else res[ai] = (int16_t)bi;
    }
    __syncthreads();

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
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kBowHistoLength; ++i) {
                const int s = hist[i];
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
    if (tid == 0) *P.nmatches = total;
}

}  // namespace

hipError_t launch_bow_search(bool frame_overload, int count, const BowPair* pairs, float nnratio, int check_ori,
                             hipStream_t st) {
    const dim3 g1(kBowTopkGroups, count);
    bow_join_kernel<<<count, kBowTopkThreads, 0, st>>>(pairs);
    if (frame_overload) {
        bow_topk_kernel<true><<<g1, kBowTopkThreads, 0, st>>>(pairs);
        bow_resolve_kernel<true><<<count, kBowResolveThreads, 0, st>>>(pairs, nnratio, check_ori);
    } else {
        bow_topk_kernel<false><<<g1, kBowTopkThreads, 0, st>>>(pairs);
        bow_resolve_kernel<false><<<count, kBowResolveThreads, 0, st>>>(pairs, nnratio, check_ori);
    }
    return hipGetLastError();
}

}  // namespace rsc
