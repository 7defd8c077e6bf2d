// rsc_orbmatch.h — ORBmatcher::SearchByBoW (src/ORBmatcher.cpp:110-240 Frame overload,
// :354-488 KeyFrame overload) on the GPU: device layout and the helpers shared by the kernels
// (orbmatch.hip) and the host.
//
// Independence.  DBoW2 FeatureVector nodes partition a view's features (every feature sits in one
// node, DBoW2 TemplatedVocabulary::transform), and the reference's sequential state — the "already
// matched" test on the inner side (vpMapPointMatches[realIdxF], :160; vbMatched2, :404) — only ever
// touches inner features of the node being walked.  So common nodes are independent; within a node
// the outer features are a greedy sequence.
//
// Three kernels per launch:
//  0. bow_join_kernel — the reference's merge walk visits exactly the node ids present in both
//     FeatureVectors (:130-211); one workgroup per pair binary-searches each outer node in the
//     inner keys and writes the compact lists of common nodes and of their 64-feature chunks.
//  1. bow_topk_kernel — the O(|A_n| x |B_n|) distance work, fully parallel: lanes = outer features
//     of a node (chunks of 64), the node's inner features read as LDS broadcasts; each
//     lane keeps the 4 smallest (distance, position) keys of its feature over the valid inner
//     features, in the reference's first-minimum order, and stores them as one 16-B record.  The
//     inner node is staged through a per-wave LDS segment.  Several workgroups per pair fill the chip.
//  2. bow_walk_kernel — the greedy walk, one wave per common node (all nodes of all pairs at once): the
//     outer features of a node sit on the lanes 64 at a time, a ballot keeps those whose first key
//     is within TH_LOW, and the wave visits them in order (readlane); the first two unmatched keys
//     of a record give bestDist1 / bestIdx / bestDist2 exactly (a record ending in an empty slot is
//     complete), with the node's matched positions held as per-lane bit masks.  Only when three of
//     the four keys are already matched does the wave rescan the node (lanes = inner positions,
//     butterfly merge of (first-min key, second-min distance)).
//  3. bow_resolve_kernel — one workgroup per pair: the matches become the reference's vector, the
//     orientation histogram (ComputeThreeMaxima, :1446-1487) filters them and the output vector is
//     written coalesced.
//
// Integer popcount + a handful of float ops: no MFMA; HBM traffic is the descriptor rows once plus
// 16 B of record per outer feature.
#pragma once
#include <cmath>
#include <cstdint>
#include <hip/hip_runtime.h>

namespace rsc {

constexpr int kBowMaxFeatures = 8192;   // features per view (positions and indices fit 16 bits)
constexpr int kBowThLow = 50;           // ORBmatcher::TH_LOW (ORBmatcher.cpp:9)
constexpr int kBowHistoLength = 30;     // ORBmatcher::HISTO_LENGTH (ORBmatcher.cpp:10)
constexpr int kBowTopkThreads = 256;    // kernel 1: 4 waves per workgroup
constexpr int kBowTopkGroups = 8;       // kernel 1: workgroups per pair
constexpr int kBowMaxSegs = 8;          // inner nodes wider than 64 positions are scanned in up to 8
                                        // segments by different waves (records merged in kernel 2)
constexpr int kBowSeg = 256;            // kernel 1: inner-node positions staged in LDS per wave at a time
constexpr int kBowResolveThreads = 1024;  // kernel 2: 16 waves, one workgroup per pair
constexpr uint32_t kBowInvalid = 0x80000000u;  // flag on a FeatureVector entry: no map point / bad
constexpr uint32_t kBowNoKey = (256u << 16) | 0xFFFFu;  // empty record slot (distance 256, no feature)

// One view (KeyFrame or Frame) resident in HBM; the header itself lives in device memory at the
// start of the view's allocation.
struct DevBow {
    const uint4* desc;          // [n][2] descriptor rows (32 B, mDescriptors.row(i))
    const uint4* desc_fv;       // [feat entries][2] the same rows in FeatureVector order (desc_fv[e] =
                                // desc[feat[e]]), so a node's rows are one contiguous coalesced range
    const float* angle;         // [n] keypoint angle in degrees
    const uint32_t* node_id;    // [n_nodes] FeatureVector keys, strictly ascending
    const int32_t* node_begin;  // [n_nodes + 1] CSR offsets into feat
    const uint32_t* feat;       // feature indices of each node in order, | kBowInvalid when the
                                // feature's map point is missing or bad
    int n;
    int n_nodes;
};

// One searched pair.  outer = the side whose features are taken in turn (pKF in the Frame
// overload, pKF1 in the KeyFrame overload), inner = the side searched (F, pKF2).
struct BowPair {
    DevBow outer;       // view headers by value: one load per workgroup instead of a dependent chain
    DevBow inner;
    uint4* rec;         // [kBowMaxSegs][outer feat entries] top-4 records per inner segment (kernel 1 -> 2)
    int4* tasks;        // [(outer n_nodes + outer feat entries / 64 + 1) * kBowMaxSegs] one per
                        // (64-feature chunk, inner segment) of each common node (kernel 0 -> kernel 1):
                        // (first | count << 16, b0 | segment << 16, nb, segment begin | length << 16)
    int4* nodes;        // [outer n_nodes] (a0, a1, b0, nb) per common node (kernel 0 -> kernel 2)
    int32_t* ntasks;    // [2] tasks, common nodes
    int16_t* mcp;       // [outer feat entries] matched inner FeatureVector entry or -1 (kernel 2 -> 3)
    int32_t* out;       // Frame overload: [inner.n] outer index per inner feature; KF: [outer.n] inner index
    int32_t* nmatches;  // [1]
};

// segments of an inner node of nb positions: one per 64 positions, at most kBowMaxSegs
__host__ __device__ inline int bow_segments(int nb) {
    const int s = (nb + 63) / 64;
    return s < 1 ? 1 : (s > kBowMaxSegs ? kBowMaxSegs : s);
}

// Orientation bin of a match (ORBmatcher.cpp:187-195, :437-445).  The reference's factor is
// 1.0f / HISTO_LENGTH, so only bins 0..12 are reached; reproduced as written.
__host__ __device__ inline int bow_rot_bin(float angle_outer, float angle_inner) {
    const float factor = 1.0f / (float)kBowHistoLength;
    float rot = angle_outer - angle_inner;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == kBowHistoLength) bin = 0;
    return bin;
}

// diagnostic phase stamps of the last launch (see orbmatch.hip), up to cap values
hipError_t read_bow_stamps(uint64_t* out, int cap);

// all kernels on `st`; frame_overload selects SearchByBoW(KeyFrame, Frame) semantics
hipError_t launch_bow_search(bool frame_overload, int count, int max_outer_nodes, const BowPair* pairs, float nnratio,
                             int check_ori, hipStream_t st);

}  // namespace rsc
