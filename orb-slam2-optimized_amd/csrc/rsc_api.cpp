// rsc_api.cpp — C ABI (include/rsc.h) and HIP backend of the RANSAC engine.
//
// Data layout in HBM (per solver, resident for the solver's lifetime):
//   PnP : pts float4[N] = (X, Y, Z, sigma^2), uv float2[N], EPnP grow-only buffers
//         pws/us/als double[N][3|2|4], best/refined inlier bitsets uint64[ceil(N/64)].
//   Sim3: x1 float4[N] = (X1c, maxErr1), x2 float4[N] = (X2c, maxErr2), pim float4[N].
// Per context (reused across calls, grown on demand): the rand() jump table (2.1 MB), pose
// records float[H][12|24], counts int32[H], inlier bitsets uint64[H][W], launch descriptors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>
#include <memory>
#include "../../include/rsc.h"
#include "rsc_kernels.h"
#include "rsc_engine.h"
#include "rsc_poseopt.h"
#include "rsc_sim3opt.h"
#include "rsc_orbmatch.h"
#include "rsc_sim3match.h"
#include "rsc_kfdb.h"

using namespace rsc;

namespace {

thread_local std::string g_last_error;

#define RSC_HIP(call)                                                                         \
    do {                                                                                      \
        hipError_t _e = (call);                                                               \
        if (_e != hipSuccess) {                                                               \
            g_last_error = std::string(#call) + ": " + hipGetErrorString(_e);                  \
            return RSC_ERR_HIP;                                                               \
        }                                                                                     \
    } while (0)

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(n, (size_t)64);
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e != hipSuccess) {
            g_last_error = std::string("hipMalloc: ") + hipGetErrorString(e);
            return RSC_ERR_OOM;
        }
        cap = want;
        return 0;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

template <typename T>
struct PinBuf {
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(n, (size_t)64);
        hipError_t e = hipHostMalloc(&p, want * sizeof(T), hipHostMallocDefault);
        if (e != hipSuccess) {
            g_last_error = std::string("hipHostMalloc: ") + hipGetErrorString(e);
            return RSC_ERR_OOM;
        }
        cap = want;
        return 0;
    }
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// XCD-aware order of a workgroup table.  The dispatcher deals blocks round-robin over the 8 XCDs
// (blocks b and b + 8 share one L2; MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"), and
// every workgroup of a problem reads that problem's correspondences (scan: all of them; solve
// stages: random samples of them).  Dealt in problem order, each problem's workgroups spread over
// all 8 XCDs and every L2 fetches the problem's points from HBM again (8x the input bytes, measured
// with FETCH_SIZE); here the problems are binned onto the 8 residues of b (greedy by workgroup
// count) so a problem's workgroups share one L2.  Placement only: results do not depend on it.
template <class T, class Prob>
void xcd_order(std::vector<T>& wgs, Prob prob_of) {
    // O(n), no allocation once the scratch has grown (this runs inside every speculation round)
    constexpr int X = 8;
    const size_t n = wgs.size();
    if (n <= (size_t)X) return;
    // thread_local scratch, addressed once (each access to a thread_local of a shared library is a
    // __tls_get_addr call)
    thread_local std::vector<T> src_tl;
    thread_local std::vector<size_t> rb_tl;  // run r = entries [rb[r], rb[r + 1]) of one problem
    thread_local std::vector<int> runs_tl[X];
    std::vector<T>& src = src_tl;
    std::vector<size_t>& rb = rb_tl;
    std::vector<int>* runs = runs_tl;
    src.assign(wgs.begin(), wgs.end());
    rb.clear();
    for (size_t i = 0; i < n; ++i)
        if (i == 0 || prob_of(src[i]) != prob_of(src[i - 1])) rb.push_back(i);
    rb.push_back(n);
    size_t left[X] = {};
    for (int x = 0; x < X; ++x) runs[x].clear();
    for (size_t r = 0; r + 1 < rb.size(); ++r) {  // each problem to the least loaded residue
        int best = 0;
        for (int x = 1; x < X; ++x) if (left[x] < left[best]) best = x;
        runs[best].push_back((int)r);
        left[best] += rb[r + 1] - rb[r];
    }
    size_t cr[X] = {}, cp[X] = {};
    for (size_t b = 0; b < n; ++b) {
        int x = (int)(b % X);
        if (!left[x])  // this residue's problems are dealt: take from the one with most left
            for (int y = 0; y < X; ++y) if (left[y] > left[x]) x = y;
        const int r = runs[x][cr[x]];
        wgs[b] = src[rb[r] + cp[x]];
        if (++cp[x] == rb[r + 1] - rb[r]) { cp[x] = 0; ++cr[x]; }
        --left[x];
    }
}

// Hypotheses per scan workgroup: enough workgroups for ~8 waves per SIMD (256 CUs x 4 SIMDs,
// 4 waves per workgroup) without going below 8 hypotheses per point load.
// RSC_SCAN_WGS overrides the workgroup target (A/B of the chunk size).
int scan_chunk(int total_hyps) {
    static const int target = [] {
        const char* m = std::getenv("RSC_SCAN_WGS");
        return m ? std::max(1, std::atoi(m)) : 2048;
    }();
    int hc = 32;
    while (hc > 8 && (total_hyps + hc - 1) / hc < target) hc >>= 1;
    return hc;
}

int ppt_for(int n) {
    int need = (n + 255) / 256;
    int p = 1;
    while (p < need) p <<= 1;
    return p;
}

}  // namespace

constexpr int kSoCoopCUs = 256;  // OptimizeSim3's cooperative form: workgroups per launch at most (MI355X CUs)
constexpr int kFaultWord = 4;  // rsc_context::h_flag[4]: the split eigen stage's fault word

struct rsc_context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    RngTable table;
    DevBuf<uint32_t> d_table;
    // speculation work buffers
    DevBuf<float> d_poses;
    DevBuf<int32_t> d_counts;
    DevBuf<uint64_t> d_masks;
    DevBuf<int32_t> d_samples;
    DevBuf<double> d_stage;  // quad path: per-hypothesis stage records between the two solve kernels
    DevBuf<double> d_berr;   // pnp_betas_kernel hand-off: error per (approximation, record)
    DevBuf<float> d_bpose;   //   float pose per (approximation, record)
    DevBuf<unsigned> d_bctr; //   one arrival counter per 64-hypothesis group (zero between launches)
    DevBuf<float> d_gather;  // gathered pose records (+ their indices)
    DevBuf<double> d_mposes; // MLPnP hypothesis poses, double[12] per record
    DevBuf<char> d_desc;
    PinBuf<char> h_desc;
    PinBuf<int32_t> h_counts;
    PinBuf<int32_t> h_qual;  // PnP rounds: 1 when a problem has a hypothesis reaching min_inliers
    // PnP work tables (eigen / betas / scan workgroups) on the device, uploaded when the round's shape
    // (pnp_tab_key) changes instead of with every round's descriptors
    DevBuf<char> d_pnp_tab;
    std::vector<int> pnp_tab_key;
    size_t pnp_tab_quad[3] = {0, 0, 0}, pnp_tab_solve[3] = {0, 0, 0}, pnp_tab_scan = 0;
    PinBuf<float> h_small;
    PinBuf<float> h_pick;  // Sim3 pick records of the last round, [solver][16]
    DevBuf<char> d_refine;
    DevBuf<RefineSelOut> d_selout;  // pnp_select_refine_kernel results of the last fused round
    PinBuf<RefineSelOut> h_selout;
    // PoseOptimization: packed inputs (problems | xw | uv), edge error scratch, results (outliers | poses)
    DevBuf<char> d_po_in;
    // OptimizeSim3: packed inputs (problems | e12 | e21 | uv), edge errors, results (out | keep)
    DevBuf<char> d_so_in;
    PinBuf<char> h_so_in;
    DevBuf<char> d_so_res;
    PinBuf<char> h_so_res;
    DevBuf<char> d_po_res;
    PinBuf<char> h_po_in;
    PinBuf<char> h_po_res;
    // SearchBySim3: packed KeyFrames + pair table + scratch + outputs (device, pinned mirror)
    DevBuf<char> d_s3m;
    PinBuf<char> h_s3m;
    // SearchByBoW: pair table + output vectors + match counts (device, pinned mirror)
    DevBuf<char> d_bow;
    PinBuf<char> h_bow;
    int mask_words = 0;  // per hypothesis, last speculation
    bool keep_samples = true;
    // timing
    bool timing = false;
    hipEvent_t ev[12] = {};  // [0..5] phase marks, [6+2g], [7+2g] eigen-stage kernel of sample-size group g
    double last_ms[6] = {0, 0, 0, 0, 0, 0};
    // host-side phase clock of the last PnP iterate_many (diagnostic): microseconds from entry to
    // [0] speculation inputs built, [1] kernels enqueued, [2] counts back (sync), [3] return
    double host_us[4] = {0, 0, 0, 0};
    bool direct_counts = true;  // env RSC_DIRECT_COUNTS=0 restores the HBM buffer + D2H copy
    bool fused_refine = true;   // env RSC_FUSED_REFINE=0: the replay's Refine always as its own launch
    bool dma_upload = false;    // env RSC_DMA_UPLOAD=1: descriptors by hipMemcpyAsync instead of the copy kernel
    // eigen stage in the rows form when it has <= W workgroups (small, latency-bound launches such as
    // one relocalization event: 125 -> 99 us, profiles/r05/bench_latency_forms_ab_r5b.json); env
    // RSC_EIG_ROWS=W or rsc_context_set_eig_rows overrides (0: lane pairs always)
    int eig_rows_max_wgs = kEigRowsDefaultWgs;
    // hypotheses per betas wave for launches small enough for the rows-form eigen stage (a wave runs
    // the union of its hypotheses' data-dependent chains; env RSC_BETAS_HB)
    int betas_small_hb = kBetasHyps;
    // eigen stages beyond the rows form's range: split form (chase and Q rotations on two waves,
    // pnp_eig_split_kernel; config-2 eigen stage 119 -> 114 us, profiles/r05/split_ab_r5q.jsonl) or
    // the pair form (env RSC_EIG_SPLIT=0)
    bool eig_split = true;
    // host wait for a speculation round's results: spin on a completion flag in pinned host memory
    // (written by signal_kernel after the round) instead of hipStreamSynchronize's wake-up; env
    // RSC_SPIN_WAIT=0/1 (stream_wait)
    bool spin_wait = false;
    // OptimizeSim3's helper workgroups per pair (the cooperative form; -1: as many as fit one per CU,
    // at most 7; 0: one workgroup per pair)
    int so_helpers = -1;
    DevBuf<char> d_so_coop;  // the cooperative form's hand-off: polled words | publications | lists | chunks
    uint32_t* h_flag = nullptr;  // [0] stream_wait's sequence flag, [kFaultWord] the eigen stage's fault word
    uint32_t flag_seq = 0;
    std::chrono::steady_clock::time_point t_entry;
};

// The process-global glibc rand() stream the reference draws every sample from (Random.cpp:47-50,
// Q3): one position shared by all solvers bound to it, advanced by each iterate() call in call order.
struct rsc_stream {
    rsc_context* ctx = nullptr;
    RngStream st;
    int64_t position = 0;  // draws consumed since srand(seed)
};

struct rsc_pnp {
    rsc_context* ctx = nullptr;
    PnPState st;
    float4* d_pts = nullptr;
    float2* d_uv = nullptr;
    double* d_pws = nullptr;
    double* d_us = nullptr;
    double* d_als = nullptr;
    uint64_t* d_best = nullptr;
    uint64_t* d_refined = nullptr;
    int words = 0;
    int last_kind = 0;  // vbInliers of the last iterate(): 0 empty, 1 refined mask, 2 best mask
    // position in the last speculation of its context
    int spec_out0 = -1, spec_H = 0;
    rsc_stream* stream = nullptr;  // shared rand() stream (rsc_pnp_bind_stream) or null: own stream
    RngStream own_rng;             // the own stream, parked while bound (st.rng follows the shared one)
    std::vector<float> h_p2d, h_p3d;  // host copies (the gated events' PoseOptimization problems)
    ~rsc_pnp() {
        for (void* p : {(void*)d_pts, (void*)d_uv, (void*)d_pws, (void*)d_us, (void*)d_als, (void*)d_best,
                        (void*)d_refined})
            if (p) (void)hipFree(p);
    }
};

struct rsc_sim3 {
    rsc_context* ctx = nullptr;
    Sim3State st;
    // prepared arrays (host copies for rsc_sim3_prepared)
    std::vector<float> X1c, X2c, P1, P2;
    std::vector<uint64_t> e1, e2;
    float K1[4], K2[4];
    float4* d_x1 = nullptr;
    float4* d_x2 = nullptr;
    float4* d_pim = nullptr;
    int spec_out0 = -1, spec_H = 0;
    rsc_stream* stream = nullptr;
    RngStream own_rng;
    ~rsc_sim3() {
        for (void* p : {(void*)d_x1, (void*)d_x2, (void*)d_pim})
            if (p) (void)hipFree(p);
    }
};

struct rsc_mlpnp {
    rsc_context* ctx = nullptr;
    MLState st;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    float4* d_pts = nullptr;
    float2* d_uv = nullptr;
    float2* d_brg = nullptr;
    double* d_cov = nullptr;  // [N][9] when covariances were set
    bool use_cov = false;
    uint64_t* d_best = nullptr;
    int words = 0;
    int spec_out0 = -1, spec_H = 0;
    rsc_stream* stream = nullptr;
    RngStream own_rng;
    ~rsc_mlpnp() {
        for (void* p : {(void*)d_pts, (void*)d_uv, (void*)d_brg, (void*)d_cov, (void*)d_best})
            if (p) (void)hipFree(p);
    }
};

namespace {

// ------------------------------------------------------------------------------------------------
// Launch-descriptor packing: one pinned blob -> one H2D copy per launch round.
// ------------------------------------------------------------------------------------------------
// Descriptor staging of one round.  The byte vector is a per-thread scratch that keeps its capacity
// across rounds (one Blob is alive at a time per thread), so a round allocates nothing here.
struct Blob {
    std::vector<char>& bytes;
    Blob() : bytes(scratch()) {
        // one Blob per thread at a time: a nested one would truncate the open one's descriptors
        if (in_use()) {
            std::fprintf(stderr, "rsc: nested launch-descriptor Blob on one thread\n");
            std::abort();
        }
        in_use() = true;
        bytes.clear();
    }
    ~Blob() { in_use() = false; }
    Blob(const Blob&) = delete;
    Blob& operator=(const Blob&) = delete;
    static std::vector<char>& scratch() {
        thread_local std::vector<char> v;
        return v;
    }
    static bool& in_use() {
        thread_local bool f = false;
        return f;
    }
    size_t add(const void* p, size_t n) {
        size_t off = (bytes.size() + 15) & ~(size_t)15;
        bytes.resize(off + n);
        std::memcpy(bytes.data() + off, p, n);
        return off;
    }
};

int upload_blob(rsc_context* C, const Blob& b) {
    const size_t n16 = (b.bytes.size() + 15) / 16;
    if (int e = C->h_desc.ensure(n16 * 16)) return e;
    if (int e = C->d_desc.ensure(n16 * 16)) return e;
    // the previous round's upload must be finished before the pinned staging is overwritten
    RSC_HIP(hipStreamSynchronize(C->stream));
    std::memcpy(C->h_desc.p, b.bytes.data(), b.bytes.size());
    // a copy kernel on the context stream, not hipMemcpyAsync: the DMA engine's start-up and its
    // completion hand-off to the first kernel cost ~15 us per round (rocprofv3 copy + kernel trace)
    if (C->dma_upload)
        RSC_HIP(hipMemcpyAsync(C->d_desc.p, C->h_desc.p, b.bytes.size(), hipMemcpyHostToDevice, C->stream));
    else
        RSC_HIP(launch_upload16(C->h_desc.p, C->d_desc.p, n16, C->stream));
    return 0;
}

// Inlier counts of a speculation round: written by the scan kernel straight into pinned host
// memory (one fewer copy and no blit launch before the host replay), or into HBM + a D2H copy.
int counts_target(rsc_context* C, int total, int32_t** dst) {
    if (int e = C->h_counts.ensure((size_t)total)) return e;
    if (C->direct_counts) {
        *dst = C->h_counts.p;
        return 0;
    }
    if (int e = C->d_counts.ensure((size_t)total)) return e;
    *dst = C->d_counts.p;
    return 0;
}

// Wait until everything enqueued on the context stream has finished.  With spin_wait a one-lane
// kernel stores a sequence number into pinned host memory behind the round and the host polls it
// (results written to pinned memory by the round's kernels are visible once the flag is: stream
// order + the flag's system-scope release); after 20 ms of polling it falls back to
// hipStreamSynchronize, which also reports a failed kernel.
int stream_wait(rsc_context* C) {
    if (!C->spin_wait || !C->h_flag || C->timing) {  // the timing pass reads events: a full sync
        RSC_HIP(hipStreamSynchronize(C->stream));
        return 0;
    }
    const uint32_t want = ++C->flag_seq;
    RSC_HIP(launch_signal(C->h_flag, want, C->stream));
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(C->h_flag, __ATOMIC_ACQUIRE) == want) return 0;
        __builtin_ia32_pause();
        if ((it & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    RSC_HIP(hipStreamSynchronize(C->stream));
    return 0;
}

// The eigen stage's fault word (h_flag[kFaultWord], set by split_wait when a hand-off gives up):
// read after the round's wait, cleared, and returned as an error instead of the round's results.
int take_fault(rsc_context* C) {
    if (__atomic_load_n(C->h_flag + kFaultWord, __ATOMIC_ACQUIRE) == 0) return 0;
    __atomic_store_n(C->h_flag + kFaultWord, 0u, __ATOMIC_RELEASE);
    g_last_error = "a device hand-off wait timed out (split_wait: eigen stage chase / row wave, or a streamed "
                   "PoseOptimization pass, or an OptimizeSim3 chunk of the cooperative form); results discarded";
    return RSC_ERR_INTERNAL;
}

void host_mark(rsc_context* C, int k) {
    C->host_us[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - C->t_entry).count();
}

void timing_begin(rsc_context* C, int slot) {
    if (C->timing) (void)hipEventRecord(C->ev[slot], C->stream);
}

// ------------------------------------------------------------------------------------------------
// PnP backend
// ------------------------------------------------------------------------------------------------
struct HipPnPBackend : PnPBackend {
    rsc_context* C;
    std::vector<rsc_pnp*> solvers;  // index = state slot in the current call
    int fused_count = 0;  // > 0: the last speculation ran pnp_select_refine_kernel over this many slots
    explicit HipPnPBackend(rsc_context* c) : C(c) {}
    rsc_pnp* of(PnPState* s) {
        for (auto* p : solvers)
            if (&p->st == s) return p;
        return nullptr;
    }
    DevPnP dev_of(rsc_pnp* p) {
        DevPnP d;
        d.pts = p->d_pts;
        d.uv = p->d_uv;
        d.n = p->st.N;
        d.fx = p->st.fx; d.fy = p->st.fy; d.cx = p->st.cx; d.cy = p->st.cy;
        d.th2 = p->st.th2;
        d.rows = p->st.max_rows;
        d.pws = p->d_pws; d.us = p->d_us; d.als = p->d_als;
        return d;
    }

    int speculate(PnPState* const* S, int count, const int* H, std::vector<std::vector<int32_t>>& counts) override {
        // group by min_set (template parameter of the solve kernel)
        int total = 0, maxN = 1;
        // per-thread scratch that keeps its capacity across rounds (no allocation per round)
        thread_local std::vector<DevPnP> probs_tl;
        thread_local std::vector<LaunchProb> lps_tl;
        std::vector<DevPnP>& probs = probs_tl;
        std::vector<LaunchProb>& lps = lps_tl;
        probs.resize(count);
        lps.resize(count);
        for (int i = 0; i < count; ++i) {
            rsc_pnp* p = of(S[i]);
            if (!p) return RSC_ERR_ARG;
            if (S[i]->mRansacMinSet < 4 || S[i]->mRansacMinSet > 6) {
                g_last_error = "min_set outside the supported range [4,6]";
                return RSC_ERR_UNSUPPORTED;
            }
            S[i]->rng.ensure(C->table, H[i] * S[i]->mRansacMinSet);
            probs[i] = dev_of(p);
            LaunchProb& lp = lps[i];
            lp.prob = i;
            lp.H = H[i];
            lp.out0 = total;
            lp.g0 = S[i]->rng.g;
            std::memcpy(lp.window, S[i]->rng.window, sizeof(lp.window));
            lp.min_inliers = S[i]->mRansacMinInliers;  // only such hypotheses' masks are ever read
            p->spec_out0 = total;
            p->spec_H = H[i];
            total += H[i];
            maxN = std::max(maxN, S[i]->N);
        }
        const int ppt = ppt_for(maxN);
        if (ppt > 32) {
            g_last_error = "more than 8192 correspondences per problem";
            return RSC_ERR_UNSUPPORTED;
        }
        const int mw = ppt * 4;
        C->mask_words = mw;
        // the replay's first Refine of every solver runs on the device with the round (small rounds)
        fused_count = 0;
        const bool fused = C->fused_refine && total <= kFusedRefineMaxHyps;
        thread_local std::vector<RefineSel> sels_tl;
        std::vector<RefineSel>& sels = sels_tl;
        sels.resize(fused ? count : 0);
        for (int i = 0; fused && i < count; ++i) {
            rsc_pnp* p = of(S[i]);
            RefineSel& r = sels[i];
            r.prob = i;
            r.out0 = lps[i].out0;
            r.H = H[i];
            r.min_inliers = S[i]->mRansacMinInliers;
            r.best0 = S[i]->mnBestInliers;
            r.rows0 = S[i]->max_rows;
            r.best = p->d_best;
            r.refined = p->d_refined;
            r.words = p->words;
        }
        // work tables
        thread_local std::vector<int2> solve_wgs_tl[3], quad_wgs_tl[3];
        thread_local std::vector<int4> scan_wgs_tl;
        std::vector<int2>* solve_wgs = solve_wgs_tl;
        std::vector<int2>* quad_wgs = quad_wgs_tl;
        std::vector<int4>& scan_wgs = scan_wgs_tl;
        const int HC = scan_chunk(total);  // hypotheses per scan workgroup
        const int hb = (total <= kEigHyps * C->eig_rows_max_wgs) ? C->betas_small_hb : kBetasHyps;

        // The tables depend only on the round's shape (count, sample size and H per problem, HC):
        // a round with the shape of the previous one on this thread reuses them (building and
        // XCD-ordering ~3.7k entries costs ~10 us of host time per config-2 round).
        thread_local std::vector<int> shape_tl;
        std::vector<int>& shape = shape_tl;
        thread_local std::vector<int> key_tl;
        std::vector<int>& key = key_tl;
        key.clear();
        key.push_back(count);
        key.push_back(HC);
        key.push_back(hb);
        for (int i = 0; i < count; ++i) {
            key.push_back(S[i]->mRansacMinSet);
            key.push_back(H[i]);
        }
        if (key != shape) {
            for (int g = 0; g < 3; ++g) { solve_wgs[g].clear(); quad_wgs[g].clear(); }
            scan_wgs.clear();
            for (int i = 0; i < count; ++i) {
                const int g = S[i]->mRansacMinSet - 4;
                for (int h0 = 0; h0 < H[i]; h0 += hb) solve_wgs[g].push_back(make_int2(i, h0));
                for (int h0 = 0; h0 < H[i]; h0 += kEigHyps) quad_wgs[g].push_back(make_int2(i, h0));
                for (int h0 = 0; h0 < H[i]; h0 += HC)
                    scan_wgs.push_back(make_int4(i, h0, std::min(HC, H[i] - h0), 0));
            }
            for (int g = 0; g < 3; ++g) {
                xcd_order(solve_wgs[g], [](const int2& w) { return w.x; });
                xcd_order(quad_wgs[g], [](const int2& w) { return w.x; });
            }
            xcd_order(scan_wgs, [](const int4& w) { return w.x; });
            shape.assign(key.begin(), key.end());
        }
        // The work tables (≈50 KB for config 2) live in the context's d_pnp_tab while the round's shape
        // repeats; only the per-round descriptors (problems, launch records, selections) travel in the
        // blob (the host copies and the upload kernel's PCIe reads shrink accordingly).
        if (C->pnp_tab_key != key || !C->d_pnp_tab.p) {
            std::vector<char> tab;
            auto put = [&](const void* p, size_t n) {
                const size_t o = tab.size();
                tab.resize(o + ((n + 15) & ~(size_t)15));
                if (n) std::memcpy(tab.data() + o, p, n);
                return o;
            };
            for (int g = 0; g < 3; ++g) C->pnp_tab_solve[g] = put(solve_wgs[g].data(), solve_wgs[g].size() * sizeof(int2));
            for (int g = 0; g < 3; ++g) C->pnp_tab_quad[g] = put(quad_wgs[g].data(), quad_wgs[g].size() * sizeof(int2));
            C->pnp_tab_scan = put(scan_wgs.data(), scan_wgs.size() * sizeof(int4));
            C->pnp_tab_key.clear();  // invalid until the copy below has landed
            if (int e = C->d_pnp_tab.ensure(std::max(tab.size(), (size_t)16))) return e;
            // the previous round (the tables' last reader) has finished: every round ends synchronized
            RSC_HIP(hipMemcpyAsync(C->d_pnp_tab.p, tab.data(), tab.size(), hipMemcpyHostToDevice, C->stream));
            RSC_HIP(hipStreamSynchronize(C->stream));
            C->pnp_tab_key = key;
        }
        Blob b;
        const size_t o_probs = b.add(probs.data(), probs.size() * sizeof(DevPnP));
        const size_t o_lps = b.add(lps.data(), lps.size() * sizeof(LaunchProb));
        const size_t o_sel = fused ? b.add(sels.data(), sels.size() * sizeof(RefineSel)) : 0;
        if (int e = upload_blob(C, b)) return e;
        const char* tab = C->d_pnp_tab.p;
        if (int e = C->d_poses.ensure((size_t)total * 12)) return e;
        int32_t* cnt_dst = nullptr;
        if (int e = counts_target(C, total, &cnt_dst)) return e;
        if (int e = C->h_qual.ensure((size_t)count)) return e;
        std::memset(C->h_qual.p, 0, (size_t)count * sizeof(int32_t));  // the previous round has finished
        int32_t* cnt_dev = nullptr;  // HBM copy of the counts for the device-side selection
        if (fused) {
            if (C->direct_counts) {
                if (int e = C->d_counts.ensure((size_t)total)) return e;
                cnt_dev = C->d_counts.p;
            }
            if (int e = C->d_selout.ensure((size_t)count)) return e;
            if (int e = C->h_selout.ensure((size_t)count)) return e;
        }
        if (int e = C->d_masks.ensure((size_t)total * mw)) return e;
        if (int e = C->d_samples.ensure((size_t)total * 8)) return e;
        if (int e = C->d_stage.ensure((size_t)total * kStageDoubles)) return e;
        if (int e = C->d_berr.ensure((size_t)total * 3)) return e;
        if (int e = C->d_bpose.ensure((size_t)total * 36)) return e;
        size_t groups = 0;
        for (int g = 0; g < 3; ++g) groups = std::max(groups, solve_wgs[g].size());
        const size_t had = C->d_bctr.cap;
        if (int e = C->d_bctr.ensure(groups)) return e;
        if (C->d_bctr.cap != had) RSC_HIP(hipMemsetAsync(C->d_bctr.p, 0, C->d_bctr.cap * sizeof(unsigned), C->stream));
        const BetasScratch bs{C->d_berr.p, C->d_bpose.p, C->d_bctr.p, (size_t)total};
        const char* base = C->d_desc.p;
        const DevPnP* dprobs = reinterpret_cast<const DevPnP*>(base + o_probs);
        const LaunchProb* dlps = reinterpret_cast<const LaunchProb*>(base + o_lps);
        host_mark(C, 0);
        timing_begin(C, 0);
        bool first_group = true;
        for (int g = 0; g < 3; ++g) {
            if (solve_wgs[g].empty()) continue;
            // the first group's eigen stage starts at ev[0]: no extra event in the queue
            hipEvent_t eb = (C->timing && !first_group) ? C->ev[6 + 2 * g] : nullptr;
            RSC_HIP(launch_pnp_solve_split(4 + g, (int)quad_wgs[g].size(),
                                          reinterpret_cast<const int2*>(tab + C->pnp_tab_quad[g]), (int)solve_wgs[g].size(),
                                          reinterpret_cast<const int2*>(tab + C->pnp_tab_solve[g]), dprobs, dlps,
                                          C->d_table.p, C->d_stage.p, C->d_poses.p, C->d_samples.p, bs, C->stream,
                                          eb, C->timing ? C->ev[7 + 2 * g] : nullptr,
                                          (int)quad_wgs[g].size() <= C->eig_rows_max_wgs, C->eig_split,
                                          C->h_flag + kFaultWord, hb));
            first_group = false;
        }
        timing_begin(C, 1);
        RSC_HIP(launch_pnp_scan(ppt, (int)scan_wgs.size(), dprobs, dlps, reinterpret_cast<const int4*>(tab + C->pnp_tab_scan),
                                C->d_poses.p, cnt_dst, cnt_dev, C->d_masks.p, mw, C->h_qual.p, C->stream));
        timing_begin(C, 2);
        if (fused) {
            timing_begin(C, 3);
            RSC_HIP(launch_pnp_select_refine(count, dprobs, reinterpret_cast<const RefineSel*>(base + o_sel),
                                             cnt_dev ? cnt_dev : cnt_dst, C->d_masks.p, mw, C->d_poses.p,
                                             C->d_selout.p, C->h_flag + kFaultWord, C->stream));
            timing_begin(C, 4);
            RSC_HIP(hipMemcpyAsync(C->h_selout.p, C->d_selout.p, sizeof(RefineSelOut) * count, hipMemcpyDeviceToHost,
                                   C->stream));
        }
        if (!C->direct_counts)
            RSC_HIP(hipMemcpyAsync(C->h_counts.p, C->d_counts.p, (size_t)total * 4, hipMemcpyDeviceToHost, C->stream));
        host_mark(C, 1);
        if (int e = stream_wait(C)) return e;
        host_mark(C, 2);
        if (int e = take_fault(C)) return e;
        if (C->timing) {
            float a = 0, s = 0;
            (void)hipEventElapsedTime(&a, C->ev[0], C->ev[1]);
            (void)hipEventElapsedTime(&s, C->ev[1], C->ev[2]);
            C->last_ms[0] += a;
            C->last_ms[1] += s;
            C->last_ms[3] += 1;
            C->last_ms[4] += total;
            bool first = true;
            for (int g = 0; g < 3; ++g) {
                if (solve_wgs[g].empty()) continue;
                float e = 0;
                (void)hipEventElapsedTime(&e, first ? C->ev[0] : C->ev[6 + 2 * g], C->ev[7 + 2 * g]);
                C->last_ms[5] += e;
                first = false;
            }
            if (fused) {
                float r = 0;
                (void)hipEventElapsedTime(&r, C->ev[3], C->ev[4]);
                C->last_ms[2] += r;
            }
        }
        // a problem none of whose hypotheses reaches min_inliers hands back no counts: the replay only
        // advances its counters (the GPU-written counts are not read back through the host caches)
        counts.resize(count);  // keeps the inner vectors' capacity
        for (int i = 0; i < count; ++i) {
            if (C->h_qual.p[i])
                counts[i].assign(C->h_counts.p + lps[i].out0, C->h_counts.p + lps[i].out0 + H[i]);
            else
                counts[i].clear();
        }
        if (fused) fused_count = count;
        return 0;
    }

    int refine(PnPState* const* S, int count, const int* spec_j, const int* pause_k, const int* adopt_k,
               const int* rows_after, int* rcount, float (*rpose)[12]) override {
        if (fused_count > 0) {
            // the device ran exactly these Refines with the round (pnp_select_refine_kernel applies the
            // replay's rules to the same counts); anything else is an engine bug, reported loudly
            const int nslots = fused_count;
            fused_count = 0;
            // every slot: the device refined exactly the listed slots (o.k >= 0) and no other one
            // (an unlisted device Refine would have overwritten that solver's best / refined masks)
            thread_local std::vector<int> listed_tl;
            std::vector<int>& listed = listed_tl;
            listed.assign((size_t)nslots, -1);
            for (int i = 0; i < count; ++i) {
                if (spec_j[i] < 0 || spec_j[i] >= nslots || listed[spec_j[i]] >= 0) {
                    g_last_error = "device-side Refine selection disagrees with the host replay";
                    return RSC_ERR_INTERNAL;
                }
                listed[spec_j[i]] = i;
            }
            for (int j = 0; j < nslots; ++j) {
                const RefineSelOut& o = C->h_selout.p[j];
                const int i = listed[j];
                const bool agree = i < 0 ? o.k < 0
                                         : o.k == pause_k[i] && (o.adopt != 0) == (adopt_k[i] >= 0) &&
                                               o.rows_after == rows_after[i];
                if (!agree) {
                    g_last_error = "device-side Refine selection disagrees with the host replay";
                    return RSC_ERR_INTERNAL;
                }
            }
            for (int i = 0; i < count; ++i) {
                const RefineSelOut& o = C->h_selout.p[spec_j[i]];
                rcount[i] = o.count;
                std::memcpy(rpose[i], o.pose, 48);
                if (adopt_k[i] >= 0) pose12_to_T(o.best_pose, S[i]->mBestTcw);
            }
            return 0;
        }
        if (count == 0) return 0;
        std::vector<DevPnP> probs(count);
        std::vector<RefineJob> jobs(count);
        // out: refined poses [count][12] | counts [count] | adopted best poses [count][12]
        if (int e = C->d_refine.ensure((size_t)count * 100)) return e;
        float* d_out_pose = reinterpret_cast<float*>(C->d_refine.p);
        int32_t* d_out_cnt = reinterpret_cast<int32_t*>(C->d_refine.p + (size_t)count * 48);
        float* d_out_best = reinterpret_cast<float*>(C->d_refine.p + (size_t)count * 52);
        for (int i = 0; i < count; ++i) {
            rsc_pnp* p = of(S[i]);
            probs[i] = dev_of(p);
            jobs[i].prob = i;
            jobs[i].rows_after = rows_after[i];
            (void)spec_j;
            if (adopt_k[i] >= 0) {
                const size_t rec = (size_t)(p->spec_out0 + adopt_k[i]);
                jobs[i].best_mask = C->d_masks.p + rec * C->mask_words;
                jobs[i].adopt_mask = p->d_best;
                jobs[i].adopt_pose = C->d_poses.p + rec * 12;
            } else {
                jobs[i].best_mask = p->d_best;
                jobs[i].adopt_mask = nullptr;
                jobs[i].adopt_pose = nullptr;
            }
            jobs[i].out_best_pose = d_out_best + 12 * i;
            jobs[i].out_pose = d_out_pose + 12 * i;
            jobs[i].out_count = d_out_cnt + i;
            jobs[i].out_mask = p->d_refined;
            jobs[i].out_words = p->words;
        }
        Blob b;
        const size_t o_probs = b.add(probs.data(), probs.size() * sizeof(DevPnP));
        const size_t o_jobs = b.add(jobs.data(), jobs.size() * sizeof(RefineJob));
        if (int e = upload_blob(C, b)) return e;
        timing_begin(C, 3);
        RSC_HIP(launch_pnp_refine(count, reinterpret_cast<const DevPnP*>(C->d_desc.p + o_probs),
                                  reinterpret_cast<const RefineJob*>(C->d_desc.p + o_jobs), C->h_flag + kFaultWord,
                                  C->stream));
        timing_begin(C, 4);
        if (int e = C->h_small.ensure((size_t)count * 25)) return e;
        RSC_HIP(hipMemcpyAsync(C->h_small.p, C->d_refine.p, (size_t)count * 100, hipMemcpyDeviceToHost, C->stream));
        RSC_HIP(hipStreamSynchronize(C->stream));
        if (int e = take_fault(C)) return e;
        if (C->timing) {
            float r = 0;
            (void)hipEventElapsedTime(&r, C->ev[3], C->ev[4]);
            C->last_ms[2] += r;
        }
        const int32_t* hc = reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(C->h_small.p) + (size_t)count * 48);
        for (int i = 0; i < count; ++i) {
            rcount[i] = hc[i];
            std::memcpy(rpose[i], C->h_small.p + 12 * i, 48);
            if (adopt_k[i] >= 0) pose12_to_T(C->h_small.p + 13 * count + 12 * i, S[i]->mBestTcw);
        }
        return 0;
    }

    int fetch_mask(PnPState* const* S, int count, const int* kind, uint8_t* const* out) override {
        std::vector<std::vector<uint64_t>> words(count);
        for (int i = 0; i < count; ++i) {
            rsc_pnp* p = of(S[i]);
            words[i].resize(p->words);
            RSC_HIP(hipMemcpyAsync(words[i].data(), kind[i] == 1 ? p->d_refined : p->d_best, (size_t)p->words * 8,
                                   hipMemcpyDeviceToHost, C->stream));
        }
        RSC_HIP(hipStreamSynchronize(C->stream));
        for (int i = 0; i < count; ++i) {
            const PnPState& s = *S[i];
            std::memset(out[i], 0, s.N_points);
            for (int j = 0; j < s.N; ++j)
                if ((words[i][j >> 6] >> (j & 63)) & 1ull) out[i][s.kp_index[j]] = 1;
        }
        return 0;
    }
};

// ------------------------------------------------------------------------------------------------
// Sim3 backend
// ------------------------------------------------------------------------------------------------
struct HipSim3Backend : Sim3Backend {
    rsc_context* C;
    std::vector<rsc_sim3*> solvers;  // slot j of the last speculation
    bool pick_valid = false;  // C->h_pick holds this round's sim3_pick_kernel records
    explicit HipSim3Backend(rsc_context* c) : C(c) {}
    rsc_sim3* of(Sim3State* s, const std::vector<rsc_sim3*>& all) {
        for (auto* p : all)
            if (&p->st == s) return p;
        return nullptr;
    }
    std::vector<rsc_sim3*> all;

    int speculate(Sim3State* const* S, int count, const int* H, std::vector<std::vector<int32_t>>& counts) override {
        pick_valid = false;  // set again only once this round's pick kernel is enqueued
        int total = 0, maxN = 1;
        // per-thread scratch that keeps its capacity across rounds (no allocation per round)
        thread_local std::vector<DevSim3> probs_tl;
        thread_local std::vector<LaunchProb> lps_tl;
        std::vector<DevSim3>& probs = probs_tl;
        std::vector<LaunchProb>& lps = lps_tl;
        probs.resize(count);
        lps.resize(count);
        solvers.assign(count, nullptr);
        for (int i = 0; i < count; ++i) {
            rsc_sim3* p = of(S[i], all);
            if (!p) return RSC_ERR_ARG;
            solvers[i] = p;
            S[i]->rng.ensure(C->table, H[i] * 3);
            DevSim3& d = probs[i];
            d.x1 = p->d_x1; d.x2 = p->d_x2; d.pim = p->d_pim; d.n = S[i]->N;
            std::memcpy(d.K1, p->K1, sizeof(d.K1));
            std::memcpy(d.K2, p->K2, sizeof(d.K2));
            LaunchProb& lp = lps[i];
            lp.prob = i; lp.H = H[i]; lp.out0 = total; lp.g0 = S[i]->rng.g;
            lp.min_inliers = S[i]->mRansacMinInliers;  // the pick kernel's return rule
            lp.best0 = S[i]->mnBestInliers;
            std::memcpy(lp.window, S[i]->rng.window, sizeof(lp.window));
            p->spec_out0 = total;
            p->spec_H = H[i];
            total += H[i];
            maxN = std::max(maxN, S[i]->N);
        }
        const int ppt = ppt_for(maxN);
        if (ppt > 32) {
            g_last_error = "more than 8192 correspondences per problem";
            return RSC_ERR_UNSUPPORTED;
        }
        const int mw = ppt * 4;
        C->mask_words = mw;
        thread_local std::vector<int2> solve_wgs_tl;
        thread_local std::vector<int4> scan_wgs_tl;
        thread_local std::vector<int> shape_tl, key_tl;
        std::vector<int2>& solve_wgs = solve_wgs_tl;
        std::vector<int4>& scan_wgs = scan_wgs_tl;
        std::vector<int>& shape = shape_tl;
        std::vector<int>& key = key_tl;
        const int HC = 32;
        key.assign(H, H + count);  // the tables depend on the per-solver H only (as the PnP tables)
        if (key != shape) {
            solve_wgs.clear();
            scan_wgs.clear();
            for (int i = 0; i < count; ++i) {
                for (int h0 = 0; h0 < H[i]; h0 += 64) solve_wgs.push_back(make_int2(i, h0));
                for (int h0 = 0; h0 < H[i]; h0 += HC) scan_wgs.push_back(make_int4(i, h0, std::min(HC, H[i] - h0), 0));
            }
            xcd_order(solve_wgs, [](const int2& w) { return w.x; });
            xcd_order(scan_wgs, [](const int4& w) { return w.x; });
            shape.assign(key.begin(), key.end());
        }
        Blob b;
        const size_t o_probs = b.add(probs.data(), probs.size() * sizeof(DevSim3));
        const size_t o_lps = b.add(lps.data(), lps.size() * sizeof(LaunchProb));
        const size_t o_solve = b.add(solve_wgs.data(), solve_wgs.size() * sizeof(int2));
        const size_t o_scan = b.add(scan_wgs.data(), scan_wgs.size() * sizeof(int4));
        if (int e = upload_blob(C, b)) return e;
        if (int e = C->d_poses.ensure((size_t)total * 24)) return e;
        // the kept pose comes back with the counts (sim3_pick_kernel) when every solver's round
        // fits the pick kernel's LDS
        bool use_pick = true;
        for (int i = 0; i < count; ++i) use_pick = use_pick && H[i] <= kPickMaxH;
        int32_t* cnt_dst = nullptr;
        if (int e = counts_target(C, total, &cnt_dst)) return e;
        if (use_pick) {
            if (int e = C->d_counts.ensure((size_t)total)) return e;
            if (int e = C->h_pick.ensure((size_t)count * 16)) return e;
        }
        if (int e = C->d_masks.ensure((size_t)total * mw)) return e;
        if (C->keep_samples)
            if (int e = C->d_samples.ensure((size_t)total * 8)) return e;
        const char* base = C->d_desc.p;
        const DevSim3* dprobs = reinterpret_cast<const DevSim3*>(base + o_probs);
        const LaunchProb* dlps = reinterpret_cast<const LaunchProb*>(base + o_lps);
        timing_begin(C, 0);
        RSC_HIP(launch_sim3_solve((int)solve_wgs.size(), dprobs, dlps, reinterpret_cast<const int2*>(base + o_solve),
                                  C->d_table.p, C->d_poses.p, C->keep_samples ? C->d_samples.p : nullptr, C->stream));
        timing_begin(C, 1);
        int32_t* cnt_dev = (use_pick && C->direct_counts) ? C->d_counts.p : nullptr;  // else cnt_dst is HBM
        RSC_HIP(launch_sim3_scan(ppt, (int)scan_wgs.size(), dprobs, dlps, reinterpret_cast<const int4*>(base + o_scan),
                                 C->d_poses.p, cnt_dst, cnt_dev, C->d_masks.p, mw, C->stream));
        timing_begin(C, 2);
        if (use_pick) {
            RSC_HIP(launch_sim3_pick(count, dlps, C->d_counts.p, C->d_poses.p, C->h_pick.p, C->stream));
            pick_valid = true;
        }
        if (!C->direct_counts)
            RSC_HIP(hipMemcpyAsync(C->h_counts.p, C->d_counts.p, (size_t)total * 4, hipMemcpyDeviceToHost, C->stream));
        if (int e = stream_wait(C)) return e;
        if (C->timing) {
            float a = 0, s = 0;
            (void)hipEventElapsedTime(&a, C->ev[0], C->ev[1]);
            (void)hipEventElapsedTime(&s, C->ev[1], C->ev[2]);
            C->last_ms[0] += a;
            C->last_ms[1] += s;
            C->last_ms[3] += 1;
            C->last_ms[4] += total;
        }
        counts.resize(count);  // keeps the inner vectors' capacity
        for (int i = 0; i < count; ++i)
            counts[i].assign(C->h_counts.p + lps[i].out0, C->h_counts.p + lps[i].out0 + H[i]);
        return 0;
    }

    int fetch_poses(const int* j, const int* k, int n, float (*pose12)[12]) override {
        // the poses the pick kernel brought back with the counts, when the replay kept the same
        // hypotheses (it always does: both apply Sim3Solver.cpp:155-166 to the same counts)
        bool from_pick = pick_valid;
        for (int q = 0; q < n && from_pick; ++q)
            from_pick = reinterpret_cast<const int32_t*>(C->h_pick.p + (size_t)j[q] * 16)[0] == k[q];
        if (from_pick) {
            for (int q = 0; q < n; ++q) std::memcpy(pose12[q], C->h_pick.p + (size_t)j[q] * 16 + 1, 48);
            return 0;
        }
        // record indices -> one gather kernel -> one D2H copy
        if (int e = C->h_small.ensure((size_t)n * 13)) return e;
        int32_t* hidx = reinterpret_cast<int32_t*>(C->h_small.p + (size_t)n * 12);
        for (int q = 0; q < n; ++q) hidx[q] = solvers[j[q]]->spec_out0 + k[q];
        if (int e = C->d_gather.ensure((size_t)n * 13)) return e;
        int32_t* didx = reinterpret_cast<int32_t*>(C->d_gather.p + (size_t)n * 12);
        RSC_HIP(hipMemcpyAsync(didx, hidx, (size_t)n * 4, hipMemcpyHostToDevice, C->stream));
        RSC_HIP(launch_gather_records(C->d_poses.p, 24, 12, didx, n, C->d_gather.p, C->stream));
        RSC_HIP(hipMemcpyAsync(C->h_small.p, C->d_gather.p, (size_t)n * 48, hipMemcpyDeviceToHost, C->stream));
        RSC_HIP(hipStreamSynchronize(C->stream));
        std::memcpy(pose12, C->h_small.p, (size_t)n * 48);
        return 0;
    }

    int fetch_mask(const int* wj, const int* wk, Sim3State* const* S, int count, uint8_t* const* out) override {
        std::vector<std::vector<uint64_t>> words(count);
        for (int q = 0; q < count; ++q) {
            rsc_sim3* p = solvers[wj[q]];
            const int nw = (S[q]->N + 63) / 64;
            words[q].resize(nw);
            RSC_HIP(hipMemcpyAsync(words[q].data(), C->d_masks.p + (size_t)(p->spec_out0 + wk[q]) * C->mask_words,
                                   (size_t)nw * 8, hipMemcpyDeviceToHost, C->stream));
        }
        RSC_HIP(hipStreamSynchronize(C->stream));
        for (int q = 0; q < count; ++q) {
            const Sim3State& s = *S[q];
            std::memset(out[q], 0, s.mN1);
            for (int j = 0; j < s.N; ++j)
                if ((words[q][j >> 6] >> (j & 63)) & 1ull) out[q][s.indices1[j]] = 1;
        }
        return 0;
    }
};

// ------------------------------------------------------------------------------------------------
// MLPnP backend
// ------------------------------------------------------------------------------------------------
struct HipMLBackend : MLBackend {
    rsc_context* C;
    std::vector<rsc_mlpnp*> all;      // solvers of the call
    std::vector<rsc_mlpnp*> solvers;  // slot j of the last speculation
    explicit HipMLBackend(rsc_context* c) : C(c) {}
    rsc_mlpnp* of(MLState* s) {
        for (auto* p : all)
            if (&p->st == s) return p;
        return nullptr;
    }

    int speculate(MLState* const* S, int count, const int* H, std::vector<std::vector<int32_t>>& counts) override {
        int total = 0, maxN = 1;
        std::vector<DevML> probs(count);
        std::vector<LaunchProb> lps(count);
        solvers.assign(count, nullptr);
        for (int i = 0; i < count; ++i) {
            rsc_mlpnp* p = of(S[i]);
            if (!p) return RSC_ERR_ARG;
            solvers[i] = p;
            S[i]->rng.ensure(C->table, H[i] * S[i]->mRansacMinSet);
            DevML& d = probs[i];
            d.pts = p->d_pts; d.uv = p->d_uv; d.brg = p->d_brg; d.cov = p->use_cov ? p->d_cov : nullptr; d.n = S[i]->N;
            d.fx = p->fx; d.fy = p->fy; d.cx = p->cx; d.cy = p->cy; d.th2 = S[i]->th2;
            LaunchProb& lp = lps[i];
            lp.prob = i;
            lp.H = H[i];
            lp.out0 = total;
            lp.g0 = S[i]->rng.g;
            std::memcpy(lp.window, S[i]->rng.window, sizeof(lp.window));
            lp.min_inliers = S[i]->mRansacMinInliers;  // only such hypotheses' masks are ever read
            p->spec_out0 = total;
            p->spec_H = H[i];
            total += H[i];
            maxN = std::max(maxN, S[i]->N);
        }
        const int ppt = ppt_for(maxN);
        if (ppt > 32) {
            g_last_error = "more than 8192 correspondences per problem";
            return RSC_ERR_UNSUPPORTED;
        }
        const int mw = ppt * 4;
        C->mask_words = mw;
        std::vector<std::vector<int2>> solve_wgs(6);  // by (min_set, covariances given)
        std::vector<int4> scan_wgs;
        const int HC = 32;
        for (int i = 0; i < count; ++i) {
            const int g = 2 * (S[i]->mRansacMinSet - 6) + (probs[i].cov ? 1 : 0);
            for (int h0 = 0; h0 < H[i]; h0 += kMlQuadHyps) solve_wgs[g].push_back(make_int2(i, h0));
            for (int h0 = 0; h0 < H[i]; h0 += HC) scan_wgs.push_back(make_int4(i, h0, std::min(HC, H[i] - h0), 0));
        }
        for (auto& t : solve_wgs) xcd_order(t, [](const int2& w) { return w.x; });
        xcd_order(scan_wgs, [](const int4& w) { return w.x; });
        Blob b;
        const size_t o_probs = b.add(probs.data(), probs.size() * sizeof(DevML));
        const size_t o_lps = b.add(lps.data(), lps.size() * sizeof(LaunchProb));
        size_t o_solve[6];
        for (int g = 0; g < 6; ++g) o_solve[g] = b.add(solve_wgs[g].data(), solve_wgs[g].size() * sizeof(int2));
        const size_t o_scan = b.add(scan_wgs.data(), scan_wgs.size() * sizeof(int4));
        if (int e = upload_blob(C, b)) return e;
        if (int e = C->d_mposes.ensure((size_t)total * 12)) return e;
        int32_t* cnt_dst = nullptr;
        if (int e = counts_target(C, total, &cnt_dst)) return e;
        if (int e = C->d_masks.ensure((size_t)total * mw)) return e;
        if (C->keep_samples)
            if (int e = C->d_samples.ensure((size_t)total * 8)) return e;
        const char* base = C->d_desc.p;
        const DevML* dprobs = reinterpret_cast<const DevML*>(base + o_probs);
        const LaunchProb* dlps = reinterpret_cast<const LaunchProb*>(base + o_lps);
        timing_begin(C, 0);
        for (int g = 0; g < 6; ++g) {
            if (solve_wgs[g].empty()) continue;
            RSC_HIP(launch_mlpnp_solve(6 + g / 2, (g & 1) != 0, (int)solve_wgs[g].size(), dprobs, dlps,
                                       reinterpret_cast<const int2*>(base + o_solve[g]), C->d_table.p, C->d_mposes.p,
                                       C->keep_samples ? C->d_samples.p : nullptr, C->stream));
        }
        timing_begin(C, 1);
        RSC_HIP(launch_mlpnp_scan(ppt, (int)scan_wgs.size(), dprobs, dlps, reinterpret_cast<const int4*>(base + o_scan),
                                  C->d_mposes.p, cnt_dst, C->d_masks.p, mw, C->stream));
        timing_begin(C, 2);
        if (!C->direct_counts)
            RSC_HIP(hipMemcpyAsync(C->h_counts.p, C->d_counts.p, (size_t)total * 4, hipMemcpyDeviceToHost, C->stream));
        if (int e = stream_wait(C)) return e;
        if (C->timing) {
            float a = 0, sc = 0;
            (void)hipEventElapsedTime(&a, C->ev[0], C->ev[1]);
            (void)hipEventElapsedTime(&sc, C->ev[1], C->ev[2]);
            C->last_ms[0] += a;
            C->last_ms[1] += sc;
            C->last_ms[3] += 1;
            C->last_ms[4] += total;
        }
        counts.resize(count);  // keeps the inner vectors' capacity
        for (int i = 0; i < count; ++i)
            counts[i].assign(C->h_counts.p + lps[i].out0, C->h_counts.p + lps[i].out0 + H[i]);
        return 0;
    }

    int pose_of(int j, int k, float* pose12) {
        // R, t double -> float (cv::Mat::convertTo(CV_32F), MLPnPsolver.cpp:152-153)
        double d[12];
        RSC_HIP(hipMemcpyAsync(d, C->d_mposes.p + (size_t)(solvers[j]->spec_out0 + k) * 12, 96, hipMemcpyDeviceToHost,
                               C->stream));
        RSC_HIP(hipStreamSynchronize(C->stream));
        for (int q = 0; q < 12; ++q) pose12[q] = (float)d[q];
        return 0;
    }

    int adopt_best(MLState* s, int j, int k) override {
        rsc_mlpnp* p = solvers[j];
        const size_t rec = (size_t)(p->spec_out0 + k);
        RSC_HIP(hipMemcpyAsync(p->d_best, C->d_masks.p + rec * C->mask_words, (size_t)p->words * 8,
                               hipMemcpyDeviceToDevice, C->stream));
        float pose[12];
        if (int e = pose_of(j, k, pose)) return e;
        pose12_to_T(pose, s->mBestTcw);
        return 0;
    }

    int fetch_poses(const int* j, const int* k, int n, float (*pose12)[12]) override {
        for (int q = 0; q < n; ++q)
            if (int e = pose_of(j[q], k[q], pose12[q])) return e;
        return 0;
    }

    int fetch_mask(MLState* const* S, int count, const int* kind, const int* j, const int* k,
                   uint8_t* const* out) override {
        std::vector<std::vector<uint64_t>> words(count);
        for (int q = 0; q < count; ++q) {
            rsc_mlpnp* p = of(S[q]);
            words[q].resize(p->words);
            const uint64_t* src = (kind[q] == 2) ? p->d_best
                                                 : C->d_masks.p + (size_t)(solvers[j[q]]->spec_out0 + k[q]) * C->mask_words;
            RSC_HIP(hipMemcpyAsync(words[q].data(), src, (size_t)p->words * 8, hipMemcpyDeviceToHost, C->stream));
        }
        RSC_HIP(hipStreamSynchronize(C->stream));
        for (int q = 0; q < count; ++q) {
            const MLState& s = *S[q];
            std::memset(out[q], 0, s.N_points);
            for (int i = 0; i < s.N; ++i)
                if ((words[q][i >> 6] >> (i & 63)) & 1ull) out[q][s.kp_index[i]] = 1;
        }
        return 0;
    }
};

void to_result(const PnPResult& r, rsc_pnp_result* o) {
    o->ok = r.ok;
    o->no_more = r.no_more;
    o->n_inliers = r.n_inliers;
    o->iterations = r.iterations;
    if (r.ok) std::memcpy(o->T, r.T, sizeof(o->T));
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
// rand() draws per hypothesis: mRansacMinSet RandomInt calls (PnPsolver.cpp:125-131,
// MLPnPsolver.cpp:84-92), 3 for Sim3 (Sim3Solver.cpp:140-147).
static inline int draws_per_hypothesis(const PnPState& s) { return s.mRansacMinSet; }
static inline int draws_per_hypothesis(const Sim3State&) { return 3; }
static inline int draws_per_hypothesis(const MLState& s) { return s.mRansacMinSet; }

// srand(seed) on a solver's own stream: while the solver is bound, that stream is the parked one
template <class Solver>
static void reset_solver(Solver* s, uint32_t seed) {
    s->st.reset(seed);
    if (s->stream) s->own_rng = s->st.rng;
}

// rsc_*_bind_stream: binding parks the own stream, unbinding resumes it where it stopped (a bound
// call overwrites st.rng with the shared stream's position); rebinding keeps the parked one
template <class Solver>
static int bind_stream(Solver* s, rsc_stream* stream) {
    if (!s || (stream && stream->ctx != s->ctx)) return RSC_ERR_ARG;
    if (!s->stream && stream) s->own_rng = s->st.rng;
    if (s->stream && !stream) s->st.rng = s->own_rng;
    s->stream = stream;
    return RSC_OK;
}

// iterate() calls of solvers bound to a shared stream draw in call order, so a bound solver's call
// starts where the previous call ended: the calls run one at a time in list order.
template <class Solver, class Impl, class Out>
static int bound_iterate_many(Solver* const* solvers, int count, const int32_t* n_its, Out* out,
                              uint8_t* const* inliers, Impl impl) {
    for (int i = 0; i < count; ++i) {
        Solver* s = solvers[i];
        if (!s) return RSC_ERR_ARG;
        const int it0 = s->st.mnIterations;
        if (s->stream) s->st.rng = s->stream->st;
        uint8_t* const m[1] = {inliers ? inliers[i] : nullptr};
        if (int st = impl(&solvers[i], 1, n_its + i, out + i, m)) return st;
        if (s->stream) {
            s->stream->st = s->st.rng;
            s->stream->position += (int64_t)(s->st.mnIterations - it0) * draws_per_hypothesis(s->st);
        }
    }
    return RSC_OK;
}

namespace {
template <class Solver, class Res, class IterFn>
int shared_events(Solver* const* solvers, const int32_t* event_begin, int n_events, rsc_stream* const* streams,
                  Res* per_candidate, rsc_event_result* per_event, IterFn iter, int (*pred_its)(const Solver*)) {
    if (n_events <= 0) return RSC_OK;
    if (!solvers || !event_begin || !streams || !per_candidate || !per_event) return RSC_ERR_ARG;
    const int total = event_begin[n_events];
    for (int e = 0; e < n_events; ++e) {
        if (event_begin[e + 1] < event_begin[e] || !streams[e] || streams[e]->ctx != streams[0]->ctx)
            return RSC_ERR_ARG;
        for (int f = 0; f < e; ++f)
            if (streams[f] == streams[e]) return RSC_ERR_ARG;  // one stream per event (calls of two events would interleave)
        per_event[e] = rsc_event_result{-1, -1, -1, 0};
    }
    std::vector<char> discarded(total, 0), resolved(n_events, 0);
    std::vector<int32_t> start_it(total);
    std::vector<RngStream> own(total);  // the calls draw from the event's stream; a solver's own
                                        // stream (st.rng of an unbound one) resumes afterwards
    for (int i = 0; i < total; ++i) {
        if (!solvers[i] || solvers[i]->ctx != streams[0]->ctx) return RSC_ERR_ARG;
        start_it[i] = solvers[i]->st.mnIterations;
        own[i] = solvers[i]->st.rng;
    }
    for (int round = 0;; ++round) {
        std::vector<Solver*> act;
        std::vector<int> idx;
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            RngStream cur = streams[e]->st;  // call positions, assuming every call runs its whole loop
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
                if (discarded[i]) continue;
                Solver* s = solvers[i];
                s->st.rng = cur;
                cur.advance(s->ctx->table, (int64_t)pred_its(s) * draws_per_hypothesis(s->st));
                act.push_back(s);
                idx.push_back(i);
            }
        }
        if (act.empty()) break;
        std::vector<int32_t> its(act.size(), 5), it0(act.size());
        for (size_t q = 0; q < act.size(); ++q) it0[q] = act[q]->st.mnIterations;
        std::vector<Res> r(act.size());
        std::vector<uint8_t*> nomask(act.size(), nullptr);
        if (int st = iter(act.data(), (int)act.size(), its.data(), r.data(), nomask.data())) return st;
        std::vector<int> slot(total, -1);
        for (size_t q = 0; q < act.size(); ++q) slot[idx[q]] = (int)q;
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            bool any_active = false;
            int64_t used = 0;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
                const int q = slot[i];
                if (q < 0) continue;  // discarded in an earlier round
                const Solver* s = act[q];
                used += (int64_t)(s->st.mnIterations - it0[q]) * draws_per_hypothesis(s->st);
                per_candidate[i] = r[q];
                if (r[q].no_more) discarded[i] = 1;  // Tracking.cpp:1257-1261, LoopClosing.cpp:292-296
                if (r[q].ok) {
                    per_event[e].winner = i - event_begin[e];
                    per_event[e].round = round;
                    per_event[e].hypothesis = r[q].iterations - 1 - start_it[i];
                    per_event[e].n_inliers = r[q].n_inliers;
                    resolved[e] = 1;
                    break;
                }
                if (!discarded[i]) any_active = true;
            }
            streams[e]->st.advance(streams[e]->ctx->table, used);
            streams[e]->position += used;
            if (!resolved[e] && !any_active) resolved[e] = 1;
        }
    }
    for (int i = 0; i < total; ++i) solvers[i]->st.rng = own[i];
    return RSC_OK;
}

// hypotheses the next iterate(5) call runs unless it succeeds: PnP's '||' loop (Q1)
// max(5, maxIts - mnIterations), Sim3's '&&' loop min(5, maxIts - mnIterations); none when N is
// below minInliers (the call returns at once)
int pnp_pred_its(const rsc_pnp* s) {
    const PnPState& t = s->st;
    return (t.N < t.mRansacMinInliers) ? 0 : std::max(0, std::max(5, t.mRansacMaxIts - t.mnIterations));
}
int sim3_pred_its(const rsc_sim3* s) {
    const Sim3State& t = s->st;
    return (t.N < t.mRansacMinInliers) ? 0 : std::max(0, std::min(5, t.mRansacMaxIts - t.mnIterations));
}
}  // namespace

extern "C" {

int rsc_version(void) { return 1; }

const char* rsc_status_string(int status) {
    switch (status) {
        case RSC_OK: return "ok";
        case RSC_ERR_ARG: return "invalid argument";
        case RSC_ERR_HIP: return g_last_error.empty() ? "HIP error" : g_last_error.c_str();
        case RSC_ERR_OOM: return g_last_error.empty() ? "out of device memory" : g_last_error.c_str();
        case RSC_ERR_UNSUPPORTED: return g_last_error.empty() ? "unsupported" : g_last_error.c_str();
        case RSC_ERR_NODEVICE: return "no HIP device";
        case RSC_ERR_INTERNAL: return g_last_error.empty() ? "internal error" : g_last_error.c_str();
        default: return "unknown status";
    }
}

int rsc_context_create(int device, rsc_context** out) {
    if (!out) return RSC_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RSC_ERR_NODEVICE;
    if (device < 0 || device >= ndev) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(device));
    std::unique_ptr<rsc_context> C(new rsc_context());
    C->device = device;
    RSC_HIP(hipStreamCreateWithFlags(&C->stream, hipStreamNonBlocking));
    C->own_stream = true;
    if (const char* m = std::getenv("RSC_DIRECT_COUNTS")) C->direct_counts = std::strcmp(m, "0") != 0;
    if (const char* m = std::getenv("RSC_FUSED_REFINE")) C->fused_refine = std::strcmp(m, "0") != 0;
    if (const char* m = std::getenv("RSC_DMA_UPLOAD")) C->dma_upload = std::strcmp(m, "0") != 0;
    if (const char* m = std::getenv("RSC_EIG_ROWS")) C->eig_rows_max_wgs = std::max(0, std::atoi(m));
    if (const char* m = std::getenv("RSC_EIG_SPLIT")) C->eig_split = std::strcmp(m, "0") != 0;
    if (const char* m = std::getenv("RSC_BETAS_HB")) C->betas_small_hb = std::min(kBetasHyps, std::max(1, std::atoi(m)));
    if (const char* m = std::getenv("RSC_SPIN_WAIT")) C->spin_wait = std::strcmp(m, "0") != 0;
    if (const char* m = std::getenv("RSC_SO_HELPERS")) C->so_helpers = std::max(-1, std::atoi(m));
    {
        void* f = nullptr;
        RSC_HIP(hipHostMalloc(&f, 64, hipHostMallocCoherent));
        C->h_flag = static_cast<uint32_t*>(f);
        std::memset(C->h_flag, 0, 64);
    }
    C->table.build();
    if (int e = C->d_table.ensure(C->table.T.size())) return e;
    RSC_HIP(hipMemcpy(C->d_table.p, C->table.T.data(), C->table.T.size() * 4, hipMemcpyHostToDevice));
    for (auto& e : C->ev) RSC_HIP(hipEventCreate(&e));
    *out = C.release();
    return RSC_OK;
}

void rsc_context_destroy(rsc_context* C) {
    if (!C) return;
    (void)hipSetDevice(C->device);
    if (C->stream) (void)hipStreamSynchronize(C->stream);
    if (C->h_flag) (void)hipHostFree(C->h_flag);
    for (auto& e : C->ev)
        if (e) (void)hipEventDestroy(e);
    if (C->own_stream && C->stream) (void)hipStreamDestroy(C->stream);
    delete C;
}

int rsc_context_set_stream(rsc_context* C, void* s) {
    if (!C) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (C->own_stream) (void)hipStreamDestroy(C->stream);
    C->stream = reinterpret_cast<hipStream_t>(s);
    C->own_stream = false;
    return RSC_OK;
}

int rsc_context_synchronize(rsc_context* C) {
    if (!C) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    return RSC_OK;
}

int rsc_context_enable_timing(rsc_context* C, int enable) {
    if (!C) return RSC_ERR_ARG;
    C->timing = enable != 0;
    return RSC_OK;
}

int rsc_context_set_eig_rows(rsc_context* C, int max_workgroups) {
    if (!C || max_workgroups < 0) return RSC_ERR_ARG;
    C->eig_rows_max_wgs = max_workgroups;
    return RSC_OK;
}

int rsc_context_set_eig_split(rsc_context* C, int on) {
    if (!C) return RSC_ERR_ARG;
    C->eig_split = on != 0;
    return RSC_OK;
}

int rsc_context_set_sim3opt_helpers(rsc_context* C, int helpers) {
    if (!C || helpers < -1) return RSC_ERR_ARG;
    C->so_helpers = helpers;
    return RSC_OK;
}

int rsc_selftest_math(rsc_context* C, int fn, const double* x, int n, double* out) {
    if (!C || fn < 0 || fn > 16 || fn == 14 || fn == 15 || n < 0 || (n > 0 && (!x || !out)) || (fn == 10 && n % 34) ||
        (fn == 16 && n % 42))
        return RSC_ERR_ARG;
    if (n == 0) return RSC_OK;
    RSC_HIP(hipSetDevice(C->device));
    double* d = nullptr;
    RSC_HIP(hipMalloc(&d, (size_t)n * 16));
    std::unique_ptr<double, void (*)(double*)> hold(d, [](double* p) { (void)hipFree(p); });
    RSC_HIP(hipMemcpyAsync(d, x, (size_t)n * 8, hipMemcpyHostToDevice, C->stream));
    if (fn == 16) RSC_HIP(launch_selftest_ldlt(d, n / 42, d + n, C->stream));
    else RSC_HIP(launch_selftest_math(fn, d, n, d + n, C->stream));
    RSC_HIP(hipMemcpyAsync(out, d + n, (size_t)n * 8, hipMemcpyDeviceToHost, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    return RSC_OK;
}

int rsc_context_last_timing(rsc_context* C, double out[5]) {
    if (!C || !out) return RSC_ERR_ARG;
    for (int i = 0; i < 5; ++i) out[i] = C->last_ms[i];
    return RSC_OK;
}

int rsc_context_last_kernel_timing(rsc_context* C, double out[6]) {
    if (!C || !out) return RSC_ERR_ARG;
    for (int i = 0; i < 6; ++i) out[i] = C->last_ms[i];
    return RSC_OK;
}

// ---- PnP ----
int rsc_pnp_create(rsc_context* C, const rsc_pnp_problem* pb, uint32_t seed, rsc_pnp** out) {
    if (!C || !pb || !out || pb->n < 0 || pb->n_points < pb->n) return RSC_ERR_ARG;
    if (pb->n > 0 && (!pb->p2d || !pb->p3dw || !pb->sigma2)) return RSC_ERR_ARG;
    *out = nullptr;
    RSC_HIP(hipSetDevice(C->device));
    std::unique_ptr<rsc_pnp> S(new rsc_pnp());
    S->ctx = C;
    PnPState& s = S->st;
    s.N = pb->n;
    s.N_points = pb->n_points;
    s.fx = pb->fx; s.fy = pb->fy; s.cx = pb->cx; s.cy = pb->cy;
    s.kp_index.resize(pb->n);
    for (int i = 0; i < pb->n; ++i) s.kp_index[i] = pb->kp_index ? pb->kp_index[i] : i;
    s.sigma2.assign(pb->sigma2, pb->sigma2 + pb->n);
    s.reset(seed);
    S->h_p2d.assign(pb->p2d, pb->p2d + 2 * (size_t)pb->n);
    S->h_p3d.assign(pb->p3dw, pb->p3dw + 3 * (size_t)pb->n);
    const int n = std::max(pb->n, 1);
    S->words = (n + 63) / 64;
    std::vector<float4> pts(n);
    std::vector<float2> uv(n);
    for (int i = 0; i < pb->n; ++i) {
        pts[i] = make_float4(pb->p3dw[3 * i], pb->p3dw[3 * i + 1], pb->p3dw[3 * i + 2], pb->sigma2[i]);
        uv[i] = make_float2(pb->p2d[2 * i], pb->p2d[2 * i + 1]);
    }
    const size_t cap = (size_t)std::max(n, 8);
    RSC_HIP(hipMalloc(&S->d_pts, n * sizeof(float4)));
    RSC_HIP(hipMalloc(&S->d_uv, n * sizeof(float2)));
    RSC_HIP(hipMalloc(&S->d_pws, cap * 3 * sizeof(double)));
    RSC_HIP(hipMalloc(&S->d_us, cap * 2 * sizeof(double)));
    RSC_HIP(hipMalloc(&S->d_als, cap * 4 * sizeof(double)));
    RSC_HIP(hipMalloc(&S->d_best, S->words * 8));
    RSC_HIP(hipMalloc(&S->d_refined, S->words * 8));
    RSC_HIP(hipMemcpy(S->d_pts, pts.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(S->d_uv, uv.data(), n * sizeof(float2), hipMemcpyHostToDevice));
    RSC_HIP(hipMemset(S->d_pws, 0, cap * 3 * sizeof(double)));
    RSC_HIP(hipMemset(S->d_us, 0, cap * 2 * sizeof(double)));
    RSC_HIP(hipMemset(S->d_als, 0, cap * 4 * sizeof(double)));
    RSC_HIP(hipMemset(S->d_best, 0, S->words * 8));
    RSC_HIP(hipMemset(S->d_refined, 0, S->words * 8));
    // PnPsolver does not call SetRansacParameters in its constructor; iterate() before it is UB in
    // the reference.  Install the declared defaults so that the object is always usable.
    pnp_set_params(s, 0.99, 8, 300, 4, 0.4f, 5.991f);
    *out = S.release();
    return RSC_OK;
}

void rsc_pnp_destroy(rsc_pnp* s) { delete s; }

int rsc_pnp_set_ransac_parameters(rsc_pnp* s, double probability, int min_inliers, int max_iterations, int min_set,
                                  float epsilon, float th2) {
    if (!s) return RSC_ERR_ARG;
    pnp_set_params(s->st, probability, min_inliers, max_iterations, min_set, epsilon, th2);
    return RSC_OK;
}

static int pnp_iterate_many_impl(rsc_pnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                                 uint8_t* const* inliers);

int rsc_pnp_iterate_many(rsc_pnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                         uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i)
        if (solvers[i] && solvers[i]->stream)
            return bound_iterate_many(solvers, count, n_its, out, inliers, pnp_iterate_many_impl);
    return pnp_iterate_many_impl(solvers, count, n_its, out, inliers);
}

static int pnp_iterate_many_impl(rsc_pnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                                 uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    rsc_context* C = solvers[0]->ctx;
    for (int i = 0; i < count; ++i)
        if (!solvers[i] || solvers[i]->ctx != C) return RSC_ERR_ARG;
    // vbInliers of a call that fails is empty (rsc_pnp_last_inliers returns 0 after it)
    for (int i = 0; i < count; ++i) solvers[i]->last_kind = 0;
    C->t_entry = std::chrono::steady_clock::now();
    RSC_HIP(hipSetDevice(C->device));
    for (double& v : C->last_ms) v = 0;
    HipPnPBackend be(C);
    be.solvers.assign(solvers, solvers + count);
    std::vector<PnPState*> S(count);
    std::vector<int> its(count);
    for (int i = 0; i < count; ++i) { S[i] = &solvers[i]->st; its[i] = n_its[i]; }
    std::vector<PnPResult> res(count);
    int st = pnp_iterate_many(be, S.data(), count, its.data(), res.data(), inliers);
    if (st) return st;
    for (int i = 0; i < count; ++i) {
        to_result(res[i], &out[i]);
        solvers[i]->last_kind = res[i].mask_kind;
    }
    host_mark(C, 3);
    return RSC_OK;
}

int rsc_diag_host_timing(rsc_context* C, double out[4]) {
    if (!C || !out) return RSC_ERR_ARG;
    for (int i = 0; i < 4; ++i) out[i] = C->host_us[i];
    return RSC_OK;
}

int rsc_pnp_iterate(rsc_pnp* s, int n_its, rsc_pnp_result* out, uint8_t* inliers) {
    if (!s || !out) return RSC_ERR_ARG;
    int32_t n = n_its;
    uint8_t* const m[1] = {inliers};
    return rsc_pnp_iterate_many(&s, 1, &n, out, m);
}

int rsc_pnp_find(rsc_pnp* s, rsc_pnp_result* out, uint8_t* inliers) {
    if (!s) return RSC_ERR_ARG;
    return rsc_pnp_iterate(s, s->st.mRansacMaxIts, out, inliers);
}

int rsc_pnp_last_inliers(rsc_pnp* s, uint8_t* out) {
    if (!s || !out) return RSC_ERR_ARG;
    const PnPState& t = s->st;
    std::memset(out, 0, (size_t)t.N_points);
    if (s->last_kind == 0) return 0;
    std::vector<uint64_t> w((size_t)s->words);
    RSC_HIP(hipMemcpyAsync(w.data(), s->last_kind == 1 ? s->d_refined : s->d_best, (size_t)s->words * 8,
                           hipMemcpyDeviceToHost, s->ctx->stream));
    RSC_HIP(hipStreamSynchronize(s->ctx->stream));
    for (int j = 0; j < t.N; ++j)
        if ((w[j >> 6] >> (j & 63)) & 1ull) out[t.kp_index[j]] = 1;
    return 1;
}

int rsc_pnp_reset(rsc_pnp* s, uint32_t seed) {
    if (!s) return RSC_ERR_ARG;
    reset_solver(s, seed);
    s->last_kind = 0;
    return RSC_OK;
}

int rsc_pnp_get_state(const rsc_pnp* s, int32_t out[8]) {
    if (!s || !out) return RSC_ERR_ARG;
    const PnPState& t = s->st;
    out[0] = t.mnIterations; out[1] = t.mRansacMaxIts; out[2] = t.mRansacMinInliers; out[3] = t.mnBestInliers;
    out[4] = t.max_rows; out[5] = t.N; out[6] = t.N_points; out[7] = t.mRansacMinSet;
    return RSC_OK;
}

int rsc_pnp_last_samples(rsc_pnp* s, int32_t* out, int cap) {
    if (!s || !out) return RSC_ERR_ARG;
    rsc_context* C = s->ctx;
    if (s->spec_out0 < 0 || !C->d_samples.p) return 0;
    const int n = std::min(cap, s->spec_H);
    RSC_HIP(hipMemcpy(out, C->d_samples.p + (size_t)s->spec_out0 * 8, (size_t)n * 8 * 4, hipMemcpyDeviceToHost));
    return n;
}

// Parity hook: counts + float poses of the last speculation of this solver.  The counts live in the
// context's pinned count buffer (valid until the context's next speculation); poses stay in HBM.
namespace {
int last_hypotheses(rsc_context* C, int out0, int H, int stride, int32_t* counts, float* poses, int cap) {
    if (out0 < 0) return 0;
    const int n = std::min(cap, H);
    if (counts) std::memcpy(counts, C->h_counts.p + out0, (size_t)n * 4);
    if (poses) {
        if (!C->d_poses.p) return RSC_ERR_ARG;
        std::vector<float> all((size_t)n * stride);
        RSC_HIP(hipMemcpy(all.data(), C->d_poses.p + (size_t)out0 * stride, all.size() * 4, hipMemcpyDeviceToHost));
        for (int h = 0; h < n; ++h) std::memcpy(poses + (size_t)h * 12, all.data() + (size_t)h * stride, 48);
    }
    return n;
}
}  // namespace

int rsc_pnp_last_hypotheses(rsc_pnp* s, int32_t* counts, float* poses, int cap) {
    if (!s) return RSC_ERR_ARG;
    return last_hypotheses(s->ctx, s->spec_out0, s->spec_H, 12, counts, poses, cap);
}

// ---- Sim3 ----
int rsc_sim3_create(rsc_context* C, const rsc_sim3_input* in, uint32_t seed, rsc_sim3** out) {
    if (!C || !in || !out || in->n1 < 0) return RSC_ERR_ARG;
    *out = nullptr;
    RSC_HIP(hipSetDevice(C->device));
    std::unique_ptr<rsc_sim3> S(new rsc_sim3());
    S->ctx = C;
    Sim3State& s = S->st;
    s.mN1 = in->n1;
    // Sim3Solver::Sim3Solver (Sim3Solver.cpp:26-68): camera-frame points (float), size_t thresholds
    for (int i1 = 0; i1 < in->n1; ++i1) {
        if (!in->valid[i1]) continue;
        S->e1.push_back((uint64_t)(9.210 * in->sigma2_1[i1]));
        S->e2.push_back((uint64_t)(9.210 * in->sigma2_2[i1]));
        s.indices1.push_back(i1);
        const float* a = &in->Xw1[3 * i1];
        const float* b = &in->Xw2[3 * i1];
        // Rcw*X3Dw + tcw (Sim3Solver.cpp:58,62): Matrix3f * Vector3f, coefficient-path reductions
        for (int r = 0; r < 3; ++r)
            S->X1c.push_back(ered3(in->R1[3 * r] * a[0], in->R1[3 * r + 1] * a[1], in->R1[3 * r + 2] * a[2]) + in->t1[r]);
        for (int r = 0; r < 3; ++r)
            S->X2c.push_back(ered3(in->R2[3 * r] * b[0], in->R2[3 * r + 1] * b[1], in->R2[3 * r + 2] * b[2]) + in->t2[r]);
    }
    s.N = (int)s.indices1.size();
    std::memcpy(S->K1, in->K1, sizeof(S->K1));
    std::memcpy(S->K2, in->K2, sizeof(S->K2));
    // FromCameraToImage (Sim3Solver.cpp:329-347)
    auto to_image = [](const std::vector<float>& X, std::vector<float>& P, const float K[4]) {
        const size_t n = X.size() / 3;
        P.resize(2 * n);
        for (size_t i = 0; i < n; ++i) {
            const float invz = 1 / X[3 * i + 2];
            const float x = X[3 * i] * invz;
            const float y = X[3 * i + 1] * invz;
            P[2 * i] = K[0] * x + K[2];
            P[2 * i + 1] = K[1] * y + K[3];
        }
    };
    to_image(S->X1c, S->P1, S->K1);
    to_image(S->X2c, S->P2, S->K2);
    const int n = std::max(s.N, 1);
    std::vector<float4> x1(n), x2(n), pim(n);
    for (int i = 0; i < s.N; ++i) {
        x1[i] = make_float4(S->X1c[3 * i], S->X1c[3 * i + 1], S->X1c[3 * i + 2], (float)S->e1[i]);
        x2[i] = make_float4(S->X2c[3 * i], S->X2c[3 * i + 1], S->X2c[3 * i + 2], (float)S->e2[i]);
        pim[i] = make_float4(S->P1[2 * i], S->P1[2 * i + 1], S->P2[2 * i], S->P2[2 * i + 1]);
    }
    RSC_HIP(hipMalloc(&S->d_x1, n * sizeof(float4)));
    RSC_HIP(hipMalloc(&S->d_x2, n * sizeof(float4)));
    RSC_HIP(hipMalloc(&S->d_pim, n * sizeof(float4)));
    RSC_HIP(hipMemcpy(S->d_x1, x1.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(S->d_x2, x2.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(S->d_pim, pim.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    s.reset(seed);
    sim3_set_params(s, 0.99, 6, 300);  // the constructor's SetRansacParameters() (:84)
    *out = S.release();
    return RSC_OK;
}

void rsc_sim3_destroy(rsc_sim3* s) { delete s; }

int rsc_sim3_set_ransac_parameters(rsc_sim3* s, double probability, int min_inliers, int max_iterations) {
    if (!s) return RSC_ERR_ARG;
    sim3_set_params(s->st, probability, min_inliers, max_iterations);
    return RSC_OK;
}

static int sim3_iterate_many_impl(rsc_sim3* const* solvers, int count, const int32_t* n_its, rsc_sim3_result* out,
                                  uint8_t* const* inliers);

int rsc_sim3_iterate_many(rsc_sim3* const* solvers, int count, const int32_t* n_its, rsc_sim3_result* out,
                          uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i)
        if (solvers[i] && solvers[i]->stream)
            return bound_iterate_many(solvers, count, n_its, out, inliers, sim3_iterate_many_impl);
    return sim3_iterate_many_impl(solvers, count, n_its, out, inliers);
}

static int sim3_iterate_many_impl(rsc_sim3* const* solvers, int count, const int32_t* n_its, rsc_sim3_result* out,
                                  uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    rsc_context* C = solvers[0]->ctx;
    for (int i = 0; i < count; ++i)
        if (!solvers[i] || solvers[i]->ctx != C) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(C->device));
    for (double& v : C->last_ms) v = 0;
    HipSim3Backend be(C);
    be.all.assign(solvers, solvers + count);
    std::vector<Sim3State*> S(count);
    std::vector<int> its(count);
    for (int i = 0; i < count; ++i) { S[i] = &solvers[i]->st; its[i] = n_its[i]; }
    std::vector<Sim3Result> res(count);
    int st = sim3_iterate_many(be, S.data(), count, its.data(), res.data(), inliers);
    if (st) return st;
    for (int i = 0; i < count; ++i) {
        out[i].ok = res[i].ok;
        out[i].no_more = res[i].no_more;
        out[i].n_inliers = res[i].n_inliers;
        out[i].iterations = res[i].iterations;
        std::memcpy(out[i].R, res[i].R, sizeof(out[i].R));
        std::memcpy(out[i].t, res[i].t, sizeof(out[i].t));
    }
    return RSC_OK;
}

int rsc_sim3_iterate(rsc_sim3* s, int n_its, rsc_sim3_result* out, uint8_t* inliers) {
    if (!s || !out) return RSC_ERR_ARG;
    int32_t n = n_its;
    uint8_t* const m[1] = {inliers};
    return rsc_sim3_iterate_many(&s, 1, &n, out, m);
}

int rsc_sim3_find(rsc_sim3* s, rsc_sim3_result* out, uint8_t* inliers) {
    if (!s) return RSC_ERR_ARG;
    return rsc_sim3_iterate(s, s->st.mRansacMaxIts, out, inliers);
}

int rsc_sim3_reset(rsc_sim3* s, uint32_t seed) {
    if (!s) return RSC_ERR_ARG;
    const int mi = s->st.mRansacMinInliers, mx = s->st.mRansacMaxIts;
    (void)mi; (void)mx;
    reset_solver(s, seed);
    return RSC_OK;
}

int rsc_sim3_get_state(const rsc_sim3* s, int32_t out[6]) {
    if (!s || !out) return RSC_ERR_ARG;
    const Sim3State& t = s->st;
    out[0] = t.mnIterations; out[1] = t.mRansacMaxIts; out[2] = t.mRansacMinInliers; out[3] = t.mnBestInliers;
    out[4] = t.N; out[5] = t.mN1;
    return RSC_OK;
}

int rsc_sim3_last_hypotheses(rsc_sim3* s, int32_t* counts, float* poses, int cap) {
    if (!s) return RSC_ERR_ARG;
    return last_hypotheses(s->ctx, s->spec_out0, s->spec_H, 24, counts, poses, cap);
}

int rsc_sim3_prepared(const rsc_sim3* s, float* X1c, float* X2c, float* P1im1, float* P2im2, uint64_t* e1,
                      uint64_t* e2, int32_t* idx) {
    if (!s) return RSC_ERR_ARG;
    const int N = s->st.N;
    if (X1c) std::memcpy(X1c, s->X1c.data(), 12 * (size_t)N);
    if (X2c) std::memcpy(X2c, s->X2c.data(), 12 * (size_t)N);
    if (P1im1) std::memcpy(P1im1, s->P1.data(), 8 * (size_t)N);
    if (P2im2) std::memcpy(P2im2, s->P2.data(), 8 * (size_t)N);
    if (e1) std::memcpy(e1, s->e1.data(), 8 * (size_t)N);
    if (e2) std::memcpy(e2, s->e2.data(), 8 * (size_t)N);
    if (idx) std::memcpy(idx, s->st.indices1.data(), 4 * (size_t)N);
    return RSC_OK;
}


// ---- Optimizer::PoseOptimization (src/Optimizer.cpp:205-424) ----
int rsc_pose_optimization_many(rsc_context* C, const rsc_poseopt_problem* P, int count, rsc_poseopt_result* out,
                               uint8_t* const* outlier) {
    if (!C || count < 0 || (count && (!P || !out))) return RSC_ERR_ARG;
    if (count == 0) return RSC_OK;
    // compaction of the slots with a map point (the edges, Optimizer.cpp:247-325), in slot order
    std::vector<int> run;             // problems with >= 3 edges (the others return 0, :329-330)
    std::vector<size_t> eoff(1, 0);   // edge offsets of the run problems
    for (int c = 0; c < count; ++c) {
        const rsc_poseopt_problem& q = P[c];
        if (q.n < 0 || (q.n > 0 && (!q.uv || !q.Xw || !q.inv_sigma2))) return RSC_ERR_ARG;
        int ne = 0;
        for (int i = 0; i < q.n; ++i) {
            if (q.has_mp && !q.has_mp[i]) continue;
            ++ne;
        }
        if (ne > kPoseMaxEdges) {
            g_last_error = "more than 8192 map-point matches in one Frame";
            return RSC_ERR_UNSUPPORTED;
        }
        rsc_poseopt_result& r = out[c];
        std::memset(&r, 0, sizeof(r));
        r.n_initial = ne;
        std::memcpy(r.Tcw, q.Tcw, sizeof(r.Tcw));
        if (outlier && outlier[c])
            for (int i = 0; i < q.n; ++i)
                if (!q.has_mp || q.has_mp[i]) outlier[c][i] = 0;
        if (ne >= 3) {
            run.push_back(c);
            eoff.push_back(eoff.back() + (size_t)ne);
        }
    }
    const int R = (int)run.size();
    if (R == 0) return RSC_OK;
    const size_t E = eoff.back();
    RSC_HIP(hipSetDevice(C->device));
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_probs = 0, o_xw = al(sizeof(DevPoseProb) * R), o_uv = o_xw + al(sizeof(float4) * E);
    const size_t o_ur = o_uv + al(sizeof(float2) * E);  // mvuRight of the edges (stereo: >= 0)
    const size_t in_bytes = o_ur + al(sizeof(float) * E);
    const size_t r_out = 0, r_flags = al(sizeof(float) * 16 * R);
    const size_t res_bytes = r_flags + al(E);
    if (int e = C->h_po_in.ensure(in_bytes)) return e;
    if (int e = C->d_po_in.ensure(in_bytes)) return e;
    if (int e = C->h_po_res.ensure(res_bytes)) return e;
    if (int e = C->d_po_res.ensure(res_bytes)) return e;
    // the previous call's copies out of the pinned staging must be complete
    RSC_HIP(hipStreamSynchronize(C->stream));
    char* h = C->h_po_in.p;
    char* d = C->d_po_in.p;
    DevPoseProb* hp = reinterpret_cast<DevPoseProb*>(h + o_probs);
    float4* hxw = reinterpret_cast<float4*>(h + o_xw);
    float2* huv = reinterpret_cast<float2*>(h + o_uv);
    float* hur = reinterpret_cast<float*>(h + o_ur);
    for (int k = 0; k < R; ++k) {
        const rsc_poseopt_problem& q = P[run[k]];
        size_t e = eoff[k];
        bool stereo = false;
        for (int i = 0; i < q.n; ++i) {
            if (q.has_mp && !q.has_mp[i]) continue;
            hxw[e] = make_float4(q.Xw[3 * i], q.Xw[3 * i + 1], q.Xw[3 * i + 2], q.inv_sigma2[i]);
            huv[e] = make_float2(q.uv[2 * i], q.uv[2 * i + 1]);
            hur[e] = q.u_right ? q.u_right[i] : -1.0f;
            stereo |= hur[e] >= 0.0f;
            ++e;
        }
        DevPoseProb& dp = hp[k];
        dp.xw = reinterpret_cast<const float4*>(d + o_xw) + eoff[k];
        dp.uv = reinterpret_cast<const float2*>(d + o_uv) + eoff[k];
        dp.ur = stereo ? reinterpret_cast<const float*>(d + o_ur) + eoff[k] : nullptr;
        dp.outlier = reinterpret_cast<uint8_t*>(C->d_po_res.p + r_flags) + eoff[k];
        dp.out = reinterpret_cast<float*>(C->d_po_res.p + r_out) + 16 * k;
        dp.n = (int)(eoff[k + 1] - eoff[k]);
        dp.fx = q.fx; dp.fy = q.fy; dp.cx = q.cx; dp.cy = q.cy; dp.bf = q.bf;
        for (int j = 0; j < 12; ++j) dp.T[j] = q.Tcw[j];
    }
    RSC_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, C->stream));
    timing_begin(C, 3);
    RSC_HIP(launch_poseopt(R, reinterpret_cast<const DevPoseProb*>(d + o_probs), C->h_flag + kFaultWord, C->stream));
    timing_begin(C, 4);
    RSC_HIP(hipMemcpyAsync(C->h_po_res.p, C->d_po_res.p, res_bytes, hipMemcpyDeviceToHost, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (int e = take_fault(C)) return e;
    if (C->timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, C->ev[3], C->ev[4]);
        C->last_ms[2] = ms;
    }
    const float* ho = reinterpret_cast<const float*>(C->h_po_res.p + r_out);
    const uint8_t* hf = reinterpret_cast<const uint8_t*>(C->h_po_res.p + r_flags);
    for (int k = 0; k < R; ++k) {
        const int c = run[k];
        const rsc_poseopt_problem& q = P[c];
        rsc_poseopt_result& r = out[c];
        const float* o = ho + 16 * k;
        for (int j = 0; j < 12; ++j) r.Tcw[j] = o[j];
        r.Tcw[12] = r.Tcw[13] = r.Tcw[14] = 0.0f;
        r.Tcw[15] = 1.0f;
        std::memcpy(&r.n_good, o + 12, 4);
        std::memcpy(&r.rounds, o + 13, 4);
        std::memcpy(&r.lm_iterations, o + 14, 4);
        std::memcpy(&r.lm_trials, o + 15, 4);
        if (outlier && outlier[c]) {
            size_t e = eoff[k];
            for (int i = 0; i < q.n; ++i) {
                if (q.has_mp && !q.has_mp[i]) continue;
                outlier[c][i] = hf[e++];
            }
        }
    }
    return RSC_OK;
}

// ---- Optimizer::OptimizeSim3 (src/Optimizer.cpp:1054-1250) ----
int rsc_optimize_sim3_many(rsc_context* C, const rsc_sim3opt_problem* P, int count, rsc_sim3opt_result* out,
                           uint8_t* const* keep) {
    if (!C || count < 0 || (count && (!P || !out))) return RSC_ERR_ARG;
    if (count == 0) return RSC_OK;
    // compaction of the correspondences (Optimizer.cpp:1108-1171), in slot order
    std::vector<int> run;
    std::vector<size_t> moff(1, 0);
    for (int c = 0; c < count; ++c) {
        const rsc_sim3opt_problem& q = P[c];
        if (q.n < 0 || (q.n > 0 && (!q.valid || !q.X1w || !q.X2w || !q.uv1 || !q.uv2 || !q.inv1 || !q.inv2)))
            return RSC_ERR_ARG;
        int m = 0;
        for (int i = 0; i < q.n; ++i) m += q.valid[i] ? 1 : 0;
        if (m > kSim3OptMaxCorr) {
            g_last_error = "more than 8192 correspondences in one OptimizeSim3 problem";
            return RSC_ERR_UNSUPPORTED;
        }
        rsc_sim3opt_result& r = out[c];
        std::memset(&r, 0, sizeof(r));
        r.n_correspondences = m;
        std::memcpy(r.S, q.S, sizeof(r.S));
        if (keep && keep[c]) std::memset(keep[c], 1, (size_t)q.n);
        if (m > 0) {  // m == 0: optimize() has no vertex to optimise, nCorrespondences - nBad < 10 -> 0
            run.push_back(c);
            moff.push_back(moff.back() + (size_t)m);
        }
    }
    const int R = (int)run.size();
    if (R == 0) return RSC_OK;
    const size_t M = moff.back();
    RSC_HIP(hipSetDevice(C->device));
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_e12 = al(sizeof(DevSim3OptProb) * R), o_e21 = o_e12 + al(sizeof(float4) * M);
    const size_t o_uv = o_e21 + al(sizeof(float4) * M), in_bytes = o_uv + al(sizeof(float4) * M);
    const size_t r_keep = al(sizeof(double) * 16 * R), res_bytes = r_keep + al(M);
    if (int e = C->h_so_in.ensure(in_bytes)) return e;
    if (int e = C->d_so_in.ensure(in_bytes)) return e;
    if (int e = C->h_so_res.ensure(res_bytes)) return e;
    if (int e = C->d_so_res.ensure(res_bytes)) return e;
    RSC_HIP(hipStreamSynchronize(C->stream));  // the previous call's copies out of the staging are done
    char* h = C->h_so_in.p;
    char* d = C->d_so_in.p;
    DevSim3OptProb* hp = reinterpret_cast<DevSim3OptProb*>(h);
    float4* h12 = reinterpret_cast<float4*>(h + o_e12);
    float4* h21 = reinterpret_cast<float4*>(h + o_e21);
    float4* huv = reinterpret_cast<float4*>(h + o_uv);
    for (int k = 0; k < R; ++k) {
        const rsc_sim3opt_problem& q = P[run[k]];
        size_t e = moff[k];
        for (int i = 0; i < q.n; ++i) {
            if (!q.valid[i]) continue;
            // P3D1c = R1w*P3D1w + t1w, P3D2c = R2w*P3D2w + t2w (float, Optimizer.cpp:1120-1136)
            const float* a = q.X1w + 3 * (size_t)i;
            const float* b = q.X2w + 3 * (size_t)i;
            float c1[3], c2[3];
            for (int r = 0; r < 3; ++r) {
                c1[r] = q.R1w[3 * r] * a[0] + q.R1w[3 * r + 1] * a[1] + q.R1w[3 * r + 2] * a[2] + q.t1w[r];
                c2[r] = q.R2w[3 * r] * b[0] + q.R2w[3 * r + 1] * b[1] + q.R2w[3 * r + 2] * b[2] + q.t2w[r];
            }
            h12[e] = make_float4(c2[0], c2[1], c2[2], q.inv1[i]);
            h21[e] = make_float4(c1[0], c1[1], c1[2], q.inv2[i]);
            huv[e] = make_float4(q.uv1[2 * i], q.uv1[2 * i + 1], q.uv2[2 * i], q.uv2[2 * i + 1]);
            ++e;
        }
        DevSim3OptProb& dp = hp[k];
        dp.e12 = reinterpret_cast<const float4*>(d + o_e12) + moff[k];
        dp.e21 = reinterpret_cast<const float4*>(d + o_e21) + moff[k];
        dp.uv = reinterpret_cast<const float4*>(d + o_uv) + moff[k];
        dp.keep = reinterpret_cast<uint8_t*>(C->d_so_res.p + r_keep) + moff[k];
        dp.out = reinterpret_cast<double*>(C->d_so_res.p) + 16 * k;
        dp.m = (int)(moff[k + 1] - moff[k]);
        dp.th2 = q.th2;
        const float deltaHuber = std::sqrt(q.th2);  // Optimizer.cpp:1104: float sqrt
        dp.delta = deltaHuber;
        std::memcpy(dp.K1, q.K1, sizeof(dp.K1));
        std::memcpy(dp.K2, q.K2, sizeof(dp.K2));
        std::memcpy(dp.S0, q.S, sizeof(dp.S0));
    }
    // the cooperative form: helper workgroups per pair, one workgroup per CU at most (its LDS)
    const int rpad = (R + 7) / 8 * 8;
    int helpers = C->so_helpers >= 0 ? C->so_helpers : std::min(7, kSoCoopCUs / rpad - 1);
    helpers = std::max(0, helpers);
    for (int k = 0; k < R; ++k) {
        hp[k].cf = nullptr;
        hp[k].cpub = hp[k].cstore = nullptr;
        hp[k].clist = nullptr;
    }
    if (helpers > 0) {
        const size_t o_pub = al(sizeof(SoCoopFlags) * R), o_list = o_pub + al(sizeof(double) * kSoCoopPub * R);
        size_t o_store = o_list + al(sizeof(int) * M), store = 0;
        for (int k = 0; k < R; ++k) {
            const size_t nch = (2 * (moff[k + 1] - moff[k]) + kSoCoopChunk - 1) / kSoCoopChunk;
            store += nch * kSoCoopJd * kSoCoopChunk;
        }
        if (int e = C->d_so_coop.ensure(o_store + sizeof(double) * store)) return e;
        char* w = C->d_so_coop.p;
        size_t so = 0;
        for (int k = 0; k < R; ++k) {
            DevSim3OptProb& dp = hp[k];
            dp.cf = reinterpret_cast<SoCoopFlags*>(w) + k;
            dp.cpub = reinterpret_cast<double*>(w + o_pub) + (size_t)kSoCoopPub * k;
            dp.clist = reinterpret_cast<int*>(w + o_list) + moff[k];
            dp.cstore = reinterpret_cast<double*>(w + o_store) + so;
            so += (2 * (moff[k + 1] - moff[k]) + kSoCoopChunk - 1) / kSoCoopChunk * kSoCoopJd * kSoCoopChunk;
        }
    }
    RSC_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, C->stream));
    if (helpers > 0) RSC_HIP(hipMemsetAsync(C->d_so_coop.p, 0, sizeof(SoCoopFlags) * R, C->stream));
    timing_begin(C, 3);
    RSC_HIP(launch_sim3opt(R, reinterpret_cast<const DevSim3OptProb*>(d), helpers, C->h_flag + kFaultWord, C->stream));
    timing_begin(C, 4);
    RSC_HIP(hipMemcpyAsync(C->h_so_res.p, C->d_so_res.p, res_bytes, hipMemcpyDeviceToHost, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (int e = take_fault(C)) return e;
    if (C->timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, C->ev[3], C->ev[4]);
        C->last_ms[2] = ms;
    }
    const double* ho = reinterpret_cast<const double*>(C->h_so_res.p);
    const uint8_t* hk = reinterpret_cast<const uint8_t*>(C->h_so_res.p + r_keep);
    for (int k = 0; k < R; ++k) {
        const int c = run[k];
        const rsc_sim3opt_problem& q = P[c];
        rsc_sim3opt_result& r = out[c];
        const double* o = ho + 16 * k;
        std::memcpy(r.S, o, 64);
        int32_t st[4];
        std::memcpy(st, o + 8, 16);
        r.n_inliers = st[0];
        r.n_bad = st[1];
        r.lm_iterations = st[2];
        r.lm_trials = st[3];
        if (keep && keep[c]) {
            size_t e = moff[k];
            for (int i = 0; i < q.n; ++i)
                if (q.valid[i]) keep[c][i] = hk[e++];
        }
    }
    return RSC_OK;
}

// ---- RNG parity hook ----

// ---- ORBmatcher::SearchByBoW (src/ORBmatcher.cpp:110-240, :354-488) ----
struct rsc_bow {
    rsc_context* ctx = nullptr;
    int n = 0;
    int n_nodes = 0;
    int n_feat = 0;
    DevBuf<char> mem;            // desc | desc_fv | angle | node_id | node_begin | feat
    size_t off_feat = 0;
    std::vector<uint32_t> feat;  // host copy of the FeatureVector entries (validity flags re-applied)
    DevBow hdr;                  // device pointers of this view (copied into every BowPair)
};

namespace {
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

void flag_invalid(std::vector<uint32_t>& feat, const uint8_t* valid) {
    for (uint32_t& x : feat) {
        x &= ~kBowInvalid;
        if (valid && !valid[x]) x |= kBowInvalid;
    }
}
}  // namespace

int rsc_bow_create(rsc_context* C, const rsc_bow_features* f, rsc_bow** out) {
    if (!C || !f || !out) return RSC_ERR_ARG;
    *out = nullptr;
    const int n = f->n, nn = f->n_nodes;
    if (n < 0 || nn < 0 || (n > 0 && (!f->desc || !f->angle)) || (nn > 0 && (!f->node_id || !f->node_begin || !f->feat)))
        return RSC_ERR_ARG;
    if (n > kBowMaxFeatures || nn > kBowMaxFeatures) {
        g_last_error = "more than 8192 keypoints (or FeatureVector nodes) in one view";
        return RSC_ERR_UNSUPPORTED;
    }
    // FeatureVector invariants the node-parallel walk relies on (DBoW2 transform guarantees them)
    const int nf = nn ? f->node_begin[nn] : 0;
    if (nn && f->node_begin[0] != 0) return RSC_ERR_ARG;
    std::vector<uint8_t> seen((size_t)n, 0);
    for (int k = 0; k < nn; ++k) {
        if (f->node_begin[k + 1] < f->node_begin[k]) return RSC_ERR_ARG;
        if (k && f->node_id[k] <= f->node_id[k - 1]) {
            g_last_error = "FeatureVector node ids must be strictly ascending";
            return RSC_ERR_ARG;
        }
    }
    for (int i = 0; i < nf; ++i) {
        const uint32_t x = f->feat[i];
        if (x >= (uint32_t)n || seen[x]) {
            g_last_error = "FeatureVector feature index out of range or repeated";
            return RSC_ERR_ARG;
        }
        seen[x] = 1;
    }
    std::unique_ptr<rsc_bow> b(new rsc_bow);
    b->ctx = C;
    b->n = n;
    b->n_nodes = nn;
    b->n_feat = nf;
    b->feat.assign(f->feat, f->feat + nf);
    flag_invalid(b->feat, f->valid);
    const size_t o_desc = 0, o_dfv = al256(32 * (size_t)n), o_ang = o_dfv + al256(32 * (size_t)nf);
    const size_t o_id = o_ang + al256(4 * (size_t)n), o_beg = o_id + al256(4 * (size_t)nn);
    const size_t o_feat = o_beg + al256(4 * ((size_t)nn + 1));
    const size_t bytes = o_feat + al256(4 * (size_t)nf);
    RSC_HIP(hipSetDevice(C->device));
    if (int e = b->mem.ensure(bytes)) return e;
    std::vector<char> h(bytes, 0);
    char* d = b->mem.p;
    DevBow hd;
    hd.desc = reinterpret_cast<const uint4*>(d + o_desc);
    hd.desc_fv = reinterpret_cast<const uint4*>(d + o_dfv);
    hd.angle = reinterpret_cast<const float*>(d + o_ang);
    hd.node_id = reinterpret_cast<const uint32_t*>(d + o_id);
    hd.node_begin = reinterpret_cast<const int32_t*>(d + o_beg);
    hd.feat = reinterpret_cast<const uint32_t*>(d + o_feat);
    hd.n = n;
    hd.n_nodes = nn;
    if (n) {
        std::memcpy(h.data() + o_desc, f->desc, 32 * (size_t)n);
        for (int e = 0; e < nf; ++e) std::memcpy(h.data() + o_dfv + 32 * (size_t)e, f->desc + 32 * (size_t)f->feat[e], 32);
        std::memcpy(h.data() + o_ang, f->angle, 4 * (size_t)n);
    }
    if (nn) {
        std::memcpy(h.data() + o_id, f->node_id, 4 * (size_t)nn);
        std::memcpy(h.data() + o_beg, f->node_begin, 4 * ((size_t)nn + 1));
        if (nf) std::memcpy(h.data() + o_feat, b->feat.data(), 4 * (size_t)nf);
    }
    RSC_HIP(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    b->off_feat = o_feat;
    b->hdr = hd;
    *out = b.release();
    return RSC_OK;
}

void rsc_bow_destroy(rsc_bow* b) {
    if (!b) return;
    // searches already enqueued on the context stream may still read the view
    (void)hipStreamSynchronize(b->ctx->stream);
    delete b;
}

int rsc_bow_set_valid(rsc_bow* b, const uint8_t* valid) {
    if (!b || (b->n && !valid)) return RSC_ERR_ARG;
    if (!b->n_feat) return RSC_OK;
    flag_invalid(b->feat, valid);
    RSC_HIP(hipStreamSynchronize(b->ctx->stream));
    RSC_HIP(hipMemcpy(b->mem.p + b->off_feat, b->feat.data(), 4 * (size_t)b->n_feat, hipMemcpyHostToDevice));
    return RSC_OK;
}

namespace {
// pairs[c] = (outer[c], inner[c]); out rows of out_n[c] int32 each
int bow_search(rsc_context* C, bool frame_overload, const rsc_bow* const* outer, const rsc_bow* const* inner,
               int count, float nnratio, int check_ori, int32_t* const* out, int32_t* nmatches) {
    std::vector<size_t> ooff(count + 1, 0), roff(count + 1, 0), joff(count + 1, 0), toff(count + 1, 0);
    for (int c = 0; c < count; ++c) {
        if (!outer[c] || !inner[c] || outer[c]->ctx != C || inner[c]->ctx != C) return RSC_ERR_ARG;
        const int on = frame_overload ? inner[c]->n : outer[c]->n;
        if (on && !out[c]) return RSC_ERR_ARG;
        ooff[c + 1] = ooff[c] + al256(4 * (size_t)on);
        roff[c + 1] = roff[c] + (size_t)outer[c]->n_feat * kBowMaxSegs;
        joff[c + 1] = joff[c] + (size_t)outer[c]->n_nodes;
        toff[c + 1] = toff[c] + ((size_t)outer[c]->n_nodes + (size_t)outer[c]->n_feat / 64 + 1) * kBowMaxSegs;
    }
    const size_t o_pairs = 0, o_cnt = al256(sizeof(BowPair) * count), o_out = o_cnt + al256(4 * (size_t)count);
    const size_t o_rec = o_out + ooff[count], o_nodes = o_rec + al256(16 * roff[count]);
    const size_t o_tasks = o_nodes + al256(16 * joff[count]), o_nt = o_tasks + al256(16 * toff[count]);
    const size_t o_mcp = o_nt + al256(8 * (size_t)count);
    const size_t bytes = o_mcp + al256(2 * roff[count] / kBowMaxSegs);
    const size_t back = o_rec;  // counts + outputs come back
    RSC_HIP(hipSetDevice(C->device));
    if (int e = C->d_bow.ensure(bytes)) return e;
    if (int e = C->h_bow.ensure(back)) return e;
    RSC_HIP(hipStreamSynchronize(C->stream));  // the pinned mirror is free again
    char* d = C->d_bow.p;
    BowPair* hp = reinterpret_cast<BowPair*>(C->h_bow.p + o_pairs);
    for (int c = 0; c < count; ++c) {
        hp[c].outer = outer[c]->hdr;
        hp[c].inner = inner[c]->hdr;  // by value
        hp[c].rec = reinterpret_cast<uint4*>(d + o_rec) + roff[c];
        hp[c].nodes = reinterpret_cast<int4*>(d + o_nodes) + joff[c];
        hp[c].tasks = reinterpret_cast<int4*>(d + o_tasks) + toff[c];
        hp[c].ntasks = reinterpret_cast<int32_t*>(d + o_nt) + 2 * c;
        hp[c].mcp = reinterpret_cast<int16_t*>(d + o_mcp) + roff[c] / kBowMaxSegs;
        hp[c].out = reinterpret_cast<int32_t*>(d + o_out + ooff[c]);
        hp[c].nmatches = reinterpret_cast<int32_t*>(d + o_cnt) + c;
    }
    RSC_HIP(hipMemcpyAsync(d, C->h_bow.p, o_cnt, hipMemcpyHostToDevice, C->stream));
    timing_begin(C, 3);
    int max_nodes = 0;
    for (int c = 0; c < count; ++c) max_nodes = std::max(max_nodes, outer[c]->n_nodes);
    RSC_HIP(launch_bow_search(frame_overload, count, max_nodes, reinterpret_cast<const BowPair*>(d + o_pairs), nnratio,
                              check_ori ? 1 : 0, C->stream));
    timing_begin(C, 4);
    RSC_HIP(hipMemcpyAsync(C->h_bow.p + o_cnt, d + o_cnt, back - o_cnt, hipMemcpyDeviceToHost, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (C->timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, C->ev[3], C->ev[4]);
        C->last_ms[2] = ms;
    }
    const int32_t* hc = reinterpret_cast<const int32_t*>(C->h_bow.p + o_cnt);
    for (int c = 0; c < count; ++c) {
        const int on = frame_overload ? inner[c]->n : outer[c]->n;
        if (on) std::memcpy(out[c], C->h_bow.p + o_out + ooff[c], 4 * (size_t)on);
        if (nmatches) nmatches[c] = hc[c];
    }
    return RSC_OK;
}
}  // namespace


// ---- ORBmatcher::SearchBySim3 (src/ORBmatcher.cpp:948-1170) ----
namespace {
struct S3Blob {
    std::vector<char> h;
    size_t add(const void* p, size_t n) {
        const size_t off = (h.size() + 255) & ~(size_t)255;
        h.resize(off + n);
        if (n) std::memcpy(h.data() + off, p, n);
        return off;
    }
    size_t reserve(size_t n) {
        const size_t off = (h.size() + 255) & ~(size_t)255;
        h.resize(off + n);
        return off;
    }
};

int check_sim3_kf(const rsc_sim3_kf& k) {
    if (k.n < 0 || k.n_levels < 1 || !k.cell_begin || !k.scale_factors) return RSC_ERR_ARG;
    if (k.n > 0 && (!k.kp || !k.octave || !k.desc || !k.mp_state || !k.mp_pos || !k.mp_dmax || !k.mp_dmin ||
                    !k.mp_desc))
        return RSC_ERR_ARG;
    const int cells = kSim3GridCols * kSim3GridRows;
    if (k.cell_begin[0] != 0) return RSC_ERR_ARG;
    for (int c = 0; c < cells; ++c)
        if (k.cell_begin[c + 1] < k.cell_begin[c]) return RSC_ERR_ARG;
    const int nf = k.cell_begin[cells];
    if (nf > 0 && !k.cell_feat) return RSC_ERR_ARG;
    for (int e = 0; e < nf; ++e)
        if (k.cell_feat[e] < 0 || k.cell_feat[e] >= k.n) {
            g_last_error = "mGrid index out of range";
            return RSC_ERR_ARG;
        }
    return 0;
}
}  // namespace

struct rsc_kfview {
    rsc_context* ctx = nullptr;
    int n = 0;
    DevBuf<char> mem;  // DevSim3KF header | kp | octave | desc | grid | scales | MapPoints
    const DevSim3KF* hdr = nullptr;
    // host copies of what OptimizeSim3 reads (the gated loop events build its problem from them)
    std::vector<float> kp, mp_pos, inv_level_sigma2;
    std::vector<int32_t> octave;
    std::vector<uint8_t> mp_state;
    float R[9], t[3], K[4];
};

int rsc_kfview_create(rsc_context* C, const rsc_sim3_kf* k, rsc_kfview** out) {
    if (!C || !k || !out) return RSC_ERR_ARG;
    *out = nullptr;
    if (int e = check_sim3_kf(*k)) return e;
    const int cells = kSim3GridCols * kSim3GridRows;
    const size_t n = (size_t)k->n, nf = (size_t)k->cell_begin[cells];
    // two passes over the same layout: sizes, then the copy into one host image
    S3Blob b;
    const size_t o_hdr = b.reserve(sizeof(DevSim3KF));
    const size_t o_kp = b.add(k->kp, 8 * n), o_oct = b.add(k->octave, 4 * n), o_desc = b.add(k->desc, 32 * n);
    const size_t o_cb = b.add(k->cell_begin, 4 * (size_t)(cells + 1)), o_cf = b.add(k->cell_feat, 4 * nf);
    const size_t o_sc = b.add(k->scale_factors, 4 * (size_t)k->n_levels), o_st = b.add(k->mp_state, n);
    const size_t o_pos = b.add(k->mp_pos, 12 * n), o_mx = b.add(k->mp_dmax, 4 * n), o_mn = b.add(k->mp_dmin, 4 * n);
    const size_t o_md = b.add(k->mp_desc, 32 * n);
    std::unique_ptr<rsc_kfview> v(new rsc_kfview);
    v->ctx = C;
    v->n = k->n;
    RSC_HIP(hipSetDevice(C->device));
    if (int e = v->mem.ensure(b.h.size())) return e;
    char* d = v->mem.p;
    DevSim3KF h;
    h.kp = reinterpret_cast<const float2*>(d + o_kp);
    h.octave = reinterpret_cast<const int32_t*>(d + o_oct);
    h.desc = reinterpret_cast<const uint4*>(d + o_desc);
    h.cell_begin = reinterpret_cast<const int32_t*>(d + o_cb);
    h.cell_feat = reinterpret_cast<const int32_t*>(d + o_cf);
    h.scale = reinterpret_cast<const float*>(d + o_sc);
    h.mp_state = reinterpret_cast<const uint8_t*>(d + o_st);
    h.mp_pos = reinterpret_cast<const float*>(d + o_pos);
    h.mp_dmax = reinterpret_cast<const float*>(d + o_mx);
    h.mp_dmin = reinterpret_cast<const float*>(d + o_mn);
    h.mp_desc = reinterpret_cast<const uint4*>(d + o_md);
    h.min_x = k->min_x; h.max_x = k->max_x; h.min_y = k->min_y; h.max_y = k->max_y;
    h.gw_inv = k->grid_w_inv; h.gh_inv = k->grid_h_inv;
    h.fx = k->fx; h.fy = k->fy; h.cx = k->cx; h.cy = k->cy;
    h.log_sf = k->log_scale_factor;
    std::memcpy(h.R, k->Rcw, sizeof(h.R));
    std::memcpy(h.t, k->tcw, sizeof(h.t));
    h.n = k->n;
    h.n_levels = k->n_levels;
    std::memcpy(b.h.data() + o_hdr, &h, sizeof(h));
    RSC_HIP(hipMemcpy(d, b.h.data(), b.h.size(), hipMemcpyHostToDevice));
    v->hdr = reinterpret_cast<const DevSim3KF*>(d + o_hdr);
    v->kp.assign(k->kp, k->kp + 2 * n);
    v->octave.assign(k->octave, k->octave + n);
    v->mp_state.assign(k->mp_state, k->mp_state + n);
    v->mp_pos.assign(k->mp_pos, k->mp_pos + 3 * n);
    // mvLevelSigma2[l] = mvScaleFactor[l]^2, mvInvLevelSigma2[l] = 1.0f / mvLevelSigma2[l] (float,
    // ORBextractor's constructor; KeyFrame copies them from the Frame)
    v->inv_level_sigma2.resize((size_t)k->n_levels);
    for (int l = 0; l < k->n_levels; ++l) {
        const float s2 = k->scale_factors[l] * k->scale_factors[l];
        v->inv_level_sigma2[l] = 1.0f / s2;
    }
    std::memcpy(v->R, k->Rcw, sizeof(v->R));
    std::memcpy(v->t, k->tcw, sizeof(v->t));
    v->K[0] = k->fx; v->K[1] = k->fy; v->K[2] = k->cx; v->K[3] = k->cy;
    *out = v.release();
    return RSC_OK;
}

void rsc_kfview_destroy(rsc_kfview* v) {
    if (!v) return;
    (void)hipStreamSynchronize(v->ctx->stream);
    delete v;
}

int rsc_search_by_sim3_many(rsc_context* C, rsc_kfview* const* kf1, rsc_kfview* const* kf2, int count,
                            const float* R12, const float* t12, float th, const int32_t* const* matched12,
                            int32_t* const* out12, int32_t* nfound) {
    if (!C || count < 0 || (count && (!kf1 || !kf2 || !R12 || !t12 || !matched12 || !out12))) return RSC_ERR_ARG;
    if (count == 0) return RSC_OK;
    int max_points = 0;
    for (int c = 0; c < count; ++c) {
        if (!kf1[c] || !kf2[c] || kf1[c]->ctx != C || kf2[c]->ctx != C) return RSC_ERR_ARG;
        if (kf1[c]->n && (!matched12[c] || !out12[c])) return RSC_ERR_ARG;
        max_points = std::max(max_points, std::max(kf1[c]->n, kf2[c]->n));
    }
    // layout: pair table | vbAlreadyMatched1/2 flags (host-derived, :972-984) | vnMatch1/2 scratch |
    // outputs (the only part that comes back)
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    std::vector<size_t> o_a1(count), o_a2(count), o_m1(count), o_m2(count), o_out(count), o_nf(count);
    size_t off = al(sizeof(Sim3MatchPair) * count);
    for (int c = 0; c < count; ++c) {
        o_a1[c] = off; off = al(off + std::max(kf1[c]->n, 1));
        o_a2[c] = off; off = al(off + std::max(kf2[c]->n, 1));
    }
    const size_t up = off;
    for (int c = 0; c < count; ++c) {
        o_m1[c] = off; off = al(off + 4 * (size_t)std::max(kf1[c]->n, 1));
        o_m2[c] = off; off = al(off + 4 * (size_t)std::max(kf2[c]->n, 1));
    }
    const size_t back = off;
    for (int c = 0; c < count; ++c) {
        o_out[c] = off; off = al(off + 4 * (size_t)std::max(kf1[c]->n, 1));
        o_nf[c] = off; off += 4;
    }
    const size_t bytes = al(off);
    RSC_HIP(hipSetDevice(C->device));
    if (int e = C->d_s3m.ensure(bytes)) return e;
    if (int e = C->h_s3m.ensure(bytes)) return e;
    RSC_HIP(hipStreamSynchronize(C->stream));  // the pinned mirror is free again
    char* h = C->h_s3m.p;
    char* d = C->d_s3m.p;
    for (int c = 0; c < count; ++c) {
        const int n1 = kf1[c]->n, n2 = kf2[c]->n;
        uint8_t* a1 = reinterpret_cast<uint8_t*>(h + o_a1[c]);
        uint8_t* a2 = reinterpret_cast<uint8_t*>(h + o_a2[c]);
        std::memset(a1, 0, (size_t)std::max(n1, 1));
        std::memset(a2, 0, (size_t)std::max(n2, 1));
        for (int i = 0; i < n1; ++i) {
            const int32_t m = matched12[c][i];
            if (m < -2 || m >= n2) return RSC_ERR_ARG;
            if (m == -1) continue;
            a1[i] = 1;
            if (m >= 0) a2[m] = 1;
        }
        Sim3MatchPair p;
        p.k1 = kf1[c]->hdr;
        p.k2 = kf2[c]->hdr;
        std::memcpy(p.R12, R12 + 9 * c, sizeof(p.R12));
        std::memcpy(p.t12, t12 + 3 * c, sizeof(p.t12));
        p.already1 = reinterpret_cast<const uint8_t*>(d + o_a1[c]);
        p.already2 = reinterpret_cast<const uint8_t*>(d + o_a2[c]);
        p.m1 = reinterpret_cast<int32_t*>(d + o_m1[c]);
        p.m2 = reinterpret_cast<int32_t*>(d + o_m2[c]);
        p.out = reinterpret_cast<int32_t*>(d + o_out[c]);
        p.nfound = reinterpret_cast<int32_t*>(d + o_nf[c]);
        std::memcpy(h + sizeof(Sim3MatchPair) * c, &p, sizeof(p));
    }
    RSC_HIP(hipMemcpyAsync(d, h, up, hipMemcpyHostToDevice, C->stream));
    timing_begin(C, 3);
    RSC_HIP(launch_search_by_sim3(count, max_points, reinterpret_cast<const Sim3MatchPair*>(d), th, C->stream));
    timing_begin(C, 4);
    RSC_HIP(hipMemcpyAsync(h + back, d + back, bytes - back, hipMemcpyDeviceToHost, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (C->timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, C->ev[3], C->ev[4]);
        C->last_ms[2] = ms;
    }
    for (int c = 0; c < count; ++c) {
        if (kf1[c]->n) std::memcpy(out12[c], h + o_out[c], 4 * (size_t)kf1[c]->n);
        if (nfound) std::memcpy(&nfound[c], h + o_nf[c], 4);
    }
    return RSC_OK;
}

// ------------------------------------------------------------------------------------------------
// KeyFrameDatabase (rsc_kfdb.h)
// ------------------------------------------------------------------------------------------------
struct rsc_kfdb {
    rsc_context* ctx = nullptr;
    int cap = 0, max_words = 0;
    int hw = 0;  // slots in use: 1 + the highest slot ever added or referenced (queries sweep [0, hw))
    uint32_t vocab = 0;
    uint32_t next_seq = 1;
    std::vector<uint8_t> present;
    PinBuf<int32_t> covis_h, covis_n_h;  // host mirror of the covisibility table (pinned: the copy kernel reads it)
    DevBuf<uint32_t> ids, seq;
    DevBuf<double> vals;
    DevBuf<char> qbuf;  // the query BowVector: ids | vals (8-aligned), one upload per query
    DevBuf<int32_t> len, covis, covis_n, words, list, scored, best, tmp, counters, out;
    DevBuf<unsigned long long> query, key;
    DevBuf<float> score, sc, acc, tscore;
    DevBuf<uint8_t> conn;
    PinBuf<char> stage;  // query upload | candidates download
    void touch(int s) { hw = std::max(hw, s + 1); }
    DevKFDB dev() const {
        DevKFDB d;
        d.cap = hw;  // the kernels' sweep bound; the arrays are sized (and strided) by cap
        d.max_words = max_words;
        d.vocab = vocab;
        d.ids = ids.p;
        d.vals = vals.p;
        d.len = len.p;
        d.seq = seq.p;
        d.covis = covis.p;
        d.covis_n = covis_n.p;
        for (int t = 0; t < 2; ++t) {
            d.query[t] = query.p + (size_t)t * cap;
            d.words[t] = words.p + (size_t)t * cap;
            d.score[t] = score.p + (size_t)t * cap;
        }
        d.tscore = tscore.p;
        d.list = list.p;
        d.key = key.p;
        d.scored = scored.p;
        d.sc = sc.p;
        d.acc = acc.p;
        d.best = best.p;
        d.tmp = tmp.p;
        d.counters = counters.p;
        d.out = out.p;
        d.qids = reinterpret_cast<const uint32_t*>(qbuf.p);
        d.qvals = reinterpret_cast<const double*>(qbuf.p);  // set per query (after the ids)
        d.conn = conn.p;
        return d;
    }
};

namespace {
int check_bow_vector(const rsc_kfdb* db, int n, const uint32_t* id, const double* val) {
    if (n < 0 || n > db->max_words || (n && (!id || !val))) return RSC_ERR_ARG;
    for (int i = 1; i < n; ++i)
        if (id[i] <= id[i - 1]) return RSC_ERR_ARG;  // a BowVector (std::map) is strictly ascending
    if (n && id[n - 1] >= db->vocab) return RSC_ERR_ARG;  // not a word of the vocabulary
    return RSC_OK;
}
}  // namespace

int rsc_kfdb_create(rsc_context* C, uint32_t vocab_words, int capacity, int max_words, rsc_kfdb** out) {
    if (!C || !out || vocab_words == 0 || vocab_words > (1u << 30) || capacity <= 0 || max_words <= 0 ||
        max_words > kKfdbMaxWords)
        return RSC_ERR_ARG;
    *out = nullptr;
    std::unique_ptr<rsc_kfdb> db(new rsc_kfdb);
    db->ctx = C;
    db->cap = capacity;
    db->max_words = max_words;
    db->vocab = vocab_words;
    db->present.assign(capacity, 0);
    RSC_HIP(hipSetDevice(C->device));
    const size_t K = (size_t)capacity;
    int e = 0;
    if ((e = db->covis_h.ensure(K * kKfdbCovis)) || (e = db->covis_n_h.ensure(K))) return e;
    std::memset(db->covis_h.p, 0, K * kKfdbCovis * sizeof(int32_t));
    std::memset(db->covis_n_h.p, 0, K * sizeof(int32_t));
    if ((e = db->ids.ensure(K * max_words)) || (e = db->vals.ensure(K * max_words)) || (e = db->len.ensure(K)) ||
        (e = db->seq.ensure(K)) || (e = db->covis.ensure(K * kKfdbCovis)) || (e = db->covis_n.ensure(K)) ||
        (e = db->query.ensure(2 * K)) || (e = db->words.ensure(2 * K)) || (e = db->score.ensure(2 * K)) ||
        (e = db->list.ensure(K)) || (e = db->key.ensure(K)) || (e = db->scored.ensure(K)) || (e = db->sc.ensure(K)) ||
        (e = db->acc.ensure(K)) || (e = db->tscore.ensure(K)) || (e = db->best.ensure(K)) || (e = db->tmp.ensure(K)) || (e = db->counters.ensure(4)) ||
        (e = db->out.ensure(K + 1)) || (e = db->qbuf.ensure(16 * (size_t)max_words + 16)) ||
        (e = db->conn.ensure(K)))
        return e;
    const size_t stage = std::max((size_t)max_words * 16 + 16 + K, (K + 1) * 4);
    if ((e = db->stage.ensure(stage))) return e;
    // KeyFrame.cpp:15: query ids and word counts start at 0; the scores (uninitialised in the
    // reference) are defined as 0
    RSC_HIP(hipMemsetAsync(db->counters.p, 0, 16, C->stream));  // the finish kernel re-zeroes n_list
    RSC_HIP(hipMemsetAsync(db->len.p, 0, 4 * K, C->stream));
    RSC_HIP(hipMemsetAsync(db->covis_n.p, 0, 4 * K, C->stream));
    RSC_HIP(hipMemsetAsync(db->covis.p, 0, 4 * K * kKfdbCovis, C->stream));  // padded rows read slot 0
    RSC_HIP(hipMemsetAsync(db->query.p, 0, 16 * K, C->stream));
    RSC_HIP(hipMemsetAsync(db->words.p, 0, 8 * K, C->stream));
    RSC_HIP(hipMemsetAsync(db->score.p, 0, 8 * K, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    *out = db.release();
    return RSC_OK;
}

void rsc_kfdb_destroy(rsc_kfdb* db) {
    if (!db) return;
    (void)hipStreamSynchronize(db->ctx->stream);
    delete db;
}

int rsc_kfdb_add(rsc_kfdb* db, int kf, int n, const uint32_t* id, const double* val) {
    if (!db || kf < 0 || kf >= db->cap) return RSC_ERR_ARG;
    if (int e = check_bow_vector(db, n, id, val)) return e;
    if (db->present[kf]) return RSC_ERR_UNSUPPORTED;
    rsc_context* C = db->ctx;
    RSC_HIP(hipSetDevice(C->device));
    const size_t o = (size_t)kf * db->max_words;
    const uint32_t s = db->next_seq++;
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (n) {
        RSC_HIP(hipMemcpy(db->ids.p + o, id, 4 * (size_t)n, hipMemcpyHostToDevice));
        RSC_HIP(hipMemcpy(db->vals.p + o, val, 8 * (size_t)n, hipMemcpyHostToDevice));
    }
    RSC_HIP(hipMemcpy(db->seq.p + kf, &s, 4, hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(db->len.p + kf, &n, 4, hipMemcpyHostToDevice));
    db->present[kf] = 1;
    db->touch(kf);
    return RSC_OK;
}

int rsc_kfdb_erase(rsc_kfdb* db, int kf) {
    if (!db || kf < 0 || kf >= db->cap) return RSC_ERR_ARG;
    if (!db->present[kf]) return RSC_OK;
    RSC_HIP(hipSetDevice(db->ctx->device));
    RSC_HIP(hipMemsetAsync(db->len.p + kf, 0, 4, db->ctx->stream));
    RSC_HIP(hipStreamSynchronize(db->ctx->stream));
    db->present[kf] = 0;
    return RSC_OK;
}

int rsc_kfdb_release(rsc_kfdb* db, int kf) {
    if (!db || kf < 0 || kf >= db->cap) return RSC_ERR_ARG;
    rsc_context* C = db->ctx;
    RSC_HIP(hipSetDevice(C->device));
    const size_t K = (size_t)db->cap;
    RSC_HIP(hipMemsetAsync(db->len.p + kf, 0, 4, C->stream));
    for (int t = 0; t < 2; ++t) {
        RSC_HIP(hipMemsetAsync(db->query.p + t * K + kf, 0, 8, C->stream));
        RSC_HIP(hipMemsetAsync(db->words.p + t * K + kf, 0, 4, C->stream));
        RSC_HIP(hipMemsetAsync(db->score.p + t * K + kf, 0, 4, C->stream));
    }
    RSC_HIP(hipMemsetAsync(db->covis.p + (size_t)kf * kKfdbCovis, 0, 4 * kKfdbCovis, C->stream));
    RSC_HIP(hipMemsetAsync(db->covis_n.p + kf, 0, 4, C->stream));
    RSC_HIP(hipStreamSynchronize(C->stream));
    std::fill(db->covis_h.p + (size_t)kf * kKfdbCovis, db->covis_h.p + (size_t)(kf + 1) * kKfdbCovis, 0);
    db->covis_n_h.p[kf] = 0;
    db->present[kf] = 0;
    return RSC_OK;
}

int rsc_kfdb_clear(rsc_kfdb* db) {
    if (!db) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(db->ctx->device));
    RSC_HIP(hipMemsetAsync(db->len.p, 0, 4 * (size_t)db->cap, db->ctx->stream));
    RSC_HIP(hipStreamSynchronize(db->ctx->stream));
    std::fill(db->present.begin(), db->present.end(), 0);
    return RSC_OK;
}

int rsc_kfdb_set_covisibility(rsc_kfdb* db, int kf, int n, const int32_t* best) {
    if (!db || kf < 0 || kf >= db->cap || n < 0 || n > kKfdbCovis || (n && !best)) return RSC_ERR_ARG;
    const int32_t nn = n;
    // one covisibility row padded to kKfdbCovis entries (the _many form reads rows of that stride)
    std::array<int32_t, kKfdbCovis> row{};
    for (int i = 0; i < n && i < kKfdbCovis; ++i) row[i] = best[i];
    return rsc_kfdb_set_covisibility_many(db, 1, &kf, &nn, row.data());
}

int rsc_kfdb_set_covisibility_many(rsc_kfdb* db, int count, const int32_t* kf, const int32_t* n,
                                   const int32_t* best) {
    if (!db || count < 0 || (count && (!kf || !n || !best))) return RSC_ERR_ARG;
    for (int c = 0; c < count; ++c) {  // validate everything before touching the mirror
        if (kf[c] < 0 || kf[c] >= db->cap || n[c] < 0 || n[c] > kKfdbCovis) return RSC_ERR_ARG;
        for (int i = 0; i < n[c]; ++i)
            if (best[(size_t)c * kKfdbCovis + i] < 0 || best[(size_t)c * kKfdbCovis + i] >= db->cap) return RSC_ERR_ARG;
    }
    // a copy of the mirror from the previous call may still be in flight
    RSC_HIP(hipSetDevice(db->ctx->device));
    RSC_HIP(hipStreamSynchronize(db->ctx->stream));
    // rows whose content changed go up as one span [lo, hi] (the mirror keeps the rest)
    int lo = INT32_MAX, hi = -1;
    for (int c = 0; c < count; ++c) {
        int32_t* row = db->covis_h.p + (size_t)kf[c] * kKfdbCovis;
        bool changed = db->covis_n_h.p[kf[c]] != n[c];
        for (int i = 0; i < kKfdbCovis; ++i) {
            const int32_t v = i < n[c] ? best[(size_t)c * kKfdbCovis + i] : 0;
            changed |= row[i] != v;
            row[i] = v;
            if (i < n[c]) db->touch(v);
        }
        db->covis_n_h.p[kf[c]] = n[c];
        db->touch(kf[c]);
        if (changed) {
            lo = std::min(lo, kf[c]);
            hi = std::max(hi, kf[c]);
        }
    }
    if (hi < 0) return RSC_OK;
    // two copy kernels on the context stream (stream order puts them before the next query's
    // kernels; the next call that rewrites the mirror synchronises first)
    const size_t rows = (size_t)(hi - lo + 1);
    RSC_HIP(launch_copy_bytes(db->covis_h.p + (size_t)lo * kKfdbCovis, db->covis.p + (size_t)lo * kKfdbCovis,
                              4 * kKfdbCovis * rows, db->ctx->stream));
    RSC_HIP(launch_copy_bytes(db->covis_n_h.p + lo, db->covis_n.p + lo, 4 * rows, db->ctx->stream));
    return RSC_OK;
}

namespace {
int kfdb_query(rsc_kfdb* db, uint64_t qid, int n, const uint32_t* id, const double* val, int loop, int n_conn,
               const int32_t* conn, float min_score, int32_t* cand, int32_t* n_cand) {
    if (!db || !cand || !n_cand) return RSC_ERR_ARG;
    if (int e = check_bow_vector(db, n, id, val)) return e;
    if (loop && (n_conn < 0 || (n_conn && !conn))) return RSC_ERR_ARG;
    rsc_context* C = db->ctx;
    const size_t K = (size_t)db->cap;
    RSC_HIP(hipSetDevice(C->device));
    RSC_HIP(hipStreamSynchronize(C->stream));  // the staging buffer is free again
    char* h = db->stage.p;
    const size_t vo = (4 * (size_t)n + 7) & ~(size_t)7;  // vals offset in the packed query
    if (n) {
        std::memcpy(h, id, 4 * (size_t)n);
        std::memcpy(h + vo, val, 8 * (size_t)n);
        RSC_HIP(launch_copy_bytes(h, db->qbuf.p, vo + 8 * (size_t)n, C->stream));
    }
    if (loop) {
        for (int i = 0; i < n_conn; ++i)
            if (conn[i] < 0 || conn[i] >= db->cap) return RSC_ERR_ARG;
        for (int i = 0; i < n_conn; ++i) db->touch(conn[i]);
    }
    if (db->hw == 0) {  // nothing was ever added: no candidates, no state to update
        *n_cand = 0;
        return RSC_OK;
    }
    const size_t H = (size_t)db->hw;  // the sweeps and the copies cover the slots in use only
    if (loop) {
        uint8_t* m = reinterpret_cast<uint8_t*>(h + 16 * (size_t)db->max_words + 16);
        std::memset(m, 0, H);
        for (int i = 0; i < n_conn; ++i) m[conn[i]] = 1;
        RSC_HIP(launch_copy_bytes(m, db->conn.p, H, C->stream));
    }
    KfdbQuery q;
    q.id = (unsigned long long)qid;
    q.n = n;
    q.loop = loop;
    q.min_score = min_score;
    timing_begin(C, 3);
    DevKFDB d = db->dev();
    d.qvals = reinterpret_cast<const double*>(db->qbuf.p + vo);
    RSC_HIP(launch_kfdb_query(d, q, C->stream));
    timing_begin(C, 4);
    RSC_HIP(launch_copy_bytes(db->out.p, h, 4 * (H + 1), C->stream));  // written into pinned memory
    RSC_HIP(hipStreamSynchronize(C->stream));
    if (C->timing) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, C->ev[3], C->ev[4]);
        C->last_ms[2] = ms;
    }
    const int32_t* o = reinterpret_cast<const int32_t*>(h);
    *n_cand = o[0];
    std::memcpy(cand, o + 1, 4 * (size_t)o[0]);
    return RSC_OK;
}
}  // namespace

int rsc_kfdb_detect_relocalization(rsc_kfdb* db, uint64_t frame_id, int n, const uint32_t* id, const double* val,
                                   int32_t* cand, int32_t* n_cand) {
    return kfdb_query(db, frame_id, n, id, val, 0, 0, nullptr, 0.0f, cand, n_cand);
}

int rsc_kfdb_detect_loop(rsc_kfdb* db, uint64_t kf_id, int n, const uint32_t* id, const double* val, int n_conn,
                         const int32_t* conn, float min_score, int32_t* cand, int32_t* n_cand) {
    return kfdb_query(db, kf_id, n, id, val, 1, n_conn, conn, min_score, cand, n_cand);
}

int rsc_kfdb_state(rsc_kfdb* db, int kf, uint64_t* q, int32_t* w, float* s) {
    if (!db || kf < 0 || kf >= db->cap || !q || !w || !s) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(db->ctx->device));
    RSC_HIP(hipStreamSynchronize(db->ctx->stream));
    for (int t = 0; t < 2; ++t) {
        unsigned long long qq = 0;
        RSC_HIP(hipMemcpy(&qq, db->query.p + (size_t)t * db->cap + kf, 8, hipMemcpyDeviceToHost));
        q[t] = qq;
        RSC_HIP(hipMemcpy(&w[t], db->words.p + (size_t)t * db->cap + kf, 4, hipMemcpyDeviceToHost));
        RSC_HIP(hipMemcpy(&s[t], db->score.p + (size_t)t * db->cap + kf, 4, hipMemcpyDeviceToHost));
    }
    return RSC_OK;
}

int rsc_diag_kfdb_stamps(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 4096 * 4) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(C->device));
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_kfdb_stamps(out));
    return RSC_OK;
}

int rsc_diag_poseopt_phases(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 64 * 8) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(C->device));
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_poseopt_phases(out, cap >= 64 * 24));
    return RSC_OK;
}

int rsc_diag_sim3opt_phases(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 64 * 8) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(C->device));
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_sim3opt_phases(out));
    return RSC_OK;
}

int rsc_diag_refine_phase_stamps(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 64 * 24) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_refine_stamps(out));
    return RSC_OK;
}

int rsc_diag_solve_phase_stamps(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 3 * 4096 * 8) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_solve_stamps(out));
    return RSC_OK;
}

int rsc_diag_mlpnp_phase_stamps(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 8192 * 8) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_ml_stamps(out));
    return RSC_OK;
}

int rsc_diag_bow_phase_stamps(rsc_context* C, uint64_t* out, int cap) {
    if (!C || !out || cap < 0) return RSC_ERR_ARG;
    RSC_HIP(hipStreamSynchronize(C->stream));
    RSC_HIP(read_bow_stamps(out, cap));
    return RSC_OK;
}

int rsc_search_by_bow_frame_many(rsc_context* C, rsc_bow* const* kfs, int count, const rsc_bow* frame, float nnratio,
                                 int check_orientation, int32_t* const* matches, int32_t* nmatches) {
    if (!C || count < 0 || (count && (!kfs || !frame || !matches))) return RSC_ERR_ARG;
    if (count == 0) return RSC_OK;
    std::vector<const rsc_bow*> inner((size_t)count, frame);
    return bow_search(C, true, kfs, inner.data(), count, nnratio, check_orientation, matches, nmatches);
}

int rsc_search_by_bow_kf_many(rsc_context* C, const rsc_bow* kf1, rsc_bow* const* kf2s, int count, float nnratio,
                              int check_orientation, int32_t* const* matches12, int32_t* nmatches) {
    if (!C || count < 0 || (count && (!kf1 || !kf2s || !matches12))) return RSC_ERR_ARG;
    if (count == 0) return RSC_OK;
    std::vector<const rsc_bow*> outer((size_t)count, kf1);
    return bow_search(C, false, outer.data(), kf2s, count, nnratio, check_orientation, matches12, nmatches);
}

int rsc_rand_stream(rsc_context* C, uint32_t seed, int n, int32_t* out) {
    if (!C || !out || n < 0) return RSC_ERR_ARG;
    if (n == 0) return RSC_OK;
    RSC_HIP(hipSetDevice(C->device));
    RngStream r;
    r.seed(seed);
    int done = 0;
    DevBuf<int32_t> d;
    if (int e = d.ensure(std::min(n, 8192))) return e;
    while (done < n) {
        const int chunk = std::min(8192, n - done);
        r.ensure(C->table, chunk);
        RSC_HIP(launch_rng_stream(C->d_table.p, r.window, r.g, chunk, d.p, C->stream));
        RSC_HIP(hipMemcpyAsync(out + done, d.p, (size_t)chunk * 4, hipMemcpyDeviceToHost, C->stream));
        RSC_HIP(hipStreamSynchronize(C->stream));
        r.g += chunk;
        done += chunk;
    }
    return RSC_OK;
}

// ---- batched state helpers ----
// ---- Shared rand() stream (Q3) ----
int rsc_stream_create(rsc_context* C, uint32_t seed, rsc_stream** out) {
    if (!C || !out) return RSC_ERR_ARG;
    rsc_stream* s = new rsc_stream();
    s->ctx = C;
    s->st.seed(seed);
    *out = s;
    return RSC_OK;
}

void rsc_stream_destroy(rsc_stream* s) { delete s; }

int rsc_stream_skip(rsc_stream* s, int64_t n) {
    if (!s || n < 0) return RSC_ERR_ARG;
    s->st.advance(s->ctx->table, n);
    s->position += n;
    return RSC_OK;
}

int rsc_stream_position(const rsc_stream* s, int64_t* out) {
    if (!s || !out) return RSC_ERR_ARG;
    *out = s->position;
    return RSC_OK;
}

int rsc_stream_peek(rsc_stream* s, int n, int32_t* out) {
    if (!s || !out || n < 0) return RSC_ERR_ARG;
    if (n == 0) return RSC_OK;
    rsc_context* C = s->ctx;
    RSC_HIP(hipSetDevice(C->device));
    RngStream r = s->st;
    DevBuf<int32_t> d;
    if (int e = d.ensure(std::min(n, 8192))) return e;
    for (int done = 0; done < n;) {
        const int chunk = std::min(8192, n - done);
        r.ensure(C->table, chunk);
        RSC_HIP(launch_rng_stream(C->d_table.p, r.window, r.g, chunk, d.p, C->stream));
        RSC_HIP(hipMemcpyAsync(out + done, d.p, (size_t)chunk * 4, hipMemcpyDeviceToHost, C->stream));
        RSC_HIP(hipStreamSynchronize(C->stream));
        r.g += chunk;
        done += chunk;
    }
    return RSC_OK;
}

int rsc_pnp_bind_stream(rsc_pnp* s, rsc_stream* stream) { return bind_stream(s, stream); }

int rsc_sim3_bind_stream(rsc_sim3* s, rsc_stream* stream) { return bind_stream(s, stream); }

int rsc_mlpnp_bind_stream(rsc_mlpnp* s, rsc_stream* stream) { return bind_stream(s, stream); }

int rsc_pnp_reset_many(rsc_pnp* const* s, int count, const uint32_t* seeds) {
    if (count < 0 || (count && (!s || !seeds))) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i) {
        if (!s[i]) return RSC_ERR_ARG;
        reset_solver(s[i], seeds[i]);
        s[i]->last_kind = 0;
    }
    return RSC_OK;
}

int rsc_pnp_set_ransac_parameters_many(rsc_pnp* const* s, int count, double probability, int min_inliers,
                                       int max_iterations, int min_set, float epsilon, float th2) {
    if (count < 0 || (count && !s)) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i) {
        if (!s[i]) return RSC_ERR_ARG;
        pnp_set_params(s[i]->st, probability, min_inliers, max_iterations, min_set, epsilon, th2);
    }
    return RSC_OK;
}

int rsc_sim3_reset_many(rsc_sim3* const* s, int count, const uint32_t* seeds) {
    if (count < 0 || (count && (!s || !seeds))) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i) {
        if (!s[i]) return RSC_ERR_ARG;
        reset_solver(s[i], seeds[i]);
    }
    return RSC_OK;
}

int rsc_sim3_set_ransac_parameters_many(rsc_sim3* const* s, int count, double probability, int min_inliers,
                                        int max_iterations) {
    if (count < 0 || (count && !s)) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i) {
        if (!s[i]) return RSC_ERR_ARG;
        sim3_set_params(s[i]->st, probability, min_inliers, max_iterations);
    }
    return RSC_OK;
}

// ---- MLPnP ----
int rsc_mlpnp_create(rsc_context* C, const rsc_pnp_problem* pb, uint32_t seed, rsc_mlpnp** out) {
    if (!C || !pb || !out || pb->n < 0 || pb->n_points < pb->n) return RSC_ERR_ARG;
    if (pb->n > 0 && (!pb->p2d || !pb->p3dw || !pb->sigma2)) return RSC_ERR_ARG;
    *out = nullptr;
    RSC_HIP(hipSetDevice(C->device));
    std::unique_ptr<rsc_mlpnp> S(new rsc_mlpnp());
    S->ctx = C;
    MLState& s = S->st;
    s.N = pb->n;
    s.N_points = pb->n_points;
    S->fx = pb->fx; S->fy = pb->fy; S->cx = pb->cx; S->cy = pb->cy;
    s.kp_index.resize(pb->n);
    for (int i = 0; i < pb->n; ++i) s.kp_index[i] = pb->kp_index ? pb->kp_index[i] : i;
    s.reset(seed);
    const int n = std::max(pb->n, 1);
    S->words = (n + 63) / 64;
    std::vector<float4> pts(n);
    std::vector<float2> uv(n), brg(n);
    for (int i = 0; i < pb->n; ++i) {
        pts[i] = make_float4(pb->p3dw[3 * i], pb->p3dw[3 * i + 1], pb->p3dw[3 * i + 2], pb->sigma2[i]);
        uv[i] = make_float2(pb->p2d[2 * i], pb->p2d[2 * i + 1]);
        // bearing (x, y, 1): float arithmetic as MLPnPsolver.cpp:32-33
        const float bx = (pb->p2d[2 * i] - pb->cx) / pb->fx;
        const float by = (pb->p2d[2 * i + 1] - pb->cy) / pb->fy;
        brg[i] = make_float2(bx, by);
    }
    RSC_HIP(hipMalloc(&S->d_pts, n * sizeof(float4)));
    RSC_HIP(hipMalloc(&S->d_uv, n * sizeof(float2)));
    RSC_HIP(hipMalloc(&S->d_brg, n * sizeof(float2)));
    RSC_HIP(hipMalloc(&S->d_best, S->words * 8));
    RSC_HIP(hipMemcpy(S->d_pts, pts.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(S->d_uv, uv.data(), n * sizeof(float2), hipMemcpyHostToDevice));
    RSC_HIP(hipMemcpy(S->d_brg, brg.data(), n * sizeof(float2), hipMemcpyHostToDevice));
    RSC_HIP(hipMemset(S->d_best, 0, S->words * 8));
    mlpnp_set_params(s, 0.99, 8, 300, 6, 0.4f, 5.991f);  // the ctor's SetRansacParameters() (:52)
    *out = S.release();
    return RSC_OK;
}

void rsc_mlpnp_destroy(rsc_mlpnp* s) { delete s; }

int rsc_mlpnp_set_covariances(rsc_mlpnp* s, const double* cov) {
    if (!s) return RSC_ERR_ARG;
    if (!cov) {
        s->use_cov = false;
        return RSC_OK;
    }
    const int n = s->st.N;
    for (size_t k = 0; k < 9 * (size_t)n; ++k)
        if (!std::isfinite(cov[k])) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(s->ctx->device));
    if (!s->d_cov && n > 0) RSC_HIP(hipMalloc(&s->d_cov, 9 * sizeof(double) * (size_t)n));
    RSC_HIP(hipStreamSynchronize(s->ctx->stream));
    if (n > 0) RSC_HIP(hipMemcpy(s->d_cov, cov, 9 * sizeof(double) * (size_t)n, hipMemcpyHostToDevice));
    s->use_cov = n > 0;
    return RSC_OK;
}

int rsc_mlpnp_set_ransac_parameters(rsc_mlpnp* s, double probability, int min_inliers, int max_iterations,
                                    int min_set, float epsilon, float th2) {
    if (!s) return RSC_ERR_ARG;
    if (min_set < 6 || min_set > 8) {
        g_last_error = "MLPnP min_set outside [6,8] (computePose asserts n > 5, MLPnPsolver.cpp:324)";
        return RSC_ERR_UNSUPPORTED;
    }
    mlpnp_set_params(s->st, probability, min_inliers, max_iterations, min_set, epsilon, th2);
    return RSC_OK;
}

int rsc_mlpnp_set_ransac_parameters_many(rsc_mlpnp* const* s, int count, double probability, int min_inliers,
                                         int max_iterations, int min_set, float epsilon, float th2) {
    for (int i = 0; i < count; ++i)
        if (int e = rsc_mlpnp_set_ransac_parameters(s[i], probability, min_inliers, max_iterations, min_set, epsilon,
                                                    th2))
            return e;
    return RSC_OK;
}

static int mlpnp_iterate_many_impl(rsc_mlpnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                                   uint8_t* const* inliers);

int rsc_mlpnp_iterate_many(rsc_mlpnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                           uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i)
        if (solvers[i] && solvers[i]->stream)
            return bound_iterate_many(solvers, count, n_its, out, inliers, mlpnp_iterate_many_impl);
    return mlpnp_iterate_many_impl(solvers, count, n_its, out, inliers);
}

static int mlpnp_iterate_many_impl(rsc_mlpnp* const* solvers, int count, const int32_t* n_its, rsc_pnp_result* out,
                                   uint8_t* const* inliers) {
    if (count <= 0) return RSC_OK;
    if (!solvers || !n_its || !out) return RSC_ERR_ARG;
    rsc_context* C = solvers[0]->ctx;
    for (int i = 0; i < count; ++i)
        if (!solvers[i] || solvers[i]->ctx != C) return RSC_ERR_ARG;
    RSC_HIP(hipSetDevice(C->device));
    for (double& v : C->last_ms) v = 0;
    HipMLBackend be(C);
    be.all.assign(solvers, solvers + count);
    std::vector<MLState*> S(count);
    for (int i = 0; i < count; ++i) S[i] = &solvers[i]->st;
    std::vector<MLResult> res(count);
    if (int st = mlpnp_iterate_many(be, S.data(), count, n_its, res.data(), inliers)) return st;
    for (int i = 0; i < count; ++i) {
        out[i].ok = res[i].ok;
        out[i].no_more = res[i].no_more;
        out[i].n_inliers = res[i].n_inliers;
        out[i].iterations = res[i].iterations;
        std::memcpy(out[i].T, res[i].T, sizeof(out[i].T));
    }
    return RSC_OK;
}

int rsc_mlpnp_iterate(rsc_mlpnp* s, int n_its, rsc_pnp_result* out, uint8_t* inliers) {
    if (!s || !out) return RSC_ERR_ARG;
    int32_t n = n_its;
    uint8_t* const m[1] = {inliers};
    return rsc_mlpnp_iterate_many(&s, 1, &n, out, m);
}

int rsc_mlpnp_reset(rsc_mlpnp* s, uint32_t seed) {
    if (!s) return RSC_ERR_ARG;
    reset_solver(s, seed);
    return RSC_OK;
}

int rsc_mlpnp_reset_many(rsc_mlpnp* const* s, int count, const uint32_t* seeds) {
    if (count > 0 && (!s || !seeds)) return RSC_ERR_ARG;
    for (int i = 0; i < count; ++i) {
        if (!s[i]) return RSC_ERR_ARG;
        reset_solver(s[i], seeds[i]);
    }
    return RSC_OK;
}

int rsc_mlpnp_get_state(const rsc_mlpnp* s, int32_t out[6]) {
    if (!s || !out) return RSC_ERR_ARG;
    const MLState& t = s->st;
    out[0] = t.mnIterations; out[1] = t.mRansacMaxIts; out[2] = t.mRansacMinInliers; out[3] = t.mnBestInliers;
    out[4] = t.N; out[5] = t.mRansacMinSet;
    return RSC_OK;
}

// Parity hook: double poses (R row-major 9 + t 3) of the last launch's hypotheses of this solver.
int rsc_mlpnp_last_poses(rsc_mlpnp* s, double* out, int cap) {
    if (!s || !out) return RSC_ERR_ARG;
    rsc_context* C = s->ctx;
    if (s->spec_out0 < 0 || !C->d_mposes.p) return 0;
    const int n = std::min(cap, s->spec_H);
    RSC_HIP(hipMemcpy(out, C->d_mposes.p + (size_t)s->spec_out0 * 12, (size_t)n * 96, hipMemcpyDeviceToHost));
    return n;
}

int rsc_mlpnp_last_counts(rsc_mlpnp* s, int32_t* counts, int cap) {
    if (!s || !counts) return RSC_ERR_ARG;
    return last_hypotheses(s->ctx, s->spec_out0, s->spec_H, 12, counts, nullptr, cap);
}

int rsc_mlpnp_last_samples(rsc_mlpnp* s, int32_t* out, int cap) {
    if (!s || !out) return RSC_ERR_ARG;
    rsc_context* C = s->ctx;
    if (s->spec_out0 < 0 || !C->d_samples.p) return 0;
    const int n = std::min(cap, s->spec_H);
    RSC_HIP(hipMemcpy(out, C->d_samples.p + (size_t)s->spec_out0 * 8, (size_t)n * 8 * 4, hipMemcpyDeviceToHost));
    return n;
}

// ---- Event drivers (config 5) ----
int rsc_reloc_events(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events, rsc_pnp_result* per_candidate,
                     rsc_event_result* per_event) {
    if (n_events <= 0) return RSC_OK;
    if (!solvers || !event_begin || !per_candidate || !per_event) return RSC_ERR_ARG;
    const int total = event_begin[n_events];
    for (int e = 0; e < n_events; ++e) {
        if (event_begin[e + 1] < event_begin[e]) return RSC_ERR_ARG;
        per_event[e] = rsc_event_result{-1, -1, -1, 0};
    }
    std::vector<char> discarded(total, 0), resolved(n_events, 0);
    std::vector<int32_t> start_it(total);
    for (int i = 0; i < total; ++i) {
        if (!solvers[i]) return RSC_ERR_ARG;
        start_it[i] = solvers[i]->st.mnIterations;
    }
    for (int round = 0;; ++round) {
        std::vector<rsc_pnp*> act;
        std::vector<int> idx;
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i)
                if (!discarded[i]) { act.push_back(solvers[i]); idx.push_back(i); }
        }
        if (act.empty()) break;
        std::vector<int32_t> its(act.size(), 5);
        std::vector<rsc_pnp_result> r(act.size());
        std::vector<uint8_t*> nomask(act.size(), nullptr);
        if (int st = rsc_pnp_iterate_many(act.data(), (int)act.size(), its.data(), r.data(), nomask.data())) return st;
        std::vector<char> iterated(total, 0);
        for (size_t q = 0; q < act.size(); ++q) {
            iterated[idx[q]] = 1;
            per_candidate[idx[q]] = r[q];
            if (r[q].no_more) discarded[idx[q]] = 1;  // Tracking.cpp:1257-1261
        }
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            bool any_active = false;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
                if (!iterated[i]) continue;  // candidates iterated this round, in order
                if (per_candidate[i].ok) {
                    per_event[e].winner = i - event_begin[e];
                    per_event[e].round = round;
                    per_event[e].hypothesis = per_candidate[i].iterations - 1 - start_it[i];
                    per_event[e].n_inliers = per_candidate[i].n_inliers;
                    resolved[e] = 1;
                    break;
                }
                if (!discarded[i]) any_active = true;
            }
            if (!resolved[e] && !any_active) resolved[e] = 1;
        }
    }
    return RSC_OK;
}

int rsc_loop_events(rsc_sim3* const* solvers, const int32_t* event_begin, int n_events,
                    rsc_sim3_result* per_candidate, rsc_event_result* per_event) {
    if (n_events <= 0) return RSC_OK;
    if (!solvers || !event_begin || !per_candidate || !per_event) return RSC_ERR_ARG;
    const int total = event_begin[n_events];
    std::vector<int32_t> its(total), start_it(total);
    for (int i = 0; i < total; ++i) {
        if (!solvers[i]) return RSC_ERR_ARG;
        start_it[i] = solvers[i]->st.mnIterations;
        its[i] = std::max(1, solvers[i]->st.mRansacMaxIts - solvers[i]->st.mnIterations);
    }
    std::vector<uint8_t*> nomask(total, nullptr);
    if (total > 0)
        if (int st = rsc_sim3_iterate_many(solvers, total, its.data(), per_candidate, nomask.data())) return st;
    for (int e = 0; e < n_events; ++e) {
        per_event[e] = rsc_event_result{-1, -1, -1, 0};
        int best_round = 0;
        for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
            if (!per_candidate[i].ok) continue;
            const int h = per_candidate[i].iterations - 1 - start_it[i];
            const int round = h / 5;
            if (per_event[e].winner < 0 || round < best_round) {
                best_round = round;
                per_event[e] = rsc_event_result{i - event_begin[e], round, h, per_candidate[i].n_inliers};
            }
        }
    }
    return RSC_OK;
}

// ---- Events on the reference's shared rand() stream (Q3) ----
// One round of the round-robin: every live candidate of every unresolved event runs iterate(5) in
// one set of launches.  A candidate's call starts where the previous candidate's call of its event
// ended, assuming every call runs its whole loop; the only call that ends early is a success, which
// resolves the event (Tracking.cpp:1284-1331 / LoopClosing.cpp:311-327 with the gate passed), so the
// candidates after it in that round are calls the reference never makes: their records are
// discarded (left as they were before the round) and the stream advances by the calls made.

int rsc_reloc_events_shared(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events,
                            rsc_stream* const* streams, rsc_pnp_result* per_candidate, rsc_event_result* per_event) {
    for (int i = 0; n_events > 0 && solvers && event_begin && i < event_begin[n_events]; ++i)
        if (solvers[i] && solvers[i]->stream) return RSC_ERR_ARG;  // events position their own calls
    return shared_events(solvers, event_begin, n_events, streams, per_candidate, per_event, pnp_iterate_many_impl,
                         pnp_pred_its);
}

int rsc_loop_events_shared(rsc_sim3* const* solvers, const int32_t* event_begin, int n_events,
                           rsc_stream* const* streams, rsc_sim3_result* per_candidate, rsc_event_result* per_event) {
    for (int i = 0; n_events > 0 && solvers && event_begin && i < event_begin[n_events]; ++i)
        if (solvers[i] && solvers[i]->stream) return RSC_ERR_ARG;
    return shared_events(solvers, event_begin, n_events, streams, per_candidate, per_event, sim3_iterate_many_impl,
                         sim3_pred_its);
}

// ---- Gated events (round 6) ----
// Tracking::Relocalization (Tracking.cpp:1239-1335): each round runs iterate(5) on every live
// candidate of every unresolved event in one set of launches (own streams: the results are the
// reference's calls whatever happens before them in the round), then walks each event's successes in
// candidate order: PoseOptimization on the success (mCurrentFrame.mvpMapPoints = the inlier matches,
// mTcw = the RANSAC pose, :1268-1284), nGood < 10 -> the next success of the round (:1286-1287),
// nGood >= 50 -> match (:1327-1331), otherwise SearchByProjection's turn (handed off).  The gate
// passes of all events run as one rsc_pose_optimization_many each.
int rsc_reloc_events_gated(rsc_pnp* const* solvers, const int32_t* event_begin, int n_events,
                           const rsc_reloc_frame* frames, rsc_pnp_result* per_candidate,
                           rsc_reloc_gate_result* per_event, uint8_t* const* outlier, uint8_t* const* inliers) {
    if (n_events <= 0) return RSC_OK;
    if (!solvers || !event_begin || !frames || !per_candidate || !per_event) return RSC_ERR_ARG;
    const int total = event_begin[n_events];
    rsc_context* C = nullptr;
    for (int e = 0; e < n_events; ++e) {
        if (event_begin[e + 1] < event_begin[e] || event_begin[e] < 0) return RSC_ERR_ARG;
        rsc_reloc_gate_result& r = per_event[e];
        std::memset(&r, 0, sizeof(r));
        r.status = RSC_GATE_NONE;
        r.winner = r.round = r.hypothesis = -1;
        for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
            if (!solvers[i]) return RSC_ERR_ARG;
            if (solvers[i]->stream) return RSC_ERR_UNSUPPORTED;  // gating moves later calls' stream positions
            if (!C) C = solvers[i]->ctx;
            // one Frame per event: every candidate's vbInliers indexes the same mCurrentFrame slots
            if (solvers[i]->ctx != C || solvers[i]->st.N_points != solvers[event_begin[e]]->st.N_points)
                return RSC_ERR_ARG;
        }
    }
    if (!C) return RSC_OK;
    std::vector<char> discarded(total, 0), resolved(n_events, 0);
    std::vector<int32_t> start_it(total);
    std::vector<std::vector<uint8_t>> mask(total);
    for (int i = 0; i < total; ++i) {
        start_it[i] = solvers[i]->st.mnIterations;
        mask[i].assign((size_t)std::max(solvers[i]->st.N_points, 1), 0);
    }
    // per gate job: the PoseOptimization problem's slot arrays (Frame::N slots)
    struct Job {
        int e, i;
        std::vector<uint8_t> has_mp, outl;
        std::vector<float> uv, Xw, inv;
    };
    for (int round = 0;; ++round) {
        std::vector<rsc_pnp*> act;
        std::vector<int> idx;
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i)
                if (!discarded[i]) { act.push_back(solvers[i]); idx.push_back(i); }
        }
        if (act.empty()) break;
        std::vector<int32_t> its(act.size(), 5);
        std::vector<rsc_pnp_result> r(act.size());
        std::vector<uint8_t*> mp(act.size());
        for (size_t q = 0; q < act.size(); ++q) mp[q] = mask[idx[q]].data();
        if (int st = rsc_pnp_iterate_many(act.data(), (int)act.size(), its.data(), r.data(), mp.data())) return st;
        std::vector<char> iterated(total, 0);
        for (size_t q = 0; q < act.size(); ++q) {
            iterated[idx[q]] = 1;
            per_candidate[idx[q]] = r[q];
            if (r[q].no_more) discarded[idx[q]] = 1;  // Tracking.cpp:1257-1261
        }
        // gate passes: each unresolved event's next success of this round, in candidate order
        std::vector<int> cursor(n_events);
        for (int e = 0; e < n_events; ++e) cursor[e] = event_begin[e];
        for (;;) {
            std::vector<Job> jobs;
            for (int e = 0; e < n_events; ++e) {
                if (resolved[e]) continue;
                int i = cursor[e];
                while (i < event_begin[e + 1] && !(iterated[i] && per_candidate[i].ok)) ++i;
                cursor[e] = i + 1;
                if (i >= event_begin[e + 1]) continue;
                const rsc_pnp* s = solvers[i];
                const PnPState& st = s->st;
                const int nf = st.N_points;
                Job j;
                j.e = e;
                j.i = i;
                j.has_mp.assign((size_t)nf, 0);
                j.outl.assign((size_t)nf, 0);
                j.uv.assign(2 * (size_t)nf, 0.f);
                j.Xw.assign(3 * (size_t)nf, 0.f);
                j.inv.assign((size_t)nf, 0.f);
                for (int c = 0; c < st.N; ++c) {
                    const int slot = st.kp_index[c];
                    if (!mask[i][slot]) continue;  // mvpMapPoints[j] = inlier ? match : NULL (:1276-1282)
                    j.has_mp[slot] = 1;
                    j.uv[2 * slot] = s->h_p2d[2 * c];
                    j.uv[2 * slot + 1] = s->h_p2d[2 * c + 1];
                    for (int k = 0; k < 3; ++k) j.Xw[3 * slot + k] = s->h_p3d[3 * c + k];
                    j.inv[slot] = 1.0f / st.sigma2[c];  // mvInvLevelSigma2 = 1.0f / mvLevelSigma2
                }
                jobs.push_back(std::move(j));
            }
            if (jobs.empty()) break;
            std::vector<rsc_poseopt_problem> pr(jobs.size());
            std::vector<rsc_poseopt_result> res(jobs.size());
            std::vector<uint8_t*> op(jobs.size());
            for (size_t q = 0; q < jobs.size(); ++q) {
                const Job& j = jobs[q];
                const PnPState& st = solvers[j.i]->st;
                rsc_poseopt_problem& P = pr[q];
                P.n = st.N_points;
                P.has_mp = j.has_mp.data();
                P.uv = j.uv.data();
                P.Xw = j.Xw.data();
                P.inv_sigma2 = j.inv.data();
                P.u_right = frames[j.e].u_right;
                P.fx = st.fx; P.fy = st.fy; P.cx = st.cx; P.cy = st.cy;
                std::memcpy(P.Tcw, per_candidate[j.i].T, sizeof(P.Tcw));
                P.bf = frames[j.e].bf;
                op[q] = jobs[q].outl.data();
            }
            if (int st = rsc_pose_optimization_many(C, pr.data(), (int)pr.size(), res.data(), op.data())) return st;
            for (size_t q = 0; q < jobs.size(); ++q) {
                const Job& j = jobs[q];
                rsc_reloc_gate_result& g = per_event[j.e];
                g.gates++;
                const int nGood = res[q].n_good;
                if (nGood < 10) {  // Tracking.cpp:1286-1287: continue with the next candidate
                    g.rejected++;
                    continue;
                }
                g.status = nGood >= 50 ? RSC_GATE_MATCH : RSC_GATE_HANDOFF;
                g.winner = j.i - event_begin[j.e];
                g.round = round;
                g.hypothesis = per_candidate[j.i].iterations - 1 - start_it[j.i];
                g.n_inliers = per_candidate[j.i].n_inliers;
                g.n_good = nGood;
                std::memcpy(g.Tcw, res[q].Tcw, sizeof(g.Tcw));
                const int nf = solvers[j.i]->st.N_points;
                if (outlier && outlier[j.e]) std::memcpy(outlier[j.e], j.outl.data(), (size_t)nf);
                if (inliers && inliers[j.e]) std::memcpy(inliers[j.e], mask[j.i].data(), (size_t)nf);
                resolved[j.e] = 1;
            }
        }
        for (int e = 0; e < n_events; ++e) {  // nCandidates == 0: the while loop ends (:1239)
            if (resolved[e]) continue;
            bool any_active = false;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) any_active |= !discarded[i];
            if (!any_active) resolved[e] = 1;
        }
    }
    return RSC_OK;
}

// LoopClosing::ComputeSim3 (LoopClosing.cpp:268-329): a candidate's k-th success comes back from the
// call that reaches it (Sim3Solver::iterate returns at the first hypothesis with more than
// mRansacMinInliers inliers, Sim3Solver.cpp:155-163), so with its own stream each candidate's
// successes are computed one at a time, each with the whole remaining budget in one call, and placed
// in the round-robin: a call starting at hypothesis p in round c covers p..p+4, so the success at
// hypothesis s is returned in round c + (s - p) / 5 and the next call starts at s + 1 in the round
// after.  The event takes its successes in (round, candidate) order: SearchBySim3(7.5) on the inliers
// (:296-309), OptimizeSim3(gScm = Sim3(R, t, 1), 10) (:310-311), accepted when nInliers >= 20
// (:314-325); a rejected candidate's next success is computed and the walk goes on.  Each pass gates
// one success per unresolved event (one launch of each stage over all of them).
int rsc_loop_events_gated(rsc_sim3* const* solvers, const rsc_loop_candidate* cands, const int32_t* event_begin,
                          int n_events, rsc_sim3_result* per_candidate, rsc_loop_gate_result* per_event,
                          int32_t* const* matches_out) {
    if (n_events <= 0) return RSC_OK;
    if (!solvers || !cands || !event_begin || !per_candidate || !per_event) return RSC_ERR_ARG;
    const int total = event_begin[n_events];
    rsc_context* C = nullptr;
    for (int e = 0; e < n_events; ++e) {
        if (event_begin[e + 1] < event_begin[e] || event_begin[e] < 0) return RSC_ERR_ARG;
        rsc_loop_gate_result& r = per_event[e];
        std::memset(&r, 0, sizeof(r));
        r.status = RSC_GATE_NONE;
        r.winner = r.round = r.hypothesis = -1;
        for (int i = event_begin[e]; i < event_begin[e + 1]; ++i) {
            const rsc_loop_candidate& k = cands[i];
            if (!solvers[i] || !k.kf1 || !k.kf2) return RSC_ERR_ARG;
            if (solvers[i]->stream) return RSC_ERR_UNSUPPORTED;
            if (!C) C = solvers[i]->ctx;
            if (solvers[i]->ctx != C || k.kf1->ctx != C || k.kf2->ctx != C) return RSC_ERR_ARG;
            if (solvers[i]->st.mN1 != k.kf1->n || (k.kf1->n > 0 && !k.matches12)) return RSC_ERR_ARG;
            if (k.kf1 != cands[event_begin[e]].kf1) return RSC_ERR_ARG;  // one mpCurrentKF per event
            for (int a = 0; a < k.kf1->n; ++a)
                if (k.matches12[a] < -2 || k.matches12[a] >= k.kf2->n) return RSC_ERR_ARG;
        }
    }
    if (!C) return RSC_OK;
    std::vector<int32_t> start_it(total), pos(total), calls(total, 0), s_round(total, -1);
    std::vector<std::vector<uint8_t>> mask(total);
    for (int i = 0; i < total; ++i) {
        start_it[i] = pos[i] = solvers[i]->st.mnIterations;
        mask[i].assign((size_t)std::max(solvers[i]->st.mN1, 1), 0);
    }
    // the next success of each listed candidate (s_round = its round, -1: none left)
    auto refill = [&](const std::vector<int>& list) -> int {
        if (list.empty()) return RSC_OK;
        std::vector<rsc_sim3*> act;
        std::vector<int32_t> its;
        std::vector<uint8_t*> mp;
        for (int i : list) {
            act.push_back(solvers[i]);
            its.push_back(std::max(1, solvers[i]->st.mRansacMaxIts - solvers[i]->st.mnIterations));
            mp.push_back(mask[i].data());
        }
        std::vector<rsc_sim3_result> r(act.size());
        if (int st = rsc_sim3_iterate_many(act.data(), (int)act.size(), its.data(), r.data(), mp.data())) return st;
        for (size_t q = 0; q < list.size(); ++q) {
            const int i = list[q];
            per_candidate[i] = r[q];
            if (!r[q].ok) {
                s_round[i] = -1;
                continue;
            }
            const int s = r[q].iterations - 1;
            s_round[i] = calls[i] + (s - pos[i]) / 5;
            pos[i] = s + 1;
            calls[i] = s_round[i] + 1;
        }
        return RSC_OK;
    };
    {
        std::vector<int> all(total);
        for (int i = 0; i < total; ++i) all[i] = i;
        if (int st = refill(all)) return st;
    }
    std::vector<char> resolved(n_events, 0);
    for (;;) {
        std::vector<int> ev, ci;  // one gate job per unresolved event: its smallest (round, candidate)
        for (int e = 0; e < n_events; ++e) {
            if (resolved[e]) continue;
            int best = -1;
            for (int i = event_begin[e]; i < event_begin[e + 1]; ++i)
                if (s_round[i] >= 0 && (best < 0 || s_round[i] < s_round[best])) best = i;
            if (best < 0) {
                resolved[e] = 1;  // every candidate discarded: bMatch stays false
                continue;
            }
            ev.push_back(e);
            ci.push_back(best);
        }
        const int J = (int)ev.size();
        if (J == 0) break;
        // SearchBySim3 over the RANSAC inliers (vpMapPointMatches[j] = inlier ? match : NULL)
        std::vector<rsc_kfview*> k1(J), k2(J);
        std::vector<float> R12(9 * (size_t)J), t12(3 * (size_t)J);
        std::vector<std::vector<int32_t>> m12(J), o12(J);
        std::vector<const int32_t*> m12p(J);
        std::vector<int32_t*> o12p(J);
        std::vector<int32_t> nfound(J, 0);
        for (int q = 0; q < J; ++q) {
            const int i = ci[q];
            const rsc_loop_candidate& k = cands[i];
            k1[q] = k.kf1;
            k2[q] = k.kf2;
            std::memcpy(&R12[9 * (size_t)q], per_candidate[i].R, 9 * sizeof(float));
            std::memcpy(&t12[3 * (size_t)q], per_candidate[i].t, 3 * sizeof(float));
            const int n1 = k.kf1->n;
            m12[q].assign((size_t)std::max(n1, 1), -1);
            o12[q].assign((size_t)std::max(n1, 1), -1);
            for (int a = 0; a < n1; ++a) m12[q][a] = mask[i][a] ? k.matches12[a] : -1;
            m12p[q] = m12[q].data();
            o12p[q] = o12[q].data();
        }
        if (int st = rsc_search_by_sim3_many(C, k1.data(), k2.data(), J, R12.data(), t12.data(), 7.5f, m12p.data(),
                                             o12p.data(), nfound.data()))
            return st;
        // OptimizeSim3 on vpMapPointMatches after the search (Optimizer.cpp:1108-1171 slot rules)
        std::vector<rsc_sim3opt_problem> pr(J);
        std::vector<rsc_sim3opt_result> res(J);
        std::vector<std::vector<uint8_t>> valid(J), keep(J);
        std::vector<std::vector<float>> X1(J), X2(J), u1(J), u2(J), i1(J), i2(J);
        std::vector<uint8_t*> keepp(J);
        for (int q = 0; q < J; ++q) {
            const int i = ci[q];
            const rsc_kfview& a = *cands[i].kf1;
            const rsc_kfview& b = *cands[i].kf2;
            const int n1 = a.n;
            for (int x = 0; x < n1; ++x)
                if (o12[q][x] >= 0) m12[q][x] = o12[q][x];  // vpMatches12[i1] = vpMapPoints2[idx2]
            valid[q].assign((size_t)std::max(n1, 1), 0);
            keep[q].assign((size_t)std::max(n1, 1), 1);
            X1[q].assign(3 * (size_t)std::max(n1, 1), 0.f);
            X2[q].assign(3 * (size_t)std::max(n1, 1), 0.f);
            u1[q].assign(2 * (size_t)std::max(n1, 1), 0.f);
            u2[q].assign(2 * (size_t)std::max(n1, 1), 0.f);
            i1[q].assign((size_t)std::max(n1, 1), 0.f);
            i2[q].assign((size_t)std::max(n1, 1), 0.f);
            for (int x = 0; x < n1; ++x) {
                const int y = m12[q][x];
                // vpMatches1[i] set, pMP1 set, neither bad, i2 = GetIndexInKeyFrame(pKF2) >= 0
                if (y < 0 || a.mp_state[x] != 1 || b.mp_state[y] != 1) continue;
                valid[q][x] = 1;
                for (int c = 0; c < 3; ++c) {
                    X1[q][3 * x + c] = a.mp_pos[3 * x + c];
                    X2[q][3 * x + c] = b.mp_pos[3 * (size_t)y + c];
                }
                u1[q][2 * x] = a.kp[2 * x];
                u1[q][2 * x + 1] = a.kp[2 * x + 1];
                u2[q][2 * x] = b.kp[2 * (size_t)y];
                u2[q][2 * x + 1] = b.kp[2 * (size_t)y + 1];
                const int o1 = a.octave[x], o2 = b.octave[y];
                if (o1 < 0 || o1 >= (int)a.inv_level_sigma2.size() || o2 < 0 || o2 >= (int)b.inv_level_sigma2.size())
                    return RSC_ERR_ARG;
                i1[q][x] = a.inv_level_sigma2[o1];
                i2[q][x] = b.inv_level_sigma2[o2];
            }
            rsc_sim3opt_problem& P = pr[q];
            P.n = n1;
            P.valid = valid[q].data();
            P.X1w = X1[q].data();
            P.X2w = X2[q].data();
            P.uv1 = u1[q].data();
            P.uv2 = u2[q].data();
            P.inv1 = i1[q].data();
            P.inv2 = i2[q].data();
            std::memcpy(P.R1w, a.R, sizeof(P.R1w));
            std::memcpy(P.t1w, a.t, sizeof(P.t1w));
            std::memcpy(P.R2w, b.R, sizeof(P.R2w));
            std::memcpy(P.t2w, b.t, sizeof(P.t2w));
            std::memcpy(P.K1, a.K, sizeof(P.K1));
            std::memcpy(P.K2, b.K, sizeof(P.K2));
            // g2o::Sim3 gScm(R.cast<double>(), t.cast<double>(), 1.0): Quaterniond(R), no normalisation
            double Rd[3][3];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) Rd[r][c] = (double)per_candidate[i].R[3 * r + c];
            const PoQuat qq = po_quat_from_R(Rd);
            P.S[0] = qq.x; P.S[1] = qq.y; P.S[2] = qq.z; P.S[3] = qq.w;
            for (int c = 0; c < 3; ++c) P.S[4 + c] = (double)per_candidate[i].t[c];
            P.S[7] = 1.0;
            P.th2 = 10.0f;
            keepp[q] = keep[q].data();
        }
        if (int st = rsc_optimize_sim3_many(C, pr.data(), J, res.data(), keepp.data())) return st;
        std::vector<int> again;
        for (int q = 0; q < J; ++q) {
            const int e = ev[q], i = ci[q];
            rsc_loop_gate_result& g = per_event[e];
            if (res[q].n_inliers < 20) {  // LoopClosing.cpp:314: not accepted, the round-robin goes on
                g.rejected++;
                again.push_back(i);
                continue;
            }
            g.status = RSC_GATE_MATCH;
            g.winner = i - event_begin[e];
            g.round = s_round[i];
            g.hypothesis = per_candidate[i].iterations - 1 - start_it[i];
            g.n_inliers = per_candidate[i].n_inliers;
            g.n_found = nfound[q];
            g.n_opt_inliers = res[q].n_inliers;
            std::memcpy(g.S, res[q].S, sizeof(g.S));
            if (matches_out && matches_out[e]) {
                const int n1 = cands[i].kf1->n;
                for (int x = 0; x < n1; ++x) matches_out[e][x] = keep[q][x] ? m12[q][x] : -1;  // outliers NULLed
            }
            resolved[e] = 1;
        }
        if (int st = refill(again)) return st;
    }
    return RSC_OK;
}
}  // extern "C"
