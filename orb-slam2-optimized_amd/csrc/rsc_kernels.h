// rsc_kernels.h — device-visible descriptors shared by kernels.hip and the HIP backend.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace rsc {

// One PnP problem (= one PnPsolver) resident in HBM.
struct DevPnP {
    const float4* pts;  // [n] x, y, z (mvP3Dw), w = sigma^2 (mvSigma2)
    const float2* uv;   // [n] mvP2D
    int n;              // N
    float fx, fy, cx, cy;  // Frame static float intrinsics (widened to double in the kernels)
    float th2;          // SetRansacParameters th2: mvMaxError[i] = sigma2[i] * th2 (float)
    int rows;           // maximum_number_of_correspondences of the grow-only EPnP buffers
    double* pws;        // [cap][3] EPnP buffers (rows >= min_set are stale rows from Refine)
    double* us;         // [cap][2]
    double* als;        // [cap][4]
};

// One Sim3 problem (= one Sim3Solver after construction).
struct DevSim3 {
    const float4* x1;   // [n] mvX3Dc1, w = (float)mvnMaxError1
    const float4* x2;   // [n] mvX3Dc2, w = (float)mvnMaxError2
    const float4* pim;  // [n] (mvP1im1.x, .y, mvP2im2.x, .y)
    int n;
    float K1[4], K2[4];  // fx, fy, cx, cy
};

// One MLPnP problem (= one MLPnPsolver) resident in HBM.
struct DevML {
    const float4* pts;  // [n] x, y, z (mvP3Dw), w = sigma^2
    const float2* uv;   // [n] mvP2D
    const float2* brg;  // [n] bearing x, y (z = 1), float arithmetic of MLPnPsolver.cpp:32-33
    const double* cov;  // [n][9] bearing-vector covariances (computePose's covMats), or null
    int n;
    float fx, fy, cx, cy;  // float members (MLPnPsolver.hpp:198)
    float th2;
};

// Per-launch, per-problem speculation record: hypotheses [0, H) of this launch use draws
// g0 + h*min_set + d of the glibc stream whose window is `window`.
struct LaunchProb {
    int prob;
    int H;
    int out0;  // first record index of this problem in the launch's pose/count/mask arrays
    int g0;
    uint32_t window[31];
    int min_inliers;  // PnP scan: masks are stored only for counts >= this (mRansacMinInliers)
    int best0 = 0;    // Sim3 pick: mnBestInliers when the call started
};

// Sim3 pick (sim3_pick_kernel): hypotheses per solver it can hold in LDS.
constexpr int kPickMaxH = 4096;

struct RefineJob {
    int prob;
    int rows_after;             // maximum_number_of_correspondences after set_maximum(n_r)
    const uint64_t* best_mask;  // mvbBestInliers as bits (the adopted hypothesis' scan record, or the solver's)
    uint64_t* adopt_mask;       // non-null: copy best_mask here (the solver's persistent mvbBestInliers)
    const float* adopt_pose;    // non-null: hypothesis pose record (12 floats) copied to out_best_pose
    float* out_best_pose;
    float* out_pose;            // 12 floats
    int32_t* out_count;
    uint64_t* out_mask;         // mvbRefinedInliers as bits
    int out_words;              // words of out_mask (the solver's ceil(N/64))
};

// pnp_select_refine_kernel: one speculation round's solver (the replay's state at launch) and what
// the kernel leaves for the host replay.
struct RefineSel {
    int prob;          // index into the round's DevPnP table
    int out0, H;       // the solver's hypothesis records in the round
    int min_inliers;   // mRansacMinInliers
    int best0;         // mnBestInliers when the round was launched
    int rows0;         // maximum_number_of_correspondences when the round was launched
    uint64_t* best;    // the solver's mvbBestInliers bits
    uint64_t* refined; // mvbRefinedInliers bits
    int words;         // words of best / refined (ceil(N/64))
};
struct RefineSelOut {
    int k;           // first hypothesis with nInliers >= mRansacMinInliers, -1: none (nothing ran)
    int adopt;       // it became the new best (mask + pose adopted on the device)
    int rows_after;  // set_maximum_number_of_correspondences(max(rows0, mnBestInliers))
    int count;       // mnRefinedInliers
    float pose[12];      // refined R (9) + t (3)
    float best_pose[12]; // adopted hypothesis pose (when adopt)
};

struct Window31 {
    uint32_t w[31];
};
// MLPnP: one quad per hypothesis, kMlQuadHyps per workgroup (min_set 6..8), poses as double[12]
// records (R row-major, t).
constexpr int kMlQuadHyps = 16;  // MLPnP hypotheses (quads) per 64-lane workgroup (rsc_mlpnp_quad.h)
// cov: the workgroups' problems carry bearing covariances (DevML::cov != null)
hipError_t launch_mlpnp_solve(int ns, bool cov, int nwg, const DevML* probs, const LaunchProb* lps, const int2* wgt,
                              const uint32_t* T, double* poses, int32_t* samples, hipStream_t st);
hipError_t launch_mlpnp_scan(int ppt, int nwg, const DevML* probs, const LaunchProb* lps, const int4* wgt,
                             const double* poses, int32_t* counts, uint64_t* masks, int mask_words, hipStream_t st);
hipError_t launch_selftest_math(int fn, const double* x, int n, double* out, hipStream_t st);
// Descriptor upload of a round: n16 16-byte words from pinned host memory (read over PCIe by the
// kernel) into device memory, in stream order with the launches that read them.
hipError_t launch_upload16(const void* host_src, void* dev_dst, size_t n16, hipStream_t st);
hipError_t launch_signal(uint32_t* host_flag, uint32_t value, hipStream_t st);
// Any-size copy between pinned host memory and HBM by a kernel (latency-bound small transfers of
// the KeyFrameDatabase queries: no DMA start-up or engine hand-off).
hipError_t launch_copy_bytes(const void* src, void* dst, size_t n, hipStream_t st);
hipError_t launch_gather_records(const float* src, int stride, int take, const int32_t* idx, int n, float* dst,
                                 hipStream_t st);
hipError_t launch_rng_stream(const uint32_t* T, const uint32_t* window, int g0, int n, int32_t* out, hipStream_t st);

constexpr int kEigLanes = 2;           // lanes per hypothesis in the eigen-stage kernel (rsc_quad.h)
#ifndef RSC_EIG_HYPS
#define RSC_EIG_HYPS 20  // build-time override for A/B runs (tools/)
#endif
constexpr int kEigHyps = RSC_EIG_HYPS;  // hypotheses per 64-lane eigen-stage workgroup (960 on config 2)
// Per-hypothesis stage record between the two kernels: eigenvectors [12][4], alphas [NS][4], cws [4][3].
constexpr int kStageDoubles = 48 + 24 + 12;
// Two-kernel hypothesis solve: eigenvectors (lane groups), then the three beta approximations
// (one wave each) + selection.
// Hand-off buffers of pnp_betas_kernel: per record and approximation the error (`err[3][hcap]`)
// and the float pose (`pose[3][12][hcap]`); one counter per 64-hypothesis group, zero between
// launches (the kernel resets what it uses).
struct BetasScratch {
    double* err;
    float* pose;
    unsigned* ctr;
    size_t hcap;
};
// Hypotheses per betas wave: 64.  Smaller waves for small (latency-bound) rounds, and eigen-stage
// waves of quads x 4 or quads x 1 instead of pairs x 20, were measured slower on the single-event
// case (tools/latency_ab.py, profiles/r03/latency_ab_r3_c.txt): the stage time is not the union of
// a wave's hypotheses' chains but the per-wave latency, which more, narrower waves do not shorten.
#ifndef RSC_BETAS_HYPS
#define RSC_BETAS_HYPS 64  // build-time override for A/B runs (tools/Makefile betas32_lib)
#endif
constexpr int kBetasHyps = RSC_BETAS_HYPS;
// Default eigen-stage form switch (rsc_context_set_eig_rows): launches of at most this many 20-hypothesis
// workgroups run the rows form.
constexpr int kEigRowsDefaultWgs = 64;
hipError_t launch_pnp_solve_split(int ns, int nwgE, const int2* wgtE, int nwgB, const int2* wgtB,
                                  const DevPnP* probs, const LaunchProb* lps, const uint32_t* T, double* stage,
                                  float* poses, int32_t* samples, const BetasScratch& bs, hipStream_t st,
                                  hipEvent_t eig_begin = nullptr, hipEvent_t eig_end = nullptr, bool eig_rows = false,
                                  bool eig_split = false, unsigned* fault = nullptr, int betas_hb = kBetasHyps);
// betas_hb: hypotheses per betas wave (<= kBetasHyps; the wg_table's groups step by it).
// fault (required by the split form): a word in pinned host memory that the split eigen stage sets to
// 1 when a chase / row-wave hand-off gives up (split_wait); the host turns it into RSC_ERR_INTERNAL.
// counts: where the host reads them (pinned memory or HBM); counts_dev (nullable): an HBM copy for
// pnp_select_refine_kernel; qual[lp] (pinned, zeroed by the host) is set to 1 when a hypothesis of
// launch problem lp reaches its min_inliers.
hipError_t launch_pnp_scan(int ppt, int nwg, const DevPnP* probs, const LaunchProb* lps, const int4* wgt,
                           const float* poses, int32_t* counts, int32_t* counts_dev, uint64_t* masks, int mask_words,
                           int32_t* qual, hipStream_t st);
// fault: the context's fault word (the Refine's split-form eigen hand-off, RSC_REFINE_SPLIT)
hipError_t launch_pnp_select_refine(int nsel, const DevPnP* probs, const RefineSel* sels, const int32_t* counts,
                                    uint64_t* masks, int mask_words, const float* poses, RefineSelOut* out,
                                    unsigned* fault, hipStream_t st);
// Rounds up to this many hypotheses run the replay's first Refine on the device right after the
// scan (pnp_select_refine_kernel): latency-bound rounds lose a host round trip; large exhaustive
// rounds (config 2), where no hypothesis qualifies, keep their launch set unchanged.
constexpr int kFusedRefineMaxHyps = 4096;
hipError_t read_refine_stamps(uint64_t* out);  // diagnostic, [64][24]
hipError_t read_solve_stamps(uint64_t* out);  // diagnostic, [3][4096][8]
hipError_t read_ml_stamps(uint64_t* out);     // diagnostic, [8192][8] (mlpnp.hip)
hipError_t launch_pnp_refine(int njobs, const DevPnP* probs, const RefineJob* jobs, unsigned* fault, hipStream_t st);
hipError_t launch_sim3_solve(int nwg, const DevSim3* probs, const LaunchProb* lps, const int2* wgt,
                             const uint32_t* T, float* poses, int32_t* samples, hipStream_t st);
// counts: where the host reads them (pinned memory or HBM); counts_dev (nullable): an HBM copy for
// sim3_pick_kernel.
hipError_t launch_sim3_scan(int ppt, int nwg, const DevSim3* probs, const LaunchProb* lps, const int4* wgt,
                            const float* poses, int32_t* counts, int32_t* counts_dev, uint64_t* masks, int mask_words,
                            hipStream_t st);
// Sim3Solver::iterate's selection evaluated after the scan (one workgroup per solver, counts from
// HBM): pick[16 j] = {kept hypothesis index (as int, -1: none), R12[9], t12[3]} — the hypothesis
// the reference's '>=' rule keeps as mBestRotation / mBestTranslation (pick: pinned host memory).
hipError_t launch_sim3_pick(int count, const LaunchProb* lps, const int32_t* counts, const float* poses,
                            float* pick, hipStream_t st);

}  // namespace rsc
