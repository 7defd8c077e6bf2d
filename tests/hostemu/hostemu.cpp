// TEST-ONLY host build of the product's per-lane device numerics (rsc_core.h / rsc_epnp.h /
// rsc_sim3.h / rsc_engine.h RNG).  The product library never contains this code path; it exists
// so that the arithmetic the kernels run can be compared with the oracle on a CPU.
#include <cstdint>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>
#include "../../orb-slam2-optimized_amd/csrc/rsc_epnp.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_sim3.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_engine.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_mlpnp.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_poseopt.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_sim3opt.h"
#include "../../tools/qr_events.h"  // diagnostic QR forms (their bit-equality is tested)

using namespace rsc;

static RngTable* g_tab = nullptr;
static const RngTable& tab() {
    if (!g_tab) { g_tab = new RngTable(); g_tab->build(); }
    return *g_tab;
}

template <int NS>
static void pnp_hyp(const uint32_t* window, int g0, int h, int n, const float* pts4, const float* uv2, const float* K,
                    int rows, const double* spw, const double* sal, int32_t* idx_out, float* R, float* t) {
    uint32_t w[31];
    std::memcpy(w, window, sizeof(w));
    uint32_t words[NS];
    for (int d = 0; d < NS; ++d) words[d] = rng_word(tab().T.data(), w, g0 + h * NS + d);
    int idx[NS];
    swap_remove_sample<NS>(words, NS, n, idx);
    HypStore<NS> st;
    for (int i = 0; i < NS; ++i) {
        st.pw_[i][0] = pts4[4 * idx[i]]; st.pw_[i][1] = pts4[4 * idx[i] + 1]; st.pw_[i][2] = pts4[4 * idx[i] + 2];
        st.u_[i][0] = uv2[2 * idx[i]]; st.u_[i][1] = uv2[2 * idx[i] + 1];
        idx_out[i] = idx[i];
    }
    st.rows_ = rows; st.spw = spw; st.sal = sal;
    std::vector<double> slab(kSlabDoubles);
    LaneMat S{slab.data(), 1};
    Intrinsics KK{(double)K[0], (double)K[1], (double)K[2], (double)K[3]};
    float Rf[9], tf[3];
    epnp_compute_pose(st, KK, S, Rf, tf);
    std::memcpy(R, Rf, sizeof(Rf));
    std::memcpy(t, tf, sizeof(tf));
}

extern "C" {

void he_rng_window(uint32_t seed, uint32_t* window, int32_t* g0) {
    RngStream r; r.seed(seed);
    std::memcpy(window, r.window, sizeof(r.window));
    *g0 = r.g;
}

void he_rand_stream(uint32_t seed, int n, int32_t* out) {
    RngStream r; r.seed(seed);
    int done = 0;
    while (done < n) {
        int chunk = n - done < 4000 ? n - done : 4000;
        r.ensure(tab(), chunk);
        for (int i = 0; i < chunk; ++i) out[done + i] = (int32_t)(tab().word(r.window, r.g + i) >> 1);
        r.g += chunk; done += chunk;
    }
}

int he_pnp_hypothesis(int ns, const uint32_t* window, int g0, int h, int n, const float* pts4, const float* uv2,
                      const float* K, int rows, const double* spw, const double* sal, int32_t* idx, float* R, float* t) {
    switch (ns) {
        case 4: pnp_hyp<4>(window, g0, h, n, pts4, uv2, K, rows, spw, sal, idx, R, t); return 0;
        case 5: pnp_hyp<5>(window, g0, h, n, pts4, uv2, K, rows, spw, sal, idx, R, t); return 0;
        case 6: pnp_hyp<6>(window, g0, h, n, pts4, uv2, K, rows, spw, sal, idx, R, t); return 0;
    }
    return -1;
}

int he_pnp_count(const float* R, const float* t, const float* K, float th2, int n, const float* pts4, const float* uv2,
                 uint8_t* mask) {
    float Rr[9], tt[3];
    std::memcpy(Rr, R, sizeof(Rr)); std::memcpy(tt, t, sizeof(tt));
    int c = 0;
    for (int i = 0; i < n; ++i) {
        bool in = pnp_inlier(Rr, tt, K[0], K[1], K[2], K[3], pts4[4 * i], pts4[4 * i + 1], pts4[4 * i + 2],
                             uv2[2 * i], uv2[2 * i + 1], pts4[4 * i + 3] * th2);
        mask[i] = in;
        c += in;
    }
    return c;
}

// Refine-style EPnP over explicit rows (RowStore): pws[rows][3], us[n][2], als[rows][4] (als rows
// >= n are the stale rows; rows < n are overwritten).
double he_pnp_rows(int n, int rows, double* pws, const double* us, double* als, const float* K, float* R, float* t) {
    RowStore st{n, rows, pws, us, als};
    std::vector<double> slab(kSlabDoubles);
    LaneMat S{slab.data(), 1};
    Intrinsics KK{(double)K[0], (double)K[1], (double)K[2], (double)K[3]};
    float Rf[9], tf[3];
    double e = epnp_compute_pose(st, KK, S, Rf, tf);
    std::memcpy(R, Rf, sizeof(Rf)); std::memcpy(t, tf, sizeof(tf));
    return e;
}

void he_sim3_hypothesis(const uint32_t* window, int g0, int h, int n, const float* x1, const float* x2, int32_t* idx_out,
                        float* pose24) {
    uint32_t w[31];
    std::memcpy(w, window, sizeof(w));
    uint32_t words[3];
    for (int d = 0; d < 3; ++d) words[d] = rng_word(tab().T.data(), w, g0 + h * 3 + d);
    int idx[3];
    swap_remove_sample<3>(words, 3, n, idx);
    float P1[3][3], P2[3][3];
    for (int i = 0; i < 3; ++i) {
        idx_out[i] = idx[i];
        for (int r = 0; r < 3; ++r) { P1[r][i] = x1[3 * idx[i] + r]; P2[r][i] = x2[3 * idx[i] + r]; }
    }
    Sim3Pose T;
    sim3_compute(P1, P2, T);
    std::memcpy(pose24, T.R12, 36); std::memcpy(pose24 + 9, T.t12, 12);
    std::memcpy(pose24 + 12, T.R21, 36); std::memcpy(pose24 + 21, T.t21, 12);
}

int he_sim3_count(const float* pose24, const float* K1, const float* K2, int n, const float* x1, const float* x2,
                  const float* p1, const float* p2, const uint64_t* e1, const uint64_t* e2, uint8_t* mask) {
    Sim3Pose T;
    std::memcpy(T.R12, pose24, 36); std::memcpy(T.t12, pose24 + 9, 12);
    std::memcpy(T.R21, pose24 + 12, 36); std::memcpy(T.t21, pose24 + 21, 12);
    float k1[4], k2[4];
    std::memcpy(k1, K1, 16); std::memcpy(k2, K2, 16);
    int c = 0;
    for (int i = 0; i < n; ++i) {
        float a[3] = {x1[3 * i], x1[3 * i + 1], x1[3 * i + 2]};
        float b[3] = {x2[3 * i], x2[3 * i + 1], x2[3 * i + 2]};
        bool in = sim3_inlier(T, k1, k2, a, b, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1], (float)e1[i], (float)e2[i]);
        mask[i] = in;
        c += in;
    }
    return c;
}

// split_wait's bounded poll (rsc_core.h poll_until) on a flag that becomes ready at the
// `ready_after`-th load: 1 when it held within `limit` polls, 0 when the wait gave up (the device
// raises the fault word then); *loads = flag loads made, *pauses = pauses between them
int he_poll_until(int limit, int ready_after, int* loads, int* pauses) {
    int n = 0, p = 0, v = -1;
    const bool ok = rsc::poll_until(limit, [&]() { return ++n; }, [&]() { ++p; },
                                    [ready_after](int x) { return x >= ready_after; }, v);
    *loads = n;
    *pauses = p;
    return ok ? 1 : 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// CPU backends of rsc_engine.h (TEST-ONLY): the same replay code the HIP backend drives, with the
// kernels replaced by loops over the per-lane functions.
// ------------------------------------------------------------------------------------------------
namespace {

struct EmuPnP {
    PnPState st;
    std::vector<float> pts4, uv;  // x,y,z,sigma2 / u,v
    std::vector<double> pws, us, als;
    std::vector<uint64_t> best, refined;
    int words = 0;
    // last speculation
    std::vector<float> poses;
    std::vector<std::vector<uint64_t>> masks;
};

struct EmuPnPBackend : PnPBackend {
    std::vector<EmuPnP*> all;
    std::vector<EmuPnP*> spec;
    EmuPnP* of(PnPState* s) { for (auto* p : all) if (&p->st == s) return p; return nullptr; }
    int speculate(PnPState* const* S, int count, const int* H, std::vector<std::vector<int32_t>>& counts) override {
        counts.assign(count, {});
        spec.assign(count, nullptr);
        for (int i = 0; i < count; ++i) {
            EmuPnP* p = of(S[i]);
            spec[i] = p;
            PnPState& s = *S[i];
            s.rng.ensure(tab(), H[i] * s.mRansacMinSet);
            const float K[4] = {s.fx, s.fy, s.cx, s.cy};
            p->poses.assign((size_t)H[i] * 12, 0.f);
            p->masks.assign(H[i], std::vector<uint64_t>(p->words, 0));
            for (int h = 0; h < H[i]; ++h) {
                int32_t idx[8];
                float R[9], t[3];
                he_pnp_hypothesis(s.mRansacMinSet, s.rng.window, s.rng.g, h, s.N, p->pts4.data(), p->uv.data(), K,
                                  s.max_rows, p->pws.data(), p->als.data(), idx, R, t);
                std::memcpy(&p->poses[12 * h], R, 36);
                std::memcpy(&p->poses[12 * h + 9], t, 12);
                std::vector<uint8_t> m(s.N);
                int c = he_pnp_count(R, t, K, s.th2, s.N, p->pts4.data(), p->uv.data(), m.data());
                for (int j = 0; j < s.N; ++j) if (m[j]) p->masks[h][j >> 6] |= 1ull << (j & 63);
                counts[i].push_back(c);
            }
        }
        return 0;
    }
    int refine(PnPState* const* S, int count, const int* spec_j, const int* /*pause_k*/, const int* adopt_k,
               const int* rows_after, int* rcount, float (*rpose)[12]) override {
        for (int i = 0; i < count; ++i) {
            EmuPnP* p = of(S[i]);
            PnPState& s = *S[i];
            if (adopt_k[i] >= 0) {
                EmuPnP* q = spec[spec_j[i]];
                p->best = q->masks[adopt_k[i]];
                pose12_to_T(&q->poses[12 * adopt_k[i]], s.mBestTcw);
            }
            int r = 0;
            for (int j = 0; j < s.N; ++j)
                if ((p->best[j >> 6] >> (j & 63)) & 1ull) {
                    for (int c = 0; c < 3; ++c) p->pws[3 * r + c] = p->pts4[4 * j + c];
                    p->us[2 * r] = p->uv[2 * j]; p->us[2 * r + 1] = p->uv[2 * j + 1];
                    ++r;
                }
            const float K[4] = {s.fx, s.fy, s.cx, s.cy};
            float R[9], t[3];
            he_pnp_rows(r, rows_after[i], p->pws.data(), p->us.data(), p->als.data(), K, R, t);
            std::vector<uint8_t> m(s.N);
            rcount[i] = he_pnp_count(R, t, K, s.th2, s.N, p->pts4.data(), p->uv.data(), m.data());
            p->refined.assign(p->words, 0);
            for (int j = 0; j < s.N; ++j) if (m[j]) p->refined[j >> 6] |= 1ull << (j & 63);
            std::memcpy(rpose[i], R, 36);
            std::memcpy(rpose[i] + 9, t, 12);
        }
        return 0;
    }
    int fetch_mask(PnPState* const* S, int count, const int* kind, uint8_t* const* out) override {
        for (int i = 0; i < count; ++i) {
            EmuPnP* p = of(S[i]);
            const std::vector<uint64_t>& w = kind[i] == 1 ? p->refined : p->best;
            std::memset(out[i], 0, S[i]->N_points);
            for (int j = 0; j < S[i]->N; ++j) if ((w[j >> 6] >> (j & 63)) & 1ull) out[i][S[i]->kp_index[j]] = 1;
        }
        return 0;
    }
};

}  // namespace

extern "C" {

void* he_pnp_create(int n, int n_points, const float* p2d, const float* p3dw, const float* sigma2,
                    const int32_t* kp_index, float fx, float fy, float cx, float cy, uint32_t seed) {
    EmuPnP* p = new EmuPnP();
    PnPState& s = p->st;
    s.N = n; s.N_points = n_points; s.fx = fx; s.fy = fy; s.cx = cx; s.cy = cy;
    s.kp_index.assign(kp_index, kp_index + n);
    s.sigma2.assign(sigma2, sigma2 + n);
    s.reset(seed);
    p->pts4.resize(4 * (size_t)n);
    p->uv.assign(p2d, p2d + 2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        for (int c = 0; c < 3; ++c) p->pts4[4 * i + c] = p3dw[3 * i + c];
        p->pts4[4 * i + 3] = sigma2[i];
    }
    const size_t cap = std::max(n, 8);
    p->pws.assign(3 * cap, 0.0); p->us.assign(2 * cap, 0.0); p->als.assign(4 * cap, 0.0);
    p->words = (std::max(n, 1) + 63) / 64;
    p->best.assign(p->words, 0); p->refined.assign(p->words, 0);
    pnp_set_params(s, 0.99, 8, 300, 4, 0.4f, 5.991f);
    return p;
}
void he_pnp_destroy(void* h) { delete static_cast<EmuPnP*>(h); }
void he_pnp_set_params(void* h, double prob, int mi, int mx, int ms, float eps, float th2) {
    pnp_set_params(static_cast<EmuPnP*>(h)->st, prob, mi, mx, ms, eps, th2);
}
// results: per solver int4 (ok, no_more, n_inliers, iterations) + T[16]; masks n_points bytes each
int he_pnp_iterate_many(void** hs, int count, const int32_t* its, int32_t* out_i4, float* out_T, uint8_t** masks) {
    EmuPnPBackend be;
    std::vector<PnPState*> S(count);
    std::vector<int> n(its, its + count);
    for (int i = 0; i < count; ++i) { be.all.push_back(static_cast<EmuPnP*>(hs[i])); S[i] = &be.all[i]->st; }
    std::vector<PnPResult> res(count);
    int st = pnp_iterate_many(be, S.data(), count, n.data(), res.data(), masks);
    for (int i = 0; i < count; ++i) {
        out_i4[4 * i] = res[i].ok; out_i4[4 * i + 1] = res[i].no_more; out_i4[4 * i + 2] = res[i].n_inliers;
        out_i4[4 * i + 3] = res[i].iterations;
        if (res[i].ok) std::memcpy(out_T + 16 * i, res[i].T, 64);
        if (!res[i].ok && masks && masks[i]) masks[i][0] = 0;
    }
    return st;
}
void he_pnp_state(void* h, int32_t* out) {
    const PnPState& t = static_cast<EmuPnP*>(h)->st;
    out[0] = t.mnIterations; out[1] = t.mRansacMaxIts; out[2] = t.mRansacMinInliers; out[3] = t.mnBestInliers;
    out[4] = t.max_rows;
}

}  // extern "C"

template <int NS>
static void mlpnp_hyp(const uint32_t* window, int g0, int h, int n, const float* pts4, const float* brg2,
                      int32_t* idx_out, double* R, double* t, const double* cov = nullptr) {
    uint32_t w[31];
    std::memcpy(w, window, sizeof(w));
    uint32_t words[NS];
    for (int d = 0; d < NS; ++d) words[d] = rng_word(tab().T.data(), w, g0 + h * NS + d);
    int idx[NS];
    swap_remove_sample<NS>(words, NS, n, idx);
    double pw[NS][3], f[NS][3];
    for (int i = 0; i < NS; ++i) {
        for (int c = 0; c < 3; ++c) pw[i][c] = pts4[4 * idx[i] + c];
        f[i][0] = brg2[2 * idx[i]];
        f[i][1] = brg2[2 * idx[i] + 1];
        f[i][2] = 1.0;
        idx_out[i] = idx[i];
    }
    std::vector<double> slab(kMlSlabDoubles);
    LaneMat S{slab.data(), 1};
    double Rm[3][3], tv[3];
    if (cov) {
        mlpnp_compute_pose<NS>(pw, f, S, Rm, tv, MlIndexedCov{cov, idx});
    } else {
        mlpnp_compute_pose<NS>(pw, f, S, Rm, tv);
    }
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R[3 * r + c] = Rm[r][c];
    for (int r = 0; r < 3; ++r) t[r] = tv[r];
}

extern "C" {
// MLPnP hypothesis h of a stream (window, g0): sample, device-path computePose (double R, t).
int he_mlpnp_hypothesis(int ns, const uint32_t* window, int g0, int h, int n, const float* pts4, const float* brg2,
                        int32_t* idx, double* R, double* t) {
    switch (ns) {
        case 6: mlpnp_hyp<6>(window, g0, h, n, pts4, brg2, idx, R, t); return 0;
        case 7: mlpnp_hyp<7>(window, g0, h, n, pts4, brg2, idx, R, t); return 0;
        case 8: mlpnp_hyp<8>(window, g0, h, n, pts4, brg2, idx, R, t); return 0;
    }
    return -1;
}
// The same with per-correspondence bearing covariances cov [n][9] (computePose's covMats branch).
int he_mlpnp_hypothesis_cov(int ns, const uint32_t* window, int g0, int h, int n, const float* pts4,
                            const float* brg2, const double* cov, int32_t* idx, double* R, double* t) {
    switch (ns) {
        case 6: mlpnp_hyp<6>(window, g0, h, n, pts4, brg2, idx, R, t, cov); return 0;
        case 7: mlpnp_hyp<7>(window, g0, h, n, pts4, brg2, idx, R, t, cov); return 0;
        case 8: mlpnp_hyp<8>(window, g0, h, n, pts4, brg2, idx, R, t, cov); return 0;
    }
    return -1;
}

int he_mlpnp_count(const double* R, const double* t, const float* K, float th2, int n, const float* pts4,
                   const float* uv2, uint8_t* mask) {
    double Rr[9], tt[3];
    std::memcpy(Rr, R, sizeof(Rr));
    std::memcpy(tt, t, sizeof(tt));
    int c = 0;
    for (int i = 0; i < n; ++i) {
        const bool in = mlpnp_inlier(Rr, tt, K[0], K[1], K[2], K[3], pts4[4 * i], pts4[4 * i + 1], pts4[4 * i + 2],
                                     uv2[2 * i], uv2[2 * i + 1], pts4[4 * i + 3] * th2);
        mask[i] = in;
        c += in;
    }
    return c;
}

// PoseOptimization in the device orchestration (poseopt.hip), run sequentially: the same per-edge
// functions, the same fused passes (errors + robust chi2 + system at one estimate, the trial's
// system adopted when the trial is accepted) and the same edge-order folds over the active edges —
// the CPU tests check it against the oracle's literal g2o control flow.  xw4 [n][4] = (X, Y, Z, invSigma2), uv [n][2].
// out[16]: Tcw rows 0..2, then n_good, rounds, lm_iterations, lm_trials (as int bits).
void he_pose_optimization(int n, const float* xw4, const float* uv, const float* K4, const float* T12, float* out,
                          uint8_t* outlier, const float* ur /* nullable: all mono */, float bf) {
    using namespace rsc;
    const PoCam K{(double)K4[0], (double)K4[1], (double)K4[2], (double)K4[3], (double)bf};
    const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);
    const double dm = deltaMono, dm2 = dm * dm, ds = deltaStereo, ds2 = ds * ds;
    auto stereo = [&](int e) { return ur && ur[e] >= 0.0f; };
    std::vector<double> err(3 * (size_t)n, 0.0);
    auto edge_error = [&](const PoSE3& est, int e) {
        const double X[3] = {xw4[4 * e], xw4[4 * e + 1], xw4[4 * e + 2]};
        po_error(est, K, X, uv[2 * e], uv[2 * e + 1], stereo(e) ? ur[e] : 0.0, stereo(e), err[3 * e], err[3 * e + 1],
                 err[3 * e + 2]);
    };
    std::vector<uint8_t> lvl(n, 0);
    double R0[3][3], t0[3];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) R0[r][c] = T12[4 * r + c];
        t0[r] = T12[4 * r + 3];
    }
    const PoSE3 init = po_from_Rt(R0, t0);
    for (int e = 0; e < n; ++e) outlier[e] = 0;
    bool robust = true;
    // one fused pass at est over the active edges in edge order (poseopt.hip po_pass): errors stored,
    // the 27 H/b terms (b's negated) and the robust chi2 term folded; returns chi2
    auto pass = [&](const PoSE3& est, double (&H)[6][6], double (&b)[6]) {
        double acc[kPoseTerms + 1];
        for (int k = 0; k <= kPoseTerms; ++k) acc[k] = 0.0;
        for (int e = 0; e < n; ++e) {
            if (lvl[e]) continue;
            edge_error(est, e);
            const double X[3] = {xw4[4 * e], xw4[4 * e + 1], xw4[4 * e + 2]};
            const bool st = stereo(e);
            double t[kPoseTerms];
            if (!po_quad_terms_finite(est, K, X, xw4[4 * e + 3], err[3 * e], err[3 * e + 1], err[3 * e + 2], st, robust,
                                      st ? ds : dm, st ? ds2 : dm2, t))
                po_quad_terms(est, K, X, xw4[4 * e + 3], err[3 * e], err[3 * e + 1], err[3 * e + 2], st, robust,
                              st ? ds : dm, st ? ds2 : dm2, t);
            const double tc = po_chi_term(robust, st, xw4[4 * e + 3], err[3 * e], err[3 * e + 1], err[3 * e + 2],
                                          st ? ds : dm, st ? ds2 : dm2);
            for (int k = 0; k < kPoseTerms; ++k) acc[k] = acc[k] + ((k >= 21) ? -t[k] : t[k]);
            acc[kPoseTerms] = acc[kPoseTerms] + tc;
        }
        int k = 0;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j <= i; ++j) { H[i][j] = acc[k++]; H[j][i] = H[i][j]; }
        for (int i = 0; i < 6; ++i) b[i] = acc[21 + i];
        return acc[kPoseTerms];
    };
    double x[6] = {0, 0, 0, 0, 0, 0};
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, rounds = 0, lm_its = 0, lm_trials = 0, nBad = 0;
    PoSE3 est = init;
    for (int it = 0; it < 4; ++it) {
        rounds++;
        est = init;
        bool any = false;
        for (int e = 0; e < n; ++e) any |= (lvl[e] == 0);
        if (any) {
            double H[6][6], b[6];
            double chiEst = pass(est, H, b);
            bool ok = true;
            for (int i = 0; i < 10 && ok; ++i) {
                lm_its++;
                double currentChi = chiEst;
                const double iniChi = currentChi;
                if (i == 0) {
                    double maxDiagonal = 0.;
                    for (int j = 0; j < 6; ++j) { const double a = std::fabs(H[j][j]); maxDiagonal = (a < maxDiagonal) ? maxDiagonal : a; }
                    lambda = 1e-5 * maxDiagonal;
                    ni = 2;
                    nBadLM = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    lm_trials++;
                    double Hd[6][6];
                    for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) Hd[r][c] = H[r][c];
                    for (int r = 0; r < 6; ++r) Hd[r][r] += lambda;
                    double xs[6];
                    const bool ok2 = po_ldlt_solve6(Hd, b, xs);
                    if (ok2) for (int j = 0; j < 6; ++j) x[j] = xs[j];
                    const PoSE3 trial = po_mul(po_exp(x), est);
                    double Ht[6][6], bt[6];
                    const double chiT = pass(trial, Ht, bt);
                    const double tempChi = ok2 ? chiT : DBL_MAX;
                    rho = (currentChi - tempChi);
                    double scale = 0.;
                    for (int j = 0; j < 6; ++j) scale += x[j] * (lambda * x[j] + b[j]);
                    scale += 1e-3;
                    rho /= scale;
                    if (rho > 0 && std::isfinite(tempChi)) {
                        double alpha = 1. - po_cube(2 * rho - 1);
                        alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;
                        const double scaleFactor = (1. / 3. < alpha) ? alpha : 1. / 3.;
                        lambda *= scaleFactor;
                        ni = 2;
                        currentChi = tempChi;
                        est = trial;
                        std::memcpy(H, Ht, sizeof(H));
                        std::memcpy(b, bt, sizeof(b));
                        chiEst = chiT;
                    } else {
                        lambda *= ni;
                        ni *= 2;
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                if (qmax == 10 || rho == 0) ok = false;
                else {
                    if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                    else nBadLM = 0;
                    ok = nBadLM < 3;
                }
            }
        }
        nBad = 0;
        for (int e = 0; e < n; ++e) {
            if (lvl[e]) edge_error(est, e);
            const float c2 = (float)po_chi2(xw4[4 * e + 3], stereo(e), err[3 * e], err[3 * e + 1], err[3 * e + 2]);
            const bool bad = c2 > (stereo(e) ? 7.815f : 5.991f);
            lvl[e] = bad;
            outlier[e] = bad;
            nBad += bad;
        }
        if (it == 2) robust = false;
        if (n < 10) break;
    }
    double R[3][3];
    po_quat_to_R(est.r, R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) out[4 * r + c] = (float)R[r][c];
        out[4 * r + 3] = (float)est.t[r];
    }
    const int ints[4] = {n - nBad, rounds, lm_its, lm_trials};
    std::memcpy(out + 12, ints, 16);
}

// The PoseOptimization folds of n edges at one estimate, with the full po_quad_terms (out[0..27]) and
// with the kernel's form (po_quad_terms_finite, po_quad_terms for an edge outside its precondition;
// out[28..55]); flags[e] bit 0 = stereo, bit 1 = robust; pose7 = quaternion (x, y, z, w), t; K5 =
// fx, fy, cx, cy, bf.  Returns the number of edges that took the full form in the kernel's.
int he_po_fold_compare(int n, const double* X3, const double* e3, const double* inv, const int32_t* flags,
                       const double* pose7, const double* K5, double* out) {
    using namespace rsc;
    PoSE3 est;
    est.r.x = pose7[0]; est.r.y = pose7[1]; est.r.z = pose7[2]; est.r.w = pose7[3];
    for (int i = 0; i < 3; ++i) est.t[i] = pose7[4 + i];
    const PoCam K{K5[0], K5[1], K5[2], K5[3], K5[4]};
    const double dm = (double)std::sqrt(5.991f), ds = (double)std::sqrt(7.815f);
    double a[kPoseTerms], b[kPoseTerms];
    for (int k = 0; k < kPoseTerms; ++k) a[k] = b[k] = 0.0;
    int full = 0;
    for (int e = 0; e < n; ++e) {
        const double X[3] = {X3[3 * e], X3[3 * e + 1], X3[3 * e + 2]};
        const bool st = flags[e] & 1, rb = flags[e] & 2;
        const double delta = st ? ds : dm, dsqr = delta * delta;
        double t[kPoseTerms], f[kPoseTerms];
        po_quad_terms(est, K, X, inv[e], e3[3 * e], e3[3 * e + 1], e3[3 * e + 2], st, rb, delta, dsqr, t);
        if (!po_quad_terms_finite(est, K, X, inv[e], e3[3 * e], e3[3 * e + 1], e3[3 * e + 2], st, rb, delta, dsqr, f)) {
            po_quad_terms(est, K, X, inv[e], e3[3 * e], e3[3 * e + 1], e3[3 * e + 2], st, rb, delta, dsqr, f);
            ++full;
        }
        for (int k = 0; k < kPoseTerms; ++k) {
            a[k] = (k >= 21) ? a[k] + (-t[k]) : a[k] + t[k];
            b[k] = (k >= 21) ? b[k] + (-f[k]) : b[k] + f[k];
        }
    }
    for (int k = 0; k < kPoseTerms; ++k) {
        out[k] = a[k];
        out[kPoseTerms + 1 + k] = b[k];
    }
    out[kPoseTerms] = out[2 * kPoseTerms + 1] = 0.0;
    return full;
}

// OptimizeSim3 in the device orchestration (sim3opt.hip), run sequentially: the same per-edge
// functions, the same fused passes, terms in the edge order e12_0, e21_0, ..., the same folds.  Inputs already compacted:
// e12/e21 [m][4] = (X, invSigma2), uv [m][4]; S[8] in/out; keep[m]; stats[4] = nIn, nBad, its, trials.
void he_optimize_sim3(int m, const float* e12, const float* e21, const float* uv, const float* K8, float th2,
                      double* S8, uint8_t* keep, int32_t* stats) {
    using namespace rsc;
    const SoCam K1{(double)K8[0], (double)K8[1], (double)K8[2], (double)K8[3]};
    const SoCam K2{(double)K8[4], (double)K8[5], (double)K8[6], (double)K8[7]};
    const float deltaHuber = std::sqrt(th2);
    const double delta = deltaHuber, dsqr = delta * delta;
    std::vector<double> err(4 * (size_t)m, 0.0);
    auto load = [&](int c, bool inv_edge, double (&X)[3], double& u, double& v, double& inv) {
        const float* a = (inv_edge ? e21 : e12) + 4 * (size_t)c;
        X[0] = a[0]; X[1] = a[1]; X[2] = a[2];
        inv = a[3];
        u = uv[4 * c + (inv_edge ? 2 : 0)];
        v = uv[4 * c + (inv_edge ? 3 : 1)];
    };
    // one fused pass at S over the kept correspondences' edges in g2o's order (sim3opt.hip so_pass):
    // errors stored, the 35 H/b terms and the robust chi2 term folded; returns chi2
    auto pass = [&](const SoSim3& S, double (&H)[7][7], double (&b)[7]) {
        SoPerturbed Pt;
        so_perturb(S, Pt);
        const SoSim3 Si = so_inverse(S);
        double acc[kSim3OptTerms + 1];
        for (int k = 0; k <= kSim3OptTerms; ++k) acc[k] = 0.0;
        for (int c = 0; c < m; ++c) {
            if (!keep[c]) continue;
            for (int side = 0; side < 2; ++side) {
                double X[3], u, v, inv, r0, r1;
                load(c, side == 1, X, u, v, inv);
                double& e0 = err[4 * c + 2 * side];
                double& e1 = err[4 * c + 2 * side + 1];
                so_edge_error(side ? Si : S, side ? K2 : K1, X, u, v, e0, e1);
                po_huber(po_chi2(inv, false, e0, e1, 0.0), delta, dsqr, r0, r1);
                double t[kSim3OptTerms];
                so_quad_terms(Pt, side == 1, side ? K2 : K1, X, u, v, inv, e0, e1, delta, dsqr, t);
                for (int k = 0; k < kSim3OptTerms; ++k) acc[k] = acc[k] + t[k];
                acc[kSim3OptTerms] = acc[kSim3OptTerms] + r0;
            }
        }
        int k = 0;
        for (int i = 0; i < 7; ++i)
            for (int j = 0; j <= i; ++j) { H[i][j] = acc[k++]; H[j][i] = H[i][j]; }
        for (int i = 0; i < 7; ++i) b[i] = acc[28 + i];
        return acc[kSim3OptTerms];
    };
    double x[7] = {0, 0, 0, 0, 0, 0, 0};
    double lambda = -1.0, ni = 2.0;
    int nBadLM = 0, its = 0, trials = 0;
    auto optimize = [&](SoSim3& S, int iterations) {
        bool any = false;
        for (int c = 0; c < m; ++c) any |= keep[c] != 0;
        if (!any) return;
        double H[7][7], b[7];
        double chiS = pass(S, H, b);
        bool ok = true;
        for (int i = 0; i < iterations && ok; ++i) {
            its++;
            double currentChi = chiS;
            const double iniChi = currentChi;
            if (i == 0) {
                double maxDiagonal = 0.;
                for (int j = 0; j < 7; ++j) { const double a = std::fabs(H[j][j]); maxDiagonal = (a < maxDiagonal) ? maxDiagonal : a; }
                lambda = 1e-5 * maxDiagonal;
                ni = 2;
                nBadLM = 0;
            }
            double rho = 0;
            int qmax = 0;
            do {
                trials++;
                double Hd[7][7];
                for (int r = 0; r < 7; ++r) for (int c = 0; c < 7; ++c) Hd[r][c] = H[r][c];
                for (int r = 0; r < 7; ++r) Hd[r][r] += lambda;
                double xs[7];
                const bool ok2 = po_ldlt_solve<7>(Hd, b, xs);
                if (ok2) for (int j = 0; j < 7; ++j) x[j] = xs[j];
                const SoSim3 trial = so_oplus(x, S);
                double Ht[7][7], bt[7];
                const double chiT = pass(trial, Ht, bt);
                const double tempChi = ok2 ? chiT : DBL_MAX;
                rho = (currentChi - tempChi);
                double scale = 0.;
                for (int j = 0; j < 7; ++j) scale += x[j] * (lambda * x[j] + b[j]);
                scale += 1e-3;
                rho /= scale;
                if (rho > 0 && std::isfinite(tempChi)) {
                    double alpha = 1. - po_cube(2 * rho - 1);
                    alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;
                    const double scaleFactor = (1. / 3. < alpha) ? alpha : 1. / 3.;
                    lambda *= scaleFactor;
                    ni = 2;
                    currentChi = tempChi;
                    S = trial;
                    std::memcpy(H, Ht, sizeof(H));
                    std::memcpy(b, bt, sizeof(b));
                    chiS = chiT;
                } else {
                    lambda *= ni;
                    ni *= 2;
                }
                qmax++;
            } while (rho < 0 && qmax < 10);
            if (qmax == 10 || rho == 0) ok = false;
            else {
                if ((iniChi - currentChi) * 1e3 < iniChi) nBadLM++;
                else nBadLM = 0;
                ok = nBadLM < 3;
            }
        }
    };
    auto outlier = [&](int c) {
        return po_chi2(e12[4 * c + 3], false, err[4 * c], err[4 * c + 1], 0.0) > (double)th2 ||
               po_chi2(e21[4 * c + 3], false, err[4 * c + 2], err[4 * c + 3], 0.0) > (double)th2;
    };
    SoSim3 S;
    S.r.x = S8[0]; S.r.y = S8[1]; S.r.z = S8[2]; S.r.w = S8[3];
    S.t[0] = S8[4]; S.t[1] = S8[5]; S.t[2] = S8[6];
    S.s = S8[7];
    for (int c = 0; c < m; ++c) keep[c] = 1;
    optimize(S, 5);
    int nBad = 0;
    for (int c = 0; c < m; ++c)
        if (outlier(c)) { keep[c] = 0; ++nBad; }
    int nIn = 0;
    if (m - nBad >= 10) {
        optimize(S, nBad > 0 ? 10 : 5);
        for (int c = 0; c < m; ++c) {
            if (!keep[c]) continue;
            if (outlier(c)) keep[c] = 0;
            else ++nIn;
        }
        S8[0] = S.r.x; S8[1] = S.r.y; S8[2] = S.r.z; S8[3] = S.r.w;
        S8[4] = S.t[0]; S8[5] = S.t[1]; S8[6] = S.t[2];
        S8[7] = S.s;
    }
    stats[0] = nIn; stats[1] = nBad; stats[2] = its; stats[3] = trials;
}

// 12x12 symmetric eigen-decomposition checks of the event-form implicit QR: A (row-major, lower
// triangle read) -> Householder tridiagonalisation (sym_eig12_tridiag), then both tridiag_qr and
// tridiag_qr_events12 on copies.  out_*: diag after the QR (sorted when ok), perm, Q (144), ok.
void he_qr_compare(const double* A, double* d_ref, int32_t* p_ref, double* q_ref, int32_t* ok_ref, double* d_ev,
                   int32_t* p_ev, double* q_ev, int32_t* ok_ev) {
    using namespace rsc;
    std::vector<double> M(A, A + 144);
    LaneMat L{M.data(), 1};
    double diag[12], sub[11];
    sym_eig12_tridiag(L, diag, sub);
    std::vector<double> Q1(M), Q2(M);
    {
        auto qapply = [&](int k, double c, double s, bool apply) {
            for (int i = 0; i < 12; ++i) {
                const double xi = Q1[i * 12 + k], yi = Q1[i * 12 + k + 1];
                Q1[i * 12 + k] = apply ? c * xi - s * yi : xi;
                Q1[i * 12 + k + 1] = apply ? s * xi + c * yi : yi;
            }
        };
        double dg[12], sb[11];
        std::memcpy(dg, diag, sizeof(dg));
        std::memcpy(sb, sub, sizeof(sb));
        int perm[12];
        *ok_ref = tridiag_qr<double, 12>(dg, sb, qapply, perm);
        for (int i = 0; i < 12; ++i) { d_ref[i] = dg[i]; p_ref[i] = perm[i]; }
        std::memcpy(q_ref, Q1.data(), 144 * 8);
    }
    {
        struct Rows {
            double* q;
            double load(int r, int c) const { return q[r * 12 + c]; }
            void store(int r, int c, double v) { q[r * 12 + c] = v; }
        } rows{Q2.data()};
        double ds[23];
        std::memcpy(ds, diag, 96);
        std::memcpy(ds + 12, sub, 88);
        int perm[12];
        *ok_ev = tridiag_qr_events12<12>(ds, rows, perm);
        for (int i = 0; i < 12; ++i) p_ev[i] = perm[i];
        std::memcpy(q_ev, Q2.data(), 144 * 8);
        // the event form returns the sorted order via perm and leaves ds[] unsorted; sort a copy the
        // same way tridiag_qr sorts its diag for the comparison
        double d2[12];
        int pp[12];
        for (int i = 0; i < 12; ++i) { d2[i] = ds[i]; pp[i] = i; }
        if (*ok_ev) eig_sort<double, 12>(d2, pp);
        for (int i = 0; i < 12; ++i) d_ev[i] = d2[i];
    }
}
// The split chase (QrChase12 + QrRowApply, rsc_core.h) with the log cut into chunks of `cap`
// rotations, as the eigen-stage kernel replays it: eigenvalues (sorted), perm, Q, converged flag.
void he_qr_split(const double* A, int cap, double* d_out, int32_t* p_out, double* q_out, int32_t* ok_out) {
    using namespace rsc;
    std::vector<double> M(A, A + 144);
    LaneMat L{M.data(), 1};
    double diag[12], sub[11];
    sym_eig12_tridiag(L, diag, sub);
    double ds[23];
    std::memcpy(ds, diag, 96);
    std::memcpy(ds + 12, sub, 88);
    auto DS = [&](int i) -> double& { return ds[i]; };
    QrChase12 ch;
    ch.init(DS);
    std::vector<int> lk(cap);
    std::vector<double> lc(cap), ls(cap);
    QrRowApply ra[12];
    while (true) {
        const int nl = ch.run(DS, [&](int e, int k, double c, double s) { lk[e] = k; lc[e] = c; ls[e] = s; }, cap);
        for (int e = 0; e < nl; ++e)
            for (int r = 0; r < 12; ++r) ra[r].step(&M[r * 12], lk[e], lc[e], ls[e]);
        if (!ch.active) break;
    }
    for (int r = 0; r < 12; ++r) ra[r].flush(&M[r * 12]);
    *ok_out = ch.converged();
    double d2[12];
    int pp[12];
    for (int i = 0; i < 12; ++i) { d2[i] = ds[i]; pp[i] = i; }
    if (*ok_out) eig_sort<double, 12>(d2, pp);
    for (int i = 0; i < 12; ++i) { d_out[i] = d2[i]; p_out[i] = pp[i]; }
    std::memcpy(q_out, M.data(), 144 * 8);
}
}  // extern "C"
