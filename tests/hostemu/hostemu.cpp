// TEST-ONLY host build of the product's per-lane device numerics (rsc_core.h / rsc_epnp.h /
// rsc_sim3.h / rsc_engine.h RNG).  The product library never contains this code path; it exists
// so that the arithmetic the kernels run can be compared with the oracle on a CPU.
#include <cstdint>
#include <cstring>
#include <vector>
#include "../../orb-slam2-optimized_amd/csrc/rsc_epnp.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_sim3.h"
#include "../../orb-slam2-optimized_amd/csrc/rsc_engine.h"

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

}  // extern "C"
