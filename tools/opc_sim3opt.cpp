// Op-counter build of the OptimizeSim3 oracle (tools/opcount_report.py loads libopcount.so).
#include <vector>
#include "opcount_libm.h"
#define double CntD
#include "../oracle/sim3opt_oracle.cpp"
#undef double

extern "C" double opc_optimize_sim3(int n, const uint8_t* valid, const float* X1w, const float* X2w, const float* uv1,
                                    const float* uv2, const float* inv1, const float* inv2, const float* poses,
                                    const float* K, float th2, const double* S0, int32_t* stats) {
    using namespace rsc_oracle;
    Sim3OptInput in;
    in.n = n; in.valid = valid; in.X1w = X1w; in.X2w = X2w; in.uv1 = uv1; in.uv2 = uv2; in.inv1 = inv1;
    in.inv2 = inv2;
    std::memcpy(in.R1w, poses, 36); std::memcpy(in.t1w, poses + 9, 12);
    std::memcpy(in.R2w, poses + 12, 36); std::memcpy(in.t2w, poses + 21, 12);
    std::memcpy(in.K1, K, 16); std::memcpy(in.K2, K + 4, 16);
    in.th2 = th2;
    Sim3Est e;
    for (int k = 0; k < 4; ++k) e.q[k] = S0[k];
    for (int k = 0; k < 3; ++k) e.t[k] = S0[4 + k];
    e.s = S0[7];
    std::vector<uint8_t> keep(n > 0 ? n : 1);
    Sim3OptStats st{};
    g_flops = g_sqrt = g_div = 0;
    optimize_sim3(in, e, keep.data(), &st);
    if (stats) { stats[0] = st.n_correspondences; stats[1] = st.n_bad; stats[2] = st.lm_iterations; stats[3] = st.lm_trials; }
    return (double)g_flops;
}
