// Op-counter build of the PoseOptimization oracle (tools/opcount_report.py loads libopcount.so).
#include <vector>
#include "opcount_libm.h"
#define double CntD
#include "../oracle/poseopt_oracle.cpp"
#undef double

extern "C" double opc_pose_optimization(int n, const float* uv, const float* Xw, const float* inv_sigma2, float fx,
                                        float fy, float cx, float cy, const float* Tcw_in, const float* u_right,
                                        float bf, int32_t* stats) {
    using namespace rsc_oracle;
    PoseOptInput in{n, nullptr, uv, Xw, inv_sigma2, fx, fy, cx, cy, {}, u_right, bf};
    std::memcpy(in.Tcw, Tcw_in, sizeof(in.Tcw));
    float T[16];
    std::vector<uint8_t> out(n > 0 ? n : 1);
    PoseOptStats st{};
    g_flops = g_sqrt = g_div = 0;
    pose_optimization(in, T, out.data(), &st);
    if (stats) { stats[0] = st.rounds; stats[1] = st.lm_iterations; stats[2] = st.lm_trials; }
    return (double)g_flops;
}
