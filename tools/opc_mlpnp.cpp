// Op-counter build of the MLPnP oracle (tools/opcount_report.py loads libopcount.so).
#include "opcount_libm.h"
#define double CntD
#include "../oracle/mlpnp_oracle.cpp"
#undef double

extern "C" void* opc_mlpnp_create(int n, const float* p2d, const float* p3dw, const float* sigma2, float fx, float fy,
                                  float cx, float cy) {
    std::vector<int32_t> kp(n);
    for (int i = 0; i < n; ++i) kp[i] = i;
    return new rsc_oracle::MLPnPOracle(n, n, p2d, p3dw, sigma2, kp.data(), fx, fy, cx, cy, 1);
}
extern "C" void opc_mlpnp_destroy(void* h) { delete static_cast<rsc_oracle::MLPnPOracle*>(h); }
extern "C" double opc_mlpnp_compute_pose(void* h, const int* idx, int k) {
    CntD R[9], t[3];
    g_flops = g_sqrt = g_div = 0;
    static_cast<rsc_oracle::MLPnPOracle*>(h)->compute_pose_public(idx, k, R, t);
    return (double)g_flops;
}
