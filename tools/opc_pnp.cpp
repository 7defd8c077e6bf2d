// Op-counter build of the EPnP oracle (tools/opcount_report.py loads libopcount.so).
#include "opcount_scalar.h"
#define double CntD
#include "../oracle/pnp_oracle.cpp"
#undef double

extern "C" void* opc_pnp_create(int n, const float* p2d, const float* p3dw, const float* sigma2, float fx, float fy,
                                float cx, float cy) {
    std::vector<int32_t> kp(n);
    for (int i = 0; i < n; ++i) kp[i] = i;
    return new rsc_oracle::PnPOracle(n, n, p2d, p3dw, sigma2, kp.data(), fx, fy, cx, cy, 1);
}
extern "C" void opc_pnp_destroy(void* h) { delete static_cast<rsc_oracle::PnPOracle*>(h); }
// FP64 flops of compute_pose on the k correspondences idx (a 4-point hypothesis or a Refine set)
extern "C" double opc_pnp_compute_pose(void* h, const int* idx, int k) {
    float R[9], t[3];
    g_flops = g_sqrt = g_div = 0;
    static_cast<rsc_oracle::PnPOracle*>(h)->compute_pose_public(idx, k, R, t);
    return (double)g_flops;
}
