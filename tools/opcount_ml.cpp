// opcount_ml — FP64 operation count of MLPnPsolver::computePose (SURVEY.md §8(d) "Solve FLOPs S_h"
// for config 4): the oracle restatement (oracle/mlpnp_oracle.cpp) compiled with `double` replaced by
// the counting scalar (opcount_scalar.h), computePose run on 6-point samples of a config-4 shaped
// scene (4096 correspondences, 40 % inliers).  sin / cos / acos / cbrt count one flop per call.
// Output: one JSON line.  Measurement tooling only.
#include <random>
#include <vector>
#include "opcount_scalar.h"
#include "../orb-slam2-optimized_amd/csrc/rsc_math.h"
#include "../oracle/ora_libm.h"

namespace ora_libm {
inline CntD sin(CntD x) { ++g_flops; return CntD(sin(x.v)); }
inline CntD cos(CntD x) { ++g_flops; return CntD(cos(x.v)); }
inline CntD acos(CntD x) { ++g_flops; return CntD(acos(x.v)); }
inline CntD pow_1_3(CntD x) { ++g_flops; return CntD(pow_1_3(x.v)); }
inline CntD pow_3_2(CntD x) { ++g_flops; return CntD(pow_3_2(x.v)); }
}  // namespace ora_libm
namespace rsc {
namespace dm {
inline CntD sin(CntD x) { ++g_flops; return CntD(sin(x.v)); }
inline CntD cos(CntD x) { ++g_flops; return CntD(cos(x.v)); }
inline CntD pow_3_2(CntD x) { ++g_flops; return CntD(pow_3_2(x.v)); }
}  // namespace dm
}  // namespace rsc
inline CntD sqrt(CntD x) { return std::sqrt(x); }  // unqualified sqrt of rsc_mlpnp_jac.h (ADL)
// the shared mlpnpJacs restatement's libm policy on the counting scalar (oracle ORA_JAC_LIBM)
struct OpcJacLibm {
    static CntD sin(CntD x) { return ora_libm::sin(x); }
    static CntD cos(CntD x) { return ora_libm::cos(x); }
    static CntD pow_3_2(CntD x) { return ora_libm::pow_3_2(x); }
};
#define ORA_JAC_LIBM OpcJacLibm
namespace std {
inline bool isfinite(CntD x) { return std::isfinite(x.v); }
inline bool isnan(CntD x) { return std::isnan(x.v); }
}  // namespace std

#define double CntD
#include "../oracle/mlpnp_oracle.cpp"
#undef double

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const int samples = argc > 2 ? atoi(argv[2]) : 5000;
    const float fx = 435.2046959714599f, fy = 435.2046959714599f, cx = 367.4517211914062f, cy = 252.2008514404297f;
    std::mt19937_64 g(2025);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> G(0.0, 1.0);
    std::vector<float> p2d(2 * n), p3d(3 * n), s2(n, 1.f);
    std::vector<int32_t> kp(n);
    const double ang = 0.7, ca = std::cos(ang), sa = std::sin(ang);
    for (int i = 0; i < n; ++i) {
        const double u = 752 * U(g), v = 480 * U(g), d = 0.5 + 7.5 * U(g);
        const double xc = (u - cx) / fx * d, yc = (v - cy) / fy * d, zc = d;
        const double a = xc - 0.3, b = yc + 0.2, c = zc - 0.5;
        p3d[3 * i] = (float)(ca * a + sa * b);
        p3d[3 * i + 1] = (float)(-sa * a + ca * b);
        p3d[3 * i + 2] = (float)c;
        const bool inl = U(g) < 0.4;
        p2d[2 * i] = (float)(inl ? u + G(g) : 752 * U(g));
        p2d[2 * i + 1] = (float)(inl ? v + G(g) : 480 * U(g));
        kp[i] = i;
    }
    rsc_oracle::MLPnPOracle o(n, n, p2d.data(), p3d.data(), s2.data(), kp.data(), fx, fy, cx, cy, 1);
    std::vector<double> f(samples);
    uint64_t sq = 0, dv = 0;
    std::uniform_int_distribution<int> pick(0, n - 1);
    for (int s = 0; s < samples; ++s) {
        int idx[6];
        for (int k = 0; k < 6; ++k) {
            bool dup;
            do {
                idx[k] = pick(g);
                dup = false;
                for (int j = 0; j < k; ++j) dup |= idx[j] == idx[k];
            } while (dup);
        }
        CntD R[9], t[3];
        g_flops = g_sqrt = g_div = 0;
        o.compute_pose_public(idx, 6, R, t);
        f[s] = (double)g_flops;
        sq += g_sqrt;
        dv += g_div;
    }
    double mean = 0, var = 0, mn = 1e300, mx = 0;
    for (double x : f) { mean += x; mn = std::min(mn, x); mx = std::max(mx, x); }
    mean /= samples;
    for (double x : f) var += (x - mean) * (x - mean);
    printf("{\"config\": \"mlpnp_compute_pose (6-point sample, N = %d)\", \"fp64_flops_mean\": %.1f, \"std\": %.1f, "
           "\"min\": %.0f, \"max\": %.0f, \"sqrt_mean\": %.2f, \"div_mean\": %.2f, \"samples\": %d}\n",
           n, mean, std::sqrt(var / samples), mn, mx, (double)sq / samples, (double)dv / samples, samples);
    return 0;
}
