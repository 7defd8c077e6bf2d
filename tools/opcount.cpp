// opcount — FP64 operation counter build of the CPU restatement (SURVEY.md §8(d) "Solve FLOPs S_h":
// "measure it by an op-counter build of the CPU restatement and report mean ± σ per config").
//
// The oracle's EPnP (oracle/pnp_oracle.cpp, test infrastructure) is compiled a second time with
// `double` replaced by a counting scalar, then compute_pose() is run on the minimal 4-point samples
// of a config-2 scene.  Counted: +, -, *, / (1 flop each), sqrt (1 flop, also counted apart),
// comparisons are not flops.  Output: one JSON line {mean, std, min, max, sqrt, div, samples}.
// Measurement tooling only; the product never links this.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <type_traits>
#include <vector>

static uint64_t g_flops = 0, g_sqrt = 0, g_div = 0;

struct CntD {
    double v;
    CntD() = default;
    CntD(double x) : v(x) {}
    explicit operator double() const { return v; }
    explicit operator float() const { return (float)v; }
    explicit operator int() const { return (int)v; }
    explicit operator bool() const { return v != 0.0; }
    CntD& operator+=(CntD o) { ++g_flops; v += o.v; return *this; }
    CntD& operator-=(CntD o) { ++g_flops; v -= o.v; return *this; }
    CntD& operator*=(CntD o) { ++g_flops; v *= o.v; return *this; }
    CntD& operator/=(CntD o) { ++g_flops; ++g_div; v /= o.v; return *this; }
    CntD operator-() const { return CntD(-v); }
    CntD operator+() const { return *this; }
};
static_assert(sizeof(CntD) == 8 && std::is_trivially_copyable<CntD>::value, "layout");

template <class T> using arith = typename std::enable_if<std::is_arithmetic<T>::value, int>::type;
#define CNT_BINOP(op, extra)                                                                          \
    inline CntD operator op(CntD a, CntD b) { ++g_flops; extra; return CntD(a.v op b.v); }            \
    template <class T, arith<T> = 0> inline CntD operator op(CntD a, T b) { ++g_flops; extra; return CntD(a.v op (double)b); } \
    template <class T, arith<T> = 0> inline CntD operator op(T a, CntD b) { ++g_flops; extra; return CntD((double)a op b.v); }
CNT_BINOP(+, )
CNT_BINOP(-, )
CNT_BINOP(*, )
CNT_BINOP(/, ++g_div)
#define CNT_CMP(op)                                                                                   \
    inline bool operator op(CntD a, CntD b) { return a.v op b.v; }                                   \
    template <class T, arith<T> = 0> inline bool operator op(CntD a, T b) { return a.v op (double)b; } \
    template <class T, arith<T> = 0> inline bool operator op(T a, CntD b) { return (double)a op b.v; }
CNT_CMP(<)
CNT_CMP(>)
CNT_CMP(<=)
CNT_CMP(>=)
CNT_CMP(==)
CNT_CMP(!=)

namespace std {
inline CntD sqrt(CntD x) { ++g_flops; ++g_sqrt; return CntD(::sqrt(x.v)); }
inline CntD fabs(CntD x) { return CntD(::fabs(x.v)); }
inline CntD abs(CntD x) { return CntD(::fabs(x.v)); }
inline CntD log(CntD x) { ++g_flops; return CntD(::log(x.v)); }
inline CntD ceil(CntD x) { return CntD(::ceil(x.v)); }
inline CntD pow(CntD x, CntD y) { ++g_flops; return CntD(::pow(x.v, y.v)); }
template <class T, arith<T> = 0> inline CntD pow(CntD x, T y) { ++g_flops; return CntD(::pow(x.v, (double)y)); }
template <class T, arith<T> = 0> inline CntD pow(T x, CntD y) { ++g_flops; return CntD(::pow((double)x, y.v)); }
template <> class numeric_limits<CntD> : public numeric_limits<decltype(0.0)> {};
}  // namespace std

#define double CntD
#include "../oracle/pnp_oracle.cpp"
#undef double

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    const int samples = argc > 2 ? atoi(argv[2]) : 20000;
    // Config-2 shaped scene: frustum points at depth [0.5, 8] m, EuRoC intrinsics, 40% inliers.
    const float fx = 435.2046959714599f, fy = 435.2046959714599f, cx = 367.4517211914062f, cy = 252.2008514404297f;
    std::mt19937_64 g(2024);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> G(0.0, 1.0);
    std::vector<float> p2d(2 * n), p3d(3 * n), s2(n, 1.f);
    std::vector<int32_t> kp(n);
    const double ang = 0.7, ca = std::cos(ang), sa = std::sin(ang);
    for (int i = 0; i < n; ++i) {
        const double u = 752 * U(g), v = 480 * U(g), d = 0.5 + 7.5 * U(g);
        const double xc = (u - cx) / fx * d, yc = (v - cy) / fy * d, zc = d;
        // Xw = R^T (Xc - t), R = rot_z(ang), t = (0.3, -0.2, 0.5)
        const double a = xc - 0.3, b = yc + 0.2, c = zc - 0.5;
        p3d[3 * i] = (float)(ca * a + sa * b);
        p3d[3 * i + 1] = (float)(-sa * a + ca * b);
        p3d[3 * i + 2] = (float)c;
        const bool inl = U(g) < 0.4;
        p2d[2 * i] = (float)(inl ? u + G(g) : 752 * U(g));
        p2d[2 * i + 1] = (float)(inl ? v + G(g) : 480 * U(g));
        kp[i] = i;
    }
    rsc_oracle::PnPOracle o(n, n, p2d.data(), p3d.data(), s2.data(), kp.data(), fx, fy, cx, cy, 1);
    std::vector<double> f(samples);
    uint64_t sq = 0, dv = 0;
    std::uniform_int_distribution<int> pick(0, n - 1);
    for (int s = 0; s < samples; ++s) {
        int idx[4];
        for (int k = 0; k < 4; ++k) {
            bool dup;
            do {
                idx[k] = pick(g);
                dup = false;
                for (int j = 0; j < k; ++j) dup |= idx[j] == idx[k];
            } while (dup);
        }
        float R[9], t[3];
        g_flops = g_sqrt = g_div = 0;
        o.compute_pose_public(idx, 4, R, t);
        f[s] = (double)g_flops;
        sq += g_sqrt;
        dv += g_div;
    }
    double mean = 0, var = 0, mn = 1e300, mx = 0;
    for (double x : f) { mean += x; mn = std::min(mn, x); mx = std::max(mx, x); }
    mean /= samples;
    for (double x : f) var += (x - mean) * (x - mean);
    printf("{\"config\": \"pnp_epnp_compute_pose (4-point sample)\", \"fp64_flops_mean\": %.1f, \"std\": %.1f, "
           "\"min\": %.0f, \"max\": %.0f, \"sqrt_mean\": %.2f, \"div_mean\": %.2f, \"samples\": %d}\n",
           mean, std::sqrt(var / samples), mn, mx, (double)sq / samples, (double)dv / samples, samples);
    return 0;
}
