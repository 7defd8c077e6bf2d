// rsc_math.h — deterministic double-precision sin, cos, acos and cbrt for host and device.
//
// MLPnPsolver (src/MLPnPsolver.cpp:628-657, :773-1020) calls sin, cos, acos and pow.  glibc's libm
// and the ROCm device libm differ in the last bit for some arguments, so the engine and its oracle
// both use these restatements of the classic fdlibm algorithms (Cody-Waite reduction by pi/2 in
// three parts, the minimax kernels __kernel_sin / __kernel_cos, the rational acos of e_acos.c, and
// the bit-seeded Newton cbrt of s_cbrt.c).  Accuracy < 1 ulp over the arguments MLPnP produces;
// tests/test_cpu_math.py checks them against glibc.  Only +, -, *, / and IEEE sqrt are used — and,
// in the two pow restatements, fma (correctly rounded on both sides: v_fma_f64, glibc fma) — so
// with -ffp-contract=off the host and gfx950 builds return identical bits.
//
// Arguments beyond |x| = 2^19 * pi/2 are reduced with the same three-part scheme (fdlibm switches to
// Payne-Hanek there); they only occur for diverged Gauss-Newton states and are deterministic.
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RSCM_HD __host__ __device__ __forceinline__
#else
#define RSCM_HD inline
#endif

namespace rsc {
namespace dm {

RSCM_HD uint32_t hi_word(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (uint32_t)(b >> 32);
}
RSCM_HD uint32_t lo_word(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (uint32_t)b;
}
RSCM_HD double from_words(uint32_t hi, uint32_t lo) {
    const uint64_t b = ((uint64_t)hi << 32) | lo;
    double x;
    std::memcpy(&x, &b, 8);
    return x;
}

// __kernel_sin(x, y, iy) on [-pi/4, pi/4]; y is the tail of x.
RSCM_HD double k_sin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix < 0x3e400000u && (int)x == 0) return x;  // |x| < 2^-27
    const double z = x * x;
    const double v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

// __kernel_cos(x, y) on [-pi/4, pi/4].
RSCM_HD double k_cos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix < 0x3e400000u && (int)x == 0) return 1.0;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3fd33333u) return 1.0 - (0.5 * z - (z * r - x * y));  // |x| < 0.3
    const double qx = (ix > 0x3fe90000u) ? 0.28125 : from_words(ix - 0x00200000u, 0u);  // x/4
    const double hz = 0.5 * z - qx;
    const double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

// High words of n*pi/2, n = 1..32 (cancellation check of the medium-size reduction).
RSCM_HD uint32_t npio2_hw(int n) {
    const uint32_t t[32] = {
        0x3ff921fbu, 0x400921fbu, 0x4012d97cu, 0x401921fbu, 0x401f6a7au, 0x4022d97cu, 0x4025fdbbu, 0x402921fbu,
        0x402c463au, 0x402f6a7au, 0x4031475cu, 0x4032d97cu, 0x40346b9cu, 0x4035fdbbu, 0x40378fdbu, 0x403921fbu,
        0x403ab41bu, 0x403c463au, 0x403dd85au, 0x403f6a7au, 0x40407e4cu, 0x4041475cu, 0x4042106cu, 0x4042d97cu,
        0x4043a28cu, 0x40446b9cu, 0x404534acu, 0x4045fdbbu, 0x4046c6cbu, 0x40478fdbu, 0x404858ebu, 0x404921fbu};
    return t[n - 1];
}

// __ieee754_rem_pio2: x = n*pi/2 + (y0 + y1), |y0 + y1| <= pi/4.
RSCM_HD int rem_pio2(double x, double& y0, double& y1) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    const uint32_t hx = hi_word(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const bool neg = (hx >> 31) != 0;
    if (ix <= 0x3fe921fbu) {
        y0 = x;
        y1 = 0.0;
        return 0;
    }
    if (ix < 0x4002d97cu) {  // |x| < 3pi/4: n = +-1
        if (!neg) {
            double z = x - pio2_1;
            if (ix != 0x3ff921fbu) {
                y0 = z - pio2_1t;
                y1 = (z - y0) - pio2_1t;
            } else {
                z -= pio2_2;
                y0 = z - pio2_2t;
                y1 = (z - y0) - pio2_2t;
            }
            return 1;
        }
        double z = x + pio2_1;
        if (ix != 0x3ff921fbu) {
            y0 = z + pio2_1t;
            y1 = (z - y0) + pio2_1t;
        } else {
            z += pio2_2;
            y0 = z + pio2_2t;
            y1 = (z - y0) + pio2_2t;
        }
        return -1;
    }
    const double t0 = std::fabs(x);
    const int n = (int)(t0 * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t0 - fn * pio2_1;
    double w = fn * pio2_1t;
    if (n < 32 && ix != npio2_hw(n)) {
        y0 = r - w;
    } else {
        const int j = (int)(ix >> 20);
        y0 = r - w;
        int i = j - (int)((hi_word(y0) >> 20) & 0x7ffu);
        if (i > 16) {
            double t = r;
            w = fn * pio2_2;
            r = t - w;
            w = fn * pio2_2t - ((t - r) - w);
            y0 = r - w;
            i = j - (int)((hi_word(y0) >> 20) & 0x7ffu);
            if (i > 49) {
                t = r;
                w = fn * pio2_3;
                r = t - w;
                w = fn * pio2_3t - ((t - r) - w);
                y0 = r - w;
            }
        }
    }
    y1 = (r - y0) - w;
    if (neg) {
        y0 = -y0;
        y1 = -y1;
        return -n;
    }
    return n;
}

RSCM_HD double sin(double x) {
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return k_sin(x, 0.0, 0);
    if (ix >= 0x7ff00000u) return x - x;
    double y0, y1;
    const int n = rem_pio2(x, y0, y1);
    switch (n & 3) {
        case 0: return k_sin(y0, y1, 1);
        case 1: return k_cos(y0, y1);
        case 2: return -k_sin(y0, y1, 1);
        default: return -k_cos(y0, y1);
    }
}

RSCM_HD double cos(double x) {
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return k_cos(x, 0.0);
    if (ix >= 0x7ff00000u) return x - x;
    double y0, y1;
    const int n = rem_pio2(x, y0, y1);
    switch (n & 3) {
        case 0: return k_cos(y0, y1);
        case 1: return -k_sin(y0, y1, 1);
        case 2: return -k_cos(y0, y1);
        default: return k_sin(y0, y1, 1);
    }
}

// __ieee754_acos.
RSCM_HD double acos(double x) {
    const double pi = 3.14159265358979311600e+00, pio2_hi = 1.57079632679489655800e+00,
                 pio2_lo = 6.12323399573676603587e-17;
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05;
    const double qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const uint32_t hx = hi_word(x);
    const uint32_t ix = hx & 0x7fffffffu;
    auto P = [&](double z) { return z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5))))); };
    auto Q = [&](double z) { return 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4))); };
    if (ix >= 0x3ff00000u) {  // |x| >= 1
        if (((ix - 0x3ff00000u) | lo_word(x)) == 0) return ((hx >> 31) == 0) ? 0.0 : pi + 2.0 * pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000u) {  // |x| < 0.5
        if (ix <= 0x3c600000u) return pio2_hi + pio2_lo;
        const double z = x * x;
        const double r = P(z) / Q(z);
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if ((hx >> 31) != 0) {  // x < -0.5
        const double z = (1.0 + x) * 0.5;
        const double s = std::sqrt(z);
        const double r = P(z) / Q(z);
        const double w = r * s - pio2_lo;
        return pi - 2.0 * (s + w);
    }
    const double z = (1.0 - x) * 0.5;  // x > 0.5
    const double s = std::sqrt(z);
    const double df = from_words(hi_word(s), 0u);
    const double c = (z - df * df) / (s + df);
    const double r = P(z) / Q(z);
    const double w = r * s + c;
    return 2.0 * (df + w);
}

// s_cbrt (fdlibm 5.3): bit-seeded rational step, chop, one Newton step.
RSCM_HD double cbrt(double x) {
    const uint32_t B1 = 715094163u, B2 = 696219795u;
    const double C = 5.42857142857142815906e-01, D = -7.05306122448979611050e-01, E = 1.41428571428571436819e+00,
                 F = 1.60714285714285720630e+00, G = 3.57142857142857150787e-01;
    uint32_t hx = hi_word(x);
    const uint32_t sign = hx & 0x80000000u;
    hx ^= sign;
    if (hx >= 0x7ff00000u) return x + x;
    if ((hx | lo_word(x)) == 0) return x;
    x = from_words(hx, lo_word(x));  // |x|
    double t;
    if (hx < 0x00100000u) {  // subnormal
        t = from_words(0x43500000u, 0u) * x;
        t = from_words(hi_word(t) / 3 + B2, 0u);
    } else {
        t = from_words(hx / 3 + B1, 0u);
    }
    double r = t * t / x;
    double s = C + r * t;
    t *= G + F / (s + E + D / s);
    t = from_words(hi_word(t) + 1u, 0u);
    s = t * t;
    r = x / s;
    const double w = t + t;
    r = (r - t) / (w + r);
    t = t + t * r;
    return from_words(hi_word(t) | sign, lo_word(t));
}

// e_log (fdlibm 5.3): argument reduction to [sqrt(2)/2, sqrt(2)], s = f/(2+f), minimax R(z).
// Used by ORBmatcher::SearchBySim3 through MapPoint::PredictScale (MapPoint.cpp:367-381, log of a
// float ratio; logf(x) is restated as the float rounding of this double log).
RSCM_HD double log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    int32_t hx = (int32_t)hi_word(x);
    const uint32_t lx = lo_word(x);
    int32_t k = 0;
    if (hx < 0x00100000) {                                  // x < 2^-1022
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -two54 / 0.0;  // log(+-0) = -inf
        if (hx < 0) return (x - x) / 0.0;                   // log(-x) = NaN
        k -= 54;
        x *= two54;
        hx = (int32_t)hi_word(x);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    x = from_words((uint32_t)(hx | (i0 ^ 0x3ff00000)), lo_word(x));  // normalise x or x/2
    k += (i0 >> 20);
    const double f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            const double dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        const double dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    int32_t i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// logf as the float rounding of the double log above.
RSCM_HD float logf(float x) { return (float)log((double)x); }

// pow(x, 3.0/2.0) of mlpnpJacs' 1.0/pow(t8,3.0/2.0) and 1.0/pow(t63,3.0/2.0)
// (MLPnPsolver.cpp:839,:901; glibc pow in the reference), correctly rounded up to a 2^-104 relative
// band around the rounding midpoints: s = sqrt(x) rounded, r = x - s^2 and x*s - fl(x*s) exact by
// fma, x^1.5 = x*s + x*r/(2s) to second order.  pow's special cases for x = +-0, +inf, < 0, NaN.
RSCM_HD double pow_3_2(double x) {
    if (!(x > 0.0)) return (x == 0.0) ? 0.0 : (x - x) / (x - x);
    const double s = sqrt(x);
    const double p = x * s;
    if (p > 1.7976931348623157e308) return p;  // overflow (and x = +inf)
    const double r = fma(-s, s, x);
    const double e = fma(x, s, -p);
    return p + (e + x * (r / (s + s)));
}

// pow(x, 1.0/3.0) of computePose's scale (MLPnPsolver.cpp:567; glibc pow in the reference, not cbrt:
// the exponent is the double nearest 1/3, 1/3 - 2^-54/3).  x^y = cbrt(x) * x^-(2^-54/3), i.e. the
// cube root in double-double — one Newton step on fdlibm's cbrt with the residual x - c^3 formed
// exactly by fma — times 1 - (2^-54/3) ln x (the dropped square term is below 2^-100).  Correctly
// rounded up to a 2^-100 band around the midpoints; x >= 0 here (the argument is an abs()).
RSCM_HD double pow_1_3(double x) {
    if (!(x > 0.0)) return (x == 0.0) ? 0.0 : (x - x) / (x - x);
    if (x > 1.7976931348623157e308) return x;
    const double c = cbrt(x);
    const double c2 = c * c, c2l = fma(c, c, -c2);           // c^2 = c2 + c2l exactly
    const double c3 = c2 * c, c3l = fma(c2, c, -c3);         // c2 * c = c3 + c3l exactly
    const double res = ((x - c3) - c3l) - c2l * c;           // x - c^3 (x - c3 exact: Sterbenz)
    const double corr = res / (3.0 * c2);                    // cbrt(x) = c + corr + O(corr^2)
    const double delta = 1.8503717077085941e-17;             // 1/3 - fl(1/3) = 2^-54 / 3
    return c + (corr - c * (delta * log(x)));
}

}  // namespace dm
}  // namespace rsc
