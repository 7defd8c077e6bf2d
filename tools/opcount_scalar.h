// opcount_scalar.h — the counting FP64 scalar of the op-counter builds (tools/opcount*.cpp): +, -,
// *, / are one flop each (divisions also counted apart), sqrt one flop (also counted apart),
// transcendental calls one flop each; comparisons, fabs and conversions are not flops.
// Measurement tooling only; the product never links this.
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <type_traits>

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

