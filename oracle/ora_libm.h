// TEST INFRASTRUCTURE — the transcendental functions the oracle's restatements call.
//
// Default build: the fdlibm restatement in csrc/rsc_math.h, i.e. the SAME functions the kernels
// compile (the product is held bit-exact to this build).  With -DRSC_ORACLE_GLIBC_LIBM (the second
// library oracle/build/librsc_oracle_glibc.so): the host glibc calls the reference actually links —
// sin/cos/acos (MLPnPsolver.cpp:636-653, g2o SE3Quat/Sim3 exp maps), std::pow(x, 1.0/3.0)
// (MLPnPsolver.cpp:567) and logf through log(float) (MapPoint.cpp:375).  tests/test_cpu_libm_choice.py
// compares the two builds' results to measure how often the restatement's libm choice changes an
// outcome (VERDICT r2 "What's weak" 1).
#pragma once
#include <cmath>
#include "../orb-slam2-optimized_amd/csrc/rsc_math.h"

namespace ora_libm {
#ifdef RSC_ORACLE_GLIBC_LIBM
inline double sin(double x) { return std::sin(x); }
inline double cos(double x) { return std::cos(x); }
inline double acos(double x) { return std::acos(x); }
inline double cbrt_pow(double x) { return std::pow(x, 1.0 / 3.0); }  // the reference's pow(x, 1/3)
inline float logf(float x) { return std::log(x); }                    // std::log(float) = glibc logf
#else
inline double sin(double x) { return rsc::dm::sin(x); }
inline double cos(double x) { return rsc::dm::cos(x); }
inline double acos(double x) { return rsc::dm::acos(x); }
inline double cbrt_pow(double x) { return rsc::dm::cbrt(x); }  // pow(x, 1/3) restated as cbrt
inline float logf(float x) { return rsc::dm::logf(x); }
#endif
}  // namespace ora_libm
