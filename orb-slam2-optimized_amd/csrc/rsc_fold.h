// rsc_fold.h — ordered folds for the g2o-restating kernels (poseopt.hip, sim3opt.hip): a g2o sum
// over the active edges is a sequential left-to-right loop in the reference, so it is folded in edge
// order on one lane (the per-edge terms having been computed in parallel into LDS).
#pragma once
#include <hip/hip_runtime.h>
#include "rsc_core.h"

namespace rsc {

// Sequential fold acc (+|-)= c[0..m) in index order (c 16-byte aligned).  The loads of the next 32
// terms are in flight while the current 32 are added.
template <bool SUB>
__device__ __forceinline__ double fold_run(double acc, const double* __restrict__ c, int m) {
    constexpr int G = 16;  // double2 per group
    const int g = m / (2 * G);
    const double2* c2 = reinterpret_cast<const double2*>(c);
    double2 nx[G];
    if (g > 0) RSC_UNROLL for (int q = 0; q < G; ++q) nx[q] = c2[q];
    for (int i = 0; i < g; ++i) {
        double2 cu[G];
        RSC_UNROLL for (int q = 0; q < G; ++q) cu[q] = nx[q];
        if (i + 1 < g) RSC_UNROLL for (int q = 0; q < G; ++q) nx[q] = c2[G * (i + 1) + q];
        RSC_UNROLL for (int q = 0; q < G; ++q) {
            acc = SUB ? acc - cu[q].x : acc + cu[q].x;
            acc = SUB ? acc - cu[q].y : acc + cu[q].y;
        }
    }
    for (int r = g * 2 * G; r < m; ++r) acc = SUB ? acc - c[r] : acc + c[r];
    return acc;
}

}  // namespace rsc
