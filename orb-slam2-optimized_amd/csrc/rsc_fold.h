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

// acc += c[0..M) in index order, straight-line: groups of 16 terms, the 8 loads of group k+1 issued
// before the additions of group k.  A compile-time recursion (not an unrolled loop over an array of
// groups, which the compiler keeps rolled and indexes through scratch) gives each group its own
// registers; sched_barrier pins the load-then-add order, so the waits count only the older group and
// no register copies sit between the additions.
constexpr int kFoldG = 8;  // double2 loads per group (16 terms)

template <int K, int NG>
__device__ __forceinline__ void fold_step(double& acc, const double2* c2, const double2 (&cur)[kFoldG]) {
    double2 nx[kFoldG];
    if constexpr (K + 1 < NG) {
        RSC_UNROLL for (int q = 0; q < kFoldG; ++q) nx[q] = c2[kFoldG * (K + 1) + q];
    }
    __builtin_amdgcn_sched_barrier(0);
    RSC_UNROLL for (int q = 0; q < kFoldG; ++q) {
        acc = acc + cur[q].x;
        acc = acc + cur[q].y;
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (K + 1 < NG) fold_step<K + 1, NG>(acc, c2, nx);
}

template <int M>
__device__ __forceinline__ double fold_fixed(double acc, const double* c) {
    static_assert(M % (2 * kFoldG) == 0, "whole groups");
    const double2* c2 = reinterpret_cast<const double2*>(c);
    double2 v[kFoldG];
    RSC_UNROLL for (int q = 0; q < kFoldG; ++q) v[q] = c2[q];
    fold_step<0, M / (2 * kFoldG)>(acc, c2, v);
    return acc;
}

}  // namespace rsc
