// sim3match.hip — ORBmatcher::SearchBySim3 kernels (src/ORBmatcher.cpp:948-1170); see rsc_sim3match.h.
#include <hip/hip_runtime.h>
#include <climits>
#include "rsc_math.h"
#include "rsc_sim3match.h"

namespace rsc {

namespace {

__device__ __forceinline__ int desc_dist(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Eigen Matrix3f * Vector3f + Vector3f, rows summed left to right
__device__ __forceinline__ void rot_add(const float* R, const float (&x)[3], const float* t, float (&o)[3]) {
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = R[3 * r] * x[0] + R[3 * r + 1] * x[1] + R[3 * r + 2] * x[2] + t[r];
}

// One MapPoint of `src` projected into `dst` (:992-1070 / :1072-1150); intrinsics are pKF1's.
__device__ int match_point(const DevSim3KF& src, const DevSim3KF& dst, const DevSim3KF& k1, const float* Rsd,
                           const float* tsd, int i, float th) {
    float pw[3] = {src.mp_pos[3 * i], src.mp_pos[3 * i + 1], src.mp_pos[3 * i + 2]};
    float pc[3], pd[3];
    rot_add(src.R, pw, src.t, pc);
    rot_add(Rsd, pc, tsd, pd);
    if (pd[2] < 0.0f) return -1;
    const float invz = (float)(1.0 / (double)pd[2]);  // `const float invz = 1.0/p3Dc2.z()` (:1011)
    const float x = pd[0] * invz;
    const float y = pd[1] * invz;
    const float u = k1.fx * x + k1.cx;
    const float v = k1.fy * y + k1.cy;
    if (!(u >= dst.min_x && u < dst.max_x && v >= dst.min_y && v < dst.max_y)) return -1;  // IsInImage
    const float maxDistance = 1.2f * src.mp_dmax[i];
    const float minDistance = 0.8f * src.mp_dmin[i];
    const float dist3D = sqrtf((pd[0] * pd[0] + pd[1] * pd[1]) + pd[2] * pd[2]);
    if (dist3D < minDistance || dist3D > maxDistance) return -1;
    // MapPoint::PredictScale (MapPoint.cpp:367-381)
    const float ratio = src.mp_dmax[i] / dist3D;
    int level = (int)ceilf(dm::logf(ratio) / dst.log_sf);
    if (level < 0) level = 0;
    else if (level >= dst.n_levels) level = dst.n_levels - 1;
    const float r = th * dst.scale[level];
    // KeyFrame::GetFeaturesInArea (KeyFrame.cpp:560-599), candidates visited in its order
    const int nMinCellX = max(0, (int)floorf((u - dst.min_x - r) * dst.gw_inv));
    if (nMinCellX >= kSim3GridCols) return -1;
    const int nMaxCellX = min(kSim3GridCols - 1, (int)ceilf((u - dst.min_x + r) * dst.gw_inv));
    if (nMaxCellX < 0) return -1;
    const int nMinCellY = max(0, (int)floorf((v - dst.min_y - r) * dst.gh_inv));
    if (nMinCellY >= kSim3GridRows) return -1;
    const int nMaxCellY = min(kSim3GridRows - 1, (int)ceilf((v - dst.min_y + r) * dst.gh_inv));
    if (nMaxCellY < 0) return -1;
    const uint4 d0 = src.mp_desc[2 * i], d1 = src.mp_desc[2 * i + 1];
    int bestDist = INT_MAX, bestIdx = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
        for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
            const int c = ix * kSim3GridRows + iy;
            const int e1 = dst.cell_begin[c + 1];
            for (int e = dst.cell_begin[c]; e < e1; ++e) {
                const int j = dst.cell_feat[e];
                const float2 kp = dst.kp[j];
                if (!(fabsf(kp.x - u) < r && fabsf(kp.y - v) < r)) continue;
                const int oct = dst.octave[j];
                if (oct < level - 1 || oct > level) continue;
                const int dist = desc_dist(d0, d1, dst.desc[2 * j], dst.desc[2 * j + 1]);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdx = j;
                }
            }
        }
    return bestDist <= kSim3ThHigh ? bestIdx : -1;
}

// grid (points / 256, 2 directions, pairs)
__global__ __launch_bounds__(256) void sim3_search_kernel(const Sim3MatchPair* __restrict__ pairs, float th) {
    const Sim3MatchPair& P = pairs[blockIdx.z];
    const DevSim3KF& k1 = *P.k1;
    const DevSim3KF& k2 = *P.k2;
    const bool fwd = blockIdx.y == 0;
    const DevSim3KF& src = fwd ? k1 : k2;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= src.n) return;
    const uint8_t done = fwd ? P.already1[i] : P.already2[i];
    int m = -1;
    // !pMP || vbAlreadyMatched || isBad (:998-1002, :1078-1082)
    if (src.mp_state[i] == 1 && !done) {
        if (fwd) {
            float R21[9], t21[3];  // R21 = R12^T, t21 = -R21 * t12 (:963-964)
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) R21[3 * r + c] = P.R12[3 * c + r];
#pragma unroll
            for (int r = 0; r < 3; ++r)
                t21[r] = -(R21[3 * r] * P.t12[0] + R21[3 * r + 1] * P.t12[1] + R21[3 * r + 2] * P.t12[2]);
            m = match_point(k1, k2, k1, R21, t21, i, th);
        } else {
            m = match_point(k2, k1, k1, P.R12, P.t12, i, th);
        }
    }
    (fwd ? P.m1 : P.m2)[i] = m;
}

// check agreement (:1152-1167), one workgroup per pair
__global__ __launch_bounds__(256) void sim3_agree_kernel(const Sim3MatchPair* __restrict__ pairs) {
    __shared__ int total;
    const Sim3MatchPair& P = pairs[blockIdx.x];
    const int n1 = P.k1->n;
    if (threadIdx.x == 0) total = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < n1; i += 256) {
        const int idx2 = P.m1[i];
        const bool ok = idx2 >= 0 && P.m2[idx2] == i;
        P.out[i] = ok ? idx2 : -1;
        cnt += ok;
    }
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&total, cnt);
    __syncthreads();
    if (threadIdx.x == 0) *P.nfound = total;
}

}  // namespace

hipError_t launch_search_by_sim3(int count, int max_points, const Sim3MatchPair* pairs, float th, hipStream_t st) {
    const dim3 g1((max_points + 255) / 256 > 0 ? (max_points + 255) / 256 : 1, 2, count);
    sim3_search_kernel<<<g1, 256, 0, st>>>(pairs, th);
    sim3_agree_kernel<<<count, 256, 0, st>>>(pairs);
    return hipGetLastError();
}

}  // namespace rsc
