// rcp_exhaustive.hip — diagnostic: is v_rcp_f32 + one FMA Newton step the IEEE float reciprocal?
// Tests every float bit pattern (2^32) against the compiler's correctly rounded 1.0f / z and
// reports mismatches per exponent field of z, for the scan kernels' invZc = 1 / p3Dc.z()
// (PnPsolver.cpp:251).  Build: make -C tools rcp_exhaustive; run: ./build/rcp_exhaustive
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float rcp_nr1(float z) {
    const float r = __builtin_amdgcn_rcpf(z);
    const float e = __builtin_fmaf(-z, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp_nr2(float z) {
    float r = __builtin_amdgcn_rcpf(z);
    float e = __builtin_fmaf(-z, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    e = __builtin_fmaf(-z, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

// bad[v][exp] += mismatches of variant v (0 raw rcp, 1 one Newton step, 2 two) for z's exponent
// field exp (0..255), both signs.
__global__ void rcp_check(unsigned long long base, unsigned* bad, unsigned* first) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned bits = (unsigned)i;
    const float z = __uint_as_float(bits);
    const float ref = 1.0f / z;
    const unsigned rb = __float_as_uint(ref);
    const unsigned ex = (bits >> 23) & 0xff;
    const float v[3] = {__builtin_amdgcn_rcpf(z), rcp_nr1(z), rcp_nr2(z)};
    for (int k = 0; k < 3; ++k) {
        const unsigned vb = __float_as_uint(v[k]);
        const bool same = vb == rb || (ref != ref && v[k] != v[k]);
        if (!same) {
            atomicAdd(&bad[k * 256 + ex], 1u);
            atomicMin(&first[k * 256 + ex], bits & 0x7fffffffu);
        }
    }
}

int main() {
    unsigned *bad, *first;
    CK(hipMalloc(&bad, 3 * 256 * 4));
    CK(hipMalloc(&first, 3 * 256 * 4));
    CK(hipMemset(bad, 0, 3 * 256 * 4));
    CK(hipMemset(first, 0xff, 3 * 256 * 4));
    const unsigned long long total = 1ull << 32, chunk = 1ull << 28;
    for (unsigned long long b = 0; b < total; b += chunk) rcp_check<<<(unsigned)(chunk / 256), 256>>>(b, bad, first);
    CK(hipDeviceSynchronize());
    unsigned hb[3 * 256], hf[3 * 256];
    CK(hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost));
    const char* names[3] = {"rcp", "rcp+1 Newton", "rcp+2 Newton"};
    for (int k = 0; k < 3; ++k) {
        unsigned long long tot = 0;
        int lo = 256, hi = -1;
        for (int e = 0; e < 256; ++e) {
            tot += hb[k * 256 + e];
            if (hb[k * 256 + e]) { lo = e < lo ? e : lo; hi = e; }
        }
        printf("%-14s mismatches %llu", names[k], tot);
        if (tot) printf("  (exponent fields %d..%d)", lo, hi);
        printf("\n");
        // exponent fields with mismatches, listed with their count and the smallest |z| pattern
        for (int e = 0; e < 256; ++e)
            if (hb[k * 256 + e] && (k > 0 || e < 3 || e > 252))
                printf("    exp %3d: %10u  first |z| bits 0x%08x (%g)\n", e, hb[k * 256 + e], hf[k * 256 + e],
                       (double)__builtin_bit_cast(float, hf[k * 256 + e]));
    }
    // the range the scans rely on: every normal z whose reciprocal is normal (exponent fields 1..252)
    unsigned long long mid = 0;
    for (int e = 1; e <= 252; ++e) mid += hb[1 * 256 + e];
    printf("rcp+1 Newton mismatches for exponent fields 1..252: %llu\n", mid);
    return 0;
}
