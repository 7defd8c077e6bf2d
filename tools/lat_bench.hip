// lat_bench.hip — diagnostic: dependent-chain latency (cycles per op, one wave per SIMD) of the
// FP64 operations on the EPnP eigen-solver's critical path (fma, IEEE division, sqrt, make_givens),
// and the same ops with 4 independent chains per lane.  Not part of the product.
// Build: make -C tools lat_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../orb-slam2-optimized_amd/csrc/rsc_core.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int OP, int CH>
__global__ __launch_bounds__(64) void chain(double* out, long long* cyc, int iters, double seed) {
    double x[CH];
    for (int c = 0; c < CH; ++c) x[c] = seed + threadIdx.x * 1e-3 + c;
    const double a = 1.0000001, b = 0.999999;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        RSC_UNROLL for (int c = 0; c < CH; ++c) {
            if (OP == 0) x[c] = x[c] * a + b;               // mul+add (no contraction)
            if (OP == 1) x[c] = a / x[c] + b;                // IEEE division
            if (OP == 2) x[c] = sqrt(x[c]) + b;              // IEEE sqrt
            if (OP == 3) { double cc, ss; rsc::make_givens(x[c], b, cc, ss); x[c] = cc + ss + a; }
            if (OP == 4) x[c] = __builtin_fma(x[c], a, b);   // one FMA
            if (OP == 8) { RSC_UNROLL for (int u = 0; u < 8; ++u) x[c] = x[c] + b; }   // 8 dependent adds
            if (OP == 9) { float f = (float)x[c]; RSC_UNROLL for (int u = 0; u < 8; ++u) f = f + 0.5f; x[c] = f; }
            if (OP == 5) { float f = (float)x[c]; f = f * 1.0000001f + 0.5f; x[c] = f; }
        }
    }
    const long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP, int CH>
int run(const char* name, int nwg) {
    const int iters = 2000;
    double* out; long long* cyc;
    CK(hipMalloc(&out, nwg * 64 * 8));
    CK(hipMalloc(&cyc, nwg * 8));
    chain<OP, CH><<<nwg, 64>>>(out, cyc, iters, 1.5);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    chain<OP, CH><<<nwg, 64>>>(out, cyc, iters, 1.5);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    long long c0;
    CK(hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost));
    printf("%-28s wgs=%5d  %7.1f clk/op-iter (per chain step)  wall %8.1f us  -> %6.1f ns/step\n", name, nwg,
           (double)c0 / iters, ms * 1e3, ms * 1e6 / iters);
    CK(hipFree(out)); CK(hipFree(cyc));
    return 0;
}

int main() {
    for (int nwg : {1024, 2048}) {
        run<0, 1>("mul+add f64 chain", nwg);
        run<0, 4>("mul+add f64 x4 chains", nwg);
        run<4, 1>("fma f64 chain", nwg);
        run<1, 1>("div f64 chain (+add)", nwg);
        run<1, 4>("div f64 x4 chains", nwg);
        run<2, 1>("sqrt f64 chain (+add)", nwg);
        run<3, 1>("make_givens chain", nwg);
        run<3, 4>("make_givens x4", nwg);
        run<5, 1>("f32 mul+add chain (+cvt)", nwg);
        run<8, 1>("8 dependent f64 adds", nwg);
        run<8, 2>("8 dep f64 adds x2 chains", nwg);
        run<9, 1>("8 dependent f32 adds (+cvt)", nwg);
    }
    return 0;
}
