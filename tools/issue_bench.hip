// issue_bench.hip — diagnostic: VALU issue cost per wave64 instruction on gfx950 for the FP64 /
// FP32 operations the solve kernels are made of, with 1, 2 and 4 waves per SIMD (independent
// chains, so latency is hidden and issue sets the time).  Prints cycles per instruction per SIMD
// from the wall time and the measured shader clock (s_memtime / wall).
// Build: make -C tools issue_bench; run: tools/bin/issue_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(64) void issue_k(double* out, float* outf, double a, double b, long long* clk) {
    const int lane = threadIdx.x;
    double x[8];
    float f[8];
    for (int k = 0; k < 8; ++k) { x[k] = 1.0 + lane * 1e-3 + k; f[k] = 1.0f + lane * 1e-3f + k; }
    const long long t0 = clock64();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (OP == 0) x[k] = __builtin_fma(x[k], a, b);        // v_fma_f64
            if (OP == 1) x[k] = x[k] * a;                         // v_mul_f64
            if (OP == 2) x[k] = x[k] + b;                         // v_add_f64
            if (OP == 3) f[k] = __builtin_fmaf(f[k], (float)a, (float)b);  // v_fma_f32
            if (OP == 4) x[k] = (double)(float)x[k];              // cvt f64->f32->f64
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const long long t1 = clock64();
    double s = 0;
    float sf = 0;
    for (int k = 0; k < 8; ++k) { s += x[k]; sf += f[k]; }
    out[blockIdx.x * 64 + lane] = s;
    outf[blockIdx.x * 64 + lane] = sf;
    if (lane == 0) clk[blockIdx.x] = t1 - t0;
}

int main() {
    const char* names[5] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_fma_f32", "cvt f64<->f32 (2 instr)"};
    double* out;
    float* outf;
    long long* clk;
    const int maxw = 4096;
    CK(hipMalloc(&out, maxw * 64 * 8));
    CK(hipMalloc(&outf, maxw * 64 * 4));
    CK(hipMalloc(&clk, maxw * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int op = 0; op < 5; ++op) {
        for (int wps = 1; wps <= 4; wps *= 2) {
            const int nwg = 1024 * wps;
            auto launch = [&] {
                switch (op) {
                    case 0: issue_k<0><<<nwg, 64>>>(out, outf, 0.999, 1e-3, clk); break;
                    case 1: issue_k<1><<<nwg, 64>>>(out, outf, 0.999, 1e-3, clk); break;
                    case 2: issue_k<2><<<nwg, 64>>>(out, outf, 0.999, 1e-3, clk); break;
                    case 3: issue_k<3><<<nwg, 64>>>(out, outf, 0.999, 1e-3, clk); break;
                    default: issue_k<4><<<nwg, 64>>>(out, outf, 0.999, 1e-3, clk); break;
                }
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            long long hc[4096];
            CK(hipMemcpy(hc, clk, nwg * 8, hipMemcpyDeviceToHost));
            double avg = 0;
            for (int i = 0; i < nwg; ++i) avg += (double)hc[i];
            avg /= nwg;
            const double instr = (double)kIters * 8 * (op == 4 ? 2 : 1);
            // per wave: clock64 cycles per instruction (the wave's own view; with wps waves on a SIMD
            // the SIMD's cost per instruction is that / wps)
            printf("%-26s waves/SIMD %d  wall %8.1f us  wave clk/instr %6.2f  SIMD clk/instr %6.2f\n", names[op], wps,
                   ms * 1e3, avg / instr, avg / instr / wps);
            fflush(stdout);
        }
    }
    return 0;
}
