// FP64 VALU throughput microbenchmark for gfx950 (roofline calibration for
// bench.py's "valu_fp64" bound). Measures v_add_f64 + v_mul_f64 (the only FP64
// ops the parity-constrained kernel may use: no contraction) and v_fma_f64.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/fp64_peak tools/fp64_peak.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kAcc = 8;
constexpr int kIters = 4096;

template <bool kFma>
__global__ __launch_bounds__(256) void peak(double* out, double m, double c) {
    double a[kAcc];
#pragma unroll
    for (int i = 0; i < kAcc; ++i) a[i] = threadIdx.x * 1e-3 + i;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < kAcc; ++i) {
            if constexpr (kFma) a[i] = __builtin_fma(a[i], m, c);
            else a[i] = a[i] * m + c;  // 2 ops (mul, add) with -ffp-contract=off
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < kAcc; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 16, threads = 256;
    double* out;
    (void)hipMalloc(&out, sizeof(double) * blocks * threads);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int fma = 0; fma < 2; ++fma) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            if (fma) hipLaunchKernelGGL(peak<true>, blocks, threads, 0, 0, out, 0.999999, 1e-7);
            else hipLaunchKernelGGL(peak<false>, blocks, threads, 0, 0, out, 0.999999, 1e-7);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double insts = (double)blocks * threads * kIters * kAcc * (fma ? 1 : 2);
        const double flops = (double)blocks * threads * kIters * kAcc * 2;
        printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"T_inst_per_s\": %.2f, \"TFLOPs\": %.2f}\n",
               fma ? "v_fma_f64" : "v_mul_f64+v_add_f64", best, insts / best / 1e9, flops / best / 1e9);
    }
    return 0;
}
