// Throughput of the expensive per-segment operations on gfx950 (diagnostic):
// Philox4x32-10 blocks, correctly rounded FP64 division and sqrt.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/op_bench tools/op_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../tray_amd/csrc/rng.hpp"

constexpr int kIters = 1024;

__global__ void philox_k(double* out, uint64_t seed) {
    double acc = 0;
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
        tray::U2 u = tray::philox_uniforms(seed, c, (uint32_t)i, 7u, 3u << 24);
        acc += u.u0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void div_k(double* out, double b) {
    double a = threadIdx.x + 1.5, acc = 0;
    for (int i = 0; i < kIters; ++i) {
        acc += a / b;
        a += 1.0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void sqrt_k(double* out) {
    double a = threadIdx.x + 1.5, acc = 0;
    for (int i = 0; i < kIters; ++i) {
        acc += __builtin_sqrt(a);
        a += 1.0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const int blocks = 256 * 16, threads = 256;
    double* out;
    (void)hipMalloc(&out, sizeof(double) * blocks * threads);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[3] = {"philox4x32_10 block", "f64 div (correctly rounded)", "f64 sqrt (correctly rounded)"};
    for (int k = 0; k < 3; ++k) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(philox_k, blocks, threads, 0, 0, out, 0x1234ull);
            if (k == 1) hipLaunchKernelGGL(div_k, blocks, threads, 0, 0, out, 3.7);
            if (k == 2) hipLaunchKernelGGL(sqrt_k, blocks, threads, 0, 0, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double ops = (double)blocks * threads * kIters;
        printf("{\"op\": \"%s\", \"G_per_s\": %.1f, \"ns_per_wave_op_per_SIMD\": %.3f}\n", names[k], ops / best / 1e6,
               best * 1e6 / (ops / 64.0 / 1024.0));
    }
    return 0;
}
