// Does a wave64 VALU instruction cost less when one 32-lane half of EXEC is
// empty? Throughput of independent FMA chains (8 accumulators, 4 waves per
// SIMD) under four lane masks: all 64, lanes 0-31, every other lane (32), 0-15.
// Prints one JSON line per (type, mask): cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#pragma clang diagnostic ignored "-Wunused-result"

// One VALU instruction each (inline asm: no SLP packing, no promotion).
__device__ __forceinline__ float fma_op(float a, float b, float c) {
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ double fma_op(double a, double b, double c) {
    double r;
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <typename T>
__global__ __launch_bounds__(1024) void fma_chain(T* out, unsigned long long* cyc, int mode, int iters) {
    const uint32_t lane = threadIdx.x & 63u;
    bool on = true;
    if (mode == 1) on = lane < 32u;
    if (mode == 2) on = (lane & 1u) == 0u;
    if (mode == 3) on = lane < 16u;
    T a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (T)(threadIdx.x + k);
    const T m = (T)1.0000001, c = (T)1e-7;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (on) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = fma_op(a[k], m, c);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    T s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64u == 0u) atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

template <typename T>
static void run(const char* name) {
    const int blocks = 256, threads = 1024, iters = 4096;
    T* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(T) * blocks * threads);
    hipMalloc(&cyc, sizeof(unsigned long long));
    const char* masks[4] = {"all64", "lanes0-31", "even32", "lanes0-15"};
    for (int mode = 0; mode < 4; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(cyc, 0, sizeof(unsigned long long));
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(fma_chain<T>, dim3(blocks), dim3(threads), 0, 0, out, cyc, mode, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        const double waves = (double)blocks * threads / 64.0;
        const double instr = 8.0 * iters;  // wave-instructions per wave
        // 4 waves share a SIMD: SIMD-cycles per wave-instruction = wave cycles / (instr * 4)
        const double per = (double)c / waves / instr / 4.0;
        printf("{\"type\": \"%s\", \"mask\": \"%s\", \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.3f}\n", name,
               masks[mode], best, per);
    }
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<float>("v_fma_f32");
    run<double>("v_fma_f64");
    return 0;
}
