// Issue cost of the 32x32 -> 64-bit products Philox4x32 needs, three ways, at
// full occupancy (diagnostic): (a) v_mad_u64_u32 (the compiler's form of
// (uint64_t)M * c), (b) v_mul_hi_u32 + v_mul_lo_u32, (c) four 16x16 v_mul_u32_u24
// partial products with carries. All three must agree (checked). Prints JSON:
// cycles per wave-round on one SIMD = time x clock x SIMDs / wave-rounds.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mul_bench tools/mul_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kRounds = 2048;
constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;

template <int kMode>
__device__ __forceinline__ void mul(uint32_t M, uint32_t a, uint32_t& hi, uint32_t& lo) {
    if constexpr (kMode == 0) {
        const uint64_t p = (uint64_t)M * a;
        hi = (uint32_t)(p >> 32);
        lo = (uint32_t)p;
    } else if constexpr (kMode == 1) {
        hi = __umulhi(M, a);
        lo = M * a;
    } else {
        const uint32_t a0 = a & 0xFFFFu, a1 = a >> 16, m0 = M & 0xFFFFu, m1 = M >> 16;
        const uint32_t p00 = __umul24(a0, m0), p01 = __umul24(a0, m1);
        const uint32_t p10 = __umul24(a1, m0), p11 = __umul24(a1, m1);
        const uint32_t mid = p01 + p10;
        const uint32_t cm = mid < p01 ? 0x10000u : 0u;
        lo = p00 + (mid << 16);
        const uint32_t cl = lo < p00 ? 1u : 0u;
        hi = p11 + (mid >> 16) + cm + cl;
    }
}

template <int kMode>
__global__ __launch_bounds__(256) void philox_rounds(uint32_t* out, uint32_t seed) {
    uint32_t c0 = blockIdx.x * blockDim.x + threadIdx.x, c1 = seed, c2 = c0 ^ 0x1234u, c3 = 7u;
    uint32_t k0 = seed, k1 = seed ^ 0xBEEFu;
    for (int r = 0; r < kRounds; ++r) {
        uint32_t h0, l0, h1, l1;
        mul<kMode>(M0, c0, h0, l0);
        mul<kMode>(M1, c2, h1, l1);
        const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
        c0 = n0, c1 = l1, c2 = n2, c3 = l0;
        k0 += 0x9E3779B9u, k1 += 0xBB67AE85u;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3;
}

__global__ __launch_bounds__(256) void fma64(double* out) {
    double a = threadIdx.x * 1e-3, b = 1.0000001, c = 0.5, d = 0.25;
    for (int r = 0; r < kRounds; ++r) {
        a = __builtin_fma(a, b, c);
        d = __builtin_fma(d, b, c);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + d;
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int blocks = prop.multiProcessorCount * 8, threads = 256;  // 8 waves per SIMD
    const size_t n = (size_t)blocks * threads;
    uint32_t *o0, *o1, *o2;
    double* od;
    (void)hipMalloc(&o0, n * 4);
    (void)hipMalloc(&o1, n * 4);
    (void)hipMalloc(&o2, n * 4);
    (void)hipMalloc(&od, n * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double clock_hz = 2.4e9, simds = prop.multiProcessorCount * 4.0, waves = n / 64.0;
    const char* names[4] = {"v_mad_u64_u32", "v_mul_hi_u32 + v_mul_lo_u32", "4 x v_mul_u32_u24 + carries",
                            "2 x v_fma_f64 (reference)"};
    for (int k = 0; k < 4; ++k) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(philox_rounds<0>, blocks, threads, 0, 0, o0, 99u);
            if (k == 1) hipLaunchKernelGGL(philox_rounds<1>, blocks, threads, 0, 0, o1, 99u);
            if (k == 2) hipLaunchKernelGGL(philox_rounds<2>, blocks, threads, 0, 0, o2, 99u);
            if (k == 3) hipLaunchKernelGGL(fma64, blocks, threads, 0, 0, od);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double cyc = best * 1e-3 * clock_hz * simds / (waves * kRounds);
        printf("{\"form\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_round_per_simd\": %.2f}\n", names[k], best, cyc);
    }
    uint32_t* h = new uint32_t[3 * n];
    (void)hipMemcpy(h, o0, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h + n, o1, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h + 2 * n, o2, n * 4, hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (size_t i = 0; i < n; ++i) diff += (h[i] != h[n + i]) + (h[i] != h[2 * n + i]);
    printf("{\"mismatches\": %zu}\n", diff);
    return 0;
}
