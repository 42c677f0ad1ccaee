// Checks tray_amd/csrc/fp64.hpp: sqrt_cr(x) must have the bits of the
// compiler's correctly rounded __builtin_sqrt(x), and rcp_cr(b) those of 1.0 / b,
// for every input: random significands over the whole exponent range (subnormals
// included), both signs, significands next to 1.0 and 2.0, zeros, infinities,
// NaN and the range boundaries 2^-767, 2^1022, 2^1024 +- a few ulps. Prints JSON.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/sqrt_rcp_check tools/sqrt_rcp_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../tray_amd/csrc/fp64.hpp"

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// mode 0: any bit pattern; 1: significand near 1.1...1; 2: near 1.0...0;
// 3: exponent within 3 of a range boundary; 4: edge values by index.
__device__ double operand(uint64_t bits, int mode, uint64_t index) {
    if (mode == 4) {
        const double edges[] = {0.0, -0.0, __builtin_inf(), -__builtin_inf(), __builtin_nan(""), 0x1p-767, 0x1p-768,
                                0x1p1022, 0x1p1023, 0x1.fffffffffffffp1023, 0x1p-1022, 0x1p-1074, 1.0, 2.0, 0.5};
        const double e = edges[index % 15];
        const int64_t step = (int64_t)((index / 15) % 9) - 4;  // +-4 ulps around each edge
        if (e == 0.0 || e != e || __builtin_isinf(e)) return e;
        return __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, e) + (uint64_t)step);
    }
    uint64_t mant = bits & 0xFFFFFFFFFFFFFull;
    if (mode == 1) mant = 0xFFFFFFFFFFFFFull - (bits & 0xFFull);
    if (mode == 2) mant = bits & 0xFFull;
    uint64_t ex = (bits >> 52) & 0x7FF;
    if (mode == 3) {
        const uint64_t b[] = {256, 255, 2044, 2045, 2046, 1, 0};
        ex = b[(bits >> 52) % 7] + ((bits >> 40) & 1);
    }
    return __builtin_bit_cast(double, (bits & 0x8000000000000000ull) | (ex << 52) | mant);
}

__global__ void check(unsigned long long* bad, uint64_t seed, int mode, int per_thread) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long ns = 0, nr = 0;
    for (int i = 0; i < per_thread; ++i) {
        const uint64_t idx = tid * (uint64_t)per_thread + (uint64_t)i;
        const double x = operand(mix(seed ^ (idx * 0x100000001ull)), mode, idx);
        const double s0 = __builtin_sqrt(x), s1 = tray::sqrt_cr(x);
        const double r0 = 1.0 / x, r1 = tray::rcp_cr(x);
        ns += __builtin_bit_cast(uint64_t, s0) != __builtin_bit_cast(uint64_t, s1) && !(s0 != s0 && s1 != s1);
        nr += __builtin_bit_cast(uint64_t, r0) != __builtin_bit_cast(uint64_t, r1) && !(r0 != r0 && r1 != r1);
    }
    atomicAdd(bad, ns);
    atomicAdd(bad + 1, nr);
}

int main() {
    unsigned long long* bad;
    (void)hipMalloc(&bad, 16);
    const char* names[5] = {"any bit pattern", "significand near 1.1...1", "significand near 1.0...0",
                            "exponent at a range boundary", "edge values +-4 ulps"};
    for (int mode = 0; mode < 5; ++mode) {
        (void)hipMemset(bad, 0, 16);
        const int per = mode == 4 ? 1 : 256, blocks = mode == 4 ? 1 : 4096;
        const int reps = mode == 4 ? 1 : 4;
        for (int rep = 0; rep < reps; ++rep)
            hipLaunchKernelGGL(check, blocks, mode == 4 ? 135 : 256, 0, 0, bad, 0x9876543ull * (rep + 1) + mode, mode,
                               per);
        unsigned long long h[2] = {0, 0};
        (void)hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
        const unsigned long long n = (unsigned long long)reps * blocks * (mode == 4 ? 135 : 256) * per;
        printf("{\"case\": \"%s\", \"operands\": %llu, \"sqrt_mismatches\": %llu, \"rcp_mismatches\": %llu}\n",
               names[mode], n, h[0], h[1]);
    }
    return 0;
}
