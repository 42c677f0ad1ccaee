// Empirical check of the division-by-known-reciprocal identity used by the
// kernel (tray_amd/csrc/tray_kernel.hip div_rcp): with y = RN(1/b),
//     q = RN(a*y); r = fma(-b, q, a) (exact); q' = RN(fma(r, y, q))
// must equal the correctly rounded quotient RN(a/b) (Markstein 1990;
// Muller et al., Handbook of Floating-Point Arithmetic, 2nd ed., §4.7) away from
// overflow/underflow. Compares against the device's correctly rounded division
// on random and adversarial operands; prints a JSON summary.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/div_check tools/div_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ double rand_double(uint64_t bits, int emin, int erange, int mode) {
    uint64_t mant = bits & 0xFFFFFFFFFFFFFull;
    if (mode == 1) mant = 0xFFFFFFFFFFFFFull - (bits & 0xFFull);  // significands near 1.111...1
    if (mode == 2) mant = bits & 0xFFull;                        // near 1.000...0
    const int e = emin + (int)((bits >> 52) % (uint64_t)erange);
    const uint64_t sign = (bits >> 63) << 63;
    const uint64_t u = sign | ((uint64_t)(e + 1023) << 52) | mant;
    return __longlong_as_double((long long)u);
}

__global__ void check(unsigned long long* bad, unsigned long long* total, uint64_t seed, int mode, int per_thread) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long nb = 0;
    for (int i = 0; i < per_thread; ++i) {
        const uint64_t r0 = mix(seed ^ (tid * 0x100000001ull + (uint64_t)i * 2));
        const uint64_t r1 = mix(r0 ^ 0xA5A5A5A5A5A5A5A5ull);
        const double a = rand_double(r0, -60, 120, mode == 3 ? 1 : 0);
        const double b = rand_double(r1, -60, 120, mode == 3 ? 0 : mode);
        const double y = 1.0 / b;
        const double q = a * y;
        const double r = __builtin_fma(-b, q, a);
        const double q1 = __builtin_fma(r, y, q);
        const double ref = a / b;
        if (__double_as_longlong(q1) != __double_as_longlong(ref)) ++nb;
    }
    atomicAdd(bad, nb);
    atomicAdd(total, (unsigned long long)per_thread);
}

int main() {
    unsigned long long *bad, *total;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&total, 8);
    const char* names[4] = {"random significands", "divisor significand near 1.1...1",
                            "divisor significand near 1.0...0", "dividend near 1.1...1"};
    for (int mode = 0; mode < 4; ++mode) {
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(total, 0, 8);
        for (int rep = 0; rep < 4; ++rep)
            hipLaunchKernelGGL(check, 4096, 256, 0, 0, bad, total, 0x1234567ull * (rep + 1) + mode, mode, 256);
        unsigned long long hb = 0, ht = 0;
        (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&ht, total, 8, hipMemcpyDeviceToHost);
        printf("{\"case\": \"%s\", \"pairs\": %llu, \"mismatches\": %llu}\n", names[mode], ht, hb);
    }
    return 0;
}
