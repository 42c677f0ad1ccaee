// Exhaustive check of tray_amd/csrc/rng.hpp: sincos_2pi_word(w) must give the
// bits of sincos_2pi(w * 2^-32) for every 32-bit word w (the kernel's samplers
// use the word form). Prints JSON.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/sincos_check tools/sincos_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../tray_amd/csrc/rng.hpp"

__global__ void check(unsigned long long* bad, uint64_t base) {
    const uint64_t w = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    double s0, c0, s1, c1;
    tray::sincos_2pi((double)(uint32_t)w * 0x1.0p-32, s0, c0);
    tray::sincos_2pi_word((uint32_t)w, s1, c1);
    const bool diff = __builtin_bit_cast(uint64_t, s0) != __builtin_bit_cast(uint64_t, s1) ||
                      __builtin_bit_cast(uint64_t, c0) != __builtin_bit_cast(uint64_t, c1);
    if (diff) atomicAdd(bad, 1ull);
}

int main() {
    unsigned long long* bad;
    (void)hipMalloc(&bad, 8);
    (void)hipMemset(bad, 0, 8);
    const uint64_t per = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += per)
        hipLaunchKernelGGL(check, (uint32_t)(per / 256), 256, 0, 0, bad, base);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    printf("{\"check\": \"sincos_2pi_word == sincos_2pi(w 2^-32)\", \"words\": %llu, \"mismatches\": %llu}\n",
           1ull << 32, h);
    return h != 0;
}
