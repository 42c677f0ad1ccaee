// Counter RNG of the tray C-ABI (include/tray.h, "Counter RNG contract").
//
// Replaces fortio.org/rand v1.1.0 (go.mod:9), whose per-row-chunk sequential
// stream (ray/tracer.go:121) cannot be reproduced here. Philox4x32-10 keyed on
// (seed) with counter (pixel, sample, bounce, purpose<<24 | attempt) makes every
// draw a pure function of where it happens, so a pixel's colour does not depend
// on launch geometry, row tiling or device count.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tray {

enum : uint32_t { kPurposeAA = 1, kPurposeLens = 2, kPurposeScatter = 3, kPurposeScene = 4 };
constexpr uint32_t kMaxAttempts = 32;

struct U2 {
    double u0, u1;
};

// One Philox4x32-10 block -> two 53-bit uniforms in [0,1).
__host__ __device__ __forceinline__ U2 philox_uniforms(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                                       uint32_t c3) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
    }
    const uint64_t a = ((uint64_t)c1 << 32) | c0;
    const uint64_t b = ((uint64_t)c3 << 32) | c2;
    U2 u;
    u.u0 = (double)(a >> 11) * 0x1.0p-53;
    u.u1 = (double)(b >> 11) * 0x1.0p-53;
    return u;
}

}  // namespace tray
