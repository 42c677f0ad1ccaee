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

enum : uint32_t { kPurposeCamera = 1, kPurposeScatter = 3, kPurposeScene = 4 };

struct U2 {
    double u0, u1;
};
struct U4 {
    double u0, u1, u2, u3;
};

struct Block {
    uint32_t x0, x1, x2, x3;
};

// Philox4x32-10 (Salmon et al. 2011, Random123 constants). TRAY_PHILOX_ROUNDS
// exists only for cost experiments (tools/build_variants.sh); the contract is 10.
#ifndef TRAY_PHILOX_ROUNDS
#define TRAY_PHILOX_ROUNDS 10
#endif
__host__ __device__ __forceinline__ Block philox4x32_10(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                                        uint32_t c3) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < TRAY_PHILOX_ROUNDS; ++r) {
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
    return Block{c0, c1, c2, c3};
}

// One block -> two 53-bit uniforms in [0,1) (host scene generation).
__host__ __device__ __forceinline__ U2 philox_uniforms(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                                       uint32_t c3) {
    const Block b = philox4x32_10(seed, c0, c1, c2, c3);
    const uint64_t a = ((uint64_t)b.x1 << 32) | b.x0;
    const uint64_t c = ((uint64_t)b.x3 << 32) | b.x2;
    U2 u;
    u.u0 = (double)(a >> 11) * 0x1.0p-53;
    u.u1 = (double)(c >> 11) * 0x1.0p-53;
    return u;
}

// One block -> four 32-bit uniforms u = x * 2^-32 in [0,1) (renderer draws).
__host__ __device__ __forceinline__ U4 philox_u4(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    const Block b = philox4x32_10(seed, c0, c1, c2, c3);
    return U4{(double)b.x0 * 0x1.0p-32, (double)b.x1 * 0x1.0p-32, (double)b.x2 * 0x1.0p-32,
              (double)b.x3 * 0x1.0p-32};
}

// sin and cos of 2*pi*u, u in [0,1), with + and * only in a fixed order (the
// "sincos2pi" of include/tray.h): quadrant and reflection into [0, pi/4], then
// Taylor polynomials of degree 15 (sin) and 16 (cos) in Horner form. Built
// with -ffp-contract=off this gives the same bits on the host and the device.
__host__ __device__ __forceinline__ void sincos_2pi(double u, double& s, double& c) {
    const double v = u * 4.0;
    const double q = __builtin_floor(v);
    const double f = v - q;
    const int quad = (int)q;
    const bool swap = f > 0.5;
    const double x = swap ? 1.0 - f : f;
    const double t = x * 0x1.921fb54442d18p+0;  // pi/2
    const double t2 = t * t;
    double sp = -0x1.ae7f3e733b81fp-41;
    sp = sp * t2 + 0x1.6124613a86d09p-33;
    sp = sp * t2 + -0x1.ae64567f544e4p-26;
    sp = sp * t2 + 0x1.71de3a556c734p-19;
    sp = sp * t2 + -0x1.a01a01a01a01ap-13;
    sp = sp * t2 + 0x1.1111111111111p-7;
    sp = sp * t2 + -0x1.5555555555555p-3;
    sp = sp * t2 + 1.0;
    double sn = t * sp;
    double cp = 0x1.ae7f3e733b81fp-45;
    cp = cp * t2 + -0x1.93974a8c07c9dp-37;
    cp = cp * t2 + 0x1.1eed8eff8d898p-29;
    cp = cp * t2 + -0x1.27e4fb7789f5cp-22;
    cp = cp * t2 + 0x1.a01a01a01a01ap-16;
    cp = cp * t2 + -0x1.6c16c16c16c17p-10;
    cp = cp * t2 + 0x1.5555555555555p-5;
    cp = cp * t2 + -0.5;
    double cs = cp * t2 + 1.0;
    if (swap) {
        const double tmp = sn;
        sn = cs;
        cs = tmp;
    }
    const int qq = quad & 3;
    s = qq == 0 ? sn : qq == 1 ? cs : qq == 2 ? -sn : -cs;
    c = qq == 0 ? cs : qq == 1 ? -sn : qq == 2 ? -cs : sn;
}

}  // namespace tray
