// Counter RNG of the tray C-ABI (include/tray.h, "Counter RNG contract").
//
// Replaces fortio.org/rand v1.1.0 (go.mod:9), whose per-row-chunk sequential
// stream (ray/tracer.go:121) cannot be reproduced here. Every renderer draw is a
// pure function of where it happens - (seed; pixel, sample, bounce, purpose) -
// so a pixel's colour does not depend on launch geometry, row tiling or device
// count. ABI 6: the draws come from draw_block (a keyed pcg4d hash, below), the
// key and the host's scene generation from Philox4x32-10.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tray {

enum : uint32_t { kPurposeCamera = 1, kPurposeScatter = 3, kPurposeScene = 4, kPurposeKey = 5 };

struct U2 {
    double u0, u1;
};
struct U4 {
    double u0, u1, u2, u3;
};

struct Block {
    uint32_t x0, x1, x2, x3;
};

// Philox4x32-10 (Salmon et al. 2011, Random123 constants): the draw key and the
// host's scene stream. TRAY_PHILOX_ROUNDS exists only for cost experiments
// (tools/build_variants.sh); the contract is 10.
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

// The renderer's draw key (include/tray.h, ABI 6): one Philox4x32-10 block of the
// seed, ctr = (0, 0, 0, kPurposeKey << 24), computed once per render on the host.
struct DrawKey {
    uint32_t k0, k1, k2, k3;
};
__host__ __device__ inline DrawKey draw_key(uint64_t seed) {
    const Block b = philox4x32_10(seed, 0u, 0u, 0u, kPurposeKey << 24);
    return DrawKey{b.x0, b.x1, b.x2, b.x3};
}

// The renderer's draw block (include/tray.h, ABI 6): pcg4d (Jarzynski & Olano,
// "Hash Functions for GPU Rendering", JCGT 9(3), 2020) of the keyed counter
// (pixel ^ k0, sample ^ k1, bounce ^ k2, purpose ^ k3), then an xorshift-16 of
// each word. The xorshift mixes the low output bits (a product's low bits depend
// only on its factors' low bits; without it flipping counter bit 17 never flips
// output bit 0), and the Philox key spreads nearby seeds. Twelve 32-bit products
// where Philox4x32-10 needs twenty 32x32 -> 64-bit ones and 40 XORs: a Philox
// block was ~7.6 % of the C2 frame (rounds 10 / 7 / 4: 78.06 / 76.33 / 74.44 ms
// per 16-frame launch, profiles/r10_ab_rng_c2.jsonl). Strict avalanche over the
// counter bits the renderer varies, bit bias and word correlations are at noise
// level (tests/test_rng_quality_cpu.py).
__host__ __device__ __forceinline__ Block draw_block(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t pixel,
                                                     uint32_t sample, uint32_t bounce, uint32_t purpose) {
    uint32_t v0 = (pixel ^ k0) * 1664525u + 1013904223u, v1 = (sample ^ k1) * 1664525u + 1013904223u;
    uint32_t v2 = (bounce ^ k2) * 1664525u + 1013904223u, v3 = (purpose ^ k3) * 1664525u + 1013904223u;
    v0 += v1 * v3;
    v1 += v2 * v0;
    v2 += v0 * v1;
    v3 += v1 * v2;
    v0 ^= v0 >> 16;
    v1 ^= v1 >> 16;
    v2 ^= v2 >> 16;
    v3 ^= v3 >> 16;
    v0 += v1 * v3;
    v1 += v2 * v0;
    v2 += v0 * v1;
    v3 += v1 * v2;
    return Block{v0 ^ (v0 >> 16), v1 ^ (v1 >> 16), v2 ^ (v2 >> 16), v3 ^ (v3 >> 16)};
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

// sin and cos of 2*pi*u, u in [0,1) (the "sincos2pi" of include/tray.h). The
// quadrant and the reflection into [0, 1/2] are exact in FP64; the polynomial
// runs in FP32: t = RN32(x) * RN32(pi/2), then Taylor polynomials of degree 9
// (sin) and 10 (cos) in t^2 by Horner's rule with correctly rounded fmaf. Both
// are accurate to ~1e-7, far finer than anything a sampled direction feeds
// (the uniforms themselves are 32-bit), and IEEE FP32 + fmaf give the same bits
// on the host oracle and the device. This is the contract's sampler transform,
// not reference arithmetic (which stays FP64, uncontracted): the FP64 form cost
// ~40 FP64 instructions and its registers, 3.5 % of the C2 frame.
__host__ __device__ __forceinline__ void sincos_2pi(double u, double& s, double& c) {
    const double v = u * 4.0;
    const double q = __builtin_floor(v);
    const double f = v - q;
    const int quad = (int)q;
    const bool swap = f > 0.5;
    const float x = (float)(swap ? 1.0 - f : f);
    const float t = x * 0x1.921fb6p+0f;  // RN32(pi/2)
    const float t2 = t * t;
    float sp = __builtin_fmaf(t2, 0x1.71de3ap-19f, -0x1.a01a02p-13f);  // 1/9!, -1/7!
    sp = __builtin_fmaf(sp, t2, 0x1.111112p-7f);                        // 1/5!
    sp = __builtin_fmaf(sp, t2, -0x1.555556p-3f);                       // -1/3!
    sp = __builtin_fmaf(sp, t2, 1.0f);
    float sn = t * sp;
    float cp = __builtin_fmaf(t2, -0x1.27e4fcp-22f, 0x1.a01a02p-16f);  // -1/10!, 1/8!
    cp = __builtin_fmaf(cp, t2, -0x1.6c16c2p-10f);                      // -1/6!
    cp = __builtin_fmaf(cp, t2, 0x1.555556p-5f);                        // 1/4!
    cp = __builtin_fmaf(cp, t2, -0.5f);
    float cs = __builtin_fmaf(cp, t2, 1.0f);
    if (swap) {
        const float tmp = sn;
        sn = cs;
        cs = tmp;
    }
    // One FP64 Newton step onto the unit circle, k = 1.5 - 0.5 (s^2 + c^2):
    // |(s, c)| = 1 within ~1e-14 (ray/vec3_test.go:505-537 pins unit vectors
    // to 1e-9; the FP32 pair alone is only within ~1e-7).
    const double sd = sn, cd = cs;
    const double k = 1.5 - 0.5 * (sd * sd + cd * cd);
    const double sk = sd * k, ck = cd * k;
    const int qq = quad & 3;
    s = qq == 0 ? sk : qq == 1 ? ck : qq == 2 ? -sk : -ck;
    c = qq == 0 ? ck : qq == 1 ? -sk : qq == 2 ? -ck : sk;
}

// sincos_2pi(w * 2^-32) from the uniform's 32-bit word, with the FP64 front
// end (4u, floor, reflection, conversion to float) done in integers: 4u =
// w 2^-30, so the quadrant is w >> 30 and f = F 2^-30 with F = w mod 2^30;
// the reflection 1 - f = (2^30 - F) 2^-30 is exact, and (float) of G 2^-30 is
// RN32(G) 2^-30 (an exact power-of-two scaling). Every step is exact or the
// same single rounding as sincos_2pi's, so the bits are identical for every w
// (tools/sincos_check.hip compares all 2^32 words on the device).
__host__ __device__ __forceinline__ void sincos_2pi_word(uint32_t w, double& s, double& c) {
    const uint32_t F = w & 0x3FFFFFFFu;
    const bool swap = F > 0x20000000u;
    const float x = (float)(swap ? 0x40000000u - F : F) * 0x1p-30f;
    const float t = x * 0x1.921fb6p+0f;  // RN32(pi/2)
    const float t2 = t * t;
    float sp = __builtin_fmaf(t2, 0x1.71de3ap-19f, -0x1.a01a02p-13f);
    sp = __builtin_fmaf(sp, t2, 0x1.111112p-7f);
    sp = __builtin_fmaf(sp, t2, -0x1.555556p-3f);
    sp = __builtin_fmaf(sp, t2, 1.0f);
    float sn = t * sp;
    float cp = __builtin_fmaf(t2, -0x1.27e4fcp-22f, 0x1.a01a02p-16f);
    cp = __builtin_fmaf(cp, t2, -0x1.6c16c2p-10f);
    cp = __builtin_fmaf(cp, t2, 0x1.555556p-5f);
    cp = __builtin_fmaf(cp, t2, -0.5f);
    float cs = __builtin_fmaf(cp, t2, 1.0f);
    if (swap) {
        const float tmp = sn;
        sn = cs;
        cs = tmp;
    }
    const double sd = sn, cd = cs;
    const double k = 1.5 - 0.5 * (sd * sd + cd * cd);
    const double sk = sd * k, ck = cd * k;
    // Quadrant rotation (sincos_2pi's qq == 0: (sk, ck), 1: (ck, -sk), 2: (-sk, -ck),
    // 3: (-ck, sk)) as one swap on bit 0 and sign flips on the high words: s is
    // negated in quadrants 2 and 3, c in 1 and 2. Negation is exact, so the bits
    // are those of the selects it replaces.
    const uint32_t qq = w >> 30;
    const bool swap_sc = (qq & 1u) != 0u;
    const double s0 = swap_sc ? ck : sk, c0 = swap_sc ? sk : ck;
    const uint64_t sflip = (uint64_t)(qq >> 1) << 63, cflip = (uint64_t)((qq ^ (qq >> 1)) & 1u) << 63;
    s = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, s0) ^ sflip);
    c = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, c0) ^ cflip);
}

}  // namespace tray
