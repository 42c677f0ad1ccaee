// Correctly rounded FP64 sqrt and reciprocal for the kernel's hot paths
// (tray_kernel.hip), bit-identical to the compiler's full lowering; checked over
// random and edge-case operands by tools/sqrt_rcp_check.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tray {

// Correctly rounded sqrt and reciprocal without their range handling.
// LLVM lowers an f64 sqrt on gfx950 to: scale x < 2^-767 up by 2^256, v_rsq_f64
// and five Newton/Goldschmidt steps (10 FP64 instructions), scale back, and
// return x itself for +-0 / +inf (v_cmp_class). For x in [2^-767, 2^1024) the
// scalings are by 2^0 and the class fix-up does not fire, so the steps alone
// give the same bits: `sqrt_core` is those steps. Likewise 1.0 / b is
// v_div_scale x2, v_rcp_f64, two Newton steps, q = 1 * r, one residual step,
// v_div_fmas and v_div_fixup; for |b| in [2^-767, 2^1022) neither div_scale
// scales (the quotient and 1/b are normal, the exponent gap is < 768) and
// div_fmas / div_fixup reduce to an fma / the identity: `rcp_core`.
// `sqrt_cr` / `rcp_cr` check the range per lane (two integer instructions on
// the exponent word) and redo the rare out-of-range lanes with the full
// lowering, so every result equals __builtin_sqrt(x) / (1.0 / b).
__device__ __forceinline__ double sqrt_core(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r;
    double h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, e, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
__device__ __forceinline__ uint32_t hi_word(double x) { return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
// x in [2^-767, 2^1024): biased exponent 256..2046, sign clear.
__device__ __forceinline__ bool sqrt_core_ok(double x) { return hi_word(x) - 0x10000000u < 0x6FF00000u; }
// Zeros also take the full lowering (it returns x for +-0): they are rare on
// every path that calls this (a tangent ray's discriminant, a Philox word of
// 0, normal incidence), so the common path carries no zero test and select.
__device__ __forceinline__ double sqrt_cr(double x) {
    double g = sqrt_core(x);
    if (__builtin_expect(!sqrt_core_ok(x), 0)) g = __builtin_sqrt(x);
    return g;
}
__device__ __forceinline__ double rcp_core(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double rem = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(rem, r, r);
}
// |b| in [2^-767, 2^1022): biased exponent 256..2044.
__device__ __forceinline__ double rcp_cr(double b) {
    double r = rcp_core(b);
    if (__builtin_expect(!((hi_word(b) & 0x7FF00000u) - 0x10000000u < 0x6FD00000u), 0)) r = 1.0 / b;
    return r;
}

}  // namespace tray
