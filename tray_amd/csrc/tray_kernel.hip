// tray_kernel.hip — the per-pixel path-tracing megakernel for gfx950.
//
// Replaces the body of Tracer.RenderLines (ray/tracer.go:120-155) and
// everything beneath it: Camera.GetRay (ray/camera.go:113-142),
// Scene.RayColor (ray/objects.go:49-62), Scene.Hit / Sphere.Hit
// (ray/objects.go:37-46, 81-104), Lambertian/Metal/Dielectric.Scatter
// (ray/materials.go:13-71), the sky (ray/objects.go:68-73) and the
// RandomUnitVector/InDisc samplers (ray/rand.go:30-32, via include/tray.h's
// counter RNG).
//
// Execution model (one launch per row set):
//   * one lane = one pixel; the lane runs all r samples of its pixel in order,
//     so the per-pixel sum has the reference's summation order
//     (ray/tracer.go:143) and needs no atomics;
//   * the recursion of RayColor becomes an iterative bounce loop with PATH
//     REGENERATION: when a lane's path ends it immediately starts its next
//     sample, so a wave iterates max-over-lanes(total segments) times instead of
//     sum-over-samples(max segments). The wave leaves the loop when a __ballot
//     of unfinished lanes is empty;
//   * the sphere geometry (cx, cy, cz, R*R: 32 B/sphere) is staged once per
//     workgroup into LDS and read by wave-uniform broadcast ds_read_b128;
//     materials are fetched from global memory only for the closest hit;
//   * a workgroup is 4 waves covering a 16x16 pixel tile (8x8 per wave), so a
//     wave's primary rays are coherent.
// Arithmetic: FP64, reference op order, compiled with -ffp-contract=off.
// The one intentional difference from the Go recursion: attenuations are
// multiplied outer-first (((att0*att1)*att2)*sky instead of
// att0*(att1*(att2*sky))), which changes colours by <= a few ulps and never a
// path decision.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "bvh.hpp"
#include "rng.hpp"
#include "tray_kernel.hpp"

namespace tray {

struct D3 {
    double x, y, z;
};

__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }
// Add(u,v) = {v.x+u.x, ...} (ray/vec3.go:25-27); IEEE addition commutes.
__device__ __forceinline__ D3 add(D3 u, D3 v) { return d3(v.x + u.x, v.y + u.y, v.z + u.z); }
__device__ __forceinline__ D3 sub(D3 u, D3 v) { return d3(u.x - v.x, u.y - v.y, u.z - v.z); }
__device__ __forceinline__ D3 smul(D3 v, double t) { return d3(v.x * t, v.y * t, v.z * t); }
__device__ __forceinline__ D3 mul(D3 u, D3 v) { return d3(u.x * v.x, u.y * v.y, u.z * v.z); }
__device__ __forceinline__ D3 sdiv(D3 v, double t) { return d3(v.x / t, v.y / t, v.z / t); }
__device__ __forceinline__ D3 neg(D3 v) { return d3(-v.x, -v.y, -v.z); }

// a / b, correctly rounded, given y = RN(1/b) (exactly rounded, e.g. a full
// division or a host-side 1.0/b): q = RN(a*y) is within 1 ulp of a/b, the
// residual fma(-b, q, a) is exact, and one correction fma(r, y, q) returns
// RN(a/b) (Markstein 1990; Muller et al., Handbook of Floating-Point Arithmetic
// §4.7). 3 FP64 instructions instead of ~10 for the generic sequence; checked
// on 10^9 pairs by tools/div_check.hip. Zero keeps its sign, and quotients near
// the overflow/underflow range (or non-finite operands) take the full division.
__device__ __forceinline__ double div_rcp(double a, double b, double y) {
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    const double q1 = __builtin_fma(r, y, q);
    const double aq = __builtin_fabs(q);
    if (a == 0) return q;
    if (!(aq > 0x1p-960 && aq < 0x1p+960)) return a / b;
    return q1;
}
__device__ __forceinline__ D3 sdiv_rcp(D3 v, double t, double y) {
    return d3(div_rcp(v.x, t, y), div_rcp(v.y, t, y), div_rcp(v.z, t, y));
}
__device__ __forceinline__ double dot(D3 u, D3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ double length_sq(D3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
// Unit (ray/vec3.go:116-119): each component divided by the length.
__device__ __forceinline__ D3 unit(D3 v) {
    const double l = __builtin_sqrt(length_sq(v));
    return sdiv_rcp(v, l, 1.0 / l);
}
__device__ __forceinline__ bool near_zero(D3 v) {
    const double s = 1e-8;
    return (__builtin_fabs(v.x) < s) && (__builtin_fabs(v.y) < s) && (__builtin_fabs(v.z) < s);
}
// Go math.Min special cases (-Inf first, then NaN, then signed zeros).
__device__ __forceinline__ double go_min(double x, double y) {
    if (__builtin_isinf(x) && x < 0) return x;
    if (__builtin_isinf(y) && y < 0) return y;
    if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
    if (x == 0 && x == y) return __builtin_signbit(x) ? x : y;
    return x < y ? x : y;
}
__device__ __forceinline__ D3 reflect(D3 v, D3 n) { return sub(v, smul(n, 2 * dot(v, n))); }
__device__ __forceinline__ D3 refract(D3 uv, D3 n, double eta) {
    const double cos_theta = go_min(dot(neg(uv), n), 1.0);
    const D3 perp = smul(add(uv, smul(n, cos_theta)), eta);
    const D3 par = smul(n, -__builtin_sqrt(__builtin_fabs(1.0 - length_sq(perp))));
    return add(perp, par);
}
// Reflectance (ray/materials.go:66-71); math.Pow(x,5) == x*((x*x)*(x*x)).
__device__ __forceinline__ double reflectance(double cosine, double ref_idx) {
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 *= r0;
    const double x = 1 - cosine;
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return r0 + (1 - r0) * (x * x4);
}

// InDisc(radius) (ray/tracer.go:138, ray/camera.go:128): polar map of two
// uniforms: r = sqrt(ua), phi = 2 pi ub.
__device__ __forceinline__ void disc(double ua, double ub, double radius, double& ox, double& oy) {
    const double r = __builtin_sqrt(ua);
    double s, c;
    sincos_2pi(ub, s, c);
    ox = (r * c) * radius;
    oy = (r * s) * radius;
}

// Camera and background, copied once per workgroup into LDS and read through a
// volatile pointer where needed: keeps ~50 dwords of loop-invariant kernel
// arguments out of the SGPR file (they otherwise spill to VGPR lanes and cost a
// v_readlane on every use).
struct Uniforms {
    CamRec cam;
    V3 bg_a, bg_b;
    double focus_time, ray_radius;
    uint64_t seed;
};
// Explicit LDS address space: a generic volatile pointer would be accessed with
// (slow, system-coherent) flat loads.
typedef const volatile __attribute__((address_space(3))) Uniforms* UniPtr;

// The RNG key, re-read per draw and made wave-uniform: Philox's round keys are
// then recomputed with scalar adds instead of being hoisted out of the loop
// (where they would be spilled to VGPR lanes and cost a v_readlane each).
__device__ __forceinline__ uint64_t uni_seed(UniPtr uni) {
    const uint64_t s = uni->seed;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)s);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(s >> 32));
    return ((uint64_t)hi << 32) | lo;
}
constexpr size_t kUniformsBytes = (sizeof(Uniforms) + 255) / 256 * 256;

__device__ __forceinline__ D3 ld3(const volatile __attribute__((address_space(3))) double* v) { return d3(v[0], v[1], v[2]); }

// RandomUnitVector (ray/rand.go:30-32): Archimedes' projection of two uniforms of
// the bounce's scatter block, z = 1 - 2 u0, phi = 2 pi u1.
__device__ __forceinline__ D3 unit_vector_from(const U4& u) {
    const double z = 1.0 - 2.0 * u.u0;
    const double r = __builtin_sqrt(1.0 - z * z);
    double s, c;
    sincos_2pi(u.u1, s, c);
    return d3(r * c, r * s, z);
}

// The sample's camera block (purpose 1): (pixel, sample, 0, 1<<24).
__device__ __forceinline__ U4 camera_block(UniPtr uni, uint32_t pixel, uint32_t sample) {
    return philox_u4(uni_seed(uni), pixel, sample, 0u, kPurposeCamera << 24);
}

// Camera.GetRay (ray/camera.go:113-142). The sample's camera block `u` feeds the
// anti-aliasing disc (words 0,1; ray/tracer.go:136-139, only when r > 1) and the
// lens disc (words 2,3, only when the aperture is open).
__device__ __forceinline__ void get_ray(const KernelParams& p, UniPtr uni, const U4& u, double px, double py,
                                        D3& origin, D3& dir) {
    double ox = 0.0, oy = 0.0;
    const double aperture = uni->cam.aperture;
    if (p.spp > 1) disc(u.u0, u.u1, uni->ray_radius, ox, oy);
    const D3 pos = ld3(uni->cam.position);
    const D3 p00 = ld3(uni->cam.pixel00);
    const D3 pxv = ld3(uni->cam.pixel_x);
    const D3 pyv = ld3(uni->cam.pixel_y);
    const D3 sample_pt = add(add(p00, smul(pxv, px + ox)), smul(pyv, py + oy));
    origin = pos;
    dir = sub(sample_pt, pos);
    if (aperture > 0) {
        double dx, dy;
        disc(u.u2, u.u3, 1.0, dx, dy);
        const D3 du = ld3(uni->cam.defocus_u);
        const D3 dv = ld3(uni->cam.defocus_v);
        const D3 offset = add(smul(du, dx), smul(dv, dy));
        const D3 focus_point = add(pos, smul(dir, uni->focus_time));
        origin = add(pos, offset);
        dir = sub(focus_point, origin);
    }
}

// ColorF.ToSRGBA channel (ray/vec3.go:173-180), IEC 61966-2-1, half-up rounding.
__device__ __forceinline__ uint32_t linear_to_srgb(double c) {
    if (!(c > 0.0)) return 0u;
    if (c >= 1.0) return 255u;
    const double s = c <= 0.0031308 ? 12.92 * c : 1.055 * pow(c, 1.0 / 2.4) - 0.055;
    return (uint32_t)__builtin_floor(s * 255.0 + 0.5);
}

// Compact output row j -> image row y (see tray_params in include/tray.h).
__device__ __forceinline__ int32_t row_of(const KernelParams& p, int32_t j) {
    if (p.tile_rows <= 0) return p.y_start + j;
    const int32_t t = j / p.tile_rows;
    const int32_t within = j - t * p.tile_rows;
    return p.y_start + (t * p.tile_count + p.tile_index) * p.tile_rows + within;
}

// Per-lane path state. A lane owns one pixel at a time and walks its samples
// in order; when the last sample ends it writes the pixel and takes another.
struct Lane {
    D3 org, dir, thr, sum;
    uint32_t pixel, sample, bounce, segments;
    int32_t x, j;  // image column, compact output row
    double fx, fy;
    bool busy;
};

template <int kFmt>
__device__ __forceinline__ void write_pixel(const KernelParams& p, const Lane& L) {
    const double inv = 1.0 / (double)p.spp;  // colorSumDiv (ray/tracer.go:123)
    const D3 mean = smul(L.sum, inv);
    const size_t off = (size_t)L.j * (size_t)p.width + (size_t)L.x;
    if constexpr (kFmt == kOutRGBF64) {
        double* o = static_cast<double*>(p.out) + off * 3;
        o[0] = mean.x;
        o[1] = mean.y;
        o[2] = mean.z;
    } else if constexpr (kFmt == kOutRGBF32) {
        float* o = static_cast<float*>(p.out) + off * 3;
        o[0] = (float)mean.x;
        o[1] = (float)mean.y;
        o[2] = (float)mean.z;
    } else {
        const uint32_t rgba = linear_to_srgb(mean.x) | (linear_to_srgb(mean.y) << 8) |
                              (linear_to_srgb(mean.z) << 16) | (255u << 24);
        static_cast<uint32_t*>(p.out)[off] = rgba;
    }
    if (p.segments) p.segments[off] = L.segments;
}

// Candidate root of one sphere whose discriminant is >= 0 (Sphere.Hit,
// ray/objects.go:86-94): the first root inside (1e-6, closest) wins. Used by the
// linear scan, which visits spheres in list order exactly like the reference.
__device__ __forceinline__ void candidate(double h, double disc, double a, double a_inv, int idx, double& closest,
                                          int& best) {
    if (disc >= 0) {
        const double sq = __builtin_sqrt(disc);
        double root = div_rcp(h - sq, a, a_inv);
        bool ok = root > 1e-6 && root < closest;
        if (!ok) {
            root = div_rcp(h + sq, a, a_inv);
            ok = root > 1e-6 && root < closest;
        }
        if (ok) {
            closest = root;
            best = idx;
        }
    }
}

// The same decision for an out-of-order visit. Sphere.Hit's root choice does
// not depend on the interval end: root2 >= root1, so the reference takes
// t = root1 if root1 > 1e-6, else root2, and accepts it iff t < closestSoFar.
// The linear scan therefore returns min over spheres of (t_i, i); accepting
// "t < closest, or t == closest with a lower index" reproduces it for any order.
__device__ __forceinline__ void candidate_any_order(double h, double disc, double a, double a_inv, int idx,
                                                    double& closest, int& best) {
    if (disc >= 0) {
        const double sq = __builtin_sqrt(disc);
        const double r1 = div_rcp(h - sq, a, a_inv);
        const double t = r1 > 1e-6 ? r1 : div_rcp(h + sq, a, a_inv);
        if (t > 1e-6 && (t < closest || (t == closest && idx < best))) {
            closest = t;
            best = idx;
        }
    }
}

// 17 FP64 add/mul per sphere, op order of Sphere.Hit (ray/objects.go:82-86).
__device__ __forceinline__ void quad(const double4 g, const D3& org, const D3& dir, double a, double& h,
                                     double& disc) {
    const double ocx = g.x - org.x;
    const double ocy = g.y - org.y;
    const double ocz = g.z - org.z;
    h = dir.x * ocx + dir.y * ocy + dir.z * ocz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - g.w;
    disc = h * h - a * c;
}

#ifndef TRAY_UNROLL
#define TRAY_UNROLL 8
#endif

// Instrumented launches only: per-lane counters, flushed once when the lane exits.
struct Stats {
    uint64_t segments = 0, spheres = 0, boxes = 0;
};

// Geometry visible to one workgroup (LDS copies, or global memory when the
// scene does not fit).
struct SceneView {
    const double4* geo;     // linear scan: list order, NaN-padded
    const BvhNode* nodes;   // BVH: depth-first nodes
    const double4* bgeo;    // BVH: spheres in leaf-slot order (+4 NaN slots)
    const int32_t* bidx;    // BVH: original list index of each slot
    const MatRec* bmat;     // BVH: shading record of each slot
    int32_t n, n_nodes;
};

// Scene.Hit (ray/objects.go:37-46) as the reference's linear scan over
// NaN-padded geometry (a NaN discriminant is never >= 0). Spheres are tested in
// groups of U that share one wave-level branch into the rare sqrt/div path;
// inside a group they are visited in list order.
template <int U, bool kStats>
__device__ __forceinline__ int scene_hit_linear(const SceneView& sv, const D3& org, const D3& dir, double& closest,
                                                Stats& st) {
    const double a = length_sq(dir);  // hoisted: same bits as per sphere
    const double a_inv = 1.0 / a;
    closest = __builtin_inf();
    int best = -1;
    const int ngroups = (sv.n + U - 1) / U;
    for (int gi = 0; gi < ngroups; ++gi) {
        const int i = gi * U;
        double h[U], d[U];
#pragma unroll
        for (int k = 0; k < U; ++k) quad(sv.geo[i + k], org, dir, a, h[k], d[k]);
        double m = d[0];
#pragma unroll
        for (int k = 1; k < U; ++k) m = __builtin_fmax(m, d[k]);  // maxNum drops NaN padding
        if (m >= 0) {
#pragma unroll
            for (int k = 0; k < U; ++k) candidate(h[k], d[k], a, a_inv, i + k, closest, best);
        }
    }
    if constexpr (kStats) st.spheres += (uint64_t)sv.n;
    return best;
}

// Round a positive (or +inf) double up to a float that is >= it.
__device__ __forceinline__ float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

// Per-lane traversal state of one Scene.Hit through the exact-culling BVH
// (tray_bvh.cpp): stackless depth-first walk with skip links, conservative FP32
// slab tests on padded boxes (culled against the current closest hit), FP64
// sphere tests with the reference's arithmetic and the any-order acceptance rule.
// Lane states of the BVH kernel.
enum : uint32_t { kIdleState = 0, kTravState = 1, kLeafState = 2, kShadeState = 3 };

struct Trav {
    float ix, iy, iz, oix, oiy, oiz;  // FP32 ray: t = box * inv - org * inv
    float tlim;                       // closest rounded up to float
    int32_t node, leaf;
    double a, a_inv, closest;
    int32_t best;  // original list index of the closest hit (tie-break key)
    int32_t slot;  // its leaf slot (LDS-resident geometry + shading record)
};

__device__ __forceinline__ void trav_begin(Trav& T, const D3& org, const D3& dir) {
    T.a = length_sq(dir);  // hoisted: same bits as per sphere
    T.a_inv = 1.0 / T.a;
    T.closest = __builtin_inf();
    T.best = -1;
    T.slot = 0;
    T.tlim = __builtin_inff();
    T.node = 0;
    T.leaf = -1;
    float dxf = (float)dir.x, dyf = (float)dir.y, dzf = (float)dir.z;
    if (__builtin_fabsf(dxf) < 1e-30f) dxf = 1e-30f;
    if (__builtin_fabsf(dyf) < 1e-30f) dyf = 1e-30f;
    if (__builtin_fabsf(dzf) < 1e-30f) dzf = 1e-30f;
    // ~1 ulp reciprocal: inside the padding's error budget (tray_bvh.cpp)
    T.ix = __builtin_amdgcn_rcpf(dxf);
    T.iy = __builtin_amdgcn_rcpf(dyf);
    T.iz = __builtin_amdgcn_rcpf(dzf);
    T.oix = (float)org.x * T.ix;
    T.oiy = (float)org.y * T.iy;
    T.oiz = (float)org.z * T.iz;
}

// One node visit. Returns the new lane state: kTrav, kLeaf (holds T.leaf) or
// kShade (traversal finished).
__device__ __forceinline__ uint32_t trav_node(Trav& T, const SceneView& sv) {
    const uint4* np = reinterpret_cast<const uint4*>(sv.nodes + T.node);
    const uint4 q0 = np[0], q1 = np[1];
    const float lox = __uint_as_float(q0.x), loy = __uint_as_float(q0.y), loz = __uint_as_float(q0.z);
    const float hix = __uint_as_float(q0.w), hiy = __uint_as_float(q1.x), hiz = __uint_as_float(q1.y);
    const int32_t skip = (int32_t)q1.z, leaf = (int32_t)q1.w;
    const float t0x = __builtin_fmaf(lox, T.ix, -T.oix), t1x = __builtin_fmaf(hix, T.ix, -T.oix);
    const float t0y = __builtin_fmaf(loy, T.iy, -T.oiy), t1y = __builtin_fmaf(hiy, T.iy, -T.oiy);
    const float t0z = __builtin_fmaf(loz, T.iz, -T.oiz), t1z = __builtin_fmaf(hiz, T.iz, -T.oiz);
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                     __builtin_fmaxf(__builtin_fminf(t0z, t1z), 0.0f));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                     __builtin_fminf(__builtin_fmaxf(t0z, t1z), T.tlim));
    const bool hit = tn <= tf;
    T.node = (hit && leaf < 0) ? T.node + 1 : skip;
    if (hit && leaf >= 0) {
        T.leaf = leaf;
        return kLeafState;
    }
    return T.node < sv.n_nodes ? kTravState : kShadeState;
}

#ifndef TRAY_LEAF_COMPACT
#define TRAY_LEAF_COMPACT 1
#endif
// Test the held leaf's <= kBvhLeafMax spheres (FP64, any-order rule).
__device__ __forceinline__ uint32_t trav_leaf(Trav& T, const SceneView& sv, const D3& org, const D3& dir) {
    const int slot = T.leaf >> 3, cnt = T.leaf & 7;
    double h[kBvhLeafMax], d[kBvhLeafMax];
#pragma unroll
    for (int k = 0; k < kBvhLeafMax; ++k) {
        quad(sv.bgeo[slot + k], org, dir, T.a, h[k], d[k]);
        if (k >= cnt) d[k] = __builtin_nan("");
    }
#if TRAY_LEAF_COMPACT
    // Only spheres whose discriminant is >= 0 need the root (a sqrt and two
    // divisions): each lane walks its own candidates, so the wave pays for
    // max-over-lanes(candidates) roots instead of kBvhLeafMax.
    uint32_t cand = 0;
#pragma unroll
    for (int k = 0; k < kBvhLeafMax; ++k) cand |= (d[k] >= 0) ? (1u << k) : 0u;
    if (cand != 0u) {
        while (cand != 0u) {
            const int k = __builtin_ctz(cand);
            cand &= cand - 1u;
            double hk = h[0], dk = d[0];
#pragma unroll
            for (int q = 1; q < kBvhLeafMax; ++q) {
                hk = k == q ? h[q] : hk;
                dk = k == q ? d[q] : dk;
            }
            const int32_t idx = sv.bidx[slot + k];
            const int32_t before = T.best;
            candidate_any_order(hk, dk, T.a, T.a_inv, idx, T.closest, T.best);
            if (T.best != before) T.slot = slot + k;
        }
        T.tlim = f32_up(T.closest);
    }
#else
    double m = d[0];
#pragma unroll
    for (int k = 1; k < kBvhLeafMax; ++k) m = __builtin_fmax(m, d[k]);
    if (m >= 0) {
#pragma unroll
        for (int k = 0; k < kBvhLeafMax; ++k) {
            const int32_t idx = sv.bidx[slot + k];
            const int32_t before = T.best;
            candidate_any_order(h[k], d[k], T.a, T.a_inv, idx, T.closest, T.best);
            if (T.best != before) T.slot = slot + k;
        }
        T.tlim = f32_up(T.closest);
    }
#endif
    T.leaf = -1;
    return T.node < sv.n_nodes ? kTravState : kShadeState;
}

// Work item w (64 pixels = one 8x8 tile of the compact row space) -> pixel.
__device__ __forceinline__ bool decode_pixel(const KernelParams& p, uint32_t item, int32_t& x, int32_t& j) {
    const uint32_t tile = item >> 6, r = item & 63u;
    const uint32_t tx = tile % (uint32_t)p.tiles_x, ty = tile / (uint32_t)p.tiles_x;
    x = (int32_t)(tx * 8u + (r & 7u));
    j = (int32_t)(ty * 8u + (r >> 3));
    return x < p.width && j < p.rows;
}

// Claim pixel (x, compact row j) for the lane; its first camera ray is generated
// by the caller (get_ray, directly or in the BVH kernel's batched phase).
__device__ __forceinline__ void start_pixel(const KernelParams& p, Lane& L, int32_t x, int32_t j) {
    const int32_t y = row_of(p, j);
    L.x = x;
    L.j = j;
    L.pixel = (uint32_t)y * (uint32_t)p.width + (uint32_t)x;  // global index: tiling-independent RNG key
    L.fx = (double)x;
    L.fy = (double)y;
    L.sample = 0;
    L.bounce = 0;
    L.segments = 0;
    L.thr = d3(1, 1, 1);
    L.sum = d3(0, 0, 0);
    L.busy = true;
}

// A path ended with `color`: accumulate (Add(colorSum, color), ray/tracer.go:143)
// and either set up the next sample or finish the pixel. Returns false when the
// pixel is done (written) and the lane is free.
template <int kFmt, bool kStats>
__device__ __forceinline__ bool finish_sample(const KernelParams& p, Lane& L, const D3& color, Stats& st) {
    L.sum = add(L.sum, color);
    ++L.sample;
    if (L.sample >= (uint32_t)p.spp) {
        write_pixel<kFmt>(p, L);
        if constexpr (kStats) st.segments += L.segments;
        L.busy = false;
        return false;
    }
    L.thr = d3(1, 1, 1);
    L.bounce = 0;
    return true;
}

// One recursion level of RayColor (ray/objects.go:49-62) after Scene.Hit gave
// (best, closest): the sky on a miss, else the hit record and the material's
// scatter; a path that ends is accumulated and the lane moves on to its next
// sample's camera ray. `geo_at`/`mat_at` give the hit sphere's geometry and
// shading record. Returns true when the lane has a new ray to trace, false when
// its pixel is finished (written) and the lane is free.
//
// Written for a wave of lanes on different branches: the work every branch
// needs is done once, before the branches — one Philox block per lane (the
// bounce's scatter block, or the next sample's camera block when the path ends
// here) and the unit direction (sky, Metal, Dielectric).
template <int kFmt, bool kStats, typename GeoAt, typename MatAt>
__device__ __forceinline__ bool shade_step(const KernelParams& p, UniPtr uni, Lane& L, int best, double closest,
                                           GeoAt geo_at, MatAt mat_at, Stats& st) {
    const bool hit = best >= 0;
    // A hit at the last level ends the path black whatever its material does
    // (RayColor(depth 0) is black), so no scatter is computed for it.
    const bool last = L.bounce + 1u >= (uint32_t)p.max_depth;
    bool ends = !hit || last;
    U4 u = philox_u4(uni_seed(uni), L.pixel, ends ? L.sample + 1u : L.sample, ends ? 0u : L.bounce,
                     (ends ? kPurposeCamera : kPurposeScatter) << 24);
    const D3 ud = unit(L.dir);
    D3 color = d3(0, 0, 0);
    if (!hit) {  // AmbientLight.Hit (ray/objects.go:68-73)
        const double t = 0.5 * (ud.y + 1.0);
        const D3 bg_a = d3(uni->bg_a.x, uni->bg_a.y, uni->bg_a.z), bg_b = d3(uni->bg_b.x, uni->bg_b.y, uni->bg_b.z);
        color = mul(L.thr, add(smul(bg_a, 1.0 - t), smul(bg_b, t)));
    } else if (!last) {
        const double4 g = geo_at();
        const MatRec m = mat_at();
        const D3 point = add(L.org, smul(L.dir, closest));                             // Ray.At (ray/ray.go:23-25)
        const D3 outward = sdiv_rcp(sub(point, d3(g.x, g.y, g.z)), m.radius, m.rinv);  // ray/objects.go:100
        const bool front = dot(L.dir, outward) < 0;                                    // SetFaceNormal (:19-26)
        const D3 normal = front ? outward : neg(outward);
        bool scattered = true;
        D3 new_dir;
        D3 att = d3(m.albedo[0], m.albedo[1], m.albedo[2]);
        const bool lambertian = m.type == kLambertian;
        D3 uv = d3(0, 0, 0);
        if (lambertian || (m.type == kMetal && m.param > 0.0)) uv = unit_vector_from(u);
        if (lambertian) {  // ray/materials.go:13-20
            new_dir = add(normal, uv);
            if (near_zero(new_dir)) new_dir = normal;
        } else if (m.type == kMetal) {  // ray/materials.go:28-37
            D3 reflected = reflect(ud, normal);
            if (m.param > 0.0) reflected = add(reflected, smul(uv, m.param));
            new_dir = reflected;
            scattered = dot(new_dir, normal) > 0;
        } else {  // Dielectric, ray/materials.go:44-64
            att = d3(1.0, 1.0, 1.0);
            const double ratio = front ? m.pinv : m.param;  // 1.0/RefIdx precomputed (same bits)
            const double cos_theta = go_min(dot(neg(ud), normal), 1.0);
            const double sin_theta = __builtin_sqrt(1.0 - cos_theta * cos_theta);
            const bool do_reflect = ratio * sin_theta > 1.0 || reflectance(cos_theta, ratio) > u.u0;
            new_dir = do_reflect ? reflect(ud, normal) : refract(ud, normal, ratio);
        }
        if (scattered) {
            L.thr = mul(L.thr, att);
            L.org = point;
            L.dir = new_dir;
            ++L.bounce;
        } else {
            ends = true;  // absorbed -> black
        }
    }
    if (!ends) return true;
    if (!finish_sample<kFmt, kStats>(p, L, color, st)) return false;
    if (hit && !last) u = camera_block(uni, L.pixel, L.sample);  // absorbed: `u` was the scatter block
    get_ray(p, uni, u, L.fx, L.fy, L.org, L.dir);
    return true;
}

#ifndef TRAY_WAVES_PER_SIMD
#define TRAY_WAVES_PER_SIMD 5
#endif
#ifndef TRAY_BVH_WAVES_PER_SIMD
#define TRAY_BVH_WAVES_PER_SIMD 3
#endif
// BVH lane scheduling: node steps per loop iteration, and how many lanes must
// be waiting before the (expensive, FP64) leaf and shading phases run. A phase
// also runs whenever nothing else can make progress.
#ifndef TRAY_NODE_STEPS
#define TRAY_NODE_STEPS 2
#endif
#ifndef TRAY_LEAF_BATCH
#define TRAY_LEAF_BATCH 24
#endif
#ifndef TRAY_SHADE_BATCH
#define TRAY_SHADE_BATCH 32
#endif

// Diagnostic build only (-DTRAY_PROFILE): per-wave s_memtime stamps around each
// phase of the BVH loop, plus phase and active-lane counts, added into
// stats[3..18] (the stats buffer must then hold 19 counters). Never part of a
// timed build: the stamps' waits serialise the phases.
#ifdef TRAY_PROFILE
#define PROF_T0() const uint64_t prof_t0_ = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot) prof[slot] += __builtin_amdgcn_s_memtime() - prof_t0_
#define PROF_CNT(slot, v) prof[slot] += (v)
#else
#define PROF_T0()
#define PROF_ADD(slot)
#define PROF_CNT(slot, v)
#endif

// Persistent megakernel: waves pull 64-pixel work items from a global counter
// and lanes refill individually, so no lane idles while the frame has work.
//
// Linear scan (kBVH = false): each loop iteration is one Scene.Hit + shading
// step for every busy lane.
// BVH (kBVH = true): each lane is a small state machine (traverse a node / test
// a leaf / shade) and one loop iteration runs a few cheap node steps for the
// traversing lanes, then the leaf phase and the shading phase only once enough
// lanes wait for them. A lane whose traversal ends early does not wait for the
// wave's slowest ray: it shades and starts its next segment while others still
// traverse.
template <bool kLDS, int kFmt, bool kBVH, bool kStats>
__global__ __launch_bounds__(256, kBVH ? TRAY_BVH_WAVES_PER_SIMD : TRAY_WAVES_PER_SIMD) void render_kernel(KernelParams p) {
    extern __shared__ __attribute__((aligned(16))) double4 smem_all[];
    __attribute__((address_space(3))) Uniforms* uni_lds =
        (__attribute__((address_space(3))) Uniforms*)reinterpret_cast<Uniforms*>(smem_all);
    double4* smem = smem_all + kUniformsBytes / sizeof(double4);
    if (threadIdx.x == 0) {  // scalar stores: an aggregate copy would go through scratch
        volatile __attribute__((address_space(3))) Uniforms* u = uni_lds;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            u->cam.position[k] = p.cam.position[k];
            u->cam.pixel00[k] = p.cam.pixel00[k];
            u->cam.pixel_x[k] = p.cam.pixel_x[k];
            u->cam.pixel_y[k] = p.cam.pixel_y[k];
            u->cam.defocus_u[k] = p.cam.defocus_u[k];
            u->cam.defocus_v[k] = p.cam.defocus_v[k];
        }
        u->cam.aperture = p.cam.aperture;
        u->bg_a.x = p.bg_a.x, u->bg_a.y = p.bg_a.y, u->bg_a.z = p.bg_a.z;
        u->bg_b.x = p.bg_b.x, u->bg_b.y = p.bg_b.y, u->bg_b.z = p.bg_b.z;
        u->focus_time = p.focus_time;
        u->ray_radius = p.ray_radius;
        u->seed = p.seed;
    }
    const UniPtr uni = uni_lds;
    SceneView sv{p.geo, p.nodes, p.bgeo, p.bidx, p.bmat, p.n, p.n_nodes};
    if constexpr (kLDS) {
        if constexpr (kBVH) {
            // [nodes: n_nodes x 32 B][bgeo: n_slots x 32 B][bidx: n_slots x 4 B]; shading
            // records (bmat) stay in global memory (L1/L2-resident, read once per hit).
            double4* lds_nodes = smem;
            double4* lds_geo = smem + p.n_nodes;
            int32_t* lds_idx = reinterpret_cast<int32_t*>(smem + p.n_nodes + p.n_slots);
            const double4* gn = reinterpret_cast<const double4*>(p.nodes);
            for (int i = threadIdx.x; i < p.n_nodes; i += blockDim.x) lds_nodes[i] = gn[i];
            for (int i = threadIdx.x; i < p.n_slots; i += blockDim.x) {
                lds_geo[i] = p.bgeo[i];
                lds_idx[i] = p.bidx[i];
            }
            sv.nodes = reinterpret_cast<const BvhNode*>(lds_nodes);
            sv.bgeo = lds_geo;
            sv.bidx = lds_idx;
        } else {
            for (int i = threadIdx.x; i < p.n_pad; i += blockDim.x) smem[i] = p.geo[i];
            sv.geo = smem;
        }
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    Lane L;
    L.busy = false;
    Stats st;
    Trav T;
    uint32_t state = kIdleState;
    uint32_t pool_next = 0, pool_end = 0;  // wave-uniform: unassigned items of the current chunk
    bool exhausted = false;
#ifdef TRAY_PROFILE
    uint64_t prof[16] = {};
#endif

    while (true) {
        PROF_CNT(10, 1);
        // Refill idle lanes from the wave's pool, fetching 64-item chunks from the global queue.
        PROF_T0();
        uint64_t idle = __ballot(!L.busy);
        while (idle != 0ull && !exhausted) {
            if (pool_next == pool_end) {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(p.queue, 1u);
                c = __shfl(c, 0);
                if (c >= p.nchunks) {
                    exhausted = true;
                    break;
                }
                pool_next = c * 64u;
                pool_end = pool_next + 64u;
            }
            const uint32_t n_idle = (uint32_t)__popcll(idle);
            const uint32_t take = min(n_idle, pool_end - pool_next);
            if (!L.busy) {
                const uint32_t rank = (uint32_t)__popcll(idle & lt_mask);
                if (rank < take) {
                    int32_t x, j;
                    if (decode_pixel(p, pool_next + rank, x, j)) {
                        start_pixel(p, L, x, j);
                        get_ray(p, uni, camera_block(uni, L.pixel, 0u), L.fx, L.fy, L.org, L.dir);
                        if constexpr (kBVH) {
                            ++L.segments;
                            trav_begin(T, L.org, L.dir);
                            state = sv.n_nodes > 0 ? kTravState : kShadeState;
                        }
                    }
                }
            }
            pool_next += take;
            idle = __ballot(!L.busy);
        }
        PROF_ADD(0);
        if (__ballot(L.busy) == 0ull) break;

        if constexpr (!kBVH) {
            if (L.busy) {
                ++L.segments;
                double closest;
                const int best = scene_hit_linear<TRAY_UNROLL, kStats>(sv, L.org, L.dir, closest, st);
                shade_step<kFmt, kStats>(p, uni, L, best, closest, [&] { return p.geo[best]; },
                                         [&] { return p.mat[best]; }, st);
            }
        } else {
            // Node steps for the traversing lanes.
            {
                PROF_T0();
#pragma unroll 1
                for (int s = 0; s < TRAY_NODE_STEPS; ++s) {
                    const uint64_t m = __ballot(state == kTravState);
                    if (m == 0ull) break;
                    PROF_CNT(4, 1);
                    PROF_CNT(5, __popcll(m));
                    if (state == kTravState) {
                        state = trav_node(T, sv);
                        if constexpr (kStats) ++st.boxes;
                    }
                }
                PROF_ADD(1);
            }
            // Leaf phase: FP64 sphere tests, batched.
            const uint64_t m_leaf = __ballot(state == kLeafState);
            if (m_leaf != 0ull &&
                (__popcll(m_leaf) >= TRAY_LEAF_BATCH || __ballot(state == kTravState) == 0ull)) {
                PROF_T0();
                PROF_CNT(6, 1);
                PROF_CNT(7, __popcll(m_leaf));
                if (state == kLeafState) {
                    if constexpr (kStats) st.spheres += (uint64_t)(T.leaf & 7);
                    state = trav_leaf(T, sv, L.org, L.dir);
                }
                PROF_ADD(2);
            }
            // Shading phase, batched.
            const uint64_t m_shade = __ballot(state == kShadeState);
            if (m_shade != 0ull && (__popcll(m_shade) >= TRAY_SHADE_BATCH ||
                                    __ballot(state == kTravState || state == kLeafState) == 0ull)) {
                PROF_T0();
                PROF_CNT(8, 1);
                PROF_CNT(9, __popcll(m_shade));
                if (state == kShadeState) {
                    if (shade_step<kFmt, kStats>(p, uni, L, T.best, T.closest, [&] { return sv.bgeo[T.slot]; },
                                                 [&] { return sv.bmat[T.slot]; }, st)) {
                        ++L.segments;
                        trav_begin(T, L.org, L.dir);
                        state = sv.n_nodes > 0 ? kTravState : kShadeState;
                    } else {
                        state = kIdleState;
                    }
                }
                PROF_ADD(3);
            }
        }
    }
    if constexpr (kStats) {
        atomicAdd(p.stats + 0, (unsigned long long)st.segments);
        atomicAdd(p.stats + 1, (unsigned long long)st.spheres);
        atomicAdd(p.stats + 2, (unsigned long long)st.boxes);
    }
#ifdef TRAY_PROFILE
    if (kStats && lane == 0)
        for (int i = 0; i < 16; ++i) atomicAdd(p.stats + 3 + i, (unsigned long long)prof[i]);
#endif
}

using KernelFn = void (*)(KernelParams);

template <bool kLDS, bool kBVH, bool kStats>
static KernelFn pick_fmt(int fmt) {
    if (fmt == kOutRGBF64) return render_kernel<kLDS, kOutRGBF64, kBVH, kStats>;
    if (fmt == kOutRGBF32) return render_kernel<kLDS, kOutRGBF32, kBVH, kStats>;
    return render_kernel<kLDS, kOutRGBA8, kBVH, kStats>;
}

static KernelFn pick_kernel(bool use_lds, bool bvh, bool stats, int fmt) {
    if (stats) {  // instrumented launches (bench roofline counts) always write f32
        if (use_lds) return bvh ? render_kernel<true, kOutRGBF32, true, true> : render_kernel<true, kOutRGBF32, false, true>;
        return bvh ? render_kernel<false, kOutRGBF32, true, true> : render_kernel<false, kOutRGBF32, false, true>;
    }
    if (use_lds) return bvh ? pick_fmt<true, true, false>(fmt) : pick_fmt<true, false, false>(fmt);
    return bvh ? pick_fmt<false, true, false>(fmt) : pick_fmt<false, false, false>(fmt);
}

// Blocks the device keeps resident for this kernel and LDS size (persistent grid cap).
static int resident_blocks(int device, KernelFn fn, size_t lds) {
    hipDeviceProp_t prop;
    int cus = 256;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), 256, lds) !=
            hipSuccess ||
        per_cu <= 0)
        per_cu = 2;
    return cus * per_cu;
}

hipError_t launch_render(KernelParams p, bool use_bvh, hipStream_t stream) {
    if (p.rows <= 0) return hipSuccess;
    p.tiles_x = (p.width + 7) / 8;
    const uint32_t tiles_y = (uint32_t)((p.rows + 7) / 8);
    p.nchunks = (uint32_t)p.tiles_x * tiles_y;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const size_t lds_bytes = use_bvh ? (size_t)p.n_nodes * sizeof(BvhNode) + (size_t)p.n_slots * (sizeof(double4) + 4)
                                     : (size_t)p.n_pad * sizeof(double4);
    const bool use_lds = lds_bytes + kUniformsBytes <= kMaxLDSBytes;
    const size_t lds = kUniformsBytes + (use_lds ? (lds_bytes + 15) / 16 * 16 : 0);
    const bool stats = p.stats != nullptr;
    const KernelFn fn = pick_kernel(use_lds, use_bvh, stats, p.out_format);
    // Per-device, per-(kernel, LDS size) launch setup, cached.
    struct Setup {
        int dev;
        KernelFn fn;
        size_t lds;
        int blocks;
    };
    static thread_local Setup cache[8] = {};
    static thread_local int cache_next = 0;
    int blocks = 0;
    for (const Setup& c : cache)
        if (c.fn == fn && c.dev == dev && c.lds == lds && c.blocks > 0) blocks = c.blocks;
    if (blocks == 0) {
        if (use_lds) {
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kMaxLDSBytes);
            if (e != hipSuccess) return e;
        }
        blocks = resident_blocks(dev, fn, lds);
        cache[cache_next] = Setup{dev, fn, lds, blocks};
        cache_next = (cache_next + 1) % 8;
    }
    // Enough waves for every item, capped at what the device keeps resident.
    const uint32_t want = (p.nchunks + 3u) / 4u;
    const uint32_t grid = std::min<uint32_t>(want, (uint32_t)blocks);
    e = hipMemsetAsync(p.queue, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    if (stats) {
#ifdef TRAY_PROFILE
        e = hipMemsetAsync(p.stats, 0, 19 * sizeof(unsigned long long), stream);
#else
        e = hipMemsetAsync(p.stats, 0, 3 * sizeof(unsigned long long), stream);
#endif
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, stream, p);
    return hipGetLastError();
}

}  // namespace tray
