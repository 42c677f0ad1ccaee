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
// Execution model (per launch band of rows):
//   * a work item is one sample (pixel, s); a lane traces one path at a time and
//     stores its colour in the band's sample buffer; resolve_kernel then adds
//     each pixel's samples in sample order (ray/tracer.go:143) and scales by 1/r;
//   * the recursion of RayColor becomes an iterative bounce loop; lanes refill
//     individually from a persistent work queue, so a wave never waits for its
//     slowest path;
//   * Scene.Hit is an exact-culling 4-wide BVH (tray_bvh.cpp) staged in LDS,
//     one 1024-lane workgroup per CU; each lane is a state machine (refill /
//     node visit / leaf / shade) and the expensive phases run batched;
//   * small scenes, or TRAY_FLAG_LINEAR_SCAN, use the reference-order linear
//     scan over NaN-padded LDS geometry instead.
// Arithmetic: FP64, reference op order, compiled with -ffp-contract=off.
// The one intentional difference from the Go recursion: attenuations are
// multiplied outer-first (((att0*att1)*att2)*sky instead of
// att0*(att1*(att2*sky))), which changes colours by <= a few ulps and never a
// path decision.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "bvh.hpp"
#include "fp64.hpp"
#include "rng.hpp"
#include "tray_internal.hpp"
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
// cond ? neg(v) : v as sign-bit flips (one mask, three XORs instead of six selects).
__device__ __forceinline__ double flip(double x, uint64_t m) {
    return __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, x) ^ m);
}
__device__ __forceinline__ D3 neg_if(D3 v, bool cond) {
    const uint64_t m = (uint64_t)cond << 63;
    return d3(flip(v.x, m), flip(v.y, m), flip(v.z, m));
}

// a / b, correctly rounded, given y = RN(1/b) (exactly rounded, e.g. a full
// division or a host-side 1.0/b): q = RN(a*y) is within 1 ulp of a/b, the
// residual fma(-b, q, a) is exact, and one correction fma(r, y, q) returns
// RN(a/b) when |q| lies in [2^-960, 2^960) (Markstein 1990; Muller et al.,
// Handbook of Floating-Point Arithmetic §4.7). 3 FP64 instructions instead of
// ~10 for the generic sequence; checked on 4.3e9 pairs by tools/div_check.hip.
// The range is tested on the high word (biased exponent 63..1982; NaN and
// infinities fail); quotients outside it take the full division in a rarely
// taken branch.
//
// A vector divided by t (Unit, the normal (P - C) / R): one range check per
// component and one branch for the three. A zero component also takes that
// branch (the sign of a zero quotient needs the full division; exact zeros do
// not occur in practice), so the common path has no zero test and no select.
__device__ __forceinline__ double div_rcp_nz(double a, double b, double y, bool& ok) {
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    ok = ok & (((hi_word(q) & 0x7FF00000u) - (63u << 20)) < (1920u << 20));
    return __builtin_fma(r, y, q);
}
__device__ __forceinline__ D3 sdiv_rcp(D3 v, double t, double y) {
    bool ok = true;
    const D3 q = d3(div_rcp_nz(v.x, t, y, ok), div_rcp_nz(v.y, t, y, ok), div_rcp_nz(v.z, t, y, ok));
    if (__builtin_expect(!ok, 0)) return sdiv(v, t);
    return q;
}
// A root of Sphere.Hit, (h -+ sqrt(disc)) / a (ray/objects.go:91,93), is used
// only through `root > 1e-6 && root < closest` and, when that holds, as the
// value itself: a quotient below 2^-960 (or a zero of either sign) fails
// root > 1e-6 whether or not it is exact, so only the upper end of the range
// is checked (q >= 2^960, infinities and NaN take the full division): two
// integer instructions and no select.
__device__ __forceinline__ double div_root(double a, double b, double y) {
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    const double q1 = __builtin_fma(r, y, q);
    // biased exponent >= 1983 (one 32-bit field extract and compare)
    if (__builtin_expect(__builtin_amdgcn_ubfe(hi_word(q), 20u, 11u) >= 1983u, 0)) return a / b;
    return q1;
}
__device__ __forceinline__ double dot(D3 u, D3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ double length_sq(D3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
// Unit (ray/vec3.go:116-119): each component divided by the length. `lsq` is
// length_sq(v) when the caller already has it (same bits).
__device__ __forceinline__ D3 unit_lsq(D3 v, double lsq) {
    const double l = sqrt_cr(lsq);
    return sdiv_rcp(v, l, rcp_cr(l));
}
__device__ __forceinline__ D3 unit(D3 v) { return unit_lsq(v, length_sq(v)); }
__device__ __forceinline__ bool near_zero(D3 v) {
    const double s = 1e-8;
    return (__builtin_fabs(v.x) < s) && (__builtin_fabs(v.y) < s) && (__builtin_fabs(v.z) < s);
}
// math.Min(x, 1): NaN propagates, everything else compares (no signed-zero or
// -Inf special case can change the result against the constant 1).
__device__ __forceinline__ double go_min1(double x) { return !(x >= 1.0) ? x : 1.0; }
__device__ __forceinline__ D3 reflect(D3 v, D3 n) { return sub(v, smul(n, 2 * dot(v, n))); }
__device__ __forceinline__ D3 refract(D3 uv, D3 n, double eta) {
    const double cos_theta = go_min1(dot(neg(uv), n));
    const D3 perp = smul(add(uv, smul(n, cos_theta)), eta);
    const D3 par = smul(n, -sqrt_cr(__builtin_fabs(1.0 - length_sq(perp))));
    return add(perp, par);
}
// Reflectance (ray/materials.go:66-71) given r0 = ((1 - ref_idx) / (1 + ref_idx))^2,
// precomputed per face on the host; math.Pow(x,5) == x*((x*x)*(x*x)).
__device__ __forceinline__ double reflectance(double cosine, double r0) {
    const double x = 1 - cosine;
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return r0 + (1 - r0) * (x * x4);
}

// The uniform u = w 2^-32 of a 32-bit word of a draw block (include/tray.h).
__device__ __forceinline__ double uniform(uint32_t w) { return (double)w * 0x1.0p-32; }

// InDisc(radius) (ray/tracer.go:138, ray/camera.go:128): polar map of two
// uniforms: r = sqrt(ua), phi = 2 pi ub (ub given as its word).
__device__ __forceinline__ void disc(uint32_t wa, uint32_t wb, double radius, double& ox, double& oy) {
    // ua = k 2^-32: 0 or >= 2^-32, inside sqrt_core's range
    const double ua = uniform(wa);
    double r = sqrt_core(ua);
    if (wa == 0) r = ua;
    double s, c;
    sincos_2pi_word(wb, s, c);
    ox = (r * c) * radius;
    oy = (r * s) * radius;
}

// The kernel's parameters read afresh from the kernel-argument segment: a use through
// this reference reloads the fields it needs (scalar loads, cached) instead of the
// compiler keeping every parameter the loop touches in a scalar register across the
// whole loop, where the product instance spilled 20 of them to vector-register lanes.
__device__ __forceinline__ const KernelParams& kp_fresh() {
    typedef const __attribute__((address_space(4))) KernelParams* ConstParams;
    ConstParams q = (ConstParams)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));  // opaque: no load through q is hoisted above this point
    return *(const KernelParams*)q;
}

// The workgroup's chunk pool, in LDS (take_chunk). The camera, background and draw key
// are read from the kernel arguments where they are used (callers pass kp_fresh()):
// scalar loads at the use, neither a register held across the loop nor an LDS copy
// re-read through vector instructions (that copy cost C2 0.7 %, C1 1.5 %, C5 0.9 %).
struct Uniforms {
    uint64_t pool;  // the workgroup's chunk pool: (end << 32) | next (take_chunk)
    uint32_t pool_chunks;  // chunks per pool refill (read only when refilling)
};
// Explicit LDS address space: a generic volatile pointer would be accessed with
// (slow, system-coherent) flat loads.
typedef const volatile __attribute__((address_space(3))) Uniforms* UniPtr;
constexpr size_t kUniformsBytes = (sizeof(Uniforms) + 255) / 256 * 256;

// The draw block of (pixel, sample, bounce, purpose) (include/tray.h, rng.hpp draw_block).
__device__ __forceinline__ Block draw(const KernelParams& p, uint32_t pixel, uint32_t sample, uint32_t bounce,
                                     uint32_t purpose) {
    return draw_block(p.key[0], p.key[1], p.key[2], p.key[3], pixel, sample, bounce, purpose);
}

__device__ __forceinline__ D3 ld3(const double v[3]) { return d3(v[0], v[1], v[2]); }

// RandomUnitVector (ray/rand.go:30-32): Archimedes' projection of two uniforms of
// the bounce's scatter block, z = 1 - 2 u0, r = sqrt(1 - z*z), phi = 2 pi u1.
__device__ __forceinline__ D3 unit_vector_from(double z, double r, uint32_t w1) {
    double s, c;
    sincos_2pi_word(w1, s, c);
    return d3(r * c, r * s, z);
}

// The sample's camera block (purpose 1): (pixel, sample, 0, 1).
__device__ __forceinline__ Block camera_block(const KernelParams& p, uint32_t pixel, uint32_t sample) {
    return draw(p, pixel, sample, 0u, kPurposeCamera);
}

// Camera.GetRay (ray/camera.go:113-142). The sample's camera block `u` feeds the
// anti-aliasing disc (words 0,1; ray/tracer.go:136-139, only when r > 1) and the
// lens disc (words 2,3, only when the aperture is open).
__device__ __forceinline__ void get_ray(const KernelParams& p, const Block& u, double px, double py, D3& origin,
                                        D3& dir) {
    double ox = 0.0, oy = 0.0;
    const double aperture = p.cam.aperture;
    if (p.spp > 1) disc(u.x0, u.x1, p.ray_radius, ox, oy);
    const D3 pos = ld3(p.cam.position);
    const D3 p00 = ld3(p.cam.pixel00);
    const D3 pxv = ld3(p.cam.pixel_x);
    const D3 pyv = ld3(p.cam.pixel_y);
    const D3 sample_pt = add(add(p00, smul(pxv, px + ox)), smul(pyv, py + oy));
    origin = pos;
    dir = sub(sample_pt, pos);
    if (aperture > 0) {
        double dx, dy;
        disc(u.x2, u.x3, 1.0, dx, dy);
        const D3 du = ld3(p.cam.defocus_u);
        const D3 dv = ld3(p.cam.defocus_v);
        const D3 offset = add(smul(du, dx), smul(dv, dy));
        const D3 focus_point = add(pos, smul(dir, p.focus_time));
        origin = add(pos, offset);
        dir = sub(focus_point, origin);
    }
}

// ColorF.ToSRGBA channel (ray/vec3.go:173-180) as the number of encoder
// thresholds <= c: t[k] (k = 1..255) is the least double the host encoder maps
// to >= k (tray::srgb_thresholds), so this returns the host encoder's byte for
// every double, NaN and the clamps included, with no device pow. `t` is the
// table in LDS; eight compares of a branch-free binary search.
__device__ __forceinline__ uint32_t srgb_encode(const double* t, double c) {
    uint32_t n = 0;
#pragma unroll
    for (uint32_t step = 128; step >= 1; step >>= 1) n += c >= t[n + step] ? step : 0u;
    return n;
}
__device__ __forceinline__ uint32_t srgba_word(const double* t, double r, double g, double b) {
    return srgb_encode(t, r) | (srgb_encode(t, g) << 8) | (srgb_encode(t, b) << 16) | (255u << 24);
}

// n / d and n % d by the launch's FastDiv (tray_kernel.hpp).
__device__ __forceinline__ uint32_t udiv(uint32_t n, const FastDiv& f, uint32_t& rem) {
    const uint32_t t = __umulhi(n, f.m);
    const uint32_t q = (t + ((n - t) >> f.s1)) >> f.s2;
    rem = n - q * f.d;
    return q;
}

// Compact output row j -> image row y (see tray_params in include/tray.h).
__device__ __forceinline__ int32_t row_of(const KernelParams& p, int32_t j) {
    if (p.tile_rows <= 0) return p.y_start + j;
    uint32_t within;
    const int32_t t = (int32_t)udiv((uint32_t)j, p.div_tile_rows, within);
    return p.y_start + (t * p.tile_count + p.tile_index) * p.tile_rows + (int32_t)within;
}

// Per-lane path state. A lane owns one pixel at a time and walks its samples
// in order; when the last sample ends it writes the pixel and takes another.
struct Lane {
    D3 org, dir, thr;
    uint32_t item;                              // work item (sample) index in the band
    uint32_t pixel, sample, bounce, segments;  // segments of this path
    int32_t x, j;                               // image column, compact output row
    uint32_t slot;                              // on-chip accumulation: the wave's slot of this sample's chunk
    bool busy;
};

// On-chip accumulation (kAcc; rays per pixel r a multiple of 64, so a 64-item
// chunk is 64 samples of one pixel, or r = 16 / 32, so a chunk is 64 / r whole
// pixel-passes; one wave takes all of a chunk's items): the wave keeps, per open
// chunk (a slot) and per pixel-pass group of the chunk, kAccCopies sets of
// three sums in LDS. A
// finishing sample adds its rounded, scaled colour there with non-returning
// LDS atomics (lanes of one wave may finish samples of one chunk in the same
// instruction; lane l adds to set l % kAccCopies, which halves the same-address
// serialisation); the adds are exact, so their order does not matter. Slots
// are retired lazily (acc_retire): when the wave needs a slot and has none
// free, every open chunk that no busy lane still traces writes its sums to
// global memory (one 32-B record per min(64, r) samples instead of 24 B per
// sample) and is freed; at exit the wave retires the rest. No per-sample
// bookkeeping. A sample's group is (item mod 64) >> rshift, with rshift =
// KernelParams::acc_rshift (6: one group per chunk; log2 r: 64 / r groups).
typedef __attribute__((address_space(3))) double LdsF64;

typedef __attribute__((address_space(3))) uint32_t LdsU32;
struct AccCtx {
    LdsF64* slabs;   // this wave's slots: groups x kAccCopies x 3 sums each
    LdsU32* counts;  // this wave's slots: Scene.Hit calls of the slot's chunk (work-order cost)
};
// kAcc: 1 one group per chunk (64 | r), 2 64 / r pixel-pass groups per chunk (r = 16, 32).
template <int kAcc>
__device__ __forceinline__ uint32_t acc_rshift(const KernelParams& p) {
    return kAcc == 2 ? p.acc_rshift : 6u;
}


// Candidate root of one sphere whose discriminant is >= 0 (Sphere.Hit,
// ray/objects.go:86-94): the first root inside (1e-6, closest) wins. Used by the
// linear scan, which visits spheres in list order exactly like the reference.
__device__ __forceinline__ void candidate(double h, double disc, double a, double a_inv, int idx, double& closest,
                                          int& best) {
    if (disc >= 0) {
        const double sq = sqrt_cr(disc);
        double root = div_root(h - sq, a, a_inv);
        bool ok = root > 1e-6 && root < closest;
        if (!ok) {
            root = div_root(h + sq, a, a_inv);
            ok = root > 1e-6 && root < closest;
        }
        if (ok) {
            closest = root;
            best = idx;
        }
    }
}

// The any-order rule (test_geo). Sphere.Hit's root choice does not depend on
// the interval end: root2 >= root1, so the reference takes t = root1 if
// root1 > 1e-6, else root2, and accepts it iff t < closestSoFar. The linear
// scan therefore returns min over spheres of (t_i, i); accepting "t < closest,
// or t == closest with a lower index" reproduces it for any visiting order.

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
#ifndef TRAY_PROFILE
struct Stats {
    uint64_t segments = 0, spheres = 0, boxes = 0;
#ifdef TRAY_STATS_PRIMARY  // diagnostic: node visits, leaf visits, box tests of primary segments; all node/leaf visits
    uint64_t nodes0 = 0, leaves0 = 0, boxes0 = 0, nodes = 0, leaves = 0;
#endif
#ifdef TRAY_STATS_GROUND  // diagnostic: segments leaving an out-of-tree sphere (upward cube face / any) and their visits
    uint64_t g_seg[2] = {0, 0}, g_nodes[2] = {0, 0}, g_leaves[2] = {0, 0}, nodes = 0, leaves = 0;
#endif
};
#else  // phase profiles count in LDS; per-lane counters would cost registers
struct NoCount {
    __device__ NoCount& operator+=(uint64_t) { return *this; }
    __device__ operator unsigned long long() const { return 0ull; }
};
struct Stats {
    NoCount segments, spheres, boxes;
};
#endif

// Geometry visible to one workgroup (LDS copies, or global memory when the
// scene does not fit).
struct SceneView {
    const double4* geo;     // linear scan: list order, NaN-padded
    const Bvh4Node* nodes;  // BVH: 4-wide nodes, root first
    const int32_t* leaves;  // BVH: per leaf (first slot << 3) | count
    bool single;            // BVH: one sphere per leaf, leaf index == slot
    const double4* bgeo;    // BVH: spheres in leaf-slot order
    const int32_t* bidx;    // BVH: original list index of each slot
    const MatRec* bmat;     // BVH: shading record of each slot
    int32_t n, n_nodes;
    int32_t n_global, global_first;  // BVH: spheres tested before the tree, their first slot
};

// Scene.Hit (ray/objects.go:37-46) as the reference's linear scan over
// NaN-padded geometry (a NaN discriminant is never >= 0). Spheres are tested in
// groups of U that share one wave-level branch into the rare sqrt/div path;
// inside a group they are visited in list order.
template <int U, bool kStats>
__device__ __forceinline__ int scene_hit_linear(const SceneView& sv, const D3& org, const D3& dir, double& closest,
                                                Stats& st) {
    const double a = length_sq(dir);  // hoisted: same bits as per sphere
    const double a_inv = rcp_cr(a);
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

// Per-lane traversal state of one Scene.Hit through the exact-culling 4-wide
// BVH (tray_bvh.cpp): conservative FP32 slab tests of a node's four child boxes
// (culled against the current closest hit), near-first descent with a per-lane
// stack in LDS, FP64 sphere tests with the reference's arithmetic and the
// any-order acceptance rule.
// Lane states of the BVH kernel, encoded in Trav::cur (no state register, no
// per-step state bookkeeping): an inner node (< kBvhLeafBit) = traversing; a
// leaf reference = waiting for the leaf phase; kBvhNone = traversal done,
// waiting for the shade phase (busy lane) or idle (Lane::busy false).

struct Trav {
    float ix, iy, iz, oix, oiy, oiz;  // FP32 ray: t = box * inv - org * inv
    float tlim;                       // closest rounded up to float
    int32_t near_x, near_y, near_z;   // byte offsets of the near planes in a node
    uint32_t cur;                     // child reference to visit next (kBvhNone: done)
    uint32_t top;                     // stack top: sort key (entry distance | reference)
    int32_t sp;                       // stack depth (the top included)
    double a, a_inv, closest;
    int32_t slot;  // leaf slot (geometry + shading record) of the closest hit, -1: none
};

// The BVH kernel runs one workgroup per CU by default (all its waves share one
// LDS copy of the scene); the linear scan runs 256-lane workgroups.
constexpr int kBvhBlock = TRAY_BVH_BLOCK;
static_assert(kBvhBlock <= 1024, "BVH workgroup larger than 1024 lanes");
// Traversal stack slots per lane are kept in LDS as far as the workgroup's LDS
// allows after the scene (4 KB per slot), at least kStackLdsMin of them.
constexpr int32_t kStackLdsMin = 8;
constexpr size_t kStackSlotBytes = (size_t)kBvhBlock * sizeof(uint32_t);

// Per-lane traversal stack of sort keys. The top entry lives in Trav::top and
// slot i >= 1 holds the entry below the i-th; slot 0 is a scratch slot, so
// pushes need no branches (stack_cap = depth bound + kStackSlack). Slots below `lds`
// are in LDS, slot i of the lane at base[i * kBvhBlock] (consecutive lanes,
// consecutive banks); a scene whose bound is deeper keeps the rest in a global
// overflow area (spill set: one wave-uniform branch per access otherwise).
template <bool kSpill>
struct Stack {
    static constexpr bool spill = kSpill;
    __attribute__((address_space(3))) uint32_t* base;  // this lane's slot 0
    uint32_t* ovf;     // this lane's slot `lds` in the overflow area (stride: grid lanes)
    uint32_t stride;
    int32_t lds;
};

template <class Stk>
__device__ __forceinline__ uint32_t stack_load(const Stk& S, int32_t i) {
    if constexpr (Stk::spill)
        if (i >= S.lds) return S.ovf[(size_t)(i - S.lds) * S.stride];
    return S.base[i * kBvhBlock];
}

template <class Stk>
__device__ __forceinline__ void stack_store(const Stk& S, int32_t i, uint32_t v) {
    if constexpr (Stk::spill) {
        if (i >= S.lds) {
            S.ovf[(size_t)(i - S.lds) * S.stride] = v;
            return;
        }
    }
    S.base[i * kBvhBlock] = v;
}

// Sort key of a hit child: the upper 16 bits of its entry distance (tn >= 0, so
// keys order like distances, to bf16 precision, and never exceed the true tn)
// over its 16-bit reference. ~0 = no entry.
__device__ __forceinline__ float key_tn(uint32_t key) { return __uint_as_float(key & 0xFFFF0000u); }

__device__ __forceinline__ bool is_trav(uint32_t cur) { return cur < kBvhLeafBit; }
__device__ __forceinline__ bool is_leaf(uint32_t cur) { return cur - kBvhLeafBit < kBvhNone - kBvhLeafBit; }

// Sphere.Hit of the sphere with geometry `g` in leaf slot `slot` under the
// any-order rule (above) with the hit kept as a slot: the
// original list index (the tie-break key, bidx) is read only on an exact tie
// t == closest, which is rare, so no index load sits on the path of every
// accepted hit (for scenes whose geometry stays in global memory it was a
// second dependent round trip after the sphere's own load).
__device__ __forceinline__ void test_geo(Trav& T, const SceneView& sv, const double4 g, int32_t slot, const D3& org,
                                         const D3& dir) {
    double h, d;
    quad(g, org, dir, T.a, h, d);
    if (d >= 0) {
        const double sq = sqrt_cr(d);
        const double r1 = div_root(h - sq, T.a, T.a_inv);
        const double t = r1 > 1e-6 ? r1 : div_root(h + sq, T.a, T.a_inv);
        // Accept with selects; only an exact tie with an earlier hit branches (to read
        // both list indices).
        const bool front = t > 1e-6;
        bool take = front & (t < T.closest);
        if (__builtin_expect(front & (t == T.closest) & (T.slot >= 0), 0)) take = sv.bidx[slot] < sv.bidx[T.slot];
        T.closest = take ? t : T.closest;
        T.slot = take ? slot : T.slot;
    }
}
__device__ __forceinline__ void test_slot(Trav& T, const SceneView& sv, int32_t slot, const D3& org, const D3& dir) {
    test_geo(T, sv, sv.bgeo[slot], slot, org, dir);
}

// Scene.Hit's FP64 setup for a new segment: a = |dir|^2 and its reciprocal,
// no hit yet, and the spheres kept out of the tree (tray_bvh.cpp, at most
// kBvhGlobals) tested first; a hit seeds the culling distance of the traversal.
__device__ __forceinline__ void trav_globals(Trav& T, const SceneView& sv, const D3& org, const D3& dir) {
    T.a = length_sq(dir);  // hoisted: same bits as per sphere
    T.a_inv = rcp_cr(T.a);
    T.closest = __builtin_inf();
    T.slot = -1;
#pragma unroll
    for (int32_t g = 0; g < kBvhGlobals; ++g)
        if (g < sv.n_global) test_slot(T, sv, sv.global_first + g, org, dir);
}

// The FP32 traversal setup of a segment whose FP64 part (trav_globals) is done.
__device__ __forceinline__ void trav_begin32(Trav& T, const SceneView& sv, const D3& org, const D3& dir) {
    T.cur = sv.n_nodes > 0 ? 0u : kBvhNone;  // the root
    T.sp = 0;
    T.top = ~0u;
    float dxf = (float)dir.x, dyf = (float)dir.y, dzf = (float)dir.z;
    if (__builtin_fabsf(dxf) < 1e-30f) dxf = 1e-30f;
    if (__builtin_fabsf(dyf) < 1e-30f) dyf = 1e-30f;
    if (__builtin_fabsf(dzf) < 1e-30f) dzf = 1e-30f;
    // ~1 ulp reciprocal: inside the padding's error budget (tray_bvh.cpp)
    const float ix = __builtin_amdgcn_rcpf(dxf);
    const float iy = __builtin_amdgcn_rcpf(dyf);
    const float iz = __builtin_amdgcn_rcpf(dzf);
    const float oix = (float)org.x * ix, oiy = (float)org.y * iy, oiz = (float)org.z * iz;
    T.ix = ix, T.iy = iy, T.iz = iz;
    T.oix = oix, T.oiy = oiy, T.oiz = oiz;
    // Bvh4Node::box[a][s]: the near plane is the low one when the ray runs up the axis.
    constexpr int32_t kPlane = 4 * kBvhWidth;  // bytes of one plane block (one float per child)
    T.near_x = ix < 0.0f ? kPlane : 0;
    T.near_y = 2 * kPlane + (iy < 0.0f ? kPlane : 0);
    T.near_z = 4 * kPlane + (iz < 0.0f ? kPlane : 0);
    T.tlim = f32_up(T.closest);
}

__device__ __forceinline__ void trav_begin(Trav& T, const SceneView& sv, const D3& org, const D3& dir) {
    T.tlim = __builtin_inff();
    trav_globals(T, sv, org, dir);
    trav_begin32(T, sv, org, dir);
}

// Push `key` if valid. The store is unconditional: with no push it writes
// slot sp, above the stack.
template <class Stk>
__device__ __forceinline__ void stack_push(Trav& T, const Stk& S, uint32_t key) {
    const bool valid = key != ~0u;
    stack_store(S, T.sp, T.top);
    T.top = valid ? key : T.top;
    T.sp += valid ? 1 : 0;
}

// Pop the next entry to visit: the top, or (when the top's box lies beyond the
// current closest hit, key_tn > tlim) the entry below it, read ahead in `below`.
// One cull at most and no further LDS round trip: an entry that is still
// beyond tlim is visited anyway, which the box tests and the any-order rule
// make harmless. Returns its reference, or kBvhNone.
template <class Stk>
__device__ __forceinline__ uint32_t stack_pop(Trav& T, const Stk& S, uint32_t below) {
    // Slot 0 always holds ~0 (written only by a push at depth 0, from the empty
    // top), so an empty stack pops ~0: key_tn(~0) is NaN (never culled) and
    // ~0 & 0xFFFF is kBvhNone. No emptiness branches: one divergent cull.
    uint32_t key = T.top;
    T.top = below;
    T.sp = max(T.sp - 1, 0);
    if (key_tn(key) > T.tlim) {
        key = T.top;
        T.sp = max(T.sp - 1, 0);
        T.top = stack_load(S, T.sp);  // the entry of depth sp sits in slot sp
        if (T.sp == 0 && key_tn(key) > T.tlim) key = ~0u;
    }
    return key & 0xFFFFu;
}


// One node visit: test the four child boxes, visit the nearest hit child next
// (an inner node or a leaf) and push the other hit children far-to-near. T.cur
// becomes the next reference (the lane's state).
template <class Stk>
__device__ __forceinline__ void trav_node(Trav& T, const SceneView& sv, const Stk& S, uint32_t& tested) {
    constexpr int32_t kPlane = 4 * kBvhWidth;  // far plane block = near ^ kPlane
    const char* nb = reinterpret_cast<const char*>(sv.nodes + T.cur);
    const uint32_t below = stack_load(S, max(T.sp - 1, 0));  // read ahead for a pop
    // Hit children: upper 16 bits of the entry distance | reference (tn >= 0, so
    // the keys order like the distances, to bf16 precision); anything else ~0.
    // An unused child's planes are (+inf, -inf): tn = +inf, never a hit.
    uint32_t key[kBvhWidth];
    tested = 0;
#pragma unroll
    for (int g = 0; g < kBvhWidth / 4; ++g) {  // four children per group of 16-B loads
        const float4 nx = *reinterpret_cast<const float4*>(nb + T.near_x + 16 * g);
        const float4 fx = *reinterpret_cast<const float4*>(nb + (T.near_x ^ kPlane) + 16 * g);
        const float4 ny = *reinterpret_cast<const float4*>(nb + T.near_y + 16 * g);
        const float4 fy = *reinterpret_cast<const float4*>(nb + (T.near_y ^ kPlane) + 16 * g);
        const float4 nz = *reinterpret_cast<const float4*>(nb + T.near_z + 16 * g);
        const float4 fz = *reinterpret_cast<const float4*>(nb + (T.near_z ^ kPlane) + 16 * g);
        const uint4 rf = *reinterpret_cast<const uint4*>(nb + 6 * kPlane + 16 * g);
        const uint32_t ref[4] = {rf.x, rf.y, rf.z, rf.w};
        const float nxa[4] = {nx.x, nx.y, nx.z, nx.w}, fxa[4] = {fx.x, fx.y, fx.z, fx.w};
        const float nya[4] = {ny.x, ny.y, ny.z, ny.w}, fya[4] = {fy.x, fy.y, fy.z, fy.w};
        const float nza[4] = {nz.x, nz.y, nz.z, nz.w}, fza[4] = {fz.x, fz.y, fz.z, fz.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // slab distances: t = plane * inv - org * inv
            const float tnx = __builtin_fmaf(nxa[k], T.ix, -T.oix), tfx = __builtin_fmaf(fxa[k], T.ix, -T.oix);
            const float tny = __builtin_fmaf(nya[k], T.iy, -T.oiy), tfy = __builtin_fmaf(fya[k], T.iy, -T.oiy);
            const float tnz = __builtin_fmaf(nza[k], T.iz, -T.oiz), tfz = __builtin_fmaf(fza[k], T.iz, -T.oiz);
            const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(tnx, tny), tnz), 0.0f);
            const float tf = __builtin_fminf(__builtin_fminf(__builtin_fminf(tfx, tfy), tfz), T.tlim);
            key[4 * g + k] = tn <= tf ? ((__float_as_uint(tn) & 0xFFFF0000u) | ref[k]) : ~0u;
            tested += ref[k] != kBvhNone ? 1u : 0u;
        }
    }
#define TRAY_CX(i, j)                             \
    {                                             \
        const uint32_t lo_ = min(key[i], key[j]); \
        key[j] = max(key[i], key[j]);             \
        key[i] = lo_;                             \
    }
    if constexpr (kBvhWidth == 4) {
        TRAY_CX(0, 1) TRAY_CX(2, 3) TRAY_CX(0, 2) TRAY_CX(1, 3) TRAY_CX(1, 2)
    } else {  // 19-exchange network for 8
        TRAY_CX(0, 2) TRAY_CX(1, 3) TRAY_CX(4, 6) TRAY_CX(5, 7)
        TRAY_CX(0, 4) TRAY_CX(1, 5) TRAY_CX(2, 6) TRAY_CX(3, 7)
        TRAY_CX(0, 1) TRAY_CX(2, 3) TRAY_CX(4, 5) TRAY_CX(6, 7)
        TRAY_CX(2, 4) TRAY_CX(3, 5)
        TRAY_CX(1, 4) TRAY_CX(3, 6)
        TRAY_CX(1, 2) TRAY_CX(3, 4) TRAY_CX(5, 6)
    }
#undef TRAY_CX
    if (key[0] != ~0u) {
        if constexpr (kBvhWidth == 4 && !Stk::spill) {
            // Branch-free push of the hit children key[1..m] (sorted: invalid keys
            // ~0 come last) far-to-near: slots sp, sp+1, sp+2 are written
            // unconditionally; those above the new top are scratch (kStackSlack).
            const bool v1 = key[1] != ~0u, v2 = key[2] != ~0u, v3 = key[3] != ~0u;
            stack_store(S, T.sp, T.top);
            stack_store(S, T.sp + 1, v3 ? key[3] : key[2]);
            stack_store(S, T.sp + 2, key[2]);
            T.top = v1 ? key[1] : T.top;
            T.sp += (int32_t)v1 + (int32_t)v2 + (int32_t)v3;
        } else {
#pragma unroll
            for (int k = kBvhWidth - 1; k >= 1; --k) stack_push(T, S, key[k]);
        }
        T.cur = key[0] & 0xFFFFu;
    } else {
        T.cur = stack_pop(T, S, below);
    }
}

// The spheres of a multi-sphere leaf `ref` (FP64, any-order rule).
// Two spheres per step, both loads issued before either test: with the
// geometry in global memory (dense scenes) a leaf's spheres are then one
// L2 round trip, not one each. The second of an odd leaf reloads the first.
// At most kBvhLeafMax spheres per leaf: straight-line pairs (C5, 2-sphere
// leaves: -0.65 % against a counted loop).
__device__ __forceinline__ void leaf_spheres(Trav& T, const SceneView& sv, uint32_t ref, const D3& org, const D3& dir,
                                             uint32_t& tested) {
    const int32_t info = sv.leaves[ref & (kBvhLeafBit - 1u)];
    const int32_t first = info >> 3, cnt = info & 7;
#pragma unroll
    for (int32_t k = 0; k < kBvhLeafMax; k += 2) {
        if (k >= cnt) break;
        const int32_t s0 = first + k, s1 = k + 1 < cnt ? s0 + 1 : s0;
        const double4 g0 = sv.bgeo[s0], g1 = sv.bgeo[s1];
        test_geo(T, sv, g0, s0, org, dir);
        if (s1 != s0) test_geo(T, sv, g1, s1, org, dir);
        tested += s1 != s0 ? 2u : 1u;
    }
}

// Test the spheres of leaf T.cur (FP64, any-order rule), then pop the next entry.
template <class Stk>
__device__ __forceinline__ void trav_leaf(Trav& T, const SceneView& sv, const Stk& S, const D3& org,
                                              const D3& dir, uint32_t& tested) {
    const uint32_t below = stack_load(S, max(T.sp - 1, 0));  // read ahead for the pop
    if (sv.single) {  // one sphere per leaf: the leaf index is its slot (no leaf table, no loop)
        test_slot(T, sv, (int32_t)(T.cur & (kBvhLeafBit - 1u)), org, dir);
        tested = 1;
    } else {
        tested = 0;
        leaf_spheres(T, sv, T.cur, org, dir, tested);
    }
    T.tlim = f32_up(T.closest);
    T.cur = stack_pop(T, S, below);
}

// The drain's wave-wide Scene.Hit (KernelParams::coop_lanes; DESIGN.md 8d, "The
// drain"). A launch ends on a few long paths, each the last of its wave: a lone
// lane's traversal is a chain of dependent LDS reads and box tests that nothing
// else in the wave hides (the timeline build measured 4-8 us of node steps per
// segment of such a path, against 1.5-2 us of shading). Instead, the whole wave
// tests every sphere of the scene for the lone ray: lane i tests slots i, i + 64,
// ... under the any-order rule (test_geo), and the lanes' closest hits are merged
// with the same rule (least t, then least list index). That is the reference's
// linear scan result (ray/objects.go:37-46), which the traversal returns too: the
// same bits, for ~8 independent sphere tests per lane at C2.
// Scene.Hit of lane `l`'s ray (its segment's FP64 setup, T.a and T.a_inv, is done)
// by the whole wave over `n` slots; lane l gets the hit and leaves the traversal.
__device__ __forceinline__ void coop_hit(Trav& T, const SceneView& sv, int32_t n, const D3& org, const D3& dir,
                                         uint32_t l, uint32_t lane) {
    // The ray through LDS permutes, into vector registers (scalar copies would add
    // to the loop's scalar-register pressure: round 6 measured 7 more spills, +2.1 %).
    const int32_t src = (int32_t)l;
    const D3 o = d3(__shfl(org.x, src, 64), __shfl(org.y, src, 64), __shfl(org.z, src, 64));
    const D3 d = d3(__shfl(dir.x, src, 64), __shfl(dir.y, src, 64), __shfl(dir.z, src, 64));
    Trav C;
    C.a = __shfl(T.a, src, 64);
    C.a_inv = __shfl(T.a_inv, src, 64);
    C.closest = __builtin_inf();
    C.slot = -1;
    // Two slots per step, both loads issued before either test (like leaf_spheres).
    for (int32_t s0 = (int32_t)lane; s0 < n; s0 += 128) {
        const int32_t s1 = s0 + 64 < n ? s0 + 64 : s0;
        const double4 g0 = sv.bgeo[s0], g1 = sv.bgeo[s1];
        test_geo(C, sv, g0, s0, o, d);
        if (s1 != s0) test_geo(C, sv, g1, s1, o, d);
    }
    // Merge the lanes' hits (usually a handful) in lane order, wave-uniformly.
    uint64_t m = __ballot(C.slot >= 0);
    double bt = __builtin_inf();
    int32_t bs = -1;
    while (m != 0ull) {
        const uint32_t k = (uint32_t)__builtin_ctzll(m);
        m &= m - 1ull;
        const double t = __shfl(C.closest, (int32_t)k, 64);
        const int32_t s = __shfl(C.slot, (int32_t)k, 64);
        bool take = t < bt;
        if (t == bt) take = sv.bidx[s] < sv.bidx[bs];  // an exact tie: the earlier sphere of the list
        bt = take ? t : bt;
        bs = take ? s : bs;
    }
    if (lane == l) {
        T.closest = bt;
        T.slot = bs;
        T.cur = kBvhNone;  // traversal done: the shade phase takes it
    }
}

// Chunks (64 work items each) a workgroup takes from the global queue per atomic.
// One queue address serves every wave of the device and its atomics serialise
// there: per-wave fetches left waves waiting on it (1 -> 16 chunks per atomic
// cut C2 from 11.3 to ~8.4 ms), and while one wave refills the pool (a
// device-scope atomic round trip) the workgroup's other hungry waves sleep:
// 16 -> 64 chunks cut C2 another 2-3 % (48-128 are within noise, 256 loses).
// Waves take single chunks from their workgroup's pool in LDS, so the end of
// the frame stays balanced at one chunk per wave. Small launches get smaller
// pools (launch_render: every workgroup refills >= 8 times on average, pools
// of 16..TRAY_POOL_CHUNKS chunks): with 64-chunk pools a 400x225 r=16 frame
// (22.5 K chunks) hands the first 256 workgroups 64 chunks each and leaves
// the rest to a few.
#ifndef TRAY_POOL_CHUNKS
#define TRAY_POOL_CHUNKS 64
#endif
constexpr uint32_t kPoolDone = 0xFFFFFFFFu;

// The next chunk for this wave (wave-uniform), or kPoolDone once the queue is
// exhausted. The pool word packs (end << 32) | next: one 64-bit LDS add hands
// out `next`; the wave that finds next == end refills the pool from the global
// queue while any other wave that overflowed waits for `end` to change.
// A wave reserves TRAY_WAVE_CHUNKS consecutive chunks per pool take (fewer at a
// pool's end; one each once the queue is near its end, so the launch's tail stays
// chunk-grained): its lanes then stay on one pixel's consecutive passes for longer.
#ifndef TRAY_WAVE_CHUNKS
#define TRAY_WAVE_CHUNKS 32
#endif
// Single-chunk takes for the last TRAY_LATE_TAKES reservations' worth of every wave of the grid.
#ifndef TRAY_LATE_TAKES
#define TRAY_LATE_TAKES 8u
#endif
__device__ __forceinline__ uint32_t take_chunk(const KernelParams& p, UniPtr uni, uint32_t lane, uint32_t G,
                                               uint32_t& count) {
    typedef __attribute__((address_space(3))) uint64_t LdsU64;
    LdsU64* pool = (LdsU64*)&uni->pool;
    const volatile __attribute__((address_space(3))) uint32_t* pool_end =
        (const volatile __attribute__((address_space(3))) uint32_t*)&uni->pool + 1;
    while (true) {
        uint64_t old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(pool, (uint64_t)G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t next = __builtin_amdgcn_readlane((uint32_t)old, 0);
        const uint32_t end = __builtin_amdgcn_readlane((uint32_t)(old >> 32), 0);
        if (end == kPoolDone) return kPoolDone;
        if (next + G <= end) {
            count = G;
            return next;
        }
        if (next <= end) {  // the take that reaches the end (exactly one per pool): refill
            uint32_t base = 0;
            const uint32_t pool_chunks = __builtin_amdgcn_readfirstlane(uni->pool_chunks);
            if (lane == 0) base = atomicAdd(p.queue, pool_chunks);
            base = __builtin_amdgcn_readlane(base, 0);
            const uint64_t fresh = base >= p.nchunks
                                       ? (uint64_t)kPoolDone << 32
                                       : ((uint64_t)min(base + pool_chunks, p.nchunks) << 32) | base;
            if (lane == 0) __hip_atomic_store(pool, fresh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (next < end) {  // the pool's last chunks are this wave's
                count = end - next;
                return next;
            }
            continue;
        }
        while (__builtin_amdgcn_readlane(*pool_end, 0) == end) __builtin_amdgcn_s_sleep(1);
    }
}

// Work item i of a band = one sample: i = (q x passes + k) x r + s, pixel q in
// 8x8-tile order of the band's compact rows, pass k within the launch, sample s
// (so a 64-item chunk is one pixel's samples of one pass at r = 64, or an 8x8
// tile at r = 1 and one pass). A pixel's passes are consecutive: a wave traces
// the same pixel for passes x r / 64 chunks in a row, whose paths stay coherent
// (the same surfaces, similar lengths). Ordering the items pass by pass instead
// cost C2 1.2 %, C5 2.2 %, C1 6.5 % and an 8-way shard 4.6 % (each
// chunk then went to another pixel).
// Work order (p.tile_order): the t-th tile of items (q >> 6 == t) renders band tile
// tile_order[t], looked up once per chunk by the caller (`tile`, chunk_tile);
// without an order, tile t. A chunk never straddles two tiles (a tile is 64
// pixels x r x passes items, a multiple of 64).
__device__ __forceinline__ bool decode_item(const KernelParams& p, uint32_t i, uint32_t tile, int32_t& x, int32_t& j,
                                            uint32_t& s, uint32_t& k) {
    k = 0;
    uint32_t q = udiv(i, p.div_spp, s);
    if (p.passes > 1) q = udiv(q, p.div_passes, k);
    const uint32_t r = q & 63u;
    if (!p.tile_order) tile = q >> 6;
    uint32_t tx;
    const uint32_t ty = udiv(tile, p.div_tiles_x, tx);
    x = (int32_t)(tx * 8u + (r & 7u));
    const int32_t jb = (int32_t)(ty * 8u + (r >> 3));
    j = p.j0 + jb;
    return x < p.width && jb < p.band_rows;
}
// The band tile chunk c renders (wave-uniform: one scalar load per chunk taken).
__device__ __forceinline__ uint32_t chunk_tile(const KernelParams& p, uint32_t c) {
    if (!p.tile_order) return 0u;  // unused: decode_item takes q >> 6
    uint32_t rem;
    return __builtin_amdgcn_readfirstlane(p.tile_order[udiv(c, p.div_chunks_per_tile, rem)]);
}

// Start sample s of pixel (x, compact row j) in the lane: its camera ray.
__device__ __forceinline__ void start_sample(const KernelParams& p, Lane& L, uint32_t item, int32_t x,
                                             int32_t j, uint32_t s) {
    const int32_t y = row_of(p, j);
    L.item = item;
    L.x = x;
    L.j = j;
    L.pixel = (uint32_t)y * (uint32_t)p.width + (uint32_t)x;  // global index: tiling-independent RNG key
    L.sample = s;  // the RNG sample word: pass * spp + sample
    L.bounce = 0;
    L.segments = 0;
    L.thr = d3(1, 1, 1);
    L.busy = true;
    get_ray(p, camera_block(p, L.pixel, s), (double)x, (double)y, L.org, L.dir);
}

// A path ended with `color`: store it in the band's sample buffer (the resolve
// kernel adds a pixel's samples in sample order, Add(colorSum, color) of
// ray/tracer.go:143), count its segments, free the lane.
// With kAcc the colour goes to the chunk's LDS accumulator instead (above):
// the colour is already scaled by 2^acc_shift (through the background) and is
// rounded to an integer (tray_kernel.hpp), added with a non-returning LDS
// atomic (exact, so in any order).
template <bool kStats, int kAcc>
__device__ __forceinline__ void end_path(const KernelParams& p, Lane& L, const D3& color, Stats& st,
                                         const AccCtx& acc) {
    if constexpr (kAcc) {
#ifdef TRAY_PROBE_NO_ACC_ADD  // diagnostic only (wrong frames): what the LDS adds cost
        if (color.x != 12345.0) return void(L.busy = false);
#endif
        const uint32_t rs = acc_rshift<kAcc>(p);
        const uint32_t group = ((L.slot << (6u - rs)) | ((L.item & 63u) >> rs));
        LdsF64* s = acc.slabs + (group * kAccCopies + (threadIdx.x % kAccCopies)) * 3u;
        __hip_atomic_fetch_add(s + 0, __builtin_rint(color.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(s + 1, __builtin_rint(color.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(s + 2, __builtin_rint(color.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        // A counting launch (the work order's costs): the chunk's sum of squared path lengths
        // (Scene.Hit calls per path, squared): a tile's few long paths - a glass rim among sky
        // pixels - decide when its last sample ends, and squares rank it by them.
#ifdef TRAY_WO_LINEAR_COST  // A/B only: the plain sum of Scene.Hit calls
        if (p.tile_cost)
            __hip_atomic_fetch_add(acc.counts + L.slot, L.segments, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#else
        if (p.tile_cost)
            __hip_atomic_fetch_add(acc.counts + L.slot, L.segments * L.segments, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
#endif
    } else {
        double* o = p.samples + (size_t)L.item * 3;
        o[0] = color.x;
        o[1] = color.y;
        o[2] = color.z;
    }
    if (p.segments) atomicAdd(p.segments + (size_t)L.j * (size_t)p.width + (size_t)L.x, L.segments);
    if constexpr (kStats) st.segments += L.segments;
    L.busy = false;
}

// Live progress (tray_render_progress): finished samples per 8-row tile row of
// compact rows, counted in HOST memory the calling thread polls while the
// launch runs (Tracer.ProgressFunc, ray/tracer.go:126-128; no device copy can
// run beside a persistent grid that holds every CU). A wave accumulates the
// count of its current tile row (wave-uniform `cur`, `cnt`) and adds it to the
// host counter with one system-scope atomic when its lanes move on to another
// tile row (a 64-item chunk lies within one tile row) and when it exits.
// 64-bit counts: a tile row holds 8 x width x rays_per_pixel samples, which can
// pass 2^32 (e.g. width 4096 at r >= 131072).
__device__ __forceinline__ void flush_progress(const KernelParams& p, int32_t t, uint64_t n, uint32_t lane) {
    if (n != 0u && lane == 0u)
        __hip_atomic_fetch_add(p.progress + t, (unsigned long long)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void count_progress(const KernelParams& p, bool ended, int32_t j, uint32_t lane,
                                               int32_t& cur, uint64_t& cnt) {
    uint64_t m = __ballot(ended);
    while (m != 0ull) {
        const uint32_t first = (uint32_t)__builtin_ctzll(m);
        const int32_t t0 = __builtin_amdgcn_readlane(j >> 3, first);
        const uint64_t same = __ballot(ended && (j >> 3) == t0) & m;
        if (t0 != cur) {
            flush_progress(p, cur, cnt, lane);
            cur = t0;
            cnt = 0u;
        }
        cnt += (uint64_t)__popcll(same);
        m &= ~same;
    }
}

template <int kFmt>
__device__ __forceinline__ void write_pixel(const KernelParams& p, const double* srgb, D3 mean, int32_t x, int32_t j,
                                            uint32_t pass) {
    const size_t off = (size_t)j * (size_t)p.width + (size_t)x;
    void* const out = static_cast<char*>(p.out) + (size_t)pass * p.out_frame_bytes;
    if constexpr (kFmt == kOutRGBF64) {
        double* o = static_cast<double*>(out) + off * 3;
        o[0] = mean.x;
        o[1] = mean.y;
        o[2] = mean.z;
    } else if constexpr (kFmt == kOutRGBF32) {
        float* o = static_cast<float*>(out) + off * 3;
        o[0] = (float)mean.x;
        o[1] = (float)mean.y;
        o[2] = (float)mean.z;
    } else {
        static_cast<uint32_t*>(out)[off] = srgba_word(srgb, mean.x, mean.y, mean.z);
    }
}
// The mean of a pixel's samples written in the output format (pixel `off` of pass `pass`).
template <int kFmt>
__device__ __forceinline__ void write_mean(const KernelParams& p, const double* srgb, D3 sum, int32_t x, int32_t j,
                                           uint32_t pass) {
    const double inv = 1.0 / (double)p.spp;  // colorSumDiv (ray/tracer.go:123)
    const D3 mean = smul(sum, inv);
    write_pixel<kFmt>(p, srgb, mean, x, j, pass);
}

// A pixel's fixed-point sums (tray_kernel.hpp): the exact integer total of its
// r samples, converted to FP64 (one rounding) and scaled back by 2^-acc_shift
// (exact); a channel with a NaN (non-finite) sample is NaN.
// kAcc, wave-uniform: retire every open chunk (a slot in `open`) that no busy
// lane still traces: its 64 samples have all been added, so its partial sums
// go to global memory (record `chunk` of the launch band, kept per slot in
// `chunk_of`: lane s holds slot s's chunk), its slot is zeroed and freed.
// Called only when the wave finds no free slot, and at exit: the busy lanes'
// slots are found by one ballot per open slot. A wave's LDS operations complete
// in issue order, so the reads see every addition its lanes made.
template <int kAcc>
__device__ __forceinline__ uint64_t acc_retire(const KernelParams& p, const AccCtx& acc, uint64_t open, bool busy,
                                               uint32_t slot, uint32_t chunk_of, uint32_t lane) {
    uint64_t freed = 0;
    while (open != 0ull) {
        const uint32_t s0 = (uint32_t)__builtin_ctzll(open);
        open &= open - 1ull;
        if (__ballot(busy && slot == s0) == 0ull) freed |= 1ull << s0;
    }
    // Lane s retires slot s (chunk_of holds slot s's chunk in lane s): all the
    // wave's retiring slots in one pass. A wave's LDS operations complete in
    // issue order, so the reads see every addition its lanes made.
    // Each of the slot's groups (one per chunk, or 64 / r pixel-passes) is one record.
    if ((freed >> lane) & 1ull) {
        const uint32_t groups = 64u >> acc_rshift<kAcc>(p);
        // the chunk's Scene.Hit calls (a counting launch; 0 otherwise) ride in group 0's pad
        uint32_t count = 0u;
        if (p.tile_cost) {
            volatile LdsU32* n = acc.counts;  // after every add of the wave's lanes (LDS issue order)
            count = n[lane];
            n[lane] = 0u;
        }
        for (uint32_t g = 0; g < groups; ++g) {
            const uint32_t slab = kAcc == 1 ? lane : lane * groups + g;
            volatile LdsF64* v = acc.slabs + slab * kAccCopies * 3u;
            double sum[3] = {0.0, 0.0, 0.0};  // integers below 2^53: exact in any order
#pragma unroll
            for (int k = 0; k < kAccCopies; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) sum[c] += v[3 * k + c];
#pragma unroll
            for (int k = 0; k < 3 * kAccCopies; ++k) v[k] = 0.0;
            AccPartial* o = reinterpret_cast<AccPartial*>(p.samples) + (kAcc == 1 ? chunk_of : chunk_of * groups + g);
            o->sum[0] = sum[0];
            o->sum[1] = sum[1];
            o->sum[2] = sum[2];
            o->pad = g == 0 ? (double)count : 0.0;
            if constexpr (kAcc == 1) break;
        }
    }
    return freed;
}

// One recursion level of RayColor (ray/objects.go:49-62) after Scene.Hit gave
// (best, closest): the sky on a miss, else the hit record and the material's
// scatter. `geo_at`/`mat_at` give the hit sphere's geometry and shading record.
// Returns true when the lane has a scattered ray to trace, false when the path
// ended (stored; the lane is free).
//
// Written for a wave of lanes on different branches: the work several branches
// need is done once, before them — the bounce's draw block and the unit
// direction (sky, Metal, Dielectric).
template <bool kStats, int kAcc, typename GeoAt, typename MatAt>
__device__ __forceinline__ bool shade_step(const KernelParams& p, Lane& L, int best, double closest,
                                           double dir_lsq, GeoAt geo_at, MatAt mat_at, Stats& st, const AccCtx& acc) {
    const bool hit = best >= 0;
    // A hit at the last level ends the path black whatever its material does
    // (RayColor(depth 0) is black), so no scatter is computed for it.
    const bool last = L.bounce + 1u >= (uint32_t)p.max_depth;
    bool ends = !hit || last;
    // Issued first, for every lane (a miss reads a valid record it ignores), so
    // the L2 round trip of the shading record overlaps the FP64 work below
    // instead of starting after it inside the hit branch.
    const double4 g = geo_at();
    const MatRec m = mat_at();
    const Block w = draw(p, L.pixel, L.sample, L.bounce, kPurposeScatter);
    const double u0 = uniform(w.x0);
    // Unit(r.Direction) is read by the sky, Metal and Dielectric, not by Lambertian
    // (nor a last-level hit): a wave whose shading lanes are all Lambertian hits
    // (a camera-ray pass of a diffuse pixel) skips the sqrt and three quotients.
    D3 ud = d3(0, 0, 0);
    if (!hit || (!last && m.type != kLambertian)) ud = unit_lsq(L.dir, dir_lsq);  // dir_lsq = length_sq(L.dir)
    D3 color = d3(0, 0, 0);
    if (!hit) {  // AmbientLight.Hit (ray/objects.go:68-73)
        const double t = 0.5 * (ud.y + 1.0);
        const D3 bg_a = d3(p.bg_a.x, p.bg_a.y, p.bg_a.z), bg_b = d3(p.bg_b.x, p.bg_b.y, p.bg_b.z);
        color = mul(L.thr, add(smul(bg_a, 1.0 - t), smul(bg_b, t)));
    } else if (!last) {
        const D3 point = add(L.org, smul(L.dir, closest));                             // Ray.At (ray/ray.go:23-25)
        const D3 outward = sdiv_rcp(sub(point, d3(g.x, g.y, g.z)), m.radius, m.rinv);  // ray/objects.go:100
        const bool front = dot(L.dir, outward) < 0;                                    // SetFaceNormal (:19-26)
        const D3 normal = neg_if(outward, !front);
        bool scattered = true;
        D3 new_dir;
        D3 att = d3(m.albedo[0], m.albedo[1], m.albedo[2]);
        const bool lambertian = m.type == kLambertian, dielectric = m.type == kDielectric;
        // One sqrt serves RandomUnitVector's sqrt(1 - z^2) and Dielectric's sin_theta.
        const double cos_theta = go_min1(dot(neg(ud), normal));
        const double z = 1.0 - 2.0 * u0;
        const double sq = sqrt_cr(dielectric ? 1.0 - cos_theta * cos_theta : 1.0 - z * z);
        D3 uv = d3(0, 0, 0);
        if (lambertian || (m.type == kMetal && m.param > 0.0)) uv = unit_vector_from(z, sq, w.x1);
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
            const double sin_theta = sq;
            const double r0 = front ? m.albedo[0] : m.albedo[1];
            const bool do_reflect = ratio * sin_theta > 1.0 || reflectance(cos_theta, r0) > u0;
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
    // Settle the shading-record loads here, on every path: vmcnt is one in-order
    // counter, so a load still pending when end_path stores would make the next
    // write of its registers wait for the stores' write-back too.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (!ends) return true;
    end_path<kStats, kAcc>(p, L, color, st, acc);
    return false;
}

#ifndef TRAY_WAVES_PER_SIMD
#define TRAY_WAVES_PER_SIMD 5
#endif
// BVH lane scheduling: node steps per loop iteration, and how many lanes must
// be waiting before the (expensive, FP64) leaf and shading phases run. A phase
// also runs whenever nothing else can make progress.
#ifndef TRAY_NODE_STEPS
#define TRAY_NODE_STEPS 3
#endif
// Up to TRAY_NODE_STEPS_MAX node steps while at least TRAY_NODE_MORE_LANES lanes still traverse
// (the steps unrolled; against a fixed 3: C2 -2.8 %, C5 -0.8 %, DESIGN.md §5 log).
#ifndef TRAY_NODE_STEPS_MAX
#define TRAY_NODE_STEPS_MAX 5
#endif
// Trees of more than kDeepNodes nodes (more node visits per segment: C5's 514-node tree against the
// book cover's 260) run a kernel instance with one more node step (C5 -1.6 %; the same step on the
// book cover costs +0.3 %, and a runtime cap in one instance cost the book cover 0.8 %).
constexpr int kDeepSteps = TRAY_NODE_STEPS_MAX + 1;
constexpr int32_t kDeepNodes = 384;
#ifndef TRAY_NODE_MORE_LANES
#define TRAY_NODE_MORE_LANES 8
#endif
#ifndef TRAY_LEAF_BATCH
#define TRAY_LEAF_BATCH 20
#endif
// 48 since round 4's pixel-inner item order (a wave's lanes end their paths more alike): 40 / 44 /
// 52 are +0.6 / +0.1 / +0.3 % on C2 (profiles/r6p_ab_shade_batch_c{2,5}.jsonl).
#ifndef TRAY_SHADE_BATCH
#define TRAY_SHADE_BATCH 48
#endif
// Idle lanes are refilled (a camera ray each) once this many wait, or the whole wave does.
#ifndef TRAY_REFILL_BATCH
#define TRAY_REFILL_BATCH 24
#endif
// Below TRAY_TRAV_SPARSE traversing lanes (node steps mostly empty) the leaf and shade phases
// already run from TRAY_LEAF_LOW / TRAY_SHADE_LOW waiting lanes (with the adaptive node steps the
// loop leaves its steps exactly then; shading from 32: C2 -0.4 %, C5 -0.65 %).
#ifndef TRAY_TRAV_SPARSE
#define TRAY_TRAV_SPARSE 8
#endif
#ifndef TRAY_LEAF_LOW
#define TRAY_LEAF_LOW 8
#endif
#ifndef TRAY_SHADE_LOW
#define TRAY_SHADE_LOW 32
#endif
// Wave priority during the leaf phase: its pair loads (sphere geometry, L2 for
// dense scenes) issue ahead of other waves' VALU work, and their latency hides
// behind it (C2 -0.30 %, C5 -0.39 %; levels 1-3 alike; raising it instead for the
// node steps, the camera rays or the shading phase gained nothing or lost).

// Cost probes (diagnostic builds only, never timed as the product): N extra
// independent VALU instructions in one phase, to measure what an instruction
// there costs (tools/ab_bench.py A/B against the plain build).
#define TRAY_PROBE_F32(n)                                                     \
    {                                                                         \
        _Pragma("unroll") for (int i_ = 0; i_ < (n); ++i_) {                  \
            float t_;                                                         \
            asm volatile("v_add_f32_e64 %0, 1.0, 1.0" : "=v"(t_));            \
        }                                                                     \
    }
#define TRAY_PROBE_F64(n)                                                     \
    {                                                                         \
        _Pragma("unroll") for (int i_ = 0; i_ < (n); ++i_) {                  \
            double t_;                                                        \
            asm volatile("v_add_f64 %0, 1.0, 1.0" : "=v"(t_));                \
        }                                                                     \
    }

// ISA census build only (-DTRAY_CENSUS, tools/isa_census.py): a comment in the
// assembly where each phase of the BVH loop starts, so the census can attribute
// instructions to phases. Never in a timed build.
#ifdef TRAY_CENSUS
#define TRAY_MARK(name) asm volatile(";@phase " name);
#else
#define TRAY_MARK(name)
#endif

// Diagnostic build only (-DTRAY_PROFILE): per-wave s_memtime stamps around each
// phase of the BVH loop, plus phase and active-lane counts, added into
// stats[3..21] (the stats buffer must then hold 22 counters). Never part of a
// timed build: the stamps' waits serialise the phases.
#ifdef TRAY_PROFILE
// Counters live in LDS (per wave, lane 0 adds): registers would change the
// kernel being measured.
#define PROF_T0() const uint64_t prof_t0_ = __builtin_amdgcn_s_memtime()
#define PROF_ADD(slot) PROF_CNT(slot, __builtin_amdgcn_s_memtime() - prof_t0_)
#define PROF_CNT(slot, v)                                  \
    {                                                      \
        const unsigned long long v_ = (v);                 \
        if (lane == 0) atomicAdd(prof + (slot), v_);       \
    }
#elif defined(TRAY_PROFILE_TIMELINE)
// The timeline build times the phases of a wave's lone last path (refill, node steps,
// leaves, shading: tl_ph[0..3]).
#define PROF_T0() const uint64_t prof_t0_ = (kStats && tl_lone) ? __builtin_amdgcn_s_memtime() : 0
#define PROF_ADD(slot) \
    if (kStats && tl_lone) tl_ph[slot] += __builtin_amdgcn_s_memtime() - prof_t0_
#define PROF_CNT(slot, v)
#else
#define PROF_T0()
#define PROF_ADD(slot)
#define PROF_CNT(slot, v)
#endif

// Diagnostic build only (-DTRAY_PROFILE -DTRAY_PROFILE_MATERIAL): the divergence
// census of the shading passes. Per site (0: camera-ray hits shaded in the
// refill, 1: the shade phase) and per class of shaded lane (0 miss/sky, 1 hit at
// the last level, 2 Lambertian, 3 Metal without fuzz, 4 Metal with fuzz, 5
// Dielectric): [c] passes with such a lane, [6 + c] such lanes; [12 + b] passes
// executing b of the three material bodies (b = 0..3); [16] passes, [17] lanes.
// Added with global atomics after the per-wave stamps (stats[32 + 2 x waves + k]).
#ifdef TRAY_PROFILE_MATERIAL
constexpr int kMatCounters = 18;
__device__ __forceinline__ void prof_material(int site, bool active, int32_t slot, uint32_t bounce, int32_t max_depth,
                                              const MatRec* bmat, uint32_t lane, unsigned long long* pm) {
    int cls = -1;
    if (active) {
        if (slot < 0) cls = 0;
        else if (bounce + 1u >= (uint32_t)max_depth) cls = 1;
        else {
            const MatRec& m = bmat[slot];
            cls = m.type == kLambertian ? 2 : m.type == kDielectric ? 5 : m.param > 0.0 ? 4 : 3;
        }
    }
    unsigned long long* c = pm + site * kMatCounters;
    int bodies = 0;
    for (int k = 0; k < 6; ++k) {
        const uint64_t m = __ballot(cls == k);
        if (lane == 0 && m) {
            atomicAdd(c + k, 1ull);
            atomicAdd(c + 6 + k, (unsigned long long)__popcll(m));
        }
    }
    bodies = (__ballot(cls == 2) ? 1 : 0) + (__ballot(cls == 3 || cls == 4) ? 1 : 0) + (__ballot(cls == 5) ? 1 : 0);
    if (lane == 0) {
        atomicAdd(c + 12 + bodies, 1ull);
        atomicAdd(c + 16, 1ull);
        atomicAdd(c + 17, (unsigned long long)__popcll(__ballot(active)));
    }
}
#define PROF_MATERIAL(site, active) prof_material(site, active, T.slot, L.bounce, p.max_depth, p.bmat, lane, prof_mat)
#else
#define PROF_MATERIAL(site, active)
#endif

// Diagnostic build only (-DTRAY_PROFILE_TIMELINE, stats instance; tools/timeline.py):
// per wave, busy lanes integrated over time in kTlTicks buckets of the shader clock
// (s_memtime, read once per loop iteration; the 100 MHz constant clock, s_memrealtime,
// only at the wave's start, dry point and end: read per iteration it stalled waves),
// constant clock, relative to the wave's start, plus its start, end, the time its
// queue ran dry and the chunks it took. Record of wave w at stats[32 + w x kTlStride]:
// [0] start, [1] end, [2] exhausted (ticks after start), [3] chunks, [4..] buckets.
#ifdef TRAY_PROFILE_TIMELINE
// [0] start, [1] end, [2] dry (constant clock), [3] chunks, [4] / [5] shader clock at start / end,
// [6 ..] buckets; the last nine: the shader ticks the wave's lone last path spent in the
// refill, node-step, leaf and shading phases, when it became the wave's only path
// (shader ticks after the start) and its segments then, and that path's segments,
// pixel and sample at the end (its latency per segment with no other path in the wave).
constexpr uint32_t kTlBuckets = 1024, kTlTicks = 25000, kTlHdr = 6, kTlStride = kTlBuckets + kTlHdr;
#endif

// Sum of a per-lane 64-bit counter over the wave (instrumented instances only).
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

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

// LDS bytes of `slots` stack slots of a BVH workgroup (32-bit entries).
__host__ __device__ constexpr size_t bvh_stack_bytes(int32_t slots) { return (size_t)slots * kStackSlotBytes; }

// kLDS: 0 scene in global memory, 1 whole scene in LDS, 2 BVH nodes + leaf table in
// LDS with sphere geometry in global memory (scenes too big for 1; BVH only).
// kProg: the live-progress instance (tray_render_progress only), so the other
// instances carry no progress code or registers.
// kAcc: on-chip fixed-point accumulation (end_path): 0 off, 1 one sum per 64-item chunk,
// 2 one per pixel-pass of a chunk (r = 16, 32).
// kSteps: node steps per loop iteration at most (kDeepSteps for deep trees, launch_render).
template <int kLDS, bool kBVH, bool kStats, bool kSpill, bool kProg, int kAcc, int kSteps = TRAY_NODE_STEPS_MAX>
__global__ __launch_bounds__(kBVH ? kBvhBlock : 256, kBVH ? TRAY_BVH_WAVES_PER_SIMD : TRAY_WAVES_PER_SIMD) void render_kernel(KernelParams p) {
    extern __shared__ __attribute__((aligned(16))) double4 smem_all[];
    __attribute__((address_space(3))) Uniforms* uni_lds =
        (__attribute__((address_space(3))) Uniforms*)reinterpret_cast<Uniforms*>(smem_all);
    double4* smem = smem_all + kUniformsBytes / sizeof(double4);
    if (threadIdx.x == 0) {
        volatile __attribute__((address_space(3))) Uniforms* u = uni_lds;
        u->pool = 0;  // empty: the first taker refills it
        u->pool_chunks = p.pool_chunks;
    }
    const UniPtr uni = uni_lds;
    SceneView sv{p.geo,  p.nodes, p.leaves,    p.leaf_single != 0,       p.bgeo, p.bidx,
                 p.bmat, p.n,     p.n_nodes,   p.n_global, p.n_slots - p.n_global};
    Stack<kSpill> S{nullptr, nullptr, 0, 0};
    if constexpr (kBVH) {
        // [stacks: stack_cap x blockDim x 4 B][nodes: n_nodes x 128 B][bgeo: n_slots x 32 B]
        // [bidx: n_slots x 4 B][leaves: n_leaves x 4 B]; shading records (bmat) stay
        // in global memory (L1/L2-resident, read once per hit).
        S.base = (__attribute__((address_space(3))) uint32_t*)reinterpret_cast<uint32_t*>(smem) + threadIdx.x;
        S.lds = p.stack_lds;
        S.stride = gridDim.x * blockDim.x;
        if constexpr (kSpill) S.ovf = p.stack_ovf + blockIdx.x * blockDim.x + threadIdx.x;
        double4* scene = smem + bvh_stack_bytes(p.stack_lds) / sizeof(double4);
        if constexpr (kLDS == 1) {
            double4* lds_nodes = scene;
            double4* lds_geo = scene + (size_t)p.n_nodes * (sizeof(Bvh4Node) / sizeof(double4));
            int32_t* lds_idx = reinterpret_cast<int32_t*>(lds_geo + p.n_slots);
            int32_t* lds_leaves = lds_idx + p.n_slots;
            const double4* gn = reinterpret_cast<const double4*>(p.nodes);
            const int n4 = p.n_nodes * (int)(sizeof(Bvh4Node) / sizeof(double4));
            for (int i = threadIdx.x; i < n4; i += blockDim.x) lds_nodes[i] = gn[i];
            for (int i = threadIdx.x; i < p.n_slots; i += blockDim.x) {
                lds_geo[i] = p.bgeo[i];
                lds_idx[i] = p.bidx[i];
            }
            for (int i = threadIdx.x; i < p.n_leaves; i += blockDim.x) lds_leaves[i] = p.leaves[i];
            sv.nodes = reinterpret_cast<const Bvh4Node*>(lds_nodes);
            sv.bgeo = lds_geo;
            sv.bidx = lds_idx;
            sv.leaves = lds_leaves;
        } else if constexpr (kLDS == 2) {
            // [nodes][leaves]: the traversal's dependent loads stay on chip; each
            // leaf's sphere is one 32-B global load (L2-resident).
            double4* lds_nodes = scene;
            int32_t* lds_leaves =
                reinterpret_cast<int32_t*>(scene + (size_t)p.n_nodes * (sizeof(Bvh4Node) / sizeof(double4)));
            const double4* gn = reinterpret_cast<const double4*>(p.nodes);
            const int n4 = p.n_nodes * (int)(sizeof(Bvh4Node) / sizeof(double4));
            for (int i = threadIdx.x; i < n4; i += blockDim.x) lds_nodes[i] = gn[i];
            for (int i = threadIdx.x; i < p.n_leaves; i += blockDim.x) lds_leaves[i] = p.leaves[i];
            sv.nodes = reinterpret_cast<const Bvh4Node*>(lds_nodes);
            sv.leaves = lds_leaves;
        }
    } else if constexpr (kLDS == 1) {
        for (int i = threadIdx.x; i < p.n_pad; i += blockDim.x) smem[i] = p.geo[i];
        sv.geo = smem;
    }
    // [acc: waves x acc_slots x groups x kAccSlotBytes][counts: waves x acc_slots x 4 B] at acc_off
    AccCtx acc{nullptr, nullptr};
    uint64_t acc_free = 0;   // kAcc, wave-uniform: free slots
    uint64_t acc_all = 0;    // kAcc, wave-uniform: every slot
    uint32_t acc_chunk = 0;  // kAcc: lane s holds the chunk of slot s
    if constexpr (kAcc) {
        LdsF64* all = (LdsF64*)reinterpret_cast<double*>(reinterpret_cast<char*>(smem_all) + p.acc_off);
        const uint32_t waves = blockDim.x / 64u, slot_f64 = (64u >> acc_rshift<kAcc>(p)) * kAccCopies * 3u;
        const uint32_t slots = (uint32_t)p.acc_slots;
        for (uint32_t i = threadIdx.x; i < waves * slots * slot_f64; i += blockDim.x) all[i] = 0.0;
        acc.slabs = all + (threadIdx.x / 64u) * slots * slot_f64;
        LdsU32* counts = (LdsU32*)(all + waves * slots * slot_f64);
        for (uint32_t i = threadIdx.x; i < waves * slots; i += blockDim.x) counts[i] = 0u;
        acc.counts = counts + (threadIdx.x / 64u) * slots;
        acc_free = acc_all = slots >= 64u ? ~0ull : (1ull << slots) - 1ull;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    Lane L;
    L.busy = false;
    Stats st;
    Trav T;
    T.cur = kBvhNone;  // idle
    uint32_t pool_next = 0, pool_end = 0;  // wave-uniform: unassigned items of the current chunk
    uint32_t grp_next = 0, grp_end = 0;    // wave-uniform: the rest of the wave's reserved chunks

    uint32_t pool_slot = 0;                 // kAcc, wave-uniform: the current chunk's accumulator slot
    uint32_t pool_tile = 0;                 // wave-uniform: the band tile the current chunk renders (work order)
    bool exhausted = false;
#ifdef TRAY_STATS_GROUND
    uint32_t gcls = 0;  // diagnostic: class of the lane's current segment (1/2: from an out-of-tree sphere, up / other)
#endif
    int32_t prog_cur = 0;  // live progress: the wave's current tile row and its unflushed count
    uint64_t prog_cnt = 0;
#ifdef TRAY_PROFILE
    __shared__ unsigned long long prof_lds[16 * 16];
    unsigned long long* prof = prof_lds + 16 * (threadIdx.x / 64u);
    if (lane == 0)
        for (int i = 0; i < 16; ++i) prof[i] = 0;
    const uint64_t prof_start = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef TRAY_PROFILE_MATERIAL  // counts only (global atomics: its timings are not used)
    unsigned long long* prof_mat = p.stats + 32 + 2 * gridDim.x * (blockDim.x / 64u);
#endif
#ifdef TRAY_PROFILE_TIMELINE
    unsigned long long* tl =  // only the stats instance has a buffer; every use is under kStats
        kStats ? p.stats + 32 + (size_t)(blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u) * kTlStride : nullptr;
    const uint64_t tl_start = __builtin_amdgcn_s_memrealtime(), tl_mt0 = __builtin_amdgcn_s_memtime();
    uint64_t tl_prev = tl_mt0, tl_acc = 0;
    uint32_t tl_busy = 0, tl_bucket = 0, tl_chunks = 0, tl_dry = 0;
    bool tl_lone = false;
    uint64_t tl_ph[4] = {0, 0, 0, 0};
#endif

    while (true) {
#ifdef TRAY_PROFILE_TIMELINE
        if constexpr (kStats) {  // p.stats is null in every other instance
            const uint64_t now = __builtin_amdgcn_s_memtime();
            const uint32_t b = min((uint32_t)((tl_prev - tl_mt0) / kTlTicks), kTlBuckets - 10u);
            if (b != tl_bucket) {
                if (lane == 0) tl[kTlHdr + tl_bucket] = tl_acc;
                tl_bucket = b;
                tl_acc = 0;
            }
            tl_acc += (now - tl_prev) * tl_busy;
            tl_prev = now;
            // The wave's last path after its queue ran dry: its segments so far, pixel, sample.
            const uint64_t m = __ballot(L.busy);
            if (exhausted && __popcll(m) == 1) {
                const uint32_t l = (uint32_t)__builtin_ctzll(m);
                const uint32_t seg = __builtin_amdgcn_readlane(L.segments, l);
                const uint32_t pix = __builtin_amdgcn_readlane(L.pixel, l);
                const uint32_t smp = __builtin_amdgcn_readlane(L.sample, l);
                if (lane == 0) {
                    if (!tl_lone) {
                        tl[kTlHdr + kTlBuckets - 5] = now - tl_mt0;
                        tl[kTlHdr + kTlBuckets - 4] = seg;
                    }
                    tl[kTlHdr + kTlBuckets - 3] = seg;
                    tl[kTlHdr + kTlBuckets - 2] = pix;
                    tl[kTlHdr + kTlBuckets - 1] = smp;
                }
                tl_lone = true;
            }
        }
#endif
#ifndef TRAY_PROFILE_REFILL  // slots 10, 13-15 hold the refill split instead
        PROF_CNT(10, 1);
#endif
        // Refill idle lanes from the wave's pool, fetching 64-item chunks from the global queue.
        PROF_T0();
        TRAY_MARK("refill_assign")
        uint64_t idle = __ballot(!L.busy);
        if (__popcll(idle) < TRAY_REFILL_BATCH && idle != ~0ull) idle = 0ull;  // batch refills
        // Items are assigned first (cheap, may span two chunks); the camera rays of
        // all newly assigned lanes are then generated together.
        uint32_t fresh_item = ~0u, fresh_slot = 0u, fresh_tile = 0u;
        bool cam_hit = false;  // a camera ray whose Scene.Hit the candidate list answered in this refill
#ifdef TRAY_PROFILE_CANDWAIT
        uint64_t prof_wait = 0;
#endif
#ifdef TRAY_PROFILE_REFILL
        uint64_t prof_cam = 0, prof_hit = 0;  // stamps after the camera ray / after its Scene.Hit
#endif
        while (idle != 0ull && !exhausted) {
            if (pool_next == pool_end) {
                if constexpr (kAcc) {
                    // A chunk needs a free accumulator: with none, the idle lanes wait
                    // for one of the wave's open chunks to finish (every open chunk
                    // has a sample in flight, so one will).
                    if (acc_free == 0ull) {
                        // Retire the chunks no busy lane traces any more (lanes assigned in
                        // this refill have not started yet: their chunk is open regardless).
                        const bool held = L.busy || fresh_item != ~0u;
                        acc_free = acc_retire<kAcc>(kp_fresh(), acc, acc_all, held, L.busy ? L.slot : fresh_slot, acc_chunk,
                                                    lane);
                    }
                    if (acc_free == 0ull) {
                        // unreachable with nothing in flight: no chunk would hold a slot
                        if (__ballot(L.busy || fresh_item != ~0u) == 0ull) __builtin_trap();
                        break;
                    }
                }
                uint32_t c = grp_next;
                if (grp_next < grp_end) {
                    ++grp_next;
                } else {
                    uint32_t cnt = 1;
                    const KernelParams& pq = kp_fresh();
                    c = take_chunk(pq, uni, lane, grp_end >= pq.late_at ? 1u : pq.wave_chunks, cnt);
                    if (c == kPoolDone) {
                        exhausted = true;
#ifdef TRAY_PROFILE_TIMELINE
                        if constexpr (kStats) tl_dry = (uint32_t)(__builtin_amdgcn_s_memrealtime() - tl_start);
#endif
                        break;
                    }
#ifdef TRAY_PROFILE_TIMELINE
                    tl_chunks += cnt;
#endif
                    grp_next = c + 1;
                    grp_end = c + cnt;
                }
                pool_next = c * 64u;
                pool_end = pool_next + 64u;
                const KernelParams& pc = kp_fresh();
                pool_tile = chunk_tile(pc, c);
                if constexpr (kAcc) {
                    // With 64 | r every item of a chunk is one pixel's: valid or padding
                    // together. A chunk of several pixel-passes (r | 64) may mix the two
                    // and always takes a slot (its padding groups retire as zeros).
                    int32_t cx, cj;
                    uint32_t cs, cp;
                    if (acc_rshift<kAcc>(p) < 6u ||
                        (pool_next < pc.items && decode_item(pc, pool_next, pool_tile, cx, cj, cs, cp))) {
                        pool_slot = (uint32_t)__builtin_ctzll(acc_free);
                        acc_free &= ~(1ull << pool_slot);
                        acc_chunk = lane == pool_slot ? c : acc_chunk;
                    }
                }
            }
            const uint32_t n_idle = (uint32_t)__popcll(idle);
            const uint32_t take = min(n_idle, pool_end - pool_next);
            if ((idle >> lane) & 1ull) {
                // idle lanes below this one (mbcnt: no per-lane mask held across the loop)
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (rank < take) {
                    fresh_item = pool_next + rank;
                    fresh_slot = pool_slot;
                    fresh_tile = pool_tile;
                }
            }
            pool_next += take;
            idle = __ballot(!L.busy && fresh_item == ~0u);
        }
#if defined(TRAY_PROFILE) && !defined(TRAY_PROFILE_REFILL)
        {
            const uint64_t fresh = __ballot(fresh_item != ~0u);
            PROF_CNT(13, fresh != 0ull ? 1 : 0);
            PROF_CNT(14, __popcll(fresh));
        }
#endif
#ifdef TRAY_PROFILE_REFILL
        const uint64_t prof_assigned = __builtin_amdgcn_s_memtime();
#endif
        if (fresh_item != ~0u) {
            TRAY_MARK("refill_cam")
            const KernelParams& pr = kp_fresh();
            int32_t x, j;
            uint32_t smp, pass;
            if (fresh_item < pr.items && decode_item(pr, fresh_item, fresh_tile, x, j, smp, pass)) {
#ifdef TRAY_PROBE_REFILL
                TRAY_PROBE_F32(TRAY_PROBE_REFILL)
#endif
                // The pixel's primary-ray candidates, loaded before the camera ray is built.
                uint4 cand = make_uint4(0u, 0u, 0u, kCandOverflow << 16);
                if constexpr (kBVH)
                    if (pr.cand) cand = pr.cand[(size_t)j * (size_t)pr.width + (size_t)x];
                start_sample(pr, L, fresh_item, x, j, (pr.pass0 + pass) * (uint32_t)pr.spp + smp);
                L.slot = fresh_slot;
#ifdef TRAY_PROFILE_REFILL
                prof_cam = __builtin_amdgcn_s_memtime();
#endif
#ifdef TRAY_STATS_GROUND
                gcls = 0;
#endif
#ifdef TRAY_PROFILE_CANDWAIT
                {  // diagnostic: the candidate record's exposed latency after the camera ray
                    const uint64_t w0 = __builtin_amdgcn_s_memtime();
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                    prof_wait = __builtin_amdgcn_s_memtime() - w0 + 1u;
                }
#endif
                if constexpr (kBVH) {
                    TRAY_MARK("refill_cand")
                    ++L.segments;
                    T.tlim = __builtin_inff();
                    trav_globals(T, sv, L.org, L.dir);
                    if constexpr (kStats) st.spheres += (uint64_t)sv.n_global;
                    const uint32_t n_cand = cand.w >> 16;
                    if (n_cand <= kCandSlots) {
                        // Scene.Hit of a camera ray: the out-of-tree spheres and the pixel's
                        // candidates under the any-order rule (every other tree sphere is out
                        // of the ray's reach), no traversal.
                        uint64_t lo = ((uint64_t)cand.y << 32) | cand.x, hi = ((uint64_t)cand.w << 32) | cand.z;
#pragma unroll 1
                        for (uint32_t k = 0; k < n_cand; ++k) {
                            test_slot(T, sv, (int32_t)(lo & 0xFFFFu), L.org, L.dir);
                            lo = (lo >> 16) | (hi << 48);
                            hi >>= 16;
                        }
                        if constexpr (kStats) st.spheres += n_cand;
                        T.cur = kBvhNone;  // traversal done: the lane waits for the shade phase
                        cam_hit = true;
                    } else {
                        trav_begin32(T, sv, L.org, L.dir);
                    }
                }
#ifdef TRAY_PROFILE_REFILL
                prof_hit = __builtin_amdgcn_s_memtime();
#endif
            }
        }
#ifdef TRAY_PROFILE_REFILL
        const uint64_t prof_shade0 = __builtin_amdgcn_s_memtime();
#endif
        // The refill's camera rays with a known hit are shaded at once (their
        // scattered rays join the node steps below) instead of waiting for the
        // shade batch; the traversal lanes' batching is unchanged.
        if constexpr (kBVH) {
            if (__ballot(cam_hit) != 0ull) {
                TRAY_MARK("refill_shade")
                PROF_MATERIAL(0, cam_hit);
                bool ended = false;
                if (cam_hit) {
                    if (shade_step<kStats, kAcc>(kp_fresh(), L, T.slot, T.closest, T.a, [&] { return sv.bgeo[max(T.slot, 0)]; },
                                                 [&] { return sv.bmat[max(T.slot, 0)]; }, st, acc)) {
                        ++L.segments;
                        trav_begin(T, sv, L.org, L.dir);
                        if constexpr (kStats) st.spheres += (uint64_t)sv.n_global;
                    } else {
                        ended = true;
                    }
                }
                if constexpr (kProg) count_progress(p, ended, L.j, lane, prog_cur, prog_cnt);
            }
        }
#ifdef TRAY_PROFILE_REFILL
        {
            const uint64_t prof_shade1 = __builtin_amdgcn_s_memtime();
            PROF_CNT(10, prof_assigned - prof_t0_);  // item assignment (pool, queue)
            PROF_CNT(15, prof_shade1 - prof_shade0);  // shading of the candidate-answered camera rays
            const uint64_t mw = __ballot(prof_cam != 0u);
            if (mw != 0ull) {
                const uint32_t lw = (uint32_t)__builtin_ctzll(mw);
                const uint64_t c = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(prof_cam >> 32), lw) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((uint32_t)prof_cam, lw);
                const uint64_t h = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(prof_hit >> 32), lw) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((uint32_t)prof_hit, lw);
                PROF_CNT(13, c - prof_assigned);  // decoding + camera ray (draw block, discs)
                PROF_CNT(14, h - c);              // out-of-tree spheres + candidates (or the FP32 setup)
            }
        }
#endif
#ifdef TRAY_PROFILE_CANDWAIT
        {
            const uint64_t mw = __ballot(prof_wait != 0u);
            if (mw != 0ull) {
                const uint32_t lw = (uint32_t)__builtin_ctzll(mw);
                const uint64_t w = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(prof_wait >> 32), lw) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((uint32_t)prof_wait, lw);
                PROF_CNT(15, w - 1u);
            }
        }
#endif
        PROF_ADD(0);
        TRAY_MARK("refill_end")
#ifdef TRAY_PROFILE_TIMELINE
        tl_busy = (uint32_t)__popcll(__ballot(L.busy));
#endif
        if (__ballot(L.busy) == 0ull) {
            if (exhausted) break;
            continue;              // every lane drew a padding item: draw again
        }

        if constexpr (!kBVH) {
            bool ended = false;
            if (L.busy) {
                ++L.segments;
                double closest;
                const int best = scene_hit_linear<TRAY_UNROLL, kStats>(sv, L.org, L.dir, closest, st);
                ended = !shade_step<kStats, kAcc>(p, L, best, closest, length_sq(L.dir), [&] { return p.geo[max(best, 0)]; },  // NaN-padded: entry 0 exists
                                                  [&] { return best >= 0 ? p.mat[best] : MatRec{}; }, st, acc);
            }
            if constexpr (kProg) count_progress(p, ended, L.j, lane, prog_cur, prog_cnt);
        } else {
            if constexpr (kLDS == 1) {
                // The drain: a dry wave with at most coop_lanes paths finds their hits
                // with the whole wave (coop_hit; the node steps below then find none).
                if (exhausted) {
                    const KernelParams& pd = kp_fresh();
                    if (pd.coop_lanes != 0u && (uint32_t)__popcll(__ballot(L.busy)) <= pd.coop_lanes) {
                        PROF_T0();
                        uint64_t m = __ballot(L.busy && T.cur != kBvhNone);
                        while (m != 0ull) {
                            const uint32_t l = (uint32_t)__builtin_ctzll(m);
                            m &= m - 1ull;
                            coop_hit(T, sv, pd.n_slots, L.org, L.dir, l, lane);
                        }
                        PROF_ADD(1);
                    }
                }
            }
            // Node steps for the traversing lanes.
            {
                PROF_T0();
                TRAY_MARK("node_ctl")
                // Unrolled: the steps are straight-line code (no loop counter, and the
                // compiler schedules across them; C2 -0.9 %, C5 -0.8 % against a rolled loop).
#pragma unroll
                for (int s = 0; s < kSteps; ++s) {
                    const uint64_t m = __ballot(is_trav(T.cur));
                    if (m == 0ull) break;
                    if (s >= TRAY_NODE_STEPS && __popcll(m) < TRAY_NODE_MORE_LANES) break;
                    PROF_CNT(4, 1);
                    PROF_CNT(5, __popcll(m));
                    PROF_CNT(11, __popcll(__ballot(is_leaf(T.cur))));             // waiting for the leaf phase
                    PROF_CNT(12, __popcll(__ballot(L.busy && T.cur == kBvhNone)));  // waiting for the shade phase
                    if (is_trav(T.cur)) {
                        TRAY_MARK("node")
                        uint32_t tested;
#ifdef TRAY_PROBE_NODE
                        TRAY_PROBE_F32(TRAY_PROBE_NODE)
#endif
                        trav_node(T, sv, S, tested);
                        if constexpr (kStats) st.boxes += tested;
#if defined(TRAY_STATS_PRIMARY) && !defined(TRAY_PROFILE)
                        if constexpr (kStats) {
                            ++st.nodes;
                            if (L.bounce == 0) ++st.nodes0, st.boxes0 += tested;
                        }
#endif
#if defined(TRAY_STATS_GROUND) && !defined(TRAY_PROFILE)
                        if constexpr (kStats) {
                            ++st.nodes;
                            if (gcls == 1) ++st.g_nodes[0];
                            if (gcls != 0) ++st.g_nodes[1];
                        }
#endif
                    }
                }
                PROF_ADD(1);
                TRAY_MARK("leaf_decide")
            }
            // Leaf phase: FP64 sphere tests, batched.
            const uint64_t m_leaf = __ballot(is_leaf(T.cur));
            const uint32_t n_trav = (uint32_t)__popcll(__ballot(is_trav(T.cur)));
            if (m_leaf != 0ull && (__popcll(m_leaf) >= TRAY_LEAF_BATCH || n_trav == 0u ||
                                   (n_trav < TRAY_TRAV_SPARSE && __popcll(m_leaf) >= TRAY_LEAF_LOW))) {
                PROF_T0();
                TRAY_MARK("leaf_ctl")
                PROF_CNT(6, 1);
                PROF_CNT(7, __popcll(m_leaf));
                __builtin_amdgcn_s_setprio(1);
                if (is_leaf(T.cur)) {
                    TRAY_MARK("leaf")
                    uint32_t tested;
#ifdef TRAY_PROBE_LEAF
                    TRAY_PROBE_F32(TRAY_PROBE_LEAF)
#endif
                    trav_leaf(T, sv, S, L.org, L.dir, tested);
                    if constexpr (kStats) st.spheres += tested;
#if defined(TRAY_STATS_PRIMARY) && !defined(TRAY_PROFILE)
                    if constexpr (kStats) {
                        ++st.leaves;
                        if (L.bounce == 0) ++st.leaves0;
                    }
#endif
#if defined(TRAY_STATS_GROUND) && !defined(TRAY_PROFILE)
                    if constexpr (kStats) {
                        ++st.leaves;
                        if (gcls == 1) ++st.g_leaves[0];
                        if (gcls != 0) ++st.g_leaves[1];
                    }
#endif
                }
                PROF_ADD(2);
                __builtin_amdgcn_s_setprio(0);
            }
            // Shading phase, batched.
            const uint64_t m_shade = __ballot(L.busy && T.cur == kBvhNone);
            if (m_shade != 0ull && (__popcll(m_shade) >= TRAY_SHADE_BATCH || __ballot(T.cur < kBvhNone) == 0ull ||
                                    (__popcll(__ballot(is_trav(T.cur))) < TRAY_TRAV_SPARSE &&
                                     __popcll(m_shade) >= TRAY_SHADE_LOW))) {
                PROF_T0();
                TRAY_MARK("shade_ctl")
                PROF_CNT(8, 1);
                PROF_CNT(9, __popcll(m_shade));
                PROF_MATERIAL(1, L.busy && T.cur == kBvhNone);
                bool ended = false;
                if (L.busy && T.cur == kBvhNone) {
                    TRAY_MARK("shade")
#ifdef TRAY_PROBE_SHADE
                    TRAY_PROBE_F32(TRAY_PROBE_SHADE)
#endif
#ifdef TRAY_PROBE_SHADE64
                    TRAY_PROBE_F64(TRAY_PROBE_SHADE64)
#endif
                    if (shade_step<kStats, kAcc>(kp_fresh(), L, T.slot, T.closest, T.a, [&] { return sv.bgeo[max(T.slot, 0)]; },
                                                 [&] { return sv.bmat[max(T.slot, 0)]; }, st, acc)) {
                        ++L.segments;
#if defined(TRAY_STATS_GROUND) && !defined(TRAY_PROFILE)
                        {
                            const bool from_g = T.slot >= sv.global_first;
                            const bool up = L.dir.y >= __builtin_fmax(__builtin_fabs(L.dir.x), __builtin_fabs(L.dir.z));
                            gcls = from_g ? (up ? 1u : 2u) : 0u;
                            if constexpr (kStats) {
                                if (gcls == 1) ++st.g_seg[0];
                                if (gcls != 0) ++st.g_seg[1];
                            }
                        }
#endif
                        trav_begin(T, sv, L.org, L.dir);
                        if constexpr (kStats) st.spheres += (uint64_t)sv.n_global;
                    } else {
                        ended = true;  // idle: T.cur stays kBvhNone, L.busy is false
                    }
                }
                if constexpr (kProg) count_progress(p, ended, L.j, lane, prog_cur, prog_cnt);
                PROF_ADD(3);
                TRAY_MARK("shade_end")
            }
        }
    }
    if constexpr (kProg) flush_progress(kp_fresh(), prog_cur, prog_cnt, lane);
    if constexpr (kAcc)  // every lane is idle
        (void)acc_retire<kAcc>(kp_fresh(), acc, acc_all & ~acc_free, false, 0u, acc_chunk, lane);
    if constexpr (kStats) {
        // One atomic per wave: 3 per lane on three addresses serialised ~9 ms of tail
        // onto every instrumented launch (786 K device-scope atomics at C2).
        const uint64_t seg_w = wave_sum_u64(st.segments), sph_w = wave_sum_u64(st.spheres),
                       box_w = wave_sum_u64(st.boxes);
        if (lane == 0) {
            atomicAdd(p.stats + 0, (unsigned long long)seg_w);
            atomicAdd(p.stats + 1, (unsigned long long)sph_w);
            atomicAdd(p.stats + 2, (unsigned long long)box_w);
        }
#if defined(TRAY_STATS_PRIMARY) && !defined(TRAY_PROFILE)
        atomicAdd(p.stats + 3, (unsigned long long)st.nodes0);
        atomicAdd(p.stats + 4, (unsigned long long)st.leaves0);
        atomicAdd(p.stats + 5, (unsigned long long)st.boxes0);
        atomicAdd(p.stats + 6, (unsigned long long)st.nodes);
        atomicAdd(p.stats + 7, (unsigned long long)st.leaves);
#endif
#if defined(TRAY_STATS_GROUND) && !defined(TRAY_PROFILE)
        for (int k = 0; k < 2; ++k) {
            atomicAdd(p.stats + 3 + k, (unsigned long long)st.g_seg[k]);
            atomicAdd(p.stats + 5 + k, (unsigned long long)st.g_nodes[k]);
            atomicAdd(p.stats + 7 + k, (unsigned long long)st.g_leaves[k]);
        }
        atomicAdd(p.stats + 9, (unsigned long long)st.nodes);
        atomicAdd(p.stats + 10, (unsigned long long)st.leaves);
#endif
    }
#ifdef TRAY_PROFILE_TIMELINE
    if (kStats && lane == 0) {
        const uint64_t end = __builtin_amdgcn_s_memrealtime();
        const uint64_t mt_end = __builtin_amdgcn_s_memtime();
        tl_acc += (mt_end - tl_prev) * tl_busy;
        tl[kTlHdr + tl_bucket] = tl_acc;
        for (int k = 0; k < 4; ++k) tl[kTlHdr + kTlBuckets - 9 + k] = tl_ph[k];
        tl[0] = tl_start;
        tl[1] = end;
        tl[2] = tl_dry;
        tl[3] = tl_chunks;
        tl[4] = tl_mt0;
        tl[5] = mt_end;
    }
#endif
#ifdef TRAY_PROFILE
    if (kStats && lane == 0) {
        for (int i = 0; i < 16; ++i) atomicAdd(p.stats + 3 + i, (unsigned long long)prof[i]);
        // Wave lifetimes on the constant-rate clock: latest exit, sum of lifetimes, earliest start.
        const uint64_t end = __builtin_amdgcn_s_memrealtime();
        atomicMax(p.stats + 19, (unsigned long long)end);
        atomicAdd(p.stats + 20, (unsigned long long)(end - prof_start));
        atomicMax(p.stats + 21, (unsigned long long)~prof_start);
        // Per-wave (start, end) from stats[32] on (the buffer must hold 32 + 2 x waves).
        const uint32_t wave = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
        p.stats[32 + 2 * wave] = prof_start;
        p.stats[33 + 2 * wave] = end;
    }
#endif
}

// A band's pixels: the mean of each pixel's samples, added in sample order
// (colorSum and colorSumDiv of ray/tracer.go:123-150), written in the output
// format. One thread per pixel of the band's 8x8-tile order.
// It also re-zeroes the work queue for the next band or launch on the stream
// (the megakernel has finished with it), so no memset launch sits between
// consecutive frames.
// blockIdx.y is the pass within the launch.
// A pixel's mean written in the output format (compact pixel (x, j) of pass `pass`).
template <int kFmt>
__device__ __forceinline__ void write_acc_mean(const KernelParams& p, const double* srgb, const int64_t s[3],
                                               uint32_t bad, int32_t x, int32_t j, uint32_t pass) {
    const double unscale = __builtin_ldexp(1.0, -p.acc_shift);
    D3 sum;
    double* c = &sum.x;
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = (bad >> k) & 1u ? __builtin_nan("") : (double)s[k] * unscale;
    write_mean<kFmt>(p, srgb, sum, x, j, pass);
}
// One rounded sample or chunk sum into a pixel's integer total; a non-finite
// value (or, for a single sample, one beyond 2^kAccBits) flags the channel.
__device__ __forceinline__ void acc_add(double v, double limit, int64_t& s, uint32_t& bad, int k) {
    if (__builtin_fabs(v) <= limit) s += (int64_t)v;
    else bad |= 1u << k;
}

// Staged resolve (rays per pixel a multiple of 8): a wave's 64 pixels are
// consecutive work items, so their samples are one contiguous region of the
// sample buffer. The wave copies each 8-sample slab of its 64 pixels (64 x 192 B)
// into LDS with 16-byte loads that walk the region in address order (about 6
// pixels per load instruction instead of 64 lines, one per lane), then every
// lane adds its pixel's 8 samples from LDS in sample order.
constexpr int kStageStride = 25;  // doubles per pixel slab in LDS: 24 + 1 of padding (bank spread)

// kMode: 0 FP64 sum in sample order, 1 the same staged through LDS (8 | r),
// 2 fixed-point sums of the per-sample buffer, 3 fixed-point sums of the chunk
// partials (on-chip accumulation, 64 | r), 4 the fixed-point sums of 2 staged
// through LDS like 1 (8 | r: r = 16, 32 renders without on-chip slots).
enum : int { kResolveF64 = 0, kResolveStaged = 1, kResolveFixed = 2, kResolvePartials = 3, kResolveFixedStaged = 4 };
template <int kFmt, int kMode>
__global__ __launch_bounds__(256) void resolve_kernel(KernelParams p) {
    constexpr bool kStaged = kMode == kResolveStaged || kMode == kResolveFixedStaged;
    constexpr bool kFixedStaged = kMode == kResolveFixedStaged;
    __shared__ double srgb[256];
    if constexpr (kFmt == kOutRGBA8) {  // the encoder table, one entry per thread
        srgb[threadIdx.x] = p.srgb[threadIdx.x];
        __syncthreads();
    }
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q == 0 && blockIdx.y == 0) *p.queue = 0u;
    const uint32_t npix = p.frame_items / (uint32_t)p.spp;  // a multiple of 64: waves are whole
    if (q >= npix) return;
    const uint32_t item0 = (q * p.passes + blockIdx.y) * (uint32_t)p.spp;
    const uint32_t pix_stride = p.passes * (uint32_t)p.spp;  // items between consecutive pixels of a pass
    int32_t x, j;
    uint32_t s0, pass;
    // A wave's 64 pixels are one tile of the item order (q >> 6): one work-order lookup.
    const uint32_t tile = p.tile_order ? __builtin_amdgcn_readfirstlane(p.tile_order[q >> 6]) : 0u;
    const bool valid = decode_item(p, item0, tile, x, j, s0, pass);
    D3 sum = d3(0, 0, 0);
    if constexpr (kMode == kResolvePartials) {
        // One record per 64 items (64 | r: r / 64 per pixel-pass) or per pixel-pass (r | 64).
        const AccPartial* part = reinterpret_cast<const AccPartial*>(p.samples) + (item0 >> p.acc_rshift);
        if (p.tile_cost) {  // a counting launch: the tile's Scene.Hit calls for the next work order
            uint64_t n = 0;
            if (valid)
                for (int32_t c = 0; c < (p.spp >> p.acc_rshift); ++c) n += (uint64_t)part[c].pad;
            n = wave_sum_u64(n);
            if ((threadIdx.x & 63u) == 0u)
                atomicAdd(p.tile_cost + (p.tile_order ? tile : q >> 6), (uint32_t)min<uint64_t>(n, 0xFFFFFFFFull));
        }
        if (!valid) return;
        int64_t s[3] = {0, 0, 0};
        uint32_t bad = 0u;
        for (int32_t c = 0; c < (p.spp >> p.acc_rshift); ++c)
#pragma unroll
            for (int k = 0; k < 3; ++k) acc_add(part[c].sum[k], 0x1p53, s[k], bad, k);
        write_acc_mean<kFmt>(p, srgb, s, bad, x, j, pass);
        return;
    } else if constexpr (kMode == kResolveFixed) {
        if (!valid) return;
        const double* smp = p.samples + (size_t)item0 * 3;
        int64_t s[3] = {0, 0, 0};
        uint32_t bad = 0u;
        for (int32_t k = 0; k < p.spp; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) acc_add(__builtin_rint(smp[3 * k + c]), 0x1p47, s[c], bad, c);
        write_acc_mean<kFmt>(p, srgb, s, bad, x, j, pass);
        return;
    } else if constexpr (kStaged) {
        __shared__ double stage[4][64 * kStageStride];
        const uint32_t lane = threadIdx.x & 63u;
        double* st = stage[threadIdx.x >> 6];
        const uint32_t q0 = q - lane;  // the wave's first pixel
        const double* base = p.samples + ((size_t)q0 * pix_stride + (size_t)blockIdx.y * (uint32_t)p.spp) * 3;
        int64_t si[3] = {0, 0, 0};  // kFixedStaged: the pixel's integer totals
        uint32_t bad = 0u;
        for (int32_t s = 0; s < p.spp; s += 8) {
#pragma unroll
            for (int k = 0; k < 12; ++k) {  // 768 16-B pieces: pixel t / 12, piece t % 12 of its 192-B slab
                const uint32_t t = (uint32_t)k * 64u + lane;
                const uint32_t i = t / 12u, c = t - i * 12u;
                const double2 v = *reinterpret_cast<const double2*>(base + ((size_t)i * pix_stride + s) * 3 + 2 * c);
                st[i * kStageStride + 2 * c] = v.x;
                st[i * kStageStride + 2 * c + 1] = v.y;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double* mine = st + lane * kStageStride;
            if constexpr (kFixedStaged) {
#pragma unroll
                for (int k = 0; k < 24; ++k) acc_add(__builtin_rint(mine[k]), 0x1p47, si[k % 3], bad, k % 3);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) sum = add(sum, d3(mine[3 * k], mine[3 * k + 1], mine[3 * k + 2]));
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();  // every lane has read the slab before it is overwritten
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if constexpr (kFixedStaged) {
            if (valid) write_acc_mean<kFmt>(p, srgb, si, bad, x, j, pass);
            return;
        }
    } else {
        if (!valid) return;
        const double* smp = p.samples + (size_t)item0 * 3;
        // Loads of 8 samples are issued together; the adds stay in sample order.
        int32_t s = 0;
        for (; s + 8 <= p.spp; s += 8) {
            double v[24];
#pragma unroll
            for (int k = 0; k < 24; ++k) v[k] = smp[3 * s + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) sum = add(sum, d3(v[3 * k], v[3 * k + 1], v[3 * k + 2]));
        }
        for (; s < p.spp; ++s) sum = add(sum, d3(smp[3 * s], smp[3 * s + 1], smp[3 * s + 2]));
    }
    if (valid) write_mean<kFmt>(p, srgb, sum, x, j, pass);
}

// Primary-ray candidates (launch_cand_build). A camera ray of pixel (x, y)
// (get_ray) runs from a lens point o = pos + du dx + dv dy, |(dx, dy)| <= 1, through
// F = pos + (S - pos) ft (aperture > 0; F = S otherwise), S = p00 + px (x + ox) +
// py (y + oy), |(ox, oy)| <= ray_radius (when r > 1). With A0 = pos, B0 = the
// disc centre's F and D = B0 - A0, the ray's point at parameter t is
// (1 - t) o + t F, within w(t) = |1 - t| rA + t rB of the axis point A0 + t D
// (rA, rB: the two disc radii). A sphere (C, R) the ray enters at t >= 0
// therefore satisfies |A0 + t D - C| <= R + w(t). With tc = the axis parameter
// closest to C (clamped to t >= 0), d_perp = C's distance from the axis line and
// L = rA + rB (w's slope bound): |t - tc| |D| <= R + w(tc) + L |t - tc| gives
// |t - tc| <= (R + w(tc)) / (|D| - L), hence the necessary condition
// d_perp <= R + w(tc) + L (R + w(tc)) / (|D| - L). The margin covers the FP64
// rounding of both this bound and the kernel's ray (orders of magnitude
// above it). Spheres outside the tree (kBvhGlobals) are tested for every ray
// anyway and are not listed.
// The beam test of one sphere against an axis pos + t D (|D|^2 = dn2) with
// disc radii ra (lens) and rb (far disc): false only when no ray of the beam
// can reach the sphere (comment above).
__device__ __forceinline__ bool beam_reaches(const D3& pos, const D3& D, double dn2, double dn, double ra, double rb,
                                             double scale, double4 g, double R) {
    const double L = ra + rb;
    const D3 rel = sub(d3(g.x, g.y, g.z), pos);
    const double tc = dot(rel, D) / dn2;
    const double tcl = __builtin_fmax(tc, 0.0);
    const double dperp = __builtin_sqrt(length_sq(sub(rel, smul(D, tc))));
    const double margin = 1e-6 * (scale + __builtin_fabs(g.x) + __builtin_fabs(g.y) + __builtin_fabs(g.z) + R);
    const double reach = R + __builtin_fabs(1.0 - tcl) * ra + tcl * rb + margin;
    return dperp <= reach + L * reach / (dn - L) + margin || !(dperp == dperp);
}

// The beam of a rectangle of pixels: columns [xa, xb], image rows [ya, yb] (one
// pixel: xa = xb, ya = yb). Its far disc is centred on the rectangle's centre
// and grown by the rectangle's half extent, so it contains every pixel's disc.
struct Beam {
    D3 pos, D;
    double dn2, dn, ra, rb, scale;
    bool ok;  // false: degenerate (the axis is not longer than twice the disc radii)
};
__device__ __forceinline__ Beam pixel_beam(const KernelParams& p, double xa, double xb, double ya, double yb) {
    Beam b;
    b.pos = d3(p.cam.position[0], p.cam.position[1], p.cam.position[2]);
    const D3 p00 = d3(p.cam.pixel00[0], p.cam.pixel00[1], p.cam.pixel00[2]);
    const D3 pxv = d3(p.cam.pixel_x[0], p.cam.pixel_x[1], p.cam.pixel_x[2]);
    const D3 pyv = d3(p.cam.pixel_y[0], p.cam.pixel_y[1], p.cam.pixel_y[2]);
    const D3 du = d3(p.cam.defocus_u[0], p.cam.defocus_u[1], p.cam.defocus_u[2]);
    const D3 dv = d3(p.cam.defocus_v[0], p.cam.defocus_v[1], p.cam.defocus_v[2]);
    const bool lens = p.cam.aperture > 0;
    const D3 s0 = add(add(p00, smul(pxv, 0.5 * (xa + xb))), smul(pyv, 0.5 * (ya + yb)));
    const D3 b0 = lens ? add(b.pos, smul(sub(s0, b.pos), p.focus_time)) : s0;
    const double lx = __builtin_sqrt(length_sq(pxv)), ly = __builtin_sqrt(length_sq(pyv));
    // |RayRadius|: Go's RenderLines accepts a negative radius and InDisc(r) is
    // symmetric (disc() scales by the signed r), so the disc's extent is |r|.
    const double aa = (p.spp > 1 ? __builtin_fabs(p.ray_radius) * __builtin_sqrt(lx * lx + ly * ly) : 0.0) +
                      0.5 * (xb - xa) * lx + 0.5 * (yb - ya) * ly;
    b.ra = lens ? __builtin_sqrt(length_sq(du) + length_sq(dv)) : 0.0;
    b.rb = lens ? aa * __builtin_fabs(p.focus_time) : aa;
    b.D = sub(b0, b.pos);
    b.dn2 = length_sq(b.D);
    b.dn = __builtin_sqrt(b.dn2);
    b.ok = b.dn > 2.0 * (b.ra + b.rb) && b.dn2 > 0;
    b.scale = 1.0 + __builtin_fmax(__builtin_fmax(__builtin_fabs(b.pos.x), __builtin_fabs(b.pos.y)), __builtin_fabs(b.pos.z));
    return b;
}

// Pass 1: one wave per 8x8 tile of compact pixels tests every tree sphere
// (lane k: spheres k, k + 64, ...) against the tile's beam and keeps up to
// kCandTileSlots of them in sphere order (else overflow: the tile's pixels test
// every tree sphere).
__global__ __launch_bounds__(256) void cand_tile_kernel(KernelParams p, uint16_t* lists, uint32_t* counts) {
    const uint32_t tiles_x = ((uint32_t)p.width + 7u) / 8u, tiles_y = ((uint32_t)p.rows + 7u) / 8u;
    const uint32_t t = blockIdx.x * 4u + threadIdx.x / 64u, lane = threadIdx.x & 63u;
    if (t >= tiles_x * tiles_y) return;  // wave-uniform
    const int32_t xa = (int32_t)(t % tiles_x) * 8, ja = (int32_t)(t / tiles_x) * 8;
    const int32_t xb = min(xa + 7, p.width - 1), jb = min(ja + 7, p.rows - 1);
    const Beam b = pixel_beam(p, (double)xa, (double)xb, (double)row_of(p, ja), (double)row_of(p, jb));
    uint32_t n = 0;
    const int32_t tree = p.n_slots - p.n_global;
    for (int32_t s0 = 0; s0 < tree && b.ok && n <= kCandTileSlots; s0 += 64) {
        const int32_t s = s0 + (int32_t)lane;
        const bool hit = s < tree && beam_reaches(b.pos, b.D, b.dn2, b.dn, b.ra, b.rb, b.scale, p.bgeo[s],
                                                   __builtin_fabs(p.bmat[s].radius));
        const uint64_t m = __ballot(hit);
        const uint32_t at = n + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (hit && at < kCandTileSlots) lists[(size_t)t * kCandTileSlots + at] = (uint16_t)s;
        n += (uint32_t)__popcll(m);
    }
    if (lane == 0) counts[t] = b.ok && n <= kCandTileSlots ? n : kCandOverflow;
}

// Pass 2: one thread per compact pixel tests its tile's spheres (all tree
// spheres when the tile overflowed) against the pixel's own beam.
__global__ __launch_bounds__(256) void cand_build_kernel(KernelParams p, uint4* out, const uint16_t* lists,
                                                        const uint32_t* counts) {
    const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= (size_t)p.rows * (size_t)p.width) return;
    const int32_t j = (int32_t)(i / (size_t)p.width), x = (int32_t)(i % (size_t)p.width);
    const double y = (double)row_of(p, j);
    const Beam b = pixel_beam(p, (double)x, (double)x, y, y);
    const uint32_t tile = (uint32_t)(j / 8) * (((uint32_t)p.width + 7u) / 8u) + (uint32_t)(x / 8);
    const uint32_t tn = counts[tile];
    const bool all = tn == kCandOverflow;
    const int32_t m = all ? p.n_slots - p.n_global : (int32_t)tn;
    uint32_t slots[kCandSlots];
    uint32_t n = 0;
    bool ok = b.ok;
    for (int32_t k = 0; k < m && ok; ++k) {
        const int32_t s = all ? k : (int32_t)lists[(size_t)tile * kCandTileSlots + k];
        if (beam_reaches(b.pos, b.D, b.dn2, b.dn, b.ra, b.rb, b.scale, p.bgeo[s], __builtin_fabs(p.bmat[s].radius))) {
            if (n == kCandSlots) ok = false;
            else slots[n++] = (uint32_t)s;
        }
    }
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (ok) {
#pragma unroll
        for (uint32_t k = 0; k < kCandSlots; ++k)
            if (k < n) w[k >> 1] |= slots[k] << (16u * (k & 1u));
    }
    w[3] = (w[3] & 0xFFFFu) | ((ok ? n : kCandOverflow) << 16);
    out[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

size_t cand_workspace_bytes(int32_t width, int32_t rows) {
    const size_t pixels = (size_t)rows * (size_t)width;
    const size_t tiles = (size_t)((width + 7) / 8) * (size_t)((rows + 7) / 8);
    return pixels * sizeof(uint4) + tiles * (kCandTileSlots * sizeof(uint16_t) + sizeof(uint32_t));
}

hipError_t launch_cand_build(const KernelParams& kp, uint4* out, hipStream_t stream) {
    KernelParams p = kp;
    p.div_tile_rows = make_fastdiv((uint32_t)std::max(p.tile_rows, 1));  // row_of
    const size_t n = (size_t)p.rows * (size_t)p.width;
    if (n == 0) return hipSuccess;
    const size_t tiles = (size_t)((p.width + 7) / 8) * (size_t)((p.rows + 7) / 8);
    uint16_t* lists = reinterpret_cast<uint16_t*>(out + n);
    uint32_t* counts = reinterpret_cast<uint32_t*>(lists + tiles * kCandTileSlots);
    hipLaunchKernelGGL(cand_tile_kernel, dim3((uint32_t)((tiles + 3) / 4)), dim3(256), 0, stream, p, lists, counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(cand_build_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, p, out, lists,
                       counts);
    return hipGetLastError();
}

// ColorF.ToSRGBA over a device buffer of linear colours (tray_linear_to_srgba_async).
__global__ __launch_bounds__(256) void to_srgba_kernel(const double* rgb, size_t n, uint32_t* rgba,
                                                      const double* table) {
    __shared__ double srgb[256];
    srgb[threadIdx.x] = table[threadIdx.x];
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u)
        rgba[i] = srgba_word(srgb, rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
}

hipError_t launch_to_srgba(const double* rgb, size_t n_pixels, uint32_t* rgba, const double* srgb,
                           hipStream_t stream) {
    if (n_pixels == 0) return hipSuccess;
    const size_t blocks = std::min<size_t>((n_pixels + 255) / 256, 4096);
    hipLaunchKernelGGL(to_srgba_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, rgb, n_pixels, rgba, srgb);
    return hipGetLastError();
}

using KernelFn = void (*)(KernelParams);

template <bool kBVH, bool kSpill, bool kStats, bool kProg, int kAcc, int kSteps>
static KernelFn pick_kernel4(int lds_mode) {
    if constexpr (kAcc == 2) {  // pixel-pass groups: only with the whole scene in LDS (launch_layout)
        (void)lds_mode;
        return render_kernel<1, kBVH, kStats, kSpill, kProg, kAcc, kSteps>;
    } else {
        if (lds_mode == 1) return render_kernel<1, kBVH, kStats, kSpill, kProg, kAcc, kSteps>;
        if constexpr (kBVH)
            if (lds_mode == 2) return render_kernel<2, kBVH, kStats, kSpill, kProg, kAcc, kSteps>;
        return render_kernel<0, kBVH, kStats, kSpill, kProg, kAcc, kSteps>;
    }
}
template <bool kBVH, bool kSpill, bool kStats, bool kProg, int kAcc>
static KernelFn pick_kernel3(int lds_mode, bool deep) {
    if constexpr (kBVH && !kSpill && kAcc != 2)
        if (deep) return pick_kernel4<kBVH, kSpill, kStats, kProg, kAcc, kDeepSteps>(lds_mode);
    return pick_kernel4<kBVH, kSpill, kStats, kProg, kAcc, TRAY_NODE_STEPS_MAX>(lds_mode);
}

// Instrumentation: the stats instance counts segments and tests; the progress
// instance feeds tray_render_progress; neither is ever timed by the bench.
template <bool kBVH, bool kSpill, int kAcc>
static KernelFn pick_kernel2(int lds_mode, bool stats, bool progress, bool deep) {
    if (stats) return pick_kernel3<kBVH, kSpill, true, false, kAcc>(lds_mode, deep);
    if (progress) return pick_kernel3<kBVH, kSpill, false, true, kAcc>(lds_mode, deep);
    return pick_kernel3<kBVH, kSpill, false, false, kAcc>(lds_mode, deep);
}

// The next launch's work order from a counting launch's tile costs (one
// workgroup; launch_render runs it after a band's resolve): the band's tiles by
// decreasing Scene.Hit calls, a counting sort over 256 logarithmic buckets (12
// per octave), so a launch hands out its most expensive tiles first and ends on
// cheap ones. A tile's longest paths (50 segments at C2) then start early instead
// of holding the last waves of the grid alone ("Work order"). The
// order inside a bucket is whatever the LDS atomics give: it changes the
// schedule, never a pixel (every pixel's sum is order-free). Zeroes the costs.
__device__ __forceinline__ uint32_t cost_bucket(uint32_t c) {
    return c == 0u ? 0u : min(255u, 1u + (uint32_t)(__builtin_log2f((float)c) * 12.0f));
}
__global__ __launch_bounds__(1024) void tile_order_kernel(uint32_t* cost, uint32_t* order, uint32_t n) {
    __shared__ uint32_t slot[256];
    for (uint32_t b = threadIdx.x; b < 256u; b += blockDim.x) slot[b] = 0u;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) atomicAdd(&slot[cost_bucket(cost[t])], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive prefix over the buckets, most expensive first
        uint32_t run = 0u;
        for (int b = 255; b >= 0; --b) {
            const uint32_t c = slot[b];
            slot[b] = run;
            run += c;
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
        order[atomicAdd(&slot[cost_bucket(cost[t])], 1u)] = t;
        cost[t] = 0u;
    }
}

// On-chip accumulation is built for the BVH kernel with the whole stack on
// chip (launch_layout grants accumulators only then); every other launch sums
// through the per-sample buffer.
static KernelFn pick_kernel(int lds_mode, bool bvh, bool stats, bool progress, bool spill, int acc, bool deep) {
    if (!bvh) return pick_kernel2<false, false, 0>(lds_mode, stats, progress, false);
    if (spill) return pick_kernel2<true, true, 0>(lds_mode, stats, progress, false);
    if (acc == 2) return pick_kernel2<true, false, 2>(lds_mode, stats, progress, false);
    return acc == 1 ? pick_kernel2<true, false, 1>(lds_mode, stats, progress, deep)
                    : pick_kernel2<true, false, 0>(lds_mode, stats, progress, deep);
}

template <int kMode>
static KernelFn pick_resolve2(int fmt) {
    if (fmt == kOutRGBF64) return resolve_kernel<kOutRGBF64, kMode>;
    if (fmt == kOutRGBF32) return resolve_kernel<kOutRGBF32, kMode>;
    return resolve_kernel<kOutRGBA8, kMode>;
}

// The staged resolve needs 8 | rays per pixel (whole 8-sample slabs).
static KernelFn pick_resolve(const KernelParams& p) {
    bool staged = p.spp % 8 == 0;
    long long v = 1;
    if (debug_knob(kKnobResolveStaged, &v)) staged = staged && v != 0;  // A/B
    if (p.acc_shift > 0) {
        if (p.acc_slots > 0) return pick_resolve2<kResolvePartials>(p.out_format);
        return staged ? pick_resolve2<kResolveFixedStaged>(p.out_format) : pick_resolve2<kResolveFixed>(p.out_format);
    }
    return staged ? pick_resolve2<kResolveStaged>(p.out_format) : pick_resolve2<kResolveF64>(p.out_format);
}

// Blocks the device keeps resident for this kernel and LDS size (persistent grid cap).
static int resident_blocks(int device, KernelFn fn, int threads, size_t lds) {
    hipDeviceProp_t prop;
    int cus = 256;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), threads, lds) !=
            hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    return cus * per_cu;
}

// Scene bytes staged in LDS (nodes, geometry, indices, leaf table), 16-B aligned.
static size_t scene_lds_bytes(int32_t n_nodes, int32_t n_slots, int32_t n_leaves) {
    const size_t b = (size_t)n_nodes * sizeof(Bvh4Node) + (size_t)n_slots * (sizeof(double4) + sizeof(int32_t)) +
                     (size_t)n_leaves * sizeof(int32_t);
    return (b + 15) / 16 * 16;
}

// The nodes-only layout (kLDS 2): nodes and leaf table.
static size_t nodes_lds_bytes(int32_t n_nodes, int32_t n_leaves) {
    return ((size_t)n_nodes * sizeof(Bvh4Node) + (size_t)n_leaves * sizeof(int32_t) + 15) / 16 * 16;
}

size_t bvh_scene_lds_bytes(int32_t n_nodes, int32_t n_slots, int32_t n_leaves, int32_t stack_cap) {
    return kUniformsBytes + bvh_stack_bytes(std::min(stack_cap, kStackLdsMin)) +
           scene_lds_bytes(n_nodes, n_slots, n_leaves);
}

// Ranked: whole scene and whole stack on chip (4) > nodes and whole stack (3) >
// whole scene, stack overflowing to global memory (2) > nodes, stack overflowing
// (1) > scene in global memory (0). A stack overflow costs more than reading
// sphere geometry from L2 (C5, 1,939 spheres: 4-sphere leaves, nodes-only with
// the whole stack on chip 6592 Mrays/s vs whole scene with overflow 6313).
LdsPlan bvh_lds_plan(int32_t n_nodes, int32_t n_slots, int32_t n_leaves, int32_t stack_cap) {
    const size_t room = kMaxLDSBytes - kUniformsBytes;
    const size_t all = scene_lds_bytes(n_nodes, n_slots, n_leaves), nodes = nodes_lds_bytes(n_nodes, n_leaves);
    const size_t full = bvh_stack_bytes(stack_cap), least = bvh_stack_bytes(std::min(stack_cap, kStackLdsMin));
    if (all + full <= room) return {1, 4};
    if (nodes + full <= room) return {2, 3};
    if (all + least <= room) return {1, 2};
    if (nodes + least <= room) return {2, 1};
    return {0, 0};
}

size_t bvh_stack_overflow_bytes(int32_t stack_cap, int device) {
    if (stack_cap <= kStackLdsMin) return 0;
    hipDeviceProp_t prop;
    size_t lanes = (size_t)256 * 2048;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess)
        lanes = (size_t)prop.multiProcessorCount * (size_t)prop.maxThreadsPerMultiProcessor;
    return (size_t)(stack_cap - kStackLdsMin) * lanes * sizeof(uint32_t);
}

uint64_t max_band_samples(bool partials) {
    const uint64_t limit = partials ? kMaxBandSamplesAcc : kMaxBandSamples;
    long long v = 0;
    if (debug_knob(kKnobBandSamples, &v) && v > 0 && (uint64_t)v < limit) return (uint64_t)v;
    return limit;
}

// Bands of 8-row tile rows, each <= max_band_samples(partials) samples over all of
// the launch's passes (at least one tile row). `spp` below counts the samples of a
// pixel in one launch: rays_per_pixel x passes. Fewer bands, fewer tails: C5's
// 16-frame launch is 4 bands instead of 8 with chunk records.
static int32_t band_tile_rows(int32_t width, uint64_t spp, bool partials) {
    const uint64_t per = (uint64_t)((width + 7) / 8) * 64u * spp;
    return (int32_t)std::max<uint64_t>(1, max_band_samples(partials) / per);
}

// Bytes of the buffer one band of `band_tiles` tile rows needs: a colour per sample, or
// one chunk record per 2^rshift samples (partials).
static size_t band_buffer_bytes(int32_t width, int32_t rows, uint64_t spp, bool partials, int32_t band_tiles,
                                uint32_t rshift = 6) {
    if (rows <= 0) return 0;
    const int32_t tile_rows = std::min(band_tiles, (rows + 7) / 8);
    const size_t samples = (size_t)((width + 7) / 8) * 64u * (size_t)tile_rows * (size_t)spp;
    return partials ? (samples >> rshift) * sizeof(AccPartial) : samples * 3 * sizeof(double);
}

size_t sample_buffer_bytes(int32_t width, int32_t rows, uint64_t spp) {
    return band_buffer_bytes(width, rows, spp, false, band_tile_rows(width, spp, false));
}

size_t accum_buffer_bytes(int32_t width, int32_t rows, uint64_t spp, bool partials, uint32_t rshift) {
    return band_buffer_bytes(width, rows, spp, partials, band_tile_rows(width, spp, partials), rshift);
}

LaunchLayout launch_layout(const KernelParams& p, bool use_bvh) {
    LaunchLayout L{0, 0, 0, 0, 0, 6u};
    if (use_bvh) {
        // Whole scene in LDS when it fits next to kStackLdsMin stack slots, else
        // the nodes and leaf table when they fit, else nothing; the stack then
        // takes what LDS is left (up to its bound), the rest spills.
        L.lds_mode = bvh_lds_plan(p.n_nodes, p.n_slots, p.n_leaves, p.stack_cap).mode;
        long long knob = 0;
        if (debug_knob(kKnobBvhLdsMode, &knob)) {  // tests / A-B: force a layout that fits
            const int want = (int)knob;
            if (want == 0 || (want == 2 && L.lds_mode != 0) ||
                (want == 1 && bvh_scene_lds_bytes(p.n_nodes, p.n_slots, p.n_leaves, p.stack_cap) <= kMaxLDSBytes))
                L.lds_mode = want;
        }
        const size_t scene = L.lds_mode == 1   ? scene_lds_bytes(p.n_nodes, p.n_slots, p.n_leaves)
                             : L.lds_mode == 2 ? nodes_lds_bytes(p.n_nodes, p.n_leaves)
                                               : 0;
        const size_t room = kMaxLDSBytes - kUniformsBytes - scene;
        L.stack_lds = std::min<int32_t>(p.stack_cap, (int32_t)(room / kStackSlotBytes));
        if (debug_knob(kKnobStackLdsSlots, &knob))  // tests: force the overflow path
            L.stack_lds = std::min(L.stack_lds, (int32_t)std::max<long long>(kStackLdsMin, std::min<long long>(knob, 1 << 20)));
        L.lds = kUniformsBytes + bvh_stack_bytes(L.stack_lds) + scene;
        // Chunk accumulators in what the whole stack leaves (fixed-point frames only).
        if (p.acc_shift > 0 && L.stack_lds == p.stack_cap && acc_groupable(p.spp) &&
            (acc_record_shift(p.spp) == 6u || L.lds_mode == 1)) {  // groups: one kernel instance (scene in LDS)
            const uint32_t rshift = acc_record_shift(p.spp);
            const size_t waves = (size_t)kBvhBlock / 64u;
            // every group of a chunk, and the chunk's Scene.Hit count (work order)
            const size_t per_slot = waves * (kAccSlotBytes * (64u >> rshift) + kAccCountBytes);
            const size_t left = kMaxLDSBytes - L.lds;
            int32_t slots = (int32_t)std::min<size_t>(kAccSlotsMax, left / per_slot);
            const bool forced = debug_knob(kKnobAccSlots, &knob);  // tests / A-B: fewer slots, 0 = off
            if (forced) slots = (int32_t)std::min<long long>(slots, std::max(0LL, knob));
            if (slots >= kAccSlotsMin || (slots > 0 && forced)) {
                L.acc_slots = slots;
                L.acc_off = (uint32_t)L.lds;
                L.acc_rshift = rshift;
                L.lds += (size_t)slots * per_slot;
            }
        }
    } else {
        const size_t geo = (size_t)p.n_pad * sizeof(double4);
        L.lds_mode = geo + kUniformsBytes <= kMaxLDSBytes ? 1 : 0;
        L.lds = kUniformsBytes + (L.lds_mode ? geo : 0);
    }
    return L;
}

bool band_fits(int32_t width, uint64_t spp) {
    return (uint64_t)((width + 7) / 8) * 64u * spp <= 0x7FFFFFFFull;
}

LaunchPlan plan_launch(const KernelParams& p, bool use_bvh) {
    LaunchPlan L;
    L.layout = launch_layout(p, use_bvh);
    const uint64_t spp_launch = (uint64_t)p.spp * std::max<uint32_t>(p.passes, 1u);
    const bool partials = L.layout.acc_slots > 0;
    L.band_tiles = band_tile_rows(p.width, spp_launch, partials);
    L.buffer_bytes = band_buffer_bytes(p.width, p.rows, spp_launch, partials, L.band_tiles, L.layout.acc_rshift);
    return L;
}

hipError_t launch_render(KernelParams p, bool use_bvh, const LaunchPlan& plan, hipStream_t stream,
                         size_t samples_bytes, uint32_t* order_out) {
    if (p.rows <= 0) return hipSuccess;
    if (p.passes < 1) p.passes = 1;
    const uint64_t spp_launch = (uint64_t)p.spp * p.passes;
    if (!band_fits(p.width, spp_launch)) return hipErrorInvalidValue;
    if (p.segments && p.passes > 1) return hipErrorInvalidValue;
    p.tiles_x = (p.width + 7) / 8;
    p.div_spp = make_fastdiv((uint32_t)p.spp);
    p.div_tiles_x = make_fastdiv((uint32_t)p.tiles_x);
    p.div_tile_rows = make_fastdiv((uint32_t)std::max(p.tile_rows, 1));
    p.div_chunks_per_tile = make_fastdiv((uint32_t)spp_launch);  // a tile: 64 pixels x r x passes items
    if (p.tile_cost && (!order_out || plan.layout.acc_slots <= 0)) return hipErrorInvalidValue;  // counting needs both
    const uint32_t* order_base = p.tile_order;
    uint32_t* cost_base = p.tile_cost;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (p.acc_shift > 0 && !acc_groupable(p.spp)) return hipErrorInvalidValue;  // the caller decides (fixed_point_shift)
    const LaunchLayout& layout = plan.layout;
    const int lds_mode = layout.lds_mode;
    const size_t lds = layout.lds;
    p.stack_lds = layout.stack_lds;
    p.acc_slots = layout.acc_slots;
    p.acc_off = layout.acc_off;
    p.acc_rshift = layout.acc_rshift;
    if (use_bvh && p.stack_cap > p.stack_lds && !p.stack_ovf) return hipErrorInvalidValue;
    // The caller sized p.samples from this plan (an invariant: the plan is decided once).
    const int32_t band_tiles = plan.band_tiles;
    if (plan.buffer_bytes > samples_bytes) return hipErrorInvalidValue;
    const int threads = use_bvh ? kBvhBlock : 256;
    const bool stats = p.stats != nullptr;
    bool deep = use_bvh && p.n_nodes > kDeepNodes;
    long long knob = 0;
    if (debug_knob(kKnobNodeDeep, &knob))  // A/B: force the instance
        deep = use_bvh && knob != 0;
    const KernelFn fn = pick_kernel(lds_mode, use_bvh, stats, p.progress != nullptr,
                                    use_bvh && p.stack_cap > p.stack_lds,
                                    p.acc_slots <= 0 ? 0 : p.acc_rshift < 6u ? 2 : 1, deep);
    const KernelFn resolve = pick_resolve(p);
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
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kMaxLDSBytes);
        if (e != hipSuccess) return e;
        blocks = resident_blocks(dev, fn, threads, lds);
        cache[cache_next] = Setup{dev, fn, lds, blocks};
        cache_next = (cache_next + 1) % 8;
    }
    if (stats) {
#ifdef TRAY_PROFILE
        e = hipMemsetAsync(p.stats, 0, 19 * sizeof(unsigned long long), stream);
#elif defined(TRAY_STATS_PRIMARY)
        e = hipMemsetAsync(p.stats, 0, 8 * sizeof(unsigned long long), stream);
#elif defined(TRAY_STATS_GROUND)
        e = hipMemsetAsync(p.stats, 0, 11 * sizeof(unsigned long long), stream);
#else
        e = hipMemsetAsync(p.stats, 0, 3 * sizeof(unsigned long long), stream);
#endif
        if (e != hipSuccess) return e;
    }
    if (p.segments) {  // summed per path with atomics
        e = hipMemsetAsync(p.segments, 0, (size_t)p.rows * (size_t)p.width * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
    }
    long long reserve_knob = 0;
    (void)debug_knob(kKnobGridReserve, &reserve_knob);
    const int reserve = (int)std::min<long long>(std::max<long long>(reserve_knob, 0), blocks - 1);
    long long wave_chunks_knob = 0;
    (void)debug_knob(kKnobWaveChunks, &wave_chunks_knob);
    wave_chunks_knob = std::min<long long>(std::max<long long>(wave_chunks_knob, 0), 64);
    const int32_t band = band_tiles * 8;
    const uint32_t waves = (uint32_t)threads / 64u;
    for (int32_t j0 = 0; j0 < p.rows; j0 += band) {
        p.j0 = j0;
        p.band_rows = std::min(band, p.rows - j0);
        const size_t tile_off = (size_t)(j0 / 8) * (size_t)p.tiles_x;  // the band's tiles in the launch's numbering
        const uint32_t band_tiles_n = (uint32_t)p.tiles_x * (uint32_t)((p.band_rows + 7) / 8);
        p.tile_order = order_base ? order_base + tile_off : nullptr;
        p.tile_cost = cost_base ? cost_base + tile_off : nullptr;
        const uint32_t pixels = (uint32_t)p.tiles_x * (uint32_t)((p.band_rows + 7) / 8) * 64u;
        p.frame_items = pixels * (uint32_t)p.spp;
        p.div_passes = make_fastdiv(p.passes);
        p.items = p.frame_items * p.passes;
        p.nchunks = (p.items + 63u) / 64u;
        p.pool_chunks = std::min<uint32_t>(TRAY_POOL_CHUNKS, std::max<uint32_t>(16u, p.nchunks / (8u * (uint32_t)blocks)));
        // Chunk reservations per wave (take_chunk): single chunks for the last 8 reservations'
        // worth of every wave of the grid, so the launch's tail stays chunk-grained.
        p.wave_chunks = std::max<uint32_t>(1u, std::min<uint32_t>(TRAY_WAVE_CHUNKS, p.pool_chunks));
        const uint64_t late_margin = (uint64_t)p.wave_chunks * TRAY_LATE_TAKES * (uint64_t)blocks * waves;
        p.late_at = p.nchunks > late_margin ? p.nchunks - (uint32_t)late_margin : 0u;
        if (wave_chunks_knob > 0) {  // tests: this reservation size everywhere, no single-chunk tail
            p.wave_chunks = (uint32_t)wave_chunks_knob;
            p.late_at = p.nchunks;
        }
        // Enough waves for every chunk, capped at what the device keeps resident
        // (less the slots the "grid_reserve" knob leaves to other kernels).
        const uint32_t grid = std::min<uint32_t>((p.nchunks + waves - 1u) / waves, (uint32_t)(blocks - reserve));
        // The queue is zero here: zeroed at allocation and by every resolve pass.
        hipLaunchKernelGGL(fn, dim3(grid), dim3(threads), lds, stream, p);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(resolve, dim3((pixels + 255u) / 256u, p.passes), dim3(256), 0, stream, p);
        e = hipGetLastError();
        if (e != hipSuccess) {
            (void)hipMemsetAsync(p.queue, 0, sizeof(uint32_t), stream);  // keep the invariant
            return e;
        }
        if (p.tile_cost) {  // a counting launch: this band's next work order (after its megakernel read the old one)
            hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, stream, p.tile_cost, order_out + tile_off,
                               band_tiles_n);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

}  // namespace tray
