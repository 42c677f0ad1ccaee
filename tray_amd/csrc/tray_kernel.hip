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
__device__ __forceinline__ double dot(D3 u, D3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
__device__ __forceinline__ double length_sq(D3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
__device__ __forceinline__ D3 unit(D3 v) {
    const double l = __builtin_sqrt(length_sq(v));
    return d3(v.x / l, v.y / l, v.z / l);
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

// RandomUnitVector (ray/rand.go:30-32): Archimedes' projection of the bounce's
// scatter block, z = 1 - 2 u0, phi = 2 pi u1.
__device__ __forceinline__ D3 unit_vector(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce) {
    const U4 u = philox_u4(seed, pixel, sample, bounce, kPurposeScatter << 24);
    const double z = 1.0 - 2.0 * u.u0;
    const double r = __builtin_sqrt(1.0 - z * z);
    double s, c;
    sincos_2pi(u.u1, s, c);
    return d3(r * c, r * s, z);
}

// Camera.GetRay (ray/camera.go:113-142). The sample's camera block feeds the
// anti-aliasing disc (words 0,1; ray/tracer.go:136-139) and the lens disc
// (words 2,3).
__device__ __forceinline__ void get_ray(const KernelParams& p, uint32_t pixel, uint32_t sample, double px, double py,
                                        D3& origin, D3& dir) {
    double ox = 0.0, oy = 0.0;
    U4 u = U4{0, 0, 0, 0};
    if (p.spp > 1 || p.cam.aperture > 0) u = philox_u4(p.seed, pixel, sample, 0u, kPurposeCamera << 24);
    if (p.spp > 1) disc(u.u0, u.u1, p.ray_radius, ox, oy);
    const D3 pos = d3(p.cam.position[0], p.cam.position[1], p.cam.position[2]);
    const D3 p00 = d3(p.cam.pixel00[0], p.cam.pixel00[1], p.cam.pixel00[2]);
    const D3 pxv = d3(p.cam.pixel_x[0], p.cam.pixel_x[1], p.cam.pixel_x[2]);
    const D3 pyv = d3(p.cam.pixel_y[0], p.cam.pixel_y[1], p.cam.pixel_y[2]);
    const D3 sample_pt = add(add(p00, smul(pxv, px + ox)), smul(pyv, py + oy));
    origin = pos;
    dir = sub(sample_pt, pos);
    if (p.cam.aperture > 0) {
        double dx, dy;
        disc(u.u2, u.u3, 1.0, dx, dy);
        const D3 du = d3(p.cam.defocus_u[0], p.cam.defocus_u[1], p.cam.defocus_u[2]);
        const D3 dv = d3(p.cam.defocus_v[0], p.cam.defocus_v[1], p.cam.defocus_v[2]);
        const D3 offset = add(smul(du, dx), smul(dv, dy));
        const D3 focus_point = add(pos, smul(dir, p.focus_time));
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
__device__ __forceinline__ void candidate(double h, double disc, double a, int idx, double& closest, int& best) {
    if (disc >= 0) {
        const double sq = __builtin_sqrt(disc);
        double root = (h - sq) / a;
        bool ok = root > 1e-6 && root < closest;
        if (!ok) {
            root = (h + sq) / a;
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
__device__ __forceinline__ void candidate_any_order(double h, double disc, double a, int idx, double& closest,
                                                    int& best) {
    if (disc >= 0) {
        const double sq = __builtin_sqrt(disc);
        const double r1 = (h - sq) / a;
        const double t = r1 > 1e-6 ? r1 : (h + sq) / a;
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

struct Stats {
    uint32_t spheres = 0, boxes = 0;
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
            for (int k = 0; k < U; ++k) candidate(h[k], d[k], a, i + k, closest, best);
        }
    }
    if constexpr (kStats) st.spheres += (uint32_t)sv.n;
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
    double a, closest;
    int32_t best;  // original list index of the closest hit (tie-break key)
    int32_t slot;  // its leaf slot (LDS-resident geometry + shading record)
};

__device__ __forceinline__ void trav_begin(Trav& T, const D3& org, const D3& dir) {
    T.a = length_sq(dir);  // hoisted: same bits as per sphere
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

// Test the held leaf's <= kBvhLeafMax spheres (FP64, any-order rule).
__device__ __forceinline__ uint32_t trav_leaf(Trav& T, const SceneView& sv, const D3& org, const D3& dir) {
    const int slot = T.leaf >> 3, cnt = T.leaf & 7;
    double h[kBvhLeafMax], d[kBvhLeafMax];
#pragma unroll
    for (int k = 0; k < kBvhLeafMax; ++k) {
        quad(sv.bgeo[slot + k], org, dir, T.a, h[k], d[k]);
        if (k >= cnt) d[k] = __builtin_nan("");
    }
    double m = d[0];
#pragma unroll
    for (int k = 1; k < kBvhLeafMax; ++k) m = __builtin_fmax(m, d[k]);
    if (m >= 0) {
#pragma unroll
        for (int k = 0; k < kBvhLeafMax; ++k) {
            const int32_t idx = sv.bidx[slot + k];
            const int32_t before = T.best;
            candidate_any_order(h[k], d[k], T.a, idx, T.closest, T.best);
            if (T.best != before) T.slot = slot + k;
        }
        T.tlim = f32_up(T.closest);
    }
    T.leaf = -1;
    return T.node < sv.n_nodes ? kTravState : kShadeState;
}

// Shading of one Scene.Hit result (one recursion level of RayColor,
// ray/objects.go:49-62): sky on a miss, else the hit record and the material's
// scatter. `g`/`mrec` give the hit sphere's geometry and shading record (LDS
// for the BVH kernel, global memory for the linear scan). Returns true when the
// path ended (its colour in `color`); otherwise the lane's ray, throughput and
// bounce advance to the scattered ray.
template <typename GeoAt, typename MatAt>
__device__ __forceinline__ bool shade(const KernelParams& p, Lane& L, int best, double closest, GeoAt geo_at,
                                      MatAt mat_at, D3& color) {
    if (best < 0) {
        // AmbientLight.Hit (ray/objects.go:68-73)
        const D3 u = unit(L.dir);
        const double t = 0.5 * (u.y + 1.0);
        const D3 sky = add(smul(d3(p.bg_a.x, p.bg_a.y, p.bg_a.z), 1.0 - t), smul(d3(p.bg_b.x, p.bg_b.y, p.bg_b.z), t));
        color = mul(L.thr, sky);
        return true;
    }
    const double4 g = geo_at();
    const MatRec m = mat_at();
    const D3 point = add(L.org, smul(L.dir, closest));                 // Ray.At (ray/ray.go:23-25)
    const D3 outward = sdiv(sub(point, d3(g.x, g.y, g.z)), m.radius);  // ray/objects.go:100
    const bool front = dot(L.dir, outward) < 0;                        // SetFaceNormal (:19-26)
    const D3 normal = front ? outward : neg(outward);
    bool scattered = true;
    D3 new_dir;
    D3 att = d3(m.albedo[0], m.albedo[1], m.albedo[2]);
    if (m.type == kLambertian) {  // ray/materials.go:13-20
        new_dir = add(normal, unit_vector(p.seed, L.pixel, L.sample, L.bounce));
        if (near_zero(new_dir)) new_dir = normal;
    } else if (m.type == kMetal) {  // ray/materials.go:28-37
        D3 reflected = reflect(unit(L.dir), normal);
        if (m.param > 0.0)
            reflected = add(reflected, smul(unit_vector(p.seed, L.pixel, L.sample, L.bounce), m.param));
        new_dir = reflected;
        scattered = dot(new_dir, normal) > 0;
    } else {  // Dielectric, ray/materials.go:44-64
        att = d3(1.0, 1.0, 1.0);
        const double ratio = front ? 1.0 / m.param : m.param;
        const D3 ud = unit(L.dir);
        const double cos_theta = go_min(dot(neg(ud), normal), 1.0);
        const double sin_theta = __builtin_sqrt(1.0 - cos_theta * cos_theta);
        bool do_reflect = ratio * sin_theta > 1.0;  // cannot refract
        if (!do_reflect) {
            const U4 u = philox_u4(p.seed, L.pixel, L.sample, L.bounce, kPurposeScatter << 24);
            do_reflect = reflectance(cos_theta, ratio) > u.u0;
        }
        new_dir = do_reflect ? reflect(ud, normal) : refract(ud, normal, ratio);
    }
    color = d3(0, 0, 0);
    if (!scattered) return true;  // absorbed -> black
    L.thr = mul(L.thr, att);
    L.org = point;
    L.dir = new_dir;
    ++L.bounce;
    return L.bounce >= (uint32_t)p.max_depth;  // RayColor(depth 0) -> black
}

// Work item w (64 pixels = one 8x8 tile of the compact row space) -> pixel.
__device__ __forceinline__ bool decode_pixel(const KernelParams& p, uint32_t item, int32_t& x, int32_t& j) {
    const uint32_t tile = item >> 6, r = item & 63u;
    const uint32_t tx = tile % (uint32_t)p.tiles_x, ty = tile / (uint32_t)p.tiles_x;
    x = (int32_t)(tx * 8u + (r & 7u));
    j = (int32_t)(ty * 8u + (r >> 3));
    return x < p.width && j < p.rows;
}

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
    get_ray(p, L.pixel, 0u, L.fx, L.fy, L.org, L.dir);
}

// A path ended with `color`: accumulate (Add(colorSum, color), ray/tracer.go:143)
// and either start the next sample or finish the pixel. Returns false when the
// pixel is done (written) and the lane is free.
template <int kFmt, bool kStats>
__device__ __forceinline__ bool end_path(const KernelParams& p, Lane& L, const D3& color, Stats& st) {
    L.sum = add(L.sum, color);
    ++L.sample;
    if (L.sample >= (uint32_t)p.spp) {
        write_pixel<kFmt>(p, L);
        if constexpr (kStats) {
            atomicAdd(p.stats + 0, (unsigned long long)L.segments);
            atomicAdd(p.stats + 1, (unsigned long long)st.spheres);
            atomicAdd(p.stats + 2, (unsigned long long)st.boxes);
            st = Stats{};
        }
        L.busy = false;
        return false;
    }
    L.thr = d3(1, 1, 1);
    L.bounce = 0;
    get_ray(p, L.pixel, L.sample, L.fx, L.fy, L.org, L.dir);
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
// stats[3..15] (the stats buffer must then hold 16 counters). Never part of a
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
    extern __shared__ __attribute__((aligned(16))) double4 smem[];
    SceneView sv{p.geo, p.nodes, p.bgeo, p.bidx, p.bmat, p.n, p.n_nodes};
    if constexpr (kLDS) {
        if constexpr (kBVH) {
            // [nodes: n_nodes x 32 B][bgeo: n_slots x 32 B][bmat: n_slots x 48 B][bidx: n_slots x 4 B]
            double4* lds_nodes = smem;
            double4* lds_geo = smem + p.n_nodes;
            MatRec* lds_mat = reinterpret_cast<MatRec*>(smem + p.n_nodes + p.n_slots);
            int32_t* lds_idx = reinterpret_cast<int32_t*>(lds_mat + p.n_slots);
            const double4* gn = reinterpret_cast<const double4*>(p.nodes);
            for (int i = threadIdx.x; i < p.n_nodes; i += blockDim.x) lds_nodes[i] = gn[i];
            for (int i = threadIdx.x; i < p.n_slots; i += blockDim.x) {
                lds_geo[i] = p.bgeo[i];
                lds_mat[i] = p.bmat[i];
                lds_idx[i] = p.bidx[i];
            }
            sv.nodes = reinterpret_cast<const BvhNode*>(lds_nodes);
            sv.bgeo = lds_geo;
            sv.bmat = lds_mat;
            sv.bidx = lds_idx;
        } else {
            for (int i = threadIdx.x; i < p.n_pad; i += blockDim.x) smem[i] = p.geo[i];
            sv.geo = smem;
        }
        __syncthreads();
    }
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
    uint64_t prof[13] = {};
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
                D3 color;
                if (shade(p, L, best, closest, [&] { return p.geo[best]; }, [&] { return p.mat[best]; }, color))
                    end_path<kFmt, kStats>(p, L, color, st);
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
                    if constexpr (kStats) st.spheres += (uint32_t)(T.leaf & 7);
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
                    D3 color;
                    bool more = true;
                    if (shade(p, L, T.best, T.closest, [&] { return sv.bgeo[T.slot]; },
                              [&] { return sv.bmat[T.slot]; }, color))
                        more = end_path<kFmt, kStats>(p, L, color, st);
                    if (more) {
                        ++L.segments;
                        trav_begin(T, L.org, L.dir);
                        state = kTravState;
                    } else {
                        state = kIdleState;
                    }
                }
                PROF_ADD(3);
            }
        }
    }
#ifdef TRAY_PROFILE
    if (kStats && lane == 0)
        for (int i = 0; i < 13; ++i) atomicAdd(p.stats + 3 + i, (unsigned long long)prof[i]);
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
    const size_t lds_bytes = use_bvh ? (size_t)p.n_nodes * sizeof(BvhNode) +
                                           (size_t)p.n_slots * (sizeof(double4) + sizeof(MatRec) + 4)
                                     : (size_t)p.n_pad * sizeof(double4);
    const bool use_lds = lds_bytes <= kMaxLDSBytes;
    const size_t lds = use_lds ? (lds_bytes + 15) / 16 * 16 : 0;
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
        e = hipMemsetAsync(p.stats, 0, 16 * sizeof(unsigned long long), stream);
#else
        e = hipMemsetAsync(p.stats, 0, 3 * sizeof(unsigned long long), stream);
#endif
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, stream, p);
    return hipGetLastError();
}

}  // namespace tray
