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

__device__ __forceinline__ void in_disc(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t purpose,
                                        double radius, double& ox, double& oy) {
    ox = 0.0;
    oy = 0.0;
    for (uint32_t a = 0; a < kMaxAttempts; ++a) {
        const U2 u = philox_uniforms(seed, pixel, sample, 0u, (purpose << 24) | a);
        const double x = 2.0 * u.u0 - 1.0;
        const double y = 2.0 * u.u1 - 1.0;
        if (x * x + y * y < 1.0) {
            ox = x * radius;
            oy = y * radius;
            break;
        }
    }
}

__device__ __forceinline__ D3 unit_vector(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce) {
    D3 r = d3(0.0, 0.0, 1.0);
    for (uint32_t a = 0; a < kMaxAttempts; ++a) {
        const U2 u = philox_uniforms(seed, pixel, sample, bounce, (kPurposeScatter << 24) | a);
        const double x1 = 2.0 * u.u0 - 1.0;
        const double x2 = 2.0 * u.u1 - 1.0;
        const double s = x1 * x1 + x2 * x2;
        if (s < 1.0 && s > 0.0) {
            const double f = 2.0 * __builtin_sqrt(1.0 - s);
            r = d3(x1 * f, x2 * f, 1.0 - 2.0 * s);
            break;
        }
    }
    return r;
}

// Camera.GetRay (ray/camera.go:113-142).
__device__ __forceinline__ void get_ray(const KernelParams& p, uint32_t pixel, uint32_t sample, double px, double py,
                                        D3& origin, D3& dir) {
    double ox = 0.0, oy = 0.0;
    if (p.spp > 1) in_disc(p.seed, pixel, sample, kPurposeAA, p.ray_radius, ox, oy);  // ray/tracer.go:136-139
    const D3 pos = d3(p.cam.position[0], p.cam.position[1], p.cam.position[2]);
    const D3 p00 = d3(p.cam.pixel00[0], p.cam.pixel00[1], p.cam.pixel00[2]);
    const D3 pxv = d3(p.cam.pixel_x[0], p.cam.pixel_x[1], p.cam.pixel_x[2]);
    const D3 pyv = d3(p.cam.pixel_y[0], p.cam.pixel_y[1], p.cam.pixel_y[2]);
    const D3 sample_pt = add(add(p00, smul(pxv, px + ox)), smul(pyv, py + oy));
    origin = pos;
    dir = sub(sample_pt, pos);
    if (p.cam.aperture > 0) {
        double dx, dy;
        in_disc(p.seed, pixel, sample, kPurposeLens, 1.0, dx, dy);
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

// Scene.Hit through the exact-culling BVH (tray_bvh.cpp). Per lane, stackless
// depth-first traversal with skip links. While-while: every lane first advances
// over nodes (cheap conservative FP32 slab tests on padded boxes, culling
// against the current closest hit) until it holds a leaf or is done; then the
// lanes holding a leaf test its <= 4 spheres together in FP64 with the
// reference's arithmetic and the any-order acceptance rule.
template <bool kStats>
__device__ __forceinline__ int scene_hit_bvh(const SceneView& sv, const D3& org, const D3& dir, double& closest,
                                             Stats& st) {
    const double a = length_sq(dir);
    closest = __builtin_inf();
    int best = -1;
    float dxf = (float)dir.x, dyf = (float)dir.y, dzf = (float)dir.z;
    if (__builtin_fabsf(dxf) < 1e-30f) dxf = 1e-30f;
    if (__builtin_fabsf(dyf) < 1e-30f) dyf = 1e-30f;
    if (__builtin_fabsf(dzf) < 1e-30f) dzf = 1e-30f;
    const float ix = 1.0f / dxf, iy = 1.0f / dyf, iz = 1.0f / dzf;
    const float oix = (float)org.x * ix, oiy = (float)org.y * iy, oiz = (float)org.z * iz;
    float tlim = __builtin_inff();  // closest rounded up to float
    int node = 0;
    while (true) {
        int leaf = -1;
        while (true) {
            const bool search = node < sv.n_nodes && leaf < 0;
            if (__ballot(search) == 0ull) break;
            if (search) {
                const BvhNode nd = sv.nodes[node];
                const float t0x = __builtin_fmaf(nd.lo[0], ix, -oix), t1x = __builtin_fmaf(nd.hi[0], ix, -oix);
                const float t0y = __builtin_fmaf(nd.lo[1], iy, -oiy), t1y = __builtin_fmaf(nd.hi[1], iy, -oiy);
                const float t0z = __builtin_fmaf(nd.lo[2], iz, -oiz), t1z = __builtin_fmaf(nd.hi[2], iz, -oiz);
                const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                                 __builtin_fmaxf(__builtin_fminf(t0z, t1z), 0.0f));
                const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                                 __builtin_fminf(__builtin_fmaxf(t0z, t1z), tlim));
                if constexpr (kStats) ++st.boxes;
                if (tn <= tf) {
                    if (nd.leaf >= 0) {
                        leaf = nd.leaf;
                        node = nd.skip;
                    } else {
                        node = node + 1;
                    }
                } else {
                    node = nd.skip;
                }
            }
        }
        if (__ballot(leaf >= 0) == 0ull) break;
        if (leaf >= 0) {
            const int slot = leaf >> 3, cnt = leaf & 7;
            double h[kBvhLeafMax], d[kBvhLeafMax];
#pragma unroll
            for (int k = 0; k < kBvhLeafMax; ++k) {
                quad(sv.bgeo[slot + k], org, dir, a, h[k], d[k]);
                if (k >= cnt) d[k] = __builtin_nan("");
            }
            double m = d[0];
#pragma unroll
            for (int k = 1; k < kBvhLeafMax; ++k) m = __builtin_fmax(m, d[k]);
            if (m >= 0) {
#pragma unroll
                for (int k = 0; k < kBvhLeafMax; ++k) candidate_any_order(h[k], d[k], a, sv.bidx[slot + k], closest, best);
                tlim = f32_up(closest);
            }
            if constexpr (kStats) st.spheres += (uint32_t)cnt;
        }
    }
    return best;
}

// One Scene.Hit + shading step of the lane's current path (one recursion level
// of RayColor, ray/objects.go:49-62). Returns true when the path ended.
template <bool kBVH, bool kStats>
__device__ __forceinline__ bool segment(const KernelParams& p, const SceneView& sv, Lane& L, D3& color, Stats& st) {
    ++L.segments;
    double closest;
    const int best = kBVH ? scene_hit_bvh<kStats>(sv, L.org, L.dir, closest, st)
                          : scene_hit_linear<TRAY_UNROLL, kStats>(sv, L.org, L.dir, closest, st);
    if (best < 0) {
        // AmbientLight.Hit (ray/objects.go:68-73)
        const D3 u = unit(L.dir);
        const double t = 0.5 * (u.y + 1.0);
        const D3 sky = add(smul(d3(p.bg_a.x, p.bg_a.y, p.bg_a.z), 1.0 - t), smul(d3(p.bg_b.x, p.bg_b.y, p.bg_b.z), t));
        color = mul(L.thr, sky);
        return true;
    }
    const double4 g = p.geo[best];
    const MatRec m = p.mat[best];
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
            const U2 u = philox_uniforms(p.seed, L.pixel, L.sample, L.bounce, kPurposeScatter << 24);
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

#ifndef TRAY_WAVES_PER_SIMD
#define TRAY_WAVES_PER_SIMD 5
#endif
#ifndef TRAY_BVH_WAVES_PER_SIMD
#define TRAY_BVH_WAVES_PER_SIMD 4
#endif

// Persistent megakernel: waves pull 64-pixel work items from a global counter
// and lanes refill individually, so no lane idles while the frame has work.
template <bool kLDS, int kFmt, bool kBVH, bool kStats>
__global__ __launch_bounds__(256, kBVH ? TRAY_BVH_WAVES_PER_SIMD : TRAY_WAVES_PER_SIMD) void render_kernel(KernelParams p) {
    extern __shared__ __attribute__((aligned(16))) double4 smem[];
    SceneView sv{p.geo, p.nodes, p.bgeo, p.bidx, p.n, p.n_nodes};
    if constexpr (kLDS) {
        if constexpr (kBVH) {
            // [nodes: n_nodes x 32 B][bgeo: n_slots x 32 B][bidx: n_slots x 4 B]
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
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    Lane L;
    L.busy = false;
    Stats st;
    uint32_t pool_next = 0, pool_end = 0;  // wave-uniform: unassigned items of the current chunk
    bool exhausted = false;

    while (true) {
        // Refill idle lanes from the wave's pool, fetching 64-item chunks from the global queue.
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
                    if (decode_pixel(p, pool_next + rank, x, j)) start_pixel(p, L, x, j);
                }
            }
            pool_next += take;
            idle = __ballot(!L.busy);
        }
        if (__ballot(L.busy) == 0ull) break;
        if (L.busy) {
            D3 color;
            if (segment<kBVH, kStats>(p, sv, L, color, st)) {
                L.sum = add(L.sum, color);  // Add(colorSum, color) (ray/tracer.go:143)
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
                } else {
                    L.thr = d3(1, 1, 1);
                    L.bounce = 0;
                    get_ray(p, L.pixel, L.sample, L.fx, L.fy, L.org, L.dir);
                }
            }
        }
    }
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
        e = hipMemsetAsync(p.stats, 0, 3 * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, stream, p);
    return hipGetLastError();
}

}  // namespace tray
