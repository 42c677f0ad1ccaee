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

template <bool kLDS>
__global__ __launch_bounds__(256) void render_kernel(KernelParams p) {
    extern __shared__ __attribute__((aligned(16))) double4 s_geo[];
    const double4* __restrict__ geo = p.geo;
    if constexpr (kLDS) {
        for (int i = threadIdx.x; i < p.n; i += blockDim.x) s_geo[i] = p.geo[i];
        __syncthreads();
        geo = s_geo;
    }

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int j = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool valid = x < p.width && j < p.rows;
    const int32_t y = valid ? row_of(p, j) : 0;
    const uint32_t pixel = (uint32_t)y * (uint32_t)p.width + (uint32_t)x;
    const double fx = (double)x, fy = (double)y;

    D3 org = d3(0, 0, 0), dir = d3(0, 0, 1);
    D3 thr = d3(1, 1, 1);
    D3 sum = d3(0, 0, 0);
    uint32_t sample = 0, bounce = 0, segments = 0;
    bool done = !valid;
    if (!done) get_ray(p, pixel, 0u, fx, fy, org, dir);

    const int n = p.n;
    while (__ballot(!done) != 0ull) {
        if (!done) {
            ++segments;
            // Scene.Hit over every sphere in list order; a = |D|^2 hoisted (same bits).
            const double a = length_sq(dir);
            double closest = __builtin_inf();
            int best = -1;
            for (int i = 0; i < n; ++i) {
                const double4 g = geo[i];
                const double ocx = g.x - org.x;
                const double ocy = g.y - org.y;
                const double ocz = g.z - org.z;
                const double h = dir.x * ocx + dir.y * ocy + dir.z * ocz;
                const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - g.w;
                const double disc = h * h - a * c;
                if (disc >= 0) {
                    const double sq = __builtin_sqrt(disc);
                    double root = (h - sq) / a;
                    if (!(root > 1e-6 && root < closest)) {
                        root = (h + sq) / a;
                        if (!(root > 1e-6 && root < closest)) continue;
                    }
                    closest = root;
                    best = i;
                }
            }

            bool path_end = false;
            D3 color = d3(0, 0, 0);
            if (best >= 0) {
                const double4 g = geo[best];
                const MatRec m = p.mat[best];
                const D3 center = d3(g.x, g.y, g.z);
                const D3 point = add(org, smul(dir, closest));
                const D3 outward = sdiv(sub(point, center), m.radius);
                const bool front = dot(dir, outward) < 0;
                const D3 normal = front ? outward : neg(outward);
                const D3 albedo = d3(m.albedo[0], m.albedo[1], m.albedo[2]);
                bool scattered = true;
                D3 new_dir;
                D3 att = albedo;
                if (m.type == kLambertian) {
                    new_dir = add(normal, unit_vector(p.seed, pixel, sample, bounce));
                    if (near_zero(new_dir)) new_dir = normal;
                } else if (m.type == kMetal) {
                    D3 reflected = reflect(unit(dir), normal);
                    if (m.param > 0.0) reflected = add(reflected, smul(unit_vector(p.seed, pixel, sample, bounce), m.param));
                    new_dir = reflected;
                    scattered = dot(new_dir, normal) > 0;
                } else {  // kDielectric
                    att = d3(1.0, 1.0, 1.0);
                    const double ratio = front ? 1.0 / m.param : m.param;
                    const D3 ud = unit(dir);
                    const double cos_theta = go_min(dot(neg(ud), normal), 1.0);
                    const double sin_theta = __builtin_sqrt(1.0 - cos_theta * cos_theta);
                    const bool cannot_refract = ratio * sin_theta > 1.0;
                    bool do_reflect = cannot_refract;
                    if (!do_reflect) {
                        const U2 u = philox_uniforms(p.seed, pixel, sample, bounce, kPurposeScatter << 24);
                        do_reflect = reflectance(cos_theta, ratio) > u.u0;
                    }
                    new_dir = do_reflect ? reflect(ud, normal) : refract(ud, normal, ratio);
                }
                if (scattered) {
                    thr = mul(thr, att);
                    org = point;
                    dir = new_dir;
                    ++bounce;
                    path_end = bounce >= (uint32_t)p.max_depth;  // RayColor(depth 0) -> black
                } else {
                    path_end = true;  // absorbed -> black
                }
            } else {
                // AmbientLight.Hit (ray/objects.go:68-73)
                const D3 u = unit(dir);
                const double t = 0.5 * (u.y + 1.0);
                const D3 sky = add(smul(d3(p.bg_a.x, p.bg_a.y, p.bg_a.z), 1.0 - t), smul(d3(p.bg_b.x, p.bg_b.y, p.bg_b.z), t));
                color = mul(thr, sky);
                path_end = true;
            }
            if (path_end) {
                sum = add(sum, color);
                ++sample;
                if (sample >= (uint32_t)p.spp) {
                    done = true;
                } else {
                    thr = d3(1, 1, 1);
                    bounce = 0;
                    get_ray(p, pixel, sample, fx, fy, org, dir);
                }
            }
        }
    }

    if (!valid) return;
    const double inv = 1.0 / (double)p.spp;  // colorSumDiv (ray/tracer.go:123)
    const D3 mean = smul(sum, inv);
    const size_t off = (size_t)j * (size_t)p.width + (size_t)x;
    if (p.out_format == kOutRGBF64) {
        double* o = static_cast<double*>(p.out) + off * 3;
        o[0] = mean.x;
        o[1] = mean.y;
        o[2] = mean.z;
    } else if (p.out_format == kOutRGBF32) {
        float* o = static_cast<float*>(p.out) + off * 3;
        o[0] = (float)mean.x;
        o[1] = (float)mean.y;
        o[2] = (float)mean.z;
    } else {
        const uint32_t rgba = linear_to_srgb(mean.x) | (linear_to_srgb(mean.y) << 8) |
                              (linear_to_srgb(mean.z) << 16) | (255u << 24);
        static_cast<uint32_t*>(p.out)[off] = rgba;
    }
    if (p.segments) p.segments[off] = segments;
}

hipError_t launch_render(const KernelParams& p, hipStream_t stream) {
    const dim3 block(256);
    const dim3 grid((unsigned)((p.width + 15) / 16), (unsigned)((p.rows + 15) / 16));
    const size_t lds = (size_t)p.n * sizeof(double4);
    if (p.rows <= 0) return hipSuccess;
    if (lds <= kMaxLDSBytes) {
        static bool attr_set[64] = {};
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev >= 0 && dev < 64 && !attr_set[dev]) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&render_kernel<true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLDSBytes);
            if (e != hipSuccess) return e;
            attr_set[dev] = true;
        }
        hipLaunchKernelGGL(render_kernel<true>, grid, block, lds, stream, p);
    } else {
        hipLaunchKernelGGL(render_kernel<false>, grid, block, 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace tray
