/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C FP64 restatement of fortio/tray's per-pixel path-tracing loop, used
 * as the parity checker for the HIP megakernel. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library. It is never linked into,
 * called by, or used as a fallback for the product path (tray_amd/).
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the fortio/tray repository root). Op order follows the Go source exactly
 * (left-to-right evaluation, no FMA contraction: build with -ffp-contract=off),
 * with one documented substitution: the random stream. fortio.org/rand v1.1.0
 * (go.mod:9) is not available, so every draw comes from the counter-based RNG
 * specified in include/tray.h ("Counter RNG contract"), keyed on
 * (seed; pixel, sample, bounce, purpose). The draw SCHEDULE (which
 * call sites draw, and when) follows the reference.
 *
 * Parity pinning: the vector/material/camera math is
 * pinned by the reference's own known-answer tests (ray/{vec3,objects,materials,camera,tracer}_test.go); RNG-free
 * scenes are pinned against an independent numpy restatement; camera + sky +
 * sRGB are pinned against the reference's own output image example.png.
 * The random stream itself is "parity unpinned" against Go (unavailable RNG).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* Data layouts (identical byte layout to include/tray.h; data only).  */
/* ------------------------------------------------------------------ */
typedef struct {
    double center[3];
    double radius;
    double albedo[3];
    double param; /* Metal.Fuzz or Dielectric.RefIdx */
    int32_t material;
    int32_t reserved;
} o_sphere; /* 72 bytes */

enum { O_LAMBERTIAN = 1, O_METAL = 2, O_DIELECTRIC = 3 };

typedef struct {
    double position[3];
    double pixel00[3];
    double pixel_x[3];
    double pixel_y[3];
    double defocus_u[3];
    double defocus_v[3];
    double aperture;
    double focus_distance;
    double focal_length;
} o_camera; /* 21 doubles */

typedef struct {
    double position[3];
    double look_at[3];
    double up[3];
    double vertical_fov;
    double focal_length;
    double focus_distance;
    double aperture;
} o_camera_setup; /* 13 doubles */

/* ------------------------------------------------------------------ */
/* Vec3 — ray/vec3.go                                                  */
/* ------------------------------------------------------------------ */
typedef struct { double x, y, z; } vec3;

static inline vec3 V(double x, double y, double z) { vec3 r = {x, y, z}; return r; }
/* Add(u,v) = {v.x+u.x, ...}  ray/vec3.go:25-27 */
static inline vec3 add(vec3 u, vec3 v) { return V(v.x + u.x, v.y + u.y, v.z + u.z); }
/* Sub  ray/vec3.go:30-32 */
static inline vec3 sub(vec3 u, vec3 v) { return V(u.x - v.x, u.y - v.y, u.z - v.z); }
/* Dot  ray/vec3.go:58-60 (left-to-right: (xx + yy) + zz) */
static inline double dot(vec3 u, vec3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
/* Cross ray/vec3.go:71-73 */
static inline vec3 cross(vec3 u, vec3 v) {
    return V(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
/* SMul ray/vec3.go:90-92 */
static inline vec3 smul(vec3 v, double t) { return V(v.x * t, v.y * t, v.z * t); }
/* Mul  ray/vec3.go:95-97 */
static inline vec3 mul(vec3 u, vec3 v) { return V(u.x * v.x, u.y * v.y, u.z * v.z); }
/* SDiv ray/vec3.go:100-102 */
static inline vec3 sdiv(vec3 v, double t) { return V(v.x / t, v.y / t, v.z / t); }
/* LengthSquared ray/vec3.go:110-112 */
static inline double length_sq(vec3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
/* Length ray/vec3.go:105-107 */
static inline double length(vec3 v) { return sqrt(length_sq(v)); }
/* Unit ray/vec3.go:116-119: divide each component by the length */
static inline vec3 unit(vec3 v) { double l = length(v); return V(v.x / l, v.y / l, v.z / l); }
/* Neg ray/vec3.go:122-124 */
static inline vec3 neg(vec3 v) { return V(-v.x, -v.y, -v.z); }
/* NearZero ray/vec3.go:127-130 */
static inline int near_zero(vec3 v) {
    const double s = 1e-8;
    return (fabs(v.x) < s) && (fabs(v.y) < s) && (fabs(v.z) < s);
}
/* Go math.Min semantics (special cases: -Inf, NaN, signed zeros). */
static inline double go_min(double x, double y) {
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}
/* Reflect ray/vec3.go:133-135 */
static inline vec3 reflect(vec3 v, vec3 n) { return sub(v, smul(n, 2 * dot(v, n))); }
/* Refract ray/vec3.go:139-144 */
static inline vec3 refract(vec3 uv, vec3 n, double etai_over_etat) {
    double cos_theta = go_min(dot(neg(uv), n), 1.0);
    vec3 r_out_perp = smul(add(uv, smul(n, cos_theta)), etai_over_etat);
    vec3 r_out_parallel = smul(n, -sqrt(fabs(1.0 - length_sq(r_out_perp))));
    return add(r_out_perp, r_out_parallel);
}
/* Go math.Pow(x, 5): integer-exponent path multiplies frexp mantissas by
 * repeated squaring (exact power-of-two rescaling), i.e. x * ((x*x)*(x*x))
 * for every normal result. */
static inline double pow5(double x) { double x2 = x * x; double x4 = x2 * x2; return x * x4; }

/* ------------------------------------------------------------------ */
/* Counter RNG (include/tray.h "Counter RNG contract"): Philox4x32-10 for the  */
/* draw key and the host's scene stream, the keyed pcg4d draw block for draws. */
/* ------------------------------------------------------------------ */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u

static void philox4x32_10(const uint32_t in[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += PH_W0; k1 += PH_W1; }
        uint64_t p0 = (uint64_t)PH_M0 * c0;
        uint64_t p1 = (uint64_t)PH_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { P_CAMERA = 1, P_SCATTER = 3, P_SCENE = 4, P_KEY = 5 };

/* The renderer's draw key (include/tray.h, ABI 6): Philox4x32-10 of the seed at
 * ctr = (0, 0, 0, P_KEY << 24). */
static void draw_key(uint64_t seed, uint32_t k[4]) {
    uint32_t ctr[4] = {0u, 0u, 0u, (uint32_t)P_KEY << 24};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    philox4x32_10(ctr, key, k);
}

/* The renderer's draw block (include/tray.h, ABI 6): pcg4d (Jarzynski & Olano,
 * JCGT 9(3) 2020) of the keyed counter, then v ^= v >> 16 on each word. All
 * arithmetic mod 2^32. */
static void draw_block(const uint32_t k[4], uint32_t pixel, uint32_t sample, uint32_t bounce, uint32_t purpose,
                       uint32_t out[4]) {
    uint32_t v[4] = {pixel ^ k[0], sample ^ k[1], bounce ^ k[2], purpose ^ k[3]};
    for (int i = 0; i < 4; ++i) v[i] = v[i] * 1664525u + 1013904223u;
    for (int round = 0; round < 2; ++round) {
        v[0] += v[1] * v[3];
        v[1] += v[2] * v[0];
        v[2] += v[0] * v[1];
        v[3] += v[1] * v[2];
        for (int i = 0; i < 4; ++i) v[i] ^= v[i] >> 16;
    }
    for (int i = 0; i < 4; ++i) out[i] = v[i];
}

/* One draw block as four 32-bit uniforms u = x * 2^-32 in [0,1). */
static void uniforms4(const uint32_t key[4], uint32_t pixel, uint32_t sample, uint32_t bounce, uint32_t purpose,
                      double u[4]) {
    uint32_t x[4];
    draw_block(key, pixel, sample, bounce, purpose, x);
    for (int i = 0; i < 4; ++i) u[i] = (double)x[i] * 0x1.0p-32;
}

/* Two uniforms in [0,1) with 53-bit resolution from one Philox block (host
 * scene generation only). */
static void uniforms2(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, double u[2]) {
    uint32_t ctr[4] = {c0, c1, c2, c3};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t x[4];
    philox4x32_10(ctr, key, x);
    uint64_t a = ((uint64_t)x[1] << 32) | x[0];
    uint64_t b = ((uint64_t)x[3] << 32) | x[2];
    u[0] = (double)(a >> 11) * 0x1.0p-53;
    u[1] = (double)(b >> 11) * 0x1.0p-53;
}

/* sin and cos of 2*pi*u for u in [0,1) (include/tray.h "sincos2pi"): exact
 * FP64 quadrant + reflection into [0, 1/2], then FP32 Taylor polynomials
 * (degree 9 / 10) in t^2 by Horner's rule with C99 fmaf() (correctly rounded,
 * as the device's v_fma_f32), so both sides produce the same bits. This is the
 * contract's sampler transform, not reference arithmetic: ray/rand.go:30-32
 * delegates to fortio.org/rand, whose stream cannot be reproduced. Needs
 * FLT_EVAL_METHOD 0 (SSE float arithmetic, the x86-64 default). */
static void sincos_2pi(double u, double *s, double *c) {
    double v = u * 4.0;
    double q = floor(v);
    double f = v - q;
    int quad = (int)q;
    int swap = f > 0.5;
    float x = (float)(swap ? 1.0 - f : f);
    float t = x * 0x1.921fb6p+0f; /* RN32(pi/2) */
    float t2 = t * t;
    float sp = fmaf(t2, 0x1.71de3ap-19f, -0x1.a01a02p-13f); /* 1/9!, -1/7! */
    sp = fmaf(sp, t2, 0x1.111112p-7f);                       /* 1/5! */
    sp = fmaf(sp, t2, -0x1.555556p-3f);                      /* -1/3! */
    sp = fmaf(sp, t2, 1.0f);
    float sn = t * sp;
    float cp = fmaf(t2, -0x1.27e4fcp-22f, 0x1.a01a02p-16f); /* -1/10!, 1/8! */
    cp = fmaf(cp, t2, -0x1.6c16c2p-10f);                     /* -1/6! */
    cp = fmaf(cp, t2, 0x1.555556p-5f);                       /* 1/4! */
    cp = fmaf(cp, t2, -0.5f);
    float cs = fmaf(cp, t2, 1.0f);
    if (swap) { float tmp = sn; sn = cs; cs = tmp; }
    /* one FP64 Newton step onto the unit circle (unit vectors are pinned to
     * 1e-9 by ray/vec3_test.go:505-537) */
    double sd = sn, cd = cs;
    double k = 1.5 - 0.5 * (sd * sd + cd * cd);
    double sk = sd * k, ck = cd * k;
    switch (quad & 3) {
    case 0: *s = sk; *c = ck; break;
    case 1: *s = ck; *c = -sk; break;
    case 2: *s = -sk; *c = -ck; break;
    default: *s = -ck; *c = sk; break;
    }
}

/* A sample's draws: the render's draw key (computed once per render) and the
 * sample's counter words. */
typedef struct { uint32_t key[4]; uint32_t pixel; uint32_t sample; } rngkey;
static rngkey make_rngkey(uint64_t seed, uint32_t pixel, uint32_t sample) {
    rngkey k;
    draw_key(seed, k.key);
    k.pixel = pixel;
    k.sample = sample;
    return k;
}

/* InDisc(radius) replacement (ray/tracer.go:138, ray/camera.go:128): polar map
 * of two uniforms of the sample's camera block; which = 0 (anti-aliasing,
 * words 0,1) or 1 (lens, words 2,3). */
static void in_disc(rngkey k, int which, double radius, double *ox, double *oy) {
    double u[4];
    uniforms4(k.key, k.pixel, k.sample, 0u, (uint32_t)P_CAMERA, u);
    double r = sqrt(u[2 * which]);
    double s, c;
    sincos_2pi(u[2 * which + 1], &s, &c);
    *ox = (r * c) * radius;
    *oy = (r * s) * radius;
}

/* RandomUnitVector (ray/rand.go:30-32 -> rand.UnitVector): uniform on S^2 by
 * Archimedes' projection, z = 1 - 2u0, phi = 2 pi u1, from the bounce's
 * scatter block. */
static vec3 random_unit_vector(rngkey k, uint32_t bounce) {
    double u[4];
    uniforms4(k.key, k.pixel, k.sample, bounce, (uint32_t)P_SCATTER, u);
    double z = 1.0 - 2.0 * u[0];
    double r = sqrt(1.0 - z * z);
    double s, c;
    sincos_2pi(u[1], &s, &c);
    return V(r * c, r * s, z);
}

/* rIn.Float64() in Dielectric.Scatter (ray/materials.go:57): word 0 of the
 * bounce's scatter block. */
static double random_float64(rngkey k, uint32_t bounce) {
    double u[4];
    uniforms4(k.key, k.pixel, k.sample, bounce, (uint32_t)P_SCATTER, u);
    return u[0];
}

/* Sequential stream for host-side scene generation (ray/objects.go:139-153). */
typedef struct { uint64_t seed; uint32_t idx; } scene_rng;
static double scene_float64(scene_rng *r) {
    double u[2];
    uniforms2(r->seed, r->idx, 0u, 0u, ((uint32_t)P_SCENE << 24), u);
    r->idx++;
    return u[0];
}
/* Float64Range(a,b) = a + (b-a)*Float64() */
static double scene_float64_range(scene_rng *r, double a, double b) { return a + (b - a) * scene_float64(r); }

/* ------------------------------------------------------------------ */
/* Ray / HitRecord / Sphere / Scene — ray/ray.go, ray/objects.go        */
/* ------------------------------------------------------------------ */
typedef struct { vec3 origin, dir; } ray;
/* At ray/ray.go:23-25 */
static inline vec3 ray_at(const ray *r, double t) { return add(r->origin, smul(r->dir, t)); }

typedef struct {
    vec3 point, normal;
    double t;
    int mat; /* index of the sphere whose material applies */
    int front_face;
} hit_record;

/* SetFaceNormal ray/objects.go:19-26 */
static inline void set_face_normal(hit_record *hr, const ray *r, vec3 outward) {
    hr->front_face = dot(r->dir, outward) < 0;
    hr->normal = hr->front_face ? outward : neg(outward);
}

/* Sphere.Hit ray/objects.go:81-104 */
static int sphere_hit(const o_sphere *s, int idx, const ray *r, double t_start, double t_end, hit_record *hr) {
    vec3 center = V(s->center[0], s->center[1], s->center[2]);
    vec3 oc = sub(center, r->origin);
    double a = length_sq(r->dir);
    double h = dot(r->dir, oc);
    double c = length_sq(oc) - s->radius * s->radius;
    double discriminant = h * h - a * c;
    if (discriminant < 0) return 0;
    double sqrt_d = sqrt(discriminant);
    double root = (h - sqrt_d) / a;
    if (!(root > t_start && root < t_end)) { /* Interval.Surrounds ray/vec3.go:198-200 */
        root = (h + sqrt_d) / a;
        if (!(root > t_start && root < t_end)) return 0;
    }
    hr->point = ray_at(r, root);
    hr->t = root;
    vec3 outward = sdiv(sub(hr->point, center), s->radius);
    set_face_normal(hr, r, outward);
    hr->mat = idx;
    return 1;
}

typedef struct {
    const o_sphere *spheres;
    int n;
    vec3 bg_a, bg_b;
} scene;

/* Scene.Hit ray/objects.go:37-46: linear scan in list order, strict shrink. */
static int scene_hit(const scene *sc, const ray *r, double t_start, double t_end, hit_record *hr) {
    int hit_anything = 0;
    double closest = t_end;
    for (int i = 0; i < sc->n; ++i) {
        if (sphere_hit(&sc->spheres[i], i, r, t_start, closest, hr)) {
            hit_anything = 1;
            closest = hr->t;
        }
    }
    return hit_anything;
}

/* AmbientLight.Hit ray/objects.go:68-73 */
static vec3 background_hit(const scene *sc, const ray *r) {
    vec3 u = unit(r->dir);
    double a = 0.5 * (u.y + 1.0);
    return add(smul(sc->bg_a, 1.0 - a), smul(sc->bg_b, a));
}

/* Reflectance ray/materials.go:66-71 */
static double reflectance(double cosine, double ref_idx) {
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 *= r0;
    return r0 + (1 - r0) * pow5(1 - cosine);
}

/* Material.Scatter ray/materials.go:13-64. Returns 1 if scattered, 0 if
 * absorbed, -1 on an unsupported material tag. */
static int scatter(const scene *sc, const ray *r_in, const hit_record *rec, rngkey k, uint32_t bounce,
                   vec3 *attenuation, ray *scattered) {
    const o_sphere *s = &sc->spheres[rec->mat];
    vec3 albedo = V(s->albedo[0], s->albedo[1], s->albedo[2]);
    switch (s->material) {
    case O_LAMBERTIAN: { /* ray/materials.go:13-20 */
        vec3 dir = add(rec->normal, random_unit_vector(k, bounce));
        if (near_zero(dir)) dir = rec->normal;
        scattered->origin = rec->point;
        scattered->dir = dir;
        *attenuation = albedo;
        return 1;
    }
    case O_METAL: { /* ray/materials.go:28-37 */
        vec3 reflected = reflect(unit(r_in->dir), rec->normal);
        if (s->param > 0.0) reflected = add(reflected, smul(random_unit_vector(k, bounce), s->param));
        scattered->origin = rec->point;
        scattered->dir = reflected;
        if (dot(scattered->dir, rec->normal) > 0) { *attenuation = albedo; return 1; }
        return 0;
    }
    case O_DIELECTRIC: { /* ray/materials.go:44-64 */
        double ratio = rec->front_face ? 1.0 / s->param : s->param;
        vec3 unit_dir = unit(r_in->dir);
        double cos_theta = go_min(dot(neg(unit_dir), rec->normal), 1.0);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        int cannot_refract = ratio * sin_theta > 1.0;
        vec3 dir;
        /* short-circuit ||: the draw is keyed, so skipping it shifts nothing */
        if (cannot_refract || reflectance(cos_theta, ratio) > random_float64(k, bounce))
            dir = reflect(unit_dir, rec->normal);
        else
            dir = refract(unit_dir, rec->normal, ratio);
        scattered->origin = rec->point;
        scattered->dir = dir;
        *attenuation = V(1.0, 1.0, 1.0);
        return 1;
    }
    default:
        return -1;
    }
}

/* Scene.RayColor ray/objects.go:49-62 — recursive, inner-first Mul. */
static vec3 ray_color(const scene *sc, const ray *r, int depth, rngkey k, uint32_t bounce, uint32_t *segments,
                      int *err) {
    if (depth <= 0) return V(0, 0, 0);
    hit_record hr;
    (*segments)++;
    if (scene_hit(sc, r, 1e-6, INFINITY, &hr)) { /* FrontEpsilon ray/vec3.go:218 */
        vec3 att;
        ray scattered;
        int s = scatter(sc, r, &hr, k, bounce, &att, &scattered);
        if (s < 0) { *err = 1; return V(0, 0, 0); }
        if (s) return mul(att, ray_color(sc, &scattered, depth - 1, k, bounce + 1, segments, err));
        return V(0, 0, 0);
    }
    return background_hit(sc, r);
}

/* Camera.GetRay ray/camera.go:113-142 */
static ray get_ray(const o_camera *c, rngkey k, double px, double py, double ox, double oy) {
    vec3 p00 = V(c->pixel00[0], c->pixel00[1], c->pixel00[2]);
    vec3 pxv = V(c->pixel_x[0], c->pixel_x[1], c->pixel_x[2]);
    vec3 pyv = V(c->pixel_y[0], c->pixel_y[1], c->pixel_y[2]);
    vec3 pos = V(c->position[0], c->position[1], c->position[2]);
    /* pixel00.Plus(a, b) = AddMultiple: Add(Add(pixel00, a), b)  ray/vec3.go:35-40 */
    vec3 sample = add(add(p00, smul(pxv, px + ox)), smul(pyv, py + oy));
    ray r;
    r.origin = pos;
    r.dir = sub(sample, pos);
    if (c->aperture > 0) {
        double dx, dy;
        in_disc(k, 1, 1.0, &dx, &dy);
        vec3 du = V(c->defocus_u[0], c->defocus_u[1], c->defocus_u[2]);
        vec3 dv = V(c->defocus_v[0], c->defocus_v[1], c->defocus_v[2]);
        vec3 offset = add(smul(du, dx), smul(dv, dy));
        double focus_time = c->focus_distance / c->focal_length;
        vec3 focus_point = add(pos, smul(r.dir, focus_time));
        r.origin = add(pos, offset);
        r.dir = sub(focus_point, r.origin);
    }
    return r;
}

typedef struct {
    int width, height, spp, max_depth;
    double ray_radius;
    uint64_t seed;
    uint32_t sample_base; /* progressive pass x spp (tray_params.pass, include/tray.h) */
    uint32_t key[4];      /* the draw key of the seed (draw_key) */
} o_params;

/* One pixel of Tracer.RenderLines ray/tracer.go:129-145 (linear mean colour). */
static int render_pixel(const scene *sc, const o_camera *cam, const o_params *p, int x, int y, double out[3],
                        uint32_t *segments) {
    int multiple_rays = p->spp > 1;
    double color_sum_div = 1.0 / (double)p->spp;
    vec3 sum = V(0, 0, 0);
    uint32_t segs = 0;
    int err = 0;
    for (int s = 0; s < p->spp; ++s) {
        rngkey k = {{p->key[0], p->key[1], p->key[2], p->key[3]}, (uint32_t)y * (uint32_t)p->width + (uint32_t)x,
                    p->sample_base + (uint32_t)s};
        double ox = 0.0, oy = 0.0;
        if (multiple_rays) in_disc(k, 0, p->ray_radius, &ox, &oy);
        ray r = get_ray(cam, k, (double)x, (double)y, ox, oy);
        vec3 c = ray_color(sc, &r, p->max_depth, k, 0u, &segs, &err);
        if (err) return -2;
        sum = add(sum, c);
    }
    vec3 m = smul(sum, color_sum_div);
    out[0] = m.x; out[1] = m.y; out[2] = m.z;
    if (segments) *segments = segs;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Scheduler — ray/tracer.go:86-116 (w==1: one pass; else a chunk queue). */
/* ------------------------------------------------------------------ */
typedef struct {
    const scene *sc;
    const o_camera *cam;
    const o_params *p;
    const int32_t *rows;
    int nrows;
    int chunk;
    double *out;
    uint32_t *segs;
    int next; /* atomic */
    int err;  /* atomic */
} job;

static void render_row_range(job *j, int r0, int r1) {
    for (int ri = r0; ri < r1; ++ri) {
        int y = j->rows[ri];
        for (int x = 0; x < j->p->width; ++x) {
            size_t off = (size_t)ri * j->p->width + x;
            uint32_t s = 0;
            if (render_pixel(j->sc, j->cam, j->p, x, y, j->out + off * 3, &s) != 0) {
                __atomic_store_n(&j->err, 1, __ATOMIC_RELAXED);
                return;
            }
            if (j->segs) j->segs[off] = s;
        }
    }
}

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (;;) {
        int c = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        int r0 = c * j->chunk;
        if (r0 >= j->nrows) break;
        int r1 = r0 + j->chunk < j->nrows ? r0 + j->chunk : j->nrows;
        render_row_range(j, r0, r1);
    }
    return NULL;
}

static int valid_scene(const o_sphere *sp, int n) {
    for (int i = 0; i < n; ++i)
        if (sp[i].material < O_LAMBERTIAN || sp[i].material > O_DIELECTRIC) return 0;
    return 1;
}

/* Render an arbitrary list of image rows into a compact (nrows x W x 3) FP64
 * buffer. workers==1 reproduces the single RenderLines pass; workers>1 the
 * chunk queue (chunk = max(4, nrows/(4w))). Returns 0, -1 bad args, -2 bad material. */
ORACLE_EXPORT int oracle_render_rows(const o_sphere *spheres, int n, const double bg[6], const o_camera *cam,
                                     int width, int height, int spp, int max_depth, double ray_radius,
                                     uint64_t seed, const int32_t *rows, int nrows, int workers, double *out_rgb,
                                     uint32_t *out_segments, int pass) {
    if (width <= 0 || height <= 0 || spp <= 0 || max_depth <= 0 || nrows < 0 || (n > 0 && !spheres)) return -1;
    if (!valid_scene(spheres, n)) return -2;
    for (int i = 0; i < nrows; ++i)
        if (rows[i] < 0 || rows[i] >= height) return -1;
    scene sc = {spheres, n, V(bg[0], bg[1], bg[2]), V(bg[3], bg[4], bg[5])};
    if (pass < 0) return -1;
    o_params p = {width, height, spp, max_depth, ray_radius, seed, (uint32_t)pass * (uint32_t)spp, {0, 0, 0, 0}};
    draw_key(seed, p.key);
    job j = {&sc, cam, &p, rows, nrows, 0, out_rgb, out_segments, 0, 0};
    if (workers <= 1) {
        render_row_range(&j, 0, nrows);
    } else {
        int chunk = nrows / (workers * 4);
        j.chunk = chunk > 4 ? chunk : 4;
        pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)workers);
        for (int w = 0; w < workers; ++w) pthread_create(&th[w], NULL, worker, &j);
        for (int w = 0; w < workers; ++w) pthread_join(th[w], NULL);
        free(th);
    }
    return j.err ? -2 : 0;
}

/* Spot-check individual pixels (size-independent parity at full configs). */
ORACLE_EXPORT int oracle_render_pixels(const o_sphere *spheres, int n, const double bg[6], const o_camera *cam,
                                       int width, int height, int spp, int max_depth, double ray_radius,
                                       uint64_t seed, const int32_t *xs, const int32_t *ys, int count,
                                       double *out_rgb, uint32_t *out_segments, int pass) {
    if (width <= 0 || height <= 0 || spp <= 0 || max_depth <= 0 || pass < 0) return -1;
    if (!valid_scene(spheres, n)) return -2;
    scene sc = {spheres, n, V(bg[0], bg[1], bg[2]), V(bg[3], bg[4], bg[5])};
    o_params p = {width, height, spp, max_depth, ray_radius, seed, (uint32_t)pass * (uint32_t)spp, {0, 0, 0, 0}};
    draw_key(seed, p.key);
    for (int i = 0; i < count; ++i) {
        uint32_t s = 0;
        if (xs[i] < 0 || xs[i] >= width || ys[i] < 0 || ys[i] >= height) return -1;
        if (render_pixel(&sc, cam, &p, xs[i], ys[i], out_rgb + 3 * (size_t)i, &s) != 0) return -2;
        if (out_segments) out_segments[i] = s;
    }
    return 0;
}

/* Scene.RayColor for one explicit ray (ray/objects_test.go style tests). */
ORACLE_EXPORT int oracle_ray_color(const o_sphere *spheres, int n, const double bg[6], const double origin[3],
                                   const double dir[3], int depth, uint64_t seed, uint32_t pixel, uint32_t sample,
                                   double out[3], uint32_t *segments) {
    scene sc = {spheres, n, V(bg[0], bg[1], bg[2]), V(bg[3], bg[4], bg[5])};
    ray r = {V(origin[0], origin[1], origin[2]), V(dir[0], dir[1], dir[2])};
    rngkey k = make_rngkey(seed, pixel, sample);
    uint32_t segs = 0;
    int err = 0;
    vec3 c = ray_color(&sc, &r, depth, k, 0u, &segs, &err);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
    if (segments) *segments = segs;
    return err ? -2 : 0;
}

/* ------------------------------------------------------------------ */
/* Small known-answer entry points (ray/{vec3,objects,materials,camera}_test.go). */
/* ------------------------------------------------------------------ */
ORACLE_EXPORT void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    philox4x32_10(ctr, key, out);
}
ORACLE_EXPORT void oracle_draw_key(uint64_t seed, uint32_t out[4]) { draw_key(seed, out); }
ORACLE_EXPORT void oracle_draw_block(const uint32_t key[4], uint32_t pixel, uint32_t sample, uint32_t bounce,
                                     uint32_t purpose, uint32_t out[4]) {
    draw_block(key, pixel, sample, bounce, purpose, out);
}
ORACLE_EXPORT void oracle_uniforms(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                   double out[2]) {
    uniforms2(seed, c0, c1, c2, c3, out);
}
ORACLE_EXPORT void oracle_unit_vector(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce,
                                      double out[3]) {
    rngkey k = make_rngkey(seed, pixel, sample);
    vec3 v = random_unit_vector(k, bounce);
    out[0] = v.x; out[1] = v.y; out[2] = v.z;
}
ORACLE_EXPORT void oracle_in_disc(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t which, double radius,
                                  double out[2]) {
    rngkey k = make_rngkey(seed, pixel, sample);
    in_disc(k, (int)which, radius, &out[0], &out[1]);
}
ORACLE_EXPORT void oracle_sincos_2pi(double u, double out[2]) { sincos_2pi(u, &out[0], &out[1]); }
ORACLE_EXPORT void oracle_reflect(const double v[3], const double n[3], double out[3]) {
    vec3 r = reflect(V(v[0], v[1], v[2]), V(n[0], n[1], n[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
ORACLE_EXPORT void oracle_refract(const double uv[3], const double n[3], double eta, double out[3]) {
    vec3 r = refract(V(uv[0], uv[1], uv[2]), V(n[0], n[1], n[2]), eta);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
ORACLE_EXPORT double oracle_reflectance(double cosine, double ref_idx) { return reflectance(cosine, ref_idx); }
ORACLE_EXPORT int oracle_near_zero(const double v[3]) { return near_zero(V(v[0], v[1], v[2])); }
ORACLE_EXPORT void oracle_unit(const double v[3], double out[3]) {
    vec3 r = unit(V(v[0], v[1], v[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* Camera.GetRay (ray/camera.go:113-142) with explicit sub-pixel offsets; the
 * lens draw (if Aperture > 0) is keyed on (seed, pixel, sample). */
ORACLE_EXPORT void oracle_get_ray(const o_camera *cam, uint64_t seed, uint32_t pixel, uint32_t sample, double px,
                                  double py, double ox, double oy, double origin[3], double dir[3]) {
    rngkey k = make_rngkey(seed, pixel, sample);
    ray r = get_ray(cam, k, px, py, ox, oy);
    origin[0] = r.origin.x; origin[1] = r.origin.y; origin[2] = r.origin.z;
    dir[0] = r.dir.x; dir[1] = r.dir.y; dir[2] = r.dir.z;
}

/* Sphere.Hit with an explicit interval. rec = point[3], normal[3], t, front_face. */
ORACLE_EXPORT int oracle_sphere_hit(const o_sphere *s, const double origin[3], const double dir[3], double t_start,
                                    double t_end, double rec[8]) {
    ray r = {V(origin[0], origin[1], origin[2]), V(dir[0], dir[1], dir[2])};
    hit_record hr;
    int hit = sphere_hit(s, 0, &r, t_start, t_end, &hr);
    if (hit) {
        rec[0] = hr.point.x; rec[1] = hr.point.y; rec[2] = hr.point.z;
        rec[3] = hr.normal.x; rec[4] = hr.normal.y; rec[5] = hr.normal.z;
        rec[6] = hr.t; rec[7] = hr.front_face;
    }
    return hit;
}

/* Scene.Hit over a sphere list; returns hit index or -1. */
ORACLE_EXPORT int oracle_scene_hit(const o_sphere *spheres, int n, const double origin[3], const double dir[3],
                                   double t_start, double t_end, double rec[8]) {
    scene sc = {spheres, n, V(0, 0, 0), V(0, 0, 0)};
    ray r = {V(origin[0], origin[1], origin[2]), V(dir[0], dir[1], dir[2])};
    hit_record hr;
    if (!scene_hit(&sc, &r, t_start, t_end, &hr)) return -1;
    rec[0] = hr.point.x; rec[1] = hr.point.y; rec[2] = hr.point.z;
    rec[3] = hr.normal.x; rec[4] = hr.normal.y; rec[5] = hr.normal.z;
    rec[6] = hr.t; rec[7] = hr.front_face;
    return hr.mat;
}

/* Material.Scatter for one hit record (ray/materials_test.go). Returns 1/0/-2;
 * att[3], sc_origin[3], sc_dir[3]. */
ORACLE_EXPORT int oracle_scatter(const o_sphere *s, const double in_origin[3], const double in_dir[3],
                                 const double point[3], const double normal[3], int front_face, uint64_t seed,
                                 uint32_t pixel, uint32_t sample, uint32_t bounce, double att[3], double sc_origin[3],
                                 double sc_dir[3]) {
    scene sc = {s, 1, V(0, 0, 0), V(0, 0, 0)};
    ray r = {V(in_origin[0], in_origin[1], in_origin[2]), V(in_dir[0], in_dir[1], in_dir[2])};
    hit_record hr;
    hr.point = V(point[0], point[1], point[2]);
    hr.normal = V(normal[0], normal[1], normal[2]);
    hr.t = 0;
    hr.mat = 0;
    hr.front_face = front_face;
    rngkey k = make_rngkey(seed, pixel, sample);
    vec3 a;
    ray out;
    int res = scatter(&sc, &r, &hr, k, bounce, &a, &out);
    if (res < 0) return -2;
    att[0] = a.x; att[1] = a.y; att[2] = a.z;
    sc_origin[0] = out.origin.x; sc_origin[1] = out.origin.y; sc_origin[2] = out.origin.z;
    sc_dir[0] = out.dir.x; sc_dir[1] = out.dir.y; sc_dir[2] = out.dir.z;
    return res;
}

/* ColorF.ToSRGBA ray/vec3.go:173-180 -> tcolor.LinearToSrgb (fortio.org/terminal
 * v0.63.4, unavailable): IEC 61966-2-1 transfer, clamped, x255 rounded half up.
 * Pinned by ray/vec3_test.go:264-289 and the sky of example.png. */
ORACLE_EXPORT uint8_t oracle_linear_to_srgb(double c) {
    if (!(c > 0.0)) return 0;
    if (c >= 1.0) return 255;
    double s = c <= 0.0031308 ? 12.92 * c : 1.055 * pow(c, 1.0 / 2.4) - 0.055;
    return (uint8_t)floor(s * 255.0 + 0.5);
}

/* oracle_linear_to_srgb over n values (test sweeps of >= 10^6 channels). */
ORACLE_EXPORT void oracle_linear_to_srgb_n(const double *c, size_t n, uint8_t *out) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_linear_to_srgb(c[i]);
}

/* ------------------------------------------------------------------ */
/* Host setup restatement: Camera.Initialize, RichScene, DefaultScene.  */
/* ------------------------------------------------------------------ */
// math.Tan of the reference's Go toolchain (Go src/math/tan.go: Cephes tan.c
// coefficients, Pi/4 in three parts, no FMA as on GOAMD64=v1). Go's toolchain
// is absent here, so this restates its published algorithm; each constant
// below matches the bit pattern Go's source gives beside it (checked by
// tests/test_abi_cpu.py). |x| >= 2^29 needs Go's Payne-Hanek reduction, which
// is not restated: libm tan serves those (no camera reaches them).
static double go_tan(double x) {
    static const double P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
    static const double Q[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7,
                                -5.38695755929454629881e7};
    const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8,
                 PI4C = 2.69515142907905952645e-15;
    if (x == 0 || x != x) return x;
    if (x - x != 0) return NAN; /* +-Inf */
    int sign = 0;
    if (x < 0) {
        x = -x;
        sign = 1;
    }
    if (x >= 536870912.0) return sign ? -tan(x) : tan(x);
    uint64_t j = (uint64_t)(x * 0x1.45f306dc9c883p+0); /* x * (4/Pi), 4/Pi rounded once as Go folds it */
    double y = (double)j;
    if (j & 1) {
        j++;
        y++;
    }
    const double z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
    const double zz = z * z;
    if (zz > 1e-14)
        y = z + z * (zz * (((P[0] * zz) + P[1]) * zz + P[2]) / ((((zz + Q[1]) * zz + Q[2]) * zz + Q[3]) * zz + Q[4]));
    else
        y = z;
    if (j & 2) y = -1 / y;
    return sign ? -y : y;
}

/* Go's math.Tan restated, for its tests. */
ORACLE_EXPORT double oracle_go_tan(double x) { return go_tan(x); }

/* Camera.Initialize ray/camera.go:43-105. `io` is updated with defaults
 * (like the Go method mutating the receiver). */
ORACLE_EXPORT void oracle_camera_initialize(o_camera_setup *io, int width, int height, o_camera *out) {
    if (io->focal_length == 0) io->focal_length = 1.0;
    if (io->vertical_fov == 0) io->vertical_fov = 90.0;
    if (io->up[0] == 0 && io->up[1] == 0 && io->up[2] == 0) { io->up[0] = 0; io->up[1] = 1; io->up[2] = 0; }
    if (io->focus_distance == 0) io->focus_distance = io->focal_length;
    vec3 pos = V(io->position[0], io->position[1], io->position[2]);
    vec3 look = V(io->look_at[0], io->look_at[1], io->look_at[2]);
    if (pos.x == 0 && pos.y == 0 && pos.z == 0 && look.x == 0 && look.y == 0 && look.z == 0) {
        io->look_at[2] = -1;
        look = V(0, 0, -1);
    }
    vec3 up = V(io->up[0], io->up[1], io->up[2]);
    vec3 view = sub(pos, look);
    if (near_zero(view)) view = V(0, 0, 1);
    vec3 w = unit(view);
    vec3 u = unit(cross(up, w));
    vec3 v = cross(w, u);
    double defocus_radius = io->aperture / 2;
    vec3 du = smul(u, defocus_radius);
    vec3 dv = smul(v, defocus_radius);
    double theta = io->vertical_fov * 0x1.1df46a2529d39p-6; /* math.Pi/180 as a Go constant */
    double viewport_h = 2.0 * io->focal_length * go_tan(theta / 2.0);
    double aspect = (double)width / (double)height;
    double viewport_w = aspect * viewport_h;
    vec3 horizontal = smul(u, viewport_w);
    vec3 vertical = smul(v, -viewport_h);
    vec3 pxv = sdiv(horizontal, (double)width);
    vec3 pyv = sdiv(vertical, (double)height);
    /* Position.Minus(a, b, c) = Sub(Position, Add(Add(a, b), c)) ray/vec3.go:44-55 */
    vec3 upper_left = sub(pos, add(add(smul(w, io->focal_length), smul(horizontal, 0.5)), smul(vertical, 0.5)));
    vec3 p00 = add(upper_left, smul(add(pxv, pyv), 0.5));
    double *dst[6] = {out->position, out->pixel00, out->pixel_x, out->pixel_y, out->defocus_u, out->defocus_v};
    vec3 src[6] = {pos, p00, pxv, pyv, du, dv};
    for (int i = 0; i < 6; ++i) { dst[i][0] = src[i].x; dst[i][1] = src[i].y; dst[i][2] = src[i].z; }
    out->aperture = io->aperture;
    out->focus_distance = io->focus_distance;
    out->focal_length = io->focal_length;
}

static void put_sphere(o_sphere *o, vec3 c, double r, int mat, vec3 albedo, double param) {
    memset(o, 0, sizeof(*o));
    o->center[0] = c.x; o->center[1] = c.y; o->center[2] = c.z;
    o->radius = r;
    o->albedo[0] = albedo.x; o->albedo[1] = albedo.y; o->albedo[2] = albedo.z;
    o->param = param;
    o->material = mat;
}

/* RichScene ray/objects.go:132-175, generalised to a grid half-extent
 * (11 = the book cover scene; 22 = the dense C5 variant). Returns the sphere
 * count, or -1 if `cap` is too small. */
ORACLE_EXPORT int oracle_rich_scene(uint64_t seed, int half_extent, o_sphere *out, int cap) {
    scene_rng rng = {seed, 0};
    int n = 0;
#define PUSH(c, r, m, alb, prm)                                                                                        \
    do {                                                                                                               \
        if (n >= cap) return -1;                                                                                       \
        put_sphere(&out[n++], c, r, m, alb, prm);                                                                      \
    } while (0)
    PUSH(V(0, -1000, 0), 1000, O_LAMBERTIAN, V(0.5, 0.5, 0.5), 0.0);
    for (int a = -half_extent; a < half_extent; ++a) {
        for (int b = -half_extent; b < half_extent; ++b) {
            double choose = scene_float64(&rng);
            double cx = (double)a + 0.9 * scene_float64(&rng);
            double cz = (double)b + 0.9 * scene_float64(&rng);
            vec3 center = V(cx, 0.2, cz);
            if (length(sub(center, V(4, 0.2, 0))) > 0.9) {
                if (choose < 0.8) {
                    /* Mul(Random(rng), Random(rng)): left argument drawn first */
                    double r1 = scene_float64(&rng), g1 = scene_float64(&rng), b1 = scene_float64(&rng);
                    double r2 = scene_float64(&rng), g2 = scene_float64(&rng), b2 = scene_float64(&rng);
                    PUSH(center, 0.2, O_LAMBERTIAN, mul(V(r1, g1, b1), V(r2, g2, b2)), 0.0);
                } else if (choose < 0.95) {
                    double ar = scene_float64_range(&rng, 0.5, 1.0);
                    double ag = scene_float64_range(&rng, 0.5, 1.0);
                    double ab = scene_float64_range(&rng, 0.5, 1.0);
                    double fuzz = scene_float64(&rng) * 0.5;
                    PUSH(center, 0.2, O_METAL, V(ar, ag, ab), fuzz);
                } else {
                    PUSH(center, 0.2, O_DIELECTRIC, V(0, 0, 0), 1.5);
                }
            }
        }
    }
    PUSH(V(0, 1, 0), 1.0, O_DIELECTRIC, V(0, 0, 0), 1.5);
    PUSH(V(-4, 1, 0), 1.0, O_LAMBERTIAN, V(0.4, 0.2, 0.1), 0.0);
    PUSH(V(4, 1, 0), 1.0, O_METAL, V(0.7, 0.6, 0.5), 0.0);
#undef PUSH
    return n;
}

/* DefaultScene ray/objects.go:112-130 */
ORACLE_EXPORT int oracle_default_scene(o_sphere *out, int cap) {
    if (cap < 5) return -1;
    put_sphere(&out[0], V(0, 0, -1.2), 0.5, O_LAMBERTIAN, V(0.1, 0.2, 0.5), 0.0);
    put_sphere(&out[1], V(0, -100.5, -1), 100, O_LAMBERTIAN, V(0.7, 0.8, 0.1), 0.0);
    put_sphere(&out[2], V(-1.0, 0, -1), 0.5, O_DIELECTRIC, V(0, 0, 0), 1.5);
    put_sphere(&out[3], V(-1.0, 0, -1), 0.4, O_DIELECTRIC, V(0, 0, 0), 1.0 / 1.5);
    put_sphere(&out[4], V(1.0, 0, -1), 0.5, O_METAL, V(1, .8, .8), 0.05);
    return 5;
}

/* ------------------------------------------------------------------ */
/* Terminal view downscale: main.go:119-128.   */
/* ------------------------------------------------------------------ */
/*
 * main.go:121-128 scales the rendered *image.RGBA into a fresh image.NewRGBA
 * (all zeros) of the terminal's size with draw.NearestNeighbor.Scale
 * (supersample < 1) or draw.BiLinear.Scale (supersample > 1), op draw.Over.
 * Both live in golang.org/x/image v0.35.0 (go.mod:11), which is NOT vendored
 * in the reference: this restates the published algorithm of its draw package
 * (scale.go: Kernel, newDistrib, kernelScaler.Scale; impl.go: the generated
 * scaleX_RGBA / scaleY_RGBA_Over and nnInterpolator scale_RGBA_RGBA_Over for
 * an *image.RGBA source and destination) in Go's op order, FP64, no FMA
 * (GOAMD64=v1; Go on arm64 may fuse `a*b + c`). Parity with the library
 * itself is UNPINNED (neither the module nor a fixture is in the tree).
 * Images are RGBA8, row pitch 4*width; dst is blended onto (Over), as Go does.
 */
typedef struct {
    int32_t i, j;             /* contribs[i..j) */
    double inv_total;         /* 1 / total weight */
    double inv_total_ffff;    /* (1 / total weight) / 0xffff */
} o_source;
typedef struct {
    int32_t coord;
    double weight;
} o_contrib;

/* BiLinear = &Kernel{Support: 1, At: func(t) { return 1 - t }}; newDistrib(q, dw, sw). */
static int bilinear_distrib(int32_t dw, int32_t sw, o_source *sources, o_contrib *contribs, int32_t cap) {
    const double support = 1.0;
    const double scale = (double)sw / (double)dw;
    double half_width = support, arg_scale = 1.0;
    if (scale > 1) { /* shrinking: widen the support to visit every source pixel */
        half_width *= scale;
        arg_scale = 1 / scale;
    }
    int32_t n = 0;
    for (int32_t x = 0; x < dw; ++x) {
        const double center = ((double)x + 0.5) * scale - 0.5;
        int32_t i = (int32_t)floor(center - half_width);
        if (i < 0) i = 0;
        int32_t j = (int32_t)ceil(center + half_width);
        if (j > sw) {
            j = sw;
            if (j < i) j = i;
        }
        double total = 0.0;
        const int32_t l = n;
        for (int32_t coord = i; coord < j; ++coord) {
            const double t = fabs((center - (double)coord) * arg_scale);
            if (t >= support) continue;
            const double w = 1 - t;
            if (w == 0) continue;
            if (n >= cap) return -1;
            total += w;
            contribs[n].coord = coord;
            contribs[n].weight = w;
            ++n;
        }
        total = 1 / total;
        sources[x].i = l;
        sources[x].j = n;
        sources[x].inv_total = total;
        sources[x].inv_total_ffff = total / 0xffff;
    }
    return n;
}

/* ftou (x/image/draw scale.go): int32(0xffff*f + 0.5) clamped to [0, 0xffff]. */
static uint32_t go_ftou(double f) {
    const double v = 0xffff * f + 0.5;
    int32_t i;
    if (!(v < 2147483648.0)) i = INT32_MAX; /* Go's int32(x) of a large float is implementation-defined; */
    else if (!(v > -2147483649.0)) i = INT32_MIN; /* clamping keeps the result in range either way */
    else i = (int32_t)v;
    if (i > 0xffff) return 0xffff;
    if (i > 0) return (uint32_t)i;
    return 0;
}

static void over_px(uint8_t *d, uint32_t r, uint32_t g, uint32_t b, uint32_t a) {
    const uint32_t a1 = (0xffff - a) * 0x101;
    d[0] = (uint8_t)(((uint32_t)d[0] * a1 / 0xffff + r) >> 8);
    d[1] = (uint8_t)(((uint32_t)d[1] * a1 / 0xffff + g) >> 8);
    d[2] = (uint8_t)(((uint32_t)d[2] * a1 / 0xffff + b) >> 8);
    d[3] = (uint8_t)(((uint32_t)d[3] * a1 / 0xffff + a) >> 8);
}

/* draw.BiLinear.Scale(dst, dst.Bounds(), src, src.Bounds(), draw.Over, nil). Returns 0, or -1. */
ORACLE_EXPORT int oracle_scale_bilinear_rgba(const uint8_t *src, int32_t sw, int32_t sh, uint8_t *dst, int32_t dw,
                                             int32_t dh) {
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return -1;
    /* every destination pixel takes at most ceil(2 * max(scale, 1)) + 1 taps */
    const int32_t capx = dw * (2 * (sw / dw + 2) + 2), capy = dh * (2 * (sh / dh + 2) + 2);
    o_source *hs = malloc(sizeof(o_source) * (size_t)dw), *vs = malloc(sizeof(o_source) * (size_t)dh);
    o_contrib *hc = malloc(sizeof(o_contrib) * (size_t)capx), *vc = malloc(sizeof(o_contrib) * (size_t)capy);
    double *tmp = malloc(sizeof(double) * 4 * (size_t)dw * (size_t)sh);
    int rc = -1;
    if (!hs || !vs || !hc || !vc || !tmp) goto out;
    if (bilinear_distrib(dw, sw, hs, hc, capx) < 0 || bilinear_distrib(dh, sh, vs, vc, capy) < 0) goto out;
    /* scaleX_RGBA: the source's columns distributed over tmp [sh][dw] */
    for (int32_t y = 0; y < sh; ++y) {
        for (int32_t x = 0; x < dw; ++x) {
            double pr = 0, pg = 0, pb = 0, pa = 0;
            for (int32_t k = hs[x].i; k < hs[x].j; ++k) {
                const uint8_t *p = src + ((size_t)y * (size_t)sw + (size_t)hc[k].coord) * 4;
                pr += (double)((uint32_t)p[0] * 0x101) * hc[k].weight;
                pg += (double)((uint32_t)p[1] * 0x101) * hc[k].weight;
                pb += (double)((uint32_t)p[2] * 0x101) * hc[k].weight;
                pa += (double)((uint32_t)p[3] * 0x101) * hc[k].weight;
            }
            double *t = tmp + ((size_t)y * (size_t)dw + (size_t)x) * 4;
            t[0] = pr * hs[x].inv_total_ffff;
            t[1] = pg * hs[x].inv_total_ffff;
            t[2] = pb * hs[x].inv_total_ffff;
            t[3] = pa * hs[x].inv_total_ffff;
        }
    }
    /* scaleY_RGBA_Over: tmp's rows distributed over dst, blended Over */
    for (int32_t x = 0; x < dw; ++x) {
        for (int32_t y = 0; y < dh; ++y) {
            double pr = 0, pg = 0, pb = 0, pa = 0;
            for (int32_t k = vs[y].i; k < vs[y].j; ++k) {
                const double *t = tmp + ((size_t)vc[k].coord * (size_t)dw + (size_t)x) * 4;
                pr += t[0] * vc[k].weight;
                pg += t[1] * vc[k].weight;
                pb += t[2] * vc[k].weight;
                pa += t[3] * vc[k].weight;
            }
            if (pr > pa) pr = pa;
            if (pg > pa) pg = pa;
            if (pb > pa) pb = pa;
            over_px(dst + ((size_t)y * (size_t)dw + (size_t)x) * 4, go_ftou(pr * vs[y].inv_total),
                    go_ftou(pg * vs[y].inv_total), go_ftou(pb * vs[y].inv_total), go_ftou(pa * vs[y].inv_total));
        }
    }
    rc = 0;
out:
    free(hs);
    free(vs);
    free(hc);
    free(vc);
    free(tmp);
    return rc;
}

/* draw.NearestNeighbor.Scale(dst, dst.Bounds(), src, src.Bounds(), draw.Over, nil):
 * source pixel ((2 dx + 1) sw / (2 dw), (2 dy + 1) sh / (2 dh)) in integers. */
ORACLE_EXPORT int oracle_scale_nearest_rgba(const uint8_t *src, int32_t sw, int32_t sh, uint8_t *dst, int32_t dw,
                                            int32_t dh) {
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0) return -1;
    const uint64_t dw2 = (uint64_t)dw * 2, dh2 = (uint64_t)dh * 2;
    for (int32_t dy = 0; dy < dh; ++dy) {
        const uint64_t sy = (2 * (uint64_t)dy + 1) * (uint64_t)sh / dh2;
        for (int32_t dx = 0; dx < dw; ++dx) {
            const uint64_t sx = (2 * (uint64_t)dx + 1) * (uint64_t)sw / dw2;
            const uint8_t *p = src + ((size_t)sy * (size_t)sw + (size_t)sx) * 4;
            over_px(dst + ((size_t)dy * (size_t)dw + (size_t)dx) * 4, (uint32_t)p[0] * 0x101, (uint32_t)p[1] * 0x101,
                    (uint32_t)p[2] * 0x101, (uint32_t)p[3] * 0x101);
        }
    }
    return 0;
}
