// tray_host.cpp — host-side setup of the C-ABI: the parts of fortio/tray that
// stay on the CPU around the kernel (camera basis, scene generators, sRGB sink).
//
//   Camera.Initialize   ray/camera.go:43-105
//   RichSceneCamera     ray/camera.go:144-154
//   DefaultBackground   ray/objects.go:106-110
//   DefaultScene        ray/objects.go:112-130
//   RichScene           ray/objects.go:132-175 (draws from the counter RNG, purpose 4)
//   ColorF.ToSRGBA      ray/vec3.go:173-180
//
// Compiled with -ffp-contract=off so the camera vectors have the reference's
// op order bit for bit (they feed every primary ray).

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <array>

#include "../../include/tray.h"
#include "rng.hpp"
#include "tray_internal.hpp"

namespace {

using Vec = std::array<double, 3>;

Vec vadd(const Vec& u, const Vec& v) { return {v[0] + u[0], v[1] + u[1], v[2] + u[2]}; }  // Add: v + u
Vec vsub(const Vec& u, const Vec& v) { return {u[0] - v[0], u[1] - v[1], u[2] - v[2]}; }
Vec vscale(const Vec& v, double t) { return {v[0] * t, v[1] * t, v[2] * t}; }
Vec vdivs(const Vec& v, double t) { return {v[0] / t, v[1] / t, v[2] / t}; }
Vec vmul(const Vec& u, const Vec& v) { return {u[0] * v[0], u[1] * v[1], u[2] * v[2]}; }
double vlen_sq(const Vec& v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; }
double vlen(const Vec& v) { return sqrt(vlen_sq(v)); }
Vec vunit(const Vec& v) {
    const double l = vlen(v);
    return {v[0] / l, v[1] / l, v[2] / l};
}
Vec vcross(const Vec& u, const Vec& v) {
    return {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
}
bool vnear_zero(const Vec& v) {
    return fabs(v[0]) < 1e-8 && fabs(v[1]) < 1e-8 && fabs(v[2]) < 1e-8;
}
bool vis_zero(const double* v) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }
Vec load(const double* v) { return {v[0], v[1], v[2]}; }
void store(double* dst, const Vec& v) {
    dst[0] = v[0];
    dst[1] = v[1];
    dst[2] = v[2];
}

void set_sphere(tray_sphere* s, const Vec& c, double r, int32_t mat, const Vec& albedo, double param) {
    memset(s, 0, sizeof(*s));
    store(s->center, c);
    s->radius = r;
    store(s->albedo, albedo);
    s->param = param;
    s->material = mat;
}

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

// Sequential draws of the scene-generation stream (counter RNG purpose 4).
struct SceneStream {
    uint64_t seed;
    uint32_t next = 0;
    double float64() { return tray::philox_uniforms(seed, next++, 0u, 0u, tray::kPurposeScene << 24).u0; }
    double range(double lo, double hi) { return lo + (hi - lo) * float64(); }
};

}  // namespace

namespace tray {

// tcolor.LinearToSrgb (fortio.org/terminal v0.63.4, not vendored): IEC 61966-2-1
// transfer, clamped, x255 rounded half up; pinned by ray/vec3_test.go:264-289
// and the sky rows of the reference's example.png.
uint8_t srgb8(double c) {
    if (!(c > 0.0)) return 0;
    if (c >= 1.0) return 255;
    const double s = c <= 0.0031308 ? 12.92 * c : 1.055 * pow(c, 1.0 / 2.4) - 0.055;
    return (uint8_t)floor(s * 255.0 + 0.5);
}

// Bisection over the bit patterns of the doubles in [0, 1] (ordered like their
// values): srgb8(0) = 0 < k and srgb8(1) = 255 >= k bracket every threshold.
static void build_srgb_thresholds(double* t) {
    t[0] = 0.0;
    for (int k = 1; k < 256; ++k) {
        uint64_t lo = 0, hi = 0x3FF0000000000000ull;  // bits of 0.0 and 1.0
        while (hi - lo > 1) {
            const uint64_t mid = lo + (hi - lo) / 2;
            double c;
            memcpy(&c, &mid, sizeof(c));
            if (srgb8(c) >= k) hi = mid;
            else lo = mid;
        }
        memcpy(&t[k], &hi, sizeof(double));
    }
}

const double* srgb_thresholds() {
    static double table[256];
    static const bool built = (build_srgb_thresholds(table), true);
    (void)built;
    return table;
}

}  // namespace tray

namespace {
using tray::srgb8;
}  // namespace

extern "C" {
#pragma GCC visibility push(default)

int tray_camera_initialize(tray_camera_setup* c, int32_t width, int32_t height, tray_camera* out) {
    if (!c || !out) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    if (width <= 0 || height <= 0) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "width/height must be > 0");
    if (c->focal_length == 0) c->focal_length = 1.0;
    if (c->vertical_fov == 0) c->vertical_fov = 90.0;
    if (vis_zero(c->up)) store(c->up, Vec{0, 1, 0});
    if (c->focus_distance == 0) c->focus_distance = c->focal_length;
    if (vis_zero(c->position) && vis_zero(c->look_at)) store(c->look_at, Vec{0, 0, -1});
    const Vec position = load(c->position);
    Vec view = vsub(position, load(c->look_at));
    if (vnear_zero(view)) view = Vec{0, 0, 1};
    const Vec w = vunit(view);
    const Vec u = vunit(vcross(load(c->up), w));
    const Vec v = vcross(w, u);
    const double defocus_radius = c->aperture / 2;
    // math.Pi/180 is folded by Go at arbitrary precision: the correctly rounded double.
    const double theta = c->vertical_fov * 0x1.1df46a2529d39p-6;
    const double viewport_h = 2.0 * c->focal_length * go_tan(theta / 2.0);
    const double aspect = (double)width / (double)height;
    const double viewport_w = aspect * viewport_h;
    const Vec horizontal = vscale(u, viewport_w);
    const Vec vertical = vscale(v, -viewport_h);
    const Vec px = vdivs(horizontal, (double)width);
    const Vec py = vdivs(vertical, (double)height);
    // Position.Minus(w*f, hor*0.5, ver*0.5) = Position - ((w*f + hor*0.5) + ver*0.5)
    const Vec upper_left =
        vsub(position, vadd(vadd(vscale(w, c->focal_length), vscale(horizontal, 0.5)), vscale(vertical, 0.5)));
    const Vec p00 = vadd(upper_left, vscale(vadd(px, py), 0.5));
    store(out->position, position);
    store(out->pixel00, p00);
    store(out->pixel_x, px);
    store(out->pixel_y, py);
    store(out->defocus_u, vscale(u, defocus_radius));
    store(out->defocus_v, vscale(v, defocus_radius));
    out->aperture = c->aperture;
    out->focus_distance = c->focus_distance;
    out->focal_length = c->focal_length;
    return TRAY_OK;
}

int tray_rich_scene_camera(tray_camera_setup* out) {
    if (!out) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof(*out));
    store(out->position, Vec{13, 2, 3});
    store(out->look_at, Vec{0, 0, 0});
    store(out->up, Vec{0, 1, 0});
    out->vertical_fov = 20.0;
    out->aperture = 0.1;
    out->focal_length = 10.0;
    out->focus_distance = 10.0;
    return TRAY_OK;
}

int tray_default_background(tray_background* out) {
    if (!out) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    store(out->color_a, Vec{1.0, 1.0, 1.0});
    store(out->color_b, Vec{0.4, 0.65, 1.0});
    return TRAY_OK;
}

int tray_default_scene(tray_sphere* out, int32_t capacity, int32_t* count) {
    if (!out || !count) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    if (capacity < 5) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "capacity < 5");
    set_sphere(&out[0], {0, 0, -1.2}, 0.5, TRAY_LAMBERTIAN, {0.1, 0.2, 0.5}, 0);       // center
    set_sphere(&out[1], {0, -100.5, -1}, 100, TRAY_LAMBERTIAN, {0.7, 0.8, 0.1}, 0);    // ground
    set_sphere(&out[2], {-1.0, 0, -1}, 0.5, TRAY_DIELECTRIC, {0, 0, 0}, 1.5);          // left
    set_sphere(&out[3], {-1.0, 0, -1}, 0.4, TRAY_DIELECTRIC, {0, 0, 0}, 1.0 / 1.5);    // bubble
    set_sphere(&out[4], {1.0, 0, -1}, 0.5, TRAY_METAL, {1, .8, .8}, 0.05);             // right
    *count = 5;
    return TRAY_OK;
}

int32_t tray_rich_scene_capacity(int32_t half_extent) {
    if (half_extent < 0) return 4;
    return 4 * half_extent * half_extent + 4;
}

int tray_rich_scene(uint64_t seed, int32_t half_extent, tray_sphere* out, int32_t capacity, int32_t* count) {
    if (!out || !count) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    if (half_extent < 0 || half_extent > 1000) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "half_extent out of range");
    SceneStream rng{seed};
    int32_t n = 0;
    auto push = [&](const Vec& c, double r, int32_t m, const Vec& albedo, double param) {
        if (n >= capacity) return false;
        set_sphere(&out[n++], c, r, m, albedo, param);
        return true;
    };
    bool ok = push({0, -1000, 0}, 1000, TRAY_LAMBERTIAN, {0.5, 0.5, 0.5}, 0);
    for (int32_t a = -half_extent; ok && a < half_extent; ++a) {
        for (int32_t b = -half_extent; ok && b < half_extent; ++b) {
            const double choose = rng.float64();
            const double cx = (double)a + 0.9 * rng.float64();  // Go evaluates the literal left to right
            const double cz = (double)b + 0.9 * rng.float64();
            const Vec center{cx, 0.2, cz};
            if (vlen(vsub(center, Vec{4, 0.2, 0})) > 0.9) {
                if (choose < 0.8) {
                    const double r1 = rng.float64(), g1 = rng.float64(), b1 = rng.float64();
                    const double r2 = rng.float64(), g2 = rng.float64(), b2 = rng.float64();
                    ok = push(center, 0.2, TRAY_LAMBERTIAN, vmul(Vec{r1, g1, b1}, Vec{r2, g2, b2}), 0);
                } else if (choose < 0.95) {
                    const double ar = rng.range(0.5, 1.0), ag = rng.range(0.5, 1.0), ab = rng.range(0.5, 1.0);
                    const double fuzz = rng.float64() * 0.5;
                    ok = push(center, 0.2, TRAY_METAL, {ar, ag, ab}, fuzz);
                } else {
                    ok = push(center, 0.2, TRAY_DIELECTRIC, {0, 0, 0}, 1.5);
                }
            }
        }
    }
    ok = ok && push({0, 1, 0}, 1.0, TRAY_DIELECTRIC, {0, 0, 0}, 1.5);
    ok = ok && push({-4, 1, 0}, 1.0, TRAY_LAMBERTIAN, {0.4, 0.2, 0.1}, 0);
    ok = ok && push({4, 1, 0}, 1.0, TRAY_METAL, {0.7, 0.6, 0.5}, 0.0);
    if (!ok) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "capacity too small (see tray_rich_scene_capacity)");
    *count = n;
    return TRAY_OK;
}

int tray_to_srgba(const double* rgb, size_t n_pixels, uint8_t* rgba) {
    if ((!rgb || !rgba) && n_pixels) return tray::fail(TRAY_ERR_INVALID_ARGUMENT, "null argument");
    for (size_t i = 0; i < n_pixels; ++i) {
        rgba[4 * i + 0] = srgb8(rgb[3 * i + 0]);
        rgba[4 * i + 1] = srgb8(rgb[3 * i + 1]);
        rgba[4 * i + 2] = srgb8(rgb[3 * i + 2]);
        rgba[4 * i + 3] = 255;
    }
    return TRAY_OK;
}

#pragma GCC visibility pop
}  // extern "C"
