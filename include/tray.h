/*
 * tray.h — C-ABI of the MI355X-native renderer for fortio/tray's per-pixel
 * path-tracing loop.
 *
 * Drop-in seam: the Go API `(*ray.Tracer).Render(scene *ray.Scene) *image.RGBA`
 * (ray/tracer.go:48) and `(*ray.Tracer).RenderLines(idx, yStart, yEnd, scene)`
 * (ray/tracer.go:120). The reference has no FFI of its own (pure Go, no cgo), so
 * each entry point below names the Go function/method whose work it replaces and
 * INTEGRATION.md shows the cgo stub a maintainer would add to `ray/`.
 *
 * Rules (cgo-clean):
 *   - plain C types only; no C++ exceptions cross this boundary;
 *   - every caller buffer is caller-owned and is never retained after return;
 *   - device-side state (uploaded scenes) is library-owned, released by
 *     tray_scene_release()/tray_shutdown();
 *   - every function returns TRAY_OK (0) or a negative tray_status; the message
 *     of the last failure on the calling thread is tray_last_error().
 *
 * Arithmetic contract: all geometry and shading is IEEE FP64 evaluated in the
 * reference's op order with no FMA contraction (ray/vec3.go, ray/objects.go,
 * ray/materials.go, ray/camera.go). Division and sqrt are correctly rounded.
 *
 * Counter RNG contract (replaces fortio.org/rand v1.1.0, go.mod:9, which is not
 * vendored). Philox4x32-10 (Salmon et al. 2011, Random123 constants), keyed by
 * (seed & 0xffffffff, seed >> 32), gives
 *     the draw key  (k0, k1, k2, k3) = Philox(ctr = (0, 0, 0, 5 << 24))
 *     host scene generation: ctr = (draw_index, 0, 0, 4 << 24),
 *                 Float64 = ((x1 << 32 | x0) >> 11) * 2^-53
 * Every renderer draw comes from one DRAW BLOCK (ABI 6; ABI 5 used a Philox
 * block here, ~7.6 % of the frame): pcg4d (Jarzynski & Olano, "Hash Functions
 * for GPU Rendering", JCGT 9(3), 2020) of the keyed counter, then an xorshift:
 *     v = (pixel ^ k0, sample ^ k1, bounce ^ k2, purpose ^ k3)
 *     v = v * 1664525 + 1013904223                        (each word, mod 2^32)
 *     twice: v0 += v1*v3; v1 += v2*v0; v2 += v0*v1; v3 += v1*v2; v ^= v >> 16
 *     pixel = y * width + x in GLOBAL image coordinates (tiling-independent)
 *     purpose 1 = the sample's camera block (bounce = 0): words 0,1 feed the
 *                 anti-aliasing disc (ray/tracer.go:138), words 2,3 the lens
 *                 disc (ray/camera.go:128)
 *     purpose 3 = the scatter block of hit number `bounce` (ray/materials.go:14,31,57)
 * Renderer uniforms are ui = xi * 2^-32 in [0,1). Samplers (no rejection loops):
 *     InDisc(r)   = (sqrt(ua) * cos(2 pi ub) * r, sqrt(ua) * sin(2 pi ub) * r)
 *     UnitVector  = z = 1 - 2 u0, s = sqrt(1 - z*z), (s cos(2 pi u1), s sin(2 pi u1), z)
 *     Float64     = u0 of the scatter block (Dielectric, ray/materials.go:57)
 * where sin/cos(2 pi u) is "sincos2pi": quadrant q = floor(4u), f = 4u - q
 * reflected into [0, 0.5] (exact, FP64), then in FP32: t = RN32(f) * RN32(pi/2),
 * Taylor polynomials in t^2 of degree 9 (sin) and 10 (cos) by Horner's rule
 * with correctly rounded fmaf; back in FP64 one Newton step onto the unit
 * circle, k = 1.5 - 0.5 (s^2 + c^2), (s, c) *= k, then the quadrant rotation
 * (tray_amd/csrc/rng.hpp). The angle is accurate to ~1e-7, the length s^2 + c^2
 * to ~1e-14. IEEE FP32 with fmaf, in a fixed
 * order, gives identical bits on the host oracle and the device. (FP32 and
 * fma appear only in this sampler transform; the reference arithmetic of
 * ray/vec3.go, objects.go, materials.go and camera.go is FP64, uncontracted.)
 * A given (seed, pixel, sample) therefore renders the same colour for any
 * tiling, row range, device count or launch geometry.
 */
#ifndef TRAY_H
#define TRAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRAY_ABI_VERSION 6 /* 2: tray_render_devices_progress, tray_release_cache; 3: tray_render_plan_get;
                              4: TRAY_FLAG_ORDERED_SUM (the library no longer reads the process environment);
                              5: a scene handle may be rendered on several streams at once (launch contexts);
                              6: renderer draws from the keyed pcg4d draw block (other pixels than ABI 5) */

typedef enum tray_status {
    TRAY_OK = 0,
    TRAY_ERR_INVALID_ARGUMENT = -1, /* bad sizes, null pointers, row range outside the image */
    TRAY_ERR_UNSUPPORTED = -2,      /* object/material kind not representable (ray/objects.go:28-30) */
    TRAY_ERR_DEVICE = -3,           /* HIP runtime failure */
    TRAY_ERR_NO_DEVICE = -4,        /* no gfx950 device visible */
    TRAY_ERR_TOO_LARGE = -5         /* scene or image exceeds a device limit */
} tray_status;

/* Material kinds: ray/materials.go:9 Lambertian, :23 Metal, :40 Dielectric. */
typedef enum tray_material {
    TRAY_LAMBERTIAN = 1,
    TRAY_METAL = 2,
    TRAY_DIELECTRIC = 3
} tray_material;

/* One *ray.Sphere with its Material (ray/objects.go:75-79). 72 bytes. */
typedef struct tray_sphere {
    double center[3];
    double radius;
    double albedo[3]; /* Lambertian.Albedo / Metal.Albedo; ignored for Dielectric */
    double param;     /* Metal.Fuzz / Dielectric.RefIdx; ignored for Lambertian */
    int32_t material; /* tray_material */
    int32_t reserved; /* must be 0 */
} tray_sphere;

/* ray.AmbientLight (ray/objects.go:64-66): ColorA at the nadir blend end, ColorB at the zenith. */
typedef struct tray_background {
    double color_a[3];
    double color_b[3];
} tray_background;

/* Public fields of ray.Camera (ray/camera.go:9-33). */
typedef struct tray_camera_setup {
    double position[3];
    double look_at[3];
    double up[3];
    double vertical_fov;
    double focal_length;
    double focus_distance;
    double aperture;
} tray_camera_setup;

/* Camera state after Camera.Initialize (ray/camera.go:34-39 computed fields). */
typedef struct tray_camera {
    double position[3];
    double pixel00[3];
    double pixel_x[3]; /* pixelXVector */
    double pixel_y[3]; /* pixelYVector */
    double defocus_u[3];
    double defocus_v[3];
    double aperture;
    double focus_distance;
    double focal_length;
} tray_camera;

/* Output pixel formats. */
typedef enum tray_output {
    TRAY_OUT_RGB_F64 = 0, /* linear mean colour, 3 x double per pixel (parity format) */
    TRAY_OUT_RGB_F32 = 1, /* linear mean colour rounded to float, 3 x float per pixel */
    TRAY_OUT_RGBA8 = 2    /* ColorF.ToSRGBA (ray/vec3.go:173-180) fused on device, A = 255; the same bytes
                             as tray_to_srgba of the TRAY_OUT_RGB_F64 frame */
} tray_output;

/* Tracer fields (ray/tracer.go:25-36) after Render's defaulting (:64-79), plus
 * the set of image rows this call renders.
 *
 * Row set: rows y in [y_start, y_end). With tile_rows > 0 the set is further
 * restricted to row tiles owned by this shard: y is rendered iff
 * ((y - y_start) / tile_rows) % tile_count == tile_index (interleaved row tiles
 * for multi-GPU sharding). Output rows are COMPACT: the i-th rendered row is
 * written at row i of the output buffer (row pitch = width pixels). */
typedef struct tray_params {
    int32_t width;
    int32_t height;
    int32_t max_depth;      /* Tracer.MaxDepth, > 0 */
    int32_t rays_per_pixel; /* Tracer.NumRaysPerPixel, > 0 */
    double ray_radius;      /* Tracer.RayRadius (AA disc radius in pixels) */
    uint64_t seed;          /* Tracer.Seed (0 is a valid fixed seed here; the Go "0 = random" is host policy) */
    int32_t y_start;
    int32_t y_end;
    int32_t tile_rows;  /* 0 = every row of [y_start, y_end) */
    int32_t tile_count; /* >= 1 when tile_rows > 0 */
    int32_t tile_index; /* 0 <= tile_index < tile_count */
    int32_t output;     /* tray_output */
    int32_t flags;      /* TRAY_FLAG_* */
    int32_t pass;       /* progressive pass, >= 0: sample s of a pixel uses the counter RNG's sample
                           word pass * rays_per_pixel + s, so passes 0, 1, ... are independent frames
                           of the same pixels (0: the single frame of Tracer.Render) */
} tray_params;

/* Force the reference-order linear scan over all spheres (Scene.Hit,
 * ray/objects.go:37-46) instead of the exact-culling BVH. Both give identical
 * results; the flag exists for verification and A/B timing. */
#define TRAY_FLAG_LINEAR_SCAN 1

/* Pixel sums. DEFAULT (flag clear): when rays_per_pixel is a multiple of 64, or
 * 16 or 32, and the scene's colour bound allows it, each pixel's samples are summed exactly
 * as fixed-point integers of 2^-k (k >= 44), so the mean is within 2^-(k+1) of
 * the exact mean of the sample colours and does not depend on the order in
 * which samples finish (tray_render_plan_get reports k; C2: k = 46, L-inf
 * 6.7e-15 against the sequential FP64 sum). With TRAY_FLAG_ORDERED_SUM the
 * samples are added in sample order in FP64, exactly as Go's RenderLines
 * accumulates colorSum (ray/tracer.go:143), at the cost of a 24-B per-sample
 * device buffer. Renders with any other r always use the ordered sum. Both are far inside the 1e-4 parity gate; the flag selects the
 * bits. */
#define TRAY_FLAG_ORDERED_SUM 2

typedef struct tray_scene_s *tray_scene_t;

/* ---- discovery / lifetime ------------------------------------------------ */
int32_t tray_abi_version(void);
const char *tray_last_error(void);
/* Number of usable gfx950 devices (0 when none). */
int tray_device_count(int32_t *count);
/* Free every library-owned device buffer on every device, and the pinned host
 * buffers tray_scale_rgba* staged its tap tables in. */
int tray_shutdown(void);
/* Free what the synchronous entry points (tray_render, tray_render_progress,
 * tray_render_devices*) keep on `device` (every device when device < 0): per
 * render slot, the last uploaded scene with its sample buffer (24 B per sample
 * of a launch band: up to ~25.8 GB at 2^30 samples, e.g. a 3840x2160 r=1024
 * band; with on-chip chunk sums 32 B per 64 samples, up to 1 GB at 2^31) and candidate records, the output workspaces, the stream and the
 * progress counters. A device listed k times in one tray_render_devices call
 * keeps k slots. Long-lived callers that share the device with other users call
 * this between renders; the next synchronous render re-uploads. Scenes from
 * tray_scene_upload are the caller's and are not touched. No reference
 * counterpart (Go's Render allocates per call, ray/tracer.go:38-45). */
int tray_release_cache(int32_t device);

/* ---- host-side setup (ray/camera.go, ray/objects.go) ------------------------ */
/* Camera.Initialize (ray/camera.go:43-105): applies zero-field defaults to
 * *setup in place (as the Go method mutates its receiver) and writes *out. */
int tray_camera_initialize(tray_camera_setup *setup, int32_t width, int32_t height, tray_camera *out);
/* RichSceneCamera (ray/camera.go:144-154). */
int tray_rich_scene_camera(tray_camera_setup *out);
/* DefaultBackground (ray/objects.go:106-110). */
int tray_default_background(tray_background *out);
/* DefaultScene (ray/objects.go:112-130): writes 5 spheres. */
int tray_default_scene(tray_sphere *out, int32_t capacity, int32_t *count);
/* RichScene (ray/objects.go:132-175) drawn from the counter RNG stream
 * (purpose 4). half_extent = 11 is the book-cover grid; larger values give the
 * dense variant used for the ~2000-sphere config. */
int tray_rich_scene(uint64_t seed, int32_t half_extent, tray_sphere *out, int32_t capacity, int32_t *count);
/* Upper bound of spheres tray_rich_scene can produce for half_extent. */
int32_t tray_rich_scene_capacity(int32_t half_extent);

/* ---- the hot path -------------------------------------------------------------- */
/* Synchronous drop-in for Tracer.RenderLines (ray/tracer.go:120-155) over the
 * row set in *params: uploads the scene (or reuses the device's copy of the same
 * scene, see tray_render_progress), renders on `device`, and copies the
 * compact rows into caller-owned host memory `out` (size: rows x width x
 * bytes-per-pixel of params->output). `segments_out` (nullable) receives the
 * per-pixel count of Scene.Hit calls summed over samples (uint32). */
int tray_render(const tray_sphere *spheres, int32_t n_spheres, const tray_background *background,
                const tray_camera *camera, const tray_params *params, int32_t device, void *out,
                uint32_t *segments_out);

/* Live progress of a synchronous render (Tracer.ProgressFunc, called per row
 * while rendering, ray/tracer.go:126-128): `rows` more rows of the row set have
 * all their samples finished. Called on the thread that called
 * tray_render_progress / tray_render_devices_progress, before it returns; the
 * rows sum to the row count.
 * The callback runs while the render holds its devices: it must not call back
 * into this library's synchronous entry points (tray_render*, tray_shutdown,
 * tray_release_cache, tray_linear_to_srgba_async), which then fail with
 * TRAY_ERR_INVALID_ARGUMENT instead of deadlocking. Keep it short (a Go
 * callback should only bump a counter, as ray/tracer_test.go:174-176 does). */
typedef void (*tray_progress_fn)(int32_t rows, void *user);

/* tray_render with live progress: the device counts finished samples per 8-row
 * tile row and the calling thread polls the counters (every ~0.5 ms) while the
 * launch runs, calling progress(rows, user) as tile rows complete. progress may
 * be NULL (then this is tray_render). The synchronous entry points keep the
 * last scene they uploaded on each device (with its sample buffer) and reuse it
 * while the caller passes identical spheres and background (compared byte for
 * byte); tray_release_cache(device) or tray_shutdown() releases it. */
int tray_render_progress(const tray_sphere *spheres, int32_t n_spheres, const tray_background *background,
                         const tray_camera *camera, const tray_params *params, int32_t device, void *out,
                         uint32_t *segments_out, tray_progress_fn progress, void *user);

/* tray_render over several devices of this process (the one-process form of
 * the multi-GPU row split): row y of the row set goes to devices[(y - y_start)
 * % n_devices] (interleaved 1-row tiles, as bench.py --gpus N splits a frame),
 * every device renders its rows concurrently, and the rows land in `out` in
 * image order (compact from y_start, exactly as tray_render writes them). A
 * device may be listed more than once (its shards render on separate streams).
 * params->tile_rows must be 0. Bit-identical to tray_render for any list: every
 * draw is keyed on the global pixel index. */
int tray_render_devices(const tray_sphere *spheres, int32_t n_spheres, const tray_background *background,
                        const tray_camera *camera, const tray_params *params, const int32_t *devices,
                        int32_t n_devices, void *out, uint32_t *segments_out);

/* tray_render_devices with live progress: every device counts its shard's
 * finished samples per 8-row tile row, and the calling thread polls all of them
 * while the devices render, calling progress(rows, user) as tile rows complete on
 * any device (ProgressFunc from any worker, ray/tracer.go:126-128). progress may
 * be NULL (then this is tray_render_devices). */
int tray_render_devices_progress(const tray_sphere *spheres, int32_t n_spheres, const tray_background *background,
                                 const tray_camera *camera, const tray_params *params, const int32_t *devices,
                                 int32_t n_devices, void *out, uint32_t *segments_out, tray_progress_fn progress,
                                 void *user);

/* Device-resident scene for repeated renders (the scene is read-only during
 * Render, ray/tracer.go:48).
 *
 * Concurrency: like a Go *Scene, which several goroutines may Render at once, a
 * scene handle may be used by any number of tray_render_*_async calls, from any
 * threads and on any streams, without ordering them. Every render takes one of
 * the scene's launch contexts (its work queue, sample or chunk buffer,
 * candidate records and traversal-stack overflow area) for as long as it runs:
 * the one last used on the same stream, else an idle one, else a new one (up to
 * 4 per scene), else the least recently used, which the new render's stream
 * then waits for on the device (hipStreamWaitEvent). A buffer that must grow is
 * freed and reallocated in the new render's stream order (hipFreeAsync /
 * hipMallocAsync), after the renders using it: the async calls only enqueue,
 * they never wait for the device. Results do not depend on which context
 * a render takes. tray_scene_release waits for the scene's enqueued renders and
 * must not race with a call still enqueueing on the same handle. */
int tray_scene_upload(const tray_sphere *spheres, int32_t n_spheres, const tray_background *background,
                      int32_t device, tray_scene_t *out);
int tray_scene_release(tray_scene_t scene);

/* How an uploaded scene is traversed (diagnostics; no reference counterpart). */
typedef struct tray_scene_info {
    int32_t n_spheres;
    int32_t has_bvh;      /* 0: every render uses the reference-order linear scan */
    int32_t leaf_max;     /* spheres per BVH leaf (1, 2 or 4: the size whose LDS layout ranks best) */
    int32_t n_nodes;      /* 4-wide BVH nodes */
    int32_t n_leaves;
    int32_t stack_depth;  /* traversal stack bound (entries) */
    int32_t lds_resident; /* 1: nodes + geometry are staged in LDS; 2: nodes only (geometry read from
                             global memory); 0: all read from global memory */
    int32_t n_global;     /* spheres kept out of the tree and tested first by every traversal */
    double bound;         /* M: the BVH needs every ray origin in [-M, M]^3 */
} tray_scene_info;
int tray_scene_get_info(tray_scene_t scene, tray_scene_info *out);

/* How a render of `params` (n_passes progressive passes from params->pass) on
 * `scene` with `camera` would run, without running it. Pixel sums: with
 * fixed_point_shift k > 0 (rays_per_pixel a multiple of 64, or 16 or 32, and a colour bound
 * that allows k >= 44) each pixel's samples are summed exactly as integers of
 * 2^-k, so the mean is within 2^-(k+1) of the exact mean of the sample colours
 * whatever order the samples finish in; k = 0: the FP64 sum in sample order of
 * Go's RenderLines (ray/tracer.go:143). acc_slots > 0: those sums are kept on
 * chip (per-wave LDS accumulators, one 32-B record per 64 samples, or per
 * pixel-pass when r is 16 or 32, in buffer_bytes); 0: through a 24-B
 * per-sample buffer. Both give the same bits. */
typedef struct tray_render_plan {
    int32_t fixed_point_shift; /* k (0: FP64 sum in sample order) */
    int32_t acc_slots;         /* on-chip accumulators per wave (0: per-sample buffer) */
    int32_t bvh;               /* 1: the BVH kernel; 0: the reference-order linear scan */
    int32_t lds_layout;        /* BVH: as tray_scene_info.lds_resident; linear scan: 1 geometry in LDS */
    int32_t stack_lds;         /* BVH: traversal stack entries per lane kept in LDS */
    int32_t reserved;          /* 0 */
    int64_t lds_bytes;         /* dynamic LDS per workgroup */
    int64_t buffer_bytes;      /* device workspace for the samples or chunk records of one launch band */
} tray_render_plan;
int tray_render_plan_get(tray_scene_t scene, const tray_camera *camera, const tray_params *params,
                         int32_t n_passes, tray_render_plan *out);

/* Asynchronous render into DEVICE memory on `stream` (a hipStream_t, or NULL for
 * the null stream of the scene's device). out_device: compact rows in the
 * params->output format; segments_device nullable. Returns after enqueueing.
 * Safe beside other renders of the same scene on other streams (see above). */
int tray_render_async(tray_scene_t scene, const tray_camera *camera, const tray_params *params, void *out_device,
                      uint32_t *segments_device, void *stream);

/* Consecutive progressive passes params->pass .. params->pass + n_passes - 1 of
 * the row set, as ONE persistent launch (per band): the work queue holds every
 * pass's samples (a pixel's passes consecutively, so waves trace one pixel's
 * samples for a long run), and there is one tail of long paths per launch, not
 * one per frame. Frame k (bit-identical to tray_render_async with pass =
 * params->pass + k) is written at out_device + k * rows * width *
 * bytes-per-pixel. No segments output. */
int tray_render_passes_async(tray_scene_t scene, const tray_camera *camera, const tray_params *params,
                             int32_t n_passes, void *out_device, void *stream);

/* tray_render_async with instrumentation, for roofline accounting: writes the
 * frame as TRAY_OUT_RGB_F32 into out_device (params->output is ignored) and
 * stats_device[0..2] = total Scene.Hit calls (segments), ray-sphere tests and
 * ray-box tests performed (summed over lanes). stats_device is zeroed first. */
int tray_render_stats_async(tray_scene_t scene, const tray_camera *camera, const tray_params *params,
                            float *out_device, uint64_t *stats_device, void *stream);

/* Rows rendered by *params (size of the compact output in rows). */
int32_t tray_params_rows(const tray_params *params);

/* ColorF.ToSRGBA on the host (ray/vec3.go:173-180): n_pixels linear RGB doubles -> RGBA8. */
int tray_to_srgba(const double *rgb, size_t n_pixels, uint8_t *rgba);

/* The same encoder on `device`, over DEVICE buffers (n_pixels x 3 doubles ->
 * n_pixels x 4 bytes, A = 255), enqueued on `stream` (e.g. to encode a frame
 * accumulated from progressive passes without a host round trip). Bit-identical
 * to tray_to_srgba: the device counts the thresholds t[k] <= c of a 255-entry
 * table the host derives from its own encoder (t[k] = least double encoding to
 * >= k), so no device pow is involved. TRAY_OUT_RGBA8 renders use the same table. */
int tray_linear_to_srgba_async(const double *rgb_device, size_t n_pixels, uint8_t *rgba_device, int32_t device,
                               void *stream);

/* ---- the terminal view's downscale (main.go:119-128) ------------------------- */
/* golang.org/x/image/draw (v0.35.0, go.mod:11) scalers, op Over: main.go scales the
 * rendered image into a fresh (zero) image of the terminal's size. */
typedef enum tray_scale_filter {
    TRAY_SCALE_NEAREST = 0, /* draw.NearestNeighbor.Scale (main.go:125, supersample < 1) */
    TRAY_SCALE_BILINEAR = 1 /* draw.BiLinear.Scale (main.go:127, supersample > 1) */
} tray_scale_filter;

/* Scales the RGBA8 image src (src_width x src_height, pitch 4 * src_width) onto
 * dst (dst_width x dst_height), blending Over dst's current contents exactly as
 * the Go scalers do, on `device`. Host buffers; synchronous. */
int tray_scale_rgba(const uint8_t *src, int32_t src_width, int32_t src_height, uint8_t *dst, int32_t dst_width,
                    int32_t dst_height, int32_t filter, int32_t device);
/* The same over DEVICE buffers, enqueued on `stream` (e.g. a TRAY_OUT_RGBA8 frame
 * still on the device: only the terminal-sized image need come back). */
int tray_scale_rgba_async(const uint8_t *src_device, int32_t src_width, int32_t src_height, uint8_t *dst_device,
                          int32_t dst_width, int32_t dst_height, int32_t filter, int32_t device, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* TRAY_H */
