/* A C99 caller of include/tray.h, the way a cgo shim binds it: plain C types,
 * caller-owned buffers, int status codes, a C progress callback.
 * Built by tests/test_c_caller.py with gcc -std=c99 -Wall -Wextra -Werror -pedantic.
 * Prints key=value lines the test checks. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "tray.h"

static void on_progress(int32_t rows, void *user) {
    int32_t *total = (int32_t *)user;
    *total += rows;
}

int main(void) {
    enum { W = 16, H = 9 };
    tray_camera_setup setup;
    tray_camera cam;
    tray_background bg;
    tray_params p = {0};
    const double lin[6] = {0.0, 0.5, 1.0, 0.0031308, -1.0, 2.0};
    uint8_t rgba[8];
    int32_t cap, n = 0, count = 0, progress_rows = 0;
    tray_sphere *spheres;
    float *out;
    int rc;

    printf("abi=%d\n", (int)tray_abi_version());
    if (tray_rich_scene_camera(&setup) != TRAY_OK) return 1;
    if (tray_camera_initialize(&setup, W, H, &cam) != TRAY_OK) return 1;
    printf("focus=%.17g\n", cam.focus_distance);
    cap = tray_rich_scene_capacity(11);
    spheres = (tray_sphere *)calloc((size_t)cap, sizeof(tray_sphere));
    if (!spheres || tray_rich_scene(2, 11, spheres, cap, &n) != TRAY_OK) return 1;
    printf("spheres=%d\n", (int)n);
    if (tray_default_background(&bg) != TRAY_OK) return 1;
    if (tray_to_srgba(lin, 2, rgba) != TRAY_OK) return 1;
    printf("srgb=%d,%d,%d,%d,%d,%d\n", rgba[0], rgba[1], rgba[2], rgba[4], rgba[5], rgba[6]);
    if (tray_device_count(&count) != TRAY_OK) return 1;
    printf("devices=%d\n", (int)count);

    p.width = W;
    p.height = H;
    p.max_depth = 10;
    p.rays_per_pixel = 2;
    p.ray_radius = 0.5;
    p.seed = 2;
    p.y_start = 0;
    p.y_end = H;
    p.output = TRAY_OUT_RGB_F32;
    printf("rows=%d\n", (int)tray_params_rows(&p));
    out = (float *)calloc((size_t)W * H * 3, sizeof(float));
    if (!out) return 1;
    rc = tray_render(spheres, n, &bg, &cam, &p, 0, out, NULL);
    printf("render=%d\n", rc);
    if (rc != TRAY_OK) printf("error=%s\n", tray_last_error());
    rc = tray_render_progress(spheres, n, &bg, &cam, &p, 0, out, NULL, on_progress, &progress_rows);
    printf("render_progress=%d progress_rows=%d\n", rc, (int)progress_rows);
    p.width = 0;
    printf("bad_width=%d\n", tray_render(spheres, n, &bg, &cam, &p, 0, out, NULL));
    spheres[3].reserved = 7;
    p.width = W;
    printf("bad_reserved=%d\n", tray_render(spheres, n, &bg, &cam, &p, 0, out, NULL));
    tray_shutdown();
    free(out);
    free(spheres);
    return 0;
}
