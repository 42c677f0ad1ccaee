"""C-ABI on the CPU: the library loads, exports every symbol include/tray.h
declares, its host-side setup matches the oracle bit for bit, argument errors
are reported before any device work, and without a GPU it fails loudly (no
fallback). No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def test_exports_match_header(L):
    header = open(os.path.join(ROOT, "include", "tray.h")).read()
    declared = set(re.findall(r"^(?:int|int32_t|const char \*)\s*\**\s*(tray_\w+)\(", header, re.M))
    assert declared == set(L.EXPORTS)
    lib = L.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.tray_abi_version() == 6  # 2: devices_progress, release_cache; 3: plan_get; 4: ORDERED_SUM flag; 5: launch contexts; 6: pcg4d draws


def test_debug_hooks_outside_stable_header(L):
    """include/tray_debug.h's knobs are exported but not part of tray.h's stable set."""
    header = open(os.path.join(ROOT, "include", "tray.h")).read()
    debug = open(os.path.join(ROOT, "include", "tray_debug.h")).read()
    declared = set(re.findall(r"^int\s+(tray_\w+)\(", debug, re.M))
    assert declared == set(L.DEBUG_EXPORTS)
    assert not any(name in header for name in declared)
    for knob in L.DEBUG_KNOBS:
        assert f'"{knob}"' in debug
    lib = L.lib()
    for knob in L.DEBUG_KNOBS:
        assert lib.tray_debug_set(knob.encode(), 1) == 0
        assert lib.tray_debug_clear(knob.encode()) == 0
    assert lib.tray_debug_set(b"no_such_knob", 1) == L.TRAY_ERR_INVALID_ARGUMENT
    assert lib.tray_debug_clear(None) == 0
    with pytest.raises(ValueError):
        L.debug_knobs(no_such_knob=1)


def test_library_never_reads_the_environment(L):
    """A stray TRAY_* variable in a host process cannot change what the library
    renders: the product .so imports no environment accessor at all (its knobs
    are set through tray_debug_set only)."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--undefined-only", L.LIB_PATH], capture_output=True, text=True, check=True)
    imported = {line.split()[-1].split("@")[0] for line in out.stdout.splitlines() if line.strip()}
    assert not imported & {"getenv", "secure_getenv", "__secure_getenv", "environ", "__environ", "setenv"}, imported
    assert "tray_debug_set" in subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                                              text=True, check=True).stdout


def _setup(L, arr):
    d3 = ctypes.c_double * 3
    return L.CameraSetup(d3(*arr[0:3]), d3(*arr[3:6]), d3(*arr[6:9]), *arr[9:13])


@pytest.mark.parametrize(
    "setup,w,h",
    [
        (np.array([13, 2, 3, 0, 0, 0, 0, 1, 0, 20.0, 10.0, 10.0, 0.1]), 1280, 720),
        (np.zeros(13), 100, 100),
        (np.array([1, 2, 3, 1, 2, 3, 0, 0, 0, 0, 0, 0, 0.0]), 64, 48),
        (np.array([-2, 2, 1, 0, 0, -1, 0, 0, 0, 20.0, 0, 3.0, 0.1]), 400, 225),
        (np.array([0, 0, 5, 0, 0, 0, 0, 1, 0, 45.0, 2.0, 0, 0.5]), 33, 77),
    ],
)
def test_camera_initialize_matches_oracle(L, O, setup, w, h):
    cs = _setup(L, setup)
    st = L.CameraState()
    L.check(L.lib().tray_camera_initialize(ctypes.byref(cs), w, h, ctypes.byref(st)))
    io, cam = O.camera_initialize(setup, w, h)
    assert np.array_equal(st.as_array(), cam)
    resolved = np.array([*cs.position, *cs.look_at, *cs.up, cs.vertical_fov, cs.focal_length, cs.focus_distance,
                         cs.aperture])
    assert np.array_equal(resolved, io)


@pytest.mark.parametrize("seed,half", [(2, 11), (7, 11), (42, 11), (7, 22), (1, 0)])
def test_rich_scene_matches_oracle(O, seed, half):
    from tray_amd import ray

    a = ray.rich_scene_array(seed, half)
    b = O.rich_scene(seed, half)
    assert a.tobytes() == b.tobytes()


def test_default_scene_and_background(L, O):
    from tray_amd import ray

    a = ray.DefaultScene()
    assert a.to_array().tobytes() == O.default_scene().tobytes()
    bg = L.Background()
    L.check(L.lib().tray_default_background(ctypes.byref(bg)))
    assert tuple(bg.color_a) + tuple(bg.color_b) == (1.0, 1.0, 1.0, 0.4, 0.65, 1.0)


def test_to_srgba_matches_oracle(L, O):
    rng = np.random.default_rng(0)
    rgb = np.concatenate([rng.random((3000, 3)), rng.random((300, 3)) * 0.004, np.array([[0.5, 1.0, 0.0]]),
                          np.array([[-1.0, 2.0, np.nan]])])
    out = np.zeros((len(rgb), 4), dtype=np.uint8)
    L.check(L.lib().tray_to_srgba(rgb.ctypes.data, len(rgb), out.ctypes.data))
    assert np.array_equal(out, O.to_srgba(rgb))


@pytest.mark.parametrize("h,tile,world", [(720, 8, 8), (720, 8, 3), (37, 5, 4), (10, 16, 2), (5, 1, 20)])
def test_params_rows_and_shard_rows(L, h, tile, world):
    from tray_amd import shard

    total = 0
    seen = []
    for r in range(world):
        p = L.make_params(17, h, 10, 1, 0.5, 1, tile_rows=tile, tile_count=world, tile_index=r)
        rows = shard.rows_for(h, tile, world, r)
        assert L.params_rows(p) == len(rows)
        total += len(rows)
        seen.extend(rows.tolist())
    assert total == h and sorted(seen) == list(range(h))
    assert L.params_rows(L.make_params(17, h, 10, 1, 0.5, 1, y_start=2, y_end=h - 1)) == h - 3


def _render_rc(L, spheres=None, **kw):
    base = dict(width=8, height=8, max_depth=5, rays_per_pixel=1, ray_radius=0.5, seed=1)
    base.update(kw)
    p = L.make_params(**base)
    bg = L.Background()
    cam = L.CameraState()
    s = L.spheres_array(spheres)
    out = np.zeros(8 * 8 * 4 * 24, dtype=np.uint8)
    return L.lib().tray_render(s.ctypes.data if len(s) else None, len(s), ctypes.byref(bg), ctypes.byref(cam),
                               ctypes.byref(p), 0, out.ctypes.data, None)


@pytest.mark.parametrize(
    "kw",
    [dict(width=0), dict(height=-1), dict(max_depth=0), dict(rays_per_pixel=0), dict(ray_radius=float("inf")),
     dict(y_start=5, y_end=3), dict(y_end=9), dict(tile_rows=4, tile_count=2, tile_index=2), dict(tile_rows=-1),
     dict(output=7), dict(pass_=-1)],
)
def test_invalid_params_rejected_before_device(L, kw):
    assert _render_rc(L, **kw) == L.TRAY_ERR_INVALID_ARGUMENT
    assert L.lib().tray_last_error()


def test_unsupported_material(L):
    s = np.zeros(2, dtype=L.SPHERE_DTYPE)
    s["material"] = [1, 9]
    assert _render_rc(L, s) == L.TRAY_ERR_UNSUPPORTED
    assert b"unsupported material" in L.lib().tray_last_error()


def test_pass_beyond_rng_sample_word(L):
    # tray_params.pass: (pass + 1) x rays_per_pixel must fit the 32-bit RNG sample word
    assert _render_rc(L, rays_per_pixel=1 << 20, pass_=4096) == L.TRAY_ERR_TOO_LARGE
    assert b"sample word" in L.lib().tray_last_error()


def test_too_many_pixels(L):
    assert _render_rc(L, width=70000, height=70000) == L.TRAY_ERR_TOO_LARGE


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_no_device_fails_loudly(L):
    assert _render_rc(L) == L.TRAY_ERR_NO_DEVICE
    n = ctypes.c_int32(-1)
    assert L.lib().tray_device_count(ctypes.byref(n)) == 0 and n.value == 0


def test_go_api_defaults_without_gpu():
    """ray/tracer_test.go:108-170 defaulting + camera_test.go defaults via the mirror (host only)."""
    from tray_amd import ray

    t = ray.New(5, 5)
    sc = t._apply_defaults(ray.DefaultScene())
    t.Camera.Initialize(5, 5)
    assert (t.FocalLength, t.VerticalFoV, t.MaxDepth, t.NumRaysPerPixel, t.RayRadius) == (1.0, 90.0, 10, 1, 0.5)
    assert t.NumWorkers == (os.cpu_count() or 1)
    assert sc.Background == ray.DefaultBackground()
    t = ray.New(5, 5)
    t.Position, t.FocalLength, t.VerticalFoV = (1, 2, 3), 10, 45.0
    t.MaxDepth, t.NumRaysPerPixel, t.RayRadius, t.NumWorkers = 20, 4, 1.0, 2
    t._apply_defaults(ray.DefaultScene())
    t.Camera.Initialize(5, 5)
    assert (t.Position, t.FocalLength, t.VerticalFoV, t.MaxDepth, t.NumRaysPerPixel, t.RayRadius, t.NumWorkers) == (
        (1.0, 2.0, 3.0), 10, 45.0, 20, 4, 1.0, 2)
    t = ray.New(10, 10)
    t._apply_defaults(None)  # Render(nil): DefaultScene + its camera (tracer.go:50-62)
    assert t.Position == (-2.0, 2.0, 1.0) and t.Aperture == 0.1 and t.VerticalFoV == 20.0
    assert t.FocusDistance == 12.0 ** 0.5  # Length(Sub(Position, LookAt)) = |(-2, 2, 2)|


def test_scene_flattening_errors():
    from tray_amd import _lib, ray

    class Weird:
        pass

    with pytest.raises(_lib.TrayError):
        ray.Scene([ray.Sphere((0, 0, 0), 1, Weird())]).to_array()
    with pytest.raises(_lib.TrayError):
        ray.Scene([Weird()]).to_array()
    arr = ray.Scene([ray.Sphere((0, 0, -1), 0.5, ray.Metal((0.8, 0.8, 0.8), 0.3))]).to_array()
    assert arr["material"][0] == _lib.METAL and arr["param"][0] == 0.3


def test_scene_info_layout(L):
    import ctypes

    assert ctypes.sizeof(L.SceneInfo) == 8 * 4 + 8
    assert ctypes.sizeof(L.RenderPlan) == 6 * 4 + 2 * 8


def test_png_sink_round_trip():
    """PNG sink (benchmark/benchmark.go:23-33 encodes Render's *image.RGBA)."""
    import numpy as np

    from tray_amd import png

    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (17, 23, 4), dtype=np.uint8)
    data = png.encode_png(img)
    assert data[:8] == b"\x89PNG\r\n\x1a\n" and data[12:16] == b"IHDR"
    assert np.array_equal(png.decode_png(data), img)


def test_bench_cpu_sample_size():
    """bench.py's cpu_baseline sample: every row for C1/C2 (the whole C2 frame is
    ~13 s on 16 threads), a row stride for the larger configs that keeps the
    oracle's linear-scan work near one C2 frame."""
    import bench

    label, seed, half, W, H, spp, depth = bench.CONFIGS["c2"]
    assert bench.auto_row_step(486, W, H, spp) == 1
    assert bench.auto_row_step(486, 400, 225, 16) == 1
    assert bench.auto_row_step(1939, 1920, 1080, 256) == 36
    assert bench.auto_row_step(486, 3840, 2160, 256) == 36
    assert bench.auto_row_step(0, 64, 64, 1) == 1


def test_srgb_threshold_encoding_equals_encoder(L, O):
    """The device's TRAY_OUT_RGBA8 encoder counts thresholds t[k] (least double
    encoding to >= k); that equals the host/oracle encoder wherever the encoder
    is monotone. Check monotonicity on sorted random values, the exact
    threshold bracketing, and the host C-ABI encoder against the oracle there."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import srgb_thresholds

    t = srgb_thresholds(O)
    k = np.arange(1, 256)
    assert np.all(np.diff(t) > 0)
    assert np.array_equal(O.linear_to_srgb_n(t).astype(int), k)
    assert np.array_equal(O.linear_to_srgb_n(np.nextafter(t, 0)).astype(int), k - 1)
    rng = np.random.default_rng(5)
    v = np.sort(np.concatenate([rng.random(1_000_000), rng.random(200_000) * 0.004]))
    enc = O.linear_to_srgb_n(v)
    assert np.all(np.diff(enc.astype(int)) >= 0)
    assert np.array_equal(np.searchsorted(t, v, side="right"), enc)  # count of t[k] <= c
    rgb = v[: len(v) // 3 * 3].reshape(-1, 3)
    host = np.zeros((len(rgb), 4), dtype=np.uint8)
    L.check(L.lib().tray_to_srgba(rgb.ctypes.data, len(rgb), host.ctypes.data))
    assert np.array_equal(host, O.to_srgba(rgb))


def test_render_devices_argument_checks(L):
    s = L.spheres_array(None)
    bg, cam = L.Background(), L.CameraState()
    out = np.zeros(8 * 8 * 24, dtype=np.uint8)
    devs = (ctypes.c_int32 * 2)(0, 0)
    lib = L.lib()
    p = L.make_params(8, 8, 5, 1, 0.5, 1)
    assert lib.tray_render_devices(None, 0, ctypes.byref(bg), ctypes.byref(cam), ctypes.byref(p), devs, 0,
                                   out.ctypes.data, None) == L.TRAY_ERR_INVALID_ARGUMENT
    q = L.make_params(8, 8, 5, 1, 0.5, 1, tile_rows=1, tile_count=2)
    assert lib.tray_render_devices(None, 0, ctypes.byref(bg), ctypes.byref(cam), ctypes.byref(q), devs, 2,
                                   out.ctypes.data, None) == L.TRAY_ERR_INVALID_ARGUMENT
    if not os.path.exists("/dev/kfd"):
        assert lib.tray_render_devices(None, 0, ctypes.byref(bg), ctypes.byref(cam), ctypes.byref(p), devs, 2,
                                       out.ctypes.data, None) == L.TRAY_ERR_NO_DEVICE


def test_import_order_library_before_torch():
    """`import tray_amd` (and loading the library) BEFORE torch: both link a
    libamdhip64.so.7, and torch only works on its own bundled copy. The binding
    loads torch first, so one HIP runtime is mapped and it is torch's."""
    import subprocess
    import sys

    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from tray_amd import _lib, ray\n"
        "_lib.lib(); ray.DefaultBackground()\n"
        "import torch\n"
        "torch.cuda.device_count()\n"
        "maps = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
        "print(len(maps), sorted(maps)[0])\n" % ROOT
    )
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    n, path = r.stdout.split()
    import torch

    assert n == "1" and os.path.realpath(path).startswith(os.path.realpath(os.path.dirname(torch.__file__))), path


def test_host_go_tan_against_independent_restatement(L):
    """The host's copy of Go's math.Tan (tray_host.cpp, Camera.Initialize's
    viewport height, ray/camera.go:93) against the independent Python
    restatement in tests/golden/make_golden.py, bit for bit. With the camera at
    the origin looking down -z (up y), focal length 0.5 and a 1x1 image,
    pixel_y = (0, -2 * 0.5 * tan(theta / 2), 0) exactly, so -pixel_y[1] IS the
    host's go_tan(vfov * Pi/180 / 2)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden

    deg = float.fromhex("0x1.1df46a2529d39p-6")  # Go's math.Pi / 180
    rng = np.random.default_rng(11)
    fovs = np.concatenate([rng.uniform(1e-3, 179.999, 3000), np.arange(1, 180, dtype=np.float64), [90.0, 20.0]])
    for fov in fovs:
        setup = _setup(L, np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, float(fov), 0.5, 0, 0.0]))
        st = L.CameraState()
        L.check(L.lib().tray_camera_initialize(ctypes.byref(setup), 1, 1, ctypes.byref(st)))
        assert st.pixel_y[0] == 0.0 and st.pixel_y[2] == 0.0
        assert -st.pixel_y[1] == make_golden.go_tan(float(fov) * deg / 2.0), fov
    st = L.CameraState()
    setup = _setup(L, np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 90.0, 0.5, 0, 0.0]))
    L.check(L.lib().tray_camera_initialize(ctypes.byref(setup), 1, 1, ctypes.byref(st)))
    assert -st.pixel_y[1] == 1.0  # Go's tan(Pi/4) = 1 (libm: 1 - 2^-53)


def test_scale_argument_checks(L):
    """tray_scale_rgba rejects bad sizes, filters and null images before any device work."""
    img = np.zeros((4, 4, 4), np.uint8)
    out = np.zeros((2, 2, 4), np.uint8)
    lib = L.lib()
    assert lib.tray_scale_rgba(img.ctypes.data, 4, 4, out.ctypes.data, 0, 2, 1, 0) == L.TRAY_ERR_INVALID_ARGUMENT
    assert lib.tray_scale_rgba(img.ctypes.data, 4, 4, out.ctypes.data, 2, 2, 7, 0) == L.TRAY_ERR_INVALID_ARGUMENT
    assert lib.tray_scale_rgba(None, 4, 4, out.ctypes.data, 2, 2, 1, 0) == L.TRAY_ERR_INVALID_ARGUMENT
    assert lib.tray_scale_rgba_async(None, 4, 4, None, 2, 2, 0, 0, None) == L.TRAY_ERR_INVALID_ARGUMENT
