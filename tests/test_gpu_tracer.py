"""fortio/tray ray/tracer_test.go and camera_test.go:245-283, run against the
Go-API mirror (tray_amd.ray) whose Render/RenderLines go through the HIP path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ray():
    from tray_amd import ray

    return ray


def test_render_default_scene(ray):  # tracer_test.go:47-78
    t = ray.New(10, 10)
    t.Seed = 1
    img = t.Render(None)
    assert img is t.imageData and img.shape == (10, 10, 4)
    assert np.all(img[..., 3] == 255) and np.any(img[..., :3] != 0)


def test_render_custom_scene_alpha(ray):  # tracer_test.go:80-106
    t = ray.New(5, 5)
    img = t.Render(ray.Scene([ray.Sphere((0, 0, -1), 0.5, ray.Lambertian((1, 0, 0)))]))
    assert np.all(img[..., 3] == 255)


def test_render_default_and_custom_parameters(ray):  # tracer_test.go:108-170
    import os

    t = ray.New(5, 5)
    t.Render(ray.DefaultScene())
    assert (t.FocalLength, t.VerticalFoV, t.MaxDepth, t.NumRaysPerPixel, t.RayRadius) == (1.0, 90.0, 10, 1, 0.5)
    assert t.NumWorkers == (os.cpu_count() or 1)
    t = ray.New(5, 5)
    t.Position, t.FocalLength, t.VerticalFoV = (1, 2, 3), 10, 45.0
    t.MaxDepth, t.NumRaysPerPixel, t.RayRadius, t.NumWorkers = 20, 4, 1.0, 2
    t.Render(ray.DefaultScene())
    assert (t.Position, t.FocalLength, t.VerticalFoV, t.MaxDepth, t.NumRaysPerPixel, t.RayRadius, t.NumWorkers) == (
        (1.0, 2.0, 3.0), 10, 45.0, 20, 4, 1.0, 2)


def test_progress_total(ray):  # tracer_test.go:172-186
    t = ray.New(10, 8)
    total = []
    t.ProgressFunc = total.append
    t.Render(ray.DefaultScene())
    assert sum(total) == 80


@pytest.mark.parametrize("workers,w,h", [(1, 10, 10), (2, 10, 10), (20, 10, 5)])
def test_parallel_rendering_all_pixels(ray, workers, w, h):  # tracer_test.go:188-222
    t = ray.New(w, h)
    t.NumWorkers = workers
    img = t.Render(ray.DefaultScene())
    assert np.all(img[..., 3] == 255)


@pytest.mark.parametrize("n", [1, 4, 10])
def test_multiple_rays_per_pixel(ray, n):  # tracer_test.go:224-256
    t = ray.New(5, 5)
    t.NumRaysPerPixel = n
    assert np.all(t.Render(ray.DefaultScene())[..., 3] == 255)


def test_render_lines(ray):  # tracer_test.go:258-297
    t = ray.New(10, 10)
    t.FocalLength, t.VerticalFoV, t.MaxDepth, t.NumRaysPerPixel, t.RayRadius = 5, 30.0, 10, 1, 0.5
    scene = ray.DefaultScene()
    t.Camera.Initialize(10, 10)
    t.RenderLines(0, 0, 3, scene)
    assert np.all(t.imageData[:3, :, 3] == 255)
    assert np.all(t.imageData[3:] == 0)


def test_render_empty_scene_is_sky(ray):  # tracer_test.go:299-321
    t = ray.New(5, 5)
    img = t.Render(ray.Scene([]))
    assert np.all(img[..., 3] == 255) and np.all(img[..., 2] > 0)


def test_rich_scene_not_black(ray):  # camera_test.go:245-283
    t = ray.New(20, 20)
    t.Camera = ray.RichSceneCamera()
    t.MaxDepth, t.NumRaysPerPixel, t.Seed = 10, 2, 42
    img = t.Render(ray.RichScene(42))
    assert (img[..., :3].max(-1) > 0).sum() >= 200


def test_seed_reproducible_and_sensitive(ray):  # Seed semantics (tracer.go:33)
    def render(seed):
        t = ray.New(16, 9)
        t.Camera = ray.RichSceneCamera()
        t.MaxDepth, t.NumRaysPerPixel, t.Seed = 12, 4, seed
        t.Render(ray.RichScene(2))
        return t.linear.copy()

    a, b, c = render(5), render(5), render(6)
    assert np.array_equal(a, b) and not np.array_equal(a, c)


def test_render_to_png(ray, tmp_path):  # benchmark/benchmark.go:23-33: png.Encode(Render(scene))
    from tray_amd import png

    t = ray.New(32, 18)
    t.Seed, t.NumRaysPerPixel, t.MaxDepth = 2, 4, 20
    t.Camera = ray.RichSceneCamera()
    img = t.Render(ray.RichScene(2))
    path = str(tmp_path / "out.png")
    png.save_png(path, img)
    assert np.array_equal(png.decode_png(open(path, "rb").read()), img)


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_progress_is_live(ray, devices):  # tracer.go:126-128: ProgressFunc per row WHILE rendering
    """tray_render_progress (one device) and tray_render_devices_progress (the
    rows split over several devices of the process; device 0 twice here) report
    rows as their samples finish, from device counters polled during the
    launches: several callbacks, the first well before the end, every row exactly
    once, and the same frame as without progress; Tracer.ProgressFunc sees width
    per row."""
    import time

    from tray_amd import _lib

    W, H = 1280, 720
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    spheres = ray.rich_scene_array(2)
    bg = ray._background(ray.DefaultBackground())
    p = _lib.make_params(W, H, 50, 256, 0.5, 2, output=_lib.OUT_RGB_F32)

    def render(**kw):
        if len(devices) == 1:
            return _lib.render(spheres, bg, cam._state, p, devices[0], **kw)[0]
        return _lib.render_devices(spheres, bg, cam._state, p, devices, **kw)[0]

    plain = render()  # also warms: scene upload + sample buffer
    calls = []
    t0 = time.perf_counter()
    live = render(progress=lambda rows: calls.append((time.perf_counter(), rows)))
    t1 = time.perf_counter()
    assert np.array_equal(plain, live)
    assert sum(r for _, r in calls) == H
    assert len(calls) >= 3, calls
    assert calls[0][1] < H and calls[0][0] < t0 + 0.8 * (t1 - t0)
    t = ray.New(64, 36)
    t.Camera = ray.RichSceneCamera()
    t.NumRaysPerPixel, t.MaxDepth, t.Seed = 16, 20, 2
    t.Devices = devices
    seen = []
    t.ProgressFunc = seen.append
    t.Render(ray.RichScene(2))
    assert seen == [64] * 36


def test_progress_callback_errors_and_reentry(ray):
    """A ProgressFunc that raises: the render finishes and the exception reaches
    the caller (ctypes would swallow it). A callback that calls back into the
    library gets an error instead of a deadlock (the render holds the device)."""
    from tray_amd import _lib

    t = ray.New(64, 36)
    t.Camera = ray.RichSceneCamera()
    t.NumRaysPerPixel, t.MaxDepth, t.Seed = 4, 20, 2

    def boom(_w):
        raise KeyError("from ProgressFunc")

    t.ProgressFunc = boom
    with pytest.raises(KeyError, match="from ProgressFunc"):
        t.Render(ray.RichScene(2))
    codes = []

    def reenter(_rows):
        codes.append(_lib.lib().tray_release_cache(0))
        codes.append(_lib.lib().tray_shutdown())

    cam = ray.RichSceneCamera()
    cam.Initialize(32, 18)
    p = _lib.make_params(32, 18, 10, 2, 0.5, 2)
    _lib.render(ray.rich_scene_array(2), ray._background(ray.DefaultBackground()), cam._state, p, progress=reenter)
    assert codes and all(c == _lib.TRAY_ERR_INVALID_ARGUMENT for c in codes)
    assert "not re-entrant" in _lib.lib().tray_last_error().decode()


def test_release_cache(ray):
    """tray_release_cache frees the synchronous renders' cached scene and
    buffers; the next render re-uploads and gives the same frame."""
    from tray_amd import _lib

    cam = ray.RichSceneCamera()
    cam.Initialize(48, 27)
    p = _lib.make_params(48, 27, 20, 4, 0.5, 2)
    args = (ray.rich_scene_array(2), ray._background(ray.DefaultBackground()), cam._state, p)
    a, _ = _lib.render(*args)
    _lib.release_cache(0)
    b, _ = _lib.render(*args)
    _lib.release_cache(-1)
    c, _ = _lib.render_devices(*args, [0, 0])
    assert np.array_equal(a, b) and np.array_equal(a, c)


def test_tracer_devices_split_is_invisible(ray):
    """Tracer.Devices (no Go counterpart): the frame's rows split over several
    devices of one process (tray_render_devices) give the same image as one device."""
    def render(devices):
        t = ray.New(48, 27)
        t.Camera = ray.RichSceneCamera()
        t.MaxDepth, t.NumRaysPerPixel, t.Seed = 20, 4, 3
        t.Devices = devices
        rows = []
        t.ProgressFunc = rows.append
        img = t.Render(ray.RichScene(2)).copy()
        assert rows == [48] * 27
        return img, t.linear.copy()

    a, la = render(None)
    b, lb = render([0, 0, 0])
    assert np.array_equal(a, b) and np.array_equal(la, lb)
