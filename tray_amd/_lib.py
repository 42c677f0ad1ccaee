"""ctypes binding of the C-ABI in include/tray.h (libtray_amd.so, built in-tree).

This is the only way the Python host reaches the renderer: there is no Python,
PyTorch or CPU fallback for the hot path. If the shared library is missing the
import fails loudly with the build command to run.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# TRAY_LIB points the binding at another build of the same ABI (A/B tooling only).
LIB_PATH = os.environ.get("TRAY_LIB") or os.path.join(_HERE, "libtray_amd.so")

# include/tray.h enums
TRAY_OK = 0
TRAY_ERR_INVALID_ARGUMENT = -1
TRAY_ERR_UNSUPPORTED = -2
TRAY_ERR_DEVICE = -3
TRAY_ERR_NO_DEVICE = -4
TRAY_ERR_TOO_LARGE = -5
LAMBERTIAN, METAL, DIELECTRIC = 1, 2, 3
OUT_RGB_F64, OUT_RGB_F32, OUT_RGBA8 = 0, 1, 2
BYTES_PER_PIXEL = {OUT_RGB_F64: 24, OUT_RGB_F32: 12, OUT_RGBA8: 4}

# tray_sphere as a numpy structured dtype (72 bytes, C layout).
SPHERE_DTYPE = np.dtype(
    [
        ("center", "<f8", (3,)),
        ("radius", "<f8"),
        ("albedo", "<f8", (3,)),
        ("param", "<f8"),
        ("material", "<i4"),
        ("reserved", "<i4"),
    ]
)
assert SPHERE_DTYPE.itemsize == 72

_d3 = ctypes.c_double * 3


class Background(ctypes.Structure):
    _fields_ = [("color_a", _d3), ("color_b", _d3)]


class CameraSetup(ctypes.Structure):
    _fields_ = [
        ("position", _d3),
        ("look_at", _d3),
        ("up", _d3),
        ("vertical_fov", ctypes.c_double),
        ("focal_length", ctypes.c_double),
        ("focus_distance", ctypes.c_double),
        ("aperture", ctypes.c_double),
    ]


class CameraState(ctypes.Structure):
    _fields_ = [
        ("position", _d3),
        ("pixel00", _d3),
        ("pixel_x", _d3),
        ("pixel_y", _d3),
        ("defocus_u", _d3),
        ("defocus_v", _d3),
        ("aperture", ctypes.c_double),
        ("focus_distance", ctypes.c_double),
        ("focal_length", ctypes.c_double),
    ]

    def as_array(self) -> np.ndarray:
        """The 21 doubles in declaration order (the oracle's camera layout)."""
        return np.frombuffer(bytes(self), dtype=np.float64).copy()


assert ctypes.sizeof(CameraState) == 21 * 8


class Params(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("max_depth", ctypes.c_int32),
        ("rays_per_pixel", ctypes.c_int32),
        ("ray_radius", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("y_start", ctypes.c_int32),
        ("y_end", ctypes.c_int32),
        ("tile_rows", ctypes.c_int32),
        ("tile_count", ctypes.c_int32),
        ("tile_index", ctypes.c_int32),
        ("output", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("pass_", ctypes.c_int32),  # tray_params.pass (progressive pass)
    ]


FLAG_LINEAR_SCAN = 1  # TRAY_FLAG_LINEAR_SCAN
FLAG_ORDERED_SUM = 2  # TRAY_FLAG_ORDERED_SUM: Go's FP64 pixel sum in sample order (include/tray.h)


class SceneInfo(ctypes.Structure):
    """tray_scene_info: how an uploaded scene is traversed."""
    _fields_ = [("n_spheres", ctypes.c_int32), ("has_bvh", ctypes.c_int32), ("leaf_max", ctypes.c_int32),
                ("n_nodes", ctypes.c_int32), ("n_leaves", ctypes.c_int32), ("stack_depth", ctypes.c_int32),
                ("lds_resident", ctypes.c_int32), ("n_global", ctypes.c_int32), ("bound", ctypes.c_double)]


class RenderPlan(ctypes.Structure):
    """tray_render_plan: how a render would run (pixel sums, kernel, LDS, workspace)."""
    _fields_ = [("fixed_point_shift", ctypes.c_int32), ("acc_slots", ctypes.c_int32), ("bvh", ctypes.c_int32),
                ("lds_layout", ctypes.c_int32), ("stack_lds", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("lds_bytes", ctypes.c_int64), ("buffer_bytes", ctypes.c_int64)]

    def as_dict(self) -> dict:
        return {name: int(getattr(self, name)) for name, _ in self._fields_ if name != "reserved"}


class TrayError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"tray error {code}: {message}")
        self.code = code


# Every symbol include/tray.h declares (tests check the library exports all of them).
EXPORTS = (
    "tray_abi_version",
    "tray_last_error",
    "tray_device_count",
    "tray_shutdown",
    "tray_camera_initialize",
    "tray_rich_scene_camera",
    "tray_default_background",
    "tray_default_scene",
    "tray_rich_scene",
    "tray_rich_scene_capacity",
    "tray_render",
    "tray_render_progress",
    "tray_render_devices",
    "tray_render_devices_progress",
    "tray_release_cache",
    "tray_scale_rgba",
    "tray_scale_rgba_async",
    "tray_scene_upload",
    "tray_scene_release",
    "tray_scene_get_info",
    "tray_render_plan_get",
    "tray_render_async",
    "tray_render_passes_async",
    "tray_render_stats_async",
    "tray_params_rows",
    "tray_to_srgba",
    "tray_linear_to_srgba_async",
)

# include/tray_debug.h: test / A-B hooks outside the stable ABI (not in EXPORTS).
DEBUG_EXPORTS = ("tray_debug_set", "tray_debug_clear")
DEBUG_KNOBS = ("acc_slots", "band_samples", "bvh_leaf", "bvh_lds_mode", "stack_lds_slots", "node_deep",
               "primary_candidates", "resolve_staged", "wave_chunks", "scene_contexts", "grid_reserve",
               "work_order", "coop_lanes")

# tray_progress_fn: void (*)(int32_t rows, void *user)
PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_int32, ctypes.c_void_p)

_libs: dict = {}


def _torch_first() -> None:
    """Load torch (when it is installed) before the library. Both link a HIP
    runtime with the same soname (libamdhip64.so.7): torch bundles its own, the
    library was linked against /opt/rocm's. Whichever is mapped first serves
    both, and torch does not work on /opt/rocm's (it then sees no GPU), while
    the library's C-ABI works on either. Importing torch here makes the import
    order of `tray_amd` and `torch` irrelevant to the caller."""
    import importlib.util

    if "torch" in sys.modules or importlib.util.find_spec("torch") is None:
        return
    import torch  # noqa: F401


def lib(path: str | None = None) -> ctypes.CDLL:
    """The C-ABI library (default: the in-tree build). `path` loads another build
    of the same ABI (used by tools/ab_bench.py to compare kernel variants)."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: the HIP renderer is not built. Run `make -C tray_amd` "
            "(or __graft_entry__.build()). There is no CPU fallback."
        )
    _torch_first()
    L = ctypes.CDLL(path)
    vp, i32, u32p = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32)
    L.tray_abi_version.restype = i32
    L.tray_last_error.restype = ctypes.c_char_p
    L.tray_device_count.argtypes = [ctypes.POINTER(i32)]
    L.tray_camera_initialize.argtypes = [ctypes.POINTER(CameraSetup), i32, i32, ctypes.POINTER(CameraState)]
    L.tray_rich_scene_camera.argtypes = [ctypes.POINTER(CameraSetup)]
    L.tray_default_background.argtypes = [ctypes.POINTER(Background)]
    L.tray_default_scene.argtypes = [vp, i32, ctypes.POINTER(i32)]
    L.tray_rich_scene.argtypes = [ctypes.c_uint64, i32, vp, i32, ctypes.POINTER(i32)]
    L.tray_rich_scene_capacity.argtypes = [i32]
    L.tray_rich_scene_capacity.restype = i32
    L.tray_render.argtypes = [vp, i32, ctypes.POINTER(Background), ctypes.POINTER(CameraState),
                              ctypes.POINTER(Params), i32, vp, u32p]
    if hasattr(L, "tray_render_progress"):  # absent from older builds (A/B tools)
        L.tray_render_progress.argtypes = L.tray_render.argtypes + [PROGRESS_FN, vp]
    if hasattr(L, "tray_render_devices"):
        L.tray_render_devices.argtypes = [vp, i32, ctypes.POINTER(Background), ctypes.POINTER(CameraState),
                                          ctypes.POINTER(Params), ctypes.POINTER(i32), i32, vp, u32p]
    if hasattr(L, "tray_render_devices_progress"):
        L.tray_render_devices_progress.argtypes = L.tray_render_devices.argtypes + [PROGRESS_FN, vp]
    if hasattr(L, "tray_release_cache"):
        L.tray_release_cache.argtypes = [i32]
    if hasattr(L, "tray_scale_rgba"):
        L.tray_scale_rgba.argtypes = [vp, i32, i32, vp, i32, i32, i32, i32]
        L.tray_scale_rgba_async.argtypes = [vp, i32, i32, vp, i32, i32, i32, i32, vp]
    if hasattr(L, "tray_linear_to_srgba_async"):
        L.tray_linear_to_srgba_async.argtypes = [vp, ctypes.c_size_t, vp, i32, vp]
    L.tray_scene_upload.argtypes = [vp, i32, ctypes.POINTER(Background), i32, ctypes.POINTER(vp)]
    L.tray_scene_release.argtypes = [vp]
    if hasattr(L, "tray_scene_get_info"):  # absent from builds older than this binding (A/B tools)
        L.tray_scene_get_info.argtypes = [vp, ctypes.POINTER(SceneInfo)]
    if hasattr(L, "tray_render_plan_get"):
        L.tray_render_plan_get.argtypes = [vp, ctypes.POINTER(CameraState), ctypes.POINTER(Params), i32,
                                           ctypes.POINTER(RenderPlan)]
    L.tray_render_async.argtypes = [vp, ctypes.POINTER(CameraState), ctypes.POINTER(Params), vp, vp, vp]
    L.tray_render_stats_async.argtypes = [vp, ctypes.POINTER(CameraState), ctypes.POINTER(Params), vp, vp, vp]
    if hasattr(L, "tray_render_passes_async"):  # absent from older builds (A/B tools)
        L.tray_render_passes_async.argtypes = [vp, ctypes.POINTER(CameraState), ctypes.POINTER(Params), i32, vp, vp]
    L.tray_params_rows.argtypes = [ctypes.POINTER(Params)]
    L.tray_params_rows.restype = i32
    L.tray_to_srgba.argtypes = [vp, ctypes.c_size_t, vp]
    if hasattr(L, "tray_debug_set"):  # absent from older builds (A/B tools)
        L.tray_debug_set.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.tray_debug_clear.argtypes = [ctypes.c_char_p]
    _libs[path] = L
    return L


def check(rc: int) -> None:
    if rc != TRAY_OK:
        msg = lib().tray_last_error()
        raise TrayError(rc, msg.decode() if msg else "")


_knobs_now: dict = {}  # the knobs this process has set (they are process-wide in the library)


def set_debug_knobs(lib_path: str | None = None, **knobs) -> dict:
    """Sets include/tray_debug.h knobs (None unsets one) and returns their
    previous values. Test and A/B use only: the library never reads the
    environment, so this is the one way to reach them."""
    unknown = set(knobs) - set(DEBUG_KNOBS)
    if unknown:
        raise ValueError(f"unknown debug knobs {sorted(unknown)}")
    L = lib(lib_path)
    before = {k: _knobs_now.get(k) for k in knobs}
    for name, value in knobs.items():
        if value is None:
            rc = L.tray_debug_clear(name.encode())
            _knobs_now.pop(name, None)
        else:
            rc = L.tray_debug_set(name.encode(), int(value))
            _knobs_now[name] = int(value)
        if rc != TRAY_OK:
            raise TrayError(rc, L.tray_last_error().decode())
    return before


def clear_debug_knobs(lib_path: str | None = None) -> None:
    check(lib(lib_path).tray_debug_clear(None))
    _knobs_now.clear()


class debug_knobs:
    """`with debug_knobs(acc_slots=0): ...` sets knobs for the block and restores
    the previous values on exit."""

    def __init__(self, lib_path: str | None = None, **knobs):
        unknown = set(knobs) - set(DEBUG_KNOBS)
        if unknown:
            raise ValueError(f"unknown debug knobs {sorted(unknown)}")
        self.lib_path, self.knobs, self.saved = lib_path, knobs, {}

    def __enter__(self):
        self.saved = set_debug_knobs(self.lib_path, **self.knobs)
        return self

    def __exit__(self, et, ev, tb):
        set_debug_knobs(self.lib_path, **self.saved)
        return False


def code_object_sha256(path: str | None = None) -> str | None:
    """sha256 of the device code (the ELF section .hip_fatbin: every gfx950 kernel
    of the library) of a libtray_amd.so build. Profile records carry it
    (tools/pmc_summary.py, tools/pmc_mix.py) so that bench.py reuses counter
    figures only for the device code they were measured on; host-only changes
    leave it unchanged. None when the file has no such section."""
    import hashlib
    import struct

    with open(path or LIB_PATH, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:  # ELF64, little endian
        return None
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    for name_off, _type, _flags, _addr, off, size, *_ in secs:
        end = data.index(b"\0", names + name_off)
        if data[names + name_off:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()
    return None


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(lib().tray_device_count(ctypes.byref(n)))
    return n.value


def spheres_array(spheres) -> np.ndarray:
    a = np.ascontiguousarray(spheres if spheres is not None else np.zeros(0, SPHERE_DTYPE))
    if a.dtype != SPHERE_DTYPE:
        raise TypeError("spheres must use tray_amd._lib.SPHERE_DTYPE")
    return a


def make_params(width, height, max_depth, rays_per_pixel, ray_radius, seed, y_start=0, y_end=None,
                tile_rows=0, tile_count=1, tile_index=0, output=OUT_RGB_F64, flags=0, pass_=0) -> Params:
    return Params(width, height, max_depth, rays_per_pixel, float(ray_radius), int(seed) & (2**64 - 1), y_start,
                  height if y_end is None else y_end, tile_rows, tile_count, tile_index, output, flags, pass_)


def params_rows(p: Params) -> int:
    return int(lib().tray_params_rows(ctypes.byref(p)))


def render(spheres, background: Background, camera: CameraState, params: Params, device: int = 0,
           segments: bool = False, progress=None):
    """Synchronous tray_render into host memory. Returns (pixels, segments-or-None);
    pixels is (rows, W, 3) f64 / (rows, W, 3) f32 / (rows, W, 4) u8 by params.output.
    progress(rows): called (tray_render_progress) as rows finish while the device renders."""
    s = spheres_array(spheres)
    rows = params_rows(params)
    shape = {OUT_RGB_F64: (rows, params.width, 3), OUT_RGB_F32: (rows, params.width, 3),
             OUT_RGBA8: (rows, params.width, 4)}[params.output]
    dtype = {OUT_RGB_F64: np.float64, OUT_RGB_F32: np.float32, OUT_RGBA8: np.uint8}[params.output]
    out = np.zeros(shape, dtype=dtype)
    seg = np.zeros((rows, params.width), dtype=np.uint32) if segments else None
    args = (s.ctypes.data if len(s) else None, len(s), ctypes.byref(background), ctypes.byref(camera),
            ctypes.byref(params), device, out.ctypes.data,
            seg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) if seg is not None else None)
    if progress is None:
        check(lib().tray_render(*args))
    else:
        with _Progress(progress) as cb:
            check(lib().tray_render_progress(*args, cb.fn, None))
    return out, seg


class _Progress:
    """A Python progress callback behind tray_progress_fn. ctypes swallows an
    exception raised inside a callback; this keeps the first one, stops calling
    the function after it, and re-raises it when the render returns."""

    def __init__(self, fn):
        self.user, self.error = fn, None
        self.fn = PROGRESS_FN(self._call)  # kept alive for the call

    def _call(self, rows, _user):
        if self.error is not None:
            return
        try:
            self.user(int(rows))
        except BaseException as e:  # noqa: BLE001 - re-raised after the render
            self.error = e

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if et is None and self.error is not None:
            raise self.error
        return False


def render_devices(spheres, background: Background, camera: CameraState, params: Params, devices,
                   segments: bool = False, progress=None):
    """tray_render_devices: the row set split over `devices` (interleaved 1-row
    tiles, a device may repeat), rows returned in image order like render().
    progress(rows): tray_render_devices_progress, called as rows finish on any device."""
    s = spheres_array(spheres)
    rows = params_rows(params)
    ch = 4 if params.output == OUT_RGBA8 else 3
    dtype = {OUT_RGB_F64: np.float64, OUT_RGB_F32: np.float32, OUT_RGBA8: np.uint8}[params.output]
    out = np.zeros((rows, params.width, ch), dtype=dtype)
    seg = np.zeros((rows, params.width), dtype=np.uint32) if segments else None
    devs = (ctypes.c_int32 * len(devices))(*devices)
    args = (s.ctypes.data if len(s) else None, len(s), ctypes.byref(background), ctypes.byref(camera),
            ctypes.byref(params), devs, len(devices), out.ctypes.data,
            seg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)) if seg is not None else None)
    if progress is None:
        check(lib().tray_render_devices(*args))
    else:
        with _Progress(progress) as cb:
            check(lib().tray_render_devices_progress(*args, cb.fn, None))
    return out, seg


SCALE_NEAREST, SCALE_BILINEAR = 0, 1  # tray_scale_filter


def scale_rgba(src: np.ndarray, dw: int, dh: int, bilinear: bool, dst: np.ndarray | None = None,
               device: int = 0) -> np.ndarray:
    """tray_scale_rgba: x/image/draw BiLinear / NearestNeighbor .Scale of an [H, W, 4]
    uint8 image onto dst (a fresh zero image by default, as main.go:123), on the device."""
    a = np.ascontiguousarray(src, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("src must be [H, W, 4] uint8")
    out = np.zeros((dh, dw, 4), dtype=np.uint8) if dst is None else np.array(dst, dtype=np.uint8, copy=True)
    if out.shape != (dh, dw, 4):
        raise ValueError("dst must be [dh, dw, 4] uint8")
    check(lib().tray_scale_rgba(a.ctypes.data, a.shape[1], a.shape[0], out.ctypes.data, dw, dh,
                                SCALE_BILINEAR if bilinear else SCALE_NEAREST, device))
    return out


def release_cache(device: int = -1) -> None:
    """tray_release_cache: free what the synchronous renders keep on `device` (all: -1)."""
    check(lib().tray_release_cache(int(device)))


def linear_to_srgba_async(rgb_ptr: int, n_pixels: int, rgba_ptr: int, device: int = 0, stream: int | None = None):
    """tray_linear_to_srgba_async: ColorF.ToSRGBA over device buffers (n x 3 f64 -> n x 4 u8)."""
    check(lib().tray_linear_to_srgba_async(rgb_ptr, n_pixels, rgba_ptr, device, stream))


class DeviceScene:
    """A scene uploaded once to one device (tray_scene_upload); render many times,
    from any thread and on any streams: each render runs in a launch context of
    its own (work queue, sample buffer, candidate records; include/tray.h)."""

    def __init__(self, spheres, background: Background, device: int = 0, lib_path: str | None = None):
        self.L = lib(lib_path)
        s = spheres_array(spheres)
        h = ctypes.c_void_p()
        rc = self.L.tray_scene_upload(s.ctypes.data if len(s) else None, len(s), ctypes.byref(background), device,
                                      ctypes.byref(h))
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())
        self.handle = h
        self.device = device
        self.n = len(s)

    def render_async(self, camera: CameraState, params: Params, out_ptr: int, segments_ptr: int | None = None,
                     stream: int | None = None) -> None:
        rc = self.L.tray_render_async(self.handle, ctypes.byref(camera), ctypes.byref(params), out_ptr, segments_ptr,
                                      stream)
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())

    def render_passes_async(self, camera: CameraState, params: Params, n_passes: int, out_ptr: int,
                            stream: int | None = None) -> None:
        """Progressive passes params.pass_ .. + n_passes - 1 in one persistent launch;
        frame k at out_ptr + k * rows * width * bytes-per-pixel."""
        rc = self.L.tray_render_passes_async(self.handle, ctypes.byref(camera), ctypes.byref(params), int(n_passes),
                                             out_ptr, stream)
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())

    def render_stats_async(self, camera: CameraState, params: Params, out_ptr: int, stats_ptr: int,
                           stream: int | None = None) -> None:
        """Instrumented render (f32 output); stats_ptr -> 3 x uint64: segments, sphere tests, box tests."""
        rc = self.L.tray_render_stats_async(self.handle, ctypes.byref(camera), ctypes.byref(params), out_ptr,
                                            stats_ptr, stream)
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())

    def plan(self, camera: CameraState, params: Params, n_passes: int = 1) -> RenderPlan:
        """tray_render_plan_get: how render_async / render_passes_async would run."""
        out = RenderPlan()
        rc = self.L.tray_render_plan_get(self.handle, ctypes.byref(camera), ctypes.byref(params), int(n_passes),
                                         ctypes.byref(out))
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())
        return out

    def info(self) -> SceneInfo:
        out = SceneInfo()
        rc = self.L.tray_scene_get_info(self.handle, ctypes.byref(out))
        if rc != TRAY_OK:
            raise TrayError(rc, self.L.tray_last_error().decode())
        return out

    def release(self) -> None:
        if self.handle:
            self.L.tray_scene_release(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass
