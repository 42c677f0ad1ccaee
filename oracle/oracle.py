"""ORACLE — test infrastructure only (ctypes wrapper over oracle/libtray_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. It is the CHECKER for the HIP path in tray_amd/, never a fallback
for it. The C restatement it wraps cites the fortio/tray file:line of every
function it follows (oracle/tray_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libtray_oracle.so")

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

LAMBERTIAN, METAL, DIELECTRIC = 1, 2, 3
P_CAMERA, P_SCATTER, P_SCENE = 1, 3, 4

_dp = ctypes.POINTER(ctypes.c_double)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p


def build() -> str:
    """Compile the oracle with its committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_render_rows.argtypes = [_vp, ctypes.c_int, _dp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_double, ctypes.c_uint64, _i32p, ctypes.c_int,
                                         ctypes.c_int, _dp, _u32p, ctypes.c_int]
        L.oracle_render_pixels.argtypes = [_vp, ctypes.c_int, _dp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_double, ctypes.c_uint64, _i32p, _i32p,
                                           ctypes.c_int, _dp, _u32p, ctypes.c_int]
        L.oracle_ray_color.argtypes = [_vp, ctypes.c_int, _dp, _dp, _dp, ctypes.c_int, ctypes.c_uint64,
                                       ctypes.c_uint32, ctypes.c_uint32, _dp, _u32p]
        L.oracle_philox4x32_10.argtypes = [_u32p, _u32p, _u32p]
        L.oracle_draw_key.argtypes = [ctypes.c_uint64, _u32p]
        L.oracle_draw_block.argtypes = [_u32p] + [ctypes.c_uint32] * 4 + [_u32p]
        L.oracle_uniforms.argtypes = [ctypes.c_uint64] + [ctypes.c_uint32] * 4 + [_dp]
        L.oracle_unit_vector.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _dp]
        L.oracle_in_disc.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_double, _dp]
        L.oracle_sincos_2pi.argtypes = [ctypes.c_double, _dp]
        L.oracle_reflect.argtypes = [_dp, _dp, _dp]
        L.oracle_refract.argtypes = [_dp, _dp, ctypes.c_double, _dp]
        L.oracle_reflectance.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oracle_reflectance.restype = ctypes.c_double
        L.oracle_near_zero.argtypes = [_dp]
        L.oracle_unit.argtypes = [_dp, _dp]
        L.oracle_sphere_hit.argtypes = [_vp, _dp, _dp, ctypes.c_double, ctypes.c_double, _dp]
        L.oracle_scene_hit.argtypes = [_vp, ctypes.c_int, _dp, _dp, ctypes.c_double, ctypes.c_double, _dp]
        L.oracle_scatter.argtypes = [_vp, _dp, _dp, _dp, _dp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, _dp, _dp, _dp]
        L.oracle_get_ray.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp, _dp]
        L.oracle_linear_to_srgb.argtypes = [ctypes.c_double]
        L.oracle_linear_to_srgb.restype = ctypes.c_uint8
        L.oracle_linear_to_srgb_n.argtypes = [_dp, ctypes.c_size_t, _vp]
        L.oracle_go_tan.argtypes = [ctypes.c_double]
        L.oracle_go_tan.restype = ctypes.c_double
        L.oracle_camera_initialize.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp]
        L.oracle_rich_scene.argtypes = [ctypes.c_uint64, ctypes.c_int, _vp, ctypes.c_int]
        L.oracle_default_scene.argtypes = [_vp, ctypes.c_int]
        for fn in (L.oracle_scale_bilinear_rgba, L.oracle_scale_nearest_rgba):
            fn.argtypes = [_vp, ctypes.c_int32, ctypes.c_int32, _vp, ctypes.c_int32, ctypes.c_int32]
        _lib = L
    return _lib


def _d(a) -> ctypes.POINTER(ctypes.c_double):
    return a.ctypes.data_as(_dp)


def _f64(v, n=None) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(v, dtype=np.float64))
    if n is not None:
        assert a.size == n
    return a


def _spheres(spheres) -> np.ndarray:
    if spheres is None:
        return np.zeros(0, dtype=SPHERE_DTYPE)
    a = np.ascontiguousarray(spheres)
    assert a.dtype == SPHERE_DTYPE
    return a


# ----------------------------------------------------------------- RNG ------
def philox4x32_10(ctr, key) -> tuple[int, int, int, int]:
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return tuple(o)


def draw_key(seed) -> tuple[int, int, int, int]:
    """The renderer's draw key of a seed (include/tray.h, ABI 6)."""
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_draw_key(seed, o)
    return tuple(o)


def draw_block(key, pixel, sample, bounce, purpose) -> tuple[int, int, int, int]:
    """The renderer's draw block (include/tray.h, ABI 6): keyed pcg4d + xorshift-16."""
    k = (ctypes.c_uint32 * 4)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_draw_block(k, pixel, sample, bounce, purpose, o)
    return tuple(o)


def uniforms(seed, c0, c1, c2, c3) -> tuple[float, float]:
    o = np.zeros(2)
    lib().oracle_uniforms(seed, c0, c1, c2, c3, _d(o))
    return float(o[0]), float(o[1])


def unit_vector(seed, pixel, sample, bounce) -> np.ndarray:
    o = np.zeros(3)
    lib().oracle_unit_vector(seed, pixel, sample, bounce, _d(o))
    return o


def in_disc(seed, pixel, sample, which, radius) -> np.ndarray:
    """which = 0: anti-aliasing disc (camera block words 0,1); 1: lens disc (words 2,3)."""
    o = np.zeros(2)
    lib().oracle_in_disc(seed, pixel, sample, which, radius, _d(o))
    return o


def sincos_2pi(u) -> np.ndarray:
    o = np.zeros(2)
    lib().oracle_sincos_2pi(u, _d(o))
    return o


# ---------------------------------------------------------------- math ------
def reflect(v, n) -> np.ndarray:
    o = np.zeros(3)
    lib().oracle_reflect(_d(_f64(v, 3)), _d(_f64(n, 3)), _d(o))
    return o


def refract(uv, n, eta) -> np.ndarray:
    o = np.zeros(3)
    lib().oracle_refract(_d(_f64(uv, 3)), _d(_f64(n, 3)), eta, _d(o))
    return o


def reflectance(cosine, ref_idx) -> float:
    return lib().oracle_reflectance(cosine, ref_idx)


def near_zero(v) -> bool:
    return bool(lib().oracle_near_zero(_d(_f64(v, 3))))


def unit(v) -> np.ndarray:
    o = np.zeros(3)
    lib().oracle_unit(_d(_f64(v, 3)), _d(o))
    return o


def linear_to_srgb(c: float) -> int:
    return int(lib().oracle_linear_to_srgb(c))


def go_tan(x: float) -> float:
    """Go's math.Tan as restated for Camera.Initialize (ray/camera.go:93)."""
    return float(lib().oracle_go_tan(x))


def linear_to_srgb_n(c: np.ndarray) -> np.ndarray:
    """oracle_linear_to_srgb elementwise over any float64 array -> uint8 of the same shape."""
    flat = np.ascontiguousarray(np.asarray(c, dtype=np.float64).reshape(-1))
    out = np.empty(flat.shape[0], dtype=np.uint8)
    lib().oracle_linear_to_srgb_n(_d(flat), flat.shape[0], out.ctypes.data)
    return out.reshape(np.shape(c))


def to_srgba(rgb: np.ndarray) -> np.ndarray:
    """ColorF.ToSRGBA over an (..., 3) array -> (..., 4) uint8."""
    rgb = np.asarray(rgb, dtype=np.float64)
    out = np.empty(rgb.shape[:-1] + (4,), dtype=np.uint8)
    out[..., :3] = linear_to_srgb_n(rgb)
    out[..., 3] = 255
    return out


def sphere_hit(sphere, origin, direction, t_start, t_end):
    s = _spheres(sphere).reshape(-1)[:1]
    rec = np.zeros(8)
    hit = lib().oracle_sphere_hit(s.ctypes.data, _d(_f64(origin, 3)), _d(_f64(direction, 3)), t_start, t_end,
                                  _d(rec))
    return bool(hit), rec


def scene_hit(spheres, origin, direction, t_start, t_end):
    s = _spheres(spheres)
    rec = np.zeros(8)
    idx = lib().oracle_scene_hit(s.ctypes.data, len(s), _d(_f64(origin, 3)), _d(_f64(direction, 3)), t_start,
                                 t_end, _d(rec))
    return idx, rec


def scatter(sphere, in_origin, in_dir, point, normal, front_face, seed=1, pixel=0, sample=0, bounce=0):
    s = _spheres(sphere).reshape(-1)[:1]
    att, o, d = np.zeros(3), np.zeros(3), np.zeros(3)
    r = lib().oracle_scatter(s.ctypes.data, _d(_f64(in_origin, 3)), _d(_f64(in_dir, 3)), _d(_f64(point, 3)),
                             _d(_f64(normal, 3)), int(bool(front_face)), seed, pixel, sample, bounce, _d(att),
                             _d(o), _d(d))
    if r < 0:
        raise ValueError("unsupported material")
    return bool(r), att, o, d


def get_ray(camera, px, py, ox=0.0, oy=0.0, seed=1, pixel=0, sample=0):
    o, d = np.zeros(3), np.zeros(3)
    lib().oracle_get_ray(_f64(camera, 21).ctypes.data, seed, pixel, sample, px, py, ox, oy, _d(o), _d(d))
    return o, d


# ------------------------------------------------------------ host setup ----
CAMERA_SETUP_FIELDS = ("position", "look_at", "up", "vertical_fov", "focal_length", "focus_distance", "aperture")


def camera_initialize(setup: np.ndarray, width: int, height: int) -> tuple[np.ndarray, np.ndarray]:
    """Camera.Initialize: setup = 13 doubles (pos3, lookat3, up3, vfov, focal, focus, aperture).
    Returns (resolved setup with defaults, camera 21 doubles)."""
    io = _f64(setup, 13).copy()
    cam = np.zeros(21)
    lib().oracle_camera_initialize(_d(io), width, height, _d(cam))
    return io, cam


def rich_scene(seed: int, half_extent: int = 11) -> np.ndarray:
    cap = (2 * half_extent) ** 2 + 4
    out = np.zeros(cap, dtype=SPHERE_DTYPE)
    n = lib().oracle_rich_scene(seed, half_extent, out.ctypes.data, cap)
    assert n > 0
    return out[:n].copy()


def default_scene() -> np.ndarray:
    out = np.zeros(5, dtype=SPHERE_DTYPE)
    n = lib().oracle_default_scene(out.ctypes.data, 5)
    assert n == 5
    return out


DEFAULT_BACKGROUND = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])  # ray/objects.go:106-110


# ---------------------------------------------------------------- render ----
def render_rows(spheres, background, camera, width, height, spp, max_depth, ray_radius, seed, rows,
                workers=1, segments=True, pass_=0):
    """Render a list of image rows -> (len(rows), W, 3) float64 [+ (len(rows), W) uint32 segments]."""
    s = _spheres(spheres)
    rows = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
    out = np.zeros((len(rows), width, 3))
    seg = np.zeros((len(rows), width), dtype=np.uint32) if segments else None
    rc = lib().oracle_render_rows(s.ctypes.data, len(s), _d(_f64(background, 6)), _f64(camera, 21).ctypes.data,
                                  width, height, spp, max_depth, ray_radius, seed, rows.ctypes.data_as(_i32p),
                                  len(rows), workers, _d(out), seg.ctypes.data_as(_u32p) if seg is not None else None,
                                  int(pass_))
    if rc != 0:
        raise ValueError(f"oracle_render_rows failed: {rc}")
    return (out, seg) if segments else out


def render(spheres, background, camera, width, height, spp, max_depth, ray_radius, seed, y_start=0, y_end=None,
           workers=1, segments=True, pass_=0):
    y_end = height if y_end is None else y_end
    return render_rows(spheres, background, camera, width, height, spp, max_depth, ray_radius, seed,
                       np.arange(y_start, y_end, dtype=np.int32), workers, segments, pass_)


def render_pixels(spheres, background, camera, width, height, spp, max_depth, ray_radius, seed, xs, ys, pass_=0):
    s = _spheres(spheres)
    xs = np.ascontiguousarray(np.asarray(xs, dtype=np.int32))
    ys = np.ascontiguousarray(np.asarray(ys, dtype=np.int32))
    out = np.zeros((len(xs), 3))
    seg = np.zeros(len(xs), dtype=np.uint32)
    rc = lib().oracle_render_pixels(s.ctypes.data, len(s), _d(_f64(background, 6)), _f64(camera, 21).ctypes.data,
                                    width, height, spp, max_depth, ray_radius, seed, xs.ctypes.data_as(_i32p),
                                    ys.ctypes.data_as(_i32p), len(xs), _d(out), seg.ctypes.data_as(_u32p), int(pass_))
    if rc != 0:
        raise ValueError(f"oracle_render_pixels failed: {rc}")
    return out, seg


def ray_color(spheres, background, origin, direction, depth, seed=1, pixel=0, sample=0):
    s = _spheres(spheres)
    out = np.zeros(3)
    seg = ctypes.c_uint32(0)
    rc = lib().oracle_ray_color(s.ctypes.data, len(s), _d(_f64(background, 6)), _d(_f64(origin, 3)),
                                _d(_f64(direction, 3)), depth, seed, pixel, sample, _d(out), ctypes.byref(seg))
    if rc != 0:
        raise ValueError("unsupported material")
    return out, seg.value


# ------------------------------------------------------- terminal downscale --
def scale_rgba(src: np.ndarray, dw: int, dh: int, bilinear: bool, dst: np.ndarray | None = None) -> np.ndarray:
    """x/image/draw {BiLinear,NearestNeighbor}.Scale(dst, dst.Bounds(), src, src.Bounds(), Over, nil)
    for [H, W, 4] uint8 images (main.go:121-128: dst is a fresh, zero image unless given)."""
    a = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = a.shape[:2]
    out = np.zeros((dh, dw, 4), dtype=np.uint8) if dst is None else np.ascontiguousarray(dst, dtype=np.uint8).copy()
    fn = lib().oracle_scale_bilinear_rgba if bilinear else lib().oracle_scale_nearest_rgba
    if fn(a.ctypes.data, sw, sh, out.ctypes.data, dw, dh) != 0:
        raise ValueError("bad sizes")
    return out
