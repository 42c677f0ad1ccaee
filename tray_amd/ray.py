"""Host-side mirror of fortio/tray's `ray` package API over the MI355X C-ABI.

Same names, field meanings and defaulting as the Go package, so code written
against `ray.New(w, h)` / `(*Tracer).Render(scene)` reads the same here:

    Go (ray/)                                   here (tray_amd.ray)
    New(w, h) *Tracer           tracer.go:38    New(w, h) -> Tracer
    (*Tracer).Render(*Scene)    tracer.go:48    Tracer.Render(scene) -> (H, W, 4) uint8 RGBA
    (*Tracer).RenderLines(...)  tracer.go:120   Tracer.RenderLines(idx, yStart, yEnd, scene)
    Camera / Initialize         camera.go:9,43  Camera / Camera.Initialize(w, h)
    RichSceneCamera()           camera.go:144   RichSceneCamera()
    Scene / Sphere / AmbientLight objects.go    Scene / Sphere / AmbientLight
    Lambertian/Metal/Dielectric materials.go    Lambertian / Metal / Dielectric
    DefaultScene(), RichScene(rng) objects.go   DefaultScene(), RichScene(seed)
    DefaultBackground()         objects.go:106  DefaultBackground()

The hot loop (everything under RenderLines) runs in the gfx950 megakernel via
tray_amd._lib; this module only applies the Go defaults and marshals data.
Differences by design: RichScene takes a seed (the scene stream is the counter
RNG of include/tray.h, not fortio.org/rand), NumWorkers is kept for API parity
but the parallelism is the GPU grid, and `idx` of RenderLines is accepted and
ignored (draws are keyed by pixel, not by row chunk).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib

Vec3 = tuple  # (x, y, z) — value semantics like the Go struct
ColorF = tuple


def _v(v) -> tuple:
    t = tuple(float(c) for c in v)
    if len(t) != 3:
        raise ValueError("expected 3 components")
    return t


# ------------------------------------------------------------------ materials
@dataclass(frozen=True)
class Lambertian:  # ray/materials.go:9-11
    Albedo: ColorF = (0.0, 0.0, 0.0)


@dataclass(frozen=True)
class Metal:  # ray/materials.go:23-26
    Albedo: ColorF = (0.0, 0.0, 0.0)
    Fuzz: float = 0.0


@dataclass(frozen=True)
class Dielectric:  # ray/materials.go:40-42
    RefIdx: float = 1.0


@dataclass
class Sphere:  # ray/objects.go:75-79
    Center: Vec3
    Radius: float
    Mat: object


@dataclass
class AmbientLight:  # ray/objects.go:64-66
    ColorA: ColorF = (0.0, 0.0, 0.0)
    ColorB: ColorF = (0.0, 0.0, 0.0)


def DefaultBackground() -> AmbientLight:  # ray/objects.go:106-110
    return AmbientLight((1.0, 1.0, 1.0), (0.4, 0.65, 1.0))


@dataclass
class Scene:  # ray/objects.go:32-35
    Objects: list = field(default_factory=list)
    Background: AmbientLight = field(default_factory=AmbientLight)

    def to_array(self) -> np.ndarray:
        """Flatten to the C-ABI's tray_sphere array; unsupported objects raise
        (the Go Hittable/Material interfaces are open, the device path is not)."""
        out = np.zeros(len(self.Objects), dtype=_lib.SPHERE_DTYPE)
        for i, o in enumerate(self.Objects):
            if not isinstance(o, Sphere):
                raise _lib.TrayError(_lib.TRAY_ERR_UNSUPPORTED, f"object {i} is not a Sphere")
            out[i]["center"] = _v(o.Center)
            out[i]["radius"] = float(o.Radius)
            m = o.Mat
            if isinstance(m, Lambertian):
                out[i]["material"], out[i]["albedo"] = _lib.LAMBERTIAN, _v(m.Albedo)
            elif isinstance(m, Metal):
                out[i]["material"], out[i]["albedo"], out[i]["param"] = _lib.METAL, _v(m.Albedo), float(m.Fuzz)
            elif isinstance(m, Dielectric):
                out[i]["material"], out[i]["param"] = _lib.DIELECTRIC, float(m.RefIdx)
            else:
                raise _lib.TrayError(_lib.TRAY_ERR_UNSUPPORTED, f"object {i}: unsupported material {type(m)}")
        return out

    @staticmethod
    def from_array(spheres: np.ndarray, background: AmbientLight | None = None) -> "Scene":
        objs = []
        for s in spheres:
            kind = int(s["material"])
            if kind == _lib.LAMBERTIAN:
                mat = Lambertian(tuple(s["albedo"].tolist()))
            elif kind == _lib.METAL:
                mat = Metal(tuple(s["albedo"].tolist()), float(s["param"]))
            else:
                mat = Dielectric(float(s["param"]))
            objs.append(Sphere(tuple(s["center"].tolist()), float(s["radius"]), mat))
        return Scene(objs, background or AmbientLight())


def _background(bg: AmbientLight) -> _lib.Background:
    return _lib.Background((ctypes.c_double * 3)(*_v(bg.ColorA)), (ctypes.c_double * 3)(*_v(bg.ColorB)))


def DefaultScene() -> Scene:  # ray/objects.go:112-130
    arr = np.zeros(5, dtype=_lib.SPHERE_DTYPE)
    n = ctypes.c_int32()
    _lib.check(_lib.lib().tray_default_scene(arr.ctypes.data, 5, ctypes.byref(n)))
    return Scene.from_array(arr[: n.value], DefaultBackground())


def rich_scene_array(seed: int, half_extent: int = 11) -> np.ndarray:
    cap = _lib.lib().tray_rich_scene_capacity(half_extent)
    arr = np.zeros(cap, dtype=_lib.SPHERE_DTYPE)
    n = ctypes.c_int32()
    _lib.check(_lib.lib().tray_rich_scene(int(seed) & (2**64 - 1), half_extent, arr.ctypes.data, cap,
                                          ctypes.byref(n)))
    return arr[: n.value].copy()


def RichScene(seed: int, half_extent: int = 11) -> Scene:  # ray/objects.go:132-175
    """Book-cover scene; Background left zero like the Go function (Render defaults it)."""
    return Scene.from_array(rich_scene_array(seed, half_extent))


# --------------------------------------------------------------------- camera
@dataclass
class Camera:  # ray/camera.go:9-39
    Position: Vec3 = (0.0, 0.0, 0.0)
    LookAt: Vec3 = (0.0, 0.0, 0.0)
    Up: Vec3 = (0.0, 0.0, 0.0)
    VerticalFoV: float = 0.0
    FocalLength: float = 0.0
    FocusDistance: float = 0.0
    Aperture: float = 0.0
    _state: _lib.CameraState | None = field(default=None, repr=False, compare=False)

    def Initialize(self, width: int, height: int) -> None:  # ray/camera.go:43-105
        cs = _lib.CameraSetup((ctypes.c_double * 3)(*_v(self.Position)), (ctypes.c_double * 3)(*_v(self.LookAt)),
                              (ctypes.c_double * 3)(*_v(self.Up)), float(self.VerticalFoV),
                              float(self.FocalLength), float(self.FocusDistance), float(self.Aperture))
        st = _lib.CameraState()
        _lib.check(_lib.lib().tray_camera_initialize(ctypes.byref(cs), width, height, ctypes.byref(st)))
        self.Position, self.LookAt, self.Up = tuple(cs.position), tuple(cs.look_at), tuple(cs.up)
        self.VerticalFoV, self.FocalLength = cs.vertical_fov, cs.focal_length
        self.FocusDistance, self.Aperture = cs.focus_distance, cs.aperture
        self._state = st

    # computed fields, named as in camera.go:34-39
    @property
    def pixel00(self) -> Vec3:
        return tuple(self._state.pixel00)

    @property
    def pixelXVector(self) -> Vec3:
        return tuple(self._state.pixel_x)

    @property
    def pixelYVector(self) -> Vec3:
        return tuple(self._state.pixel_y)

    @property
    def defocusDiskU(self) -> Vec3:
        return tuple(self._state.defocus_u)

    @property
    def defocusDiskV(self) -> Vec3:
        return tuple(self._state.defocus_v)


def RichSceneCamera() -> Camera:  # ray/camera.go:144-154
    cs = _lib.CameraSetup()
    _lib.check(_lib.lib().tray_rich_scene_camera(ctypes.byref(cs)))
    return Camera(tuple(cs.position), tuple(cs.look_at), tuple(cs.up), cs.vertical_fov, cs.focal_length,
                  cs.focus_distance, cs.aperture)


# --------------------------------------------------------------------- tracer
_CAMERA_FIELDS = ("Position", "LookAt", "Up", "VerticalFoV", "FocalLength", "FocusDistance", "Aperture")


class Tracer:  # ray/tracer.go:25-36
    """Go's Tracer embeds Camera: t.Position etc. forward to t.Camera."""

    def __init__(self, width: int, height: int):
        object.__setattr__(self, "Camera", Camera())
        self.MaxDepth = 0
        self.NumRaysPerPixel = 0
        self.RayRadius = 0.0
        self.NumWorkers = 0
        self.ProgressFunc = None
        self.Seed = 0
        self.Device = 0  # which gfx950 device renders (no Go counterpart)
        self.Devices = None  # several devices: rows split over them (tray_render_devices; no Go counterpart)
        self.width = width
        self.height = height
        self.imageData = np.zeros((height, width, 4), dtype=np.uint8)  # image.NewRGBA, tracer.go:43
        self.linear = np.zeros((height, width, 3), dtype=np.float64)   # FP64 mean colour (parity format)
        self.segments = np.zeros((height, width), dtype=np.uint32)     # Scene.Hit calls per pixel

    def __getattr__(self, name):
        if name in _CAMERA_FIELDS:
            return getattr(object.__getattribute__(self, "Camera"), name)
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in _CAMERA_FIELDS:
            setattr(self.Camera, name, value)
        else:
            object.__setattr__(self, name, value)

    def _apply_defaults(self, scene: Scene | None) -> Scene:  # ray/tracer.go:50-79
        if scene is None:
            scene = DefaultScene()
            self.Position = (-2.0, 2.0, 1.0)
            self.LookAt = (0.0, 0.0, -1.0)
            self.VerticalFoV = 20.0
            self.Aperture = 0.1
            d = [p - q for p, q in zip(self.Position, self.LookAt)]
            self.FocusDistance = math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])
        zero = (0.0, 0.0, 0.0)
        if tuple(scene.Background.ColorA) == zero and tuple(scene.Background.ColorB) == zero:
            scene.Background = DefaultBackground()
        if self.MaxDepth <= 0:
            self.MaxDepth = 10
        if self.NumRaysPerPixel <= 0:
            self.NumRaysPerPixel = 1
        if self.RayRadius <= 0:
            self.RayRadius = 0.5
        if self.NumWorkers <= 0:
            self.NumWorkers = os.cpu_count() or 1  # runtime.GOMAXPROCS(0)
        return scene

    def _seed(self) -> int:
        # Seed 0 means "randomized each time" (tracer.go:33).
        return self.Seed if self.Seed else int.from_bytes(os.urandom(8), "little") or 1

    def _render_rows(self, y0: int, y1: int, scene: Scene) -> None:
        params = _lib.make_params(self.width, self.height, self.MaxDepth, self.NumRaysPerPixel, self.RayRadius,
                                  self._seed(), y0, y1)
        progress = None
        if self.ProgressFunc is not None:  # per row, while the device renders (tracer.go:126-128)
            def progress(rows):
                for _ in range(rows):
                    self.ProgressFunc(self.width)
        if self.Devices and len(self.Devices) > 1:  # one process, several GPUs, live progress from all of them
            rgb, seg = _lib.render_devices(scene.to_array(), _background(scene.Background), self.Camera._state,
                                           params, list(self.Devices), segments=True, progress=progress)
        else:
            rgb, seg = _lib.render(scene.to_array(), _background(scene.Background), self.Camera._state, params,
                                   self.Devices[0] if self.Devices else self.Device, segments=True,
                                   progress=progress)
        self.linear[y0:y1] = rgb
        self.segments[y0:y1] = seg
        rgba = np.zeros((y1 - y0, self.width, 4), dtype=np.uint8)
        _lib.check(_lib.lib().tray_to_srgba(rgb.ctypes.data, rgb.shape[0] * rgb.shape[1], rgba.ctypes.data))
        self.imageData[y0:y1] = rgba

    def Render(self, scene: Scene | None) -> np.ndarray:  # ray/tracer.go:48-118
        scene = self._apply_defaults(scene)
        self.Camera.Initialize(self.width, self.height)
        self._render_rows(0, self.height, scene)
        return self.imageData

    def RenderLines(self, idx: int, yStart: int, yEnd: int, scene: Scene) -> None:  # ray/tracer.go:120-155
        """Render rows [yStart, yEnd) with the current (initialized) camera and
        fields; like Go, no defaulting happens here."""
        if self.Camera._state is None:
            raise _lib.TrayError(_lib.TRAY_ERR_INVALID_ARGUMENT, "Camera.Initialize must be called first")
        self._render_rows(yStart, yEnd, scene)


def New(width: int, height: int) -> Tracer:  # ray/tracer.go:38-45
    return Tracer(width, height)
