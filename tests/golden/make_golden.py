"""Generate the committed golden fixtures in tests/golden/ (run from the repo root).

    python tests/golden/make_golden.py [--reference /root/reference]

1. rngfree_*.npz — RNG-FREE scenes rendered by an INDEPENDENT numpy restatement
   of the reference written straight from the Go source (not from oracle/).
   With rays_per_pixel = 1 (no AA draw, ray/tracer.go:122,136), Aperture = 0
   (no lens draw, ray/camera.go:126) and only Metal{Fuzz: 0} spheres (no
   scatter draw, ray/materials.go:30) the output is a pure function of the
   reference's arithmetic, so the C oracle and the HIP kernel must match it
   without any RNG assumption. Camera vectors come from the same numpy
   restatement of Camera.Initialize (ray/camera.go:43-105).
2. example_sky_rows.npz — rows 0..48 of the reference's own output image
   example.png (`tray -save example.png -r 64 -s 8 -d 50 -seed 2` on a 160x45
   terminal, README.md:30-31 = 1280x720, r=64, d=50). These rows are sky
   only, so they pin camera + AmbientLight + LinearToSrgb against the real Go
   binary independently of its RNG.

numpy elementwise float64 ops are IEEE-754 binary64 with no FMA contraction,
sqrt/division correctly rounded; evaluation order below follows the Go source.
"""
from __future__ import annotations

import argparse
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

SPHERE_DTYPE = np.dtype([("center", "<f8", (3,)), ("radius", "<f8"), ("albedo", "<f8", (3,)), ("param", "<f8"),
                         ("material", "<i4"), ("reserved", "<i4")])
METAL = 2


# ---------------------------------------------------------------- vec3.go ----
def add(u, v):  # Add(u, v) = {v.x + u.x, ...}
    return (v[0] + u[0], v[1] + u[1], v[2] + u[2])


def sub(u, v):
    return (u[0] - v[0], u[1] - v[1], u[2] - v[2])


def smul(v, t):
    return (v[0] * t, v[1] * t, v[2] * t)


def mul(u, v):
    return (u[0] * v[0], u[1] * v[1], u[2] * v[2])


def dot(u, v):
    return u[0] * v[0] + u[1] * v[1] + u[2] * v[2]


def unit(v):
    length = np.sqrt(dot(v, v))
    return (v[0] / length, v[1] / length, v[2] / length)


def cross(u, v):
    return (u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0])


def reflect(v, n):  # Sub(v, SMul(n, 2*Dot(v, n)))
    return sub(v, smul(n, 2 * dot(v, n)))


# -------------------------------------------------------- camera.go (host) ----
_TAN_P = (-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7)
_TAN_Q = (1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7,
          -5.38695755929454629881e7)


def go_tan(x):
    """Go's math.Tan (src/math/tan.go, Cephes coefficients; no FMA, as GOAMD64=v1
    compiles it) for |x| < 2^29, in Python floats (IEEE binary64)."""
    pi4a, pi4b, pi4c = 7.85398125648498535156e-1, 3.77489470793079817668e-8, 2.69515142907905952645e-15
    if x == 0 or x != x:
        return x
    sign = x < 0
    x = -x if sign else x
    assert x < 2.0 ** 29
    j = int(x * float.fromhex("0x1.45f306dc9c883p+0"))  # x * (4/Pi), the constant rounded once
    y = float(j)
    if j & 1:
        j, y = j + 1, y + 1
    z = ((x - y * pi4a) - y * pi4b) - y * pi4c
    zz = z * z
    if zz > 1e-14:
        y = z + z * (zz * (((_TAN_P[0] * zz) + _TAN_P[1]) * zz + _TAN_P[2])
                     / ((((zz + _TAN_Q[1]) * zz + _TAN_Q[2]) * zz + _TAN_Q[3]) * zz + _TAN_Q[4]))
    else:
        y = z
    if j & 2:
        y = -1 / y
    return -y if sign else y


def camera_initialize(position, look_at, up, vfov, focal, width, height):
    f64 = np.float64
    position = tuple(f64(c) for c in position)
    view = sub(position, tuple(f64(c) for c in look_at))
    w = unit(view)
    u = unit(cross(tuple(f64(c) for c in up), w))
    v = cross(w, u)
    theta = f64(vfov) * f64(float.fromhex("0x1.1df46a2529d39p-6"))  # math.Pi/180, folded exactly by Go
    viewport_h = f64(2.0) * f64(focal) * f64(go_tan(float(theta / f64(2.0))))
    viewport_w = (f64(width) / f64(height)) * viewport_h
    horizontal = smul(u, viewport_w)
    vertical = smul(v, -viewport_h)
    px = smul(horizontal, f64(1.0))
    px = (px[0] / f64(width), px[1] / f64(width), px[2] / f64(width))
    py = (vertical[0] / f64(height), vertical[1] / f64(height), vertical[2] / f64(height))
    upper_left = sub(position, add(add(smul(w, f64(focal)), smul(horizontal, f64(0.5))), smul(vertical, f64(0.5))))
    p00 = add(upper_left, smul(add(px, py), f64(0.5)))
    zero = (f64(0), f64(0), f64(0))
    # tray_camera layout: position, pixel00, pixel_x, pixel_y, defocus_u, defocus_v, aperture, focus, focal
    return np.array([*position, *p00, *px, *py, *zero, *zero, 0.0, float(focal), float(focal)])


# ---------------------------------------------------- objects.go, vectorised --
def render_rngfree(spheres, cam, width, height, max_depth, bg):
    """Vectorised over all pixels: RenderLines with r=1 (tracer.go:120-155) ->
    GetRay without aperture (camera.go:113-124) -> RayColor (objects.go:49-62)
    with Metal{Fuzz:0}.Scatter (materials.go:28-37). Inner-first attenuation
    product, as the Go recursion computes it."""
    ys, xs = np.mgrid[0:height, 0:width]
    xs = xs.ravel().astype(np.float64)
    ys = ys.ravel().astype(np.float64)
    npx = xs.size
    pos, p00, pxv, pyv = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    sample = add(add(tuple(p00), smul(tuple(pxv), xs + 0.0)), smul(tuple(pyv), ys + 0.0))
    org = tuple(np.full(npx, c) for c in pos)
    dirn = sub(sample, tuple(pos))
    alive = np.ones(npx, dtype=bool)
    segments = np.zeros(npx, dtype=np.uint32)
    atts = []  # per bounce: (attenuation tuple, mask of lanes that scattered)
    final = (np.zeros(npx), np.zeros(npx), np.zeros(npx))  # colour returned at the deepest level
    for depth in range(max_depth, 0, -1):
        segments += alive
        # Scene.Hit: linear scan, strict shrink (objects.go:37-46)
        closest = np.full(npx, np.inf)
        best = np.full(npx, -1)
        a = dot(dirn, dirn)
        for i, s in enumerate(spheres):
            c = tuple(s["center"])
            oc = sub(c, org)
            h = dot(dirn, oc)
            cc = dot(oc, oc) - s["radius"] * s["radius"]
            disc = h * h - a * cc
            ok = disc >= 0
            sq = np.sqrt(np.where(ok, disc, 0.0))
            with np.errstate(invalid="ignore", divide="ignore"):
                r1 = (h - sq) / a
                r2 = (h + sq) / a
            in1 = (r1 > 1e-6) & (r1 < closest)
            in2 = (r2 > 1e-6) & (r2 < closest)
            root = np.where(in1, r1, r2)
            hit = ok & alive & (in1 | in2)
            closest = np.where(hit, root, closest)
            best = np.where(hit, i, best)
        hit_any = best >= 0
        # sky for the lanes that missed (AmbientLight.Hit, objects.go:68-73)
        miss = alive & ~hit_any
        u = unit(dirn)
        t = 0.5 * (u[1] + 1.0)
        sky = add(smul(tuple(bg[0:3]), 1.0 - t), smul(tuple(bg[3:6]), t))
        final = tuple(np.where(miss, sky[k], final[k]) for k in range(3))
        # hit lanes: HitRecord (objects.go:95-102) + Metal scatter
        hb = np.where(hit_any, best, 0)
        cen = tuple(spheres["center"][hb, k] for k in range(3))
        rad = spheres["radius"][hb]
        point = add(org, smul(dirn, closest))
        outward = sub(point, cen)
        outward = (outward[0] / rad, outward[1] / rad, outward[2] / rad)
        front = dot(dirn, outward) < 0
        normal = tuple(np.where(front, outward[k], -outward[k]) for k in range(3))
        reflected = reflect(unit(dirn), normal)
        scat = alive & hit_any & (dot(reflected, normal) > 0)
        att = tuple(spheres["albedo"][hb, k] for k in range(3))
        atts.append((att, scat))
        # absorbed lanes end black; scattered lanes continue
        final = tuple(np.where(alive & hit_any, 0.0, final[k]) for k in range(3))
        org = tuple(np.where(scat, point[k], org[k]) for k in range(3))
        dirn = tuple(np.where(scat, reflected[k], dirn[k]) for k in range(3))
        alive = scat
    # lanes still alive after max_depth hits: RayColor(depth 0) -> black (already 0)
    col = final
    for att, scat in reversed(atts):  # Mul(attenuation, RayColor(...)), innermost first
        col = tuple(np.where(scat, att[k] * col[k], col[k]) for k in range(3))
    img = np.stack(col, axis=-1).reshape(height, width, 3)
    return img, segments.reshape(height, width)


def mirror_scene():
    spheres = np.zeros(7, dtype=SPHERE_DTYPE)
    rows = [
        ((0.0, -1000.0, 0.0), 1000.0, (0.7, 0.7, 0.75)),  # mirror ground (R=1000: FP64 cancellation)
        ((0.0, 0.6, 0.0), 0.6, (0.9, 0.8, 0.7)),
        ((-1.3, 0.45, 0.4), 0.45, (0.6, 0.9, 0.6)),
        ((1.2, 0.5, -0.3), 0.5, (0.95, 0.95, 0.95)),
        ((0.45, 0.2, 1.0), 0.2, (0.8, 0.5, 0.9)),
        ((-0.5, 1.6, -1.5), 0.7, (0.85, 0.85, 0.6)),
        ((0.45, 0.2, 1.0), 0.2, (0.1, 0.1, 0.1)),  # exact duplicate: the tie must keep the first one
    ]
    for i, (c, r, a) in enumerate(rows):
        spheres[i]["center"], spheres[i]["radius"], spheres[i]["albedo"] = c, r, a
        spheres[i]["material"] = METAL
    return spheres


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    bg = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])
    cases = {
        "rngfree_mirrors": dict(pos=(0.3, 1.1, 3.2), look=(0.0, 0.5, 0.0), vfov=40.0, w=96, h=54, depth=12),
        "rngfree_mirrors_deep": dict(pos=(-2.5, 0.35, 1.5), look=(0.2, 0.6, 0.0), vfov=60.0, w=64, h=48,
                                     depth=50),
    }
    spheres = mirror_scene()
    for name, c in cases.items():
        cam = camera_initialize(c["pos"], c["look"], (0, 1, 0), c["vfov"], 1.0, c["w"], c["h"])
        img, seg = render_rngfree(spheres, cam, c["w"], c["h"], c["depth"], bg)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), spheres=spheres, camera=cam,
                            camera_setup=np.array([*c["pos"], *c["look"], 0, 1, 0, c["vfov"], 1.0, 1.0, 0.0]),
                            background=bg, width=c["w"], height=c["h"], max_depth=c["depth"], rgb=img,
                            segments=seg)
        print(name, img.shape, "segments", int(seg.sum()), "max", int(seg.max()))
    png = os.path.join(args.reference, "example.png")
    if os.path.exists(png):
        from PIL import Image

        rows = np.asarray(Image.open(png).convert("RGB"))[:49]
        np.savez_compressed(os.path.join(HERE, "example_sky_rows.npz"), rows=rows,
                            note="rows 0..48 of fortio/tray example.png (1280x720, -r 64 -d 50 -seed 2)")
        print("example_sky_rows", rows.shape)


if __name__ == "__main__":
    main()
