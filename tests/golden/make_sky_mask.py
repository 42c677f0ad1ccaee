"""Generate tests/golden/example_sky_mask.npz (run from the repo root):

    python tests/golden/make_sky_mask.py [--reference /root/reference]

The reference's own output example.png (`tray -save example.png -r 64 -s 8
-d 50 -seed 2` on a 160x45 terminal, README.md:30-31 = 1280x720, r=64, d=50)
holds the Go binary's pixels. Its seed-2 scene comes from fortio.org/rand, which
is not vendored, so which small spheres it holds is unknown. But every
RichScene (ray/objects.go:132-175) lies inside a fixed set: the ground sphere
(0,-1000,0) R=1000, the three R=1 spheres at (0,1,0), (-4,1,0), (4,1,0), and small
spheres of radius 0.2 centred at (a + 0.9u, 0.2, b + 0.9u'), a, b in [-11, 11),
u in [0, 1): all inside the box [-11.2, 11.1] x [0, 0.4] x [-11.2, 11.1].

A pixel is SKY for any RichScene when no camera ray it can cast reaches that
set. RichSceneCamera (ray/camera.go:144-154): aperture 0.1 (lens disc radius
rA = 0.05 on the orthonormal u, v), focus 10 = focal 10 (focusTime 1); anti-
aliasing offsets in a disc of radius 0.5 px (ray/tracer.go:136-139,
RayRadius 0.5). A sample's ray (camera.go:113-142) is
    X(t) = pos + offset + t (focusPoint - pos - offset)
         = A(t) + (1 - t) offset + t dS,
with A(t) = pos + t (Sc - pos) the pixel-centre pinhole ray, |offset| <= rA and
|dS| <= rS = 0.5 |pixel_x| (pixel_x, pixel_y orthogonal, equal length). So at
every t >= 0 the sample lies within w(t) = |1 - t| rA + t rS of A(t), t in the
ray's own units (the root Sphere.Hit compares with 1e-6). The pixel is sky when
for every obstacle  min_t>=0 [dist(A(t), obstacle) - w(t)] > 1e-6: dist to a
ball or a box is convex in the point, A is affine and w linear on [0, 1] and on
[1, inf), so each piece is a convex function of t, minimised by golden-section
search. Camera vectors come from make_golden.py's numpy restatement of
Camera.Initialize (independent of oracle/ and of the kernel).

The fixture holds the mask (np.packbits of [720, 1280]) and example.png's RGB
bytes at those pixels, in row-major order. Every sky pixel's samples escape at
their first segment in ANY RichScene, so the kernel's and the oracle's frames
there are the camera, AmbientLight.Hit (objects.go:68-73) and LinearToSrgb alone,
checked against the real Go binary's bytes by the tests.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import camera_initialize  # noqa: E402

W, H = 1280, 720
RA = 0.05            # lens disc radius: Aperture / 2 (camera.go:84-86), u and v unit vectors
MARGIN = 1e-6        # >> FP64 rounding of the rays (~1e-14 at these magnitudes)
SPHERES = [((0.0, -1000.0, 0.0), 1000.0), ((0.0, 1.0, 0.0), 1.0), ((-4.0, 1.0, 0.0), 1.0), ((4.0, 1.0, 0.0), 1.0)]
BOX = (np.array([-11.2, 0.0, -11.2]), np.array([11.1, 0.4, 11.1]))  # every possible small sphere


def _golden_min(f, lo, hi, iters=160):
    """Vectorised golden-section minimum of convex f over [lo, hi] (arrays), ends included."""
    g = (np.sqrt(5.0) - 1.0) / 2.0
    a, b = np.array(lo, dtype=np.float64), np.array(hi, dtype=np.float64)
    c, d = b - g * (b - a), a + g * (b - a)
    fc, fd = f(c), f(d)
    for _ in range(iters):
        left = fc < fd
        b = np.where(left, d, b)
        a = np.where(left, a, c)
        nc, nd = b - g * (b - a), a + g * (b - a)
        c, d = np.where(left, nc, d), np.where(left, c, nd)
        fnew = f(np.where(left, c, d))
        fc, fd = np.where(left, fnew, fd), np.where(left, fc, fnew)
    return np.minimum(np.minimum(fc, fd), np.minimum(f(np.asarray(lo, np.float64)), f(np.asarray(hi, np.float64))))


def sky_mask():
    cam = camera_initialize((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 10.0, W, H)
    pos, p00, pxv, pyv = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    assert abs(np.dot(pxv, pyv)) < 1e-15 and abs(np.linalg.norm(pxv) - np.linalg.norm(pyv)) < 1e-15
    rs = 0.5 * max(np.linalg.norm(pxv), np.linalg.norm(pyv)) * (1 + 1e-9)
    ra = RA * (1 + 1e-9)
    ys, xs = np.mgrid[0:H, 0:W]
    sc = p00[None, :] + xs.reshape(-1, 1) * pxv[None, :] + ys.reshape(-1, 1) * pyv[None, :]
    d = sc - pos[None, :]  # A(t) = pos + t d

    def w(t):
        return np.abs(1.0 - t) * ra + t * rs

    def point(t):
        return pos[None, :] + t[:, None] * d

    def ball(c, r):
        c = np.array(c)
        return lambda t: np.linalg.norm(point(t) - c[None, :], axis=1) - r - w(t)

    def box(t):
        p = point(t)
        q = np.maximum(np.maximum(BOX[0][None, :] - p, p - BOX[1][None, :]), 0.0)
        return np.linalg.norm(q, axis=1) - w(t)

    n = d.shape[0]
    ok = np.ones(n, dtype=bool)
    for f in [ball(c, r) for c, r in SPHERES] + [box]:
        m1 = _golden_min(f, np.zeros(n), np.ones(n))
        m2 = _golden_min(f, np.ones(n), np.full(n, 1e5))
        ok &= (m1 > MARGIN) & (m2 > MARGIN)
    return ok.reshape(H, W)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    from PIL import Image

    mask = sky_mask()
    img = np.asarray(Image.open(os.path.join(args.reference, "example.png")).convert("RGB"))
    assert img.shape == (H, W, 3)
    assert mask[:49].all(), "rows 0..48 (example_sky_rows.npz) must be sky"
    rgb = img[mask]
    np.savez_compressed(os.path.join(HERE, "example_sky_mask.npz"), mask=np.packbits(mask), shape=np.array([H, W]),
                        rgb=rgb, note="example.png pixels no ray of any RichScene's camera footprint can reach a "
                                      "sphere in (tests/golden/make_sky_mask.py)")
    rows = np.nonzero(mask.any(1))[0]
    print("example_sky_mask", int(mask.sum()), "pixels, rows", int(rows.min()), "..", int(rows.max()))


if __name__ == "__main__":
    main()
