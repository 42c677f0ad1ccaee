"""The primary-ray candidate bound (tray_kernel.hip: pixel_beam / beam_reaches,
DESIGN.md §5) restated in numpy and checked on the CPU: for every sampled pixel,
every sphere that ANY camera ray of the pixel enters at t > 1e-6 — rays from
points of the lens disc through points of the pixel's anti-aliasing disc on the
focus plane, sampled uniformly and on both rims, intersected in FP64 — must be
in the pixel's candidate set, and a tile's set must contain its pixels' sets.
This is the soundness the device path's bit-exactness rests on (the GPU tests in
tests/test_gpu_candidates.py compare whole frames with the traversal)."""
import ctypes

import numpy as np
import pytest

from conftest import RICH_SETUP


def camera(L, setup, w, h):
    d3 = ctypes.c_double * 3
    cs = L.CameraSetup(d3(*setup[0:3]), d3(*setup[3:6]), d3(*setup[6:9]), *[float(v) for v in setup[9:13]])
    st = L.CameraState()
    L.check(L.lib().tray_camera_initialize(ctypes.byref(cs), w, h, ctypes.byref(st)))
    return st


def beam(cam, spp, ray_radius, xa, xb, ya, yb):
    """pixel_beam: axis pos -> far-disc centre, lens radius ra, far radius rb."""
    pos = np.array(cam.position[:]); p00 = np.array(cam.pixel00[:])
    pxv = np.array(cam.pixel_x[:]); pyv = np.array(cam.pixel_y[:])
    du = np.array(cam.defocus_u[:]); dv = np.array(cam.defocus_v[:])
    ft = cam.focus_distance / cam.focal_length
    lens = cam.aperture > 0
    s0 = p00 + pxv * (0.5 * (xa + xb)) + pyv * (0.5 * (ya + yb))
    b0 = pos + (s0 - pos) * ft if lens else s0
    lx, ly = np.linalg.norm(pxv), np.linalg.norm(pyv)
    aa = (abs(ray_radius) * np.hypot(lx, ly) if spp > 1 else 0.0) + 0.5 * (xb - xa) * lx + 0.5 * (yb - ya) * ly
    ra = np.sqrt(du @ du + dv @ dv) if lens else 0.0
    rb = aa * abs(ft) if lens else aa
    return pos, b0 - pos, ra, rb


def reaches(pos, D, ra, rb, centers, radii):
    """beam_reaches for every sphere (vectorised)."""
    dn2 = D @ D
    dn = np.sqrt(dn2)
    L = ra + rb
    assert dn > 2 * L
    scale = 1.0 + np.abs(pos).max()
    rel = centers - pos
    tc = rel @ D / dn2
    tcl = np.maximum(tc, 0.0)
    dperp = np.linalg.norm(rel - tc[:, None] * D[None], axis=1)
    margin = 1e-6 * (scale + np.abs(centers).sum(1) + radii)
    reach = radii + np.abs(1.0 - tcl) * ra + tcl * rb + margin
    return dperp <= reach + L * reach / (dn - L) + margin


def disc_points(rng, n, rim):
    """Points of the unit disc: uniform, and (rim) on the boundary."""
    phi = rng.uniform(0, 2 * np.pi, n)
    r = np.ones(n) if rim else np.sqrt(rng.uniform(0, 1, n))
    return np.stack([r * np.cos(phi), r * np.sin(phi)], 1)


def camera_rays(cam, spp, ray_radius, x, y, rng, n):
    """Rays of pixel (x, y) as get_ray builds them, for lens/AA offsets sampled
    uniformly in their discs and on their rims."""
    pos = np.array(cam.position[:]); p00 = np.array(cam.pixel00[:])
    pxv = np.array(cam.pixel_x[:]); pyv = np.array(cam.pixel_y[:])
    du = np.array(cam.defocus_u[:]); dv = np.array(cam.defocus_v[:])
    ft = cam.focus_distance / cam.focal_length
    aa = np.concatenate([disc_points(rng, n // 2, False), disc_points(rng, n - n // 2, True)]) * ray_radius
    if spp <= 1:
        aa[:] = 0.0
    sample = p00 + pxv * (x + aa[:, :1]) + pyv * (y + aa[:, 1:])
    org = np.broadcast_to(pos, sample.shape).copy()
    dirs = sample - pos
    if cam.aperture > 0:
        ln = np.concatenate([disc_points(rng, n - n // 2, True), disc_points(rng, n // 2, False)])
        rng.shuffle(ln)
        offset = du * ln[:, :1] + dv * ln[:, 1:]
        focus = pos + dirs * ft
        org = pos + offset
        dirs = focus - org
    return org, dirs


def hits(org, dirs, centers, radii):
    """[rays, spheres]: does the ray enter the sphere at t > 1e-6 (Sphere.Hit's roots)."""
    a = (dirs * dirs).sum(1)[:, None]
    oc = centers[None] - org[:, None]
    h = (dirs[:, None] * oc).sum(2)
    c = (oc * oc).sum(2) - radii[None] ** 2
    disc = h * h - a * c
    ok = disc >= 0
    sq = np.sqrt(np.where(ok, disc, 0.0))
    r1, r2 = (h - sq) / a, (h + sq) / a
    return ok & ((r1 > 1e-6) | (r2 > 1e-6))


def tree_spheres(O, seed, half):
    s = O.rich_scene(seed, half)
    big = np.abs(s["radius"]) > 100  # the ground: out of the tree, tested for every ray anyway
    return s["center"][~big], np.abs(s["radius"][~big])


CAMS = {
    "rich_dof": (RICH_SETUP, 64, 0.5),
    "rich_pinhole_r1": (np.r_[RICH_SETUP[:12], 0.0], 1, 0.5),
    "rich_big_aperture_radius2": (np.r_[RICH_SETUP[:12], 1.5], 16, 2.0),
    # Go accepts a negative RayRadius (InDisc(r) scales by the signed r): the disc's extent is |r|
    "rich_negative_radius": (RICH_SETUP, 16, -1.5),
    "top_down": (np.array([0.5, 15, 0.2, 0, 0, 0, 0, 0, 1, 60.0, 1.0, 15.0, 0.3]), 4, 0.5),
}


@pytest.mark.parametrize("name", sorted(CAMS))
def test_every_hit_sphere_is_a_candidate(L, O, name):
    setup, spp, radius = CAMS[name]
    W, H = 160, 90
    cam = camera(L, setup, W, H)
    centers, radii = tree_spheres(O, 2, 11)
    rng = np.random.default_rng(7)
    pixels = [(x, y) for x in rng.integers(0, W, 60) for y in rng.integers(0, H, 1)]
    pixels += [(0, 0), (W - 1, H - 1), (W // 2, H // 2), (0, H - 1)]
    checked = 0
    for x, y in pixels:
        cand = reaches(*beam(cam, spp, radius, x, x, y, y), centers, radii)
        org, dirs = camera_rays(cam, spp, radius, float(x), float(y), rng, 400)
        hit = hits(org, dirs, centers, radii).any(0)
        missing = np.flatnonzero(hit & ~cand)
        assert missing.size == 0, (name, x, y, missing)
        checked += int(hit.sum())
        # the tile beam (8x8 block holding the pixel) contains the pixel beam
        xa, ya = x - x % 8, y - y % 8
        tile = reaches(*beam(cam, spp, radius, xa, min(xa + 7, W - 1), ya, min(ya + 7, H - 1)), centers, radii)
        assert not np.any(cand & ~tile), (name, x, y)
    assert checked > 0  # the sampled pixels do hit spheres


def test_sampling_catches_an_unsound_bound(L, O):
    """Negative control: the same ray sampling finds hits outside a beam whose
    disc radii are halved, so the soundness test above is not vacuous."""
    cam = camera(L, RICH_SETUP, 160, 90)
    centers, radii = tree_spheres(O, 2, 11)
    rng = np.random.default_rng(7)
    missed = 0
    for x in range(0, 160, 9):
        for y in range(0, 90, 9):
            pos, D, ra, rb = beam(cam, 64, 0.5, x, x, y, y)
            cand = reaches(pos, D, 0.5 * ra, 0.5 * rb, centers, radii)
            org, dirs = camera_rays(cam, 64, 0.5, float(x), float(y), rng, 400)
            missed += int((hits(org, dirs, centers, radii).any(0) & ~cand).sum())
    assert missed > 0


def test_candidate_counts_are_small_for_the_book_cover(L, O):
    """The bound stays selective (1.08 candidates per pixel on C2)."""
    W, H = 320, 180
    cam = camera(L, RICH_SETUP, W, H)
    centers, radii = tree_spheres(O, 2, 11)
    counts = [int(reaches(*beam(cam, 64, 0.5, x, x, y, y), centers, radii).sum())
              for x in range(0, W, 7) for y in range(0, H, 7)]
    assert np.mean(counts) < 2.0 and np.mean(np.array(counts) <= 7) > 0.99, (np.mean(counts), max(counts))
