"""Oracle: sampler statistics (the reference's only pins on its sampler,
ray/vec3_test.go:539-741), RNG-free golden scenes (independent numpy
restatement, tests/golden/make_golden.py) and the sky of the reference's own
example.png. CPU only."""
import os

import numpy as np
import pytest

from conftest import (DEFAULT_BG, RICH_SETUP, SKY_EDGE_AA, SKY_EDGE_PINHOLE, example_sky_mask, load_golden,
                      srgb_boundary_distance)


def test_unit_vector_distribution(O):  # ray/vec3_test.go:539-649 (100k samples)
    n = 100_000
    v = np.array([O.unit_vector(42, i, i % 7, i % 50) for i in range(n)])
    assert np.all(np.abs(v.mean(0)) <= 0.015)
    assert np.all(np.abs(v.var(0) - 1.0 / 3.0) <= 0.01)
    octant = (v[:, 0] > 0) * 4 + (v[:, 1] > 0) * 2 + (v[:, 2] > 0)
    counts = np.bincount(octant, minlength=8)
    assert np.all(np.abs(counts - n / 8) <= 0.15 * n / 8)
    z_hist = np.histogram(v[:, 2], bins=20, range=(-1, 1))[0]  # Archimedes: z is uniform (vec3_test.go:651-705)
    assert np.all(np.abs(z_hist - n / 20) <= 0.1 * n / 20)


@pytest.mark.parametrize("which,radius", [(0, 0.5), (1, 1.0), (0, 1.0)])
def test_in_disc(O, which, radius):  # InDisc: inside the disc, uniform over its area
    d = np.array([O.in_disc(3, i, 0, which, radius) for i in range(40_000)])
    r2 = (d**2).sum(1)
    assert np.all(r2 < radius * radius)
    assert abs(r2.mean() / (radius * radius) - 0.5) < 0.01  # E[r^2] = R^2/2 for a uniform disc
    assert np.all(np.abs(d.mean(0)) < 0.01 * radius)


def test_sincos_2pi(O):
    """The contract's sin/cos(2 pi u): exact FP64 quadrant reduction, FP32 Horner
    polynomials with fmaf, one FP64 Newton step onto the unit circle
    (include/tray.h): the angle within ~1e-7 (far finer than a sampled direction
    needs), the length within ~1e-14."""
    us = np.concatenate([np.linspace(0, 1, 4001, endpoint=False), np.random.default_rng(1).random(4000),
                         [0.125, 0.25 - 2**-40, 0.5, 0.75, 1 - 2**-32]])
    got = np.array([O.sincos_2pi(u) for u in us])
    assert np.max(np.abs(got[:, 0] - np.sin(2 * np.pi * us))) < 2.5e-7
    assert np.max(np.abs(got[:, 1] - np.cos(2 * np.pi * us))) < 2.5e-7
    assert np.max(np.abs((got**2).sum(1) - 1.0)) < 5e-14  # one FP64 Newton step: (3/4) * (2e-7)^2
    assert tuple(O.sincos_2pi(0.0)) == (0.0, 1.0) and tuple(O.sincos_2pi(0.25)) == (1.0, -0.0)


def test_camera_block_shared(O):
    """AA (words 0,1) and lens (words 2,3) discs come from one draw block per sample
    (purpose 1, include/tray.h)."""
    a = O.in_disc(5, 77, 3, 0, 1.0)
    b = O.in_disc(5, 77, 3, 1, 1.0)
    assert tuple(a) != tuple(b)
    x = O.draw_block(O.draw_key(5), 77, 3, 0, 1)
    u = [v * 2.0**-32 for v in x]
    s, c = O.sincos_2pi(u[1])
    assert tuple(a) == ((u[0] ** 0.5 * c) * 1.0, (u[0] ** 0.5 * s) * 1.0)


@pytest.mark.parametrize("name", ["rngfree_mirrors", "rngfree_mirrors_deep"])
def test_rngfree_golden(O, name):
    g = load_golden(name)
    io, cam = O.camera_initialize(g["camera_setup"], int(g["width"]), int(g["height"]))
    assert np.array_equal(cam, g["camera"])
    img, seg = O.render(g["spheres"], g["background"], g["camera"], int(g["width"]), int(g["height"]), 1,
                        int(g["max_depth"]), 0.5, 12345)
    assert np.array_equal(seg, g["segments"])
    assert np.array_equal(img, g["rgb"])  # bit-exact: same op order, no RNG involved


def test_example_png_sky_rows(O):
    """Rows 0..48 of the reference's own output (1280x720, r=64, d=50, seed 2).
    Pure sky, so camera + AmbientLight + LinearToSrgb are checked against the
    real Go binary; the +-1 LSB is AA noise of a different random stream."""
    rows = load_golden("example_sky_rows")["rows"]
    _, cam = O.camera_initialize(RICH_SETUP, 1280, 720)
    sc = O.rich_scene(2)
    img, seg = O.render(sc, DEFAULT_BG, cam, 1280, 720, 64, 50, 0.5, 2, 0, 49, workers=os.cpu_count() or 4)
    assert np.all(seg == 64)  # every sample escaped to the sky at its first segment
    diff = np.abs(O.to_srgba(img)[..., :3].astype(int) - rows.astype(int))
    assert diff.max() <= 1
    assert (diff.max(-1) == 0).mean() >= 0.98
    # a 1-LSB miss only next to an encoder rounding boundary (AA noise of another stream)
    assert not np.any((diff > 0) & (srgb_boundary_distance(img) >= SKY_EDGE_AA))
    # pixel-centre rays through a pinhole: the analytic recomputation of SURVEY.md §8(c).
    # No random stream is involved, so the bytes must be EXACT except where the
    # encoded value sits within SKY_EDGE_PINHOLE of a rounding boundary.
    setup = RICH_SETUP.copy()
    setup[12] = 0.0
    _, cam0 = O.camera_initialize(setup, 1280, 720)
    img0, _ = O.render(None, DEFAULT_BG, cam0, 1280, 720, 1, 50, 0.5, 2, 0, 49)
    d0 = np.abs(O.to_srgba(img0)[..., :3].astype(int) - rows.astype(int))
    assert d0.max() <= 1 and (d0.max(-1) == 0).mean() >= 0.985
    near = srgb_boundary_distance(img0) < SKY_EDGE_PINHOLE
    assert near.mean() < 0.03  # the exemption covers < 3 % of channels
    assert np.array_equal(d0[~near], np.zeros_like(d0[~near]))


def test_example_png_sky_mask(O):
    """145,582 pixels of the reference's own output (rows 0..156: the sky above the
    horizon, and below it where rays descend too little to meet the R=1000 ground,
    between and above the spheres), pinned with example_sky_rows' rules: every
    sample escapes at its first segment, the r=64 frame differs by at most 1 LSB
    and only next to an encoder rounding boundary, the pixel-centre pinhole frame
    is exact except within SKY_EDGE_PINHOLE of a boundary."""
    mask, rgb, ymax = example_sky_mask()
    assert mask.sum() >= 120_000 and mask[:49].all()
    _, cam = O.camera_initialize(RICH_SETUP, 1280, 720)
    img, seg = O.render(O.rich_scene(2), DEFAULT_BG, cam, 1280, 720, 64, 50, 0.5, 2, 0, ymax,
                        workers=os.cpu_count() or 4)
    m = mask[:ymax]
    assert np.all(seg[m] == 64)
    diff = np.abs(O.to_srgba(img)[..., :3][m].astype(int) - rgb.astype(int))
    assert diff.max() <= 1 and (diff.max(-1) == 0).mean() >= 0.98
    assert not np.any((diff > 0) & (srgb_boundary_distance(img)[m] >= SKY_EDGE_AA))
    setup = RICH_SETUP.copy()
    setup[12] = 0.0
    _, cam0 = O.camera_initialize(setup, 1280, 720)
    img0, _ = O.render(None, DEFAULT_BG, cam0, 1280, 720, 1, 50, 0.5, 2, 0, ymax)
    d0 = np.abs(O.to_srgba(img0)[..., :3][m].astype(int) - rgb.astype(int))
    near = srgb_boundary_distance(img0)[m] < SKY_EDGE_PINHOLE
    assert d0.max() <= 1 and near.mean() < 0.05
    assert np.array_equal(d0[~near], np.zeros_like(d0[~near]))


def test_oracle_workers_invariant(O):
    """The counter RNG removes the reference's -w dependence (ray/tracer.go:93,121)."""
    _, cam = O.camera_initialize(RICH_SETUP, 40, 24)
    sc = O.rich_scene(2)
    a, sa = O.render(sc, DEFAULT_BG, cam, 40, 24, 3, 12, 0.5, 9, workers=1)
    b, sb = O.render(sc, DEFAULT_BG, cam, 40, 24, 3, 12, 0.5, 9, workers=5)
    assert np.array_equal(a, b) and np.array_equal(sa, sb)


def test_rich_scene_structure(O):  # ray/objects.go:132-175; benchmark/benchmark.go:42 (486 objects @ seed 7)
    for seed in (2, 7, 42):
        sc = O.rich_scene(seed)
        assert 4 < len(sc) <= 488
        assert sc[0]["radius"] == 1000 and tuple(sc[0]["center"]) == (0, -1000, 0)
        small = sc[1:-3]
        assert np.all(small["radius"] == 0.2) and np.all(small["center"][:, 1] == 0.2)
        assert np.all(np.linalg.norm(small["center"] - np.array([4, 0.2, 0]), axis=1) > 0.9)
        mats = np.bincount(small["material"], minlength=4)[1:]
        assert mats[0] > mats[1] > mats[2] > 0  # ~80 / 15 / 5 %
        assert tuple(sc[-3]["center"]) == (0, 1, 0) and sc[-3]["material"] == 3
    dense = O.rich_scene(7, 22)
    assert 1800 < len(dense) <= 44 * 44 + 4
