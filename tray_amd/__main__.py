"""Render the book-cover scene to a PNG through the MI355X path: the flags of the
reference's benchmark binary (benchmark/benchmark.go:37-47; -w and -profile-cpu
have no meaning here).

    python -m tray_amd [-width 1280] [-height 720] [-r 64] [-d 50] [-seed 2] [-save out.png]
    python -m tray_amd -ansi [-s 4] ...   # main.go's terminal view, non-interactive (-exit)
"""
from __future__ import annotations

import argparse
import sys
import time

from . import png, ray, terminal


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m tray_amd")
    ap.add_argument("-width", type=int, default=1280)
    ap.add_argument("-height", type=int, default=720)
    ap.add_argument("-r", type=int, default=64, help="rays per pixel")
    ap.add_argument("-d", type=int, default=50, help="max depth")
    ap.add_argument("-seed", type=int, default=2)
    ap.add_argument("-save", default="out.png", help="output PNG ('' to skip)")
    ap.add_argument("-ansi", action="store_true",
                    help="render at -s x the terminal size and draw it in the terminal (main.go:86-131)")
    ap.add_argument("-s", type=float, default=4, help="supersampling factor of -ansi")
    a = ap.parse_args(argv)
    if a.ansi:
        a.width, a.height = terminal.image_size(*terminal.terminal_size(), a.s)
    t = ray.New(a.width, a.height)
    t.Camera = ray.RichSceneCamera()
    t.NumRaysPerPixel, t.MaxDepth, t.Seed = a.r, a.d, a.seed
    scene = ray.RichScene(a.seed)
    t0 = time.perf_counter()
    img = t.Render(scene)
    dt = time.perf_counter() - t0
    print(f"rendered {a.width}x{a.height} r={a.r} d={a.d} ({len(scene.Objects)} objects) in {dt:.3f} s: "
          f"{a.width * a.height * a.r / dt / 1e6:.1f} Mrays/s end to end", file=sys.stderr)
    if a.save:
        png.save_png(a.save, img)
    if a.ansi:
        cols, rows = terminal.terminal_size()
        print(terminal.ansi_halfblocks(terminal.scale_image(img, cols, rows * 2, a.s)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
