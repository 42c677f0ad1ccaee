#!/usr/bin/env python3
"""Interleaved A/B timing of libtray_amd.so builds in ONE process (same device,
same data): per round every variant renders the frame once; reports the median
and min kernel time per variant (HIP events on the launch stream).

    python tools/ab_bench.py [--config c2] [--rounds 5] NAME=path/libtray_amd.so[@KEY=VAL,...] ...

`@KEY=VAL,...` sets include/tray_debug.h knobs for that variant's scene upload and
launches (e.g. bvh_leaf=4, bvh_lds_mode=2; a legacy TRAY_BVH_LEAF-style name maps to
its knob). `@ordered_sum=1` renders the variant with TRAY_FLAG_ORDERED_SUM. Builds
older than the knob API read the same settings from the environment.
"""
import argparse
import contextlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@contextlib.contextmanager
def _env(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _knobs(path, kv):
    """The variant's settings: tray_debug_set knobs, or the environment for builds that predate them."""
    from tray_amd import _lib

    names = {k.lower().removeprefix("tray_"): v for k, v in kv.items()}
    if hasattr(_lib.lib(path), "tray_debug_set"):
        return _lib.debug_knobs(path, **{k: int(v) for k, v in names.items()})
    return _env({"TRAY_" + k.upper(): str(v) for k, v in names.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--linear", action="store_true", help="force the linear-scan kernel")
    ap.add_argument("--half", type=int, default=None, help="override the scene's grid half-extent (density)")
    ap.add_argument("--spp", type=int, default=None, help="override rays per pixel")
    ap.add_argument("--passes", type=int, default=1,
                    help="frames per launch (tray_render_passes_async; bench.py's launch shape is 16)")
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    half = args.half or half
    spp = args.spp or spp
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    params = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32,
                              flags=_lib.FLAG_LINEAR_SCAN if args.linear else 0)
    stream = torch.cuda.current_stream()
    runs = {}
    for v in args.variants:
        name, path = v.split("=", 1)
        path, _, envs = path.partition("@")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        ordered = int(env.pop("ordered_sum", 0))
        path = os.path.abspath(path)
        with _knobs(path, env):
            scene = _lib.DeviceScene(spheres, bg, 0, path)
        p = _lib.Params.from_buffer_copy(params)
        if ordered:
            p.flags |= _lib.FLAG_ORDERED_SUM
        runs[name] = dict(scene=scene, env=env, path=path, params=p,
                          out=torch.empty((args.passes, H, W, 3), dtype=torch.float32, device="cuda"), ms=[])
    ref = None
    for r in range(args.rounds + 1):
        for name, st in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with _knobs(st["path"], st["env"]):
                a.record(stream)
                if args.passes == 1:
                    st["scene"].render_async(cam._state, st["params"], st["out"].data_ptr(), None, stream.cuda_stream)
                else:
                    st["scene"].render_passes_async(cam._state, st["params"], args.passes, st["out"].data_ptr(),
                                                    stream.cuda_stream)
                b.record(stream)
            torch.cuda.synchronize()
            if r > 0:
                st["ms"].append(a.elapsed_time(b))
            if ref is None:
                ref = st["out"].clone()
            elif r == 0:
                st["equal_to_first"] = bool(torch.equal(ref, st["out"]))
    samples = W * H * spp * args.passes
    for name, st in runs.items():
        med = float(np.median(st["ms"]))
        print(json.dumps({"variant": name, "config": args.config, "passes": args.passes, "median_ms": round(med, 3),
                          "min_ms": round(min(st["ms"]), 3), "ms_per_frame": round(med / args.passes, 4),
                          "mrays": round(samples / med / 1e3, 1), "equal_to_first": st.get("equal_to_first", True)}),
              flush=True)


if __name__ == "__main__":
    main()
