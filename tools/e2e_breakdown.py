#!/usr/bin/env python3
"""Where a synchronous drop-in Render's time goes (bench.py `e2e`): host-timed
pieces of a C2 render with a scene the device has not seen — the scene upload
(BVH build + copies), the first launch on it (sample-buffer allocation,
candidate build), a warm launch, and the whole synchronous tray_render call
with a new scene and with the cached one. Median of --reps runs, milliseconds;
`render_first_at_size` is the process's first render at this size (what
bench.py's `e2e_ms_new_scene` measures).

    python tools/e2e_breakdown.py [--config c2] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--first-split", action="store_true", help="first time the process renders at this size, piece by piece")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    base = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    p = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGBA8)
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    _lib.render(ray.DefaultScene().to_array(), bg, cam._state, _lib.make_params(8, 8, 4, 1, 0.5, seed))  # runtime setup

    def fresh(k):  # a scene no cache has seen (k >= -1): one sphere nudged
        s = base.copy()
        s["center"][1][0] += 1e-9 * (k + 2)
        return s

    def ms(f):
        t0 = time.perf_counter()
        r = f()
        return (time.perf_counter() - t0) * 1e3, r

    if args.first_split:  # the first-at-size costs, piece by piece (a fresh process)
        t_up, sc0 = ms(lambda: _lib.DeviceScene(fresh(-1), bg))

        def go0():
            sc0.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
            torch.cuda.synchronize()
        t_l1, _ = ms(go0)
        t_l2, _ = ms(go0)
        host = np.empty((H, W, 4), dtype=np.uint8)
        t_d2h1, _ = ms(lambda: host.__setitem__(slice(None), out.cpu().numpy()))
        t_d2h2, _ = ms(lambda: host.__setitem__(slice(None), out.cpu().numpy()))
        sc0.release()
        print(json.dumps({"first_upload": round(t_up, 3), "first_launch_at_size": round(t_l1, 3),
                          "second_launch": round(t_l2, 3), "first_d2h_torch": round(t_d2h1, 3),
                          "second_d2h_torch": round(t_d2h2, 3)}))
    first_at_size, _ = ms(lambda: _lib.render(fresh(-1), bg, cam._state, p))  # bench.py's e2e_ms_new_scene
    rows = {"upload": [], "first_launch": [], "warm_launch": [], "render_new_scene": [], "render_cached": []}
    for k in range(args.reps):
        t, sc = ms(lambda: _lib.DeviceScene(fresh(2 * k), bg))
        rows["upload"].append(t)
        for key in ("first_launch", "warm_launch"):
            def go():
                sc.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
                torch.cuda.synchronize()
            rows[key].append(ms(go)[0])
        sc.release()
        s = fresh(2 * k + 1)
        rows["render_new_scene"].append(ms(lambda: _lib.render(s, bg, cam._state, p))[0])
        rows["render_cached"].append(ms(lambda: _lib.render(s, bg, cam._state, p))[0])
    print(json.dumps({"config": args.config, "reps": args.reps, "render_first_at_size": round(first_at_size, 3),
                      **{k: round(float(np.median(v)), 3) for k, v in rows.items()}}))


if __name__ == "__main__":
    main()
