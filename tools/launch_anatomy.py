#!/usr/bin/env python3
"""Where a one-frame launch's time goes (the drop-in tray_render shape): R
one-frame launches of a config, one at a time, each between two HIP events on
the launch stream; under `rocprofv3 --kernel-trace` the trace then splits every
launch into its dispatches (megakernel, resolve, tile order) and the gaps
between them.

    rocprofv3 --kernel-trace -d DIR -o kt -- python3 tools/launch_anatomy.py --config c1 --reps 30 > run.json
    python3 tools/launch_anatomy.py --summarize DIR/kt_results.db (or a kt_kernel_trace.csv) [--run run.json]

The run prints one JSON line (event-timed ms per launch, median / mean); the
summary prints, per dispatch kind, the median duration and the median gap from
the previous dispatch of the same launch, over the launches after the first two.
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = ("render_kernel", "resolve_kernel", "tile_order_kernel", "cand_")


def kind(name):
    for k in KINDS:
        if k in name:
            return k
    return None


def summarize(path, run_path=None):
    import numpy as np

    rows = []
    if path.endswith(".db"):  # rocprofv3's default rocpd (SQLite) output
        import sqlite3

        with sqlite3.connect(path) as db:
            for name, start, end in db.execute("select name, start, end from kernels"):
                k = kind(name)
                if k:
                    rows.append((int(start), int(end), k))
    else:
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                k = kind(r["Kernel_Name"])
                if k:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    launches, cur = [], []
    for s, e, k in rows:  # a launch starts at each megakernel dispatch
        if k == "render_kernel" and cur:
            launches.append(cur)
            cur = []
        cur.append((s, e, k))
    if cur:
        launches.append(cur)
    launches = launches[2:]  # the counting launch and one more: warm-up
    dur, gap = {}, {}
    span = []
    for L in launches:
        prev_end = None
        for s, e, k in L:
            dur.setdefault(k, []).append((e - s) / 1e3)
            if prev_end is not None:
                gap.setdefault(k, []).append((s - prev_end) / 1e3)
            prev_end = e
        span.append((L[-1][1] - L[0][0]) / 1e3)
    rec = {"trace": os.path.basename(path), "launches": len(launches),
           "span_us": round(float(np.median(span)), 2) if span else None,
           "dispatch_us": {k: round(float(np.median(v)), 2) for k, v in dur.items()},
           "gap_before_us": {k: round(float(np.median(v)), 2) for k, v in gap.items()}}
    if run_path:
        with open(run_path) as f:
            run = json.loads([ln for ln in f if ln.startswith("{")][-1])
        rec["event_ms_median"] = run["event_ms_median"]
        rec["outside_dispatches_us"] = round(run["event_ms_median"] * 1e3 - rec["span_us"], 2) if span else None
    print(json.dumps(rec))


def run(args):
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    _, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    p = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGBA8 if args.rgba else _lib.OUT_RGB_F32)
    dev = _lib.DeviceScene(spheres, bg, 0)
    out = torch.empty((H, W, 4 if args.rgba else 3), dtype=torch.uint8 if args.rgba else torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    ms = []
    for i in range(args.reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        dev.render_async(cam._state, p, out.data_ptr(), None, stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        if i >= 2:
            ms.append(a.elapsed_time(b))
    dev.release()
    print(json.dumps({"config": args.config, "reps": args.reps, "rgba8": args.rgba,
                      "event_ms_median": round(float(np.median(ms)), 4), "event_ms_mean": round(float(np.mean(ms)), 4),
                      "event_ms_min": round(float(min(ms)), 4)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rgba", action="store_true", help="RGBA8 output (the drop-in call's format)")
    ap.add_argument("--summarize", default=None, help="a rocprofv3 kernel trace of a run (rocpd .db or kernel_trace.csv)")
    ap.add_argument("--run", default=None, help="the run's JSON output (for the event-timed span)")
    args = ap.parse_args()
    if args.summarize:
        summarize(args.summarize, args.run)
    else:
        run(args)


if __name__ == "__main__":
    main()
