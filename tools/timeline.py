#!/usr/bin/env python3
"""Diagnostic: where a launch's ramp and drain go. Needs a -DTRAY_PROFILE_TIMELINE
build (tools/build_variants.sh tl "-DTRAY_PROFILE_TIMELINE"); renders one frame
through the stats instance and reports, from every wave's record
(tray_kernel.hip, kTlStride): busy lanes of the whole grid over time (10-us
buckets), the time the work queue first and last ran dry in a wave, wave end
times, chunks per wave, and the lane-time lost before the first dry wave, between
first dry and the last wave's end.

    python tools/timeline.py path/to/libtray_amd.so [--config c2] [--shard N,K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BUCKETS, MT_TICKS, HDR = 1024, 25000, 6  # kTlBuckets, kTlTicks (shader clock), kTlHdr
TICKS = 1000  # output buckets: 10 us of the 100 MHz constant clock
STRIDE = BUCKETS + HDR


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--shard", default=None, help="N,K: rank K's row tiles of an N-way split (1-row tiles)")
    ap.add_argument("--waves", type=int, default=256 * 16)
    ap.add_argument("--reps", type=int, default=3, help="renders; the last one is reported")
    ap.add_argument("--curve", action="store_true", help="print the per-bucket utilisation curve too")
    ap.add_argument("--knob", action="append", default=[], help="NAME=VALUE include/tray_debug.h knob (repeatable)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from bench import CONFIGS
    from tray_amd import _lib, ray

    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    if args.knob:
        _lib.set_debug_knobs(os.path.abspath(args.lib), **{k: int(v) for k, v in (kv.split("=", 1) for kv in args.knob)})
    scene = _lib.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0, os.path.abspath(args.lib))
    params = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32)
    if args.shard:
        from tray_amd import shard
        n, k = (int(v) for v in args.shard.split(","))
        params = shard.shard_params(params, 1, n, k)
    out = torch.empty((_lib.params_rows(params), W, 3), dtype=torch.float32, device="cuda")
    stats = torch.zeros(32 + STRIDE * args.waves, dtype=torch.int64, device="cuda")
    for _ in range(args.reps):
        stats.zero_()
        scene.render_stats_async(cam._state, params, out.data_ptr(), stats.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    rec = stats[32:].view(args.waves, STRIDE).cpu().numpy().astype(np.float64)
    seen = rec[:, 1] > 0
    rec = rec[seen]
    last = rec[:, HDR + BUCKETS - 3:HDR + BUCKETS].astype(np.int64)  # last path: segments, pixel, sample
    lone_t, lone_seg = rec[:, HDR + BUCKETS - 5].copy(), rec[:, HDR + BUCKETS - 4].astype(np.int64)
    lone_ph = rec[:, HDR + BUCKETS - 9:HDR + BUCKETS - 5].copy()  # shader ticks: refill, node, leaf, shade
    rec[:, HDR + BUCKETS - 9:] = 0
    start, end, dry, chunks = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3]
    ratio = (end - start) / np.maximum(rec[:, 5] - rec[:, 4], 1)  # constant-clock ticks per shader tick
    g0 = start.min()
    span = end.max() - g0
    lanes = 64 * len(rec)
    nb = int(span // TICKS) + 2
    curve = np.zeros(nb)
    for w in range(len(rec)):
        b = rec[w, HDR:HDR + BUCKETS - 9] * ratio[w]  # busy lane x constant-clock ticks
        mid = start[w] - g0 + (np.arange(b.size) + 0.5) * MT_TICKS * ratio[w]
        idx = np.minimum((mid // TICKS).astype(np.int64), nb - 1)
        np.add.at(curve, idx, b)
    util = curve / (TICKS * lanes)  # busy-lane fraction of the whole grid per bucket
    dry_abs = start + dry - g0
    has_dry = dry > 0
    first_dry, last_dry = dry_abs[has_dry].min(), dry_abs[has_dry].max()
    end_rel = end - g0
    busy_total = curve.sum()
    t_first = int(first_dry // TICKS)
    q = [0, 1, 10, 50, 90, 99, 100]
    d = {
        "config": args.config, "shard": args.shard, "knobs": args.knob, "shader_ghz": round(float(np.median(100e6 / ratio)) / 1e9, 3), "waves": int(len(rec)), "span_us": round(span / 100, 1),
        "lane_util_overall": round(busy_total / (span * lanes), 4),
        "first_dry_us": round(first_dry / 100, 1), "last_dry_us": round(last_dry / 100, 1),
        "end_us_pct": {str(k): round(float(np.percentile(end_rel, k)) / 100, 1) for k in q},
        "start_us_pct": {str(k): round(float(np.percentile(start - g0, k)) / 100, 1) for k in q},
        "chunks_per_wave_pct": {str(k): float(np.percentile(chunks, k)) for k in q},
        # lane-time lost: before the first dry wave (ramp + refill waits) and after (the drain)
        "lost_before_dry_us": round((first_dry * lanes - curve[:t_first].sum()) / lanes / 100, 1),
        "lost_after_dry_us": round(((span - first_dry) * lanes - curve[t_first:].sum()) / lanes / 100, 1),
        "util_first_100us": round(float(util[:10].mean()), 4),
        "util_steady": round(float(util[10:max(11, t_first)].mean()), 4),
    }
    # what the last waves trace: the wave's final lone path (segments so far, pixel, sample)
    order = np.argsort(end_rel)[::-1][:32]
    d["last_waves"] = [{"end_us": round(float(end_rel[w]) / 100, 1), "drain_us": round(float(end[w] - start[w] - dry[w]) / 100, 1),
                        "segments": int(last[w, 0]), "x": int(last[w, 1] % W), "y": int(last[w, 1] // W),
                        "sample": int(last[w, 2])} for w in order]
    seg_all = last[:, 0][last[:, 0] > 0]
    d["last_path_segments_pct"] = {str(k): float(np.percentile(seg_all, k)) for k in q} if seg_all.size else None
    drain = (end - start - dry)[has_dry] / 100
    d["wave_drain_us_pct"] = {str(k): round(float(np.percentile(drain, k)), 1) for k in q}
    # the lone path's latency per segment: from the moment it was the wave's only path
    # to the wave's end, over the segments it traced in that time
    lone = (lone_t > 0) & (last[:, 0] > lone_seg)
    if lone.any():
        dt = (rec[:, 5] - rec[:, 4] - lone_t)[lone] * ratio[lone] / 100  # us
        dseg = (last[:, 0] - lone_seg)[lone]
        lone_start = (start + lone_t * ratio - g0)[lone]
        alive = np.array([(end_rel > t).sum() for t in lone_start])  # waves alive then (of the grid)
        per = dt / dseg
        d["lone_path_us_per_segment_pct"] = {str(k): round(float(np.percentile(per, k)), 2) for k in q}
        d["lone_segments_pct"] = {str(k): float(np.percentile(dseg, k)) for k in q}
        d["lone_waves"] = int(lone.sum())
        late = lone_start >= np.percentile(lone_start, 90)  # the last tenth to go lone
        d["lone_late_us_per_segment_median"] = round(float(np.median(per[late])), 2)
        d["lone_late_waves_alive_median"] = int(np.median(alive[late]))
        ph = (lone_ph[lone] * ratio[lone, None] / 100) / dseg[:, None]  # us per segment per phase
        d["lone_phase_us_per_segment_median"] = dict(zip(("refill", "node", "leaf", "shade"),
                                                         (round(float(v), 3) for v in np.median(ph, axis=0))))
    if args.curve:
        d["util_curve"] = [round(float(u), 3) for u in util]
    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
