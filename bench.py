#!/usr/bin/env python3
"""Benchmark: Mrays/s of the MI355X path-tracing megakernel on BASELINE.json's
headline workload (config 2: book-cover scene, seed 2, 1280x720, r=64, d=50).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches its
own N ranks (one child process per GPU, started before this process touches
torch or the GPU; RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT
set per child), waits for all of them and exits non-zero if any fails; rank 0
prints the JSON line. Under a launcher (WORLD_SIZE set) the ranks are the
launcher's. Every N > 1 line reports the world RCCL formed and the device
(PCI bus id, UUID) each rank rendered on; under RCCL the devices must be
distinct.

A step = one full frame rendered through the C-ABI with the scene already
resident in HBM; for N > 1 the frame is split into interleaved row tiles
(default 1 row: rank k renders rows y = k mod N; one shard per rank, no
collective inside the render) and the frames are gathered to rank 0 by RCCL
over xGMI ("scaling": "strong": the frame is fixed as N grows).
value = W*H*r*steps / max-over-ranks wall time.
Frames are progressive passes (tray_params.pass = frame index: every frame
draws fresh samples). --passes F (default 16, THE SAME AT EVERY N, so the N = 1
line and every point of a 1 -> 8 curve share one launch shape) renders F
frames per launch (tray_render_passes_async: lanes flow from one frame's
samples into the next, so a launch has one tail of long paths, not F); at
N > 1 one gather per launch moves its F frames to rank 0, on a stream of its
own. Launches rotate over --frames-in-flight slots (own output and stream, and
the one device scene's launch context of that stream - work queue, chunk
records -; default 2), so a launch's
workgroups start on the CUs the previous launch's last long paths leave idle.
Every step still renders its whole frame inside the timed region.

Also reported (rank 0):
  roofline     the megakernel against the FP64 VALU roof (it is compute and
               latency bound; HBM traffic, by PMC, is far below its roof and is
               reported against the algorithmic W*H*12 B per frame): achieved = algorithmic VALU work per launch / mean
               launch time, in FP64-op equivalents. No FMA is allowed in the FP64
               arithmetic, so the peak is 78.6 TFLOP/s / 2 = 39.3 T ops/s (a
               wave64 FP64 op issues in 4 cycles on a SIMD-32); an FP32 op issues
               in 2 cycles (MI355X_MICROARCH.md) and counts 1/2. Work = 17 FP64
               ops per ray-sphere test + 60 per segment + 40 per
               sample + 11 FP32 ops per ray-box test of the exact-culling BVH (6
               FMA + 5 min/max/compare). Segments, sphere and box tests are
               counted by the kernel itself in an untimed instrumented launch
               (segments are bit-exact with the oracle). The timed launch is the
               megakernel plus its per-pixel resolve passes (all on the stream
               between the two HIP events). Beside the spec peak: the measured
               FP64 mul+add peak, and the counter-derived VALU issue and lane
               utilisation of this build (profiles/pmc_mix_<config>.json), which a
               worse BVH cannot inflate. "brute_force_equiv" rates the same frame
               at the reference's all-spheres-per-segment work (not a fraction).
  single_launch_ms  one frame, one launch, nothing overlapped.
  e2e          the drop-in call: one synchronous tray_render of the frame into
               host memory as RGBA8 (what benchmark.go:88 times around
               rt.Render), cold (BVH build, upload, allocation) and warm.
  cpu_baseline the oracle (C port of the reference's CPU loop with the
               reference's chunk-queue scheduler, ray/tracer.go:86-116) timed on
               a bounded row sample of the same frame on the host cores (frames
               smaller than --cpu-min-seconds of work, C1, are rendered as
               several progressive passes until that much time has passed).
  parity       the per-pixel L-inf of the metric: pass 0 of the frame rendered
               on the device (untimed) against the oracle's render of the same
               pass that cpu_baseline produced, over every pixel of the rows the
               oracle rendered (the whole frame at C1/C2; every k-th row at
               C3/C5): the FP64 output (tray_render_async, TRAY_OUT_RGB_F64) and
               frame 0 of a passes launch in the timed shape (TRAY_OUT_RGB_F32),
               plus the per-pixel Scene.Hit counts (bit-exact). Gate 1e-4.
               At N > 1 the same check runs on the frame rank 0 ASSEMBLES: every
               rank renders pass 0 of its rows again (untimed), the timed run's
               gather brings the row tiles to rank 0, and the oracle renders the
               same rows there (gather_pass0, gathered_parity).
  ranks        (N > 1) each rank's render time per frame (HIP events, one
               launch of F frames of its rows) and one gather of F frames, so
               a measured curve separates imbalance from the gather.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec, seed-2 book-cover scene 1280x720 r=64 d=50; per-pixel L∞ vs ref"

CONFIGS = {
    # name: (label, seed, half_extent, W, H, spp, depth)
    "c1": ("C1 book-cover seed 2 400x225 r=16 d=12", 2, 11, 400, 225, 16, 12),
    "c2": ("C2 book-cover seed 2 1280x720 r=64 d=50", 2, 11, 1280, 720, 64, 50),
    "c3": ("C3 book-cover seed 2 3840x2160 r=256 d=50", 2, 11, 3840, 2160, 256, 50),
    "c4": ("C4 book-cover seed 2 3840x2160 r=1024 d=50 (8-GPU row tiles)", 2, 11, 3840, 2160, 1024, 50),
    "c5": ("C5 dense RichScene(half-extent 22) seed 7 1920x1080 r=256 d=50", 7, 22, 1920, 1080, 256, 50),
}

FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector, AMD spec, FMA counted as 2 flops
FP64_PEAK_OPS = FP64_PEAK_TFLOPS / 2  # T non-FMA FP64 ops/s (parity forbids contraction): 39.3
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


FP64_PEAK_MEASURED = 34.03    # T v_mul_f64 + v_add_f64 per s, tools/fp64_peak.hip (profiles/r1_fp64_peak.json)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _profile_json(name, config, frames, code_hash, profiles_dir=None):
    """profiles/<name>_<config>.json when it was measured on this launch shape (N = 1,
    F frames/launch) AND on the device code the process loaded (the record's
    code_object_sha256 equals the library's; tools/pmc_summary.py, pmc_mix.py).
    Returns (record or None, source path or None, reason when None)."""
    path = os.path.join(profiles_dir or os.path.join(ROOT, "profiles"), f"{name}_{config}.json")
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None, None, f"no {os.path.basename(path)}"
    if rec.get("frames_per_launch", 1) != frames:
        return None, None, f"{os.path.basename(path)} was measured at {rec.get('frames_per_launch', 1)} frames per launch"
    if not code_hash or rec.get("code_object_sha256") != code_hash:
        return None, None, (f"{os.path.basename(path)} was measured on device code "
                            f"{str(rec.get('code_object_sha256'))[:12]}, the loaded library is {str(code_hash)[:12]}")
    return rec, os.path.relpath(path, ROOT), None


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base: dict | None = None) -> list:
    """The environment of each of the n ranks bench.py launches itself (the
    variables torch.distributed.run would set for --nnodes 1 --nproc-per-node n)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                  "TRAY_BENCH_LAUNCHER": "bench.py"})
        envs.append(e)
    return envs


def launch_ranks(n: int, argv: list, timeout: float | None = None, script: str | None = None) -> int:
    """Run this script once per rank as child processes (no exec: this process
    never initialises the GPU) and return 0 only if every rank exits 0. Rank 0's
    JSON line reaches stdout directly (the children inherit it). When one rank
    fails the others are stopped (their exact PIDs), so a rank stuck in a
    collective does not outlive the job."""
    import subprocess

    cmd = [sys.executable, script or os.path.abspath(__file__)] + list(argv)
    procs = [subprocess.Popen(cmd, env=e) for e in rank_envs(n, free_port())]
    rc = 0
    deadline = None if timeout is None else time.monotonic() + timeout
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
        if deadline is not None and time.monotonic() > deadline and live:
            stuck = sorted(procs.index(q) for q in live)
            print(f"bench.py: rank(s) {stuck} still running after {timeout} s (--rank-timeout): stopping them",
                  file=sys.stderr)
            for q in live:
                q.kill()
            rc = rc or 124
            deadline = None
        time.sleep(0.05)
    return rc


_PHASE = ["start", time.monotonic()]


def set_phase(name: str) -> None:
    """What this rank is doing, for the watchdog's message; re-arms the watchdog's
    per-phase deadline (start_watchdog)."""
    _PHASE[:] = [name, time.monotonic()]


def start_watchdog(rank: int, seconds: float) -> None:
    """A daemon thread that ends this rank (exit status 124) once it has spent
    `seconds` in ONE phase (set_phase re-arms the deadline), naming the rank and
    the phase: a collective that never completes (a peer that died, an RCCL hang)
    then fails the job instead of holding it, while a long but progressing run
    (many --steps, a big config) is never cut off for its total length."""
    import threading

    def watch():
        while True:
            name, t0 = _PHASE
            left = t0 + seconds - time.monotonic()
            if left <= 0:
                break
            time.sleep(min(left, 1.0))
        print(f"bench.py: rank {rank} still running after {seconds} s (--rank-timeout) in phase "
              f"'{_PHASE[0]}': exiting", file=sys.stderr, flush=True)
        os._exit(124)

    threading.Thread(target=watch, daemon=True, name="rank-watchdog").start()


def device_record(torch, local_rank: int) -> dict:
    """Which device this rank renders on (bench line, `dist.devices`)."""
    pr = torch.cuda.get_device_properties(local_rank)
    bus = getattr(pr, "pci_bus_id", None)
    dom = getattr(pr, "pci_domain_id", 0)
    dev = getattr(pr, "pci_device_id", 0)
    return {"device": local_rank, "name": pr.name,
            "pci": f"{dom:04x}:{bus:02x}:{dev:02x}.0" if bus is not None else None,
            "uuid": str(getattr(pr, "uuid", "")) or None}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--tile-rows", type=int, default=1, help="rows per interleaved tile (N > 1): 1 balances best")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the synchronous tray_render (drop-in) timings")
    ap.add_argument("--no-single", action="store_true", help="skip the one-frame launch timing (profiling runs)")
    ap.add_argument("--cpu-row-step", type=int, default=0,
                    help="oracle renders every k-th row of the frame (0: about a C2 frame's work, ~13 s)")
    ap.add_argument("--linear", action="store_true", help="force the reference-order linear scan (no BVH)")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="launches overlap this deep (own scene copy, output and stream each): a launch's "
                         "blocks start on CUs the previous launch's last paths leave idle")
    ap.add_argument("--passes", type=int, default=16,
                    help="frames per launch, the same at every N (tray_render_passes_async: consecutive "
                         "progressive passes in one persistent launch, one tail of long paths per launch)")
    ap.add_argument("--rank-timeout", type=float, default=900.0,
                    help="N > 1: a rank that spends this many seconds in one phase (scene upload, warmup, timed "
                         "frames, ...) exits 124 naming it (under any launcher; also the process group's collective "
                         "timeout); bench.py's own launcher stops every rank once one fails, and the ranks still "
                         "running after 8x this long in total (0: no limit)")
    ap.add_argument("--cpu-min-seconds", type=float, default=10.0,
                    help="cpu_baseline: render further progressive passes of the sample until this much time has "
                         "passed (small frames, C1)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # No launcher: start the N ranks here, before anything touches the GPU.
        # The ranks' watchdogs bound each phase; this bounds the whole run as a backstop.
        return launch_ranks(args.gpus, sys.argv[1:], 8 * args.rank_timeout if args.rank_timeout > 0 else None)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and args.rank_timeout > 0:
        # Under any launcher (torchrun included) a rank stuck in a collective ends with a
        # non-zero exit that names it and the phase it was in, instead of hanging.
        start_watchdog(rank, args.rank_timeout)

    import torch

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # TRAY_BENCH_BACKEND=gloo rehearses the N > 1 code path on ONE GPU (ranks
    # share device 0; RCCL refuses two ranks on one device). Never for numbers.
    backend = os.environ.get("TRAY_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local_rank = 0
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and ndev == 1:
        # A launcher that gives each rank one visible GPU (HIP_VISIBLE_DEVICES per rank):
        # every rank renders on its device 0; distinct devices are checked below.
        local_rank = 0
    elif world > 1 and backend == "nccl" and ndev < world:
        print(f"bench.py: --gpus {world} needs {world} visible GPUs (or one per rank), found {ndev}",
              file=sys.stderr)
        return 2
    torch.cuda.set_device(local_rank)
    dist = None
    dist_rec = None
    if world > 1:
        import torch.distributed as dist

        from datetime import timedelta

        set_phase("init_process_group")
        to = {"timeout": timedelta(seconds=args.rank_timeout)} if args.rank_timeout > 0 else {}
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), **to)
        else:
            dist.init_process_group(backend, **to)
        # What the process group saw: its size and every rank's device.
        devs = [None] * world
        dist.all_gather_object(devs, dict(device_record(torch, local_rank), rank=rank))
        keys = [d["pci"] or d["uuid"] or str(d["device"]) for d in devs]
        if backend == "nccl" and len(set(keys)) != world:
            print(f"bench.py: RCCL ranks share devices: {keys}", file=sys.stderr)
            return 3
        dist_rec = {"backend": backend, "world": dist.get_world_size(), "devices": devs,
                    "launcher": os.environ.get("TRAY_BENCH_LAUNCHER", "external")}

    from tray_amd import _lib, ray, shard

    set_phase("scene upload")
    label, seed, half, W, H, spp, depth = CONFIGS[args.config]
    spheres = ray.rich_scene_array(seed, half)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    bg = ray._background(ray.DefaultBackground())
    params = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGB_F32,
                              flags=_lib.FLAG_LINEAR_SCAN if args.linear else 0)
    params = shard.shard_params(params, args.tile_rows, world, rank)
    rows = _lib.params_rows(params)
    # A step is one frame. Frames are rendered F per launch at every N (progressive
    # passes of tray_render_passes_async: lanes flow from one frame's samples into
    # the next, so a launch has one tail of long paths, not F), and launches
    # rotate over frame slots (own output and stream; the scene's launch context of
    # that stream holds the work queue and chunk records), so launch j+1 starts on
    # the CUs launch j's last paths leave idle. At N > 1 each launch's F frames are gathered to rank 0 with ONE
    # gather on a stream of its own; the next launch into the same slot waits for it.
    F = max(1, min(args.passes, args.steps))
    nslot = max(1, args.frames_in_flight)
    # ONE device scene for every slot: each slot's stream gets a launch context of its own
    # (work queue, chunk records, candidate records; include/tray.h "Concurrency"), so the
    # launches in flight share the scene as goroutines share a *Scene.
    scene = _lib.DeviceScene(spheres, bg, local_rank)
    plan = scene.plan(cam._state, params, F).as_dict()  # tray_render_plan_get: how the timed launches run
    outs = [torch.empty((F, rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nslot)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nslot - 1)]
    comm = torch.cuda.Stream() if world > 1 else None
    gathered = [None] * nslot
    gathers = {}  # (slot, frames) -> shard.FrameGather: receive and frame buffers allocated once

    def gather_for(k, n):
        if (k, n) not in gathers:
            gathers[(k, n)] = shard.FrameGather(n, H, W, (3,), args.tile_rows, world, rank, torch.float32,
                                                torch.device("cuda", local_rank))
        return gathers[(k, n)]
    out, stream = outs[0], streams[0]

    def launch(k, first, n):
        """Frames first .. first + n - 1 (progressive passes) in slot k."""
        p = _lib.Params.from_buffer_copy(params)
        p.pass_ = first % 4096
        if n == 1:
            scene.render_async(cam._state, p, outs[k].data_ptr(), None, streams[k].cuda_stream)
        else:
            scene.render_passes_async(cam._state, p, n, outs[k].data_ptr(), streams[k].cuda_stream)

    def frames(first, count):
        j = 0
        for i in range(first, first + count, F):
            n = min(F, first + count - i)
            k = j % nslot
            if gathered[k] is not None:  # slot k's previous frames have left for rank 0
                streams[k].wait_event(gathered[k])
            with torch.cuda.stream(streams[k]):
                launch(k, i, n)
            if world > 1:
                comm.wait_stream(streams[k])
                with torch.cuda.stream(comm):
                    gather_for(k, n)(outs[k][:n])
                    gathered[k] = torch.cuda.Event()
                    gathered[k].record(comm)
            j += 1

    # Untimed instrumented launches: segments, ray-sphere and ray-box tests for the
    # roofline, one per frame of the roofline's launch (passes 0 .. F-1).
    segments_local = sphere_tests = box_tests = 0
    for k in range(F):
        stats = torch.zeros(3, dtype=torch.int64, device="cuda")
        p = _lib.Params.from_buffer_copy(params)
        p.pass_ = k
        scene.render_stats_async(cam._state, p, out.data_ptr(), stats.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        seg_k, sph_k, box_k = (int(v) for v in stats.tolist())
        segments_local, sphere_tests, box_tests = segments_local + seg_k, sphere_tests + sph_k, box_tests + box_k

    for k in range(nslot):  # setup: each slot's sample buffer and launch state
        launch(k, 0, F)
        if world > 1:  # and its gather buffers, for every launch size the timed frames use
            for n in {F, args.steps % F} - {0}:
                gather_for(k, n)
    set_phase("warmup")
    frames(0, args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    set_phase("timed frames")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames(args.warmup, args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # Untimed: one launch at a time, HIP events on the launch stream.
    def launch_ms(n, reps=3):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(stream)
            launch(0, 0, n)
            b.record(stream)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev]))

    set_phase("launch timings")
    kernel_ms = launch_ms(F)  # the timed launch shape: F frames, megakernel + F resolves
    single_ms = kernel_ms if F == 1 else None if args.no_single else launch_ms(1)  # one frame, nothing overlapped
    ranks_rec = parity_n = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        set_phase("per-rank gather timing")
        # Untimed, per rank: the render of its rows (kernel_ms above) and one gather of F frames
        # (HIP events on the gather's stream), so a measured curve separates imbalance from the gather.
        torch.cuda.synchronize()
        dist.barrier()
        g = gather_for(0, F)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a, b in evs:
            with torch.cuda.stream(comm):
                a.record(comm)
                g(outs[0][:F])
                b.record(comm)
        torch.cuda.synchronize()
        mine = {"rank": rank, "rows": rows, "render_ms_per_frame": round(kernel_ms / F, 4),
                "gather_ms_per_launch": round(float(np.mean([a.elapsed_time(b) for a, b in evs])), 4)}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        r_ms = [r["render_ms_per_frame"] for r in allr]
        ranks_rec = {"per_rank": allr, "render_ms_per_frame_max": max(r_ms), "render_ms_per_frame_min": min(r_ms),
                     "imbalance": round(max(r_ms) / min(r_ms), 4),
                     "gather_ms_per_launch_max": max(r["gather_ms_per_launch"] for r in allr),
                     "what": "untimed: one launch of F frames of each rank's rows (HIP events) and one gather of "
                             "F frames to rank 0 (HIP events on the gather stream); ms_per_step is the timed run"}
        if not args.no_cpu_baseline:
            # Untimed: is the frame the N ranks assemble the right image? Every rank renders
            # pass 0 again in the timed shape and as FP64 with segment counts; all three are
            # gathered to rank 0, which checks them against the oracle (ray/tracer.go:86-116
            # splits rows over goroutines; here over ranks, and the pixels must not change).
            set_phase("gathered-frame parity")
            torch.cuda.synchronize()
            dist.barrier()
            gathered = gather_pass0(torch, _lib, shard, scene, cam, params, F, launch, outs[0], gather_for(0, F),
                                    args.tile_rows, world, rank)
            if rank == 0:
                row_step = args.cpu_row_step or auto_row_step(len(spheres), W, H, spp)
                parity_n = gathered_parity(gathered, spheres, cam._state.as_array(), W, H, spp, depth, seed, row_step)
            dist.barrier()

    samples = W * H * spp
    value = samples * args.steps / elapsed / 1e6
    rec = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,  # BASELINE.json "published" is empty
        "reference_readme_mrays": 0.33,  # derived from README.md:30-31 (M3 Pro, 11 cores, C2, ~3 min); context only
        "dtype": "f64",
        "data": "synthetic: RichScene book-cover generator on the counter RNG (include/tray.h), RichSceneCamera",
        "config": {
            "workload": label,
            "traversal": "linear" if args.linear else "bvh",
            "width": W, "height": H, "rays_per_pixel": spp, "max_depth": depth, "scene_seed": seed,
            "spheres": int(len(spheres)), "output": "float3 f32 linear", "parallelism": f"row-tiles x{world}",
            "tile_rows": args.tile_rows if world > 1 else 0,
            "frames_in_flight": nslot,
            "frames_per_launch": F,
        },
        "single_launch_ms": round(single_ms, 4) if single_ms else None,
        "accumulation": ("fixed-point chunk sums in LDS (exact, order-free; DESIGN.md 5)" if plan["acc_slots"] > 0
                         else "fixed-point sums through the per-sample buffer" if plan["fixed_point_shift"] > 0
                         else "FP64 sum in sample order"),
        "plan": plan,
    }
    if dist_rec:
        rec["rccl_world"] = dist_rec["world"] if backend == "nccl" else None
        rec["dist"] = dist_rec
        rec["ranks"] = ranks_rec
    if world > 1 and backend != "nccl":
        rec["rehearsal_backend"] = backend  # code-path check only, not a measurement
    if rank == 0:
        local_samples = rows * W * spp * F  # per launch: F frames
        ops64 = 17.0 * sphere_tests + 60.0 * segments_local + 40.0 * local_samples
        ops32 = 11.0 * box_tests
        ops = ops64 + 0.5 * ops32
        brute = 17.0 * len(spheres) * segments_local + 60.0 * segments_local + 40.0 * local_samples
        achieved = ops / (kernel_ms * 1e-3) / 1e12
        alg_bytes = rows * W * 12 * F  # the float3 frames the launch writes
        traffic = util = pmc_src = mix_src = None
        code_hash = _lib.code_object_sha256(_lib.LIB_PATH)
        why_null = {}
        if world == 1:
            pmc, pmc_src, why_null["traffic"] = _profile_json("pmc", args.config, F, code_hash)
            traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
            util, mix_src, why_null["util"] = _profile_json("pmc_mix", args.config, F, code_hash)
        else:
            why_null = {"traffic": "counters are profiled at N = 1", "util": "counters are profiled at N = 1"}
        roof = {
            "bound": "valu",
            "achieved": round(achieved, 3),
            "peak": FP64_PEAK_OPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / FP64_PEAK_OPS, 4),
            "traffic": traffic,
            # achieved HBM bandwidth of the megakernel launch against the 8 TB/s roof (PMC bytes / launch time)
            "hbm_gbs": round(traffic / (kernel_ms * 1e-3) / 1e9, 2) if traffic else None,
            "hbm_frac": round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6) if traffic else None,
            "hbm_peak_gbs": HBM_PEAK_GBS,
            "code_object_sha256": code_hash,
            "kernel_ms": round(kernel_ms, 4),
            "frames_per_launch": F,
            "peak_measured": FP64_PEAK_MEASURED,
            "frac_of_measured_peak": round(achieved / FP64_PEAK_MEASURED, 4),
            "peak_measured_source": "profiles/r1_fp64_peak.json (tools/fp64_peak.hip, v_mul_f64 + v_add_f64)",
            "segments_per_launch": segments_local,
            "sphere_tests_per_launch": sphere_tests,
            "box_tests_per_launch": box_tests,
            "fp64_ops_per_launch": ops64,
            "fp32_ops_per_launch": ops32,
            "ops_model": "FP64-op equivalents: 17/sphere test + 60/segment + 40/sample (FP64, no FMA; SURVEY.md 8d) "
                         "+ 0.5 x 11/box test (FP32 issues at 2x FP64 on SIMD-32); "
                         "peak = 78.6 TFLOP/s FP64 vector spec / 2 = 39.3 T ops/s",
            "algorithmic_bytes_per_launch": alg_bytes,
            "traffic_over_algorithmic": round(traffic / alg_bytes, 2) if traffic else None,
            "traffic_note": "megakernel HBM bytes by PMC (FETCH_SIZE x2 + WRITE_SIZE). With 64 | r (or r = 16, 32) "
                            "each pixel's samples are summed exactly in LDS as fixed-point integers and the megakernel "
                            "writes one 32-B record per 64-sample chunk (per pixel-pass at r = 16, 32; DESIGN.md 5, "
                            "Accumulation); the resolve pass turns them into the frames",
            "traversal": "linear scan" if args.linear else "exact-culling 4-wide BVH; camera rays: per-pixel "
                                                            "candidate lists (no traversal)",
            "ops_note": "achieved counts the work executed: the candidate lists removed ~35 % of the box tests "
                        "(C2), which lowered frac while the frame got faster; valu_issue_util and lane_util are "
                        "the counter figures no acceleration structure moves (DESIGN.md 5)",
            "brute_force_equiv": {"ops_per_launch": brute,
                                  "TFLOPs": round(brute / (kernel_ms * 1e-3) / 1e12, 3),
                                  "note": "NOT a roofline fraction: the reference's work (every sphere tested per "
                                          "segment) over the measured time; the BVH skips ~99.7 % of it exactly"},
        }
        # BASELINE.md's secondary metrics, over the same timed launch
        sec = kernel_ms * 1e-3
        rec["secondary"] = {"segments_per_s": round(segments_local / sec, 1),
                            "sphere_tests_per_s": round(sphere_tests / sec, 1),
                            "box_tests_per_s": round(box_tests / sec, 1),
                            "segments_per_sample": round(segments_local / local_samples, 4),
                            "scope": "rank 0's rows, one launch of F frames (kernel_ms)"}
        if util:
            roof["valu_issue_util"] = util.get("valu_issue_utilisation")
            roof["lane_util"] = util.get("valu_lane_utilisation")
            roof["util_source"] = mix_src
            if roof["valu_issue_util"] and roof["lane_util"]:
                # the same instruction stream at full issue on 64 active lanes (tools/attainable.py)
                roof["attainable"] = round(roof["frac"] / (roof["valu_issue_util"] * roof["lane_util"]), 4)
                roof["attainable_note"] = ("frac / (valu_issue_util x lane_util): what the parity contract's "
                                           "instruction stream allows; the rest of the gap to it is divergence "
                                           "(1/lane_util) and issue stalls (1/valu_issue_util), DESIGN.md 8b")
        else:
            roof["valu_issue_util"] = roof["lane_util"] = None
            roof["util_null_reason"] = why_null.get("util")
        if traffic:
            roof["traffic_source"] = pmc_src
        else:
            roof["traffic_null_reason"] = why_null.get("traffic")
        rec["roofline"] = roof
        if world == 1 and not args.no_e2e:
            rec["e2e"] = e2e_timings(_lib, spheres, bg, cam, W, H, depth, spp, seed)
        if world == 1 and not args.no_cpu_baseline:
            row_step = args.cpu_row_step or auto_row_step(len(spheres), W, H, spp)
            rec["cpu_baseline"], ref = cpu_baseline(spheres, cam._state.as_array(), W, H, spp, depth, seed, row_step,
                                                    args.cpu_min_seconds)
            rec["parity"] = device_parity(torch, _lib, scene, cam, params, F, launch, outs[0], ref, row_step)
        elif parity_n is not None:
            rec["parity"] = parity_n
        else:
            rec["parity"] = None
            rec["parity_null_reason"] = "--no-cpu-baseline: no oracle frame"
    if rank == 0:
        print(json.dumps(rec), flush=True)
    set_phase("teardown")
    scene.release()
    if dist:
        dist.destroy_process_group()
    return 0


def e2e_timings(_lib, spheres, bg, cam, W, H, depth, spp, seed):
    """The drop-in call a Go caller makes instead of Tracer.Render (benchmark.go:88
    times rt.Render): one synchronous tray_render of the whole frame into host
    memory as RGBA8 (image.RGBA.Pix). `first_call_ms`: the process's first
    synchronous call (a tiny render), which pays the HIP runtime's one-time costs
    (a new hardware queue for the library's stream, the pageable-copy staging
    buffer; tools/hip_setup_costs.hip measures ~8 ms each). `e2e_ms_new_scene`:
    the next call, with the config's scene not yet on the device (BVH build,
    upload, sample-buffer allocation, render, copy). `e2e_ms`: the same scene
    again (the library keeps the last scene it uploaded), median of 7.
    `e2e_ms_new_scene_warm`: three more scenes the device has not seen (one
    sphere nudged), median: a new scene once the buffers exist."""
    import numpy as np

    from tray_amd import ray

    tiny = _lib.make_params(8, 8, 4, 1, 0.5, seed, output=_lib.OUT_RGBA8)
    t0 = time.perf_counter()
    _lib.render(ray.DefaultScene().to_array(), bg, cam._state, tiny)
    first = (time.perf_counter() - t0) * 1e3
    p = _lib.make_params(W, H, depth, spp, 0.5, seed, output=_lib.OUT_RGBA8)
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        _lib.render(spheres, bg, cam._state, p)
        ts.append((time.perf_counter() - t0) * 1e3)
    warm = float(np.median(ts[1:]))
    news = []
    for k in range(3):  # scenes the process has not seen, after it has rendered at this size
        other = np.array(spheres, copy=True)
        other["center"][-1][0] += 1e-9 * (k + 1)
        t0 = time.perf_counter()
        _lib.render(other, bg, cam._state, p)
        news.append((time.perf_counter() - t0) * 1e3)
    return {"first_call_ms": round(first, 3), "e2e_ms_new_scene": round(ts[0], 3), "e2e_ms": round(warm, 3),
            "e2e_ms_new_scene_warm": round(float(np.median(news)), 3),
            "e2e_mrays": round(W * H * spp / warm / 1e3, 1),
            "what": "tray_render, RGBA8 into host memory; new_scene: the first call at this size (BVH build, upload, "
                    "allocations); new_scene_warm: a new scene once the process has rendered at this size"}


def auto_row_step(n_spheres, W, H, spp):
    """Row stride that keeps the CPU sample near the whole C2 frame's linear-scan
    work (1280x720 px x r=64 x 486 spheres): C1, C2 every row; C3, C5 every 36th."""
    return max(1, round(W * H * spp * max(n_spheres, 1) / (1280 * 720 * 64 * 486)))


def cpu_share() -> tuple:
    """Threads for the CPU baseline: the CPUs this job may use, not the machine's.
    BASELINE.md planned w = nproc (GOMAXPROCS, ray/tracer.go:77-79), but on the
    GPU box nproc reports the whole host while a one-GPU job's share is 16
    (OMP_NUM_THREADS there); more threads than the share would time the
    scheduler, not the port. The smallest of the cgroup CPU quota, the affinity
    mask and OMP_NUM_THREADS, with each figure stated."""
    seen = {"nproc": os.cpu_count() or 1}
    try:
        seen["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            seen["cgroup_quota"] = max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        seen["OMP_NUM_THREADS"] = int(omp)
    cores = min(seen.values())
    return cores, "min of " + ", ".join(f"{k}={v}" for k, v in seen.items())


def cpu_baseline(spheres, camera, W, H, spp, depth, seed, row_step, min_seconds=0.0):
    """Oracle (C FP64 port of the reference CPU path, chunk-queue scheduler of
    ray/tracer.go:86-116) on every `row_step`-th row of the same frame, pass 0;
    while less than `min_seconds` have passed, passes 1, 2, ... of the same rows
    (a frame as small as C1's renders in well under a second). Returns the
    record and pass 0's (rows, segments) for the parity check. Pass 0 is timed
    with segments=True: the oracle counts every path's Scene.Hit calls whether or
    not they are asked for (tray_oracle.c render_pixel), the flag only stores one
    uint32 per pixel, so the timed work is the same as with segments=False."""
    from oracle import oracle as O

    cores, why = cpu_share()
    rows = np.arange(0, H, row_step, dtype=np.int32)
    bg = np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0])
    t0 = time.perf_counter()
    ref = O.render_rows(spheres, bg, camera, W, H, spp, depth, 0.5, seed, rows, workers=cores, segments=True)
    passes = 1
    while time.perf_counter() - t0 < min_seconds:
        O.render_rows(spheres, bg, camera, W, H, spp, depth, 0.5, seed, rows, workers=cores, segments=False,
                      pass_=passes)
        passes += 1
    dt = time.perf_counter() - t0
    samples = len(rows) * W * spp * passes
    what = f"{len(rows)} rows x {W} px x r={spp}" + (f" x {passes} passes" if passes > 1 else "")
    return ({"value": round(samples / dt / 1e6, 4), "unit": "Mrays/s", "cores": cores, "kind": "port",
             "seconds": round(dt, 3), "cpu_model": cpu_model(), "cores_reason": why, "passes": passes,
             "sample": f"every {row_step}. row of the same frame ({what}), oracle/tray_oracle.c, {cores} pthreads"},
            (rows, ref))


def frame_parity(ref, ref_seg, f64, seg, f32, tol=1e-4):
    """Per-pixel parity of device frames against the oracle's frame of the same
    pass (ray/tracer.go:120-155): `f64` (TRAY_OUT_RGB_F64) and `f32`
    (TRAY_OUT_RGB_F32) are [rows, W, 3], `seg`/`ref_seg` the per-pixel Scene.Hit
    counts. The f32 bound: one f32 rounding (<= 2^-24 |v|) of a value within
    1e-12 of the oracle's mean."""
    ref = np.asarray(ref, dtype=np.float64)
    d64 = np.abs(np.asarray(f64, dtype=np.float64) - ref)
    g32 = np.asarray(f32, dtype=np.float32)
    d32 = np.abs(g32.astype(np.float64) - ref)
    linf = float(d64.max()) if d64.size else 0.0
    linf32 = float(d32.max()) if d32.size else 0.0
    rec = {"pixels": int(ref.shape[0] * ref.shape[1]), "rows": int(ref.shape[0]), "linf": linf, "linf_f32": linf32,
           "segments_equal": bool(np.array_equal(seg, ref_seg)), "segments_differing": int((seg != ref_seg).sum()),
           "f64_bit_equal_frac": round(float((f64 == ref).mean()), 4),
           "f32_within_one_rounding": bool(np.all(d32 <= np.abs(ref) * 2.0**-24 + 1e-12)),
           "f32_equal_frac": round(float((g32 == ref.astype(np.float32)).mean()), 4),
           "tol": tol}
    rec["ok"] = bool(rec["segments_equal"] and linf <= tol and linf32 <= tol and np.isfinite(ref).all())
    return rec


def gather_pass0(torch, _lib, shard, scene, cam, params, F, launch, out, gather32, tile_rows, world, rank):
    """N > 1, every rank (untimed): pass 0 of its rows (a) as frame 0 of a passes
    launch in the timed shape (slot 0, F frames, TRAY_OUT_RGB_F32) gathered to rank 0
    by the timed frames' own FrameGather, and (b) through tray_render_async as
    TRAY_OUT_RGB_F64 with per-pixel Scene.Hit counts, gathered likewise. Returns
    rank 0's assembled (f64 [H, W, 3], segments [H, W], f32 [H, W, 3]) as numpy,
    None on the other ranks."""
    W, H = params.width, params.height
    rows = _lib.params_rows(params)
    dev = torch.device("cuda", torch.cuda.current_device())
    p = _lib.Params.from_buffer_copy(params)
    p.output, p.pass_ = _lib.OUT_RGB_F64, 0
    f64 = torch.empty((1, rows, W, 3), dtype=torch.float64, device=dev)
    seg = torch.zeros((1, rows, W), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    scene.render_async(cam._state, p, f64.data_ptr(), seg.data_ptr(), stream.cuda_stream)
    with torch.cuda.stream(stream):
        launch(0, 0, F)  # frames 0 .. F-1 of this rank's rows, as the timed launches render them
    torch.cuda.synchronize()
    g32 = gather32(out[:F])
    g64 = shard.FrameGather(1, H, W, (3,), tile_rows, world, rank, torch.float64, dev)(f64)
    gseg = shard.FrameGather(1, H, W, (), tile_rows, world, rank, torch.int32, dev)(seg)
    torch.cuda.synchronize()
    if rank != 0:
        return None
    return (g64[0].cpu().numpy(), gseg[0].cpu().numpy().astype(np.uint32), g32[0].cpu().numpy())


def gathered_parity(gathered, spheres, camera, W, H, spp, depth, seed, row_step, workers=None):
    """N > 1, rank 0: the frame the ranks assembled (gather_pass0) against the
    oracle's pass 0 on every `row_step`-th row (the rows cpu_baseline renders at
    N = 1), with frame_parity's bar: segment counts bit-exact, L-inf <= 1e-4."""
    from oracle import oracle as O

    f64, seg, f32 = gathered
    rows = np.arange(0, H, row_step, dtype=np.int32)
    cores = workers or cpu_share()[0]
    t0 = time.perf_counter()
    ref, ref_seg = O.render_rows(spheres, np.array([1.0, 1.0, 1.0, 0.4, 0.65, 1.0]), camera, W, H, spp, depth, 0.5,
                                 seed, rows, workers=cores, segments=True)
    rec = frame_parity(ref, ref_seg, f64[rows], seg[rows], f32[rows])
    rec.update({"pass": 0, "oracle_seconds": round(time.perf_counter() - t0, 2),
                "scope": ("the whole gathered frame" if row_step == 1 else
                          f"every {row_step}. row of the gathered frame ({len(rows)} of {H} rows)"),
                "frame": "assembled on rank 0 from every rank's row tiles by the timed run's gather "
                         "(shard.FrameGather), f32 frame 0 of a passes launch and an f64 render with segment counts",
                "reference": "oracle/tray_oracle.c (ray/*.go restated; per-pixel parity with the Go binary's "
                             "fortio.org/rand stream is unpinned, DESIGN.md 3)"})
    return rec


def device_parity(torch, _lib, scene, cam, params, F, launch, out, oracle_frame, row_step):
    """Untimed: pass 0 of the frame on the device, (a) through tray_render_async into
    TRAY_OUT_RGB_F64 with segment counts and (b) as frame 0 of a passes launch in
    the timed shape (slot 0: F frames into TRAY_OUT_RGB_F32), against the oracle's
    pass 0 that cpu_baseline rendered, on the rows the oracle rendered."""
    rows_idx, (ref, ref_seg) = oracle_frame
    W, H = params.width, params.height
    p = _lib.Params.from_buffer_copy(params)
    p.output, p.pass_ = _lib.OUT_RGB_F64, 0
    f64 = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    seg = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    scene.render_async(cam._state, p, f64.data_ptr(), seg.data_ptr(), stream.cuda_stream)
    with torch.cuda.stream(stream):
        launch(0, 0, F)  # frames 0 .. F-1 into `out`, exactly as the timed launches render them
    torch.cuda.synchronize()
    idx = torch.as_tensor(rows_idx, dtype=torch.long, device="cuda")
    rec = frame_parity(ref, ref_seg, f64[idx].cpu().numpy(), seg[idx].cpu().numpy().astype(np.uint32),
                       out[0][idx].cpu().numpy())
    rec["pass"] = 0
    rec["scope"] = ("the whole frame" if row_step == 1 else
                    f"every {row_step}. row ({len(rows_idx)} of {H} rows: the rows cpu_baseline rendered)")
    rec["reference"] = "oracle/tray_oracle.c (ray/*.go restated; per-pixel parity with the Go binary's " \
                       "fortio.org/rand stream is unpinned, DESIGN.md 3)"
    return rec


if __name__ == "__main__":
    sys.exit(main())
