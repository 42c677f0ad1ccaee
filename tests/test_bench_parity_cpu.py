"""bench.py's N > 1 parity on CPU (gloo, world 2 and 3): every rank's row tiles
(the oracle stands in for the device renderer) are assembled on rank 0 by
shard.FrameGather, exactly as bench.gather_pass0 assembles the device frames, and
bench.gathered_parity checks the assembled frame against the oracle's own render
(ray/tracer.go:86-116 splits rows over goroutines; the pixels must not change).
A corrupted shard - one colour off by 1e-3, or one Scene.Hit count off by one, on
one rank - must turn parity.ok false."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import DEFAULT_BG, RICH_SETUP

W, H, SPP, DEPTH, SEED = 40, 29, 4, 12, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_path, corrupt):
    import json

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import oracle as O
    from tray_amd import shard

    _, cam = O.camera_initialize(RICH_SETUP, W, H)
    spheres = O.rich_scene(2)
    rows = shard.rows_for(H, 1, world, rank)
    f64, seg = O.render_rows(spheres, DEFAULT_BG, cam, W, H, SPP, DEPTH, 0.5, SEED, rows, segments=True)
    f64, seg = np.array(f64), np.array(seg).astype(np.int32)
    if rank == world - 1 and corrupt == "colour":
        f64[len(rows) // 2, 7, 1] += 1e-3
    if rank == world - 1 and corrupt == "segments":
        seg[0, 3] += 1
    f32 = f64.astype(np.float32)
    dev = torch.device("cpu")
    g = [shard.FrameGather(1, H, W, c, 1, world, rank, torch.from_numpy(a).dtype, dev)(torch.from_numpy(a)[None])
         for a, c in ((f64, (3,)), (seg, ()), (f32, (3,)))]
    if rank == 0:
        gathered = (g[0][0].numpy(), g[1][0].numpy().astype(np.uint32), g[2][0].numpy())
        rec = bench.gathered_parity(gathered, spheres, cam, W, H, SPP, DEPTH, SEED, 1, workers=2)
        with open(result_path, "w") as f:
            json.dump(rec, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, None), (3, None), (2, "colour"), (3, "segments")])
def test_gathered_frame_parity(tmp_path, world, corrupt):
    import json

    path = str(tmp_path / "parity.json")
    mp.spawn(_worker, args=(world, _free_port(), path, corrupt), nprocs=world, join=True)
    rec = json.load(open(path))
    assert rec["pixels"] == W * H and rec["rows"] == H
    if corrupt is None:
        assert rec["ok"] and rec["linf"] == 0.0 and rec["segments_equal"]
    else:
        assert not rec["ok"]
        if corrupt == "colour":
            assert rec["linf"] > 1e-4 and rec["segments_equal"]
        else:
            assert rec["segments_differing"] == 1
