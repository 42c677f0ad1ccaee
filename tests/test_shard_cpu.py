"""N > 1 path on CPU: world_size-2 gloo. Each rank renders its interleaved row
tiles (here with the oracle standing in for the device renderer) and
tray_amd.shard.gather_image assembles them on rank 0; the image must equal a
single-process render bit for bit (the counter RNG is keyed on global pixels)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import DEFAULT_BG, RICH_SETUP

W, H, SPP, DEPTH, SEED = 40, 29, 2, 12, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_path, tile):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from tray_amd import shard

    _, cam = O.camera_initialize(RICH_SETUP, W, H)
    rows = shard.rows_for(H, tile, world, rank)
    local = O.render_rows(O.rich_scene(2), DEFAULT_BG, cam, W, H, SPP, DEPTH, 0.5, SEED, rows, segments=False)
    full = shard.gather_image(torch.from_numpy(local), H, tile, world, rank)
    if rank == 0:
        np.save(result_path, full.numpy())
    else:
        assert full is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 4), (3, 4), (2, 1)])
def test_gather_row_tiles_gloo(O, tmp_path, world, tile):
    path = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), path, tile), nprocs=world, join=True)
    got = np.load(path)
    _, cam = O.camera_initialize(RICH_SETUP, W, H)
    ref = O.render(O.rich_scene(2), DEFAULT_BG, cam, W, H, SPP, DEPTH, 0.5, SEED, segments=False)
    assert np.array_equal(got, ref)


def _worker_frames(rank, world, port, result_path, tile):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from tray_amd import shard

    _, cam = O.camera_initialize(RICH_SETUP, W, H)
    rows = shard.rows_for(H, tile, world, rank)
    # a batch of progressive passes 1..3, as one tray_render_passes_async launch would produce
    local = np.stack([O.render_rows(O.rich_scene(2), DEFAULT_BG, cam, W, H, SPP, DEPTH, 0.5, SEED, rows,
                                    segments=False, pass_=k) for k in (1, 2, 3)])
    full = shard.gather_frames(torch.from_numpy(local), H, tile, world, rank)
    if rank == 0:
        np.save(result_path, full.numpy())
    else:
        assert full is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 1), (3, 2)])
def test_gather_pass_batch_gloo(O, tmp_path, world, tile):
    """N > 1 with several progressive passes per launch: ONE gather per batch
    reassembles every frame bit for bit."""
    path = str(tmp_path / "frames.npy")
    mp.spawn(_worker_frames, args=(world, _free_port(), path, tile), nprocs=world, join=True)
    got = np.load(path)
    _, cam = O.camera_initialize(RICH_SETUP, W, H)
    for i, k in enumerate((1, 2, 3)):
        ref = O.render(O.rich_scene(2), DEFAULT_BG, cam, W, H, SPP, DEPTH, 0.5, SEED, segments=False, pass_=k)
        assert np.array_equal(got[i], ref)
    assert not np.array_equal(got[0], got[1])


def _old_gather(local, height, tile, world, rank):
    """The round-3 gather (per call: padded send buffer, `world` receive buffers,
    a fresh frame and one index_copy_ per rank), kept as the reference."""
    import torch
    import torch.distributed as dist

    from tray_amd import shard

    counts = [len(shard.rows_for(height, tile, world, r)) for r in range(world)]
    pad = torch.zeros((local.shape[0], max(counts)) + tuple(local.shape[2:]), dtype=local.dtype)
    pad[:, : local.shape[1]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0)
    if rank != 0:
        return None
    full = torch.empty((local.shape[0], height) + tuple(local.shape[2:]), dtype=local.dtype)
    for r in range(world):
        idx = torch.as_tensor(shard.rows_for(height, tile, world, r), dtype=torch.long)
        full.index_copy_(1, idx, bufs[r][:, : counts[r]])
    return full


def _worker_framegather(rank, world, port, result_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tray_amd import shard

    ok = True
    for height, tile in [(29, 1), (29, 4), (24, 1), (31, 3), (5, 8), (90, 1)]:
        rows = shard.rows_for(height, tile, world, rank)
        g = shard.FrameGather(3, height, 7, (3,), tile, world, rank, torch.float32, torch.device("cpu"))
        for call in range(3):  # the buffers are reused from call to call
            gen = torch.Generator().manual_seed(1000 * height + 10 * tile + call)
            frame = torch.rand((3, height, 7, 3), generator=gen)
            local = frame[:, torch.as_tensor(rows, dtype=torch.long)].contiguous()
            new = g(local)
            old = _old_gather(local, height, tile, world, rank)
            if rank == 0:
                ok &= bool(torch.equal(new, old)) and bool(torch.equal(new, frame))
            else:
                ok &= new is None and old is None
    flags = [None] * world
    dist.all_gather_object(flags, ok)
    if rank == 0:
        np.save(result_path, np.array(flags))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_frame_gather_equals_round3_gather(tmp_path, world):
    """shard.FrameGather (buffers allocated once, one strided copy into image
    order) equals the round-3 gather bit for bit, over ragged heights, tiles with
    a partial last tile, ranks with fewer rows than others and repeated calls."""
    path = str(tmp_path / "ok.npy")
    mp.spawn(_worker_framegather, args=(world, _free_port(), path), nprocs=world, join=True)
    assert np.load(path).all()


def _worker_owned(rank, world, port, result_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tray_amd import shard

    ok = True
    kept = []
    for call in range(shard._GATHERS_MAX + 3):  # more shapes than the cache keeps, then the first again
        height = 9 + (call % (shard._GATHERS_MAX + 2))
        rows = shard.rows_for(height, 1, world, rank)
        frame = torch.full((2, height, 5, 3), float(call))
        got = shard.gather_frames(frame[:, torch.as_tensor(rows, dtype=torch.long)].contiguous(), height, 1, world,
                                  rank)
        if rank == 0:
            kept.append((got, frame))
            ok &= all(bool(torch.equal(g, f)) for g, f in kept)  # earlier results untouched by later gathers
        else:
            ok &= got is None
        ok &= len(shard._GATHERS) <= shard._GATHERS_MAX
    flags = [None] * world
    dist.all_gather_object(flags, ok)
    if rank == 0:
        np.save(result_path, np.array(flags))
    dist.destroy_process_group()


def test_gather_frames_returns_owned_tensors(tmp_path):
    """gather_frames / gather_image return tensors of the caller's own: a later
    gather of the same shape does not overwrite an earlier result, and the
    per-shape buffers kept between calls are bounded."""
    path = str(tmp_path / "ok.npy")
    mp.spawn(_worker_owned, args=(2, _free_port(), path), nprocs=2, join=True)
    assert np.load(path).all()
