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
