"""The multi-GPU path end to end on the device: 2 and 3 ranks (gloo, all on
device 0: RCCL refuses two ranks on one device, and 8-GPU runs are the
driver's) each render their interleaved row tiles with the megakernel
(tray_render_passes_async: several progressive passes in one launch) and
tray_amd.shard.gather_frames assembles the frames on rank 0. The result must
equal a single-rank render bit for bit: every draw is keyed on the global pixel
index (include/tray.h), unlike the reference's per-row-chunk stream
(ray/tracer.go:86-116, 121)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, SPP, DEPTH, SEED, PASSES = 96, 45, 4, 30, 6, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frames(L, ray, params, rows, passes):
    import torch

    spheres = ray.rich_scene_array(2)
    cam = ray.RichSceneCamera()
    cam.Initialize(W, H)
    dev = L.DeviceScene(spheres, ray._background(ray.DefaultBackground()), 0)
    out = torch.empty((passes, rows, W, 3), dtype=torch.float32, device="cuda")
    dev.render_passes_async(cam._state, params, passes, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    dev.release()
    return out


def _worker(rank, world, port, tile, path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tray_amd import _lib as L
    from tray_amd import ray, shard

    p = shard.shard_params(L.make_params(W, H, DEPTH, SPP, 0.5, SEED, output=L.OUT_RGB_F32, pass_=1), tile, world,
                           rank)
    local = _frames(L, ray, p, L.params_rows(p), PASSES)
    full = shard.gather_frames(local, H, tile, world, rank)
    if rank == 0:
        assert full.is_cuda
        np.save(path, full.cpu().numpy())
    else:
        assert full is None
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tile", [(2, 1), (3, 4)])
def test_device_shards_gathered_equal_single_rank(L, tmp_path, world, tile):
    from tray_amd import ray

    path = str(tmp_path / "frames.npy")
    mp.spawn(_worker, args=(world, _free_port(), tile, path), nprocs=world, join=True)
    got = np.load(path)
    ref = _frames(L, ray, L.make_params(W, H, DEPTH, SPP, 0.5, SEED, output=L.OUT_RGB_F32, pass_=1), H,
                  PASSES).cpu().numpy()
    assert got.shape == ref.shape == (PASSES, H, W, 3)
    assert np.array_equal(got, ref)
    assert not np.array_equal(got[0], got[1])
