"""Multi-GPU row-tile sharding.

Pixels are independent and every draw is keyed on the GLOBAL pixel index
(include/tray.h), so an image split into interleaved row tiles and reassembled
is bit-identical to a single-device render. Tile k of `tile_rows` rows goes to
rank k mod world: interleaving balances cheap sky rows against ground rows
(the reference's own scheduler balances with a chunk queue instead,
ray/tracer.go:93-116). Each rank renders its tiles into a COMPACT buffer; the
only exchange is one gather of those buffers to the destination rank (RCCL over
xGMI with the nccl backend, gloo on CPU in tests).
"""
from __future__ import annotations

import numpy as np

from . import _lib


def rows_for(height: int, tile_rows: int, world: int, rank: int, y_start: int = 0, y_end: int | None = None
             ) -> np.ndarray:
    """Image rows owned by `rank`, in compact order (mirrors row_of() in the kernel)."""
    y_end = height if y_end is None else y_end
    ys = np.arange(y_start, y_end, dtype=np.int64)
    if tile_rows <= 0:
        return ys.astype(np.int32)
    tile = (ys - y_start) // tile_rows
    return ys[tile % world == rank].astype(np.int32)


def shard_params(params: _lib.Params, tile_rows: int, world: int, rank: int) -> _lib.Params:
    p = _lib.Params.from_buffer_copy(params)
    if world > 1:
        p.tile_rows, p.tile_count, p.tile_index = tile_rows, world, rank
    return p


def gather_image(local, height: int, tile_rows: int, world: int, rank: int, dst: int = 0, group=None):
    """Gather every rank's compact rows (torch tensor [rows_r, W, C]) to `dst` and
    return the assembled [height, W, C] image there (None elsewhere).

    Uses ONE torch.distributed.gather of equal-size (padded) buffers."""
    full = gather_frames(local.unsqueeze(0), height, tile_rows, world, rank, dst, group)
    return None if full is None else full[0]


def gather_frames(local, height: int, tile_rows: int, world: int, rank: int, dst: int = 0, group=None):
    """gather_image for a batch of frames (the passes of one
    tray_render_passes_async launch): local [n, rows_r, W, C] -> [n, height, W, C]
    on `dst`, with ONE gather for the whole batch (fewer, larger transfers over
    xGMI). Returns a tensor of the caller's own: the receive buffers are kept
    per shape (a FrameGather, at most _GATHERS_MAX shapes) and the result is
    copied out of them. Callers that gather every launch (bench.py's frame
    slots) hold a FrameGather each and use its zero-copy view instead."""
    key = (tuple(local.shape), str(local.dtype), str(local.device), height, tile_rows, world, rank, dst, id(group))
    g = _GATHERS.pop(key, None)
    if g is None:
        g = FrameGather(local.shape[0], height, local.shape[2], tuple(local.shape[3:]), tile_rows, world, rank,
                        local.dtype, local.device, dst, group)
    _GATHERS[key] = g  # most recently used last
    while len(_GATHERS) > _GATHERS_MAX:
        _GATHERS.pop(next(iter(_GATHERS)))
    full = g(local)
    return None if full is None else full.clone()


_GATHERS: dict = {}
_GATHERS_MAX = 4


class FrameGather:
    """Rank `dst` assembles every rank's compact rows of F frames into image
    order, with buffers allocated once:

    * every rank sends an equal-size [F, max_rows, W, C] buffer (its own output
      when it holds max_rows rows, else a preallocated padded copy);
    * `dst` receives the world's buffers into ONE contiguous [world, F, max_rows,
      W, C] tensor (the gather list is views of it);
    * one strided copy puts them in image order: with tiles of t rows, rank k's
      compact row i is image row (k + world * (i // t)) * t + i % t, i.e. the
      image padded to Hpad = world * max_rows rows is
      recv.view(world, F, max_rows / t, t, W, C) permuted to
      (F, max_rows / t, world, t, W, C); rows >= height are padding.

    This replaces a per-launch allocation of `world` receive buffers and a full
    frame plus `world` index_copy_ scatters on `dst` (round 3), which made the
    destination rank the straggler of every launch."""

    def __init__(self, frames, height, width, channels, tile_rows, world, rank, dtype, device, dst=0, group=None):
        import torch
        import torch.distributed as dist

        self.F, self.H, self.W, self.C = frames, height, width, tuple(channels)
        self.t = tile_rows if tile_rows > 0 else height
        self.world, self.rank, self.dst, self.group = world, rank, dst, group
        self.counts = [len(rows_for(height, tile_rows, world, r)) for r in range(world)]
        tiles = -(-height // self.t)
        self.tiles_per_rank = -(-tiles // world)
        self.max_rows = self.tiles_per_rank * self.t  # a multiple of t, >= every count
        self.device = device
        self.host_staged = str(device).startswith("cuda") and dist.get_backend(group) == "gloo"
        buf_dev = "cpu" if self.host_staged else device
        shape = (frames, self.max_rows, width) + self.C
        self.send = torch.zeros(shape, dtype=dtype, device=buf_dev)
        self.recv = self.full = None
        if rank == dst:
            self.recv = torch.zeros((world,) + shape, dtype=dtype, device=buf_dev)
            self.recv_list = list(self.recv.unbind(0))
            self.full = torch.empty((frames, world * self.max_rows, width) + self.C, dtype=dtype, device=device)

    def __call__(self, local):
        import torch.distributed as dist

        n = self.counts[self.rank]
        if tuple(local.shape) != (self.F, n, self.W) + self.C:
            raise ValueError(f"local frames {tuple(local.shape)} != {(self.F, n, self.W) + self.C}")
        if self.host_staged or n != self.max_rows or not local.is_contiguous():
            self.send[:, :n].copy_(local)
            out = self.send
        else:
            out = local  # already the equal-size buffer: sent as is
        dist.gather(out, gather_list=self.recv_list if self.rank == self.dst else None, dst=self.dst,
                    group=self.group)
        if self.rank != self.dst:
            return None
        tpr, t, w = self.tiles_per_rank, self.t, self.world
        src = self.recv.view((w, self.F, tpr, t, self.W) + self.C).permute(1, 2, 0, 3, 4, *range(5, 5 + len(self.C)))
        self.full.view((self.F, tpr, w, t, self.W) + self.C).copy_(src)
        return self.full[:, : self.H]
