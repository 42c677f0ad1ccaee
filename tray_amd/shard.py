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
    xGMI)."""
    import torch
    import torch.distributed as dist

    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo gathers host tensors only (RCCL, the nccl backend, gathers device
        # memory directly over xGMI): stage through the host, hand back a device frame.
        full = gather_frames(local.cpu(), height, tile_rows, world, rank, dst, group)
        return None if full is None else full.to(local.device)
    counts = [len(rows_for(height, tile_rows, world, r)) for r in range(world)]
    max_rows = max(counts)
    pad = local
    if local.shape[1] < max_rows:
        pad = torch.zeros((local.shape[0], max_rows) + tuple(local.shape[2:]), dtype=local.dtype,
                          device=local.device)
        pad[:, : local.shape[1]] = local
    elif not local.is_contiguous():
        pad = local.contiguous()
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.empty((local.shape[0], height) + tuple(local.shape[2:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        full.index_copy_(1, _row_index(height, tile_rows, world, r, local.device), bufs[r][:, : counts[r]])
    return full


_ROW_INDEX = {}


def _row_index(height, tile_rows, world, rank, device):
    """Device tensor of rows_for(...), built once (no host copy per gather)."""
    import torch

    key = (height, tile_rows, world, rank, str(device))
    if key not in _ROW_INDEX:
        _ROW_INDEX[key] = torch.as_tensor(rows_for(height, tile_rows, world, rank), dtype=torch.long, device=device)
    return _ROW_INDEX[key]
