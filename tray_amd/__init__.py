"""tray_amd — MI355X-native renderer for fortio/tray's per-pixel path-tracing loop.

Layout:
  csrc/          gfx950 megakernel (tray_kernel.hip), C-ABI glue (tray_abi.hip),
                 host setup (tray_host.cpp); built into libtray_amd.so
  _lib.py        ctypes binding of include/tray.h (no fallback path)
  ray.py         mirror of the Go `ray` package API (New/Render/RenderLines/...)
  shard.py       interleaved row-tile sharding + gather for multi-GPU renders
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
