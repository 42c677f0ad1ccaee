"""The drain's wave-wide Scene.Hit (DESIGN.md §5 "The drain"; KernelParams::coop_lanes):
once a wave's work queue has run dry and it holds at most `coop_lanes` paths, the whole
wave scans every sphere for each of their segments instead of one lane traversing the
BVH. It returns the linear scan's closest hit, as the traversal does, so the frames and
the Scene.Hit counts per pixel must equal those with it off, bit for bit — whether it
takes over only the lone last paths (1, the default 2) or every path of a dry wave (64).
The rest of the GPU suite runs with the default and compares against the oracle."""
import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import WORKERS, bg_struct, camera, check

pytestmark = pytest.mark.gpu


def _render(L, torch, sc, st, p, passes, coop):
    with L.debug_knobs(coop_lanes=coop):
        dev = L.DeviceScene(sc, bg_struct(L, DEFAULT_BG), 0)
        try:
            rows = L.params_rows(p)
            out = torch.empty((passes, rows, p.width, 3), dtype=torch.float64, device="cuda")
            s = torch.cuda.current_stream()
            seg = None
            if passes == 1:
                seg = torch.zeros((rows, p.width), dtype=torch.int32, device="cuda")
                dev.render_async(st, p, out.data_ptr(), seg.data_ptr(), s.cuda_stream)
            else:
                dev.render_passes_async(st, p, passes, out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            return out.cpu().numpy(), None if seg is None else seg.cpu().numpy()
        finally:
            dev.release()


@pytest.mark.parametrize("spp,depth,passes,tiles", [(64, 9, 1, {}), (16, 12, 1, {}), (64, 50, 3, {}),
                                                    (16, 50, 4, {}),
                                                    (64, 50, 1, dict(tile_rows=1, tile_count=8, tile_index=3))])
def test_coop_drain_is_invisible(L, O, spp, depth, passes, tiles):
    import torch

    sc = O.rich_scene(2)
    w, h = 96, 54
    st = camera(L, RICH_SETUP, w, h)
    p = L.make_params(w, h, depth, spp, 0.5, 9, output=L.OUT_RGB_F64, **tiles)
    off, off_seg = _render(L, torch, sc, st, p, passes, 0)
    for coop in (1, 2, 64):
        on, on_seg = _render(L, torch, sc, st, p, passes, coop)
        assert np.array_equal(on, off), coop
        if off_seg is not None:
            assert np.array_equal(on_seg, off_seg), coop


def test_coop_drain_matches_the_oracle_everywhere(L, O):
    """Every dry wave's paths through the wave-wide scan (coop_lanes 64): pass 0 of a
    small frame against the oracle's, colours and Scene.Hit counts."""
    import torch

    sc = O.rich_scene(2)
    w, h, spp, depth = 40, 24, 64, 20
    st = camera(L, RICH_SETUP, w, h)
    p = L.make_params(w, h, depth, spp, 0.5, 5, output=L.OUT_RGB_F64)
    got, seg = _render(L, torch, sc, st, p, 1, 64)
    want, want_seg = O.render(sc, DEFAULT_BG, st.as_array(), w, h, spp, depth, 0.5, 5, workers=WORKERS)
    check(got[0], seg.astype(np.uint32), want, want_seg)
