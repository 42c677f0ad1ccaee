"""The synchronous C-ABI under concurrent callers (tray_abi.hip lock order).

A render takes its device's lock and, when the scene changed, uploads the new
one (which looks the device up under the global device-table lock);
tray_release_cache / tray_shutdown take the table lock only to copy the device
states and then lock each device. One thread renders alternating scenes while
another releases the cache in a loop: both must finish (no lock-order
deadlock), and every frame must equal its scene's reference frame."""
import threading

import numpy as np
import pytest

from conftest import DEFAULT_BG, RICH_SETUP
from test_gpu_parity import bg_struct, camera

pytestmark = pytest.mark.gpu


def test_release_cache_while_rendering_alternating_scenes(L, O):
    w, h = 48, 27
    st = camera(L, RICH_SETUP, w, h)
    scenes = [O.rich_scene(2), O.rich_scene(3)]
    p = L.make_params(w, h, 20, 4, 0.5, 5)
    refs = [L.render(s, bg_struct(L, DEFAULT_BG), st, p, 0)[0] for s in scenes]
    stop = threading.Event()
    errors, frames = [], []

    def renderer():
        try:
            for i in range(40):
                rgb, _ = L.render(scenes[i % 2], bg_struct(L, DEFAULT_BG), st, p, 0)
                frames.append((i % 2, rgb))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(e)
        finally:
            stop.set()

    def releaser():
        try:
            n = 0
            while not stop.is_set():
                L.release_cache(0 if n % 2 else -1)
                n += 1
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=renderer), threading.Thread(target=releaser)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not any(t.is_alive() for t in threads), "deadlock: a thread did not finish"
    assert not errors, errors
    assert len(frames) == 40
    for k, rgb in frames:
        assert np.array_equal(rgb, refs[k])
