"""bench.py's own N-rank launcher (`--gpus N` with no WORLD_SIZE): the rank
environments, the child-process supervision and the refusal paths, on CPU.

The reference's parallelism lives inside one Render call (NumWorkers
goroutines, ray/tracer.go:86-116); bench.py's N-GPU line must come out of
`python bench.py --gpus N` alone, one process per GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_envs_match_torchrun_single_node():
    envs = bench.rank_envs(4, 29555, base={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"  # inherited
        assert e["TRAY_BENCH_LAUNCHER"] == "bench.py"


def test_free_port_is_bindable():
    import socket

    p = bench.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


def _script(tmp_path, body):
    path = tmp_path / "rank.py"
    path.write_text("import os, sys, time\n" + body)
    return str(path)


def test_launch_ranks_runs_every_rank(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    script = _script(tmp_path, f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write("
                               "os.environ['WORLD_SIZE'] + ' ' + os.environ['MASTER_PORT'] + ' ' + ' '.join(sys.argv[1:]))\n")
    assert bench.launch_ranks(3, ["--steps", "7"], timeout=60, script=script) == 0
    got = sorted(os.listdir(out))
    assert got == ["0", "1", "2"]
    lines = {(out / r).read_text() for r in got}
    assert len(lines) == 1  # one port, one world, the same arguments for every rank
    world, port, *argv = lines.pop().split()
    assert world == "3" and int(port) > 0 and argv == ["--steps", "7"]


def test_launch_ranks_fails_and_stops_the_others(tmp_path):
    # rank 1 fails at once; rank 0 would sleep for a minute (a rank stuck in a collective)
    script = _script(tmp_path, "if os.environ['RANK'] == '1': sys.exit(5)\ntime.sleep(60)\n")
    t0 = __import__("time").monotonic()
    assert bench.launch_ranks(2, [], timeout=120, script=script) == 5
    assert __import__("time").monotonic() - t0 < 30


def test_launch_ranks_timeout(tmp_path):
    script = _script(tmp_path, "time.sleep(60)\n")
    assert bench.launch_ranks(2, [], timeout=1.0, script=script) == 124


def test_cpu_share_states_its_reason():
    cores, why = bench.cpu_share()
    assert 1 <= cores <= (os.cpu_count() or 1)
    assert "nproc=" in why


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU refusal")
def test_self_launch_without_gpus_fails_loudly():
    """`bench.py --gpus 2` with no launcher starts two ranks; without GPUs each
    refuses (RCCL needs one device per rank) and the parent exits non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TRAY_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rank-timeout", "240"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line from a failed job


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_profile_records_only_for_the_loaded_device_code(tmp_path):
    """bench.py copies PMC figures (traffic, VALU issue / lane utilisation) into
    its roofline record only when the profile was measured on the device code
    the process loaded: a record with another code-object hash, none, or
    another launch shape yields null with the reason."""
    import json

    import bench
    from tray_amd import _lib

    h = _lib.code_object_sha256()
    assert h and len(h) == 64
    rec = {"frames_per_launch": 16, "hbm_bytes_per_launch": 123, "code_object_sha256": h}
    (tmp_path / "pmc_c2.json").write_text(json.dumps(rec))
    got, src, why = bench._profile_json("pmc", "c2", 16, h, profiles_dir=str(tmp_path))
    assert got == rec and why is None
    got, src, why = bench._profile_json("pmc", "c2", 16, "0" * 64, profiles_dir=str(tmp_path))
    assert got is None and src is None and "device code" in why
    got, _, why = bench._profile_json("pmc", "c2", 8, h, profiles_dir=str(tmp_path))
    assert got is None and "frames per launch" in why
    (tmp_path / "pmc_c2.json").write_text(json.dumps({"frames_per_launch": 16, "hbm_bytes_per_launch": 1}))
    got, _, why = bench._profile_json("pmc", "c2", 16, h, profiles_dir=str(tmp_path))
    assert got is None and "None" in why  # records from before the hash existed are not trusted
    got, _, why = bench._profile_json("pmc_mix", "c9", 16, h, profiles_dir=str(tmp_path))
    assert got is None and "no pmc_mix_c9.json" in why


def test_rank_stuck_in_a_collective_is_stopped_and_named(tmp_path, capsys):
    """Rank 1 sleeps past the limit while rank 0 waits for it in a gloo barrier (a
    rank stuck in the gather): the launcher stops both within the limit, exits
    non-zero and names the ranks it stopped."""
    import time

    script = _script(tmp_path, "import torch.distributed as dist\n"
                               "dist.init_process_group('gloo')\n"
                               "if os.environ['RANK'] == '1': time.sleep(120)\n"
                               "dist.barrier()\n")
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, [], timeout=20.0, script=script)
    took = time.monotonic() - t0
    assert rc == 124 and took < 40
    err = capsys.readouterr().err
    assert "rank(s) [0, 1] still running after 20.0 s" in err


def test_rank_timeout_has_a_finite_default():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0
    import re

    m = re.search(r"--rank-timeout RANK_TIMEOUT", r.stdout)
    assert m
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'ap.add_argument("--rank-timeout", type=float, default=900.0' in src


def test_frame_parity_record():
    """bench.frame_parity (the `parity` field of the bench line) on synthetic frames."""
    import numpy as np

    rng = np.random.default_rng(1)
    ref = rng.random((4, 5, 3))
    seg = rng.integers(64, 200, (4, 5)).astype(np.uint32)
    rec = bench.frame_parity(ref, seg, ref.copy(), seg.copy(), ref.astype(np.float32))
    assert rec["ok"] and rec["linf"] == 0.0 and rec["pixels"] == 20 and rec["segments_equal"]
    assert rec["f32_within_one_rounding"] and rec["f32_equal_frac"] == 1.0
    bad = ref.copy()
    bad[1, 2, 0] += 2e-4
    seg2 = seg.copy()
    seg2[0, 0] += 1
    rec = bench.frame_parity(ref, seg, bad, seg2, ref.astype(np.float32))
    assert not rec["ok"] and abs(rec["linf"] - 2e-4) < 1e-12 and rec["segments_differing"] == 1


def test_rank_watchdog_names_rank_and_phase():
    """Under any launcher (torchrun included) an N > 1 rank that is still running
    after --rank-timeout exits 124 and names itself and its phase (bench.py
    start_watchdog), so a collective that never completes fails the job."""
    import time

    code = ("import sys, time; sys.path.insert(0, %r); import bench; bench.start_watchdog(3, 1.0); "
            "bench.set_phase('timed frames'); time.sleep(60)" % ROOT)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 124 and time.monotonic() - t0 < 30
    assert "rank 3 still running after 1.0 s" in r.stderr and "'timed frames'" in r.stderr


def test_rank_watchdog_is_per_phase():
    """The watchdog bounds each phase, not the run: a rank whose phases
    each finish within the limit runs on past it in total and exits normally."""
    import time

    code = ("import sys, time; sys.path.insert(0, %r); import bench; bench.start_watchdog(4, 1.5)\n"
            "for k in range(4):\n    bench.set_phase('phase %%d' %% k); time.sleep(0.8)\n"
            "print('done')" % ROOT)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "done", r.stderr
    assert time.monotonic() - t0 > 3.0  # longer in total than the limit
