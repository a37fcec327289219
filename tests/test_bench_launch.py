"""CPU tests of bench.py's rank launcher: `--gpus N` either runs N ranks or fails loudly,
never a silent 1-GPU measurement.  PICO_BENCH_DRY=1 makes each rank
print its RANK / WORLD_SIZE and exit before any GPU call."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=300)


def test_gpus_mismatch_with_world_size_fails():
    r = _run(["--gpus", "8"], WORLD_SIZE="1", PICO_BENCH_DRY="1")
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_gpus_more_than_visible_fails():
    r = _run(["--gpus", "2"], PICO_BENCH_DRY="1", HIP_VISIBLE_DEVICES="")
    assert r.returncode != 0
    assert "HIP device" in r.stderr


def test_gpus_n_self_launches_n_ranks():
    # same-device rehearsal switch lets the launcher run without N visible GPUs; the dry
    # ranks report what they were given and exit before touching a device
    r = _run(["--gpus", "2", "--config", "c4"], PICO_BENCH_DRY="1", PICO_BENCH_SAME_DEVICE="1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus"] == 2 for x in lines)


def test_gpus_one_runs_in_process():
    r = _run(["--gpus", "1"], PICO_BENCH_DRY="1")
    assert r.returncode == 0
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line == {"rank": 0, "world": 1, "gpus": 1}
