"""bench.py's multi-GPU launch (CPU only): --gpus N starts N ranks itself, a launcher's
WORLD_SIZE must match --gpus, and at N > 1 every rank builds BASELINE config 4's shard
(50M x 16 B, m = 5e8, k = 10, seed 0x5EED0040 + rank; compactors/sized.rs:170-200)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_launch_plan():
    import bench
    assert bench.launch_plan(None, {}) == ("run", 1)
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(None, {"WORLD_SIZE": "8"}) == ("run", 8)
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == ("run", 8)
    with pytest.raises(ValueError):
        bench.launch_plan(2, {"WORLD_SIZE": "4"})  # the driver's N must be the N measured
    with pytest.raises(ValueError):
        bench.launch_plan(0, {})


def test_spawn_command():
    import bench
    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5] == os.path.join(ROOT, "bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def _plan(args, env=None):
    e = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(v, None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan-only"] + args, env=e,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_two_rank_spawn_gets_config4_shards():
    """`python bench.py --gpus 2` with no launcher: two ranks, one process group, config 4."""
    r = _plan(["--gpus", "2"])
    assert r["world_size"] == 2 and r["n_gpus"] == 2
    assert [x["rank"] for x in r["ranks"]] == [0, 1]
    assert {x["local_rank"] for x in r["ranks"]} == {0, 1}
    for x in r["ranks"]:
        assert (x["config"], x["keys"], x["m"], x["k"]) == (4, 50_000_000, 500_000_000, 10)
        assert x["seed"] == 0x5EED0040 + x["rank"]


def test_eight_rank_spawn_gets_config4_shards():
    """The driver's 8-GPU scaling run, rehearsed on CPU: `bench.py --gpus 8` with no launcher
    starts 8 ranks in one process group, each on its own local rank, rank r on config 4's shard r
    (seed 0x5EED0040 + r) -- one merged table's filter per GPU (compactors/sized.rs:170-200)."""
    r = _plan(["--gpus", "8"])
    assert r["world_size"] == 8 and r["n_gpus"] == 8
    assert [x["rank"] for x in r["ranks"]] == list(range(8))
    assert sorted(x["local_rank"] for x in r["ranks"]) == list(range(8))
    for x in r["ranks"]:
        assert (x["config"], x["keys"], x["m"], x["k"]) == (4, 50_000_000, 500_000_000, 10)
        assert x["seed"] == 0x5EED0040 + x["rank"]
    assert len({x["seed"] for x in r["ranks"]}) == 8


def test_one_gpu_default_is_config2():
    r = _plan([])
    assert r["world_size"] == 1
    assert [(x["config"], x["keys"], x["m"], x["k"], x["seed"]) for x in r["ranks"]] == \
        [(2, 100_000_000, 1_000_000_000, 10, 0x5EED0001)]


def test_mismatched_launcher_world_fails():
    e = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan-only", "--gpus", "2"], env=e,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=3" in out.stderr
