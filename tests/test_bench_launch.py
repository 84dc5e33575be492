"""bench.py --gpus N (the driver's contract): without a launcher bench.py starts N rank processes
itself, under one it refuses a WORLD_SIZE that disagrees with --gpus; it never runs fewer ranks than
asked. CPU only: --launch-check meets the ranks over gloo and exits before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launch_plan_cases():
    assert bench.launch_plan(1, {}, []) == ("run", None)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, []) == ("run", None)
    how, why = bench.launch_plan(8, {"WORLD_SIZE": "1"}, [])
    assert how == "refuse" and "WORLD_SIZE=1" in why
    assert bench.launch_plan(0, {}, [])[0] == "refuse"
    how, cmd = bench.launch_plan(2, {}, ["--gpus", "2", "--dist-backend", "gloo"])
    assert how == "spawn"
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--dist-backend", "gloo"]


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--dist-backend", "gloo", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout  # rank 0 alone prints
    got = json.loads(line[0])
    rep = got.pop("dist")
    fields = got.pop("group_fields")
    assert got == {"launch_check": True, "gpus": n, "world_size": n, "ranks_met": n}
    # every rank's own report of the world size, as the bench line's `dist` field carries it
    assert rep["all_ranks_saw_world"] and rep["backend"] == "gloo"
    assert [r["rank"] for r in rep["ranks"]] == list(range(n)) and all(r["world_size"] == n for r in rep["ranks"])
    # the device-group leg's line names the devices it spanned and their peer access
    assert {"n_devices", "devices", "peer_access"} <= set(fields)


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
    assert not r.stdout.strip()
