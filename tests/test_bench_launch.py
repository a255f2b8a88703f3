"""bench.py --gpus N launch contract (CPU, no GPU touched).

The driver runs `python3 bench.py --gpus N` without torchrun's env for its
1/2/4/8-GPU scaling curve (BASELINE configs[3]); bench.py must then start N
rank processes itself, before any GPU call, and refuse to run a world that
differs from N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _import_bench():
    sys.path.insert(0, ROOT)
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_plan_decisions():
    b = _import_bench()
    assert b.launch_plan(1, {}, [], 0) == ("run", None)
    assert b.launch_plan(4, {"WORLD_SIZE": "4"}, [], 0) == ("run", None)
    what, msg = b.launch_plan(8, {"WORLD_SIZE": "1"}, [], 8)
    assert what == "error" and "WORLD_SIZE=1" in msg
    what, msg = b.launch_plan(8, {}, [], 1)
    assert what == "error" and "1 GPU(s) visible" in msg
    what, cmd = b.launch_plan(4, {}, ["--gpus", "4", "--steps", "3"], 8)
    assert what == "launch"
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_yields_n_ranks(n):
    """No WORLD_SIZE in the env: bench.py starts n ranks (torch.distributed.run
    child), each sees RANK / LOCAL_RANK / WORLD_SIZE = n; --dry-run joins a
    gloo group instead of touching a GPU."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env=_env(),
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["ok"] and out["world_size"] == n and out["gpus"] == n
    assert sorted((x["rank"], x["local_rank"], x["world_size"]) for x in out["ranks"]) == \
        [(i, i, n) for i in range(n)]


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_more_gpus_than_visible_fails():
    """Here no GPU is visible: --gpus 2 must fail, not fall back to one
    process (the driver would read a 1-GPU number as the 2-GPU point)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], env=_env(),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
