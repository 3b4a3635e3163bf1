"""bench.py --gpus N on the CPU: N means N GPUs or an error, never a silent 1-GPU line.

  * WORLD_SIZE unset, N > 1: bench.py starts N ranks through torch.distributed.run as a child
    process (one process per GPU, nothing in the parent touches the GPU), after checking that N GPUs
    are visible (counted from the KFD topology, without initialising HIP);
  * under a launcher: WORLD_SIZE must equal N;
  * fewer GPUs than N, or a mismatch: rc != 0 and no JSON line.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture
def bench():
    sys.path.insert(0, str(ROOT))
    import bench as b

    yield b
    sys.path.remove(str(ROOT))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_2_without_gpus_refuses(tmp_path):
    # this container has no GPU: --gpus 2 must fail before rendering anything
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=_env(), cwd=str(tmp_path), timeout=120)
    assert r.returncode != 0
    assert "only 0 GPU(s) visible" in r.stderr + r.stdout
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_launch_plan(bench):
    # in-process: 1 GPU, or N ranks started by a launcher with WORLD_SIZE == N
    assert bench.launch_plan(1, {}, 0, []) is None
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, 0, []) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.launch_plan(4, {"WORLD_SIZE": "2"}, 8, [])
    with pytest.raises(SystemExit, match="only 3 GPU"):
        bench.launch_plan(4, {}, 3, [])
    cmd = bench.launch_plan(8, {}, 8, ["--gpus", "8", "--steps", "5"])
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and cmd[i + 1:i + 4] == ["--nnodes=1", "--nproc-per-node", "8"]
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")


def test_visible_gpus_honours_visibility_lists(bench, monkeypatch):
    n = bench.visible_gpus()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert bench.visible_gpus() == min(n, 2)


def test_gpus_2_with_mocked_count_launches_two_ranks(bench, monkeypatch, capsys):
    """With 2 GPUs 'visible' (mocked) the bench starts 2 ranks through torch.distributed.run; here the
    ranks find no GPU and fail, so the job fails -- it does not fall back to a 1-GPU line."""
    monkeypatch.setattr(bench, "visible_gpus", lambda: 2)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    seen = {}
    real_run = subprocess.run

    def spy(cmd, *a, **kw):
        seen["cmd"] = cmd
        kw.setdefault("capture_output", True)
        kw.setdefault("timeout", 240)
        r = real_run(cmd, *a, text=True, **kw)
        seen["out"] = r.stdout
        return r

    monkeypatch.setattr(bench.subprocess, "run", spy)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code != 0
    assert "--nproc-per-node" in seen["cmd"] and seen["cmd"][seen["cmd"].index("--nproc-per-node") + 1] == "2"
    lines = [json.loads(ln) for ln in seen["out"].splitlines() if ln.startswith("{")]
    assert not any(d.get("n_gpus") == 1 for d in lines)
