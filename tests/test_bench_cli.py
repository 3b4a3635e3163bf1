"""bench.py --gpus N on the CPU: N means N GPUs or an error, never a silent 1-GPU line.

  * WORLD_SIZE unset, N > 1: bench.py drives the N GPUs from this one process through the library's
    own multi-GPU group (srt_comm_init_all + pipelined srt_render_group; no torch, no launcher), after
    checking that N GPUs are visible (counted from the KFD topology, without initialising HIP);
  * under a launcher (one process per GPU): WORLD_SIZE must equal N;
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
    assert bench.launch_plan(8, {}, 8, ["--gpus", "8", "--steps", "5"]) == bench.GROUP


def test_visible_gpus_honours_visibility_lists(bench, monkeypatch):
    n = bench.visible_gpus()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert bench.visible_gpus() == min(n, 2)


def test_gpus_2_with_mocked_count_runs_the_group_in_process(bench, monkeypatch, capsys):
    """With 2 GPUs 'visible' (mocked) and no launcher, main() runs the in-process group plan with N = 2
    and prints its line; nothing goes through torch.distributed.run or a second process."""
    monkeypatch.setattr(bench, "visible_gpus", lambda: 2)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    seen = {}

    def fake_group(args, gpus):
        seen["gpus"] = gpus
        seen["steps"] = args.steps
        return {"metric": "m", "n_gpus": gpus, "nranks": gpus}

    def no_subprocess(*a, **kw):
        raise AssertionError("no child process expected: %r" % (a,))

    monkeypatch.setattr(bench, "run_group", fake_group)
    monkeypatch.setattr(bench.subprocess, "run", no_subprocess)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3", "--warmup", "0", "--no-cpu-baseline"])
    bench.main()
    assert seen == {"gpus": 2, "steps": 3}
    lines = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert lines == [{"metric": "m", "n_gpus": 2, "nranks": 2}]


def test_gpus_2_group_without_gpus_fails_without_a_line(tmp_path):
    """The in-process group plan with 2 GPUs 'visible' (HIP sees none here): srt_comm_init_all fails,
    the run fails, and no JSON line (in particular no 1-GPU line) is printed."""
    code = ("import sys; sys.argv = ['bench.py', '--gpus', '2', '--steps', '1', '--warmup', '0', '--no-cpu-baseline'];"
            "sys.path.insert(0, %r); import bench; bench.visible_gpus = lambda: 2; bench.main()" % str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(), cwd=str(tmp_path),
                       timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_hw_queues_range_checked_and_exported(bench, monkeypatch, capsys):
    """--hw-queues is set in the environment before HIP initialises (the boxes export 4) and is
    range-checked (1..32)."""
    monkeypatch.setattr(bench, "visible_gpus", lambda: 2)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--hw-queues", "40"])
    with pytest.raises(SystemExit, match="hw-queues"):
        bench.main()
    seen = {}
    monkeypatch.setattr(bench, "run_group", lambda args, gpus: seen.setdefault("q", os.environ["GPU_MAX_HW_QUEUES"]) and {})
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    bench.main()
    assert seen == {"q": "7"}
