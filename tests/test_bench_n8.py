"""Pre-flight of the driver's 8-GPU run on the CPU: `bench.py --gpus 8 --steps K --warmup W`, both ways
the driver may start it, against tests/fake_srt.py (the C ABI restated in Python, checking every
call) instead of libsightpy_hip.so:

  * one process per GPU, as `torch.distributed.run --nproc-per-node 8` starts it: 8 processes with
    WORLD_SIZE / RANK / LOCAL_RANK / MASTER_PORT, the RCCL id handed from rank 0 through the file
    bench.py writes, the linear RGB in POSIX shared memory registered by every rank, max-over-ranks
    timing through srt_comm_allreduce, one JSON line from rank 0;
  * no launcher: one process drives the 8 GPUs through the library's own group (run_group:
    srt_comm_init_all + pipelined srt_render_group).

What is checked is the plumbing of srt_render / srt_render_group at N = 8 (flags, which rank passes
which output, the shared frame's registration, the row bands each rank writes: exactly the frame's
rows, once), not the GPU work.  The RCCL exchange itself has not run with more than one rank (the
round's GPU lease is one GPU)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HERE = Path(__file__).resolve().parent

_BOOT = r"""
import os, sys
sys.path[:0] = [%(root)r, %(tests)r, %(pkg)r]
import bench, fake_srt
from sightpy import _backend as B
world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
B._STATE["lib"] = fake_srt.FakeSrt(%(W)d, %(H)d, %(spp)d, world, rank, %(sync)r)
sys.argv = ["bench.py"] + %(argv)r
bench.main()
"""


def _boot(tmp, W, H, spp, argv):
    return _BOOT % {"root": str(ROOT), "tests": str(HERE), "pkg": str(ROOT / "python-raytracer_amd"), "W": W,
                    "H": H, "spp": spp, "sync": str(tmp), "argv": argv}


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    env["OMP_NUM_THREADS"] = "1"
    env["OPENBLAS_NUM_THREADS"] = "1"
    return env


@pytest.mark.parametrize("extra", [[], ["--rgb-to-host"]])
def test_bench_gpus_8_one_process_per_rank(tmp_path, extra):
    """The driver's N = 8 command under a launcher (8 ranks): every rank's srt_render gets SHARDED frames
    of the whole height, rank 0 alone a (pinned) uint8 output, the RGB rows go into the registered
    shared frame and tile it exactly; the JSON line comes from rank 0 alone, n_gpus = nranks = 8,
    value = the 8 ranks' rays / the slowest rank's time."""
    W, H, spp, world = 96, 64, 2, 8
    argv = ["--gpus", "8", "--steps", "4", "--warmup", "2", "--config", "example1_1080p_d5", "--size", "%dx%d" % (W, H),
            "--spp", str(spp)] + extra
    port = str(20000 + os.getpid() % 20000)
    procs = []
    for r in range(world):
        env = _env(WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-c", _boot(tmp_path, W, H, spp, argv)], env=env,
                                      cwd=str(tmp_path), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=300)
            outs.append((p.returncode, out, err))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (rc, out, err) in enumerate(outs):
        assert rc == 0, "rank %d rc %d:\n%s" % (r, rc, err[-3000:])
    lines = [[json.loads(ln) for ln in out.splitlines() if ln.startswith("{")] for _, out, _ in outs]
    assert [len(x) for x in lines] == [1] + [0] * (world - 1)
    rec = lines[0][0]
    assert rec["n_gpus"] == world and rec["nranks"] == world and rec["steps"] == 4 and rec["warmup"] == 2
    from sightpy._shard import shard_kmax, shard_rows

    kmax = shard_kmax(H, world, 0, 1)
    rays = sum(len(shard_rows(H, world, q, kmax)) * W * spp * (1 + 1 / 2 + 1 / 8) for q in range(world))
    assert rec["config"]["rays_per_frame"] == int(rays)
    assert abs(rec["value"] - rec["config"]["rays_per_frame"] / rec["ms_per_step"] / 1e3) <= 1e-3 * rec["value"] + 1e-3
    assert "cpu_baseline" not in rec  # (rank 0 at N = 1 only)
    logs = [json.load(open(tmp_path / ("fake_rank%d.json" % r))) for r in range(world)]
    assert all("errors" not in g for g in logs), [g.get("errors") for g in logs]
    frames = {g["frames"] for g in logs}
    assert len(frames) == 1  # every rank rendered the same number of frames (the gathers pair up)
    rgb_checks = [c for c in logs[0]["checks"] if c["frame"] == "rgb_rows"]
    assert rgb_checks and all(c["tiled_exactly"] for c in rgb_checks)
    assert all(g.get("lane_frames") == 2 for g in logs)


def test_bench_gpus_8_in_process_group(tmp_path, monkeypatch, capsys):
    """The driver's N = 8 command without a launcher: run_group drives the 8 'GPUs' (mocked count)
    through srt_comm_init_all and srt_render_group; the RGB_ROWS frames' host buffer is the pinned
    whole frame, tiled exactly by the 8 contexts' row bands."""
    sys.path[:0] = [str(ROOT), str(HERE)]
    try:
        import bench
        import fake_srt
        from sightpy import _backend as B

        W, H, spp = 96, 64, 2
        fake = fake_srt.FakeSrt(W, H, spp, 8, 0, str(tmp_path), group=True)
        monkeypatch.setitem(B._STATE, "lib", fake)
        monkeypatch.setattr(bench, "visible_gpus", lambda: 8)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            monkeypatch.delenv(k, raising=False)
        monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "4", "--warmup", "2", "--size",
                                          "%dx%d" % (W, H), "--spp", str(spp)])
        bench.main()
    finally:
        sys.path.remove(str(ROOT))
        sys.path.remove(str(HERE))
    lines = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["n_gpus"] == 8 and rec["nranks"] == 8
    assert "errors" not in fake.log, fake.log.get("errors")
    # warm-up 2 + timed 4 + the host_rgb figure's 4 + 3 latency frames
    assert len(fake.frames) == 2 + 4 + 4 + 3
    rgb_checks = [c for c in fake.log["checks"] if c["frame"] == "rgb_rows"]
    assert len(rgb_checks) == 3 and all(c["tiled_exactly"] for c in rgb_checks)


def test_bench_gpus_8_line_survives_a_failed_secondary_figure(tmp_path):
    """A library error in the secondary frames of the N = 8 run (here every rank's SRT_RENDER_RGB_ROWS
    frame fails, injected in the stand-in) costs the secondary figures, not the line: rank 0 still
    prints its one JSON line, with the timed value and the error in `secondary_error`, and every rank
    exits cleanly (the ranks take the same branch, no collective is left waiting)."""
    W, H, spp, world = 96, 64, 2, 8
    argv = ["--gpus", "8", "--steps", "4", "--warmup", "2", "--config", "example1_1080p_d5", "--size", "%dx%d" % (W, H),
            "--spp", str(spp)]
    port = str(20000 + (os.getpid() + 7919) % 20000)
    procs = []
    for r in range(world):
        env = _env(WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   FAKE_SRT_FAIL_RGB_ROWS="1")
        procs.append(subprocess.Popen([sys.executable, "-c", _boot(tmp_path, W, H, spp, argv)], env=env,
                                      cwd=str(tmp_path), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=300)
            outs.append((p.returncode, out, err))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (rc, out, err) in enumerate(outs):
        assert rc == 0, "rank %d rc %d:\n%s" % (r, rc, err[-3000:])
    lines = [[json.loads(ln) for ln in out.splitlines() if ln.startswith("{")] for _, out, _ in outs]
    assert [len(x) for x in lines] == [1] + [0] * (world - 1)
    rec = lines[0][0]
    assert rec["n_gpus"] == world and rec["value"] > 0
    assert "injected" in rec["secondary_error"] and "host_rgb" not in rec
