"""Headline benchmark: Mrays/s (primary + secondary) on example1 at 1920x1080, depth 5, 6 spp
(BASELINE.json configs[1]) through the C ABI of libsightpy_hip.so.

One step = one full frame: every spp sample traced through every depth, plus the sRGB resolve, with
the scene, camera tables and the sample jitter already resident in HBM (the jitter is the
reference's numpy stream for seed 0, uploaded once before timing).  With N GPUs
(torch.distributed, one process per GPU) the frame's rows are dealt round-robin in 8-row bands,
each rank renders its shard and the uint8 tiles are gathered to rank 0 over RCCL; the frame is
fixed, so scaling is strong.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config example1_1080p_d5]
"""
import os

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")  # the CPU baseline is a single-core number
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
for p in (ROOT / "python-raytracer_amd", ROOT / "tests", ROOT / "oracle"):
    sys.path.insert(0, str(p))

BYTES_PER_RAY = 280  # algorithmic bytes per ray segment of the fp64 wavefront
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (builder, width, height, depth, spp, label)
    "example1_1080p_d5": ("example1", 1920, 1080, 5, 6, "example1.py (spheres+plane) 1920x1080 depth 5, 6 spp"),
    "example3_1080p_d8": ("example3", 1920, 1080, 8, 4, "example3.py (glass cuboid) 1920x1080 depth 8, 4 spp"),
    "example4_4k_d6": ("example4", 3840, 2160, 6, 10, "example4.py (thin film) 3840x2160 depth 6, 10 spp"),
    "cornell_800_s512": ("cornell", 800, 800, None, 512, "example_cornellbox.py 800x800, 512 spp (MC)"),
    "example1_400x300_d3": ("example1", 400, 300, None, 6, "example1.py 400x300 depth 3, 6 spp"),
    "mesh_1080p_d3": ("mesh_bench", 1920, 1080, 3, 2,
                      "TriangleMesh (20480-triangle icosphere, BVH) + sphere + floor + sky 1920x1080 depth 3, 2 spp"),
}


def cpu_baseline(builder, W, H, depth, spp, budget_s=20.0):
    """Oracle (numpy port of the reference algorithm) timed on this host's CPU, one process, on the
    same frame: samples are traced one after another until the frame is done or `budget_s` of CPU
    time is spent (the sample count is reported)."""
    import sightpy_oracle as O
    import scenes

    sc = getattr(scenes, builder)(W, H, depth)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(spp)
    counts = {}
    done = 0
    t0 = time.perf_counter()
    for s in range(spp):
        Oo, Do = O.primary_rays(sc.camera, jit[s])
        O.raycolor(sc, O.Rays(np.ascontiguousarray(np.broadcast_to(Oo, Do.shape)), Do, O.scene_medium(sc), 0), counts)
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    rays = sum(counts["depth"].values())
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": "oracle/sightpy_oracle.py (numpy restatement of the reference), 1 process, "
                      "OPENBLAS_NUM_THREADS=1: %d of %d samples of the same %dx%d frame (%d rays, %.1f s)"
                      % (done, spp, W, H, rays, dt),
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count()}


def pmc_traffic(config, kernel="k_primary"):
    """HBM bytes per k_primary launch from the newest committed PMC summary of this config
    (profiles/rNN_traffic_<config>.json, written by tools/pmc_traffic.py from two separate
    rocprofv3 --pmc passes of this same bench command), or None."""
    files = sorted(ROOT.glob("profiles/r*_traffic_%s.json" % config))
    if not files:
        return None, None
    rec = json.loads(files[-1].read_text())
    for name, k in rec["kernels"].items():
        if kernel in name and "traffic_bytes" in k:
            return k["traffic_bytes"] / 1e9, files[-1].name
    return None, None


def _cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if "Model name" in line:
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="example1_1080p_d5", choices=sorted(CONFIGS))
    ap.add_argument("--rng", default="numpy", choices=["numpy", "device", "mt"],
                    help="numpy: reference jitter stream resident in HBM; mt: the same stream generated on "
                         "the GPU inside every step (srt_mt19937_uniforms); device: Philox raygen")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--occupancy", type=int, default=0, help="experiment: kernel variant with this waves/SIMD bound")
    ap.add_argument("--option", action="append", default=[],
                    help="experiment: srt_set_option KEY=VALUE before rendering (repeatable)")
    ap.add_argument("--sync", action="store_true",
                    help="one frame at a time (host waits for each frame) instead of pipelined frames")
    ap.add_argument("--size", default=None, help="diagnostic: WxH override of the config's frame size")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic (1 GPU): render only rank 0's rows of an N-rank job, to size the per-rank work "
                         "of the multi-GPU run without the gather")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="diagnostic (1 GPU, with --shard-of N): run the N-rank step as one rank would, including "
                         "the per-frame RCCL all-gather call (a 1-rank group) and row assembly, to size the host "
                         "and stream overhead of the multi-GPU step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on a box with fewer GPUs (never used by the driver):
    # SIGHTPY_BENCH_DEVICE=k puts every rank on GPU k, SIGHTPY_BENCH_BACKEND=gloo gathers on the host
    dev = int(os.environ.get("SIGHTPY_BENCH_DEVICE", local))
    backend = os.environ.get("SIGHTPY_BENCH_BACKEND", "nccl")
    os.environ.setdefault("SIGHTPY_DEVICE", str(dev))
    dist = None
    if args.rehearse_gather and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.rehearse_gather:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(dev)
        dist.init_process_group(backend)

    import scenes
    from sightpy import _backend as B, _native as N
    from sightpy._shard import shard_rows, max_shard_rows, RowGather

    builder, W, H, depth, spp, label = CONFIGS[args.config]
    if args.spp:
        spp = args.spp
    if args.size:
        W, H = (int(v) for v in args.size.lower().split("x"))
    sc = getattr(scenes, builder)(W, H, depth)
    lib, ctx = B.context()
    if args.occupancy:
        N.check(lib, lib.srt_set_option(ctx, b"occupancy", args.occupancy))
    if not args.sync:
        # size every frame slot during the warmup (the first pipelined frame would allocate them)
        N.check(lib, lib.srt_set_option(ctx, b"pipeline", 1))
    for kv in args.option:
        k, v = kv.split("=")
        N.check(lib, lib.srt_set_option(ctx, k.encode(), int(v)))
    B.upload(sc)
    rows = shard_rows(H, world, rank) if world > 1 else np.arange(H)
    if args.shard_of > 1 and world == 1:
        rows = shard_rows(H, args.shard_of, 0)
    npix = len(rows) * W
    # resident inputs: jitter (reference stream, seed 0) in HBM
    jit_dev = None
    np.random.seed(0)
    mt_state = np.random.get_state()
    mt_key = np.ascontiguousarray(mt_state[1], dtype=np.uint32)
    mt_key_out = np.empty(624, dtype=np.uint32)
    mt_pos_out = ctypes.c_int32(0)
    if args.rng == "mt" and world > 1:
        raise SystemExit("--rng mt renders the full frame's stream; use it with --gpus 1")
    if args.rng == "mt":
        p = ctypes.c_void_p()
        N.check(lib, lib.srt_device_alloc(ctx, spp * 4 * npix * 8, ctypes.byref(p)))
        jit_dev = p
    if args.rng == "numpy":
        np.random.seed(0)
        jit = np.random.rand(spp * 4 * H * W).reshape(spp, 4, H, W)[:, :, rows].reshape(spp, 4, npix)
        jit = np.ascontiguousarray(jit)
        p = ctypes.c_void_p()
        N.check(lib, lib.srt_device_alloc(ctx, jit.nbytes, ctypes.byref(p)))
        N.check(lib, lib.srt_memcpy(ctx, p, N.ptr(jit), jit.nbytes))
        jit_dev = p
        del jit
    out_u8 = ctypes.c_void_p()
    out_rgb = ctypes.c_void_p()
    N.check(lib, lib.srt_device_alloc(ctx, 3 * npix, ctypes.byref(out_u8)))
    N.check(lib, lib.srt_device_alloc(ctx, 3 * npix * 8, ctypes.byref(out_rgb)))
    cd = B.camera_desc(sc.camera)
    rows32 = np.ascontiguousarray(rows, dtype=np.int32)
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, len(rows), 0
    a.rows = N.ptr(rows32)
    a.jitter = jit_dev
    a.seed = 12345
    a.out_rgb, a.out_srgb8, a.out_hit_id = out_rgb, out_u8, None

    # Frames are pipelined: each step queues its frame on the library's stream (SRT_RENDER_ASYNC)
    # and returns, so the host prepares frame k+1 while the GPU renders frame k; srt_render_finish
    # at the end checks every frame's error flags.  With N ranks the frame's uint8 tile (written in
    # place by k_resolve, double-buffered) is all-gathered over RCCL on torch's stream after the
    # frame, overlapping the next frame's rendering.
    pipelined = not args.sync and args.rng != "mt"
    NTILE = int(os.environ.get("SIGHTPY_BENCH_NTILE", "5"))  # uint8 tiles in flight (gather ring)
    tiles, done = None, [None] * NTILE
    if dist is not None:
        import torch

        # each rank's uint8 tile, padded to the largest shard: the send buffer of the all-gather
        tiles = [torch.zeros((max_shard_rows(H, world), W, 3), dtype=torch.uint8, device="cuda") for _ in range(NTILE)]
        gather = RowGather(H, world, (W, 3), torch.uint8, "cuda" if backend == "nccl" else "cpu")
        if world == 1:  # --rehearse-gather: rank 0's tile of an N-rank job through a 1-rank group
            tiles = [torch.zeros((len(rows), W, 3), dtype=torch.uint8, device="cuda") for _ in range(NTILE)]
            gather = RowGather(len(rows), 1, (W, 3), torch.uint8, "cuda" if backend == "nccl" else "cpu")
    streams = {}

    def frame_stream():
        """torch handle of the stream the library queued its last frame on (pipelined frames
        alternate between two streams)."""
        import torch

        sp = ctypes.c_void_p()
        N.check(lib, lib.srt_stream(ctx, ctypes.byref(sp)))
        if sp.value not in streams:
            streams[sp.value] = torch.cuda.ExternalStream(sp.value, device=torch.device("cuda", dev))
        return streams[sp.value]

    frame = {"k": 0}

    def step(st, async_ok=True):
        if args.rng == "mt":
            # the reference's stream (seed 0): spp x 4 x npix jitter + the sizing draw, on the GPU
            N.check(lib, lib.srt_mt19937_uniforms(ctx, N.ptr(mt_key), int(mt_state[2]), spp * 4 * npix, 4 * npix,
                                                  jit_dev, N.ptr(mt_key_out), ctypes.byref(mt_pos_out)))
        i = frame["k"] % NTILE
        frame["k"] += 1
        a.flags = N.RENDER_ASYNC if (pipelined and async_ok) else 0
        if tiles is not None:
            if done[i] is not None:
                # the gather that read this tile NTILE frames ago must be done before this frame's
                # resolve overwrites it (a host wait: by now it has long finished)
                done[i].synchronize()
            a.out_srgb8 = ctypes.c_void_p(tiles[i].data_ptr())
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), ctypes.byref(st)))
        if tiles is not None:
            import torch

            cur = torch.cuda.current_stream()
            cur.wait_stream(frame_stream())  # this frame's tile is complete
            if backend == "nccl":
                frame["image"] = gather(tiles[i])
            else:
                cur.synchronize()
                frame["image"] = gather(tiles[i].cpu())
            ev = torch.cuda.Event()
            ev.record(cur)
            done[i] = ev

    st = N.Stats()
    for w in range(args.warmup):
        step(st, async_ok=w > 0)  # the first frame runs synchronously (sizes the queues)

    def barrier():
        if dist is not None:
            dist.barrier()
            import torch
            torch.cuda.synchronize()
        N.check(lib, lib.srt_synchronize(ctx))

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(st)
    barrier()
    elapsed = time.perf_counter() - t0
    N.check(lib, lib.srt_render_finish(ctx, ctypes.byref(st)))  # error flags of every pipelined frame
    # kernel durations (HIP events on the library's stream) of the same frame, rendered one at a
    # time so that every frame's events can be read: the roofline's per-launch times
    stats = []
    for _ in range(max(1, min(args.steps, 10))):
        s = N.Stats()
        step(s, async_ok=False)
        stats.append(s.as_dict())
    barrier()
    if dist is not None:
        import torch

        cdev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        rays_local = torch.tensor([stats[0]["total_rays"]], dtype=torch.float64, device=cdev)
        dist.all_reduce(rays_local)
        total_rays = float(rays_local.item())
    else:
        total_rays = float(stats[0]["total_rays"])

    ms_step = elapsed / args.steps * 1e3
    value = total_rays * args.steps / elapsed / 1e6
    # roofline of the dominant kernel (depth-0 trace = raygen + trace; HIP events on its stream)
    prim_ms = np.mean([s["ms_primary_kernel"] for s in stats])
    trace_ms = np.mean([s["ms_trace_kernels"] for s in stats])
    rpd = stats[0]["rays_per_depth"]
    frame_path = stats[0]["kernel_path"] == "frame"
    # the dominant kernel: k_primary (depth 0) on the wavefront path; k_frame (every ray of the
    # pass) on the frame-kernel path used for branching scenes
    prim_rays = stats[0]["total_rays"] if frame_path else rpd[0]
    achieved = prim_rays * BYTES_PER_RAY / (prim_ms * 1e-3) / 1e9
    family = stats[0]["total_rays"] * BYTES_PER_RAY / (trace_ms * 1e-3) / 1e9
    # (PMC summaries are per launch of the full configuration: none for diagnostic shapes)
    traffic_gb, traffic_src = (None, None) if (args.shard_of or args.size or args.spp) else \
        pmc_traffic(args.config, "k_frame" if frame_path else "k_primary")
    if rank == 0:
        rec = {
            "metric": "Mrays/sec (primary+secondary) at 1920x1080 depth 5" if args.config == "example1_1080p_d5"
            else "Mrays/sec (primary+secondary)",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: %s; jitter = reference numpy stream seed 0 (%s)" % (label, args.rng),
            "config": {"workload": label, "width": W, "height": H, "max_ray_depth": depth, "spp": spp,
                       "rays_per_frame": int(total_rays), "rays_per_depth_rank0": rpd,
                       "shadow_rays_rank0": stats[0]["shadow_rays"], "kernel_path": stats[0]["kernel_path"],
                       "chain_from_depth": stats[0]["chain_from"], "parallelism": ("row-band shards x%d" % world) if not args.shard_of
                       else "diagnostic: rank 0 of %d row-band shards, %s" % (
                           args.shard_of, "1-rank RCCL all-gather + assembly per frame" if args.rehearse_gather
                           else "no gather"),
                       "frame_ms": round(ms_step, 4)},
            "roofline": {"bound": "hbm",
                         "kernel": "k_frame (whole pass: every ray of every depth, one wave per 64-pixel tile)"
                         if frame_path else "k_primary (depth 0: raygen + nearest hit + shading, fused)",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic_gb is None else round(traffic_gb, 4),
                         "traffic_unit": "GB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "algorithmic_GB_per_launch": round(prim_rays * BYTES_PER_RAY / 1e9, 4),
                         "bytes_per_ray": BYTES_PER_RAY, "kernel_ms": round(float(prim_ms), 4),
                         "all_trace_kernels": {"ms": round(float(trace_ms), 4), "achieved_GBs": round(family, 2),
                                               "frac": round(family / HBM_PEAK_GBS, 4)}},
        }
        if not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(builder, W, H, depth, spp)
        print(json.dumps(rec))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    lib.srt_device_free(ctx, out_u8)
    lib.srt_device_free(ctx, out_rgb)
    if jit_dev is not None:
        lib.srt_device_free(ctx, jit_dev)


if __name__ == "__main__":
    main()
