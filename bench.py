"""Headline benchmark: Mrays/s (primary + secondary) and frame ms on example1 at 1920x1080, depth 5,
6 spp (BASELINE.json configs[1]) through the C ABI of libsightpy_hip.so.

One step = one SURVEY 8(d) frame, from render() entry (scene already uploaded) to the image in host
memory:
  * the camera jitter is the reference's numpy stream (np.random.seed(0) before the first frame,
    every frame continuing it, as consecutive Scene.render calls do), generated on the GPU inside the
    step (rt_mt.h; bit-equal to np.random.rand);
  * every sample traced through every depth, the sRGB resolve: the linear RGB (f64) computed and
    stored in HBM, the uint8 image copied to pinned host memory -- what Scene.render hands back (the
    reference's render returns the uint8 image only, scene.py:118-140; SRT_RENDER_RGB_LOCAL).
Frames are pipelined (each step queues its frame and returns; the timed region ends when all K
frames are in host memory).  With N GPUs the library splits each frame into row bands dealt
round-robin (SRT_RENDER_SHARDED), every rank draws the same stream and reads its rows, the uint8
tiles are gathered to rank 0 over RCCL (xGMI) and every rank keeps its rows of the linear RGB in its
HBM; the frame is fixed, so scaling is strong.  `--rgb-to-host` copies the linear RGB to pinned host
memory as well (rounds 1-4's step: 50 MB per 1080p frame over PCIe, every rank its own rows at
N > 1); the default line reports that form too (`host_rgb`).  Two launches, no
torch imported in either: one process per GPU (WORLD_SIZE set by a launcher such as the driver's
`torch.distributed.run`; the ranks meet through the library's srt_comm_init), or -- `--gpus N` with no
launcher -- this one process driving all N GPUs through the library's group (srt_comm_init_all +
pipelined srt_render_group).

Secondary figures in the same line: `host_rgb` (the same frames with the linear RGB copied to host
memory too), `frame_latency_ms` (one synchronous frame), `device_resident`
(jitter pre-resident in HBM and outputs left in HBM: the round-1 headline), the roofline of the
dominant kernel, and the CPU baseline (oracle: one core, and a multiprocessing.Pool over samples
structured like the reference's Scene.render).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config example1_1080p_d5] [--rng mt|device]
"""
import os

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")  # CPU baseline legs: one BLAS thread per process
import argparse
import ctypes
import json
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
for p in (ROOT / "python-raytracer_amd", ROOT / "tests", ROOT / "oracle"):
    sys.path.insert(0, str(p))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6  # MI355X fp64 vector spec: 256 CU x 64 FMA/clk x 2 x 2.4 GHz

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

RAY_BYTES = 84  # one queued ray record (rt_kernels.hip Queue): O, D, throughput f64 x 9 + 3 u32
BYTES_MODEL = {
    "primary": "jitter read (2 f64 per sample, 4 for a thin lens) + the depth-1 children written to the queue "
               "(84 B each) + the framebuffer store (3 f64 per pixel); depth-0 rays live in registers",
    "fused": "jitter read (2 f64 per sample, 4 for a thin lens) + per pixel the resolved linear RGB (3 f64) and "
             "uint8 (3 B) of a single-pass frame (the fused resolve), else its fixed-point sums (3 x 8 B + 4 B) "
             "read and written; every ray of every depth lives in registers",
    "frame": "jitter read + every secondary ray written to and read back from its wave's ring (2 x 84 B) + the "
             "fused resolve's uint8 and linear-RGB stores (27 B per pixel)",
}


def kernel_bytes_model(stats, spp, npix, lens, npass=1):
    """Algorithmic HBM bytes of one launch of the dominant kernel, from what it moves;
    texture and scene-table reads are cache-resident and not counted (BYTES_MODEL)."""
    planes = 4 if lens else 2
    rpd = stats["rays_per_depth"]
    if stats["kernel_path"] == "frame":
        return spp * npix * planes * 8 + sum(rpd[1:]) * 2 * RAY_BYTES + npix * 27
    if stats["kernel_path"] == "fused":
        return spp * npix * planes * 8 + npix * (27 if npass == 1 else 2 * 28)
    children = rpd[1] if len(rpd) > 1 else 0
    return spp * npix * planes * 8 + children * RAY_BYTES + npix * 24


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if "Model name" in line:
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def _pool_warm(args):
    builder, W, H, depth = args
    import scenes
    import sightpy_oracle  # noqa: F401

    getattr(scenes, builder)(W, H, depth)
    return os.getpid()


def _oracle_samples(sc, jit, rows, counts):
    """The oracle's get_raycolor of the samples `jit` (rows: a row tile; jit holds its pixels):
    summed colour.  Monte-Carlo draws come from numpy's global RNG, as in the reference."""
    import sightpy_oracle as O

    acc = 0.0
    for j in jit:
        Oo, Do = O.primary_rays(sc.camera, j, rows)
        acc = acc + O.raycolor(sc, O.Rays(np.ascontiguousarray(np.broadcast_to(Oo, Do.shape)), Do,
                                          O.scene_medium(sc), 0), counts)
    return acc


def _pool_task(args):
    """One Pool task: the oracle's get_raycolor of a batch of samples (reference scene.py:16-17,
    98-116: each task traces its samples and returns their summed colour)."""
    builder, W, H, depth, jit, rows = args
    import scenes

    sc = getattr(scenes, builder)(W, H, depth)
    counts = {}
    acc = _oracle_samples(sc, jit, rows, counts)
    return acc, sum(counts["depth"].values())


# CPU sample per config: the headline frames whole; the 4K and 512-spp frames on
# one row tile (rank 0's rows of an 8-rank job), rates extrapolated to the frame
CPU_TILE = {"example4_4k_d6": 8, "cornell_800_s512": 8}
# configs without a CPU leg: the oracle intersects all 20,480 triangles of the mesh per ray (the
# reference's linear collider loop), minutes for a few rows, beyond the bench's time budget
CPU_SKIP = {"mesh_1080p_d3": "TriangleMesh frame: the oracle's linear loop over 20,480 triangles per ray takes "
                             "minutes per row tile; not a BASELINE config"}


def cpu_baseline(builder, W, H, depth, spp, frame_rays, tile_of=0, budget_s=15.0):
    """The oracle (numpy restatement of the reference, oracle/sightpy_oracle.py) timed on this host's
    CPU on the same frame, or on a row tile of it (`tile_of` > 1: rank 0's rows of a tile_of-rank
    job) for frames whose single sample would run for minutes: (1) one core, samples one after another
    until the frame (tile) is done or `budget_s` is spent; (2) a multiprocessing.Pool over samples
    structured like the reference's Scene.render (scene.py:80-116: ceil(spp / workers) samples per
    task, results summed), with as many workers as this process may use (capped at 16, the GPU box's
    CPU share per GPU) -- on a tile, min(spp, workers) samples.  The extrapolated frame time is the
    GPU-counted frame's rays at the measured rate."""
    import multiprocessing as mp
    import scenes
    from sightpy._shard import scene_fanout, shard_rows

    sc = getattr(scenes, builder)(W, H, depth)
    np.random.seed(0)
    # (rank 0's rows as the library deals them: 2-row bands for a Diffuse fan-out scene)
    rows = shard_rows(H, tile_of, 0, fanout=scene_fanout(sc)) if tile_of > 1 else None
    npx = (len(rows) if rows is not None else H) * W
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    workers = max(1, min(avail, 16))
    ns = spp if rows is None else min(spp, workers)
    jit = sc.camera.draw_jitter(ns)
    if rows is not None:
        jit = np.ascontiguousarray(jit.reshape(ns, 4, H, W)[:, :, rows].reshape(ns, 4, -1))
    what = ("the whole %dx%d frame" % (W, H) if rows is None else
            "a row tile of the %dx%d frame (rank 0's %d rows of an %d-rank job, %d pixels)" % (W, H, len(rows),
                                                                                             tile_of, npx))
    counts = {}
    done = 0
    t0 = time.perf_counter()
    for s in range(ns):
        _oracle_samples(sc, jit[s:s + 1], rows, counts)
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    rays1 = sum(counts["depth"].values())
    rate1 = rays1 / dt
    one = {"value": round(rate1 / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "port",
           "sample": "oracle/sightpy_oracle.py, 1 process, OPENBLAS_NUM_THREADS=1: %d of %d samples of %s "
                     "(%d rays, %.1f s)" % (done, spp, what, rays1, dt),
           "frame_s_extrapolated": round(frame_rays / rate1, 2) if rows is not None or done < spp else None,
           "extrapolated": rows is not None or done < spp}
    per_task = -(-ns // workers)
    tasks = [(builder, W, H, depth, jit[i:i + per_task], rows) for i in range(0, ns, per_task)]
    # spawned workers (fresh interpreters: this process holds the GPU, forked children would inherit
    # its device handles), warmed up with the imports and scene build before the timed tasks
    ctx = mp.get_context("spawn")
    with ctx.Pool(min(workers, len(tasks))) as pool:
        pool.map(_pool_warm, [(builder, 8, 8, depth)] * min(workers, len(tasks)))
        t0 = time.perf_counter()
        res = list(pool.imap_unordered(_pool_task, tasks))
        dtp = time.perf_counter() - t0
    raysp = sum(r[1] for r in res)
    ratep = raysp / dtp
    pool_leg = {"value": round(ratep / 1e6, 4), "unit": "Mrays/s", "cores": min(workers, len(tasks)),
                "workers": workers, "kind": "port",
                "sample": "oracle/sightpy_oracle.py in multiprocessing.Pool(%d) over samples like scene.py:80-116 "
                          "(%d tasks of %d sample(s)): %d of %d samples of %s (%d rays, %.2f s wall incl. the scene "
                          "build per task)" % (workers, len(tasks), per_task, ns, spp, what, raysp, dtp),
                "frame_s_extrapolated": round(frame_rays / ratep, 2) if rows is not None else round(dtp, 2),
                "extrapolated": rows is not None,
                "note": "the reference splits a frame over samples, one task per ceil(spp / cpus) samples, so it "
                        "keeps at most spp cores busy (%d here) however many the host has" % spp}
    one.update({"cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "usable_cpus": avail, "pool": pool_leg})
    return one


def pmc_counters(config, kernel, variant=None):
    """Per-launch counters of `kernel` from the newest committed PMC summary of this config
    (profiles/rNN_counters_<config>.json, tools/pmc_summary.py over separate rocprofv3 --pmc passes of
    this bench: FETCH_SIZE, WRITE_SIZE, SQ fp64/VALU/wait counters), or (None, None)."""
    files = sorted(ROOT.glob("profiles/r*_counters_%s.json" % config))
    if not files:
        return None, None
    rec = json.loads(files[-1].read_text())
    for name, k in rec["kernels"].items():
        if kernel in name and (variant is None or variant in name):
            return k, files[-1].name
    return None, None


ROCPROF_TAG = {"example1_1080p_d5": "ex1_1080p_d5", "example3_1080p_d8": "ex3_1080p_d8"}


def rocprof_kernel_ms(config, kernel, sync_kind):
    """The committed rocprofv3 --kernel-trace --stats average of `kernel` (ms) over synchronous frames
    of this config (profiles/rNN*_<tag>_kernel_stats_<sync_kind>.csv, newest round first), or
    (None, None): the time base the roofline's HIP-event kernel_ms is checked against."""
    tag = ROCPROF_TAG.get(config)
    if tag is None:
        return None, None
    for f in sorted(ROOT.glob("profiles/r*_%s_kernel_stats_%s.csv" % (tag, sync_kind)), reverse=True):
        import csv

        for row in csv.DictReader(open(f)):
            if (kernel + "<") in row["Name"] and ", true>" not in row["Name"]:
                return float(row["AverageNs"]) / 1e6, "%s (%s launches)" % (f.name, row["Calls"])
    return None, None


def lane_summary(raw):
    """srt_debug_lane_stats counters -> per-depth active lane fractions of the depth loop."""
    out = []
    for d, (it, lanes) in enumerate(raw):
        if it:
            out.append({"depth": d, "wave_iterations": int(it), "live_lanes": int(lanes),
                        "frac": round(lanes / (64.0 * it), 4)})
    it_all = sum(x["wave_iterations"] for x in out)
    return {"per_depth": out,
            "overall": round(sum(x["live_lanes"] for x in out) / (64.0 * it_all), 4) if it_all else None,
            "what": "live lanes / (64 x wave iterations) of the fused depth loop, per depth (srt_debug_lane_stats "
                    "over one pipelined frame); a wave runs a depth while any of its lanes' samples still has a "
                    "ray there"}


def roofline(kname, kms, model_bytes, path, krec, src):
    """The dominant kernel against the MI355X roofline.  achieved = algorithmic bytes / launch time
    (HIP events); traffic = PMC HBM bytes per launch; the arithmetic intensity (counted fp64 FLOP per
    PMC byte) against the ridge (78.6 TF / 8 TB/s) classifies the bound; the counters then say what
    holds the kernel below that roof."""
    sec = kms * 1e-3
    roof = {"kernel": kname, "kernel_ms": round(kms, 4), "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
            "achieved": round(model_bytes / sec / 1e9, 2), "frac": round(model_bytes / sec / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_GB_per_launch": round(model_bytes / 1e9, 4),
            "bytes_model": BYTES_MODEL[path], "traffic": None}
    if krec is None or "traffic_bytes" not in krec:
        return roof
    tb = krec["traffic_bytes"]
    roof["traffic"] = round(tb / 1e9, 4)
    roof["traffic_unit"] = "GB per launch (PMC 2 x FETCH_SIZE + WRITE_SIZE)"
    roof["traffic_frac"] = round(tb / sec / 1e9 / HBM_PEAK_GBS, 4)
    roof["model_over_traffic"] = round(model_bytes / tb, 3)
    roof["source"] = src
    c = krec.get("counters", {})
    if krec.get("fp64_flop"):
        ai = krec["fp64_flop"] / tb
        ridge = FP64_PEAK_TFS * 1e3 / HBM_PEAK_GBS
        tf = krec["fp64_flop"] / sec / 1e12
        roof["arith_intensity_flop_per_byte"] = round(ai, 2)
        roof["ridge_flop_per_byte"] = round(ridge, 2)
        roof["fp64"] = {"achieved_TFLOPs": round(tf, 3), "peak": FP64_PEAK_TFS, "frac": round(tf / FP64_PEAK_TFS, 4),
                        "note": "64 x (ADD + MUL + TRANS + 2 FMA) f64 wave instructions: counts masked lanes"}
        if krec.get("valu_lane_util") is not None:
            # the flops the active lanes executed: the count weighted by the VALU instructions' active
            # lanes (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU)
            u = krec["valu_lane_util"]
            roof["fp64"].update({"valu_lane_util": round(u, 4), "achieved_TFLOPs_active_lanes": round(tf * u, 3),
                                 "frac_active_lanes": round(tf * u / FP64_PEAK_TFS, 4)})
        if ai >= ridge:
            # the fp64 side of the ridge: the kernel is measured against the vector fp64 peak (there is
            # no MFMA work here); the HBM figures stay beside it
            roof["hbm"] = {k: roof[k] for k in ("achieved", "peak", "unit", "frac")}
            roof.update({"bound": "fp64", "achieved": round(tf, 3), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": round(tf / FP64_PEAK_TFS, 4)})
    # (tools/pmc_summary.py: VALU issue cycles over the dispatch's SIMD cycles, GRBM_GUI_ACTIVE / 8 XCDs)
    if krec.get("valu_issue_frac") is not None:
        roof["valu_issue_frac"] = round(krec["valu_issue_frac"], 4)
    if krec.get("wave_wait_frac") is not None:
        roof["wave_wait_frac"] = round(krec["wave_wait_frac"], 4)
    if "valu_issue_frac" in roof and "wave_wait_frac" in roof:
        roof["limiter"] = ("latency: 3 waves/SIMD; waves wait on memory %.0f%% of their cycles, VALU "
                           "issue %.0f%% busy, HBM %.0f%% of peak" % (100 * roof["wave_wait_frac"],
                                                                    100 * roof["valu_issue_frac"],
                                                                    100 * roof["traffic_frac"]))
    return roof


def shared_frames(create, world, count, nbytes):
    """`count` host frames in POSIX shared memory, named after the launcher (one node: every rank is a
    child of one torch.distributed.run agent), as (SharedMemory, address) pairs."""
    from multiprocessing import resource_tracker, shared_memory

    out = []
    for k in range(count):
        name = "sightpy_%d_%s_%d" % (os.getppid(), os.environ.get("MASTER_PORT", "0"), k)
        if create:
            shm = shared_memory.SharedMemory(name=name, create=True, size=nbytes)
        else:
            shm = shared_memory.SharedMemory(name=name)
            resource_tracker.unregister(shm._name, "shared_memory")  # rank 0 owns (and unlinks) it
        addr = ctypes.addressof(ctypes.c_char.from_buffer(shm.buf))
        out.append((shm, addr))
    return out


def comm_id_exchange(lib, N, rank, world):
    """RCCL unique id from rank 0 to every rank through a file keyed by the launcher's pid and port
    (one node: torch.distributed.run starts every rank as a child of one agent process)."""
    path = Path("/tmp") / ("sightpy_comm_%d_%s.id" % (os.getppid(), os.environ.get("MASTER_PORT", "0")))
    buf = (ctypes.c_uint8 * N.COMM_ID_BYTES)()
    if rank == 0:
        N.check(lib, lib.srt_comm_unique_id(buf))
        tmp = path.with_suffix(".tmp")
        tmp.write_bytes(bytes(buf))
        os.replace(tmp, path)
    else:
        t0 = time.time()
        while not path.exists():
            if time.time() - t0 > 120:
                raise SystemExit("rank %d: no communicator id from rank 0 (%s)" % (rank, path))
            time.sleep(0.02)
        time.sleep(0.05)
        data = path.read_bytes()
        ctypes.memmove(buf, data, N.COMM_ID_BYTES)
    return buf, path


def visible_gpus():
    """GPUs this process may use, counted WITHOUT initialising HIP (the launcher below must not touch
    the GPU before it starts the ranks): KFD topology nodes with SIMDs (GPU agents), capped by the
    HIP/ROCR/CUDA_VISIBLE_DEVICES lists; rocminfo (a child process) if sysfs is unreadable."""
    n = None
    topo = Path("/sys/class/kfd/kfd/topology/nodes")
    try:
        n = 0
        for node in topo.iterdir():
            props = (node / "properties").read_text().split("\n")
            simd = [ln.split()[1] for ln in props if ln.startswith("simd_count ")]
            if simd and int(simd[0]) > 0:
                n += 1
    except (OSError, ValueError, IndexError):
        n = None
    if n is None:
        try:
            out = subprocess.run(["/opt/rocm/bin/rocminfo"], capture_output=True, text=True, timeout=60).stdout
            n = sum(1 for ln in out.splitlines() if ln.strip().startswith("Name:") and "gfx" in ln)
        except (OSError, subprocess.SubprocessError):
            n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


GROUP = "group"  # launch_plan: one process drives the N GPUs through the library's own group


def launch_plan(gpus, env, n_visible, argv):
    """How `bench.py --gpus N` runs: None = one rank in this process (N == 1, or N == WORLD_SIZE: one
    process per GPU, as the driver launches it through torch.distributed.run); GROUP = this process
    drives all N GPUs itself (WORLD_SIZE unset, N > 1) through the library's torch-free multi-GPU path
    -- srt_comm_init_all (one RCCL communicator over the N devices) and pipelined srt_render_group
    frames.  Refuses (SystemExit, rc 2) rather than measure fewer GPUs than asked: fewer than N GPUs
    visible, or a launcher whose WORLD_SIZE differs from N."""
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (gpus, world))
        return None
    if gpus == 1:
        return None
    if n_visible < gpus:
        raise SystemExit("bench.py: --gpus %d but only %d GPU(s) visible; refusing to report an N=%d line "
                         "measured on fewer GPUs" % (gpus, n_visible, gpus))
    return GROUP


def run_group(args, gpus):
    """`bench.py --gpus N` in one process (no launcher, no torch): contexts on devices 0..N-1 with one
    RCCL communicator (srt_comm_init_all), every frame a pipelined srt_render_group -- each GPU renders
    its row bands (SRT_RENDER_SHARDED), the uint8 tiles are gathered to device 0 over RCCL (xGMI) and
    every GPU writes its rows of the linear RGB into the pinned host frame over its own PCIe link
    (SRT_RENDER_RGB_ROWS).  Returns the JSON record (without the CPU baseline)."""
    import scenes
    from sightpy import _backend as B, _native as N
    from sightpy._shard import band_height, scene_fanout, shard_kmax

    builder, W, H, depth, spp, label = CONFIGS[args.config]
    if args.spp:
        spp = args.spp
    if args.size:
        W, H = (int(v) for v in args.size.lower().split("x"))
    sc = getattr(scenes, builder)(W, H, depth)
    lib = B.library()
    devs = (ctypes.c_int * gpus)(*range(gpus))
    ctxs = (ctypes.c_void_p * gpus)()
    N.check(lib, lib.srt_comm_init_all(gpus, devs, ctxs))
    ctx = [ctypes.c_void_p(ctxs[q]) for q in range(gpus)]
    nr, rk = ctypes.c_int(0), ctypes.c_int(0)
    N.check(lib, lib.srt_comm_rank(ctx[0], ctypes.byref(nr), ctypes.byref(rk)))
    if nr.value != gpus:
        raise SystemExit("bench.py: the library's group has %d ranks, asked for %d" % (nr.value, gpus))
    for c in ctx:
        N.check(lib, lib.srt_set_option(c, b"pipeline", 1))
        if args.shard_bands:
            N.check(lib, lib.srt_set_option(c, b"shard_bands", args.shard_bands))
        for kv in args.option:
            k, v = kv.split("=")
            N.check(lib, lib.srt_set_option(c, k.encode(), int(v)))
        B.upload(sc, ctx=c)
    cd = B.camera_desc(sc.camera)
    NOUT = 3
    outs = []
    for _ in range(NOUT):
        pu, pr = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(lib, lib.srt_host_alloc(ctx[0], 3 * W * H, ctypes.byref(pu)))
        N.check(lib, lib.srt_host_alloc(ctx[0], 3 * W * H * 8, ctypes.byref(pr)))
        outs.append((pu, pr))
    np.random.seed(0)
    mt = N.MtState.from_numpy()
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
    a.rows, a.jitter, a.out_hit_id = None, None, None
    a.mt = ctypes.pointer(mt) if args.rng == "mt" else None
    a.seed = 12345
    frame = {"k": 0}

    def step(async_ok=True, st=None, host_rgb=args.rgb_to_host):
        u8, rgb = outs[frame["k"] % NOUT]
        frame["k"] += 1
        # host_rgb: every GPU writes its rows of the linear RGB into the pinned host frame (RGB_ROWS,
        # pipelined frames) or rank 0 gathers it (synchronous); else every GPU keeps its rows in HBM
        a.out_srgb8, a.out_rgb = u8, (rgb if host_rgb else None)
        a.flags = ((N.RENDER_ASYNC | (N.RENDER_RGB_ROWS if host_rgb else 0)) if async_ok else 0) | \
            (0 if host_rgb else N.RENDER_RGB_LOCAL)
        N.check(lib, lib.srt_render_group(ctxs, gpus, ctypes.byref(cd), ctypes.byref(a),
                                          ctypes.byref(st) if st is not None else None))

    for w in range(args.warmup):
        step(async_ok=w > 0)  # the first frame synchronously (sizes queues and rings on every GPU)
    N.check(lib, lib.srt_render_group_finish(ctxs, gpus, None))
    for c in ctx:
        N.check(lib, lib.srt_synchronize(c))

    def timed(host_rgb):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(async_ok=not args.sync, host_rgb=host_rgb)
        st = N.Stats()
        N.check(lib, lib.srt_render_group_finish(ctxs, gpus, ctypes.byref(st)))  # every GPU's frames done
        for c in ctx:
            N.check(lib, lib.srt_synchronize(c))
        return time.perf_counter() - t0, st.as_dict()

    el, last = timed(args.rgb_to_host)
    ms_step = el / args.steps * 1e3
    rec = {
        "metric": "Mrays/sec (primary+secondary) + frame ms at 1920x1080 depth 5" if args.config == "example1_1080p_d5"
        else "Mrays/sec (primary+secondary) + frame ms",
        "value": round(last["total_rays"] * args.steps / el / 1e6, 3),
        "unit": "Mrays/s", "n_gpus": gpus, "nranks": nr.value, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: %s; jitter = the reference's numpy stream (seed 0, continued frame to frame) %s"
                % (label, "generated on every GPU inside each step" if args.rng == "mt" else "replaced by device Philox"),
        "config": {"workload": label, "width": W, "height": H, "max_ray_depth": depth, "spp": spp,
                   "rays_per_frame": int(last["total_rays"]), "rays_per_depth": last["rays_per_depth"],
                   "shadow_rays": last["shadow_rays"], "kernel_path_rank0": last["kernel_path"],
                   "parallelism": "row-band shards x%d in one process (srt_comm_init_all + pipelined "
                                  "srt_render_group, no torch): uint8 tiles gathered to GPU 0 over RCCL (xGMI); every "
                                  "GPU %s" % (gpus, "writes its rows of the linear RGB into the pinned host frame over "
                                                    "its own PCIe link" if args.rgb_to_host else
                                                    "keeps its rows of the linear RGB in its HBM"),
                   "frame": "render_group() entry (scene resident on every GPU) -> jitter stream on every GPU -> all "
                            "samples and depths -> sRGB resolve -> gather -> uint8 image in pinned host memory, %s; "
                            "frames pipelined" % ("linear RGB (f64) in pinned host memory too" if args.rgb_to_host
                                                  else "every GPU's rows of the linear RGB (f64) stored in its HBM"),
                   "frame_ms": round(ms_step, 4),
                   "row_bands": {"kmax": shard_kmax(H, gpus, args.shard_bands, scene_fanout(sc)),
                                 "band_height": band_height(H, gpus, shard_kmax(H, gpus, args.shard_bands,
                                                                                scene_fanout(sc)))}},
    }
    if not args.no_secondary:
        if not args.rgb_to_host:
            el2, st2 = timed(True)
            rec["host_rgb"] = {"value": round(st2["total_rays"] * args.steps / el2 / 1e6, 3),
                               "ms_per_step": round(el2 / args.steps * 1e3, 4),
                               "what": "same frames with every GPU's rows of the linear RGB copied into the pinned "
                                       "host frame as well (SRT_RENDER_RGB_ROWS)"}
        lat = []
        for _ in range(3):
            t1 = time.perf_counter()
            step(async_ok=False, st=N.Stats())
            lat.append((time.perf_counter() - t1) * 1e3)
        rec["config"]["frame_latency_ms"] = round(float(np.median(lat)), 4)
    for pu, pr in outs:
        lib.srt_host_free(ctx[0], pu)
        lib.srt_host_free(ctx[0], pr)
    for c in ctx:
        lib.srt_destroy(c)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--config", default="example1_1080p_d5", choices=sorted(CONFIGS))
    ap.add_argument("--rng", default="mt", choices=["mt", "device"],
                    help="mt: the reference's numpy stream generated on the GPU inside every step; device: Philox")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the latency / device-resident / roofline runs")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--size", default=None, help="diagnostic: WxH override of the config's frame size")
    ap.add_argument("--option", action="append", default=[],
                    help="experiment: srt_set_option KEY=VALUE before rendering (repeatable)")
    ap.add_argument("--hw-queues", type=int, default=7,
                    help="GPU_MAX_HW_QUEUES for this process (read when HIP initialises): the library keeps one "
                         "frame in flight per hardware queue but one (rt_kernels.hip default_slots); 7 -> six "
                         "frames.  Set here, not inherited: the GPU boxes export HIP's default of 4, which "
                         "leaves four frame slots sharing three queues")
    ap.add_argument("--rgb-to-host", action="store_true",
                    help="headline frames copy the linear RGB (f64) to pinned host memory as well as the uint8 image "
                         "(rounds 1-4's step); default: the uint8 image to host memory, the linear RGB kept in HBM")
    ap.add_argument("--device-outputs", action="store_true",
                    help="diagnostic (one process): the frames' outputs left in HBM instead of host memory")
    ap.add_argument("--sync", action="store_true",
                    help="diagnostic: synchronous timed frames (no pipelining), so a rocprofv3 kernel trace shows each "
                         "kernel's launch time alone, as the roofline's HIP-event kernel_ms measures it")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic (1 GPU): render only one rank's rows of an N-rank job (its per-frame work "
                         "without the gather)")
    ap.add_argument("--shard-rank", default="0",
                    help="with --shard-of: the rank rehearsed, or 'all' / 'all-reversed' (every rank in turn, "
                         "from rank 0 or from the last; ms_per_step = the slowest rank, value = all ranks' rays / "
                         "that time)")
    ap.add_argument("--rehearse-assemble", action="store_true",
                    help="with --shard-of N: rank 0's rehearsed frame also assembles the whole frame from its tile and N-1 "
                         "stand-in tiles (k_assemble) and copies the whole uint8 frame to the host, as a sharded rank 0 "
                         "does after the RCCL gather (library option rehearse_assemble)")
    ap.add_argument("--shard-bands", type=int, default=0,
                    help="most row bands per rank (library option shard_bands; default rt_device.h shard_kmax)")
    args = ap.parse_args()
    if not 1 <= args.hw_queues <= 32:
        raise SystemExit("bench.py: --hw-queues 1 .. 32")
    os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)  # (before anything initialises HIP)

    plan = launch_plan(args.gpus, os.environ, visible_gpus() if "WORLD_SIZE" not in os.environ and args.gpus > 1
                       else args.gpus, sys.argv[1:])
    if plan == GROUP:
        # this process drives the N GPUs (the library's RCCL group); no CPU baseline at N > 1
        print(json.dumps(run_group(args, args.gpus)), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["SIGHTPY_DEVICE"] = str(local)

    import scenes
    from sightpy import _backend as B, _native as N

    builder, W, H, depth, spp, label = CONFIGS[args.config]
    if args.spp:
        spp = args.spp
    if args.size:
        W, H = (int(v) for v in args.size.lower().split("x"))
    sc = getattr(scenes, builder)(W, H, depth)
    lib, ctx = B.context()
    id_path = None
    NOUT = 3  # output buffers: one per frame in flight
    shm_frames = []
    if world > 1:
        # the frame's linear RGB in host shared memory: every rank writes its own rows into it over
        # its own PCIe link (SRT_RENDER_RGB_ROWS); created by rank 0 before it publishes the RCCL id
        if rank == 0:
            shm_frames = shared_frames(True, world, NOUT, 3 * W * H * 8)
        cid, id_path = comm_id_exchange(lib, N, rank, world)
        if rank != 0:
            shm_frames = shared_frames(False, world, NOUT, 3 * W * H * 8)
        N.check(lib, lib.srt_comm_init(ctx, world, rank, cid))
    nr, rk = ctypes.c_int(0), ctypes.c_int(0)
    N.check(lib, lib.srt_comm_rank(ctx, ctypes.byref(nr), ctypes.byref(rk)))
    if (nr.value, rk.value) != (world, rank):
        raise SystemExit("bench.py: the library's communicator has %d ranks (this is %d), the launcher %d (rank %d)"
                         % (nr.value, rk.value, world, rank))
    N.check(lib, lib.srt_set_option(ctx, b"pipeline", 1))  # size every frame slot during the warmup
    if args.shard_bands:
        N.check(lib, lib.srt_set_option(ctx, b"shard_bands", args.shard_bands))
    for kv in args.option:
        k, v = kv.split("=")
        N.check(lib, lib.srt_set_option(ctx, k.encode(), int(v)))
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    npix_full = W * H
    # the linear RGB: host memory (--rgb-to-host: every rank its own rows over its PCIe link at N > 1)
    # or each rank's rows kept in its HBM (SRT_RENDER_RGB_LOCAL)
    base_flags = N.RENDER_SHARDED if world > 1 else 0

    def frame_flags(host_rgb):
        return base_flags | ((N.RENDER_RGB_ROWS if world > 1 else 0) if host_rgb else N.RENDER_RGB_LOCAL)
    rows32 = None
    from sightpy._shard import band_height, scene_fanout, shard_kmax, shard_rows

    # the library's band count (rt_device.h shard_kmax: depends on the scene's fan-out)
    kmax = shard_kmax(H, max(world, args.shard_of, 1), args.shard_bands, scene_fanout(sc))
    rehearse = {None: None}  # rank -> its rows (None: the frame as the launcher splits it)
    if args.shard_of > 1 and world == 1:
        ranks = (range(args.shard_of) if args.shard_rank == "all" else
                 range(args.shard_of - 1, -1, -1) if args.shard_rank == "all-reversed" else [int(args.shard_rank)])
        rehearse = {r: np.ascontiguousarray(shard_rows(H, args.shard_of, r, kmax), dtype=np.int32)
                    for r in ranks}
        rows32 = rehearse[min(ranks)]
        npix_full = max(len(v) for v in rehearse.values()) * W  # the shards' outputs
        if args.rehearse_assemble:
            N.check(lib, lib.srt_set_option(ctx, b"rehearse_assemble", args.shard_of))
            npix_full = W * H  # (rank 0 hands back the whole frame)

    # outputs: the whole frame in pinned host memory, one pair of buffers per frame in flight (N > 1:
    # the uint8 image on rank 0, gathered over RCCL; the linear RGB in the shared frames, every rank)
    outs = []
    for k in range(NOUT):
        pu, pr = ctypes.c_void_p(), ctypes.c_void_p()
        if args.device_outputs and world == 1:  # (diagnostic: no host copies)
            N.check(lib, lib.srt_device_alloc(ctx, 3 * npix_full, ctypes.byref(pu)))
            N.check(lib, lib.srt_device_alloc(ctx, 3 * npix_full * 8, ctypes.byref(pr)))
            outs.append((pu, pr))
            continue
        if rank == 0:
            N.check(lib, lib.srt_host_alloc(ctx, 3 * npix_full, ctypes.byref(pu)))
        if world > 1:
            pr = ctypes.c_void_p(shm_frames[k][1])
            N.check(lib, lib.srt_host_register(ctx, pr, 3 * W * H * 8))
        else:
            N.check(lib, lib.srt_host_alloc(ctx, 3 * npix_full * 8, ctypes.byref(pr)))
        outs.append((pu, pr))

    np.random.seed(0)
    mt = N.MtState.from_numpy()
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
    a.rows = None
    if rows32 is not None:
        a.rows, a.n_rows = N.ptr(rows32), len(rows32)
    a.jitter = None
    a.mt = ctypes.pointer(mt) if args.rng == "mt" else None
    a.seed = 12345
    a.out_hit_id = None
    frame = {"k": 0}

    def step(async_ok=True, st=None, host_rgb=args.rgb_to_host):
        u8, rgb = outs[frame["k"] % NOUT]
        a.out_srgb8, a.out_rgb = (u8 if u8.value else None), (rgb if host_rgb else None)
        frame["k"] += 1
        a.flags = frame_flags(host_rgb) | (N.RENDER_ASYNC if async_ok else 0)
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), ctypes.byref(st) if st else None))

    def barrier():
        N.check(lib, lib.srt_render_finish(ctx, None))
        N.check(lib, lib.srt_synchronize(ctx))
        if world > 1:
            N.check(lib, lib.srt_comm_barrier(ctx))

    def timed(host_rgb):
        """args.steps pipelined frames after a barrier: (seconds, last frame's stats)"""
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(async_ok=not args.sync, host_rgb=host_rgb)
        enq_ms = (time.perf_counter() - t0) / args.steps * 1e3  # host time to queue a frame
        st = N.Stats()
        N.check(lib, lib.srt_render_finish(ctx, ctypes.byref(st)))  # every frame in host memory, flags checked
        if world > 1:
            N.check(lib, lib.srt_comm_barrier(ctx))
        return time.perf_counter() - t0, st.as_dict(), enq_ms

    rank_ms, rank_rays, enq = [], [], []
    for i, (rr, rows_r) in enumerate(rehearse.items()):
        if rows_r is not None:
            rows32 = rows_r
            a.rows, a.n_rows = N.ptr(rows32), len(rows32)
        t_w = time.perf_counter()
        w = 0
        # rehearsing several ranks: the first one's warm-up also runs >= 1.5 s of frames, so that it
        # does not carry the GPU's own warm-up into the slowest-rank figure
        prime_s = 1.5 if (i == 0 and len(rehearse) > 1) else 0.0
        while w < args.warmup or time.perf_counter() - t_w < prime_s:
            step(async_ok=w > 0 and not args.sync)  # the first frame runs synchronously (sizes queues and rings)
            w += 1
            if w % 50 == 0:
                barrier()  # (bounded queue depth while priming)
        barrier()
        el, last, enq_ms = timed(args.rgb_to_host)
        enq.append(enq_ms)
        rank_ms.append(el / args.steps * 1e3)
        rank_rays.append(last["total_rays"])
    elapsed = max(rank_ms) * args.steps / 1e3
    if len(rehearse) > 1:
        last["total_rays"] = sum(rank_rays)
    vals = (ctypes.c_double * 2)(elapsed, float(last["total_rays"]))
    if world > 1:
        N.check(lib, lib.srt_comm_allreduce(ctx, vals, 1, 1))  # max elapsed over ranks
        tot = (ctypes.c_double * 1)(float(last["total_rays"]))
        N.check(lib, lib.srt_comm_allreduce(ctx, tot, 1, 0))  # rays of the frame, all ranks
        elapsed, total_rays = vals[0], tot[0]
    else:
        total_rays = float(last["total_rays"])
    ms_step = elapsed / args.steps * 1e3
    value = total_rays * args.steps / elapsed / 1e6

    # ---- secondary figures --------------------------------------------------------------------
    sec = {}

    def secondaries():
        if not args.no_secondary and not args.rgb_to_host and not args.device_outputs and len(rehearse) == 1:
            # the same frames with the linear RGB copied to host memory as well (rounds 1-4's step)
            barrier()
            el2, st2, _ = timed(True)
            vals2 = (ctypes.c_double * 1)(el2)
            if world > 1:
                N.check(lib, lib.srt_comm_allreduce(ctx, vals2, 1, 1))
            sec["host_rgb"] = {"value": round(total_rays * args.steps / vals2[0] / 1e6, 3),
                               "ms_per_step": round(vals2[0] / args.steps * 1e3, 4),
                               "what": "same frames with the linear RGB (f64) copied to pinned host memory as well "
                                       "(%s)" % ("every rank its rows into the shared host frame, SRT_RENDER_RGB_ROWS"
                                                 if world > 1 else "50 MB per 1080p frame over one PCIe link")}
        if not args.no_secondary:
            # one synchronous frame, render() entry -> host memory (latency, not throughput)
            lat = []
            stats = []
            for _ in range(3):
                s = N.Stats()
                t1 = time.perf_counter()
                step(async_ok=False, st=s)
                lat.append((time.perf_counter() - t1) * 1e3)
                stats.append(s.as_dict())
            sec["frame_latency_ms"] = round(float(np.median(lat)), 4)
            sec["stats"] = stats
            if stats[0]["kernel_path"] == "fused" and not args.sync:
                # the pipelined frames' kernel (k_primary_lean, when the scene has one) timed alone in the same
                # synchronous frames (option sync_lean), for the roofline
                n0, n1 = ctypes.c_int64(0), ctypes.c_int64(0)
                N.check(lib, lib.srt_debug_lean_launches(ctx, ctypes.byref(n0)))
                N.check(lib, lib.srt_set_option(ctx, b"sync_lean", 1))
                lean_stats = []
                try:
                    for _ in range(3):
                        s = N.Stats()
                        step(async_ok=False, st=s)
                        lean_stats.append(s.as_dict())
                finally:
                    N.check(lib, lib.srt_set_option(ctx, b"sync_lean", 0))
                N.check(lib, lib.srt_debug_lean_launches(ctx, ctypes.byref(n1)))
                if n1.value > n0.value:
                    sec["stats_lean"] = lean_stats
                    # lane utilisation of the pipelined frames' depth loop: one more pipelined frame with the
                    # kernel's counting instantiation (not timed)
                    raw = (ctypes.c_int64 * (2 * 16))()
                    N.check(lib, lib.srt_debug_lane_stats(ctx, 1, None, 0))
                    step()
                    step()
                    N.check(lib, lib.srt_debug_lane_stats(ctx, 0, raw, 16))
                    sec["lane_stats"] = lane_summary([(raw[2 * d] / 2, raw[2 * d + 1] / 2) for d in range(16)])
            if world == 1 and rows32 is None:
                # the round-1 headline form: jitter resident in HBM, outputs left in HBM
                nj = spp * 4 * npix_full
                jd, od, ud = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
                N.check(lib, lib.srt_device_alloc(ctx, nj * 8, ctypes.byref(jd)))
                N.check(lib, lib.srt_device_alloc(ctx, 3 * npix_full * 8, ctypes.byref(od)))
                N.check(lib, lib.srt_device_alloc(ctx, 3 * npix_full, ctypes.byref(ud)))
                np.random.seed(0)
                jh = np.random.rand(nj)
                N.check(lib, lib.srt_memcpy(ctx, jd, N.ptr(jh), jh.nbytes))
                del jh
                r = N.RenderArgs()
                r.spp, r.n_rows, r.jitter, r.seed, r.out_rgb, r.out_srgb8 = spp, H, jd, 12345, od, ud
                r.flags = 0
                N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(r), None))
                r.flags = N.RENDER_ASYNC
                N.check(lib, lib.srt_synchronize(ctx))
                t1 = time.perf_counter()
                for _ in range(args.steps):
                    N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(r), None))
                s = N.Stats()
                N.check(lib, lib.srt_render_finish(ctx, ctypes.byref(s)))
                dt = time.perf_counter() - t1
                sec["device_resident"] = {
                    "value": round(s.total_rays * args.steps / dt / 1e6, 3), "ms_per_step": round(dt / args.steps * 1e3, 4),
                    "what": "same frames with the jitter pre-resident in HBM (uploaded once) and the outputs left in HBM "
                            "(the round-1 headline; excludes the in-step jitter generation and the host copies)"}
                for p in (jd, od, ud):
                    lib.srt_device_free(ctx, p)

    if world > 1:
        # (the N > 1 line must not be lost to a figure beside it: a library error in the secondary
        # frames -- the host-RGB rows into the shared frame, synchronous sharded frames -- is reported in
        # the line instead; every rank takes the same branch, so no collective is left waiting)
        try:
            secondaries()
        except (RuntimeError, OSError) as e:
            sec.clear()
            sec["error"] = "%s: %s" % (type(e).__name__, e)
    else:
        secondaries()

    if rank == 0:
        rec = {
            "metric": "Mrays/sec (primary+secondary) + frame ms at 1920x1080 depth 5" if args.config == "example1_1080p_d5"
            else "Mrays/sec (primary+secondary) + frame ms",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "nranks": nr.value,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: %s; jitter = the reference's numpy stream (seed 0, continued frame to frame) %s"
                    % (label, "generated on the GPU inside each step" if args.rng == "mt" else "replaced by device Philox"),
            "config": {"workload": label, "width": W, "height": H, "max_ray_depth": depth, "spp": spp,
                       "rays_per_frame": int(total_rays), "rays_per_depth_rank0": last["rays_per_depth"],
                       "shadow_rays_rank0": last["shadow_rays"], "kernel_path": last["kernel_path"],
                       "chain_from_depth": last["chain_from"],
                       "parallelism": "row-band shards x%d: uint8 tiles gathered to rank 0 over RCCL (xGMI); every rank "
                                      "%s" % (world, "writes its rows of the linear RGB into the shared host frame over "
                                                     "its own PCIe link" if args.rgb_to_host else
                                                     "keeps its rows of the linear RGB in its HBM")
                       if world > 1 else (("diagnostic: rank %s's rows of a %d-rank job, no gather" % (
                                              args.shard_rank, args.shard_of) if len(rehearse) == 1 else
                                              "diagnostic: every rank's rows of a %d-rank job rendered in turn on "
                                              "one GPU, no gather; ms_per_step = the slowest rank's frame"
                                              % args.shard_of) if rows32 is not None else "1 GPU"),
                       "frame": "render() entry (scene resident) -> jitter stream on the GPU -> all samples and depths "
                                "-> sRGB resolve -> uint8 image in pinned host memory, %s; frames pipelined"
                                % ("linear RGB (f64) in pinned host memory too" if args.rgb_to_host else
                                   "the linear RGB (f64) stored in HBM (what Scene.render keeps; the reference "
                                   "returns the uint8 image, scene.py:118-140)"),
                       "frame_ms": round(ms_step, 4),
                       "host_enqueue_ms": round(max(enq), 4),
                       "row_bands": {"kmax": kmax,
                                     "band_height": band_height(H, max(world, args.shard_of, 1), kmax)}},
        }
        if len(rehearse) > 1:
            order = list(rehearse)  # (rank of each rehearsal, in the order run)
            rec["rank_frame_ms"] = [round(rank_ms[order.index(r)], 4) for r in sorted(order)]
            rec["rank_rays"] = [rank_rays[order.index(r)] for r in sorted(order)]
            rec["rehearsal_order"] = order
        if "host_rgb" in sec:
            rec["host_rgb"] = sec["host_rgb"]
        if "error" in sec:
            rec["secondary_error"] = sec["error"]
        if "frame_latency_ms" in sec:
            rec["config"]["frame_latency_ms"] = sec["frame_latency_ms"]
            if "device_resident" in sec:
                rec["device_resident"] = sec["device_resident"]
            st0 = sec["stats"]
            path = {"frame": "frame", "fused": "fused"}.get(st0[0]["kernel_path"], "primary")
            frame_path = path == "frame"
            kname = "k_frame" if frame_path else "k_primary"
            # one launch of the dominant kernel: a frame of `passes` passes launches it once per pass
            npass = max(1, st0[0]["passes"])
            kms = float(np.mean([x["ms_primary_kernel"] for x in st0])) / npass
            kms_sync = None
            variant = {"fused": ", true>", "primary": ", false>"}.get(path)
            if "stats_lean" in sec:
                # the timed region's kernel: the lean form the pipelined frames run
                kms_sync, kname, variant = kms, "k_primary_lean", None
                kms = float(np.mean([x["ms_primary_kernel"] for x in sec["stats_lean"]])) / npass
            krec, src = (None, None) if (args.size or args.spp or world > 1 or rows32 is not None) else \
                pmc_counters(args.config, kname, variant)
            from sightpy._shard import shard_rows

            npix_rank = len(shard_rows(H, max(world, args.shard_of, 1), 0, kmax)) * W
            st_pass = dict(st0[0])
            st_pass["rays_per_depth"] = [r / npass for r in st0[0]["rays_per_depth"]]
            model = kernel_bytes_model(st_pass, spp / npass, npix_rank, sc.camera.lens_radius != 0.0, npass)
            roof = roofline(kname + (" (fused paths)" if path == "fused" else ""), kms, model, path, krec, src)
            if npass > 1:
                roof["passes_per_frame"] = npass
            roof["kernel_ms_note"] = ("one launch in a synchronous frame (HIP events); pipelined frames overlap one "
                                      "frame's tail with the next, so ms_per_step can be below it")
            if kms_sync is not None:
                roof["kernel_ms_note"] += ("; the kernel the pipelined frames run (k_primary_lean), timed alone in "
                                           "synchronous frames (option sync_lean)")
                roof["sync_frames_kernel"] = {"kernel": "k_primary (fused paths: synchronous frames, Scene.render)",
                                              "kernel_ms": round(kms_sync / 1.0, 4)}
            rp_ms, rp_src = (None, None) if (args.size or args.spp or world > 1 or rows32 is not None) else \
                rocprof_kernel_ms(args.config, kname, "sync_lean" if kname == "k_primary_lean" else "sync")
            if rp_ms is not None:
                # the same launch's rocprofv3 dispatch time (the events bracket it ~0.05 ms wider)
                roof["kernel_ms_rocprof"] = round(rp_ms, 4)
                roof["kernel_ms_rocprof_source"] = rp_src
                if "fp64" in roof:
                    f = roof["fp64"]
                    f["frac_rocprof"] = round(f["frac"] * kms / rp_ms, 4)
                    if "frac_active_lanes" in f:
                        f["frac_active_lanes_rocprof"] = round(f["frac_active_lanes"] * kms / rp_ms, 4)
            if "lane_stats" in sec:
                roof["active_lane_frac"] = sec["lane_stats"]
            rec["roofline"] = roof
        if not args.no_cpu_baseline and world == 1 and args.config in CPU_SKIP:
            rec["cpu_baseline"] = {"value": None, "skipped": CPU_SKIP[args.config]}
        elif not args.no_cpu_baseline and world == 1:
            rec["cpu_baseline"] = cpu_baseline(builder, W, H, depth, spp, total_rays, CPU_TILE.get(args.config, 0))
        print(json.dumps(rec), flush=True)
    if world > 1:
        N.check(lib, lib.srt_comm_barrier(ctx))
        if rank == 0 and id_path is not None:
            try:
                id_path.unlink()
            except OSError:
                pass
    for pu, pr in outs:
        if pu.value:
            lib.srt_host_free(ctx, pu)
        if world > 1:
            lib.srt_host_unregister(ctx, pr)
        else:
            lib.srt_host_free(ctx, pr)
    if world > 1:
        N.check(lib, lib.srt_comm_barrier(ctx))  # every rank unregistered before rank 0 unlinks
        for shm, _ in shm_frames:
            shm.close()
            if rank == 0:
                shm.unlink()


if __name__ == "__main__":
    main()
