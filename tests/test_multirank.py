"""Multi-GPU row sharding.

The product path is torch-free: the library splits a frame into 8-row bands dealt round-robin over
the ranks (SRT_RENDER_SHARDED, rt_device.h shard_of_row / shard_local_row) and gathers the tiles
to rank 0 over RCCL (rt_kernels.hip gather_post / k_assemble).  On the CPU:
  * the kernels' shard map (compiled for the CPU) against the numpy restatement (sightpy._shard);
  * a world-size-2 `gloo` job replays the gather protocol -- each rank sends its unpadded tile,
    rank 0 receives into padded staging and assembles with the kernels' map -- and must rebuild
    the frame exactly.
On the GPU (one card): the sharded render through a 1-rank communicator (multi-process API) and a
1-device srt_comm_init_all group (single-process API) equal the plain render, and every rank's
shard of an N-rank frame, rendered in turn, assembles into the plain render (the numpy-stream
jitter is indexed by global pixel).  The N > 1 RCCL exchange itself runs only on a multi-GPU node.
"""
import ctypes
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_rows_partition():
    from sightpy._shard import shard_rows, assemble_index, max_shard_rows

    for H in (1, 7, 8, 37, 300, 1080):
        for world in (1, 2, 3, 4, 8):
            parts = [shard_rows(H, world, r) for r in range(world)]
            allrows = np.sort(np.concatenate(parts))
            assert np.array_equal(allrows, np.arange(H))
            assert max(len(p) for p in parts) == max_shard_rows(H, world)
            idx = assemble_index(H, world)
            buf = np.full(world * max_shard_rows(H, world), -1)
            for r, p in enumerate(parts):
                buf[r * max_shard_rows(H, world) + np.arange(len(p))] = p
            assert np.array_equal(buf[idx], np.arange(H))
    # 1080 rows over 8 ranks: 40 bands of 27 rows, 5 per rank, 135 rows each (the busiest rank has no
    # more rows than 1080 / 8; kmax = 8 allows 4..8 bands per rank, and 5 is the most that balance)
    from sightpy._shard import band_height

    assert band_height(1080, 8) == 27
    assert [len(shard_rows(1080, 8, r)) for r in range(8)] == [135] * 8
    # ex4 4K over 8 ranks: 270 rows each; cornell 800 over 8: 100 rows each in 5 bands of 20
    assert [len(shard_rows(2160, 8, r)) for r in range(8)] == [270] * 8
    assert band_height(800, 8) == 20 and [len(shard_rows(800, 8, r)) for r in range(8)] == [100] * 8
    # one band per rank allowed: contiguous blocks
    assert band_height(1080, 8, kmax=1) == 135
    # round-robin: rank 0 takes band 0 of every period
    assert list(shard_rows(40, 2, 0, kmax=2)) == list(range(0, 10)) + list(range(20, 30))


def _kernel_shard_map(H, n, kmax=8):
    import hostcheck as HC

    owner = np.empty(H, dtype=np.int32)
    local = np.empty(H, dtype=np.int64)
    lib = HC.lib()
    lib.hc_shard_map.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.hc_shard_map.restype = ctypes.c_int64
    h = lib.hc_shard_map(H, n, kmax, owner.ctypes.data, local.ctypes.data)
    return owner, local, h


@pytest.mark.parametrize("H", [8, 9, 13, 37, 300, 800, 1080, 2160])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("kmax", [1, 4, 8, 17])
def test_kernel_shard_map_matches_partition(H, n, kmax):
    from sightpy._shard import shard_rows, band_height, rank_rows

    owner, local, h = _kernel_shard_map(H, n, kmax)
    assert h == band_height(H, n, kmax)
    for q in range(n):
        rows = shard_rows(H, n, q, kmax)
        assert len(rows) > 0  # (H >= n) every rank gets rows, e.g. H = 9 over 8 ranks with one band each
        assert len(rows) == rank_rows(H, n, q, h)
        assert np.array_equal(np.where(owner == q)[0], rows)
        assert np.array_equal(local[rows], np.arange(len(rows)))
        # a rank's j-th band lies in period j (the RGB row copies and the local-row map rely on it)
        assert np.array_equal(rows // (h * n), np.arange(len(rows)) // h)


@pytest.mark.parametrize("H,n", [(800, 8), (800, 2), (1080, 8), (2160, 8), (37, 3), (8, 8)])
@pytest.mark.parametrize("kmax,fanout", [(0, 1), (0, 2), (0, 20), (5, 20), (0, 3)])
def test_kernel_band_count_rule_matches_partition(H, n, kmax, fanout):
    """The library's automatic band count (rt_device.h shard_kmax: 8 bands per rank, or 2-row bands
    for a Diffuse fan-out scene) is the one sightpy._shard restates."""
    import hostcheck as HC
    from sightpy._shard import shard_kmax, band_height

    lib = HC.lib()
    lib.hc_shard_kmax.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.hc_shard_kmax.restype = ctypes.c_int
    k = lib.hc_shard_kmax(H, n, kmax, fanout)
    assert k == shard_kmax(H, n, kmax, fanout)
    owner, local, h = _kernel_shard_map(H, n, k)
    assert h == band_height(H, n, kmax, fanout)
    if fanout > 2 and not kmax and H >= 4 * n * 8:
        assert h <= 4  # k in [kmax / 2, kmax]: at most twice the 2-row bands


def test_cornell_scene_takes_two_row_bands():
    import scenes
    from sightpy._shard import scene_fanout, band_height

    assert scene_fanout(scenes.cornell(40, 40)) == 20
    assert scene_fanout(scenes.example1(16, 12)) == 1
    assert scene_fanout(scenes.example4(16, 12, 2)) == 2
    assert band_height(800, 8, fanout=20) == 2 and band_height(1080, 8, fanout=1) == 27


def _gather_worker(rank, world, port, H, W):
    for p in (ROOT / "python-raytracer_amd", ROOT / "tests", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from sightpy._shard import shard_rows, max_shard_rows

    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = np.random.default_rng(7).integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    rgb = np.random.default_rng(8).random((3, H * W))
    rows = shard_rows(H, world, rank)
    tile_u8 = full[rows].copy()
    tile_rgb = rgb.reshape(3, H, W)[:, rows].reshape(3, -1).copy()
    if rank == 0:
        maxpix = max_shard_rows(H, world) * W
        g_u8 = np.zeros((world, maxpix * 3), dtype=np.uint8)
        g_rgb = np.zeros((world, 3 * maxpix))
        g_u8[0, : tile_u8.size] = tile_u8.reshape(-1)
        g_rgb[0, : tile_rgb.size] = tile_rgb.reshape(-1)
        for q in range(1, world):
            npq = len(shard_rows(H, world, q)) * W
            bu = torch.zeros(3 * npq, dtype=torch.uint8)
            br = torch.zeros(3 * npq, dtype=torch.float64)
            dist.recv(bu, q)
            dist.recv(br, q)
            g_u8[q, : 3 * npq] = bu.numpy()
            g_rgb[q, : 3 * npq] = br.numpy()
        # k_assemble with the kernels' map
        owner, local, _ = _kernel_shard_map(H, world)
        out_u8 = np.empty((H, W, 3), dtype=np.uint8)
        out_rgb = np.empty((3, H, W))
        for y in range(H):
            q, i = owner[y], local[y]
            npq = len(shard_rows(H, world, q)) * W
            out_u8[y] = g_u8[q, 3 * i * W: 3 * (i + 1) * W].reshape(W, 3)
            for ch in range(3):
                out_rgb[ch, y] = g_rgb[q, ch * npq + i * W: ch * npq + (i + 1) * W]
        assert np.array_equal(out_u8, full)
        assert np.array_equal(out_rgb.reshape(3, -1), rgb)
    else:
        dist.send(torch.from_numpy(tile_u8.reshape(-1)), 0)
        dist.send(torch.from_numpy(tile_rgb.reshape(-1)), 0)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("H", [37, 48])
def test_gather_protocol_gloo_world2(H):
    import torch.multiprocessing as mp

    mp.start_processes(_gather_worker, args=(2, _free_port(), H, 5), nprocs=2, join=True, start_method="spawn")


# ---- GPU ------------------------------------------------------------------------------------


def _render_args(N, spp, H, flags, mt=None, u8=None, rgb=None, seed=5):
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
    a.mt = ctypes.pointer(mt) if mt is not None else None
    a.seed = seed
    a.flags = flags
    a.out_srgb8 = N.ptr(u8)
    a.out_rgb = N.ptr(rgb)
    return a


@pytest.mark.gpu
def test_gpu_sharded_frame_one_rank_communicator_equals_plain_render():
    """SRT_RENDER_SHARDED through a 1-rank RCCL communicator (srt_comm_unique_id / srt_comm_init, the
    multi-process API bench.py uses), synchronous and pipelined, equals the plain render."""
    import scenes
    from sightpy import _backend as B, _native as N

    sc = scenes.example1(96, 40, 3)
    np.random.seed(11)
    ref = B.render_scene(sc, 2, seed=5, mt=True)
    after_ref = np.random.get_state()[1].copy()
    lib = B.library()
    ctx = ctypes.c_void_p()
    N.check(lib, lib.srt_create(int(B.devices()[0]), ctypes.byref(ctx)))
    try:
        cid = (ctypes.c_uint8 * N.COMM_ID_BYTES)()
        N.check(lib, lib.srt_comm_unique_id(cid))
        N.check(lib, lib.srt_comm_init(ctx, 1, 0, cid))
        B.upload(sc, ctx=ctx)
        cd = B.camera_desc(sc.camera)
        np.random.seed(11)
        mt = N.MtState.from_numpy()
        u8 = np.empty((40 * 96, 3), np.uint8)
        rgb = np.empty((3, 40 * 96))
        a = _render_args(N, 2, 40, N.RENDER_SHARDED | N.RENDER_GATHER_RGB, mt, u8, rgb)
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        np.testing.assert_allclose(rgb, ref.rgb, rtol=1e-12, atol=1e-15)
        assert np.array_equal(u8.reshape(40, 96, 3), ref.srgb8)
        assert np.array_equal(np.ctypeslib.as_array(mt.key), after_ref)
        # four pipelined frames into pinned host buffers, the stream continuing on the device
        bufs = []
        for _ in range(4):
            pu, pr = ctypes.c_void_p(), ctypes.c_void_p()
            N.check(lib, lib.srt_host_alloc(ctx, 3 * 40 * 96, ctypes.byref(pu)))
            N.check(lib, lib.srt_host_alloc(ctx, 3 * 40 * 96 * 8, ctypes.byref(pr)))
            bufs.append((pu, pr))
        np.random.seed(11)
        mt2 = N.MtState.from_numpy()
        a2 = _render_args(N, 2, 40, N.RENDER_SHARDED | N.RENDER_GATHER_RGB | N.RENDER_ASYNC, mt2)
        for pu, pr in bufs:
            a2.out_srgb8, a2.out_rgb = pu, pr
            N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a2), None))
        N.check(lib, lib.srt_render_finish(ctx, None))
        np.random.seed(11)
        for pu, pr in bufs:
            want = B.render_scene(sc, 2, seed=5, mt=True)
            got = np.ctypeslib.as_array(ctypes.cast(pr, ctypes.POINTER(ctypes.c_double)), shape=(3, 40 * 96))
            np.testing.assert_allclose(got, want.rgb, rtol=1e-12, atol=1e-15)
            got8 = np.ctypeslib.as_array(ctypes.cast(pu, ctypes.POINTER(ctypes.c_uint8)), shape=(40 * 96 * 3,))
            assert np.array_equal(got8.reshape(40, 96, 3), want.srgb8)
        assert np.array_equal(np.ctypeslib.as_array(mt2.key), np.random.get_state()[1])
        assert mt2.pos == np.random.get_state()[2]
        for pu, pr in bufs:
            lib.srt_host_free(ctx, pu)
            lib.srt_host_free(ctx, pr)
    finally:
        lib.srt_destroy(ctx)


@pytest.mark.gpu
def test_gpu_group_render_one_device_equals_plain_render(monkeypatch):
    """srt_comm_init_all + srt_render_group (the single-process multi-GPU API Scene.render uses with
    $SIGHTPY_DEVICES) on a group of one device."""
    import scenes
    from sightpy import _backend as B

    monkeypatch.setenv("SIGHTPY_DEVICES", str(B.devices()[0]))
    sc = scenes.example3(64, 48, 6)
    np.random.seed(4)
    ref = B.render_scene(sc, 2, seed=5, mt=True)
    np.random.seed(4)
    got = B.render_group(sc, 2, seed=5, mt=True)
    np.testing.assert_allclose(got.rgb, ref.rgb, rtol=1e-12, atol=1e-15)
    assert np.array_equal(got.srgb8, ref.srgb8)
    assert got.stats["total_rays"] == ref.stats["total_rays"]


@pytest.mark.gpu
def test_gpu_async_group_frames_equal_plain_render(monkeypatch):
    """Pipelined group frames (srt_render_group with SRT_RENDER_ASYNC | SRT_RENDER_RGB_ROWS, then
    srt_render_group_finish: the in-process multi-GPU bench's frame loop, bench.py --gpus N) on a group
    of one device: every frame's uint8 image and linear RGB in pinned host memory equal the synchronous
    render from the same numpy state, and the numpy stream continues frame to frame as Scene.render's."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N

    monkeypatch.setenv("SIGHTPY_DEVICES", str(B.devices()[0]))
    sc = scenes.example1(96, 64, 4)
    W, H = 96, 64
    np.random.seed(8)
    refs = [B.render_scene(sc, 2, seed=5, mt=True) for _ in range(3)]
    lib, ctxs = B.group()
    c0 = ctypes.c_void_p(ctxs[0])
    B.upload(sc, ctx=c0)
    cd = B.camera_desc(sc.camera)
    bufs = []
    for _ in range(3):
        pu, pr = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(lib, lib.srt_host_alloc(c0, 3 * W * H, ctypes.byref(pu)))
        N.check(lib, lib.srt_host_alloc(c0, 3 * W * H * 8, ctypes.byref(pr)))
        bufs.append((pu, pr))
    try:
        np.random.seed(8)
        mt = N.MtState.from_numpy()
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, H, 0
        a.rows, a.jitter, a.out_hit_id = None, None, None
        a.mt = ctypes.pointer(mt)
        a.seed = 5
        a.flags = N.RENDER_ASYNC | N.RENDER_RGB_ROWS
        for pu, pr in bufs:
            a.out_srgb8, a.out_rgb = pu, pr
            N.check(lib, lib.srt_render_group(ctxs, 1, ctypes.byref(cd), ctypes.byref(a), None))
        st = N.Stats()
        N.check(lib, lib.srt_render_group_finish(ctxs, 1, ctypes.byref(st)))
        assert st.as_dict()["total_rays"] == refs[-1].stats["total_rays"]
        for (pu, pr), ref in zip(bufs, refs):
            u8 = np.ctypeslib.as_array(ctypes.cast(pu, ctypes.POINTER(ctypes.c_uint8)), (H, W, 3)).copy()
            rgb = np.ctypeslib.as_array(ctypes.cast(pr, ctypes.POINTER(ctypes.c_double)), (3, W * H)).copy()
            assert np.array_equal(u8, ref.srgb8)
            assert np.array_equal(rgb, ref.rgb)
        np.random.seed(8)
        for _ in range(3):
            np.random.rand(3 * 4 * W * H)  # each frame: 2 samples + the sizing draw (scene.py:78-81)
        assert np.array_equal(np.random.get_state()[1], np.ctypeslib.as_array(mt.key))
        assert np.random.get_state()[2] == mt.pos
    finally:
        for pu, pr in bufs:
            lib.srt_host_free(c0, pu)
            lib.srt_host_free(c0, pr)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_gpu_every_shard_of_an_n_rank_frame_assembles_to_the_plain_render(world):
    """What each rank of an N-rank job renders (its 8-row bands, jitter read from the whole frame's
    numpy stream by global pixel), rendered here one shard after another on one card and assembled
    with the partition, equals the single-GPU frame; numpy's state advances identically."""
    import scenes
    from sightpy import _backend as B
    from sightpy._shard import shard_rows

    sc = scenes.example1(120, 64, 4)
    np.random.seed(21)
    full = B.render_scene(sc, 3, seed=5, mt=True)
    after = np.random.get_state()[1].copy()
    rgb = np.zeros((3, 64, 120))
    for q in range(world):
        rows = shard_rows(64, world, q)
        np.random.seed(21)
        part = B.render_scene(sc, 3, seed=5, mt=True, rows=rows)
        assert np.array_equal(np.random.get_state()[1], after)
        rgb[:, rows] = part.rgb.reshape(3, len(rows), 120)
    np.testing.assert_allclose(rgb.reshape(3, -1), full.rgb, rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("world,kmax", [(2, 8), (3, 8), (3, 3), (8, 2), (8, 17)])
def test_gpu_rgb_rows_shards_fill_the_shared_host_frame(world, kmax):
    """SRT_RENDER_RGB_ROWS (the multi-GPU bench's output path): each rank writes its own rows of the
    linear RGB into one host frame with pitched copies.  Rehearsed on one card (option
    rehearse_shard: act as rank r of N without a communicator): the N shards, rendered in turn into
    one pinned host frame, fill every row exactly once and equal the single-GPU frame."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N

    W, H, spp = 120, 70, 2  # 70 rows: a short last band
    sc = scenes.example1(W, H, 4)
    np.random.seed(4)
    full = B.render_scene(sc, spp, seed=5, mt=True)
    lib, ctx = B.context()
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    host = ctypes.c_void_p()
    N.check(lib, lib.srt_host_alloc(ctx, 3 * W * H * 8, ctypes.byref(host)))
    N.check(lib, lib.srt_set_option(ctx, b"shard_bands", kmax))
    try:
        frame = np.ctypeslib.as_array((ctypes.c_double * (3 * W * H)).from_address(host.value))
        frame[:] = np.nan
        for r in range(world):
            N.check(lib, lib.srt_set_option(ctx, b"rehearse_shard", (world << 8) | r))
            np.random.seed(4)
            st = N.MtState.from_numpy()
            a = N.RenderArgs()
            a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
            a.rows = a.jitter = a.out_srgb8 = a.out_hit_id = None
            a.mt = ctypes.pointer(st)
            a.seed = 5
            a.out_rgb = host
            a.flags = N.RENDER_SHARDED | N.RENDER_RGB_ROWS
            N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        N.check(lib, lib.srt_set_option(ctx, b"rehearse_shard", 0))
        assert not np.isnan(frame).any()
        assert np.array_equal(frame.reshape(3, -1), full.rgb)
    finally:
        lib.srt_set_option(ctx, b"rehearse_shard", 0)
        lib.srt_set_option(ctx, b"shard_bands", 0)  # back to the automatic choice
        lib.srt_host_free(ctx, host)


def _set_option(key, value):
    from sightpy import _backend as B, _native as N

    lib, ctx = B.context()
    N.check(lib, lib.srt_set_option(ctx, key.encode(), int(value)))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["multipass", "thin_lens", "odd_rows"])
def test_gpu_band_mode_stream_equals_tabulated_stream(case):
    """A shard's numpy stream in band mode (only its rows' runs generated, each jumped to from the
    key by a host-made polynomial; rt_mt_kernel.h MtArgs::bands) against the tabulated 2^19-word
    segments (option mt_bands=0), through several passes (full and last-pass band tables), a thin-lens
    camera (all four planes stored) and an arbitrary row set; numpy's state advances identically."""
    import scenes
    from sightpy import _backend as B
    from sightpy._shard import shard_rows

    W, H = 96, 72
    sc = scenes.example1(W, H, 3)
    spp, batch, rows = 2, None, shard_rows(H, 4, 1)
    if case == "multipass":
        spp, batch = 5, 2
    elif case == "thin_lens":
        sc.camera.lens_radius = 0.05
    else:
        rows = np.array([0, 1, 2, 9, 10, 33, 50, 51, 52, 53, 71])
    out, states = {}, {}
    try:
        for bands in (0, 1):
            _set_option("mt_bands", bands)
            np.random.seed(33)
            out[bands] = B.render_scene(sc, spp, seed=5, mt=True, rows=rows, batch_size=batch)
            states[bands] = np.random.get_state()
    finally:
        _set_option("mt_bands", 1)
    assert np.array_equal(out[0].rgb, out[1].rgb)
    assert np.array_equal(out[0].srgb8, out[1].srgb8)
    assert states[0][2] == states[1][2] and np.array_equal(states[0][1], states[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_gpu_async_band_mode_shard_frames_match_sync_frames(world):
    """Pipelined frames of one rank's shard (the multi-GPU bench loop, rehearsed on one card): in band
    mode each frame's key and its y words come from the previous frame's end block; every frame equals
    the synchronous shard render from the same numpy state, and the state after the sequence matches."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N
    from sightpy._shard import shard_rows

    W, H, K, spp = 160, 96, 5, 2
    sc = scenes.example1(W, H, 4)
    rows = shard_rows(H, world, world - 1)
    np.random.seed(9)
    ref = [B.render_scene(sc, spp, seed=5, mt=True, rows=rows) for _ in range(K)]
    want = np.random.get_state()
    lib, ctx = B.context()
    np.random.seed(9)
    mt = N.MtState.from_numpy()
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    hosts = []
    try:
        for k in range(K):
            h = ctypes.c_void_p()
            N.check(lib, lib.srt_host_alloc(ctx, 3 * W * H * 8, ctypes.byref(h)))
            hosts.append(h)
        N.check(lib, lib.srt_set_option(ctx, b"rehearse_shard", (world << 8) | (world - 1)))
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
        a.jitter, a.seed, a.out_hit_id, a.rows, a.out_srgb8 = None, 5, None, None, None
        a.mt = ctypes.pointer(mt)
        a.flags = N.RENDER_ASYNC | N.RENDER_SHARDED | N.RENDER_RGB_ROWS
        for k in range(K):
            a.out_rgb = hosts[k]
            N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        N.check(lib, lib.srt_render_finish(ctx, None))
        mt.to_numpy()
        got = np.random.get_state()
        assert got[2] == want[2] and np.array_equal(got[1], want[1])
        for k in range(K):
            frame = np.ctypeslib.as_array((ctypes.c_double * (3 * W * H)).from_address(hosts[k].value))
            mine = frame.reshape(3, H, W)[:, rows].reshape(3, -1)
            assert np.array_equal(mine, ref[k].rgb), "frame %d" % k
    finally:
        lib.srt_set_option(ctx, b"rehearse_shard", 0)
        for h in hosts:
            lib.srt_host_free(ctx, h)


@pytest.mark.gpu
def test_gpu_many_shard_shapes_keep_band_mode_exact():
    """More row sets than the context keeps band tables for (16): the tables are dropped between
    frames and rebuilt; every shard still equals the tabulated stream's render and numpy's state
    advances identically."""
    import scenes
    from sightpy import _backend as B
    from sightpy._shard import shard_rows

    W, H = 64, 80
    sc = scenes.example1(W, H, 3)
    cases = [(n, r) for n in (2, 3, 4, 5, 6, 7) for r in range(3) if r < n][:18]
    try:
        for n, r in cases:
            rows = shard_rows(H, n, r)
            out = {}
            for bands in (1, 0):
                _set_option("mt_bands", bands)
                np.random.seed(n * 10 + r)
                out[bands] = (B.render_scene(sc, 2, seed=5, mt=True, rows=rows), np.random.get_state()[1].copy())
            assert np.array_equal(out[0][0].rgb, out[1][0].rgb), (n, r)
            assert np.array_equal(out[0][1], out[1][1])
    finally:
        _set_option("mt_bands", 1)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_gpu_rehearsed_rank0_assembly_places_its_rows(world):
    """Option rehearse_assemble (bench.py --shard-of N --rehearse-assemble): rank 0's rows of an N-rank
    frame rendered on one card also run rank 0's k_assemble over its tile and N - 1 stand-in tiles
    (zeros) and hand back the whole frame: rank 0's rows equal the single-GPU frame's rows, every other
    row is the stand-ins' zeros.  Other rows sets (not rank 0's) hand back their own tile."""
    import ctypes

    import scenes
    from sightpy import _backend as B, _native as N
    from sightpy._shard import shard_rows

    W, H, spp = 160, 96, 2
    sc = scenes.example1(W, H, 3)
    np.random.seed(8)
    full = B.render_scene(sc, spp, seed=5, mt=True)
    lib, ctx = B.context()
    N.check(lib, lib.srt_set_option(ctx, b"rehearse_assemble", world))
    try:
        rows0 = shard_rows(H, world, 0)
        np.random.seed(8)
        B.upload(sc)
        cd = B.camera_desc(sc.camera)
        r32 = np.ascontiguousarray(rows0, dtype=np.int32)
        mt = N.MtState.from_numpy()
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, len(r32), 0
        a.rows, a.jitter, a.out_hit_id, a.seed = N.ptr(r32), None, None, 5
        a.mt = ctypes.pointer(mt)
        out = B.pinned_buffer("rehearse_u8", 3 * W * H)
        out[:] = 7
        a.out_srgb8, a.out_rgb = out.ctypes.data, None
        a.flags = N.RENDER_ASYNC | N.RENDER_RGB_LOCAL
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        N.check(lib, lib.srt_render_finish(ctx, None))
        img = out.reshape(H, W, 3).copy()
        mask = np.zeros(H, dtype=bool)
        mask[rows0] = True
        assert np.array_equal(img[mask], full.srgb8[mask])
        assert not img[~mask].any()
        # rank 1's rows: no assembly, its own tile
        rows1 = shard_rows(H, world, 1)
        np.random.seed(8)
        part = B.render_scene(sc, spp, seed=5, mt=True, rows=rows1)
        assert np.array_equal(part.srgb8, full.srgb8[rows1])
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"rehearse_assemble", 0))
