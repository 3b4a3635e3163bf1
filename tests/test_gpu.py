"""GPU parity tests: the HIP path (libsightpy_hip.so through the C ABI) against the reference
fixtures, the oracle, and size-independent properties at the BASELINE sizes.

Bar: primary hit-id masks exact; linear RGB within 1e-5 relative (north_star tolerance, with a
1e-12 absolute floor for near-black values); uint8 images equal up to rare +-1 at rounding
boundaries (transcendental ulps differ between numpy's SIMD libm and the device libm)."""
import numpy as np
import pytest

import scenes
import sightpy_oracle as O
from conftest import golden
from test_oracle import kat_colliders, DETERMINISTIC

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-5, 1e-12


def _backend():
    from sightpy import _backend

    return _backend


def _close_u8(a, b):
    d = np.abs(a.astype(int) - b.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())


def test_library_loads_on_gpu():
    lib, ctx = _backend().context()
    assert ctx.value


@pytest.mark.parametrize("name", ["sphere", "plane", "plane_tilted", "cuboid_rot30", "cuboid_axis", "triangle"])
def test_gpu_collider_kat(name):
    from sightpy import vec3

    g = golden("colliders")
    c = kat_colliders()[name]
    out = c.intersect(vec3(*g["O"]), vec3(*g["D"]))  # Collider.intersect -> srt_intersect_collider
    assert np.array_equal(out, g[name], equal_nan=True)


def test_gpu_camera_rays_exact():
    g = golden("camera")
    sc = scenes.example1(64, 48)
    np.random.seed(0)
    j = sc.camera.draw_jitter(1)[0]
    Og, Dg = _backend().primary_rays(sc.camera, j)
    assert np.array_equal(np.stack([Og.x, Og.y, Og.z]), g["O"])
    assert np.array_equal(np.stack([Dg.x, Dg.y, Dg.z]), g["D"])


@pytest.mark.parametrize("name,builder,depth", DETERMINISTIC)
def test_gpu_examples_match_reference(name, builder, depth):
    g = golden(name)
    W, H, spp = int(g["width"]), int(g["height"]), int(g["spp"])
    sc = builder(W, H, depth)
    np.random.seed(int(g["seed"]))
    jit = sc.camera.draw_jitter(spp)
    out = _backend().render_scene(sc, spp, jitter=jit, seed=1, want_hits=True)
    assert np.array_equal(out.hit_ids, g["hit_id"])
    assert out.stats["rays_per_depth"][: len(g["depth_counts"])] == g["depth_counts"].tolist()
    np.testing.assert_allclose(out.rgb, g["rgb"], rtol=RTOL, atol=ATOL)
    _close_u8(out.srgb8, g["srgb8"])


def test_gpu_example1_plumbing_config_400x300():
    g = golden("ex1_400x300_d3_s6")
    sc = scenes.example1(400, 300)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(6)
    out = _backend().render_scene(sc, 6, jitter=jit, seed=1, want_hits=True)
    assert np.array_equal(out.hit_ids, g["hit_id"])
    assert out.stats["rays_per_depth"][:4] == g["depth_counts"].tolist()
    np.testing.assert_allclose(out.rgb, g["rgb"].astype(np.float64), rtol=RTOL, atol=1e-9)
    _close_u8(out.srgb8, g["srgb8"])


def test_scene_render_api_matches_reference_image():
    # Scene.render draws the jitter from numpy's global RNG like the reference (+ the extra draw)
    g = golden("ex1_64x48_d3_s2")
    sc = scenes.example1(64, 48)
    np.random.seed(0)
    img = sc.render(samples_per_pixel=2)
    _close_u8(np.asarray(img), g["srgb8"])
    assert np.random.rand() == _rng_after(0, 2, 64 * 48)


def _rng_after(seed, spp, n):
    np.random.seed(seed)
    np.random.rand((spp + 1) * 4 * n)
    return np.random.rand()


def test_get_raycolor_dropin_matches_oracle():
    from sightpy import Ray, get_raycolor, vec3

    sc = scenes.example3(48, 36, 6)
    np.random.seed(4)
    jit = sc.camera.draw_jitter(1)[0]
    Oo, Do = O.primary_rays(sc.camera, jit)
    ray = Ray(vec3(*np.broadcast_to(Oo, Do.shape)), vec3(*Do), 0, sc.n, 0, 0, 0)
    col = get_raycolor(ray, sc)
    ref = O.raycolor(sc, O.Rays(np.broadcast_to(Oo, Do.shape), Do, O.scene_medium(sc), 0), {})
    np.testing.assert_allclose(np.stack([col.x, col.y, col.z]), ref, rtol=RTOL, atol=ATOL)
    # a secondary batch (depth 2, inside-glass medium) through the same entry point
    ray2 = Ray(vec3(*np.broadcast_to(Oo, Do.shape)), vec3(*Do), 2, vec3(1.5 + 4e-8j, 1.5 + 0j, 1.5 + 4e-8j), 0, 0, 0)
    col2 = get_raycolor(ray2, sc)
    n2 = np.array([[1.5 + 4e-8j], [1.5 + 0j], [1.5 + 4e-8j]])
    ref2 = O.raycolor(sc, O.Rays(np.broadcast_to(Oo, Do.shape), Do, n2, 2), {})
    np.testing.assert_allclose(np.stack([col2.x, col2.y, col2.z]), ref2, rtol=RTOL, atol=ATOL)


def test_get_distances_matches_oracle():
    sc = scenes.example1(64, 48)
    np.random.seed(2)
    img = np.asarray(sc.get_distances())
    np.random.seed(2)
    jit = sc.camera.draw_jitter(1)[0]
    Oo, Do = O.primary_rays(sc.camera, jit)
    near, _ = O.nearest(sc, np.broadcast_to(Oo, Do.shape), Do)
    g = np.where(near <= 10, near, 10) / 10
    ref = (255 * np.clip(g, 0, 1).reshape(48, 64)).astype(np.uint8)
    assert np.array_equal(img[..., 0], ref)


def test_cornell_monte_carlo_deterministic():
    """(Sample-for-sample parity of the MC paths: tests/test_gpu_mc.py.)  The primary hit ids match
    the reference's fixture, and the device RNG is deterministic: identical seeds, identical images."""
    g = golden("cornell_24x24_s1")
    sc = scenes.cornell(24, 24)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(16)
    out = _backend().render_scene(sc, 16, jitter=jit, seed=3, want_hits=True)
    assert np.array_equal(out.hit_ids[0], g["hit_id"][0])
    out2 = _backend().render_scene(sc, 16, jitter=jit, seed=3)
    np.testing.assert_allclose(out2.rgb, out.rgb, rtol=1e-12, atol=1e-12)


def test_thinfilm_index_error_like_reference():
    # cos(theta_i) == 1 indexes row 400 of the 400-row table: the reference raises IndexError
    from sightpy import Ray, get_raycolor, vec3

    sc = scenes.example4(16, 12, 6)
    c = sc.collider_list[0]
    o = vec3(np.array([c.center.x - 5.0]), np.array([c.center.y]), np.array([c.center.z]))
    d = vec3(np.array([1.0]), np.array([0.0]), np.array([0.0]))
    with pytest.raises(IndexError):
        get_raycolor(Ray(o, d, 0, sc.n, 0, 0, 0), sc)


# ---- BASELINE sizes: size-independent properties -------------------------------------------
def test_example1_1080p_d5_properties():
    """At the headline config: exact hit ids vs the oracle (one sample), per-depth counts vs the
    reference's published counts, and sample linearity (2-sample render == mean of 1-sample ones)."""
    sc = scenes.example1(1920, 1080, 5)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(2)
    be = _backend()
    full = be.render_scene(sc, 2, jitter=jit, seed=1, want_hits=True)
    a = be.render_scene(sc, 1, jitter=jit[:1], seed=1)
    b = be.render_scene(sc, 1, jitter=jit[1:], seed=1)
    np.testing.assert_allclose(full.rgb, (a.rgb + b.rgb) / 2, rtol=1e-12, atol=1e-14)
    Oo, Do = O.primary_rays(sc.camera, jit[0])
    _, ids = O.hit_ids(sc, np.broadcast_to(Oo, Do.shape), Do)
    assert np.array_equal(full.hit_ids[0], ids)
    # row shards render the same pixels as the full frame (multi-GPU partitioning)
    rows = np.arange(3, 1080, 8)
    shard = be.render_scene(sc, 2, jitter=jit.reshape(2, 4, 1080, 1920)[:, :, rows].reshape(2, 4, -1), seed=1,
                            rows=rows)
    np.testing.assert_allclose(shard.rgb, full.rgb.reshape(3, 1080, 1920)[:, rows].reshape(3, -1), rtol=1e-12,
                               atol=1e-14)


@pytest.mark.parametrize("builder,depth,spp,seed", [(scenes.example1, 5, 2, 0), (scenes.example3, 8, 1, 0)],
                         ids=["example1_1080p_d5_2spp", "example3_1080p_d8_1spp"])
def test_headline_configs_1080p_rgb_match_oracle(builder, depth, spp, seed):
    """Full-size RGB parity at the BASELINE headline configurations (1920x1080): hit ids exact,
    per-depth ray counts equal, linear RGB within 1e-5 relative of the oracle on the same jitter."""
    sc = builder(1920, 1080, depth)
    np.random.seed(seed)
    jit = sc.camera.draw_jitter(spp)
    out = _backend().render_scene(sc, spp, jitter=jit, seed=1, want_hits=True)
    rgb, ids, counts = O.render_linear(sc, jit)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)
    _close_u8(out.srgb8, O.srgb_u8(rgb, 1080, 1920))


def test_headline_frame_through_the_bench_path_matches_oracle():
    """The exact headline frame (BASELINE configs[1]: example1 1920x1080, depth 5, 6 spp) through the
    bench's own path -- numpy's stream generated on the GPU from a seeded numpy state, pipelined
    (SRT_RENDER_ASYNC) frames into pinned host buffers, the fused kernel's in-kernel resolve -- against
    the oracle on the same numpy draws (reference scene.py:71-140, example1.py:73).  The second of two
    pipelined frames is checked (its key window comes from the first frame's end jump): linear RGB
    within a pure 1e-5 relative bound on every value (no absolute floor), uint8 within +-1 at < 0.1 %
    of the pixels, primary hit ids exact (a synchronous re-render from the same numpy state with hit
    ids requested, equal to the pipelined frame bit for bit), per-depth ray counts equal, and numpy's
    state advanced past both frames' sizing draws (scene.py:81)."""
    import ctypes
    from sightpy import _native as N
    from oracle_pool import render_linear_pool

    B = _backend()
    W, H, D, spp, npix = 1920, 1080, 5, 6, 1920 * 1080
    sc = scenes.example1(W, H, D)
    # the reference's draws: per frame 6 samples x (x, y, disk r, disk phi), then one sizing get_ray
    np.random.seed(0)
    state0 = np.random.get_state()
    sc.camera.draw_jitter(spp)
    sc.camera.draw_jitter(1)
    state1 = np.random.get_state()
    jit2 = sc.camera.draw_jitter(spp)
    sc.camera.draw_jitter(1)
    state2 = np.random.get_state()

    lib, ctx = B.context()
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    N.check(lib, lib.srt_set_option(ctx, b"pipeline", 1))
    outs = []
    try:
        for _ in range(2):
            pu, pr = ctypes.c_void_p(), ctypes.c_void_p()
            N.check(lib, lib.srt_host_alloc(ctx, 3 * npix, ctypes.byref(pu)))
            N.check(lib, lib.srt_host_alloc(ctx, 3 * npix * 8, ctypes.byref(pr)))
            outs.append((pu, pr))
        np.random.set_state(state0)
        mt = N.MtState.from_numpy()
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, H, 0
        a.rows, a.jitter, a.out_hit_id = None, None, None
        a.mt = ctypes.pointer(mt)
        a.seed = 12345
        a.flags = N.RENDER_ASYNC
        for pu, pr in outs:
            a.out_srgb8, a.out_rgb = pu, pr
            N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
        st = N.Stats()
        N.check(lib, lib.srt_render_finish(ctx, ctypes.byref(st)))
        st = st.as_dict()
        assert st["kernel_path"] == "fused"
        mt.to_numpy()
        got = np.random.get_state()
        assert got[2] == state2[2] and np.array_equal(got[1], state2[1])
        u8 = np.ctypeslib.as_array(ctypes.cast(outs[1][0], ctypes.POINTER(ctypes.c_uint8)), (H, W, 3)).copy()
        rgb = np.ctypeslib.as_array(ctypes.cast(outs[1][1], ctypes.POINTER(ctypes.c_double)), (3, npix)).copy()
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"pipeline", 0))
        for pu, pr in outs:
            lib.srt_host_free(ctx, pu)
            lib.srt_host_free(ctx, pr)
    # the same frame again, synchronously, with the primary hit ids
    np.random.set_state(state1)
    again = B.render_scene(sc, spp, seed=12345, mt=True, want_hits=True)
    assert np.array_equal(again.rgb, rgb) and np.array_equal(again.srgb8, u8)
    ref, ids, counts = render_linear_pool("example1", W, H, D, jit2)
    assert np.array_equal(again.hit_ids, ids)
    assert st["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    nz = ref != 0.0
    assert np.all(rgb[~nz] == 0.0)
    rel = np.abs(rgb[nz] - ref[nz]) / np.abs(ref[nz])
    assert rel.max() <= RTOL, rel.max()
    _close_u8(u8, O.srgb_u8(ref, H, W))


def test_example1_1080p_d5_ray_counts_match_reference_survey():
    # seed 0, 6 spp -> rays per depth measured with the reference
    sc = scenes.example1(1920, 1080, 5)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(6)
    out = _backend().render_scene(sc, 6, jitter=jit, seed=1)
    assert out.stats["rays_per_depth"] == [12441600, 6413569, 1326285, 537874, 163811, 95648]


def test_gpu_lane_stats_count_the_depth_loop():
    """srt_debug_lane_stats on the headline frame's lean kernel (its counting instantiation): the live
    lanes of each depth are exactly the rays entering that depth (the reference's per-depth counts),
    depth 0 runs one wave iteration per 32 pixels x 3 samples (two sample groups), and the image is
    the non-counting kernel's bit for bit."""
    import ctypes
    from sightpy import _native as N

    sc = scenes.example1(1920, 1080, 5)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(6)
    lib, ctx = _backend().context()
    N.check(lib, lib.srt_set_option(ctx, b"sync_lean", 1))
    raw = (ctypes.c_int64 * 32)()
    try:
        plain = _backend().render_scene(sc, 6, jitter=jit, seed=1)
        N.check(lib, lib.srt_debug_lane_stats(ctx, 1, None, 0))
        out = _backend().render_scene(sc, 6, jitter=jit, seed=1)
        N.check(lib, lib.srt_debug_lane_stats(ctx, 0, raw, 16))
    finally:
        N.check(lib, lib.srt_set_option(ctx, b"sync_lean", 0))
    assert out.stats["kernel_path"] == "fused"
    assert np.array_equal(out.rgb, plain.rgb) and np.array_equal(out.srgb8, plain.srgb8)
    rpd = out.stats["rays_per_depth"]
    assert [raw[2 * d + 1] for d in range(len(rpd))] == rpd
    assert raw[0] == 1920 * 1080 // 32 * 3
    for d in range(len(rpd)):
        assert 64 * raw[2 * d] >= raw[2 * d + 1] > 0
    assert raw[2 * len(rpd)] == 0
    assert lib.srt_debug_lane_stats(ctx, 0, raw, 16) != 0  # (stopped: nothing to read)


def test_example3_1080p_d8_counts_match_reference_survey():
    sc = scenes.example3(1920, 1080, 8)
    np.random.seed(0)
    jit = sc.camera.draw_jitter(4)
    out = _backend().render_scene(sc, 4, jitter=jit, seed=1)
    assert out.stats["rays_per_depth"] == [8294400, 4847603, 2862842, 2874155, 2799708, 2840696, 2741719,
                                           2752695, 2692499]


def _set_option(key, value):
    import ctypes

    lib, ctx = _backend().context()
    rc = lib.srt_set_option(ctx, key.encode(), ctypes.c_int64(value))
    assert rc == 0, lib.srt_last_error()


@pytest.mark.parametrize("name,builder,depth", DETERMINISTIC)
@pytest.mark.parametrize("mode", ["wavefront", "wavefront+chain", "frame", "fused"])
def test_gpu_every_kernel_path_matches_reference(name, builder, depth, mode):
    """Every example through each trace strategy, whatever the automatic choice would be: the
    per-depth wavefront kernels, the same with chain mode from depth 2 (the second render of a
    shape; single-child scenes only), the frame kernel, and the fused paths (every depth of a
    single-child scene in k_primary)."""
    g = golden(name)
    W, H, spp = int(g["width"]), int(g["height"]), int(g["spp"])
    sc = builder(W, H, depth)
    np.random.seed(int(g["seed"]))
    jit = sc.camera.draw_jitter(spp)
    _set_option("frame_kernel", 1 if mode == "frame" else 0)
    _set_option("chain_rays", 1 << 40 if mode == "wavefront+chain" else 0)
    _set_option("fuse_primary", 1 if mode == "fused" else 0)
    try:
        B = _backend()
        for _ in range(2 if mode == "wavefront+chain" else 1):
            out = B.render_scene(sc, spp, jitter=jit, seed=1, want_hits=True)
    finally:
        _set_option("frame_kernel", -1)
        _set_option("chain_rays", 1000000)
        _set_option("fuse_primary", -1)
    if mode == "fused" and builder is scenes.example1:
        assert out.stats["kernel_path"] == "fused"
    assert np.array_equal(out.hit_ids, g["hit_id"])
    assert out.stats["rays_per_depth"][: len(g["depth_counts"])] == g["depth_counts"].tolist()
    np.testing.assert_allclose(out.rgb, g["rgb"], rtol=RTOL, atol=ATOL)
    _close_u8(out.srgb8, g["srgb8"])


def test_gpu_async_frames_match_sync_frame():
    """SRT_RENDER_ASYNC frames (pipelined, device outputs) equal a synchronous render."""
    import ctypes
    from sightpy import _native as N

    B = _backend()
    sc = scenes.example1(160, 120, 4)
    np.random.seed(3)
    jit = np.ascontiguousarray(sc.camera.draw_jitter(2))
    ref = B.render_scene(sc, 2, jitter=jit, seed=5)
    lib, ctx = B.context()
    npix = 160 * 120
    dj = B.device_buffer("test_jit", jit.nbytes)
    N.check(lib, lib.srt_memcpy(ctx, dj, N.ptr(jit), jit.nbytes))
    drgb = B.device_buffer("test_rgb", 3 * npix * 8)
    du8 = B.device_buffer("test_u8", 3 * npix)
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, 120, 0
    a.jitter, a.seed, a.out_rgb, a.out_srgb8, a.out_hit_id = dj, 5, drgb, du8, None
    a.flags = N.RENDER_ASYNC
    cd = B.camera_desc(sc.camera)
    st = N.Stats()
    for _ in range(4):
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
    N.check(lib, lib.srt_render_finish(ctx, ctypes.byref(st)))
    rgb = np.empty((3, npix))
    u8 = np.empty((npix, 3), dtype=np.uint8)
    N.check(lib, lib.srt_memcpy(ctx, N.ptr(rgb), drgb, rgb.nbytes))
    N.check(lib, lib.srt_memcpy(ctx, N.ptr(u8), du8, u8.nbytes))
    assert st.as_dict()["total_rays"] == ref.stats["total_rays"]
    assert np.array_equal(rgb, ref.rgb)  # (order-independent framebuffer sums: bit-identical)
    assert np.array_equal(u8.reshape(120, 160, 3), ref.srgb8)


def test_gpu_frames_are_bit_reproducible():
    """The reference is deterministic; so are these frames: depth-0 colours are summed in the pixel's
    own thread and every other contribution goes into an order-independent fixed-point sum, so
    repeated renders, a render whose depths run in chain mode, and the split-sample path of small
    frames give bit-identical linear RGB."""
    B = _backend()
    sc = scenes.example1(160, 120, 5)
    np.random.seed(2)
    jit = sc.camera.draw_jitter(3)
    a = B.render_scene(sc, 3, jitter=jit, seed=5)
    b = B.render_scene(sc, 3, jitter=jit, seed=5)  # (same shape: chain mode from the hinted depth)
    assert np.array_equal(a.rgb, b.rgb) and np.array_equal(a.srgb8, b.srgb8)
    _set_option("chain_rays", 0)
    try:
        c = B.render_scene(sc, 3, jitter=jit, seed=5)
    finally:
        _set_option("chain_rays", 1000000)
    assert np.array_equal(a.rgb, c.rgb)
    small = scenes.example1(40, 30, 5)
    jit_s = small.camera.draw_jitter(8)
    d = B.render_scene(small, 8, jitter=jit_s, seed=5)  # split samples: depth-0 sums also fixed point
    e = B.render_scene(small, 8, jitter=jit_s, seed=5)
    assert np.array_equal(d.rgb, e.rgb)


def test_gpu_colour_beyond_fixed_point_range_falls_back_to_f64_sums():
    """A contribution of magnitude >= 2^17 (here a very bright Emissive dome seen in the floor's
    reflection) does not fit the fixed-point framebuffer sums: the frame is rendered again with f64
    atomics, and the result still matches the oracle."""
    from sightpy import Emissive, Sphere, rgb, vec3

    B = _backend()
    sc = scenes.example1(48, 36, 3)
    sc.add(Sphere(material=Emissive(color=rgb(1e7, 1e7, 1e7)), center=vec3(0.0, 60.0, -3.0), radius=55.0,
                  shadow=False, max_ray_depth=3))
    np.random.seed(6)
    jit = sc.camera.draw_jitter(2)
    out = B.render_scene(sc, 2, jitter=jit, seed=1)
    assert out.stats["retries"] >= 1
    rgb_o, ids, counts = O.render_linear(sc, jit)
    np.testing.assert_allclose(out.rgb, rgb_o, rtol=RTOL, atol=ATOL)


def test_gpu_fixed_point_sums_near_wrap_fall_back_to_f64_sums():
    """Every contribution below the per-term limit (2^17), but a pixel's reflected contributions
    summing past the coarse magnitude limit (rt_kernels.hip FX_MAG_LIMIT, the guard against a
    fixed-point sum wrapping): the frame is rendered again with f64 atomics and matches the oracle."""
    from sightpy import Emissive, Sphere, rgb, vec3

    B = _backend()
    sc = scenes.example1(48, 36, 3)
    sc.add(Sphere(material=Emissive(color=rgb(3e4, 3e4, 3e4)), center=vec3(0.0, 60.0, -3.0), radius=55.0,
                  shadow=False, max_ray_depth=3))
    np.random.seed(6)
    jit = sc.camera.draw_jitter(2)
    out = B.render_scene(sc, 2, jitter=jit, seed=1)
    assert out.stats["retries"] >= 1
    rgb_o, ids, counts = O.render_linear(sc, jit)
    np.testing.assert_allclose(out.rgb, rgb_o, rtol=RTOL, atol=ATOL)


def _bright_light_example1(W, H, depth, color):
    """example1 with a second DirectionalLight of the given colour: a Glossy-only scene (the
    glossy+sky kernel variant, which has the fused paths) whose reflected terms can leave the
    fixed-point range."""
    from sightpy import rgb, vec3

    sc = scenes.example1(W, H, depth)
    sc.add_DirectionalLight(Ldir=vec3(-0.3, 0.8, -0.2), color=rgb(color, color, color))
    return sc


@pytest.mark.parametrize("color", [1e6, 3e4], ids=["term_beyond_2^17", "sum_past_magnitude_limit"])
def test_gpu_fused_path_leaves_fixed_point_range_and_falls_back(color):
    """The fused paths (every depth in k_primary) with terms beyond the fixed-point range: each
    term is checked as fb_add checks it (|term| < 2^17, else left out of the sums and flagged
    through the independent magnitude), the frame is rendered again with every depth summed in
    the pixel's thread in f64, and matches the oracle."""
    B = _backend()
    sc = _bright_light_example1(64, 48, 4, color)
    np.random.seed(11)
    jit = sc.camera.draw_jitter(3)
    _set_option("fuse_primary", 1)
    try:
        out = B.render_scene(sc, 3, jitter=jit, seed=1)
        again = B.render_scene(sc, 3, jitter=jit, seed=1)  # (fixed-point sums now off for this scene)
    finally:
        _set_option("fuse_primary", -1)
    assert out.stats["kernel_path"] == "fused" and again.stats["kernel_path"] == "fused"
    assert out.stats["retries"] >= 1
    rgb_o, ids, counts = O.render_linear(sc, jit)
    np.testing.assert_allclose(out.rgb, rgb_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(again.rgb, rgb_o, rtol=RTOL, atol=ATOL)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]


def test_gpu_fused_path_without_fixed_point_sums_keeps_every_depth():
    """Option deterministic=0 (f64 sums) on the fused paths: the deeper depths' colour goes into the
    pixel's register sum, stored once with the depth-0 colour (an atomic add into the
    framebuffer there was overwritten by the single-pass store, dropping the reflections)."""
    B = _backend()
    sc = scenes.example1(160, 120, 5)
    np.random.seed(12)
    jit = sc.camera.draw_jitter(2)
    _set_option("fuse_primary", 1)
    _set_option("deterministic", 0)
    try:
        out = B.render_scene(sc, 2, jitter=jit, seed=1)
    finally:
        _set_option("deterministic", 1)
        _set_option("fuse_primary", -1)
    assert out.stats["kernel_path"] == "fused"
    rgb_o, ids, counts = O.render_linear(sc, jit)
    np.testing.assert_allclose(out.rgb, rgb_o, rtol=RTOL, atol=ATOL)


def test_gpu_point_light_raises_name_error_like_reference():
    """PointLight.get_L reads undefined names (reference lights.py:30-31): the reference's render
    raises NameError at the first Glossy hit.  So does this one; a scene whose rays never reach a
    Glossy surface never consults the light and renders."""
    from sightpy import rgb, vec3

    sc = scenes.example1(32, 24, 2)
    sc.add_PointLight(pos=vec3(0.0, 2.0, -3.0), color=rgb(1.0, 1.0, 1.0))
    np.random.seed(0)
    with pytest.raises(NameError):
        sc.render(samples_per_pixel=1)
    cb = scenes.cornell(16, 16)  # Diffuse / Emissive / Refractive only
    cb.add_PointLight(pos=vec3(0.0, 0.2, 0.0), color=rgb(1.0, 1.0, 1.0))
    np.random.seed(0)
    img = cb.render(samples_per_pixel=1)
    assert np.asarray(img).shape == (16, 16, 3)


def test_gpu_group_render_retries_a_frame_on_every_context():
    """srt_render_group (Scene.render over $SIGHTPY_DEVICES) renders a frame that left the
    fixed-point range again on every context, as the single-GPU path does, instead of failing."""
    from sightpy import Emissive, Sphere, rgb, vec3

    B = _backend()
    sc = scenes.example1(48, 40, 3)
    sc.add(Sphere(material=Emissive(color=rgb(1e7, 1e7, 1e7)), center=vec3(0.0, 60.0, -3.0), radius=55.0,
                  shadow=False, max_ray_depth=3))
    np.random.seed(9)
    ref = B.render_scene(sc, 2, seed=3, mt=True)
    assert ref.stats["retries"] >= 1
    np.random.seed(9)
    import os

    old = os.environ.get("SIGHTPY_DEVICES")
    os.environ["SIGHTPY_DEVICES"] = str(B.devices()[0])
    try:
        got = B.render_group(sc, 2, seed=3, mt=True)
    finally:
        if old is None:
            os.environ.pop("SIGHTPY_DEVICES")
        else:
            os.environ["SIGHTPY_DEVICES"] = old
    np.testing.assert_allclose(got.rgb, ref.rgb, rtol=1e-12, atol=1e-6)
    assert got.stats["total_rays"] == ref.stats["total_rays"]


def test_gpu_async_numpy_stream_frames_match_sync_frames():
    """Pipelined frames drawing numpy's stream on the device (the bench's frame loop): each frame's key
    window comes from the previous frame's end jump (k_mt_jump's last block) while that frame's
    generators still run.  Every frame equals the synchronous render from the same numpy state, and
    numpy's state after the sequence equals the state after the synchronous frames."""
    import ctypes
    from sightpy import _native as N

    B = _backend()
    sc = scenes.example1(160, 120, 4)
    K, spp, npix = 5, 2, 160 * 120
    np.random.seed(7)
    ref = [B.render_scene(sc, spp, seed=5, mt=True) for _ in range(K)]
    want_state = np.random.get_state()
    np.random.seed(7)
    mt = N.MtState.from_numpy()
    lib, ctx = B.context()
    B.upload(sc)
    cd = B.camera_desc(sc.camera)
    bufs = [(B.device_buffer("mt_rgb%d" % k, 3 * npix * 8), B.device_buffer("mt_u8%d" % k, 3 * npix)) for k in range(K)]
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, 120, 0
    a.jitter, a.seed, a.out_hit_id, a.rows = None, 5, None, None
    a.mt = ctypes.pointer(mt)
    a.flags = N.RENDER_ASYNC
    for k in range(K):
        a.out_rgb, a.out_srgb8 = bufs[k]
        N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
    N.check(lib, lib.srt_render_finish(ctx, None))
    mt.to_numpy()
    got_state = np.random.get_state()
    assert got_state[2] == want_state[2] and np.array_equal(got_state[1], want_state[1])
    for k in range(K):
        rgb = np.empty((3, npix))
        N.check(lib, lib.srt_memcpy(ctx, N.ptr(rgb), bufs[k][0], rgb.nbytes))
        assert np.array_equal(rgb, ref[k].rgb)


@pytest.mark.parametrize("mode", ["wavefront", "frame", "fused"])
def test_gpu_triangle_mesh_bvh_matches_oracle(tmp_path, mode):
    """TriangleMesh through the device BVH (320 triangles + a tie-making duplicate set) against the
    oracle's linear loop over the collider list: hit ids exact, per-depth counts, RGB -- per-depth
    kernels, the frame kernel, and the fused single-child paths (the glossy BVH variant)."""
    for dup in (0, 12):
        path = str(tmp_path / ("ico%d.obj" % dup))
        scenes.write_icosphere_obj(path, subdiv=2, duplicate_faces=dup)
        sc = scenes.mesh_scene(path, 48, 36, 3)
        np.random.seed(9)
        jit = sc.camera.draw_jitter(2)
        _set_option("frame_kernel", 1 if mode == "frame" else 0)
        _set_option("fuse_primary", 1 if mode == "fused" else 0)
        try:
            out = _backend().render_scene(sc, 2, jitter=jit, seed=1, want_hits=True)
        finally:
            _set_option("frame_kernel", -1)
            _set_option("fuse_primary", -1)
        rgb, ids, counts = O.render_linear(sc, jit)
        assert np.array_equal(out.hit_ids, ids)
        assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
        np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)


def test_gpu_mesh_nearest_matches_oracle(tmp_path):
    import test_mesh

    path = str(tmp_path / "ico.obj")
    scenes.write_icosphere_obj(path, subdiv=3)
    sc = scenes.mesh_scene(path)
    Oa, Da = test_mesh._probe_rays(sc, np.random.default_rng(3), n=20000)
    from sightpy import vec3

    t, ids, orient = _backend().nearest_hits(sc, vec3(*Oa), vec3(*Da))
    near, ref = O.hit_ids(sc, Oa, Da)
    assert np.array_equal(ids, ref)
    hit = ref >= 0
    assert np.array_equal(t[hit], near[hit])


def test_gpu_bvh_f32_box_test_is_conservative(tmp_path):
    """The device's f32 BVH box test (NaN-disabled axes, the widened entry / exit) on rays at its
    error bound (test_mesh._box_edge_rays): the same nearest hits as the oracle's linear loop."""
    import test_mesh

    path = str(tmp_path / "ico.obj")
    scenes.write_icosphere_obj(path, subdiv=3)
    sc = scenes.mesh_scene(path)
    Oa, Da = test_mesh._box_edge_rays(sc, np.random.default_rng(29))
    from sightpy import vec3

    t, ids, orient = _backend().nearest_hits(sc, vec3(*Oa), vec3(*Da))
    near, ref = O.hit_ids(sc, Oa, Da)
    assert np.array_equal(ids, ref)
    hit = ref >= 0
    assert np.array_equal(t[hit], near[hit])
    assert hit.mean() > 0.3


def test_gpu_bvh_f32_box_test_tiny_mesh(tmp_path):
    """A mesh ~1e-2 across at the origin and direction components ~1e-39 (f32(1/D) overflows while
    the 1e37 guard passes: test_mesh._tiny_mesh_rays): the device's nearest hits equal the oracle's."""
    import test_mesh

    path = str(tmp_path / "ico_tiny.obj")
    scenes.write_icosphere_obj(path, subdiv=3, radius=5e-3)
    sc = scenes.mesh_scene(path, center=(0.0, 0.0, 0.0))
    Oa, Da = test_mesh._tiny_mesh_rays(sc, np.random.default_rng(37))
    from sightpy import vec3

    t, ids, orient = _backend().nearest_hits(sc, vec3(*Oa), vec3(*Da))
    near, ref = O.hit_ids(sc, Oa, Da)
    assert np.array_equal(ids, ref)
    hit = ref >= 0
    assert np.array_equal(t[hit], near[hit])
    assert (ref >= 1).mean() > 0.3


def test_gpu_create_animation_frames(tmp_path, monkeypatch):
    """create_animation (persistent device scene, background frame writer) writes the same frames
    as rendering them one by one."""
    from PIL import Image
    from sightpy import create_animation, vec3

    monkeypatch.chdir(tmp_path)

    def update(scene, t):
        scene.collider_list[0].center = vec3(-0.75 + t, 0.1, -3.0)

    sc = scenes.example1(48, 36, 3)
    np.random.seed(4)
    create_animation(sc, 1, 3, 0.0, 1.0, update, "anim")
    sc2 = scenes.example1(48, 36, 3)
    np.random.seed(4)
    t = 0.0
    for i in range(3):
        update(sc2, t)
        ref = np.array(sc2.render(1))
        got = np.array(Image.open(tmp_path / "frames" / ("anim_%d.png" % i)))
        assert np.array_equal(got, ref), i
        t += 1.0 / 3


@pytest.mark.parametrize("mode", ["wavefront", "frame"])
@pytest.mark.parametrize("shape", [(1, 1), (67, 13), (13, 67), (129, 3)])
def test_gpu_edge_shapes_match_oracle(shape, mode):
    """Frame shapes that leave partial waves / blocks / tiles everywhere (1x1, odd sizes) through
    both trace strategies, against the oracle on the same jitter."""
    W, H = shape
    sc = scenes.example1(W, H, 3)
    np.random.seed(2)
    jit = sc.camera.draw_jitter(3)
    _set_option("frame_kernel", 1 if mode == "frame" else 0)
    try:
        out = _backend().render_scene(sc, 3, jitter=jit, seed=1, want_hits=True)
    finally:
        _set_option("frame_kernel", -1)
    rgb, ids, counts = O.render_linear(sc, jit)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("which", ["no_background", "background_only"])
def test_gpu_degenerate_scenes(which):
    """Rays that miss everything (no SkyBox: black, ray.py:134-146) and a scene with nothing but the
    background."""
    from sightpy import Scene, rgb as RGB, vec3

    if which == "no_background":
        sc = scenes.example1(40, 30, 3)
        sc.collider_list = [c for c in sc.collider_list if type(c.assigned_primitive).__name__ != "SkyBox"]
        sc.scene_primitives = [p for p in sc.scene_primitives if type(p).__name__ != "SkyBox"]
    else:
        sc = Scene(ambient_color=RGB(0.05, 0.05, 0.05))
        sc.add_Camera(look_from=vec3(0.0, 0.25, 1.0), look_at=vec3(0.0, 0.25, -3.0), screen_width=40,
                      screen_height=30)
        sc.add_Background("stormydays.png")
    np.random.seed(6)
    jit = sc.camera.draw_jitter(2)
    out = _backend().render_scene(sc, 2, jitter=jit, seed=1, want_hits=True)
    rgb, ids, counts = O.render_linear(sc, jit)
    assert np.array_equal(out.hit_ids, ids)
    np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)
    if which == "no_background":
        assert (ids == -1).any()


def test_gpu_chain_mode_recovers_from_ties(tmp_path):
    """A tie (duplicated mesh faces: two colliders at the same distance, both shaded, ray.py:131-146)
    gives a chained ray two children.  The frame is rendered again without chain mode (not with
    bigger queues, which would never help), and the result equals the oracle."""
    path = str(tmp_path / "ico_dup.obj")
    scenes.write_icosphere_obj(path, subdiv=2, duplicate_faces=320)  # every face twice
    sc = scenes.mesh_scene(path, 48, 36, 3)
    np.random.seed(9)
    jit = sc.camera.draw_jitter(2)
    _set_option("frame_kernel", 0)
    _set_option("chain_rays", 1 << 40)
    try:
        B = _backend()
        outs = [B.render_scene(sc, 2, jitter=jit, seed=1, want_hits=True) for _ in range(3)]
    finally:
        _set_option("frame_kernel", -1)
        _set_option("chain_rays", 1000000)
    rgb, ids, counts = O.render_linear(sc, jit)
    for out in outs:
        assert np.array_equal(out.hit_ids, ids)
        assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
        np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)
    assert all(out.stats["retries"] <= 1 for out in outs)


def test_gpu_rgbx_output_is_the_uint8_image_with_opaque_alpha():
    """SRT_RENDER_RGBX (Scene.render's output path, PIL's own RGB layout): the same pixels as the
    3-byte image, alpha 255, into pageable, pinned and device memory; Scene.render returns a mode-RGB
    image equal to the one built from the 3-byte pixels."""
    import ctypes
    from PIL import Image
    from sightpy import _native as N

    B = _backend()
    sc = scenes.example1(160, 90, 3)
    np.random.seed(2)
    jit = sc.camera.draw_jitter(2)
    ref = B.render_scene(sc, 2, jitter=jit, seed=1)
    got = B.render_scene(sc, 2, jitter=jit, seed=1, want_rgb=False, rgbx=True)
    assert got.srgb8.shape == (90, 160, 4)
    assert np.array_equal(got.srgb8[..., :3], ref.srgb8) and np.all(got.srgb8[..., 3] == 255)
    pin = B.render_scene(sc, 2, jitter=jit, seed=1, want_rgb=False, rgbx=True, pinned_u8=True)
    assert np.array_equal(pin.srgb8, got.srgb8)
    lib, ctx = B.context()
    d = B.device_buffer("rgbx_out", 4 * 160 * 90)
    cd = B.camera_desc(sc.camera)
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, 90, 0
    a.rows, a.out_hit_id, a.mt, a.seed = None, None, None, 1
    jd = np.ascontiguousarray(jit)
    a.jitter = N.ptr(jd)
    a.out_rgb, a.out_srgb8 = None, d
    a.flags = N.RENDER_RGB_LOCAL | N.RENDER_RGBX
    N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
    h = np.empty((90, 160, 4), dtype=np.uint8)
    N.check(lib, lib.srt_memcpy(ctx, N.ptr(h), d, h.nbytes))
    assert np.array_equal(h, got.srgb8)
    np.random.seed(2)
    img = sc.render(2, rng="numpy-host", seed=1)
    assert img.mode == "RGB" and np.array_equal(np.asarray(img), ref.srgb8)


def test_gpu_render_prefetch_is_used_and_changes_nothing():
    """srt_render_prefetch (render_scene queues the numpy-stream generation before lowering and
    uploading the scene): frames rendered after a prefetch equal frames without one bit for bit, with
    numpy's state advanced alike; a prefetch the next render does not match -- another spp, a host
    draw or a device stream draw in between, an option change -- is dropped, and one for a frame of
    another scene of the same shape is used (the jitter depends only on the stream)."""
    import ctypes
    from sightpy import _native as N

    B = _backend()
    lib, ctx = B.context()

    def counts():
        u, q = ctypes.c_int64(0), ctypes.c_int64(0)
        N.check(lib, lib.srt_debug_prefetch_counts(ctx, ctypes.byref(u), ctypes.byref(q)))
        return u.value, q.value

    def render(scene, spp, prefetch):
        out = B.render_scene(scene, spp, mt=True, prefetch=prefetch)
        return out.rgb.copy(), out.srgb8.copy(), np.random.get_state()

    def same(x, y):
        assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1])
        assert np.array_equal(x[2][1], y[2][1]) and x[2][2] == y[2][2]

    def prefetch_only(scene, spp):
        cd = B.camera_desc(scene.camera)
        a = N.RenderArgs()
        a.spp, a.sample_base, a.n_rows, a.batch_spp = spp, 0, int(scene.camera.screen_height), 0
        a.rows, a.jitter, a.out_hit_id, a.out_rgb, a.out_srgb8, a.seed = None, None, None, None, None, 1
        st = N.MtState.from_numpy()
        a.mt = ctypes.pointer(st)
        N.check(lib, lib.srt_render_prefetch(ctx, ctypes.byref(cd), ctypes.byref(a)))

    sc = scenes.example1(320, 180, 3)
    sc2 = scenes.example2(320, 180, 3)
    for spp in (1, 3):
        np.random.seed(5)
        ref = render(sc, spp, False)
        u0, q0 = counts()
        np.random.seed(5)
        got = render(sc, spp, True)
        assert counts() == (u0 + 1, q0 + 1)
        same(got, ref)
    # dropped: another spp
    np.random.seed(7)
    ref = render(sc, 2, False)
    u0, _ = counts()
    np.random.seed(7)
    prefetch_only(sc, 3)
    same(render(sc, 2, False), ref)
    assert counts()[0] == u0
    # dropped: a host draw, then a device draw of numpy's stream in between
    np.random.seed(8)
    np.random.rand(3)
    ref = render(sc, 2, False)
    np.random.seed(8)
    prefetch_only(sc, 2)
    np.random.rand(3)
    same(render(sc, 2, False), ref)
    np.random.seed(9)
    B.numpy_uniforms(1000)
    ref = render(sc, 2, False)
    np.random.seed(9)
    prefetch_only(sc, 2)
    B.numpy_uniforms(1000)
    same(render(sc, 2, False), ref)
    assert counts()[0] == u0
    # dropped: an option set in between
    np.random.seed(10)
    ref = render(sc, 2, False)
    np.random.seed(10)
    prefetch_only(sc, 2)
    N.check(lib, lib.srt_set_option(ctx, b"mt_short", 65536))
    same(render(sc, 2, False), ref)
    assert counts()[0] == u0
    # used: another scene (lowered and uploaded after the prefetch) of the same frame shape
    np.random.seed(11)
    ref2 = render(sc2, 2, False)
    np.random.seed(11)
    prefetch_only(sc2, 2)
    B.upload(sc)
    got2 = render(sc2, 2, False)  # (uploads sc2 again after the prefetch)
    assert counts()[0] == u0 + 1
    same(got2, ref2)


def test_gpu_scene_render_images_own_their_pixels():
    """Scene.render's image maps pinned memory of its own (image_block): a later render does not
    change an earlier image, a change to an image does not reach another one, the images equal the
    reference's fromarray of the uint8 frame, and past the pool's cap of live images the pixels are
    copied instead (same images)."""
    import gc

    B = _backend()
    sc = scenes.example1(160, 90, 3)
    np.random.seed(3)
    jit = sc.camera.draw_jitter(2)
    ref = B.render_scene(sc, 2, jitter=jit, seed=1).srgb8
    np.random.seed(3)
    a = sc.render(2)
    a_px = np.asarray(a).copy()
    assert np.array_equal(a_px, ref)
    np.random.seed(4)
    b = sc.render(2)
    assert np.array_equal(np.asarray(a), a_px) and not np.array_equal(np.asarray(b), a_px)
    a.putpixel((0, 0), (1, 2, 3))
    np.random.seed(3)
    c = sc.render(2)
    assert np.array_equal(np.asarray(c), a_px) and a.getpixel((0, 0)) == (1, 2, 3)
    imgs = []
    for _ in range(B._BLOCKS_OUT_MAX + 4):
        np.random.seed(3)
        imgs.append(sc.render(2))
    assert B._STATE["blocks_out"] <= B._BLOCKS_OUT_MAX
    for im in imgs:
        assert im.mode == "RGB" and np.array_equal(np.asarray(im), a_px)
    del imgs, a, b, c
    gc.collect()
    assert B._STATE["blocks_out"] == 0
    assert sum(len(v) for v in B._STATE["blocks"].values()) <= B._BLOCKS_FREE_MAX


def test_gpu_grid_and_kernel_form_options_give_the_same_frames():
    """The kernel forms -- the synchronous launch's full grid, the lean kernel of pipelined frames on
    its grid-stride grid, and the lean kernel in synchronous frames (sync_lean) -- change how the work
    is spread, not what is summed: the same images, whole frames and a shard's rows, synchronous and
    pipelined (fixed-point sums are exact in any grouping)."""
    import ctypes
    from sightpy import _native as N

    B = _backend()
    lib, ctx = B.context()
    sc = scenes.example1(640, 360, 3)
    rows = np.ascontiguousarray([r for r in range(360) if (r // 9) % 4 == 1], dtype=np.int32)
    cd = B.camera_desc(sc.camera)

    def frames():
        outs = []
        for rr in (None, rows):
            n = 360 if rr is None else len(rr)
            np.random.seed(31)
            jit = np.ascontiguousarray(np.random.rand(2, 4, 640 * n))
            sync = B.render_scene(sc, 2, jitter=jit, seed=1, rows=rr)
            outs += [sync.rgb.copy(), sync.srgb8.copy()]
            jd = B.device_buffer("grid_jit_%d" % n, jit.nbytes)
            N.check(lib, lib.srt_memcpy(ctx, jd, N.ptr(jit), jit.nbytes))
            a = N.RenderArgs()
            a.spp, a.sample_base, a.n_rows, a.batch_spp = 2, 0, n, 0
            a.rows, a.jitter, a.out_hit_id, a.mt, a.seed = N.ptr(rr), jd, None, None, 1
            a.flags = N.RENDER_ASYNC
            bufs = [B.pinned_buffer("grid_u8_%d_%d" % (n, k), 3 * 640 * n) for k in range(3)]
            for k in range(3):
                a.out_srgb8 = N.ptr(bufs[k])
                N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), None))
            N.check(lib, lib.srt_render_finish(ctx, None))
            outs += [b.copy().reshape(n, 640, 3) for b in bufs]
        return outs

    def opts(**kv):
        for k, v in kv.items():
            N.check(lib, lib.srt_set_option(ctx, k.encode(), v))

    ref = frames()
    try:
        opts(sync_lean=1)
        got = frames()
        for x, y in zip(ref, got):
            assert np.array_equal(x, y)
    finally:
        opts(sync_lean=0)
    assert np.array_equal(ref[2], ref[1]) and np.array_equal(ref[3], ref[1])  # pipelined == synchronous


OPTION_KEYS = {"frame_kernel": -1, "fuse_primary": -1, "chain_rays": 1000000, "bvh": 1, "collider_seq": 1,
               "sync_lean": 0, "deterministic": 1, "pipeline": 0, "mt_bands": 1, "mt_short": 65536,
               "mt_pipe_split": 1 << 18, "mt_gen_nt": 0, "mt_jump_parts": 0, "shard_bands": 0,
               "rehearse_shard": 0, "rehearse_assemble": 0}


def test_gpu_option_surface():
    """srt_set_option takes exactly the 16 documented keys (include/sightpy_rt.h); the round-1..5
    experiment switches removed in round 6 fail as unknown."""
    lib, ctx = _backend().context()
    assert len(OPTION_KEYS) == 16
    for k, v in OPTION_KEYS.items():
        _set_option(k, v)
    for k in ("queue_bytes", "occupancy", "mt_gen_stream", "mt_short_all", "lean_blocks", "lean_blocks_shard",
              "sync_blocks", "texel_rgbx", "sky_prefetch", "frame_groups", "shard_snake", "pix_groups",
              "max_blocks", "slots", "mt_stream", "copy_stream"):
        assert lib.srt_set_option(ctx, k.encode(), 0) != 0, k


def test_gpu_collider_seq_and_bvh_options_give_the_same_frames(tmp_path):
    """The specialised kernels (collider_seq: ex1's straight-line sphere, sphere, plane, sky box
    variant; bvh: the triangle BVH) against the generic paths they replace: the same frames bit for
    bit (options "collider_seq" 0 and "bvh" 0)."""
    sc = scenes.example1(320, 180, 5)
    np.random.seed(7)
    jit = sc.camera.draw_jitter(2)
    path = str(tmp_path / "ico.obj")
    scenes.write_icosphere_obj(path, subdiv=2)
    mesh = scenes.mesh_scene(path, 96, 64, 3)
    jm = mesh.camera.draw_jitter(2)
    for key, scene, j in (("collider_seq", sc, jit), ("bvh", mesh, jm)):
        on = _backend().render_scene(scene, 2, jitter=j, seed=1, want_hits=True)
        _set_option(key, 0)
        try:
            off = _backend().render_scene(scene, 2, jitter=j, seed=1, want_hits=True)
        finally:
            _set_option(key, 1)
        assert np.array_equal(on.rgb, off.rgb) and np.array_equal(on.srgb8, off.srgb8), key
        assert np.array_equal(on.hit_ids, off.hit_ids), key
