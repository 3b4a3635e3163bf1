"""GPU parity of the Monte-Carlo paths (Diffuse PDFs, mc=True refraction, device-RNG raygen).

The HIP kernels draw their Monte-Carlo numbers from Philox4x32-10 keyed by (seed, global pixel,
child-path hash, tag).  The oracle, pinned to the reference on the reference's own numpy stream
(tests/test_mc.py), consumes that same stream here (`sightpy_oracle.DeviceStream`), so every
sample is compared deterministically: primary hit ids exact, per-depth ray counts equal, linear
RGB within the north_star tolerance (1e-5 relative, 1e-12 absolute floor).  On top, the cornell
box is compared statistically with the reference's own renders (per-10x10-block means
over 16 seeds, tests/golden/cornell_stats_80x80.npz).
"""
import numpy as np
import pytest

import scenes
import sightpy_oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-5, 1e-12


def _backend():
    from sightpy import _backend

    return _backend


def _set_option(key, value):
    lib, ctx = _backend().context()
    import ctypes

    rc = lib.srt_set_option(ctx, key.encode(), ctypes.c_int64(value))
    assert rc == 0, lib.srt_last_error()


MC_SCENES = [
    ("cornell_32x32", lambda: scenes.cornell(32, 32), 2),
    ("cornell_mc_24x24", lambda: scenes.cornell(24, 24, mc=True), 2),
    ("features_mc_48x36", lambda: scenes.features(48, 36, 4, mc=True), 2),
]


@pytest.mark.parametrize("name,build,spp", MC_SCENES)
@pytest.mark.parametrize("mode", ["wavefront", "frame"])
def test_gpu_mc_matches_oracle_on_device_stream(name, build, spp, mode):
    sc = build()
    np.random.seed(0)
    jit = sc.camera.draw_jitter(spp)
    _set_option("frame_kernel", 1 if mode == "frame" else 0)
    try:
        out = _backend().render_scene(sc, spp, jitter=jit, seed=2024, want_hits=True)
    finally:
        _set_option("frame_kernel", -1)
    rgb, ids, counts = O.render_linear(sc, jit, stream=O.DeviceStream(2024))
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)


def test_gpu_device_rng_raygen_matches_oracle():
    """Device-RNG mode (no host jitter): the camera uniforms come from Philox as well."""
    sc = scenes.cornell(24, 24)
    out = _backend().render_scene(sc, 2, jitter=None, seed=77, want_hits=True)
    st = O.DeviceStream(77)
    rgb, ids, counts = O.render_linear(sc, st.jitter(24 * 24, 2), stream=st)
    assert np.array_equal(out.hit_ids, ids)
    np.testing.assert_allclose(out.rgb, rgb, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("dfl", [0, 1])
def test_gpu_diffuse_batch_matches_oracle(dfl):
    """get_raycolor (srt_trace) of a batch hitting the cornell walls: the 20-ray fan-out of
    diffuse.py:34-83 (dfl 0) and the single ray of :85-121 (dfl 1)."""
    from sightpy import Ray, vec3
    from sightpy._backend import trace_rays

    sc = scenes.cornell(16, 16)
    rng = np.random.default_rng(dfl)
    n = 2000
    # origins in the box above the tall block and the glass sphere (a ray starting inside the block
    # meets its bottom face and the coplanar floor at distances one rounding apart: a tie or not
    # depending on the last bit of the direction, i.e. on the libm)
    Ob = np.stack([rng.uniform(20, 535, n), rng.uniform(350, 540, n), rng.uniform(-535, -20, n)])
    D = rng.standard_normal((3, n))
    D /= np.sqrt((D * D).sum(0))
    ray = Ray(vec3(*Ob), vec3(*D), 0, sc.n, 0, 0, dfl)
    col, st = trace_rays(ray, sc, seed=99, return_stats=True)
    ref, counts = O.trace_linear(sc, Ob, D, O.scene_medium(sc), 0, dfl, stream=O.DeviceStream(99))
    assert st["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(np.stack([col.x, col.y, col.z]), ref, rtol=RTOL, atol=ATOL)


def test_gpu_mc_row_shards_equal_full_frame():
    """Monte-Carlo draws are keyed by the global pixel: the rows of a shard (one GPU of N) come out
    exactly as in the full frame, so a multi-GPU image does not depend on the GPU count."""
    sc = scenes.cornell(40, 40)
    np.random.seed(3)
    jit = sc.camera.draw_jitter(2)
    be = _backend()
    full = be.render_scene(sc, 2, jitter=jit, seed=5)
    for world in (2, 3):
        from sightpy._shard import shard_rows

        rows = shard_rows(40, world, world - 1)
        part = np.ascontiguousarray(jit.reshape(2, 4, 40, 40)[:, :, rows].reshape(2, 4, -1))
        sh = be.render_scene(sc, 2, jitter=part, seed=5, rows=rows)
        np.testing.assert_allclose(sh.rgb, full.rgb.reshape(3, 40, 40)[:, rows].reshape(3, -1), rtol=1e-13,
                                   atol=1e-15)


def test_gpu_cornell_block_statistics_vs_reference():
    """the device's cornell box (Philox) against the reference's (numpy MT19937)
    per-10x10-block means, 16 seeds x 8 spp on each side.  Each block and channel must agree within
    5 combined standard errors, the whole image within 3."""
    g = golden("cornell_stats_80x80")
    ref = g["block_means"]  # (seeds, 3, 8, 8)
    W, H, spp, nseeds = int(g["width"]), int(g["height"]), int(g["spp"]), ref.shape[0]
    sc = scenes.cornell(W, H)
    be = _backend()
    dev = np.empty_like(ref)
    for k in range(nseeds):
        out = be.render_scene(sc, spp, jitter=None, seed=0xC0FFEE + k)
        dev[k] = out.rgb.reshape(3, H // 10, 10, W // 10, 10).mean(axis=(2, 4))
    from test_mc import block_stats_z

    z, z_img = block_stats_z(ref, dev)
    assert z.max() < 5.0 and (z_img < 3.0).all(), (z.max(), z_img)
