"""Monte-Carlo shading pinned deterministically on the CPU (no GPU needed).

Two links make the chain from the reference to the kernels:

1. oracle == reference: the oracle draws from numpy's global RNG in the reference's order, so a
   seeded single-process render of an MC scene (Diffuse with the cosine / spherical-caps / mixed
   PDFs of utils/random.py:50-174, and the `mc=True` refraction pick of refractive.py:95-101)
   reproduces the reference's fixture to rounding (tests/golden/{cornell,cornell_mc,features_mc}_*).
2. kernels == oracle: the device draws its MC numbers from a counter-based stream (Philox4x32-10
   keyed by seed, global pixel, child-path hash and a tag).  The oracle restates that stream
   (`DeviceStream`) and consumes it in place of numpy's, so the kernel math -- here the same
   rt_device.h compiled for the CPU, on the GPU in tests/test_gpu_mc.py -- must match it sample for
   sample: same ray counts per depth, colours equal to rounding.
"""
import numpy as np
import pytest

import hostcheck as HC
import scenes
import sightpy_oracle as O
from conftest import golden

# Random123's published known-answer vectors for philox4x32-10 (counter, key, result)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]

RTOL, ATOL = 1e-10, 1e-14  # measured <= 8e-16 relative (libm ulps only)


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(ctr, key, want):
    assert [int(x) for x in O.philox4x32_10(*ctr, *key)] == list(want)
    assert HC.philox(ctr, *key).tolist() == list(want)


def test_mix32_and_child_path_agree_with_kernels():
    rng = np.random.default_rng(5)
    h = rng.integers(0, 2**32, 200, dtype=np.uint64).astype(np.uint32)
    v = rng.integers(0, 2**32, 200, dtype=np.uint64).astype(np.uint32)
    got = O.mix32(h, v)
    assert [HC.mix32(a, b) for a, b in zip(h, v)] == got.tolist()


@pytest.mark.parametrize("name,build", [
    ("cornell_mc_24x24_s1", lambda W, H, d: scenes.cornell(W, H, d, mc=True)),
    ("features_mc_48x36_d4_s2", lambda W, H, d: scenes.features(W, H, d, mc=True)),
])
def test_oracle_mc_refraction_matches_reference(name, build):
    """The mc=True pick (refractive.py:95-101) consumes numpy's stream as the reference does."""
    g = golden(name)
    W, H, spp, depth = int(g["width"]), int(g["height"]), int(g["spp"]), int(g["depth"])
    sc = build(W, H, None if depth < 0 else depth)
    np.random.seed(int(g["seed"]))
    jit = sc.camera.draw_jitter(spp)
    sc.camera.draw_jitter(1)
    rgb, ids, counts = O.render_linear(sc, jit)
    assert np.array_equal(ids, g["hit_id"])
    assert [counts["depth"].get(d, 0) for d in range(len(g["depth_counts"]))] == g["depth_counts"].tolist()
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-12, atol=1e-15)


MC_SCENES = [
    ("cornell", lambda: scenes.cornell(24, 24)),
    ("cornell_mc", lambda: scenes.cornell(24, 24, mc=True)),
    ("features_mc", lambda: scenes.features(32, 24, 4, mc=True)),
]


@pytest.mark.parametrize("name,build", MC_SCENES)
def test_device_math_mc_matches_oracle_on_device_stream(name, build):
    sc = build()
    np.random.seed(0)
    jit = sc.camera.draw_jitter(2)
    rgb, _, hits, st = HC.render(sc, jit, seed=7)
    ref, ids, counts = O.render_linear(sc, jit, stream=O.DeviceStream(7))
    assert np.array_equal(hits, ids)
    assert st["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(rgb, ref, rtol=RTOL, atol=ATOL)


def test_device_math_mc_row_shard_draws_as_full_frame():
    """MC draws are keyed by the global pixel: a row shard renders its rows exactly as the full
    frame does (multi-GPU images are independent of the GPU count)."""
    sc = scenes.cornell(24, 24)
    np.random.seed(1)
    jit = sc.camera.draw_jitter(2)
    full, *_ = HC.render(sc, jit, seed=11)
    rows = np.arange(5, 24, 3)
    part = np.ascontiguousarray(jit.reshape(2, 4, 24, 24)[:, :, rows].reshape(2, 4, -1))
    shard, *_ = HC.render(sc, part, seed=11, rows=rows)
    np.testing.assert_array_equal(shard, full.reshape(3, 24, 24)[:, rows].reshape(3, -1))


@pytest.mark.parametrize("dfl", [0, 1])
def test_device_math_diffuse_batch_kat(dfl):
    """get_raycolor of a batch hitting the cornell walls (diffuse.py:34-83 fan-out of 20 at
    diffuse_reflections 0, the single ray of :85-121 at 1) through the kernel math vs the oracle."""
    sc = scenes.cornell(16, 16)
    rng = np.random.default_rng(dfl)
    n = 300
    # origins in the box above the tall block and the glass sphere (a ray starting inside the block
    # meets its bottom face and the coplanar floor at distances one rounding apart: a tie or not
    # depending on the last bit of the direction, i.e. on the libm)
    Ob = np.stack([rng.uniform(20, 535, n), rng.uniform(350, 540, n), rng.uniform(-535, -20, n)])
    D = rng.standard_normal((3, n))
    D /= np.sqrt((D * D).sum(0))
    got, st = HC.trace(sc, Ob, D, depth=0, dfl=dfl, seed=99)
    ref, counts = O.trace_linear(sc, Ob, D, O.scene_medium(sc), 0, dfl, stream=O.DeviceStream(99))
    assert [st["rays_per_depth"][d] for d in sorted(counts["depth"])] == \
        [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)


def block_stats_z(ref, dev):
    """Per-block and whole-image z-scores of two sets of per-seed 10x10-block means (seeds, 3, by, bx)."""
    n_r, n_d = ref.shape[0], dev.shape[0]
    se = np.sqrt(ref.var(0, ddof=1) / n_r + dev.var(0, ddof=1) / n_d)
    z = np.abs(dev.mean(0) - ref.mean(0)) / np.maximum(se, 1e-12)
    ir, idv = ref.mean(axis=(2, 3)), dev.mean(axis=(2, 3))
    se_img = np.sqrt(ir.var(0, ddof=1) / n_r + idv.var(0, ddof=1) / n_d)
    return z, np.abs(idv.mean(0) - ir.mean(0)) / se_img


def test_device_math_cornell_block_statistics_vs_reference():
    """SURVEY 8(c) statistical pin: the kernels' cornell box (Philox stream, CPU build) against the
    reference's own renders (numpy stream): per-10x10-block means over 16 seeds x 8 spp agree within
    5 standard errors in every block and channel, the image mean within 3 (block SE ~1% relative)."""
    g = golden("cornell_stats_80x80")
    ref = g["block_means"]
    W, H, spp, ns = int(g["width"]), int(g["height"]), int(g["spp"]), ref.shape[0]
    sc = scenes.cornell(W, H)
    dev = np.empty_like(ref)
    for k in range(ns):
        jit = np.random.default_rng(k).random((spp, 4, W * H))
        rgb, *_ = HC.render(sc, jit, seed=0xC0FFEE + k)
        dev[k] = rgb.reshape(3, H // 10, 10, W // 10, 10).mean(axis=(2, 4))
    z, z_img = block_stats_z(ref, dev)
    assert z.max() < 5.0 and (z_img < 3.0).all(), (z.max(), z_img)
