"""GPU parity at the two 8-GPU BASELINE configurations, at their own frame size.

Each test renders ONE rank's row shard of an 8-rank frame at full frame width -- exactly the rows
rank r renders in the multi-GPU job (sightpy._shard.shard_rows, the library's SRT_RENDER_SHARDED
map) -- through the C ABI, and compares it with the oracle on those rows:
  * example4.py 3840x2160, max_ray_depth 6 (reference example4.py:34): thin-film bubble, blurred
    lake skybox with lightmap; jitter = the reference's numpy stream;
  * example_cornellbox.py 800x800 (reference example_cornellbox.py:126): Diffuse PDFs with 20-ray
    fan-out, Monte-Carlo draws from the device's Philox stream, which the oracle restates
    (sightpy_oracle.DeviceStream, keyed by GLOBAL pixel as on the device).
One sample per pixel (the oracle takes ~10-40 s per shard); the per-sample work is what spp
multiplies.  Bar (north_star): primary hit ids exact, per-depth ray counts equal, linear RGB within
1e-5 relative -- checked with NO absolute floor on every value above 1e-9 (the fixed-point
framebuffer sums quantise each term to 2^-44, rt_kernels.hip fx_add), and within 1e-14 absolute
below it.
"""
import numpy as np
import pytest

import scenes
import sightpy_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def assert_rel_no_floor(got, ref, rtol=RTOL, floor=1e-9, atol_below=1e-14):
    """max |got - ref| / |ref| <= rtol over every value with |ref| > floor (no absolute floor), and
    |got - ref| <= atol_below on the rest.  Returns the worst relative error."""
    got, ref = np.asarray(got), np.asarray(ref)
    big = np.abs(ref) > floor
    rel = np.abs(got[big] - ref[big]) / np.abs(ref[big])
    worst = float(rel.max()) if rel.size else 0.0
    assert worst <= rtol, ("max relative error %.3e at %d values above %.0e" % (worst, big.sum(), floor))
    small_err = float(np.abs(got[~big] - ref[~big]).max()) if (~big).any() else 0.0
    assert small_err <= atol_below, small_err
    return worst


def _render_shard(sc, jit_full, rows, seed, stream=None):
    from sightpy import _backend as B

    W, H = int(sc.camera.screen_width), int(sc.camera.screen_height)
    spp = jit_full.shape[0]
    part = np.ascontiguousarray(jit_full.reshape(spp, 4, H, W)[:, :, rows].reshape(spp, 4, -1))
    out = B.render_scene(sc, spp, jitter=part, seed=seed, rows=rows, want_hits=True)
    rgb, ids, counts = O.render_linear(sc, part, stream=stream, rows=rows)
    return out, rgb, ids, counts


@pytest.mark.parametrize("rank", [5])
def test_example4_4k_d6_rank_of_8_full_width_matches_oracle(rank):
    from sightpy._shard import shard_rows

    sc = scenes.example4(3840, 2160, 6)
    rows = shard_rows(2160, 8, rank)
    np.random.seed(4)
    jit = sc.camera.draw_jitter(1)
    out, rgb, ids, counts = _render_shard(sc, jit, rows, seed=1)
    assert out.rgb.shape == (3, len(rows) * 3840)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    worst = assert_rel_no_floor(out.rgb, rgb)
    print("example4 4K d6 rank %d of 8: %d rays, worst relative RGB error %.3e" % (rank, out.stats["total_rays"],
                                                                                     worst))


@pytest.mark.parametrize("rank", [3])
def test_cornell_800_rank_of_8_full_width_matches_oracle_device_stream(rank):
    from sightpy._shard import scene_fanout, shard_rows

    sc = scenes.cornell(800, 800)
    rows = shard_rows(800, 8, rank, fanout=scene_fanout(sc))  # (the library's 2-row bands of a fan-out scene)
    np.random.seed(8)
    jit = sc.camera.draw_jitter(1)
    out, rgb, ids, counts = _render_shard(sc, jit, rows, seed=2025, stream=O.DeviceStream(2025))
    assert out.rgb.shape == (3, len(rows) * 800)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    worst = assert_rel_no_floor(out.rgb, rgb)
    print("cornell 800x800 rank %d of 8: %d rays, worst relative RGB error %.3e" % (rank, out.stats["total_rays"],
                                                                                      worst))


# ---- multi-pass accumulation at the 8-GPU configurations ------------------------------------------
# The multi-GPU frames run several passes per frame (cornell 512 spp: 11 passes; ex4 10 spp): the
# first pass stores the pixels' fixed-point sums, later passes add to them.  batch_size=1 forces one
# pass per sample on a few full-width rows of a rank's shard, compared with the oracle.


def test_cornell_800_multipass_band_of_rank_3_matches_oracle_device_stream():
    """One 2-row band of rank 3's shard of the 8-rank cornell frame (800 wide), 4 spp in 4 passes
    (batch_size 1), Monte-Carlo draws from the device stream the oracle restates
    (reference example_cornellbox.py:126 renders 100 spp; the BASELINE config 512)."""
    from sightpy._shard import scene_fanout, shard_rows

    sc = scenes.cornell(800, 800)
    rows = shard_rows(800, 8, 3, fanout=scene_fanout(sc))[:2]
    assert rows[1] == rows[0] + 1  # one band
    np.random.seed(13)
    jit = sc.camera.draw_jitter(4)
    from sightpy import _backend as B

    part = np.ascontiguousarray(jit.reshape(4, 4, 800, 800)[:, :, rows].reshape(4, 4, -1))
    out = B.render_scene(sc, 4, jitter=part, seed=77, rows=rows, batch_size=1, want_hits=True)
    assert out.stats["passes"] == 4
    rgb, ids, counts = O.render_linear(sc, part, stream=O.DeviceStream(77), rows=rows)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    worst = assert_rel_no_floor(out.rgb, rgb)
    print("cornell 800 rank 3 band, 4 spp in 4 passes: worst relative RGB error %.3e" % worst)


def test_example4_4k_multipass_rows_of_rank_5_match_oracle():
    """Four 3840-wide rows of rank 5's shard of the 8-rank ex4 frame, 3 spp in 3 passes (batch_size 1)
    on the reference's numpy stream (example4.py:34 renders 10 spp)."""
    from sightpy._shard import shard_rows

    sc = scenes.example4(3840, 2160, 6)
    rows = shard_rows(2160, 8, 5)[:4]
    np.random.seed(14)
    jit = sc.camera.draw_jitter(3)
    from sightpy import _backend as B

    part = np.ascontiguousarray(jit.reshape(3, 4, 2160, 3840)[:, :, rows].reshape(3, 4, -1))
    out = B.render_scene(sc, 3, jitter=part, seed=1, rows=rows, batch_size=1, want_hits=True)
    assert out.stats["passes"] == 3
    rgb, ids, counts = O.render_linear(sc, part, rows=rows)
    assert np.array_equal(out.hit_ids, ids)
    assert out.stats["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    worst = assert_rel_no_floor(out.rgb, rgb)
    print("example4 4K rank 5 rows, 3 spp in 3 passes: worst relative RGB error %.3e" % worst)
