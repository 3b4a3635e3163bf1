"""Row-band sharding of a frame across GPUs: the partition the library uses (SRT_RENDER_SHARDED,
csrc/rt_device.h shard_band_height / shard_band_owner / shard_local_row), restated with numpy for
callers and tests.

The reference parallelises `Scene.render` over samples with `multiprocessing.Pool`
(`sightpy/scene.py:80-116`).  Pixels are independent, so here the frame is split instead: the rows
are cut into bands of h rows (the last one shorter) and every period of `world` bands is dealt one
band per rank, round-robin.  Interleaving balances the cheap sky rows
against the reflective floor rows; every rank renders its rows with the same per-pixel random
numbers the single-GPU render would use; the library gathers the uint8 (and linear-RGB) tiles to
rank 0 over RCCL and assembles the frame there.  The image is independent of the number of ranks.

Every band of a rank is a run of numpy's stream that the rank's generator jumps to (one ~110 us jump
per band, plane and sample), so h is as large as the balance allows: at most `kmax` bands per rank
(at least kmax // 2), the fewest rows on the busiest rank first, then the most bands; a Diffuse
fan-out scene, whose rows cost ~30x more, takes 2-row bands (shard_kmax).
"""
import numpy as np

SHARD_BANDS = 8  # kmax (library option "shard_bands"; 0 = shard_kmax's choice)
SHARD_FANOUT_ROWS = 2  # band rows of a Diffuse fan-out scene (rt_device.h shard_kmax)


def shard_kmax(height, world, kmax=0, fanout=1):
    """Most bands per rank (rt_device.h shard_kmax): `kmax` if set, else SHARD_BANDS, or for a scene
    with a Diffuse fan-out (fanout > 2: ~50 rays per pixel and sample, a jump is a fraction of one
    row's work) as many as SHARD_FANOUT_ROWS-row bands give."""
    if kmax:
        return int(kmax)
    if fanout > 2 and world > 0:
        return max(SHARD_BANDS, int(height) // (int(world) * SHARD_FANOUT_ROWS))
    return SHARD_BANDS


def scene_fanout(scene):
    """Most children one hit spawns (the library's rule, srt_upload_scene): 2 for refraction and thin
    film, diffuse_rays for Diffuse, else 1."""
    from . import _native as N
    from ._lower import lower_scene

    fan = 1
    for m in lower_scene(scene).materials:
        if m["type"] in (N.REFRACTIVE, N.THINFILM):
            fan = max(fan, 2)
        elif m["type"] == N.DIFFUSE:
            fan = max(fan, max(1, int(m["ival"])))
    return fan


def band_owner(b, world):
    """Rank of band `b` (rt_device.h shard_band_owner); b may be an array."""
    return np.asarray(b) % world


def rank_rows(height, world, rank, band):
    """Rows of `rank` with bands of `band` rows (rt_device.h shard_rank_rows)."""
    B = -(-int(height) // band)
    owners = band_owner(np.arange(B), world)
    nb = int((owners == rank).sum())
    return nb * band - ((B * band - height) if owners[-1] == rank else 0)


def band_height(height, world, kmax=0, fanout=1):
    """Band height of a `world`-rank frame of `height` rows (rt_device.h shard_band_height)."""
    height = int(height)
    if world <= 1 or height <= 1:
        return max(height, 1)
    kmax = max(shard_kmax(height, world, kmax, fanout), 1)
    best_h, best_rows = 1, None
    for k in range(kmax, max(kmax // 2, 1) - 1, -1):
        h = max(-(-height // (world * k)), 1)
        if -(-height // h) < world:  # fewer bands than ranks: a rank would get no rows
            continue
        m = max(rank_rows(height, world, q, h) for q in range(world))
        if best_rows is None or m < best_rows:
            best_h, best_rows = h, m
    return best_h


def shard_rows(height, world, rank, kmax=0, fanout=1):
    """Image rows owned by `rank` (ascending)."""
    h = band_height(height, world, kmax, fanout)
    rows = np.arange(int(height))
    return rows[band_owner(rows // h, world) == rank]


def max_shard_rows(height, world, kmax=0, fanout=1):
    """Largest per-rank row count (the padded tile height of the gather)."""
    return max(len(shard_rows(height, world, r, kmax, fanout)) for r in range(world))


def assemble_index(height, world, kmax=0, fanout=1):
    """For every image row, its position in the gathered buffer of padded tiles:
    `gathered.reshape(world * maxrows, ...)[idx]` is the image."""
    maxrows = max_shard_rows(height, world, kmax, fanout)
    idx = np.empty(int(height), dtype=np.int64)
    for r in range(world):
        rows = shard_rows(height, world, r, kmax, fanout)
        idx[rows] = r * maxrows + np.arange(len(rows))
    return idx
