"""Row-band sharding of a frame across GPUs: the partition the library uses (SRT_RENDER_SHARDED,
csrc/rt_device.h shard_band_height / shard_band_owner / shard_local_row), restated with numpy for
callers and tests.

The reference parallelises `Scene.render` over samples with `multiprocessing.Pool`
(`sightpy/scene.py:80-116`).  Pixels are independent, so here the frame is split instead: the rows
are cut into bands of h rows (the last one shorter) and every period of `world` bands is dealt one
band per rank -- round-robin, or with `snake` in alternating direction (odd periods dealt
world-1 .. 0, cancelling a top-to-bottom cost gradient).  Interleaving balances the cheap sky rows
against the reflective floor rows; every rank renders its rows with the same per-pixel random
numbers the single-GPU render would use; the library gathers the uint8 (and linear-RGB) tiles to
rank 0 over RCCL and assembles the frame there.  The image is independent of the number of ranks.

Every band of a rank is a run of numpy's stream that the rank's generator jumps to (one ~110 us jump
per band, plane and sample), so h is as large as the balance allows: at most `kmax` bands per rank
(at least kmax // 2), the fewest rows on the busiest rank first, then the most bands.
"""
import numpy as np

SHARD_BANDS = 8  # kmax (library option "shard_bands")
SHARD_SNAKE = 1  # dealing order (library option "shard_snake")


def band_owner(b, world, snake=SHARD_SNAKE):
    """Rank of band `b` (rt_device.h shard_band_owner); b may be an array."""
    b = np.asarray(b)
    i = b % world
    return np.where(np.logical_and(bool(snake), (b // world) % 2 == 1), world - 1 - i, i)


def rank_rows(height, world, rank, band, snake=SHARD_SNAKE):
    """Rows of `rank` with bands of `band` rows (rt_device.h shard_rank_rows)."""
    B = -(-int(height) // band)
    owners = band_owner(np.arange(B), world, snake)
    nb = int((owners == rank).sum())
    return nb * band - ((B * band - height) if owners[-1] == rank else 0)


def band_height(height, world, kmax=SHARD_BANDS, snake=SHARD_SNAKE):
    """Band height of a `world`-rank frame of `height` rows (rt_device.h shard_band_height)."""
    height = int(height)
    if world <= 1 or height <= 1:
        return max(height, 1)
    kmax = max(int(kmax), 1)
    best_h, best_rows = 1, None
    for k in range(kmax, max(kmax // 2, 1) - 1, -1):
        h = max(-(-height // (world * k)), 1)
        m = max(rank_rows(height, world, q, h, snake) for q in range(world))
        if best_rows is None or m < best_rows:
            best_h, best_rows = h, m
    return best_h


def shard_rows(height, world, rank, kmax=SHARD_BANDS, snake=SHARD_SNAKE):
    """Image rows owned by `rank` (ascending)."""
    h = band_height(height, world, kmax, snake)
    rows = np.arange(int(height))
    return rows[band_owner(rows // h, world, snake) == rank]


def max_shard_rows(height, world, kmax=SHARD_BANDS, snake=SHARD_SNAKE):
    """Largest per-rank row count (the padded tile height of the gather)."""
    return max(len(shard_rows(height, world, r, kmax, snake)) for r in range(world))


def assemble_index(height, world, kmax=SHARD_BANDS, snake=SHARD_SNAKE):
    """For every image row, its position in the gathered buffer of padded tiles:
    `gathered.reshape(world * maxrows, ...)[idx]` is the image."""
    maxrows = max_shard_rows(height, world, kmax, snake)
    idx = np.empty(int(height), dtype=np.int64)
    for r in range(world):
        rows = shard_rows(height, world, r, kmax, snake)
        idx[rows] = r * maxrows + np.arange(len(rows))
    return idx
