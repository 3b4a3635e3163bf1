"""Row-band sharding of a frame across GPUs: the partition the library uses (SRT_RENDER_SHARDED,
csrc/rt_device.h shard_of_row / shard_local_row), restated with numpy for callers and tests.

The reference parallelises `Scene.render` over samples with `multiprocessing.Pool`
(`sightpy/scene.py:80-116`).  Pixels are independent, so here the frame is split instead: rank r
owns the rows `{y : (y // band) % world == r}` (bands dealt round-robin, which balances the cheap
sky rows against the reflective floor rows) and renders them with the same per-pixel random numbers
the single-GPU render would use; the library gathers the uint8 (and linear-RGB) tiles to rank 0
over RCCL and assembles the frame there.  The image is independent of the number of ranks.
"""
import numpy as np

BAND = 8


def shard_rows(height, world, rank, band=BAND):
    """Image rows owned by `rank` (ascending)."""
    rows = np.arange(int(height))
    return rows[(rows // band) % world == rank]


def max_shard_rows(height, world, band=BAND):
    """Largest per-rank row count (rank 0's: the padded tile height of the gather)."""
    return max(len(shard_rows(height, world, r, band)) for r in range(world))


def assemble_index(height, world, band=BAND):
    """For every image row, its position in the gathered buffer of padded tiles:
    `gathered.reshape(world * maxrows, ...)[idx]` is the image."""
    maxrows = max_shard_rows(height, world, band)
    idx = np.empty(int(height), dtype=np.int64)
    for r in range(world):
        rows = shard_rows(height, world, r, band)
        idx[rows] = r * maxrows + np.arange(len(rows))
    return idx
