"""Row-band sharding of a frame across ranks (one process per GPU) and the final gather.

The reference parallelises `Scene.render` over samples with `multiprocessing.Pool`
(`sightpy/scene.py:80-116`).  Pixels are independent, so here the frame is split instead: rank r
owns the rows `{y : (y // band) % world == r}` (bands dealt round-robin, which balances the cheap
sky rows against the reflective floor rows), renders them with the same per-pixel jitter the
single-GPU render would use, and the uint8 tiles are all-gathered (`torch.distributed`; backend
`nccl` = RCCL over xGMI on MI355X, `gloo` on CPU for tests).  The assembled image is independent of
the number of ranks.
"""
import numpy as np

BAND = 8


def shard_rows(height, world, rank, band=BAND):
    """Image rows owned by `rank` (ascending)."""
    rows = np.arange(int(height))
    return rows[(rows // band) % world == rank]


def max_shard_rows(height, world, band=BAND):
    """Largest per-rank row count (the padded tile height of the gather)."""
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


class RowGather:
    """Reusable all-gather of padded row tiles for one (height, world, tile shape, device): the
    gathered buffer and the row-assembly index are allocated once, so each frame costs one RCCL
    `all_gather_into_tensor` plus one on-device row permutation (`index_select`)."""

    def __init__(self, height, world, rest, dtype, device, group=None, band=BAND):
        import torch

        self.height, self.world, self.group, self.band = int(height), int(world), group, band
        self.maxrows = max_shard_rows(height, world, band)
        self.full = torch.empty((world * self.maxrows,) + tuple(rest), dtype=dtype, device=device)
        self.idx = torch.as_tensor(assemble_index(height, world, band), device=device)

    def __call__(self, padded):
        """`padded`: this rank's tile with `maxrows` rows (rows beyond its shard are ignored)."""
        import torch.distributed as dist

        if dist.get_backend(self.group) == "gloo":
            dist.all_gather(list(self.full.chunk(self.world)), padded, group=self.group)
        else:
            dist.all_gather_into_tensor(self.full, padded, group=self.group)
        return self.full.index_select(0, self.idx)


def gather_rows(tile, height, world, group=None, band=BAND):
    """All-gather each rank's row tile and return the full image on every rank.

    `tile` is a torch tensor of shape (len(shard_rows(...)), ...) on the collective's device
    (cuda for nccl, cpu for gloo).  Tiles are padded to the largest shard so a single
    `all_gather_into_tensor` (one RCCL collective) moves the frame."""
    g = RowGather(height, world, tile.shape[1:], tile.dtype, tile.device, group, band)
    padded = tile.new_zeros((g.maxrows,) + tuple(tile.shape[1:]))
    padded[: tile.shape[0]] = tile
    return g(padded)
