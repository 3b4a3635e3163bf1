"""The oracle over several host processes (test infrastructure): one sample of a frame per task, so a
full-size multi-sample parity check costs about one sample's oracle time.

Workers are spawned (fresh interpreters: the test process holds the GPU), each rebuilds the scene from
tests/scenes.py and returns the oracle's summed colour, primary hit ids and per-depth ray counts of
its sample -- sightpy_oracle.render_linear split over samples (its loop is over samples, each
independent: oracle/sightpy_oracle.py render_linear)."""
import multiprocessing as mp
import os

import numpy as np


def _sample(args):
    builder, W, H, depth, jit = args
    import scenes
    import sightpy_oracle as O

    sc = getattr(scenes, builder)(W, H, depth)
    rgb, ids, counts = O.render_linear(sc, jit[None])
    return rgb, ids[0], counts


def render_linear_pool(builder, W, H, depth, jit, workers=None):
    """sightpy_oracle.render_linear(scene, jit) for a deterministic scene (no Monte-Carlo draws),
    computed one sample per worker: (mean rgb (3, n), hit ids (spp, n), {"depth": {d: rays}, ...})."""
    spp = jit.shape[0]
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    n = max(1, min(spp, workers or avail, 16))
    with mp.get_context("spawn").Pool(n) as pool:
        res = pool.map(_sample, [(builder, W, H, depth, np.ascontiguousarray(jit[s])) for s in range(spp)])
    acc = 0.0
    for rgb, _, _ in res:
        acc = acc + rgb * 1.0  # (render_linear returns the per-sample mean: here spp = 1)
    counts = {"depth": {}, "shadow": 0}
    for _, _, c in res:
        for d, v in c["depth"].items():
            counts["depth"][d] = counts["depth"].get(d, 0) + v
        counts["shadow"] += c.get("shadow", 0)
    return acc / spp, np.array([r[1] for r in res]), counts
