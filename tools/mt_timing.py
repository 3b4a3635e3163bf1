"""Time srt_mt19937_uniforms for a few sizes (device output) to separate jump and generation cost."""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "python-raytracer_amd"))
from sightpy import _backend as B, _native as N  # noqa: E402

L2 = (1 << 19) // 2
lib, ctx = B.context()
key = np.ascontiguousarray(np.random.RandomState(0).get_state()[1], dtype=np.uint32)
ko = np.empty(624, dtype=np.uint32)
po = ctypes.c_int32()
for label, n in [("1 seg (no jump)", L2 - 8), ("2 segs", 2 * L2 - 8), ("17 segs", 17 * L2 - 8), ("256 segs", 256 * L2 - 8),
                 ("1080p x 7 draws", 7 * 4 * 1920 * 1080), ("tiny", 1000)]:
    p = B.device_buffer("t", 8 * n)
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        N.check(lib, lib.srt_mt19937_uniforms(ctx, N.ptr(key), 624, n, 0, p, N.ptr(ko), ctypes.byref(po)))
        ts.append(time.perf_counter() - t0)
    print("%-20s n=%10d  %.3f ms" % (label, n, 1e3 * np.median(ts[1:])), flush=True)
