"""Per-section wave time of the trace kernels from the RT_PROF diagnostic build (see
tools/build_ablations.sh PROF): renders the bench frame a few times and prints, per section,
total sampled wave-cycles, number of (wave, section) entries and cycles per entry.

    SIGHTPY_HIP_LIB=build/abl/libsightpy_hip_PROF.so python tools/prof_sections.py [--config ...]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "python-raytracer_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

NAMES = {0: "k_primary raygen (uniform loads + primary_ray)", 1: "nearest_hit", 2: "waterfall (all shading)",
         3: "k_primary trace_one", 4: "glossy: normal + uv + texture", 5: "glossy: shadow_nearest",
         6: "glossy: pow (Dphong)", 7: "glossy: light loop (incl. shadow, pow)", 8: "glossy: child math",
         9: "glossy: child append (reserve + store)", 10: "sky: P + uv", 11: "sky: texture", 12: "waterfall passes",
         13: "k_trace queue load", 14: "k_trace trace_one",
         15: "k_frame primary setup (jitter + raygen)", 16: "k_frame ring chunk load", 17: "k_frame trace_one",
         18: "k_frame prologue (LUTs + ring lock)", 19: "k_frame epilogue"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--builder", default="example1")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--spp", type=int, default=6)
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    import scenes
    from sightpy import _backend as B

    W, H = (int(v) for v in a.size.split("x"))
    sc = getattr(scenes, a.builder)(W, H, a.depth)
    lib, ctx = B.context()
    lib.srt_debug_prof.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    np.random.seed(0)
    jit = sc.camera.draw_jitter(a.spp)
    B.render_scene(sc, a.spp, jitter=jit, seed=1)
    lib.srt_debug_prof(ctx, buf, 1)
    for _ in range(a.frames):
        B.render_scene(sc, a.spp, jitter=jit, seed=1)
    lib.srt_debug_prof(ctx, buf, 1)
    v = np.array(buf[:], dtype=np.float64)
    print("%-48s %14s %10s %10s" % ("section", "cycles", "entries", "cyc/entry"))
    for k in sorted(NAMES):
        n = v[32 + k]
        if n:
            print("%-48s %14.4g %10d %10.0f" % (NAMES[k], v[k], n, v[k] / n))


if __name__ == "__main__":
    main()
