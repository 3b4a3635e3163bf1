"""Diagnostic: the srt_render_group retry of test_gpu.py::test_gpu_group_render_retries_a_frame_on_every_context
outside pytest (stderr not captured, so HIP/RCCL messages survive an abort), step by step."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "python-raytracer_amd", ROOT / "tests", ROOT / "oracle"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    import scenes
    from sightpy import Emissive, Sphere, rgb, vec3
    from sightpy import _backend as B

    sc = scenes.example1(48, 40, 3)
    sc.add(Sphere(material=Emissive(color=rgb(1e7, 1e7, 1e7)), center=vec3(0.0, 60.0, -3.0), radius=55.0,
                  shadow=False, max_ray_depth=3))
    mode = sys.argv[1] if len(sys.argv) > 1 else "retry"
    log("step 1: render_scene (process context)")
    np.random.seed(9)
    ref = B.render_scene(sc, 2, seed=3, mt=True)
    log("  retries", ref.stats["retries"])
    os.environ["SIGHTPY_DEVICES"] = str(B.devices()[0])
    if mode == "plain":
        sc2 = scenes.example1(48, 40, 3)
        log("step 2: render_group of a scene that needs no retry")
        np.random.seed(9)
        got = B.render_group(sc2, 2, seed=3, mt=True)
        log("  ok", got.stats["total_rays"])
        return
    log("step 2: render_group (group context, retry expected)")
    np.random.seed(9)
    got = B.render_group(sc, 2, seed=3, mt=True)
    log("  ok; max |d rgb|", float(np.abs(got.rgb - ref.rgb).max()), "rays", got.stats["total_rays"],
        ref.stats["total_rays"])


if __name__ == "__main__":
    main()
