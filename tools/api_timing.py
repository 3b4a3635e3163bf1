"""End-to-end rate of the public API: `Scene.render(spp)` exactly as an example script calls it
(scene.py:60-104 here, reference scene.py:71-140): the reference's numpy jitter stream generated on
the GPU, every sample and depth traced, the uint8 image copied to host memory over PCIe (Scene.render
returns only the PIL image, so the linear RGB stays on the device), and the PIL image built.  Compare
bench.py, whose frame also brings the linear RGB (f64) to the host.

    python tools/api_timing.py [--config example1_1080p_d5] [--repeats 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "python-raytracer_amd", ROOT / "tests", ROOT):
    sys.path.insert(0, str(p))


def main():
    import numpy as np
    import scenes
    from bench import CONFIGS

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="example1_1080p_d5", choices=sorted(CONFIGS))
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--profile", action="store_true", help="cProfile one render (host-side breakdown)")
    ap.add_argument("--phases", action="store_true", help="median ms of the call's steps (lowering, device frame, PIL)")
    ap.add_argument("--option", action="append", default=[], help="srt_set_option KEY=VALUE (repeatable)")
    a = ap.parse_args()
    builder, W, H, depth, spp, label = CONFIGS[a.config]
    sc = getattr(scenes, builder)(W, H, depth)
    if a.option:
        from sightpy import _backend as B, _native as N

        lib, ctx = B.context()
        for kv in a.option:
            k, v = kv.split("=")
            N.check(lib, lib.srt_set_option(ctx, k.encode(), int(v)))
    np.random.seed(0)
    sc.render(spp)  # warmup: scene upload, queue sizing
    times = []
    for _ in range(a.repeats):
        np.random.seed(0)
        t0 = time.perf_counter()
        img = sc.render(spp)
        times.append(time.perf_counter() - t0)
    if a.profile:
        import cProfile
        import pstats

        np.random.seed(0)
        pr = cProfile.Profile()
        pr.enable()
        sc.render(spp)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(25)
    phases = None
    if a.phases:
        # the same call in its steps (scene.py render): lowering alone, lowering + signature check, the
        # device frame (render_scene: its own lowering, RGBX image into the image's pinned block), the
        # PIL image over that block
        from sightpy import _backend as B

        acc = {"lower_only": [], "lower_upload": [], "device_frame": [], "pil": []}
        for _ in range(a.repeats):
            np.random.seed(0)
            tl = time.perf_counter()
            B.lower_scene(sc)
            t0 = time.perf_counter()
            B.upload(sc)
            t1 = time.perf_counter()
            blk = B.image_block(4 * W * H)
            out = B.render_scene(sc, spp, want_rgb=False, mt=True, pinned_u8=True, rgbx=True, out_u8=blk)
            t2 = time.perf_counter()
            im = B.rgb_image(out.srgb8, W, H, mapped=blk is not None)
            t3 = time.perf_counter()
            del im, out, blk
            for k, v in zip(acc, (t0 - tl, t1 - t0, t2 - t1, t3 - t2)):
                acc[k].append(v)
        phases = {k: round(float(np.median(v)) * 1e3, 3) for k, v in acc.items()}
    rays = sc.last_stats["total_rays"]
    best, med = min(times), float(np.median(times))
    print(json.dumps({"what": "Scene.render(%d) via the public API, host buffers (PCIe-inclusive)" % spp,
                      "options": a.option,
                      "workload": label, "image": list(img.size), "rays_per_frame": int(rays),
                      "ms_median": round(med * 1e3, 3), "ms_min": round(best * 1e3, 3),
                      "Mrays_per_s_median": round(rays / med / 1e6, 1), "repeats": a.repeats, "phases_ms_median": phases}))


if __name__ == "__main__":
    main()
