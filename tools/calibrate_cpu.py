"""CPU-baseline calibration (BASELINE.md "CPU-baseline plan", step 3): time the oracle restatement
(oracle/sightpy_oracle.py, what bench.py's cpu_baseline runs on the GPU box) against the reference
itself on BASELINE configs 1 and 2, one core each, in this (build) container.

The reference is imported read-only from /root/reference with tests/golden/gen_golden.py's harness
(numpy-2 shim, scratch directory); both run the same frames: np.random.seed(0), every sample's
Camera.get_ray first, then get_raycolor per sample (the single-process form of Scene.render).

    OPENBLAS_NUM_THREADS=1 python tools/calibrate_cpu.py [--configs 1 2]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
import numpy as np  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "tests" / "golden", ROOT / "tests", ROOT / "oracle", ROOT / "python-raytracer_amd"):
    sys.path.insert(0, str(p))

CONFIGS = {1: ("example1.py", "example1", 400, 300, None, 6), 2: ("example1.py", "example1", 1920, 1080, 5, 6)}


def time_reference(gg, sp, script, W, H, depth, spp):
    scene = gg.capture_scene(sp, script, W, H, depth)
    counts, get_rc = gg.instrument(sp)
    np.random.seed(0)
    t0 = time.perf_counter()
    rays = [scene.camera.get_ray(scene.n) for _ in range(spp)]
    acc = sp.rgb(0.0, 0.0, 0.0)
    for r in rays:
        acc = acc + get_rc(r, scene)
    dt = time.perf_counter() - t0
    return dt, sum(counts.values()), (acc / spp).to_array()


def time_oracle(builder, W, H, depth, spp):
    import scenes
    import sightpy_oracle as O

    sc = getattr(scenes, builder)(W, H, depth)
    np.random.seed(0)
    counts = {}
    t0 = time.perf_counter()
    jit = sc.camera.draw_jitter(spp)
    acc = 0.0
    for s in range(spp):
        Oo, Do = O.primary_rays(sc.camera, jit[s])
        acc = acc + O.raycolor(sc, O.Rays(np.ascontiguousarray(np.broadcast_to(Oo, Do.shape)), Do,
                                          O.scene_medium(sc), 0), counts)
    dt = time.perf_counter() - t0
    return dt, sum(counts["depth"].values()), acc / spp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--side", choices=["reference", "oracle"], default=None)
    ap.add_argument("--rgb-out", default=None)
    a = ap.parse_args()
    if a.side:  # one side in this process (both packages are called `sightpy`)
        script, builder, W, H, depth, spp = CONFIGS[a.configs[0]]
        if a.side == "reference":
            import gen_golden as gg

            dt, n, rgb = time_reference(gg, gg.import_reference(), script, W, H, depth, spp)
        else:
            dt, n, rgb = time_oracle(builder, W, H, depth, spp)
        np.save(a.rgb_out, rgb)
        print(json.dumps({"s": dt, "rays": n}))
        return
    import subprocess
    import tempfile

    for k in a.configs:
        res = {}
        with tempfile.TemporaryDirectory() as tmp:
            for side in ("reference", "oracle"):
                f = os.path.join(tmp, side + ".npy")
                r = subprocess.run([sys.executable, __file__, "--configs", str(k), "--side", side, "--rgb-out", f],
                                   capture_output=True, text=True, check=True)
                res[side] = json.loads(r.stdout.strip().splitlines()[-1])
                res[side]["rgb"] = np.load(f)
        script, builder, W, H, depth, spp = CONFIGS[k]
        ref, ora = res["reference"], res["oracle"]
        rec = {"config": k, "frame": "%s %dx%d depth %s spp %d" % (script, W, H, depth, spp),
               "rays_reference": ref["rays"], "rays_oracle": ora["rays"], "reference_s": round(ref["s"], 3),
               "oracle_s": round(ora["s"], 3), "ratio_oracle_over_reference": round(ora["s"] / ref["s"], 3),
               "max_rel_rgb_diff": float(np.max(np.abs(ora["rgb"] - ref["rgb"]) /
                                                np.maximum(np.abs(ref["rgb"]), 1e-300)))}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
