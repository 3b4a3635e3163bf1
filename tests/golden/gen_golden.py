"""Generate the parity fixtures in tests/golden/ by running the REFERENCE implementation.

Runs only in the build container, where the reference is mounted read-only at /root/reference:

    python tests/golden/gen_golden.py            # writes tests/golden/*.npz

The reference (lmondada/Python-Raytracer @ 2025-02-14) is imported from a scratch directory
holding a symlink `sightpy -> /root/reference/sightpy` (its asset paths are CWD-relative) with
bytecode writing disabled.  Nothing of the reference is copied: the example scripts are executed
in place with `runpy`, `Scene.render` is intercepted to capture the scene, camera size and
max_ray_depth are overridden, and the golden path is the reference's own single-process form of
render(): all `Camera.get_ray` draws first (plus the extra sizing draw of scene.py:81), then
`get_raycolor` per sample, summed in sample order and divided by spp.

Runtime shim (no file edits): with numpy >= 2, `np.abs(vec3)` no longer dispatches to
`vec3.__abs__` (cuboid.py:145, glossy.py:66, glossy.py:91); a component-wise `__array_ufunc__`
restores the behaviour the reference was written for (validated against its published images).
The progressbar module is stubbed for example_cornellbox.py.
"""
import os
import runpy
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def import_reference():
    work = Path(tempfile.mkdtemp(prefix="refharn_"))
    (work / "sightpy").symlink_to(REF / "sightpy")
    os.chdir(work)
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(work))
    sys.modules.setdefault("progressbar", types.ModuleType("progressbar"))
    import sightpy
    from sightpy.utils.vector3 import vec3

    def _ufunc(self, uf, method, *ins, **kw):
        if method != "__call__":
            return NotImplemented
        return vec3(*[uf(*[getattr(i, c) if isinstance(i, vec3) else i for i in ins], **kw) for c in "xyz"])

    vec3.__array_ufunc__ = _ufunc
    return sightpy


class _Captured(Exception):
    pass


def capture_scene(sp, script, width, height, depth):
    """Execute an example script with the camera size and depth overridden; return its Scene."""
    orig_cam = sp.Scene.add_Camera
    orig_render = sp.Scene.render
    box = {}

    def add_camera(self, look_from, look_at, **kw):
        kw["screen_width"], kw["screen_height"] = width, height
        return orig_cam(self, look_from, look_at, **kw)

    def render(self, *a, **k):
        box["scene"] = self
        raise _Captured()

    sp.Scene.add_Camera, sp.Scene.render = add_camera, render
    try:
        runpy.run_path(str(REF / script), run_name="__main__")
    except _Captured:
        pass
    finally:
        sp.Scene.add_Camera, sp.Scene.render = orig_cam, orig_render
    sc = box["scene"]
    if depth is not None:
        for p in sc.scene_primitives:
            p.max_ray_depth = depth
    return sc


def instrument(sp):
    """Wrap get_raycolor everywhere it is referenced to count rays per depth."""
    import importlib

    counts = {}
    orig = getattr(sp.ray, "_golden_original", None) or sp.ray.get_raycolor
    sp.ray._golden_original = orig

    def counted(ray, scene):
        counts[ray.depth] = counts.get(ray.depth, 0) + len(ray)
        return orig(ray, scene)

    for mod in ["sightpy.ray", "sightpy.materials.glossy", "sightpy.materials.refractive",
                "sightpy.materials.thin_film_interference", "sightpy.materials.diffuse"]:
        setattr(importlib.import_module(mod), "get_raycolor", counted)
    return counts, counted


def primary_hit_ids(sp, scene, ray):
    from functools import reduce

    inters = [c.intersect(ray.origin, ray.dir) for c in scene.collider_list]
    near = reduce(np.minimum, [i[0] for i in inters])
    ids = np.full(len(ray), -1, dtype=np.int32)
    for k in range(len(inters) - 1, -1, -1):
        ids = np.where((near != sp.FARAWAY) & (inters[k][0] == near), k, ids)
    return ids, near


def render_golden(sp, scene, spp, seed):
    counts, get_rc = instrument(sp)
    np.random.seed(seed)
    rays = [scene.camera.get_ray(scene.n) for _ in range(spp)]
    scene.camera.get_ray(scene.n)  # scene.py:81
    acc = sp.rgb(0.0, 0.0, 0.0)
    hits, nears = [], []
    for r in rays:
        ids, near = primary_hit_ids(sp, scene, r)
        hits.append(ids)
        nears.append(near)
        acc = acc + get_rc(r, scene)
    lin = (acc / spp).to_array()
    enc = sp.sRGB_linear_to_sRGB(lin)
    H, W = scene.camera.screen_height, scene.camera.screen_width
    u8 = np.stack([(255 * np.clip(c, 0, 1).reshape((H, W))).astype(np.uint8) for c in enc], axis=-1)
    depth_counts = np.array([counts.get(d, 0) for d in range(max(counts) + 1)], dtype=np.int64)
    return lin, u8, np.array(hits), np.array(nears), depth_counts


CONFIGS = [
    # name, script, W, H, depth, spp, seed, store linear RGB as
    ("ex1_64x48_d3_s2", "example1.py", 64, 48, None, 2, 0, "f8"),
    ("ex1_160x120_d5_s1", "example1.py", 160, 120, 5, 1, 3, "f8"),
    ("ex2_64x48_d3_s2", "example2.py", 64, 48, None, 2, 0, "f8"),
    ("ex3_64x48_d8_s2", "example3.py", 64, 48, 8, 2, 0, "f8"),
    ("ex4_48x36_d6_s1", "example4.py", 48, 36, 6, 1, 0, "f8"),
    ("cornell_24x24_s1", "example_cornellbox.py", 24, 24, None, 1, 0, "f8"),
    ("ex1_400x300_d3_s6", "example1.py", 400, 300, None, 6, 0, "f4"),
]


def gen_examples(sp, only=None):
    for name, script, W, H, depth, spp, seed, rgb_dtype in CONFIGS:
        if only and name not in only:
            continue
        scene = capture_scene(sp, script, W, H, depth)
        lin, u8, hits, nears, counts = render_golden(sp, scene, spp, seed)
        extra = {} if rgb_dtype == "f4" else {"nearest": nears}
        np.savez_compressed(OUT / (name + ".npz"), rgb=lin.astype(rgb_dtype), srgb8=u8, hit_id=hits.astype(np.int16),
                            depth_counts=counts, seed=seed, spp=spp, width=W, height=H,
                            depth=-1 if depth is None else depth, **extra)
        print(name, "rays per depth", counts.tolist(), "rgb mean", lin.mean())


FEATURE_CONFIGS = [
    # name, W, H, depth, spp, seed: tests/scenes.py:features built with the reference's module
    ("features_64x48_d4_s2", 64, 48, 4, 2, 0),
]


def gen_features(sp):
    sys.path.insert(0, str(OUT.parent))
    import scenes

    for name, W, H, depth, spp, seed in FEATURE_CONFIGS:
        scene = scenes.features(W, H, depth, sp=sp)
        lin, u8, hits, nears, counts = render_golden(sp, scene, spp, seed)
        np.savez_compressed(OUT / (name + ".npz"), rgb=lin, srgb8=u8, hit_id=hits.astype(np.int16), nearest=nears,
                            depth_counts=counts, seed=seed, spp=spp, width=W, height=H, depth=depth)
        print(name, "rays per depth", counts.tolist(), "rgb mean", lin.mean())


MC_CONFIGS = [
    # name, W, H, depth, spp, seed: Monte-Carlo refraction (Primitive.mc, refractive.py:95-101) -- the
    # glass sphere of the cornell box / of tests/scenes.py:features with mc=True, rendered by the
    # reference in one process (seeded, hence deterministic)
    ("cornell_mc_24x24_s1", 24, 24, None, 1, 0),
    ("features_mc_48x36_d4_s2", 48, 36, 4, 2, 0),
]


def gen_mc(sp):
    sys.path.insert(0, str(OUT.parent))
    import scenes

    for name, W, H, depth, spp, seed in MC_CONFIGS:
        if name.startswith("cornell"):
            scene = capture_scene(sp, "example_cornellbox.py", W, H, depth)
            glass = [p for p in scene.scene_primitives if type(p.material).__name__ == "Refractive"]
            assert len(glass) == 1
            glass[0].mc = True
        else:
            scene = scenes.features(W, H, depth, sp=sp, mc=True)
        lin, u8, hits, nears, counts = render_golden(sp, scene, spp, seed)
        np.savez_compressed(OUT / (name + ".npz"), rgb=lin, srgb8=u8, hit_id=hits.astype(np.int16), nearest=nears,
                            depth_counts=counts, seed=seed, spp=spp, width=W, height=H, depth=-1 if depth is None else depth)
        print(name, "rays per depth", counts.tolist(), "rgb mean", lin.mean())


# SURVEY 8(c) statistical pin of the cornell box: per-seed means of every 10x10 pixel block (linear
# RGB) of single-process seeded renders by the reference
CORNELL_STATS = ("cornell_stats_80x80", 80, 80, 8, 16)  # name, W, H, spp per seed, seeds


def gen_cornell_stats(sp):
    name, W, H, spp, nseeds = CORNELL_STATS
    scene = capture_scene(sp, "example_cornellbox.py", W, H, None)
    blocks = np.empty((nseeds, 3, H // 10, W // 10))
    for s in range(nseeds):
        lin, _, _, _, counts = render_golden(sp, scene, spp, 1000 + s)
        blocks[s] = lin.reshape(3, H // 10, 10, W // 10, 10).mean(axis=(2, 4))
        print(name, "seed", s, "rays", int(counts.sum()), "mean", lin.mean())
    np.savez_compressed(OUT / (name + ".npz"), block_means=blocks, seeds=1000 + np.arange(nseeds), spp=spp, width=W,
                        height=H, block=10)


def gen_colliders(sp):
    """Known-answer tests of every collider's intersect on random and edge-case rays."""
    from sightpy.geometry.triangle import Triangle_Collider
    from sightpy.geometry.sphere import Sphere_Collider
    from sightpy.geometry.plane import Plane_Collider
    from sightpy.geometry.cuboid import Cuboid_Collider

    vec3 = sp.vec3
    rng = np.random.default_rng(7)
    n = 4000
    O = rng.uniform(-3, 3, (3, n))
    D = rng.standard_normal((3, n))
    D /= np.sqrt((D * D).sum(0))
    # edge cases: axis-parallel directions, rays from inside, grazing, zero components
    D[:, :6] = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]]).T
    O[:, 6:12] = 0.0
    D[:, 12:18] = D[:, 12:18] * np.array([[1.0], [0.0], [1.0]])
    D[:, 12:18] /= np.sqrt((D[:, 12:18] ** 2).sum(0))
    out = {"O": O, "D": D}
    Ov, Dv = vec3(O[0], O[1], O[2]), vec3(D[0], D[1], D[2])
    prim = types.SimpleNamespace()
    sph = Sphere_Collider(assigned_primitive=prim, center=vec3(0.3, -0.2, 0.1), radius=1.1)
    pl = Plane_Collider(assigned_primitive=prim, center=vec3(0.1, -0.5, 0.2), u_axis=vec3(1.0, 0.0, 0.0),
                        v_axis=vec3(0.0, 0.0, -1.0), w=1.5, h=0.8)
    pl2 = Plane_Collider(assigned_primitive=prim, center=vec3(0.0, 0.2, -0.3), u_axis=vec3(0.6, 0.0, 0.8),
                         v_axis=vec3(0.0, 1.0, 0.0), w=1.0, h=2.0)
    cb = Cuboid_Collider(assigned_primitive=prim, center=vec3(0.2, 0.1, -0.4), width=0.9, height=1.0, length=0.4)
    M = sp.Primitive.__new__(sp.Primitive)
    M.collider_list = [cb]
    M.center = vec3(0.2, 0.1, -0.4)
    sp.Primitive.rotate(M, 30, vec3(0, 1, 0))
    cb_axis = Cuboid_Collider(assigned_primitive=prim, center=vec3(0.0, 0.0, 0.0), width=2.0, height=2.0,
                              length=2.0)
    tri = Triangle_Collider(assigned_surface=prim, p1=vec3(-1.0, -0.5, 0.0), p2=vec3(1.2, -0.4, 0.1),
                            p3=vec3(0.1, 1.3, -0.2))
    for name, c in [("sphere", sph), ("plane", pl), ("plane_tilted", pl2), ("cuboid_rot30", cb),
                    ("cuboid_axis", cb_axis), ("triangle", tri)]:
        out[name] = np.asarray(c.intersect(Ov, Dv), dtype=np.float64)
    out["cuboid_rot30_basis"] = cb.basis_matrix
    out["cuboid_rot30_lb"] = np.array([cb.lb_local_basis.x, cb.lb_local_basis.y, cb.lb_local_basis.z], dtype=np.float64)
    out["cuboid_rot30_rt"] = np.array([cb.rt_local_basis.x, cb.rt_local_basis.y, cb.rt_local_basis.z], dtype=np.float64)
    np.savez_compressed(OUT / "colliders.npz", **out)
    print("colliders", {k: v.shape for k, v in out.items()})


def gen_camera(sp):
    scene = capture_scene(sp, "example1.py", 64, 48, None)
    np.random.seed(0)
    r = scene.camera.get_ray(scene.n)
    after = np.random.rand(3)
    np.savez_compressed(OUT / "camera.npz", O=r.origin.to_array(), D=r.dir.to_array(), rng_after=after,
                        width=64, height=48)
    print("camera", r.origin.to_array().shape)


def gen_textures(sp):
    """The reference's float texture arrays at a few texels (pins the u8 + LUT representation)."""
    from sightpy.utils.image_functions import load_image_as_linear_sRGB, load_image
    from sightpy.backgrounds.util.blur_background import blur_skybox

    rng = np.random.default_rng(3)
    out = {}
    for name, arr in [("checkered", load_image_as_linear_sRGB("sightpy/textures/checkered_floor.png")),
                      ("lake_lightmap", load_image("sightpy/backgrounds/lightmaps/lake.png")),
                      ("lake_blur10", blur_skybox(load_image("sightpy/backgrounds/lake.png"), 10.0, "lake.png"))]:
        r = rng.integers(0, arr.shape[0], 5000)
        c = rng.integers(0, arr.shape[1], 5000)
        out[name + "_rc"] = np.stack([r, c])
        out[name + "_val"] = arr[r, c, :3]
        out[name + "_shape"] = np.array(arr.shape)
    np.savez_compressed(OUT / "textures.npz", **out)
    print("textures", list(out))


if __name__ == "__main__":
    only = sys.argv[1:]
    sp = import_reference()
    if not only or "colliders" in only:
        gen_colliders(sp)
    if not only or "camera" in only:
        gen_camera(sp)
    if not only or "textures" in only:
        gen_textures(sp)
    if not only or "features" in only:
        gen_features(sp)
    if not only or "mc" in only:
        gen_mc(sp)
    if not only or "cornell_stats" in only:
        gen_cornell_stats(sp)
    rest = [o for o in only if o not in ("colliders", "camera", "textures", "features", "mc", "cornell_stats")]
    if not only or rest:
        gen_examples(sp, rest or None)
