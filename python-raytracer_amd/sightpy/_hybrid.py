"""Scenes holding user subclasses of `Collider` or `Material`: the reference's duck-typed plugin
dispatch (`ray.py:122-148` calls `intersect` and `get_color` on whatever the lists hold; contracts
at `geometry/collider.py:12-14` and `materials/material.py:42-44`).

A user class's Python methods cannot run inside a kernel, so such a scene is traced by the
reference's own recursion structure, driven from the host one batch level at a time, with every
step the device can take on the device:

  * intersect: built-in colliders on the device (`srt_intersect_collider`), a user collider's own
    `intersect(O, D)` (its code, on its batch);
  * nearest hit and the tie rule: as ray.py:127-135 (every collider at the nearest distance shades
    its rays, the colours added);
  * get_color: a user material's own `get_color(scene, ray, hit)` (its recursion through
    `get_raycolor` comes back here); a built-in material on a built-in collider shades its rays on
    the device one level deep (`srt_shade_level`: the colour it adds before its children, and the
    children with the factor their colour is multiplied by), and the children are traced by this
    same recursion, so they can hit user colliders.

Scenes made only of built-in classes never come here: they render in the device kernels whole.

What the device cannot do for a user class is refused (NotImplementedError) rather than computed
on the CPU: a built-in material on a user collider (the device shaders take the surface from the
built-in colliders' device code), and a user collider casting shadows (`shadow=True`) in a scene
with built-in Glossy materials (their shadow rays, glossy.py:54-67, are traced on the device
against the device's colliders; a built-in collider with a user material is one of them).  Monte-Carlo materials (Diffuse, `mc=True` Refractive) shaded on
the device here draw from the device stream keyed by each level's ray index: valid samples, but not
the ones a whole-device render of the same pixel draws.
"""
from functools import reduce

import numpy as np

from .utils.constants import FARAWAY
from .utils.vector3 import vec3, rgb, extract

__all__ = ["device_collider", "device_material", "on_device", "is_hybrid", "raycolor", "shade_level",
           "render_linear", "nearest_distance"]

_SURFACE_METHODS = ("intersect", "get_Normal", "get_uv")


def _builtin_colliders():
    from .geometry.sphere import Sphere_Collider
    from .geometry.plane import Plane_Collider
    from .geometry.cuboid import Cuboid_Collider
    from .geometry.triangle import Triangle_Collider

    return (Sphere_Collider, Plane_Collider, Cuboid_Collider, Triangle_Collider)


def _builtin_materials():
    from .materials import Glossy, Refractive, ThinFilmInterference, Diffuse, Emissive
    from .backgrounds.skybox import SkyBox_Material

    return (Glossy, Refractive, ThinFilmInterference, Diffuse, Emissive, SkyBox_Material)


def device_collider(c):
    """A built-in collider (or a subclass of one that keeps its intersect / get_Normal / get_uv):
    its intersection and surface run in the device code."""
    for base in _builtin_colliders():
        if isinstance(c, base):
            t = type(c)
            return all(getattr(t, m, None) is getattr(base, m, None) for m in _SURFACE_METHODS)
    return False


def device_material(m):
    """A built-in material (or a subclass of one that keeps its get_color)."""
    from .materials.material import Material

    return isinstance(m, _builtin_materials()) and type(m).get_color is Material.get_color


def on_device(c):
    """The collider and its material both lower to the device tables."""
    return device_collider(c) and device_material(c.assigned_primitive.material)


def is_hybrid(scene):
    """Whether `scene` holds a user Collider / Material subclass (cached per collider list)."""
    key = (id(scene.collider_list), len(scene.collider_list))
    cached = getattr(scene, "_hybrid_key", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    res = not all(on_device(c) for c in scene.collider_list)
    if res:
        _check(scene)
    scene._hybrid_key = (key, res)
    return res


def _check(scene):
    from .materials import Glossy

    for c in scene.collider_list:
        m = c.assigned_primitive.material
        if not device_collider(c) and device_material(m):
            raise NotImplementedError(
                "built-in material %s on the user collider %s: the device shaders take the hit's surface from "
                "the built-in colliders; give the collider a user Material" % (type(m).__name__, type(c).__name__))
    shadowing = [c for c in scene.shadowed_collider_list if not device_collider(c)]
    glossy = [c for c in scene.collider_list if on_device(c) and isinstance(c.assigned_primitive.material, Glossy)]
    if shadowing and glossy:
        raise NotImplementedError(
            "the user collider %s casts shadows (shadow=True) on built-in Glossy materials, whose shadow rays "
            "(glossy.py:54-67) are traced on the device; add its primitive with shadow=False"
            % type(shadowing[0]).__name__)


def _intersect(c, ray):
    """(distance, orientation) arrays of collider c for the batch (collider.py:12-14 contract)."""
    if device_collider(c):
        from ._backend import intersect_collider

        out = intersect_collider(c, ray.origin, ray.dir)
        return out[0], out[1]
    d, o = c.intersect(ray.origin, ray.dir)
    n = len(ray)
    return (np.broadcast_to(np.asarray(d, dtype=np.float64), (n,)),
            np.broadcast_to(np.asarray(o, dtype=np.float64), (n,)))


def nearest_distance(ray, scene):
    """reduce(np.minimum, distances) over every collider (ray.py:125-129)."""
    return reduce(np.minimum, [_intersect(c, ray)[0] for c in scene.collider_list])


def raycolor(ray, scene):
    """get_raycolor (ray.py:122-148) of a batch in a scene with user classes."""
    from .ray import Hit

    inters = [_intersect(c, ray) for c in scene.collider_list]
    distances, orientations = zip(*inters)
    nearest = reduce(np.minimum, distances)
    color = rgb(0.0, 0.0, 0.0)
    for coll, dis, orient in zip(scene.collider_list, distances, orientations):
        hit_check = (nearest != FARAWAY) & (dis == nearest)
        if np.any(hit_check):
            material = coll.assigned_primitive.material
            hit = Hit(extract(hit_check, dis), extract(hit_check, orient), material, coll, coll.assigned_primitive)
            cc = material.get_color(scene, ray.extract(hit_check), hit)
            color += cc.place(hit_check)
    return color


def shade_level(scene, material, ray, hit):
    """A built-in material's get_color in a scene with user classes: its own colour from the
    device (srt_shade_level), plus each child's colour (this recursion) times its factor."""
    import ctypes

    from . import _backend as B, _native as N
    from .ray import Ray

    lib, ctx = B.context()
    n = len(ray)
    uniq, inv = B._media_of(ray.n, n)
    L = B.upload(scene, extra_media=uniq)
    remap = np.array([L.media_keys.index(k) for k in uniq], dtype=np.int32)
    med = np.ascontiguousarray(remap[inv])
    dev = L.device_index[scene.collider_list.index(hit.collider)]
    O, D = B._planar(ray.origin, n), B._planar(ray.dir, n)
    local = np.empty((3, n))
    a = N.TraceArgs()
    a.n = n
    a.origin, a.dir, a.medium = N.ptr(O), N.ptr(D), N.ptr(med)
    a.depth, a.diffuse_reflections = int(ray.depth), int(ray.diffuse_reflections)
    a.seed = int(B._default_seed()) & (2**64 - 1)
    a.out_rgb = N.ptr(local)
    ids = np.full(n, dev, dtype=np.int32)
    t = np.ascontiguousarray(np.broadcast_to(np.asarray(hit.distance, dtype=np.float64), (n,)))
    o = np.ascontiguousarray(np.broadcast_to(np.asarray(hit.orientation, dtype=np.float64), (n,)))
    cap = 2 * n  # (a refractive hit's two children; a Diffuse fan-out asks for more, below)
    for _ in range(2):
        arrs = {"origin": np.empty((3, cap)), "dir": np.empty((3, cap)), "weight": np.empty((3, cap)),
                "parent": np.empty(cap, np.int32), "medium": np.empty(cap, np.int32),
                "depth": np.empty(cap, np.int32), "diffuse_reflections": np.empty(cap, np.int32)}
        kids = N.Children()
        kids.cap = cap
        for k, v in arrs.items():
            setattr(kids, k, N.ptr(v))
        rc = lib.srt_shade_level(ctx, ctypes.byref(a), N.ptr(ids), N.ptr(t), N.ptr(o), ctypes.byref(kids), None)
        if rc != 0 and kids.n > cap:
            cap = int(kids.n)  # room for them all, then once more
            continue
        N.check(lib, rc)
        break
    color = [local[0].copy(), local[1].copy(), local[2].copy()]
    nk = int(kids.n)
    if nk:
        media = np.array([[complex(v) for v in L.media_keys[m]] for m in range(len(L.media_keys))])
        depth, dfl = arrs["depth"][:nk], arrs["diffuse_reflections"][:nk]
        # the reference's batches carry one depth and one diffuse count: one batch per pair
        for dv, fv in sorted(set(zip(depth.tolist(), dfl.tolist()))):
            sel = np.nonzero((depth == dv) & (dfl == fv))[0]
            mk = media[arrs["medium"][:nk][sel]]
            child = Ray(vec3(*(arrs["origin"][k, sel] for k in range(3))), vec3(*(arrs["dir"][k, sel] for k in range(3))),
                        dv, vec3(mk[:, 0], mk[:, 1], mk[:, 2]), 0, 0, fv)
            cc = raycolor(child, scene)
            par = arrs["parent"][:nk][sel]
            for k, comp in enumerate((cc.x, cc.y, cc.z)):
                np.add.at(color[k], par, arrs["weight"][k, sel] * np.broadcast_to(comp, sel.shape))
    return rgb(color[0], color[1], color[2])


def render_linear(scene, samples_per_pixel):
    """Scene.render's linear colour (scene.py:71-118) for a scene with user classes: numpy's stream
    drawn in the reference's order (spp get_ray draws, then the sizing draw), every sample's batch
    through raycolor, averaged."""
    rays = [scene.camera.get_ray(scene.n) for _ in range(samples_per_pixel)]
    scene.camera.get_ray(scene.n)  # the reference's sizing draw (scene.py:81)
    color = rgb(0.0, 0.0, 0.0)
    for r in rays:
        color += raycolor(r, scene)
    return color / samples_per_pixel
