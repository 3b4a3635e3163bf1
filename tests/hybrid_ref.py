"""The reference's get_raycolor recursion (ray.py:122-148) for scenes with user classes, on the CPU,
for the duck-typed plugin tests: built-in colliders and materials through the oracle
(oracle/sightpy_oracle.py: intersect, shade), user ones through their own methods.  Test
infrastructure: the expected frames of tests/test_gpu_hybrid.py."""
import numpy as np

import sightpy_oracle as O
from sightpy import _hybrid
from sightpy.ray import Ray, Hit
from sightpy.utils.vector3 import vec3


def _rays_of(ray):
    """sightpy Ray batch -> oracle Rays"""
    n = len(ray)
    nn = np.array([np.broadcast_to(np.asarray(c, dtype=np.complex128), (n,)) for c in (ray.n.x, ray.n.y, ray.n.z)])
    Oa = np.array([np.broadcast_to(np.asarray(c, dtype=np.float64), (n,)) for c in (ray.origin.x, ray.origin.y, ray.origin.z)])
    Da = np.array([np.broadcast_to(np.asarray(c, dtype=np.float64), (n,)) for c in (ray.dir.x, ray.dir.y, ray.dir.z)])
    return O.Rays(Oa, Da, nn, ray.depth, ray.diffuse_reflections)


def _ray_of(r):
    n = len(r)
    nn = np.broadcast_to(r.n, (3, n))
    return Ray(vec3(*r.O), vec3(*r.D), r.depth, vec3(nn[0], nn[1], nn[2]), 0, 0, r.dfl)


def raycolor(scene, r, counts):
    """oracle.raycolor with user classes (installed over it while expected frames are made, so the
    oracle's shaders recurse through it)."""
    dists = []
    for c in scene.collider_list:
        if _hybrid.device_collider(c):
            dists.append(O.intersect(c, r.O, r.D))
        else:
            d, o = c.intersect(vec3(*r.O), vec3(*r.D))
            dists.append(np.array([np.broadcast_to(d, (len(r),)), np.broadcast_to(o, (len(r),))], dtype=np.float64))
    near = dists[0][0]
    for d in dists[1:]:
        near = np.minimum(near, d[0])
    color = np.zeros((3, len(r)))
    for c, d in zip(scene.collider_list, dists):
        hit = (near != O.FARAWAY) & (d[0] == near)
        if np.any(hit):
            m = c.assigned_primitive.material
            sub = r.take(hit)
            if _hybrid.device_material(m):
                cc = O.shade(scene, c, sub, d[0][hit], d[1][hit], counts)
            else:
                h = Hit(d[0][hit], d[1][hit], m, c, c.assigned_primitive)
                v = m.get_color(scene, _ray_of(sub), h)
                cc = np.array([np.broadcast_to(np.asarray(x, dtype=np.float64), (sub.O.shape[1],)) for x in (v.x, v.y, v.z)])
            color = color + O.place(cc, hit)
    return color


def trace(ray, scene):
    """get_raycolor for Tinted's children in the expected frames"""
    col = raycolor(scene, _rays_of(ray), {})
    return vec3(col[0], col[1], col[2])


def render_linear(scene, jit):
    """Sum over samples / spp with raycolor above (jit: (spp, 4, n), numpy's draws)."""
    saved = O.raycolor
    O.raycolor = raycolor
    try:
        acc = 0.0
        for s in range(jit.shape[0]):
            Oa, Da = O.primary_rays(scene.camera, jit[s])
            acc = acc + raycolor(scene, O.Rays(Oa, Da, O.scene_medium(scene), 0, 0), {})
    finally:
        O.raycolor = saved
    return acc / jit.shape[0]
