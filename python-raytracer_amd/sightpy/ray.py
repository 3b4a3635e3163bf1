"""Ray batches and the recursive colour entry point (reference `sightpy/ray.py:7-163`).

`Ray` and `Hit` keep the reference's batch containers.  `get_raycolor(ray, scene)` — the
reference's recursive numpy driver (ray.py:122-148) — is served by the device wavefront tracer:
the batch is uploaded, traced to completion by the HIP kernels (intersect -> nearest -> shade ->
child rays, depth by depth) and the per-ray colours are returned.  A scene holding user subclasses of
Collider / Material (duck-typed plugins) goes through `_hybrid.raycolor`, this recursion driven
from the host with the device doing every built-in step.  `get_distances` is the
nearest-hit probe (ray.py:151-163).
"""
import numpy as np

from .utils.constants import *
from .utils.vector3 import vec3, extract, rgb

__all__ = ["Ray", "Hit", "get_raycolor", "get_distances"]


class Ray:
    """Info of the ray batch and the media it travels in (reference ray.py:7-94)."""

    def __init__(self, origin, dir, depth, n, reflections, transmissions, diffuse_reflections):
        self.length = max(len(origin), len(dir), len(n))
        shape = [self.length]
        self.origin = origin.broadcast_to(shape)
        self.dir = dir.broadcast_to(shape)
        self.depth = depth
        self.n = n.broadcast_to(shape)
        self.reflections = reflections
        self.transmissions = transmissions
        self.diffuse_reflections = diffuse_reflections

    def extract(self, hit_check):
        return Ray(self.origin.extract(hit_check), self.dir.extract(hit_check), self.depth,
                   self.n.extract(hit_check), self.reflections, self.transmissions,
                   self.diffuse_reflections)

    def __len__(self):
        return self.length

    def __getitem__(self, ind):
        return Ray(self.origin[ind], self.dir[ind], self.depth, self.n[ind], self.reflections,
                   self.transmissions, self.diffuse_reflections)

    @staticmethod
    def where(cond, x, y):
        if x.depth != y.depth:
            raise ValueError("Both rays must have same depth")
        return Ray(vec3.where(cond, x.origin, y.origin), vec3.where(cond, x.dir, y.dir), x.depth,
                   vec3.where(cond, x.n, y.n), max(x.reflections, y.reflections),
                   max(x.transmissions, y.transmissions),
                   max(x.diffuse_reflections, y.diffuse_reflections))

    @staticmethod
    def concatenate(rays):
        depth = rays[0].depth
        if not all(r.depth == depth for r in rays):
            print("All rays must have same depth!")
        return Ray(vec3.concatenate([r.origin for r in rays]), vec3.concatenate([r.dir for r in rays]),
                   depth, vec3.concatenate([r.n for r in rays]),
                   max(r.reflections for r in rays), max(r.transmissions for r in rays),
                   max(r.diffuse_reflections for r in rays))


class Hit:
    """Info of a ray-surface intersection batch (reference ray.py:97-119)."""

    def __init__(self, distance, orientation, material, collider, surface):
        self.distance = distance
        self.orientation = orientation
        self.material = material
        self.collider = collider
        self.surface = surface
        self.u = None
        self.v = None
        self.N = None
        self.point = None

    def get_uv(self):
        if self.u is None:  # computed once per hit (ray.py:111-114)
            self.u, self.v = self.collider.assigned_primitive.get_uv(self)
        return self.u, self.v

    def get_normal(self):
        # ray.py:116-119 calls collider.get_N, which no collider defines; get_Normal is meant
        if self.N is None:
            self.N = self.collider.get_Normal(self)
        return self.N


def get_raycolor(ray, scene):
    """Colour of every ray of the batch (reference ray.py:122-148), traced on the GPU; a scene with
    user Collider / Material subclasses through the host-driven recursion (_hybrid.py)."""
    from ._backend import trace_rays
    from . import _hybrid

    if _hybrid.is_hybrid(scene):
        return _hybrid.raycolor(ray, scene)
    return trace_rays(ray, scene)


def get_distances(ray, scene):
    """Grey map min(nearest, 10)/10 of the batch (reference ray.py:151-163), on the GPU."""
    from ._backend import nearest_hits
    from . import _hybrid

    if _hybrid.is_hybrid(scene):
        t = _hybrid.nearest_distance(ray, scene)
    else:
        t, _, _ = nearest_hits(scene, ray.origin, ray.dir)
    g = np.where(t <= 10, t, 10) / 10
    return rgb(g, g, g)
