"""Collider base class (reference `geometry/collider.py:6-18`).

`intersect(O, D)` returns a (2, N) float64 array `[distance; orientation]` with FARAWAY for
misses.  `get_Normal(hit)` / `get_uv(hit)` evaluate the collider's normal and surface
coordinates at `hit.point` (sphere.py:54-64, plane.py:98-105, cuboid.py:142-187,
triangle.py:85-86).  Every one runs on the GPU (`srt_intersect_collider`, `srt_collider_surface`
in `csrc/rt_kernels.hip`); subclasses only describe their parameters (lowered by `_lower.py`).
"""
from ..utils.vector3 import vec3

__all__ = ["Collider"]


def _hit_point(hit):
    if hit.point is None:
        # the reference's materials set it first (glossy.py:27, skybox.py:93, ...)
        raise ValueError("hit.point is unset: set hit.point = ray.origin + ray.dir * hit.distance first")
    return hit.point


class Collider:
    def __init__(self, assigned_primitive, center):
        self.assigned_primitive = assigned_primitive
        self.center = center

    def intersect(self, O, D):
        from .._backend import intersect_collider

        return intersect_collider(self, O, D)

    def get_Normal(self, hit):
        from .._backend import collider_surface

        N, _ = collider_surface(self, _hit_point(hit), uv=False)
        return vec3(N[0], N[1], N[2])

    def get_uv(self, hit):
        from .._backend import collider_surface

        _, uv = collider_surface(self, _hit_point(hit), normal=False)
        return uv[0], uv[1]
