"""Collider base class (reference `geometry/collider.py:6-18`).

`intersect(O, D)` returns a (2, N) float64 array `[distance; orientation]` with FARAWAY for
misses.  In this package the computation runs on the GPU (`srt_intersect_collider` in
`csrc/rt_kernels.hip`); subclasses only describe their parameters via `_lower()`.
"""
import numpy as np

__all__ = ["Collider"]


class Collider:
    def __init__(self, assigned_primitive, center):
        self.assigned_primitive = assigned_primitive
        self.center = center

    def intersect(self, O, D):
        from .._backend import intersect_collider

        return intersect_collider(self, O, D)

    def get_Normal(self, hit):
        raise NotImplementedError(
            "%s.get_Normal is evaluated on the device inside the shading kernels"
            % type(self).__name__
        )
