"""Sphere primitive (reference `geometry/sphere.py:7-64`)."""
import numpy as np

from .primitive import Primitive
from .collider import Collider

__all__ = ["Sphere", "Sphere_Collider"]


class Sphere(Primitive):
    def __init__(self, center, material, radius, max_ray_depth=5, shadow=True, mc=False):
        super().__init__(center, material, max_ray_depth, shadow=shadow, mc=mc)
        self.collider_list += [Sphere_Collider(assigned_primitive=self, center=center, radius=radius)]
        self.bounded_sphere_radius = radius


class Sphere_Collider(Collider):
    """Ray/sphere quadratic, unit-length D assumed (device: `rt_sphere_hit`)."""

    def __init__(self, radius, **kwargs):
        super().__init__(**kwargs)
        self.radius = radius

    def rotate(self, M, center):
        # the reference sphere collider has no rotate(); a sphere is rotation invariant
        # except for its uv frame, which the reference never rotates either.
        pass
