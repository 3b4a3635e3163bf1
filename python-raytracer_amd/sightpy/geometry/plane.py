"""Finite rectangle primitive (reference `geometry/plane.py:7-105`)."""
import numpy as np

from .primitive import Primitive
from .collider import Collider

__all__ = ["Plane", "Plane_Collider"]


class Plane(Primitive):
    def __init__(self, center, material, width, height, u_axis, v_axis, max_ray_depth=5, shadow=True):
        super().__init__(center, material, max_ray_depth, shadow=shadow)
        self.collider_list += [
            Plane_Collider(
                assigned_primitive=self,
                center=center,
                u_axis=u_axis,
                v_axis=v_axis,
                w=width / 2,
                h=height / 2,
            )
        ]
        self.width = width
        self.height = height
        self.bounded_sphere_radius = np.sqrt((width / 2) ** 2 + (height / 2) ** 2)


def _basis_from_columns(a, b, c):
    return np.array([[a.x, b.x, c.x], [a.y, b.y, c.y], [a.z, b.z, c.z]])


class Plane_Collider(Collider):
    """Ray/rectangle test (device: `rt_plane_hit`)."""

    def __init__(self, u_axis, v_axis, w, h, uv_shift=(0.0, 0.0), **kwargs):
        super().__init__(**kwargs)
        self.normal = u_axis.cross(v_axis).normalize()
        self.w = w
        self.h = h
        self.u_axis = u_axis
        self.v_axis = v_axis
        self.uv_shift = uv_shift
        self.inverse_basis_matrix = _basis_from_columns(self.u_axis, self.v_axis, self.normal)
        self.basis_matrix = self.inverse_basis_matrix.T

    def rotate(self, M, center):
        self.u_axis = self.u_axis.matmul(M)
        self.v_axis = self.v_axis.matmul(M)
        self.normal = self.normal.matmul(M)
        self.center = center + (self.center - center).matmul(M)
