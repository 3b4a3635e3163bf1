"""Oriented box primitive (reference `geometry/cuboid.py:7-187`)."""
import numpy as np

from ..utils.vector3 import vec3
from .primitive import Primitive
from .collider import Collider

__all__ = ["Cuboid", "Cuboid_Collider"]


class Cuboid(Primitive):
    def __init__(self, center, material, width, height, length, max_ray_depth=5, shadow=True):
        super().__init__(center, material, max_ray_depth, shadow=shadow)
        self.width = width
        self.height = height
        self.length = length
        self.bounded_sphere_radius = np.sqrt(
            (self.width / 2) ** 2 + (self.height / 2) ** 2 + (self.length / 2) ** 2
        )
        self.collider_list += [
            Cuboid_Collider(
                assigned_primitive=self, center=center, width=width, height=height, length=length
            )
        ]

    # Primitive.get_uv of a cuboid divides the 4x3 cross coordinates by (4, 3); the device
    # applies it through the collider's UV_CUBE_CROSS flag (reference cuboid.py:29-32).
    uv_cube_cross = True


class Cuboid_Collider(Collider):
    """Slab test in the box's local basis (device: `rt_cuboid_hit`)."""

    def __init__(self, width, height, length, **kwargs):
        super().__init__(**kwargs)
        half = vec3(width / 2, height / 2, length / 2)
        self.lb = self.center - half
        self.rt = self.center + half
        self.lb_local_basis = self.lb
        self.rt_local_basis = self.rt
        self.width = width
        self.height = height
        self.length = length
        self.ax_w = vec3(1.0, 0.0, 0.0)
        self.ax_h = vec3(0.0, 1.0, 0.0)
        self.ax_l = vec3(0.0, 0.0, 1.0)
        self._refresh_basis()

    def _refresh_basis(self):
        a, b, c = self.ax_w, self.ax_h, self.ax_l
        self.inverse_basis_matrix = np.array([[a.x, b.x, c.x], [a.y, b.y, c.y], [a.z, b.z, c.z]])
        self.basis_matrix = self.inverse_basis_matrix.T

    def rotate(self, M, center):
        self.ax_w = self.ax_w.matmul(M)
        self.ax_h = self.ax_h.matmul(M)
        self.ax_l = self.ax_l.matmul(M)
        self._refresh_basis()
        self.lb = center + (self.lb - center).matmul(M)
        self.rt = center + (self.rt - center).matmul(M)
        self.lb_local_basis = self.lb.matmul(self.basis_matrix)
        self.rt_local_basis = self.rt.matmul(self.basis_matrix)
