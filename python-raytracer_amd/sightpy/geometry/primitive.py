"""Primitive base class (reference `geometry/primitive.py:6-44`).

A primitive owns colliders, a material and the per-primitive recursion limit.  All fields are
lowered to the device collider table by `sightpy/_lower.py`.
"""
import numpy as np

__all__ = ["Primitive", "rotation_matrix"]


def rotation_matrix(theta_deg, axis):
    """Rodrigues rotation matrix, evaluated exactly as reference `primitive.py:16-40`.

    `sin` is derived from `cos` (sqrt(1 - cos^2) * sign), which is what the reference does, so
    rotated cuboid/plane bases uploaded to the device are bit-identical.
    """
    u = axis.normalize()
    t = theta_deg / 180 * np.pi
    c = np.cos(t)
    s = np.sqrt(1 - c ** 2) * np.sign(t)
    k = 1 - c
    return np.array(
        [
            [c + u.x * u.x * k, u.x * u.y * k - u.z * s, u.x * u.z * k + u.y * s],
            [u.y * u.x * k + u.z * s, c + u.y ** 2 * k, u.y * u.z * k - u.x * s],
            [u.z * u.x * k - u.y * s, u.z * u.y * k + u.x * s, c + u.z * u.z * k],
        ]
    )


class Primitive:
    def __init__(self, center, material, max_ray_depth=1, shadow=True, mc=False):
        self.center = center
        self.material = material
        self.material.assigned_primitive = self
        self.shadow = shadow
        self.collider_list = []
        self.max_ray_depth = max_ray_depth
        self.mc = mc

    def rotate(self, θ, u):
        M = rotation_matrix(θ, u)
        for c in self.collider_list:
            c.rotate(M, self.center)

    uv_cube_cross = False  # Cuboid / SkyBox: the cube-cross texture layout (cuboid.py:29-32)

    def get_uv(self, hit):
        """Texture coordinates of the hit (sphere.py:17, plane.py:34, cuboid.py:29-32)."""
        u, v = hit.collider.get_uv(hit)
        if self.uv_cube_cross:
            u, v = u / 4, v / 3
        return u, v
