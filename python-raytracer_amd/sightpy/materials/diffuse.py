"""Lambertian Monte-Carlo material (reference `materials/diffuse.py:11-124`).

First diffuse bounce fans out `diffuse_rays` rays (cosine or cosine/spherical-cap mixture
importance sampling), the second bounce one ray, none after two.  Device: `rt_shade_diffuse`
with a counter-based Philox RNG keyed by (seed, pixel, sample, path, depth).
"""
from ..utils.vector3 import vec3
from ..textures.texture import texture, solid_color
from .material import Material

__all__ = ["Diffuse"]


class Diffuse(Material):
    def __init__(self, diff_color, diffuse_rays=20, ambient_weight=0.5, **kwargs):
        super().__init__(**kwargs)
        if isinstance(diff_color, vec3):
            self.diff_texture = solid_color(diff_color)
        elif isinstance(diff_color, texture):
            self.diff_texture = diff_color
        self.diffuse_rays = diffuse_rays
        self.max_diffuse_reflections = 2
        self.ambient_weight = ambient_weight
