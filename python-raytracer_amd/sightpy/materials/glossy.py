"""Glossy material (reference `materials/glossy.py:11-110`).

Ambient + per-light Lambert with a shadow ray + Schlick/Phong specular + Fresnel-weighted
mirror reflection.  Device: `rt_shade_glossy` (csrc/rt_device.h).
"""
from ..utils.vector3 import vec3
from ..textures.texture import texture, solid_color
from .material import Material

__all__ = ["Glossy"]


class Glossy(Material):
    def __init__(self, diff_color, roughness, spec_coeff, diff_coeff, n, **kwargs):
        super().__init__(**kwargs)
        if isinstance(diff_color, vec3):
            self.diff_texture = solid_color(diff_color)
        elif isinstance(diff_color, texture):
            self.diff_texture = diff_color
        self.roughness = roughness
        self.diff_coeff = diff_coeff
        self.spec_coeff = spec_coeff
        self.n = n
