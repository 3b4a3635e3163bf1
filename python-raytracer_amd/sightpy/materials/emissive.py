"""Emissive material (reference `materials/emissive.py:11-23`): returns its texture colour."""
from ..utils.vector3 import vec3
from ..textures.texture import texture, solid_color
from .material import Material

__all__ = ["Emissive"]


class Emissive(Material):
    def __init__(self, color, **kwargs):
        if isinstance(color, vec3):
            self.texture_color = solid_color(color)
        elif isinstance(color, texture):
            self.texture_color = color
        super().__init__(**kwargs)
