"""Textures (reference `textures/texture.py:8-39`).

`image` keeps the decoded uint8 texels; the device gathers `lut[byte]` with the reference's
index arithmetic (truncate, floor-mod, negative-row wrap).  `img` is provided for API parity and
equals the reference's `load_image_as_linear_sRGB` array.
"""
from functools import cached_property

import numpy as np

from ..utils.image_functions import load_image_u8
from ..utils.colour_functions import sRGB_to_sRGB_linear
from ..utils.vector3 import vec3

__all__ = ["texture", "solid_color", "image"]


class texture:
    def get_color(self, hit):
        raise NotImplementedError


class solid_color(texture):
    def __init__(self, color):
        self.color = color

    def get_color(self, hit):
        return self.color


class image(texture):
    def __init__(self, img, repeat=1.0):
        print("proccesing " + img.split("/")[-1])
        self.name = img
        self.u8 = load_image_u8("sightpy/textures/" + img)
        self.repeat = repeat

    @cached_property
    def img(self):
        return sRGB_to_sRGB_linear(self.u8 / 256.0)

    def get_color(self, hit):
        """The texel at hit.get_uv() (texture.py:32-39), gathered on the device (srt_texture_lookup)."""
        from .._backend import texture_lookup

        u, v = hit.get_uv()
        c = texture_lookup(self.u8, self.repeat, u, v)
        return vec3(c[0], c[1], c[2])
