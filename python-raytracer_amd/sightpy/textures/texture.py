"""Textures (reference `textures/texture.py:8-39`).

`image` keeps the decoded uint8 texels; the device gathers `lut[byte]` with the reference's
index arithmetic (truncate, floor-mod, negative-row wrap).  `img` is provided for API parity and
equals the reference's `load_image_as_linear_sRGB` array.
"""
from functools import cached_property

import numpy as np

from ..utils.image_functions import load_image_u8
from ..utils.colour_functions import sRGB_to_sRGB_linear

__all__ = ["texture", "solid_color", "image"]


class texture:
    def get_color(self, hit):
        raise NotImplementedError("texture lookups run on the device")


class solid_color(texture):
    def __init__(self, color):
        self.color = color


class image(texture):
    def __init__(self, img, repeat=1.0):
        print("proccesing " + img.split("/")[-1])
        self.name = img
        self.u8 = load_image_u8("sightpy/textures/" + img)
        self.repeat = repeat

    @cached_property
    def img(self):
        return sRGB_to_sRGB_linear(self.u8 / 256.0)
