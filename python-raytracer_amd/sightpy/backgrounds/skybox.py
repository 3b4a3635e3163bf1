"""Cube-map background (reference `backgrounds/skybox.py:9-94`).

A 2e6-wide `Cuboid_Collider` around `center` shaded by `SkyBox_Material`: texel of the 4x3 cross
(optionally the seam-aware blurred cross) plus `light_intensity * lightmap` for non-primary rays.
Device: `rt_shade_sky`.
"""
from functools import cached_property

from ..geometry import Cuboid_Collider, Primitive
from ..materials import Material
from ..utils.vector3 import vec3
from ..utils.constants import SKYBOX_DISTANCE
from ..utils.image_functions import load_image_u8
from ..utils.colour_functions import sRGB_to_sRGB_linear
from .util.blur_background import blur_skybox_u8

__all__ = ["SkyBox", "SkyBox_Material"]


class SkyBox(Primitive):
    uv_cube_cross = True

    def __init__(self, cubemap, center=vec3(0.0, 0.0, 0.0), light_intensity=0.0, blur=0.0):
        super().__init__(center, SkyBox_Material(cubemap, light_intensity, blur), shadow=False)
        l = SKYBOX_DISTANCE
        self.light_intensity = light_intensity
        self.collider_list += [
            Cuboid_Collider(assigned_primitive=self, center=center, width=2 * l, height=2 * l, length=2 * l)
        ]


class SkyBox_Material(Material):
    def __init__(self, cubemap, light_intensity, blur):
        self.normalmap = None
        self.cubemap = cubemap
        print("proccesing " + cubemap)
        self.texture_u8 = load_image_u8("sightpy/backgrounds/" + cubemap)
        self.lightmap_u8 = None
        self.blur_u8 = None
        if light_intensity != 0.0:
            self.lightmap_u8 = load_image_u8("sightpy/backgrounds/lightmaps/" + cubemap)
        if blur != 0.0:
            self.blur_u8 = blur_skybox_u8(self.texture_u8, blur, cubemap)
        self.blur = blur
        self.light_intensity = light_intensity
        self.repeat = 1.0

    @cached_property
    def texture(self):
        return sRGB_to_sRGB_linear(self.texture_u8 / 256.0)

    @cached_property
    def lightmap(self):
        return None if self.lightmap_u8 is None else self.lightmap_u8 / 256.0

    @cached_property
    def blur_image(self):
        return None if self.blur_u8 is None else sRGB_to_sRGB_linear(self.blur_u8 / 256.0)
