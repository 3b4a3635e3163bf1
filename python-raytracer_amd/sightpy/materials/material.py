"""Material base class (reference `materials/material.py:11-44`).

A material here is a parameter record.  Its `get_color(scene, ray, hit)` — the reference's
per-batch shading entry point — runs on the device: the shading kernels in
`csrc/rt_device.h` (`rt_shade_*`) implement each subclass.  Normal maps (material.py:18-40) are
supported for Plane and Cuboid colliders (the only ones with `inverse_basis_matrix`).
"""
from ..utils.image_functions import load_image_u8

__all__ = ["Material"]


class Material:
    def __init__(self, normalmap=None):
        self.normalmap = None
        self.normalmap_u8 = None
        self.repeat = 1.0
        if normalmap is not None:
            self.set_normalmap(normalmap)

    def set_normalmap(self, normalmap, repeat=1.0):
        self.normalmap_u8 = load_image_u8("sightpy/normalmaps/" + normalmap)
        self.normalmap = self.normalmap_u8 / 256.0
        self.repeat = repeat

    def get_color(self, scene, ray, hit):
        raise NotImplementedError(
            "%s shading runs on the device; trace rays with sightpy.get_raycolor" % type(self).__name__
        )
