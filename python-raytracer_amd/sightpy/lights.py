"""Lights (reference `sightpy/lights.py:6-52`).  Lights only affect Glossy materials.

`DirectionalLight` is lowered to the device light table.  The reference `PointLight.get_L`
references undefined names (lights.py:30-31) and raises NameError whenever a Glossy surface is
shaded; here a point light is evaluated with its evident intent (L = (pos - P)/|pos - P|,
irradiance = color * NdotL / dist^2 * 100) -- parity unpinned, no reference output exists.
"""
import numpy as np

from .utils.constants import SKYBOX_DISTANCE

__all__ = ["Light", "PointLight", "DirectionalLight"]


class Light:
    def __init__(self, pos, color):
        self.pos = pos
        self.color = color


class PointLight(Light):
    def get_distance(self, M):
        return np.sqrt((self.pos - M).dot(self.pos - M))

    def get_irradiance(self, dist_light, NdotL):
        return self.color * NdotL / (dist_light ** 2.0) * 100


class DirectionalLight(Light):
    def __init__(self, Ldir, color):
        self.Ldir = Ldir
        self.color = color

    def get_L(self):
        return self.Ldir

    def get_distance(self, M):
        return SKYBOX_DISTANCE

    def get_irradiance(self, dist_light, NdotL):
        return self.color * NdotL
