"""Lights (reference `sightpy/lights.py:6-52`).  Lights only affect Glossy materials.

`DirectionalLight` is lowered to the device light table.  The reference `PointLight.get_L`
references undefined names (lights.py:30-31), so rendering a scene with a point light raises
NameError as soon as a Glossy surface is shaded (glossy.py:38 calls get_L for every light).  Here
the point light is lowered as a record and the device raises the same way: a Glossy hit under a
point light sets an error bit and the render fails with SRT_ERR_NAME -> NameError.  Scenes whose
rays never hit a Glossy surface render as in the reference (the light is never consulted).
"""
import numpy as np

from .utils.constants import SKYBOX_DISTANCE

__all__ = ["Light", "PointLight", "DirectionalLight"]


class Light:
    def __init__(self, pos, color):
        self.pos = pos
        self.color = color


class PointLight(Light):
    def get_L(self):
        # lights.py:30-31: `(self.pos - M) * (1.0 / (dist_light))` with M, dist_light undefined
        raise NameError("name 'M' is not defined")

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
