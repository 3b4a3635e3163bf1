"""Equirectangular background (reference `backgrounds/panorama.py:10-26`): a radius-1e6
`Sphere_Collider` with the sky material, sampled with the sphere's (atan2, asin) uv."""
from ..geometry import Sphere_Collider, Primitive
from ..utils.vector3 import vec3
from ..utils.constants import SKYBOX_DISTANCE
from .skybox import SkyBox_Material

__all__ = ["Panorama"]


class Panorama(Primitive):
    def __init__(self, panorama, center=vec3(0.0, 0.0, 0.0), light_intensity=0.0, blur=0.0):
        super().__init__(center, SkyBox_Material(panorama, light_intensity, blur), shadow=False)
        self.light_intensity = light_intensity
        self.collider_list += [
            Sphere_Collider(assigned_primitive=self, center=center, radius=SKYBOX_DISTANCE)
        ]
