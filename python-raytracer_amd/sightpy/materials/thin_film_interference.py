"""Thin-film interference material (reference `materials/thin_film_interference.py:11-115`).

Reflectance comes from the 400x400 precomputed table `thin_film_interference_n=1.4.png`
indexed by (cos(theta_i) * 400, thickness); the thickness is jittered by the `noise.png` red
channel.  Device: `rt_shade_thinfilm`.
"""
from ..utils.image_functions import load_image_u8
from .material import Material

__all__ = ["ThinFilmInterference"]


class ThinFilmInterference(Material):
    def __init__(self, thickness, noise=0.0, **kwargs):
        super().__init__(**kwargs)
        self.thickness = thickness
        self.reflectance_u8 = load_image_u8("sightpy/textures/thin_film_interference_n=1.4.png")
        self.noise_u8 = load_image_u8("sightpy/textures/noise.png")
        self.thin_film_interference_reflectance = self.reflectance_u8 / 256.0
        self.thickness_noise = (self.noise_u8 / 256.0)[:, :, 0]
        self.noise_factor = noise
