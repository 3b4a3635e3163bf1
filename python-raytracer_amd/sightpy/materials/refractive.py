"""Refractive (dielectric / absorbing) material (reference `materials/refractive.py:10-123`).

Complex-IOR Fresnel, reflection + Snell refraction (RGB-averaged IOR), total internal reflection,
Beer absorption; deterministic split or Monte-Carlo pick when the primitive has `mc=True`.
Device: `rt_shade_refractive`.
"""
from .material import Material

__all__ = ["Refractive"]


class Refractive(Material):
    def __init__(self, n, **kwargs):
        super().__init__(**kwargs)
        self.n = n
