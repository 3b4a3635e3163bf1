"""Pinhole / thin-lens camera (reference `sightpy/camera.py:7-85`).

The constructor computes the camera basis and the pixel grid on the host exactly as the
reference does; `_lower()` hands the device the per-column x and per-row y coordinates plus the
basis scalars, and the raygen kernel (`rt_primary_ray` in csrc/rt_device.h) reproduces
`get_ray` for every (sample, pixel) from the four uniforms [x-jitter, y-jitter, disk r, disk phi].
"""
import numpy as np

from .utils.vector3 import vec3, rgb
from .ray import Ray

__all__ = ["Camera"]


class Camera:
    def __init__(
        self,
        look_from,
        look_at,
        screen_width=400,
        screen_height=300,
        field_of_view=90.0,
        aperture=0.0,
        focal_distance=1.0,
    ):
        self.screen_width = screen_width
        self.screen_height = screen_height
        self.aspect_ratio = float(screen_width) / screen_height
        self.look_from = look_from
        self.look_at = look_at
        self.field_of_view = field_of_view
        self.camera_width = np.tan(field_of_view * np.pi / 180 / 2.0) * 2.0
        self.camera_height = self.camera_width / self.aspect_ratio
        self.cameraFwd = (look_at - look_from).normalize()
        self.cameraRight = (self.cameraFwd.cross(vec3(0.0, 1.0, 0.0))).normalize()
        self.cameraUp = self.cameraRight.cross(self.cameraFwd)
        self.lens_radius = aperture / 2.0
        self.focal_distance = focal_distance
        # per-column / per-row image-plane coordinates (the reference flattens a meshgrid of these)
        self.xs = np.linspace(-self.camera_width / 2.0, self.camera_width / 2.0, self.screen_width)
        self.ys = np.linspace(self.camera_height / 2.0, -self.camera_height / 2.0, self.screen_height)

    @property
    def x(self):
        return np.tile(self.xs, self.screen_height)

    @property
    def y(self):
        return np.repeat(self.ys, self.screen_width)

    def draw_jitter(self, samples):
        """Draw the uniforms `get_ray` consumes, in the reference's order, from numpy's global
        legacy RNG: per sample rand(N) x-jitter, rand(N) y-jitter, rand(N) disk r, rand(N) disk phi
        (camera.py:56-64, utils/random.py:6-9).  Shape (samples, 4, N)."""
        n = self.screen_width * self.screen_height
        return np.random.rand(samples * 4 * n).reshape(samples, 4, n)

    def get_ray(self, n):
        """One sample of primary rays for every pixel, generated on the device."""
        from ._backend import primary_rays

        jitter = self.draw_jitter(1)
        origin, direction = primary_rays(self, jitter[0])
        return Ray(origin=origin, dir=direction, depth=0, n=n, reflections=0, transmissions=0,
                   diffuse_reflections=0)
