"""Scene assembly and the render entry point (reference `sightpy/scene.py:28-166`).

`Scene` keeps the reference's assembly API.  `render()` is the drop-in boundary: instead of the
reference's `multiprocessing.Pool` over samples (scene.py:80-116) it lowers the scene to flat
device tables once, generates the camera jitter of numpy's global RNG in the reference's order on
the GPU (so a seeded render consumes the same random stream), and runs the whole
samples x depths wavefront plus the sRGB resolve on the GPU(s) through `libsightpy_hip.so`.
"""
import time

import numpy as np
from PIL import Image

from .camera import Camera
from .utils.constants import *
from .utils.vector3 import vec3, rgb
from . import lights
from .backgrounds.skybox import SkyBox
from .backgrounds.panorama import Panorama

__all__ = ["Scene"]


class Scene:
    def __init__(self, ambient_color=rgb(0.01, 0.01, 0.01), n=vec3(1.0, 1.0, 1.0)):
        self.scene_primitives = []
        self.collider_list = []
        self.shadowed_collider_list = []
        self.Light_list = []
        self.importance_sampled_list = []
        self.ambient_color = ambient_color
        self.n = n
        self.last_stats = None

    def add_Camera(self, look_from, look_at, **kwargs):
        self.camera = Camera(look_from, look_at, **kwargs)

    def add_PointLight(self, pos, color):
        self.Light_list += [lights.PointLight(pos, color)]

    def add_DirectionalLight(self, Ldir, color):
        self.Light_list += [lights.DirectionalLight(Ldir.normalize(), color)]

    def add(self, primitive, importance_sampled=False):
        self.scene_primitives += [primitive]
        self.collider_list += primitive.collider_list
        if importance_sampled == True:
            self.importance_sampled_list += [primitive]
        if primitive.shadow == True:
            self.shadowed_collider_list += primitive.collider_list

    def add_Background(self, img, light_intensity=0.0, blur=0.0, spherical=False):
        if spherical == False:
            primitive = SkyBox(img, light_intensity=light_intensity, blur=blur)
        else:
            primitive = Panorama(img, light_intensity=light_intensity, blur=blur)
        self.scene_primitives += [primitive]
        self.collider_list += primitive.collider_list

    def render(self, samples_per_pixel, progress_bar=False, batch_size=None, rng="numpy", seed=None):
        """Render `samples_per_pixel` samples and return a PIL RGB image.

        rng="numpy" (default) draws the primary-ray jitter from numpy's global legacy RNG exactly
        as the reference does (including the extra sizing draw at scene.py:81), so seeded renders
        match the reference: the stream is generated on the GPU inside the render (rt_mt.h,
        bit-equal to np.random.rand) and numpy's global state is advanced past it.
        rng="numpy-host" draws the same stream with numpy on the host.  rng="device" generates
        independent jitter on the GPU (Philox keyed by pixel and sample).  `batch_size` bounds the
        samples per device pass.

        With several GPUs ($SIGHTPY_DEVICES, e.g. "0,1,2,3" or "all") the frame is split into row
        bands dealt round-robin over the GPUs (at most 8 bands per GPU: e.g. 27-row bands at 1080p
        on 8 GPUs, 2-row bands for a Diffuse fan-out scene; rt_device.h shard_band_height) and
        gathered over RCCL (the reference's
        multiprocessing.Pool over samples, scene.py:80-116, is replaced); the image does not depend
        on the number of GPUs.
        """
        from . import _backend as B
        from . import _hybrid

        print("Rendering...")
        t0 = time.time()
        if rng not in ("numpy", "numpy-host", "device"):
            raise ValueError("rng must be 'numpy', 'numpy-host' or 'device'")
        H, W = int(self.camera.screen_height), int(self.camera.screen_width)
        if _hybrid.is_hybrid(self):
            # user Collider / Material subclasses: the reference's recursion driven from the host,
            # the built-in steps on the device (_hybrid.py); numpy's stream as the reference draws it
            from .utils.colour_functions import sRGB_linear_to_sRGB

            lin = _hybrid.render_linear(self, samples_per_pixel)
            color = sRGB_linear_to_sRGB(lin.to_array())
            u8 = [(255 * np.clip(c, 0, 1).reshape((H, W))).astype(np.uint8) for c in color]
            print("Render Took", time.time() - t0)
            return Image.fromarray(np.stack(u8, axis=-1), "RGB")
        ndev = len(B.devices())
        if ndev > 1 and rng != "numpy-host" and H >= 8 * ndev:
            out = B.render_group(self, samples_per_pixel, seed=seed, batch_size=batch_size, want_rgb=False,
                                 mt=(rng == "numpy"))
        else:
            jitter = None
            if rng == "numpy-host":
                jitter = self.camera.draw_jitter(samples_per_pixel)
                self.camera.draw_jitter(1)  # reference draws one more get_ray for sizing (scene.py:81)
            # only the uint8 image leaves the GPU (the linear RGB stays there: 8x fewer PCIe bytes), as
            # 4-byte pixels -- PIL's layout of an RGB image -- into pinned memory of the image's own,
            # which the returned image maps (no host copy)
            blk = B.image_block(4 * W * H)
            out = B.render_scene(self, samples_per_pixel, jitter=jitter, seed=seed, batch_size=batch_size,
                                 want_rgb=False, mt=(rng == "numpy"), pinned_u8=True, rgbx=True, out_u8=blk)
            self.last_stats = out.stats
            print("Render Took", time.time() - t0)
            return B.rgb_image(out.srgb8, W, H, mapped=blk is not None)
        self.last_stats = out.stats
        print("Render Took", time.time() - t0)
        return Image.fromarray(out.srgb8, "RGB")

    def get_distances(self):
        """Grey depth map of one primary sample (reference scene.py:142-166)."""
        from ._backend import primary_rays, nearest_hits

        print("Rendering...")
        t0 = time.time()
        from . import _hybrid

        jitter = self.camera.draw_jitter(1)[0]
        O, D = primary_rays(self.camera, jitter)
        if _hybrid.is_hybrid(self):
            from .ray import Ray

            t = _hybrid.nearest_distance(Ray(vec3(*O), vec3(*D), 0, self.n, 0, 0, 0), self)
        else:
            t, _, _ = nearest_hits(self, O, D)
        g = np.where(t <= 10, t, 10) / 10
        print("Render Took", time.time() - t0)
        h, w = self.camera.screen_height, self.camera.screen_width
        u8 = (255 * np.clip(g, 0, 1).reshape((h, w))).astype(np.uint8)
        return Image.fromarray(np.stack([u8, u8, u8], axis=-1), "RGB")


def get_raycolor_tuple(x):
    """Reference scene.py:16-17 (Pool worker shim); kept for API compatibility."""
    from .ray import get_raycolor

    return get_raycolor(*x)


def batch_rays(rays, batch_size):
    """Reference scene.py:20-25: concatenate per-sample Ray batches in groups of batch_size."""
    from .ray import Ray

    return [Ray.concatenate(rays[i:i + batch_size]) for i in range(0, len(rays), batch_size)]
