"""Material base class (reference `materials/material.py:11-44`).

A material here is a parameter record.  Its `get_color(scene, ray, hit)` — the reference's
per-batch shading entry point — runs on the device (`srt_shade`): the shading kernels in
`csrc/rt_device.h` (`rt_shade_*`) implement each subclass, and the reflected / refracted /
diffuse rays a hit spawns are traced to completion as in get_raycolor.  In a scene holding user
Collider / Material subclasses the children are traced by the host-driven recursion instead
(`sightpy/_hybrid.py`: one device shading level per call).  Normal maps
(material.py:18-40) are supported for Plane and Cuboid colliders (the only ones with
`inverse_basis_matrix`), in shading and through get_Normal (srt_material_normal).
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

    def get_Normal(self, hit):
        """Shading normal (material.py:18-36) at hit.point: without a normal map the collider's
        normal times the hit orientation, as the reference composes it (the collider's get_Normal is
        its own device entry point); with one, on the device (srt_material_normal): the normal map's
        texel at the primitive's uv through the collider's inverse_basis_matrix, normalised, times
        the hit orientation."""
        if self.normalmap is None:
            return hit.collider.get_Normal(hit) * hit.orientation
        from .._backend import material_normal
        from ..utils.vector3 import vec3

        N = material_normal(self, hit)
        return vec3(N[0], N[1], N[2])

    def get_color(self, scene, ray, hit):
        """Colour of the batch `ray` at `hit` (all rays hit `hit.collider` at `hit.distance` with
        `hit.orientation`), as get_raycolor adds it (ray.py:131-146): srt_shade on the device."""
        from .._backend import trace_rays
        from .. import _hybrid

        if hit.collider.assigned_primitive.material is not self:
            raise ValueError("a hit is shaded by the material of its collider's primitive")
        hit.point = ray.origin + ray.dir * hit.distance
        if _hybrid.is_hybrid(scene):  # user classes in the scene: one level here, the children traced by _hybrid
            return _hybrid.shade_level(scene, self, ray, hit)
        ids = scene.collider_list.index(hit.collider)
        return trace_rays(ray, scene, hits=(ids, hit.distance, hit.orientation))
