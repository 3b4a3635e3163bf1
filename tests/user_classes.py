"""User subclasses of sightpy's Collider, Primitive and Material, written the way a reference user
writes them (numpy on vec3 batches, recursion through get_raycolor; contracts at reference
geometry/collider.py:12-14 and materials/material.py:42-44), for the duck-typed plugin tests
(tests/test_hybrid.py, tests/test_gpu_hybrid.py).  Nothing here is library code."""
import numpy as np

from sightpy import rgb, vec3
from sightpy.geometry.collider import Collider
from sightpy.geometry.primitive import Primitive
from sightpy.materials.material import Material
from sightpy.ray import Ray
from sightpy.utils.constants import FARAWAY, UPDOWN, UPWARDS

# how Tinted traces its reflected rays: sightpy.ray.get_raycolor, or the test's CPU recursion
TRACE = {"fn": None}


class PySphereCollider(Collider):
    """A sphere the user wrote (the quadratic of reference sphere.py:26-52, on vec3 batches)."""

    def __init__(self, assigned_primitive, center, radius):
        super().__init__(assigned_primitive, center)
        self.radius = radius

    def intersect(self, O, D):
        b = 2 * D.dot(O - self.center)
        c = self.center.square_length() + O.square_length() - 2 * self.center.dot(O) - self.radius * self.radius
        disc = b ** 2 - 4 * c
        sq = np.sqrt(np.maximum(0, disc))
        h0 = (-b - sq) / 2
        h1 = (-b + sq) / 2
        h = np.where((h0 > 0) & (h0 < h1), h0, h1)
        nd = ((O + D * h - self.center) * (1.0 / self.radius)).dot(D)
        hit = (disc > 0) & (h > 0)
        dist = np.where(hit, h, FARAWAY)
        orient = np.where(hit & (nd > 0), UPDOWN, np.where(hit & (nd < 0), UPWARDS, FARAWAY))
        return dist, orient

    def get_Normal(self, hit):
        return (hit.point - self.center) * (1.0 / self.radius)


class PyBall(Primitive):
    def __init__(self, center, material, radius, max_ray_depth=3, shadow=False):
        super().__init__(center, material, max_ray_depth, shadow=shadow)
        self.collider_list += [PySphereCollider(self, center, radius)]
        self.bounded_sphere_radius = radius


class Tinted(Material):
    """A user material: a Lambert-tinted base colour under one light direction plus `k` times the
    colour of the mirror ray (traced through TRACE["fn"] while the depth allows)."""

    def __init__(self, color, k, light=vec3(0.52, 0.45, -0.5)):
        super().__init__()
        self.color = color
        self.k = k
        self.light = light.normalize()

    def get_color(self, scene, ray, hit):
        hit.point = ray.origin + ray.dir * hit.distance
        N = hit.collider.get_Normal(hit) * hit.orientation
        color = self.color * (0.2 + 0.8 * np.maximum(N.dot(self.light), 0.0))
        if ray.depth < hit.surface.max_ray_depth:
            R = ray.dir - N * 2.0 * ray.dir.dot(N)
            child = Ray(hit.point + N * 0.000001, R, ray.depth + 1, ray.n, ray.reflections + 1, ray.transmissions,
                        ray.diffuse_reflections)
            color = color + TRACE["fn"](child, scene) * self.k
        return color


def scene(kind, width=48, height=36, depth=3):
    """example1's setting with user classes: 'material' -- the blue sphere's Glossy replaced by a
    Tinted (a built-in Sphere collider: it keeps casting shadows), 'collider' -- the blue sphere
    replaced by a PyBall with a Tinted material (shadow=False), 'collider_shadow' -- the same with
    shadow=True (refused: it would shadow the device's glossy floor)."""
    from sightpy import Scene, Sphere, Plane, Glossy, image

    gold = Glossy(diff_color=rgb(1.0, 0.572, 0.184), n=vec3(0.15 + 3.58j, 0.4 + 2.37j, 1.54 + 1.91j),
                  roughness=0.0, spec_coeff=0.2, diff_coeff=0.8)
    floor = Glossy(diff_color=image("checkered_floor.png", repeat=80.0), n=vec3(1.2 + 0.3j, 1.2 + 0.3j, 1.1 + 0.3j),
                   roughness=0.2, spec_coeff=0.3, diff_coeff=0.9)
    tint = Tinted(rgb(0.2, 0.4, 0.9), 0.5)
    sc = Scene(ambient_color=rgb(0.05, 0.05, 0.05))
    angle = -np.pi / 2 * 0.3
    sc.add_Camera(look_from=vec3(2.5 * np.sin(angle), 0.25, 2.5 * np.cos(angle) - 1.5),
                  look_at=vec3(0.0, 0.25, -3.0), screen_width=width, screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.52, 0.45, -0.5), color=rgb(0.15, 0.15, 0.15))
    sc.add(Sphere(material=gold, center=vec3(-0.75, 0.1, -3.0), radius=0.6, max_ray_depth=depth))
    if kind == "material":
        sc.add(Sphere(material=tint, center=vec3(1.25, 0.1, -3.0), radius=0.6, max_ray_depth=depth))
    else:
        sc.add(PyBall(vec3(1.25, 0.1, -3.0), tint, 0.6, max_ray_depth=depth, shadow=(kind == "collider_shadow")))
    sc.add(Plane(material=floor, center=vec3(0, -0.5, -3.0), width=120.0, height=120.0,
                 u_axis=vec3(1.0, 0, 0), v_axis=vec3(0, 0, -1.0), max_ray_depth=depth))
    sc.add_Background("stormydays.png")
    return sc


def glass_scene(width=40, height=30, depth=4):
    """example3's glass cuboid (built-in Refractive: two children per hit, rays inside the glass in
    its medium) over a floor whose material is a user Tinted: srt_shade_level's children carry media
    rows back to the host recursion."""
    from sightpy import Scene, Plane, Cuboid, Refractive

    green = Refractive(n=vec3(1.5 + 4e-8j, 1.5 + 0.0j, 1.5 + 4e-8j))
    sc = Scene()
    sc.add_Camera(look_from=vec3(0.0, 0.25, 1.0), look_at=vec3(0.0, 0.25, -3.0), screen_width=width,
                  screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.0, 0.5, 0.5), color=rgb(0.5, 0.5, 0.5))
    sc.add(Plane(material=Tinted(rgb(0.7, 0.6, 0.4), 0.3), center=vec3(0, -0.5, -3.0), width=6.0, height=6.0,
                 u_axis=vec3(1.0, 0, 0), v_axis=vec3(0, 0, -1.0), max_ray_depth=depth))
    cb = Cuboid(material=green, center=vec3(0.00, 0.0001, -0.8), width=0.9, height=1.0, length=0.4, shadow=False,
                max_ray_depth=depth)
    cb.rotate(θ=30, u=vec3(0, 1, 0))
    sc.add(cb)
    sc.add_Background("stormydays.png")
    return sc
