"""Workload scenes for tests and bench, built with this package's sightpy API.

These restate the scene *parameters* of the reference's example scripts (example1.py, example2.py,
example3.py, example4.py, example_cornellbox.py) as functions of resolution and recursion depth, so
the BASELINE.json configurations (e.g. example1 at 1920x1080 depth 5) can be built without editing
the scripts.  `depth=None` keeps each primitive's own max_ray_depth from the script.
tests/golden/gen_golden.py renders the reference's own scripts with the same overrides.
"""
import numpy as np

from sightpy import (Scene, Sphere, Plane, Cuboid, Glossy, Refractive, ThinFilmInterference, Diffuse,
                     Emissive, TriangleMesh, image, rgb, vec3)


def _depth(scene, depth):
    if depth is not None:
        for p in scene.scene_primitives:
            p.max_ray_depth = depth
    return scene


def example1(width=400, height=300, depth=None):
    gold = Glossy(diff_color=rgb(1.0, 0.572, 0.184), n=vec3(0.15 + 3.58j, 0.4 + 2.37j, 1.54 + 1.91j),
                  roughness=0.0, spec_coeff=0.2, diff_coeff=0.8)
    blue = Glossy(diff_color=rgb(0.0, 0, 0.1), n=vec3(1.3 + 1.91j, 1.3 + 1.91j, 1.4 + 2.91j),
                  roughness=0.2, spec_coeff=0.5, diff_coeff=0.3)
    floor = Glossy(diff_color=image("checkered_floor.png", repeat=80.0), n=vec3(1.2 + 0.3j, 1.2 + 0.3j, 1.1 + 0.3j),
                   roughness=0.2, spec_coeff=0.3, diff_coeff=0.9)
    sc = Scene(ambient_color=rgb(0.05, 0.05, 0.05))
    angle = -np.pi / 2 * 0.3
    sc.add_Camera(look_from=vec3(2.5 * np.sin(angle), 0.25, 2.5 * np.cos(angle) - 1.5),
                  look_at=vec3(0.0, 0.25, -3.0), screen_width=width, screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.52, 0.45, -0.5), color=rgb(0.15, 0.15, 0.15))
    sc.add(Sphere(material=gold, center=vec3(-0.75, 0.1, -3.0), radius=0.6, max_ray_depth=3))
    sc.add(Sphere(material=blue, center=vec3(1.25, 0.1, -3.0), radius=0.6, max_ray_depth=3))
    sc.add(Plane(material=floor, center=vec3(0, -0.5, -3.0), width=120.0, height=120.0,
                 u_axis=vec3(1.0, 0, 0), v_axis=vec3(0, 0, -1.0), max_ray_depth=3))
    sc.add_Background("stormydays.png")
    return _depth(sc, depth)


def example2(width=400, height=300, depth=None):
    blue = Refractive(n=vec3(1.5 + 4e-8j, 1.5 + 4e-8j, 1.5 + 0.0j))
    green = Refractive(n=vec3(1.5 + 4e-8j, 1.5 + 0.0j, 1.5 + 4e-8j))
    red = Refractive(n=vec3(1.5 + 0.0j, 1.5 + 5e-8j, 1.5 + 5e-8j))
    floor = Glossy(diff_color=image("checkered_floor.png", repeat=80.0), n=vec3(1.2 + 0.3j, 1.2 + 0.3j, 1.1 + 0.3j),
                   roughness=0.2, spec_coeff=0.3, diff_coeff=0.9)
    sc = Scene(ambient_color=rgb(0.05, 0.05, 0.05))
    angle = np.pi / 2 * 0.3
    sc.add_Camera(look_from=vec3(2.5 * np.sin(angle), 0.25, 2.5 * np.cos(angle) - 1.5),
                  look_at=vec3(0.0, 0.25, -1.5), screen_width=width, screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.52, 0.45, -0.5), color=rgb(0.15, 0.15, 0.15))
    for mat, x in ((blue, -1.2), (green, 0.0), (red, 1.2)):
        sc.add(Sphere(material=mat, center=vec3(x, 0.0, -1.5), radius=0.5, shadow=False, max_ray_depth=3))
    sc.add(Plane(material=floor, center=vec3(0, -0.5, -3.0), width=120.0, height=120.0,
                 u_axis=vec3(1.0, 0, 0), v_axis=vec3(0, 0, -1.0), max_ray_depth=3))
    sc.add_Background("miramar.jpeg")
    return _depth(sc, depth)


def example3(width=400, height=300, depth=None):
    floor = Glossy(diff_color=image("checkered_floor.png", repeat=2.0), roughness=0.2, spec_coeff=0.3,
                   diff_coeff=0.7, n=vec3(2.2, 2.2, 2.2))
    green = Refractive(n=vec3(1.5 + 4e-8j, 1.5 + 0.0j, 1.5 + 4e-8j))
    sc = Scene()
    sc.add_Camera(look_from=vec3(0.0, 0.25, 1.0), look_at=vec3(0.0, 0.25, -3.0), screen_width=width,
                  screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.0, 0.5, 0.5), color=rgb(0.5, 0.5, 0.5))
    sc.add(Plane(material=floor, center=vec3(0, -0.5, -3.0), width=6.0, height=6.0, u_axis=vec3(1.0, 0, 0),
                 v_axis=vec3(0, 0, -1.0), max_ray_depth=5))
    cb = Cuboid(material=green, center=vec3(0.00, 0.0001, -0.8), width=0.9, height=1.0, length=0.4, shadow=False,
                max_ray_depth=5)
    cb.rotate(θ=30, u=vec3(0, 1, 0))
    sc.add(cb)
    sc.add_Background("stormydays.png")
    return _depth(sc, depth)


def example4(width=400, height=300, depth=None):
    sc = Scene(ambient_color=rgb(0.01, 0.01, 0.01))
    angle = -np.pi * 0.5
    sc.add_Camera(screen_height=height, screen_width=width,
                  look_from=vec3(4.0 * np.sin(angle), 0.00, 4.0 * np.cos(angle)), look_at=vec3(0.0, 0.05, 0.0))
    bubble = ThinFilmInterference(thickness=330, noise=60.0)
    sc.add(Sphere(material=bubble, center=vec3(1.0, 0.0, 1.5), radius=1.7, shadow=False, max_ray_depth=5))
    sc.add_Background("lake.png", light_intensity=5.0, blur=10.0)
    return _depth(sc, depth)


def cornell(width=100, height=100, depth=None, mc=False):
    """example_cornellbox.py; `mc=True` makes the glass sphere pick reflection or refraction by
    Monte Carlo (refractive.py:95-101), which no example script does."""
    sc = Scene(ambient_color=rgb(0.00, 0.00, 0.00))
    sc.add_Camera(screen_width=width, screen_height=height, look_from=vec3(278, 278, 800),
                  look_at=vec3(278, 278, 0), focal_distance=1.0, field_of_view=40)
    green = Diffuse(diff_color=rgb(0.12, 0.45, 0.15))
    red = Diffuse(diff_color=rgb(0.65, 0.05, 0.05))
    white = Diffuse(diff_color=rgb(0.73, 0.73, 0.73))
    light = Emissive(color=rgb(15.0, 15.0, 15.0))
    glass = Refractive(n=vec3(1.5 + 0.05e-8j, 1.5 + 0.02e-8j, 1.5 + 0.0j))
    sc.add(Plane(material=light, center=vec3(213 + 130 / 2, 554, -227.0 - 105 / 2), width=130.0, height=105.0,
                 u_axis=vec3(1.0, 0.0, 0), v_axis=vec3(0.0, 0, 1.0)), importance_sampled=True)
    sc.add(Plane(material=white, center=vec3(555 / 2, 555 / 2, -555.0), width=555.0, height=555.0,
                 u_axis=vec3(0.0, 1.0, 0), v_axis=vec3(1.0, 0, 0.0)))
    sc.add(Plane(material=green, center=vec3(-0.0, 555 / 2, -555 / 2), width=555.0, height=555.0,
                 u_axis=vec3(0.0, 1.0, 0), v_axis=vec3(0.0, 0, -1.0)))
    sc.add(Plane(material=red, center=vec3(555.0, 555 / 2, -555 / 2), width=555.0, height=555.0,
                 u_axis=vec3(0.0, 1.0, 0), v_axis=vec3(0.0, 0, -1.0)))
    sc.add(Plane(material=white, center=vec3(555 / 2, 555, -555 / 2), width=555.0, height=555.0,
                 u_axis=vec3(1.0, 0.0, 0), v_axis=vec3(0.0, 0, -1.0)))
    sc.add(Plane(material=white, center=vec3(555 / 2, 0.0, -555 / 2), width=555.0, height=555.0,
                 u_axis=vec3(1.0, 0.0, 0), v_axis=vec3(0.0, 0, -1.0)))
    cb = Cuboid(material=white, center=vec3(182.5, 165, -285 - 160 / 2), width=165, height=165 * 2, length=165,
                shadow=False)
    cb.rotate(θ=15, u=vec3(0, 1, 0))
    sc.add(cb)
    sc.add(Sphere(material=glass, center=vec3(370.5, 165 / 2, -65 - 185 / 2), radius=165 / 2, shadow=False,
                  max_ray_depth=3, mc=mc), importance_sampled=True)
    return _depth(sc, depth)


BUILDERS = {"example1": example1, "example2": example2, "example3": example3, "example4": example4,
            "cornell": cornell}


def features(width=64, height=48, depth=4, sp=None, mc=False):
    """Feature scene (not one of the reference's scripts): exercises the API paths the examples do
    not reach -- normal map on a textured floor (material.py:18-40), a rotated textured Cuboid
    (cuboid.py:84-187 uv cross), an absorbing glass sphere, an Emissive sphere, a metal with
    roughness, two directional lights and a spherical Panorama background (panorama.py:10-26).

    `sp` is the sightpy module to build with: this package by default; tests/golden/gen_golden.py
    passes the reference's module so the fixture comes from the reference itself.  `mc=True`: the
    glass sphere picks reflection or refraction by Monte Carlo (refractive.py:95-101)."""
    if sp is None:
        import sightpy as sp
    vec3, rgb = sp.vec3, sp.rgb
    floor = sp.Glossy(diff_color=sp.image("checkered_floor.png", repeat=6.0), n=vec3(1.2 + 0.3j, 1.2 + 0.3j, 1.1 + 0.3j),
                      roughness=0.3, spec_coeff=0.4, diff_coeff=0.9)
    floor.set_normalmap("floor.jpg", repeat=4.0)
    wood = sp.Glossy(diff_color=sp.image("wood.jpg"), n=vec3(1.5 + 0j, 1.5 + 0j, 1.5 + 0j), roughness=0.5,
                     spec_coeff=0.2, diff_coeff=0.8)
    glass = sp.Refractive(n=vec3(1.5 + 4e-8j, 1.5 + 1e-8j, 1.5 + 0j))
    metal = sp.Glossy(diff_color=rgb(0.8, 0.7, 0.3), n=vec3(0.2 + 3.0j, 0.5 + 2.5j, 1.3 + 2.0j), roughness=0.15,
                      spec_coeff=0.6, diff_coeff=0.2)
    lamp = sp.Emissive(color=rgb(3.0, 2.5, 2.0))
    sc = sp.Scene(ambient_color=rgb(0.05, 0.05, 0.05))
    sc.add_Camera(look_from=vec3(0.5, 1.2, 3.0), look_at=vec3(0.0, 0.1, -1.0), screen_width=width,
                  screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.5, 0.6, 0.4), color=rgb(0.6, 0.6, 0.55))
    sc.add_DirectionalLight(Ldir=vec3(-0.7, 0.3, 0.2), color=rgb(0.2, 0.2, 0.3))
    sc.add(sp.Plane(material=floor, center=vec3(0.0, -0.5, -1.0), width=20.0, height=20.0, u_axis=vec3(1.0, 0, 0),
                    v_axis=vec3(0, 0, -1.0), max_ray_depth=depth))
    cb = sp.Cuboid(material=wood, center=vec3(-1.0, 0.0, -1.2), width=0.8, height=1.0, length=0.6,
                   max_ray_depth=depth, shadow=True)
    cb.rotate(θ=25, u=vec3(0, 1, 0))
    sc.add(cb)
    sc.add(sp.Sphere(material=glass, center=vec3(0.6, 0.0, -0.8), radius=0.5, max_ray_depth=depth, shadow=False,
                     mc=mc))
    sc.add(sp.Sphere(material=metal, center=vec3(0.1, -0.25, 0.2), radius=0.25, max_ray_depth=depth))
    sc.add(sp.Sphere(material=lamp, center=vec3(1.5, 0.8, -2.0), radius=0.3, max_ray_depth=depth, shadow=False))
    sc.add_Background("miramar.jpeg", spherical=True)
    return sc


def write_icosphere_obj(path, subdiv=2, radius=0.5, duplicate_faces=0, slash_format=True):
    """Write an icosphere as a Wavefront OBJ (v / f records, 1-based, 'i/t/n' face syntax when
    `slash_format`).  `duplicate_faces` repeats the first faces at the end (exact ties: two
    colliders at the same distance, both shaded by the reference, ray.py:131-146)."""
    t = (1.0 + 5 ** 0.5) / 2.0
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    V = [np.array(v, dtype=np.float64) / np.linalg.norm(v) for v in V]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    for _ in range(subdiv):
        mids = {}

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in mids:
                m = V[a] + V[b]
                V.append(m / np.linalg.norm(m))
                mids[k] = len(V) - 1
            return mids[k]

        F = [f for a, b, c in F for f in ((a, mid(a, b), mid(c, a)), (b, mid(b, c), mid(a, b)),
                                          (c, mid(c, a), mid(b, c)), (mid(a, b), mid(b, c), mid(c, a)))]
    F = F + F[:duplicate_faces]
    with open(path, "w") as fh:
        fh.write("# icosphere, %d faces\n" % len(F))
        for v in V:
            fh.write("v %.17g %.17g %.17g\n" % tuple(radius * v))
        for a, b, c in F:
            if slash_format:
                fh.write("f %d/%d/%d %d//%d %d\n" % (a + 1, a + 1, a + 1, b + 1, b + 1, c + 1))
            else:
                fh.write("f %d %d %d\n" % (a + 1, b + 1, c + 1))
    return len(F)


def mesh_scene(obj_path, width=64, height=48, depth=3, center=(0.35, 0.05, -1.0)):
    """A TriangleMesh in the ex1 setting: a glossy icosphere mesh next to a
    sphere over the textured floor, sky box background, one shadowing light."""
    red = Glossy(diff_color=rgb(0.6, 0.1, 0.1), n=vec3(1.5 + 0.2j, 1.5 + 0.2j, 1.5 + 0.2j), roughness=0.2,
                 spec_coeff=0.4, diff_coeff=0.8)
    gold = Glossy(diff_color=rgb(1.0, 0.572, 0.184), n=vec3(0.15 + 3.58j, 0.4 + 2.37j, 1.54 + 1.91j),
                  roughness=0.0, spec_coeff=0.2, diff_coeff=0.8)
    floor = Glossy(diff_color=image("checkered_floor.png", repeat=20.0), n=vec3(1.2 + 0.3j, 1.2 + 0.3j, 1.1 + 0.3j),
                   roughness=0.2, spec_coeff=0.3, diff_coeff=0.9)
    sc = Scene(ambient_color=rgb(0.05, 0.05, 0.05))
    sc.add_Camera(look_from=vec3(0.3, 0.6, 1.8), look_at=vec3(0.0, 0.0, -1.0), screen_width=width,
                  screen_height=height)
    sc.add_DirectionalLight(Ldir=vec3(0.52, 0.45, -0.5), color=rgb(0.5, 0.5, 0.5))
    sc.add(Sphere(material=gold, center=vec3(-0.8, 0.0, -1.2), radius=0.45, max_ray_depth=depth))
    sc.add(TriangleMesh(obj_path, center=vec3(*center), material=red, max_ray_depth=depth))
    sc.add(Plane(material=floor, center=vec3(0, -0.5, -2.0), width=40.0, height=40.0, u_axis=vec3(1.0, 0, 0),
                 v_axis=vec3(0, 0, -1.0), max_ray_depth=depth))
    sc.add_Background("stormydays.png")
    return sc


def mesh_bench(width=1920, height=1080, depth=3, subdiv=5):
    """Bench workload for the BVH: mesh_scene with an icosphere of 20 * 4**subdiv triangles."""
    import os
    import tempfile

    path = os.path.join(tempfile.gettempdir(), "sightpy_icosphere_%d.obj" % subdiv)
    if not os.path.exists(path):
        write_icosphere_obj(path, subdiv=subdiv)
    return mesh_scene(path, width, height, depth)
