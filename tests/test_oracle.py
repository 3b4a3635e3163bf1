"""The CPU oracle (oracle/sightpy_oracle.py) against fixtures produced by the reference itself
(tests/golden/gen_golden.py).  Geometry is bit-exact; colours agree to <= 1e-12 relative."""
import numpy as np
import pytest

import sightpy_oracle as O
import scenes
from conftest import golden
from sightpy import vec3
from sightpy.geometry.sphere import Sphere_Collider
from sightpy.geometry.plane import Plane_Collider
from sightpy.geometry.cuboid import Cuboid_Collider
from sightpy.geometry.triangle import Triangle_Collider
from sightpy.geometry.primitive import rotation_matrix


class _Prim:
    pass


def kat_colliders():
    prim = _Prim()
    sph = Sphere_Collider(assigned_primitive=prim, center=vec3(0.3, -0.2, 0.1), radius=1.1)
    pl = Plane_Collider(assigned_primitive=prim, center=vec3(0.1, -0.5, 0.2), u_axis=vec3(1.0, 0.0, 0.0),
                        v_axis=vec3(0.0, 0.0, -1.0), w=1.5, h=0.8)
    pl2 = Plane_Collider(assigned_primitive=prim, center=vec3(0.0, 0.2, -0.3), u_axis=vec3(0.6, 0.0, 0.8),
                         v_axis=vec3(0.0, 1.0, 0.0), w=1.0, h=2.0)
    cb = Cuboid_Collider(assigned_primitive=prim, center=vec3(0.2, 0.1, -0.4), width=0.9, height=1.0, length=0.4)
    cb.rotate(rotation_matrix(30, vec3(0, 1, 0)), vec3(0.2, 0.1, -0.4))
    cb_axis = Cuboid_Collider(assigned_primitive=prim, center=vec3(0.0, 0.0, 0.0), width=2.0, height=2.0, length=2.0)
    tri = Triangle_Collider(assigned_surface=prim, p1=vec3(-1.0, -0.5, 0.0), p2=vec3(1.2, -0.4, 0.1),
                            p3=vec3(0.1, 1.3, -0.2))
    return {"sphere": sph, "plane": pl, "plane_tilted": pl2, "cuboid_rot30": cb, "cuboid_axis": cb_axis,
            "triangle": tri}


def same(a, b):
    """bit-exact incl. NaN positions"""
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("name", ["sphere", "plane", "plane_tilted", "cuboid_rot30", "cuboid_axis", "triangle"])
def test_collider_kat(name):
    g = golden("colliders")
    c = kat_colliders()[name]
    out = O.intersect(c, g["O"], g["D"])
    assert same(out, g[name]), "oracle %s intersect differs from the reference" % name


def test_rotated_cuboid_basis_matches_reference():
    g = golden("colliders")
    cb = kat_colliders()["cuboid_rot30"]
    assert np.array_equal(cb.basis_matrix, g["cuboid_rot30_basis"])
    assert np.array_equal([cb.lb_local_basis.x, cb.lb_local_basis.y, cb.lb_local_basis.z], g["cuboid_rot30_lb"])
    assert np.array_equal([cb.rt_local_basis.x, cb.rt_local_basis.y, cb.rt_local_basis.z], g["cuboid_rot30_rt"])


def test_camera_kat_and_rng_stream():
    g = golden("camera")
    sc = scenes.example1(64, 48)
    np.random.seed(0)
    j = sc.camera.draw_jitter(1)[0]
    after = np.random.rand(3)
    Og, Dg = O.primary_rays(sc.camera, j)
    assert np.array_equal(np.broadcast_to(Og, g["O"].shape), g["O"])
    assert np.array_equal(Dg, g["D"])
    assert np.array_equal(after, g["rng_after"]), "jitter draw must consume the reference's RNG stream"


def test_texture_tables_match_reference():
    from sightpy._lower import _LIN_LUT, _RAW_LUT
    from sightpy.utils.image_functions import load_image_u8
    from sightpy.backgrounds.util.blur_background import blur_skybox_u8

    g = golden("textures")
    for name, u8, lut in [("checkered", load_image_u8("sightpy/textures/checkered_floor.png"), _LIN_LUT),
                          ("lake_lightmap", load_image_u8("sightpy/backgrounds/lightmaps/lake.png"), _RAW_LUT),
                          ("lake_blur10", None, _LIN_LUT)]:
        if u8 is None:
            u8 = blur_skybox_u8(load_image_u8("sightpy/backgrounds/lake.png"), 10.0, "lake.png")
        r, c = g[name + "_rc"]
        assert tuple(u8.shape) == tuple(g[name + "_shape"])
        assert np.array_equal(lut[u8[r, c, :3]], g[name + "_val"]), name


def _render_oracle(name, builder, W, H, depth, spp, seed):
    sc = builder(W, H, depth)
    np.random.seed(seed)
    jit = sc.camera.draw_jitter(spp)
    sc.camera.draw_jitter(1)
    return sc, O.render_linear(sc, jit)


DETERMINISTIC = [
    ("ex1_64x48_d3_s2", scenes.example1, None),
    ("ex1_160x120_d5_s1", scenes.example1, 5),
    ("ex2_64x48_d3_s2", scenes.example2, None),
    ("ex3_64x48_d8_s2", scenes.example3, 8),
    ("ex4_48x36_d6_s1", scenes.example4, 6),
    ("features_64x48_d4_s2", scenes.features, 4),
]


@pytest.mark.parametrize("name,builder,depth", DETERMINISTIC)
def test_oracle_examples_match_reference(name, builder, depth):
    g = golden(name)
    sc, (rgb, ids, counts) = _render_oracle(name, builder, int(g["width"]), int(g["height"]), depth, int(g["spp"]),
                                            int(g["seed"]))
    assert np.array_equal(ids, g["hit_id"]), "primary hit-id mask must be exact"
    assert [counts["depth"].get(d, 0) for d in range(len(g["depth_counts"]))] == g["depth_counts"].tolist()
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-12, atol=1e-15)
    u8 = O.srgb_u8(rgb, int(g["height"]), int(g["width"]))
    assert np.array_equal(u8, g["srgb8"])


def test_oracle_cornell_matches_reference_single_process():
    # Monte-Carlo: the oracle consumes numpy's RNG in the reference's order, so a seeded
    # single-process render reproduces the reference exactly (the GPU path is statistical).
    g = golden("cornell_24x24_s1")
    sc, (rgb, ids, counts) = _render_oracle("cornell", scenes.cornell, 24, 24, None, 1, 0)
    assert np.array_equal(ids, g["hit_id"])
    assert [counts["depth"].get(d, 0) for d in range(len(g["depth_counts"]))] == g["depth_counts"].tolist()
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-12, atol=1e-15)


@pytest.mark.slow
def test_oracle_example1_full_plumbing_config():
    g = golden("ex1_400x300_d3_s6")
    sc, (rgb, ids, counts) = _render_oracle("ex1", scenes.example1, 400, 300, None, 6, 0)
    assert np.array_equal(ids, g["hit_id"])
    assert [counts["depth"].get(d, 0) for d in range(4)] == g["depth_counts"].tolist()
    np.testing.assert_allclose(rgb, g["rgb"].astype(np.float64), rtol=1e-6, atol=1e-9)  # fixture stored as f32
    assert np.array_equal(O.srgb_u8(rgb, 300, 400), g["srgb8"])
