"""GPU parity of the reference's per-hit plugin points, through the C ABI:

  Collider.get_Normal / get_uv, Primitive.get_uv  -> srt_collider_surface
  image.get_color                                 -> srt_texture_lookup
  Material.get_color(scene, ray, hit)             -> srt_shade

each against the oracle's restatement (oracle/sightpy_oracle.py collider_normal, collider_uv,
primitive_uv, texel, shade_linear) on the reference's collider fixtures and example scenes.
Bar: texel gathers and hit/face selections exact; float64 results within 1e-12 relative
(transcendentals: device libm vs numpy's), colours within the north_star 1e-5."""
import numpy as np
import pytest

import scenes
import sightpy_oracle as O
from conftest import golden
from test_oracle import kat_colliders

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-5, 1e-12
FTOL = 1e-12


def _backend():
    from sightpy import _backend

    return _backend


def _kat_points(name):
    """Points on collider `name` where the fixture's rays hit it (plus the rays' origins)."""
    g = golden("colliders")
    c = kat_colliders()[name]
    t = g[name][0]
    hit = t < O.FARAWAY
    P = g["O"][:, hit] + g["D"][:, hit] * t[hit]
    return c, P


class _Hit:
    """A Hit record whose point is set, as the reference's materials do before get_Normal."""

    def __init__(self, collider, P, orientation=1.0):
        from sightpy import Hit, vec3

        prim = collider.assigned_primitive
        self.h = Hit(None, orientation, getattr(prim, "material", None), collider, prim)
        self.h.point = vec3(P[0], P[1], P[2])


@pytest.mark.parametrize("name", ["sphere", "plane", "plane_tilted", "cuboid_rot30", "cuboid_axis", "triangle"])
def test_gpu_collider_normal_matches_oracle(name):
    c, P = _kat_points(name)
    assert P.shape[1] > 16
    N = c.get_Normal(_Hit(c, P).h)  # Collider.get_Normal -> srt_collider_surface
    got = np.stack([np.broadcast_to(N.x, P.shape[1]), np.broadcast_to(N.y, P.shape[1]),
                    np.broadcast_to(N.z, P.shape[1])])
    ref = np.broadcast_to(O.collider_normal(c, P), P.shape)
    if name.startswith("cuboid"):  # face selection exact: the same signed axis
        assert np.array_equal(np.sign(np.round(got, 9)), np.sign(np.round(ref, 9)))
    np.testing.assert_allclose(got, ref, rtol=FTOL, atol=1e-15)


@pytest.mark.parametrize("name", ["sphere", "plane", "plane_tilted", "cuboid_rot30", "cuboid_axis"])
def test_gpu_collider_uv_matches_oracle(name):
    c, P = _kat_points(name)
    u, v = c.get_uv(_Hit(c, P).h)  # Collider.get_uv -> srt_collider_surface
    ru, rv = O.collider_uv(c, P)
    np.testing.assert_allclose(u, ru, rtol=FTOL, atol=1e-15)
    np.testing.assert_allclose(v, rv, rtol=FTOL, atol=1e-15)


def test_gpu_cube_cross_primitive_uv():
    """Cuboid / SkyBox primitives divide the collider's uv by (4, 3) (cuboid.py:29-32), on the device
    (primitive_uv = 1) and through Primitive.get_uv."""
    c, P = _kat_points("cuboid_rot30")

    from sightpy.geometry.primitive import Primitive

    class CrossPrim:
        uv_cube_cross = True
        get_uv = Primitive.get_uv

    c.assigned_primitive = CrossPrim()
    ru, rv = O.collider_uv(c, P)
    from sightpy import vec3

    _, uv = _backend().collider_surface(c, vec3(*P), normal=False, primitive_uv=True)
    np.testing.assert_allclose(uv[0], ru / 4, rtol=FTOL, atol=1e-15)
    np.testing.assert_allclose(uv[1], rv / 3, rtol=FTOL, atol=1e-15)
    h = _Hit(c, P).h
    u, v = h.get_uv()  # Hit.get_uv -> Primitive.get_uv -> Collider.get_uv
    np.testing.assert_allclose(u, ru / 4, rtol=FTOL, atol=1e-15)
    np.testing.assert_allclose(v, rv / 3, rtol=FTOL, atol=1e-15)


def test_gpu_triangle_uv_is_undefined_like_reference():
    from sightpy import _native

    c, P = _kat_points("triangle")
    with pytest.raises(NotImplementedError):
        c.get_uv(_Hit(c, P).h)
    with pytest.raises(_native.SrtError):  # the C ABI refuses it as well
        _backend().collider_surface(c, _Hit(c, P).h.point, normal=False)


def test_gpu_texture_lookup_matches_oracle():
    """image.get_color's gather (texture.py:32-39): negative-row wrap, truncation toward zero,
    floor-mod of negative indices, repeat; every texel exact."""
    from sightpy.utils.colour_functions import sRGB_to_sRGB_linear

    rng = np.random.default_rng(5)
    u8 = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    img = sRGB_to_sRGB_linear(u8 / 256.0)
    n = 4099
    u, v = rng.uniform(-2.5, 2.5, n), rng.uniform(-2.5, 2.5, n)
    u[:5] = [0.0, 1.0, -1e-300, 0.999999999, 2.0]
    for rep in (1.0, 1.5, 0.25):
        got = _backend().texture_lookup(u8, rep, u, v)
        assert np.array_equal(got, O.texel(img, u, v, rep))


def test_gpu_image_get_color_at_hits():
    """image.get_color(hit): Hit.get_uv (device) then the device gather, vs the oracle."""
    from sightpy.textures.texture import image
    from sightpy.utils.colour_functions import sRGB_to_sRGB_linear

    from sightpy.geometry.primitive import Primitive

    class PlanePrim:
        uv_cube_cross = False
        get_uv = Primitive.get_uv

    c, P = _kat_points("plane_tilted")
    c.assigned_primitive = PlanePrim()
    tex = image.__new__(image)
    tex.u8 = np.random.default_rng(9).integers(0, 256, (16, 24, 3), dtype=np.uint8)
    tex.repeat = 2.0
    col = tex.get_color(_Hit(c, P).h)
    ru, rv = O.collider_uv(c, P)
    ref = O.texel(sRGB_to_sRGB_linear(tex.u8 / 256.0), ru, rv, 2.0)
    assert np.array_equal(np.stack([col.x, col.y, col.z]), ref)


def _primary(sc, seed):
    np.random.seed(seed)
    jit = sc.camera.draw_jitter(1)[0]
    Oo, Do = O.primary_rays(sc.camera, jit)
    return np.ascontiguousarray(np.broadcast_to(Oo, Do.shape)), Do


@pytest.mark.parametrize("builder,depth", [("example1", 5), ("example3", 6), ("example4", 6), ("features", 4)])
def test_gpu_material_get_color_matches_oracle(builder, depth):
    """Material.get_color(scene, ray.extract(hit_check), hit) per collider, as get_raycolor's loop
    calls it (ray.py:131-146), vs the oracle's shade at the same hits; the sum over colliders of
    the shaded colours equals get_raycolor."""
    from sightpy import Hit, Ray, get_raycolor, vec3

    sc = getattr(scenes, builder)(40, 30, depth)
    Ob, Do = _primary(sc, 3)
    ray = Ray(vec3(*Ob), vec3(*Do), 0, sc.n, 0, 0, 0)
    near, dists = O.nearest(sc, Ob, Do)
    total = np.zeros_like(Do)
    shaded = 0
    for k, coll in enumerate(sc.collider_list):
        hit = (near != O.FARAWAY) & (dists[k][0] == near)
        if not hit.any():
            continue
        m = coll.assigned_primitive.material
        h = Hit(dists[k][0][hit], dists[k][1][hit], m, coll, coll.assigned_primitive)
        cc = m.get_color(sc, ray.extract(hit), h)  # -> srt_shade
        got = np.stack([np.broadcast_to(cc.x, hit.sum()), np.broadcast_to(cc.y, hit.sum()),
                        np.broadcast_to(cc.z, hit.sum())])
        ci = np.full(hit.sum(), k, dtype=np.int32)
        ref, _ = O.shade_linear(sc, ci, Ob[:, hit], Do[:, hit], O.scene_medium(sc), 0, dists[k][0][hit],
                                dists[k][1][hit])
        np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
        total[:, hit] += got
        shaded += 1
    assert shaded >= 2
    col = get_raycolor(ray, sc)
    np.testing.assert_allclose(total, np.stack([col.x, col.y, col.z]), rtol=RTOL, atol=ATOL)


def test_gpu_shade_whole_batch_and_misses():
    """srt_shade over a mixed batch: collider -1 adds nothing; other rays match the oracle."""
    from sightpy import Ray, vec3

    sc = scenes.example3(32, 24, 6)
    Ob, Do = _primary(sc, 8)
    near, ids = O.hit_ids(sc, Ob, Do)
    orient = np.ones_like(near)
    for k in range(len(sc.collider_list)):
        m = ids == k
        orient[m] = O.intersect(sc.collider_list[k], Ob[:, m], Do[:, m])[1]
    ids[::7] = -1  # "no hit" rows among the hits
    ray = Ray(vec3(*Ob), vec3(*Do), 0, sc.n, 0, 0, 0)
    col = _backend().trace_rays(ray, sc, hits=(ids, near, orient))
    got = np.stack([col.x, col.y, col.z])
    ref, _ = O.shade_linear(sc, ids, Ob, Do, O.scene_medium(sc), 0, near, orient)
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    assert (got[:, ids < 0] == 0).all() and (got[:, ids >= 0] != 0).any()


def test_gpu_shade_monte_carlo_matches_oracle_stream():
    """Diffuse shading at given hits with the device stream (ray i keyed like srt_trace's ray i)."""
    from sightpy import Ray, vec3

    sc = scenes.cornell(16, 16)
    rng = np.random.default_rng(2)
    n = 257
    Ob = np.stack([rng.uniform(20, 535, n), rng.uniform(350, 540, n), rng.uniform(-535, -20, n)])
    D = rng.standard_normal((3, n))
    D /= np.sqrt((D * D).sum(0))
    near, ids = O.hit_ids(sc, Ob, D)
    orient = np.ones_like(near)
    for k in range(len(sc.collider_list)):
        m = ids == k
        orient[m] = O.intersect(sc.collider_list[k], Ob[:, m], D[:, m])[1]
    ray = Ray(vec3(*Ob), vec3(*D), 0, sc.n, 0, 0, 0)
    col = _backend().trace_rays(ray, sc, seed=41, hits=(ids, near, orient))
    ref, _ = O.shade_linear(sc, ids, Ob, D, O.scene_medium(sc), 0, near, orient, stream=O.DeviceStream(41))
    np.testing.assert_allclose(np.stack([col.x, col.y, col.z]), ref, rtol=RTOL, atol=ATOL)


def test_gpu_shade_rejects_foreign_collider_index():
    from sightpy import Ray, vec3

    sc = scenes.example1(8, 6)
    Ob, Do = _primary(sc, 1)
    ray = Ray(vec3(*Ob), vec3(*Do), 0, sc.n, 0, 0, 0)
    with pytest.raises(IndexError):
        _backend().trace_rays(ray, sc, hits=(len(sc.collider_list), np.ones(48), np.ones(48)))


def _primary_hits(sc, ci, seed=5):
    """Points where one sample of primary rays of `sc` hits collider index `ci` nearest, with the
    orientations there (oracle nearest hit)."""
    np.random.seed(seed)
    jit = sc.camera.draw_jitter(1)[0]
    Oo, Do = O.primary_rays(sc.camera, jit)
    Ob = np.ascontiguousarray(np.broadcast_to(Oo, Do.shape))
    near, ids = O.hit_ids(sc, Ob, Do)
    sel = ids == ci
    t, orient = O.intersect(sc.collider_list[ci], Ob[:, sel], Do[:, sel])
    return Ob[:, sel] + Do[:, sel] * t, orient


@pytest.mark.parametrize("which", ["floor_plane", "rotated_cuboid", "plain_sphere"])
def test_gpu_material_get_normal_matches_oracle(which):
    """Material.get_Normal(hit) (material.py:18-36) through srt_material_normal: the normal-mapped
    floor of the features scene (the map's texel at the primitive's uv, through the Plane's
    inverse_basis_matrix), a normal-mapped rotated Cuboid (its 4x3 cross uv and basis), and a plain
    material (collider normal x orientation) -- against the oracle's shading_normal."""
    from sightpy import Cuboid, Glossy, rgb, vec3

    sc = scenes.features(96, 72, 3)
    if which == "floor_plane":
        ci = 0
    elif which == "plain_sphere":
        ci = 3
    else:
        m = Glossy(diff_color=rgb(0.5, 0.4, 0.3), n=vec3(1.5 + 0j, 1.5 + 0j, 1.5 + 0j), roughness=0.3, spec_coeff=0.3,
                   diff_coeff=0.7)
        m.set_normalmap("floor.jpg", repeat=2.0)
        cb = Cuboid(material=m, center=vec3(0.2, 0.2, 0.5), width=0.9, height=0.7, length=0.8, max_ray_depth=3)
        cb.rotate(θ=35, u=vec3(0.3, 1, 0.2))
        sc.add(cb)
        ci = len(sc.collider_list) - 1
    c = sc.collider_list[ci]
    mat = c.assigned_primitive.material
    P, orient = _primary_hits(sc, ci)
    assert P.shape[1] > 16
    from sightpy import Hit

    h = Hit(None, orient, mat, c, c.assigned_primitive)
    h.point = vec3(P[0], P[1], P[2])
    got = mat.get_Normal(h)
    got = np.stack([got.x, got.y, got.z])
    ref = O.shading_normal(mat, c, P, orient)
    np.testing.assert_allclose(got, ref, rtol=FTOL, atol=1e-15)
    if which != "plain_sphere":
        # the map moved the normals off the collider's (so the texel path was exercised)
        plain = np.broadcast_to(O.collider_normal(c, P), P.shape) * orient
        assert np.abs(got - plain).max() > 1e-3


def test_gpu_material_get_normal_needs_inverse_basis_like_reference():
    """A normal-mapped material on a Sphere: the reference reads hit.collider.inverse_basis_matrix,
    which a Sphere_Collider lacks (AttributeError); so does this."""
    from sightpy import Glossy, Hit, rgb, vec3

    sc = scenes.features(64, 48, 3)
    c = sc.collider_list[3]
    m = Glossy(diff_color=rgb(0.5, 0.4, 0.3), n=vec3(1.5 + 0j, 1.5 + 0j, 1.5 + 0j), roughness=0.3, spec_coeff=0.3,
               diff_coeff=0.7)
    m.set_normalmap("floor.jpg")
    P, orient = _primary_hits(sc, 3)
    h = Hit(None, orient, m, c, c.assigned_primitive)
    h.point = vec3(P[0], P[1], P[2])
    with pytest.raises(AttributeError):
        m.get_Normal(h)
