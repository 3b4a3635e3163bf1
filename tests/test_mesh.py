"""TriangleMesh: the OBJ loader and the BVH that intersects large meshes on
the device.  The reference's TriangleMesh raises NameError (`geometry/triangle_mesh.py:40`), so mesh
parity is pinned through its Triangle_Collider, whose intersection the oracle reproduces bit-exactly
(collider KATs from the reference, tests/golden/colliders.npz): the BVH path must give exactly the
linear loop's nearest distance, first collider index and tie flag, and the same images.

CPU tests run the kernels' math through the host harness (tests/_build, rt_device.h + rt_bvh.h
compiled by g++); the GPU versions are in test_gpu.py."""
import numpy as np
import pytest

import hostcheck as HC
import scenes
import sightpy_oracle as O


@pytest.fixture(scope="module")
def obj(tmp_path_factory):
    p = tmp_path_factory.mktemp("mesh") / "icosphere.obj"
    nf = scenes.write_icosphere_obj(str(p), subdiv=2)
    return str(p), nf


@pytest.fixture(scope="module")
def obj_ties(tmp_path_factory):
    p = tmp_path_factory.mktemp("mesh") / "icosphere_dup.obj"
    nf = scenes.write_icosphere_obj(str(p), subdiv=1, duplicate_faces=12, slash_format=False)
    return str(p), nf


def test_obj_loader(obj):
    from sightpy import TriangleMesh, Glossy, rgb, vec3

    path, nf = obj
    m = TriangleMesh(path, center=vec3(1.0, 2.0, 3.0), material=Glossy(diff_color=rgb(0.5, 0.5, 0.5), roughness=0.2,
                                                                     spec_coeff=0.3, diff_coeff=0.8, n=vec3(1.5, 1.5, 1.5)),
                     max_ray_depth=2)
    assert len(m.collider_list) == nf == 320
    verts = [np.array(l.split()[1:4], dtype=float) for l in open(path) if l.startswith("v ")]
    face = [int(t.split("/")[0]) - 1 for t in [l for l in open(path) if l.startswith("f ")][7].split()[1:4]]
    c = m.collider_list[7]
    assert np.array_equal([c.p1.x, c.p1.y, c.p1.z], verts[face[0]] + [1.0, 2.0, 3.0])
    assert np.array_equal([c.p3.x, c.p3.y, c.p3.z], verts[face[2]] + [1.0, 2.0, 3.0])


def test_bvh_built_only_for_meshes(obj):
    assert HC.bvh_nodes(scenes.mesh_scene(obj[0])) > 16
    assert HC.bvh_nodes(scenes.example1(8, 6)) == 0


def _probe_rays(sc, rng, n=6000):
    """Random rays at the mesh plus the awkward ones: axis-parallel, through vertices exactly,
    starting inside the mesh, grazing along the floor."""
    mesh = [c for c in sc.collider_list if type(c).__name__ == "Triangle_Collider"]
    verts = np.array([[c.p1.x, c.p1.y, c.p1.z] for c in mesh])
    Os, Ds = [], []
    O0 = rng.uniform(-2, 2, size=(n, 3)) + [0.0, 0.5, 1.0]
    tgt = verts[rng.integers(0, len(verts), n)] + rng.normal(scale=0.05, size=(n, 3))
    Os.append(O0), Ds.append(tgt - O0)
    k = 400
    Os.append(O0[:k]), Ds.append(verts[rng.integers(0, len(verts), k)] - O0[:k])  # exactly at vertices
    ax = np.zeros((k, 3))
    ax[np.arange(k), rng.integers(0, 3, k)] = rng.choice([-1.0, 1.0], k)
    Os.append(np.array([0.35, 0.05, -1.0]) + rng.uniform(-0.6, 0.6, size=(k, 3))), Ds.append(ax)  # axis-parallel
    Os.append(np.tile([0.35, 0.05, -1.0], (k, 1))), Ds.append(rng.normal(size=(k, 3)))  # from inside
    Ds.append(np.tile([1.0, 0.0, 0.0], (k, 1))), Os.append(np.c_[np.full(k, -3.0), np.full(k, -0.5),
                                                             rng.uniform(-2, 0, k)])  # along the floor
    Oa, Da = np.concatenate(Os), np.concatenate(Ds)
    Da = Da / np.linalg.norm(Da, axis=1, keepdims=True)
    return np.ascontiguousarray(Oa.T), np.ascontiguousarray(Da.T)


@pytest.mark.parametrize("which", ["plain", "ties"])
def test_bvh_nearest_equals_linear_and_oracle(obj, obj_ties, which):
    path = obj[0] if which == "plain" else obj_ties[0]
    sc = scenes.mesh_scene(path)
    Oa, Da = _probe_rays(sc, np.random.default_rng(11))
    HC.set_bvh(1)
    tb, ib, ob = HC.nearest(sc, Oa, Da)
    HC.set_bvh(0)
    try:
        tl, il, ol = HC.nearest(sc, Oa, Da)
    finally:
        HC.set_bvh(1)
    assert np.array_equal(ib, il)
    assert np.array_equal(tb, tl, equal_nan=True)
    assert np.array_equal(ob, ol, equal_nan=True)
    near, ids = O.hit_ids(sc, Oa, Da)
    assert np.array_equal(ib, ids)
    hit = ids >= 0
    assert np.array_equal(tb[hit], near[hit])
    assert (ib >= 1).mean() > 0.3  # the probe hits the mesh a lot
    if which == "ties":
        # the duplicated faces (the last 12 mesh colliders) tie with their originals: the lower index
        # is reported (ray.py:131-132), so none of them is ever the hit id
        dup = set(range(1 + obj_ties[1] - 12, 1 + obj_ties[1]))
        assert not dup & set(ib.tolist())


def _box_edge_rays(sc, rng, k=1500):
    """Rays whose slab distances sit at the f32 box test's error bound: starting on the mesh surface
    (every vertex, edge and face point lies on or inside box planes), nearly axis-parallel (1/D up
    to 1e300: the f32 axis switched off), from far away (|O| = 1e5 with a 2-unit mesh)."""
    mesh = [c for c in sc.collider_list if type(c).__name__ == "Triangle_Collider"]
    tri = np.array([[[c.p1.x, c.p1.y, c.p1.z], [c.p2.x, c.p2.y, c.p2.z], [c.p3.x, c.p3.y, c.p3.z]] for c in mesh])
    pick = tri[rng.integers(0, len(tri), k)]
    w = rng.dirichlet([1.0, 1.0, 1.0], size=k)
    w[: k // 3] = np.eye(3)[rng.integers(0, 3, k // 3)]  # exactly at vertices
    w[k // 3: 2 * k // 3, rng.integers(0, 3)] = 0.0  # on edges
    w /= w.sum(axis=1, keepdims=True)
    surf = np.einsum("kv,kvc->kc", w, pick)
    Os = [surf, surf]
    Ds = [rng.normal(size=(k, 3)), tri.mean(axis=(0, 1)) - surf]
    nearly = rng.normal(size=(k, 3))
    nearly[np.arange(k), rng.integers(0, 3, k)] = rng.choice([1e-300, -1e-12, 1e-7], k)
    Os.append(surf + rng.normal(scale=0.3, size=(k, 3))), Ds.append(nearly)
    far = rng.normal(size=(k, 3))
    far *= 1e5 / np.linalg.norm(far, axis=1, keepdims=True)
    Os.append(far), Ds.append(pick.mean(axis=1) - far)
    Oa, Da = np.concatenate(Os), np.concatenate(Ds)
    Da = Da / np.linalg.norm(Da, axis=1, keepdims=True)
    return np.ascontiguousarray(Oa.T), np.ascontiguousarray(Da.T)


def _tiny_mesh_rays(sc, rng, k=3000):
    """Rays through a mesh ~1e-2 across at the origin with one direction component ~1e-39: that
    axis's s = |1/D| (bound + |O|) stays below the 1e37 guard while f32(1/D) overflows to inf
    (the axis must then constrain nothing, as for axis-parallel rays)."""
    Os, Ds = [], []
    for a in range(3):
        O = rng.uniform(-4e-3, 4e-3, size=(k, 3))
        b = (a + 1) % 3
        O[:, b] = rng.choice([-0.02, 0.02], k)  # outside the mesh along axis b, aimed back through it
        D = rng.normal(scale=0.3, size=(k, 3))
        D[:, b] = -np.sign(O[:, b])
        D[:, a] = rng.choice([1e-39, -1e-39, 3e-39], k)
        Os.append(O), Ds.append(D)
    Oa, Da = np.concatenate(Os), np.concatenate(Ds)
    Da = Da / np.linalg.norm(Da, axis=1, keepdims=True)
    return np.ascontiguousarray(Oa.T), np.ascontiguousarray(Da.T)


@pytest.fixture(scope="module")
def tiny_obj(tmp_path_factory):
    p = tmp_path_factory.mktemp("mesh") / "icosphere_tiny.obj"
    scenes.write_icosphere_obj(str(p), subdiv=2, radius=5e-3)
    return str(p)


def test_bvh_f32_box_test_tiny_mesh_overflowing_inverse(tiny_obj):
    """A direction component whose f32 inverse overflows on a mesh ~1e-2 across at the origin: the
    BVH gives exactly the linear loop's nearest hits (before the |1/D| < 3e38 guard in box_ray the
    boxes beside the ray's origin on that axis were dropped)."""
    sc = scenes.mesh_scene(tiny_obj, center=(0.0, 0.0, 0.0))
    Oa, Da = _tiny_mesh_rays(sc, np.random.default_rng(31))
    HC.set_bvh(1)
    tb, ib, ob = HC.nearest(sc, Oa, Da)
    HC.set_bvh(0)
    try:
        tl, il, ol = HC.nearest(sc, Oa, Da)
    finally:
        HC.set_bvh(1)
    assert np.array_equal(ib, il)
    assert np.array_equal(tb, tl, equal_nan=True)
    assert np.array_equal(ob, ol, equal_nan=True)
    assert (ib >= 1).mean() > 0.3


def test_bvh_f32_box_test_is_conservative(obj):
    """The BVH's box test runs in f32 (rt_device.h box_ray / box4f_hit), widened to hold the exact
    slab interval: on rays at its error bound it gives exactly the linear loop's nearest hit."""
    sc = scenes.mesh_scene(obj[0])
    Oa, Da = _box_edge_rays(sc, np.random.default_rng(23))
    HC.set_bvh(1)
    tb, ib, ob = HC.nearest(sc, Oa, Da)
    HC.set_bvh(0)
    try:
        tl, il, ol = HC.nearest(sc, Oa, Da)
    finally:
        HC.set_bvh(1)
    assert np.array_equal(ib, il)
    assert np.array_equal(tb, tl, equal_nan=True)
    assert np.array_equal(ob, ol, equal_nan=True)
    assert (ib >= 1).mean() > 0.3


@pytest.mark.parametrize("which", ["plain", "ties"])
def test_mesh_render_matches_oracle(obj, obj_ties, which):
    path = obj[0] if which == "plain" else obj_ties[0]
    sc = scenes.mesh_scene(path, 32, 24, 3)
    np.random.seed(5)
    jit = sc.camera.draw_jitter(1)
    rgb, u8, hits, st = HC.render(sc, jit)
    ref, ids, counts = O.render_linear(sc, jit)
    assert np.array_equal(hits, ids)
    assert st["rays_per_depth"] == [counts["depth"][d] for d in sorted(counts["depth"])]
    np.testing.assert_allclose(rgb, ref, rtol=1e-12, atol=1e-15)
    assert (hits >= 1).any() and (hits <= 320).any()
