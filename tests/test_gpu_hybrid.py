"""Duck-typed plugins on the device (reference ray.py:122-148: intersect and get_color called on
whatever the scene's lists hold; collider.py:12-14, material.py:42-44): scenes with a user Material
on a built-in Sphere, and a user Collider (a Python sphere) with a user Material, rendered through
sightpy (_hybrid.py: built-in colliders intersected and built-in materials shaded on the device one
level at a time, srt_shade_level; the user classes' own code on their batches) against the
reference recursion on the CPU (tests/hybrid_ref.py: the oracle for built-in classes, the same user
classes).  Bar: linear RGB within 1e-5 relative, uint8 within +-1 at rounding boundaries."""
import numpy as np
import pytest

import hybrid_ref
import sightpy_oracle as O
import user_classes as U

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["material", "collider"])
def test_gpu_user_classes_frame_matches_reference_recursion(kind):
    from sightpy import _hybrid
    from sightpy.ray import get_raycolor

    W, H, spp = 48, 36, 2
    sc = U.scene(kind, W, H, 3)
    np.random.seed(11)
    state = np.random.get_state()
    jit = sc.camera.draw_jitter(spp)
    U.TRACE["fn"] = hybrid_ref.trace
    ref = hybrid_ref.render_linear(sc, jit)
    calls = {"n": 0}
    orig = U.Tinted.get_color

    def counted(self, scene, ray, hit):
        calls["n"] += 1
        return orig(self, scene, ray, hit)

    U.TRACE["fn"] = get_raycolor
    U.Tinted.get_color = counted
    try:
        np.random.set_state(state)
        lin = _hybrid.render_linear(sc, spp)
        np.random.set_state(state)
        img = np.asarray(sc.render(spp))
    finally:
        U.Tinted.get_color = orig
    assert calls["n"] >= 2  # the user's get_color ran on its batches (primaries and reflections)
    got = np.array([np.broadcast_to(np.asarray(c, dtype=np.float64), (W * H,)) for c in (lin.x, lin.y, lin.z)])
    nz = ref != 0.0
    assert np.all(got[~nz] == 0.0)
    rel = np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])
    assert rel.max() <= 1e-5, rel.max()
    want = O.srgb_u8(ref, H, W)
    d = np.abs(img.astype(int) - want.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-2


def test_gpu_user_classes_get_distances():
    from sightpy import _hybrid
    from sightpy.ray import get_distances

    sc = U.scene("collider", 32, 24, 3)
    np.random.seed(5)
    ray = sc.camera.get_ray(sc.n)
    g = get_distances(ray, sc)
    near = _hybrid.nearest_distance(ray, sc)
    r = hybrid_ref._rays_of(ray)
    dists = [O.intersect(c, r.O, r.D)[0] if _hybrid.device_collider(c) else c.intersect(ray.origin, ray.dir)[0]
             for c in sc.collider_list]
    want = np.minimum.reduce(dists)
    assert np.array_equal(near, want)
    assert np.array_equal(np.asarray(g.x), np.where(want <= 10, want, 10) / 10)


def test_gpu_user_floor_under_builtin_glass():
    """A built-in Refractive cuboid (srt_shade_level returns its reflected and refracted children,
    the refracted ones in the glass's medium) over a user-material floor: the frame equals the
    reference recursion on the CPU."""
    from sightpy import _hybrid
    from sightpy.ray import get_raycolor

    W, H, spp = 40, 30, 2
    sc = U.glass_scene(W, H, 4)
    np.random.seed(17)
    state = np.random.get_state()
    jit = sc.camera.draw_jitter(spp)
    U.TRACE["fn"] = hybrid_ref.trace
    ref = hybrid_ref.render_linear(sc, jit)
    U.TRACE["fn"] = get_raycolor
    np.random.set_state(state)
    lin = _hybrid.render_linear(sc, spp)
    got = np.array([np.broadcast_to(np.asarray(c, dtype=np.float64), (W * H,)) for c in (lin.x, lin.y, lin.z)])
    nz = ref != 0.0
    assert np.all(got[~nz] == 0.0)
    rel = np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])
    assert rel.max() <= 1e-5, rel.max()
