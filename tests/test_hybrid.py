"""Duck-typed plugins on the CPU (SURVEY §2 plugin points: reference ray.py:122-148 calls intersect /
get_color on whatever the scene lists hold): which classes the device implements, how a scene with
user classes lowers, what is refused, and the expected-frame harness (tests/hybrid_ref.py) against
the oracle on a scene without user classes.  The device frames are in test_gpu_hybrid.py."""
import numpy as np
import pytest

import hybrid_ref
import scenes
import sightpy_oracle as O
import user_classes as U
from sightpy import _hybrid
from sightpy._lower import lower_scene


def test_builtin_scenes_are_not_hybrid():
    for b in ("example1", "example3", "example4", "cornell"):
        assert not _hybrid.is_hybrid(getattr(scenes, b)(16, 12))


def test_user_material_on_builtin_collider_lowers_as_placeholder():
    sc = U.scene("material")
    assert _hybrid.is_hybrid(sc)
    assert [_hybrid.on_device(c) for c in sc.collider_list] == [True, False, True, True]
    L = lower_scene(sc)
    # every built-in collider is on the device (the user material's sphere still casts shadows)
    assert L.device_index == [0, 1, 2, 3] and len(L.colliders) == 4
    from sightpy import _native as N

    tint = L.colliders["material"][1]
    assert L.materials["type"][tint] == N.EMISSIVE and not L.materials["p"][tint].any()


def test_user_collider_is_left_to_the_host():
    sc = U.scene("collider")
    L = lower_scene(sc)
    assert L.device_index == [0, -1, 1, 2] and len(L.colliders) == 3


def test_overriding_a_builtin_method_makes_a_user_class():
    from sightpy import Sphere, Glossy, rgb, vec3
    from sightpy.geometry.sphere import Sphere_Collider

    class Odd(Sphere_Collider):
        def intersect(self, O, D):
            return super().intersect(O, D)

    class Keeps(Sphere_Collider):
        pass

    s = Sphere(material=Glossy(diff_color=rgb(1, 1, 1), roughness=0.2, spec_coeff=0.3, diff_coeff=0.8, n=vec3(1.5, 1.5, 1.5)), center=vec3(0, 0, 0), radius=1.0)
    assert _hybrid.device_collider(Keeps(radius=1.0, assigned_primitive=s, center=vec3(0, 0, 0)))
    assert not _hybrid.device_collider(Odd(radius=1.0, assigned_primitive=s, center=vec3(0, 0, 0)))

    class MyGlossy(Glossy):
        def get_color(self, scene, ray, hit):
            return super().get_color(scene, ray, hit)

    assert _hybrid.device_material(Glossy(diff_color=rgb(1, 1, 1), roughness=0.2, spec_coeff=0.3, diff_coeff=0.8, n=vec3(1.5, 1.5, 1.5)))
    assert not _hybrid.device_material(MyGlossy(diff_color=rgb(1, 1, 1), roughness=0.2, spec_coeff=0.3, diff_coeff=0.8, n=vec3(1.5, 1.5, 1.5)))


def test_refused_combinations():
    with pytest.raises(NotImplementedError, match="casts shadows"):
        _hybrid.is_hybrid(U.scene("collider_shadow"))
    sc = U.scene("collider")
    from sightpy import Glossy, rgb, vec3

    sc.collider_list[1].assigned_primitive.material = Glossy(diff_color=rgb(1, 1, 1), roughness=0.2, spec_coeff=0.3, diff_coeff=0.8, n=vec3(1.5, 1.5, 1.5))
    sc._hybrid_key = None
    with pytest.raises(NotImplementedError, match="built-in material"):
        _hybrid.is_hybrid(sc)


def test_expected_frame_harness_equals_the_oracle_without_user_classes():
    sc = scenes.example1(24, 18, 3)
    np.random.seed(3)
    jit = sc.camera.draw_jitter(2)
    ref, _, _ = O.render_linear(sc, jit)
    got = hybrid_ref.render_linear(sc, jit)
    assert np.array_equal(got, ref)

