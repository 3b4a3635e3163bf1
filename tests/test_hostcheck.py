"""Kernel math (csrc/rt_device.h compiled for the CPU by the test-only host harness) and the
scene lowering (sightpy/_lower.py) against the reference fixtures and the oracle."""
import numpy as np
import pytest

import hostcheck as HC
import scenes
import sightpy_oracle as O
from conftest import golden
from test_oracle import kat_colliders, DETERMINISTIC


@pytest.mark.parametrize("name", ["sphere", "plane", "plane_tilted", "cuboid_rot30", "cuboid_axis", "triangle"])
def test_device_collider_kat(name):
    g = golden("colliders")
    out = HC.intersect(kat_colliders()[name], g["O"], g["D"])
    assert np.array_equal(out, g[name], equal_nan=True)


@pytest.mark.parametrize("name,builder,depth", DETERMINISTIC)
def test_device_math_examples(name, builder, depth):
    g = golden(name)
    W, H, spp = int(g["width"]), int(g["height"]), int(g["spp"])
    sc = builder(W, H, depth)
    np.random.seed(int(g["seed"]))
    jit = sc.camera.draw_jitter(spp)
    rgb, u8, hits, st = HC.render(sc, jit)
    assert np.array_equal(hits, g["hit_id"]), "primary hit-id mask must be exact"
    assert st["rays_per_depth"][: len(g["depth_counts"])] == g["depth_counts"].tolist()
    np.testing.assert_allclose(rgb, g["rgb"], rtol=1e-5, atol=1e-12)
    rel = np.abs(rgb - g["rgb"]) / np.maximum(np.abs(g["rgb"]), 1e-300)
    print(name, "max rel err", rel.max())
    diff = np.abs(u8.astype(int) - g["srgb8"].astype(int))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3


def test_texel_pool_persists_across_lowerings():
    """Frame sequences re-lower the scene every frame: same images -> same texel_key and the cached
    pool (the device then keeps its copy); another image -> another key."""
    from sightpy._lower import lower_scene
    from sightpy import image

    sc = scenes.example1(16, 12)
    a, b = lower_scene(sc), lower_scene(sc)
    assert a.texel_key == b.texel_key != 0
    assert a.texels is b.texels
    assert a.signature() == b.signature()
    sc.collider_list[0].assigned_primitive.center.x = sc.collider_list[0].assigned_primitive.center.x + 0.0
    floor = sc.collider_list[2].assigned_primitive.material
    floor.diff_texture = image("wood.jpg", repeat=80.0)
    c = lower_scene(sc)
    assert c.texel_key != a.texel_key and c.texels.size != a.texels.size


def test_fingerprint_cached_only_for_immutable_texels(monkeypatch):
    """Scene.render re-lowers its scene every call: decoded images (read-only views of immutable
    bytes, also the blurred skybox) are hashed once; a writeable texel array is hashed on every
    lowering, so an in-place edit still changes the key."""
    from sightpy import _lower

    calls = []
    real = _lower._xxhash.xxh3_64_intdigest

    def counting(buf):
        calls.append(len(buf))
        return real(buf)

    monkeypatch.setattr(_lower._xxhash, "xxh3_64_intdigest", counting)
    frozen = np.frombuffer(bytes(range(256)) * 3, dtype=np.uint8).reshape(16, 16, 3)
    assert _lower._immutable_root(frozen) is not None
    k1 = _lower._fingerprint(frozen)
    assert _lower._fingerprint(frozen) == k1 and len(calls) == 1
    live = np.array(frozen)
    assert _lower._immutable_root(live) is None
    assert _lower._fingerprint(live) == k1 and len(calls) == 2
    live[0, 0, 0] ^= 1
    assert _lower._fingerprint(live) != k1 and len(calls) == 3
    sc = scenes.example4(16, 12, 2)
    _lower.lower_scene(sc)
    n = len(calls)
    _lower.lower_scene(sc)
    assert len(calls) == n, "a second lowering of the same scene re-hashed its textures"


def test_glossy_integer_lobe_exponent():
    """Glossy lobe exponent a = 2/roughness^2 - 2 (glossy.py:71): lowered with an integer k in
    `ival` only when a is within 4 ulp of k (roughness 0.2 -> 47.99999999999999 -> 48, 0.5 -> 6),
    otherwise the device keeps pow (0.3 -> 20.22..., 0.15 -> 86.88...)."""
    from sightpy._lower import lower_scene
    from sightpy import _native as N

    L = lower_scene(scenes.features(16, 12))
    seen = {}
    for r in L.materials:
        if r["type"] == N.GLOSSY and r["flags"] & N.MF_ROUGH:
            a = float(r["p"][4])
            seen[round(a, 6)] = int(r["ival"])
            if r["ival"]:
                assert abs(a - r["ival"]) <= 4 * np.spacing(a)
                x = np.linspace(0.0, 1.0, 1001)
                np.testing.assert_allclose(x ** r["ival"], x ** a, rtol=1e-12, atol=1e-300)
    assert seen[6.0] == 6 and seen[round(2 / 0.3 ** 2 - 2, 6)] == 0
