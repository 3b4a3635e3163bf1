"""Loader for the test-only host check harness (python-raytracer_amd/csrc/rt_hostcheck.cpp):
the kernels' per-ray functions compiled for the CPU, driven sequentially.  Used by the CPU test
suite to check the device math and the scene lowering against the oracle without a GPU."""
import ctypes
from pathlib import Path

import numpy as np

from sightpy import _native as N
from sightpy._lower import lower_scene, camera_desc, collider_record

LIB = Path(__file__).resolve().parent / "_build" / "libsightpy_hostcheck.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            import subprocess
            subprocess.run(["make", "-C", str(Path(__file__).resolve().parent.parent / "python-raytracer_amd" / "csrc"),
                            str(LIB.relative_to(LIB.parent.parent.parent).as_posix()).replace("tests/", "../../tests/")],
                           check=True)
        _lib = ctypes.CDLL(str(LIB))
        _lib.hc_render.argtypes = [ctypes.POINTER(N.SceneDesc), ctypes.POINTER(N.CameraDesc),
                                   ctypes.POINTER(N.RenderArgs), ctypes.POINTER(N.Stats)]
        _lib.hc_trace.argtypes = [ctypes.POINTER(N.SceneDesc), ctypes.POINTER(N.TraceArgs), ctypes.POINTER(N.Stats)]
        _lib.hc_nearest.argtypes = [ctypes.POINTER(N.SceneDesc)] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + \
                                   [ctypes.c_void_p] * 3
        _lib.hc_intersect_collider.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p]
        _lib.hc_primary_rays.argtypes = [ctypes.POINTER(N.CameraDesc)] + [ctypes.c_void_p] * 3
        _lib.hc_mt_uniforms.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        _lib.hc_xpow_mod.argtypes = [ctypes.c_uint64, ctypes.c_void_p]
        _lib.hc_jump_window.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        _lib.hc_last_error.restype = ctypes.c_char_p
        _lib.hc_philox.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        _lib.hc_mix32.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        _lib.hc_mix32.restype = ctypes.c_uint32
        _lib.hc_set_bvh.argtypes = [ctypes.c_int]
        _lib.hc_bvh_nodes.argtypes = [ctypes.POINTER(N.SceneDesc)]
    return _lib


def set_bvh(on):
    """1: large meshes through the BVH (the GPU's behaviour), 0: every collider in the linear loop."""
    lib().hc_set_bvh(int(on))


def bvh_nodes(scene):
    L = lower_scene(scene)
    return lib().hc_bvh_nodes(ctypes.byref(L.desc()))


def nearest(scene, O, D):
    """nearest_hit for rays (3, n): (t, collider id, orientation)."""
    L = lower_scene(scene)
    d = L.desc()
    O = np.ascontiguousarray(O, dtype=np.float64)
    D = np.ascontiguousarray(D, dtype=np.float64)
    n = O.shape[1]
    t, ids, orient = np.empty(n), np.empty(n, np.int32), np.empty(n)
    lib().hc_nearest(ctypes.byref(d), N.ptr(O), N.ptr(D), n, N.ptr(t), N.ptr(ids), N.ptr(orient))
    return t, ids, orient


def render(scene, jitter, seed=0, rows=None):
    L = lower_scene(scene)
    d = L.desc()
    cd = camera_desc(scene.camera)
    spp = jitter.shape[0] if jitter is not None else 1
    nrows = scene.camera.screen_height if rows is None else len(rows)
    npix = nrows * scene.camera.screen_width
    a = N.RenderArgs()
    a.spp = spp
    a.n_rows = nrows
    rows_arr = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    a.rows = N.ptr(rows_arr)
    j = None if jitter is None else np.ascontiguousarray(jitter)
    a.jitter = N.ptr(j)
    a.seed = seed
    rgb = np.empty((3, npix))
    u8 = np.empty((npix, 3), np.uint8)
    hits = np.empty((spp, npix), np.int32)
    a.out_rgb, a.out_srgb8, a.out_hit_id = N.ptr(rgb), N.ptr(u8), N.ptr(hits)
    st = N.Stats()
    rc = lib().hc_render(ctypes.byref(d), ctypes.byref(cd), ctypes.byref(a), ctypes.byref(st))
    if rc:
        if rc == N.ERR_INDEX:
            raise IndexError(lib().hc_last_error().decode())
        raise RuntimeError(lib().hc_last_error().decode())
    return rgb, u8.reshape(nrows, scene.camera.screen_width, 3), hits, st.as_dict()


def intersect(collider, O, D):
    rec = np.ascontiguousarray(collider_record(collider)).reshape(1)
    O = np.ascontiguousarray(O, dtype=np.float64)
    D = np.ascontiguousarray(D, dtype=np.float64)
    out = np.empty((2, O.shape[1]))
    lib().hc_intersect_collider(N.ptr(rec), N.ptr(O), N.ptr(D), O.shape[1], N.ptr(out))
    return out


def mt_uniforms(key, pos, n_out, n_skip=0):
    """rt_mt.h's segmented numpy-stream generator, run serially on the CPU."""
    key = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.empty(n_out)
    key_out = np.empty(624, dtype=np.uint32)
    pos_out = ctypes.c_int(0)
    rc = lib().hc_mt_uniforms(key.ctypes.data, int(pos), int(n_out), int(n_skip), out.ctypes.data,
                              key_out.ctypes.data, ctypes.byref(pos_out))
    assert rc == 0, rc
    return out, key_out, pos_out.value


def xpow_mod(J):
    """rt_mt.h xpow_mod: x^J mod phi as 624 uint32 words."""
    out = np.empty(624, dtype=np.uint32)
    lib().hc_xpow_mod(int(J), out.ctypes.data)
    return out


def jump_window(key, J):
    """The MT19937 window J words past `key` by rt_mt.h's polynomial jump (exact from word 1 on)."""
    key = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.empty(624, dtype=np.uint32)
    lib().hc_jump_window(key.ctypes.data, int(J), out.ctypes.data)
    return out


def philox(ctr, k0, k1):
    """rt_device.h philox(ctr[4], k0, k1) -> 4 uint32."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    out = np.empty(4, dtype=np.uint32)
    lib().hc_philox(c.ctypes.data, int(k0), int(k1), out.ctypes.data)
    return out


def mix32(h, v):
    return int(lib().hc_mix32(int(h), int(v)))


def trace(scene, O, D, depth=0, dfl=0, seed=0, medium=None):
    """hc_trace: get_raycolor of a batch (3, n) on the CPU build of the kernels."""
    L = lower_scene(scene)
    d = L.desc()
    O = np.ascontiguousarray(O, dtype=np.float64)
    D = np.ascontiguousarray(D, dtype=np.float64)
    n = O.shape[1]
    a = N.TraceArgs()
    a.n, a.origin, a.dir = n, N.ptr(O), N.ptr(D)
    med = None if medium is None else np.ascontiguousarray(medium, dtype=np.int32)
    a.medium = N.ptr(med)
    a.depth, a.diffuse_reflections, a.seed = depth, dfl, seed
    out = np.empty((3, n))
    a.out_rgb = N.ptr(out)
    st = N.Stats()
    rc = lib().hc_trace(ctypes.byref(d), ctypes.byref(a), ctypes.byref(st))
    if rc:
        raise RuntimeError(lib().hc_last_error().decode())
    return out, st.as_dict()
