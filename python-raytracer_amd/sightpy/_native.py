"""ctypes binding of the C ABI in include/sightpy_rt.h (libsightpy_hip.so).

This is the reference-side binding a maintainer adds to sightpy: every entry point of the header is
declared here with its argument types.  Table records (colliders, materials, textures, lights) are
numpy structured dtypes laid out exactly like the C structs, so lowering builds them with vectorised
numpy and passes plain pointers.

The library is loaded lazily; if it is missing, or no GPU is visible, the first call raises
`BackendUnavailable` -- there is no CPU fallback in the product path.
"""
import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_NAME = "libsightpy_hip.so"

SRT_MAX_DEPTHS = 64
SRT_COLLIDER_PARAMS = 48
SRT_MATERIAL_PARAMS = 16

SPHERE, PLANE, CUBOID, TRIANGLE = 0, 1, 2, 3
GLOSSY, REFRACTIVE, THINFILM, DIFFUSE, EMISSIVE, SKY = 0, 1, 2, 3, 4, 5
CF_SHADOW, CF_MC, CF_UV_CROSS = 1, 2, 4
MF_ROUGH, MF_LIGHTMAP, MF_NOISE = 1, 2, 4
LIGHT_DIRECTIONAL, LIGHT_POINT = 0, 1

ERR_ARG, ERR_HIP, ERR_NOSCENE, ERR_MEMORY, ERR_INDEX, ERR_DEPTH, ERR_NAME = -1, -2, -3, -4, -5, -6, -7

COLLIDER_DTYPE = np.dtype(
    [
        ("type", "<i4"),
        ("material", "<i4"),
        ("max_ray_depth", "<i4"),
        ("flags", "<u4"),
        ("primitive", "<i4"),
        ("reserved", "<i4", (3,)),
        ("p", "<f8", (SRT_COLLIDER_PARAMS,)),
    ],
    align=True,
)
MATERIAL_DTYPE = np.dtype(
    [
        ("type", "<i4"),
        ("tex", "<i4"),
        ("tex_aux0", "<i4"),
        ("tex_aux1", "<i4"),
        ("normalmap", "<i4"),
        ("medium", "<i4"),
        ("flags", "<u4"),
        ("ival", "<i4"),
        ("p", "<f8", (SRT_MATERIAL_PARAMS,)),
    ],
    align=True,
)
TEXTURE_DTYPE = np.dtype(
    [
        ("offset", "<i8"),
        ("height", "<i4"),
        ("width", "<i4"),
        ("channels", "<i4"),
        ("channel0", "<i4"),
        ("idx_h", "<i4"),
        ("idx_w", "<i4"),
        ("repeat", "<f8"),
        ("lut", "<f8", (256,)),
    ],
    align=True,
)
LIGHT_DTYPE = np.dtype(
    [("type", "<i4"), ("reserved", "<i4"), ("dir", "<f8", (3,)), ("color", "<f8", (3,)), ("pos", "<f8", (3,))],
    align=True,
)
assert COLLIDER_DTYPE.itemsize == 416 and MATERIAL_DTYPE.itemsize == 160
assert TEXTURE_DTYPE.itemsize == 2088 and LIGHT_DTYPE.itemsize == 80

_p = ctypes.c_void_p
_d3 = ctypes.c_double * 3


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("n_colliders", ctypes.c_int32),
        ("n_materials", ctypes.c_int32),
        ("n_textures", ctypes.c_int32),
        ("n_lights", ctypes.c_int32),
        ("n_media", ctypes.c_int32),
        ("n_importance", ctypes.c_int32),
        ("colliders", _p),
        ("materials", _p),
        ("textures", _p),
        ("texels", _p),
        ("texel_bytes", ctypes.c_int64),
        ("lights", _p),
        ("media", _p),
        ("glossy_f0", _p),
        ("light_local", _p),
        ("importance", _p),
        ("ambient", _d3),
        ("max_ray_depth", ctypes.c_int32),
        ("has_diffuse", ctypes.c_int32),
        ("texel_key", ctypes.c_uint64),
    ]


class CameraDesc(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("xs", _p),
        ("ys", _p),
        ("look_from", _d3),
        ("right", _d3),
        ("up", _d3),
        ("fwd_fd", _d3),
        ("cam_width", ctypes.c_double),
        ("cam_height", ctypes.c_double),
        ("lens_radius", ctypes.c_double),
        ("focal_distance", ctypes.c_double),
    ]


class MtState(ctypes.Structure):
    """np.random.get_state() of numpy's legacy MT19937 RandomState (srt_mt_state)."""
    _fields_ = [("key", ctypes.c_uint32 * 624), ("pos", ctypes.c_int32), ("reserved", ctypes.c_int32)]

    @classmethod
    def from_numpy(cls, state=None):
        name, key, pos, _, _ = np.random.get_state() if state is None else state
        if name != "MT19937":
            raise ValueError("numpy's global generator is not MT19937")
        m = cls()
        np.ctypeslib.as_array(m.key)[:] = np.asarray(key, dtype=np.uint32)
        m.pos = int(pos)
        return m

    def to_numpy(self):
        """Set numpy's global RandomState to this state (the gauss cache is reset, as rand leaves it)."""
        np.random.set_state(("MT19937", np.ctypeslib.as_array(self.key).copy(), int(self.pos), 0, 0.0))


class RenderArgs(ctypes.Structure):
    _fields_ = [
        ("spp", ctypes.c_int32),
        ("sample_base", ctypes.c_int32),
        ("n_rows", ctypes.c_int32),
        ("batch_spp", ctypes.c_int32),
        ("rows", _p),
        ("jitter", _p),
        ("mt", ctypes.POINTER(MtState)),
        ("seed", ctypes.c_uint64),
        ("out_rgb", _p),
        ("out_srgb8", _p),
        ("out_hit_id", _p),
        ("flags", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("rays_per_depth", ctypes.c_int64 * SRT_MAX_DEPTHS),
        ("total_rays", ctypes.c_int64),
        ("shadow_rays", ctypes.c_int64),
        ("n_depths", ctypes.c_int32),
        ("passes", ctypes.c_int32),
        ("ms_wall", ctypes.c_double),
        ("ms_device", ctypes.c_double),
        ("ms_trace_kernels", ctypes.c_double),
        ("ms_primary_kernel", ctypes.c_double),
        ("retries", ctypes.c_int64),
        ("kernel_path", ctypes.c_int32),
        ("chain_from", ctypes.c_int32),
    ]

    def as_dict(self):
        n = max(int(self.n_depths), 0)
        rpd = [int(x) for x in self.rays_per_depth[:n]]
        while rpd and rpd[-1] == 0:
            rpd.pop()
        return {
            "rays_per_depth": rpd,
            "total_rays": int(self.total_rays),
            "shadow_rays": int(self.shadow_rays),
            "passes": int(self.passes),
            "ms_wall": float(self.ms_wall),
            "ms_device": float(self.ms_device),
            "ms_trace_kernels": float(self.ms_trace_kernels),
            "ms_primary_kernel": float(self.ms_primary_kernel),
            "retries": int(self.retries),
            "kernel_path": {1: "frame", 2: "fused"}.get(int(self.kernel_path), "wavefront"),
            "chain_from": int(self.chain_from),
        }


class TraceArgs(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64),
        ("origin", _p),
        ("dir", _p),
        ("medium", _p),
        ("depth", ctypes.c_int32),
        ("diffuse_reflections", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("out_rgb", _p),
    ]


class Children(ctypes.Structure):
    """srt_children: the rays one level of shading spawns (srt_shade_level)."""
    _fields_ = [
        ("cap", ctypes.c_int64),
        ("n", ctypes.c_int64),
        ("origin", _p),
        ("dir", _p),
        ("weight", _p),
        ("parent", _p),
        ("medium", _p),
        ("depth", _p),
        ("diffuse_reflections", _p),
    ]


# name -> (restype, argtypes) for every entry point of include/sightpy_rt.h
RENDER_ASYNC, RENDER_SHARDED, RENDER_GATHER_RGB, RENDER_RGB_ROWS, RENDER_RGB_LOCAL, RENDER_RGBX = 1, 2, 4, 8, 16, 32  # SRT_RENDER_*
ABI_VERSION = 5  # SRT_ABI_VERSION of include/sightpy_rt.h
COMM_ID_BYTES = 128

SIGNATURES = {
    "srt_abi_version": (ctypes.c_int, []),
    "srt_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "srt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "srt_destroy": (ctypes.c_int, [_p]),
    "srt_set_option": (ctypes.c_int, [_p, ctypes.c_char_p, ctypes.c_int64]),
    "srt_upload_scene": (ctypes.c_int, [_p, ctypes.POINTER(SceneDesc)]),
    "srt_render": (ctypes.c_int, [_p, ctypes.POINTER(CameraDesc), ctypes.POINTER(RenderArgs), ctypes.POINTER(Stats)]),
    "srt_trace": (ctypes.c_int, [_p, ctypes.POINTER(TraceArgs), ctypes.POINTER(Stats)]),
    "srt_nearest": (ctypes.c_int, [_p, _p, _p, ctypes.c_int64, _p, _p, _p]),
    "srt_intersect_collider": (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int64, _p]),
    "srt_shade": (ctypes.c_int, [_p, ctypes.POINTER(TraceArgs), _p, _p, _p, ctypes.POINTER(Stats)]),
    "srt_shade_level": (ctypes.c_int, [_p, ctypes.POINTER(TraceArgs), _p, _p, _p, ctypes.POINTER(Children),
                                       ctypes.POINTER(Stats)]),
    "srt_collider_surface": (ctypes.c_int, [_p, _p, _p, ctypes.c_int64, _p, _p, ctypes.c_int]),
    "srt_texture_lookup": (ctypes.c_int, [_p, _p, _p, ctypes.c_int64, _p, ctypes.c_int64, _p]),
    "srt_primary_rays": (ctypes.c_int, [_p, ctypes.POINTER(CameraDesc), _p, _p, _p]),
    "srt_mt19937_uniforms": (ctypes.c_int, [_p, _p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, _p, _p,
                                            ctypes.POINTER(ctypes.c_int32)]),
    "srt_device_alloc": (ctypes.c_int, [_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "srt_device_free": (ctypes.c_int, [_p, _p]),
    "srt_memcpy": (ctypes.c_int, [_p, _p, _p, ctypes.c_int64]),
    "srt_synchronize": (ctypes.c_int, [_p]),
    "srt_debug_mt_residue": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_int64)]),
    "srt_debug_prefetch_counts": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "srt_debug_lane_stats": (ctypes.c_int, [_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "srt_debug_lean_launches": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_int64)]),
    "srt_render_prefetch": (ctypes.c_int, [_p, ctypes.POINTER(CameraDesc), ctypes.POINTER(RenderArgs)]),
    "srt_render_finish": (ctypes.c_int, [_p, ctypes.POINTER(Stats)]),
    "srt_stream": (ctypes.c_int, [_p, ctypes.POINTER(_p)]),
    "srt_comm_unique_id": (ctypes.c_int, [_p]),
    "srt_comm_init": (ctypes.c_int, [_p, ctypes.c_int, ctypes.c_int, _p]),
    "srt_comm_init_all": (ctypes.c_int, [ctypes.c_int, _p, _p]),
    "srt_comm_rank": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "srt_render_group": (ctypes.c_int, [_p, ctypes.c_int, ctypes.POINTER(CameraDesc), ctypes.POINTER(RenderArgs),
                                        ctypes.POINTER(Stats)]),
    "srt_render_group_finish": (ctypes.c_int, [_p, ctypes.c_int, ctypes.POINTER(Stats)]),
    "srt_material_normal": (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_int64, _p, _p, ctypes.c_int64, _p]),
    "srt_comm_allreduce": (ctypes.c_int, [_p, _p, ctypes.c_int, ctypes.c_int]),
    "srt_comm_barrier": (ctypes.c_int, [_p]),
    "srt_host_alloc": (ctypes.c_int, [_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "srt_host_free": (ctypes.c_int, [_p, _p]),
    "srt_host_register": (ctypes.c_int, [_p, _p, ctypes.c_int64]),
    "srt_host_unregister": (ctypes.c_int, [_p, _p]),
    "srt_last_error": (ctypes.c_char_p, []),
}


class BackendUnavailable(RuntimeError):
    """libsightpy_hip.so is missing or no GPU is visible; sightpy has no CPU fallback."""


class SrtError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("%s (code %d)" % (message, code))
        self.code = code


def lib_path():
    return Path(os.environ.get("SIGHTPY_HIP_LIB", HERE / LIB_NAME))


def load_library(path=None):
    path = Path(path) if path is not None else lib_path()
    if not path.exists():
        raise BackendUnavailable(
            "%s not found: build it with `make -C python-raytracer_amd/csrc` (hipcc, gfx950)" % path
        )
    lib = ctypes.CDLL(str(path))
    # an older build picked by SIGHTPY_HIP_LIB (same-box A/B of library versions) may lack entry
    # points added since; those stay unbound there (calling one raises AttributeError)
    lenient = "SIGHTPY_HIP_LIB" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if lenient and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.srt_abi_version() != ABI_VERSION:
        raise BackendUnavailable("ABI version mismatch in %s" % path)
    return lib


def check(lib, rc):
    if rc == 0:
        return
    msg = lib.srt_last_error().decode(errors="replace")
    if rc == ERR_INDEX:
        raise IndexError(msg)
    if rc == ERR_NAME:
        raise NameError(msg)
    raise SrtError(rc, msg)


def ptr(a):
    """Data pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data
