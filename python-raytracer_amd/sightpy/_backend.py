"""Device backend: one libsightpy_hip.so context per process, scene upload cache, entry points used
by the public API (Scene.render, get_raycolor, get_distances, Collider.intersect, Camera.get_ray).

There is deliberately no CPU path here: if the HIP library or a GPU is missing every entry point
raises `BackendUnavailable`.
"""
import ctypes
import os

import numpy as np

from . import _native as N
from ._lower import lower_scene, camera_desc, collider_record
from .utils.vector3 import vec3

_STATE = {"lib": None, "ctx": None, "device": None, "scene_sig": {}, "buffers": {}, "pinned": {}, "group": None}


class RenderResult:
    def __init__(self, srgb8, rgb, hit_ids, stats):
        self.srgb8 = srgb8
        self.rgb = rgb
        self.hit_ids = hit_ids
        self.stats = stats


def library():
    if _STATE["lib"] is None:
        _STATE["lib"] = N.load_library()
    return _STATE["lib"]


def _env_options(lib, ctx):
    """Options every context of this process takes from the environment (the process context and
    the contexts of a multi-GPU group alike)."""
    if os.environ.get("SIGHTPY_FRAME_KERNEL") is not None:  # A/B switch: 0 = per-depth wavefront kernels
        N.check(lib, lib.srt_set_option(ctx, b"frame_kernel", int(os.environ["SIGHTPY_FRAME_KERNEL"])))
    if os.environ.get("SIGHTPY_DETERMINISTIC") is not None:  # 0: f64 atomics instead of fixed-point sums
        N.check(lib, lib.srt_set_option(ctx, b"deterministic", int(os.environ["SIGHTPY_DETERMINISTIC"])))
    # any library option: SIGHTPY_OPTIONS="key=value,key=value" (srt_set_option; e.g. A/B runs of the
    # whole test suite on another generator or kernel strategy)
    for kv in os.environ.get("SIGHTPY_OPTIONS", "").split(","):
        if kv.strip():
            k, v = kv.split("=")
            N.check(lib, lib.srt_set_option(ctx, k.strip().encode(), int(v)))


def _device_spec():
    """$SIGHTPY_DEVICES as a list of ints, or None (unset / empty / "all")."""
    spec = os.environ.get("SIGHTPY_DEVICES", "").strip()
    if not spec or spec == "all":
        return None
    return [int(v) for v in spec.split(",") if v.strip()]


def context():
    """The process's device context: device = $SIGHTPY_DEVICE, else a one-entry $SIGHTPY_DEVICES,
    else $LOCAL_RANK, else 0."""
    if _STATE["ctx"] is None:
        lib = library()
        n = ctypes.c_int(0)
        rc = lib.srt_device_count(ctypes.byref(n))
        if rc != 0 or n.value < 1:
            raise N.BackendUnavailable(
                "no HIP device visible (%s); sightpy on MI355X has no CPU fallback"
                % lib.srt_last_error().decode(errors="replace")
            )
        spec = _device_spec()
        if os.environ.get("SIGHTPY_DEVICE") is not None:
            dev = int(os.environ["SIGHTPY_DEVICE"])
        elif spec is not None and len(spec) == 1:
            dev = spec[0]
        else:
            dev = int(os.environ.get("LOCAL_RANK", "0"))
        if not 0 <= dev < n.value:
            raise ValueError("sightpy: device %d requested, %d visible" % (dev, n.value))
        ctx = ctypes.c_void_p()
        N.check(lib, lib.srt_create(dev, ctypes.byref(ctx)))
        _env_options(lib, ctx)
        _STATE["ctx"] = ctx
        _STATE["device"] = dev
    return _STATE["lib"], _STATE["ctx"]


def devices():
    """GPUs Scene.render uses: $SIGHTPY_DEVICES ("0,1,2,3" or "all"), else the one context device
    ($SIGHTPY_DEVICE, else $LOCAL_RANK, else 0)."""
    spec = os.environ.get("SIGHTPY_DEVICES", "").strip()
    if not spec:
        return [int(os.environ.get("SIGHTPY_DEVICE", os.environ.get("LOCAL_RANK", "0")))]
    if spec == "all":
        n = ctypes.c_int(0)
        N.check(library(), library().srt_device_count(ctypes.byref(n)))
        return list(range(n.value))
    return _device_spec()


def group():
    """Contexts of the multi-GPU group over devices() (srt_comm_init_all: one RCCL communicator in
    this process, rank q on devices()[q]), created once."""
    devs = devices()
    g = _STATE["group"]
    if g is not None and g[0] == devs:
        return library(), g[1]
    lib = library()
    arr = (ctypes.c_int * len(devs))(*devs)
    ctxs = (ctypes.c_void_p * len(devs))()
    N.check(lib, lib.srt_comm_init_all(len(devs), arr, ctxs))
    for q in range(len(devs)):
        _env_options(lib, ctypes.c_void_p(ctxs[q]))
    _STATE["group"] = (devs, ctxs)
    return lib, ctxs


def upload(scene, extra_media=(), force=False, ctx=None):
    """Lower and upload `scene` to `ctx` (default: the process context) unless the identical tables
    are already resident there."""
    lib = library()
    if ctx is None:
        ctx = context()[1]
    L = lower_scene(scene, extra_media)
    sig = L.signature()
    key = ctx.value if isinstance(ctx, ctypes.c_void_p) else int(ctx)
    if force or sig != _STATE["scene_sig"].get(key):
        _STATE["scene_sig"].pop(key, None)
        N.check(lib, lib.srt_upload_scene(ctx, ctypes.byref(L.desc())))
        _STATE["scene_sig"][key] = sig
    return L


def pinned_buffer(name, nbytes):
    """A named pinned host allocation of the context (srt_host_alloc), grown on demand and kept across
    calls, as a uint8 numpy array: the device copies into it at full PCIe rate (a pageable destination
    goes through the runtime's staging copies)."""
    lib, ctx = context()
    cur = _STATE["pinned"].get(name)
    if cur is None or cur[1] < nbytes:
        if cur is not None:
            N.check(lib, lib.srt_host_free(ctx, cur[0]))
            del _STATE["pinned"][name]
        p = ctypes.c_void_p()
        N.check(lib, lib.srt_host_alloc(ctx, max(int(nbytes), 8), ctypes.byref(p)))
        cur = (p, int(nbytes))
        _STATE["pinned"][name] = cur
    return np.ctypeslib.as_array(ctypes.cast(cur[0], ctypes.POINTER(ctypes.c_uint8)), (cur[1],))[:nbytes]


class _HostBlock:
    """A pinned host allocation of the context lent to numpy as the base of one array (and through it
    to a PIL image mapping that array): when the last of them is gone the allocation goes back to a
    small pool for the next image (image_block)."""

    __slots__ = ("ptr", "nbytes")

    def __init__(self, ptr, nbytes):
        self.ptr, self.nbytes = ptr, nbytes

    @property
    def __array_interface__(self):
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 3}

    def __del__(self):
        try:
            _STATE["blocks_out"] -= 1
            if _STATE["ctx"] is None:
                return
            if sum(len(v) for v in _STATE["blocks"].values()) < _BLOCKS_FREE_MAX:
                _STATE["blocks"].setdefault(self.nbytes, []).append(self.ptr)
            else:
                _STATE["lib"].srt_host_free(_STATE["ctx"], ctypes.c_void_p(self.ptr))
        except Exception:  # (interpreter shutdown: the process frees it)
            pass


_STATE["blocks"] = {}      # nbytes -> free pinned allocations (pointers), _BLOCKS_FREE_MAX in all
_STATE["blocks_out"] = 0   # allocations lent to live arrays
_BLOCKS_FREE_MAX = 4
_BLOCKS_OUT_MAX = 16


def image_block(nbytes):
    """A uint8 array of `nbytes` in pinned host memory of its own, for an output that outlives the call
    (Scene.render's image maps it: the device copies the frame into it at full PCIe rate and PIL takes
    it without a copy), or None when _BLOCKS_OUT_MAX such arrays are alive already (the caller then
    copies out of the shared pinned buffer)."""
    lib, ctx = context()
    if _STATE["blocks_out"] >= _BLOCKS_OUT_MAX:
        return None
    free = _STATE["blocks"].get(nbytes)
    if free:
        ptr = free.pop()
    else:
        p = ctypes.c_void_p()
        N.check(lib, lib.srt_host_alloc(ctx, max(int(nbytes), 8), ctypes.byref(p)))
        ptr = p.value
    _STATE["blocks_out"] += 1
    return np.asarray(_HostBlock(ptr, int(nbytes)))


def rgb_image(rgbx, width, height, mapped):
    """PIL RGB image of 4-byte pixels (R, G, B, 255: PIL's own layout of mode RGB).  `mapped`: the image
    maps `rgbx` (which it keeps alive; read-only, so PIL copies it before any change), else the pixels
    are copied into a new image.  Either way the image equals Image.fromarray(rgbx[..., :3], "RGB")."""
    from PIL import Image

    if mapped:
        try:
            im = Image.frombuffer("RGBX", (width, height), rgbx, "raw", "RGBX", 0, 1)
            core = im.im
            core.setmode("RGB")
            img = im._new(core)
            img.readonly = 1
            if img.mode == "RGB" and img.size == (width, height):
                return img
        except Exception:  # (a Pillow without these internals: the copy below)
            pass
    img = Image.new("RGB", (width, height), None)
    img.frombytes(rgbx, "raw", "RGBX")
    return img


def device_buffer(name, nbytes):
    """A named device allocation of the context, grown on demand (kept across calls)."""
    lib, ctx = context()
    cur = _STATE["buffers"].get(name)
    if cur is not None and cur[1] >= nbytes:
        return cur[0]
    if cur is not None:
        N.check(lib, lib.srt_device_free(ctx, cur[0]))
        del _STATE["buffers"][name]
    p = ctypes.c_void_p()
    N.check(lib, lib.srt_device_alloc(ctx, max(int(nbytes), 8), ctypes.byref(p)))
    _STATE["buffers"][name] = (p, int(nbytes))
    return p


def release_buffer(name):
    """Free a named device allocation of the context."""
    cur = _STATE["buffers"].pop(name, None)
    if cur is not None:
        lib, ctx = context()
        N.check(lib, lib.srt_device_free(ctx, cur[0]))


def numpy_uniforms(n_out, n_skip=0, out=None):
    """`np.random.rand(n_out)` computed on the GPU (then `n_skip` more draws), advancing numpy's
    global RandomState exactly as the host draws would (srt_mt19937_uniforms).

    Returns the doubles in a device buffer (a ctypes pointer, valid until the next call) when `out`
    is None, else writes the host array `out`."""
    lib, ctx = context()
    name, key, pos, has_gauss, gauss = np.random.get_state()
    if name != "MT19937":
        raise ValueError("numpy's global generator is not MT19937")
    key = np.ascontiguousarray(key, dtype=np.uint32)
    if out is None:
        release_buffer("uniforms")  # sized per call, not kept at the largest request ever made
    dst = device_buffer("uniforms", 8 * n_out) if out is None else N.ptr(out)
    key_out = np.empty(624, dtype=np.uint32)
    pos_out = ctypes.c_int32(0)
    N.check(lib, lib.srt_mt19937_uniforms(ctx, N.ptr(key), int(pos), int(n_out), int(n_skip), dst, N.ptr(key_out),
                                          ctypes.byref(pos_out)))
    np.random.set_state((name, key_out, pos_out.value, has_gauss, gauss))
    return dst


def _planar(v, n=None):
    """vec3 (scalars or arrays) -> C-contiguous float64 (3, n)."""
    comps = [np.asarray(c, dtype=np.float64) for c in (v.x, v.y, v.z)]
    if n is None:
        n = max([c.size for c in comps])
    return np.ascontiguousarray(np.stack([np.broadcast_to(c.reshape(-1) if c.ndim else c, (n,)) for c in comps]))


def _default_seed():
    """Seed for the device RNG derived from numpy's global RNG state WITHOUT consuming it (the
    reference's render consumes only the camera draws from the parent's stream)."""
    key, pos = np.random.get_state()[1:3]
    return (int(key[pos % 624]) << 32 | int(key[(pos + 397) % 624])) ^ (int(pos) * 0x9E3779B97F4A7C15) & (2**64 - 1)


def render_scene(scene, spp, jitter=None, seed=None, batch_size=None, rows=None, want_rgb=True, want_hits=False,
                 jitter_device=None, mt=False, pinned_u8=False, rgbx=False, prefetch=None, out_u8=None):
    """Scene.render on the device.  `jitter` (spp, 4, H*W) from numpy or None for the device RNG;
    `jitter_device`: the same uniforms already in device memory (numpy_uniforms); `mt=True`: the
    jitter is numpy's global stream generated on the device (the reference's draws, including the
    sizing draw of scene.py:81), and numpy's global state is advanced past it.  `pinned_u8`: the
    uint8 image lands in the context's pinned host buffer (a view, valid until the next such call)
    instead of a new array.  Without `want_rgb` the linear RGB is resolved and kept in HBM
    (SRT_RENDER_RGB_LOCAL), as the reference keeps it internal.  `rgbx`: the image as 4-byte pixels
    (R, G, B, 255; SRT_RENDER_RGBX), srgb8 of shape (rows, W, 4).  `prefetch` (whole frames with
    `mt`): the jitter's generation is queued on the GPU (srt_render_prefetch) before the scene is
    lowered and uploaded, so the two overlap (default on; $SIGHTPY_PREFETCH=0 turns it off).
    `out_u8`: a host uint8 array of the image's size to write the image into (image_block)."""
    lib, ctx = context()
    if prefetch is None:
        prefetch = os.environ.get("SIGHTPY_PREFETCH", "1") != "0"
    cam = scene.camera
    W, H = int(cam.screen_width), int(cam.screen_height)
    rows_arr = None if rows is None else np.ascontiguousarray(rows, dtype=np.int32)
    nrows = H if rows_arr is None else len(rows_arr)
    npix = nrows * W
    cd = camera_desc(cam)
    a = N.RenderArgs()
    a.spp = int(spp)
    a.sample_base = 0
    a.n_rows = nrows
    a.batch_spp = int(batch_size or 0)
    a.rows = N.ptr(rows_arr)
    j = None
    if jitter_device is not None:
        a.jitter = jitter_device.value if isinstance(jitter_device, ctypes.c_void_p) else jitter_device
    elif jitter is not None:
        j = np.ascontiguousarray(jitter, dtype=np.float64)
        if j.shape != (spp, 4, npix):
            raise ValueError("jitter must have shape (spp, 4, %d)" % npix)
        a.jitter = N.ptr(j)
    a.seed = int(seed if seed is not None else _default_seed()) & (2**64 - 1)
    state = None
    if mt:
        if j is not None or jitter_device is not None:
            raise ValueError("mt=True draws the jitter itself")
        state = N.MtState.from_numpy()
        a.mt = ctypes.pointer(state)
    a.flags = (0 if want_rgb else N.RENDER_RGB_LOCAL) | (N.RENDER_RGBX if rgbx else 0)
    if mt and prefetch and rows_arr is None and nrows == H:
        N.check(lib, lib.srt_render_prefetch(ctx, ctypes.byref(cd), ctypes.byref(a)))
    upload(scene)
    rgb = np.empty((3, npix)) if want_rgb else None
    ch = 4 if rgbx else 3
    if out_u8 is not None:
        if out_u8.dtype != np.uint8 or out_u8.size != ch * npix or not out_u8.flags.c_contiguous:
            raise ValueError("out_u8 must be a contiguous uint8 array of %d bytes" % (ch * npix))
        u8 = out_u8.reshape(npix, ch)
    else:
        u8 = (pinned_buffer("render_u8", ch * npix) if pinned_u8 else np.empty(ch * npix, dtype=np.uint8)).reshape(npix, ch)
    hits = np.empty((spp, npix), dtype=np.int32) if want_hits else None
    a.out_rgb = N.ptr(rgb)
    a.out_srgb8 = N.ptr(u8)
    a.out_hit_id = N.ptr(hits)
    st = N.Stats()
    N.check(lib, lib.srt_render(ctx, ctypes.byref(cd), ctypes.byref(a), ctypes.byref(st)))
    if state is not None:
        state.to_numpy()
    return RenderResult(u8.reshape(nrows, W, ch), rgb, hits, st.as_dict())


def render_group(scene, spp, seed=None, batch_size=None, want_rgb=True, mt=True):
    """Scene.render on every GPU of devices(): each renders its row bands (SRT_RENDER_SHARDED; at
    most shard_kmax bands per GPU, rt_device.h shard_band_height: 27 rows at 1080p on 8 GPUs) and
    the tiles are gathered to the first over RCCL (srt_render_group).  `mt`: numpy's stream as in
    render_scene (else the device RNG)."""
    lib, ctxs = group()
    for q in range(len(ctxs)):
        upload(scene, ctx=ctypes.c_void_p(ctxs[q]))
    cam = scene.camera
    W, H = int(cam.screen_width), int(cam.screen_height)
    cd = camera_desc(cam)
    a = N.RenderArgs()
    a.spp, a.sample_base, a.n_rows, a.batch_spp = int(spp), 0, H, int(batch_size or 0)
    a.seed = int(seed if seed is not None else _default_seed()) & (2**64 - 1)
    state = None
    if mt:
        state = N.MtState.from_numpy()
        a.mt = ctypes.pointer(state)
    rgb = np.empty((3, W * H)) if want_rgb else None
    u8 = np.empty((W * H, 3), dtype=np.uint8)
    a.out_rgb, a.out_srgb8 = N.ptr(rgb), N.ptr(u8)
    a.flags = 0 if want_rgb else N.RENDER_RGB_LOCAL  # (every GPU keeps its rows of the linear RGB)
    st = N.Stats()
    N.check(lib, lib.srt_render_group(ctxs, len(ctxs), ctypes.byref(cd), ctypes.byref(a), ctypes.byref(st)))
    if state is not None:
        state.to_numpy()
    return RenderResult(u8.reshape(H, W, 3), rgb, None, st.as_dict())


def _media_of(ray_n, count):
    """Per-ray complex IOR triples -> (unique triples, index per ray)."""
    comps = [np.asarray(c) for c in (ray_n.x, ray_n.y, ray_n.z)]
    cols = [np.broadcast_to(c.astype(np.complex128), (count,)) for c in comps]
    tri = np.stack(cols, axis=1)
    uniq, inv = np.unique(tri, axis=0, return_inverse=True)
    return [tuple(complex(v) for v in row) for row in uniq], inv.reshape(-1).astype(np.int32)


def trace_rays(ray, scene, seed=None, return_stats=False, hits=None):
    """get_raycolor(ray, scene) on the device: colour of every ray of the batch.  `hits`:
    (collider index per ray, distance, orientation) -- Material.get_color at those hits
    (srt_shade) instead of the nearest-hit search of the first depth."""
    lib, ctx = context()
    n = len(ray)
    uniq, inv = _media_of(ray.n, n)
    L = upload(scene, extra_media=uniq)
    remap = np.array([L.media_keys.index(k) for k in uniq], dtype=np.int32)
    med = np.ascontiguousarray(remap[inv])
    O = _planar(ray.origin, n)
    D = _planar(ray.dir, n)
    out = np.empty((3, n))
    a = N.TraceArgs()
    a.n = n
    a.origin, a.dir, a.medium = N.ptr(O), N.ptr(D), N.ptr(med)
    a.depth = int(ray.depth)
    a.diffuse_reflections = int(ray.diffuse_reflections)
    a.seed = int(seed if seed is not None else _default_seed()) & (2**64 - 1)
    a.out_rgb = N.ptr(out)
    st = N.Stats()
    if hits is None:
        N.check(lib, lib.srt_trace(ctx, ctypes.byref(a), ctypes.byref(st)))
    else:
        ids = np.ascontiguousarray(np.broadcast_to(np.asarray(hits[0], dtype=np.int32), (n,)))
        t = np.ascontiguousarray(np.broadcast_to(np.asarray(hits[1], dtype=np.float64), (n,)))
        o = np.ascontiguousarray(np.broadcast_to(np.asarray(hits[2], dtype=np.float64), (n,)))
        N.check(lib, lib.srt_shade(ctx, ctypes.byref(a), N.ptr(ids), N.ptr(t), N.ptr(o), ctypes.byref(st)))
    col = vec3(out[0], out[1], out[2])
    return (col, st.as_dict()) if return_stats else col


def nearest_hits(scene, O, D):
    """Nearest hit over scene.collider_list: (t, collider index or -1, orientation)."""
    lib, ctx = context()
    upload(scene)
    Oa = _planar(O)
    n = Oa.shape[1]
    Da = _planar(D, n)
    t = np.empty(n)
    ids = np.empty(n, dtype=np.int32)
    orient = np.empty(n)
    N.check(lib, lib.srt_nearest(ctx, N.ptr(Oa), N.ptr(Da), n, N.ptr(t), N.ptr(ids), N.ptr(orient)))
    return t, ids, orient


def intersect_collider(collider, O, D):
    """Collider.intersect(O, D) -> (2, N) [distance; orientation] on the device."""
    lib, ctx = context()
    rec = np.ascontiguousarray(collider_record(collider))
    Oa = _planar(O)
    n = Oa.shape[1]
    Da = _planar(D, n)
    out = np.empty((2, n))
    N.check(lib, lib.srt_intersect_collider(ctx, N.ptr(rec.reshape(1)), N.ptr(Oa), N.ptr(Da), n, N.ptr(out)))
    return out


def collider_surface(collider, P, normal=True, uv=True, primitive_uv=False):
    """Collider.get_Normal (3, n) and get_uv (2, n) at points P on the device
    (srt_collider_surface); `primitive_uv` applies the owning Cuboid/SkyBox's (4, 3) divide."""
    lib, ctx = context()
    rec = np.ascontiguousarray(collider_record(collider))
    if getattr(getattr(collider, "assigned_primitive", None), "uv_cube_cross", False):
        rec["flags"] |= N.CF_UV_CROSS
    Pa = _planar(P)
    n = Pa.shape[1]
    Nout = np.empty((3, n)) if normal else None
    uvout = np.empty((2, n)) if uv else None
    N.check(lib, lib.srt_collider_surface(ctx, N.ptr(rec.reshape(1)), N.ptr(Pa), n, N.ptr(Nout), N.ptr(uvout),
                                          int(bool(primitive_uv))))
    return Nout, uvout


def material_normal(material, hit):
    """Material.get_Normal(hit) on the device (srt_material_normal): the collider normal, or the
    material's normal map through the collider's inverse_basis_matrix, times hit.orientation (3, n)."""
    from ._lower import texture_record

    lib, ctx = context()
    c = hit.collider
    rec = np.ascontiguousarray(collider_record(c))
    if getattr(getattr(c, "assigned_primitive", None), "uv_cube_cross", False):
        rec["flags"] |= N.CF_UV_CROSS  # (the primitive's uv, as hit.get_uv() takes it)
    Pa = _planar(hit.point)
    n = Pa.shape[1]
    orient = np.ascontiguousarray(np.broadcast_to(np.asarray(hit.orientation, dtype=np.float64).reshape(-1)
                                                  if np.ndim(hit.orientation) else hit.orientation, (n,)))
    tex, texels = None, None
    if material.normalmap is not None:
        if not hasattr(c, "inverse_basis_matrix"):
            raise AttributeError("'%s' object has no attribute 'inverse_basis_matrix'" % type(c).__name__)
        tex, texels = texture_record(material.normalmap_u8, material.repeat, linear=False)
        tex = np.ascontiguousarray(tex).reshape(1)
    out = np.empty((3, n))
    N.check(lib, lib.srt_material_normal(ctx, N.ptr(rec.reshape(1)), N.ptr(tex), N.ptr(texels),
                                         0 if texels is None else texels.size, N.ptr(Pa), N.ptr(orient), n,
                                         N.ptr(out)))
    return out


def texture_lookup(u8, repeat, u, v, linear=True):
    """image.get_color at (u, v) on the device (srt_texture_lookup): rgb (3, n)."""
    from ._lower import texture_record

    lib, ctx = context()
    rec, texels = texture_record(u8, repeat, linear)
    uv = np.ascontiguousarray(np.stack(np.broadcast_arrays(np.asarray(u, dtype=np.float64),
                                                           np.asarray(v, dtype=np.float64))).reshape(2, -1))
    n = uv.shape[1]
    out = np.empty((3, n))
    N.check(lib, lib.srt_texture_lookup(ctx, N.ptr(rec.reshape(1)), N.ptr(texels), texels.size, N.ptr(uv), n,
                                        N.ptr(out)))
    return out


def primary_rays(camera, jitter):
    """Camera.get_ray geometry for one sample; jitter (4, H*W).  Returns (origin, dir) vec3."""
    lib, ctx = context()
    cd = camera_desc(camera)
    n = int(camera.screen_width) * int(camera.screen_height)
    J = np.ascontiguousarray(jitter, dtype=np.float64).reshape(4, n)
    O = np.empty((3, n))
    D = np.empty((3, n))
    N.check(lib, lib.srt_primary_rays(ctx, ctypes.byref(cd), N.ptr(J), N.ptr(O), N.ptr(D)))
    return vec3(O[0], O[1], O[2]), vec3(D[0], D[1], D[2])
