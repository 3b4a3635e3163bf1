"""Scene lowering: sightpy objects -> the flat POD tables of include/sightpy_rt.h.

Every scalar the kernels consume is computed here with the same expression the reference
evaluates (mostly inside its per-call numpy code, e.g. the Glossy Schlick F0 at glossy.py:66/91,
the plane normal at plane.py:41, the cuboid basis at cuboid.py:84-103), so the device sees
bit-identical constants.  Per-medium quantities (the specular F0 depends on the ray's index of
refraction) are tabulated over the finite set of media a ray can be in: scene.n and the n of
every Refractive material.
"""
import collections
import os
import zlib

import numpy as np

try:
    import xxhash as _xxhash
except ImportError:  # pragma: no cover - zlib fallback
    _xxhash = None

from . import _native as N
from .utils.vector3 import vec3
from .utils.colour_functions import sRGB_to_sRGB_linear
from .geometry.sphere import Sphere_Collider
from .geometry.plane import Plane_Collider
from .geometry.cuboid import Cuboid_Collider
from .geometry.triangle import Triangle_Collider
from .materials.glossy import Glossy
from .materials.refractive import Refractive
from .materials.thin_film_interference import ThinFilmInterference
from .materials.diffuse import Diffuse
from .materials.emissive import Emissive
from .textures.texture import image, solid_color
from .backgrounds.skybox import SkyBox_Material
from .lights import DirectionalLight, PointLight

_LIN_LUT = sRGB_to_sRGB_linear(np.arange(256) / 256.0)  # image textures (load_image_as_linear_sRGB)
_RAW_LUT = np.arange(256) / 256.0                        # load_image (lightmap, tables, noise, normal maps)


def _c(v):
    """Components of a vec3 as complex (Python scalars)."""
    return [complex(v.x), complex(v.y), complex(v.z)]


def _f3(v):
    return [float(v.x), float(v.y), float(v.z)]


class Lowered:
    """Tables for srt_upload_scene plus host-side bookkeeping (keeps the arrays alive)."""

    def __init__(self):
        self.colliders = None
        self.materials = None
        self.textures = None
        self.texels = None
        self.lights = None
        self.media = None
        self.glossy_f0 = None
        self.light_local = None
        self.importance = None
        self.ambient = (0.0, 0.0, 0.0)
        self.max_ray_depth = 0
        self.has_diffuse = 0
        self.media_keys = []
        self.scene_n = None
        self.texel_key = 0
        self.device_index = []  # scene.collider_list index -> device collider index (-1: a user class, _hybrid)

    def desc(self):
        d = N.SceneDesc()
        d.n_colliders = len(self.colliders)
        d.n_materials = len(self.materials)
        d.n_textures = len(self.textures)
        d.n_lights = len(self.lights)
        d.n_media = len(self.media)
        d.n_importance = len(self.importance)
        d.colliders = N.ptr(self.colliders) if len(self.colliders) else None
        d.materials = N.ptr(self.materials) if len(self.materials) else None
        d.textures = N.ptr(self.textures) if len(self.textures) else None
        d.texels = N.ptr(self.texels) if self.texels.size else None
        d.texel_bytes = int(self.texels.size)
        d.lights = N.ptr(self.lights) if len(self.lights) else None
        d.media = N.ptr(self.media)
        d.glossy_f0 = N.ptr(self.glossy_f0) if self.glossy_f0.size else None
        d.light_local = N.ptr(self.light_local) if self.light_local.size else None
        d.importance = N.ptr(self.importance) if self.importance.size else None
        d.ambient[:] = list(self.ambient)
        d.max_ray_depth = int(self.max_ray_depth)
        d.has_diffuse = int(self.has_diffuse)
        d.texel_key = int(self.texel_key)
        return d

    def signature(self):
        parts = [self.colliders.tobytes(), self.materials.tobytes(), self.textures.tobytes(),
                 self.lights.tobytes(), self.media.tobytes(), self.glossy_f0.tobytes(),
                 self.light_local.tobytes(), self.importance.tobytes(), repr(self.ambient).encode(),
                 str(self.max_ray_depth).encode()]
        return hash((tuple(parts), self.texels.size, self.texel_key))


class _TexturePool:
    def __init__(self):
        self.records = []
        self.images = []
        self.offsets = {}
        self.size = 0

    def add(self, u8, lut, repeat=1.0, channel0=0, idx_shape=None):
        u8 = np.ascontiguousarray(u8)
        if u8.dtype != np.uint8:
            raise TypeError("textures must be uint8 images")
        if u8.ndim == 2:
            u8 = u8[:, :, None]
        if u8.shape[2] < 3:  # grey images: replicate to RGB (device reads 3 channels per texel)
            src = u8
            hit = _GREY_CACHE.get(id(src))
            if hit is None or hit[0] is not src or hit[2] != _fingerprint(src):
                hit = (src, np.ascontiguousarray(np.repeat(src[:, :, :1], 3, axis=2)), _fingerprint(src))
                _GREY_CACHE[id(src)] = hit  # (keeps src alive, so its id stays unique)
                while len(_GREY_CACHE) > _GREY_CACHE_MAX:
                    _GREY_CACHE.popitem(last=False)
            else:
                _GREY_CACHE.move_to_end(id(src))
            u8 = hit[1]
        key = id(u8) if u8.base is None else (id(u8.base), u8.__array_interface__["data"][0])
        if key not in self.offsets:
            self.offsets[key] = self.size
            self.images.append(u8)
            self.size += u8.size
        rec = np.zeros((), dtype=N.TEXTURE_DTYPE)
        rec["offset"] = self.offsets[key]
        rec["height"], rec["width"], rec["channels"] = u8.shape[0], u8.shape[1], u8.shape[2]
        rec["channel0"] = channel0
        ih, iw = idx_shape if idx_shape is not None else u8.shape[:2]
        rec["idx_h"], rec["idx_w"] = ih, iw
        rec["repeat"] = repeat
        rec["lut"] = lut
        self.records.append(rec)
        return len(self.records) - 1

    def key(self):
        """Identity of the pool's images: the same image objects in the same order, with the same
        contents (a content hash per image, so an image edited in place is uploaded again)."""
        if not self.images:
            return 0
        ident = tuple((id(im), im.__array_interface__["data"][0], im.shape, _fingerprint(im)) for im in self.images)
        return hash(ident) & (2**64 - 1) or 1

    def finish(self):
        """Records and the concatenated texel pool.  The pool of the last key is cached: a frame
        sequence (create_animation) re-lowers its scene every frame with the same images, and the
        device keeps the resident copy for an unchanged texel_key (srt_upload_scene)."""
        tex = np.array(self.records, dtype=N.TEXTURE_DTYPE) if self.records else np.zeros(0, N.TEXTURE_DTYPE)
        key = self.key()
        cached = _POOL_CACHE.get("pool")
        if cached is not None and cached[0] == key and key != 0:
            return tex, cached[1], key
        texels = np.concatenate([im.reshape(-1) for im in self.images]) if self.images else np.zeros(0, np.uint8)
        # the cache holds the images too, so their ids cannot be reused by other arrays meanwhile
        _POOL_CACHE["pool"] = (key, texels, list(self.images))
        return tex, texels, key


_POOL_CACHE = {}
_GREY_CACHE = collections.OrderedDict()  # id(grey image) -> (image, RGB copy, fingerprint), LRU
_GREY_CACHE_MAX = 16


_FP_CACHE = collections.OrderedDict()  # (id(root), address, shape, strides) -> (root, fingerprint), LRU
_FP_CACHE_MAX = 64


def _immutable_root(a):
    """The `bytes` object holding `a`'s texels when nothing can write them (images decoded by PIL:
    np.asarray(img) is a read-only view of immutable bytes), else None."""
    b = a
    while isinstance(b, np.ndarray):
        if b.flags.writeable:
            return None
        if b.base is None:
            return None
        b = b.base
    return b if isinstance(b, bytes) else None


def _fingerprint(a):
    """Content hash of a texture (xxh3: ~2 ms for the 37.7 MB stormydays image on every Scene.render).
    Texels that no one can modify (a read-only view of immutable bytes) are hashed once: the hash is
    cached by their memory, and the cache holds the bytes so the key stays unique."""
    root = _immutable_root(a) if isinstance(a, np.ndarray) else None
    if root is not None:
        key = (id(root), a.__array_interface__["data"][0], a.shape, a.strides)
        hit = _FP_CACHE.get(key)
        if hit is not None and hit[0] is root:
            _FP_CACHE.move_to_end(key)
            return hit[1]
    buf = memoryview(np.ascontiguousarray(a)).cast("B")
    fp = _xxhash.xxh3_64_intdigest(buf) if _xxhash is not None else zlib.crc32(buf)
    if root is not None:
        _FP_CACHE[key] = (root, fp)
        while len(_FP_CACHE) > _FP_CACHE_MAX:
            _FP_CACHE.popitem(last=False)
    return fp


# Memo of the pure per-material expressions below (each ~15-20 us of numpy scalar/vec3 arithmetic,
# evaluated on every Scene.render): keyed by the operands' types and exact values (repr keeps -0.0
# and nan apart), so a memo hit returns what the expression would.  Operands that are not Python or
# numpy scalars / small arrays are not memoised.
_EXPR_MEMO = {}
_EXPR_MEMO_MAX = 4096


def _vkey(v):
    """Exact key of a scalar or small array operand, or None."""
    if isinstance(v, (float, complex, int)) and not isinstance(v, bool):
        return (type(v).__name__, repr(v))
    if isinstance(v, np.ndarray) and v.size <= 4:
        return ("nd", v.dtype.str, v.shape, v.tobytes())
    if isinstance(v, np.generic):
        return ("np", v.dtype.str, v.tobytes())
    return None


def _memo(tag, operands, fn):
    keys = tuple(_vkey(v) for v in operands)
    if any(k is None for k in keys):
        return fn()
    key = (tag,) + keys
    hit = _EXPR_MEMO.get(key)
    if hit is None:
        if len(_EXPR_MEMO) >= _EXPR_MEMO_MAX:
            _EXPR_MEMO.clear()
        hit = _EXPR_MEMO[key] = fn()
    return hit


def _medium_f0(n_ray, n_mat):
    """|(n_ray - n)/(n_ray + n)|^2 per component with numpy array semantics (glossy.py:66):
    n_ray is a length-1 array of the ray's n dtype, n_mat the material's Python scalars."""
    def f0():
        return [float((np.abs((a - b) / (a + b)) ** 2)[0]) for a, b in zip(n_ray, n_mat)]

    return list(_memo("medium_f0", tuple(n_ray) + tuple(n_mat), f0))


def _glossy_f0(scene_n, m_n):
    """np.abs((scene.n - m.n) / (scene.n + m.n)) ** 2 as in glossy.py:91 (vec3 of Python scalars)."""
    def f0():
        return _f3(np.abs((scene_n - m_n) / (scene_n + m_n)) ** 2)

    ops = (scene_n.x, scene_n.y, scene_n.z, m_n.x, m_n.y, m_n.z)
    return list(_memo("glossy_f0", ops, f0))


def texture_record(u8, repeat=1.0, linear=True):
    """One srt_texture record over its own texel array (offset 0): image.get_color's lookup
    (srt_texture_lookup).  `linear`: the load_image_as_linear_sRGB table, else load_image's."""
    pool = _TexturePool()
    i = pool.add(u8, _LIN_LUT if linear else _RAW_LUT, repeat=repeat)
    return pool.records[i], np.ascontiguousarray(np.concatenate([im.reshape(-1) for im in pool.images]))


def collider_record(c):
    """One srt_collider record (no material/primitive fields)."""
    rec = np.zeros((), dtype=N.COLLIDER_DTYPE)
    p = np.zeros(N.SRT_COLLIDER_PARAMS)
    if isinstance(c, Sphere_Collider):
        rec["type"] = N.SPHERE
        p[0:3] = _f3(c.center)
        p[3] = c.radius
        p[4] = 1.0 / c.radius
        p[5] = c.center.square_length()
        p[6] = c.radius * c.radius
    elif isinstance(c, Plane_Collider):
        rec["type"] = N.PLANE
        p[0:3] = _f3(c.center)
        p[3:6] = _f3(c.normal)
        p[6:9] = _f3(c.u_axis)
        p[9:12] = _f3(c.v_axis)
        p[12] = c.w
        p[13] = c.h
        p[14:16] = [float(c.uv_shift[0]), float(c.uv_shift[1])]
        p[16:25] = np.asarray(c.inverse_basis_matrix, dtype=np.float64).reshape(-1)
    elif isinstance(c, Cuboid_Collider):
        rec["type"] = N.CUBOID
        p[0:3] = _f3(c.center)
        p[3:12] = np.asarray(c.basis_matrix, dtype=np.float64).reshape(-1)
        p[12:15] = _f3(c.lb_local_basis)
        p[15:18] = _f3(c.rt_local_basis)
        p[18:21] = _f3(c.ax_w)
        p[21:24] = _f3(c.ax_h)
        p[24:27] = _f3(c.ax_l)
        p[27], p[28], p[29] = c.width, c.height, c.length
        p[30:39] = np.asarray(c.inverse_basis_matrix, dtype=np.float64).reshape(-1)
        p[39], p[40], p[41] = 1.0 / c.width, 1.0 / c.height, 1.0 / c.length
        eye = np.eye(3)
        p[42] = 1.0 if (np.array_equal(c.basis_matrix, eye) and np.array_equal(c.inverse_basis_matrix, eye)) else 0.0
    elif isinstance(c, Triangle_Collider):
        rec["type"] = N.TRIANGLE
        p[0:3] = _f3(c.centroid)
        p[3:6] = _f3(c.normal)
        p[6:9] = _f3(c.p1)
        p[9:12] = _f3(c.p2)
        p[12:15] = _f3(c.p3)
        p[15:18] = _f3(c.n31)
        p[18:21] = _f3(c.n12)
        p[21:24] = _f3(c.n23)
    else:
        raise NotImplementedError(
            "collider type %s has no device kernel (sightpy on MI355X has no CPU fallback)" % type(c).__name__
        )
    rec["p"] = p
    return rec


def camera_desc(cam):
    """srt_camera for a Camera (pointers into cam.xs / cam.ys)."""
    d = N.CameraDesc()
    d.width = int(cam.screen_width)
    d.height = int(cam.screen_height)
    cam._xs_c = np.ascontiguousarray(cam.xs, dtype=np.float64)
    cam._ys_c = np.ascontiguousarray(cam.ys, dtype=np.float64)
    d.xs = N.ptr(cam._xs_c)
    d.ys = N.ptr(cam._ys_c)
    d.look_from[:] = _f3(cam.look_from)
    d.right[:] = _f3(cam.cameraRight)
    d.up[:] = _f3(cam.cameraUp)
    d.fwd_fd[:] = _f3(cam.cameraFwd * cam.focal_distance)
    d.cam_width = float(cam.camera_width)
    d.cam_height = float(cam.camera_height)
    d.lens_radius = float(cam.lens_radius)
    d.focal_distance = float(cam.focal_distance)
    return d


def lower_scene(scene, extra_media=()):
    from ._hybrid import is_hybrid, device_collider, device_material

    L = Lowered()
    pool = _TexturePool()
    # a scene with user Collider / Material subclasses (_hybrid.py) keeps the colliders whose geometry
    # the device code implements (a user material's collider too: it casts shadows on the device's
    # glossy hits, and the host never has the device shade it: its material is a black placeholder)
    hybrid = is_hybrid(scene)
    colliders = [c for c in scene.collider_list if device_collider(c)] if hybrid else scene.collider_list
    dev = {id(c): i for i, c in enumerate(colliders)}
    L.device_index = [dev.get(id(c), -1) for c in scene.collider_list]
    # ---- media: row 0 = scene.n, then each refractive material's n, then caller extras -------
    media = [_c(scene.n)]
    keys = [tuple(media[0])]
    ray_n0 = [np.broadcast_to(np.asarray(v), (1,)) for v in (scene.n.x, scene.n.y, scene.n.z)]
    media_arrays = [ray_n0]

    def medium_of(cvals):
        k = tuple(cvals)
        if k not in keys:
            keys.append(k)
            media.append(list(cvals))
            media_arrays.append([np.array([v], dtype=np.complex128) for v in cvals])
        return keys.index(k)

    materials, mat_index = [], {}
    prims = []
    for c in colliders:
        m = c.assigned_primitive.material
        if id(m) not in mat_index:
            mat_index[id(m)] = len(materials)
            materials.append(m)
        if isinstance(m, Refractive):
            medium_of(_c(m.n))
    for e in extra_media:
        medium_of(list(e))

    # ---- materials --------------------------------------------------------------------------
    mrecs = np.zeros(len(materials), dtype=N.MATERIAL_DTYPE)
    mrecs["tex"] = -1
    mrecs["tex_aux0"] = -1
    mrecs["tex_aux1"] = -1
    mrecs["normalmap"] = -1
    glossy_f0 = np.zeros((len(materials), len(media), 3))
    for i, m in enumerate(materials):
        r = mrecs[i]
        p = np.zeros(N.SRT_MATERIAL_PARAMS)
        if hybrid and not device_material(m):
            r["type"] = N.EMISSIVE  # (placeholder: never shaded on the device)
            r["p"] = p
            mrecs[i] = r
            continue
        if getattr(m, "normalmap_u8", None) is not None:
            r["normalmap"] = pool.add(m.normalmap_u8, _RAW_LUT, repeat=m.repeat)
        if isinstance(m, Glossy):
            r["type"] = N.GLOSSY
            if isinstance(m.diff_texture, image):
                r["tex"] = pool.add(m.diff_texture.u8, _LIN_LUT, repeat=m.diff_texture.repeat)
            else:
                p[0:3] = _f3(m.diff_texture.color * m.diff_coeff)
            p[3] = m.diff_coeff
            if m.roughness != 0.0:
                r["flags"] |= N.MF_ROUGH
                a = 2.0 / (m.roughness ** 2.0) - 2.0
                p[4] = a
                p[5] = a + 2.0
                k = int(round(a))
                if 1 <= k <= 1 << 20 and abs(a - k) <= 4.0 * np.spacing(a) and not os.environ.get("SIGHTPY_NO_POWI"):
                    r["ival"] = k  # device evaluates x**a as x**k (rt_device.h powi)
            p[6] = 2.0 * np.pi
            p[7] = m.spec_coeff
            p[8:11] = _glossy_f0(scene.n, m.n)  # glossy.py:91 (Python scalars)
            for k, arrs in enumerate(media_arrays):
                glossy_f0[i, k] = _medium_f0(arrs, [m.n.x, m.n.y, m.n.z])
            p[11:14] = glossy_f0[i, 0]  # medium 0 copy, read with scalar loads
        elif isinstance(m, Refractive):
            r["type"] = N.REFRACTIVE
            r["medium"] = medium_of(_c(m.n))
        elif isinstance(m, ThinFilmInterference):
            r["type"] = N.THINFILM
            r["tex_aux0"] = pool.add(m.reflectance_u8, _RAW_LUT)
            r["tex_aux1"] = pool.add(m.noise_u8, _RAW_LUT, repeat=0.5, channel0=0)
            p[0] = m.thickness
            p[1] = m.noise_factor
            if m.noise_factor != 0.0:
                r["flags"] |= N.MF_NOISE
        elif isinstance(m, Diffuse):
            r["type"] = N.DIFFUSE
            if isinstance(m.diff_texture, image):
                r["tex"] = pool.add(m.diff_texture.u8, _LIN_LUT, repeat=m.diff_texture.repeat)
            else:
                p[0:3] = _f3(m.diff_texture.color)
            p[3] = m.ambient_weight
            p[4] = 1.0 - m.ambient_weight
            r["ival"] = m.diffuse_rays
            L.has_diffuse = 1
        elif isinstance(m, Emissive):
            r["type"] = N.EMISSIVE
            if isinstance(m.texture_color, image):
                r["tex"] = pool.add(m.texture_color.u8, _LIN_LUT, repeat=m.texture_color.repeat)
            else:
                p[0:3] = _f3(m.texture_color.color)
        elif isinstance(m, SkyBox_Material):
            r["type"] = N.SKY
            if m.blur != 0.0:
                r["tex"] = pool.add(m.blur_u8, _LIN_LUT, repeat=m.repeat)
            else:
                r["tex"] = pool.add(m.texture_u8, _LIN_LUT, repeat=m.repeat)
            p[0] = m.light_intensity
            if m.light_intensity != 0.0:
                r["flags"] |= N.MF_LIGHTMAP
                r["tex_aux0"] = pool.add(m.lightmap_u8, _RAW_LUT, repeat=m.repeat, idx_shape=m.texture_u8.shape[:2])
        else:
            raise NotImplementedError(
                "material %s has no device kernel (sightpy on MI355X has no CPU fallback)" % type(m).__name__
            )
        r["p"] = p
        mrecs[i] = r

    # ---- colliders --------------------------------------------------------------------------
    shadow_ids = {id(c) for c in scene.shadowed_collider_list}
    crecs = np.zeros(len(colliders), dtype=N.COLLIDER_DTYPE)
    prim_index = {}
    for i, c in enumerate(colliders):
        prim = c.assigned_primitive
        rec = collider_record(c)
        rec["material"] = mat_index[id(prim.material)]
        rec["max_ray_depth"] = int(prim.max_ray_depth)
        flags = 0
        if id(c) in shadow_ids:
            flags |= N.CF_SHADOW
        if getattr(prim, "mc", False):
            flags |= N.CF_MC
        if getattr(prim, "uv_cube_cross", False):
            flags |= N.CF_UV_CROSS
        rec["flags"] = flags
        rec["primitive"] = prim_index.setdefault(id(prim), len(prim_index))
        m = prim.material
        if isinstance(c, Triangle_Collider) and (
            getattr(m, "normalmap_u8", None) is not None
            or isinstance(getattr(m, "diff_texture", None), image)
            or isinstance(m, ThinFilmInterference)
        ):
            raise NotImplementedError("Triangle uv is undefined in the reference (triangle.py:79-83)")
        if getattr(m, "normalmap_u8", None) is not None and isinstance(c, Sphere_Collider):
            raise AttributeError("'Sphere_Collider' object has no attribute 'inverse_basis_matrix'")
        crecs[i] = rec
    L.colliders = crecs
    L.max_ray_depth = int(max([int(c.assigned_primitive.max_ray_depth) for c in colliders], default=0))

    # ---- lights -----------------------------------------------------------------------------
    lrecs = np.zeros(len(scene.Light_list), dtype=N.LIGHT_DTYPE)
    light_local = np.zeros((len(scene.Light_list), len(colliders), 3))
    for i, lt in enumerate(scene.Light_list):
        if isinstance(lt, DirectionalLight):
            lrecs[i]["type"] = N.LIGHT_DIRECTIONAL
            lrecs[i]["dir"] = _f3(lt.Ldir)
            for j, c in enumerate(colliders):
                if isinstance(c, Cuboid_Collider):
                    # shadow rays: D is a scalar vec3, so D.matmul goes through BLAS gemv
                    light_local[i, j] = _f3(lt.Ldir.matmul(c.basis_matrix))
        elif isinstance(lt, PointLight):
            lrecs[i]["type"] = N.LIGHT_POINT
            lrecs[i]["pos"] = _f3(lt.pos)
        else:
            raise NotImplementedError("light type %s" % type(lt).__name__)
        lrecs[i]["color"] = _f3(lt.color)
    L.lights = lrecs
    L.light_local = np.ascontiguousarray(light_local)

    imp = np.zeros((len(scene.importance_sampled_list), 4))
    for i, prim in enumerate(scene.importance_sampled_list):
        imp[i, 0:3] = _f3(prim.center)
        imp[i, 3] = prim.bounded_sphere_radius
    L.importance = imp

    L.materials = mrecs
    L.glossy_f0 = np.ascontiguousarray(glossy_f0)
    med = np.zeros((len(media), 6))
    for k, cv in enumerate(media):
        med[k, 0:3] = [v.real for v in cv]
        med[k, 3:6] = [v.imag for v in cv]
    L.media = med
    L.media_keys = keys
    L.textures, L.texels, L.texel_key = pool.finish()
    L.ambient = tuple(_f3(scene.ambient_color))
    return L
