"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the sightpy ray-trace hot path.

A from-scratch numpy restatement of the reference algorithm (lmondada/Python-Raytracer, the
`sightpy` package; file:line citations below are into that repository).  It is the parity checker
for the HIP kernels: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
it, and never as the thing measured or shipped.

Structure (deliberately the reference's, so that rounding and random-number consumption match):
the whole ray batch is intersected against every collider, the nearest distance is reduced with
np.minimum, rays are compacted per hit collider (np.extract), the material shades the compacted
batch and recurses into `raycolor` for secondary rays, and results are scattered back
(np.place) and summed (ray.py:122-148).  Vectors are planar float64 arrays of shape (3, n);
scene constants are (3, 1) arrays so that broadcasting reproduces the reference's
scalar-vec3-times-array expressions element for element.

Pinned against the reference itself: tests/golden/*.npz were produced by importing the reference
in the build container (tests/golden/gen_golden.py); tests/test_oracle.py checks this module
against them (bit-exact for geometry, <=1e-12 relative for colours), Monte-Carlo scenes included
(single-process seeded renders of the reference are deterministic).

Random numbers.  By default every draw comes from numpy's global RNG in the reference's order
(camera jitter, `mixed_pdf`/`cosine_pdf`/`spherical_caps_pdf` draws, the `mc=True` pick), which is
what pins this module to the reference.  With `rng=DeviceStream(seed)` the Monte-Carlo draws
instead come from the device's counter-based stream -- Philox4x32-10 keyed by (seed, global pixel,
child-path hash, tag), restated here from csrc/rt_device.h and rt_kernels.hip -- so the GPU's
Monte-Carlo paths can be compared with this restatement sample for sample (tests/test_gpu_mc.py).
The algorithm code is the same in both modes; only the source of the uniforms differs.
"""
import numpy as np

FARAWAY = 1.0e39
SKYBOX_DISTANCE = 1.0e6
UPWARDS, UPDOWN = 1, -1


# ---- planar vector helpers (utils/vector3.py) ------------------------------------------------
def col3(v):
    """scene vec3 (scalar components) -> (3, 1) array of its components' numpy dtype."""
    return np.array([[v.x], [v.y], [v.z]])


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def length(v):
    return np.sqrt(dot(v, v))


def normalize(v):  # vector3.py:158-160
    mag = length(v)
    return v * (1.0 / np.where(mag == 0, 1, mag))


def mat_apply(M, v):  # vec3.matmul on array components: np.tensordot -> BLAS (vector3.py:93-97)
    return np.tensordot(M, v, axes=([1, 0]))


def reflect(D, N):  # glossy.py:93, refractive.py:61
    return normalize(D - N * 2.0 * dot(D, N))


def texel(img, u, v, rep, shape=None):
    """img[-(int(v*H*rep) % H), int(u*W*rep) % W] (texture.py:32-39); shape: index arithmetic."""
    h, w = (img.shape[0], img.shape[1]) if shape is None else shape
    return img[-((v * h * rep).astype(int) % h), (u * w * rep).astype(int) % w].T


# ---- the device's counter-based stream (csrc/rt_device.h Rng / philox / mix32) -----------------
_M32 = 0xFFFFFFFF


def mix32(h, v):
    """rt_device.h mix32 on uint32 arrays."""
    h = np.asarray(h).astype(np.uint64)
    v = np.asarray(v).astype(np.uint64)
    h = h ^ ((v + 0x9E3779B9 + ((h << np.uint64(6)) & _M32) + (h >> np.uint64(2))) & _M32)
    h = (h * 0x85EBCA6B) & _M32
    return (h ^ (h >> np.uint64(13))).astype(np.uint32)


def child_path(path, slot, rnd):
    """rt_device.h child_path: the RNG identity of a child ray (slot, tie round)."""
    return mix32(path, (np.asarray(slot).astype(np.uint64) + 4096 * np.asarray(rnd).astype(np.uint64)) & _M32)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al., SC'11), as rt_device.h philox: four uint32 counter words."""
    a, b, c, d = (np.asarray(x).astype(np.uint64) for x in (c0, c1, c2, c3))
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = a * np.uint64(0xD2511F53)
        p1 = c * np.uint64(0xCD9E8D57)
        a, b, c, d = (p1 >> np.uint64(32)) ^ b ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ d ^ k1, p0 & _M32
        k0 = (k0 + np.uint64(0x9E3779B9)) & np.uint64(_M32)
        k1 = (k1 + np.uint64(0xBB67AE85)) & np.uint64(_M32)
    return a, b, c, d


def u01(a, b):
    """numpy's 53-bit double from two 32-bit words (rt_device.h u01)."""
    return ((a >> np.uint64(5)).astype(np.float64) * 67108864.0 + (b >> np.uint64(6)).astype(np.float64)) / 9007199254740992.0


class DeviceStream:
    """The uniforms the GPU draws for its Monte-Carlo shading: Rng.init(seed, pix, path, tag), call n
    returns the pair (u01(r.a, r.b), u01(r.c, r.d)) of philox((pix, path, tag, n), seed)."""

    def __init__(self, seed):
        seed = int(seed) & (2**64 - 1)
        self.k0, self.k1 = seed & _M32, seed >> 32

    def pair(self, pix, path, tag, n):
        size = np.broadcast(np.asarray(pix), np.asarray(path), np.asarray(tag)).shape
        a, b, c, d = philox4x32_10(np.broadcast_to(pix, size), np.broadcast_to(path, size),
                                   np.broadcast_to(tag, size), np.full(size, n), self.k0, self.k1)
        return u01(a, b), u01(c, d)


    def jitter(self, npix, spp, sample_base=0):
        """The camera uniforms of the device-RNG render mode (render jitter NULL; rt_kernels.hip
        primary_uniforms): pixel p, sample s -> pairs 0, 1 of Rng(seed, p, sample_base + s, TAG_RAYGEN)."""
        pix = np.arange(npix, dtype=np.uint32)
        out = np.empty((spp, 4, npix))
        for s in range(spp):
            out[s, 0], out[s, 1] = self.pair(pix, sample_base + s, TAG_RAYGEN, 0)
            out[s, 2], out[s, 3] = self.pair(pix, sample_base + s, TAG_RAYGEN, 1)
        return out


TAG_RAYGEN = 0xCA3E0000
PRIMARY_PATH = 0x5EED0000  # k_primary / k_frame: path of sample s = mix32(PRIMARY_PATH, s)
TRACE_PATH = 0x7A11  # srt_trace: path of batch ray i = mix32(TRACE_PATH, i)
TAG_DIFFUSE, TAG_MC = 0xD1000000, 0x3C000000


class Rays:
    """A batch: origin/dir (3, n), medium index n (3, n) or (3, 1), batch-scalar counters.  With a
    DeviceStream, `pix` (global pixel), `path` (child-path hash) and `rnd` (tie round of the hit
    being shaded) identify each ray's random numbers as on the device; otherwise they are None."""

    def __init__(self, O, D, n, depth, diffuse_reflections=0, pix=None, path=None):
        self.O, self.D, self.n = O, D, n
        self.depth = depth
        self.dfl = diffuse_reflections
        self.pix, self.path, self.rnd = pix, path, None

    def __len__(self):
        return self.O.shape[1]

    def take(self, mask):
        n = self.n if self.n.shape[1] == 1 else self.n[:, mask]
        r = Rays(self.O[:, mask], self.D[:, mask], n, self.depth, self.dfl)
        if self.path is not None:
            r.pix, r.path = self.pix[mask], self.path[mask]
            if self.rnd is not None:
                r.rnd = self.rnd[mask]
        return r

    def child(self, O, D, n, depth, dfl, slot):
        """A child batch of this (shaded) batch: RNG identity child_path(path, slot, round)."""
        r = Rays(O, D, n, depth, dfl)
        if self.path is not None:
            r.pix, r.path = self.pix, child_path(self.path, slot, self.rnd)
        return r


_RNG = {"stream": None}  # DeviceStream while render_linear / trace run in device-stream mode


def place(vals, mask):  # vec3.place (vector3.py:195-200)
    out = np.zeros((3, mask.shape[0]))
    for k in range(3):
        np.place(out[k], mask, vals[k])
    return out


# ---- colliders (sightpy/geometry) ------------------------------------------------------------
def _kind(c):
    return type(c).__name__


def intersect(c, O, D, scalar_D=False):
    """Collider.intersect -> (2, n) [distance; orientation], FARAWAY for misses.
    scalar_D: D is a vec3 of scalars in the reference (shadow rays toward a directional light)."""
    k = _kind(c)
    if k == "Sphere_Collider":  # sphere.py:26-52
        C = col3(c.center)
        b = 2 * dot(D, O - C)
        cc = c.center.square_length() + dot(O, O) - 2 * dot(C, O) - (c.radius * c.radius)
        disc = (b ** 2) - (4 * cc)
        sq = np.sqrt(np.maximum(0, disc))
        h0 = (-b - sq) / 2
        h1 = (-b + sq) / 2
        h = np.where((h0 > 0) & (h0 < h1), h0, h1)
        M = O + D * h
        nd = dot((M - C) * (1.0 / c.radius), D)
        hit = (disc > 0) & (h > 0)
        return np.select([hit & (nd > 0), hit & (nd < 0), True],
                         [[h, np.tile(UPDOWN, h.shape)], [h, np.tile(UPWARDS, h.shape)], FARAWAY])
    if k in ("Plane_Collider", "Triangle_Collider"):  # plane.py:57-90, triangle.py:36-66
        Nn = col3(c.normal)
        nd = dot(Nn, D)
        nd = np.where(nd == 0.0, nd + 0.0001, nd)
        Cc = col3(c.center if k == "Plane_Collider" else c.centroid)
        nco = dot(Nn, Cc - O)
        d = D * nco / nd
        M = O + d
        dis = length(d)
        if k == "Plane_Collider":
            MC = M - Cc
            inside = (np.abs(dot(col3(c.u_axis), MC)) <= c.w) & (np.abs(dot(col3(c.v_axis), MC)) <= c.h) & (nco * nd > 0)
        else:
            inside = ((dot(col3(c.n31), M - col3(c.p1)) >= 0) & (dot(col3(c.n12), M - col3(c.p2)) >= 0)
                      & (dot(col3(c.n23), M - col3(c.p3)) >= 0) & (nco * nd > 0))
        up = nd < 0
        return np.select([inside & up, inside & ~up, True],
                         [[dis, np.tile(UPWARDS, dis.shape)], [dis, np.tile(UPDOWN, dis.shape)], FARAWAY])
    if k == "Cuboid_Collider":  # cuboid.py:105-140
        Ol = mat_apply(c.basis_matrix, O)
        if scalar_D:
            # scalar D (shadow rays): vec3.matmul of scalars goes through np.dot (gemv)
            Dl = np.dot(c.basis_matrix, D[:, 0])[:, None]
        else:
            Dl = mat_apply(c.basis_matrix, D)
        f = 1.0 / Dl
        lb, rt = col3(c.lb_local_basis), col3(c.rt_local_basis)
        t1, t2 = (lb[0] - Ol[0]) * f[0], (rt[0] - Ol[0]) * f[0]
        t3, t4 = (lb[1] - Ol[1]) * f[1], (rt[1] - Ol[1]) * f[1]
        t5, t6 = (lb[2] - Ol[2]) * f[2], (rt[2] - Ol[2]) * f[2]
        tmin = np.maximum(np.maximum(np.minimum(t1, t2), np.minimum(t3, t4)), np.minimum(t5, t6))
        tmax = np.minimum(np.minimum(np.maximum(t1, t2), np.maximum(t3, t4)), np.maximum(t5, t6))
        miss = (tmax < 0) | (tmin > tmax)
        return np.select([miss, tmin < 0, True],
                         [FARAWAY, [tmax, np.tile(UPDOWN, tmin.shape)], [tmin, np.tile(UPWARDS, tmin.shape)]])
    raise TypeError("oracle: unknown collider %s" % k)


def cuboid_normal(c, P):  # cuboid.py:142-151
    L = mat_apply(c.basis_matrix, P - col3(c.center))
    a = np.array([[1.0 / c.width], [1.0 / c.height], [1.0 / c.length]]) * np.abs(L)
    m = np.maximum(np.maximum(a[0], a[1]), a[2])
    s = np.array([np.where(m == a[k], np.sign(L[k]), 0.0) for k in range(3)])
    return mat_apply(c.inverse_basis_matrix, s)


def collider_normal(c, P):
    k = _kind(c)
    if k == "Sphere_Collider":
        return (P - col3(c.center)) * (1.0 / c.radius)
    if k == "Cuboid_Collider":
        return cuboid_normal(c, P)
    return col3(c.normal)


def _cross_coord(ax, MC, width, shift):
    return (dot(ax, MC) / width * 2 * 0.985 + 1) / 2 + shift


def collider_uv(c, P):
    k = _kind(c)
    if k == "Sphere_Collider":  # sphere.py:58-64
        M = (P - col3(c.center)) / c.radius
        return (np.arctan2(M[2], M[0]) + np.pi) / (2 * np.pi), (np.arcsin(M[1]) + np.pi / 2) / np.pi
    if k == "Plane_Collider":  # plane.py:98-102
        MC = P - col3(c.center)
        return ((dot(col3(c.u_axis), MC) / c.w + 1) / 2 + c.uv_shift[0],
                (dot(col3(c.v_axis), MC) / c.h + 1) / 2 + c.uv_shift[1])
    if k == "Cuboid_Collider":  # cuboid.py:153-187
        Nn = cuboid_normal(c, P)
        MC = P - col3(c.center)
        aw, ah, al = col3(c.ax_w), col3(c.ax_h), col3(c.ax_l)
        w = c.width

        def face(x, y, z):
            return (Nn[0] == x) & (Nn[1] == y) & (Nn[2] == z)

        faces = [face(0.0, -1.0, 0.0), face(0.0, 1.0, 0.0), face(1.0, 0.0, 0.0),
                 face(-1.0, 0.0, 0.0), face(0.0, 0.0, 1.0), face(0.0, 0.0, -1.0)]
        u = np.select(faces, [_cross_coord(aw, MC, w, 1), _cross_coord(aw, MC, w, 1), _cross_coord(al, MC, w, 2),
                              _cross_coord(al * -1, MC, w, 0), _cross_coord(aw * -1, MC, w, 3),
                              _cross_coord(aw, MC, w, 1)])
        v = np.select(faces, [_cross_coord(al * -1, MC, w, 0), _cross_coord(al, MC, w, 2), _cross_coord(ah, MC, w, 1),
                              _cross_coord(ah, MC, w, 1), _cross_coord(ah, MC, w, 1), _cross_coord(ah, MC, w, 1)])
        return u, v
    raise TypeError("oracle: uv undefined for %s (triangle.py:79-83)" % k)


def primitive_uv(c, P):  # Primitive.get_uv; Cuboid/SkyBox divide by (4, 3)
    u, v = collider_uv(c, P)
    if type(c.assigned_primitive).__name__ in ("Cuboid", "SkyBox"):
        u, v = u / 4, v / 3
    return u, v


def shading_normal(mat, c, P, orient):  # material.py:18-36
    nm = getattr(mat, "normalmap", None)
    if nm is not None:
        u, v = primitive_uv(c, P)
        im = texel(nm, u, v, mat.repeat)
        Nmap = np.array([im[0] - 0.5, im[1] - 0.5, im[2] - 0.5]) * 2.0
        return normalize(mat_apply(c.inverse_basis_matrix, Nmap)) * orient
    return collider_normal(c, P) * orient


# ---- materials (sightpy/materials, backgrounds) -----------------------------------------------
def _tex_color(tex, c, P):
    if type(tex).__name__ == "solid_color":
        return col3(tex.color)
    u, v = primitive_uv(c, P)
    return texel(tex.img, u, v, tex.repeat)


def shade_glossy(scene, m, c, r, t, orient, counts):  # glossy.py:25-110
    P = r.O + r.D * t
    Nn = shading_normal(m, c, P, orient)
    diff = _tex_color(m.diff_texture, c, P) * m.diff_coeff
    color = col3(scene.ambient_color) * diff
    V = r.D * -1.0
    nudged = P + Nn * 0.000001
    for light in scene.Light_list:
        L = col3(light.Ldir)
        dist = SKYBOX_DISTANCE
        NdotL = np.maximum(dot(Nn, L), 0.0)
        lv = col3(light.color) * NdotL
        H = normalize(L + V)
        if scene.shadowed_collider_list:
            ln = None
            for s in scene.shadowed_collider_list:
                d = intersect(s, nudged, L, scalar_D=True)[0]
                ln = d if ln is None else np.minimum(ln, d)
            seelight = ln >= dist
            counts["shadow"] = counts.get("shadow", 0) + len(r)
        else:
            seelight = 1.0
        color = color + diff * lv * seelight
        if m.roughness != 0.0:
            F0 = np.abs((r.n - col3(m.n)) / (r.n + col3(m.n))) ** 2
            cos_t = np.clip(dot(V, H), 0.0, 1.0)
            F = F0 + (1.0 - F0) * (1.0 - cos_t) ** 5
            a = 2.0 / (m.roughness ** 2.0) - 2.0
            Dp = np.power(np.clip(dot(Nn, H), 0.0, 1.0), a) * (a + 2.0) / (2.0 * np.pi)
            color = color + F * Dp / (4.0 * np.clip(dot(Nn, V) * NdotL, 0.001, 1.0)) * seelight * lv * m.spec_coeff
    if r.depth < c.assigned_primitive.max_ray_depth:
        F0 = np.abs((scene.n - m.n) / (scene.n + m.n)) ** 2  # Python scalar complex arithmetic
        F0 = col3(F0)
        cos_t = np.clip(dot(V, Nn), 0.0, 1.0)
        F = F0 + (1.0 - F0) * (1.0 - cos_t) ** 5
        child = r.child(nudged, reflect(r.D, Nn), r.n, r.depth + 1, r.dfl, 1)
        color = color + raycolor(scene, child, counts) * F
    return color


def shade_refractive(scene, m, c, r, t, orient, counts):  # refractive.py:24-123
    if not r.depth < c.assigned_primitive.max_ray_depth:
        return np.zeros((3, len(r)))
    P = r.O + r.D * t
    Nn = shading_normal(m, c, P, orient)
    V = r.D * -1.0
    nudged = P + Nn * 0.000001
    n1 = np.broadcast_to(r.n, (3, len(r)))
    n2 = np.where(orient == UPWARDS, col3(m.n), col3(scene.n))
    ratio = np.real(n1) / np.real(n2)
    cos_i = dot(V, Nn)
    cos_t = np.sqrt(1.0 - (n1 / n2) ** 2 * (1.0 - cos_i ** 2))
    r_per = (n1 * cos_i - n2 * cos_t) / (n1 * cos_i + n2 * cos_t)
    r_par = -1.0 * (n1 * cos_t - n2 * cos_i) / (n1 * cos_t + n2 * cos_i)
    F = (np.abs(r_per) ** 2 + np.abs(r_par) ** 2) / 2.0
    T = 1.0 - F
    refl = r.child(nudged, reflect(r.D, Nn), n1, r.depth + 1, r.dfl, 1)
    aver = (ratio[0] + ratio[1] + ratio[2]) / 3
    sin2 = aver ** 2 * (1.0 - cos_i ** 2)
    non_tir = sin2 <= 1.0
    Rt = normalize(r.D * aver + Nn * (aver * cos_i - np.sqrt(1 - np.clip(sin2, 0, 1))))
    refr = r.child(P - Nn * 0.000001, Rt, n2, r.depth + 1, r.dfl, 2)
    if c.assigned_primitive.mc:
        if _RNG["stream"] is None:
            u = np.random.rand(len(refl))  # refractive.py:100
        else:
            u = _RNG["stream"].pair(r.pix, r.path, TAG_MC | (r.depth << 8) | r.rnd, 0)[0]
        pick = (u > (F[0] + F[1] + F[2]) / 3) & non_tir
        both = r.child(np.where(pick, refr.O, refl.O), np.where(pick, refr.D, refl.D), np.where(pick, n2, n1),
                       r.depth + 1, r.dfl, 1)
        color = raycolor(scene, both, counts)
    else:
        color = raycolor(scene, refl, counts) * F
        if np.any(non_tir):
            color = color + place(raycolor(scene, refr.take(non_tir), counts), non_tir) * T
    lam = np.array([[630], [550], [475]])
    return color * np.exp(-2.0 * np.imag(n1) * 2.0 * np.pi / lam * 1e9 * t)


def shade_thinfilm(scene, m, c, r, t, orient, counts):  # thin_film_interference.py:24-115
    if not r.depth < c.assigned_primitive.max_ray_depth:
        return np.zeros((3, len(r)))
    P = r.O + r.D * t
    Nn = shading_normal(m, c, P, orient)
    V = r.D * -1.0
    cos_i = dot(V, Nn)
    lut = m.thin_film_interference_reflectance
    if m.noise_factor != 0.0:
        u, v = primitive_uv(c, P)
        thick = m.thickness + m.noise_factor * (texel(m.thickness_noise, u, v, 0.5) - 0.5)
        Fim = lut[(cos_i * lut.shape[0]).astype(int), thick.astype(int)]
    else:
        Fim = lut[(cos_i * lut.shape[0]).astype(int), int(m.thickness)]
    F = np.array([Fim[:, 0], Fim[:, 1], Fim[:, 2]])
    refl = r.child(P + Nn * 0.000001, reflect(r.D, Nn), r.n, r.depth + 1, r.dfl, 1)
    color = (col3(scene.ambient_color) + raycolor(scene, refl, counts)) * F
    trans = r.child(P - Nn * 0.000001, r.D, r.n, r.depth + 1, r.dfl, 2)
    return color + raycolor(scene, trans, counts) * (1.0 - F)


def shade_sky(scene, m, c, r, t):  # skybox.py:51-94
    P = r.O + r.D * t
    u, v = primitive_uv(c, P)
    img = m.blur_image if m.blur != 0.0 else m.texture
    im = texel(img, u, v, m.repeat)
    if r.depth != 0 and m.light_intensity != 0.0:
        ls = texel(m.lightmap, u, v, m.repeat, shape=m.texture.shape[:2])
        return np.array([im[0] + m.light_intensity * ls[0], im[1] + m.light_intensity * ls[1],
                         im[2] + m.light_intensity * ls[2]])
    return np.array([im[0], im[1], im[2]])


# -- Monte-Carlo sampling (utils/random.py:58-174), numpy's global RNG in the reference's order --
def _onb(w):
    a = np.where(np.abs(w[0]) > 0.9, np.array([[0], [1], [0]]), np.array([[1], [0], [0]]))
    cr = lambda p, q: np.array([p[1] * q[2] - p[2] * q[1], -p[0] * q[2] + p[2] * q[0], p[0] * q[1] - p[1] * q[0]])
    v = normalize(cr(w, a))
    return cr(w, v), v


def _cosine_generate(size, Nn, draws=None):
    u, v = _onb(Nn)
    a, r2 = (np.random.rand(size), np.random.rand(size)) if draws is None else draws
    phi = a * 2 * np.pi
    z = np.sqrt(1 - r2)
    return u * (np.cos(phi) * np.sqrt(r2)) + v * (np.sin(phi) * np.sqrt(r2)) + Nn * z


def _caps_generate(size, origin, prims, draws=None):
    nl = len(prims)
    pick_u = np.random.rand(size) if draws is None else draws[0]
    pick = (pick_u * nl).astype(int)
    ws, cmaxs, us, vs = [], [], [], []
    for p in prims:
        tc = col3(p.center) - origin
        w = normalize(tc)
        u, v = _onb(w)
        dist = np.sqrt(dot(tc, tc))
        ws.append(w), us.append(u), vs.append(v)
        cmaxs.append(np.sqrt(1 - np.clip(p.bounded_sphere_radius / dist, 0.0, 1.0) ** 2))
    masks = [pick == i for i in range(nl)]
    a, r2 = (np.random.rand(size), np.random.rand(size)) if draws is None else draws[1:]
    phi = a * 2 * np.pi
    cmax = np.select(masks, cmaxs)
    sel = lambda lst: np.array([np.select(masks, [x[k] for x in lst]) for k in range(3)])
    z = 1.0 + r2 * (cmax - 1.0)
    xy = np.sqrt(1.0 - z ** 2)
    return sel(us) * (np.cos(phi) * xy) + sel(vs) * (np.sin(phi) * xy) + sel(ws) * z, ws, cmaxs


def _caps_value(d, ws, cmaxs):
    val = 0.0
    for w, cm in zip(ws, cmaxs):
        val = val + np.where(dot(d, w) > cm, 1 / ((1 - cm) * 2 * np.pi), 0.0)
    return val / len(ws)


def shade_diffuse(scene, m, c, r, t, orient, counts):  # diffuse.py:25-124
    P = r.O + r.D * t
    Nn = shading_normal(m, c, P, orient)
    diff = _tex_color(m.diff_texture, c, P)
    if r.dfl >= m.max_diffuse_reflections:
        return np.zeros((3, len(r)))
    k = m.diffuse_rays if r.dfl < 1 else 1
    nudged = P + Nn * 0.000001
    Nr, Or = np.repeat(Nn, k, axis=1), np.repeat(nudged, k, axis=1)
    size = Nr.shape[1]
    prims = scene.importance_sampled_list
    stream = _RNG["stream"]
    cos_draws = caps_draws = sel = cpix = cpath = None
    if r.path is not None:
        # child j of ray i: child_path(path_i, 0x100 + j, round_i); Rng calls 0: (mixture select,
        # unused), 1: cosine (phi, r2) or caps (pick, phi), 2: caps r2 (rt_device.h diffuse_child)
        cpix = np.repeat(r.pix, k)
        cpath = child_path(np.repeat(r.path, k), 0x100 + np.tile(np.arange(k), len(r)), np.repeat(r.rnd, k))
    if stream is not None:
        tag = TAG_DIFFUSE | r.depth
        sel = stream.pair(cpix, cpath, tag, 0)[0]
        cos_draws = caps_draws = stream.pair(cpix, cpath, tag, 1)
        caps_draws = caps_draws + (stream.pair(cpix, cpath, tag, 2)[0],)
    if not prims:
        d = _cosine_generate(size, Nr, cos_draws)
        pdf = np.clip(dot(d, Nr), 0.0, 1.0) / np.pi
    else:
        w = m.ambient_weight
        mask = np.random.rand(size) if stream is None else sel
        d1 = _cosine_generate(size, Nr, cos_draws)
        d2, ws, cm = _caps_generate(size, Or, prims, caps_draws)
        d = np.where(mask < w, d1, d2)
        pdf = (np.clip(dot(d, Nr), 0.0, 1.0) / np.pi) * w + _caps_value(d, ws, cm) * (1.0 - w)
    nr = r.n if r.n.shape[1] == 1 else np.repeat(r.n, k, axis=1)
    child = Rays(Or, d, nr, r.depth + 1, r.dfl + 1, cpix, cpath)
    ndl = np.clip(dot(d, Nr), 0.0, 1.0)
    if k == 1 and r.dfl >= 1:  # second bounce (diffuse.py:85-121)
        return diff * raycolor(scene, child, counts) * ndl / pdf / np.pi
    est = raycolor(scene, child, counts) * ndl / pdf / np.pi
    return diff * est.reshape(3, len(r), k).mean(axis=2)


def shade(scene, c, r, t, orient, counts):
    m = c.assigned_primitive.material
    kind = type(m).__name__
    if kind == "Glossy":
        return shade_glossy(scene, m, c, r, t, orient, counts)
    if kind == "Refractive":
        return shade_refractive(scene, m, c, r, t, orient, counts)
    if kind == "ThinFilmInterference":
        return shade_thinfilm(scene, m, c, r, t, orient, counts)
    if kind == "Diffuse":
        return shade_diffuse(scene, m, c, r, t, orient, counts)
    if kind == "Emissive":
        return _tex_color(m.texture_color, c, r.O + r.D * t) * np.ones((1, len(r)))
    if kind == "SkyBox_Material":
        return shade_sky(scene, m, c, r, t)
    raise TypeError("oracle: unknown material %s" % kind)


# ---- the recursion (ray.py:122-148) -----------------------------------------------------------
def nearest(scene, O, D):
    dists = [intersect(c, O, D) for c in scene.collider_list]
    near = dists[0][0]
    for d in dists[1:]:
        near = np.minimum(near, d[0])
    return near, dists


def raycolor(scene, r, counts):
    counts.setdefault("depth", {})
    counts["depth"][r.depth] = counts["depth"].get(r.depth, 0) + len(r)
    near, dists = nearest(scene, r.O, r.D)
    color = np.zeros((3, len(r)))
    # tie round of each (ray, collider) hit: earlier colliders hit at the same distance (the device
    # shades the first one in round 0 and the tied ones in rounds 1, 2, ...)
    rnd = np.zeros(len(r), dtype=np.int64) if r.path is not None else None
    for c, d in zip(scene.collider_list, dists):
        hit = (near != FARAWAY) & (d[0] == near)
        if np.any(hit):
            sub = r.take(hit)
            if rnd is not None:
                sub.rnd = rnd[hit]
            cc = shade(scene, c, sub, d[0][hit], d[1][hit], counts)
            color = color + place(cc, hit)
            if rnd is not None:
                rnd = rnd + hit
    return color


def hit_ids(scene, O, D):
    """Index of the first collider with distance == nearest (-1: miss / NaN)."""
    near, dists = nearest(scene, O, D)
    ids = np.full(O.shape[1], -1, dtype=np.int32)
    for i in range(len(dists) - 1, -1, -1):
        ids = np.where((near != FARAWAY) & (dists[i][0] == near), i, ids)
    return near, ids


# ---- camera and render driver (camera.py:51-85, scene.py:71-140) -----------------------------
def primary_rays(cam, j, rows=None):
    """j: (4, n) uniforms [x-jitter, y-jitter, disk r, disk phi] -> O, D (3, n).  `rows`: only these
    image rows (a row shard of a multi-GPU frame; j holds their pixels, row-major)."""
    W, H = cam.screen_width, cam.screen_height
    xs = np.linspace(-cam.camera_width / 2.0, cam.camera_width / 2.0, W)
    ys = np.linspace(cam.camera_height / 2.0, -cam.camera_height / 2.0, H)
    if rows is not None:
        ys = ys[np.asarray(rows)]
    xx, yy = np.meshgrid(xs, ys)
    x = xx.flatten() + (j[0] - 0.5) * cam.camera_width / W
    y = yy.flatten() + (j[1] - 0.5) * cam.camera_height / H
    rr = np.sqrt(j[2])
    phi = j[3] * 2 * np.pi
    rx, ry = rr * np.cos(phi), rr * np.sin(phi)
    lf, R, U, Fw = col3(cam.look_from), col3(cam.cameraRight), col3(cam.cameraUp), col3(cam.cameraFwd)
    O = lf + R * rx * cam.lens_radius + U * ry * cam.lens_radius
    D = normalize(lf + U * y * cam.focal_distance + R * x * cam.focal_distance + Fw * cam.focal_distance - O)
    return O, D


def scene_medium(scene):
    return np.array([[scene.n.x], [scene.n.y], [scene.n.z]])


def render_linear(scene, jitter, stream=None, sample_base=0, rows=None):
    """Sum over samples of raycolor / spp.  jitter (spp, 4, n).  Returns rgb (3, n), hit ids
    (spp, n) of the primary rays and the per-depth / shadow ray counts.  `stream`: a DeviceStream
    for the Monte-Carlo draws (default: numpy's global RNG, the reference's order).  `rows`: render
    only these image rows (a row shard; jitter holds their pixels), the Monte-Carlo draws keyed by
    global pixel as on the device."""
    spp = jitter.shape[0]
    counts = {}
    acc = 0.0
    ids = []
    _RNG["stream"] = stream
    try:
        for s in range(spp):
            O, D = primary_rays(scene.camera, jitter[s], rows)
            ids.append(hit_ids(scene, O, D)[1])
            r = Rays(O, D, scene_medium(scene), 0, 0)
            if stream is not None:
                n = D.shape[1]
                W = int(scene.camera.screen_width)
                r.pix = (np.arange(n, dtype=np.uint32) if rows is None else
                         (np.asarray(rows, dtype=np.uint32)[:, None] * np.uint32(W) +
                          np.arange(W, dtype=np.uint32)[None, :]).reshape(-1))
                r.path = np.full(n, mix32(PRIMARY_PATH, sample_base + s), dtype=np.uint32)
            acc = acc + raycolor(scene, r, counts)
    finally:
        _RNG["stream"] = None
    return acc / spp, np.array(ids), counts


def trace_linear(scene, O, D, n, depth, dfl=0, stream=None):
    """get_raycolor of one batch (srt_trace), MC draws from `stream` when given (ray i is keyed
    like the device: pixel i, path mix32(TRACE_PATH, i))."""
    r = Rays(O, D, n, depth, dfl)
    counts = {}
    _RNG["stream"] = stream
    try:
        if stream is not None:
            k = D.shape[1]
            r.pix = np.arange(k, dtype=np.uint32)
            r.path = mix32(TRACE_PATH, np.arange(k, dtype=np.uint32))
        return raycolor(scene, r, counts), counts
    finally:
        _RNG["stream"] = None


def shade_linear(scene, ci, O, D, n, depth, t, orient, dfl=0, stream=None):
    """Material.get_color at given hits (srt_shade): ray i shaded by collider ci[i] (-1: nothing)
    at distance t[i], orientation orient[i], as material.get_color(scene, ray.extract(hit_check),
    hit_info) in ray.py:131-146 with the hit supplied by the caller; children traced by raycolor."""
    r = Rays(O, D, n, depth, dfl)
    counts = {}
    _RNG["stream"] = stream
    try:
        k = D.shape[1]
        if stream is not None:
            r.pix = np.arange(k, dtype=np.uint32)
            r.path = mix32(TRACE_PATH, np.arange(k, dtype=np.uint32))
        color = np.zeros((3, k))
        for i, c in enumerate(scene.collider_list):
            hit = ci == i
            if np.any(hit):
                sub = r.take(hit)
                if stream is not None:
                    sub.rnd = np.zeros(int(hit.sum()), dtype=np.int64)
                color = color + place(shade(scene, c, sub, t[hit], orient[hit], counts), hit)
        return color, counts
    finally:
        _RNG["stream"] = None


def srgb_u8(rgb_lin, H, W):  # colour_functions.py:4-18 + scene.py:125-140
    rgb = np.where(rgb_lin <= 0.00304, 12.92 * rgb_lin, 1.055 * np.power(rgb_lin, 1.0 / 2.4) - 0.055)
    peak = np.amax(rgb, axis=0) + 0.00001
    rgb = np.where(peak > 1.0, rgb * 1.0 / peak, rgb)
    return np.stack([(255 * np.clip(c, 0, 1).reshape((H, W))).astype(np.uint8) for c in rgb], axis=-1)
