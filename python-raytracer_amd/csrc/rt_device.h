// rt_device.h -- per-ray math of the sightpy hot path, shared by the gfx950 kernels
// (rt_kernels.hip) and the sequential host check harness (rt_hostcheck.cpp, tests only).
//
// Every function restates a numpy expression of the reference (lmondada/Python-Raytracer,
// cited file:line) for ONE ray, in the reference's evaluation order: numpy evaluates
// `a + b + c` as ((a+b)+c) and `x * y / z` as ((x*y)/z), vec3.dot is ((x*x'+y*y')+z*z'),
// and vec3.matmul goes through OpenBLAS dgemm, i.e. fma(B[i][2], z, fma(B[i][1], y, B[i][0]*x)).
// The file must be compiled with -ffp-contract=off so that only the explicit fma() calls fuse.
// With that, + - * / sqrt are IEEE-exact on both sides, so intersections, normals, directions
// and texel indices match the numpy reference bit for bit; transcendental functions (pow, exp,
// atan2, asin, sin, cos, hypot) differ from numpy's SIMD versions by ~1 ulp.
#pragma once

#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <utility>

#include "../../include/sightpy_rt.h"

// Scene tables are read-only while a kernel runs.  In the device compilation they are addressed
// through the constant address space so that wave-uniform reads (the collider loop, the
// per-material waterfall) become scalar loads into SGPRs instead of per-lane loads into VGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_RO __attribute__((address_space(4)))
#define RT_LDS __attribute__((address_space(3)))
#else
#define RT_RO
#define RT_LDS
#endif

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#define RT_HDM __host__ __device__ __forceinline__
// out of line on the device: code on rare paths that would otherwise be inlined at every call site
// (instruction-cache footprint of the trace kernels) and hold registers in every kernel that calls it
#define RT_OOL __host__ __device__ __attribute__((noinline))
#else
#define RT_HD static inline
#define RT_HDM inline
#define RT_OOL static inline
#endif

// Diagnostic build only (-DRT_PROF): wave-time per code section, sampled on 1/16 of the blocks,
// read back with srt_debug_prof (tools/prof_sections.py).  Compiles to nothing otherwise.
#if defined(RT_PROF) && defined(__HIPCC__)
__device__ unsigned long long g_rt_prof[64];
#endif
#if defined(RT_PROF) && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint64_t rt_clock() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void rt_prof_add(int k, uint64_t dt) {
    if ((blockIdx.x & 15) != 0) return;
    const uint64_t m = __ballot(1);
    if ((uint64_t)__lane_id() == (uint64_t)__builtin_ctzll(m)) {
        atomicAdd(&g_rt_prof[k], (unsigned long long)dt);
        atomicAdd(&g_rt_prof[32 + k], 1ull);
    }
}
#define RT_T0(v) const uint64_t v = rt_clock()
#define RT_ACC(k, v) rt_prof_add(k, rt_clock() - v)
#else
#define RT_T0(v)
#define RT_ACC(k, v)
#endif

namespace rt {

// constants (reference utils/constants.py:1-4)
constexpr double FARAWAY = 1.0e39;
constexpr double SKYBOX_DISTANCE = 1.0e6;
constexpr double PI = 3.141592653589793;      // np.pi
constexpr double TWO_PI = 6.283185307179586;  // 2 * np.pi
constexpr double HALF_PI = 1.5707963267948966;  // np.pi / 2
constexpr double NUDGE = 0.000001;              // glossy.py:35 etc.

// error bits raised by a kernel (folded into SRT_ERR_* by the host)
constexpr uint32_t ERR_INDEX = 1u;      // texture/table index outside the array (IndexError)
constexpr uint32_t ERR_UNSUPPORTED = 2u;  // uv of a Triangle (undefined in the reference)
constexpr uint32_t ERR_NAME = 4u;         // a PointLight met by a Glossy hit (NameError in the reference)

// Feature masks of the kernel variants: a kernel instantiated for MATS contains only these shading
// paths and scene features (the host picks the first variant covering the scene).
constexpr uint32_t MAT_ALL = 0x3Fu;   // every material type (1 << SRT_GLOSSY .. 1 << SRT_SKY)
constexpr uint32_t MAT_BVH = 0x40u;   // a triangle BVH (the traversal code)
constexpr uint32_t MAT_TRI = 0x80u;   // Triangle colliders intersected one by one (collider loops, tie re-tests)
constexpr uint32_t MAT_NMAP = 0x100u; // a normal-mapped material (shading_normal's texel path)
constexpr uint32_t MAT_LDS_STACK = 0x200u;   // the BVH traversal stack's first entries in LDS (256-thread blocks)
constexpr uint32_t MAT_LDS_NARROW = 0x400u;  // ... in k_frame's 64-thread blocks (half as many entries)
constexpr uint32_t MAT_GENERIC = MAT_ALL | MAT_TRI | MAT_NMAP;
constexpr uint32_t mat_bit(int type) { return 1u << type; }
// Collider sequence known at compile time (bits 12..31 of a variant's feature mask, 0: the scene's
// collider list read at run time): bits 0..3 of the sequence hold the count n (1..8), then 2 bits per
// collider its type (SRT_SPHERE .. SRT_TRIANGLE), collider 0 first.  A kernel instantiated for a
// sequence intersects the colliders in straight-line code (no loop, no type switch: the compiler
// shares common subexpressions between colliders and interleaves their independent arithmetic); the
// host runs it only on scenes whose colliders have exactly those types in that order.
constexpr int SEQ_SHIFT = 12;
constexpr int SEQ_MAX = 8;
constexpr uint32_t seq_of(uint32_t feat) { return feat >> SEQ_SHIFT; }
constexpr int seq_count(uint32_t q) { return (int)(q & 15u); }
constexpr int seq_type(uint32_t q, int k) { return (int)((q >> (4 + 2 * k)) & 3u); }
// the sequence code of n collider types (n <= SEQ_MAX), 0 if it cannot be encoded
RT_HD uint32_t seq_encode(const int* types, int n) {
    if (n < 1 || n > SEQ_MAX) return 0u;
    uint32_t q = (uint32_t)n;
    for (int k = 0; k < n; ++k) {
        if (types[k] < 0 || types[k] > 3) return 0u;
        q |= (uint32_t)types[k] << (4 + 2 * k);
    }
    return q;
}

struct d3 {
    double x, y, z;
};

RT_HD d3 mk(double x, double y, double z) { return d3{x, y, z}; }
template <class P>
RT_HD d3 ld3(P p) { return d3{p[0], p[1], p[2]}; }
RT_HD d3 add(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD d3 sub(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD d3 mul(d3 a, d3 b) { return d3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD d3 mul(d3 a, double s) { return d3{a.x * s, a.y * s, a.z * s}; }
RT_HD d3 rsub(double s, d3 a) { return d3{s - a.x, s - a.y, s - a.z}; }
RT_HD d3 divs(d3 a, double s) { return d3{a.x / s, a.y / s, a.z / s}; }
RT_HD double dot(d3 a, d3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_HD bool is_zero(d3 a) { return a.x == 0.0 && a.y == 0.0 && a.z == 0.0; }

// Several quotients a_i / b with one divisor.  On the GPU a float64 division is an 11-instruction
// sequence (div_scale x2, rcp, two Newton steps, q = a*y, r = fma(-b, q, a), div_fmas, div_fixup);
// for operands in the normal range div_scale/div_fmas/div_fixup change nothing, so the refined
// reciprocal y can be computed once and each further quotient costs q = a*y, r = fma(-b, q, a),
// q' = fma(r, y, q) -- the same instructions, hence bit-identical (correctly rounded, as numpy).
// Divisors outside [1e-100, 1e100] (or NaN/inf/0) take the plain division.  Numerators must be
// finite and below 1e100 in magnitude (true at every call site: geometry within FARAWAY = 1e39).
struct Quot {
    double b, y;
    bool fast;
    RT_HDM explicit Quot(double den) : b(den), y(0.0), fast(false) {
#if defined(__HIP_DEVICE_COMPILE__)
        const double ab = fabs(den);
        fast = ab > 1e-100 && ab < 1e100;
        if (fast) {
            double r = __builtin_amdgcn_rcp(den);
            r = fma(r, fma(-den, r, 1.0), r);
            y = fma(r, fma(-den, r, 1.0), r);
        }
#endif
    }
    RT_HDM double operator()(double a) const {
#if defined(__HIP_DEVICE_COMPILE__)
        if (fast) {
            const double q = a * y;
            return fma(fma(-b, q, a), y, q);
        }
#endif
        return a / b;
    }
};

// vec3.normalize (vector3.py:158-160): v * (1.0 / where(|v| == 0, 1, |v|))
RT_HD d3 normalize(d3 v) {
    double mag = sqrt(dot(v, v));
    double inv = 1.0 / (mag == 0.0 ? 1.0 : mag);
    return mul(v, inv);
}

// vec3.matmul on arrays = np.tensordot(B, v) -> OpenBLAS dgemm: one fma chain per row
// (vector3.py:93-97; order verified bit-exact against OpenBLAS 0.3.29)
template <class P>
RT_HD d3 matmul_rows(P B, d3 v) {
    return d3{fma(B[2], v.z, fma(B[1], v.y, B[0] * v.x)),
              fma(B[5], v.z, fma(B[4], v.y, B[3] * v.x)),
              fma(B[8], v.z, fma(B[7], v.y, B[6] * v.x))};
}

// np.minimum / np.maximum: NaN-propagating, first operand wins on NaN
RT_HD double np_min(double a, double b) { return (a < b || a != a) ? a : b; }
RT_HD double np_max(double a, double b) { return (a > b || a != a) ? a : b; }
RT_HD double np_clip(double x, double lo, double hi) { return np_min(np_max(x, lo), hi); }
// np.sign
RT_HD double np_sign(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x)); }

// ndarray.astype(int) of float64: truncation; out-of-range / NaN give INT64_MIN (x86 cvttsd2si)
// (fast path: one v_cvt_i32_f64 when the value fits 32 bits, which texel indices always do)
RT_HD int64_t np_trunc(double x) {
    if (x > -2147483648.0 && x < 2147483648.0) return (int64_t)(int32_t)x;
    return (x > -9.2e18 && x < 9.2e18) ? (int64_t)x : (int64_t)(-9223372036854775807LL - 1);
}
// Python/numpy integer floor-mod (result has the sign of m); 64-bit division is emulated on the
// GPU, so in-range and 32-bit operands take cheaper paths with identical results
RT_OOL int64_t py_mod_wide(int64_t a, int64_t m) {  // emulated 64-bit division: ~150 instructions
    int64_t r = a % m;
    return (r != 0 && (r < 0) != (m < 0)) ? r + m : r;
}
RT_HD int64_t py_mod(int64_t a, int64_t m) {
    if (a >= 0 && a < m) return a;
    if (a >= 0 && a <= 0x7FFFFFFFLL && m > 0 && m <= 0x7FFFFFFFLL) return (int64_t)((uint32_t)a % (uint32_t)m);
    return py_mod_wide(a, m);
}

// ---- complex128 (numpy semantics) ---------------------------------------------------------
struct cplx {
    double re, im;
};
RT_HD cplx cadd(cplx a, cplx b) { return cplx{a.re + b.re, a.im + b.im}; }
RT_HD cplx csub(cplx a, cplx b) { return cplx{a.re - b.re, a.im - b.im}; }
RT_HD cplx cmul(cplx a, cplx b) { return cplx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
// complex * real array (numpy promotes the real operand to (x, 0))
RT_HD cplx cmulr(cplx a, double x) { return cplx{a.re * x - a.im * 0.0, a.re * 0.0 + a.im * x}; }
// numpy complex division (Smith's algorithm, umath loops)
RT_HD cplx cdiv(cplx a, cplx b) {
    double abr = fabs(b.re), abi = fabs(b.im);
    if (abr >= abi) {
        if (abr == 0.0 && abi == 0.0) return cplx{a.re / abr, a.im / abr};
        double rat = b.im / b.re;
        double scl = 1.0 / (b.re + b.im * rat);
        return cplx{(a.re + a.im * rat) * scl, (a.im - a.re * rat) * scl};
    }
    double rat = b.re / b.im;
    double scl = 1.0 / (b.im + b.re * rat);
    return cplx{(a.re * rat + a.im) * scl, (a.im * rat - a.re) * scl};
}
RT_HD double cabs(cplx a) { return hypot(a.re, a.im); }
// principal square root (glibc csqrt arrangement)
RT_HD cplx csqrt_np(cplx z) {
    double x = z.re, y = z.im;
    if (x == 0.0 && y == 0.0) return cplx{0.0, y};
    double d = hypot(x, y);
    double r, s;
    if (x > 0.0) {
        r = sqrt(0.5 * (d + x));
        s = 0.5 * (y / r);
    } else {
        s = sqrt(0.5 * (d - x));
        r = fabs(0.5 * (y / s));
    }
    return cplx{r, copysign(s, y)};
}

// ---- scene view ---------------------------------------------------------------------------
struct SceneView {
    const RT_RO srt_collider* col;
    const RT_RO srt_material* mat;
    const RT_RO srt_texture* tex;
    const RT_RO uint8_t* texels;
    const RT_RO srt_light* lights;
    const RT_RO double* media;
    const RT_RO double* glossy_f0;
    const RT_RO double* light_local;
    const RT_RO double* importance;
    int ncol, nmat, ntex, nlights, nmedia, nimp;
    int nshadow;  // colliders flagged SRT_CF_SHADOW
    double ambient[3];
    // texture lookup tables staged in LDS by the kernel (textures [0, nlut_lds)); the host
    // harness leaves nlut_lds = 0 and reads the tables from the texture records.  An LDS pointer
    // is 32-bit in device code and 64-bit on the host; the union keeps the struct (a kernel
    // argument built by the host) the same layout on both sides.
    union {
        const RT_LDS double* lut_lds;
        uint64_t lut_lds_bits_;
    };
    int nlut_lds;
    // Triangle colliders of large meshes live in a BVH (rt_bvh.h); `lin` lists the colliders
    // intersected one by one (ascending; every collider when there is no BVH)
    int nlin;
    const RT_RO int32_t* lin;
    const RT_RO struct BvhNode* bvh;
    const RT_RO int32_t* bvh_tri;  // collider index of each BVH leaf slot
    int bvh_nodes;                 // 0: no BVH
    int sky_col;                   // the one collider shaded by a SkyBox / Panorama material, else -1
    float bvh_bound;               // max |coordinate| of the BVH's boxes (the f32 box test's error bound)
    int32_t pad_;
};
// the host builds SceneView/TraceParams and the device reads them: the layout must agree
static_assert(sizeof(SceneView) == 184 && offsetof(SceneView, nlut_lds) == 136, "SceneView layout");

// BVH node, 4-wide (128 B: one traversal step loads one cache line and tests four boxes): child k's
// box [lo[.][k], hi[.][k]] in float, rounded outward from the build's f64 boxes (which are inflated so
// that rounding never excludes a triangle's hit point), tested by the widened f32 slab test
// (box4f_hit), which is conservative against the exact test on these bounds; child[k] >= 0: inner node; child[k] < 0 (and != BVH_EMPTY): leaf of the triangles
// bvh_tri[-child[k] - 1, .. + count[k]); BVH_EMPTY: no child in slot k
struct BvhNode {
    float lo[3][4], hi[3][4];
    int32_t child[4];
    int32_t count[4];
};
static_assert(sizeof(BvhNode) == 128, "one 128-byte line per BVH node");
constexpr int32_t BVH_EMPTY = (int32_t)0x80000000;
constexpr int BVH_STACK = 32;  // (3 entries per 4-wide level at most: depth <= 10 levels)
#ifndef RT_BVH_LDS
#define RT_BVH_LDS 16  // (-DRT_BVH_LDS=2: a check build whose stacks overflow into the private part)
#endif
constexpr int BVH_LDS = RT_BVH_LDS;  // (MAT_LDS_STACK) entries of a thread's stack kept in LDS, the rest private

// The kernel's dynamic LDS: the texture tables [0, nlut_lds) staged by the trace kernels first
// (rt_kernels.hip stage_luts), read directly (no pointer in the scene view, so the kernels' scene view
// needs no per-block copy of their arguments)
#if defined(__HIPCC__)
extern __shared__ double rt_lds_dyn[];
#endif

// lut[b] of texture `tid` (LDS copy when staged)
RT_HD double tex_lut(const SceneView& S, int tid, uint8_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (tid < S.nlut_lds) return rt_lds_dyn[tid * 256 + b];
#endif
    return S.tex[tid].lut[b];
}

// ---- ray/primitive intersection (returns distance; orientation through `o`) -----------------
// sphere.py:26-52
RT_HD double sphere_hit(const RT_RO double* p, d3 O, d3 D, double& o) {
    d3 C = ld3(p);
    double b = 2.0 * dot(D, sub(O, C));
    double c = ((p[5] + dot(O, O)) - 2.0 * dot(C, O)) - p[6];
    double disc = b * b - 4.0 * c;
    // disc <= 0 (or NaN) misses whatever h is (ok below needs disc > 0): skip the rest
    if (!(disc > 0.0)) { o = FARAWAY; return FARAWAY; }
    double sq = sqrt(np_max(0.0, disc));
    double h0 = (-b - sq) / 2.0;
    double h1 = (-b + sq) / 2.0;
    double h = (h0 > 0.0 && h0 < h1) ? h0 : h1;
    d3 M = add(O, mul(D, h));
    double nd = dot(mul(sub(M, C), p[4]), D);
    bool ok = disc > 0.0 && h > 0.0;
    if (ok && nd > 0.0) { o = -1.0; return h; }
    if (ok && nd < 0.0) { o = 1.0; return h; }
    o = FARAWAY;
    return FARAWAY;
}

// plane.py:57-90 (rectangle: |u| <= w, |v| <= h in the plane basis)
RT_HD double plane_hit(const RT_RO double* p, d3 O, d3 D, double& o) {
    d3 N = ld3(p + 3);
    double nd = dot(N, D);
    nd = (nd == 0.0) ? nd + 0.0001 : nd;
    double nco = dot(N, sub(ld3(p), O));
    // the hit needs nco * nd > 0 (same product as below; NaN fails too): skip the rest otherwise
    if (!(nco * nd > 0.0)) { o = FARAWAY; return FARAWAY; }
    const Quot q(nd);
    d3 d = d3{q(D.x * nco), q(D.y * nco), q(D.z * nco)};
    d3 M = add(O, d);
    double dis = sqrt(dot(d, d));
    d3 MC = sub(M, ld3(p));
    double u = dot(ld3(p + 6), MC);
    double v = dot(ld3(p + 9), MC);
    if (fabs(u) <= p[12] && fabs(v) <= p[13] && nco * nd > 0.0) {
        o = (nd < 0.0) ? 1.0 : -1.0;
        return dis;
    }
    o = FARAWAY;
    return FARAWAY;
}

// cuboid.py:105-140 (slab test in the local basis).  `Dl` is D.matmul(basis); it is passed in
// because for shadow rays D is a scalar vec3 whose matmul goes through BLAS gemv on the host.
// p[42] != 0: the basis is exactly the identity (every SkyBox, unrotated cuboids).  The fma chain
// then returns its input except for the sign of a zero component, which changes no result here
// (|.| and np.sign ignore it; an axis-parallel slab gives t = +-inf pairs that either miss on
// both signs or span (-inf, inf) and drop out of the min/max), so the matmuls are skipped.
RT_HD double cuboid_hit_local(const RT_RO double* p, d3 O, d3 Dl, double& o) {
    d3 Ol = (p[42] != 0.0) ? O : matmul_rows(p + 3, O);
    d3 f = d3{1.0 / Dl.x, 1.0 / Dl.y, 1.0 / Dl.z};
    double t1 = (p[12] - Ol.x) * f.x, t2 = (p[15] - Ol.x) * f.x;
    double t3 = (p[13] - Ol.y) * f.y, t4 = (p[16] - Ol.y) * f.y;
    double t5 = (p[14] - Ol.z) * f.z, t6 = (p[17] - Ol.z) * f.z;
    double tmin = np_max(np_max(np_min(t1, t2), np_min(t3, t4)), np_min(t5, t6));
    double tmax = np_min(np_min(np_max(t1, t2), np_max(t3, t4)), np_max(t5, t6));
    if (tmax < 0.0 || tmin > tmax) { o = FARAWAY; return FARAWAY; }
    if (tmin < 0.0) { o = -1.0; return tmax; }
    o = 1.0;
    return tmin;
}
RT_HD double cuboid_hit(const RT_RO double* p, d3 O, d3 D, double& o) {
    return cuboid_hit_local(p, O, (p[42] != 0.0) ? D : matmul_rows(p + 3, D), o);
}

// triangle.py:36-66 (plane through the centroid + edge half-spaces)
RT_HD double triangle_hit(const RT_RO double* p, d3 O, d3 D, double& o) {
    d3 N = ld3(p + 3);
    double nd = dot(N, D);
    nd = (nd == 0.0) ? nd + 0.0001 : nd;
    double nco = dot(N, sub(ld3(p), O));
    if (!(nco * nd > 0.0)) { o = FARAWAY; return FARAWAY; }  // as plane_hit
    const Quot q(nd);
    d3 d = d3{q(D.x * nco), q(D.y * nco), q(D.z * nco)};
    d3 M = add(O, d);
    double dis = sqrt(dot(d, d));
    bool inside = dot(ld3(p + 15), sub(M, ld3(p + 6))) >= 0.0 &&
                  dot(ld3(p + 18), sub(M, ld3(p + 9))) >= 0.0 &&
                  dot(ld3(p + 21), sub(M, ld3(p + 12))) >= 0.0 && nco * nd > 0.0;
    if (inside) {
        o = (nd < 0.0) ? 1.0 : -1.0;
        return dis;
    }
    o = FARAWAY;
    return FARAWAY;
}

template <uint32_t FEAT = MAT_GENERIC>
RT_HD double collider_hit(const RT_RO srt_collider& c, d3 O, d3 D, double& o) {
    switch (c.type) {
        case SRT_SPHERE: return sphere_hit(c.p, O, D, o);
        case SRT_PLANE: return plane_hit(c.p, O, D, o);
        case SRT_CUBOID: return cuboid_hit(c.p, O, D, o);
        default:
            if (FEAT & MAT_TRI) return triangle_hit(c.p, O, D, o);
            o = FARAWAY;  // (a variant without MAT_TRI is never picked for a scene with triangles)
            return FARAWAY;
    }
}

// Large libm routines called only on rare paths (the Glossy lobe's non-integer power, sphere uv, the
// resolve's sRGB power) are kept out of line: inlined, their temporaries set the register
// allocation of every shading kernel (k_primary<33> at 3 waves/SIMD: 127 VGPRs spilled inlined,
// none out of line); the call returns the same value as the inlined routine
RT_OOL double pow_ool(double x, double y) { return pow(x, y); }
RT_OOL double atan2_ool(double y, double x) { return atan2(y, x); }
RT_OOL double asin_ool(double x) { return asin(x); }

// ---- normals and uv (per collider) ---------------------------------------------------------
// cuboid.py:142-151: face normal picked by the largest scaled |local coordinate|
RT_HD d3 cuboid_normal(const RT_RO double* p, d3 P) {
    const bool axis = p[42] != 0.0;
    d3 L = axis ? sub(P, ld3(p)) : matmul_rows(p + 3, sub(P, ld3(p)));
    double ax = p[39] * fabs(L.x), ay = p[40] * fabs(L.y), az = p[41] * fabs(L.z);
    double m = np_max(np_max(ax, ay), az);
    d3 s = d3{m == ax ? np_sign(L.x) : 0.0, m == ay ? np_sign(L.y) : 0.0, m == az ? np_sign(L.z) : 0.0};
    return axis ? s : matmul_rows(p + 30, s);
}

// un-oriented collider normal at P (Collider.get_Normal)
RT_HD d3 collider_normal(const RT_RO srt_collider& c, d3 P) {
    switch (c.type) {
        case SRT_SPHERE: return mul(sub(P, ld3(c.p)), c.p[4]);  // sphere.py:54-56
        case SRT_PLANE: return ld3(c.p + 3);                       // plane.py:104-105
        case SRT_CUBOID: return cuboid_normal(c.p, P);
        default: return ld3(c.p + 3);                              // triangle.py:85-86
    }
}

// cuboid.py:153-187: 4x3 cube-cross coordinates; every face divides by `width`
RT_HD double cross_coord(d3 ax, double sgn, d3 MC, const Quot& width, double shift) {
    d3 a = d3{ax.x * sgn, ax.y * sgn, ax.z * sgn};
    return (((width(dot(a, MC)) * 2.0) * 0.985 + 1.0) / 2.0) + shift;
}
RT_HD void cuboid_uv(const RT_RO double* p, d3 P, double& u, double& v) {
    d3 N = cuboid_normal(p, P);
    d3 MC = sub(P, ld3(p));
    d3 aw = ld3(p + 18), ah = ld3(p + 21), al = ld3(p + 24);
    const Quot w(p[27]);  // both coordinates divide by the width
    if (N.x == 0.0 && N.y == -1.0 && N.z == 0.0) {  // BOTTOM
        u = cross_coord(aw, 1.0, MC, w, 1.0); v = cross_coord(al, -1.0, MC, w, 0.0);
    } else if (N.x == 0.0 && N.y == 1.0 && N.z == 0.0) {  // TOP
        u = cross_coord(aw, 1.0, MC, w, 1.0); v = cross_coord(al, 1.0, MC, w, 2.0);
    } else if (N.x == 1.0 && N.y == 0.0 && N.z == 0.0) {  // RIGHT
        u = cross_coord(al, 1.0, MC, w, 2.0); v = cross_coord(ah, 1.0, MC, w, 1.0);
    } else if (N.x == -1.0 && N.y == 0.0 && N.z == 0.0) {  // LEFT
        u = cross_coord(al, -1.0, MC, w, 0.0); v = cross_coord(ah, 1.0, MC, w, 1.0);
    } else if (N.x == 0.0 && N.y == 0.0 && N.z == 1.0) {  // FRONT
        u = cross_coord(aw, -1.0, MC, w, 3.0); v = cross_coord(ah, 1.0, MC, w, 1.0);
    } else if (N.x == 0.0 && N.y == 0.0 && N.z == -1.0) {  // BACK
        u = cross_coord(aw, 1.0, MC, w, 1.0); v = cross_coord(ah, 1.0, MC, w, 1.0);
    } else {  // np.select default
        u = 0.0; v = 0.0;
    }
}

// Primitive.get_uv(hit) for the collider's primitive; returns false for the undefined Triangle uv
RT_HD bool collider_uv(const RT_RO srt_collider& c, d3 P, double& u, double& v) {
    switch (c.type) {
        case SRT_SPHERE: {  // sphere.py:58-64
            d3 M = divs(sub(P, ld3(c.p)), c.p[3]);
            u = (atan2_ool(M.z, M.x) + PI) / TWO_PI;
            v = (asin_ool(M.y) + HALF_PI) / PI;
            break;
        }
        case SRT_PLANE: {  // plane.py:98-102
            d3 MC = sub(P, ld3(c.p));
            u = (dot(ld3(c.p + 6), MC) / c.p[12] + 1.0) / 2.0 + c.p[14];
            v = (dot(ld3(c.p + 9), MC) / c.p[13] + 1.0) / 2.0 + c.p[15];
            break;
        }
        case SRT_CUBOID: cuboid_uv(c.p, P, u, v); break;
        default: u = 0.0; v = 0.0; return false;
    }
    if (c.flags & SRT_CF_UV_CROSS) {  // cuboid.py:29-32, skybox.py:29-32
        u = u / 4.0;  // exact: a multiplication by 0.25
        v = Quot(3.0)(v);
    }
    return true;
}

// ---- textures -------------------------------------------------------------------------------
// numpy fancy-index semantics for one axis: -n <= i < n, negative wraps
RT_HD int64_t np_index(int64_t i, int64_t n, uint32_t& err) {
    if (i < 0) i += n;
    if (i < 0 || i >= n) {
        err |= ERR_INDEX;
        i = i < 0 ? 0 : n - 1;
    }
    return i;
}
RT_HD const RT_RO uint8_t* texel_at(const SceneView& S, const RT_RO srt_texture& T, int64_t row, int64_t col, uint32_t& err) {
    row = np_index(row, T.height, err);
    col = np_index(col, T.width, err);
    return S.texels + T.offset + (row * (int64_t)T.width + col) * T.channels + T.channel0;
}
// img[-(int(v*H*rep) % H), int(u*W*rep) % W] (texture.py:32-39, skybox.py:54-86)
RT_HD const RT_RO uint8_t* tex_uv(const SceneView& S, const RT_RO srt_texture& T, double u, double v, uint32_t& err) {
    int64_t m = py_mod(np_trunc((v * (double)T.idx_h) * T.repeat), T.idx_h);
    int64_t col = py_mod(np_trunc((u * (double)T.idx_w) * T.repeat), T.idx_w);
    return texel_at(S, T, -m, col, err);
}
// The three bytes of a texel through the texture's table.  A 4-byte texel read from its first byte
// (RGBX: srt_upload_scene stores 3-channel images that way, and RGBA images are) is one aligned
// dword load instead of three byte loads; other layouts read the bytes.
// A texture whose texels can be read as one dword each: 4 channels from the first, and the image
// 4-byte aligned in the pool (srt_upload_scene pads the RGBX pool so; a caller's own pool or offsets
// may not be).  Wave-uniform: scalar operations on the texture record.
RT_HD bool texel_dword(const SceneView& S, const RT_RO srt_texture& T) {
    return T.channels == 4 && T.channel0 == 0 && (((uintptr_t)S.texels + (uint64_t)T.offset) & 3u) == 0;
}
RT_HD d3 texel_rgb(const SceneView& S, const RT_RO srt_texture& T, int tid, const RT_RO uint8_t* px) {
    uint32_t b0, b1, b2;
    if (texel_dword(S, T)) {
        const uint32_t w = *reinterpret_cast<const RT_RO uint32_t*>(px);
        b0 = w & 0xFFu;
        b1 = (w >> 8) & 0xFFu;
        b2 = (w >> 16) & 0xFFu;
    } else {
        b0 = px[0];
        b1 = px[1];
        b2 = px[2];
    }
    return d3{tex_lut(S, tid, (uint8_t)b0), tex_lut(S, tid, (uint8_t)b1), tex_lut(S, tid, (uint8_t)b2)};
}
RT_HD d3 tex_rgb(const SceneView& S, int tid, double u, double v, uint32_t& err) {
    const RT_RO srt_texture& T = S.tex[tid];
#ifdef RT_ABL_TEX  // diagnostic build only: no gathers
    return d3{u * T.repeat, v, u + v};
#endif
    return texel_rgb(S, T, tid, tex_uv(S, T, u, v, err));
}

// A texel's 4 bytes as one word (texel_rgb's layouts): one dword load for RGBX / RGBA texels
RT_HD uint32_t texel_word(const SceneView& S, const RT_RO srt_texture& T, const RT_RO uint8_t* px) {
    if (texel_dword(S, T)) return *reinterpret_cast<const RT_RO uint32_t*>(px);
    return (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
}
RT_HD d3 word_rgb(const SceneView& S, int tid, uint32_t w) {
    return d3{tex_lut(S, tid, (uint8_t)(w & 0xFFu)), tex_lut(S, tid, (uint8_t)((w >> 8) & 0xFFu)),
              tex_lut(S, tid, (uint8_t)((w >> 16) & 0xFFu))};
}

// Material.get_Normal (material.py:18-36): collider normal (or normal map) times orientation
template <uint32_t FEAT = MAT_GENERIC>
RT_HD d3 shading_normal(const SceneView& S, const RT_RO srt_collider& c, const RT_RO srt_material& m, d3 P,
                        double orient, uint32_t& err) {
    if ((FEAT & MAT_NMAP) && m.normalmap >= 0) {
        double u, v;
        if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
        const RT_RO srt_texture& T = S.tex[m.normalmap];
        const d3 t = texel_rgb(S, T, m.normalmap, tex_uv(S, T, u, v, err));
        d3 nm = d3{(t.x - 0.5) * 2.0, (t.y - 0.5) * 2.0, (t.z - 0.5) * 2.0};
        const RT_RO double* ib = (c.type == SRT_PLANE) ? c.p + 16 : c.p + 30;
        return mul(normalize(matmul_rows(ib, nm)), orient);
    }
    return mul(collider_normal(c, P), orient);
}

// ---- counter-based RNG (Philox4x32-10) for Monte-Carlo shading and device jitter -------------
struct u4 {
    uint32_t a, b, c, d;
};
RT_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
RT_HD u4 philox(u4 ctr, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint32_t h0 = mulhi32(0xD2511F53u, ctr.a), l0 = 0xD2511F53u * ctr.a;
        uint32_t h1 = mulhi32(0xCD9E8D57u, ctr.c), l1 = 0xCD9E8D57u * ctr.c;
        ctr = u4{h1 ^ ctr.b ^ k0, l1, h0 ^ ctr.d ^ k1, l0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return ctr;
}
// numpy's 53-bit double from two 32-bit words
RT_HD double u01(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}
struct Rng {
    uint32_t k0, k1, c0, c1, c2, n;
    RT_HDM void init(uint64_t seed, uint32_t pix, uint32_t path, uint32_t tag) {
        k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32); c0 = pix; c1 = path; c2 = tag; n = 0;
    }
    RT_HDM void two(double& x, double& y) {
        u4 r = philox(u4{c0, c1, c2, n++}, k0, k1);
        x = u01(r.a, r.b);
        y = u01(r.c, r.d);
    }
    RT_HDM double one() {
        double x, y;
        two(x, y);
        return x;
    }
};
RT_HD uint32_t mix32(uint32_t h, uint32_t v) {
    h ^= v + 0x9E3779B9u + (h << 6) + (h >> 2);
    h *= 0x85EBCA6Bu;
    return h ^ (h >> 13);
}

// ---- rays -----------------------------------------------------------------------------------
// meta word: medium (8) | depth (8) | diffuse reflections (8)
RT_HD uint32_t pack_meta(uint32_t medium, uint32_t depth, uint32_t diffuse) {
    return (medium & 0xFFu) | ((depth & 0xFFu) << 8) | ((diffuse & 0xFFu) << 16);
}
RT_HD uint32_t meta_medium(uint32_t m) { return m & 0xFFu; }
RT_HD uint32_t meta_depth(uint32_t m) { return (m >> 8) & 0xFFu; }
RT_HD uint32_t meta_diffuse(uint32_t m) { return (m >> 16) & 0xFFu; }

struct Ray {
    d3 o, d, w;  // origin, direction, throughput (product of the Fresnel/absorption weights)
    uint32_t pix, meta, path;
};

// Camera.get_ray for one pixel (camera.py:51-85, utils/random.py:6-9)
// qw, qh: the divisions by the screen size (Quot: the kernels build them once per thread)
RT_HD void primary_ray(const srt_camera& cam, const Quot& qw, const Quot& qh, double xc, double yr,
                       const double j[4], d3& O, d3& D) {
    double x = xc + qw((j[0] - 0.5) * cam.cam_width);
    double y = yr + qh((j[1] - 0.5) * cam.cam_height);
    // pinhole (lens_radius == 0, every example): the disk offsets are (r cos, r sin) * 0 = +-0 and
    // leave O = look_from, so the sqrt/sincos of the disk sample are skipped (0 stands in for them)
    double rx = 0.0, ry = 0.0;
    if (cam.lens_radius != 0.0) {
        double r = sqrt(j[2]);
        double phi = (j[3] * 2.0) * PI;
        rx = r * cos(phi);
        ry = r * sin(phi);
    }
    d3 lf = ld3(cam.look_from), R = ld3(cam.right), U = ld3(cam.up);
    O = add(add(lf, mul(mul(R, rx), cam.lens_radius)), mul(mul(U, ry), cam.lens_radius));
    d3 t = add(add(add(lf, mul(mul(U, y), cam.focal_distance)), mul(mul(R, x), cam.focal_distance)),
               ld3(cam.fwd_fd));
    D = normalize(sub(t, O));
}
RT_HD void primary_ray(const srt_camera& cam, double xc, double yr, const double j[4], d3& O, d3& D) {
    primary_ray(cam, Quot((double)cam.width), Quot((double)cam.height), xc, yr, j, O, D);
}

// Nearest collider over the scene (ray.py:124-132): nearest = reduce(np.minimum, distances);
// a collider is hit where nearest != FARAWAY and its distance == nearest.  Returns the first
// such collider (-1 if none); `ties` reports that a later collider hit at the same distance.
// Ray/box slab test of child k of a 4-wide node (f64 arithmetic on the float bounds): entry
// distance `tnear`; an axis whose slab product is NaN (an axis-parallel ray exactly on a slab plane)
// constrains nothing (conservative).
#ifdef RT_BVH_F64
RT_HD bool box4_hit(const RT_RO BvhNode& nd, int k, d3 O, d3 inv, double& tnear) {
    double t0 = -INFINITY, t1 = INFINITY;
    const double o[3] = {O.x, O.y, O.z}, iv[3] = {inv.x, inv.y, inv.z};
    for (int a = 0; a < 3; ++a) {
        const double lo = (double)nd.lo[a][k], hi = (double)nd.hi[a][k];
        const double p = (lo - o[a]) * iv[a], q = (hi - o[a]) * iv[a];
        if (p != p || q != q) continue;
        t0 = fmax(t0, fmin(p, q));
        t1 = fmin(t1, fmax(p, q));
    }
    tnear = t0;
    return t0 <= t1 && t1 >= 0.0;
}
#endif

// The same slab test in f32 arithmetic (half the registers and VALU cycles of the f64 test above,
// which the RT_BVH_F64 experiment build keeps), widened so that it never rejects a box the exact
// test accepts.  Per ray and axis: iv = f32(1/D), noiv = -f32(O/D), so a slab plane's distance is
// one fma, fma(x, iv, noiv) -- within 2.001 * 2^-24 * s of (x - O)/D, s = |1/D| (bound + |O|) and x
// a box bound (|x| <= S.bvh_bound).  The box's entry / exit (max / min over the axes) are then moved
// out by e = 2^-20 max(s) over the axes, 8x every axis's error bound and 16x the f32 rounding of the
// subtraction / addition (|entry| <= 2^20 e), so the f32 interval holds the exact one and `tnear`
// is a lower bound of the exact entry distance.  An axis whose s is not below 1e37 (an
// axis-parallel ray: 1/D = inf; NaN) or whose 1/D does not fit a float (|D| < ~3e-39 on a tiny mesh
// near the origin, where s stays small but f32(1/D) would be inf) constrains nothing
// (conservative): its noiv is a quiet NaN, which fminf / fmaxf (IEEE minNum / maxNum) pass over;
// every other product stays finite.
#ifndef RT_BOX_MARGIN
#define RT_BOX_MARGIN 0x1p-20  // (tests/test_mesh.py checks that 0 fails the conservativeness probe)
#endif
struct BoxRay {
    float iv[3], noiv[3], e;
};
RT_HD BoxRay box_ray(d3 O, d3 inv, float bound) {
    BoxRay r;
    const double o[3] = {O.x, O.y, O.z}, iv[3] = {inv.x, inv.y, inv.z};
    double smax = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double s = fabs(iv[a]) * ((double)bound + fabs(o[a]));
        const bool ok = s < 1e37 && fabs(iv[a]) < 3e38;
        r.iv[a] = ok ? (float)iv[a] : 0.0f;
        r.noiv[a] = ok ? -(float)(o[a] * iv[a]) : __builtin_nanf("");
        smax = ok ? fmax(smax, s) : smax;
    }
    r.e = (float)(RT_BOX_MARGIN * smax);
    return r;
}
RT_HD bool box4f_hit(const RT_RO BvhNode& nd, int k, const BoxRay& r, float& tnear) {
    float t0 = -INFINITY, t1 = INFINITY;
    for (int a = 0; a < 3; ++a) {
        const float p = fmaf(nd.lo[a][k], r.iv[a], r.noiv[a]), q = fmaf(nd.hi[a][k], r.iv[a], r.noiv[a]);
        t0 = fmaxf(t0, fminf(p, q));
        t1 = fminf(t1, fmaxf(p, q));
    }
    t0 -= r.e;
    t1 += r.e;
    tnear = t0;
    return t0 <= t1 && t1 >= 0.0f;
}

// Traversal stack entries, one 64-bit word each: the entry distance as float bits (rounded down: a
// lower bound, so pruning never drops a box that holds a hit) over a child code -- an inner node's
// index (>= 0) or a leaf, -(1 + (first << 6 | count)) (rt_bvh.h keeps leaves below 64 triangles and
// 2^25 slots).  Leaves go on the stack like nodes, so the triangle loop appears once.
#if defined(__HIPCC__)
#define RT_UNROLL _Pragma("unroll")
#else
#define RT_UNROLL
#endif
RT_HD uint32_t bvh_f2u(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}
RT_HD float bvh_u2f(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f;
    memcpy(&f, &u, 4);
    return f;
#endif
}
// the box test's distance type and its per-ray operands
#ifdef RT_BVH_F64
using bvh_t = double;
struct BvhRay {
    d3 O, inv;
};
RT_HD BvhRay bvh_ray(const SceneView&, d3 O, d3 D) { return BvhRay{O, d3{1.0 / D.x, 1.0 / D.y, 1.0 / D.z}}; }
#else
using bvh_t = float;
struct BvhRay {
    BoxRay b;
};
RT_HD BvhRay bvh_ray(const SceneView& S, d3 O, d3 D) {
    return BvhRay{box_ray(O, d3{1.0 / D.x, 1.0 / D.y, 1.0 / D.z}, S.bvh_bound)};
}
#endif
RT_HD uint64_t bvh_entry(bvh_t tn, int32_t code) {
    float f = (float)tn;
    if ((double)f > (double)tn) f = nextafterf(f, -INFINITY);
    return ((uint64_t)bvh_f2u(f) << 32) | (uint32_t)code;
}
RT_HD int32_t bvh_code(int32_t child, int32_t count) {
    // (the negation in uint32_t: defined for every input, BVH_EMPTY included)
    if (child >= 0) return child;
    const uint32_t leaf = (0u - (uint32_t)child) - 1u;
    return (int32_t)(0u - (1u + ((leaf << 6) | (uint32_t)count)));
}

// The four children of a node against the ray: entry distances t[k] (INFINITY: missed, empty, or
// entered beyond `limit`) and child codes c[k], sorted by distance (a sorting network on registers).
RT_HD void bvh_children(const RT_RO BvhNode& nd, const BvhRay& R, double limit, bool strict, bvh_t t[4],
                        int32_t c[4]) {
RT_UNROLL
    for (int k = 0; k < 4; ++k) {
        c[k] = bvh_code(nd.child[k], nd.count[k]);  // (an empty slot's code is never used: t = INFINITY)
        bvh_t tn;
#ifdef RT_BVH_F64
        const bool box = box4_hit(nd, k, R.O, R.inv, tn);
#else
        const bool box = box4f_hit(nd, k, R.b, tn);
#endif
        const bool hit = nd.child[k] != BVH_EMPTY && box && (strict ? (double)tn < limit : (double)tn <= limit);
        t[k] = hit ? tn : (bvh_t)INFINITY;
    }
    auto cs = [&](int a, int b) {
        const bool sw = t[b] < t[a];
        const bvh_t ta = sw ? t[b] : t[a], tb = sw ? t[a] : t[b];
        const int32_t ca = sw ? c[b] : c[a], cb = sw ? c[a] : c[b];
        t[a] = ta;
        t[b] = tb;
        c[a] = ca;
        c[b] = cb;
    };
    cs(0, 1);
    cs(2, 3);
    cs(0, 2);
    cs(1, 3);
    cs(1, 2);
}

// A thread's traversal stack: a private array (scratch: its dynamic indexing keeps it out of
// registers), or (MAT_LDS_STACK) its first NL entries in LDS, column threadIdx.x of an [NL][NT]
// array (a wave's 64 lanes on consecutive words: conflict-free), the rest private.  Scratch entries
// go through L1/L2 and, a whole chip of stacks outgrowing them, to HBM, and a pop's latency is on the
// traversal's critical path: the fused mesh kernel 4.44 -> 3.20 ms per launch, spilled VGPRs 121 -> 29
// (profiles/r06_bvh_lds_stack_ab.txt).
constexpr int bvh_lds_entries(uint32_t feat) {
    return !(feat & MAT_LDS_STACK) ? 0 : (feat & MAT_LDS_NARROW) ? BVH_LDS / 2 : BVH_LDS;
}
constexpr int bvh_lds_threads(uint32_t feat) { return (feat & MAT_LDS_NARROW) ? 64 : 256; }
#if defined(__HIP_DEVICE_COMPILE__)
template <int NL, int NT>
__device__ __forceinline__ uint64_t* bvh_lds_column() {
    __shared__ uint64_t stack_lds[NL * NT];
    return stack_lds + threadIdx.x;
}
#endif
template <uint32_t FEAT>
struct BvhStack {
#if defined(__HIP_DEVICE_COMPILE__)
    static constexpr int NL = bvh_lds_entries(FEAT), NT = bvh_lds_threads(FEAT);
    uint64_t* col = NL > 0 ? bvh_lds_column<(NL > 0 ? NL : 1), NT>() : nullptr;
#else
    static constexpr int NL = 0, NT = 1;
#endif
    uint64_t priv[BVH_STACK - NL];
    RT_HDM void put(int i, uint64_t e) {
#if defined(__HIP_DEVICE_COMPILE__)
        if (NL > 0 && i < NL) { col[i * NT] = e; return; }
#endif
        priv[i - NL] = e;
    }
    RT_HDM uint64_t get(int i) const {
#if defined(__HIP_DEVICE_COMPILE__)
        if (NL > 0 && i < NL) return col[i * NT];
#endif
        return priv[i - NL];
    }
};

// Nearest BVH triangle, merged into (best, id, bo, ties) with the reference's rule independent of
// visiting order: the smallest distance wins, among equal distances the lowest collider index,
// and `ties` records that another collider hit at that distance.  Boxes entered beyond `best` are
// pruned (a box entered exactly at `best` is still visited: it may hold a tie); a node's hit children
// are pushed farthest first (the nearest is popped next) with their entry distance, which prunes them
// again on pop.  Triangles never return NaN (a NaN ray fails every comparison of triangle_hit and
// misses).
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH>
RT_HD void bvh_nearest(const SceneView& S, d3 O, d3 D, double& best, int& id, double& bo, bool& ties) {
    const BvhRay R = bvh_ray(S, O, D);
    BvhStack<FEAT> stack;
    int sp = 0;
    // the node (or leaf) visited next stays in a register: a node's nearest hit child is taken
    // directly, the others pushed; the stack is read only when a subtree is done
    int32_t code = 0;
    for (;;) {
        if (code < 0) {
            const int first = (-code - 1) >> 6, cnt = (-code - 1) & 63;
            for (int j = first; j < first + cnt; ++j) {
                const int c = S.bvh_tri[j];
                double o;
                const double t = triangle_hit(S.col[c].p, O, D, o);
                if (t < best) { best = t; id = c; bo = o; ties = false; }
                else if (t == best && best != FARAWAY) {
                    ties = true;
                    if (c < id) { id = c; bo = o; }
                }
            }
        } else {
            bvh_t t[4];
            int32_t c[4];
            bvh_children(S.bvh[code], R, best, false, t, c);
            if (t[0] != INFINITY) {
                RT_UNROLL
                for (int k = 3; k >= 1; --k)
                    if (t[k] != INFINITY && sp < BVH_STACK) stack.put(sp++, bvh_entry(t[k], c[k]));
                code = c[0];
                continue;
            }
        }
        // pop the nearest pending subtree not entered beyond `best`
        bool more = false;
        while (sp > 0) {
            const uint64_t e = stack.get(--sp);
            if ((double)bvh_u2f((uint32_t)(e >> 32)) > best) continue;
            code = (int32_t)(uint32_t)e;
            more = true;
            break;
        }
        if (!more) break;
    }
}

// Any shadowed BVH triangle closer than `stop` along L: returns its distance, else FARAWAY.
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH>
RT_HD double bvh_shadow(const SceneView& S, d3 O, d3 L, double stop) {
    const BvhRay R = bvh_ray(S, O, L);
    BvhStack<FEAT> stack;
    int sp = 0;
    int32_t code = 0;
    for (;;) {
        if (code < 0) {
            const int first = (-code - 1) >> 6, cnt = (-code - 1) & 63;
            for (int j = first; j < first + cnt; ++j) {
                const RT_RO srt_collider& cc = S.col[S.bvh_tri[j]];
                if (!(cc.flags & SRT_CF_SHADOW)) continue;
                double o;
                const double t = triangle_hit(cc.p, O, L, o);
                if (t < stop) return t;
            }
        } else {
            bvh_t t[4];
            int32_t c[4];
            bvh_children(S.bvh[code], R, stop, true, t, c);
            if (t[0] != INFINITY) {
                RT_UNROLL
                for (int k = 3; k >= 1; --k)
                    if (t[k] != INFINITY && sp < BVH_STACK) stack.put(sp++, (uint32_t)c[k]);
                code = c[0];
                continue;
            }
        }
        if (sp == 0) break;
        code = (int32_t)(uint32_t)stack.get(--sp);
    }
    return FARAWAY;
}

// BVH: compile the mesh traversal in (kernels instantiated for scenes without a BVH leave it out:
// its stack would otherwise cost scratch and registers in every kernel)
// One collider of the nearest-hit search of a collider sequence (its TYPE known at compile time),
// merged into (best, id, bo, ties, nan) as nearest_hit's loop does
template <uint32_t FEAT, int TYPE>
RT_HD void nearest_step(const RT_RO srt_collider& cc, int c, d3 O, d3 D, double& best, int& id, double& bo,
                        bool& ties, bool& nan) {
    double o;
    if (TYPE == SRT_CUBOID && cc.p[42] != 0.0 && id >= 0) {
        // axis-aligned box around O (a SkyBox): leaving it takes t >= dmin / max|D_i|, dmin the
        // distance from O to the nearest face, and its slab t's are NaN-free (no face passes
        // through O).  Far beyond the nearest hit so far it can be neither nearest nor tied.
        const RT_RO double* p = cc.p;
        double dmin = np_min(np_min(np_min(O.x - p[12], p[15] - O.x), np_min(O.y - p[13], p[16] - O.y)),
                             np_min(O.z - p[14], p[17] - O.z));
        double dmax = np_max(np_max(fabs(D.x), fabs(D.y)), fabs(D.z));
        if (dmin > 0.0 && best * dmax < 0.5 * dmin) return;
    }
    double t;
    if constexpr (TYPE == SRT_SPHERE) t = sphere_hit(cc.p, O, D, o);
    else if constexpr (TYPE == SRT_PLANE) t = plane_hit(cc.p, O, D, o);
    else if constexpr (TYPE == SRT_CUBOID) t = cuboid_hit(cc.p, O, D, o);
    else t = triangle_hit(cc.p, O, D, o);
    if (t != t) nan = true;
    if (t < best) { best = t; id = c; bo = o; ties = false; }
    else if (t == best && id >= 0) ties = true;
}
template <uint32_t FEAT, int... K>
RT_HD void nearest_seq(const SceneView& S, d3 O, d3 D, double& best, int& id, double& bo, bool& ties, bool& nan,
                       std::integer_sequence<int, K...>) {
    (nearest_step<FEAT, seq_type(seq_of(FEAT), K)>(S.col[K], K, O, D, best, id, bo, ties, nan), ...);
}

template <uint32_t FEAT = MAT_GENERIC | MAT_BVH>
RT_HD int nearest_hit(const SceneView& S, d3 O, d3 D, double& tn, double& on, bool& ties) {
    constexpr bool BVH = (FEAT & MAT_BVH) != 0;
    double best = FARAWAY;
    int id = -1;
    double bo = FARAWAY;
    ties = false;
    bool nan = false;
    if constexpr (seq_of(FEAT) != 0u && !BVH) {
        // the scene's colliders in straight-line code, in index order (the same merge as the loop)
        nearest_seq<FEAT>(S, O, D, best, id, bo, ties, nan, std::make_integer_sequence<int, seq_count(seq_of(FEAT))>{});
    } else {
        // without a BVH `lin` is the identity: the loop then indexes the collider table directly
        const int nl = BVH ? S.nlin : S.ncol;
        for (int li = 0; li < nl; ++li) {
            const int c = BVH ? S.lin[li] : li;
            double o;
            const RT_RO srt_collider& cc = S.col[c];
            if (cc.type == SRT_CUBOID && cc.p[42] != 0.0 && id >= 0) {
                // axis-aligned box around O (a SkyBox): see nearest_step
                const RT_RO double* p = cc.p;
                double dmin = np_min(np_min(np_min(O.x - p[12], p[15] - O.x), np_min(O.y - p[13], p[16] - O.y)),
                                     np_min(O.z - p[14], p[17] - O.z));
                double dmax = np_max(np_max(fabs(D.x), fabs(D.y)), fabs(D.z));
                if (dmin > 0.0 && best * dmax < 0.5 * dmin) continue;
            }
            double t = collider_hit<FEAT>(cc, O, D, o);
            if (t != t) nan = true;
            if (t < best) { best = t; id = c; bo = o; ties = false; }
            else if (t == best && id >= 0) ties = true;
        }
    }
    if (BVH && S.bvh_nodes > 0) bvh_nearest<FEAT>(S, O, D, best, id, bo, ties);
    if (nan || best == FARAWAY) { tn = nan ? NAN : FARAWAY; on = FARAWAY; ties = false; return -1; }
    tn = best;
    on = bo;
    return id;
}

// ---- shading --------------------------------------------------------------------------------
// Shading functions report their results to an emitter `E` as they are produced:
//   em.local(c)        colour added at this hit (the caller multiplies by the ray throughput)
//   em.child(ch)       one child ray (weight relative to the parent's throughput)
//   em.diffuse(g, m)   a Diffuse fan-out of g.count children (generated by diffuse_child)
//   em.shadow(n)       n shadow rays were traced
// On the GPU the emitter appends children with one atomic per wave (rt_kernels.hip); in the host
// check harness it pushes to a vector.  Nothing is held per lane between hits.
struct Child {
    d3 o, d, w;       // w: weight relative to the parent's throughput
    uint32_t medium;  // media row the child travels in
    uint32_t dfl;     // diffuse reflections of the child
    uint32_t slot;    // child index (path hash)
};
// Diffuse fan-out descriptor
struct DiffuseGen {
    d3 P;       // nudged origin
    d3 N;       // oriented normal
    d3 w;       // diff colour / (pi * count)
    int count;  // diffuse_rays (first bounce) or 1
    uint32_t medium, dfl;
};

// (1 - cos)^5 by repeated products; numpy evaluates `** 5` with its SIMD pow, both are within a
// few ulp of the exact power (far inside the 1e-5 colour tolerance)
RT_HD double pow5(double x) {
    double x2 = x * x;
    return (x2 * x2) * x;
}

// x^k for a wave-uniform integer k >= 1 by binary powering (a few multiplies instead of pow): the
// Glossy lobe exponent 2/roughness^2 - 2 is an integer up to rounding for the usual roughnesses
// (0.2 -> 47.99999999999999); within 4 ulp of k, x^a / x^k = x^(a-k) differs from 1 by
// |(a-k) ln x| < 4 * 2^-52 * a * 745 / a < 1e-12 wherever x^a is a normal double
RT_HD double powi(double x, int k) {
    double r = 1.0;
    bool first = true;
    for (;;) {
        if (k & 1) { r = first ? x : r * x; first = false; }
        k >>= 1;
        if (!k) return r;
        x = x * x;
    }
}

RT_HD d3 schlick(d3 F0, double cos_t) {
    double p = pow5(1.0 - cos_t);
    d3 one_m = rsub(1.0, F0);
    return add(F0, mul(one_m, p));
}

RT_HD d3 reflect_dir(d3 D, d3 N) {
    double dn = dot(D, N);
    d3 N2 = mul(N, 2.0);
    return normalize(sub(D, mul(N2, dn)));
}

RT_HD Child mkchild(d3 o, d3 d, d3 w, uint32_t medium, uint32_t dfl, uint32_t slot) {
    Child c;
    c.o = o; c.d = d; c.w = w; c.medium = medium; c.dfl = dfl; c.slot = slot;
    return c;
}

// min over the shadowed colliders of the distance along the light direction (glossy.py:53-59)
// `stop`: the caller only asks whether the result is >= stop (seelight), so the BVH pass may stop
// at the first shadowing triangle closer than that
// One collider of the shadow test (glossy.py:53-59) of a collider sequence, as shadow_nearest's loop
template <uint32_t FEAT, int TYPE>
RT_HD void shadow_step(const SceneView& S, const RT_RO srt_collider& cc, int c, int light, d3 O, d3 L, double& best,
                       bool& first) {
    if (!(cc.flags & SRT_CF_SHADOW)) return;
    double o, t;
    if constexpr (TYPE == SRT_CUBOID) t = cuboid_hit_local(cc.p, O, ld3(S.light_local + ((int64_t)light * S.ncol + c) * 3), o);
    else if constexpr (TYPE == SRT_SPHERE) t = sphere_hit(cc.p, O, L, o);
    else if constexpr (TYPE == SRT_PLANE) t = plane_hit(cc.p, O, L, o);
    else t = triangle_hit(cc.p, O, L, o);
    best = first ? t : np_min(best, t);
    first = false;
}
template <uint32_t FEAT, int... K>
RT_HD void shadow_seq(const SceneView& S, int light, d3 O, d3 L, double& best, bool& first,
                      std::integer_sequence<int, K...>) {
    (shadow_step<FEAT, seq_type(seq_of(FEAT), K)>(S, S.col[K], K, light, O, L, best, first), ...);
}

template <uint32_t FEAT = MAT_GENERIC | MAT_BVH>
RT_HD double shadow_nearest(const SceneView& S, int light, d3 O, d3 L, double stop) {
    constexpr bool BVH = (FEAT & MAT_BVH) != 0;
    double best = FARAWAY;
    bool first = true;
    if constexpr (seq_of(FEAT) != 0u && !BVH) {
        shadow_seq<FEAT>(S, light, O, L, best, first, std::make_integer_sequence<int, seq_count(seq_of(FEAT))>{});
    } else {
        const int nl = BVH ? S.nlin : S.ncol;
        for (int li = 0; li < nl; ++li) {
            const int c = BVH ? S.lin[li] : li;
            const RT_RO srt_collider& cc = S.col[c];
            if (!(cc.flags & SRT_CF_SHADOW)) continue;
            double o, t;
            if (cc.type == SRT_CUBOID)
                t = cuboid_hit_local(cc.p, O, ld3(S.light_local + ((int64_t)light * S.ncol + c) * 3), o);
            else
                t = collider_hit<FEAT>(cc, O, L, o);
            best = first ? t : np_min(best, t);
            first = false;
        }
    }
    if (BVH && S.bvh_nodes > 0 && best >= stop)
        best = np_min(best, bvh_shadow<FEAT>(S, O, L, stop));
    return best;
}

// Glossy.get_color (glossy.py:25-110)
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH, class E>
RT_HD void shade_glossy(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t, double orient,
                        E& em, uint32_t& err) {
    const RT_RO srt_material& m = S.mat[mi];
    RT_T0(tg0);
    d3 P = add(r.o, mul(r.d, t));
    d3 N = shading_normal<FEAT>(S, c, m, P, orient, err);
    // the texel word of a textured material is loaded first and read after the shadow tests of the
    // lights (which do not depend on it), so its latency overlaps them; the colour is then composed
    // in the reference's order (glossy.py:30-84)
    uint32_t tw = 0u;
    if (m.tex >= 0) {
        double u, v;
        if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
        tw = texel_word(S, S.tex[m.tex], tex_uv(S, S.tex[m.tex], u, v, err));
    }
    RT_ACC(4, tg0);
    RT_T0(tg1);
    d3 V = mul(r.d, -1.0);
    d3 nudged = add(P, mul(N, NUDGE));
    uint32_t med = meta_medium(r.meta);
    // seelight of the first 32 lights (glossy.py:53-59), tested before the texel is read
    uint32_t see = 0u;
    for (int l = 0; l < S.nlights && l < 32; ++l) {
        const RT_RO srt_light& Lt = S.lights[l];
        if (Lt.type != SRT_LIGHT_DIRECTIONAL) continue;
#ifndef RT_ABL_SHADOW  // (diagnostic build only: time without the shadow test)
        if (S.nshadow > 0) {
            RT_T0(ts0);
            const double ln = shadow_nearest<FEAT>(S, l, nudged, ld3(Lt.dir), SKYBOX_DISTANCE);
            RT_ACC(5, ts0);
            if (ln >= SKYBOX_DISTANCE) see |= 1u << l;
            em.shadow(1);
        } else
#endif
        {
            see |= 1u << l;
        }
    }
    const d3 diff = m.tex >= 0 ? mul(word_rgb(S, m.tex, tw), m.p[3]) : ld3(m.p);
    d3 color = mul(ld3(S.ambient), diff);
    for (int l = 0; l < S.nlights; ++l) {
        const RT_RO srt_light& Lt = S.lights[l];
        if (Lt.type != SRT_LIGHT_DIRECTIONAL) {
            // PointLight.get_L reads the undefined names M and dist_light (lights.py:30-31): the
            // reference's render raises NameError at the first Glossy hit, so does this one
            err |= ERR_NAME;
            continue;
        }
        const d3 L = ld3(Lt.dir);
        const double dist = SKYBOX_DISTANCE;
        double NdotL = np_max(dot(N, L), 0.0);
        const d3 lv = mul(ld3(Lt.color), NdotL);
        d3 H = normalize(add(L, V));
        double seelight = 1.0;
        if (l < 32) {
            seelight = ((see >> l) & 1u) ? 1.0 : 0.0;
#ifndef RT_ABL_SHADOW
        } else if (S.nshadow > 0) {
            double ln = shadow_nearest<FEAT>(S, l, nudged, L, dist);
            seelight = (ln >= dist) ? 1.0 : 0.0;
            em.shadow(1);
#endif
        }
        color = add(color, mul(mul(diff, lv), seelight));
        if (m.flags & SRT_MF_ROUGH) {
            // medium 0 (scene.n, nearly every ray) has its F0 in the material record (scalar loads)
            d3 F0 = (med == 0) ? ld3(m.p + 11) : ld3(S.glossy_f0 + ((int64_t)mi * S.nmedia + med) * 3);
            double cos_t = np_clip(dot(V, H), 0.0, 1.0);
            d3 F = schlick(F0, cos_t);
#ifdef RT_ABL_POW  // diagnostic build only
            double Dphong = (pow5(np_clip(dot(N, H), 0.0, 1.0)) * m.p[5]) / m.p[6];
#else
            RT_T0(tp0);
            const double nh = np_clip(dot(N, H), 0.0, 1.0);
            double Dphong = ((m.ival > 0 ? powi(nh, m.ival) : pow_ool(nh, m.p[4])) * m.p[5]) / m.p[6];
            RT_ACC(6, tp0);
#endif
            double den = 4.0 * np_clip(dot(N, V) * NdotL, 0.001, 1.0);
            const Quot qd(den);
            d3 FD = mul(F, Dphong);
            d3 spec = mul(mul(mul(d3{qd(FD.x), qd(FD.y), qd(FD.z)}, seelight), lv), m.p[7]);
            color = add(color, spec);
        }
    }
    RT_ACC(7, tg1);
    em.local(color);
#ifdef RT_ABL_NOEMIT  // diagnostic build only
    return;
#endif
    if ((int)meta_depth(r.meta) < c.max_ray_depth) {
        RT_T0(tc0);
        double cos_t = np_clip(dot(V, N), 0.0, 1.0);
        d3 F = schlick(ld3(m.p + 8), cos_t);
        Child ch = mkchild(nudged, reflect_dir(r.d, N), F, med, meta_diffuse(r.meta), 1);
        RT_ACC(8, tc0);
        RT_T0(tc1);
        em.child(ch);
        RT_ACC(9, tc1);
    }
}

// Refractive.get_color (refractive.py:24-123); `mc_u` is the uniform for the MC pick
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH, class E>
RT_HD void shade_refractive(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t,
                            double orient, E& em, uint32_t& err, double mc_u) {
    if ((int)meta_depth(r.meta) >= c.max_ray_depth) return;  // black beyond max_ray_depth
    const RT_RO srt_material& m = S.mat[mi];
    d3 P = add(r.o, mul(r.d, t));
    d3 N = shading_normal<FEAT>(S, c, m, P, orient, err);
    d3 V = mul(r.d, -1.0);
    uint32_t m1 = meta_medium(r.meta);
    uint32_t m2 = (orient == 1.0) ? (uint32_t)m.medium : 0u;
    const RT_RO double* n1 = S.media + m1 * 6;
    const RT_RO double* n2 = S.media + m2 * 6;
    double cos_i = dot(V, N);
    double s = 1.0 - cos_i * cos_i;
    double F[3], ratio[3];
    for (int k = 0; k < 3; ++k) {
        cplx a1 = cplx{n1[k], n1[3 + k]}, a2 = cplx{n2[k], n2[3 + k]};
        ratio[k] = n1[k] / n2[k];
        cplx q = cdiv(a1, a2);
        cplx z = cmulr(cmul(q, q), s);
        cplx cos_t = csqrt_np(cplx{1.0 - z.re, 0.0 - z.im});
        cplx x1 = cmulr(a1, cos_i), x2 = cmul(a2, cos_t);
        cplx r_per = cdiv(csub(x1, x2), cadd(x1, x2));
        cplx y1 = cmul(a1, cos_t), y2 = cmulr(a2, cos_i);
        cplx r_par = cdiv(cmul(cplx{-1.0, 0.0}, csub(y1, y2)), cadd(y1, y2));
        double ap = cabs(r_per), aq = cabs(r_par);
        F[k] = (ap * ap + aq * aq) / 2.0;
    }
    // absorption: exp(-2 * Im(n_ray) * 2 * pi / lambda * 1e9 * distance), lambda = (630, 550, 475)
    const double lam[3] = {630.0, 550.0, 475.0};
    double ab[3];
    for (int k = 0; k < 3; ++k) ab[k] = exp(((((-2.0 * n1[3 + k]) * 2.0) * PI) / lam[k]) * 1e9 * t);
    double aver = ((ratio[0] + ratio[1]) + ratio[2]) / 3.0;
    double sin2 = (aver * aver) * (1.0 - cos_i * cos_i);
    bool non_tir = sin2 <= 1.0;
    uint32_t dfl = meta_diffuse(r.meta);
    if (c.flags & SRT_CF_MC) {
        double favg = ((F[0] + F[1]) + F[2]) / 3.0;
        bool refr = (mc_u > favg) && non_tir;
        d3 w = d3{ab[0], ab[1], ab[2]};
        if (refr) {
            double kk = aver * cos_i - sqrt(1.0 - np_clip(sin2, 0.0, 1.0));
            d3 Rt = normalize(add(mul(r.d, aver), mul(N, kk)));
            em.child(mkchild(sub(P, mul(N, NUDGE)), Rt, w, m2, dfl, 1));
        } else {
            em.child(mkchild(add(P, mul(N, NUDGE)), reflect_dir(r.d, N), w, m1, dfl, 1));
        }
        return;
    }
    em.child(mkchild(add(P, mul(N, NUDGE)), reflect_dir(r.d, N), d3{F[0] * ab[0], F[1] * ab[1], F[2] * ab[2]},
                     m1, dfl, 1));
    if (non_tir) {
        double kk = aver * cos_i - sqrt(1.0 - np_clip(sin2, 0.0, 1.0));
        d3 Rt = normalize(add(mul(r.d, aver), mul(N, kk)));
        em.child(mkchild(sub(P, mul(N, NUDGE)), Rt,
                         d3{(1.0 - F[0]) * ab[0], (1.0 - F[1]) * ab[1], (1.0 - F[2]) * ab[2]}, m2, dfl, 2));
    }
}

// ThinFilmInterference.get_color (thin_film_interference.py:24-115)
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH, class E>
RT_HD void shade_thinfilm(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t,
                          double orient, E& em, uint32_t& err) {
    if ((int)meta_depth(r.meta) >= c.max_ray_depth) return;
    const RT_RO srt_material& m = S.mat[mi];
    d3 P = add(r.o, mul(r.d, t));
    d3 N = shading_normal<FEAT>(S, c, m, P, orient, err);
    d3 V = mul(r.d, -1.0);
    double cos_i = dot(V, N);
    const RT_RO srt_texture& lut = S.tex[m.tex_aux0];
    int64_t li = np_trunc(cos_i * (double)lut.height);
    int64_t ti;
    if (m.flags & SRT_MF_NOISE) {
        double u, v;
        if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
        const RT_RO srt_texture& nt = S.tex[m.tex_aux1];
        double nz = tex_lut(S, m.tex_aux1, *tex_uv(S, nt, u, v, err));
        double thick = m.p[0] + m.p[1] * (nz - 0.5);
        ti = np_trunc(thick);
    } else {
        ti = (int64_t)m.p[0];
    }
    d3 F = texel_rgb(S, lut, m.tex_aux0, texel_at(S, lut, li, ti, err));
    em.local(mul(ld3(S.ambient), F));
    uint32_t med = meta_medium(r.meta), dfl = meta_diffuse(r.meta);
    em.child(mkchild(add(P, mul(N, NUDGE)), reflect_dir(r.d, N), F, med, dfl, 1));
    em.child(mkchild(sub(P, mul(N, NUDGE)), r.d, rsub(1.0, F), med, dfl, 2));
}

// SkyBox_Material.get_texture_color (skybox.py:51-94)
template <class E>
RT_HD void shade_sky(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t, E& em,
                     uint32_t& err) {
#ifdef RT_ABL_NOSKY  // diagnostic build only
    em.local(d3{t, 0.5, 0.5});
    return;
#endif
    const RT_RO srt_material& m = S.mat[mi];
    RT_T0(tk0);
    d3 P = add(r.o, mul(r.d, t));
    double u, v;
    if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
    RT_ACC(10, tk0);
    RT_T0(tk1);
    d3 col = tex_rgb(S, m.tex, u, v, err);
    RT_ACC(11, tk1);
    if (meta_depth(r.meta) != 0 && (m.flags & SRT_MF_LIGHTMAP)) {
        const RT_RO srt_texture& L = S.tex[m.tex_aux0];
        const d3 lt = texel_rgb(S, L, m.tex_aux0, tex_uv(S, L, u, v, err));
        col = d3{col.x + m.p[0] * lt.x, col.y + m.p[0] * lt.y, col.z + m.p[0] * lt.z};
    }
    em.local(col);
}

// The collider whose material is the scene's SkyBox / Panorama (SceneView::sky_col), when exactly one
// collider has a sky material; else -1
RT_HD int sky_collider(const srt_collider* col, int n, const srt_material* mat) {
    int k = -1;
    for (int i = 0; i < n; ++i)
        if (mat[col[i].material].type == SRT_SKY) {
            if (k >= 0) return -1;
            k = i;
        }
    return k;
}

// shade_sky in two halves around the waterfall of the other colliders (trace_one): the texel words
// of a sky hit (colour, and the lightmap's on a non-primary ray) fetched first, so their load latency
// overlaps the other colliders' shading; the colour made from them afterwards -- the same values
// shade_sky computes (skybox.py:51-94)
RT_HD void sky_fetch(const SceneView& S, const Ray& r, double t, uint32_t& w0, uint32_t& w1, uint32_t& err) {
    const RT_RO srt_collider& c = S.col[S.sky_col];
    const RT_RO srt_material& m = S.mat[c.material];
    const d3 P = add(r.o, mul(r.d, t));
    double u, v;
    if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
    w0 = texel_word(S, S.tex[m.tex], tex_uv(S, S.tex[m.tex], u, v, err));
    w1 = 0u;
    if (meta_depth(r.meta) != 0 && (m.flags & SRT_MF_LIGHTMAP))
        w1 = texel_word(S, S.tex[m.tex_aux0], tex_uv(S, S.tex[m.tex_aux0], u, v, err));
}
RT_HD d3 sky_color(const SceneView& S, const Ray& r, uint32_t w0, uint32_t w1) {
    const RT_RO srt_material& m = S.mat[S.col[S.sky_col].material];
    d3 col = word_rgb(S, m.tex, w0);
    if (meta_depth(r.meta) != 0 && (m.flags & SRT_MF_LIGHTMAP)) {
        const d3 lt = word_rgb(S, m.tex_aux0, w1);
        col = d3{col.x + m.p[0] * lt.x, col.y + m.p[0] * lt.y, col.z + m.p[0] * lt.z};
    }
    return col;
}

// Emissive.get_color (emissive.py:21-23)
template <class E>
RT_HD void shade_emissive(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t, E& em,
                          uint32_t& err) {
    const RT_RO srt_material& m = S.mat[mi];
    if (m.tex >= 0) {
        double u, v;
        d3 P = add(r.o, mul(r.d, t));
        if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
        em.local(tex_rgb(S, m.tex, u, v, err));
    } else {
        em.local(ld3(m.p));
    }
}

// Diffuse.get_color (diffuse.py:25-124): no local colour; the children carry the estimate
template <uint32_t FEAT = MAT_GENERIC | MAT_BVH, class E>
RT_HD void shade_diffuse(const SceneView& S, const RT_RO srt_collider& c, int mi, const Ray& r, double t, double orient,
                         E& em, uint32_t& err) {
    uint32_t dfl = meta_diffuse(r.meta);
    if (dfl >= 2) return;
    const RT_RO srt_material& m = S.mat[mi];
    d3 P = add(r.o, mul(r.d, t));
    d3 N = shading_normal<FEAT>(S, c, m, P, orient, err);
    d3 diff;
    if (m.tex >= 0) {
        double u, v;
        if (!collider_uv(c, P, u, v)) err |= ERR_UNSUPPORTED;
        diff = tex_rgb(S, m.tex, u, v, err);
    } else {
        diff = ld3(m.p);
    }
    DiffuseGen g;
    g.count = (dfl < 1) ? m.ival : 1;
    g.P = add(P, mul(N, NUDGE));
    g.N = N;
    g.w = mul(diff, 1.0 / (PI * (double)g.count));
    g.medium = meta_medium(r.meta);
    g.dfl = dfl + 1;
    em.diffuse(g, mi);
}

// ONB of utils/random.py:72-76 (ax_w given)
RT_HD void onb(d3 w, d3& u, d3& v) {
    d3 a = (fabs(w.x) > 0.9) ? d3{0.0, 1.0, 0.0} : d3{1.0, 0.0, 0.0};
    d3 c = d3{w.y * a.z - w.z * a.y, -w.x * a.z + w.z * a.x, w.x * a.y - w.y * a.x};
    v = normalize(c);
    u = d3{w.y * v.z - w.z * v.y, -w.x * v.z + w.z * v.x, w.x * v.y - w.y * v.x};
}

// One diffuse child: direction from the cosine PDF or the cosine/spherical-caps mixture
// (utils/random.py:58-174), weight = w * clip(N.d) / pdf(d).
RT_HD Child diffuse_child(const SceneView& S, const RT_RO srt_material& m, const DiffuseGen& g, Rng& rng, uint32_t k) {
    double pdf1w = m.p[3];
    double sel, dummy;
    rng.two(sel, dummy);
    bool caps = (S.nimp > 0) && !(sel < pdf1w);
    d3 dir;
    if (!caps) {
        d3 u, v;
        onb(g.N, u, v);
        double a, b;
        rng.two(a, b);
        double phi = (a * 2.0) * PI;
        double z = sqrt(1.0 - b), x = cos(phi) * sqrt(b), y = sin(phi) * sqrt(b);
        dir = add(add(mul(u, x), mul(v, y)), mul(g.N, z));
    } else {
        double pick, a;
        rng.two(pick, a);
        int i = (int)(pick * (double)S.nimp);
        if (i >= S.nimp) i = S.nimp - 1;
        const RT_RO double* im = S.importance + 4 * i;
        d3 tc = sub(ld3(im), g.P);
        d3 w = normalize(tc);
        double dist = sqrt(dot(tc, tc));
        double rr = np_clip(im[3] / dist, 0.0, 1.0);
        double cmax = sqrt(1.0 - rr * rr);
        d3 u, v;
        onb(w, u, v);
        double b = rng.one();
        double phi = (a * 2.0) * PI;
        double z = 1.0 + b * (cmax - 1.0);
        double sz = sqrt(1.0 - z * z);
        dir = add(add(mul(u, cos(phi) * sz), mul(v, sin(phi) * sz)), mul(w, z));
    }
    double cosp = np_clip(dot(dir, g.N), 0.0, 1.0) / PI;
    double pdf = cosp;
    if (S.nimp > 0) {
        double caps_pdf = 0.0;
        for (int i = 0; i < S.nimp; ++i) {
            const RT_RO double* im = S.importance + 4 * i;
            d3 tc = sub(ld3(im), g.P);
            d3 w = normalize(tc);
            double dist = sqrt(dot(tc, tc));
            double rr = np_clip(im[3] / dist, 0.0, 1.0);
            double cmax = sqrt(1.0 - rr * rr);
            if (dot(dir, w) > cmax) caps_pdf += 1.0 / ((1.0 - cmax) * TWO_PI);
        }
        caps_pdf = caps_pdf / (double)S.nimp;
        pdf = cosp * pdf1w + caps_pdf * m.p[4];
    }
    double ndl = np_clip(dot(dir, g.N), 0.0, 1.0);
    return mkchild(g.P, dir, mul(g.w, ndl / pdf), g.medium, g.dfl, 0x100u + k);
}


// Shade one (ray, collider) hit with a per-lane (possibly divergent) material.
template <uint32_t MATS = MAT_GENERIC | MAT_BVH, class E>
RT_HD void shade_hit(const SceneView& S, int cid, int mi, const Ray& r, double t, double orient, E& em,
                     uint32_t& err, double mc_u) {
    const RT_RO srt_collider& c = S.col[cid];
    switch (S.mat[mi].type) {
        case SRT_GLOSSY:
            if (MATS & mat_bit(SRT_GLOSSY)) shade_glossy<MATS>(S, c, mi, r, t, orient, em, err);
            break;
        case SRT_REFRACTIVE:
            if (MATS & mat_bit(SRT_REFRACTIVE)) shade_refractive<MATS>(S, c, mi, r, t, orient, em, err, mc_u);
            break;
        case SRT_THINFILM:
            if (MATS & mat_bit(SRT_THINFILM)) shade_thinfilm<MATS>(S, c, mi, r, t, orient, em, err);
            break;
        case SRT_DIFFUSE:
            if (MATS & mat_bit(SRT_DIFFUSE)) shade_diffuse<MATS>(S, c, mi, r, t, orient, em, err);
            break;
        case SRT_EMISSIVE:
            if (MATS & mat_bit(SRT_EMISSIVE)) shade_emissive(S, c, mi, r, t, em, err);
            break;
        default:
            if (MATS & mat_bit(SRT_SKY)) shade_sky(S, c, mi, r, t, em, err);
            break;
    }
}

// RNG stream of the Monte-Carlo refraction pick / diffuse children of a ray
RT_HD uint32_t child_path(uint32_t path, uint32_t slot, uint32_t round) { return mix32(path, slot + 4096u * round); }

// ---- row-band shards of a frame over ranks (SRT_RENDER_SHARDED) ---------------------------------
// The frame's rows are cut into bands of h rows (the last band shorter), dealt round-robin to the n
// ranks, one band per rank per period of n bands (rank q takes band q of every period; the reference
// parallelises over samples instead, scene.py:80-116).  A rank's j-th band lies in period j, so its
// local row i holds a row of period i / h.  Interleaving balances the cheap sky rows against the
// reflective floor rows; each band of a rank is a run of the numpy stream a rank jumps to (~110 us
// of a CU per jump), so the bands are as tall as the balance allows: h is chosen per (H, n) with at
// most `kmax` bands per rank (and at least kmax / 2), the fewest rows on the busiest rank first, then
// the most bands.  (A snake order -- odd periods dealt n-1 .. 0 -- gave the first and the last rank
// two adjacent bands at every turn, one run of the numpy stream twice as long to generate: ex1 1080p,
// slowest of 8 ranks 0.317 vs 0.288 ms round-robin, ex4 4K 2.47 vs 2.35 ms,
// profiles/r03_band_order_ab.txt; removed in round 6.)
constexpr int SHARD_BANDS = 8;  // kmax: most bands per rank (option "shard_bands"; 0 = shard_kmax's choice)
// A Diffuse fan-out scene costs ~50 rays per pixel and sample, so a jump is a fraction of one row's
// work and the balance wins: bands of SHARD_FANOUT_ROWS rows (cornell 800x800 on 8 ranks, slowest
// rank of the same frame: 618 ms with 20-row bands, 583 with 4, 570 with 2; profiles/r03_*)
constexpr int SHARD_FANOUT_ROWS = 2;
RT_HD int shard_kmax(int64_t H, int n, int kmax_opt, int fanout) {
    if (kmax_opt > 0) return kmax_opt;
    if (fanout > 2 && n > 0) {
        const int64_t k = H / ((int64_t)n * SHARD_FANOUT_ROWS);
        return k > SHARD_BANDS ? (int)k : SHARD_BANDS;
    }
    return SHARD_BANDS;
}
RT_HD int shard_band_owner(int64_t b, int n) { return (int)(b % n); }
RT_HD int64_t shard_rank_rows(int64_t H, int n, int q, int64_t h) {
    const int64_t B = (H + h - 1) / h;  // bands
    const int64_t full = B / n, rem = B % n;
    const int64_t nb = full + (q < rem ? 1 : 0);  // one band per full period, then bands 0 .. rem-1
    return nb * h - (shard_band_owner(B - 1, n) == q ? B * h - H : 0);
}
RT_HD int64_t shard_max_rows(int64_t H, int n, int64_t h) {
    int64_t m = 0;
    for (int q = 0; q < n; ++q) {
        const int64_t r = shard_rank_rows(H, n, q, h);
        m = r > m ? r : m;
    }
    return m;
}
RT_HD int64_t shard_band_height(int64_t H, int n, int kmax) {
    if (n <= 1 || H <= 1) return H > 0 ? H : 1;
    if (kmax < 1) kmax = 1;
    int64_t best_h = 1, best_rows = (int64_t)1 << 62;
    for (int k = kmax; k >= (kmax / 2 > 1 ? kmax / 2 : 1); --k) {
        int64_t h = (H + (int64_t)n * k - 1) / ((int64_t)n * k);
        if (h < 1) h = 1;
        if ((H + h - 1) / h < n) continue;  // fewer bands than ranks: a rank would get no rows (then h = 1)
        const int64_t m = shard_max_rows(H, n, h);
        if (m < best_rows) { best_rows = m; best_h = h; }
    }
    return best_h;
}
RT_HD int shard_of_row(int64_t y, int n, int64_t h) { return shard_band_owner(y / h, n); }
RT_HD int64_t shard_local_row(int64_t y, int n, int64_t h) { return (y / (h * n)) * h + y % h; }

// sRGB_linear_to_sRGB + clip + uint8 for one pixel (colour_functions.py:4-18, scene.py:125-140)
RT_HD void resolve_pixel(double r, double g, double b, double& orr, double& og, double& ob, uint8_t px[3]) {
    double c[3] = {r, g, b}, e[3];
    for (int k = 0; k < 3; ++k)
        e[k] = (c[k] <= 0.00304) ? 12.92 * c[k] : 1.055 * pow_ool(c[k], 1.0 / 2.4) - 0.055;
    double peak = np_max(np_max(e[0], e[1]), e[2]) + 0.00001;
    if (peak > 1.0)
        for (int k = 0; k < 3; ++k) e[k] = (e[k] * 1.0) / peak;
    for (int k = 0; k < 3; ++k) {
        double q = 255.0 * np_clip(e[k], 0.0, 1.0);
        px[k] = (q == q) ? (uint8_t)(int)q : (uint8_t)0;
    }
    orr = r; og = g; ob = b;
}

}  // namespace rt
