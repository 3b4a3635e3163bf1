// rt_kernels.hip -- gfx950 wavefront tracer behind the C ABI of include/sightpy_rt.h.
//
// The reference (sightpy) recursively evaluates numpy batches: intersect every collider, reduce
// the nearest hit, compact the rays per collider, shade, recurse (ray.py:122-148).  Here the
// recursion is flattened into a breadth-first wavefront over structure-of-arrays ray queues in
// HBM, one launch per depth:
//
//   k_primary      depth 0: primary-ray generation (camera.py:51-85) fused with the trace step,
//                  one thread per pixel looping over the pass's samples
//   k_trace        depth d: read ray d from queue, nearest hit over all colliders, shade,
//                  add throughput * local colour to the framebuffer, append children to d+1
//   k_resolve      spp average + sRGB + intensity clip + uint8 (scene.py:118-140)
//
// A colour composes linearly along the ray tree (colour = local + F * child), so each queued ray
// carries the product of the weights above it (its throughput) and contributions are summed into
// the per-pixel framebuffer with float64 atomics.  Scene tables are read through wave-uniform
// indices (scalar loads) in the collider loop; shading runs as a waterfall over the materials
// present in a wave so each material's parameters are wave-uniform too.  Children are appended
// with one block-wide exclusive scan and one atomicAdd per block.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_mt.h"
#include "rt_mt_kernel.h"

using namespace rt;
using namespace rtmt_dev;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return fail(SRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
    } while (0)

constexpr int BLOCK = 256;
#ifndef RT_NSHARD
#define RT_NSHARD 256
#endif
// queue shards, one append counter each: blocks b, b + NSHARD, ... share one.  Appends are
// device-scope atomics executed at the memory side; with 16 counters their serialisation cost the
// depth-0 kernel ~40 % (1.39 vs 0.87 ms, ex1 1080p), 64-256 counters remove it.
constexpr int NSHARD = RT_NSHARD;
constexpr size_t TRACE_PARAMS_BYTES = 864;
constexpr int MAX_LUT_LDS = 12;  // texture tables staged in LDS per block (2 KiB each)
// retry bits of flags[1]: a queue shard / ring overflowed (re-render with bigger queues); a tie gave
// a chained ray a second child (re-render without chain mode)
constexpr uint32_t RETRY_OVERFLOW = 1u;
constexpr uint32_t RETRY_CHAIN_TIE = 2u;
constexpr uint32_t RETRY_FIXED_RANGE = 4u;  // a contribution beyond the fixed-point range (fx_add)

struct Queue {
    double *ox, *oy, *oz, *dx, *dy, *dz, *wr, *wg, *wb;
    uint32_t *pix, *meta, *path;
};
constexpr int64_t RAY_BYTES = 9 * 8 + 3 * 4;  // 84 B per queued ray

struct TraceParams {
    SceneView S;
    Queue qin, qout;
    const uint32_t* cnt_in;  // [NSHARD] rays per input shard (depth d)
    uint32_t* cnt_out;       // [NSHARD] append counters of the output shards (depth d+1)
    uint32_t* flags;         // [0] error bits, [1] overflow
    unsigned long long* shadow;
    double* fb;              // [3][npix] depth-0 colour (stored by the pixel's own thread)
    unsigned long long* fbx; // [3][npix] fixed-point sums of every added contribution (fb_add), or null:
                             // f64 atomics into fb (option "deterministic" 0, order-dependent rounding)
    int64_t npix;
    int64_t seg;             // capacity of one queue shard (rays)
    uint64_t seed;
    int depth;
    int fb_first;  // depth 0 of the first pass: store the pixel instead of adding (no memset)
    // primary generation
    int64_t n_primary;
    srt_camera cam;
    const int32_t* rows;
    const double* jitter;  // [spp][4][jit_plane] (device) or null
    int64_t jit_plane;     // doubles per jitter plane: npix, or width*height when jit_global
    int jit_global;        // 1: jitter indexed by the global pixel (the whole frame's numpy stream)
    int sample_base;
    int spp;           // samples of this pass (k_primary)
    int pix_groups;    // k_primary: sample groups per pixel (a power of two <= 64; lanes of one wave)
    int chain;         // k_trace: trace each ray's whole (single-child) chain in-thread, see k_trace
    int32_t* hit_out;  // [spp][npix] or null
    // frame kernel (k_frame): per-wave ray rings in HBM, slot s = rays [s * ring_cap, (s+1) * ring_cap)
    Queue ring;
    uint32_t* ring_lock;  // [nslot] 0 = free, 1 = owned by a running wave
    int64_t ring_cap;     // rays per ring (power of two)
    double* out_rgb;      // fused resolve (single-pass frames): [3][npix] linear RGB or null
    uint8_t* out_u8;      //                                     [npix][3] sRGB8 or null
    int nslot;
    int dcap;             // deepest depth traced; deeper children are counted and dropped
    int fuse_resolve;     // 1: k_frame resolves its pixels (no framebuffer); 0: adds to fb
    int spp_total;        // samples of the frame (resolve average)
    // k_shade_forced (srt_shade, Material.get_color): the first depth's hit per ray (index = pix)
    const int32_t* force_id;
    const double* force_t;
    const double* force_o;
    // k_frame sample groups: block b takes tile b % ntiles and the samples [g spg, (g+1) spg) of the
    // pass, g = b / ntiles; groups > 1 store their partial sums to fbg[g][3][npix] (k_fb_groups adds them)
    double* fbg;
    int groups;
    int ntiles;
    // srt_debug_lane_stats: [depth][2] u64 = (wave iterations that traced the depth, live lanes in
    // them) of the fused paths' depth loop, or null (counting off)
    unsigned long long* lane_stats;
};
// kernel argument: host and device passes must agree on the layout (catches address-space pointer
// size differences, see SceneView)
static_assert(sizeof(TraceParams) == TRACE_PARAMS_BYTES, "TraceParams layout");

// Pixel identity that keys the Monte-Carlo draws: the global pixel row * width + col of the frame
// (`pix` indexes the rows this call renders), so that an image sharded over any number of GPUs draws
// the same numbers as the single-GPU render; srt_trace (no rows) keys by the ray's batch index.
__device__ __forceinline__ uint32_t key_pix(const TraceParams& P, uint32_t pix) {
    if (!P.rows) return pix;
    const uint32_t W = (uint32_t)P.cam.width;
    const uint32_t lr = pix / W;
    return (uint32_t)P.rows[lr] * W + (pix - lr * W);
}

__device__ __forceinline__ void queue_store(const Queue& q, int64_t i, d3 o, d3 d, d3 w, uint32_t pix,
                                            uint32_t meta, uint32_t path) {
    q.ox[i] = o.x; q.oy[i] = o.y; q.oz[i] = o.z;
    q.dx[i] = d.x; q.dy[i] = d.y; q.dz[i] = d.z;
    q.wr[i] = w.x; q.wg[i] = w.y; q.wb[i] = w.z;
    q.pix[i] = pix; q.meta[i] = meta; q.path[i] = path;
}

__device__ __forceinline__ Ray queue_load(const Queue& q, int64_t i) {
    Ray r;
    r.o = d3{q.ox[i], q.oy[i], q.oz[i]};
    r.d = d3{q.dx[i], q.dy[i], q.dz[i]};
    r.w = d3{q.wr[i], q.wg[i], q.wb[i]};
    r.pix = q.pix[i]; r.meta = q.meta[i]; r.path = q.path[i];
    return r;
}

// Contributions added to a pixel by other threads (depth >= 1, split samples) go into an
// order-independent fixed-point sum, so a frame is bit-reproducible (the reference is
// deterministic; f64 atomics are not, their rounding depends on arrival order): each contribution
// rounded to a multiple of 2^-FX_BITS and summed with one int64 atomic per channel (the count of f64
// atomics it replaces); the resolve adds sum 2^-FX_BITS to the depth-0 colour.  Rounding error
// <= 2^-45 = 2.8e-14 per contribution; a contribution of magnitude >= 2^17 (sums up to 2^19 stay in
// range) raises RETRY_FIXED_RANGE and the frame is rendered again with f64 atomics.
constexpr int FX_BITS = 44;
constexpr double FX_SCALE = (double)(1ull << FX_BITS);
constexpr double FX_UNIT = 1.0 / FX_SCALE;
constexpr double FX_MAX = 131072.0;                 // 2^17

// Range of the sums: a pixel-channel sum wraps only beyond 2^20 (2^64 scaled).  Besides the three
// sums, every pixel keeps a coarse magnitude -- the f32 sum of |r| + |g| + |b| of its terms, one
// more fire-and-forget atomic (fx_mag, behind the sums in the same buffer) -- and the resolve
// distrusts a pixel whose magnitude reached FX_MAG_LIMIT (2^16; f32 rounding keeps it within a factor
// 1 + n 2^-24 of the true magnitude, so no sum of fewer than 2^23 terms gets near 2^20 unseen).
// A returning atomic per term (checking each partial sum) cost 6.6 % of the device frame.
constexpr float FX_MAG_LIMIT = 65536.0f;
RT_HD int64_t fx_words(int64_t npix) { return 3 * npix + (npix + 1) / 2; }  // u64 words of fbx
__device__ __forceinline__ float* fx_mag(unsigned long long* fbx, int64_t npix) {
    return reinterpret_cast<float*>(fbx + 3 * npix);
}
__device__ __forceinline__ const float* fx_mag(const unsigned long long* fbx, int64_t npix) {
    return reinterpret_cast<const float*>(fbx + 3 * npix);
}

__device__ __forceinline__ bool fx_add(unsigned long long* acc, double v) {
    if (!(fabs(v) < FX_MAX)) return false;  // (also NaN)
    atomicAdd(acc, (unsigned long long)__double2ll_rn(v * FX_SCALE));
    return true;
}

__device__ __forceinline__ void fb_add(double* fb, unsigned long long* fbx, uint32_t* flags, int64_t npix,
                                       uint32_t pix, d3 w, d3 c) {
    if (is_zero(c)) return;  // adding an exact zero is a no-op
#ifdef RT_ABL_FB  // diagnostic build only: no framebuffer atomics
    if (w.x * c.x == 12345.678) fb[pix] = 0.0;
    return;
#endif
    if (fbx) {
        // all three channels added (no short-circuit), then one range check
        const double tx = w.x * c.x, ty = w.y * c.y, tz = w.z * c.z;
        const int ok = (int)fx_add(fbx + pix, tx) & (int)fx_add(fbx + npix + pix, ty) & (int)fx_add(fbx + 2 * npix + pix, tz);
        if (!ok) atomicOr(flags + 1, RETRY_FIXED_RANGE);
        unsafeAtomicAdd(fx_mag(fbx, npix) + pix, (float)((fabs(tx) + fabs(ty)) + fabs(tz)));
    } else {
        unsafeAtomicAdd(fb + pix, w.x * c.x);
        unsafeAtomicAdd(fb + npix + pix, w.y * c.y);
        unsafeAtomicAdd(fb + 2 * npix + pix, w.z * c.z);
    }
}

__device__ __forceinline__ double fx_value(const unsigned long long* fbx, int64_t npix, int ch, int64_t p) {
    return (double)(long long)fbx[ch * npix + p] * FX_UNIT;
}

// a pixel the resolve must not trust: its coarse magnitude reached FX_MAG_LIMIT (or is NaN), or a
// channel sum lies in [2^61, 2^64) scaled (>= 2^17 in colour units; negative = wrapped)
__device__ __forceinline__ bool fx_suspect(const unsigned long long* fbx, int64_t npix, int64_t p) {
    bool bad = !(fx_mag(fbx, npix)[p] < FX_MAG_LIMIT);
    for (int ch = 0; ch < 3; ++ch) bad |= (fbx[ch * npix + p] >> 61) != 0;
    return bad;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Reserve `cnt` consecutive slots of the output shard for every active lane: one atomic per wave.
// The exclusive prefix of the (small) per-lane counts is assembled from one ballot per bit, which
// is exact in divergent code (inactive lanes contribute nothing).
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* ctr, uint32_t cnt) {
    uint32_t total = 0, below = 0;
    uint64_t any = __ballot(cnt != 0);
    if (!any) return 0;
    for (int b = 0; b < 8; ++b) {
        uint64_t m = __ballot((cnt >> b) & 1u);
        total += (uint32_t)__builtin_popcountll(m) << b;
        below += lanes_below(m) << b;
    }
    uint32_t base = 0;
#ifdef RT_ABL_NOATOMIC  // diagnostic build only: no counter traffic at all
    return below + (total & 0u);
#endif
#ifdef RT_ABL_APPEND  // diagnostic build only: counts kept, slots not waited for (wrong images)
    if (lanes_below(__ballot(1)) == 0) atomicAdd(ctr, total);
    return ((blockIdx.x * 256u + threadIdx.x) * 2u + below % 2u) % 400000u;
#endif
    if (lanes_below(__ballot(1)) == 0) base = atomicAdd(ctr, total);  // first active lane
    base = __builtin_amdgcn_readfirstlane(base);
    return base + below;
}

// the exclusive prefix of `cnt` over the active lanes below this one (wave_reserve's `below`)
__device__ __forceinline__ uint32_t wave_below(uint32_t cnt) {
    uint32_t below = 0;
    for (int b = 0; b < 8; ++b) below += lanes_below(__ballot((cnt >> b) & 1u)) << b;
    return below;
}

// A pixel's colour summed in the thread that traces (some of) its samples, in one of two forms
// sharing the same registers:
//  * fixed point (P.fbx set, the default): every term -- depth 0 included -- rounded to a multiple of
//    2^-FX_BITS and summed as an integer (unsigned: wrapping is defined), exactly fb_add's terms, plus
//    fb_add's coarse magnitude (the f32 sum of |r| + |g| + |b| of the terms, independent of the sums).
//    Integer sums do not depend on the order or grouping of the terms, so a pixel's samples may be
//    split over any number of threads (sample groups, k_primary) or GPUs and the totals are the same
//    bits.  A term of magnitude >= 2^17 (or NaN) is left out of the sums and shows in the magnitude
//    (>= FX_MAG_LIMIT or NaN): the frame is then rendered again in f64.
//  * f64 (option deterministic 0, or that fallback): the f64 sums, in the words' bits.
struct PixAcc {
    unsigned long long w[3] = {0ull, 0ull, 0ull};
    float mag = 0.0f;

    __device__ __forceinline__ void add(bool fx, d3 t) {
        if (fx) {
            const double m = (fabs(t.x) + fabs(t.y)) + fabs(t.z);
            if (m < FX_MAX) {  // every |term| < 2^17: the conversions are in range (NaN fails too)
                w[0] += (unsigned long long)__double2ll_rn(t.x * FX_SCALE);
                w[1] += (unsigned long long)__double2ll_rn(t.y * FX_SCALE);
                w[2] += (unsigned long long)__double2ll_rn(t.z * FX_SCALE);
            }
            mag += (float)m;
        } else {
            w[0] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)w[0]) + t.x);
            w[1] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)w[1]) + t.y);
            w[2] = (unsigned long long)__double_as_longlong(__longlong_as_double((long long)w[2]) + t.z);
        }
    }
    __device__ __forceinline__ double value(bool fx, int k) const {
        return fx ? (double)(long long)w[k] * FX_UNIT : __longlong_as_double((long long)w[k]);
    }
    // the pixel's fixed-point totals the resolve must not trust (fx_suspect's rule)
    __device__ __forceinline__ bool suspect() const {
        return !(mag < FX_MAG_LIMIT) || ((w[0] | w[1] | w[2]) >> 61) != 0;
    }
    // sum over the lanes l ^ off, off = 32, 16, .. >= lo (the sample groups of a pixel, k_primary):
    // integer sums exactly; f64 sums pairwise, commutative, so every lane ends with the same value
    __device__ __forceinline__ void reduce_lanes(bool fx, int lo) {
        for (int off = 32; off >= lo; off >>= 1) {
            for (int k = 0; k < 3; ++k) {
                const unsigned long long o = __shfl_xor(w[k], off);
                w[k] = fx ? w[k] + o
                          : (unsigned long long)__double_as_longlong(__longlong_as_double((long long)w[k]) +
                                                                     __longlong_as_double((long long)o));
            }
            mag += __shfl_xor(mag, off);
        }
    }
};


// Emitter of the GPU trace step: colour -> framebuffer atomics, children -> output queue shard.
struct GpuEmit {
    const TraceParams& P;
    const Ray& r;
    uint32_t shard;
    uint32_t round;
    uint32_t* shadow_acc;
    PixAcc* acc;  // depth 0: the pixel's sums in the thread (no framebuffer atomics)

    __device__ void local(d3 c) const {
        if (acc) {
            if (!is_zero(c)) acc->add(P.fbx != nullptr, mul(r.w, c));
        } else {
            fb_add(P.fb, P.fbx, P.flags, P.npix, r.pix, r.w, c);
        }
    }
    __device__ void shadow(int n) const { *shadow_acc += (uint32_t)n; }
    __device__ void store(uint32_t slot, const Child& c, uint32_t path) const {
#if defined(RT_ABL_QSTORE) || defined(RT_ABL_NOATOMIC)  // diagnostic build only: no queue stores
        if (c.o.x == 12345.678) P.flags[1] = path;
        return;
#endif
        if (slot < (uint64_t)P.seg) {
            queue_store(P.qout, (int64_t)shard * P.seg + slot, c.o, c.d, mul(r.w, c.w), r.pix,
                        pack_meta(c.medium, meta_depth(r.meta) + 1, c.dfl), path);
        } else {
            atomicOr(&P.flags[1], RETRY_OVERFLOW);
        }
    }
    __device__ void child(const Child& c) const {
        uint32_t slot = wave_reserve(P.cnt_out + shard, 1u);
        store(slot, c, child_path(r.path, c.slot, round));
    }
    // the fan-out child-major: the k-th children of the wave's lanes take consecutive slots, so every
    // store of a child is one coalesced run (lane-major slots scattered each store over 64 lines)
    __device__ void diffuse(const DiffuseGen& g, int mi) const {
        const uint32_t cnt = (uint32_t)g.count;
        const uint32_t base = wave_reserve(P.cnt_out + shard, cnt) - wave_below(cnt);
        const auto& m = P.S.mat[mi];
        uint32_t off = 0;
        for (uint32_t k = 0;; ++k) {
            const uint64_t mk = __ballot(cnt > k);
            if (!mk) break;
            if (cnt > k) {
                Rng rng;
                const uint32_t cpath = child_path(r.path, 0x100u + k, round);
                rng.init(P.seed, key_pix(P, r.pix), cpath, 0xD1000000u | meta_depth(r.meta));
                store(base + off + lanes_below(mk), diffuse_child(P.S, m, g, rng, k), cpath);
            }
            off += (uint32_t)__builtin_popcountll(mk);
        }
    }
};

__device__ __forceinline__ double mc_uniform(const TraceParams& P, const Ray& r, int cid, uint32_t round) {
    if (!(P.S.col[cid].flags & SRT_CF_MC)) return 0.0;
    Rng g;
    g.init(P.seed, key_pix(P, r.pix), r.path, 0x3C000000u | (meta_depth(r.meta) << 8) | round);
    return g.one();
}

// Uniforms for primary ray of sample s at local pixel p.
__device__ __forceinline__ void primary_uniforms(const TraceParams& P, int s, uint32_t p, uint32_t gpix,
                                                 double j[4]) {
    if (P.jitter) {
        const int64_t plane = P.jit_plane;
        const double* base = P.jitter + (int64_t)s * 4 * plane + (P.jit_global ? gpix : p);
        j[0] = base[0]; j[1] = base[plane];
        // the lens-disk pair is read only by a thin-lens camera (pinhole: primary_ray skips it)
        if (P.cam.lens_radius != 0.0) { j[2] = base[2 * plane]; j[3] = base[3 * plane]; }
    } else {
        Rng g;
        g.init(P.seed, gpix, (uint32_t)(P.sample_base + s), 0xCA3E0000u);
        g.two(j[0], j[1]);
        g.two(j[2], j[3]);
    }
}

// k_primary's split of primary_uniforms: the pixel-jitter pair (prefetched a sample ahead) and the
// lens-disk pair (thin-lens cameras only), the same values
__device__ __forceinline__ void primary_jitter(const TraceParams& P, int s, uint32_t p, uint32_t gpix, double j[2]) {
#ifdef RT_ABL_JIT  // diagnostic build only: no jitter loads (wrong images; timing only)
    j[0] = 0.5 + 1e-9 * (double)(s & 7);
    j[1] = 0.5;
    return;
#endif
    if (P.jitter) {
        const int64_t plane = P.jit_plane;
        const double* base = P.jitter + (int64_t)s * 4 * plane + (P.jit_global ? gpix : p);
        j[0] = base[0];
        j[1] = base[plane];
    } else {
        double j4[4];
        primary_uniforms(P, s, p, gpix, j4);
        j[0] = j4[0];
        j[1] = j4[1];
    }
}
__device__ __forceinline__ void lens_jitter(const TraceParams& P, int s, uint32_t p, uint32_t gpix, double j[4]) {
    double j4[4] = {0.0, 0.0, 0.0, 0.0};
    primary_uniforms(P, s, p, gpix, j4);
    j[2] = j4[2];
    j[3] = j4[3];
}

// an emitter whose child replaces the traced ray in place (Em::kInPlace)
template <class Em, class = void>
struct em_in_place : std::false_type {};
template <class Em>
struct em_in_place<Em, std::void_t<decltype(Em::kInPlace)>> : std::bool_constant<Em::kInPlace> {};

// One trace step for one ray (all lanes of the wave call it; `active` masks the tail).
// MATS: material types compiled into this instantiation (the host picks one covering the scene).
// Em: the emitter (GpuEmit: wavefront queues; FrameEmit: the frame kernel's per-wave ring); `em0`
// is round 0's, tied colliders get copies with rounds 1, 2, ...
template <uint32_t MATS, class Em, bool FORCED = false>
__device__ __forceinline__ void trace_one(const TraceParams& P, Ray& r, bool active, uint32_t& err, int32_t* hit_slot,
                                          const Em& em0) {
    const SceneView& S = P.S;
    double t = FARAWAY, o = FARAWAY;
    bool ties = false;
    int id = -1;
    RT_T0(tn0);
    if (FORCED) {  // the caller's hit (Material.get_color): that collider only, no tie loop
        if (active) {
            id = P.force_id[r.pix];
            t = P.force_t[r.pix];
            o = P.force_o[r.pix];
            if (id < -1 || id >= (int32_t)S.ncol) {  // not a collider of the scene (IndexError)
                err |= ERR_INDEX;
                id = -1;
            }
        }
    } else if (active) {
        id = nearest_hit<MATS>(S, r.o, r.d, t, o, ties);
    }
    if constexpr (em_in_place<Em>::value) {
        // the emitter writes the child over `r` (the fused path): no tie loop, which would read the
        // ray after shading; a tie renders the frame again without the fused path
        if (ties) atomicOr(&P.flags[1], RETRY_CHAIN_TIE);
        ties = false;
    }
    RT_ACC(1, tn0);
    if (hit_slot && active) *hit_slot = id;
#ifdef RT_ABL_NOSHADE  // diagnostic build only: raygen + nearest hit, no shading
    if (id == 12345) em0.local(d3{t, o, 0.0});
    return;
#endif
    // waterfall over the colliders hit in this wave: inside each pass the collider index, and so
    // its material and every table entry they reference, is wave-uniform (scalar loads into SGPRs,
    // uniform branches); a wave usually sees one to three distinct colliders
    // Exact ties (ray.py:131-146: every collider at the nearest distance is shaded and the colours
    // added) go through the same waterfall: after shading its collider a tied lane moves on to the
    // next collider (in index order) hit at the same distance, with the next emission round.  One
    // copy of the shaders per kernel (a separate tie loop held a second one: the kernels waited on
    // ~10 % of their wave cycles in SQ_WAIT_INST_ANY; round 6: issue stalls, the i-cache misses 0.004 %).
    RT_T0(tw0);
    // a SkyBox / Panorama hit without a tie: its texel words fetched now, its colour added after the
    // waterfall of the other colliders (the load latency overlaps their shading; fixed-point sums do
    // not depend on the order of the terms)
    bool sky_pre = false;
    uint32_t sky_w0 = 0u, sky_w1 = 0u;
    if constexpr (!FORCED && (MATS & mat_bit(SRT_SKY)) != 0) {
        sky_pre = S.sky_col >= 0 && id == S.sky_col && !ties;
        if (sky_pre) sky_fetch(S, r, t, sky_w0, sky_w1, err);
    }
    int cur = sky_pre ? -1 : id;  // collider this lane shades next (-1: done)
    double co = o;    // its orientation
    uint32_t rnd = 0;  // emission round: 0 the nearest collider, k the k-th tied one
    uint64_t pending = __ballot(cur >= 0);
    while (pending) {
        RT_ACC(12, tw0);  // counts waterfall passes (k = 12 calls)
        const int lead = __builtin_ctzll(pending);
        const int cu = __builtin_amdgcn_readfirstlane(__shfl(cur, lead));
        const bool mine = (cur == cu);
        if (mine) {
            // re-derive the uniform index inside the branch: here cur == cu on every active lane, and
            // the compiler would otherwise substitute the per-lane id back into every table
            // address (vector loads into VGPRs instead of scalar loads)
            const int cs = __builtin_amdgcn_readfirstlane(cur);
            const auto& c = S.col[cs];
            const int m = c.material;
            Em em = em0;
            if (rnd) em.round = rnd;
            switch (S.mat[m].type) {
                case SRT_GLOSSY:
                    if (MATS & mat_bit(SRT_GLOSSY)) shade_glossy<MATS>(S, c, m, r, t, co, em, err);
                    break;
                case SRT_REFRACTIVE:
                    if (MATS & mat_bit(SRT_REFRACTIVE))
                        shade_refractive<MATS>(S, c, m, r, t, co, em, err, mc_uniform(P, r, cs, rnd));
                    break;
                case SRT_THINFILM:
                    if (MATS & mat_bit(SRT_THINFILM)) shade_thinfilm<MATS>(S, c, m, r, t, co, em, err);
                    break;
                case SRT_DIFFUSE:
                    if (MATS & mat_bit(SRT_DIFFUSE)) shade_diffuse<MATS>(S, c, m, r, t, co, em, err);
                    break;
                case SRT_EMISSIVE:
                    if (MATS & mat_bit(SRT_EMISSIVE)) shade_emissive(S, c, m, r, t, em, err);
                    break;
                default:
                    if (MATS & mat_bit(SRT_SKY)) shade_sky(S, c, m, r, t, em, err);
                    break;
            }
        }
        if (!FORCED && __ballot(mine && ties)) {
            // the lanes just shaded find their next tied collider: a wave-uniform collider loop
            // (scalar table loads) from cu + 1
            int nxt = -1;
            double no = FARAWAY;
            for (int c = cu + 1; c < S.ncol; ++c) {
                double oc;
                if (mine && ties && nxt < 0 && collider_hit<MATS>(S.col[c], r.o, r.d, oc) == t) {
                    nxt = c;
                    no = oc;
                }
            }
            if (mine) {
                cur = nxt;
                co = no;
                ++rnd;
            }
        } else if (mine) {
            cur = -1;
        }
        pending = __ballot(cur >= 0);
    }
    if (sky_pre) em0.local(sky_color(S, r, sky_w0, sky_w1));
    RT_ACC(2, tw0);
}

// Chain mode emitter (scenes whose rays have at most one child): the child replaces the ray in the
// thread instead of going to the next depth's queue.  A second child (two colliders tied at the
// same distance) has no place: it raises the retry flag and the host renders the frame again
// without chain mode.
struct ChainEmit {
    const TraceParams& P;
    const Ray& r;
    uint32_t round;
    uint32_t* shadow_acc;
    Ray* next;
    bool* has;

    __device__ void local(d3 c) const { fb_add(P.fb, P.fbx, P.flags, P.npix, r.pix, r.w, c); }
    __device__ void shadow(int n) const { *shadow_acc += (uint32_t)n; }
    __device__ void put(const Child& c, uint32_t path) const {
        if (*has) {
            atomicOr(&P.flags[1], RETRY_CHAIN_TIE);
            return;
        }
        *has = true;
        next->o = c.o;
        next->d = c.d;
        next->w = mul(r.w, c.w);
        next->pix = r.pix;
        next->meta = pack_meta(c.medium, meta_depth(r.meta) + 1, c.dfl);
        next->path = path;
    }
    __device__ void child(const Child& c) const { put(c, child_path(r.path, c.slot, round)); }
    __device__ void diffuse(const DiffuseGen& g, int mi) const {
        const auto& m = P.S.mat[mi];
        for (int k = 0; k < g.count; ++k) {
            Rng rng;
            const uint32_t cpath = child_path(r.path, 0x100u + (uint32_t)k, round);
            rng.init(P.seed, key_pix(P, r.pix), cpath, 0xD1000000u | meta_depth(r.meta));
            put(diffuse_child(P.S, m, g, rng, (uint32_t)k), cpath);
        }
    }
};

// Fused-path emitter (k_primary<.., FUSE>: single-child scenes traced pixel by pixel, every depth
// in the pixel's own thread): the one child replaces the ray.  A second child (an exact tie) raises
// RETRY_CHAIN_TIE as in chain mode.  Every depth's colour goes into the thread's PixAcc: the same
// fixed-point terms the per-depth kernels add (their k_primary keeps depth 0 in a PixAcc, k_trace
// adds the deeper terms with fb_add), so the fused and the per-depth paths give the same image bit
// for bit; in f64 mode the terms are summed in the thread in trace order.
struct FusedEmit {
    static constexpr bool kInPlace = true;  // `next` is the traced ray itself (see trace_one)
    const TraceParams& P;
    const Ray& r;
    uint32_t round;
    uint32_t* shadow_acc;
    PixAcc* acc;
    Ray* next;
    bool* has;

    __device__ void local(d3 c) const {
        if (!is_zero(c)) acc->add(P.fbx != nullptr, mul(r.w, c));
    }
    __device__ void shadow(int n) const { *shadow_acc += (uint32_t)n; }
    __device__ void child(const Child& c) const {
        ChainEmit{P, r, round, shadow_acc, next, has}.child(c);
    }
    __device__ void diffuse(const DiffuseGen& g, int mi) const {
        ChainEmit{P, r, round, shadow_acc, next, has}.diffuse(g, mi);
    }
};

// srt_debug_lane_stats: one wave iteration of a depth with the live lanes m, counted by the lowest
// live lane ([0] iterations, [1] live lanes)
__device__ __forceinline__ void lane_count(unsigned long long* st, uint64_t m) {
    if (lanes_below(m) == 0) {
        atomicAdd(st, 1ull);
        atomicAdd(st + 1, (unsigned long long)__builtin_popcountll(m));
    }
}

// Copy the first `nlut` texture lookup tables into LDS (dynamic shared memory) and point the
// scene view at them: texel -> value becomes an LDS read instead of a dependent global load.
__device__ __forceinline__ void stage_luts(const TraceParams& P) {
    const int n = P.S.nlut_lds;
    for (int i = threadIdx.x; i < n * 256; i += BLOCK) rt_lds_dyn[i] = P.S.tex[i >> 8].lut[i & 255];
    __syncthreads();
}

// The uint8 RGB of n consecutive pixels (lane l < n holds pixel p0 + l; dst = out + 3 p0) as 3n/4
// dword stores instead of 3n byte stores (n a multiple of 4, dst 4-byte aligned); otherwise byte
// stores.  Every lane of the wave must call it (cross-lane reads).
__device__ __forceinline__ void store_u8_chunk(uint8_t* dst, const uint8_t px[3], int lane, int n) {
    const uint32_t v = (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(dst) & 3) == 0) {
        const int nd = (3 * n) / 4;
        const int w = lane < nd ? lane : nd - 1;
        const int q0 = (4 * w) / 3, r0 = (4 * w) % 3;  // dword w = bytes 4w..4w+3: pixels q0, q0 + 1
        const uint32_t x0 = __shfl(v, q0), x1 = __shfl(v, q0 + 1);
        if (lane < nd) reinterpret_cast<uint32_t*>(dst)[lane] = (x0 >> (8 * r0)) | (x1 << (8 * (3 - r0)));
    } else if (lane < n) {
        dst[3 * lane] = px[0];
        dst[3 * lane + 1] = px[1];
        dst[3 * lane + 2] = px[2];
    }
}

// The uint8 RGB of a tw x th pixel tile (lane l < tw th holds local pixel (row0 + l / tw, col0 + l % tw))
// of a frame of W columns and nrows rows: per tile row of tw = 8 (4) pixels, 6 (3) dword stores when
// the row is whole and dword-aligned, else byte stores.  Every lane of the wave must call it.
__device__ __forceinline__ void store_u8_tile(uint8_t* out, const uint8_t px[3], int lane, int tw, int th,
                                              int64_t row0, int64_t col0, int64_t W, int64_t nrows) {
    const uint32_t v = (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
    const int nd = (3 * tw) / 4;  // dwords per tile row
    const int ry = lane / nd, w = lane % nd;
    const int q0 = (4 * w) / 3, r0 = (4 * w) % 3;
    const uint32_t x0 = __shfl(v, ry * tw + q0), x1 = __shfl(v, ry * tw + q0 + 1);
    const int64_t row = row0 + ry;
    uint8_t* dst = out + 3 * (row * W + col0);
    const bool whole = col0 + tw <= W && (reinterpret_cast<uintptr_t>(dst) & 3) == 0;
    if (ry < th && row < nrows && whole) reinterpret_cast<uint32_t*>(dst)[w] = (x0 >> (8 * r0)) | (x1 << (8 * (3 - r0)));
    // rows that are cut by the frame's edge or unaligned: byte stores by the pixel's own lane
    const int py = lane / tw, pxl = lane % tw;
    const int64_t prow = row0 + py, pcol = col0 + pxl;
    uint8_t* pd = out + 3 * (prow * W + col0);
    const bool pwhole = col0 + tw <= W && (reinterpret_cast<uintptr_t>(pd) & 3) == 0;
    if (lane < tw * th && prow < nrows && pcol < W && !pwhole) {
        pd[3 * pxl] = px[0];
        pd[3 * pxl + 1] = px[1];
        pd[3 * pxl + 2] = px[2];
    }
}

// Depth 0: primary-ray generation (camera.py:51-85) fused with the trace step.  A wave takes
// ppw = 64 / G consecutive pixels of the pass: lane l traces pixel l % ppw through the samples of
// its sample group l / ppw (G = P.pix_groups, a power of two; G > 1 gives a small frame -- one GPU's
// shard of a multi-GPU frame -- enough threads to fill the GPU).  A pixel's colour is summed in the
// thread (PixAcc), its groups combined by lane shuffles, and its lane of group 0 stores the pixel:
// no framebuffer atomics, no memset.  FUSE (single-child scenes): every depth of the sample's path
// is traced in the thread too (no ray queues), and a single-pass frame resolves the pixel here
// (P.fuse_resolve: average, sRGB, uint8; no framebuffer at all).  Otherwise the children are appended
// to the depth-1 queue for k_trace.
template <uint32_t MATS, int OCC = 2, bool FUSE = false>
__global__ __launch_bounds__(BLOCK, OCC) void k_primary(TraceParams P0) {
    constexpr bool LEAN = false, LANE_STATS = false;
#include "rt_primary_body.inc"
}

// The lean form of the fused paths of single-child scenes without a BVH, for pipelined frames (the
// headline's kernel; a synchronous frame has no generation beside it and takes k_primary<.., true>):
// built to 160 VGPRs instead of the 168 of 3 waves/SIMD (amdgpu_num_vgpr counts half the unified
// VGPR+AGPR file on gfx950), so three trace waves leave 32 registers per SIMD -- room for one
// four-wave generator workgroup of the next frames' numpy stream (mt_gen_nt: 256 threads, one wave per
// SIMD) beside them instead of it waiting for a trace wave to end -- and reading the camera coordinates
// and jitter per sample (LEAN), which holds its spills to the 168-VGPR build's.  Same box, ex1 1080p d5
// 6 spp pipelined frames 0.901 -> 0.876 ms; the kernel alone (device-resident frames) 0.752 -> 0.762
// (profiles/r05_lean_primary_ab.txt).
// LANE_STATS: the instantiation srt_debug_lane_stats selects (the counting cost 2 spilled VGPRs as a
// run-time branch in the default kernels).
template <uint32_t MATS, int OCC, bool LANE_STATS = false>
__global__ __launch_bounds__(BLOCK, OCC) __attribute__((amdgpu_num_vgpr(80))) void k_primary_lean(TraceParams P0) {
    constexpr bool FUSE = true, LEAN = true;
#include "rt_primary_body.inc"
}

// Depth d >= 1: blocks b, b + NSHARD, ... drain input shard b % NSHARD and append to output shard
// b % NSHARD.
template <uint32_t MATS, int OCC = 2, bool CHAIN = false>
__global__ __launch_bounds__(BLOCK, OCC) void k_trace(TraceParams P0) {
    const TraceParams& P = P0;
    const uint32_t shard = blockIdx.x % NSHARD;
    const int64_t n = min((int64_t)P.cnt_in[shard], P.seg);
    const int64_t blk = blockIdx.x / NSHARD, nblk = gridDim.x / NSHARD;
    if (blk * BLOCK >= n) return;  // nothing in this block's part of the shard (block-uniform)
    stage_luts(P);
    uint32_t err = 0;
    uint32_t shadow = 0;
    const int64_t off = (int64_t)shard * P.seg;
    for (int64_t base = blk * BLOCK; base < n; base += nblk * BLOCK) {
        const int64_t i = base + threadIdx.x;
        const bool active = i < n;
        Ray r;
        RT_T0(tq0);
        if (active) {
            r = queue_load(P.qin, off + i);
        } else {
            r.o = r.d = r.w = d3{0.0, 0.0, 0.0};
            r.pix = 0; r.meta = 0; r.path = 0;
        }
        RT_ACC(13, tq0);
        RT_T0(tt1);
        if (!CHAIN) {
            trace_one<MATS>(P, r, active, err, nullptr, GpuEmit{P, r, shard, 0u, &shadow, nullptr});
        } else {
            // the rest of each ray's path in this thread: lanes advance one depth per iteration, so
            // the live lanes of an iteration share a depth (counted per wave into the shard's
            // counter of that depth, as the queue appends would have)
            bool live = active;
            int d = P.depth;
            for (;;) {
                Ray nx = r;
                bool has = false;
                trace_one<MATS>(P, r, live, err, nullptr, ChainEmit{P, r, 0u, &shadow, &nx, &has});
                live = live && has;
                r = nx;
                ++d;
                const uint64_t m = __ballot(live);
                if (m == 0) break;
                if (live && lanes_below(m) == 0 && d < SRT_MAX_DEPTHS)  // the lowest live lane
                    atomicAdd(P.cnt_out + (int64_t)(d - P.depth - 1) * NSHARD + shard, (uint32_t)__builtin_popcountll(m));
                if (d > P.dcap) break;  // counted (the host reports rays beyond the cap), not traced
            }
        }
        RT_ACC(14, tt1);
    }
    if (err) atomicOr(&P.flags[0], err);
    if (shadow) atomicAdd(P.shadow, (unsigned long long)shadow);
}

// srt_shade's first depth: each queued ray shaded at the caller's hit (Material.get_color,
// material.py:42-44), its children appended for the ordinary k_trace depths
template <uint32_t MATS>
__global__ __launch_bounds__(BLOCK) void k_shade_forced(TraceParams P0) {
    const TraceParams& P = P0;
    const uint32_t shard = blockIdx.x % NSHARD;
    const int64_t n = min((int64_t)P.cnt_in[shard], P.seg);
    const int64_t blk = blockIdx.x / NSHARD, nblk = gridDim.x / NSHARD;
    if (blk * BLOCK >= n) return;
    stage_luts(P);
    uint32_t err = 0;
    uint32_t shadow = 0;
    const int64_t off = (int64_t)shard * P.seg;
    for (int64_t base = blk * BLOCK; base < n; base += nblk * BLOCK) {
        const int64_t i = base + threadIdx.x;
        const bool active = i < n;
        Ray r;
        if (active) {
            r = queue_load(P.qin, off + i);
        } else {
            r.o = r.d = r.w = d3{0.0, 0.0, 0.0};
            r.pix = 0; r.meta = 0; r.path = 0;
        }
        trace_one<MATS, GpuEmit, true>(P, r, active, err, nullptr, GpuEmit{P, r, shard, 0u, &shadow, nullptr});
    }
    if (err) atomicOr(&P.flags[0], err);
    if (shadow) atomicAdd(P.shadow, (unsigned long long)shadow);
}

// ---- the frame kernel ----------------------------------------------------------------------
// One wave (a 64-thread block) owns a tile of 64 consecutive pixels and traces their whole ray
// trees: it generates the tile's primary rays sample by sample, appends every child to a private
// ring in HBM and drains the ring in FIFO order, taking a full 64-ray chunk whenever one is
// pending and new primaries otherwise.  Colours go to per-pixel accumulators in LDS; at the end
// the wave writes (or resolves) its 64 pixels.  No atomics between waves, no per-depth launches:
// the depth tails of different tiles overlap on the GPU instead of serialising kernel after
// kernel, and all samples of a pixel are queued together, which keeps lanes ~95 % busy
// (simulated on the ex1 1080p path-length distribution: 94.6 % with pure chunks).
constexpr int FRAME_BLOCK = 64;

struct FrameLds {
    double acc[3][FRAME_BLOCK];  // per-pixel colour sums of the tile
    uint32_t depth_cnt[SRT_MAX_DEPTHS];
    uint32_t head, tail;         // ring positions (wave-uniform; kept in LDS so that updates made
                                 // under divergent control flow are seen by every lane)
    uint32_t head1, tail1;       // (FRAME_SPLIT) the second ring's: rays travelling inside a medium
    uint32_t slot;
    uint32_t overflow;
};

// The ring positions are shared by the wave's lanes through LDS.  Plain loads/stores would let the
// compiler forward a lane's own earlier value past another lane's update (a data race under the
// single-thread model), so every access is an atomic at workgroup scope and the reserving lane's
// result is broadcast with a cross-lane read.
__device__ __forceinline__ uint32_t lds_get(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// k_frame's tile: 8 x 8 pixels of the pass or 64 consecutive ones of a row; the tile's first pixel is
// tile0, and the LDS accumulator of pixel tile0 + d is the lane that owns it.  A square tile's rays
// stay coherent deeper (fewer chunks mix colliders): same box, ex3 1080p d8 frame 2.755 -> 2.605 ms,
// cornell 800x800 512 spp 4006 -> 3939 ms, but the thin-film example4 4K 13.95 -> 14.09 ms, so the
// thin-film variants keep rows (profiles/r06_frame_tile_ab.txt).
constexpr bool frame_tile_for(uint32_t mats) { return (mats & mat_bit(SRT_THINFILM)) == 0; }
// k_frame's ring split in two halves for the refractive variants without thin films or Diffuse: rays
// travelling inside a medium (which next hit the body they are in) in one, the rest in the other, so
// that a chunk of the first shades one collider in one pass of the material waterfall: ex3 1080p d8
// frame 2.647 -> 2.552 ms, k_frame 2.86 -> 2.65 ms; the thin-film example4 4K 13.53 -> 14.04 ms, and
// cornell's Diffuse fan-out overflows half a ring (profiles/r06_frame_split_ab.txt)
constexpr bool frame_split_for(uint32_t mats) {
    return (mats & mat_bit(SRT_REFRACTIVE)) != 0 && (mats & (mat_bit(SRT_THINFILM) | mat_bit(SRT_DIFFUSE))) == 0;
}
// k_frame's rings drained newest first (a stack: the chunk taken is the last 64 rays pushed, usually
// the children of the chunk just traced, still in L2) for the thin-film variants (ex4 4K frame 13.83 ->
// 13.58 ms) and the split-ring ones (ex3 1080p d8, same box: frame 2.55-2.58 -> 2.45-2.47 ms,
// device-resident 2.41-2.43 -> 2.14-2.18 ms, profiles/r06_frame_split_lifo_ab.txt; before the split,
// one FIFO-or-stack ring gave ex3 no change); oldest first for the rest (cornell's Diffuse fan-out
// outgrows a stack's ring: 4.02 -> 5.24 s; profiles/r06_rejected_frame_lifo.txt)
constexpr bool frame_lifo_for(uint32_t mats) {
    return (mats & mat_bit(SRT_THINFILM)) != 0 || frame_split_for(mats);
}
__device__ __forceinline__ uint32_t frame_tile_index(bool tiled, uint32_t d, uint32_t W) {
    if (!tiled) return d;
    const uint32_t ly = d / W;
    return ly * 8u + (d - ly * W);
}
inline int64_t frame_tiles(bool tiled, int64_t W, int64_t nrows) {
    return tiled ? ((W + 7) / 8) * ((nrows + 7) / 8) : (W * nrows + FRAME_BLOCK - 1) / FRAME_BLOCK;
}

struct FrameEmit {
    const TraceParams& P;
    const Ray& r;
    uint32_t round;
    uint32_t* shadow_acc;
    FrameLds* L;
    uint32_t tile0;
    int64_t ring_base;
    bool tiled;  // (k_frame's FRAME_TILE)
    bool split;  // (k_frame's FRAME_SPLIT) rays inside a medium (child medium != 0) go to ring 1

    __device__ void local(d3 c) const {
        if (is_zero(c)) return;
        const uint32_t k = frame_tile_index(tiled, r.pix - tile0, (uint32_t)P.cam.width);
        __hip_atomic_fetch_add(&L->acc[0][k], r.w.x * c.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&L->acc[1][k], r.w.y * c.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&L->acc[2][k], r.w.z * c.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ void shadow(int n) const { *shadow_acc += (uint32_t)n; }
    // `cnt` consecutive ring positions for every active lane (wave-local: LDS counter, no atomics)
    __device__ uint32_t reserve(uint32_t cnt) const {
        uint32_t total = 0, below = 0;
        for (int b = 0; b < 8; ++b) {
            uint64_t m = __ballot((cnt >> b) & 1u);
            total += (uint32_t)__builtin_popcountll(m) << b;
            below += lanes_below(m) << b;
        }
        const uint64_t act = __ballot(1);
        const int leader = __builtin_ctzll(act);
        uint32_t base = 0;
        if (lanes_below(act) == 0)
            base = __hip_atomic_fetch_add(&L->tail, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        base = (uint32_t)__shfl((int)base, leader);
        return base + below;
    }
    // ring q (split: half the slot each) at its position pos
    __device__ void store(uint32_t pos, const Child& c, uint32_t path, int q = 0) const {
        const uint32_t depth = meta_depth(r.meta) + 1;
        const uint32_t cap = split ? (uint32_t)P.ring_cap >> 1 : (uint32_t)P.ring_cap;
        if (pos - lds_get(q ? &L->head1 : &L->head) >= cap) {  // ring full: the frame is re-rendered with bigger rings
            lds_put(&L->overflow, 1u);
            return;
        }
        queue_store(P.ring, ring_base + (int64_t)(q ? cap : 0u) + (int64_t)(pos & (cap - 1u)), c.o, c.d, mul(r.w, c.w),
                    r.pix, pack_meta(c.medium, depth, c.dfl), path);
    }
    __device__ void child(const Child& c) const {
        if (!split) {
            store(reserve(1u), c, child_path(r.path, c.slot, round));
            return;
        }
        // a ray inside a medium (a refractive body: it next hits that body from inside) to ring 1, the
        // rest to ring 0, so that chunks of ring 1 shade one collider in one waterfall pass
        const bool in = c.medium != 0u;
        const uint64_t m1 = __ballot(in), m0 = __ballot(!in), act = __ballot(1);
        const int leader = __builtin_ctzll(act);
        uint32_t b0 = 0, b1 = 0;
        if (lanes_below(act) == 0) {
            if (m0) b0 = __hip_atomic_fetch_add(&L->tail, (uint32_t)__builtin_popcountll(m0), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
            if (m1) b1 = __hip_atomic_fetch_add(&L->tail1, (uint32_t)__builtin_popcountll(m1), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        b0 = (uint32_t)__shfl((int)b0, leader);
        b1 = (uint32_t)__shfl((int)b1, leader);
        store(in ? b1 + lanes_below(m1) : b0 + lanes_below(m0), c, child_path(r.path, c.slot, round), in ? 1 : 0);
    }
    // the fan-out child-major in the ring (as GpuEmit::diffuse): the k-th children of the lanes are
    // consecutive, every store a coalesced run.  Lane-major positions scattered each store over 64
    // cache lines and doubled the ring's HBM writes (cornell k_frame: 309 GB written per pass for
    // 143 GB of rays, PMC WRITE_SIZE)
    __device__ void diffuse(const DiffuseGen& g, int mi) const {
        const uint32_t cnt = (uint32_t)g.count;
        const uint32_t base = reserve(cnt) - wave_below(cnt);
        const auto& m = P.S.mat[mi];
        uint32_t off = 0;
        for (uint32_t k = 0;; ++k) {
            const uint64_t mk = __ballot(cnt > k);
            if (!mk) break;
            if (cnt > k) {
                Rng rng;
                const uint32_t cpath = child_path(r.path, 0x100u + k, round);
                rng.init(P.seed, key_pix(P, r.pix), cpath, 0xD1000000u | meta_depth(r.meta));
                store(base + off + lanes_below(mk), diffuse_child(P.S, m, g, rng, k), cpath);
            }
            off += (uint32_t)__builtin_popcountll(mk);
        }
    }
};

template <uint32_t MATS, int OCC = 2>
__global__ __launch_bounds__(FRAME_BLOCK, OCC) void k_frame(TraceParams P0) {
    constexpr bool FRAME_TILE = frame_tile_for(MATS), FRAME_LIFO = frame_lifo_for(MATS);
    constexpr bool FRAME_SPLIT = frame_split_for(MATS);
    const TraceParams& P = P0;
    {
        const int nl = P.S.nlut_lds;
        for (int i = threadIdx.x; i < nl * 256; i += FRAME_BLOCK) rt_lds_dyn[i] = P.S.tex[i >> 8].lut[i & 255];
    }
    __shared__ FrameLds L;
    RT_T0(tf0);
    const uint32_t lane = threadIdx.x;
    for (int k = 0; k < 3; ++k) L.acc[k][lane] = 0.0;
    for (int d = lane; d < SRT_MAX_DEPTHS; d += FRAME_BLOCK) L.depth_cnt[d] = 0u;
    if (lane == 0) {
        // a free ring: slots are tried from blockIdx on; there are twice as many as resident waves
        uint32_t s = blockIdx.x % (uint32_t)P.nslot;
        while (atomicCAS(&P.ring_lock[s], 0u, 1u) != 0u) s = (s + 1u) % (uint32_t)P.nslot;
        L.slot = s;
        L.head = 0u;
        L.tail = 0u;
        L.head1 = 0u;
        L.tail1 = 0u;
        L.overflow = 0u;
    }
    __syncthreads();
    RT_ACC(18, tf0);
    const uint32_t tile = blockIdx.x % (uint32_t)P.ntiles, grp = blockIdx.x / (uint32_t)P.ntiles;
    const uint32_t Wc = (uint32_t)P.cam.width, nrows = (uint32_t)(P.npix / P.cam.width);
    const uint32_t tiles_x = (Wc + 7u) >> 3, ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const uint32_t tile0 = FRAME_TILE ? (ty * 8u) * Wc + tx * 8u : tile * FRAME_BLOCK;
    const int spg = (P.spp + P.groups - 1) / P.groups;
    const int s_end = min(P.spp, (int)(grp + 1) * spg);
    const int64_t ring_base = (int64_t)L.slot * P.ring_cap;
    const uint32_t shard = blockIdx.x % NSHARD;
    uint32_t err = 0;
    uint32_t shadow = 0;
    // this lane's pixel of the tile
    uint32_t p, lr, col;
    bool pact;
    if (FRAME_TILE) {
        const uint32_t r = ty * 8u + (lane >> 3), cx = tx * 8u + (lane & 7u);
        pact = r < nrows && cx < Wc;
        lr = pact ? r : 0u;
        col = pact ? cx : 0u;
        p = pact ? lr * Wc + col : tile0;
    } else {
        p = tile0 + lane;
        pact = p < (uint32_t)P.npix;
        lr = pact ? p / (uint32_t)P.cam.width : 0u;
        col = pact ? p - lr * (uint32_t)P.cam.width : 0u;
    }
    const int grow = pact ? P.rows[lr] : 0;
    const double xc = pact ? P.cam.xs[col] : 0.0, yr = pact ? P.cam.ys[grow] : 0.0;
    const uint32_t gpix = (uint32_t)grow * (uint32_t)P.cam.width + col;
    const Quot qw((double)P.cam.width), qh((double)P.cam.height);
    int s_next = (int)grp * spg;
    const uint32_t rcap = FRAME_SPLIT ? (uint32_t)P.ring_cap >> 1 : (uint32_t)P.ring_cap;  // rays per ring
    for (;;) {
        const uint32_t head0 = lds_get(&L.head), tail0 = lds_get(&L.tail);
        const uint32_t head1 = FRAME_SPLIT ? lds_get(&L.head1) : 0u, tail1 = FRAME_SPLIT ? lds_get(&L.tail1) : 0u;
        const uint32_t pend0 = tail0 - head0, pend1 = tail1 - head1;
        if (pend0 == 0u && pend1 == 0u && s_next >= s_end) break;
        // a ring overflowed: the frame is re-rendered with bigger rings, and the positions past the
        // overflow hold no rays of this launch
        if (lds_get(&L.overflow)) break;
        // the ring a chunk comes from: the fuller of two full chunks (ring 1 on a tie), else the one
        // holding a full chunk, else (primaries done) ring 1 then ring 0
        const int q = pend1 >= (uint32_t)FRAME_BLOCK ? (pend1 >= pend0 ? 1 : 0)
                                                     : (pend0 < (uint32_t)FRAME_BLOCK && pend1 > 0u ? 1 : 0);
        const uint32_t head = q ? head1 : head0, tail = q ? tail1 : tail0, pending = q ? pend1 : pend0;
        Ray r;
        bool active;
        uint32_t depth = 0;
        int32_t* hs = nullptr;
        if (pending >= (uint32_t)FRAME_BLOCK || s_next >= s_end) {
            // a chunk of the ring: its oldest rays, or (FRAME_LIFO) its newest, whose children are then
            // pushed over them (their stores follow every lane's loads: the loaded rays are read first)
            const uint32_t take = min(pending, (uint32_t)FRAME_BLOCK);
            active = lane < take;
            RT_T0(tl0);
            const uint32_t first = FRAME_LIFO ? tail - take : head;
            if (active) {
                r = queue_load(P.ring, ring_base + (int64_t)(q ? rcap : 0u) + (int64_t)((first + lane) & (rcap - 1u)));
                depth = meta_depth(r.meta);
            } else {
                r.o = r.d = r.w = d3{0.0, 0.0, 0.0};
                r.pix = tile0; r.meta = 0; r.path = 0;
            }
            if (lane == 0) {
                if (FRAME_LIFO)
                    lds_put(q ? &L.tail1 : &L.tail, first);
                else
                    lds_put(q ? &L.head1 : &L.head, head + take);
            }
            RT_ACC(16, tl0);
        } else {
            // primary rays of sample s_next for the tile's pixels (camera.py:51-85)
            const int s = s_next++;
            active = pact;
            r.o = r.d = d3{0.0, 0.0, 0.0};
            r.w = d3{1.0, 1.0, 1.0};
            r.meta = pack_meta(0, 0, 0);
            r.pix = pact ? p : tile0;
            r.path = mix32(0x5EED0000u, (uint32_t)(P.sample_base + s));
            RT_T0(tg0);
            if (active) {
                double j[4] = {0.0, 0.0, 0.0, 0.0};
                primary_uniforms(P, s, p, gpix, j);
                primary_ray(P.cam, qw, qh, xc, yr, j, r.o, r.d);
            }
            RT_ACC(15, tg0);
            if (P.hit_out && active) hs = P.hit_out + (int64_t)s * P.npix + p;
        }
        // rays entering each depth; a ray beyond the depth cap is counted (the host reports it as an
        // error) and dropped, so every ring drains
        if (active) {
            __hip_atomic_fetch_add(&L.depth_cnt[min(depth, (uint32_t)SRT_MAX_DEPTHS - 1u)], 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((int)depth > P.dcap) active = false;
        }
        RT_T0(tt2);
        trace_one<MATS>(P, r, active, err, hs, FrameEmit{P, r, 0u, &shadow, &L, tile0, ring_base, FRAME_TILE, FRAME_SPLIT});
        RT_ACC(17, tt2);
    }
    RT_T0(te0);
    // tile pixels out
    if (P.fuse_resolve) {
        uint8_t px[3] = {0, 0, 0};
        if (pact) {
            const double spp = (double)P.spp_total;
            double rr = L.acc[0][lane] / spp, gg = L.acc[1][lane] / spp, bb = L.acc[2][lane] / spp;
            double a0, a1, a2;
            resolve_pixel(rr, gg, bb, a0, a1, a2, px);
            if (P.out_rgb) { P.out_rgb[p] = rr; P.out_rgb[P.npix + p] = gg; P.out_rgb[2 * P.npix + p] = bb; }
        }
        if (P.out_u8) {
            if (FRAME_TILE) {
                store_u8_tile(P.out_u8, px, lane, 8, 8, (int64_t)(ty * 8u), (int64_t)(tx * 8u), (int64_t)Wc, (int64_t)nrows);
            } else {
                const int64_t p0 = p - lane;
                store_u8_chunk(P.out_u8 + 3 * p0, px, lane, (int)min<int64_t>(64, P.npix - p0));
            }
        }
    } else if (pact && P.groups > 1) {
        double* part = P.fbg + (int64_t)grp * 3 * P.npix;
        part[p] = L.acc[0][lane]; part[P.npix + p] = L.acc[1][lane]; part[2 * P.npix + p] = L.acc[2][lane];
    } else if (pact) {
        const double ar = L.acc[0][lane], ag = L.acc[1][lane], ab = L.acc[2][lane];
        if (P.fb_first) {
            P.fb[p] = ar; P.fb[P.npix + p] = ag; P.fb[2 * P.npix + p] = ab;
        } else {
            P.fb[p] += ar; P.fb[P.npix + p] += ag; P.fb[2 * P.npix + p] += ab;
        }
    }
    __syncthreads();
    for (int d = lane; d <= P.dcap + 1 && d < SRT_MAX_DEPTHS; d += FRAME_BLOCK)
        if (L.depth_cnt[d]) atomicAdd(P.cnt_out + (int64_t)d * NSHARD + shard, L.depth_cnt[d]);
    if (err) atomicOr(&P.flags[0], err);
    if (lane == 0 && lds_get(&L.overflow)) atomicOr(&P.flags[1], RETRY_OVERFLOW);
    // the wave's shadow-ray count into its shard's counter
    for (int off = 32; off > 0; off >>= 1) shadow += __shfl_xor(shadow, off);
    if (lane == 0) {
        if (shadow) atomicAdd(P.shadow + shard, (unsigned long long)shadow);
        __threadfence();
        atomicExch(&P.ring_lock[L.slot], 0u);
    }
    RT_ACC(19, te0);
}

// Kernel variants by the material types they contain; the host picks the first covering the scene.
constexpr uint32_t MATS_GLOSSY_SKY = mat_bit(SRT_GLOSSY) | mat_bit(SRT_SKY);
constexpr uint32_t MATS_DIELECTRIC = MATS_GLOSSY_SKY | mat_bit(SRT_REFRACTIVE) | mat_bit(SRT_EMISSIVE);
constexpr uint32_t MATS_FILM = mat_bit(SRT_THINFILM) | mat_bit(SRT_SKY) | mat_bit(SRT_GLOSSY);
constexpr uint32_t MATS_MC = mat_bit(SRT_DIFFUSE) | mat_bit(SRT_EMISSIVE) | mat_bit(SRT_REFRACTIVE);
struct Variant {
    uint32_t mats;
    void (*primary)(TraceParams);
    void (*trace)(TraceParams);
    void (*frame)(TraceParams);
    void (*chain)(TraceParams);
    void (*fused)(TraceParams) = nullptr;  // k_primary<.., FUSE>: whole single-child paths per pixel
    // k_primary_lean (160 VGPRs): the fused paths of pipelined frames, whose numpy-stream generators
    // then run beside them (mt_gen_launch); synchronous frames take `fused`
    void (*lean)(TraceParams) = nullptr;
    void (*lean_stats)(TraceParams) = nullptr;  // k_primary_lean<.., LANE_STATS> (srt_debug_lane_stats)
};
// The trace kernels are built for RT_OCC = 3 waves/SIMD.  Same-box A/B against 2 waves/SIMD
// (profiles/r03_occ_ab.txt): device-resident ex1 1080p 1.22 -> 1.10 ms, ex3 k_frame 3.36 -> 3.06 ms,
// ex4 4K 14.5 -> 13.2 ms, cornell 4.87 -> 4.05 s, mesh 12.2 -> 10.2 ms.
#ifndef RT_OCC
#define RT_OCC 3
#endif
constexpr int OCC = RT_OCC;  // waves/SIMD the trace kernels are built for (register cap 512 / OCC)
#ifndef RT_FUSE_OCC
#define RT_FUSE_OCC 3  // waves/SIMD of the fused k_primary (168 VGPRs; its spills: DESIGN.md §3)
#endif
#ifndef RT_BVH_LDS_STACK
#define RT_BVH_LDS_STACK 1  // the BVH variants' traversal stacks start in LDS (rt_device.h BvhStack)
#endif
constexpr uint32_t LDS_STK = RT_BVH_LDS_STACK ? MAT_LDS_STACK : 0u, LDS_STK_FRAME = RT_BVH_LDS_STACK ? MAT_LDS_STACK | MAT_LDS_NARROW : 0u;
#ifndef RT_MESH_FUSE_OCC
#define RT_MESH_FUSE_OCC RT_FUSE_OCC  // the glossy BVH variant's fused k_primary
#endif
constexpr uint32_t MATS_MESH = MATS_GLOSSY_SKY | MAT_TRI | MAT_BVH;  // a glossy TriangleMesh in the ex1 setting
const Variant VARIANTS[] = {
    {MATS_GLOSSY_SKY, k_primary<MATS_GLOSSY_SKY, OCC>, k_trace<MATS_GLOSSY_SKY, OCC>, k_frame<MATS_GLOSSY_SKY, OCC>, k_trace<MATS_GLOSSY_SKY, OCC, true>,
     k_primary<MATS_GLOSSY_SKY, RT_FUSE_OCC, true>, k_primary_lean<MATS_GLOSSY_SKY, RT_FUSE_OCC>,
     k_primary_lean<MATS_GLOSSY_SKY, RT_FUSE_OCC, true>},
#ifndef RT_EXP_MIN  // (register-usage experiments, tools/resource_usage.py: the headline variants only, a quicker compile)
    {MATS_DIELECTRIC, k_primary<MATS_DIELECTRIC, OCC>, k_trace<MATS_DIELECTRIC, OCC>, k_frame<MATS_DIELECTRIC, OCC>, k_trace<MATS_DIELECTRIC, OCC, true>},
    {MATS_FILM, k_primary<MATS_FILM, OCC>, k_trace<MATS_FILM, OCC>, k_frame<MATS_FILM, OCC>, k_trace<MATS_FILM, OCC, true>},
    {MATS_MC, k_primary<MATS_MC, OCC>, k_trace<MATS_MC, OCC>, k_frame<MATS_MC, OCC>, k_trace<MATS_MC, OCC, true>},
    // a glossy TriangleMesh in the ex1 setting (the mesh bench): the BVH traversal, no other features
    {MATS_MESH, k_primary<MATS_MESH | LDS_STK, OCC>, k_trace<MATS_MESH | LDS_STK, OCC>, k_frame<MATS_MESH | LDS_STK_FRAME, OCC>,
     k_trace<MATS_MESH | LDS_STK, OCC, true>, k_primary<MATS_MESH | LDS_STK, RT_MESH_FUSE_OCC, true>},
    {MAT_GENERIC, k_primary<MAT_GENERIC, OCC>, k_trace<MAT_GENERIC, OCC>, k_frame<MAT_GENERIC, OCC>,
     k_trace<MAT_GENERIC, OCC, true>},
    // scenes with a triangle BVH (TriangleMesh)
    {MAT_GENERIC | MAT_BVH, k_primary<MAT_GENERIC | MAT_BVH | LDS_STK, OCC>, k_trace<MAT_GENERIC | MAT_BVH | LDS_STK, OCC>,
     k_frame<MAT_GENERIC | MAT_BVH | LDS_STK_FRAME, OCC>, k_trace<MAT_GENERIC | MAT_BVH | LDS_STK, OCC, true>},
#endif
};
// Variants for scenes of a given collider sequence (rt_device.h seq_of: the colliders intersected in
// straight-line code); a scene runs one when its colliders have exactly these types in this order
// and its materials are covered.
#ifndef RT_NO_SEQ_VARIANTS
#define RT_SEQ_VARIANTS
#endif
#ifdef RT_SEQ_VARIANTS
constexpr uint32_t seq_bits(std::initializer_list<int> t) {
    uint32_t q = (uint32_t)t.size();
    int k = 0;
    for (int v : t) q |= (uint32_t)v << (4 + 2 * k++);
    return q << SEQ_SHIFT;
}
// example1 / the headline: two spheres, a plane, the sky box (same box, ex1 1080p d5 6 spp: device-
// resident frame 0.837 -> 0.750 ms, k_primary 1.05 -> 0.95 ms; profiles/r05_collider_seq_ab.txt)
constexpr uint32_t MATS_SEQ_SSPC = MATS_GLOSSY_SKY | seq_bits({SRT_SPHERE, SRT_SPHERE, SRT_PLANE, SRT_CUBOID});
// the branching scenes of two other BASELINE configs, whose frames run k_frame: example3 (floor, glass
// cuboid, sky box; same box, ex3 1080p d8 frame 2.81 -> 2.73 ms, k_frame 2.94 -> 2.82 ms) and example4
// (thin-film sphere, sky box; 4K frame 14.08 -> 13.96 ms), profiles/r06_collider_seq_frame_ab.txt.  The
// cornell box's eight colliders in sequence were 1.7 % slower (4024 -> 4092 ms), so it keeps the loop.
constexpr uint32_t MATS_SEQ_PCC = MATS_DIELECTRIC | seq_bits({SRT_PLANE, SRT_CUBOID, SRT_CUBOID});
constexpr uint32_t MATS_SEQ_SC = MATS_FILM | seq_bits({SRT_SPHERE, SRT_CUBOID});
#define RT_SEQ_FRAME_VARIANT(M) {M, k_primary<M, OCC>, k_trace<M, OCC>, k_frame<M, OCC>, k_trace<M, OCC, true>}
const Variant SEQ_VARIANTS[] = {
    {MATS_SEQ_SSPC, k_primary<MATS_SEQ_SSPC, OCC>, k_trace<MATS_SEQ_SSPC, OCC>, k_frame<MATS_SEQ_SSPC, OCC>,
     k_trace<MATS_SEQ_SSPC, OCC, true>, k_primary<MATS_SEQ_SSPC, RT_FUSE_OCC, true>, k_primary_lean<MATS_SEQ_SSPC, RT_FUSE_OCC>,
     k_primary_lean<MATS_SEQ_SSPC, RT_FUSE_OCC, true>},
#ifndef RT_EXP_MIN
    RT_SEQ_FRAME_VARIANT(MATS_SEQ_PCC),
    RT_SEQ_FRAME_VARIANT(MATS_SEQ_SC),
#endif
};
#endif
const Variant& pick_variant(uint32_t mats, uint32_t seq = 0) {
#ifdef RT_SEQ_VARIANTS
    if (seq)
        for (const Variant& v : SEQ_VARIANTS)
            if (seq_of(v.mats) == seq && (v.mats & mats) == mats) return v;
#endif
    for (const Variant& v : VARIANTS)
        if ((v.mats & mats) == mats) return v;
    return VARIANTS[sizeof(VARIANTS) / sizeof(VARIANTS[0]) - 1];
}

// End of a pass (one block): hand the per-depth append counters and the error/overflow flags to
// the host through pinned memory and zero them for the next pass (replaces two memsets and two
// copies per pass; the frame's stream needs no host round trip until its end).
__global__ __launch_bounds__(BLOCK) void k_pass_end(uint32_t* counts, int64_t words, uint32_t* flags,
                                                   uint32_t* host, uint32_t* host_flags) {
    for (int64_t i = threadIdx.x; i < words; i += BLOCK) {
        host[i] = counts[i];
        counts[i] = 0u;
    }
    if (threadIdx.x < 2) {
        host_flags[threadIdx.x] |= flags[threadIdx.x];  // accumulated until the host checks them
        flags[threadIdx.x] = 0u;
    }
}

__global__ __launch_bounds__(BLOCK) void k_resolve(const double* fb, const unsigned long long* fbx, int64_t npix,
                                                  unsigned long long* shadow,
                                                  uint32_t* shadow_host, double spp, double* rgb, uint8_t* u8,
                                                  uint32_t* counts, int64_t words, uint32_t* flags, uint32_t* host,
                                                  uint32_t* host_flags) {
    // block 0 also ends the last pass (the work of k_pass_end, one launch less per frame)
    if (blockIdx.x == 0 && words > 0) {
        for (int64_t i = threadIdx.x; i < words; i += BLOCK) {
            host[i] = counts[i];
            counts[i] = 0u;
        }
        if (threadIdx.x < 2) {
            host_flags[threadIdx.x] |= flags[threadIdx.x];
            flags[threadIdx.x] = 0u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        // the frame's shadow-ray count (NSHARD counters) to the host, zeroed for the next frame (no
        // kernel of this frame adds to them any more): wave 0 reads them in parallel and reduces
        // across lanes
        unsigned long long v = 0;
        for (int k = threadIdx.x; k < NSHARD; k += 64) {
            v += shadow[k];
            shadow[k] = 0ull;
        }
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (threadIdx.x == 0) {
            shadow_host[0] = (uint32_t)v;
            shadow_host[1] = (uint32_t)(v >> 32);
        }
    }
    // wave-uniform trip count: each wave takes 64 consecutive pixels per step
    const int lane = threadIdx.x & 63;
    for (int64_t p0 = (int64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63); p0 < npix; p0 += (int64_t)gridDim.x * BLOCK) {
        const int64_t p = p0 + lane;
        const int n = (int)min<int64_t>(64, npix - p0);
        uint8_t px[3] = {0, 0, 0};
        if (p < npix) {
            double r, g, b;
            if (fbx) {  // every contribution as a fixed-point term (order-independent sums)
                r = fx_value(fbx, npix, 0, p);
                g = fx_value(fbx, npix, 1, p);
                b = fx_value(fbx, npix, 2, p);
                if (fx_suspect(fbx, npix, p)) shadow_host[2] = RETRY_FIXED_RANGE;  // render again with f64
            } else {
                r = fb[p];
                g = fb[npix + p];
                b = fb[2 * npix + p];
            }
            r /= spp;
            g /= spp;
            b /= spp;
            double a0, a1, a2;
            resolve_pixel(r, g, b, a0, a1, a2, px);
            if (rgb) { rgb[p] = r; rgb[npix + p] = g; rgb[2 * npix + p] = b; }
        }
        if (u8) store_u8_chunk(u8 + 3 * p0, px, lane, n);
    }
}

// fb += the fixed-point sums (srt_trace's colours)
__global__ __launch_bounds__(BLOCK) void k_fx_combine(double* fb, const unsigned long long* fbx, int64_t npix,
                                                     uint32_t* flags) {
    bool bad = false;
    for (int64_t p = (int64_t)blockIdx.x * BLOCK + threadIdx.x; p < npix; p += (int64_t)gridDim.x * BLOCK) {
        for (int ch = 0; ch < 3; ++ch) fb[ch * npix + p] += fx_value(fbx, npix, ch, p);
        bad |= fx_suspect(fbx, npix, p);
    }
    if (bad) atomicOr(flags + 1, RETRY_FIXED_RANGE);
}

// the sample groups' partial sums of a frame-kernel pass into the framebuffer, in group order
__global__ __launch_bounds__(BLOCK) void k_fb_groups(double* fb, const double* fbg, int groups, int64_t npix, int first) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < 3 * npix; i += (int64_t)gridDim.x * BLOCK) {
        double v = fbg[i];
        for (int g = 1; g < groups; ++g) v += fbg[(int64_t)g * 3 * npix + i];
        fb[i] = first ? v : fb[i] + v;
    }
}

__global__ __launch_bounds__(BLOCK) void k_nearest(SceneView S, const double* O, const double* D, int64_t n, double* t,
                                                  int32_t* id, double* orient) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        d3 o = d3{O[i], O[n + i], O[2 * n + i]}, d = d3{D[i], D[n + i], D[2 * n + i]};
        double tn, on;
        bool ties;
        int c = nearest_hit(S, o, d, tn, on, ties);
        if (t) t[i] = tn;
        if (id) id[i] = c;
        if (orient) orient[i] = on;
    }
}

__global__ __launch_bounds__(BLOCK) void k_intersect_one(const srt_collider* c_generic, const double* O,
                                                        const double* D, int64_t n, double* out) {
    // generic pointer in the signature (kernel arguments stay in the global address space),
    // read through the constant address space inside
    const RT_RO srt_collider* c = (const RT_RO srt_collider*)c_generic;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        d3 o = d3{O[i], O[n + i], O[2 * n + i]}, d = d3{D[i], D[n + i], D[2 * n + i]};
        double orient;
        double t = collider_hit(*c, o, d, orient);
        out[i] = t;
        out[n + i] = orient;
    }
}

// Collider.get_Normal / get_uv and Primitive.get_uv at points P (the reference's per-hit plugin
// points, collider.py:12-17, sphere.py:54-64, plane.py:98-105, cuboid.py:142-187, skybox.py:29-32)
__global__ __launch_bounds__(BLOCK) void k_collider_surface(const srt_collider* c_generic, const double* P, int64_t n,
                                                           double* N, double* uv) {
    const RT_RO srt_collider* c = (const RT_RO srt_collider*)c_generic;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        const d3 p = d3{P[i], P[n + i], P[2 * n + i]};
        if (N) {
            const d3 v = collider_normal(*c, p);
            N[i] = v.x;
            N[n + i] = v.y;
            N[2 * n + i] = v.z;
        }
        if (uv) {
            double u = 0.0, v = 0.0;
            collider_uv(*c, p, u, v);
            uv[i] = u;
            uv[n + i] = v;
        }
    }
}

// Material.get_Normal(hit) (material.py:18-36) at points P: the collider's normal, or with a normal
// map the map's texel (texture 0 of S) through the collider's inverse_basis_matrix, normalised;
// times the hit orientation
__global__ __launch_bounds__(BLOCK) void k_material_normal(SceneView S, const srt_collider* c_generic,
                                                          const srt_material* m_generic, const double* P,
                                                          const double* orient, int64_t n, double* N,
                                                          uint32_t* flags) {
    const RT_RO srt_collider* c = (const RT_RO srt_collider*)c_generic;
    const RT_RO srt_material* m = (const RT_RO srt_material*)m_generic;
    uint32_t err = 0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        const d3 v = shading_normal(S, *c, *m, d3{P[i], P[n + i], P[2 * n + i]}, orient[i], err);
        N[i] = v.x;
        N[n + i] = v.y;
        N[2 * n + i] = v.z;
    }
    if (err) atomicOr(flags, err);
}

// image.get_color(hit): the texel of (u, v) through texture 0 of S (texture.py:27-39)
__global__ __launch_bounds__(BLOCK) void k_texture_lookup(SceneView S, const double* uv, int64_t n, double* rgb,
                                                         uint32_t* flags) {
    uint32_t err = 0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        const d3 c = tex_rgb(S, 0, uv[i], uv[n + i], err);
        rgb[i] = c.x;
        rgb[n + i] = c.y;
        rgb[2 * n + i] = c.z;
    }
    if (err) atomicOr(flags, err);
}

__global__ __launch_bounds__(BLOCK) void k_primary_rays(srt_camera cam, const double* J, int64_t n, double* O,
                                                       double* D) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        uint32_t row = (uint32_t)(i / cam.width), col = (uint32_t)(i - (int64_t)row * cam.width);
        double j[4] = {J[i], J[n + i], J[2 * n + i], J[3 * n + i]};
        d3 o, d;
        primary_ray(cam, cam.xs[col], cam.ys[row], j, o, d);
        O[i] = o.x; O[n + i] = o.y; O[2 * n + i] = o.z;
        D[i] = d.x; D[n + i] = d.y; D[2 * n + i] = d.z;
    }
}

// ---- row-band shards (SRT_RENDER_SHARDED, rt_device.h shard_of_row) -----------------------------
// Rank 0 gathers every rank's tiles (RCCL) and k_assemble writes them into the frame.
constexpr int MAX_RANKS = 64;
struct GatherTiles {
    const uint8_t* u8[MAX_RANKS];  // [rows_q][W][3]
    const double* rgb[MAX_RANKS];  // [3][rows_q * W]
    int64_t npix[MAX_RANKS];       // rows_q * W
};

__global__ __launch_bounds__(BLOCK) void k_assemble(GatherTiles T, int nranks, int64_t band, int64_t W,
                                                   int64_t H, uint8_t* u8, double* rgb) {
    const int64_t n = W * H;
    for (int64_t g = (int64_t)blockIdx.x * BLOCK + threadIdx.x; g < n; g += (int64_t)gridDim.x * BLOCK) {
        const int64_t y = g / W, x = g - y * W;
        const int q = shard_of_row(y, nranks, band);
        const int64_t l = shard_local_row(y, nranks, band) * W + x;
        if (u8) {
            const uint8_t* s = T.u8[q] + 3 * l;
            u8[3 * g] = s[0]; u8[3 * g + 1] = s[1]; u8[3 * g + 2] = s[2];
        }
        if (rgb) {
            const double* s = T.rgb[q];
            const int64_t np = T.npix[q];
            rgb[g] = s[l]; rgb[n + g] = s[np + l]; rgb[2 * n + g] = s[2 * np + l];
        }
    }
}

// SRT_RENDER_RGBX: the uint8 image as 4-byte pixels (R, G, B, 255) -- PIL's own layout of an "RGB"
// image, which it then takes in with a word copy per pixel instead of unpacking 3-byte pixels
__global__ __launch_bounds__(BLOCK) void k_rgbx(const uint8_t* rgb, uint32_t* rgbx, int64_t npix) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < npix; i += (int64_t)gridDim.x * BLOCK)
        rgbx[i] = (uint32_t)rgb[3 * i] | ((uint32_t)rgb[3 * i + 1] << 8) | ((uint32_t)rgb[3 * i + 2] << 16) | 0xFF000000u;
}

std::vector<int32_t> band_rows(int64_t H, int n, int q, int64_t band) {
    std::vector<int32_t> r;
    for (int64_t y = 0; y < H; ++y)
        if (shard_of_row(y, n, band) == q) r.push_back((int32_t)y);
    return r;
}

template <typename T>
hipError_t dalloc(T** p, int64_t count) {
    return hipMalloc((void**)p, (size_t)std::max<int64_t>(count, 1) * sizeof(T));
}

// Device buffers of one API call, freed on every exit path (the early HIP_TRY returns included)
struct CallBufs {
    std::vector<void*> p;
    CallBufs() = default;
    CallBufs(const CallBufs&) = delete;
    CallBufs& operator=(const CallBufs&) = delete;
    ~CallBufs() {
        for (void* b : p) (void)hipFree(b);
    }
    template <typename T>
    hipError_t alloc(T** out, int64_t count) {
        *out = nullptr;
        const hipError_t e = dalloc(out, count);
        if (e == hipSuccess) p.push_back(*out);
        return e;
    }
};

int grid_for(int64_t n, int max_blocks) {
    int64_t b = (n + BLOCK - 1) / BLOCK;
    if (b < 1) b = 1;
    return (int)std::min<int64_t>(b, max_blocks);
}

// seed the queue from caller rays (get_raycolor): ray i -> shard i % NSHARD, slot i / NSHARD
__global__ __launch_bounds__(BLOCK) void k_seed_queue(Queue q, int64_t seg, const double* O, const double* D,
                                                     const int32_t* med, int64_t n, uint32_t depth, uint32_t dfl,
                                                     uint32_t nmedia) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        int64_t dst = (i % NSHARD) * seg + i / NSHARD;
        uint32_t m = med ? (uint32_t)med[i] : 0u;
        if (m >= nmedia) m = 0u;  // out-of-table medium index: scene.n
        queue_store(q, dst, d3{O[i], O[n + i], O[2 * n + i]}, d3{D[i], D[n + i], D[2 * n + i]}, d3{1.0, 1.0, 1.0},
                    (uint32_t)i, pack_meta(m, depth, dfl), mix32(0x7A11u, (uint32_t)i));
    }
}

// srt_shade_level: the children one shading level appended to the queue shards, packed in shard
// order (block b = shard b, its rays at prefix[b] ..) into planar arrays of `total` rays
__global__ __launch_bounds__(BLOCK) void k_gather_children(Queue q, int64_t seg, const uint32_t* cnt,
                                                          const int64_t* prefix, int64_t total, double* O, double* D,
                                                          double* Wt, int32_t* parent, int32_t* medium, int32_t* depth,
                                                          int32_t* dfl) {
    const int s = blockIdx.x;
    const int64_t n = min((int64_t)cnt[s], seg);
    for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
        const Ray r = queue_load(q, (int64_t)s * seg + i);
        const int64_t k = prefix[s] + i;
        O[k] = r.o.x; O[total + k] = r.o.y; O[2 * total + k] = r.o.z;
        D[k] = r.d.x; D[total + k] = r.d.y; D[2 * total + k] = r.d.z;
        Wt[k] = r.w.x; Wt[total + k] = r.w.y; Wt[2 * total + k] = r.w.z;
        parent[k] = (int32_t)r.pix;
        medium[k] = (int32_t)meta_medium(r.meta);
        depth[k] = (int32_t)meta_depth(r.meta);
        dfl[k] = (int32_t)meta_diffuse(r.meta);
    }
}


}  // namespace

// shape of one frame's passes (what the read-back of its counters needs)
struct FramePlan {
    bool frame = false;  // rendered by k_frame (counts are totals, not queue fills)
    int chain_from = 0;  // > 0: k_trace at this depth runs in chain mode and no deeper kernel is launched
    bool fuse = false;   // k_primary traces every depth (single-child scenes): no k_trace launch
    int64_t npix = 0;
    int64_t W = 0, H = 0;  // frame shape (a shard renders npix of W * H)
    bool sharded = false, gather_rgb = false, use_mt = false;
    int spp = 0, batch = 0, npass = 0, dcap = 0, nev = 0;
    int groups = 1;  // k_frame sample groups per tile (the largest pass's)
    int64_t cnt_words = 0, pass_words = 0;
};

constexpr int MAX_FRAME_SLOTS = 8;

// Buffers and stream of one frame in flight.  Synchronous calls use slot 0; pipelined
// (SRT_RENDER_ASYNC) frames rotate over the slots, each with its own stream, so one frame's
// low-occupancy tail (deep depths, resolve) overlaps the next frame's primary kernel.  Measured on
// ex1 1080p (ms/frame, device-resident): 1 slot 1.47, 2 slots 1.308, 3 slots 1.292; 1/8 shard 0.28 /
// 0.202 / 0.199.  HIP gives a process four hardware queues by default, and a stream that shares a
// queue with another waits behind that stream's work: the slot count follows the queues
// (default_slots), and host outputs are copied on the frame's own stream.
struct FrameSlot {
    hipStream_t stream = nullptr;
    hipEvent_t jit_ready = nullptr;  // recorded on the MT stream after this slot's jitter is generated
    hipEvent_t jit_free = nullptr;   // recorded on `stream` after the last kernel that reads the jitter
    hipEvent_t mt_jumped = nullptr;  // recorded on the MT stream after this slot's jump kernel
    bool jit_busy = false;           // `jit_free` guards the jitter buffer
    uint32_t* mt_win = nullptr;      // segment windows of this slot's numpy-stream generation
    int64_t mt_win_cap = 0;
    // ray queues: 2 x NSHARD segments of `seg` rays
    Queue q[2]{};
    int64_t seg = 0;
    std::vector<void*> queue_bufs;
    // frame kernel rings (k_frame): nslot rings of ring_cap rays, one lock word per ring
    Queue ring{};
    int64_t ring_cap = 0;
    int nslot = 0;
    uint32_t* ring_lock = nullptr;
    std::vector<void*> ring_bufs;
    // frame buffers
    double* fb = nullptr;
    int64_t fb_cap = 0;
    double* fbg = nullptr;  // k_frame sample groups' partial sums [groups][3][npix]
    int64_t fbg_cap = 0;
    unsigned long long* fbx = nullptr;  // [3][npix] fixed-point sums + [npix] f32 magnitudes (fb_add)
    int64_t fbx_cap = 0;
    double* rgb = nullptr;
    int64_t rgb_cap = 0;
    uint8_t* u8 = nullptr;
    int64_t u8_cap = 0;
    double* jit = nullptr;
    int64_t jit_cap = 0;
    int32_t* hit = nullptr;
    int64_t hit_cap = 0;
    uint32_t* counts = nullptr;  // [SRT_MAX_DEPTHS][NSHARD]
    uint32_t* flags = nullptr;   // [2]
    unsigned long long* shadow = nullptr;  // [NSHARD]
    std::vector<hipEvent_t> ev;
    uint32_t* host = nullptr;  // pinned: per-pass counters/flags, shadow count
    int64_t host_words = 0;
    // SRT_RENDER_SHARDED on rank 0: every rank's tiles (padded to the largest shard) and the frame
    uint8_t* g_u8 = nullptr;
    int64_t g_u8_cap = 0;
    double* g_rgb = nullptr;
    int64_t g_rgb_cap = 0;
    uint8_t* full_u8 = nullptr;
    int64_t full_u8_cap = 0;
    double* full_rgb = nullptr;
    int64_t full_rgb_cap = 0;
    // the frame's gather (srt_render_group posts it for all its contexts in one RCCL group)
    struct Gather {
        bool on = false;
        int64_t W = 0, H = 0, npix = 0, maxpix = 0, band = 1;
        bool want_u8 = false, want_rgb = false;
        uint8_t* dst_u8 = nullptr;  // where k_assemble writes (caller's device buffer or full_u8)
        double* dst_rgb = nullptr;
        uint8_t* host_u8 = nullptr;  // caller's host buffer (copied after k_assemble) or null
        double* host_rgb = nullptr;
    } gather;
    // counts/flags/shadow are zeroed by the kernels that consume them (k_pass_end, k_resolve); a
    // frame that did not complete leaves them dirty and the next one clears them first
    bool dirty = true;
    // asynchronous frames queued on this slot since the last synchronisation point
    int pending = 0;
    FramePlan plan;
};

struct srt_ctx {
    int device = 0;
    int max_blocks = 2048;
    int ncu = 256;
    static constexpr int64_t queue_budget = (int64_t)96 << 30;  // bytes for both ray queues
    // scene
    bool has_scene = false;
    SceneView S{};
    int max_depth = 0;
    int has_diffuse = 0;
    int fanout = 1;
    uint32_t mats = 0;  // material types present (selects the kernel variant)
    uint32_t seq = 0;   // the scene's collider sequence (rt_device.h seq_encode; 0: none, or option collider_seq 0)
    bool seq_on = true;  // option "collider_seq": kernels specialised to the scene's collider sequence when built
    std::vector<void*> scene_bufs;
    // texel pool (outside scene_bufs: survives re-uploads with the same texel_key)
    uint8_t* texels = nullptr;
    uint64_t texel_key = 0;
    int64_t texel_bytes = 0;
    uint64_t texel_layout = 0;  // hash of the pool layout the records' offsets were remapped to
    bool texels_rgbx = false;  // the resident pool holds 3-channel images as RGBX
    // option "mt_jump_parts": blocks per jump window (0: mt_jump_parts's choice)
    int mt_parts_opt = 0;
    // camera tables (shared by the slots; uploaded only when they change)
    double* xs = nullptr;
    double* ys = nullptr;
    int32_t* rows = nullptr;
    int64_t cam_cap[3] = {0, 0, 0};
    std::vector<uint8_t> cam_host[3];  // host copies of what xs / ys / rows hold
    uint32_t* mt = nullptr;    // MT19937 jump tables (255 x 624), two round keys, two final windows
    // the y words (k_mt_y) of a generation's key: [0] / [1] those of the two final windows (made
    // by the end block that made the window, valid flag per window), [2] scratch for other keys
    uint32_t* mt_y = nullptr;
    bool mt_y_valid[2] = {false, false};
    // band mode (a shard's rows of the numpy stream, rt_mt_kernel.h MtArgs::bands): per pass shape,
    // the segment list and its jump polynomials (host-made once, kept for the context's life)
    struct MtBandTab {
        int64_t key[6];
        uint64_t rows_hash;
        int nseg;
        int64_t band_len, band_period;  // merged segments store k % band_period < band_len (doubles)
        int64_t* bands;   // device [nseg][4]
        uint32_t* polys;  // device [nseg][624]
    };
    std::deque<MtBandTab> mt_bandtabs;  // (stable addresses: frames hold pointers into it)
    std::vector<std::pair<int64_t, uint32_t*>> mt_end_polys;  // frame-end jump polynomial per word count
    bool mt_bands_on = true;  // option "mt_bands"
    // option "mt_short": doubles per segment of a whole frame's stream when nothing else is in flight
    // (a synchronous frame -- Scene.render -- or the first of a pipeline): its generation cannot hide
    // behind earlier frames, and a segment's serial generator (624-word blocks, ~0.5 us each) sets the
    // frame's latency: 2^19-word tabulated segments 0.42 ms, 2^17-word ones ~0.1 ms for 4x the jumps,
    // made in band mode (host jump polynomials, cached per frame shape); 0: tabulated segments
    int64_t mt_short = 65536;
    // option "mt_pipe_split": doubles per band-mode segment of a pipelined whole frame behind others in
    // flight (0: the tabulated 2^19-word segments).  Band mode generates exactly the stored planes' runs
    // (a tabulated segment straddling a stored and a skipped plane generates both), each run cut at the
    // split: same box, ex1 1080p pipelined frames 0.84 ms tabulated, 0.794 at 2^18 doubles (the
    // tabulated segments' length), 1.12 at 2^19 (longer generator chains); profiles/r05_pipe_split_ab.txt
    int64_t mt_pipe_split = (int64_t)1 << 18;
    double* mt_out = nullptr;  // staging for srt_mt19937_uniforms into host memory
    int64_t mt_out_cap = 0;
    // -1 auto: k_frame for scenes whose rays branch (refractive / thin-film / diffuse fan-out),
    // per-depth wavefront kernels otherwise.  Measured (one MI355X, Mrays/s, wavefront vs frame):
    // ex1 1080p d5 13388 vs 10478, ex3 1080p d8 8950 vs 9585, ex4 4K d6 14081 vs 17494,
    // cornell 800x800 512 spp 3542 vs 4073.
    int use_frame = -1;
    bool use_bvh = true;  // option "bvh": 0 intersects mesh triangles one by one (comparison runs)
    // chain mode of the wavefront path (single-child scenes): from the first depth >= 1 whose ray
    // count in the previous frame of the same shape was below chain_rays
    int64_t chain_rays = 1000000;
    bool chain_ok = true;  // cleared when a tie produced a second child in chain mode
    int64_t hint_key[3] = {-1, -1, -1};
    int64_t hint[SRT_MAX_DEPTHS] = {};
    // frame slots; `f` is the one the current call works on
    FrameSlot slots[MAX_FRAME_SLOTS];
    // pipelined frames: slots they rotate over; the numpy-stream generation of single-pass frames on a
    // stream of its own (round 2-3 options "slots", "mt_stream", "copy_stream", removed in round 6: the
    // host-output copies on a stream of their own did not pay).  ex1 1080p, host outputs, one MI355X,
    // ms/frame: 3 slots 1.83; 2 slots
    // + copy stream 1.83; 3 slots + MT stream 1.82; 2 slots 2.20; 2 slots + MT stream 2.00; one rank's
    // shard of an 8-GPU frame (bench --shard-of 8, same box): 3 slots 0.627, 4 slots 0.544, 3 slots +
    // MT stream 0.857.  Default (default_slots): one slot per hardware queue HIP gives the process
    // but one, at least four: GPU_MAX_HW_QUEUES=7 (bench.py sets it) -> 6 slots: one rank of 8,
    // slowest rank 0.318 -> 0.265 ms per frame, the whole ex1 frame 1.30 -> 1.26 ms (8 slots: 0.41 /
    // 1.28; profiles/r03_slots_ab.txt)
    int nslots = 4;
    // where the numpy-stream generation runs: a high-priority stream of its own for whole frames (ex1
    // 1080p 1.80 -> 1.64 ms/frame, same box), the frame's stream for shards (round 4, same box: one
    // rank of 2 0.87 ms on a stream of its own, 0.67 on a high-priority one, 0.55 on the frame's
    // stream; of 4 0.33 / 0.48 / 0.32; of 8 0.20 / 0.33 / 0.21, profiles/r04_mt_stream_ab.txt).  The
    // generators of a whole pipelined frame run after its jump kernel on that stream (frame k+1's
    // jumps then wait behind frame k's generators); on the frame's own stream or on two high-priority
    // generator streams taken in turn (round-5 option "mt_gen_stream", removed in round 6) pipelined
    // ex1 frames took ~1.05 and 1.014-1.028 ms against 0.940 (profiles/r05_mt_generator_ab.txt).
    // option "deterministic" (default 1): contributions added to a pixel by other threads go into
    // order-independent fixed-point sums (bit-reproducible frames); 0: f64 atomics
    bool deterministic = true;
    bool fx_ok = true;  // cleared when a contribution left the fixed-point range (until the next scene)
    FrameSlot* f = &slots[0];
    bool pipeline = false;  // option "pipeline": size every slot on every frame (no first-use allocation)
    int next_slot = 0;      // slot of the next asynchronous frame
    int last_slot = 0;      // slot of the last asynchronous frame (its stats are reported)
    int async_pending = 0;  // asynchronous frames in flight (all slots)
    srt_stats async_stats{};
    // numpy-stream jitter generated on the device (render args `mt`): the state after the last
    // queued frame stays on the device (mt dump window) while consecutive asynchronous frames pass the
    // same host state, which srt_render_finish then writes
    srt_mt_state* mt_chain = nullptr;
    int mt_pos = 0;
    hipEvent_t mt_done = nullptr;  // recorded after the last frame's stream generation
    int mt_cur = 0;                // which of the two final-window buffers is current (mt_dump)
    // a generation stopped between its jump and its generator launches (an error return) leaves
    // windows that are not zero and possibly a partial end accumulator: every slot's window table,
    // end_acc and end_cnt are cleared before the next generation (mt_win_ensure)
    bool mt_dirty = false;
    // single-pass frames generate their numpy stream on a stream of their own, so the generation of
    // frame k+1 runs beside frame k's trace (their order is this stream's order)
    hipStream_t mt_stream = nullptr;
    bool mt_tables = false;
    // multi-GPU (srt_comm_init / srt_comm_init_all)
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool defer_gather = false;  // srt_render_group posts the gathers of all its contexts in one group
    bool retry_frame = false;   // the last finish_async failed only with RETRY_* bits (render the frame again)
    int shard_bands = 0;  // option "shard_bands": most row bands per rank (0: rt_device.h shard_kmax by the scene's fan-out)
    // option "fuse_primary": single-child scenes traced whole-path per pixel in k_primary (same image
    // bit for bit as the per-depth kernels); -1 (default) for frames of at least two resident
    // rounds of threads: ex1 1080p 1.308 -> 1.209 ms per frame, a rank of 4 0.47 -> 0.44, while a rank
    // of 8 (1.3 rounds) is faster per depth, 0.29 vs 0.35 (profiles/r03_fused_ab.txt)
    int fuse_primary = -1;
    // option "rehearse_assemble" = n (diagnostic, one GPU): a frame rendering rank 0's rows of an
    // n-rank job (rows given, not SRT_RENDER_SHARDED) also does rank 0's assembly -- k_assemble of its
    // tile and n - 1 stand-in tiles of the other ranks' shapes into the whole frame -- and hands back
    // the whole frame's uint8 image (host copy of W x H x 3 bytes), as a sharded rank 0 does after the
    // RCCL gather (the transfers themselves are not rehearsed)
    int rehearse_assemble = 0;
    int lean_blocks = 0;  // grid of k_primary_lean in pipelined whole frames (set to 2 blocks per CU)
    // the same for a shard's rows (set to 4 per CU: every rank of 4 rehearsed, slowest 0.321 -> 0.275 ms
    // per frame; of 8 unchanged, profiles/r05_lean_grid_ab.txt)
    int lean_blocks_shard = 0;
    bool sync_lean = false;     // option "sync_lean": synchronous frames run k_primary_lean too (measurement)
    int64_t lean_launches = 0;  // (srt_debug_lean_launches)
    // generator workgroup size of the current generation (mt_gen_launch): 256 for the pipelined frames
    // of a lean k_primary, else MT_GEN_THREADS; option "mt_gen_nt" (0 auto, 256 or 320) forces one
    int gen_nt = rtmt_dev::MT_GEN_THREADS;
    int mt_gen_nt_opt = 0;
    double* red = nullptr;      // srt_comm_allreduce scratch
    // srt_render_prefetch: the numpy-stream generation of the synchronous whole frame srt_render is
    // about to be called for, queued before the caller lowers and uploads its scene (Scene.render);
    // the next srt_render with the same stream state and frame shape finds it queued and skips its
    // own launch.  Any other call that generates from the stream drops it.
    struct MtPrefetch {
        bool valid = false;
        uint32_t key[rtmt::N];
        int pos = 0;
        int64_t shape[8] = {};       // W, H, spp, batch, plane mask, slot, stream, generation flavour
        const void* bt[2] = {nullptr, nullptr};  // the band tables it used
        int final_pos = 0;
        hipStream_t gen_on = nullptr;
    } pf;
    int64_t pf_used = 0, pf_queued = 0;  // (srt_debug_prefetch_counts)
    unsigned long long* lane_stats = nullptr;  // (srt_debug_lane_stats) [SRT_MAX_DEPTHS][2] or null
};

namespace {

void free_list(std::vector<void*>& v) {
    for (void* p : v)
        if (p) (void)hipFree(p);
    v.clear();
}

// make room for `rays` queued rays per depth (spread over the shards with slack)
int ensure_queues(srt_ctx* c, int64_t rays) {
    int64_t seg = (rays + NSHARD - 1) / NSHARD;
    seg = seg + seg / 8 + 1024;
    if (seg <= c->f->seg) return SRT_OK;
    free_list(c->f->queue_bufs);
    c->f->seg = 0;
    const int64_t n = seg * NSHARD;
    for (int k = 0; k < 2; ++k) {
        Queue& q = c->f->q[k];
        double** dptr[9] = {&q.ox, &q.oy, &q.oz, &q.dx, &q.dy, &q.dz, &q.wr, &q.wg, &q.wb};
        for (double** p : dptr) {
            if (dalloc(p, n) != hipSuccess) return fail(SRT_ERR_MEMORY, "ray queue allocation failed");
            c->f->queue_bufs.push_back(*p);
        }
        uint32_t** uptr[3] = {&q.pix, &q.meta, &q.path};
        for (uint32_t** p : uptr) {
            if (dalloc(p, n) != hipSuccess) return fail(SRT_ERR_MEMORY, "ray queue allocation failed");
            c->f->queue_bufs.push_back(*p);
        }
    }
    c->f->seg = seg;
    return SRT_OK;
}

// rings of the frame kernel: more rings than waves can ever be resident (32 per CU), so a wave
// always finds a free one; `cap` rays each (power of two)
int ensure_ring(srt_ctx* c, int64_t cap) {
    int64_t k = 256;
    while (k < cap) k <<= 1;
    cap = k;
    const int nslot = std::max(1024, 2 * 32 * c->ncu);
    if (cap <= c->f->ring_cap && nslot <= c->f->nslot) return SRT_OK;
    free_list(c->f->ring_bufs);
    c->f->ring_cap = 0;
    c->f->nslot = 0;
    const int64_t n = cap * nslot;
    Queue& q = c->f->ring;
    double** dptr[9] = {&q.ox, &q.oy, &q.oz, &q.dx, &q.dy, &q.dz, &q.wr, &q.wg, &q.wb};
    for (double** p : dptr) {
        if (dalloc(p, n) != hipSuccess) return fail(SRT_ERR_MEMORY, "ray ring allocation failed");
        c->f->ring_bufs.push_back(*p);
    }
    uint32_t** uptr[3] = {&q.pix, &q.meta, &q.path};
    for (uint32_t** p : uptr) {
        if (dalloc(p, n) != hipSuccess) return fail(SRT_ERR_MEMORY, "ray ring allocation failed");
        c->f->ring_bufs.push_back(*p);
    }
    if (dalloc(&c->f->ring_lock, nslot) != hipSuccess) return fail(SRT_ERR_MEMORY, "ring lock allocation failed");
    c->f->ring_bufs.push_back(c->f->ring_lock);
    HIP_TRY(hipMemset(c->f->ring_lock, 0, (size_t)nslot * 4));
    c->f->ring_cap = cap;
    c->f->nslot = nslot;
    return SRT_OK;
}

template <typename T>
int ensure_buf(T** p, int64_t& cap, int64_t count) {
    if (count <= cap && *p) return SRT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (dalloc(p, count) != hipSuccess) return fail(SRT_ERR_MEMORY, "device allocation failed");
    cap = count;
    return SRT_OK;
}

// The segment-window table of a slot's numpy-stream generation: zero when (re)allocated; from then
// on every window a jump XORs into is zeroed again by the generator that reads it.  After a
// generation that stopped between its jump and generator launches (srt_ctx::mt_dirty) every slot's
// table and the end accumulator are cleared first (device-synchronous: an error path only).
int mt_end_reset(srt_ctx* c);
int mt_win_ensure(srt_ctx* c, FrameSlot& f, int64_t count) {
    if (c->mt_dirty) {
        HIP_TRY(hipDeviceSynchronize());
        for (FrameSlot& s : c->slots)
            if (s.mt_win) HIP_TRY(hipMemset(s.mt_win, 0, (size_t)s.mt_win_cap * 4));
        int rc = mt_end_reset(c);
        if (rc) return rc;
        c->mt_dirty = false;
    }
    if (count <= f.mt_win_cap && f.mt_win) return SRT_OK;
    int rc = ensure_buf(&f.mt_win, f.mt_win_cap, count);
    if (rc) return rc;
    HIP_TRY(hipMemset(f.mt_win, 0, (size_t)count * 4));
    return SRT_OK;
}

template <typename T>
int upload(srt_ctx* c, const T* src, int64_t count, T** dst) {
    *dst = nullptr;
    if (count <= 0 || !src) return SRT_OK;
    HIP_TRY(dalloc(dst, count));
    c->scene_bufs.push_back(*dst);
    HIP_TRY(hipMemcpy(*dst, src, (size_t)count * sizeof(T), hipMemcpyDefault));
    return SRT_OK;
}

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

// 0: null, 1: device memory, 2: pinned host memory (hipHostMalloc / registered), 3: other host memory
int ptr_kind(const void* p) {
    if (!p) return 0;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 3;
    }
    if (a.type == hipMemoryTypeDevice) return 1;
    if (a.type == hipMemoryTypeHost) return 2;
    return 3;
}

#define NCCL_TRY(expr)                                                                          \
    do {                                                                                        \
        ncclResult_t _r = (expr);                                                               \
        if (_r != ncclSuccess)                                                                  \
            return fail(SRT_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r));      \
    } while (0)

int check_flags(uint32_t f0) {
    if (f0 & ERR_INDEX)
        return fail(SRT_ERR_INDEX, "index out of bounds in a texture/table lookup (reference raises IndexError)");
    if (f0 & ERR_UNSUPPORTED) return fail(SRT_ERR_ARG, "uv requested on a Triangle (undefined in the reference)");
    if (f0 & ERR_NAME)
        return fail(SRT_ERR_NAME, "name 'M' is not defined (PointLight.get_L at a Glossy hit, as the reference "
                                  "sightpy/lights.py:30-31 raises)");
    return SRT_OK;
}

TraceParams base_params(srt_ctx* c, uint64_t seed) {
    TraceParams P{};
    P.S = c->S;
    P.flags = c->f->flags;
    P.shadow = c->f->shadow;
    P.seg = c->f->seg;
    P.seed = seed;
    P.lane_stats = c->lane_stats;  // (read by k_primary_lean<.., true> only)
    return P;
}

// deepest depth index that can hold rays: max_ray_depth, +2 diffuse bounces without depth check
// (a child is made only while depth < max_ray_depth, so depth max_ray_depth is the last with rays;
// Diffuse bounces ignore max_ray_depth (diffuse.py:25-124) and add at most two more)
int depth_cap(const srt_ctx* c) { return std::min(SRT_MAX_DEPTHS - 2, c->max_depth + (c->has_diffuse ? 2 : 0)); }

// threads the fused paths want per pass: two rounds of the resident threads (4 SIMDs x OCC waves per CU)
int64_t fused_items(const srt_ctx* c) { return 2 * (int64_t)c->ncu * 4 * OCC * 64; }

// k_primary's sample groups per pixel (TraceParams::pix_groups): the fewest (a power of two, at most
// the pass's samples and 64) that give the pass enough threads
int pix_groups(const srt_ctx* c, int64_t npix, int ns, bool fused) {
    const int64_t want = fused ? fused_items(c) : (int64_t)c->max_blocks * 64;
    int g = 1;
    while (g * 2 <= std::min(ns, 64) && npix * g < want) g *= 2;
    // a BVH scene's paths differ widely in length (mesh hits traverse, the rest do not): one sample
    // per lane where the spp allows (up to 4 groups, dividing the samples evenly) gives the GPU twice
    // the waves to balance -- mesh 1080p 2 spp 5.94 -> 4.33 ms per frame, same box
    // (profiles/r04_mesh_pix_groups_ab.txt)
    if (c->mats & MAT_BVH)
        while (g * 2 <= std::min(ns, 4) && ns % (g * 2) == 0) g *= 2;
    // the fused paths take two groups whenever the samples split evenly: ex1 1080p 6 spp, same box,
    // the fused kernel 1.095 -> 1.050 ms per launch, device-resident frame 0.841 -> 0.830 ms
    // (profiles/r04_pix_groups_ab.txt)
    if (fused && g < 2 && ns % 2 == 0) g = 2;
    // the fused paths' tiles of 8 x 64 / g pixels (rt_primary_body.inc) need g <= 8
    if (fused && !(c->mats & MAT_BVH)) g = std::min(g, 8);
    return g;
}

size_t lut_bytes(const srt_ctx* c) { return (size_t)c->S.nlut_lds * 256 * sizeof(double); }

int trace_grid(const srt_ctx* c) { return std::max(NSHARD, (c->max_blocks / NSHARD) * NSHARD); }

// copy `bytes` from host `src` to device `dst` unless `shadow` (the host copy of what dst holds)
// already equals it.  The shadow is invalidated whenever the buffer is reallocated (ensure_buf).
int finish_async(srt_ctx* c, srt_stats* st);

// the camera tables are shared by the frame slots: wait for the frames in flight before changing
// them (keeps the current slot)
int quiesce_for_shared_write(srt_ctx* c) {
    if (c->async_pending == 0) return SRT_OK;
    FrameSlot* keep = c->f;
    int rc = finish_async(c, nullptr);
    c->f = keep;
    return rc;
}

int upload_if_changed(srt_ctx* c, void* dst, std::vector<uint8_t>& shadow, const void* src, size_t bytes) {
    if (is_device_ptr(src)) {
        int rc = quiesce_for_shared_write(c);
        if (rc) return rc;
        shadow.clear();
        HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->f->stream));
        return SRT_OK;
    }
    if (shadow.size() == bytes && !memcmp(shadow.data(), src, bytes)) return SRT_OK;
    int rc = quiesce_for_shared_write(c);
    if (rc) return rc;
    shadow.assign((const uint8_t*)src, (const uint8_t*)src + bytes);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->f->stream));
    return SRT_OK;
}

int64_t depth_total(const uint32_t* cnt, int64_t seg) {
    int64_t t = 0;
    for (int s = 0; s < NSHARD; ++s) t += std::min<int64_t>(cnt[s], seg);
    return t;
}

}  // namespace

namespace {

// ---- numpy's stream on the device (rt_mt.h): scratch c->mt = jump tables | key 0 | key 1 | dump ----
constexpr int64_t MT_NTAB = rtmt::TABLE_WORDS;
uint32_t* mt_key0(srt_ctx* c) { return c->mt + MT_NTAB; }
// the final window of the last queued generation (two alternate, so the next frame's generation
// reads the previous one in place while writing its own)
uint32_t* mt_dump(srt_ctx* c) { return c->mt + MT_NTAB + (2 + c->mt_cur) * rtmt::N; }

int mt_ensure(srt_ctx* c) {
    if (c->mt) return SRT_OK;
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mt_jump),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)MT_LDS_BYTES));
    // jump tables | two round keys | two final windows | the end window's accumulator + its counter
    HIP_TRY(dalloc(&c->mt, MT_NTAB + 5 * rtmt::N + 1));
    HIP_TRY(hipMemcpy(c->mt, rtmt::tables_flat(), MT_NTAB * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(c->mt + MT_NTAB + 4 * rtmt::N, 0, (rtmt::N + 1) * 4));
    HIP_TRY(dalloc(&c->mt_y, (int64_t)3 * MT_YBLOCKS * rtmt::N));
    return SRT_OK;
}

uint32_t* mt_dump_at(srt_ctx* c, int d) { return c->mt + MT_NTAB + (2 + d) * rtmt::N; }
uint32_t* mt_end_acc(srt_ctx* c) { return c->mt + MT_NTAB + 4 * rtmt::N; }
uint32_t* mt_end_cnt(srt_ctx* c) { return c->mt + MT_NTAB + 5 * rtmt::N; }
uint32_t* mt_ybuf(srt_ctx* c, int i) { return c->mt_y + (int64_t)i * MT_YBLOCKS * rtmt::N; }
int mt_end_reset(srt_ctx* c) {
    if (c->mt) HIP_TRY(hipMemset(mt_end_acc(c), 0, (rtmt::N + 1) * 4));  // end_acc [624] and end_cnt [1]
    return SRT_OK;
}

// Blocks per jump window (k_mt_jump parts): the option, else 4 (final build, same box, against 8:
// device-side whole frame 0.988 -> 0.979 ms, a rank of 8 0.204 -> 0.202, of 4 0.328 -> 0.318;
// profiles/r04_jump_parts_ab.txt)
int mt_jump_parts(const srt_ctx* c) { return c->mt_parts_opt ? c->mt_parts_opt : 4; }



// The y words of `key` for a generation on `st`: those an end block made with the key (a final
// window), else k_mt_y into the scratch buffer (one workgroup, ~34 blocks).  Generations of
// different frames are ordered by the key they hand on, so one scratch buffer suffices.
const uint32_t* mt_y_for(srt_ctx* c, hipStream_t st, const uint32_t* key) {
    for (int d = 0; d < 2; ++d)
        if (key == mt_dump_at(c, d) && c->mt_y_valid[d]) return mt_ybuf(c, d);
    hipLaunchKernelGGL(k_mt_y, dim3(1), dim3(MT_THREADS), 0, st, key, mt_ybuf(c, 2));
    return mt_ybuf(c, 2);
}

// x^end_jump(n_words) mod phi on the device, made once per word count (a few shapes per context)
int mt_end_poly_for(srt_ctx* c, int64_t n_words, const uint32_t** out) {
    for (auto& e : c->mt_end_polys)
        if (e.first == n_words) { *out = e.second; return SRT_OK; }
    uint32_t* d = nullptr;
    HIP_TRY(dalloc(&d, rtmt::N));
    const std::vector<uint32_t> poly = rtmt::xpow_mod(rtmt::end_jump(n_words));
    HIP_TRY(hipMemcpy(d, poly.data(), rtmt::N * 4, hipMemcpyHostToDevice));
    c->mt_end_polys.emplace_back(n_words, d);
    *out = d;
    return SRT_OK;
}

// The generators of `nseg` segments, one workgroup each: five waves, or four (one per SIMD) for the
// frames of a lean k_primary (srt_ctx::gen_nt), which leaves room for exactly that beside its waves
void mt_gen_launch(srt_ctx* c, const MtArgs& G, int nseg, hipStream_t st, uint32_t* win) {
    if (c->gen_nt == 256)
        hipLaunchKernelGGL(k_mt_gen<256>, dim3(nseg), dim3(256), 0, st, G, win);
    else
        hipLaunchKernelGGL(k_mt_gen<MT_GEN_THREADS>, dim3(nseg), dim3(MT_GEN_THREADS), 0, st, G, win);
}

// Band mode table of one pass shape: the rows' runs of `ns` samples' stored planes, each segment
// with its jump polynomial x^(2 d0 - 1) mod phi (xpow_mod, ~2.5 ms each, over a few host threads).
// Regular runs (a shard's row bands: equal length, equal spacing) with short gaps are merged while
// a segment spans at most MT_MERGE_DOUBLES: it then generates through the other ranks' rows between
// them (stores masked by band_len / band_period), trading one jump (~110 us of a CU) for a few
// hundred generated blocks (a CU fraction); other runs are split at `split` doubles (2^18 for a
// shard's rows, srt_ctx::mt_short for a whole frame generated with nothing else in flight).
constexpr int MT_MAX_BANDS = 2048;
constexpr int64_t MT_MERGE_DOUBLES = 150000;
int mt_band_table(srt_ctx* c, int64_t W, int64_t Hf, int ns, int plane_mask, const int32_t* rows, int n_rows,
                  int64_t split, const srt_ctx::MtBandTab** out) {
    uint64_t h = 1469598103934665603ull;
    for (int k = 0; k < n_rows; ++k) h = (h ^ (uint64_t)(uint32_t)rows[k]) * 1099511628211ull;
    const int64_t key[6] = {W, Hf, ns, plane_mask, n_rows, split};
    for (auto& t : c->mt_bandtabs)
        if (!memcmp(t.key, key, sizeof key) && t.rows_hash == h) { *out = &t; return SRT_OK; }
    // runs of consecutive rows (first row, count)
    std::vector<std::pair<int, int>> runs;
    for (int k = 0; k < n_rows;) {
        int e = k + 1;
        while (e < n_rows && rows[e] == rows[e - 1] + 1) ++e;
        runs.emplace_back(rows[k], e - k);
        k = e;
    }
    // the regular pattern (the first run's length and the spacing of the first two runs), if any
    const int rlen = runs[0].second;
    const int rper = runs.size() > 1 ? runs[1].first - runs[0].first : 0;
    // merged only when the gaps are no longer than the runs (N = 2 shards): the merged segments' longer
    // generation is on the frame's critical path, and with longer gaps it cost more than the jumps it
    // saves (same box, ms per rank-frame, ex1 1080p, unmerged vs merged: N = 2 1.076 vs 0.991, N = 4
    // 0.579 vs 0.614, N = 8 0.339 vs 0.422)
    const bool regular_ok = rper > rlen && rper - rlen <= rlen;
    // local row of each run's first row (the shard's compact jitter layout [s][plane][rows][W])
    std::vector<int64_t> run_lrow(runs.size(), 0);
    for (size_t k = 1; k < runs.size(); ++k) run_lrow[k] = run_lrow[k - 1] + runs[k - 1].second;
    const int64_t npix = (int64_t)n_rows * W;
    std::vector<int64_t> segs;  // (first double, doubles, masked, local offset)
    for (int s = 0; s < ns; ++s)
        for (int j = 0; j < 4; ++j) {
            if (!((plane_mask >> j) & 1)) continue;
            const int64_t pbase = (int64_t)(s * 4 + j) * Hf;
            const int64_t lbase = (int64_t)(s * 4 + j) * npix;
            for (size_t k = 0; k < runs.size();) {
                size_t e = k + 1;
                if (regular_ok && runs[k].second == rlen)
                    while (e < runs.size() && runs[e].second == rlen && runs[e].first - runs[e - 1].first == rper &&
                           (int64_t)(runs[e].first + rlen - runs[k].first) * W <= MT_MERGE_DOUBLES)
                        ++e;
                int64_t d0 = (pbase + runs[k].first) * W;
                int64_t l0 = lbase + run_lrow[k] * W;
                if (e > k + 1) {
                    segs.insert(segs.end(), {d0, (int64_t)(runs[e - 1].first + rlen - runs[k].first) * W, 1, l0});
                } else {
                    int64_t n = (int64_t)runs[k].second * W;
                    while (n > 0) {
                        const int64_t m = std::min<int64_t>(n, split);
                        segs.insert(segs.end(), {d0, m, 0, l0});
                        d0 += m;
                        l0 += m;
                        n -= m;
                    }
                }
                k = e;
            }
        }
    const int nseg = (int)(segs.size() / 4);
    *out = nullptr;
    if (nseg > MT_MAX_BANDS || nseg == 0) return SRT_OK;  // (the tabulated segments instead)
    std::vector<uint32_t> polys((size_t)nseg * rtmt::N, 0u);
    // (xpow_mod ~2.5 ms per polynomial: up to 16 host threads, the GPU boxes' CPU share per GPU)
    const int nth = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int w = 0; w < nth; ++w)
        th.emplace_back([&, w] {
            for (int i = w; i < nseg; i += nth) {
                if (segs[4 * i] == 0) continue;  // starts from the key
                const std::vector<uint32_t> p = rtmt::xpow_mod((uint64_t)(2 * segs[4 * i] - 1));
                std::copy(p.begin(), p.end(), polys.begin() + (size_t)i * rtmt::N);
            }
        });
    for (auto& t : th) t.join();
    srt_ctx::MtBandTab T{};
    memcpy(T.key, key, sizeof key);
    T.rows_hash = h;
    T.nseg = nseg;
    T.band_len = (int64_t)rlen * W;
    T.band_period = (int64_t)std::max(rper, 1) * W;
    HIP_TRY(dalloc(&T.bands, (int64_t)segs.size()));
    HIP_TRY(dalloc(&T.polys, (int64_t)polys.size()));
    HIP_TRY(hipMemcpy(T.bands, segs.data(), segs.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(T.polys, polys.data(), polys.size() * 4, hipMemcpyHostToDevice));
    c->mt_bandtabs.push_back(T);
    *out = &c->mt_bandtabs.back();
    return SRT_OK;
}

// Band mode generation of n_words words from (key, pos): only the table's segments are generated
// (their doubles at their place in `out`, the whole pass's layout), every one jumped to from the key;
// the final window (next key) and its y come from the jump kernel's end block.
int mt_launch_bands(srt_ctx* c, hipStream_t st, uint32_t* win, const uint32_t* key, int pos, int64_t n_words,
                    const srt_ctx::MtBandTab& T, double* out, int* final_pos, const uint32_t* end_poly,
                    hipEvent_t key_ready, hipStream_t gst = nullptr, hipEvent_t jumped = nullptr,
                    hipStream_t* gen_on = nullptr) {
    const int64_t abs_end = pos + n_words;
    const int64_t dump_abs = ((abs_end + rtmt::N - 1) / rtmt::N - 1) * rtmt::N;
    MtArgs A{};
    A.key = key;
    A.tab = T.polys;
    A.bands = T.bands;
    A.band_len = T.band_len;
    A.band_period = T.band_period;
    A.out = out;
    A.words = n_words;
    A.double_base = 0;
    A.n_out = INT64_MAX;
    A.pos = pos;
    A.dump_at = dump_abs;
    A.dump_dst = mt_dump_at(c, c->mt_cur ^ 1);
    A.end_poly = end_poly;
    A.end_at = (int64_t)rtmt::end_jump(n_words);
    A.key_in_win = 1;
    A.compact = 1;  // the shard's own layout (srt_render reads it by local pixel)
    A.y = mt_y_for(c, st, key);
    A.y_next = mt_ybuf(c, c->mt_cur ^ 1);
    A.end_acc = mt_end_acc(c);
    A.end_cnt = mt_end_cnt(c);
    A.parts = mt_jump_parts(c);
    // the segment windows are XOR-accumulated by their jump parts into the table, which is zero here:
    // zeroed when allocated (mt_win_ensure), and every generator zeroes the window it read
    c->mt_dirty = true;  // (until the generators that zero the windows are queued)
    hipLaunchKernelGGL(k_mt_jump, dim3((T.nseg + 1) * A.parts), dim3(MT_THREADS), mt_jump_lds_bytes(A.parts), st, A,
                       win);
    HIP_TRY(hipGetLastError());
    if (key_ready) HIP_TRY(hipEventRecord(key_ready, st));
    MtArgs G = A;
    G.dump_dst = nullptr;
    G.y_next = nullptr;
    if (gst && gst != st) {  // the generators on their own stream, after the windows they start from
        HIP_TRY(hipEventRecord(jumped, st));
        HIP_TRY(hipStreamWaitEvent(gst, jumped, 0));
    } else {
        gst = st;
    }
    mt_gen_launch(c, G, T.nseg, gst, win);
    HIP_TRY(hipGetLastError());
    if (gen_on) *gen_on = gst;
    c->mt_dirty = false;
    c->mt_y_valid[c->mt_cur ^ 1] = true;
    c->mt_cur ^= 1;
    *final_pos = (int)(abs_end - dump_abs);
    return SRT_OK;
}

// Queue on `st`: from the key window `key` (device) at position `pos`, n_out doubles into `out`
// (device) and n_skip more draws; the window holding the last consumed word becomes mt_dump(c).  Returns the
// numpy position of that window in *final_pos.  `plane` > 0: only the doubles of the planes
// (index % 4) in `plane_mask` are stored (a pinhole camera reads no lens-disk pair).
// `win`: the segment-window table of this generation (SEGS x 624 words; per frame slot, as pipelined
// frames generate concurrently).  `end_poly` (x^end_at mod phi, device) on a one-round generation:
// k_mt_jump also makes the final window, and `key_ready` is recorded right after it -- the next
// frame's generation may start then, beside this one's generators.
int mt_launch(srt_ctx* c, hipStream_t st, uint32_t* win, const uint32_t* key, int pos, int64_t n_out, int64_t n_skip,
              double* out, int* final_pos, int64_t plane = 0, int plane_mask = 15, const uint32_t* end_poly = nullptr,
              int64_t end_at = 0, hipEvent_t key_ready = nullptr, hipStream_t gst = nullptr,
              hipEvent_t jumped = nullptr, hipStream_t* gen_on = nullptr) {
    if (gen_on) *gen_on = st;
    uint32_t* keys[2] = {c->mt + MT_NTAB, c->mt + MT_NTAB + rtmt::N};
    const rtmt::Plan plan = rtmt::make_plan(pos, 2 * (n_out + n_skip));
    if (plan.rounds.size() != 1) end_poly = nullptr;
    for (size_t r = 0; r < plan.rounds.size(); ++r) {
        const rtmt::Round& R = plan.rounds[r];
        MtArgs A{};
        A.key = r == 0 ? key : keys[r & 1];
        A.tab = c->mt;
        A.out = out;
        A.chain_dst = R.chain ? keys[(r + 1) & 1] : nullptr;
        A.dump_dst = R.dump_at >= 0 ? c->mt + MT_NTAB + (2 + (c->mt_cur ^ 1)) * rtmt::N : nullptr;
        A.words = R.words;
        A.double_base = R.double_base;
        A.n_out = n_out;
        A.dump_at = R.dump_at;
        A.pos = R.pos;
        // the block's doubles span at most two planes when a plane holds >= 312 of them
        A.plane = plane >= 1024 ? plane : 0;
        A.plane_mask = plane_mask;
        // segment windows (and the final window), then the generators
        const bool end = end_poly && A.dump_dst;
        if (end) {
            A.end_poly = end_poly;
            A.end_at = end_at;
        }
        const int jump_blocks = (R.nseg - 1) + (end ? 1 : 0);
        A.key_in_win = jump_blocks > 0;
        if (A.dump_dst) {
            A.y_next = end ? mt_ybuf(c, c->mt_cur ^ 1) : nullptr;
            c->mt_y_valid[c->mt_cur ^ 1] = end;  // (a generator segment makes the window, not its y)
        }
        if (jump_blocks > 0) {
            c->mt_dirty = true;  // (until the generators that zero the windows are queued)
            A.y = mt_y_for(c, st, A.key);
            A.end_acc = mt_end_acc(c);
            A.end_cnt = mt_end_cnt(c);
            A.parts = mt_jump_parts(c);
            // the segment windows are XOR-accumulated by their jump parts (into zeroed windows: see
            // mt_launch_bands)
            hipLaunchKernelGGL(k_mt_jump, dim3(jump_blocks * A.parts), dim3(MT_THREADS), mt_jump_lds_bytes(A.parts),
                               st, A, win);
            HIP_TRY(hipGetLastError());
        }
        if (end && key_ready) HIP_TRY(hipEventRecord(key_ready, st));
        MtArgs G = A;
        G.y_next = nullptr;
        if (end) G.dump_dst = nullptr;  // (made by the jump kernel)
        // the generators on their own stream when the jump kernel made the final window (a one-round
        // generation with the frame-end jump): nothing after them on `st` reads what they write
        hipStream_t g = st;
        if (gst && gst != st && end && plan.rounds.size() == 1) {
            HIP_TRY(hipEventRecord(jumped, st));
            HIP_TRY(hipStreamWaitEvent(gst, jumped, 0));
            g = gst;
        }
        mt_gen_launch(c, G, R.nseg, g, win);
        HIP_TRY(hipGetLastError());
        if (gen_on) *gen_on = g;
        c->mt_dirty = false;
    }
    c->mt_cur ^= 1;
    *final_pos = plan.final_pos;
    return SRT_OK;
}

// Read back a completed frame (its stream has been synchronised): error/overflow flags OR-ed over
// every pass (and every asynchronous frame since the last synchronisation point), per-depth counts
// and kernel times of the frame's passes.  Returns SRT_RETRY_OVERFLOW when a queue shard overflowed.
// `retry` receives the RETRY_* bits of every pass.
constexpr int SRT_RETRY = 1;
int collect_frame(srt_ctx* c, const FramePlan& F, srt_stats& S, uint32_t* retry = nullptr) {
    uint32_t bits = 0;
    for (int p = 0; p < F.npass; ++p) {
        const uint32_t* hp = c->f->host + p * F.pass_words;
        int rc;
        if ((rc = check_flags(hp[F.cnt_words]))) return rc;
        bits |= hp[F.cnt_words + 1];
    }
    bits |= c->f->host[F.npass * F.pass_words + 2];
    if (bits & RETRY_CHAIN_TIE) c->chain_ok = false;  // no chain mode for this scene any more
    if (bits & RETRY_FIXED_RANGE) c->fx_ok = false;   // f64 atomics for this scene
    if (retry) *retry = bits;
    if (bits) return SRT_RETRY;
    double ms_trace = 0.0, ms_primary = 0.0;
    for (int d = 0; d < SRT_MAX_DEPTHS; ++d) S.rays_per_depth[d] = 0;
    for (int p = 0; p < F.npass; ++p) {
        const uint32_t* hp = c->f->host + p * F.pass_words;
        if (depth_total(hp + (int64_t)(F.dcap + 1) * NSHARD, (F.frame || F.fuse) ? INT64_MAX : c->f->seg) != 0)
            return fail(SRT_ERR_DEPTH, "rays alive after the depth cap");
        if (F.frame) {
            // k_frame counts every ray it traces (per shard), depth 0 included
            for (int d = 0; d <= F.dcap; ++d)
                for (int k = 0; k < NSHARD; ++k) S.rays_per_depth[d] += hp[(int64_t)d * NSHARD + k];
        } else {
            S.rays_per_depth[0] += (int64_t)std::min(F.batch, F.spp - p * F.batch) * F.npix;
            for (int d = 1; d <= F.dcap; ++d)
                S.rays_per_depth[d] += depth_total(hp + (int64_t)d * NSHARD, F.fuse ? INT64_MAX : c->f->seg);
        }
        const hipEvent_t* ev = c->f->ev.data() + (int64_t)p * F.nev;
        float ms;
        HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
        ms_primary += ms;
        HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[F.chain_from > 0 ? F.chain_from + 1 : F.dcap + 1]));
        ms_trace += ms;
    }
    const uint32_t* hshadow = c->f->host + F.npass * F.pass_words;
    S.passes = F.npass;
    S.ms_trace_kernels = ms_trace;
    S.ms_primary_kernel = ms_primary;
    S.ms_device = ms_trace;
    S.shadow_rays = (int64_t)(hshadow[0] | (uint64_t)hshadow[1] << 32);
    S.n_depths = F.dcap + 1;
    S.kernel_path = F.frame ? 1 : (F.fuse ? 2 : 0);
    S.chain_from = F.chain_from;
    S.total_rays = 0;
    for (int d = 0; d <= F.dcap; ++d) S.total_rays += S.rays_per_depth[d];
    // per-pass ray counts of this frame shape: the next frame's chain-mode plan
    c->hint_key[0] = F.npix; c->hint_key[1] = F.spp; c->hint_key[2] = F.batch;
    for (int d = 0; d < SRT_MAX_DEPTHS; ++d) c->hint[d] = S.rays_per_depth[d] / std::max(1, F.npass);
    return SRT_OK;
}

// zero the pinned flag words of every pass (only while no frame is in flight)
void clear_host_flags(srt_ctx* c, const FramePlan& F) {
    for (int p = 0; p < F.npass; ++p) {
        c->f->host[p * F.pass_words + F.cnt_words] = 0u;
        c->f->host[p * F.pass_words + F.cnt_words + 1] = 0u;
    }
    c->f->host[F.npass * F.pass_words + 2] = 0u;  // k_resolve's fixed-point range check
}

// Stream and counters of a slot, created on first use.
int ensure_slot(FrameSlot& f) {
    if (f.stream) return SRT_OK;
    HIP_TRY(hipStreamCreateWithFlags(&f.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&f.jit_ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&f.jit_free, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&f.mt_jumped, hipEventDisableTiming));
    HIP_TRY(dalloc(&f.counts, SRT_MAX_DEPTHS * NSHARD));
    HIP_TRY(dalloc(&f.flags, 2));
    HIP_TRY(dalloc(&f.shadow, NSHARD));
    f.dirty = true;
    return SRT_OK;
}

void free_slot(FrameSlot& f) {
    if (!f.stream) return;
    (void)hipStreamSynchronize(f.stream);
    free_list(f.queue_bufs);
    free_list(f.ring_bufs);
    void* bufs[] = {f.fb, f.fbg, f.fbx, f.rgb, f.u8, f.jit, f.hit, f.counts, f.flags, f.shadow, f.g_u8, f.g_rgb, f.full_u8, f.full_rgb,
                    f.mt_win};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : f.ev) (void)hipEventDestroy(e);
    if (f.host) (void)hipHostFree(f.host);
    (void)hipEventDestroy(f.jit_ready);
    (void)hipEventDestroy(f.jit_free);
    (void)hipEventDestroy(f.mt_jumped);
    (void)hipStreamDestroy(f.stream);
    f = FrameSlot{};
}

// Wait for the asynchronous frames in flight and check them (flags accumulated over all of them,
// stats of the last).  An overflow grows the queues and is reported as an error: those frames are
// wrong and must be rendered again.  Leaves slot 0 current.
int finish_async(srt_ctx* c, srt_stats* st) {
    c->retry_frame = false;
    if (c->async_pending == 0) {
        c->f = &c->slots[0];
        if (st) *st = c->async_stats;
        return SRT_OK;
    }
    for (FrameSlot& f : c->slots)
        if (f.stream) HIP_TRY(hipStreamSynchronize(f.stream));
    c->async_pending = 0;
    if (c->mt_chain) {  // numpy's state after the last asynchronous frame's draws
        HIP_TRY(hipMemcpy(c->mt_chain->key, mt_dump(c), rtmt::N * 4, hipMemcpyDeviceToHost));
        c->mt_chain->pos = c->mt_pos;
        c->mt_chain = nullptr;
    }
    int first_err = SRT_OK;
    bool overflow = false;
    srt_stats last{};
    for (int k = 0; k < MAX_FRAME_SLOTS; ++k) {
        FrameSlot& f = c->slots[(c->last_slot + 1 + k) % MAX_FRAME_SLOTS];  // the last frame's slot last
        if (!f.pending) continue;
        c->f = &f;
        srt_stats S{};
        uint32_t bits = 0;
        int rc = collect_frame(c, f.plan, S, &bits);
        clear_host_flags(c, f.plan);
        f.pending = 0;
        if (rc == SRT_RETRY) {
            overflow = true;
            if ((bits & RETRY_OVERFLOW) &&
                (rc = f.plan.frame ? ensure_ring(c, 2 * f.ring_cap) : ensure_queues(c, 2 * f.seg * NSHARD))) {
                first_err = first_err ? first_err : rc;
            }
        } else if (rc) {
            first_err = first_err ? first_err : rc;
        } else {
            last = S;
        }
    }
    c->f = &c->slots[0];
    if (first_err) return first_err;
    c->retry_frame = overflow;
    if (overflow)
        return fail(SRT_ERR_MEMORY, "a ray queue overflowed (queues grown), a tie met chain mode (chain mode "
                                    "off) or a colour left the fixed-point range (f64 sums from now on) during an "
                                    "asynchronous frame: render that frame again");
    c->async_stats = last;
    if (st) *st = last;
    return SRT_OK;
}

int64_t shard_npix(const FrameSlot::Gather& G, int nranks, int q) {
    return shard_rank_rows(G.H, nranks, q, G.band) * G.W;
}

// Post this rank's part of the frame's gather on its stream (inside an RCCL group): rank 0 receives
// every other rank's uint8 (and linear-RGB) tile, the others send theirs.
int gather_post(srt_ctx* c) {
    const FrameSlot::Gather& G = c->f->gather;
    if (!G.on || c->nranks == 1 || !c->comm) return SRT_OK;  // (no communicator: a rehearsed shard)
    hipStream_t st = c->f->stream;
    if (c->rank == 0) {
        for (int q = 1; q < c->nranks; ++q) {
            const int64_t np = shard_npix(G, c->nranks, q);
            NCCL_TRY(ncclRecv(c->f->g_u8 + (int64_t)q * G.maxpix * 3, (size_t)(3 * np), ncclUint8, q, c->comm, st));
            if (G.want_rgb)
                NCCL_TRY(ncclRecv(c->f->g_rgb + (int64_t)q * G.maxpix * 3, (size_t)(3 * np), ncclFloat64, q, c->comm, st));
        }
    } else {
        NCCL_TRY(ncclSend(c->f->u8, (size_t)(3 * G.npix), ncclUint8, 0, c->comm, st));
        if (G.want_rgb) NCCL_TRY(ncclSend(c->f->rgb, (size_t)(3 * G.npix), ncclFloat64, 0, c->comm, st));
    }
    return SRT_OK;
}

int gather_finish(srt_ctx* c);

// The frame's gather on its own (one rank per process): post it in a group, assemble on rank 0.
int gather_frame(srt_ctx* c) {
    if (c->nranks > 1) {
        NCCL_TRY(ncclGroupStart());
        int rc = gather_post(c);
        NCCL_TRY(ncclGroupEnd());
        if (rc) return rc;
    }
    return gather_finish(c);
}

// Rank 0, after the gather: the tiles into the frame, then to the caller's host buffers if any.
int gather_finish(srt_ctx* c) {
    const FrameSlot::Gather& G = c->f->gather;
    if (!G.on || c->rank != 0 || (c->nranks > 1 && !c->comm)) return SRT_OK;
    GatherTiles T{};
    for (int q = 0; q < c->nranks; ++q) {
        T.u8[q] = q == 0 ? c->f->u8 : c->f->g_u8 + (int64_t)q * G.maxpix * 3;
        T.rgb[q] = q == 0 ? c->f->rgb : c->f->g_rgb + (int64_t)q * G.maxpix * 3;
        T.npix[q] = shard_npix(G, c->nranks, q);
    }
    hipStream_t st = c->f->stream;
    hipLaunchKernelGGL(k_assemble, dim3(grid_for(G.W * G.H, c->max_blocks)), dim3(BLOCK), 0, st, T, c->nranks, G.band, G.W, G.H,
                       G.want_u8 ? G.dst_u8 : nullptr, G.want_rgb ? G.dst_rgb : nullptr);
    HIP_TRY(hipGetLastError());
    if (G.host_u8) HIP_TRY(hipMemcpyAsync(G.host_u8, G.dst_u8, (size_t)3 * G.W * G.H, hipMemcpyDeviceToHost, st));
    if (G.host_rgb)
        HIP_TRY(hipMemcpyAsync(G.host_rgb, G.dst_rgb, (size_t)3 * G.W * G.H * 8, hipMemcpyDeviceToHost, st));
    return SRT_OK;
}

}  // namespace

extern "C" {

int srt_abi_version(void) { return SRT_ABI_VERSION; }

const char* srt_last_error(void) { return g_err.c_str(); }

int srt_device_count(int* count) {
    if (!count) return fail(SRT_ERR_ARG, "count is null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(SRT_ERR_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return SRT_OK;
}

// frame slots by default: HIP's hardware queues per process (GPU_MAX_HW_QUEUES, default 4) but one
// for the generation stream, at least 4, at most MAX_FRAME_SLOTS
static int default_slots() {
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    const int q = e ? atoi(e) : 4;
    return std::max(4, std::min(MAX_FRAME_SLOTS, q - 1));
}

int srt_create(int device, srt_ctx** out) {
    if (!out) return fail(SRT_ERR_ARG, "out is null");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    srt_ctx* c = new srt_ctx();
    c->nslots = default_slots();
    c->device = device;
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    c->ncu = prop.multiProcessorCount;
    // 4 x OCC blocks per CU = the CU's resident wave slots (OCC per SIMD): one wave-sized block
    // (the frame kernel) per slot, or four rounds of the OCC resident 256-thread blocks of the
    // grid-stride kernels
    c->max_blocks = prop.multiProcessorCount * 4 * OCC;
    c->lean_blocks = prop.multiProcessorCount * 2;
    c->lean_blocks_shard = prop.multiProcessorCount * 4;
    int rc = ensure_slot(c->slots[0]);
    if (rc) {
        delete c;
        return rc;
    }
    *out = c;
    return SRT_OK;
}

int srt_destroy(srt_ctx* c) {
    if (!c) return SRT_OK;
    (void)hipSetDevice(c->device);
    (void)finish_async(c, nullptr);
    for (FrameSlot& f : c->slots) free_slot(f);
    free_list(c->scene_bufs);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->mt_done) (void)hipEventDestroy(c->mt_done);
    if (c->mt_stream) (void)hipStreamDestroy(c->mt_stream);
    void* bufs[] = {c->xs, c->ys, c->rows, c->mt, c->mt_out, c->texels, c->red, c->mt_y, c->lane_stats};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (auto& t : c->mt_bandtabs) {
        (void)hipFree(t.bands);
        (void)hipFree(t.polys);
    }
    for (auto& e : c->mt_end_polys) (void)hipFree(e.second);
    delete c;
    return SRT_OK;
}

int srt_set_option(srt_ctx* c, const char* key, int64_t value) {
    if (!c || !key) return fail(SRT_ERR_ARG, "null ctx/key");
    c->pf.valid = false;  // (an option may change the streams or the generation a prefetch assumed)
    if (!strcmp(key, "pipeline")) { c->pipeline = value != 0; return SRT_OK; }
    if (!strcmp(key, "bvh")) { c->use_bvh = value != 0; return SRT_OK; }
    if (!strcmp(key, "mt_bands")) { c->mt_bands_on = value != 0; return SRT_OK; }
    if (!strcmp(key, "collider_seq")) { c->seq_on = value != 0; return SRT_OK; }
    if (!strcmp(key, "mt_pipe_split")) {
        if (value != 0 && (value < 4096 || value > ((int64_t)1 << 24)))
            return fail(SRT_ERR_ARG, "mt_pipe_split: 0 or 4096 .. 2^24 doubles");
        c->mt_pipe_split = value;
        return SRT_OK;
    }
    if (!strcmp(key, "mt_gen_nt")) {
        if (value != 0 && value != 256 && value != 320) return fail(SRT_ERR_ARG, "mt_gen_nt: 0 (auto), 256 or 320");
        c->mt_gen_nt_opt = (int)value;
        return SRT_OK;
    }
    if (!strcmp(key, "sync_lean")) { c->sync_lean = value != 0; return SRT_OK; }
    if (!strcmp(key, "rehearse_assemble")) {
        if (value != 0 && (value < 2 || value > MAX_RANKS)) return fail(SRT_ERR_ARG, "rehearse_assemble: 0 or 2 .. 64");
        c->rehearse_assemble = (int)value;
        return SRT_OK;
    }
    if (!strcmp(key, "mt_short")) {
        if (value != 0 && (value < 4096 || value > ((int64_t)1 << 24))) return fail(SRT_ERR_ARG, "mt_short: 0 or 4096 .. 2^24 doubles");
        c->mt_short = value;
        return SRT_OK;
    }
    if (!strcmp(key, "mt_jump_parts")) {
        if (value != 0 && (value < MT_MIN_PARTS || value > MT_MAX_PARTS))
            return fail(SRT_ERR_ARG, "mt_jump_parts: 0 (auto) or 2 .. 8");
        c->mt_parts_opt = (int)value;
        return SRT_OK;
    }
    if (!strcmp(key, "shard_bands")) {
        if (value < 0 || value > 4096) return fail(SRT_ERR_ARG, "shard_bands: 0 (auto) .. 4096");
        c->shard_bands = (int)value;
        return SRT_OK;
    }
    if (!strcmp(key, "chain_rays")) { c->chain_rays = value; return SRT_OK; }
    if (!strcmp(key, "fuse_primary")) { c->fuse_primary = (int)value; return SRT_OK; }
    if (!strcmp(key, "frame_kernel")) { c->use_frame = value < 0 ? -1 : (value != 0); return SRT_OK; }
    if (!strcmp(key, "deterministic")) {
        HIP_TRY(hipSetDevice(c->device));
        int rc = finish_async(c, nullptr);
        if (rc) return rc;
        c->deterministic = value != 0;
        return SRT_OK;
    }
    if (!strcmp(key, "rehearse_shard")) {
        // diagnostic: act as rank (value & 255) of (value >> 8) ranks without a communicator, so one
        // GPU can render the shards of an N-rank frame in turn (no gather; SRT_RENDER_RGB_ROWS still
        // writes the rank's rows into the host frame).  0 ends the rehearsal.
        if (c->comm) return fail(SRT_ERR_ARG, "the context has a communicator");
        const int n = value ? (int)(value >> 8) : 1, r = value ? (int)(value & 255) : 0;
        if (n < 1 || n > MAX_RANKS || r >= n) return fail(SRT_ERR_ARG, "rehearse_shard: (nranks << 8) | rank");
        HIP_TRY(hipSetDevice(c->device));
        int rc = finish_async(c, nullptr);
        if (rc) return rc;
        c->nranks = n;
        c->rank = r;
        return SRT_OK;
    }
    return fail(SRT_ERR_ARG, std::string("unknown option ") + key);
}

int srt_upload_scene(srt_ctx* c, const srt_scene_desc* d) {
    if (!c || !d) return fail(SRT_ERR_ARG, "null ctx/scene");
    if (d->n_colliders < 0 || d->n_materials < 0 || d->n_media < 1 || d->n_media > 255)
        return fail(SRT_ERR_ARG, "scene needs 1 <= n_media <= 255 (row 0 = scene.n)");
    for (int i = 0; i < d->n_colliders; ++i) {
        const srt_collider& cc = d->colliders[i];
        if (cc.type < 0 || cc.type > 3) return fail(SRT_ERR_ARG, "bad collider type");
        if (cc.material < 0 || cc.material >= d->n_materials) return fail(SRT_ERR_ARG, "collider material out of range");
    }
    if (!d->media) return fail(SRT_ERR_ARG, "media table is null");
    if (d->n_lights > 0 && d->n_colliders > 0 && !d->light_local) return fail(SRT_ERR_ARG, "light_local is null");
    if (d->n_importance > 0 && !d->importance) return fail(SRT_ERR_ARG, "importance table is null");
    if (d->n_textures > 0 && (!d->textures || (d->texel_bytes > 0 && !d->texels)))
        return fail(SRT_ERR_ARG, "texture tables are null");
    for (int i = 0; i < d->n_textures; ++i) {
        const srt_texture& t = d->textures[i];
        if (t.height <= 0 || t.width <= 0 || t.channels < 3 || t.channel0 < 0 || t.channel0 + 3 > t.channels ||
            t.idx_h <= 0 || t.idx_w <= 0 || t.offset < 0 ||
            t.offset + (int64_t)t.height * t.width * t.channels > d->texel_bytes)
            return fail(SRT_ERR_ARG, "texture record out of the texel pool");
    }
    for (int i = 0; i < d->n_materials; ++i) {
        const srt_material& m = d->materials[i];
        if (m.type == SRT_GLOSSY && !d->glossy_f0) return fail(SRT_ERR_ARG, "glossy_f0 table is null");
        int texs[4] = {m.tex, m.tex_aux0, m.tex_aux1, m.normalmap};
        for (int t : texs)
            if (t >= d->n_textures) return fail(SRT_ERR_ARG, "material texture index out of range");
        if (m.type == SRT_REFRACTIVE && (m.medium < 0 || m.medium >= d->n_media))
            return fail(SRT_ERR_ARG, "refractive medium out of range");
        if ((m.type == SRT_SKY && m.tex < 0) || (m.type == SRT_THINFILM && (m.tex_aux0 < 0 || m.tex_aux1 < 0)))
            return fail(SRT_ERR_ARG, "material is missing a required texture");
        if (m.type == SRT_DIFFUSE && (m.ival < 1 || m.ival > 255)) return fail(SRT_ERR_ARG, "diffuse_rays must be 1..255");
    }
    HIP_TRY(hipSetDevice(c->device));
    int rc0 = finish_async(c, nullptr);  // frames in flight read the scene tables freed below
    if (rc0) return rc0;
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    free_list(c->scene_bufs);
    c->has_scene = false;
    SceneView S{};
    int rc;
    srt_collider* col;
    srt_material* mat;
    srt_texture* tex;
    uint8_t* texels;
    srt_light* lights;
    double *media, *f0, *ll, *imp;
    if ((rc = upload(c, d->colliders, d->n_colliders, &col))) return rc;
    if ((rc = upload(c, d->materials, d->n_materials, &mat))) return rc;
    // texel pool in HBM: 3-channel images as 4-byte texels (RGBX), so that a texel is one aligned
    // dword load (texel_rgb) instead of three byte loads; the records point into that layout
    std::vector<srt_texture> tex_h(d->textures, d->textures + std::max(0, d->n_textures));
    std::vector<std::array<int64_t, 4>> imgs;  // (offset, bytes, new offset, expand) per image
    bool rgbx = d->texel_bytes > 0 && d->texels && !is_device_ptr(d->texels);
    if (rgbx) {
        for (const srt_texture& t : tex_h) {
            const int64_t bytes = (int64_t)t.height * t.width * t.channels;
            bool seen = false;
            for (auto& im : imgs)
                if (im[0] == t.offset) {
                    seen = true;
                    rgbx = rgbx && im[1] == bytes;  // (one image per offset, else the pool stays as given)
                }
            if (!seen) imgs.push_back({t.offset, bytes, 0, t.channels == 3 ? 1 : 0});
        }
        std::sort(imgs.begin(), imgs.end());
        for (size_t k = 1; k < imgs.size(); ++k) rgbx = rgbx && imgs[k][0] >= imgs[k - 1][0] + imgs[k - 1][1];
    }
    int64_t pool_bytes = d->texel_bytes;
    if (rgbx) {
        pool_bytes = 0;
        for (auto& im : imgs) {
            im[2] = pool_bytes;
            pool_bytes += ((im[3] ? im[1] / 3 * 4 : im[1]) + 3) / 4 * 4;
        }
        for (srt_texture& t : tex_h)
            for (auto& im : imgs)
                if (im[0] == t.offset) {
                    t.offset = im[2];
                    if (im[3]) t.channels = 4;
                }
    }
    if ((rc = upload(c, tex_h.data(), d->n_textures, &tex))) return rc;
    // the pool's layout: the images (caller offset, bytes, pool offset, expanded) it holds, or the
    // caller's pool as given -- a key reused with another image set must not reuse the pool
    uint64_t layout = 1469598103934665603ull;
    auto mix = [&layout](int64_t v) { layout = (layout ^ (uint64_t)v) * 1099511628211ull; };
    mix(pool_bytes);
    mix(rgbx);
    if (rgbx)
        for (const auto& im : imgs)
            for (int64_t v : im) mix(v);
    // kept in HBM across uploads while the caller's key and size and the layout are unchanged
    if (d->texel_key != 0 && d->texel_key == c->texel_key && d->texel_bytes == c->texel_bytes && c->texels &&
        rgbx == c->texels_rgbx && layout == c->texel_layout) {
        texels = c->texels;
    } else {
        if (c->texels) (void)hipFree(c->texels);
        c->texels = nullptr;
        c->texel_key = 0;
        c->texel_bytes = 0;
        texels = nullptr;
        if (d->texel_bytes > 0 && d->texels) {
            HIP_TRY(dalloc(&texels, pool_bytes));
            if (rgbx) {
                std::vector<uint8_t> h((size_t)pool_bytes, 0);
                for (const auto& im : imgs) {
                    const uint8_t* src = d->texels + im[0];
                    uint8_t* dst = h.data() + im[2];
                    if (im[3]) {
                        for (int64_t i = 0, n = im[1] / 3; i < n; ++i) memcpy(dst + 4 * i, src + 3 * i, 3);
                    } else {
                        memcpy(dst, src, (size_t)im[1]);
                    }
                }
                HIP_TRY(hipMemcpy(texels, h.data(), (size_t)pool_bytes, hipMemcpyHostToDevice));
            } else {
                HIP_TRY(hipMemcpy(texels, d->texels, (size_t)d->texel_bytes, hipMemcpyDefault));
            }
            c->texels = texels;
            c->texel_key = d->texel_key;
            c->texel_bytes = d->texel_bytes;
            c->texels_rgbx = rgbx;
            c->texel_layout = layout;
        }
    }
    if ((rc = upload(c, d->lights, d->n_lights, &lights))) return rc;
    if ((rc = upload(c, d->media, (int64_t)d->n_media * 6, &media))) return rc;
    if ((rc = upload(c, d->glossy_f0, (int64_t)d->n_materials * d->n_media * 3, &f0))) return rc;
    if ((rc = upload(c, d->light_local, (int64_t)d->n_lights * d->n_colliders * 3, &ll))) return rc;
    if ((rc = upload(c, d->importance, (int64_t)d->n_importance * 4, &imp))) return rc;
    // (casts: in the device compilation the SceneView fields are constant-address-space pointers)
    S.col = (decltype(S.col))col; S.mat = (decltype(S.mat))mat; S.tex = (decltype(S.tex))tex;
    S.texels = (decltype(S.texels))texels; S.lights = (decltype(S.lights))lights;
    S.media = (decltype(S.media))media; S.glossy_f0 = (decltype(S.glossy_f0))f0;
    S.light_local = (decltype(S.light_local))ll; S.importance = (decltype(S.importance))imp;
    S.ncol = d->n_colliders; S.nmat = d->n_materials; S.ntex = d->n_textures; S.nlights = d->n_lights;
    S.nmedia = d->n_media; S.nimp = d->n_importance;
    S.sky_col = sky_collider(d->colliders, d->n_colliders, d->materials);
    S.nshadow = 0;
    bool lin_tri = false;
    {
        // triangle meshes: BVH over the Triangle colliders, the rest intersected one by one
        BvhBuild B;
        lin_tri = false;
        if (c->use_bvh) {
            bvh_build(d->colliders, d->n_colliders, B);
        } else {
            for (int i = 0; i < d->n_colliders; ++i) B.lin.push_back(i);
        }
        int32_t *lin, *tri;
        BvhNode* nodes;
        if ((rc = upload(c, B.lin.data(), (int64_t)B.lin.size(), &lin))) return rc;
        if ((rc = upload(c, B.tri.data(), (int64_t)B.tri.size(), &tri))) return rc;
        if ((rc = upload(c, B.nodes.data(), (int64_t)B.nodes.size(), &nodes))) return rc;
        S.nlin = (int)B.lin.size();
        S.lin = (decltype(S.lin))lin;
        S.bvh_tri = (decltype(S.bvh_tri))tri;
        S.bvh = (decltype(S.bvh))nodes;
        S.bvh_nodes = (int)B.nodes.size();
        S.bvh_bound = B.bound;
        for (int k : B.lin) lin_tri |= d->colliders[k].type == SRT_TRIANGLE;
    }
    int fan = 1;
    c->has_diffuse = 0;
    for (int i = 0; i < d->n_colliders; ++i)
        if (d->colliders[i].flags & SRT_CF_SHADOW) S.nshadow++;
    for (int i = 0; i < d->n_materials; ++i) {
        const srt_material& m = d->materials[i];
        if (m.type == SRT_REFRACTIVE || m.type == SRT_THINFILM) fan = std::max(fan, 2);
        if (m.type == SRT_DIFFUSE) { fan = std::max(fan, std::max(1, (int)m.ival)); c->has_diffuse = 1; }
    }
    for (int k = 0; k < 3; ++k) S.ambient[k] = d->ambient[k];
    S.lut_lds = nullptr;
    S.nlut_lds = std::min(d->n_textures, MAX_LUT_LDS);
    c->S = S;
    c->max_depth = std::max(0, (int)d->max_ray_depth);
    c->fanout = fan;
    c->mats = 0;
    for (int i = 0; i < d->n_materials; ++i) c->mats |= mat_bit(d->materials[i].type);
    if (S.bvh_nodes > 0) c->mats |= MAT_BVH | MAT_TRI;  // (a tied ray re-tests its colliders, triangles too)
    if (lin_tri) c->mats |= MAT_TRI;  // Triangle colliders outside the BVH
    for (int i = 0; i < d->n_materials; ++i)
        if (d->materials[i].normalmap >= 0) c->mats |= MAT_NMAP;
    c->seq = 0;
    if (S.bvh_nodes == 0 && d->n_colliders <= SEQ_MAX) {
        int types[SEQ_MAX];
        for (int i = 0; i < d->n_colliders; ++i) types[i] = d->colliders[i].type;
        c->seq = seq_encode(types, d->n_colliders);
    }
    c->chain_ok = true;
    c->hint_key[0] = -1;  // ray counts of another scene are no plan for this one
    c->has_scene = true;
    c->fx_ok = true;
    return SRT_OK;
}


}  // extern "C"
namespace {
// srt_render, or with `prefetch` srt_render_prefetch: the same planning, then only the first pass's
// numpy-stream generation is queued (srt_ctx::pf) and the call returns
int render_impl(srt_ctx* c, const srt_camera* cam, const srt_render_args* a, srt_stats* st, bool prefetch) {
    auto t_start = std::chrono::steady_clock::now();
    if (!c || !cam || !a) return fail(SRT_ERR_ARG, "null argument");
    const srt_ctx::MtPrefetch pf_in = c->pf;  // (a prefetch is used by the next render only)
    c->pf.valid = false;
    if (!prefetch && !c->has_scene) return fail(SRT_ERR_NOSCENE, "no scene uploaded");
    if (a->flags & ~(SRT_RENDER_ASYNC | SRT_RENDER_SHARDED | SRT_RENDER_GATHER_RGB | SRT_RENDER_RGB_ROWS |
                     SRT_RENDER_RGB_LOCAL | SRT_RENDER_RGBX))
        return fail(SRT_ERR_ARG, "unknown render flag");
    if ((a->flags & SRT_RENDER_RGBX) && (a->flags & SRT_RENDER_SHARDED))
        return fail(SRT_ERR_ARG, "SRT_RENDER_RGBX: not with SRT_RENDER_SHARDED");
    if ((a->flags & SRT_RENDER_RGB_LOCAL) && (a->out_rgb || (a->flags & (SRT_RENDER_GATHER_RGB | SRT_RENDER_RGB_ROWS))))
        return fail(SRT_ERR_ARG, "SRT_RENDER_RGB_LOCAL needs out_rgb NULL and no SRT_RENDER_GATHER_RGB / RGB_ROWS");
    if ((a->flags & SRT_RENDER_RGB_ROWS) &&
        (!(a->flags & SRT_RENDER_SHARDED) || (a->flags & SRT_RENDER_GATHER_RGB) || !a->out_rgb))
        return fail(SRT_ERR_ARG, "SRT_RENDER_RGB_ROWS needs SRT_RENDER_SHARDED, out_rgb and no SRT_RENDER_GATHER_RGB");
    const bool async = (a->flags & SRT_RENDER_ASYNC) != 0;
    const bool sharded = (a->flags & SRT_RENDER_SHARDED) != 0;
    if (a->spp <= 0 || cam->width <= 0 || cam->height <= 0 || (!sharded && a->n_rows <= 0) || !cam->xs || !cam->ys)
        return fail(SRT_ERR_ARG, "spp, width, height, n_rows must be positive and xs/ys set");
    if (a->jitter && a->mt) return fail(SRT_ERR_ARG, "jitter and mt are exclusive");
    const bool use_mt = a->mt != nullptr;
    if (use_mt && (a->mt->pos < 0 || a->mt->pos > rtmt::N)) return fail(SRT_ERR_ARG, "bad numpy RNG position");
    // a prefetch covers synchronous whole frames drawing numpy's stream (Scene.render); others: nothing
    if (prefetch && (async || sharded || !use_mt || a->rows || a->n_rows != cam->height)) return SRT_OK;
    // rows of this call
    std::vector<int32_t> rows_h;
    const int32_t* rows_src = nullptr;
    int n_rows = a->n_rows;
    int64_t band = 1;  // row-band height of a sharded frame
    if (sharded) {
        if (c->nranks > MAX_RANKS) return fail(SRT_ERR_ARG, "too many ranks");
        if (cam->height < c->nranks) return fail(SRT_ERR_ARG, "a sharded frame needs at least one row per rank");
        if (a->out_hit_id) return fail(SRT_ERR_ARG, "hit ids of a sharded frame are not gathered");
        band = shard_band_height(cam->height, c->nranks, shard_kmax(cam->height, c->nranks, c->shard_bands, c->fanout));
        rows_h = band_rows(cam->height, c->nranks, c->rank, band);
        n_rows = (int)rows_h.size();
        if (n_rows == 0) return fail(SRT_ERR_ARG, "a sharded frame left this rank without rows");
        rows_src = rows_h.data();
    } else if (a->rows) {
        if (is_device_ptr(a->rows)) return fail(SRT_ERR_ARG, "rows must be host memory");
        for (int k = 0; k < a->n_rows; ++k)
            if (a->rows[k] < 0 || a->rows[k] >= cam->height) return fail(SRT_ERR_ARG, "row index out of range");
        rows_src = a->rows;
    } else {
        if (a->n_rows > cam->height) return fail(SRT_ERR_ARG, "n_rows > height");
        rows_h.resize(a->n_rows);
        for (int k = 0; k < a->n_rows; ++k) rows_h[k] = k;
        rows_src = rows_h.data();
    }
    HIP_TRY(hipSetDevice(c->device));
    const int64_t W = cam->width, Hf = cam->height;
    const int64_t npix = (int64_t)n_rows * W;
    if (W * Hf >= ((int64_t)1 << 31)) return fail(SRT_ERR_ARG, "image too large");
    const int jk = ptr_kind(a->jitter), hk = ptr_kind(a->out_hit_id);
    const int rk = ptr_kind(a->out_rgb), uk = ptr_kind(a->out_srgb8);
    const bool jit_dev = jk == 1, hit_dev = hk == 1, rgb_dev = rk == 1, u8_dev = uk == 1;
    if (async && (jk >= 2 || hk >= 2 || rk == 3 || uk == 3))
        return fail(SRT_ERR_ARG, "an asynchronous render takes device (or NULL) jitter and hit ids, and device or "
                                 "pinned host (srt_host_alloc) outputs");
    // outputs written by this rank: a shard's tiles stay on the device (the gather reads them); rank 0
    // of a sharded frame writes the whole frame to the caller's buffers after the gather
    const bool gather_rgb = sharded && (a->flags & SRT_RENDER_GATHER_RGB) != 0;
    const bool rgb_rows = sharded && (a->flags & SRT_RENDER_RGB_ROWS) != 0;
    if (rgb_rows && ptr_kind(a->out_rgb) != 2)
        return fail(SRT_ERR_ARG, "SRT_RENDER_RGB_ROWS: out_rgb must be pinned or registered host memory");
    int rc;
    // samples per pass: both queues must hold spp_pass * npix * fanout rays
    const int64_t per_sample = npix * c->fanout;
    const int64_t budget_rays = c->queue_budget / (2 * RAY_BYTES);
    int batch = a->batch_spp > 0 ? a->batch_spp
                                 : (int)std::max<int64_t>(1, std::min<int64_t>(1 << 20, budget_rays / per_sample));
    batch = std::min(batch, a->spp);
    while (batch > 1 && (int64_t)batch * npix * c->fanout >= ((int64_t)1 << 32) - 1) batch /= 2;
    // the numpy stream of a pass (its samples of the whole frame) is generated into the jitter buffer
    if (use_mt) while (batch > 1 && (int64_t)batch * 4 * W * Hf * 8 > ((int64_t)8 << 30)) batch /= 2;
    FramePlan F;
    F.npix = npix;
    F.W = W;
    F.H = Hf;
    F.sharded = sharded;
    F.gather_rgb = gather_rgb;
    F.use_mt = use_mt;
    F.spp = a->spp;
    F.batch = batch;
    F.npass = (a->spp + batch - 1) / batch;
    F.dcap = depth_cap(c);
    F.nev = F.dcap + 2;  // events per pass: before k_primary, after each depth
    F.cnt_words = (int64_t)SRT_MAX_DEPTHS * NSHARD;
    F.pass_words = F.cnt_words + 2;
    F.frame = c->use_frame < 0 ? c->fanout > 1 : c->use_frame != 0;
    const int64_t ntiles = frame_tiles(frame_tile_for(pick_variant(c->mats, c->seq_on ? c->seq : 0).mats), W, npix / W);
    if (F.frame) {
        // a frame kernel block traces one 64-pixel tile through the pass's samples: a small frame (a
        // shard of a multi-GPU frame) has too few tiles to fill the GPU, so its samples are split
        // into groups, one block per (tile, group), until there are ~4 blocks per resident wave
        // slot (c->max_blocks = 4 OCC per CU)
        const int64_t want = 4 * (int64_t)c->max_blocks;
        const int64_t g = (want + ntiles - 1) / ntiles;
        F.groups = (int)std::max<int64_t>(1, std::min<int64_t>(g, batch));
    }
    // fused paths (single-child scenes): by default when the frame's threads (sample groups
    // included, pix_groups) fill two rounds of the resident threads
    F.fuse = !F.frame && c->fanout == 1 && c->chain_ok && pick_variant(c->mats, c->seq_on ? c->seq : 0).fused &&
             (c->fuse_primary > 0 ||
              (c->fuse_primary < 0 && npix * pix_groups(c, npix, batch, true) >= fused_items(c)));
    if (!F.fuse && !F.frame && c->fanout == 1 && c->chain_ok && c->hint_key[0] == npix && c->hint_key[1] == a->spp &&
        c->hint_key[2] == batch) {
        for (int d = 1; d <= F.dcap; ++d)
            if (c->hint[d] < c->chain_rays) { F.chain_from = d; break; }
    }
    // the slot of this frame: slot 0 for a synchronous frame (after the frames in flight),
    // alternating slots for asynchronous ones
    if (!async) {
        if ((rc = finish_async(c, nullptr))) return rc;
    } else {
        FrameSlot& f = c->slots[c->next_slot];
        if ((rc = ensure_slot(f))) return rc;
        c->f = &f;
    }
    // numpy stream of a shard (rows not the whole frame): band mode, only the rows' runs generated
    // (rt_mt_kernel.h MtArgs::bands); tables for the full passes and the last pass
    const int mt_pm = cam->lens_radius != 0.0 ? 15 : 3;  // a pinhole camera reads planes 0 and 1 only
    const srt_ctx::MtBandTab* mt_bt[2] = {nullptr, nullptr};
    int64_t mt_win_need = (int64_t)rtmt::SEGS * rtmt::N;
    // (the band tables and end polynomials are kept per frame shape; a context that has seen many
    // shapes drops them between frames, when no frame in flight reads them)
    if (c->async_pending == 0 && (c->mt_bandtabs.size() >= 16 || c->mt_end_polys.size() >= 64)) {
        HIP_TRY(hipDeviceSynchronize());
        for (auto& t : c->mt_bandtabs) {
            (void)hipFree(t.bands);
            (void)hipFree(t.polys);
        }
        c->mt_bandtabs.clear();
        for (auto& e : c->mt_end_polys) (void)hipFree(e.second);
        c->mt_end_polys.clear();
    }
    // a whole frame with nothing in flight (synchronous, or the first of a pipeline): short segments in
    // band mode (srt_ctx::mt_short); later pipelined frames generate behind their predecessors in
    // band-mode segments of mt_pipe_split doubles (0: the tabulated 2^19-word segments)
    const int64_t whole_split = n_rows < Hf ? 0
                              : c->async_pending == 0 ? c->mt_short
                                                                           : c->mt_pipe_split;
    if (use_mt && c->mt_bands_on && (n_rows < Hf || whole_split > 0)) {
        const int last_ns = a->spp - (F.npass - 1) * batch;
        const int64_t split = n_rows < Hf ? (int64_t)1 << 18 : whole_split;
        for (int k = 0; k < 2; ++k) {
            if ((rc = mt_band_table(c, W, Hf, k == 0 ? batch : last_ns, mt_pm, rows_src, n_rows, split, &mt_bt[k])))
                return rc;
            if (mt_bt[k]) mt_win_need = std::max(mt_win_need, (int64_t)(mt_bt[k]->nseg + 1) * rtmt::N);
        }
        if (!mt_bt[0] || !mt_bt[1]) mt_bt[0] = mt_bt[1] = nullptr;
    }
    // band mode stores a shard's jitter in its own layout [s][plane][its rows][W] (1/N of the frame's)
    // when every pass generates in band mode (a pass whose generation ends inside the key window
    // takes the tabulated segments and the frame's layout)
    auto pass_words = [&](int ns, bool last) { return 2 * ((int64_t)ns * 4 * W * Hf + (last ? 4 * W * Hf : 0)); };
    const bool jit_compact = mt_bt[0] && rtmt::end_jump(pass_words(a->spp - (F.npass - 1) * batch, true)) > 0 &&
                             (F.npass == 1 || rtmt::end_jump(pass_words(batch, false)) > 0);
    const int64_t jit_doubles = use_mt ? (int64_t)batch * 4 * (jit_compact ? npix : W * Hf)
                                       : (a->jitter && !jit_dev ? (int64_t)batch * 4 * npix : 0);
    const int64_t maxpix = sharded ? shard_max_rows(Hf, c->nranks, band) * W : 0;  // the gather's tile
    // rank 0's assembly rehearsed (srt_ctx::rehearse_assemble): these rows are rank 0's of an n-rank job
    int reh_n = 0;
    int64_t reh_band = 1, reh_maxpix = 0;
    if (c->rehearse_assemble > 1 && !sharded && a->rows && a->out_srgb8 && ptr_kind(a->out_srgb8) != 1 &&
        !(a->flags & SRT_RENDER_RGBX)) {
        const int n = c->rehearse_assemble;
        reh_band = shard_band_height(Hf, n, shard_kmax(Hf, n, c->shard_bands, c->fanout));
        const std::vector<int32_t> r0 = band_rows(Hf, n, 0, reh_band);
        if ((int)r0.size() == n_rows && std::equal(r0.begin(), r0.end(), rows_src)) {
            reh_n = n;
            reh_maxpix = shard_max_rows(Hf, n, reh_band) * W;
        }
    }
    // frames in flight use the buffers below: a frame that would reallocate anything first waits
    // for them (and reports their errors)
    if (async && c->async_pending > 0) {
        const FramePlan& pp = c->f->pending ? c->f->plan : c->slots[c->last_slot].plan;
        const bool same = W <= c->cam_cap[0] && cam->height <= c->cam_cap[1] && n_rows <= c->cam_cap[2] &&
                          3 * npix <= c->f->fb_cap && fx_words(npix) <= c->f->fbx_cap && 3 * npix <= c->f->rgb_cap &&
                          3 * npix <= c->f->u8_cap &&
                          jit_doubles <= c->f->jit_cap && (!use_mt || (mt_win_need <= c->f->mt_win_cap && !c->mt_dirty)) &&
                          (F.frame || (int64_t)batch * npix * c->fanout <= c->f->seg * NSHARD) &&
                          (!F.frame || c->f->ring_cap > 0) && F.npass == pp.npass && F.dcap == pp.dcap &&
                          F.frame == pp.frame && F.chain_from == pp.chain_from && F.fuse == pp.fuse && F.W == pp.W && F.H == pp.H &&
                          F.groups == pp.groups && (F.groups == 1 || (int64_t)F.groups * 3 * npix <= c->f->fbg_cap) &&
                          F.sharded == pp.sharded && F.gather_rgb == pp.gather_rgb && F.use_mt == pp.use_mt &&
                          (!reh_n || (c->f->g_u8_cap >= reh_n * reh_maxpix * 3 && c->f->full_u8_cap >= 3 * W * Hf)) &&
                          (!(a->flags & SRT_RENDER_RGBX) || c->f->full_u8_cap >= 4 * npix) &&
                          (!sharded || c->rank != 0 ||
                           (c->f->g_u8_cap >= c->nranks * maxpix * 3 && c->f->full_u8_cap >= 3 * W * Hf &&
                            (!gather_rgb || (c->f->g_rgb_cap >= c->nranks * maxpix * 3 && c->f->full_rgb_cap >= 3 * W * Hf)))) &&
                          (int)c->f->ev.size() >= F.npass * F.nev && c->f->host_words >= F.npass * F.pass_words + 2;
        if (!same) {
            FrameSlot* keep = c->f;
            if ((rc = finish_async(c, nullptr))) return rc;
            c->f = keep;
        }
    }
    {
        const void* old[3] = {c->xs, c->ys, c->rows};
        if ((rc = ensure_buf(&c->xs, c->cam_cap[0], W))) return rc;
        if ((rc = ensure_buf(&c->ys, c->cam_cap[1], cam->height))) return rc;
        if ((rc = ensure_buf(&c->rows, c->cam_cap[2], n_rows))) return rc;
        const void* now[3] = {c->xs, c->ys, c->rows};
        for (int k = 0; k < 3; ++k)
            if (old[k] != now[k]) c->cam_host[k].clear();
    }
    // camera tables: uploaded only when they change (a render loop re-sends the same ones)
    if ((rc = upload_if_changed(c, c->xs, c->cam_host[0], cam->xs, (size_t)W * 8))) return rc;
    if ((rc = upload_if_changed(c, c->ys, c->cam_host[1], cam->ys, (size_t)cam->height * 8))) return rc;
    if ((rc = upload_if_changed(c, c->rows, c->cam_host[2], rows_src, (size_t)n_rows * 4))) return rc;
    if (use_mt && (rc = mt_ensure(c))) return rc;
    // per-slot buffers of this frame shape (for an asynchronous frame also those of the other slot
    // while it is idle, so that the pipeline's first frame on it allocates nothing)
    auto ensure_frame = [&](FrameSlot& fs) -> int {
        FrameSlot* keep = c->f;
        c->f = &fs;
        int r = SRT_OK;
        if (!r) r = ensure_buf(&c->f->fb, c->f->fb_cap, 3 * npix);
        if (!r && F.groups > 1) r = ensure_buf(&c->f->fbg, c->f->fbg_cap, (int64_t)F.groups * 3 * npix);
        if (!r) r = ensure_buf(&c->f->fbx, c->f->fbx_cap, fx_words(npix));
        if (!r) r = ensure_buf(&c->f->rgb, c->f->rgb_cap, 3 * npix);
        if (!r) r = ensure_buf(&c->f->u8, c->f->u8_cap, 3 * npix);
        if (!r && jit_doubles > 0) r = ensure_buf(&c->f->jit, c->f->jit_cap, jit_doubles);
        if (!r && use_mt) r = mt_win_ensure(c, *c->f, mt_win_need);
        if (!r && a->out_hit_id && !hit_dev) r = ensure_buf(&c->f->hit, c->f->hit_cap, (int64_t)batch * npix);
        if (!r && (a->flags & SRT_RENDER_RGBX)) r = ensure_buf(&c->f->full_u8, c->f->full_u8_cap, 4 * npix);
        if (!r && reh_n) {
            const int64_t had = c->f->g_u8_cap;
            r = ensure_buf(&c->f->g_u8, c->f->g_u8_cap, reh_n * reh_maxpix * 3);
            if (!r && c->f->g_u8_cap != had && hipMemset(c->f->g_u8, 0, (size_t)c->f->g_u8_cap) != hipSuccess)
                r = fail(SRT_ERR_HIP, "hipMemset failed");  // (stand-in tiles: defined bytes)
            if (!r) r = ensure_buf(&c->f->full_u8, c->f->full_u8_cap, 3 * W * Hf);
        }
        if (!r && sharded && c->rank == 0) {
            r = ensure_buf(&c->f->g_u8, c->f->g_u8_cap, c->nranks * maxpix * 3);
            if (!r) r = ensure_buf(&c->f->full_u8, c->f->full_u8_cap, 3 * W * Hf);
            if (!r && gather_rgb) r = ensure_buf(&c->f->g_rgb, c->f->g_rgb_cap, c->nranks * maxpix * 3);
            if (!r && gather_rgb) r = ensure_buf(&c->f->full_rgb, c->f->full_rgb_cap, 3 * W * Hf);
        }
        // (a split ring: each half that size)
        if (!r) r = F.frame ? ensure_ring(c, (int64_t)FRAME_BLOCK * (c->fanout + 2) * 2 *
                                                 (frame_split_for(pick_variant(c->mats, c->seq_on ? c->seq : 0).mats) ? 2 : 1))
                            : ensure_queues(c, (int64_t)batch * npix * c->fanout);
        if (!r && (int)c->f->ev.size() < F.npass * F.nev) {
            for (hipEvent_t e : c->f->ev) (void)hipEventDestroy(e);
            c->f->ev.assign(F.npass * F.nev, nullptr);
            for (auto& e : c->f->ev)
                if (hipEventCreate(&e) != hipSuccess) r = fail(SRT_ERR_HIP, "hipEventCreate failed");
        }
        // per-pass counters and flags come back through pinned memory once, at the end of the
        // frame: the passes, the resolve and the output copies are queued without a host round trip
        if (!r && c->f->host_words < F.npass * F.pass_words + 3) {
            if (c->f->host) (void)hipHostFree(c->f->host);
            c->f->host = nullptr;
            c->f->host_words = 0;
            if (hipHostMalloc((void**)&c->f->host, (size_t)(F.npass * F.pass_words + 3) * 4, hipHostMallocDefault) !=
                hipSuccess) {
                r = fail(SRT_ERR_MEMORY, "pinned host allocation failed");
            } else {
                c->f->host_words = F.npass * F.pass_words + 3;  // + shadow count (2), resolve's fx check
                memset(c->f->host, 0, (size_t)c->f->host_words * 4);  // depths beyond used_words stay zero
            }
        }
        c->f = keep;
        return r;
    };
    if ((rc = ensure_frame(*c->f))) return rc;
    if (async || c->pipeline) {
        for (int k = 0; k < c->nslots; ++k) {
            FrameSlot& other = c->slots[k];
            if (&other != c->f && other.pending == 0) {
                if ((rc = ensure_slot(other))) return rc;
                if ((rc = ensure_frame(other))) return rc;
            }
        }
    }
    if (use_mt && !c->mt_done) HIP_TRY(hipEventCreateWithFlags(&c->mt_done, hipEventDisableTiming));
    const Variant& V = pick_variant(c->mats, c->seq_on ? c->seq : 0);
    // resolve targets: outputs in device memory are written in place by the resolve; host outputs
    // are resolved into the slot buffers and copied by DMA on the frame's stream (57 GB/s measured
    // for the ex1 1080p RGB, against 28 GB/s for a resolve kernel storing straight into pinned
    // memory over PCIe); a shard resolves into its slot tiles (gathered afterwards)
    const bool rgb_direct = rk == 1, u8_direct = uk == 1;
    const bool rgb_local = (a->flags & SRT_RENDER_RGB_LOCAL) != 0;
    double* res_rgb = rgb_local ? c->f->rgb
                    : sharded ? ((gather_rgb || rgb_rows) ? c->f->rgb : nullptr)
                              : a->out_rgb ? (rgb_direct ? a->out_rgb : c->f->rgb) : nullptr;
    const bool rgbx = (a->flags & SRT_RENDER_RGBX) && a->out_srgb8;
    uint8_t* res_u8 = (sharded || rgbx) ? c->f->u8 : a->out_srgb8 ? (u8_direct ? a->out_srgb8 : c->f->u8) : nullptr;
    // only the depths this frame can reach are handed back and cleared per pass
    const int64_t used_words = std::min<int64_t>(F.cnt_words, (int64_t)(F.dcap + 2) * NSHARD);
    // the numpy stream continues on the device from the previous asynchronous frame (same `mt`)
    const bool mt_chained = use_mt && async && c->async_pending > 0 && c->mt_chain == a->mt;
    srt_stats S{};
    // this frame's first-pass generation already queued by srt_render_prefetch (same stream state,
    // same frame shape, nothing generated since): not launched again (the first iteration only)
    // generator width: four waves (one per SIMD) beside the lean fused kernel of the frames in flight
    c->gen_nt = c->mt_gen_nt_opt ? c->mt_gen_nt_opt
                                 : ((async && F.fuse && pick_variant(c->mats, c->seq_on ? c->seq : 0).lean != nullptr) ? 256
                                                                                                          : rtmt_dev::MT_GEN_THREADS);
    bool pf_hit = false;
    const int mts = use_mt ? (n_rows >= Hf ? 2 : 0) : 0;
    const int64_t pf_shape[8] = {W, Hf, a->spp, batch, mt_pm, (int64_t)(c->f - c->slots), mts,
                                 (int64_t)c->mt_bands_on * 2 + (c->mt_short > 0)};
    if (prefetch && (F.npass != 1 || !mts)) return SRT_OK;  // (the generation would run on the frame's stream)
    if (!prefetch && use_mt && pf_in.valid && !async && !sharded && !a->rows && n_rows == Hf && F.npass == 1 && mts &&
        !memcmp(pf_in.shape, pf_shape, sizeof pf_shape) && pf_in.bt[0] == mt_bt[0] && pf_in.bt[1] == mt_bt[1] &&
        pf_in.pos == a->mt->pos && !memcmp(pf_in.key, a->mt->key, sizeof pf_in.key))
        pf_hit = true;
    for (;;) {
        if (!prefetch) {
            if (c->f->pending == 0) clear_host_flags(c, F);  // k_pass_end ORs into them
            if (c->f->dirty) {
                HIP_TRY(hipMemsetAsync(c->f->shadow, 0, 8 * NSHARD, c->f->stream));
                HIP_TRY(hipMemsetAsync(c->f->counts, 0, (size_t)F.cnt_words * 4, c->f->stream));
                HIP_TRY(hipMemsetAsync(c->f->flags, 0, 8, c->f->stream));
            }
            c->f->dirty = true;
        }
        int mt_pos = 0;
        const uint32_t* mt_key = nullptr;
        // the stream the numpy-stream generation runs on: the MT stream for a single-pass frame
        // (it waits until the slot's previous frame has read its jitter), else the frame's stream
        hipStream_t mst = c->f->stream;
        if (use_mt) {
            // (auto: whole frames on the high-priority stream, shards on the frame's stream: a stream
            // shared by the frames serialises their generations, and a shard's band segments -- one
            // serial generator block each -- are long: a rank of 2's 130k-double bands take ~0.4 ms)
            if (F.npass == 1 && mts) {
                if (!c->mt_stream) {
                    // a high-priority queue (mt_stream 2): the generation's blocks are dispatched ahead
                    // of the trace kernels' as CUs free up
                    int lo = 0, hi = 0;
                    if (mts == 2 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
                        HIP_TRY(hipStreamCreateWithPriority(&c->mt_stream, hipStreamNonBlocking, hi));
                    else
                        HIP_TRY(hipStreamCreateWithFlags(&c->mt_stream, hipStreamNonBlocking));
                }
                mst = c->mt_stream;
                if (c->f->jit_busy && !pf_hit) HIP_TRY(hipStreamWaitEvent(mst, c->f->jit_free, 0));
            }
            // this frame's stream starts where the previous frame's ended (device dump window) or at
            // the caller's state
            if (c->mt_done && !pf_hit) HIP_TRY(hipStreamWaitEvent(mst, c->mt_done, 0));
            if (mt_chained) {
                mt_key = mt_dump(c);
                mt_pos = c->mt_pos;
            } else {
                if (!pf_hit) HIP_TRY(hipMemcpyAsync(mt_key0(c), a->mt->key, rtmt::N * 4, hipMemcpyHostToDevice, mst));
                mt_key = mt_key0(c);
                mt_pos = a->mt->pos;
            }
        }
        for (int p = 0; p < F.npass; ++p) {
            const int s0 = p * batch;
            const int ns = std::min(batch, a->spp - s0);
            const int64_t nrays = (int64_t)ns * npix;
            TraceParams P = base_params(c, a->seed);
            P.fb = c->f->fb;
            P.fbx = (c->deterministic && c->fx_ok) ? c->f->fbx : nullptr;
            P.fb_first = (p == 0);  // the first pass's depth-0 kernel stores the framebuffer (no memset)
            // sample groups per pixel (k_primary): one (all of the pass's samples in one thread, summed
            // in registers) unless the frame has too few pixels to fill the GPU -- one GPU's shard of a
            // multi-GPU frame -- then 2, 4, .. groups on lanes of the pixel's wave (their fixed-point
            // sums are exact in any grouping: the image does not depend on it).  Enough means one
            // round of the resident threads for the per-depth kernels (a 1/8 shard of ex1 1080p, 261k
            // pixels: 6 samples per thread 118 us, 1 sample 133 us) and two for the fused paths, whose
            // threads trace whole paths (long tails: a 1/8 shard on one group per pixel 0.35 ms, 1.3
            // rounds, against 0.29 ms on the per-depth kernels)
            P.pix_groups = pix_groups(c, npix, ns, F.fuse);
            P.npix = npix;
            P.cam = *cam;
            P.cam.xs = c->xs;
            P.cam.ys = c->ys;
            P.rows = c->rows;
            P.sample_base = a->sample_base + s0;
            P.spp = ns;
            P.jit_plane = npix;
            if (use_mt) {
                // the pass's samples of the whole frame's stream (then the sizing draw after the last
                // pass); a shard reads its rows by global pixel
                const int64_t n_out = (int64_t)ns * 4 * W * Hf;
                const int64_t n_skip = (p + 1 == F.npass) ? 4 * W * Hf : 0;
                if (p > 0) mt_key = mt_dump(c);  // the previous pass's final window
                // a pipelined one-pass frame: its final window (the next frame's key) by one jump, so
                // the next frame's generation starts once this one's jump kernel has run
                const int64_t n_words = 2 * (n_out + n_skip);
                const srt_ctx::MtBandTab* bt = mt_bt[p + 1 == F.npass ? 1 : 0];
                const bool band = bt && rtmt::end_jump(n_words) > 0;
                const bool end = band || (async && F.npass == 1 && n_words <= (int64_t)rtmt::SEGS * rtmt::L &&
                                          rtmt::end_jump(n_words) > 0);
                const uint32_t* end_poly = nullptr;
                if (end && (rc = mt_end_poly_for(c, n_words, &end_poly))) return rc;
                // (a pinhole camera reads only the pixel-jitter planes 0 and 1 of each sample)
                const hipStream_t gst = mst;
                hipStream_t gen_on = mst;
                if (pf_hit && p == 0) {  // queued by srt_render_prefetch
                    mt_pos = pf_in.final_pos;
                    gen_on = pf_in.gen_on;
                    c->pf_used++;
                } else {
                    if (band) {
                        if ((rc = mt_launch_bands(c, mst, c->f->mt_win, mt_key, mt_pos, n_words, *bt, c->f->jit, &mt_pos,
                                                  end_poly, p + 1 == F.npass ? c->mt_done : nullptr, gst,
                                                  c->f->mt_jumped, &gen_on)))
                            return rc;
                    } else if ((rc = mt_launch(c, mst, c->f->mt_win, mt_key, mt_pos, n_out, n_skip, c->f->jit, &mt_pos,
                                               W * Hf, mt_pm, end_poly, end ? (int64_t)rtmt::end_jump(n_words) : 0,
                                               end ? c->mt_done : nullptr, gst, c->f->mt_jumped, &gen_on))) {
                        return rc;
                    }
                    // otherwise the next frame's stream may start as soon as this one's is generated
                    if (p + 1 == F.npass && !end) HIP_TRY(hipEventRecord(c->mt_done, mst));
                }
                if (prefetch) {
                    // queued: the frame's stream waits for it when srt_render comes (a wait queued
                    // here would also hold up the scene upload's synchronisation of that stream)
                    srt_ctx::MtPrefetch& q = c->pf;
                    memcpy(q.key, a->mt->key, sizeof q.key);
                    q.pos = a->mt->pos;
                    memcpy(q.shape, pf_shape, sizeof pf_shape);
                    q.bt[0] = mt_bt[0];
                    q.bt[1] = mt_bt[1];
                    q.final_pos = mt_pos;
                    q.gen_on = gen_on;
                    q.valid = true;
                    c->pf_queued++;
                    return SRT_OK;
                }
                if (gen_on != c->f->stream) {
                    HIP_TRY(hipEventRecord(c->f->jit_ready, gen_on));
                    HIP_TRY(hipStreamWaitEvent(c->f->stream, c->f->jit_ready, 0));
                }
                P.jitter = c->f->jit;
                P.jit_plane = band ? npix : W * Hf;
                P.jit_global = band ? 0 : 1;
            } else if (a->jitter) {
                const double* src = a->jitter + (int64_t)s0 * 4 * npix;
                if (jit_dev) {
                    P.jitter = src;
                } else {
                    HIP_TRY(hipMemcpyAsync(c->f->jit, src, (size_t)nrays * 4 * 8, hipMemcpyHostToDevice, c->f->stream));
                    P.jitter = c->f->jit;
                }
            }
            if (a->out_hit_id) P.hit_out = hit_dev ? a->out_hit_id + (int64_t)s0 * npix : c->f->hit;
            hipEvent_t* ev = c->f->ev.data() + (int64_t)p * F.nev;
            if (F.frame) {
                // the whole pass in one launch: one wave per 64-pixel tile
                P.ring = c->f->ring;
                P.ring_lock = c->f->ring_lock;
                P.ring_cap = c->f->ring_cap;
                P.nslot = c->f->nslot;
                P.dcap = F.dcap;
                P.cnt_out = c->f->counts;
                P.groups = std::min(F.groups, ns);
                P.ntiles = (int)ntiles;
                P.fbg = c->f->fbg;
                P.fuse_resolve = (F.npass == 1 && F.groups == 1);
                P.out_rgb = res_rgb;
                P.out_u8 = res_u8;
                P.spp_total = a->spp;
                HIP_TRY(hipEventRecord(ev[0], c->f->stream));
                hipLaunchKernelGGL(V.frame, dim3((unsigned)(ntiles * P.groups)), dim3(FRAME_BLOCK), lut_bytes(c),
                                   c->f->stream, P);
                HIP_TRY(hipGetLastError());
                if (P.groups > 1) {
                    hipLaunchKernelGGL(k_fb_groups, dim3(grid_for(3 * npix, c->max_blocks)), dim3(BLOCK), 0, c->f->stream,
                                       c->f->fb, (const double*)c->f->fbg, P.groups, npix, (int)P.fb_first);
                    HIP_TRY(hipGetLastError());
                }
                HIP_TRY(hipEventRecord(ev[1], c->f->stream));
                HIP_TRY(hipEventRecord(ev[F.dcap + 1], c->f->stream));
                if (mst != c->f->stream) {  // the next generation into this slot may start
                    HIP_TRY(hipEventRecord(c->f->jit_free, c->f->stream));
                    c->f->jit_busy = true;
                }
            } else {
            // depth 0: raygen fused with the trace step
            P.depth = 0;
            P.n_primary = nrays;
            P.qout = c->f->q[1];
            P.cnt_out = c->f->counts + NSHARD;
            P.dcap = F.dcap;
            HIP_TRY(hipEventRecord(ev[0], c->f->stream));
            // a single-pass fused frame resolves its pixels in k_primary (no framebuffer)
            P.fuse_resolve = F.fuse && F.npass == 1;
            P.out_rgb = res_rgb;
            P.out_u8 = res_u8;
            P.spp_total = a->spp;
            // grid: frames in flight overlap one frame's tail with the next, and fewer, longer blocks
            // (grid-stride, max_blocks: four rounds of the resident blocks) leave the numpy-stream
            // generators of the frames behind more room; a synchronous frame has nothing to overlap,
            // so it takes one block per 256 threads and the hardware fills the tail as blocks finish
            // (same box, ex1 1080p: the synchronous launch 0.950 -> 0.908 ms; pipelined frames with the
            // full grid 0.902 -> 0.986 ms, profiles/r05_primary_grid_ab.txt)
            // the lean kernel of pipelined whole frames (its generators beside it): two blocks per CU,
            // each grid-striding over ~30 wave iterations of a 1080p frame; the frames in flight fill
            // the rest of the CU (ex1 1080p: 0.878 ms per frame at 3072 blocks, 0.838 at 512; a rank of
            // 8's shard, 2025 blocks at most, was slower with it: profiles/r05_lean_grid_ab.txt).  A
            // pipeline's first frame, with nothing in flight to fill the CUs around its blocks, keeps
            // the full four rounds (max_blocks).
            // (option sync_lean: synchronous frames take the lean kernel too -- bench.py times the pipelined
            // frames' kernel alone that way for its roofline)
            const bool lean = F.fuse && (async || c->sync_lean) && V.lean;
            if (lean) c->lean_launches++;
            const int pgrid = !async ? INT_MAX
                                     : (!lean || c->async_pending == 0               ? c->max_blocks
                                        : n_rows == Hf && c->lean_blocks > 0              ? c->lean_blocks
                                        : n_rows < Hf && c->lean_blocks_shard > 0         ? c->lean_blocks_shard
                                                                                            : c->max_blocks);
            hipLaunchKernelGGL(F.fuse ? (lean ? (c->lane_stats && V.lean_stats ? V.lean_stats : V.lean) : V.fused) : V.primary,
                               dim3(grid_for(((npix * P.pix_groups + 63) / 64) * 64, pgrid)), dim3(BLOCK),
                               lut_bytes(c), c->f->stream, P);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(ev[1], c->f->stream));
            if (F.fuse)  // every depth traced: the deeper depths' events mark the same point
                for (int d = 1; d <= F.dcap; ++d) HIP_TRY(hipEventRecord(ev[1 + d], c->f->stream));
            if (mst != c->f->stream) {  // the next generation into this slot may start
                HIP_TRY(hipEventRecord(c->f->jit_free, c->f->stream));
                c->f->jit_busy = true;
            }
            P.fb_first = 0;
            for (int d = 1; d <= F.dcap && !F.fuse; ++d) {
                if (F.chain_from > 0 && d > F.chain_from) break;  // traced by the chain kernel
                P.depth = d;
                P.qin = c->f->q[d & 1];
                P.qout = c->f->q[(d + 1) & 1];
                P.cnt_in = c->f->counts + (int64_t)d * NSHARD;
                P.cnt_out = c->f->counts + (int64_t)(d + 1) * NSHARD;
                P.chain = (d == F.chain_from);
                P.dcap = F.dcap;
                hipLaunchKernelGGL(P.chain ? V.chain : V.trace, dim3(trace_grid(c)), dim3(BLOCK),
                                   lut_bytes(c), c->f->stream, P);
                HIP_TRY(hipGetLastError());
                HIP_TRY(hipEventRecord(ev[1 + d], c->f->stream));
            }
            }
            uint32_t* hp = c->f->host + p * F.pass_words;
            // counters of this pass -> pinned host words [0, used_words) (the unused depths are zero
            // on the host), flags OR-ed into the two words at [cnt_words, cnt_words + 2); the last
            // pass's are handed over by k_resolve
            if (p + 1 < F.npass) {
                hipLaunchKernelGGL(k_pass_end, dim3(1), dim3(BLOCK), 0, c->f->stream, c->f->counts, used_words, c->f->flags,
                                   hp, hp + F.cnt_words);
                HIP_TRY(hipGetLastError());
            }
            if (a->out_hit_id && !hit_dev)
                HIP_TRY(hipMemcpyAsync(a->out_hit_id + (int64_t)s0 * npix, c->f->hit, (size_t)nrays * 4,
                                       hipMemcpyDeviceToHost, c->f->stream));
        }
        if (use_mt) c->mt_pos = mt_pos;
        uint32_t* hshadow = c->f->host + F.npass * F.pass_words;
        // (a single-pass frame kernel or fused frame has resolved its pixels: k_resolve only hands over
        // the counters and the shadow count)
        const bool fused = F.npass == 1 && ((F.frame && F.groups == 1) || F.fuse);
        uint32_t* hlast = c->f->host + (F.npass - 1) * F.pass_words;
        hipLaunchKernelGGL(k_resolve, dim3(fused ? 1 : grid_for(npix, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, c->f->fb,
                           (F.frame || !c->deterministic || !c->fx_ok) ? nullptr
                                                                       : (const unsigned long long*)c->f->fbx,
                           fused ? (int64_t)0 : npix, c->f->shadow, hshadow, (double)a->spp, res_rgb, res_u8, c->f->counts,
                           used_words, c->f->flags, hlast, hlast + F.cnt_words);
        HIP_TRY(hipGetLastError());
        c->f->dirty = false;  // the kernels above leave counts/flags/shadow zeroed
        // this rank's rows of the linear RGB into the shared host frame: per plane, the rank's band j
        // at frame band j n + rank, one pitched copy of the full bands, then a short last band
        if (rgb_rows) {
            const int64_t band_px = band * W;
            const int64_t nb = npix / band_px, tail = npix - nb * band_px;
            for (int pl = 0; pl < 3; ++pl) {
                double* dst = a->out_rgb + (int64_t)pl * W * Hf;
                const double* src = c->f->rgb + (int64_t)pl * npix;
                if (nb > 0)
                    HIP_TRY(hipMemcpy2DAsync(dst + (int64_t)c->rank * band_px, (size_t)(c->nranks * band_px * 8), src,
                                             (size_t)(band_px * 8), (size_t)(band_px * 8), (size_t)nb,
                                             hipMemcpyDeviceToHost, c->f->stream));
                if (tail > 0) {
                    // (the rank's band nb, in period nb)
                    const int64_t bt = nb * c->nranks + c->rank;
                    HIP_TRY(hipMemcpyAsync(dst + bt * band_px, src + nb * band_px, (size_t)(tail * 8),
                                           hipMemcpyDeviceToHost, c->f->stream));
                }
            }
        }
        // the shard's tiles to rank 0 (RCCL over xGMI), assembled into the frame there
        FrameSlot::Gather& G = c->f->gather;
        G = FrameSlot::Gather{};
        if (sharded) {
            G.on = true;
            G.W = W;
            G.H = Hf;
            G.npix = npix;
            G.maxpix = maxpix;
            G.band = band;
            G.want_u8 = true;
            G.want_rgb = gather_rgb;
            if (c->rank == 0) {
                G.dst_u8 = (a->out_srgb8 && u8_dev) ? a->out_srgb8 : c->f->full_u8;
                G.dst_rgb = (a->out_rgb && rgb_dev) ? a->out_rgb : c->f->full_rgb;
                G.host_u8 = (a->out_srgb8 && !u8_dev) ? a->out_srgb8 : nullptr;
                G.host_rgb = (a->out_rgb && !rgb_dev && gather_rgb) ? a->out_rgb : nullptr;
            }
        }
        const uint8_t* u8_src = c->f->u8;
        int64_t u8_bytes = 3 * npix;
        if (reh_n) {
            GatherTiles T{};
            for (int q = 0; q < reh_n; ++q) {
                T.u8[q] = q == 0 ? c->f->u8 : c->f->g_u8 + (int64_t)q * reh_maxpix * 3;
                T.npix[q] = shard_rank_rows(Hf, reh_n, q, reh_band) * W;
            }
            hipLaunchKernelGGL(k_assemble, dim3(grid_for(W * Hf, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, T, reh_n,
                               reh_band, W, Hf, c->f->full_u8, (double*)nullptr);
            HIP_TRY(hipGetLastError());
            u8_src = c->f->full_u8;
            u8_bytes = 3 * W * Hf;
        }
        if (rgbx) {
            uint32_t* dst4 = reinterpret_cast<uint32_t*>(u8_direct ? a->out_srgb8 : c->f->full_u8);
            hipLaunchKernelGGL(k_rgbx, dim3(grid_for(npix, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, c->f->u8, dst4,
                               npix);
            HIP_TRY(hipGetLastError());
            u8_src = c->f->full_u8;
            u8_bytes = 4 * npix;
        }
        if (async) {
            // (a synchronous frame gathers after its retries: every rank gathers each frame once)
            if (sharded && !c->defer_gather && (rc = gather_frame(c))) return rc;
            if (!sharded && ((a->out_srgb8 && !u8_direct) || (a->out_rgb && !rgb_direct))) {
                hipStream_t cs = c->f->stream;
                if (a->out_srgb8 && !u8_direct)
                    HIP_TRY(hipMemcpyAsync(a->out_srgb8, u8_src, (size_t)u8_bytes, hipMemcpyDeviceToHost, cs));
                if (a->out_rgb && !rgb_direct)
                    HIP_TRY(hipMemcpyAsync(a->out_rgb, c->f->rgb, (size_t)3 * npix * 8, hipMemcpyDeviceToHost, cs));
            }
            // host outputs (pinned) are copied on the frame's stream; stats and errors come with
            // srt_render_finish; the next asynchronous frame goes to the next slot
            if (use_mt) c->mt_chain = a->mt;
            c->async_pending++;
            c->f->pending++;
            c->f->plan = F;
            c->last_slot = (int)(c->f - c->slots);
            c->next_slot = (c->last_slot + 1) % c->nslots;
            return SRT_OK;
        }
        if (!sharded && a->out_rgb && !rgb_direct)
            HIP_TRY(hipMemcpyAsync(a->out_rgb, c->f->rgb, (size_t)3 * npix * 8, hipMemcpyDeviceToHost, c->f->stream));
        if (!sharded && a->out_srgb8 && !u8_direct)
            HIP_TRY(hipMemcpyAsync(a->out_srgb8, u8_src, (size_t)u8_bytes, hipMemcpyDeviceToHost, c->f->stream));
        c->f->dirty = true;
        HIP_TRY(hipStreamSynchronize(c->f->stream));
        c->f->dirty = false;
        const int64_t retries = S.retries;
        uint32_t bits = 0;
        rc = collect_frame(c, F, S, &bits);
        if (rc == SRT_RETRY) {
            // render the frame again: without chain mode after a tie gave a chained ray a second
            // child (the same tie would recur), with bigger queues after an overflow
            S.retries = retries + 1;
            if (S.retries > 8) return fail(SRT_ERR_MEMORY, "ray queues keep overflowing");
            if (bits & RETRY_CHAIN_TIE) {
                F.chain_from = 0;
                F.fuse = false;
            }
            if ((bits & RETRY_OVERFLOW) &&
                (rc = F.frame ? ensure_ring(c, 2 * c->f->ring_cap) : ensure_queues(c, 2 * c->f->seg * NSHARD)))
                return rc;
            pf_hit = false;  // (the retry generates its stream again from the caller's state)
            continue;
        }
        S.retries = retries;
        if (rc) return rc;
        break;
    }
    if (sharded && !c->defer_gather) {
        if ((rc = gather_frame(c))) return rc;
        HIP_TRY(hipStreamSynchronize(c->f->stream));
    }
    if (use_mt) {  // numpy's state after this frame's draws
        HIP_TRY(hipMemcpy(a->mt->key, mt_dump(c), rtmt::N * 4, hipMemcpyDeviceToHost));
        a->mt->pos = c->mt_pos;
    }
    if (st) {
        S.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        *st = S;
    }
    return SRT_OK;
}
}  // namespace

extern "C" {
int srt_render(srt_ctx* c, const srt_camera* cam, const srt_render_args* a, srt_stats* st) {
    return render_impl(c, cam, a, st, false);
}

int srt_render_prefetch(srt_ctx* c, const srt_camera* cam, const srt_render_args* a) {
    return render_impl(c, cam, a, nullptr, true);
}

int srt_render_finish(srt_ctx* c, srt_stats* st) {
    if (!c) return fail(SRT_ERR_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    return finish_async(c, st);
}

int srt_stream(srt_ctx* c, void** stream) {
    if (!c || !stream) return fail(SRT_ERR_ARG, "null argument");
    *stream = (void*)c->f->stream;
    return SRT_OK;
}

}  // extern "C"

namespace {
// get_raycolor (srt_trace) or Material.get_color at given hits (srt_shade: fid/ft/fo non-null)
// kids (srt_shade_level): shade the first depth only and hand its children back instead of tracing them
int trace_impl(srt_ctx* c, const srt_trace_args* a, const int32_t* fid, const double* ft, const double* fo,
               srt_stats* st, srt_children* kids = nullptr) {
    auto t_start = std::chrono::steady_clock::now();
    if (!c || !a || !a->origin || !a->dir || !a->out_rgb) return fail(SRT_ERR_ARG, "null argument");
    c->pf.valid = false;  // (slot 0's buffers are reused here)
    if (!c->has_scene) return fail(SRT_ERR_NOSCENE, "no scene uploaded");
    if (a->depth < 0 || a->depth > 200 || a->diffuse_reflections < 0) return fail(SRT_ERR_ARG, "bad depth");
    if (a->n <= 0) return SRT_OK;
    if (a->n >= ((int64_t)1 << 31)) return fail(SRT_ERR_ARG, "batch too large");
    HIP_TRY(hipSetDevice(c->device));
    int rc0 = finish_async(c, nullptr);
    if (rc0) return rc0;
    c->f->dirty = true;  // counts/flags/shadow are left as this call's memsets and kernels leave them
    const int64_t n = a->n;
    int rc = SRT_OK;
    CallBufs bufs;  // (freed on every return)
    double *O = nullptr, *D = nullptr;
    int32_t* med = nullptr;
    HIP_TRY(bufs.alloc(&O, 3 * n));
    HIP_TRY(bufs.alloc(&D, 3 * n));
    if (a->medium) HIP_TRY(bufs.alloc(&med, n));
    HIP_TRY(hipMemcpyAsync(O, a->origin, (size_t)3 * n * 8, hipMemcpyDefault, c->f->stream));
    HIP_TRY(hipMemcpyAsync(D, a->dir, (size_t)3 * n * 8, hipMemcpyDefault, c->f->stream));
    if (med) HIP_TRY(hipMemcpyAsync(med, a->medium, (size_t)n * 4, hipMemcpyDefault, c->f->stream));
    int32_t* dfid = nullptr;
    double *dft = nullptr, *dfo = nullptr;
    if (fid) {
        HIP_TRY(bufs.alloc(&dfid, n));
        HIP_TRY(bufs.alloc(&dft, n));
        HIP_TRY(bufs.alloc(&dfo, n));
        HIP_TRY(hipMemcpyAsync(dfid, fid, (size_t)n * 4, hipMemcpyDefault, c->f->stream));
        HIP_TRY(hipMemcpyAsync(dft, ft, (size_t)n * 8, hipMemcpyDefault, c->f->stream));
        HIP_TRY(hipMemcpyAsync(dfo, fo, (size_t)n * 8, hipMemcpyDefault, c->f->stream));
    }
    if ((rc = ensure_buf(&c->f->fb, c->f->fb_cap, 3 * n))) return rc;
    if ((rc = ensure_buf(&c->f->fbx, c->f->fbx_cap, fx_words(n)))) return rc;
    if ((rc = ensure_queues(c, n * c->fanout))) return rc;
    // depths a->depth .. a->depth + cap (the batch's depth is a scalar in the reference)
    const int d0 = a->depth;
    const int dlast = kids ? d0 : std::min(SRT_MAX_DEPTHS - 2, d0 + depth_cap(c));
    srt_stats S{};
    std::vector<uint32_t> counts(SRT_MAX_DEPTHS * NSHARD);
    bool fx = c->deterministic;  // fixed-point colour sums (fb_add)
    for (int attempt = 0;; ++attempt) {
        if (attempt > 8) { rc = fail(SRT_ERR_MEMORY, "ray queues keep overflowing"); break; }
        HIP_TRY(hipMemsetAsync(c->f->fb, 0, (size_t)3 * n * 8, c->f->stream));
        HIP_TRY(hipMemsetAsync(c->f->fbx, 0, (size_t)fx_words(n) * 8, c->f->stream));
        HIP_TRY(hipMemsetAsync(c->f->counts, 0, (size_t)SRT_MAX_DEPTHS * NSHARD * 4, c->f->stream));
        HIP_TRY(hipMemsetAsync(c->f->flags, 0, 8, c->f->stream));
        HIP_TRY(hipMemsetAsync(c->f->shadow, 0, 8 * NSHARD, c->f->stream));
        uint32_t seed_counts[NSHARD];
        for (int s = 0; s < NSHARD; ++s) seed_counts[s] = (uint32_t)((n - s + NSHARD - 1) / NSHARD);
        HIP_TRY(hipMemcpyAsync(c->f->counts + (int64_t)d0 * NSHARD, seed_counts, sizeof(seed_counts),
                               hipMemcpyHostToDevice, c->f->stream));
        hipLaunchKernelGGL(k_seed_queue, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, c->f->q[d0 & 1],
                           c->f->seg, O, D, med, n, (uint32_t)d0, (uint32_t)a->diffuse_reflections, (uint32_t)c->S.nmedia);
        HIP_TRY(hipGetLastError());
        TraceParams P = base_params(c, a->seed);
        P.fb = c->f->fb;
        P.fbx = fx ? c->f->fbx : nullptr;
        P.npix = n;
        const Variant& V = pick_variant(c->mats, c->seq_on ? c->seq : 0);
        for (int d = d0; d <= dlast; ++d) {
            P.depth = d;
            P.qin = c->f->q[d & 1];
            P.qout = c->f->q[(d + 1) & 1];
            P.cnt_in = c->f->counts + (int64_t)d * NSHARD;
            P.cnt_out = c->f->counts + (int64_t)(d + 1) * NSHARD;
            if (fid && d == d0) {
                P.force_id = dfid;
                P.force_t = dft;
                P.force_o = dfo;
                hipLaunchKernelGGL((c->mats & MAT_BVH) ? k_shade_forced<MAT_GENERIC | MAT_BVH> : k_shade_forced<MAT_GENERIC>,
                                   dim3(trace_grid(c)), dim3(BLOCK), lut_bytes(c), c->f->stream, P);
                P.force_id = nullptr;
                P.force_t = P.force_o = nullptr;
            } else {
                hipLaunchKernelGGL(V.trace, dim3(trace_grid(c)), dim3(BLOCK), lut_bytes(c), c->f->stream, P);
            }
            HIP_TRY(hipGetLastError());
        }
        uint32_t flags[2];
        unsigned long long shadow = 0;
        HIP_TRY(hipMemcpyAsync(counts.data(), c->f->counts, counts.size() * 4, hipMemcpyDeviceToHost, c->f->stream));
        HIP_TRY(hipMemcpyAsync(flags, c->f->flags, sizeof(flags), hipMemcpyDeviceToHost, c->f->stream));
        HIP_TRY(hipMemcpyAsync(&shadow, c->f->shadow, 8, hipMemcpyDeviceToHost, c->f->stream));
        HIP_TRY(hipStreamSynchronize(c->f->stream));
        if ((rc = check_flags(flags[0]))) break;
        if (flags[1]) {
            S.retries++;
            if (flags[1] & RETRY_FIXED_RANGE) fx = false;  // again with f64 atomics
            if ((flags[1] & RETRY_OVERFLOW) && (rc = ensure_queues(c, 2 * c->f->seg * NSHARD))) break;
            continue;
        }
        if (!kids && depth_total(counts.data() + (int64_t)(dlast + 1) * NSHARD, c->f->seg) != 0) {
            rc = fail(SRT_ERR_DEPTH, "rays alive after the depth cap");
            break;
        }
        for (int d = d0; d <= dlast; ++d) S.rays_per_depth[d] = depth_total(counts.data() + (int64_t)d * NSHARD, c->f->seg);
        S.n_depths = dlast + 1;
        for (int d = 0; d < SRT_MAX_DEPTHS; ++d) S.total_rays += S.rays_per_depth[d];
        S.shadow_rays = (int64_t)shadow;
        if (fx) {
            hipLaunchKernelGGL(k_fx_combine, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, c->f->fb,
                               (const unsigned long long*)c->f->fbx, n, c->f->flags);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(flags, c->f->flags, sizeof(flags), hipMemcpyDeviceToHost, c->f->stream));
            HIP_TRY(hipStreamSynchronize(c->f->stream));
            if (flags[1] & RETRY_FIXED_RANGE) {
                S.retries++;
                fx = false;  // again with f64 atomics
                continue;
            }
        }
        HIP_TRY(hipMemcpyAsync(a->out_rgb, c->f->fb, (size_t)3 * n * 8, hipMemcpyDefault, c->f->stream));
        HIP_TRY(hipStreamSynchronize(c->f->stream));
        if (kids) {
            // the first depth's children, packed shard by shard (the order the queue appends gave them)
            const uint32_t* kc = counts.data() + (int64_t)(d0 + 1) * NSHARD;
            std::vector<int64_t> prefix(NSHARD);
            int64_t total = 0;
            for (int s = 0; s < NSHARD; ++s) {
                prefix[s] = total;
                total += std::min<int64_t>(kc[s], c->f->seg);
            }
            kids->n = total;
            if (total > kids->cap) {
                rc = fail(SRT_ERR_MEMORY, "children exceed srt_children.cap (n holds the count)");
                break;
            }
            if (total > 0) {
                double *kO, *kD, *kW;
                int32_t *kp, *km, *kd, *kf;
                int64_t* kpre;
                HIP_TRY(bufs.alloc(&kO, 3 * total));
                HIP_TRY(bufs.alloc(&kD, 3 * total));
                HIP_TRY(bufs.alloc(&kW, 3 * total));
                HIP_TRY(bufs.alloc(&kp, total));
                HIP_TRY(bufs.alloc(&km, total));
                HIP_TRY(bufs.alloc(&kd, total));
                HIP_TRY(bufs.alloc(&kf, total));
                HIP_TRY(bufs.alloc(&kpre, NSHARD));
                HIP_TRY(hipMemcpyAsync(kpre, prefix.data(), NSHARD * 8, hipMemcpyHostToDevice, c->f->stream));
                hipLaunchKernelGGL(k_gather_children, dim3(NSHARD), dim3(BLOCK), 0, c->f->stream, c->f->q[(d0 + 1) & 1],
                                   c->f->seg, c->f->counts + (int64_t)(d0 + 1) * NSHARD, kpre, total, kO, kD, kW, kp, km,
                                   kd, kf);
                HIP_TRY(hipGetLastError());
                for (int k = 0; k < 3; ++k) {
                    HIP_TRY(hipMemcpyAsync(kids->origin + k * kids->cap, kO + k * total, (size_t)total * 8,
                                           hipMemcpyDefault, c->f->stream));
                    HIP_TRY(hipMemcpyAsync(kids->dir + k * kids->cap, kD + k * total, (size_t)total * 8,
                                           hipMemcpyDefault, c->f->stream));
                    HIP_TRY(hipMemcpyAsync(kids->weight + k * kids->cap, kW + k * total, (size_t)total * 8,
                                           hipMemcpyDefault, c->f->stream));
                }
                HIP_TRY(hipMemcpyAsync(kids->parent, kp, (size_t)total * 4, hipMemcpyDefault, c->f->stream));
                HIP_TRY(hipMemcpyAsync(kids->medium, km, (size_t)total * 4, hipMemcpyDefault, c->f->stream));
                HIP_TRY(hipMemcpyAsync(kids->depth, kd, (size_t)total * 4, hipMemcpyDefault, c->f->stream));
                HIP_TRY(hipMemcpyAsync(kids->diffuse_reflections, kf, (size_t)total * 4, hipMemcpyDefault,
                                       c->f->stream));
                HIP_TRY(hipStreamSynchronize(c->f->stream));
            }
        }
        break;
    }
    if (rc) return rc;
    S.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (st) *st = S;
    return SRT_OK;
}
}  // namespace

extern "C" {

int srt_trace(srt_ctx* c, const srt_trace_args* a, srt_stats* st) {
    return trace_impl(c, a, nullptr, nullptr, nullptr, st);
}

int srt_shade(srt_ctx* c, const srt_trace_args* a, const int32_t* collider, const double* t, const double* orient,
              srt_stats* st) {
    if (!collider || !t || !orient) return fail(SRT_ERR_ARG, "null hit arrays");
    return trace_impl(c, a, collider, t, orient, st);
}

int srt_shade_level(srt_ctx* c, const srt_trace_args* a, const int32_t* collider, const double* t, const double* orient,
                    srt_children* kids, srt_stats* st) {
    if (!collider || !t || !orient || !kids) return fail(SRT_ERR_ARG, "null hit / children arrays");
    kids->n = 0;
    if (kids->cap < 0 || (kids->cap > 0 && (!kids->origin || !kids->dir || !kids->weight || !kids->parent ||
                                            !kids->medium || !kids->depth || !kids->diffuse_reflections)))
        return fail(SRT_ERR_ARG, "srt_children arrays");
    return trace_impl(c, a, collider, t, orient, st, kids);
}

int srt_nearest(srt_ctx* c, const double* O, const double* D, int64_t n, double* t, int32_t* id, double* orient) {
    if (!c || !O || !D) return fail(SRT_ERR_ARG, "null argument");
    if (!c->has_scene) return fail(SRT_ERR_NOSCENE, "no scene uploaded");
    if (n <= 0) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    double *dO, *dD, *dt, *dor;
    int32_t* did;
    HIP_TRY(bufs.alloc(&dO, 3 * n));
    HIP_TRY(bufs.alloc(&dD, 3 * n));
    HIP_TRY(bufs.alloc(&dt, n));
    HIP_TRY(bufs.alloc(&dor, n));
    HIP_TRY(bufs.alloc(&did, n));
    HIP_TRY(hipMemcpy(dO, O, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dD, D, (size_t)3 * n * 8, hipMemcpyDefault));
    hipLaunchKernelGGL(k_nearest, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, c->S, dO, dD, n, dt, did,
                       dor);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    if (t) HIP_TRY(hipMemcpy(t, dt, (size_t)n * 8, hipMemcpyDefault));
    if (id) HIP_TRY(hipMemcpy(id, did, (size_t)n * 4, hipMemcpyDefault));
    if (orient) HIP_TRY(hipMemcpy(orient, dor, (size_t)n * 8, hipMemcpyDefault));
    return SRT_OK;
}

int srt_intersect_collider(srt_ctx* c, const srt_collider* col, const double* O, const double* D, int64_t n,
                           double* out) {
    if (!c || !col || !O || !D || !out) return fail(SRT_ERR_ARG, "null argument");
    if (col->type < 0 || col->type > 3) return fail(SRT_ERR_ARG, "bad collider type");
    if (n <= 0) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    double *dO, *dD, *dout;
    srt_collider* dcol;
    HIP_TRY(bufs.alloc(&dO, 3 * n));
    HIP_TRY(bufs.alloc(&dD, 3 * n));
    HIP_TRY(bufs.alloc(&dout, 2 * n));
    HIP_TRY(bufs.alloc(&dcol, 1));
    HIP_TRY(hipMemcpy(dO, O, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dD, D, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dcol, col, sizeof(srt_collider), hipMemcpyDefault));
    hipLaunchKernelGGL(k_intersect_one, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, dcol, dO, dD, n,
                       dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    HIP_TRY(hipMemcpy(out, dout, (size_t)2 * n * 8, hipMemcpyDefault));
    return SRT_OK;
}

int srt_collider_surface(srt_ctx* c, const srt_collider* col, const double* P, int64_t n, double* N, double* uv,
                         int primitive_uv) {
    if (!c || !col || !P || (!N && !uv)) return fail(SRT_ERR_ARG, "null argument");
    if (col->type < 0 || col->type > 3) return fail(SRT_ERR_ARG, "bad collider type");
    if (uv && col->type == SRT_TRIANGLE)
        return fail(SRT_ERR_ARG, "Triangle uv is undefined in the reference (triangle.py:79-83)");
    if (n <= 0) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    srt_collider rec = *col;
    if (!primitive_uv) rec.flags &= ~SRT_CF_UV_CROSS;  // the collider's own 4x3 cross coordinates
    double *dP, *dN = nullptr, *duv = nullptr;
    srt_collider* dcol;
    HIP_TRY(bufs.alloc(&dP, 3 * n));
    if (N) HIP_TRY(bufs.alloc(&dN, 3 * n));
    if (uv) HIP_TRY(bufs.alloc(&duv, 2 * n));
    HIP_TRY(bufs.alloc(&dcol, 1));
    HIP_TRY(hipMemcpy(dP, P, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dcol, &rec, sizeof(srt_collider), hipMemcpyDefault));
    hipLaunchKernelGGL(k_collider_surface, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, dcol, dP, n,
                       dN, duv);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    if (N) HIP_TRY(hipMemcpy(N, dN, (size_t)3 * n * 8, hipMemcpyDefault));
    if (uv) HIP_TRY(hipMemcpy(uv, duv, (size_t)2 * n * 8, hipMemcpyDefault));
    return SRT_OK;
}

int srt_texture_lookup(srt_ctx* c, const srt_texture* tex, const uint8_t* texels, int64_t texel_bytes,
                       const double* uv, int64_t n, double* rgb) {
    if (!c || !tex || !texels || !uv || !rgb) return fail(SRT_ERR_ARG, "null argument");
    if (tex->offset < 0 || tex->offset + tex->height * tex->width * tex->channels > texel_bytes)
        return fail(SRT_ERR_ARG, "texture record outside the texel array");
    if (n <= 0) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    uint8_t* dtexels;
    srt_texture* dtex;
    double *duv, *drgb;
    uint32_t* dflags;
    HIP_TRY(bufs.alloc(&dtexels, texel_bytes));
    HIP_TRY(bufs.alloc(&dtex, 1));
    HIP_TRY(bufs.alloc(&duv, 2 * n));
    HIP_TRY(bufs.alloc(&drgb, 3 * n));
    HIP_TRY(bufs.alloc(&dflags, 1));
    HIP_TRY(hipMemcpy(dtexels, texels, (size_t)texel_bytes, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dtex, tex, sizeof(srt_texture), hipMemcpyDefault));
    HIP_TRY(hipMemcpy(duv, uv, (size_t)2 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemset(dflags, 0, 4));
    SceneView S{};
    S.tex = (const RT_RO srt_texture*)dtex;
    S.texels = (const RT_RO uint8_t*)dtexels;
    S.ntex = 1;
    hipLaunchKernelGGL(k_texture_lookup, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, S, duv, n, drgb,
                       dflags);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    uint32_t flags = 0;
    HIP_TRY(hipMemcpy(&flags, dflags, 4, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(rgb, drgb, (size_t)3 * n * 8, hipMemcpyDefault));
    return check_flags(flags);
}

int srt_material_normal(srt_ctx* c, const srt_collider* col, const srt_texture* normalmap, const uint8_t* texels,
                        int64_t texel_bytes, const double* P, const double* orient, int64_t n, double* N) {
    if (!c || !col || !P || !orient || !N) return fail(SRT_ERR_ARG, "null argument");
    if (col->type < 0 || col->type > 3) return fail(SRT_ERR_ARG, "bad collider type");
    if (normalmap) {
        if (!texels || normalmap->offset < 0 || normalmap->channels < 3 || normalmap->channel0 < 0 ||
            normalmap->channel0 + 3 > normalmap->channels ||
            normalmap->offset + (int64_t)normalmap->height * normalmap->width * normalmap->channels > texel_bytes)
            return fail(SRT_ERR_ARG, "normal-map record outside the texel array");
        if (col->type != SRT_PLANE && col->type != SRT_CUBOID)
            return fail(SRT_ERR_ARG, "a normal map needs the collider's inverse_basis_matrix (Plane, Cuboid)");
    }
    if (n <= 0) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    srt_material mrec{};
    mrec.type = SRT_GLOSSY;
    mrec.tex = mrec.tex_aux0 = mrec.tex_aux1 = -1;
    mrec.normalmap = normalmap ? 0 : -1;
    srt_collider* dcol;
    srt_material* dmat;
    srt_texture* dtex = nullptr;
    uint8_t* dtexels = nullptr;
    double *dP, *dor, *dN;
    uint32_t* dflags;
    HIP_TRY(bufs.alloc(&dcol, 1));
    HIP_TRY(bufs.alloc(&dmat, 1));
    HIP_TRY(bufs.alloc(&dP, 3 * n));
    HIP_TRY(bufs.alloc(&dor, n));
    HIP_TRY(bufs.alloc(&dN, 3 * n));
    HIP_TRY(bufs.alloc(&dflags, 1));
    HIP_TRY(hipMemcpy(dcol, col, sizeof(srt_collider), hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dmat, &mrec, sizeof(srt_material), hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dP, P, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(dor, orient, (size_t)n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemset(dflags, 0, 4));
    SceneView S{};
    if (normalmap) {
        HIP_TRY(bufs.alloc(&dtex, 1));
        HIP_TRY(bufs.alloc(&dtexels, texel_bytes));
        HIP_TRY(hipMemcpy(dtex, normalmap, sizeof(srt_texture), hipMemcpyDefault));
        HIP_TRY(hipMemcpy(dtexels, texels, (size_t)texel_bytes, hipMemcpyDefault));
        S.tex = (const RT_RO srt_texture*)dtex;
        S.texels = (const RT_RO uint8_t*)dtexels;
        S.ntex = 1;
    }
    hipLaunchKernelGGL(k_material_normal, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, S, dcol, dmat,
                       dP, dor, n, dN, dflags);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    uint32_t flags = 0;
    HIP_TRY(hipMemcpy(&flags, dflags, 4, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(N, dN, (size_t)3 * n * 8, hipMemcpyDefault));
    return check_flags(flags);
}

int srt_primary_rays(srt_ctx* c, const srt_camera* cam, const double* J, double* O, double* D) {
    if (!c || !cam || !J || !O || !D) return fail(SRT_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    CallBufs bufs;
    const int64_t n = (int64_t)cam->width * cam->height;
    double *dJ, *dO, *dD, *xs, *ys;
    HIP_TRY(bufs.alloc(&dJ, 4 * n));
    HIP_TRY(bufs.alloc(&dO, 3 * n));
    HIP_TRY(bufs.alloc(&dD, 3 * n));
    HIP_TRY(bufs.alloc(&xs, cam->width));
    HIP_TRY(bufs.alloc(&ys, cam->height));
    HIP_TRY(hipMemcpy(dJ, J, (size_t)4 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(xs, cam->xs, (size_t)cam->width * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(ys, cam->ys, (size_t)cam->height * 8, hipMemcpyDefault));
    srt_camera k = *cam;
    k.xs = xs;
    k.ys = ys;
    hipLaunchKernelGGL(k_primary_rays, dim3(grid_for(n, c->max_blocks)), dim3(BLOCK), 0, c->f->stream, k, dJ, n, dO, dD);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    HIP_TRY(hipMemcpy(O, dO, (size_t)3 * n * 8, hipMemcpyDefault));
    HIP_TRY(hipMemcpy(D, dD, (size_t)3 * n * 8, hipMemcpyDefault));
    return SRT_OK;
}

int srt_device_alloc(srt_ctx* c, int64_t bytes, void** out) {
    if (!c || !out || bytes <= 0) return fail(SRT_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMalloc(out, (size_t)bytes));
    return SRT_OK;
}

int srt_device_free(srt_ctx* c, void* p) {
    if (!c) return fail(SRT_ERR_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    if (p) HIP_TRY(hipFree(p));
    return SRT_OK;
}

int srt_memcpy(srt_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c || !dst || !src || bytes < 0) return fail(SRT_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
    return SRT_OK;
}

int srt_mt19937_uniforms(srt_ctx* c, const uint32_t* key, int32_t pos, int64_t n_out, int64_t n_skip, double* out,
                         uint32_t* key_out, int32_t* pos_out) {
    if (!c || !key || !key_out || !pos_out || (n_out > 0 && !out)) return fail(SRT_ERR_ARG, "null argument");
    c->pf.valid = false;  // (generates from the stream state a prefetch assumed)
    if (pos < 0 || pos > rtmt::N || n_out < 0 || n_skip < 0) return fail(SRT_ERR_ARG, "bad position or count");
    if (is_device_ptr(key) || is_device_ptr(key_out)) return fail(SRT_ERR_ARG, "key and key_out are host arrays");
    if (n_out + n_skip == 0) {
        memcpy(key_out, key, rtmt::N * 4);
        *pos_out = pos;
        return SRT_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    int rc = finish_async(c, nullptr);  // frames in flight may use the generator's scratch
    if (rc) return rc;
    if ((rc = mt_ensure(c))) return rc;
    double* dst = out;
    const bool host_out = n_out > 0 && !is_device_ptr(out);
    if (host_out) {
        if ((rc = ensure_buf(&c->mt_out, c->mt_out_cap, n_out))) return rc;
        dst = c->mt_out;
    }
    hipStream_t st = c->f->stream;
    HIP_TRY(hipMemcpyAsync(mt_key0(c), key, rtmt::N * 4, hipMemcpyHostToDevice, st));
    int final_pos = 0;
    if ((rc = mt_win_ensure(c, *c->f, (int64_t)rtmt::SEGS * rtmt::N))) return rc;
    if ((rc = mt_launch(c, st, c->f->mt_win, mt_key0(c), pos, n_out, n_skip, dst, &final_pos))) return rc;
    if (host_out) HIP_TRY(hipMemcpyAsync(out, dst, (size_t)n_out * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(key_out, mt_dump(c), rtmt::N * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *pos_out = final_pos;
    return SRT_OK;
}

// ---- multi-GPU ------------------------------------------------------------------------------
int srt_comm_unique_id(uint8_t* id) {
    if (!id) return fail(SRT_ERR_ARG, "null id");
    static_assert(sizeof(ncclUniqueId) == SRT_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return SRT_OK;
}

int srt_comm_init(srt_ctx* c, int nranks, int rank, const uint8_t* id) {
    if (!c || !id || nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks)
        return fail(SRT_ERR_ARG, "bad communicator arguments");
    if (c->comm) return fail(SRT_ERR_ARG, "context already has a communicator");
    HIP_TRY(hipSetDevice(c->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    NCCL_TRY(ncclCommInitRank(&c->comm, nranks, u, rank));
    c->nranks = nranks;
    c->rank = rank;
    return SRT_OK;
}

int srt_comm_init_all(int ndev, const int* devs, srt_ctx** ctxs) {
    if (ndev < 1 || ndev > MAX_RANKS || !devs || !ctxs) return fail(SRT_ERR_ARG, "bad device list");
    for (int q = 0; q < ndev; ++q) ctxs[q] = nullptr;
    for (int q = 0; q < ndev; ++q) {
        int rc = srt_create(devs[q], &ctxs[q]);
        if (rc) {
            for (int k = 0; k < q; ++k) srt_destroy(ctxs[k]);
            return rc;
        }
    }
    std::vector<ncclComm_t> comms(ndev);
    ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devs);
    if (r != ncclSuccess) {
        for (int k = 0; k < ndev; ++k) srt_destroy(ctxs[k]);
        return fail(SRT_ERR_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
    for (int q = 0; q < ndev; ++q) {
        ctxs[q]->comm = comms[q];
        ctxs[q]->nranks = ndev;
        ctxs[q]->rank = q;
    }
    return SRT_OK;
}

int srt_comm_rank(srt_ctx* c, int* nranks, int* rank) {
    if (!c || !nranks || !rank) return fail(SRT_ERR_ARG, "null argument");
    *nranks = c->nranks;
    *rank = c->rank;
    return SRT_OK;
}

}  // extern "C"
static int render_group_once(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* a, srt_stats* st);
static int render_group_async(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* a);
extern "C" {

int srt_render_group(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* a, srt_stats* st) {
    if (!ctxs || n < 1 || !cam || !a) return fail(SRT_ERR_ARG, "null argument");
    for (int q = 0; q < n; ++q)
        if (!ctxs[q] || ctxs[q]->nranks != n || ctxs[q]->rank != q)
            return fail(SRT_ERR_ARG, "contexts must be the ranks 0..n-1 of one srt_comm_init_all group");
    for (int q = 0; q < n; ++q) ctxs[q]->pf.valid = false;
    if (a->jitter) return fail(SRT_ERR_ARG, "a group frame draws its jitter on the devices (mt or Philox)");
    if (a->out_hit_id) return fail(SRT_ERR_ARG, "hit ids of a sharded frame are not gathered");
    if (a->flags & ~(SRT_RENDER_ASYNC | SRT_RENDER_RGB_ROWS | SRT_RENDER_RGB_LOCAL))
        return fail(SRT_ERR_ARG, "group flags: ASYNC, RGB_ROWS, RGB_LOCAL");
    if ((a->flags & SRT_RENDER_RGB_LOCAL) && (a->out_rgb || (a->flags & SRT_RENDER_RGB_ROWS)))
        return fail(SRT_ERR_ARG, "SRT_RENDER_RGB_LOCAL needs out_rgb NULL and no SRT_RENDER_RGB_ROWS");
    if (a->flags & SRT_RENDER_ASYNC) return render_group_async(ctxs, n, cam, a);
    // A frame whose passes overflowed a queue/ring, met a chain-mode tie or left the fixed-point range
    // is rendered again on every context (the gather pairs the ranks' tiles), from the same numpy
    // state, as the synchronous single-GPU path does; the contexts already grew their queues or
    // dropped chain mode / fixed-point sums in finish_async.
    srt_mt_state mt0{};
    if (a->mt) mt0 = *a->mt;
    int rc = SRT_OK;
    for (int attempt = 0;; ++attempt) {
        if (a->mt) *a->mt = mt0;
        // (a flag left by an earlier frame must not make a failure of this one look retryable)
        for (int q = 0; q < n; ++q) ctxs[q]->retry_frame = false;
        rc = render_group_once(ctxs, n, cam, a, st);
        bool again = false;
        for (int q = 0; q < n; ++q) again |= ctxs[q]->retry_frame;
        if (rc == SRT_OK && st) st->retries += attempt;  // frames rendered again, as srt_render counts them
        if (rc == SRT_OK || !again || attempt >= 8) return rc;
    }
}

}  // extern "C"

static int render_group_once(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* a, srt_stats* st) {
    const bool want_rgb = a->out_rgb != nullptr;
    int rc = SRT_OK;
    srt_render_args aq = *a;
    aq.flags = SRT_RENDER_ASYNC | SRT_RENDER_SHARDED | (want_rgb ? SRT_RENDER_GATHER_RGB : (a->flags & SRT_RENDER_RGB_LOCAL));
    aq.out_rgb = nullptr;  // rank 0 assembles into its slot buffers; copied to the caller's below
    aq.out_srgb8 = nullptr;
    for (int q = 0; q < n && !rc; ++q) {
        if ((rc = finish_async(ctxs[q], nullptr))) break;
        ctxs[q]->defer_gather = true;
        rc = srt_render(ctxs[q], cam, &aq, nullptr);
    }
    FrameSlot* f0 = ctxs[0]->f;
    if (!rc && n > 1) {
        ncclResult_t r = ncclGroupStart();
        for (int q = 0; q < n && !rc && r == ncclSuccess; ++q) {
            (void)hipSetDevice(ctxs[q]->device);
            rc = gather_post(ctxs[q]);
        }
        ncclResult_t r2 = ncclGroupEnd();
        if (!rc && (r != ncclSuccess || r2 != ncclSuccess))
            rc = fail(SRT_ERR_HIP, std::string("RCCL group gather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    }
    if (!rc) {
        (void)hipSetDevice(ctxs[0]->device);
        rc = gather_finish(ctxs[0]);
    }
    srt_stats sum{};
    for (int q = 0; q < n; ++q) {
        ctxs[q]->defer_gather = false;
        srt_stats sq{};
        int r = srt_render_finish(ctxs[q], &sq);
        if (!rc) rc = r;
        if (q == 0) sum = sq;
        else {
            for (int d = 0; d < SRT_MAX_DEPTHS; ++d) sum.rays_per_depth[d] += sq.rays_per_depth[d];
            sum.total_rays += sq.total_rays;
            sum.shadow_rays += sq.shadow_rays;
            sum.n_depths = std::max(sum.n_depths, sq.n_depths);
        }
    }
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctxs[0]->device));
    const int64_t np = (int64_t)cam->width * cam->height;
    if (a->out_srgb8) HIP_TRY(hipMemcpy(a->out_srgb8, f0->full_u8, (size_t)3 * np, hipMemcpyDefault));
    if (want_rgb) HIP_TRY(hipMemcpy(a->out_rgb, f0->full_rgb, (size_t)3 * np * 8, hipMemcpyDefault));
    if (st) *st = sum;
    return SRT_OK;
}

// A pipelined group frame (SRT_RENDER_ASYNC): every context queues its shard (asynchronous
// srt_render, SRT_RENDER_SHARDED), the uint8 tiles' RCCL gather is posted for all of them in one
// group, rank 0 assembles the frame and copies it to the caller's out_srgb8 (pinned host memory or
// device memory of rank 0); the linear RGB goes to out_rgb (pinned host memory visible to every
// context, srt_host_alloc) either gathered to rank 0 or, with SRT_RENDER_RGB_ROWS, as every rank's
// rows over its own PCIe link.  Nothing waits: srt_render_group_finish checks every context.
static int render_group_async(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* a) {
    srt_render_args aq = *a;
    const bool rows = (a->flags & SRT_RENDER_RGB_ROWS) != 0;
    aq.flags = SRT_RENDER_ASYNC | SRT_RENDER_SHARDED | (a->flags & SRT_RENDER_RGB_LOCAL) |
               (rows ? SRT_RENDER_RGB_ROWS : (a->out_rgb ? SRT_RENDER_GATHER_RGB : 0));
    int rc = SRT_OK;
    int queued = 0;
    for (int q = 0; q < n && !rc; ++q) {
        aq.out_srgb8 = q == 0 ? a->out_srgb8 : nullptr;
        aq.out_rgb = (rows || q == 0) ? a->out_rgb : nullptr;
        ctxs[q]->defer_gather = true;
        rc = srt_render(ctxs[q], cam, &aq, nullptr);
        if (!rc) ++queued;
    }
    if (!rc && n > 1) {
        ncclResult_t r = ncclGroupStart();
        for (int q = 0; q < n && !rc && r == ncclSuccess; ++q) {
            (void)hipSetDevice(ctxs[q]->device);
            rc = gather_post(ctxs[q]);
        }
        ncclResult_t r2 = ncclGroupEnd();
        if (!rc && (r != ncclSuccess || r2 != ncclSuccess))
            rc = fail(SRT_ERR_HIP, std::string("RCCL group gather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    }
    if (!rc) {
        (void)hipSetDevice(ctxs[0]->device);
        rc = gather_finish(ctxs[0]);
    }
    for (int q = 0; q < n; ++q) ctxs[q]->defer_gather = false;
    if (rc && queued < n) {
        // a context refused the frame: the others' shards are queued without the gather; wait for them
        // (their frames are dropped) so that no rank is left a send without its receive
        for (int q = 0; q < queued; ++q) (void)srt_render_finish(ctxs[q], nullptr);
    }
    return rc;
}

extern "C" {

int srt_render_group_finish(srt_ctx** ctxs, int n, srt_stats* st) {
    if (!ctxs || n < 1) return fail(SRT_ERR_ARG, "null argument");
    int rc = SRT_OK;
    srt_stats sum{};
    for (int q = 0; q < n; ++q) {
        srt_stats sq{};
        const int r = srt_render_finish(ctxs[q], &sq);
        if (!rc) rc = r;
        if (q == 0) {
            sum = sq;
        } else {
            for (int d = 0; d < SRT_MAX_DEPTHS; ++d) sum.rays_per_depth[d] += sq.rays_per_depth[d];
            sum.total_rays += sq.total_rays;
            sum.shadow_rays += sq.shadow_rays;
            sum.n_depths = std::max(sum.n_depths, sq.n_depths);
        }
    }
    if (st && !rc) *st = sum;
    return rc;
}

int srt_comm_allreduce(srt_ctx* c, double* vals, int n, int op) {
    if (!c || !vals || n < 1 || n > 64 || op < 0 || op > 1) return fail(SRT_ERR_ARG, "bad allreduce arguments");
    if (c->nranks == 1 || !c->comm) return SRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc = finish_async(c, nullptr);
    if (rc) return rc;
    if (!c->red) HIP_TRY(dalloc(&c->red, 64));
    hipStream_t st = c->f->stream;
    HIP_TRY(hipMemcpyAsync(c->red, vals, (size_t)n * 8, hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllReduce(c->red, c->red, (size_t)n, ncclFloat64, op == 0 ? ncclSum : ncclMax, c->comm, st));
    HIP_TRY(hipMemcpyAsync(vals, c->red, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SRT_OK;
}

int srt_comm_barrier(srt_ctx* c) {
    double v = 0.0;
    return srt_comm_allreduce(c, &v, 1, 0);
}

// (hipHostMalloc places the buffer on the GPU's NUMA node: tools/pcie_probe.py, 56 GB/s either way
// the calling process is pinned)
int srt_host_alloc(srt_ctx* c, int64_t bytes, void** out) {
    if (!c || !out || bytes <= 0) return fail(SRT_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipHostMalloc(out, (size_t)bytes, hipHostMallocPortable));  // (pinned for every context's device)
    return SRT_OK;
}

int srt_host_register(srt_ctx* c, void* p, int64_t bytes) {
    if (!c || !p || bytes <= 0) return fail(SRT_ERR_ARG, "null ctx/pointer or bad size");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipHostRegister(p, (size_t)bytes, hipHostRegisterPortable));
    return SRT_OK;
}

int srt_host_unregister(srt_ctx* c, void* p) {
    if (!c || !p) return fail(SRT_ERR_ARG, "null ctx/pointer");
    HIP_TRY(hipSetDevice(c->device));
    int rc = finish_async(c, nullptr);  // frames in flight may still write into it
    if (rc) return rc;
    HIP_TRY(hipHostUnregister(p));
    return SRT_OK;
}

int srt_host_free(srt_ctx* c, void* p) {
    if (!c) return fail(SRT_ERR_ARG, "null ctx");
    if (p) HIP_TRY(hipHostFree(p));
    return SRT_OK;
}

#ifdef RT_PROF
// diagnostic build only: section counters of rt_device.h (64 words: 32 cycle sums, 32 counts)
int srt_debug_prof(srt_ctx* c, unsigned long long* out, int reset) {
    if (!c || !out) return fail(SRT_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->f->stream));
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_prof), sizeof(unsigned long long) * 64));
    if (reset) {
        unsigned long long z[64] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rt_prof), z, sizeof(z)));
    }
    return SRT_OK;
}
#endif

int srt_debug_lean_launches(srt_ctx* c, int64_t* launches) {
    if (!c || !launches) return fail(SRT_ERR_ARG, "null argument");
    *launches = c->lean_launches;
    return SRT_OK;
}

int srt_debug_lane_stats(srt_ctx* c, int mode, int64_t* out, int n) {
    if (!c) return fail(SRT_ERR_ARG, "null ctx");
    if (mode != 0 && mode != 1) return fail(SRT_ERR_ARG, "lane stats mode: 1 start, 0 read and stop");
    HIP_TRY(hipSetDevice(c->device));
    int rc = finish_async(c, nullptr);  // (the frames in flight were queued with the old pointer)
    if (rc) return rc;
    const size_t bytes = (size_t)SRT_MAX_DEPTHS * 2 * sizeof(unsigned long long);
    if (mode == 1) {
        if (!c->lane_stats) HIP_TRY(hipMalloc(&c->lane_stats, bytes));
        HIP_TRY(hipMemset(c->lane_stats, 0, bytes));
        return SRT_OK;
    }
    if (!out || n < 0 || n > SRT_MAX_DEPTHS) return fail(SRT_ERR_ARG, "lane stats: out[n][2], n <= SRT_MAX_DEPTHS");
    if (!c->lane_stats) return fail(SRT_ERR_ARG, "lane stats were not started");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, c->lane_stats, (size_t)n * 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(c->lane_stats));
    c->lane_stats = nullptr;
    return SRT_OK;
}

int srt_debug_prefetch_counts(srt_ctx* c, int64_t* used, int64_t* queued) {
    if (!c || !used || !queued) return fail(SRT_ERR_ARG, "null argument");
    *used = c->pf_used;
    *queued = c->pf_queued;
    return SRT_OK;
}

int srt_debug_mt_residue(srt_ctx* c, int64_t* nonzero_words) {
    if (!c || !nonzero_words) return fail(SRT_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    int rc = finish_async(c, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    int64_t nz = 0;
    std::vector<uint32_t> h;
    auto count = [&](const uint32_t* d, int64_t words) -> int {
        h.resize((size_t)words);
        HIP_TRY(hipMemcpy(h.data(), d, (size_t)words * 4, hipMemcpyDeviceToHost));
        for (uint32_t w : h) nz += w != 0u;
        return SRT_OK;
    };
    // (window 0 of a table holds a copy of the key, written by a plain store at every generation that
    // jumps -- never an XOR target -- and left there when no segment starts at the key: not counted)
    for (FrameSlot& f : c->slots)
        if (f.mt_win && f.mt_win_cap > rtmt::N && (rc = count(f.mt_win + rtmt::N, f.mt_win_cap - rtmt::N))) return rc;
    if (c->mt && (rc = count(mt_end_acc(c), rtmt::N + 1))) return rc;
    *nonzero_words = nz;
    return SRT_OK;
}

int srt_synchronize(srt_ctx* c) {
    if (!c) return fail(SRT_ERR_ARG, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    for (FrameSlot& f : c->slots)
        if (f.stream) HIP_TRY(hipStreamSynchronize(f.stream));
    return SRT_OK;
}

}  // extern "C"
