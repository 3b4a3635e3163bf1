// rt_hostcheck.cpp -- TEST HARNESS ONLY (tests/_build/libsightpy_hostcheck.so).
//
// A sequential, breadth-first CPU driver over the *same* per-ray functions the gfx950 kernels
// use (rt_device.h), compiled by g++ with -ffp-contract=off.  It lets the CPU test suite check
// the kernel math against the numpy oracle in a container without a GPU.  It is never loaded by
// the product package (sightpy/_native.py loads only libsightpy_hip.so and fails loudly without
// it); it mirrors the kernel's RNG keys and child-path hashing, so Monte-Carlo scenes give the
// same samples as the GPU path up to transcendental-function ulps.
#include <cstring>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_mt.h"

using namespace rt;

namespace {

thread_local std::string g_err;

struct Scene {
    SceneView S{};
    int max_depth = 0;
    int has_diffuse = 0;
};

thread_local BvhBuild g_bvh;  // the BVH of the scene of the current call
thread_local int g_use_bvh = 1;
// rows of the current hc_render (null: identity / hc_trace): Monte-Carlo draws are keyed by the
// global pixel, as key_pix in rt_kernels.hip
thread_local const int32_t* g_rows = nullptr;
thread_local int64_t g_width = 0;

uint32_t key_pix(uint32_t pix) {
    if (!g_rows) return pix;
    const uint32_t W = (uint32_t)g_width, lr = pix / W;
    return (uint32_t)g_rows[lr] * W + (pix - lr * W);
}

SceneView view_of(const srt_scene_desc* d) {
    SceneView S{};
    if (g_use_bvh) {
        bvh_build(d->colliders, d->n_colliders, g_bvh);
    } else {
        g_bvh = BvhBuild{};
        for (int i = 0; i < d->n_colliders; ++i) g_bvh.lin.push_back(i);
    }
    S.nlin = (int)g_bvh.lin.size();
    S.lin = g_bvh.lin.data();
    S.bvh = g_bvh.nodes.empty() ? nullptr : g_bvh.nodes.data();
    S.bvh_tri = g_bvh.tri.empty() ? nullptr : g_bvh.tri.data();
    S.bvh_nodes = (int)g_bvh.nodes.size();
    S.bvh_bound = g_bvh.bound;
    S.col = d->colliders; S.mat = d->materials; S.tex = d->textures; S.texels = d->texels;
    S.lights = d->lights; S.media = d->media; S.glossy_f0 = d->glossy_f0; S.light_local = d->light_local;
    S.importance = d->importance;
    S.ncol = d->n_colliders; S.nmat = d->n_materials; S.ntex = d->n_textures; S.nlights = d->n_lights;
    S.nmedia = d->n_media; S.nimp = d->n_importance;
    S.sky_col = sky_collider(d->colliders, d->n_colliders, d->materials);
    S.nshadow = 0;
    for (int i = 0; i < d->n_colliders; ++i)
        if (d->colliders[i].flags & SRT_CF_SHADOW) S.nshadow++;
    for (int k = 0; k < 3; ++k) S.ambient[k] = d->ambient[k];
    return S;
}

int depth_cap(const srt_scene_desc* d) {
    int diff = 0;
    for (int i = 0; i < d->n_materials; ++i)
        if (d->materials[i].type == SRT_DIFFUSE) diff = 1;
    return d->max_ray_depth + 1 + (diff ? 2 : 0);
}

struct HostEmit {
    const SceneView& S;
    const Ray& r;
    std::vector<Ray>& next;
    double* fb;
    int64_t npix;
    uint64_t seed;
    int depth;
    uint32_t round;
    int64_t* sh;

    void local(d3 c) const {
        if (is_zero(c)) return;
        fb[r.pix] += r.w.x * c.x;
        fb[npix + r.pix] += r.w.y * c.y;
        fb[2 * npix + r.pix] += r.w.z * c.z;
    }
    void shadow(int n) const { *sh += n; }
    void push(const Child& c, uint32_t path) const {
        Ray k;
        k.o = c.o; k.d = c.d; k.w = mul(r.w, c.w);
        k.pix = r.pix;
        k.meta = pack_meta(c.medium, meta_depth(r.meta) + 1, c.dfl);
        k.path = path;
        next.push_back(k);
    }
    void child(const Child& c) const { push(c, child_path(r.path, c.slot, round)); }
    void diffuse(const DiffuseGen& g, int mi) const {
        for (int k = 0; k < g.count; ++k) {
            Rng rng;
            const uint32_t cpath = child_path(r.path, 0x100u + (uint32_t)k, round);
            rng.init(seed, key_pix(r.pix), cpath, 0xD1000000u | (uint32_t)depth);
            push(diffuse_child(S, S.mat[mi], g, rng, (uint32_t)k), cpath);
        }
    }
};

double mc_uniform(const SceneView& S, uint64_t seed, int depth, const Ray& r, int cid, uint32_t round) {
    if (!(S.col[cid].flags & SRT_CF_MC)) return 0.0;
    Rng g;
    g.init(seed, key_pix(r.pix), r.path, 0x3C000000u | ((uint32_t)depth << 8) | round);
    return g.one();
}

void trace_one(const SceneView& S, const Ray& r, int depth, uint64_t seed, std::vector<Ray>& next, double* fb,
               int64_t npix, uint32_t& err, int64_t& shadow, int32_t* hit_slot) {
    double t, o;
    bool ties;
    int id = nearest_hit(S, r.o, r.d, t, o, ties);
    if (hit_slot) *hit_slot = id;
    if (id < 0) return;
    HostEmit em{S, r, next, fb, npix, seed, depth, 0u, &shadow};
    shade_hit<MAT_GENERIC | MAT_BVH>(S, id, S.col[id].material, r, t, o, em, err, mc_uniform(S, seed, depth, r, id, 0));
    if (ties) {
        uint32_t round = 1;
        for (int c = id + 1; c < S.ncol; ++c) {
            double oc;
            if (collider_hit(S.col[c], r.o, r.d, oc) == t) {
                HostEmit et{S, r, next, fb, npix, seed, depth, round, &shadow};
                shade_hit<MAT_GENERIC | MAT_BVH>(S, c, S.col[c].material, r, t, oc, et, err,
                                             mc_uniform(S, seed, depth, r, c, round));
                ++round;
            }
        }
    }
}

int err_code(uint32_t e) {
    if (e & ERR_INDEX) { g_err = "index out of bounds in a texture/table lookup"; return SRT_ERR_INDEX; }
    if (e & ERR_UNSUPPORTED) { g_err = "uv requested on a Triangle"; return SRT_ERR_ARG; }
    if (e & ERR_NAME) { g_err = "name 'M' is not defined (PointLight.get_L)"; return SRT_ERR_NAME; }
    return SRT_OK;
}

}  // namespace

extern "C" {

const char* hc_last_error(void) { return g_err.c_str(); }

// 1: triangle colliders of large meshes go through the BVH (as on the GPU); 0: linear loop only
void hc_set_bvh(int on) { g_use_bvh = on; }
int hc_bvh_nodes(const srt_scene_desc* d) {
    BvhBuild b;
    bvh_build(d->colliders, d->n_colliders, b);
    return (int)b.nodes.size();
}

// Breadth-first render of `args->spp` samples (host pointers only); out_rgb = linear RGB / spp.
int hc_render(const srt_scene_desc* d, const srt_camera* cam, const srt_render_args* a, srt_stats* st) {
    SceneView S = view_of(d);
    const int64_t W = cam->width, npix = (int64_t)a->n_rows * W;
    std::vector<double> fb(3 * npix, 0.0);
    uint32_t err = 0;
    int64_t shadow = 0;
    srt_stats stats{};
    const int dcap = depth_cap(d);
    g_rows = a->rows;
    g_width = W;
    for (int s = 0; s < a->spp; ++s) {
        std::vector<Ray> cur, next;
        for (int64_t p = 0; p < npix; ++p) {
            int64_t lr = p / W, col = p % W;
            int grow = a->rows ? a->rows[lr] : (int)lr;
            double j[4];
            if (a->jitter) {
                const double* b = a->jitter + (int64_t)s * 4 * npix + p;
                j[0] = b[0]; j[1] = b[npix]; j[2] = b[2 * npix]; j[3] = b[3 * npix];
            } else {
                Rng g;
                g.init(a->seed, (uint32_t)(grow * W + col), (uint32_t)(a->sample_base + s), 0xCA3E0000u);
                g.two(j[0], j[1]);
                g.two(j[2], j[3]);
            }
            Ray r;
            primary_ray(*cam, cam->xs[col], cam->ys[grow], j, r.o, r.d);
            r.w = d3{1.0, 1.0, 1.0};
            r.pix = (uint32_t)p;
            r.meta = pack_meta(0, 0, 0);
            r.path = mix32(0x5EED0000u, (uint32_t)(a->sample_base + s));
            int32_t* hs = a->out_hit_id ? a->out_hit_id + (int64_t)s * npix + p : nullptr;
            trace_one(S, r, 0, a->seed, next, fb.data(), npix, err, shadow, hs);
        }
        stats.rays_per_depth[0] += npix;
        for (int dpt = 1; dpt <= dcap && !next.empty(); ++dpt) {
            cur.swap(next);
            next.clear();
            stats.rays_per_depth[dpt] += (int64_t)cur.size();
            for (const Ray& r : cur) trace_one(S, r, dpt, a->seed, next, fb.data(), npix, err, shadow, nullptr);
        }
        if (!next.empty()) { g_err = "rays alive after the depth cap"; return SRT_ERR_DEPTH; }
    }
    if (int rc = err_code(err)) return rc;
    for (int64_t p = 0; p < npix; ++p) {
        double r = fb[p] / a->spp, g = fb[npix + p] / a->spp, b = fb[2 * npix + p] / a->spp;
        uint8_t px[3];
        double q0, q1, q2;
        resolve_pixel(r, g, b, q0, q1, q2, px);
        if (a->out_rgb) { a->out_rgb[p] = r; a->out_rgb[npix + p] = g; a->out_rgb[2 * npix + p] = b; }
        if (a->out_srgb8) { a->out_srgb8[3 * p] = px[0]; a->out_srgb8[3 * p + 1] = px[1]; a->out_srgb8[3 * p + 2] = px[2]; }
    }
    stats.n_depths = dcap + 1;
    for (int k = 0; k <= dcap; ++k) stats.total_rays += stats.rays_per_depth[k];
    stats.shadow_rays = shadow;
    stats.passes = 1;
    if (st) *st = stats;
    return SRT_OK;
}

int hc_trace(const srt_scene_desc* d, const srt_trace_args* a, srt_stats* st) {
    SceneView S = view_of(d);
    g_rows = nullptr;
    const int64_t n = a->n;
    std::vector<double> fb(3 * n, 0.0);
    std::vector<Ray> cur, next;
    for (int64_t i = 0; i < n; ++i) {
        Ray r;
        r.o = d3{a->origin[i], a->origin[n + i], a->origin[2 * n + i]};
        r.d = d3{a->dir[i], a->dir[n + i], a->dir[2 * n + i]};
        r.w = d3{1.0, 1.0, 1.0};
        r.pix = (uint32_t)i;
        r.meta = pack_meta(a->medium ? (uint32_t)a->medium[i] : 0u, (uint32_t)a->depth, (uint32_t)a->diffuse_reflections);
        r.path = mix32(0x7A11u, (uint32_t)i);
        cur.push_back(r);
    }
    uint32_t err = 0;
    int64_t shadow = 0;
    srt_stats stats{};
    const int dlast = a->depth + depth_cap(d);
    for (int dpt = a->depth; dpt <= dlast && !cur.empty(); ++dpt) {
        stats.rays_per_depth[dpt] = (int64_t)cur.size();
        next.clear();
        for (const Ray& r : cur) trace_one(S, r, dpt, a->seed, next, fb.data(), n, err, shadow, nullptr);
        cur.swap(next);
    }
    if (!cur.empty()) { g_err = "rays alive after the depth cap"; return SRT_ERR_DEPTH; }
    if (int rc = err_code(err)) return rc;
    std::memcpy(a->out_rgb, fb.data(), 3 * n * sizeof(double));
    stats.n_depths = dlast + 1;
    for (int k = 0; k < SRT_MAX_DEPTHS; ++k) stats.total_rays += stats.rays_per_depth[k];
    stats.shadow_rays = shadow;
    if (st) *st = stats;
    return SRT_OK;
}

int hc_nearest(const srt_scene_desc* d, const double* O, const double* D, int64_t n, double* t, int32_t* id,
               double* orient) {
    SceneView S = view_of(d);
    for (int64_t i = 0; i < n; ++i) {
        double tn, on;
        bool ties;
        int c = nearest_hit(S, d3{O[i], O[n + i], O[2 * n + i]}, d3{D[i], D[n + i], D[2 * n + i]}, tn, on, ties);
        if (t) t[i] = tn;
        if (id) id[i] = c;
        if (orient) orient[i] = on;
    }
    return SRT_OK;
}

int hc_intersect_collider(const srt_collider* c, const double* O, const double* D, int64_t n, double* out) {
    for (int64_t i = 0; i < n; ++i) {
        double o;
        out[i] = collider_hit(*c, d3{O[i], O[n + i], O[2 * n + i]}, d3{D[i], D[n + i], D[2 * n + i]}, o);
        out[n + i] = o;
    }
    return SRT_OK;
}

int hc_primary_rays(const srt_camera* cam, const double* J, double* O, double* D) {
    const int64_t n = (int64_t)cam->width * cam->height;
    for (int64_t i = 0; i < n; ++i) {
        int64_t row = i / cam->width, col = i % cam->width;
        double j[4] = {J[i], J[n + i], J[2 * n + i], J[3 * n + i]};
        d3 o, d;
        primary_ray(*cam, cam->xs[col], cam->ys[row], j, o, d);
        O[i] = o.x; O[n + i] = o.y; O[2 * n + i] = o.z;
        D[i] = d.x; D[n + i] = d.y; D[2 * n + i] = d.z;
    }
    return SRT_OK;
}

// rt_device.h's Philox4x32-10 and path hash (known-answer tests of the Monte-Carlo stream)
void hc_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out) {
    const u4 r = philox(u4{ctr[0], ctr[1], ctr[2], ctr[3]}, k0, k1);
    out[0] = r.a; out[1] = r.b; out[2] = r.c; out[3] = r.d;
}
uint32_t hc_mix32(uint32_t h, uint32_t v) { return mix32(h, v); }

// row-band shard map of the sharded render (rt_device.h): band height, owner rank and local row of
// global row y, with at most kmax bands per rank, dealt round-robin
int hc_shard_kmax(int64_t H, int n, int kmax, int fanout) { return shard_kmax(H, n, kmax, fanout); }
int64_t hc_shard_map(int64_t H, int n, int kmax, int32_t* owner, int64_t* local) {
    const int64_t h = shard_band_height(H, n, kmax);
    for (int64_t y = 0; y < H; ++y) {
        owner[y] = shard_of_row(y, n, h);
        local[y] = shard_local_row(y, n, h);
    }
    return h;
}

// numpy legacy rand stream by the segmented jump-ahead scheme of rt_mt.h, run serially
int hc_mt_uniforms(const uint32_t* key, int pos, int64_t n_out, int64_t n_skip, double* out, uint32_t* key_out,
                   int* pos_out) {
    if (pos < 0 || pos > rtmt::N || n_out < 0 || n_skip < 0 || n_out + n_skip == 0) return SRT_ERR_ARG;
    rtmt::uniforms_serial(key, pos, n_out, n_skip, out, key_out, pos_out);
    return SRT_OK;
}

// x^J mod phi (rt_mt.h xpow_mod), 624 words
void hc_xpow_mod(uint64_t J, uint32_t* out) {
    const std::vector<uint32_t> p = rtmt::xpow_mod(J);
    memcpy(out, p.data(), rtmt::N * 4);
}

// the window J words past `key` by the polynomial jump (rt_mt.h jump_serial with x^J)
void hc_jump_window(const uint32_t* key, uint64_t J, uint32_t* out) {
    const std::vector<uint32_t> p = rtmt::xpow_mod(J);
    rtmt::jump_serial(key, p.data(), out);
}

}  // extern "C"
