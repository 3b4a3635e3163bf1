/*
 * sightpy_rt.h -- C ABI of the MI355X (gfx950) ray-trace backend, libsightpy_hip.so.
 *
 * This is the drop-in boundary for the hot path of lmondada/Python-Raytracer ("sightpy").
 * The reference is pure Python/numpy with no FFI; each entry point below replaces one Python
 * interface of the reference and is what a ctypes binding of that interface calls
 * (the binding is python-raytracer_amd/sightpy/_native.py):
 *
 *   srt_render             <- Scene.render            sightpy/scene.py:71-140
 *                             (camera.get_ray per sample, get_raycolor recursion, spp average,
 *                              sRGB_linear_to_sRGB + clip + uint8 resolve)
 *   srt_trace              <- get_raycolor(ray, scene) sightpy/ray.py:122-148
 *   srt_nearest            <- get_distances / the nearest-hit reduction
 *                                                     sightpy/ray.py:124-132, 151-163
 *   srt_intersect_collider <- Collider.intersect(O, D) sightpy/geometry/collider.py:12-14
 *                             (sphere.py:26-52, plane.py:57-90, cuboid.py:105-140,
 *                              triangle.py:36-66)
 *   srt_shade              <- Material.get_color(scene, ray, hit) at given hits
 *                             (material.py:43, glossy.py:25, refractive.py:24, diffuse.py:25,
 *                              thin_film_interference.py:24, emissive.py:21; the children it
 *                              spawns are traced as in get_raycolor)
 *   srt_collider_surface   <- Collider.get_Normal(hit) / Collider.get_uv(hit) / Primitive.get_uv
 *                             (sphere.py:17,54-64, plane.py:34,98-105, cuboid.py:29,142-187,
 *                              triangle.py:85, skybox.py:29)
 *   srt_texture_lookup     <- image.get_color(hit)     sightpy/textures/texture.py:32-39
 *   srt_material_normal    <- Material.get_Normal(hit) sightpy/materials/material.py:18-36
 *   srt_primary_rays       <- Camera.get_ray(n)       sightpy/camera.py:51-85
 *   srt_upload_scene       <- (scene lowering; the reference deep-copies the Scene per task,
 *                              scene.py:85)
 *
 * Conventions
 *   - Every entry point returns 0 on success or a negative SRT_ERR_* code; the message of the
 *     last failure on the calling thread is srt_last_error().  No C++ exception crosses the ABI.
 *   - Array arguments are plain pointers + sizes.  Vectors are planar [3][n] float64 (the
 *     reference's vec3.to_array() layout).  A pointer may address host memory or device memory
 *     of the context's GPU (copies use hipMemcpyDefault); host memory is borrowed for the call.
 *   - All arithmetic is IEEE float64 (complex128 for the index of refraction), evaluated in the
 *     reference's operation order with FP contraction disabled.
 *   - One context = one GPU; a context must be used by one host thread at a time.
 */
#ifndef SIGHTPY_RT_H
#define SIGHTPY_RT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRT_ABI_VERSION 5

/* ---- error codes ------------------------------------------------------------------------ */
#define SRT_OK 0
#define SRT_ERR_ARG -1      /* bad argument / unsupported scene feature */
#define SRT_ERR_HIP -2      /* HIP runtime failure (message has the hipError string) */
#define SRT_ERR_NOSCENE -3  /* render/trace before srt_upload_scene */
#define SRT_ERR_MEMORY -4   /* queue / framebuffer allocation failed */
#define SRT_ERR_INDEX -5    /* a table index left its array (the reference raises IndexError) */
#define SRT_ERR_DEPTH -6    /* rays still alive after the depth cap */
#define SRT_ERR_NAME -7     /* a Glossy hit shaded under a PointLight: the reference raises NameError
                               (PointLight.get_L uses undefined names, sightpy/lights.py:30-31) */

/* ---- scene tables --------------------------------------------------------------------- */
enum { SRT_SPHERE = 0, SRT_PLANE = 1, SRT_CUBOID = 2, SRT_TRIANGLE = 3 };
enum {
    SRT_GLOSSY = 0,
    SRT_REFRACTIVE = 1,
    SRT_THINFILM = 2,
    SRT_DIFFUSE = 3,
    SRT_EMISSIVE = 4,
    SRT_SKY = 5
};
/* collider flags */
#define SRT_CF_SHADOW 1u   /* member of scene.shadowed_collider_list */
#define SRT_CF_MC 2u       /* primitive.mc: Monte-Carlo refraction pick */
#define SRT_CF_UV_CROSS 4u /* Cuboid/SkyBox primitive: uv /= (4, 3) */
/* material flags */
#define SRT_MF_ROUGH 1u    /* Glossy: roughness != 0 (specular lobe on) */
#define SRT_MF_LIGHTMAP 2u /* SkyBox: light_intensity != 0 (lightmap on non-primary rays) */
#define SRT_MF_NOISE 4u    /* ThinFilm: noise != 0 (thickness jitter from noise texture) */

#define SRT_COLLIDER_PARAMS 48
#define SRT_MATERIAL_PARAMS 16

/*
 * Collider parameter layout (p[]), all float64, host-precomputed exactly as the reference:
 *   SPHERE   0-2 center, 3 radius, 4 1.0/radius, 5 center.square_length(), 6 radius*radius
 *   PLANE    0-2 center, 3-5 normal, 6-8 u_axis, 9-11 v_axis, 12 w, 13 h, 14-15 uv_shift,
 *            16-24 inverse_basis_matrix (row-major)
 *   CUBOID   0-2 center, 3-11 basis_matrix (row-major), 12-14 lb_local_basis,
 *            15-17 rt_local_basis, 18-20 ax_w, 21-23 ax_h, 24-26 ax_l, 27 width, 28 height,
 *            29 length, 30-38 inverse_basis_matrix (row-major), 39-41 (1/width,1/height,1/length),
 *            42 1.0 if basis_matrix is exactly the identity (else 0.0)
 *   TRIANGLE 0-2 centroid, 3-5 normal, 6-8 p1, 9-11 p2, 12-14 p3, 15-17 n31, 18-20 n12,
 *            21-23 n23
 */
typedef struct srt_collider {
    int32_t type;          /* SRT_SPHERE .. */
    int32_t material;      /* index into the material table */
    int32_t max_ray_depth; /* primitive.max_ray_depth */
    uint32_t flags;        /* SRT_CF_* */
    int32_t primitive;     /* index of the owning primitive (diagnostics) */
    int32_t reserved[3];
    double p[SRT_COLLIDER_PARAMS];
} srt_collider;

/*
 * Material parameter layout (p[]):
 *   GLOSSY     0-2 solid diffuse colour * diff_coeff (tex < 0), 3 diff_coeff, 4 a = 2/r^2 - 2,
 *              5 a + 2.0, 6 2.0*pi, 7 spec_coeff, 8-10 F0 of the reflection term (scene.n vs n),
 *              11-13 specular F0 for medium 0 (= glossy_f0[m][0]; the specular F0 depends on the
 *              ray's medium: srt_scene_desc.glossy_f0)
 *   REFRACTIVE (index of refraction = media[medium])
 *   THINFILM   0 thickness, 1 noise factor
 *   DIFFUSE    0-2 solid colour, 3 ambient_weight, 4 1 - ambient_weight
 *   EMISSIVE   0-2 solid colour
 *   SKY        0 light_intensity
 */
typedef struct srt_material {
    int32_t type;      /* SRT_GLOSSY .. */
    int32_t tex;       /* colour texture (GLOSSY/DIFFUSE/EMISSIVE/SKY), -1 = solid colour */
    int32_t tex_aux0;  /* THINFILM: reflectance table; SKY: lightmap */
    int32_t tex_aux1;  /* THINFILM: thickness noise */
    int32_t normalmap; /* normal-map texture, -1 = none */
    int32_t medium;    /* REFRACTIVE: media[] row holding its n */
    uint32_t flags;    /* SRT_MF_* */
    int32_t ival;      /* DIFFUSE: diffuse_rays; GLOSSY: k > 0 when the lobe exponent p[4] is within
                          4 ulp of the integer k (x^p[4] is then evaluated as x^k, < 1e-12 relative
                          apart), 0 = general pow */
    double p[SRT_MATERIAL_PARAMS];
} srt_material;

/*
 * A texture is a uint8 image in the shared texel pool plus a 256-entry float64 table: a texel
 * byte b reads as lut[b].  lut = sRGB_to_sRGB_linear(b/256) for linear-sRGB images, b/256 for
 * raw ones, which reproduces the reference's float arrays bit for bit.  The lookup index is
 *   row = -(trunc(v*idx_h*repeat) mod idx_h), col = trunc(u*idx_w*repeat) mod idx_w
 * (texture.py:32-39), with numpy negative-index wrap against `height`.
 */
typedef struct srt_texture {
    int64_t offset;   /* byte offset of texel (0,0) in the pool */
    int32_t height;   /* rows of the stored image */
    int32_t width;    /* columns */
    int32_t channels; /* bytes per texel (>= 3, or 1..4 with channel0) */
    int32_t channel0; /* first channel read */
    int32_t idx_h;    /* shape used by the index arithmetic (== height except the lightmap) */
    int32_t idx_w;
    double repeat;
    double lut[256];
} srt_texture;

enum { SRT_LIGHT_DIRECTIONAL = 0, SRT_LIGHT_POINT = 1 };
typedef struct srt_light {
    int32_t type;
    int32_t reserved;
    double dir[3]; /* DirectionalLight.Ldir (normalised by Scene.add_DirectionalLight) */
    double color[3];
    double pos[3]; /* PointLight.pos (kept for the record: shading a Glossy hit under a point light
                      fails with SRT_ERR_NAME, as the reference raises NameError) */
} srt_light;

typedef struct srt_scene_desc {
    int32_t n_colliders;
    int32_t n_materials;
    int32_t n_textures;
    int32_t n_lights;
    int32_t n_media;      /* rows of media[]; row 0 is scene.n */
    int32_t n_importance; /* scene.importance_sampled_list */
    const srt_collider* colliders; /* scene.collider_list order */
    const srt_material* materials;
    const srt_texture* textures;
    const uint8_t* texels;
    int64_t texel_bytes;
    const srt_light* lights;
    const double* media;       /* [n_media][6]: Re n (3), Im n (3) */
    const double* glossy_f0;   /* [n_materials][n_media][3]: |(n_ray-n)/(n_ray+n)|^2 */
    const double* light_local; /* [n_lights][n_colliders][3]: Ldir.matmul(basis) (cuboids) */
    const double* importance;  /* [n_importance][4]: center xyz, bounded_sphere_radius */
    double ambient[3];         /* scene.ambient_color */
    int32_t max_ray_depth;     /* max over colliders (depth cap = this + 1, +2 with Diffuse) */
    int32_t has_diffuse;
    uint64_t texel_key;        /* caller's identity of the texel pool (0 = none): when it and
                                  texel_bytes equal the resident pool's, the pool stays in HBM and is
                                  not copied again (frame sequences re-upload only the small tables) */
} srt_scene_desc;

/* ---- camera / render ------------------------------------------------------------------ */
typedef struct srt_camera {
    int32_t width;  /* screen_width */
    int32_t height; /* screen_height */
    const double* xs; /* [width]  np.linspace(-cw/2, cw/2, width) */
    const double* ys; /* [height] np.linspace(ch/2, -ch/2, height) */
    double look_from[3];
    double right[3];  /* cameraRight */
    double up[3];     /* cameraUp */
    double fwd_fd[3]; /* cameraFwd * focal_distance */
    double cam_width;
    double cam_height;
    double lens_radius;
    double focal_distance;
} srt_camera;

/* numpy's legacy global RandomState (np.random.get_state(): MT19937 key window and position) */
typedef struct srt_mt_state {
    uint32_t key[624];
    int32_t pos; /* 0..624 */
    int32_t reserved;
} srt_mt_state;

typedef struct srt_render_args {
    int32_t spp;          /* samples traced by this call */
    int32_t sample_base;  /* global index of the first sample (RNG key) */
    int32_t n_rows;       /* rows rendered by this call (a shard of the image) */
    int32_t batch_spp;    /* samples per device pass (0 = fit to the HBM budget) */
    const int32_t* rows;  /* [n_rows] global row index of each local row; NULL = 0..n_rows-1 */
    const double* jitter; /* [spp][4][n_rows*width] uniforms (x-jitter, y-jitter, r, phi) in
                             numpy's draw order, or NULL (then `mt`, else device Philox keyed by
                             (seed, pixel, sample)) */
    srt_mt_state* mt;     /* jitter == NULL, mt != NULL: the jitter is numpy's legacy rand stream
                             from *mt exactly as Scene.render draws it (Camera.get_ray per sample,
                             camera.py:56-64, then one more get_ray for sizing, scene.py:81: that is
                             spp*4*width*height doubles of which a shard reads its rows, then
                             4*width*height skipped), generated on the device (rt_mt.h); *mt is
                             advanced past them.  Consecutive asynchronous frames that pass the same
                             `mt` continue the stream on the device; *mt is written by
                             srt_render_finish */
    uint64_t seed;        /* device RNG key (jitter when jitter == NULL, Monte-Carlo shading) */
    double* out_rgb;      /* [3][n_rows*width] linear RGB averaged over spp, or NULL */
    uint8_t* out_srgb8;   /* [n_rows*width][3] resolved image, or NULL */
    int32_t* out_hit_id;  /* [spp][n_rows*width] primary nearest collider (-1 miss), or NULL */
    int32_t flags;        /* SRT_RENDER_* */
    int32_t reserved;
} srt_render_args;

/* SRT_RENDER_ASYNC: queue the frame on the context's stream and return at once (jitter must be
 * device memory or NULL, outputs device memory, pinned host memory from srt_host_alloc, or NULL;
 * `stats` is not written).  Consecutive asynchronous frames of the same shape pipeline back to back
 * without host round trips; srt_render_finish waits for them, checks their error flags and returns
 * the last one's stats.  Any other call on the context first finishes pending frames.  (No
 * reference counterpart: Scene.render is synchronous; this serves frame sequences such as
 * create_animation and the multi-GPU frame loop.) */
#define SRT_RENDER_ASYNC 1
/* SRT_RENDER_SHARDED: the context's communicator (srt_comm_init / srt_comm_init_all) splits the
 * frame: this rank renders the rows {y : (y / h) % nranks == rank} (h-row bands dealt round-robin,
 * which balances cheap sky rows against reflective floor rows; h = shard_band_height in rt_device.h,
 * at most 8 bands per rank; rows / n_rows are ignored) and the
 * uint8 and linear-RGB tiles are gathered over RCCL to rank 0, whose out_srgb8 / out_rgb receive the
 * whole frame ([height][width][3], [3][height*width]); the other ranks' outputs are not written.
 * Replaces the reference's multiprocessing.Pool over samples (scene.py:80-116). */
#define SRT_RENDER_SHARDED 2
/* with SRT_RENDER_SHARDED: gather the linear RGB as well (every rank passes the same flags) */
#define SRT_RENDER_GATHER_RGB 4
/* with SRT_RENDER_SHARDED, instead of SRT_RENDER_GATHER_RGB: every rank writes its own rows of the
 * linear RGB straight into out_rgb, the whole frame's [3][height*width] buffer in host memory that
 * all ranks share (e.g. POSIX shared memory registered in every process with srt_host_register),
 * each over its own PCIe link; the RCCL gather to rank 0 then carries only the uint8 image.  The
 * frame's linear RGB is complete in host memory when every rank's frame has finished. */
#define SRT_RENDER_RGB_ROWS 8
/* SRT_RENDER_RGB_LOCAL (out_rgb NULL, without GATHER_RGB / RGB_ROWS): the linear RGB of the rows this
 * call renders is resolved into the context's frame buffer in HBM and stays there -- what
 * Scene.render keeps (the reference returns only the uint8 image, scene.py:118-140): the whole RGB
 * is computed and stored, nothing crosses PCIe or xGMI but the uint8 image. */
#define SRT_RENDER_RGB_LOCAL 16
/* SRT_RENDER_RGBX (not with SRT_RENDER_SHARDED): out_srgb8 receives 4-byte pixels [n_rows*width][4]
 * (R, G, B, 255) instead of 3-byte ones -- PIL's in-memory layout of an RGB image, so that
 * Scene.render's PIL image is built by a word copy per pixel */
#define SRT_RENDER_RGBX 32

#define SRT_MAX_DEPTHS 64
typedef struct srt_stats {
    int64_t rays_per_depth[SRT_MAX_DEPTHS]; /* rays entering each trace depth (all passes) */
    int64_t total_rays;                     /* sum of rays_per_depth */
    int64_t shadow_rays;
    int32_t n_depths;
    int32_t passes;
    double ms_wall;          /* host wall time inside the call */
    double ms_device;        /* first launch -> last kernel end, HIP events */
    double ms_trace_kernels; /* sum of trace-kernel durations, HIP events */
    double ms_primary_kernel;
    int64_t retries;         /* passes re-run after a queue overflow */
    int32_t kernel_path;     /* 0: per-depth wavefront kernels (ms_primary_kernel = k_primary),
                                1: frame kernel (ms_primary_kernel = k_frame, the whole pass),
                                2: fused paths (k_primary traces every depth; option fuse_primary) */
    int32_t chain_from;      /* > 0: depths >= chain_from traced in chain mode by one k_trace */
} srt_stats;

typedef struct srt_trace_args {
    int64_t n;
    const double* origin; /* [3][n] */
    const double* dir;    /* [3][n] */
    const int32_t* medium; /* [n] rows of media[] (ray.n), or NULL = all scene.n */
    int32_t depth;        /* Ray.depth (a batch scalar in the reference) */
    int32_t diffuse_reflections;
    uint64_t seed;
    double* out_rgb;      /* [3][n] colour of each ray */
} srt_trace_args;

typedef struct srt_ctx srt_ctx;

int srt_abi_version(void);
int srt_device_count(int* count);
int srt_create(int device, srt_ctx** out);
int srt_destroy(srt_ctx* ctx);
/* options (16 keys; unknown keys fail with SRT_ERR_ARG):
 *   strategy: "frame_kernel" (-1 auto = frame kernel for branching scenes, 0 per-depth wavefront
 *     kernels, 1 frame kernel), "fuse_primary" (-1 auto, 0/1: single-child paths traced whole in
 *     k_primary), "chain_rays" (the per-depth path traces whole chains from the first depth with fewer
 *     rays than this), "bvh" (0: mesh triangles intersected one by one), "collider_seq" (0: no
 *     straight-line collider-sequence kernel), "sync_lean" (1: synchronous frames run the lean kernel
 *     too, for measurement), "deterministic" (0: f64 atomics instead of fixed-point sums),
 *     "pipeline" (1: size every frame slot on each render, so the first pipelined frame allocates
 *     nothing);
 *   numpy's stream on the device: "mt_bands" (0: whole-frame stream on every rank), "mt_short" /
 *     "mt_pipe_split" (band-mode segment lengths, 0: tabulated 2^19-word segments), "mt_gen_nt"
 *     (generator workgroup, 0 auto / 256 / 320), "mt_jump_parts" (0 auto, 2..8);
 *   multi-GPU: "shard_bands" (most row bands per rank, 0 auto), "rehearse_shard" ((nranks << 8) |
 *     rank: act as that rank without a communicator), "rehearse_assemble" (n: rank 0's assembly of an
 *     n-rank frame rehearsed). */
int srt_set_option(srt_ctx* ctx, const char* key, int64_t value);
int srt_upload_scene(srt_ctx* ctx, const srt_scene_desc* scene);
int srt_render(srt_ctx* ctx, const srt_camera* cam, const srt_render_args* args, srt_stats* stats);
/* Queue the numpy-stream generation of the synchronous whole frame that srt_render will be called
 * for next with the same camera size and args (args->mt set, no rows, not SRT_RENDER_ASYNC /
 * SHARDED; otherwise it does nothing), so that it runs on the GPU while the caller lowers and uploads
 * its scene -- reference scene.py:71-83 draws the jitter before the samples are traced.  That
 * srt_render finds it queued (same stream state, frame shape and options) and does not launch it
 * again; any other render, option change, srt_trace/srt_shade or srt_mt19937_uniforms call drops it.
 * Does not advance args->mt (srt_render does).  Needs no scene. */
int srt_render_prefetch(srt_ctx* ctx, const srt_camera* cam, const srt_render_args* args);
int srt_render_finish(srt_ctx* ctx, srt_stats* stats);
/* the hipStream_t every call on ctx is ordered on (for stream/event interop, e.g. torch) */
int srt_stream(srt_ctx* ctx, void** stream);
int srt_trace(srt_ctx* ctx, const srt_trace_args* args, srt_stats* stats);
int srt_nearest(srt_ctx* ctx, const double* origin, const double* dir, int64_t n, double* t,
                int32_t* id, double* orient);
int srt_intersect_collider(srt_ctx* ctx, const srt_collider* collider, const double* origin,
                           const double* dir, int64_t n, double* out /* [2][n] */);
/* Material.get_color at the caller's hits: ray i is shaded as if its nearest hit were collider
 * collider[i] at distance t[i] with orientation orient[i] (the values srt_nearest returns;
 * -1 = no hit, nothing added), with no tie resolution; the reflected/refracted/diffuse rays
 * it spawns are traced by get_raycolor's rules.  out_rgb[3][n] as srt_trace.  A collider index
 * outside the scene fails with SRT_ERR_INDEX. */
int srt_shade(srt_ctx* ctx, const srt_trace_args* args, const int32_t* collider, const double* t,
              const double* orient, srt_stats* stats);
/* One level of Material.get_color (materials/material.py:42-44, as get_raycolor calls it,
 * ray.py:131-146) for a recursion the host drives through user Collider / Material subclasses
 * (sightpy/_hybrid.py): ray i is shaded at the caller's hit as srt_shade shades it, its own colour
 * (the terms the material adds before its children's) written to args->out_rgb, and the rays it
 * spawns handed back instead of traced.  Child k: origin / dir, the factor its colour is multiplied
 * by (weight; glossy.py:110, refractive.py:105-123, diffuse.py:85-124), the index of the ray it came
 * from (parent), its medium row, depth and diffuse-reflection count.  More children than `cap`:
 * SRT_ERR_MEMORY with `n` set to the count (call again with room for them). */
typedef struct srt_children {
    int64_t cap;                  /* in: room, in rays */
    int64_t n;                    /* out: children */
    double* origin;               /* [3][cap] */
    double* dir;                  /* [3][cap] */
    double* weight;               /* [3][cap] */
    int32_t* parent;              /* [cap] */
    int32_t* medium;              /* [cap] rows of the scene's media table */
    int32_t* depth;               /* [cap] */
    int32_t* diffuse_reflections; /* [cap] */
} srt_children;
int srt_shade_level(srt_ctx* ctx, const srt_trace_args* args, const int32_t* collider, const double* t,
                    const double* orient, srt_children* children, srt_stats* stats);
/* Collider.get_Normal (N [3][n]) and get_uv (uv [2][n], u then v) at points P [3][n] on the
 * collider; primitive_uv = 1 applies a Cuboid/SkyBox primitive's (4, 3) cross divide
 * (SRT_CF_UV_CROSS, cuboid.py:29-34), 0 returns the collider's own coordinates.  Either output may
 * be NULL.  Triangle uv is undefined in the reference (triangle.py:79-83): SRT_ERR_ARG. */
int srt_collider_surface(srt_ctx* ctx, const srt_collider* collider, const double* P, int64_t n,
                         double* N, double* uv, int primitive_uv);
/* image.get_color: the texel at uv [2][n] of the texture record `tex` over `texels`
 * (texel_bytes bytes, tex->offset into it), rgb [3][n] in [0, 1].  Indices outside the image
 * fail with SRT_ERR_INDEX as numpy indexing raises. */
int srt_texture_lookup(srt_ctx* ctx, const srt_texture* tex, const uint8_t* texels, int64_t texel_bytes,
                       const double* uv, int64_t n, double* rgb);
/* Material.get_Normal(hit) at points P [3][n] on the collider with orientations orient [n]: the
 * collider's normal, or -- normalmap not NULL, a record over `texels` (texel_bytes bytes) whose
 * table maps a byte b to b/256 -- the map's texel at the primitive's uv taken through the
 * collider's inverse_basis_matrix and normalised (Plane and Cuboid colliders: the reference's other
 * colliders have no inverse_basis_matrix), times the orientation; N [3][n].
 * Replaces sightpy/materials/material.py:18-36. */
int srt_material_normal(srt_ctx* ctx, const srt_collider* collider, const srt_texture* normalmap,
                        const uint8_t* texels, int64_t texel_bytes, const double* P, const double* orient,
                        int64_t n, double* N);
int srt_primary_rays(srt_ctx* ctx, const srt_camera* cam, const double* jitter /* [4][n] */,
                     double* origin /* [3][n] */, double* dir /* [3][n] */);
/* numpy's legacy global-RNG stream on the device: writes the n_out doubles that
 * `np.random.rand(n_out)` would return for the RandomState with MT19937 key[624] and position
 * pos (0..624, as in np.random.get_state()), then consumes n_skip more draws, and returns the
 * resulting state (key_out, *pos_out) for np.random.set_state.  `out` may be device or host memory.
 * Replaces the camera jitter draws of Camera.get_ray (sightpy/camera.py:56-64,
 * utils/random.py:6-9) and the extra sizing draw of Scene.render (sightpy/scene.py:81), so that
 * parity-mode renders need no host RNG and no host-to-device jitter copy. */
int srt_mt19937_uniforms(srt_ctx* ctx, const uint32_t* key, int32_t pos, int64_t n_out, int64_t n_skip,
                         double* out, uint32_t* key_out, int32_t* pos_out);

/* ---- multi-GPU: row-band shards + RCCL gather over xGMI -------------------------
 * One context per GPU.  Several processes (one per GPU): rank 0 makes an id with
 * srt_comm_unique_id, every rank passes it to srt_comm_init.  One process driving several GPUs:
 * srt_comm_init_all creates one context per device with one communicator (ncclCommInitAll), and
 * srt_render_group renders a frame on all of them (each its shard, SRT_RENDER_SHARDED) and gathers
 * it to the first. */
#define SRT_COMM_ID_BYTES 128
int srt_comm_unique_id(uint8_t* id /* [SRT_COMM_ID_BYTES] */);
int srt_comm_init(srt_ctx* ctx, int nranks, int rank, const uint8_t* id);
int srt_comm_init_all(int ndev, const int* devs, srt_ctx** ctxs /* [ndev], out */);
int srt_comm_rank(srt_ctx* ctx, int* nranks, int* rank);
/* frame of srt_render on every context of an srt_comm_init_all group; args of rank 0 (its outputs
 * receive the frame), stats of rank 0 plus total_rays / rays_per_depth / shadow_rays summed.
 * args->flags may hold SRT_RENDER_ASYNC (queue the frame on every context, gather posted, return at
 * once; outputs in pinned host memory from srt_host_alloc; `stats` not written; finish with
 * srt_render_group_finish), SRT_RENDER_RGB_ROWS (with ASYNC: every context writes its rows of the
 * linear RGB into out_rgb over its own PCIe link instead of the RCCL gather to rank 0) and
 * SRT_RENDER_RGB_LOCAL (out_rgb NULL: every context keeps its rows of the linear RGB in its HBM). */
int srt_render_group(srt_ctx** ctxs, int n, const srt_camera* cam, const srt_render_args* args, srt_stats* stats);
/* wait for the group's asynchronous frames: errors of every context, the last frame's stats summed as
 * srt_render_group returns them */
int srt_render_group_finish(srt_ctx** ctxs, int n, srt_stats* stats);
/* collectives over the communicator for callers' bookkeeping (host values, blocking):
 * op 0 = sum, 1 = max; n doubles */
int srt_comm_allreduce(srt_ctx* ctx, double* vals, int n, int op);
int srt_comm_barrier(srt_ctx* ctx);

/* Pinned host memory (outputs of asynchronous frames are copied into it by the frame's stream). */
int srt_host_alloc(srt_ctx* ctx, int64_t bytes, void** out);
int srt_host_free(srt_ctx* ctx, void* ptr);
/* Pin caller-owned host memory (e.g. a shared-memory frame for SRT_RENDER_RGB_ROWS) for the
 * context's device, and release it again (hipHostRegister / hipHostUnregister). */
int srt_host_register(srt_ctx* ctx, void* ptr, int64_t bytes);
int srt_host_unregister(srt_ctx* ctx, void* ptr);
/* Device memory helpers for callers that keep inputs resident in HBM (bench, multi-GPU). */
int srt_device_alloc(srt_ctx* ctx, int64_t bytes, void** out);
int srt_device_free(srt_ctx* ctx, void* ptr);
int srt_memcpy(srt_ctx* ctx, void* dst, const void* src, int64_t bytes);
int srt_synchronize(srt_ctx* ctx);
/* Diagnostic: waits for the context's frames and counts the nonzero words of the numpy-stream
 * generator's state that must be zero between generations (every frame slot's segment windows -- the
 * XOR targets of the jump parts, all but window 0, the key's copy --, the end-window accumulator and
 * its arrival counter): 0 on a healthy context. */
int srt_debug_mt_residue(srt_ctx* ctx, int64_t* nonzero_words);
/* Diagnostic: renders that found their generation queued by srt_render_prefetch (used, not
 * launched again) and prefetches queued, since the context was created. */
int srt_debug_prefetch_counts(srt_ctx* ctx, int64_t* used, int64_t* queued);
/* Diagnostic: lane utilisation of the lean fused kernel's depth loop (k_primary_lean: the headline's
 * pipelined frames, or synchronous ones with option "sync_lean"; ray.py:122-148's recursion traced in
 * one thread per sample; while counting, the kernel's counting instantiation runs).  mode 1 zeroes
 * and starts the counters for the frames rendered next; mode 0 waits for them and writes out[d][0]
 * = wave iterations that traced depth d, out[d][1] = live lanes in those iterations (d < n <=
 * SRT_MAX_DEPTHS), then stops counting.  active lane fraction(d) = out[d][1] / (64 out[d][0]). */
int srt_debug_lane_stats(srt_ctx* ctx, int mode, int64_t* out, int n);
/* Diagnostic: launches of the lean fused kernel (k_primary_lean: pipelined frames of single-child
 * scenes without a BVH, or any frame with option "sync_lean") since the context was created. */
int srt_debug_lean_launches(srt_ctx* ctx, int64_t* launches);
const char* srt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SIGHTPY_RT_H */
