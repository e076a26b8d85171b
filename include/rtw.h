/*
 * rtw.h -- C-ABI of the MI355X (gfx950) path tracer: the drop-in boundary for
 * the reference's per-pixel / per-sample ray_colour loop.
 *
 * Reference interfaces replaced (paths relative to N9199/ray_tracing_weekend):
 *   Camera::render(&self, world: &dyn Hittable, lights: &dyn Hittable)
 *       -> Vec<Vec<SampledColour>>            shared/src/camera.rs:295-297
 *   Camera::render_debug(...)                 shared/src/camera.rs:299-312
 *   (both through render_internal            shared/src/camera.rs:315-388)
 *   CameraBuilder::build(self) -> Camera      shared/src/camera.rs:114-218
 *   scenes::simple() (the input producer)     scenes/src/lib.rs:155-233
 *   SampledColour Display / PPM writer        shared/src/colour.rs:14-36,136-148;
 *                                             bin/src/main.rs:89-104
 *
 * Plain C types only (no torch, no HIP types): pointers, sizes, POD structs.
 * Every entry point returns 0 on success and a negative RTW_E* code on error
 * (the reference panics instead; this library never aborts the caller).
 * The rtw_ctx is reentrant across contexts; one context is single-threaded.
 * The GPU work runs on gfx950 only; there is no CPU fallback in this library.
 *
 * Output convention (mirrors render_internal's Vec<Vec<Colour>> before it is
 * wrapped in SampledColour): out[(j * W + i) * 3 + c] is the SUM of the
 * samples of pixel (i, j) -- not the mean -- and j = 0 is the BOTTOM row
 * (camera.rs:179-188: viewport_v = +v * h).  NaN samples are not scrubbed
 * (the live integrator never calls fix_nan, camera.rs:459-522).
 */
#ifndef RTW_H
#define RTW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 10

/* error codes */
#define RTW_OK 0
#define RTW_E_INVALID (-1)       /* bad argument / inconsistent scene */
#define RTW_E_DEVICE (-2)        /* HIP runtime error (message in rtw_last_error) */
#define RTW_E_NO_LIGHTS (-3)     /* a Lambertian bounce drew a light sample from an empty
                                    light list: hittable_list.rs:417 panics there */
#define RTW_E_NO_SCENE (-4)      /* render before a scene was set */
#define RTW_E_UNSUPPORTED (-5)   /* scene/feature outside this build's scope */
#define RTW_E_PANIC (-6)         /* the render reached a point where the reference panics:
                                    a non-finite plane UV (plane.rs:66-69) */

/* precision of the device arithmetic */
#define RTW_F32 0                /* speed mode: f32 + FMA + native sqrt/rcp/sin/cos */
#define RTW_F64 1                /* parity mode: f64, no FMA contraction, same op order
                                    as the reference (bit-comparable with the oracle) */

/* material kinds (shared/src/material.rs) */
#define RTW_LAMBERTIAN 0         /* material.rs:327-376 (SolidColour texture) */
#define RTW_METAL 1              /* material.rs:378-421 */
#define RTW_DIELECTRIC 2         /* material.rs:423-488 ("Dialectric") */
#define RTW_INVISIBLE 3          /* material.rs:321-325 */
#define RTW_DIFFUSE_LIGHT 4      /* material.rs:490-514: emits albedo, scatter() None */

/* texture kinds (shared/src/texture.rs) */
#define RTW_TEX_SOLID 0          /* SolidColour, texture.rs:15-22 */
#define RTW_TEX_CHECKER 1        /* CheckerTexture, texture.rs:24-55 */
#define RTW_TEX_NOISE 2          /* NoiseTexture over a Perlin table, texture.rs:57-102, perlin.rs */

/* light-list entry kinds (rtw_scene.light_kinds) */
#define RTW_LIGHT_SPHERE 0       /* Sphere::pdf_value / random, sphere.rs:101-127 */
#define RTW_LIGHT_QUAD 1         /* Quad::pdf_value / random, quadrilateral.rs:100-118 */
#define RTW_LIGHT_DEFAULT 2      /* a hittable without its own pdf (Plane, Transformed<Cuboid>):
                                    the trait defaults pdf_value = 0, random = (1, 0, 0),
                                    hittable.rs:175-181 */
/* rtw_scene.light_flags */
#define RTW_LIGHTS_BVH_LEAF 1    /* the light list is a BoundedVolumeHierarchy of <= 5 entries
                                    (a leaf): pdf_value = (sum / n * n) / n, bvh.rs:67-76,191-194 */

/* Stream arguments (hipStream_t as void*): NULL = the context's own stream
 * (non-blocking); RTW_STREAM_NULL = the device's null (legacy default)
 * stream, which orders with every blocking stream -- e.g. PyTorch's default
 * stream, whose handle is 0; anything else is a hipStream_t of that device. */
#define RTW_STREAM_NULL ((void *)1)

/* World acceleration used by the render kernel */
#define RTW_ACCEL_AUTO 0         /* pick per scene */
#define RTW_ACCEL_BRUTE 1        /* every ray tests every sphere, sphere list in LDS */
#define RTW_ACCEL_BVH 2          /* device BVH (closest-hit semantics unchanged) */

/* CameraBuilder (camera.rs:29-42).  has_* == 0 encodes Option::None. */
typedef struct rtw_camera_builder {
    int32_t has_aspect_ratio, has_image_width, has_image_height;
    double aspect_ratio;
    uint32_t image_width, image_height;
    uint32_t samples_per_pixel;  /* u16 in the reference */
    uint32_t max_depth;
    double background[3];
    double vfov;
    double lookfrom[3], lookat[3], vup[3];
    double defocus_angle, focus_dist;
} rtw_camera_builder;

/* The derived Camera fields the render loop reads (camera.rs:228-261). */
typedef struct rtw_camera {
    uint32_t image_width, image_height;
    uint32_t samples_per_pixel, max_depth;
    double background[3];
    double defocus_angle;
    double center[3], pixel00_loc[3], pixel_delta_u[3], pixel_delta_v[3];
    double defocus_disk_u[3], defocus_disk_v[3];
} rtw_camera;

/* Flattened world + lights, struct-of-arrays, caller-owned host memory.
 * world  = planes + spheres + quads + transformed cuboids (closest hit over
 *          all of them, bvh.rs:164-188), materials and their textures
 * lights = the light list in order: spheres, quads and entries with the
 *          Hittable defaults (HittableList::pdf_value / random,
 *          hittable_list.rs:408-419) */
typedef struct rtw_scene {
    uint32_t n_spheres;
    const double *spheres;        /* n_spheres x {cx, cy, cz, radius} */
    const uint32_t *sphere_mat;   /* n_spheres material ids */
    uint32_t n_planes;
    const double *planes;         /* n_planes x {px, py, pz, nx, ny, nz}, unit normal */
    const uint32_t *plane_mat;
    uint32_t n_materials;
    const uint32_t *mat_type;     /* RTW_LAMBERTIAN ... RTW_DIFFUSE_LIGHT */
    const double *mat_params;     /* n_materials x {albedo r, g, b, fuzz, ior} */
    uint32_t n_lights;
    const double *lights;         /* n_lights x {cx, cy, cz, radius}: the light list's spheres */
    /* Quads (quadrilateral.rs:21-56): Quad::new(Q, u, v, mat) */
    uint32_t n_quads;
    const double *quads;          /* n_quads x {Qx, Qy, Qz, ux, uy, uz, vx, vy, vz} */
    const uint32_t *quad_mat;
    uint32_t n_light_quads;
    const double *light_quads;    /* the light list's quads, n x 9 as quads */
    /* light-list order (HittableList insertion order, hittable_list.rs:408-419):
     * n_lights + n_light_quads + n_light_other RTW_LIGHT_* kinds, each taking
     * the next entry of its array (RTW_LIGHT_DEFAULT has no data);
     * NULL = all spheres, then all quads */
    const uint32_t *light_kinds;
    /* Transformed<Cuboid> (cuboid.rs:26-71, entities/transformations.rs:10-30):
     * Cuboid::new(p, q, mat) under the composed Transformation (rotation R,
     * translation T; Transformation::then order, geometry transformations.rs) */
    uint32_t n_boxes;
    const double *boxes;          /* n_boxes x {p xyz, q xyz, R[3][3] row-major, T xyz} = 18 */
    const uint32_t *box_mat;
    /* Textures (texture.rs, perlin.rs).  mat_tex == NULL: every material's
     * colour is the SolidColour albedo in mat_params.  Otherwise mat_tex[m] is
     * the texture of material m (Lambertian attenuation, DiffuseLight emission),
     * evaluated at the hit's (u, v, p) (sphere.rs:49-54, plane.rs:40-54,
     * quadrilateral.rs:58-63):
     *   RTW_TEX_SOLID    tex_params {r, g, b, -}
     *   RTW_TEX_CHECKER  tex_params {-, -, -, inv_scale = 1 / scale}, tex_refs {even, odd} texture ids
     *   RTW_TEX_NOISE    tex_params {-, -, -, scale}, tex_refs {Perlin table id, -} */
    const uint32_t *mat_tex;
    uint32_t n_textures;
    const uint32_t *tex_type;
    const double *tex_params;     /* n_textures x 4 */
    const uint32_t *tex_refs;     /* n_textures x 2 */
    uint32_t n_perlin;
    const double *perlin_vec;     /* n_perlin x 256 x 3: Perlin::rand_vec */
    const uint32_t *perlin_perm;  /* n_perlin x 3 x 256: perm_x, perm_y, perm_z (0..255) */
    /* light-list entries of kind RTW_LIGHT_DEFAULT (light_kinds == 2) */
    uint32_t n_light_other;
    uint32_t light_flags;         /* RTW_LIGHTS_BVH_LEAF */
} rtw_scene;

typedef struct rtw_stats {
    uint64_t samples;             /* W*H*spp of the rendered tiles */
    uint64_t segments;            /* world.hit calls */
    uint64_t lambertian;          /* Scatter-branch bounces (light pdf loop) */
    double kernel_ms;             /* device time of the last render (HIP events) */
    uint32_t accel;               /* RTW_ACCEL_* actually used */
    uint32_t chunk;               /* samples per work item */
    uint64_t node_visits;         /* BVH inner nodes entered (RTW_ACCEL_BVH) */
    uint64_t sphere_tests;        /* ray-sphere discriminant evaluations */
    uint32_t bvh_width;           /* child boxes tested per node visit (4, 2; 0 = no BVH) */
    uint32_t kernel;              /* render-kernel variant: 0 brute/L2, 1 brute/LDS, 2 BVH one
                                     loop, 3 BVH while-while, 4 BVH 4-wide, 5 BVH while-while
                                     with the tree in LDS */
    /* samples that reached a reference panic (the render then returns an
     * error): a non-finite plane UV (plane.rs:66-69) -> RTW_E_PANIC;
     * HittableList::random on an empty light list (hittable_list.rs:417)
     * -> RTW_E_NO_LIGHTS */
    uint64_t panic_plane_uv, panic_no_lights;
    /* light-pdf work (ABI 9): light tests = (bounce, light) pairs tested by the
     * light pdf -- every Lambertian bounce x every light for the linear list
     * loop (hittable_list.rs:408-412), the lights of the big list, the visited
     * grid cells or light-BVH leaves for the light grid / BVH (counted by the
     * kernel); grid_cells = light-grid cells those walks visited.  For the
     * light grid these are WALK-WORK counters, not properties of the samples:
     * the cooperative walks visit a piece boundary's cell twice, size pieces
     * by the wave's pending cells and count a re-walk again, so they depend
     * on how rays are grouped into waves (the image does not). */
    uint64_t light_tests, grid_cells;
} rtw_stats;

typedef struct rtw_ctx rtw_ctx;

/* ---- context ---------------------------------------------------------- */
int rtw_abi_version(void);
/* A context on one GPU (HIP device index `device`). */
rtw_ctx *rtw_create(int device, int precision);
/* A context over several GPUs of this node: SURVEY.md §8(b)(1)'s
 * rtw_create(device_mask, precision), the drop-in for render_internal's use of
 * every host core (camera.rs:340-353: one rayon task per pixel over the
 * global pool) -- here one rank per GPU, all in the calling process.
 * devices[k] is rank k's HIP device; rank k renders the 8x8 tiles
 * T = k (mod n_devices) (rtw_tiles_for_rank), and ONE RCCL gather
 * (ncclGather, rccl.h:745-746, a single-process clique from ncclCommInitAll)
 * brings the ranks' packed tiles to rank 0's device, which un-interleaves them
 * (rtw_assemble_tiles).  Every knob (rtw_set_tuning / rtw_set_chunk /
 * rtw_set_accel) and the scene (rtw_set_scene, staged once) apply to all
 * ranks; rtw_render and rtw_render_image_device render on all of them, and
 * the image is bit-identical to a one-GPU render of the same seed.
 * RTW_E_INVALID: NULL / empty list, a negative, repeated or not visible
 * device (checked before any HIP call for the first two); RTW_E_DEVICE: a HIP
 * or RCCL failure (RCCL is loaded at run time: librccl.so.1). */
int rtw_create_devices(const int *devices, uint32_t n_devices, int precision, rtw_ctx **out);
/* The same over the devices whose bits are set (bit k = HIP device k, in
 * increasing order); NULL on error (an empty mask included). */
rtw_ctx *rtw_create_mask(uint64_t device_mask, int precision);
/* rtw_create_mask with its error code (ABI 9): RTW_E_INVALID for an empty mask
 * or a device that is not visible (compare rtw_visible_devices), RTW_E_DEVICE
 * for a HIP / RCCL failure -- which a caller must not answer by dropping GPUs. */
int rtw_create_mask_ex(uint64_t device_mask, int precision, rtw_ctx **out);
/* HIP devices visible to this process (RTW_E_DEVICE if HIP fails). */
int rtw_visible_devices(void);
/* TEST MODE (ABI 9): a multi-device context of n_ranks ranks that all live on
 * one device, with every product code path of rtw_create_devices -- per-rank
 * contexts, streams, work buffers and scene copies, rank 0 rendering into its
 * gather slot, the equal-size slots, the assembly, the summed stats -- except
 * the transport: the gather is n_ranks - 1 device copies on rank 0's stream,
 * each after its rank's render, instead of ncclGather.  It lets a one-GPU box
 * execute and check the n-rank path; RCCL stays the only product transport. */
int rtw_create_virtual(int device, uint32_t n_ranks, int precision, rtw_ctx **out);
/* Ranks of a context (1 for rtw_create), and rank k's per-device context
 * (k = 0: ctx itself) for rtw_get_stats / rtw_get_timings / rtw_last_kernel
 * of that rank; owned by ctx (do not destroy).  rtw_device_of: its HIP device. */
uint32_t rtw_device_count(const rtw_ctx *ctx);
rtw_ctx *rtw_device_ctx(rtw_ctx *ctx, uint32_t k);
int rtw_device_of(const rtw_ctx *ctx);
void rtw_destroy(rtw_ctx *ctx);
const char *rtw_last_error(const rtw_ctx *ctx);
int rtw_precision(const rtw_ctx *ctx);
/* knobs: samples per work item (0 = auto), acceleration (RTW_ACCEL_*) */
int rtw_set_chunk(rtw_ctx *ctx, uint32_t chunk);
int rtw_set_accel(rtw_ctx *ctx, int accel);
/* scheduling knobs (benchmarking): "chunk" (samples per item, 0 = auto),
 * "auto_chunk", "group" (chunks per wave task, 0 = auto: 4..32), "target_tasks"
 * (auto group: about this many tasks; 0 = 2^17),
 * "persist" (workgroups of persistent waves that take tasks from a global counter;
 * 1 = as many as are resident at once, the default; 0 = one task per wave),
 * "lds" (1 = stage the sphere list in LDS when it fits, 0 = read it from HBM),
 * "robust" (f32 ray-sphere tests in closest-approach form: 1 on, 0 off,
 * 2 = by the scene's distance-to-radius ratio, the default),
 * "item_order" (wave item pool: 1 = sample-major, the default; 0 = pixel-major),
 * "lpt" (longest tiles first: the segments of each pixel's first 2 samples,
 * summed per tile, order the tasks, cached until the scene, camera or rank split
 * changes; 1 = for worlds held in LDS or of at most 4 MiB (an XCD's L2), the
 * default, 2 = for every world, 0 = tiles in index order),
 * "lpt_inline" (1 = the default: the first render of a scene / camera / split
 * runs in tile index order and counts those segments itself, the next render
 * reads them back (waiting for it once) and takes the ordered tasks; 0 = a
 * blocking 2-spp pilot render before the first render),
 * "lpt_pilot_spp" (samples per pixel counted, default 2), "lpt_pilot_depth" (the
 * separate pilot's max depth, 0 = the camera's),
 * "lpt_min_spp" (renders of fewer samples per pixel keep the index order, default 32),
 * "bvh_leaf" (spheres per BVH leaf, 1..15; 0 = auto, the default: 4, 8 for
 * scenes of >= 100k spheres, 2 for f64 contexts on scenes of 4096..100k; takes effect at the
 * next rtw_set_scene), "light_bvh_min" (light lists this long or longer take the light grid
 * or light BVH in the BVH kernels, default 64), "light_grid" (light-grid resolution in
 * 1/16 cells per light, default 8; 0 = the light BVH instead; next rtw_set_scene),
 * "max_group" (longest-first task list: at most this many chunks per task, default 32),
 * "grid_piece" (f32 light-grid walks: cells per piece of the wave's cooperative walk,
 * default by grid size: its widest side / 14, 4..16; 0 = every lane walks its own ray),
 * "light_leaf" (light spheres per light-BVH leaf, 1..15; 0 = 4), "partial_max" (bytes of chunk sums an auto chunk may use, default 128 GiB, at most half the device's memory; an auto chunk doubles if the allocation fails),
 * "bvh_kind" (3 = binary while-while on the tree staged in LDS, the
 * default, 1 = binary while-while from L1/L2, 2 = 4-wide octant BVH, 0 =
 * binary single loop), "bvh_lds_max" (LDS bytes per workgroup bvh_kind 3 may
 * use; 0 = by precision: 36 KiB f32, 52 KiB f64), "bvh_ww" (legacy: 1 -> bvh_kind 1, 0 -> 0), "auto_accel" */
int rtw_set_tuning(rtw_ctx *ctx, const char *key, int64_t value);

/* ---- CameraBuilder::build (camera.rs:114-218) ------------------------- */
int rtw_camera_build(const rtw_camera_builder *builder, rtw_camera *out);
/* CameraBuilder::new() defaults (camera.rs:45-60) */
void rtw_camera_builder_default(rtw_camera_builder *out);

/* ---- scene ------------------------------------------------------------ */
/* Validate, convert to the device layout and upload (copied; the caller may
 * free its arrays afterwards). */
int rtw_set_scene(rtw_ctx *ctx, const rtw_scene *scene);

/* ---- Camera::render (camera.rs:295-297) ------------------------------- */
/* Synchronous drop-in: uploads `scene` (if non-NULL), renders every pixel and
 * writes H*W*3 doubles (sums, j = 0 bottom row) to host `out_sum`.  On a
 * multi-device context every GPU renders its share (rtw_create_devices);
 * `stats` then sums the ranks' counters (kernel_ms: the slowest rank). */
int rtw_render(rtw_ctx *ctx, const rtw_camera *cam, const rtw_scene *scene,
               uint64_t seed, double *out_sum, rtw_stats *stats);

/* The whole image into device memory of the context's first device: d_image
 * holds H*W*3 elements of the context's precision (sums, j = 0 bottom row).
 * Asynchronous on `stream` (a hipStream_t of that device; NULL = the
 * context's own): rank 0 renders on it, the other ranks on their own
 * streams; the RCCL gather and the assembly are ordered on `stream` after
 * every rank's render, so work queued on `stream` afterwards sees the image. */
int rtw_render_image_device(rtw_ctx *ctx, const rtw_camera *cam, uint64_t seed, void *d_image,
                            size_t image_bytes, void *stream);

/* Device-resident form for benchmarking and multi-GPU sharding.
 * The image is cut into 8x8 tiles T = ty * tiles_x + tx (tiles_x = ceil(W/8),
 * row j = 0 at the bottom); rank `rank` of `nranks` renders the tiles
 * T = rank, rank + nranks, ... (a fine interleave: every rank samples the
 * whole image, so the ranks' costs match).  d_out receives them packed: a
 * device buffer of rtw_tiles_for_rank(W, H, rank, nranks) * 64 * 3 elements of
 * the context's precision (float or double), the rank's k-th tile at
 * d_out[(k * 64 + ly * 8 + lx) * 3 + c] (pixels outside the image: 0).
 * d_out may be NULL when the rank has no tiles.  Asynchronous on `stream`
 * (a hipStream_t; NULL = the context's own stream).  No host synchronisation
 * inside, except once per (scene, camera, rank split) when tuning "lpt" is on
 * and spp >= "lpt_min_spp": the second render of the key waits for the first,
 * whose tile costs order its tasks, and reads them back (then cached; with
 * "lpt_inline" 0 the first render runs and reads back a 2-spp pilot instead).
 * On a multi-device context it renders on the first device only (each rank's
 * context: rtw_device_ctx). */
int rtw_render_device(rtw_ctx *ctx, const rtw_camera *cam, uint64_t seed,
                      uint32_t rank, uint32_t nranks, void *d_out, size_t out_bytes,
                      void *stream);
uint32_t rtw_tile_size(void);                        /* tile edge in pixels (8) */
uint32_t rtw_tiles_for_rank(uint32_t image_width, uint32_t image_height, uint32_t rank,
                            uint32_t nranks);
/* The gathered packed tiles of all ranks -> the image [H][W][3] (sums, j = 0
 * bottom row), on the device: d_ranks holds nranks rank buffers, each
 * rank_stride_bytes apart (>= rank 0's packed size; equal-size buffers as an
 * RCCL gather delivers them).  Follows the context's split for (W, H,
 * nranks) (rtw_set_split; the round robin without one).  Asynchronous on
 * `stream`. */
int rtw_assemble_tiles(rtw_ctx *ctx, const void *d_ranks, size_t rank_stride_bytes, uint32_t nranks,
                       uint32_t image_width, uint32_t image_height, void *d_image, void *stream);

/* ---- cost-balanced rank split (ABI 10) ---------------------------------
 * The round robin (T mod nranks) gives every rank the same NUMBER of tiles
 * but not the same work: a rank's share of glass and mirror tiles varies.
 * The reference balances dynamically -- one rayon task per pixel,
 * work-stealing over every host core (camera.rs:340-353); across GPUs the
 * tiles are dealt once by their costs instead.  A split keeps the round
 * robin's per-rank tile counts (rtw_tiles_for_rank), so packed buffers and the
 * gather stay the same size, and the image does not depend on the split. */
#define RTW_MAX_RANKS 256
/* Deal the tiles of a W x H image (n_tiles = ceil(W/8) * ceil(H/8) entries of
 * tile_cost, any cost unit) to nranks ranks: costliest first (ties: lower
 * tile index), each to the rank of least dealt cost (ties: lower rank) that
 * still has room below its round-robin count.  Writes tile_rank[n_tiles].
 * Deterministic: every process dealing the same costs gets the same split. */
int rtw_split_deal(const uint32_t *tile_cost, uint32_t image_width, uint32_t image_height,
                   uint32_t nranks, uint32_t *tile_rank);
/* Renders (rtw_render_device with this nranks, and the multi-device paths)
 * and rtw_assemble_tiles of a W x H image over nranks ranks follow this split
 * from now on: rank r renders the tiles T with tile_rank[T] == r, packed in
 * increasing T.  tile_rank == NULL restores the round robin.  tile_cost
 * (optional, n_tiles) orders each rank's tasks longest first without a
 * counting render.  RTW_E_INVALID unless every rank r gets exactly
 * rtw_tiles_for_rank(W, H, r, nranks) tiles.  A multi-device context sets it
 * on every rank. */
int rtw_set_split(rtw_ctx *ctx, uint32_t image_width, uint32_t image_height, uint32_t nranks,
                  const uint32_t *tile_rank, const uint32_t *tile_cost);
/* The split renders of (W, H, nranks) follow: 0 = the round robin (tile_rank
 * untouched), 1 = set by rtw_set_split, 2 = dealt by the context itself
 * (tuning "balance"); for 1 and 2 tile_rank (may be NULL) receives it. */
int rtw_get_split(rtw_ctx *ctx, uint32_t image_width, uint32_t image_height, uint32_t nranks,
                  uint32_t *tile_rank);
/* The tile costs the context counted in its first render of (cam, rank,
 * nranks) under its current split (tuning "lpt", spp >= "lpt_min_spp": BVH
 * node visits + sphere tests + 12 per segment of each pixel's first
 * "lpt_pilot_spp" samples, summed per tile), written to tile_cost[T] for the
 * rank's tiles T (other entries untouched: the ranks' arrays summed give the
 * whole image's).  Waits for that render.  RTW_E_INVALID when there is no
 * such count.  With tuning "balance" (1, the default) a multi-device
 * context deals its split from these costs by itself: the first
 * rtw_render_image_device of a camera counts, the second deals and renders
 * balanced (re-dealt when the scene or camera changes). */
int rtw_tile_costs(rtw_ctx *ctx, const rtw_camera *cam, uint32_t rank, uint32_t nranks, uint32_t *tile_cost);
/* Counters of the last render (waits for it to finish).  Returns
 * RTW_E_NO_LIGHTS / RTW_E_PANIC (stats still filled) when a sample reached a
 * reference panic, RTW_E_INVALID before the first render.  A multi-device
 * context sums the ranks that took part in its last render (all of them after
 * rtw_render / rtw_render_image_device; rank 0 after rtw_render_device). */
int rtw_get_stats(rtw_ctx *ctx, rtw_stats *stats);
/* Rank k's own counters of its last render (k = 0 included: rtw_get_stats on
 * rtw_device_ctx(ctx, 0) == ctx sums the ranks), ABI 9. */
int rtw_get_stats_rank(rtw_ctx *ctx, uint32_t k, rtw_stats *stats);
/* Device times (HIP events) of the last min(max, 64) renders, oldest first:
 * render_ms = the render kernel alone, total_ms = render + chunk reduction.
 * Waits for them; returns how many were written. */
int rtw_get_timings(rtw_ctx *ctx, float *render_ms, float *total_ms, int max);
/* The render-kernel variant of the last render: (kernel << 8) | options, with
 * kernel as rtw_stats.kernel and options the compile-time option bits of the
 * launched instantiation (1 closest-approach f32 tests, 2 light BVH / grid,
 * 4 textures, 8 quads / cuboids / mixed light lists, 16 f64 hit points);
 * 0 when no render kernel has run.  Measurement tooling uses it to name the
 * exact machine code that ran (render_kernel<R, kernel, options>). */
int rtw_last_kernel(const rtw_ctx *ctx);

/* ---- scenes::simple (scenes/src/lib.rs:155-233) ----------------------- */
/* The library owns the arrays; view them through rtw_world_scene(). grid_n =
 * 11 is the reference scene; larger n gives the synthetic C3/C5 fields. */
typedef struct rtw_world rtw_world;
rtw_world *rtw_scene_simple(uint64_t seed, int grid_n);
const rtw_scene *rtw_world_scene(const rtw_world *w);
/* the camera builder scenes::simple returns (lib.rs:219-226) + main.rs's vfov */
void rtw_world_camera_builder(const rtw_world *w, rtw_camera_builder *out);
void rtw_world_free(rtw_world *w);
/* a reference scene by its bin/src/main.rs name (scenes/src/lib.rs):
 * "simple" (seeded, grid 11), "cornell_box", "debug", "checkered_spheres",
 * "perlin_spheres", "plane", "simple_light", "simple_transform"; the seed
 * drives simple's generator and the Perlin tables.  NULL for other names. */
rtw_world *rtw_scene_named(const char *name, uint64_t seed);

/* ---- Perlin::new (perlin.rs:46-58) ------------------------------------- */
/* The reference fills the tables from thread_rng; here from the build's
 * seeded xoshiro256++: rand_vec = 256 UnitSphere samples, then perm_x, perm_y,
 * perm_z, each the identity shuffled by j = Uniform::new(i, 256) for i < 255.
 * rand_vec: 768 doubles; perm: 768 values (perm_x, perm_y, perm_z). */
int rtw_perlin_generate(uint64_t seed, double *rand_vec, uint32_t *perm);

/* ---- SampledColour / PPM (colour.rs:14-36; main.rs:89-104) ------------ */
/* sums -> 8-bit RGB, rows flipped so that row 0 is the TOP row:
 * (256 * clamp(sqrt(sum / spp), 0, 1)) as u8, saturating, NaN -> 0. */
int rtw_encode_rgb8(const double *sums, uint32_t width, uint32_t height, uint32_t spp,
                    uint8_t *out_rgb);
/* Writes the reference's P3 "image.ppm" text; returns bytes written or < 0. */
int rtw_write_ppm(const char *path, const double *sums, uint32_t width, uint32_t height,
                  uint32_t spp);
/* The same for the f32 sums of a speed-mode render (each sum widened to f64
 * exactly, then encoded as above). */
int rtw_encode_rgb8_f32(const float *sums, uint32_t width, uint32_t height, uint32_t spp,
                        uint8_t *out_rgb);
int rtw_write_ppm_f32(const char *path, const float *sums, uint32_t width, uint32_t height,
                      uint32_t spp);

#ifdef __cplusplus
}
#endif
#endif /* RTW_H */
