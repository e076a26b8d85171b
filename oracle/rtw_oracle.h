/*
 * rtw_oracle.h -- CPU restatement of the reference's per-pixel/per-sample
 * ray_colour loop (N9199/ray_tracing_weekend), f64, plain C.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ray_tracing_weekend_amd/)
 * links or calls this.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and there only as the checker / the timed
 * CPU baseline ("kind": "port").
 *
 * Parity status: the Rust reference cannot be built or run here (no cargo /
 * rustc) and its own tests pin no numeric output
 * (integration-tests/src/lib.rs:7-112 has no asserts).  The restatement is
 * pinned by hand-derived known-answer tests taken from the cited formulas
 * (tests/test_oracle_kat.py) -- "parity unpinned" against the reference
 * binary itself.
 *
 * Conventions shared with the GPU path (the C-ABI in include/rtw.h):
 *   out[(j*W + i)*3 + c]: per-pixel SUM over samples (not a mean), j = 0 is
 *   the bottom row (camera.rs:179-188, 381-387).
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material type codes (material.rs:321-488). */
enum { RTWO_LAMBERTIAN = 0, RTWO_METAL = 1, RTWO_DIELECTRIC = 2, RTWO_INVISIBLE = 3, RTWO_DIFFUSE_LIGHT = 4 };

/* World-acceleration choice for the closest-hit query.  All three return the
 * same closest hit (bvh.rs:164-188 keeps "min t over every primitive").
 *   0 = brute force over the flat primitive list (the checker)
 *   1 = restatement of the reference BVH (bvh.rs:106-188, hittable_list.rs:
 *       296-406) including its per-visit recursive node-AABB recomputation
 *       (bvh.rs:147-152) -- the faithful CPU baseline
 *   2 = the same BVH with node AABBs cached once (a kinder CPU baseline) */
enum { RTWO_ACCEL_BRUTE = 0, RTWO_ACCEL_BVH_REF = 1, RTWO_ACCEL_BVH_CACHED = 2 };

typedef struct rtwo_camera {
    /* Derived fields of Camera (camera.rs:228-261) the render loop reads. */
    uint32_t image_width, image_height;
    uint32_t samples_per_pixel, max_depth;
    double background[3];
    double defocus_angle;
    double center[3], pixel00_loc[3], pixel_delta_u[3], pixel_delta_v[3];
    double defocus_disk_u[3], defocus_disk_v[3];
} rtwo_camera;

typedef struct rtwo_camera_builder {
    /* CameraBuilder (camera.rs:29-42).  has_* = 0 means Option::None. */
    int has_aspect_ratio, has_image_width, has_image_height;
    double aspect_ratio;
    uint32_t image_width, image_height;
    uint32_t samples_per_pixel, max_depth;
    double background[3];
    double vfov;
    double lookfrom[3], lookat[3], vup[3];
    double defocus_angle, focus_dist;
} rtwo_camera_builder;

typedef struct rtwo_scene {
    uint32_t n_spheres;
    const double *spheres;      /* n x {cx, cy, cz, r} */
    const uint32_t *sphere_mat; /* n material ids */
    uint32_t n_planes;
    const double *planes;       /* n x {px, py, pz, nx, ny, nz} (normal already normalized, plane.rs:175) */
    const uint32_t *plane_mat;
    uint32_t n_materials;
    const uint32_t *mat_type;   /* n */
    const double *mat_params;   /* n x {albedo r, g, b, fuzz, ior} */
    uint32_t n_lights;
    const double *lights;       /* n x {cx, cy, cz, r}  (the light list's Spheres) */
    /* Quads (quadrilateral.rs): world quads and the light list's quads */
    uint32_t n_quads;
    const double *quads;        /* n x {Qx, Qy, Qz, ux, uy, uz, vx, vy, vz} */
    const uint32_t *quad_mat;
    uint32_t n_light_quads;
    const double *light_quads;  /* n x 9, as quads */
    /* light-list order: n_lights + n_light_quads kinds (0 sphere, 1 quad),
     * each taking the next entry of its array; NULL = spheres then quads */
    const uint32_t *light_kinds;
    /* Transformed<Cuboid> (cuboid.rs:26-59, entities/transformations.rs,
     * geometry/src/transformations.rs): Cuboid::new(p, q, mat) under the
     * composed Transformation {rotation R (row-major), translation T} */
    uint32_t n_boxes;
    const double *boxes;        /* n x {p xyz, q xyz, R[3][3], T xyz} = 18 */
    const uint32_t *box_mat;
    /* Textures (texture.rs, perlin.rs).  mat_tex NULL: every material's colour
     * is its SolidColour albedo from mat_params.  Otherwise mat_tex[m] is the
     * texture of material m (Lambertian attenuation, DiffuseLight emission):
     *   RTWO_TEX_SOLID   params {r, g, b, -}
     *   RTWO_TEX_CHECKER params {-, -, -, inv_scale}, refs {even, odd} texture ids
     *   RTWO_TEX_NOISE   params {-, -, -, scale},     refs {perlin table id, -} */
    const uint32_t *mat_tex;
    uint32_t n_textures;
    const uint32_t *tex_type;
    const double *tex_params;   /* n x 4 */
    const uint32_t *tex_refs;   /* n x 2 */
    uint32_t n_perlin;
    const double *perlin_vec;   /* n x 256 x 3: Perlin::rand_vec */
    const uint32_t *perlin_perm;/* n x 3 x 256: perm_x, perm_y, perm_z */
    /* light-list entries with the Hittable trait defaults (hittable.rs:175-181:
     * pdf_value 0, random (1, 0, 0)), e.g. a Transformed<Cuboid>: light_kinds 2 */
    uint32_t n_light_other;
    uint32_t light_flags;       /* RTWO_LIGHTS_BVH_LEAF */
} rtwo_scene;

enum { RTWO_TEX_SOLID = 0, RTWO_TEX_CHECKER = 1, RTWO_TEX_NOISE = 2 };
/* the light list is a BoundedVolumeHierarchy leaf (<= 5 entries): pdf_value =
 * (HittableList::pdf_value * len) / len (bvh.rs:67-76, 191-194) */
enum { RTWO_LIGHTS_BVH_LEAF = 1 };

typedef struct rtwo_stats {
    uint64_t samples;
    uint64_t segments;          /* world.hit calls (one per bounce) */
    uint64_t lambertian;        /* Scatter-branch bounces (light-list pdf loop) */
    uint64_t nan_samples;
    /* samples on which the reference panics: a non-finite plane UV
     * (plane.rs:66-69), or HittableList::random on an empty light list
     * (hittable_list.rs:414-419) */
    uint64_t panic_plane_uv, panic_no_lights;
} rtwo_stats;

/* Quad::hit (quadrilateral.rs:79-100) with Quad::new's derived fields
 * (:37-56); out = {t, alpha, beta, normal xyz (front-face adjusted)}.
 * Returns 1 on a hit. */
int rtwo_quad_hit(const double quad[9], const double o[3], const double d[3],
                  double tmin, double tmax, double out[6]);
/* Quad::pdf_value / Quad::random (quadrilateral.rs:102-118) */
double rtwo_quad_pdf_value(const double quad[9], const double o[3], const double d[3]);
void rtwo_quad_random(const double quad[9], const double o[3], uint64_t st[4], double out[3]);
/* Quad::new's AABBox::from_points (aabox.rs:199-211, padded per enclose) */
void rtwo_quad_aabb(const double quad[9], double box[6]);

/* Transformed<Cuboid>::hit for one box record (18 doubles, see rtwo_scene):
 * out = {t, world point xyz, normal xyz (object space, front-face adjusted
 * against the object-space ray -- the reference does not transform it back),
 * front}.  Returns 1 on a hit. */
int rtwo_box_hit(const double box[18], const double o[3], const double d[3],
                 double tmin, double tmax, double out[8]);
/* its world-space AABB (Transformed::get_aabbox) */
void rtwo_box_aabb(const double box[18], double aabb_out[6]);

/* world.hit(&r, EPSILON..=INFINITY) for one ray with the given accel:
 * object id (planes, quads, boxes, spheres) or -1; out = {t, p, normal, front} */
int rtwo_world_hit(const rtwo_scene *sc, int accel, const double o[3], const double d[3], double out[8]);

/* CameraBuilder::build, camera.rs:114-218. Returns 0. */
int rtwo_camera_build(const rtwo_camera_builder *b, rtwo_camera *out);

/* Render a window of the image.  Rows j in [row_begin, row_end) stepping by
 * row_step, columns [col_begin, col_end).  Untouched pixels are left as is.
 * chunk: samples are summed in chunks of `chunk` (chunk >= spp = the
 * reference's single fold, camera.rs:323-335); the per-pixel sum is
 * ((0 + chunk_0) + chunk_1) + ..., each chunk ((0 + s_a) + s_a+1) + ...
 * Returns 0 on success, -1 on invalid input, -2 when a sample hit a point
 * where the reference panics (stats->panic_*: a non-finite plane UV,
 * plane.rs:66-69; HittableList::random on an empty light list,
 * hittable_list.rs:417) -- the image is still written. */
int rtwo_render(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed,
                uint32_t chunk, int accel, int nthreads,
                uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                uint32_t col_begin, uint32_t col_end,
                double *out, rtwo_stats *stats);

/* One sample, exposed for tests (returns the colour, fills segment counts). */
void rtwo_trace_sample(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed,
                       uint32_t i, uint32_t j, uint32_t s, double out_rgb[3],
                       rtwo_stats *stats);
/* rtwo_trace_sample with an accel and (debugging) the path: per segment
 * {origin xyz, direction xyz, hit object id or -1, t}; returns segments */
uint32_t rtwo_trace_path(const rtwo_camera *cam, const rtwo_scene *sc, uint64_t seed, uint32_t i, uint32_t j,
                         uint32_t s, int accel, double out_rgb[3], rtwo_stats *stats, double *path,
                         uint32_t path_cap);

/* scenes::simple (scenes/src/lib.rs:155-233) driven by the build's seeded
 * RNG; grid a,b in [-n, n) (the reference uses n = 11).  Writes at most
 * max_* entries; returns 0, or -1 if a capacity is too small.  Counts are
 * returned through the *_count pointers.  Material ids: 0 = ground plane
 * material, then one per sphere in insertion order. */
int rtwo_scene_simple(uint64_t seed, int n,
                      uint32_t max_spheres, double *spheres, uint32_t *sphere_mat,
                      uint32_t *n_spheres,
                      double *planes, uint32_t *plane_mat, uint32_t *n_planes,
                      uint32_t max_mats, uint32_t *mat_type, double *mat_params,
                      uint32_t *n_mats,
                      uint32_t max_lights, double *lights, uint32_t *n_lights);

/* ---- primitive-level entry points for the known-answer tests ---- */
void rtwo_rng_seed(uint64_t seed, uint64_t pixel_index, uint64_t sample_index, uint64_t st[4]);
uint64_t rtwo_rng_next(uint64_t st[4]);
double rtwo_rand_std(uint64_t st[4]);
double rtwo_rand_open01(uint64_t st[4]);
double rtwo_rand_uniform_incl(uint64_t st[4], double low, double high);
uint32_t rtwo_rand_index(uint64_t st[4], uint32_t n);
void rtwo_sincos_2pi(double r, double *s, double *c);
/* Sphere::hit (sphere.rs:61-99): returns 1 and t/normal/front on hit. */
int rtwo_sphere_hit(const double sph[4], const double o[3], const double d[3],
                    double tmin, double tmax, double *t, double normal[3], int *front);
/* Plane::hit (plane.rs:61-76). plane = {px,py,pz,nx,ny,nz}. */
int rtwo_plane_hit(const double pl[6], const double o[3], const double d[3],
                   double tmin, double tmax, double *t, double normal[3], int *front);
/* AABBox slab test (hittable.rs:291-339). box = {minx,miny,minz,maxx,maxy,maxz}. */
int rtwo_aabb_hit(const double box[6], const double o[3], const double d[3],
                  double tmin, double tmax);
double rtwo_sphere_pdf_value(const double sph[4], const double o[3], const double d[3]);
void rtwo_onb(const double n[3], double u[3], double v[3], double w[3]);
double rtwo_reflectance(double cosine, double ref_idx);
void rtwo_reflect(const double v[3], const double n[3], double out[3]);
void rtwo_refract(const double v[3], const double n[3], double eta, double out[3]);
void rtwo_unit_sphere(uint64_t st[4], double out[3]);
void rtwo_cosine_hemisphere(uint64_t st[4], double out[3]);
void rtwo_sphere_random(const double sph[4], const double o[3], uint64_t st[4], double out[3]);
/* Number of BVH nodes/leaves built for a scene (tests of the BVH restatement). */
int rtwo_bvh_stats(const rtwo_scene *sc, uint32_t *nodes, uint32_t *leaves, uint32_t *depth);

/* ---- texture KATs ---- */
/* sin(x) as the build evaluates it on CPU and GPU (fdlibm: medium-size
 * Cody-Waite reduction by pi/2 + __kernel_sin/__kernel_cos) */
double rtwo_sin(double x);
/* Sphere::get_sphere_uv (sphere.rs:49-54) of an outward unit normal */
void rtwo_sphere_uv(const double n[3], double uv[2]);
/* Plane::get_plane_uv (plane.rs:40-54); plane = {p, unit normal} */
void rtwo_plane_uv(const double pl[6], const double p[3], double uv[2]);
/* Perlin::noise / Perlin::turb (perlin.rs:59-94) over one table */
double rtwo_perlin_noise(const double *vec, const uint32_t *perm, const double p[3]);
double rtwo_perlin_turb(const double *vec, const uint32_t *perm, const double p[3], int depth);
/* Texture::get_colour (texture.rs) of texture `tid` of the scene */
void rtwo_texture_colour(const rtwo_scene *sc, uint32_t tid, double u, double v, const double p[3],
                         double out[3]);

#ifdef __cplusplus
}
#endif
#endif
