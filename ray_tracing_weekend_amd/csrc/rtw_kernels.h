// rtw_kernels.h -- host-visible description of the device scene layout and the
// launch entry points of the gfx950 render kernels (render_f32.hip /
// render_f64.hip).  Included by the C-ABI (capi.cpp) and by the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace rtw {

constexpr uint32_t kTile = 8;          // 8 x 8 pixel tile = one wavefront of 64 lanes
constexpr uint32_t kWavesPerBlock = 4; // 256-thread workgroups, one tile item per wave
constexpr uint32_t kBlock = 64 * kWavesPerBlock;
// Wide workgroups (round 6): the f64 sphere + plane kernel with the tree in
// LDS runs 16 waves per workgroup -- the 4 waves per SIMD of one CU, so ONE
// LDS copy of the scene per CU instead of four -- and spends the freed LDS on
// the f64 leaf spheres, which the 4-wave layout had to read from L1 / L2 in
// the leaf loop (a dependent global load per candidate).  0: 4 waves.
#ifndef RTW_WIDE_F64
#define RTW_WIDE_F64 1
#endif
// RTW_WIDE_SPH64: the wide kernel's LDS also holds the f64 spheres in id order
// (the own-sphere test that starts each traversal)
#ifndef RTW_WIDE_SPH64
#define RTW_WIDE_SPH64 1
#endif
constexpr uint32_t kWavesWide = 16;
// waves per workgroup of a render kernel: `wide` = f64, tree in LDS, no
// light BVH / grid, no quads / cuboids / textures (the Book-1 family)
__host__ __device__ constexpr uint32_t block_waves(bool wide) {
    return (RTW_WIDE_F64 != 0 && wide) ? kWavesWide : kWavesPerBlock;
}

// world query of the render kernel
enum WorldMode : int {
    kWorldGlobal = 0,   // brute force, sphere list read from HBM/L2
    kWorldLds = 1,      // brute force, sphere list staged in LDS
    kWorldBvh = 2,      // binary BVH, single-loop traversal
    kWorldBvhWW = 3,    // binary BVH, while-while + leaf postponing
    kWorldBvh4 = 4,     // 4-wide octant BVH, while-while + leaf postponing
    kWorldBvhLds = 5,   // kWorldBvhWW with nodes + leaf spheres staged in LDS
};

// material kinds (same codes as RTW_LAMBERTIAN.. in include/rtw.h)
enum : uint32_t { kMatLambertian = 0, kMatMetal = 1, kMatDielectric = 2, kMatInvisible = 3, kMatDiffuseLight = 4 };

template <typename R>
struct alignas(4 * sizeof(R)) R4 {
    R x, y, z, w;
};

// Device-resident scene, precision R.  HBM layout (all arrays tightly packed):
//   sph      : n_sph   x R4 {cx, cy, cz, r*r}   -- staged into LDS by the brute kernel
//   sph_r    : n_sph   x R  radius              -- read once per hit (normal)
//   sph_mat  : n_sph   x u32 {material id (bits 0-23), kind (24-30), isolated (31)}
//   sph_shade: n_sph   x R4 {albedo r, g, b, fuzz | ior} -- the material's, per sphere
//   planes   : n_pl    x kPlaneR R {p, n, aabb lo, aabb hi, uv mode, cos, sin, k} (layout below)
//   plane_mat: n_pl    x u32
//   mat_type : n_mat   x u32
//   mat_p    : n_mat   x R4 {albedo r, g, b, fuzz | ior}
//   lights   : n_li    x R4 {cx, cy, cz, r}     -- staged into LDS
//   bvh      : n_nodes x BvhNode<R>            -- RTW_ACCEL_BVH
//   bsph     : n_sph   x R4 {cx, cy, cz, r*r} in BVH leaf order
//   bid      : n_sph   x u32 original sphere index of bsph[k]
//   bvh32    : n_nodes x BvhNode<float>        -- R = double: the same tree in f32 (while-while culling)
//   bvh4     : 8 x n_nodes4 x Bvh4Node<R>      -- RTW_ACCEL_BVH, 4-wide
//   lbvh     : n_lnodes x BvhNode<R>           -- light pdf query (BVH kernels)
//   lsph/lid : n_li x R4 {c, r} / u32 in light-BVH leaf order
//   lg_start : n_cells + 1 x u32                -- light grid (light pdf, long light lists)
//   lg_sph/lg_id : n_items x R4 {c, r} / u32    -- big list, then each cell's lights
//   lg_rec   : n_cells x 4 x R4<float>          -- each cell's first lights inline (the walk's one load per cell)
template <typename R>
struct BvhNode {
    // two child boxes per node (children tested together, the classic
    // "both children in one fetch" layout); a child index c >= 0 is an inner
    // node, c < 0 encodes a leaf: spheres [first, first + count) of the
    // BVH-ordered sphere arrays, first = (~c) >> 4, count = (~c) & 15.
    R lo_x[2], lo_y[2], lo_z[2], hi_x[2], hi_y[2], hi_z[2];
    int32_t child[2];
    int32_t pad[2];
};

// 4-wide node, one copy of the tree per ray-direction octant (bit a of the
// octant set: the ray goes -a).  In the copy for octant o the slab planes are
// pre-selected -- near = the plane a ray of that octant enters through, far =
// the one it leaves through -- and the children are stored in front-to-back
// order for that octant, so a visit is 6 FMAs + 4 min/max per child and no
// sort.  Child slot q is two R4s: a[q] = {near x, y, z, far x}, b[q] = {far y,
// far z, child link (bits), 0}.  Empty slots map to near = +inf, far = -inf
// in ray space (never hit) and an empty leaf.  Links index the same copy.
template <typename R>
struct alignas(sizeof(R) == 4 ? 128 : 256) Bvh4Node {
    R4<R> a[4];
    R4<R> b[4];
};

// f64 scenes also carry the binary tree in f32 (boxes rounded outward): the
// while-while traversal culls on f32 nodes in both precisions (R = float:
// `bvh` itself; the empty base keeps the f32 layout unchanged).
template <typename R>
struct DevSceneCull {};
template <>
struct DevSceneCull<double> {
    const BvhNode<float>* bvh32;
    const R4<float>* bsph32;          // bsph rounded to f32 {c, r^2}: the leaf pre-pass
    const R4<float>* lg_sph32;        // lg_sph rounded to f32 {c, |r|}: the light grid's f32 walk
};

template <typename R>
struct DevScene : DevSceneCull<R> {
    const R4<R>* sph;
    const R* sph_r;
    const uint32_t* sph_mat;
    const R4<R>* sph_shade;
    const R* planes;
    const uint32_t* plane_mat;
    const uint32_t* mat_type;
    const R4<R>* mat_p;
    const R4<R>* lights;
    const BvhNode<R>* bvh;
    const R4<R>* bsph;
    const uint32_t* bid;
    const Bvh4Node<R>* bvh4;          // 8 x n_nodes4 (octant copies)
    const BvhNode<R>* lbvh;           // binary BVH over the light spheres
    const R4<R>* lsph;                // lights {cx, cy, cz, r} in light-BVH leaf order
    const uint32_t* lid;              // light-list index of lsph[k]
    const uint32_t* lg_start;         // light grid: n_cells + 1 offsets into lg_sph / lg_id
    const R4<R>* lg_sph;              // light grid items {c, r}: the big list, then cell by cell
    const uint32_t* lg_id;            // light-list index of lg_sph[k]
    const R4<float>* lg_rec;          // light grid cell records (light_grid.hpp kGridRecSlots): the
                                      // cell's lights as the f32 walk reads them, inline, or 3 + a link
    const R* quads;                   // n_quads x kQuadR (see quad layout below)
    const uint32_t* quad_mat;
    const R* lquads;                  // the light list's quads, n_lquads x kQuadR
    const R4<double>* sph64;          // spheres {cx, cy, cz, radius} as given (f64): the f32
                                      // kernels' f64 hit points (kOptHit64)
    const R4<double>* pl64;           // planes {point, 0}, {normal, 0} as given (f64): kOptHit64
    const R4<double>* mat64;          // per material (f64; kOptHit64 and the f64 kernels): {1/ior, r0 at 1/ior, r0 at ior,
                                      // ior} (Dialectric), {-, -, -, fuzz} (Metal)
    const uint32_t* lref;             // light list in order (kLref* bits | index; null when the
                                      // list is spheres only)
    const R* boxes;                   // n_boxes x kBoxR (transformed cuboids, layout below)
    const uint32_t* box_mat;
    // textures (null mat_tex: every material is its SolidColour albedo, mat_p)
    const uint32_t* mat_tex;          // n_mat texture ids
    const uint32_t* tex_type;         // RTW_TEX_*
    const R4<R>* tex_p;               // {r, g, b, inv_scale | scale}
    const uint32_t* tex_refs;         // 2 per texture: checker even/odd, noise Perlin table
    const R4<R>* perlin_vec;          // 256 per table: rand_vec {x, y, z, 0}
    const uint32_t* perlin_perm;      // 768 per table: perm_x, perm_y, perm_z
    uint32_t n_sph, n_planes, n_mat, n_lights, n_nodes, bvh_depth;
    uint32_t n_nodes4, bvh4_stack, n_lnodes, lbvh_depth;
    uint32_t robust;                  // f32: closest-approach sphere / light tests (far geometry)
    uint32_t n_quads, n_lquads, n_list;   // world quads, light quads, light-list length
    uint32_t n_boxes;
    uint32_t light_flags;             // RTW_LIGHTS_BVH_LEAF
    uint32_t emissive;                // a DiffuseLight material exists (its scenes run the kOptPrims
                                      // kernels, which keep the emission accumulator)
    // light grid (host/bvh.hpp LightGrid): box lo / hi, cell size and its
    // inverse, cells per axis, big-list length, 1 when staged
    R lg_lo[3], lg_hi[3], lg_cell[3], lg_inv[3];
    uint32_t lg_n[3], lg_big, lg_on;
};

// Plane record, kPlaneR values of precision R: point [0..2], unit normal
// [3..5], the reference's AABB lo [6..8] hi [9..11] (plane.rs:79-102), and
// Plane::get_plane_uv's per-plane constants (plane.rs:40-54): [12] mode (0:
// theta <= EPSILON, uv = (x, z); 1: Rodrigues rotation; 2: k is not finite,
// so every uv is NaN and Plane::hit panics), [13] cos(theta), [14]
// sin(theta), [15..17] k = normalize(n x (0, 1, 0)).
constexpr uint32_t kPlaneR = 20;
// light-list entry encoding (DevScene::lref): bit 31 quad, bit 30 an entry
// with the Hittable defaults (pdf 0, random (1, 0, 0)), else a sphere
constexpr uint32_t kLrefQuad = 0x80000000u, kLrefDefault = 0x40000000u;

// Quad record (Quad::new's derived fields, quadrilateral.rs:37-56), kQuadR
// values of precision R: Q[0..2], u[3..5], v[6..8], w = n/|n|^2 [9..11],
// unit normal [12..14], area [15], AABB lo [16..18], hi [19..21], pad.
constexpr uint32_t kQuadR = 24;

// Transformed<Cuboid> record, kBoxR values of precision R: the six object-
// space quads (6 x kQuadR), rotation R [144..152] and its inverse [153..161]
// (row-major), translation T [162..164], -(R^-1 T) [165..167], world AABB lo
// [168..170] hi [171..173], invertible flag [174], pad.
constexpr uint32_t kBoxR = 176;
constexpr uint32_t kBoxRot = 144, kBoxInv = 153, kBoxT = 162, kBoxTi = 165, kBoxLo = 168, kBoxHi = 171,
                   kBoxOk = 174;

constexpr uint32_t kBvhStack = 32;    // per-lane traversal stack entries (LDS)
constexpr uint32_t kWalkStashMax = 48; // per-lane LDS words the light grid's walk may ask for
// f32 light-grid kernels: the cooperative walk parks up to this many words of
// path state per lane in the wave's stack area (render_kernel.hpp), so the
// host gives them at least kCoopStash + 1 entries
constexpr uint32_t kCoopStash = 20;
// f64 light-grid kernels: the walk parks the RNG state, the ray and (when
// RTW_STASH64_EXTRA) the path throughput and the pending bounce's weights
#ifndef RTW_STASH64_EXTRA
#define RTW_STASH64_EXTRA 1
#endif
constexpr uint32_t kCoopStash64 = RTW_STASH64_EXTRA ? 34u : 20u;
// the f64 cooperative grid walk (lights_pdf_grid_coop64): list indices one
// piece keeps per pass (its LDS slot: count + ids), and that a ray's owner
// sums per pass
#ifndef RTW_COOP64_PIECE_IDS
#define RTW_COOP64_PIECE_IDS 6
#endif
// the f64 list walk's owners merge only the pieces that hold a candidate
// (a ballot mask per round of <= 64 pieces); 0: every piece's slot
#ifndef RTW_COOP_HELD
#define RTW_COOP_HELD 1
#endif
// the f64 list walk's pieces keep their candidates in registers (one
// compare-exchange insert each) and write their slot once (C5 f64 1527 ->
// 1460 ms, C3 1042 -> 1004, profiles/r06m_ab_piece_reg.jsonl); 0: insertion in LDS
#ifndef RTW_PIECE_REG
#define RTW_PIECE_REG 1
#endif
// the light grid's piece walks load each cell's record one cell ahead of its
// tests (two loads in flight per lane); 0: load, then test
#ifndef RTW_GRID_PF
#define RTW_GRID_PF 0
#endif
#ifndef RTW_COOP64_MAX
#define RTW_COOP64_MAX 8
#endif
constexpr uint32_t kCoop64PieceIds = RTW_COOP64_PIECE_IDS;
// ... and the LDS words of one piece's slot per round: [count, list indices],
// padded to 8 (16-byte reads).  The host gives the f64 light-grid kernels
// kCoopStash64 + kCoop64Slot words per lane, so that a round holds >= 64
// pieces (the walk has no per-lane fallback)
constexpr uint32_t kCoop64Slot = 8;
static_assert(kCoop64PieceIds + 1 <= kCoop64Slot, "a piece's slot holds its count and ids");
static_assert(kCoopStash64 + kCoop64Slot <= kWalkStashMax, "the walk's LDS area fits the host's bound");
// Subtree stealing in the while-while traversal (render_kernel.hpp
// bvh_traverse_steal): per wave the result slots of its 64 rays (f32: a u64
// key; f64: u64 t bits + u32 id) and 64 rendezvous bytes, in LDS right after
// the traversal stacks of the workgroup's waves.
template <typename R>
constexpr uint32_t kStealSlotBytes = sizeof(R) == 4 ? 64 * 8 : 64 * 20;   // f64: + a culling bound per ray
template <typename R>
constexpr uint32_t kStealLdsPerWave = kStealSlotBytes<R> + 64;
// light-pdf work counters of a wave (u64 light tests, u64 light-grid cells:
// KParams::counters[7], [8]); the kernels with the light BVH / grid
// (light_bvh != 0) keep them right after the traversal area
constexpr uint32_t kLightWorkBytes = 16;
// LDS of the traversal stacks + the stealing area of one workgroup (+ the
// light-work counters when `light_work`)
template <typename R>
__host__ __device__ inline size_t traversal_lds(uint32_t stack, bool light_work = false,
                                               uint32_t waves = kWavesPerBlock) {
    return (size_t)waves * ((size_t)stack * 64 * sizeof(int32_t) + kStealLdsPerWave<R> +
                                     (light_work ? kLightWorkBytes : 0));
}
constexpr uint32_t kPersistResident = 0xFFFFFFFFu;   // KParams::persist: one resident grid


template <typename R>
struct KParams {
    DevScene<R> sc;
    R* partial;                       // [n_local_tiles][64][n_chunks][3] item (chunk) sums
    unsigned long long* counters;     // [0] segments, [1] lambertian, [2] node visits,
                                      // [3] sphere tests, [4] plane-UV panics, [5] empty-light panics,
                                      // [6] next task (persistent waves), [7] light tests and
                                      // [8] light-grid cells of the light BVH / grid walks
    R center[3], p00[3], du[3], dv[3], disk_u[3], disk_v[3], bg[3];
    R u_scale;                        // Uniform::new_inclusive(-0.5, 0.5) scale
    uint64_t seed;
    uint32_t defocus;                 // defocus_angle > f64::EPSILON
    uint32_t W, H, spp, max_depth;
    uint32_t chunk, n_chunks;         // samples per item, items per pixel
    uint32_t group, n_groups;         // chunks per wave task, tasks per tile
    uint32_t tiles_x, n_local_tiles, rank, nranks;   // local tile lt = global tile lt * nranks + rank
    uint32_t n_tasks;                 // n_local_tiles * n_groups
    uint32_t stack;                   // BVH traversal stack entries per lane (LDS)
    uint32_t light_bvh;               // light pdf (BVH kernels only): 1 through sc.lbvh, 2 the light grid
    uint32_t item_order;              // 0: pixel-major item pool, 1: sample-major
    uint32_t hit64;                   // f32 BVH kernels: f64 ray origin / own-sphere re-hit / hit point
    uint32_t persist;                 // > 0: workgroups launched (waves take tasks from
                                      // counters[6]; kPersistResident: as many as fit on the
                                      // GPU at once); 0: one task per wave
    const uint32_t* task_table;       // non-null: task t = {local tile, first chunk | chunks << 20}
                                      // at [2t, 2t + 1] (longest tiles first, sized by a pilot
                                      // render's costs); null: t = tile * n_groups + group
    uint32_t* tile_cost;              // non-null: [local tile] += the cost of each sample s < cost_spp
    uint32_t cost_spp;                //   (a pilot render, or the first render of a split)
    uint32_t cost_time;               //   ... the cost: 1 the sample's share of its wave's clock
                                      //   cycles (each trip's / its lanes); 0 node visits + sphere
                                      //   tests + kCostPerSegment per segment
    uint32_t grid_piece;              // f32 light grid: cells per piece of the wave-cooperative
                                      // walk (lights_pdf_grid_coop); 0: one lane per ray
    const uint32_t* tile_map;         // non-null: local tile lt -> global tile (a dealt split,
                                      // rtw_set_split); null: lt * nranks + rank (the round robin)
};

// the global 8x8 tile of local tile lt
template <typename R>
__host__ __device__ inline uint32_t global_tile(const KParams<R>& p, uint32_t lt) {
    return p.tile_map ? p.tile_map[lt] : lt * p.nranks + p.rank;
}

// The cost of a sample for the task order (KParams::tile_cost): its BVH node
// visits + sphere tests + this many per segment (a segment's hit record and
// scatter, in node-visit units).  Segments alone miss C5's horizon tiles,
// whose rays skim the sphere field through thousands of nodes per segment.
constexpr uint32_t kCostPerSegment = 12;

// Host-side launch helpers (defined in render_f32.hip / render_f64.hip).
// world: a WorldMode; lds_bytes: dynamic LDS of the kWorldLds variant.
// `mid` (may be null) is recorded on `stream` between the render kernel and
// the chunk reduction, so the render kernel can be timed on its own.
int launch_render_f32(const KParams<float>& p, int world, size_t lds_bytes, float* out,
                      hipStream_t stream, hipEvent_t mid);
int launch_render_f64(const KParams<double>& p, int world, size_t lds_bytes, double* out,
                      hipStream_t stream, hipEvent_t mid);
// The ranks' packed tiles (nranks buffers, rank_stride elements apart) -> the
// image [H][W][3] (rtw_assemble_tiles).  slot (may be null: the round robin,
// T itself): global tile T -> lt * nranks + rank of a dealt split.
int launch_assemble_f32(const float* ranks, size_t rank_stride, uint32_t nranks, uint32_t W, uint32_t H,
                        const uint32_t* slot, float* img, hipStream_t stream);
int launch_assemble_f64(const double* ranks, size_t rank_stride, uint32_t nranks, uint32_t W, uint32_t H,
                        const uint32_t* slot, double* img, hipStream_t stream);

}  // namespace rtw
