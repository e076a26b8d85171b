// bvh.hpp -- host-side BVH over the world's spheres for the RTW_ACCEL_BVH
// render kernel.
//
// The reference builds a median-split binary BVH with <= 5 objects per leaf
// and visits BOTH children of every node it enters (bvh.rs:106-188); only its
// closest-hit semantics are part of the contract.  This
// build is a binned-SAH binary tree with <= kLeafMax spheres per leaf, stored
// "children in the parent" (one node = both child boxes + both child links),
// traversed near-child-first with t-culling.  Box tests only cull: every
// sphere that survives is tested with exactly the brute-force arithmetic, and
// boxes are padded outward so that rounding can never cull the true closest
// sphere.
#pragma once

#include <stdint.h>

#include <vector>

namespace rtw {

struct BvhBuild {
    struct Node {
        double lo[2][3], hi[2][3];   // child boxes (padded)
        int32_t child[2];            // >= 0 inner node; < 0 leaf, see leaf_code()
    };
    std::vector<Node> nodes;         // nodes[0] is the root
    std::vector<uint32_t> order;     // BVH position -> original sphere index
    uint32_t depth = 0;              // inner-node levels on the deepest path
    uint32_t leaves = 0;
};

constexpr uint32_t kLeafMax = 4;

// leaf code: ~((first << 4) | count), count in [0, 15]
inline int32_t leaf_code(uint32_t first, uint32_t count) { return ~(int32_t)((first << 4) | count); }

// spheres: n x {cx, cy, cz, r}.  pad_rel: relative outward padding of every
// box (absorbs the rounding of the device slab test in the kernel precision).
// leaf_max: spheres per leaf (1..15; the kernel tests leaves in groups of 4).
BvhBuild build_bvh(const double* spheres, uint32_t n, double pad_rel, uint32_t leaf_max = kLeafMax);

// 4-wide BVH collapsed from the binary one (same leaves, same boxes): every
// node takes the up-to-4 descendants reached by repeatedly opening its
// largest-area inner child.  For each of the 8 ray-direction octants the
// children get a front-to-back order from the binary splits they came from
// (near side first along each split axis), so the kernel needs no sort.
struct Bvh4Build {
    struct Node {
        double lo[4][3], hi[4][3];   // child boxes; slots >= n are empty
        int32_t child[4];            // >= 0 inner node; < 0 leaf code (leaf_code(0,0) if empty)
        uint8_t order[8][4];         // per octant: slot of the 1st, 2nd, ... child to visit
        uint32_t n;
    };
    std::vector<Node> nodes;         // nodes[0] is the root
    uint32_t max_stack = 0;          // most traversal-stack entries any path can hold
    uint32_t depth = 0;
};

Bvh4Build collapse_bvh4(const BvhBuild& b);

// Spheres whose closed ball is at least `margin` away from every other
// sphere's (negative radii never hit and are ignored).  A ray that starts on
// such a sphere and hits it again reaches that hit along a chord of the ball,
// which no other sphere touches -- so that hit is the closest sphere hit and
// the render kernel skips the traversal for it (self-hit shortcut).
std::vector<uint8_t> isolated_spheres(const double* spheres, uint32_t n, const BvhBuild& b, double margin);

// Uniform grid over the light spheres for the light pdf's all-hits query
// (render_kernel.hpp light_grid_walk).  Cell c lists every light whose
// padded AABB overlaps it, in ascending light index; lights that are not
// finite, larger than kGridBigRadius x the median radius or span more than
// kGridBigCells cells form the "big" list every ray tests.  The grid box (lo, lo + n * cell) holds every listed light's AABB.
struct LightGrid {
    double lo[3] = {0, 0, 0}, cell[3] = {1, 1, 1};
    uint32_t n[3] = {1, 1, 1};
    uint32_t n_big = 0;
    std::vector<uint32_t> start;     // n_cells + 1 offsets into items (start[0] = n_big)
    std::vector<uint32_t> items;     // light indices: the big list, then cell by cell
};

constexpr uint32_t kGridBigCells = 64;
constexpr double kGridBigRadius = 3.0;   // x the median light radius

// lights: n x {cx, cy, cz, r}; cells_per_light: grid resolution target.
LightGrid build_light_grid(const double* lights, uint32_t n, double cells_per_light);

// light grid cell records (DevScene::lg_rec, light_grid.hpp light_grid_walk_piece_rec)
constexpr uint32_t kGridRecSlots = 4;
constexpr uint32_t kGridRecLink = 0x7fc0dea1u;   // a quiet NaN: slot 3's z of a link

// The cells' records of the f32 walk (DevScene::lg_rec, light_grid.hpp
// light_grid_walk_piece_rec): kGridRecSlots x {cx, cy, cz, r} floats per cell
// -- a cell of n <= kGridRecSlots lights holds them then all-NaN slots, a
// larger one its first kGridRecSlots - 1 and a link {first bits, count bits,
// kGridRecLink bits, NaN} to the rest of its list (g.items order).  The
// radius is |r| rounded when `abs_radius` (the f64 kernels' lg_sph32), else r.
std::vector<float> light_grid_records(const LightGrid& g, const double* lights, bool abs_radius);

}  // namespace rtw
