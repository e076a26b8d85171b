// capi.cpp -- the C-ABI (include/rtw.h): context, scene upload, CameraBuilder::
// build, the render entry points, scenes::simple and the PPM encoding.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>   // types only: the functions are resolved at run time (rccl_api)
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <new>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/rtw.h"
#include "host/bvh.hpp"
#include "host/rtw_host.hpp"
#include "rtw_kernels.h"

struct rtw_ctx {
    int device = 0;
    int precision = RTW_F32;
    int accel = RTW_ACCEL_AUTO;
    uint32_t chunk = 0;           // samples per item (0 = auto_chunk)
    uint32_t auto_chunk = 1;      // one sample per item: the chunk fold is then the reference's
                                  // sample-by-sample fold exactly
    // cap of the chunk-sum buffer (the auto chunk grows beyond it), at most half
    // the device's memory: 128 GiB of the 288 GB of HBM keeps every BASELINE
    // config at one sample per item -- the reference's fold order exactly (C2
    // f64: 11.5 GB, C3 f64 51 GB, a C4 f64 8-way share 102 GB).  Chunk 1 is
    // also the faster form: a chunk > 1 reads its running sum back at every
    // sample's end (C3 f64 1083 vs 1121 ms at chunk 2, a C4 share 958 vs 993
    // ms at chunk 4, profiles/r06h_ab_chunk.jsonl, r06i_ab_c4_chunk.jsonl)
    size_t partial_max = (size_t)128 << 30;
    size_t dev_total = 0;         // the device's memory (hipMemGetInfo), 0 until asked
    uint32_t group = 0;           // chunks per wave task (0 = from target_tasks)
    uint64_t target_tasks = 0;   // auto chunks-per-task: about this many tasks (0: 2^19 with
                                 // persistent waves, 2^17 without), 4..32 chunks per task
    int world_pref = 1;           // 1: LDS-staged sphere list when it fits, 0: global
    int auto_accel = RTW_ACCEL_AUTO;    // RTW_ACCEL_AUTO resolves to this (AUTO: by scene size)
    int bvh_kind = 3;             // BVH traversal: 3 = binary while-while + leaf postponing on the
                                  // tree staged in LDS (falls back to 1 when it does not fit),
                                  // 1 = the same from L1/L2, 2 = 4-wide octant tree, 0 = binary
                                  // single loop
    // LDS per workgroup allowed for bvh_kind 3 (0: by precision -- f32 36 KiB, four
    // 256-thread workgroups per CU at 4 waves/SIMD; f64 52 KiB)
    size_t bvh_lds_max = 0;
    int robust = 2;                   // f32 closest-approach tests: 1 on, 0 off, 2 by scene scale
    double scene_extent = 0.0, min_radius = 0.0;   // of the staged scene (robust = 2)
    uint32_t bvh_leaf = 0;            // spheres per BVH leaf (set before rtw_set_scene); 0 = auto:
                                      // 4, 8 for scenes of >= 100k spheres (C5: +12 %), 2 for
                                      // f64 scenes of 4096..100k (rtw_set_scene)
    uint32_t persist = rtw::kPersistResident;   // workgroups of persistent waves (tasks from a
                                      // counter; default: as many as are resident at once);
                                      // 0: one task per wave
    uint32_t light_leaf = 0;          // light spheres per light-BVH leaf; 0 = 4
    uint32_t light_grid = 8;          // light pdf through the light grid at light_grid / 16
                                      // cells per light (set before rtw_set_scene); 0: light BVH
    uint32_t hit64 = 1;               // f32: f64 hit points (the reference's self-intersection odds)
    uint32_t item_order = 1;          // wave item pool: 1 sample-major (C2 +1.3 %, C3 +5 %, C5 +2 %), 0 pixel-major
    uint32_t lpt = 1;                 // longest tiles first: task order from a pilot render's
                                      // per-tile segment counts (cached per scene / camera / split);
                                      // 1: for worlds in LDS or within an L2, 2: always, 0: never
    uint32_t lpt_min_spp = 32;        // ... for renders of at least this many samples per pixel
    uint32_t lpt_inline = 1;          // 1: no separate pilot -- the first render of a (scene,
                                      // camera, split) runs in the plain tile order and counts the
                                      // segments of each pixel's first lpt_pilot_spp samples; the
                                      // renders after it take the task list of those counts
                                      // 0: a pilot render before the first render
    uint32_t lpt_pilot_spp = 2;       // the pilot render: samples per pixel
    uint32_t lpt_pilot_depth = 0;     // ... and its max depth (0: the camera's); a path's segments
                                      // run one after another, so the pilot lasts as long as its
                                      // longest path
    static constexpr uint32_t kGridPieceAuto = 0xFFFFFFFFu;
    uint32_t grid_piece = kGridPieceAuto;   // light grid walks: cells per piece of the wave's
                                      // cooperative walk (0: one lane walks its own ray)
    uint32_t light_bvh_min = 64;      // light lists at least this long use the light BVH
                                      // (C2, 19 lights: the linear masked loop is faster)
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // ring of per-render event triples: [start, after render kernel, after reduce]
    static constexpr int kRing = 64;
    hipEvent_t ring[kRing][3] = {};
    uint64_t n_renders = 0;
    // device scene (one allocation holding every array)
    void* d_scene = nullptr;
    size_t scene_bytes = 0;           // allocation
    size_t scene_used = 0;            // the current scene's bytes
    size_t tree_bytes = 0;            // ... of them the BVH nodes + leaf spheres + ids
    rtw::DevScene<float> sc32{};
    rtw::DevScene<double> sc64{};
    bool has_scene = false;
    // work buffers
    void* d_partial = nullptr;
    size_t partial_cap = 0;
    void* d_out = nullptr;        // rtw_render: the packed tiles, then the image
    size_t out_cap = 0;
    void* d_img = nullptr;
    size_t img_cap = 0;
    static constexpr int kCounters = 9;   // rtw_kernels.h KParams::counters
    unsigned long long* d_counters = nullptr;
    std::vector<unsigned char> h_out;
    // longest-tiles-first task list (pilot render, see lpt_pilot / lpt_tasks)
    uint64_t scene_serial = 0;        // ++ per rtw_upload_scene
    static constexpr uint32_t kMaxGroup = 32;
    uint32_t max_group = kMaxGroup;   // longest-first task list: at most this many chunks per task
    // longest-first task list with guided sizes (lpt_tasks; guide_div 0: equal-cost
    // tasks of max_group chunks at most): a task costs the remaining work / guide_div,
    // at least total / guide_floor, at most guide_max chunks
    // (C2 f64, max of 8 rank shares, 3 runs each: 16.32 ms vs equal-cost tasks 16.79;
    // one GPU 117.35 vs 118.46 ms; profiles/r06i_ab_split.jsonl)
    uint32_t guide_div = 16384, guide_max = 128;
    uint32_t cost_time = 1;           // tile costs in wave-time shares (KParams::cost_time); 0: work counts
    uint64_t guide_floor = 1u << 20;
    void* d_lpt = nullptr;            // pilot: [tile cost | chunk sums | tiles]
    size_t lpt_cap = 0;
    bool lpt_valid = false;           // h_lpt_cost is the pilot of (lpt_cam, lpt_serial, rank split, precision)
    bool lpt_pending = false;         // ... still on the device: counted by the render before (lpt_ev)
    hipEvent_t lpt_ev = nullptr;
    rtw_camera lpt_cam{};
    uint64_t lpt_serial = 0;
    uint32_t lpt_rank = 0, lpt_nranks = 0, lpt_prec = 0;
    uint64_t lpt_split = 0;           // ... and split id (split_id: 0 = the round robin)
    std::vector<uint32_t> h_lpt_cost;
    void* d_lpt_tasks = nullptr;      // the task list of (h_lpt_cost, lpt_tab_*)
    size_t lpt_tasks_cap = 0;
    bool lpt_tab_valid = false;
    uint32_t lpt_tab_chunks = 0, lpt_tab_group = 0;
    uint64_t lpt_tab_target = 0;
    std::vector<uint32_t> h_lpt_tasks;
    rtw_stats last{};
    int last_variant = 0;             // render kernel of the last render: launch_render_impl's code
    uint32_t last_n_sph = 0;
    uint32_t last_light_bvh = 0;      // KParams::light_bvh of the last render (0: the linear light loop)
    uint32_t last_n_list = 0;         // ... and its light-list length
    std::string err;
    // multi-device context (rtw_create_devices): this context is rank 0 on the
    // first device; peers[k - 1] is the context of rank k on device k of the
    // list, mirroring every knob and the scene.  One RCCL communicator per rank
    // (a single-process clique) for the framebuffer gather to rank 0.
    bool multi = false;
    std::vector<rtw_ctx*> peers;
    std::vector<ncclComm_t> comms;
    void* d_gather = nullptr;         // rank 0's device: the n ranks' packed tiles (gather target)
    size_t gather_cap = 0;
    // virtual ranks (rtw_create_virtual, a test mode): every rank on one device,
    // the gather done by device copies on rank 0's stream after peer_ev[k - 1]
    bool virt = false;
    std::vector<hipEvent_t> peer_ev;
    // the last multi-device gather + assembly, on rank 0's stream of that call:
    // the next call's renders (every rank) wait for it before they overwrite
    // d_gather or a peer's packed tiles
    hipEvent_t gather_ev = nullptr;
    bool gather_pending = false;
    // ranks whose counters the last render filled (rtw_get_stats): n after
    // rtw_render / rtw_render_image_device, 1 after rtw_render_device
    uint32_t stats_ranks = 1;
    // Rank split (ABI 10): renders of a split_W x split_H image over split_n
    // ranks give tile T to rank split_rank[T] (rtw_set_split; empty: T mod n,
    // the round robin).  Each rank keeps the round robin's tile COUNT, so the
    // packed buffers and the gather are unchanged.  split_cost: the tile costs
    // the split was dealt by -- they order the next renders' tasks (no counting
    // render after a deal).  split_auto: dealt by rtw_render_image_device
    // (tuning "balance") for split_cam / split_scene, re-dealt when they change.
    uint32_t split_W = 0, split_H = 0, split_n = 0;
    uint64_t split_serial = 0;        // ++ per split set: the split's id in the task-order key
    bool split_auto = false;
    rtw_camera split_cam{};
    uint64_t split_scene = 0;
    std::vector<uint32_t> split_rank, split_cost;
    uint32_t balance = 1;             // multi-device renders: deal tiles by their counted costs
    // the device copies of the split: this rank's local tile -> global tile (render
    // kernel) and global tile -> lt * n + rank (assembly), for split id *_key
    std::vector<uint32_t> h_tile_map;
    void* d_tile_map = nullptr;
    size_t tile_map_cap = 0;
    uint64_t tile_map_key = 0;
    uint32_t tile_map_rank = 0;
    void* d_tile_slot = nullptr;
    size_t tile_slot_cap = 0;
    uint64_t tile_slot_key = 0;
};

namespace {

constexpr size_t kLdsLimit = 160 * 1024;
constexpr uint64_t kAutoTasks = 1u << 17;   // auto task size: about this many tasks per render
constexpr uint32_t kTaskMaxChunks = 4095;    // task-table entry {first chunk | chunks << 20}: 12 bits

int fail(rtw_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
int hip_fail(rtw_ctx* c, hipError_t e, const char* what) {
    return fail(c, RTW_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(ctx, expr)                                   \
    do {                                                     \
        hipError_t e_ = (expr);                              \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
    } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// RCCL for the multi-device gather, resolved at the first multi-device
// context: dlopen by SONAME, so a process that already holds PyTorch's
// librccl.so.1 shares that copy (one RCCL per process); a plain C caller gets
// ROCm's.  Single-device contexts never load it.
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const RcclApi& rccl_api() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
        if (!h) {
            api.err = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && api.err.empty()) api.err = std::string("librccl.so.1 lacks ") + name;
        };
        sym(api.comm_init_all, "ncclCommInitAll");
        sym(api.comm_destroy, "ncclCommDestroy");
        sym(api.gather, "ncclGather");
        sym(api.group_start, "ncclGroupStart");
        sym(api.group_end, "ncclGroupEnd");
        sym(api.error_string, "ncclGetErrorString");
        api.ok = api.err.empty();
    });
    return api;
}

// the caller's stream argument: NULL = the context's own stream,
// RTW_STREAM_NULL = the device's null (legacy default) stream, else a hipStream_t
hipStream_t resolve_stream(const rtw_ctx* c, void* stream) {
    if (!stream) return c->stream;
    if (stream == RTW_STREAM_NULL) return nullptr;
    return reinterpret_cast<hipStream_t>(stream);
}

int rccl_fail(rtw_ctx* c, ncclResult_t r, const char* what) {
    const RcclApi& a = rccl_api();
    return fail(c, RTW_E_DEVICE, std::string(what) + ": " + (a.error_string ? a.error_string(r) : "RCCL error"));
}

// Quad::new (quadrilateral.rs:37-56) in f64, in the oracle's operation order
// (rtw_oracle.c quad_new): out = {Q, u, v, w, normal, area, box lo, box hi}.
void quad_derive(const double* p, double* out) {
    const double q[3] = {p[0], p[1], p[2]}, u[3] = {p[3], p[4], p[5]}, v[3] = {p[6], p[7], p[8]};
    // AABBox::from_points([q + (u + v) * 0.5, q, q + v, q + u, q + u + v]),
    // each enclose followed by pad_to_minimum (aabox.rs:129-175)
    double pts[5][3];
    for (int a = 0; a < 3; ++a) {
        pts[0][a] = q[a] + (u[a] + v[a]) * 0.5;
        pts[1][a] = q[a];
        pts[2][a] = q[a] + v[a];
        pts[3][a] = q[a] + u[a];
        pts[4][a] = (q[a] + u[a]) + v[a];
    }
    double mn[3], mx[3];
    for (int a = 0; a < 3; ++a) mn[a] = mx[a] = pts[0][a];
    for (int i = 1; i < 5; ++i) {
        for (int a = 0; a < 3; ++a) {
            mn[a] = fmin(mn[a], pts[i][a]);
            mx[a] = fmax(mx[a], pts[i][a]);
        }
        for (int a = 0; a < 3; ++a)
            if (mx[a] - mn[a] < 0.0001) {
                mn[a] -= 0.0001;
                mx[a] += 0.0001;
            }
    }
    const double n[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
    const double n2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    const double area = sqrt(n2);
    for (int a = 0; a < 3; ++a) {
        out[a] = q[a];
        out[3 + a] = u[a];
        out[6 + a] = v[a];
        out[9 + a] = n[a] / n2;
        out[12 + a] = n[a] / area;
        out[16 + a] = mn[a];
        out[19 + a] = mx[a];
    }
    out[15] = area;
    out[22] = out[23] = 0.0;
}

// Transformed<Cuboid> derived record in f64, in the oracle's operation order
// (rtw_oracle.c box_new); layout rtw_kernels.h kBoxR.
void box_derive(const double* b, double* out) {
    auto enclose_pad = [](double* mn, double* mx, const double* pmn, const double* pmx) {
        for (int a = 0; a < 3; ++a) {
            mn[a] = fmin(mn[a], pmn[a]);
            mx[a] = fmax(mx[a], pmx[a]);
        }
        for (int a = 0; a < 3; ++a)
            if (mx[a] - mn[a] < 0.0001) {
                mn[a] -= 0.0001;
                mx[a] += 0.0001;
            }
    };
    // Cuboid::new: the padded box of p and q, then the six quads
    double mn[3] = {b[0], b[1], b[2]}, mx[3] = {b[0], b[1], b[2]};
    enclose_pad(mn, mx, b + 3, b + 3);
    const double delta[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
    const double dx[3] = {delta[0], 0.0, 0.0}, dy[3] = {0.0, delta[1], 0.0}, dz[3] = {0.0, 0.0, delta[2]};
    const double ndx[3] = {-dx[0], -dx[1], -dx[2]}, ndy[3] = {-dy[0], -dy[1], -dy[2]},
                 ndz[3] = {-dz[0], -dz[1], -dz[2]};
    const double* args[6][3] = {{mn, dx, dy}, {mn, dy, dz}, {mn, dx, dz}, {mx, ndx, ndy}, {mx, ndy, ndz}, {mx, ndx, ndz}};
    double cmn[3] = {0, 0, 0}, cmx[3] = {0, 0, 0};
    for (int i = 0; i < 6; ++i) {
        double q[9];
        for (int a = 0; a < 3; ++a) {
            q[a] = args[i][0][a];
            q[3 + a] = args[i][1][a];
            q[6 + a] = args[i][2][a];
        }
        double* Q = out + rtw::kQuadR * i;
        quad_derive(q, Q);
        // Cuboid::get_aabbox: fold of the quads' boxes
        if (i == 0) {
            for (int a = 0; a < 3; ++a) {
                cmn[a] = Q[16 + a];
                cmx[a] = Q[19 + a];
            }
        } else {
            enclose_pad(cmn, cmx, Q + 16, Q + 19);
        }
    }
    double* Rm = out + rtw::kBoxRot;
    for (int k = 0; k < 9; ++k) Rm[k] = b[6 + k];
    for (int a = 0; a < 3; ++a) out[rtw::kBoxT + a] = b[15 + a];
    auto mul = [&](const double* M, const double* p, double* o) {
        for (int r = 0; r < 3; ++r) o[r] = M[3 * r] * p[0] + M[3 * r + 1] * p[1] + M[3 * r + 2] * p[2];
    };
    // world AABB: from_points of the cuboid box corners (get_points order) mapped by R p + T
    const double* lo = cmn;
    const double* hi = cmx;
    const double corners[8][3] = {{lo[0], lo[1], lo[2]}, {lo[0], hi[1], lo[2]}, {lo[0], lo[1], hi[2]},
                                  {lo[0], hi[1], hi[2]}, {hi[0], lo[1], lo[2]}, {hi[0], hi[1], lo[2]},
                                  {hi[0], lo[1], hi[2]}, {hi[0], hi[1], hi[2]}};
    double wmn[3], wmx[3];
    for (int i = 0; i < 8; ++i) {
        double w[3];
        mul(Rm, corners[i], w);
        for (int a = 0; a < 3; ++a) w[a] = w[a] + b[15 + a];
        if (i == 0) {
            for (int a = 0; a < 3; ++a) wmn[a] = wmx[a] = w[a];
        } else {
            enclose_pad(wmn, wmx, w, w);
        }
    }
    for (int a = 0; a < 3; ++a) {
        out[rtw::kBoxLo + a] = wmn[a];
        out[rtw::kBoxHi + a] = wmx[a];
    }
    // Matrix3::inverse (matrix3.rs:9-28), Transformation::inverse
    const double a = Rm[0], bb = Rm[1], c = Rm[2], d = Rm[3], e = Rm[4], f = Rm[5], g = Rm[6], h = Rm[7],
                 i = Rm[8];
    const double det = a * (e * i - f * h) + bb * (f * g - d * i) + c * (d * h - e * g);
    out[rtw::kBoxOk] = std::isnormal(det) ? 1.0 : 0.0;
    const double A = e * i - f * h, Bc = f * g - d * i, C = d * h - e * g;
    const double D = c * h - bb * i, E = a * i - c * g, F = bb * g - a * h;
    const double G = bb * f - c * e, H = c * d - a * f, I = a * e - bb * d;
    double* Ri = out + rtw::kBoxInv;
    Ri[0] = A / det; Ri[1] = D / det; Ri[2] = G / det;
    Ri[3] = Bc / det; Ri[4] = E / det; Ri[5] = H / det;
    Ri[6] = C / det; Ri[7] = F / det; Ri[8] = I / det;
    double rt[3];
    mul(Ri, b + 15, rt);
    for (int a2 = 0; a2 < 3; ++a2) out[rtw::kBoxTi + a2] = -rt[a2];
    out[rtw::kBoxOk + 1] = 0.0;
}

// Convert the caller's f64 SoA into the device layout of precision R, in one
// host staging blob, and fill the DevScene pointers relative to `base`.
template <typename R>
std::vector<unsigned char> stage_scene(const rtw_scene* s, rtw::DevScene<R>* ds, uintptr_t base,
                                       uint32_t leaf_max, uint32_t light_leaf, double grid_density) {
    using R4 = rtw::R4<R>;
    size_t off = 0;
    auto reserve = [&](size_t bytes) {
        size_t o = align_up(off, 64);
        off = o + bytes;
        return o;
    };
    const size_t o_sph = reserve(sizeof(R4) * s->n_spheres);
    // the f64 copies read by the f32 kernels' kOptHit64 parts only
    constexpr bool k64 = std::is_same<R, float>::value;
    const size_t o_s64 = reserve(k64 ? sizeof(double) * 4 * s->n_spheres : 0);
    const size_t o_pl64 = reserve(k64 ? sizeof(double) * 8 * s->n_planes : 0);
    // the per-material f64 scatter record: both precisions (the f64 kernels' one-pass
    // Metal / Dielectric scatter reads it too)
    const size_t o_m64 = reserve(sizeof(double) * 4 * s->n_materials);
    const size_t o_r = reserve(sizeof(R) * s->n_spheres);
    const size_t o_smat = reserve(sizeof(uint32_t) * s->n_spheres);
    const size_t o_sshade = reserve(sizeof(R4) * s->n_spheres);
    const size_t o_pl = reserve(sizeof(R) * rtw::kPlaneR * s->n_planes);
    const size_t o_quads = reserve(sizeof(R) * rtw::kQuadR * s->n_quads);
    const size_t o_qmat = reserve(sizeof(uint32_t) * s->n_quads);
    const size_t o_lquads = reserve(sizeof(R) * rtw::kQuadR * s->n_light_quads);
    const uint32_t n_list = s->n_lights + s->n_light_quads + s->n_light_other;
    const size_t o_lref = reserve(sizeof(uint32_t) * n_list);
    const size_t o_boxes = reserve(sizeof(R) * rtw::kBoxR * s->n_boxes);
    const size_t o_bmat = reserve(sizeof(uint32_t) * s->n_boxes);
    const size_t o_pmat = reserve(sizeof(uint32_t) * s->n_planes);
    const size_t o_mt = reserve(sizeof(uint32_t) * s->n_materials);
    const size_t o_mp = reserve(sizeof(R4) * s->n_materials);
    const size_t o_li = reserve(sizeof(R4) * s->n_lights);
    const bool tex = s->mat_tex != nullptr;
    const size_t o_mtex = reserve(sizeof(uint32_t) * (tex ? s->n_materials : 0));
    const size_t o_ttype = reserve(sizeof(uint32_t) * (tex ? s->n_textures : 0));
    const size_t o_tp = reserve(sizeof(R4) * (tex ? s->n_textures : 0));
    const size_t o_trefs = reserve(sizeof(uint32_t) * 2 * (tex ? s->n_textures : 0));
    const size_t o_pvec = reserve(sizeof(R4) * 256 * (tex ? s->n_perlin : 0));
    const size_t o_pperm = reserve(sizeof(uint32_t) * 768 * (tex ? s->n_perlin : 0));
    // BVH over the spheres; boxes padded outward by a margin that absorbs the
    // rounding of the slab test in precision R (it only ever culls)
    const rtw::BvhBuild bb = rtw::build_bvh(s->spheres, s->n_spheres,
                                            std::is_same<R, float>::value ? 1e-5 : 1e-12, leaf_max);
    const size_t o_nodes = reserve(sizeof(rtw::BvhNode<R>) * bb.nodes.size());
    // f64: the same tree in f32 (boxes rounded outward), which the while-while
    // traversal culls on with an error slack (bvh_traverse_ww)
    const size_t o_nodes32 = reserve(std::is_same<R, double>::value ? sizeof(rtw::BvhNode<float>) * bb.nodes.size() : 0);
    // f64: the leaf spheres {c, r^2} rounded to f32, the leaf pre-pass of the f64 kernels
    const size_t o_bsph32 = reserve(std::is_same<R, double>::value ? sizeof(rtw::R4<float>) * s->n_spheres : 0);
    const size_t o_bsph = reserve(sizeof(R4) * s->n_spheres);
    const size_t o_bid = reserve(sizeof(uint32_t) * s->n_spheres);
    // isolated spheres (self-hit shortcut): bit 31 of sphere_mat.  The margin
    // covers the rounding of the hit point the next segment starts from and
    // of the precision-R sphere tests of nearby spheres (grazing hits).
    double scale = 0.0;
    for (uint32_t k = 0; k < s->n_spheres; ++k)
        for (int a = 0; a < 3; ++a) scale = std::max(scale, fabs(s->spheres[4 * k + a]) + fabs(s->spheres[4 * k + 3]));
    const double iso_margin = std::is_same<R, float>::value ? 1e-2 + 1e-5 * scale : 1e-6 + 1e-12 * scale;
    const std::vector<uint8_t> iso = rtw::isolated_spheres(s->spheres, s->n_spheres, bb, iso_margin);
    const rtw::Bvh4Build b4 = rtw::collapse_bvh4(bb);
    const size_t o_nodes4 = reserve(sizeof(rtw::Bvh4Node<R>) * 8 * b4.nodes.size());
    // BVH over the light spheres for the light pdf (a query for EVERY light
    // the ray hits, so boxes only cull; the sum itself keeps list order in f64)
    const rtw::BvhBuild lb = rtw::build_bvh(s->lights, s->n_lights,
                                            std::is_same<R, float>::value ? 1e-5 : 1e-12, light_leaf);
    const size_t o_lnodes = reserve(sizeof(rtw::BvhNode<R>) * lb.nodes.size());
    const size_t o_lsph = reserve(sizeof(R4) * s->n_lights);
    const size_t o_lid = reserve(sizeof(uint32_t) * s->n_lights);
    // uniform grid over the light spheres (grid_density cells per light; 0: none)
    const rtw::LightGrid lg = grid_density > 0 ? rtw::build_light_grid(s->lights, s->n_lights, grid_density)
                                               : rtw::LightGrid{};
    const size_t o_lgs = reserve(sizeof(uint32_t) * lg.start.size());
    const size_t o_lgsph = reserve(sizeof(R4) * lg.items.size());
    const size_t o_lgid = reserve(sizeof(uint32_t) * lg.items.size());
    // f64: the grid's lights rounded to f32 with |r| -- the f64 kernels' walk runs
    // in f32 on them (render_kernel.hpp lights_pdf_grid_coop64)
    const size_t o_lgsph32 = reserve(std::is_same<R, double>::value ? sizeof(rtw::R4<float>) * lg.items.size() : 0);
    // the cells' records (light_grid.hpp light_grid_walk_piece_rec): 64 B per cell
    const size_t n_cells = lg.start.empty() ? 0 : lg.start.size() - 1;
    const size_t o_lgrec = reserve(sizeof(rtw::R4<float>) * rtw::kGridRecSlots * n_cells);
    std::vector<unsigned char> blob(align_up(off, 64) + 64, 0);
    unsigned char* b = blob.data();
    for (uint32_t k = 0; k < s->n_spheres; ++k) {
        const double* p = s->spheres + 4 * k;
        R r = (R)p[3];
        // a negative radius inverts the sphere's AABB, which bounded_hit never
        // passes (sphere.rs:42-45): r^2 = -inf makes the discriminant -inf
        reinterpret_cast<R4*>(b + o_sph)[k] = R4{(R)p[0], (R)p[1], (R)p[2], p[3] < 0 ? (R)-INFINITY : r * r};
        reinterpret_cast<R*>(b + o_r)[k] = r;
        if (k64)
            for (int a = 0; a < 4; ++a) reinterpret_cast<double*>(b + o_s64)[4 * k + a] = p[a];
        const uint32_t m = s->sphere_mat[k], t = s->mat_type[m];
        reinterpret_cast<uint32_t*>(b + o_smat)[k] = m | (t << 24);
        const double* mp = s->mat_params + 5 * m;
        const double w = t == RTW_METAL ? mp[3] : (t == RTW_DIELECTRIC ? mp[4] : 0.0);
        reinterpret_cast<R4*>(b + o_sshade)[k] = R4{(R)mp[0], (R)mp[1], (R)mp[2], (R)w};
    }
    for (uint32_t k = 0; k < s->n_spheres; ++k)
        if (iso[k]) reinterpret_cast<uint32_t*>(b + o_smat)[k] |= 0x80000000u;
    for (uint32_t k = 0; k < s->n_planes; ++k) {
        // {point, normal, AABB lo, AABB hi}: Plane::get_aabbox (plane.rs:218-242)
        // pins the normal axis at 0 and leaves the others infinite
        const double* pl = s->planes + 6 * k;
        const double e = 2.220446049250313080847e-16;
        const bool fx = fabs(pl[5]) < e && fabs(pl[4]) < e, fy = fabs(pl[3]) < e && fabs(pl[5]) < e,
                   fz = fabs(pl[3]) < e && fabs(pl[4]) < e;
        const double box[6] = {fx ? 0.0 : -INFINITY, fy ? 0.0 : -INFINITY, fz ? 0.0 : -INFINITY,
                               fx ? 0.0 : INFINITY, fy ? 0.0 : INFINITY, fz ? 0.0 : INFINITY};
        R* dst = reinterpret_cast<R*>(b + o_pl) + rtw::kPlaneR * k;
        for (int q = 0; q < 6; ++q) dst[q] = (R)pl[q];
        for (int q = 0; k64 && q < 3; ++q) {
            reinterpret_cast<double*>(b + o_pl64)[8 * k + q] = pl[q];
            reinterpret_cast<double*>(b + o_pl64)[8 * k + 4 + q] = pl[3 + q];
        }
        for (int q = 0; q < 6; ++q) dst[6 + q] = (R)box[q];
        // Plane::get_plane_uv's constants (plane.rs:40-54), computed as the
        // oracle's plane_uv does: theta = atan2(|n x V|, n . V), V = (0, 1, 0)
        const double c[3] = {pl[4] * 0.0 - pl[5] * 1.0, pl[5] * 0.0 - pl[3] * 0.0, pl[3] * 1.0 - pl[4] * 0.0};
        const double clen = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        const double theta = atan2(clen, pl[3] * 0.0 + pl[4] * 1.0 + pl[5] * 0.0);
        const double kv[3] = {c[0] / clen, c[1] / clen, c[2] / clen};
        const bool kfin = std::isfinite(kv[0]) && std::isfinite(kv[1]) && std::isfinite(kv[2]);
        dst[12] = theta <= e ? (R)0 : (kfin ? (R)1 : (R)2);
        dst[13] = (R)cos(theta);
        dst[14] = (R)sin(theta);
        for (int q = 0; q < 3; ++q) dst[15 + q] = kfin ? (R)kv[q] : (R)0;
        dst[18] = dst[19] = (R)0;
    }
    for (uint32_t k = 0; k < s->n_planes; ++k) reinterpret_cast<uint32_t*>(b + o_pmat)[k] = s->plane_mat[k];
    // quads: derived in f64; the AABB is rounded outward into R (a cull only)
    auto put_quad = [&](const double* src, R* dst) {
        double q[rtw::kQuadR];
        quad_derive(src, q);
        for (uint32_t a = 0; a < rtw::kQuadR; ++a) dst[a] = (R)q[a];
        for (int a = 0; a < 3; ++a) {
            R lo = (R)q[16 + a], hi = (R)q[19 + a];
            if ((double)lo > q[16 + a]) lo = std::nextafter(lo, (R)-INFINITY);
            if ((double)hi < q[19 + a]) hi = std::nextafter(hi, (R)INFINITY);
            dst[16 + a] = lo;
            dst[19 + a] = hi;
        }
    };
    for (uint32_t k = 0; k < s->n_quads; ++k) {
        put_quad(s->quads + 9 * k, reinterpret_cast<R*>(b + o_quads) + rtw::kQuadR * k);
        reinterpret_cast<uint32_t*>(b + o_qmat)[k] = s->quad_mat[k];
    }
    for (uint32_t k = 0; k < s->n_light_quads; ++k)
        put_quad(s->light_quads + 9 * k, reinterpret_cast<R*>(b + o_lquads) + rtw::kQuadR * k);
    for (uint32_t k = 0; k < s->n_boxes; ++k) {
        double bx[rtw::kBoxR];
        box_derive(s->boxes + 18 * k, bx);
        R* dst = reinterpret_cast<R*>(b + o_boxes) + rtw::kBoxR * k;
        for (uint32_t a = 0; a < rtw::kBoxR; ++a) dst[a] = (R)bx[a];
        auto outward = [&](uint32_t lo_at, uint32_t hi_at) {   // AABBs round outward (culls only)
            for (int a = 0; a < 3; ++a) {
                R lo = (R)bx[lo_at + a], hi = (R)bx[hi_at + a];
                if ((double)lo > bx[lo_at + a]) lo = std::nextafter(lo, (R)-INFINITY);
                if ((double)hi < bx[hi_at + a]) hi = std::nextafter(hi, (R)INFINITY);
                dst[lo_at + a] = lo;
                dst[hi_at + a] = hi;
            }
        };
        outward(rtw::kBoxLo, rtw::kBoxHi);
        for (uint32_t qd = 0; qd < 6; ++qd) outward(rtw::kQuadR * qd + 16, rtw::kQuadR * qd + 19);
        reinterpret_cast<uint32_t*>(b + o_bmat)[k] = s->box_mat[k];
    }
    {
        uint32_t ns = 0, nq = 0;
        for (uint32_t k = 0; k < n_list; ++k) {
            const uint32_t kind = s->light_kinds ? s->light_kinds[k] : (k >= s->n_lights ? 1u : 0u);
            reinterpret_cast<uint32_t*>(b + o_lref)[k] =
                kind == RTW_LIGHT_QUAD ? (rtw::kLrefQuad | nq++) : (kind == RTW_LIGHT_DEFAULT ? rtw::kLrefDefault : ns++);
        }
    }
    if (tex) {
        for (uint32_t k = 0; k < s->n_materials; ++k) reinterpret_cast<uint32_t*>(b + o_mtex)[k] = s->mat_tex[k];
        for (uint32_t k = 0; k < s->n_textures; ++k) {
            const double* tp = s->tex_params + 4 * k;
            reinterpret_cast<uint32_t*>(b + o_ttype)[k] = s->tex_type[k];
            reinterpret_cast<R4*>(b + o_tp)[k] = R4{(R)tp[0], (R)tp[1], (R)tp[2], (R)tp[3]};
            reinterpret_cast<uint32_t*>(b + o_trefs)[2 * k] = s->tex_refs[2 * k];
            reinterpret_cast<uint32_t*>(b + o_trefs)[2 * k + 1] = s->tex_refs[2 * k + 1];
        }
        for (uint32_t k = 0; k < 256 * s->n_perlin; ++k) {
            const double* v = s->perlin_vec + 3 * k;
            reinterpret_cast<R4*>(b + o_pvec)[k] = R4{(R)v[0], (R)v[1], (R)v[2], (R)0};
        }
        for (uint32_t k = 0; k < 768 * s->n_perlin; ++k)
            reinterpret_cast<uint32_t*>(b + o_pperm)[k] = s->perlin_perm[k];
    }
    ds->mat_tex = tex ? reinterpret_cast<const uint32_t*>(base + o_mtex) : nullptr;
    ds->tex_type = reinterpret_cast<const uint32_t*>(base + o_ttype);
    ds->tex_p = reinterpret_cast<const R4*>(base + o_tp);
    ds->tex_refs = reinterpret_cast<const uint32_t*>(base + o_trefs);
    ds->perlin_vec = reinterpret_cast<const R4*>(base + o_pvec);
    ds->perlin_perm = reinterpret_cast<const uint32_t*>(base + o_pperm);
    ds->light_flags = s->light_flags;
    ds->emissive = 0;
    for (uint32_t k = 0; k < s->n_materials; ++k)
        if (s->mat_type[k] == RTW_DIFFUSE_LIGHT) ds->emissive = 1;
    for (uint32_t k = 0; k < s->n_materials; ++k) {
        const double* m = s->mat_params + 5 * k;
        const uint32_t t = s->mat_type[k];
        // the f64 scatter constants of kOptHit64 (dielectric_dir64): Dialectric's
        // index_of_refraction.recip() and reflectance's r0 for both faces, with the
        // reference's operations (material.rs:450-454, 464-468); Metal's fuzz
        double* m64 = reinterpret_cast<double*>(b + o_m64) + 4 * k;
        if (t == RTW_DIELECTRIC) {
            const double ior = m[4], rf = 1.0 / ior;
            const double r0f = (1.0 - rf) / (1.0 + rf), r0b = (1.0 - ior) / (1.0 + ior);
            m64[0] = rf;
            m64[1] = r0f * r0f;
            m64[2] = r0b * r0b;
            m64[3] = ior;
        } else {
            m64[0] = m64[1] = m64[2] = 0.0;
            m64[3] = t == RTW_METAL ? m[3] : 0.0;
        }
        reinterpret_cast<uint32_t*>(b + o_mt)[k] = t;
        const double w = t == RTW_METAL ? m[3] : (t == RTW_DIELECTRIC ? m[4] : 0.0);
        reinterpret_cast<R4*>(b + o_mp)[k] = R4{(R)m[0], (R)m[1], (R)m[2], (R)w};
    }
    for (uint32_t k = 0; k < s->n_lights; ++k) {
        const double* p = s->lights + 4 * k;
        reinterpret_cast<R4*>(b + o_li)[k] = R4{(R)p[0], (R)p[1], (R)p[2], (R)p[3]};
    }
    ds->sph = reinterpret_cast<const R4*>(base + o_sph);
    ds->sph_r = reinterpret_cast<const R*>(base + o_r);
    ds->sph64 = reinterpret_cast<const rtw::R4<double>*>(base + o_s64);
    ds->pl64 = reinterpret_cast<const rtw::R4<double>*>(base + o_pl64);
    ds->mat64 = reinterpret_cast<const rtw::R4<double>*>(base + o_m64);
    ds->sph_mat = reinterpret_cast<const uint32_t*>(base + o_smat);
    ds->sph_shade = reinterpret_cast<const R4*>(base + o_sshade);
    ds->planes = reinterpret_cast<const R*>(base + o_pl);
    ds->plane_mat = reinterpret_cast<const uint32_t*>(base + o_pmat);
    ds->mat_type = reinterpret_cast<const uint32_t*>(base + o_mt);
    ds->mat_p = reinterpret_cast<const R4*>(base + o_mp);
    ds->lights = reinterpret_cast<const R4*>(base + o_li);
    ds->quads = reinterpret_cast<const R*>(base + o_quads);
    ds->quad_mat = reinterpret_cast<const uint32_t*>(base + o_qmat);
    ds->lquads = reinterpret_cast<const R*>(base + o_lquads);
    ds->lref = (s->n_light_quads || s->n_light_other) ? reinterpret_cast<const uint32_t*>(base + o_lref) : nullptr;
    ds->n_quads = s->n_quads;
    ds->n_lquads = s->n_light_quads;
    ds->n_list = n_list;
    ds->boxes = reinterpret_cast<const R*>(base + o_boxes);
    ds->box_mat = reinterpret_cast<const uint32_t*>(base + o_bmat);
    ds->n_boxes = s->n_boxes;
    // round box bounds outward into precision R
    auto down = [](double x) {
        R r = (R)x;
        return (double)r > x ? std::nextafter(r, (R)-INFINITY) : r;
    };
    auto up = [](double x) {
        R r = (R)x;
        return (double)r < x ? std::nextafter(r, (R)INFINITY) : r;
    };
    auto pack_node = [&](const rtw::BvhBuild::Node& n) {
        rtw::BvhNode<R> d{};
        for (int c = 0; c < 2; ++c) {
            d.lo_x[c] = down(n.lo[c][0]);
            d.lo_y[c] = down(n.lo[c][1]);
            d.lo_z[c] = down(n.lo[c][2]);
            d.hi_x[c] = up(n.hi[c][0]);
            d.hi_y[c] = up(n.hi[c][1]);
            d.hi_z[c] = up(n.hi[c][2]);
            d.child[c] = n.child[c];
        }
        return d;
    };
    for (size_t k = 0; k < bb.nodes.size(); ++k)
        reinterpret_cast<rtw::BvhNode<R>*>(b + o_nodes)[k] = pack_node(bb.nodes[k]);
    if constexpr (std::is_same<R, double>::value) {
        auto down32 = [](double x) {
            float r = (float)x;
            return (double)r > x ? std::nextafter(r, -INFINITY) : r;
        };
        auto up32 = [](double x) {
            float r = (float)x;
            return (double)r < x ? std::nextafter(r, INFINITY) : r;
        };
        for (size_t k = 0; k < bb.nodes.size(); ++k) {
            const rtw::BvhBuild::Node& n = bb.nodes[k];
            rtw::BvhNode<float> d{};
            for (int c = 0; c < 2; ++c) {
                d.lo_x[c] = down32(n.lo[c][0]);
                d.lo_y[c] = down32(n.lo[c][1]);
                d.lo_z[c] = down32(n.lo[c][2]);
                d.hi_x[c] = up32(n.hi[c][0]);
                d.hi_y[c] = up32(n.hi[c][1]);
                d.hi_z[c] = up32(n.hi[c][2]);
                d.child[c] = n.child[c];
            }
            reinterpret_cast<rtw::BvhNode<float>*>(b + o_nodes32)[k] = d;
        }
    }
    for (uint32_t k = 0; k < s->n_spheres; ++k) {
        const uint32_t id = bb.order[k];
        const R4 sk = reinterpret_cast<const R4*>(b + o_sph)[id];
        reinterpret_cast<R4*>(b + o_bsph)[k] = sk;
        reinterpret_cast<uint32_t*>(b + o_bid)[k] = id;
        if constexpr (std::is_same<R, double>::value)
            reinterpret_cast<rtw::R4<float>*>(b + o_bsph32)[k] =
                rtw::R4<float>{(float)sk.x, (float)sk.y, (float)sk.z, (float)sk.w};
    }
    // 4-wide tree, one copy per ray octant: slots in that octant's
    // front-to-back order, slab planes pre-selected as near/far (see Bvh4Node)
    const size_t n4 = b4.nodes.size();
    for (int oct = 0; oct < 8; ++oct) {
        for (size_t k = 0; k < n4; ++k) {
            const rtw::Bvh4Build::Node& n = b4.nodes[k];
            rtw::Bvh4Node<R> d{};
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t slot = n.order[oct][q];
                const bool valid = q < n.n;
                R nr[3], fr[3];
                for (int a = 0; a < 3; ++a) {
                    const bool neg = (oct >> a) & 1;
                    const R lo = valid ? down(n.lo[slot][a]) : (R)INFINITY;
                    const R hi = valid ? up(n.hi[slot][a]) : (R)-INFINITY;
                    // a ray going -a enters through hi and leaves through lo;
                    // an empty slot maps to near = +inf, far = -inf in ray space
                    nr[a] = neg ? hi : lo;
                    fr[a] = neg ? lo : hi;
                }
                const int32_t link = valid ? n.child[slot] : rtw::leaf_code(0, 0);
                R lr = 0;   // the link's bits in an R slot (low 32 bits for double)
                if constexpr (sizeof(R) == 4) {
                    memcpy(&lr, &link, 4);
                } else {
                    const int64_t l64 = (int64_t)(uint32_t)link;
                    memcpy(&lr, &l64, 8);
                }
                d.a[q] = rtw::R4<R>{nr[0], nr[1], nr[2], fr[0]};
                d.b[q] = rtw::R4<R>{fr[1], fr[2], lr, (R)0};
            }
            reinterpret_cast<rtw::Bvh4Node<R>*>(b + o_nodes4)[oct * n4 + k] = d;
        }
    }
    for (size_t k = 0; k < lb.nodes.size(); ++k)
        reinterpret_cast<rtw::BvhNode<R>*>(b + o_lnodes)[k] = pack_node(lb.nodes[k]);
    for (uint32_t k = 0; k < s->n_lights; ++k) {
        const uint32_t id = lb.order[k];
        reinterpret_cast<R4*>(b + o_lsph)[k] = reinterpret_cast<const R4*>(b + o_li)[id];
        reinterpret_cast<uint32_t*>(b + o_lid)[k] = id;
    }
    ds->lbvh = reinterpret_cast<const rtw::BvhNode<R>*>(base + o_lnodes);
    ds->lsph = reinterpret_cast<const R4*>(base + o_lsph);
    ds->lid = reinterpret_cast<const uint32_t*>(base + o_lid);
    ds->n_lnodes = (uint32_t)lb.nodes.size();
    ds->lbvh_depth = lb.depth;
    if (!lg.start.empty())
        memcpy(b + o_lgs, lg.start.data(), sizeof(uint32_t) * lg.start.size());
    for (size_t k = 0; k < lg.items.size(); ++k) {
        const uint32_t id = lg.items[k];
        reinterpret_cast<R4*>(b + o_lgsph)[k] = reinterpret_cast<const R4*>(b + o_li)[id];
        reinterpret_cast<uint32_t*>(b + o_lgid)[k] = id;
        if constexpr (std::is_same<R, double>::value) {
            const double* l = s->lights + 4 * (size_t)id;
            reinterpret_cast<rtw::R4<float>*>(b + o_lgsph32)[k] =
                rtw::R4<float>{(float)l[0], (float)l[1], (float)l[2], fabsf((float)l[3])};
        }
    }
    if (n_cells) {   // each cell's lights as the f32 walk reads them (f32: lg_sph; f64: lg_sph32)
        const std::vector<float> rec = rtw::light_grid_records(lg, s->lights, std::is_same<R, double>::value);
        memcpy(b + o_lgrec, rec.data(), sizeof(float) * rec.size());
    }
    ds->lg_rec = reinterpret_cast<const rtw::R4<float>*>(base + o_lgrec);
    ds->lg_start = reinterpret_cast<const uint32_t*>(base + o_lgs);
    ds->lg_sph = reinterpret_cast<const R4*>(base + o_lgsph);
    ds->lg_id = reinterpret_cast<const uint32_t*>(base + o_lgid);
    for (int a = 0; a < 3; ++a) {
        ds->lg_lo[a] = (R)lg.lo[a];
        ds->lg_hi[a] = (R)(lg.lo[a] + lg.n[a] * lg.cell[a]);
        ds->lg_cell[a] = (R)lg.cell[a];
        ds->lg_inv[a] = (R)(1.0 / lg.cell[a]);
        ds->lg_n[a] = lg.n[a];
    }
    ds->lg_big = lg.n_big;
    ds->lg_on = lg.start.empty() ? 0u : 1u;
    ds->bvh4 = reinterpret_cast<const rtw::Bvh4Node<R>*>(base + o_nodes4);
    ds->n_nodes4 = (uint32_t)n4;
    ds->bvh4_stack = b4.max_stack;
    ds->bvh = reinterpret_cast<const rtw::BvhNode<R>*>(base + o_nodes);
    if constexpr (std::is_same<R, double>::value) {
        ds->bvh32 = reinterpret_cast<const rtw::BvhNode<float>*>(base + o_nodes32);
        ds->bsph32 = reinterpret_cast<const rtw::R4<float>*>(base + o_bsph32);
        ds->lg_sph32 = reinterpret_cast<const rtw::R4<float>*>(base + o_lgsph32);
    }
    ds->bsph = reinterpret_cast<const R4*>(base + o_bsph);
    ds->bid = reinterpret_cast<const uint32_t*>(base + o_bid);
    ds->n_sph = s->n_spheres;
    ds->n_planes = s->n_planes;
    ds->n_mat = s->n_materials;
    ds->n_lights = s->n_lights;
    ds->n_nodes = (uint32_t)bb.nodes.size();
    ds->bvh_depth = bb.depth;
    return blob;
}

int validate_scene(rtw_ctx* c, const rtw_scene* s) {
    if (!s) return fail(c, RTW_E_INVALID, "scene is NULL");
    if ((s->n_spheres && (!s->spheres || !s->sphere_mat)) || (s->n_planes && (!s->planes || !s->plane_mat)) ||
        (s->n_materials && (!s->mat_type || !s->mat_params)) || (s->n_lights && !s->lights) ||
        (s->n_quads && (!s->quads || !s->quad_mat)) || (s->n_light_quads && !s->light_quads) ||
        (s->n_boxes && (!s->boxes || !s->box_mat)))
        return fail(c, RTW_E_INVALID, "scene array pointer is NULL");
    const uint32_t n_list = s->n_lights + s->n_light_quads + s->n_light_other;
    if (s->light_kinds) {
        uint32_t cnt[3] = {0, 0, 0};
        for (uint32_t k = 0; k < n_list; ++k) {
            if (s->light_kinds[k] > RTW_LIGHT_DEFAULT) return fail(c, RTW_E_INVALID, "unknown light kind");
            ++cnt[s->light_kinds[k]];
        }
        if (cnt[0] != s->n_lights || cnt[1] != s->n_light_quads || cnt[2] != s->n_light_other)
            return fail(c, RTW_E_INVALID, "light_kinds does not match the light counts");
    } else if (s->n_light_other) {
        return fail(c, RTW_E_INVALID, "n_light_other needs light_kinds");
    }
    if (s->light_flags & ~(uint32_t)RTW_LIGHTS_BVH_LEAF) return fail(c, RTW_E_INVALID, "unknown light_flags");
    if ((s->light_flags & RTW_LIGHTS_BVH_LEAF) && n_list > 5)
        return fail(c, RTW_E_UNSUPPORTED, "a BVH light list of more than 5 entries is not a leaf: the reference's "
                                          "BVH aux_random indexes it inconsistently (bvh.rs:78-92)");
    for (uint32_t k = 0; k < s->n_materials; ++k)
        if (s->mat_type[k] > RTW_DIFFUSE_LIGHT) return fail(c, RTW_E_INVALID, "unknown material type");
    if (s->n_materials >= (1u << 24)) return fail(c, RTW_E_UNSUPPORTED, "more than 2^24 materials");
    if (s->mat_tex) {
        if ((s->n_textures && (!s->tex_type || !s->tex_params || !s->tex_refs)) ||
            (s->n_perlin && (!s->perlin_vec || !s->perlin_perm)))
            return fail(c, RTW_E_INVALID, "texture array pointer is NULL");
        for (uint32_t k = 0; k < s->n_materials; ++k)
            if (s->mat_tex[k] >= s->n_textures) return fail(c, RTW_E_INVALID, "material texture id out of range");
        for (uint32_t k = 0; k < s->n_textures; ++k) {
            const uint32_t t = s->tex_type[k];
            if (t > RTW_TEX_NOISE) return fail(c, RTW_E_INVALID, "unknown texture type");
            if (t == RTW_TEX_CHECKER && (s->tex_refs[2 * k] >= s->n_textures || s->tex_refs[2 * k + 1] >= s->n_textures))
                return fail(c, RTW_E_INVALID, "checker texture id out of range");
            if (t == RTW_TEX_NOISE && s->tex_refs[2 * k] >= s->n_perlin)
                return fail(c, RTW_E_INVALID, "noise texture Perlin table id out of range");
        }
        // nested checkers must bottom out (the reference's Arc<dyn Texture> tree)
        for (uint32_t k = 0; k < s->n_textures; ++k) {
            std::vector<uint32_t> stack{k};
            uint32_t steps = 0;
            while (!stack.empty()) {
                const uint32_t t = stack.back();
                stack.pop_back();
                if (++steps > 4096) return fail(c, RTW_E_INVALID, "checker textures form a cycle or are too deep");
                if (s->tex_type[t] == RTW_TEX_CHECKER) {
                    stack.push_back(s->tex_refs[2 * t]);
                    stack.push_back(s->tex_refs[2 * t + 1]);
                }
            }
        }
        for (uint32_t k = 0; k < 768 * s->n_perlin; ++k)
            if (s->perlin_perm[k] > 255) return fail(c, RTW_E_INVALID, "Perlin permutation entry > 255");
    }
    for (uint32_t k = 0; k < s->n_spheres; ++k)
        if (s->sphere_mat[k] >= s->n_materials) return fail(c, RTW_E_INVALID, "sphere material id out of range");
    for (uint32_t k = 0; k < s->n_planes; ++k)
        if (s->plane_mat[k] >= s->n_materials) return fail(c, RTW_E_INVALID, "plane material id out of range");
    for (uint32_t k = 0; k < s->n_quads; ++k)
        if (s->quad_mat[k] >= s->n_materials) return fail(c, RTW_E_INVALID, "quad material id out of range");
    for (uint32_t k = 0; k < s->n_boxes; ++k)
        if (s->box_mat[k] >= s->n_materials) return fail(c, RTW_E_INVALID, "box material id out of range");
    return RTW_OK;
}

int ensure(rtw_ctx* c, void** buf, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return RTW_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    HIP_TRY(c, hipMalloc(buf, bytes));
    *cap = bytes;
    return RTW_OK;
}

uint64_t n_tiles_of(uint32_t W, uint32_t H) {
    return (uint64_t)((W + rtw::kTile - 1) / rtw::kTile) * ((H + rtw::kTile - 1) / rtw::kTile);
}

// a split is set for renders of this image size and rank count
bool split_active(const rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks) {
    return !c->split_rank.empty() && c->split_W == W && c->split_H == H && c->split_n == nranks;
}
// the id of the split renders of (W, H, nranks) follow: 0 = the round robin
uint64_t split_id(const rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks) {
    return split_active(c, W, H, nranks) ? c->split_serial : 0;
}

// the global tiles of `rank`, in the order they are packed (increasing T)
void local_tiles(const rtw_ctx* c, uint32_t W, uint32_t H, uint32_t rank, uint32_t nranks,
                 std::vector<uint32_t>& out) {
    out.clear();
    const uint64_t n = n_tiles_of(W, H);
    if (split_active(c, W, H, nranks)) {
        for (uint64_t T = 0; T < n; ++T)
            if (c->split_rank[T] == rank) out.push_back((uint32_t)T);
    } else {
        for (uint64_t T = rank; T < n; T += nranks) out.push_back((uint32_t)T);
    }
}

// pixels inside the image of the rank's tiles
uint64_t rank_pixels(const rtw_ctx* c, uint32_t W, uint32_t H, uint32_t rank, uint32_t nranks) {
    const uint32_t tiles_x = (W + rtw::kTile - 1) / rtw::kTile;
    std::vector<uint32_t> tiles;
    local_tiles(c, W, H, rank, nranks, tiles);
    uint64_t px = 0;
    for (uint32_t T : tiles) {
        const uint32_t tx = T % tiles_x, ty = T / tiles_x;
        px += (uint64_t)std::min(rtw::kTile, W - tx * rtw::kTile) * std::min(rtw::kTile, H - ty * rtw::kTile);
    }
    return px;
}

// The device copy of a buffer the kernels read (the split's maps): rewritten
// only when the split changes, after the device is idle -- a render still
// queued on another stream may read the old contents.
int upload_map(rtw_ctx* c, void** buf, size_t* cap, const std::vector<uint32_t>& h) {
    HIP_TRY(c, hipDeviceSynchronize());
    int rc = ensure(c, buf, cap, std::max<size_t>(h.size(), 1) * sizeof(uint32_t));
    if (rc) return rc;
    if (!h.empty()) HIP_TRY(c, hipMemcpy(*buf, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return RTW_OK;
}

// this rank's local tile -> global tile map of the active split on the device
int ensure_tile_map(rtw_ctx* c, uint32_t W, uint32_t H, uint32_t rank, uint32_t nranks) {
    if (c->d_tile_map && c->tile_map_key == c->split_serial && c->tile_map_rank == rank) return RTW_OK;
    local_tiles(c, W, H, rank, nranks, c->h_tile_map);
    const int rc = upload_map(c, &c->d_tile_map, &c->tile_map_cap, c->h_tile_map);
    if (rc) return rc;
    c->tile_map_key = c->split_serial;
    c->tile_map_rank = rank;
    return RTW_OK;
}

// the assembly's map of the active split: global tile T -> lt * n + rank (the
// round robin's own index form, so the assembly kernel decodes both alike)
int ensure_tile_slot(rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks) {
    if (c->d_tile_slot && c->tile_slot_key == c->split_serial) return RTW_OK;
    std::vector<uint32_t> slot(n_tiles_of(W, H));
    std::vector<uint32_t> next(nranks, 0);
    for (size_t T = 0; T < slot.size(); ++T) {
        const uint32_t k = c->split_rank[T];
        slot[T] = next[k]++ * nranks + k;
    }
    const int rc = upload_map(c, &c->d_tile_slot, &c->tile_slot_cap, slot);
    if (rc) return rc;
    c->tile_slot_key = c->split_serial;
    return RTW_OK;
}

template <typename R>
void fill_camera(rtw::KParams<R>& p, const rtw_camera* cam) {
    for (int k = 0; k < 3; ++k) {
        p.center[k] = (R)cam->center[k];
        p.p00[k] = (R)cam->pixel00_loc[k];
        p.du[k] = (R)cam->pixel_delta_u[k];
        p.dv[k] = (R)cam->pixel_delta_v[k];
        p.disk_u[k] = (R)cam->defocus_disk_u[k];
        p.disk_v[k] = (R)cam->defocus_disk_v[k];
        p.bg[k] = (R)cam->background[k];
    }
    // Uniform::new_inclusive(-0.5, 0.5) scale (rand 0.8.6)
    double max_rand = 1.0 - 2.220446049250313080847e-16;
    double scale = (0.5 - -0.5) / max_rand;
    while (scale * max_rand + -0.5 > 0.5) scale = nextafter(scale, 0.0);
    p.u_scale = (R)scale;
    p.defocus = cam->defocus_angle > 2.220446049250313080847e-16 ? 1u : 0u;
    p.W = cam->image_width;
    p.H = cam->image_height;
    p.spp = cam->samples_per_pixel;
    p.max_depth = cam->max_depth;
}

// The tile costs counted by the last counting render (lpt_pending) -> h_lpt_cost
// (waits for that render: once per key)
int lpt_readback(rtw_ctx* c, uint32_t nt) {
    c->lpt_pending = false;   // (an error below recounts at the next render)
    HIP_TRY(c, hipEventSynchronize(c->lpt_ev));
    c->h_lpt_cost.resize(nt);
    // on the context's own (idle, non-blocking) stream: waits for nothing but the copy
    if (nt) {
        HIP_TRY(c, hipMemcpyAsync(c->h_lpt_cost.data(), c->d_lpt, (size_t)nt * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->lpt_valid = true;
    return RTW_OK;
}

// the context holds (or has pending) tile costs of this camera, scene, rank and split
bool lpt_has(const rtw_ctx* c, const rtw_camera* cam, uint32_t rank, uint32_t nranks) {
    return (c->lpt_valid || c->lpt_pending) && c->lpt_serial == c->scene_serial && c->lpt_rank == rank &&
           c->lpt_nranks == nranks && c->lpt_prec == (c->precision == RTW_F32 ? 4u : 8u) &&
           c->lpt_split == split_id(c, cam->image_width, cam->image_height, nranks) &&
           memcmp(&c->lpt_cam, cam, sizeof *cam) == 0;
}

// Longest tiles first: a 2-sample-per-pixel pilot render of the rank's tiles
// counts each tile's segments (h_lpt_cost); lpt_tasks turns them into the task
// list.  Blocking (reads the counts back); cached by the caller.
template <typename R>
int lpt_pilot(rtw_ctx* c, const rtw::KParams<R>& p, int world, size_t launch_lds, hipStream_t stream) {
    const uint32_t nt = p.n_local_tiles;
    rtw::KParams<R> q = p;
    q.spp = std::min(p.spp, std::max(c->lpt_pilot_spp, 1u));
    if (c->lpt_pilot_depth) q.max_depth = std::min(p.max_depth, c->lpt_pilot_depth);
    q.chunk = 1;
    q.n_chunks = q.spp;
    q.group = q.n_chunks;
    q.n_groups = 1;
    q.n_tasks = nt;
    q.seed = p.seed ^ 0x5851F42D4C957F2Dull;
    q.task_table = nullptr;
    const size_t words = align_up((size_t)nt, 64);
    const size_t tile_bytes = (size_t)nt * 64 * 3 * sizeof(R);
    const size_t bytes = words * sizeof(uint32_t) + (size_t)q.n_chunks * tile_bytes + tile_bytes;
    int rc = ensure(c, &c->d_lpt, &c->lpt_cap, bytes);
    if (rc) return rc;
    uint32_t* d_cost = reinterpret_cast<uint32_t*>(c->d_lpt);
    R* d_part = reinterpret_cast<R*>(d_cost + words);
    R* d_pout = d_part + (size_t)q.n_chunks * nt * 64 * 3;
    q.partial = d_part;
    q.tile_cost = d_cost;
    q.cost_spp = q.spp;
    q.cost_time = c->cost_time;
    HIP_TRY(c, hipMemsetAsync(d_cost, 0, (size_t)nt * sizeof(uint32_t), stream));
    HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, rtw_ctx::kCounters * sizeof(unsigned long long), stream));
    int lrc;
    if constexpr (std::is_same<R, float>::value) lrc = rtw::launch_render_f32(q, world, launch_lds, d_pout, stream, nullptr);
    else lrc = rtw::launch_render_f64(q, world, launch_lds, d_pout, stream, nullptr);
    if (lrc < 0) return fail(c, RTW_E_DEVICE, std::string("pilot launch failed: ") + hipGetErrorString(hipGetLastError()));
    c->h_lpt_cost.resize(nt);
    HIP_TRY(c, hipMemcpyAsync(c->h_lpt_cost.data(), d_cost, (size_t)nt * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    HIP_TRY(c, hipStreamSynchronize(stream));
    return RTW_OK;
}

// The task list from the pilot's tile costs: tiles longest first (ties by
// index), each cut into tasks of g chunks.  With the auto task size, g is
// sized per tile so that tasks cost about the same (total cost / target
// tasks, 1..kMaxGroup chunks): a tile whose every sample bounces max_depth
// times (a glass sphere's interior) gets 1-chunk tasks and no task outlasts
// the launch's tail; cheap tiles (sky) get long ones, fewer task switches.
// Only the order and cut of tasks change: every item is still one (pixel,
// chunk) folded in sample order by the reduce, the image is the same bit for
// bit.  Entry: {local tile, first chunk | chunks << 20}.
template <typename R>
int lpt_tasks(rtw_ctx* c, const rtw::KParams<R>& p, uint32_t fixed_group, uint64_t target, hipStream_t stream) {
    const uint32_t nt = p.n_local_tiles;
    const std::vector<uint32_t>& cost = c->h_lpt_cost;
    std::vector<uint32_t> order(nt);
    for (uint32_t k = 0; k < nt; ++k) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
    double total = 0;
    for (uint32_t k = 0; k < nt; ++k) total += std::max<uint32_t>(cost[k], 1);
    const double per_task = total * p.n_chunks / (double)std::max<uint64_t>(target, 1);   // pilot-cost units x chunks
    std::vector<uint32_t>& tab = c->h_lpt_tasks;
    tab.clear();
    if (!fixed_group && c->guide_div) {
        // Guided sizes (guided self-scheduling): each task costs about the work
        // still left after it / guide_div (~ 2 x the resident waves), between
        // total / guide_floor and guide_max chunks.  The launch starts on large
        // tasks (few task switches: a wave's lanes then stay on one tile) and
        // ends on small ones, so the waves run dry together: an 8-rank C2
        // share's equal-cost 2^17 tasks left 3.4 % of its wave-time idle at the
        // end and switched tasks 32 times per wave (profiles/r06a_timeline_*).
        double remaining = total * p.n_chunks;
        const double floor_cost = total * p.n_chunks / (double)std::max<uint64_t>(c->guide_floor, 1);
        const uint32_t gmax = std::min<uint32_t>(std::max(c->guide_max, 1u), kTaskMaxChunks);
        for (uint32_t k : order) {
            const double ck = (double)std::max<uint32_t>(cost[k], 1);
            for (uint32_t cb = 0; cb < p.n_chunks;) {
                const double want = std::max(remaining / (double)c->guide_div, floor_cost) / ck;
                uint32_t g = (uint32_t)std::max(1.0, std::min((double)gmax, std::floor(want + 0.5)));
                g = std::min(g, p.n_chunks - cb);
                tab.push_back(k);
                tab.push_back(cb | (g << 20));
                cb += g;
                remaining -= g * ck;
            }
        }
    }
    for (uint32_t k : order) {
        if (!fixed_group && c->guide_div) break;
        uint32_t g = fixed_group;
        if (!g) {
            const double want = per_task / (double)std::max<uint32_t>(cost[k], 1);
            g = (uint32_t)std::max(1.0, std::min((double)std::max(c->max_group, 1u), std::floor(want + 0.5)));
        }
        // the entry holds the chunk count in 12 bits (first chunk < 2^20 in the low 20)
        g = std::min(std::min(g, p.n_chunks), kTaskMaxChunks);
        for (uint32_t cb = 0; cb < p.n_chunks; cb += g) {
            tab.push_back(k);
            tab.push_back(cb | (std::min(g, p.n_chunks - cb) << 20));
        }
    }
    int rc = ensure(c, &c->d_lpt_tasks, &c->lpt_tasks_cap, tab.size() * sizeof(uint32_t));
    if (rc) return rc;
    HIP_TRY(c, hipMemcpyAsync(c->d_lpt_tasks, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    HIP_TRY(c, hipStreamSynchronize(stream));
    return RTW_OK;
}

template <typename R>
int render_device_t(rtw_ctx* c, const rtw_camera* cam, uint64_t seed, uint32_t rank, uint32_t nranks,
                    void* d_out, size_t out_bytes, hipStream_t stream) {
    rtw::KParams<R> p{};
    p.sc = *reinterpret_cast<const rtw::DevScene<R>*>(
        std::is_same<R, float>::value ? (const void*)&c->sc32 : (const void*)&c->sc64);
    fill_camera(p, cam);
    // the kernel holds a lane's pixel as i | j << 16
    if (p.W > 65535 || p.H > 65535) return fail(c, RTW_E_UNSUPPORTED, "image width or height beyond 65535");
    p.seed = seed;
    p.rank = rank;
    p.nranks = nranks;
    p.tiles_x = (p.W + rtw::kTile - 1) / rtw::kTile;
    p.n_local_tiles = rtw_tiles_for_rank(p.W, p.H, rank, nranks);
    const size_t need_out = (size_t)p.n_local_tiles * 64 * 3 * sizeof(R);
    if (out_bytes < need_out) return fail(c, RTW_E_INVALID, "d_out is smaller than tiles_for_rank*64*3");
    if (need_out && !d_out) return fail(c, RTW_E_INVALID, "d_out is NULL");
    // the split's local -> global tile map (a dealt split; null: the round robin)
    const bool split = split_active(c, p.W, p.H, nranks);
    const uint64_t sid = split_id(c, p.W, p.H, nranks);
    p.tile_map = nullptr;
    if (split && p.n_local_tiles) {
        const int mrc = ensure_tile_map(c, p.W, p.H, rank, nranks);
        if (mrc) return mrc;
        p.tile_map = reinterpret_cast<const uint32_t*>(c->d_tile_map);
    }
    // Work decomposition: ITEM = (pixel, chunk of `chunk` samples) -- the unit
    // a lane folds in sample order; TASK = (8x8 tile, group of chunks) -- one
    // wavefront's dynamic item pool.  Small chunks balance the lanes of a
    // wave; enough tasks keep the dispatcher fed to the end of the launch.
    uint32_t chunk = c->chunk ? c->chunk : c->auto_chunk;
    const size_t per_chunk = (size_t)p.n_local_tiles * 64 * 3 * sizeof(R);
    if (!c->chunk && p.spp) {
        // keep the chunk sums within partial_max and half the device's memory
        // (deterministic: the chunk, and so the fold order, never depends on
        // what else holds memory): bytes = ceil(spp/chunk) * tiles * 64 * 3 * sizeof(R)
        size_t pmax = c->partial_max;
        if (!c->dev_total) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess) c->dev_total = tot;
        }
        if (c->dev_total) pmax = std::min(pmax, c->dev_total / 2);
        const size_t max_chunks = std::max<size_t>(1, pmax / std::max<size_t>(per_chunk, 1));
        while ((p.spp + chunk - 1) / chunk > max_chunks) ++chunk;
    }
    chunk = std::max<uint32_t>(1, std::min<uint32_t>(chunk, std::max<uint32_t>(p.spp, 1)));
    // the chunk-sum buffer; when the device cannot hold it (other allocations)
    // an auto chunk doubles instead of failing -- stats.chunk reports it, the
    // fold is then chunk-associated (rounding level)
    for (;;) {
        const uint32_t nc = p.spp ? (p.spp + chunk - 1) / chunk : 0;
        const size_t bytes = std::max<size_t>((size_t)nc * per_chunk, 64);
        if (c->partial_cap >= bytes) break;
        if (c->d_partial) (void)hipFree(c->d_partial);
        c->d_partial = nullptr;
        c->partial_cap = 0;
        const hipError_t e = hipMalloc(&c->d_partial, bytes);
        if (e == hipSuccess) { c->partial_cap = bytes; break; }
        c->d_partial = nullptr;
        (void)hipGetLastError();
        if (c->chunk || chunk >= p.spp || e != hipErrorOutOfMemory) return hip_fail(c, e, "hipMalloc(chunk sums)");
        chunk = std::min<uint32_t>(chunk * 2, p.spp);
    }
    p.chunk = chunk;
    p.n_chunks = p.spp ? (p.spp + chunk - 1) / chunk : 0;
    uint32_t group = c->group;
    if (group == 0) {
        // Persistent waves (default) have no per-task drain; a task boundary
        // mixes two tiles' items in the wave (less coherent), the launch's tail
        // grows with the task size.  Longest tiles first leaves cheap tiles
        // for the end, so ~2^17 tasks (~32 per resident wave): C2 split over
        // 1 / 2 / 4 / 8 ranks -> 32 / 28 / 15 / 8 chunks per task (N = 1:
        // group 32 93.7 ms vs 16 94.4, 4 104.4; an 8-way share: 8 13.2 ms vs
        // 4 13.6).  One task per wave instead pays a drain per task: ~2^17.
        constexpr uint32_t kMinAutoGroup = 4, kMaxAutoGroup = 32;
        const uint64_t target = c->target_tasks ? c->target_tasks : kAutoTasks;
        const uint64_t n_groups = p.n_local_tiles ? (target + p.n_local_tiles - 1) / p.n_local_tiles : 1;
        group = (uint32_t)((p.n_chunks + n_groups - 1) / std::max<uint64_t>(n_groups, 1));
        group = std::max(kMinAutoGroup, std::min(group, kMaxAutoGroup));
    }
    // at most 4096 chunks per task: the kernel divides item indices q < 64 * group
    // by the group with a multiply-high by ceil(2^32 / group), exact while 64 group^2 < 2^32
    p.group = std::max<uint32_t>(1, std::min<uint32_t>(std::min<uint32_t>(group, 4096u), std::max<uint32_t>(p.n_chunks, 1)));
    p.n_groups = p.n_chunks ? (p.n_chunks + p.group - 1) / p.group : 0;
    p.n_tasks = p.n_local_tiles * p.n_groups;
    p.item_order = c->item_order;
    p.persist = c->persist;
    int rc = RTW_OK;
    p.partial = reinterpret_cast<R*>(c->d_partial);
    p.counters = c->d_counters;
    HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, rtw_ctx::kCounters * sizeof(unsigned long long), stream));
    const size_t lds = (size_t)(p.sc.n_sph + p.sc.n_lights) * sizeof(rtw::R4<R>);
    int accel = c->accel == RTW_ACCEL_AUTO ? c->auto_accel : c->accel;
    if (accel == RTW_ACCEL_AUTO) accel = p.sc.n_sph >= 64 ? RTW_ACCEL_BVH : RTW_ACCEL_BRUTE;
    int world = (c->world_pref == 0 || lds > kLdsLimit) ? rtw::kWorldGlobal : rtw::kWorldLds;
    p.stack = rtw::kBvhStack;
    uint32_t bvh_width = 0;
    size_t launch_lds = lds;
    // f32 sphere/light tests: the reference's hb^2 - a c loses r^2 to
    // rounding once (distance / radius)^2 * 2^-24 is no longer small (C3/C5
    // seen from afar); the closest-approach form is then used.
    {
        const double far = std::max(c->scene_extent, sqrt((double)p.center[0] * p.center[0] +
                                                          (double)p.center[1] * p.center[1] +
                                                          (double)p.center[2] * p.center[2]));
        const double rel = std::isfinite(c->min_radius) ? (far / c->min_radius) * (far / c->min_radius) * 5.96e-8
                                                        : 0.0;
        p.sc.robust = c->robust == 2 ? (rel > 1e-3 ? 1u : 0u) : (uint32_t)c->robust;
    }
    p.light_bvh = 0;
    if (accel == RTW_ACCEL_BVH) {
        // the light pdf goes through the light BVH (same per-lane stack) for
        // longer light lists
        const uint32_t light_stack = p.sc.lbvh_depth + 1;
        if (p.sc.n_lights >= c->light_bvh_min && p.sc.n_lquads == 0) {
            if (p.sc.lg_on) p.light_bvh = 2;                          // light grid
            else if (light_stack <= rtw::kBvhStack) p.light_bvh = 1;  // light BVH
        }
        // the light grid's cooperative walk parks path state in the stack area
        // (f64: one kCoop64Slot-word slot per piece of the walk -- [count, list
        // indices] -- after the kCoopStash64-word stash: 64 pieces per round)
        const uint32_t min_stack = p.light_bvh == 1 ? light_stack
                                   : (p.light_bvh == 2 ? (sizeof(R) == 8 ? rtw::kCoopStash64 + rtw::kCoop64Slot
                                                                         : rtw::kCoopStash + 1u)
                                                       : 1u);
        // binary traversal pushes at most one entry per inner level: a leaf at
        // level `bvh_depth` has that many inner nodes above it (host/bvh.cpp)
        const uint32_t bin_stack = std::max(p.sc.bvh_depth, min_stack);
        // kWorldBvhLds layout: stacks + stealing area (+ light-work counters) (traversal_lds) | f32 nodes
        // (bvh32) | leaf spheres | ids (padded to 8) | lights | (f32) light pairs | (f64) the lights rounded to f32
        // wide workgroups (rtw_kernels.h block_waves): the f64 kernel of sphere + plane
        // scenes with a linear light list -- 16 waves share one copy, which then also
        // holds the f64 leaf spheres (32 B each, 32-B aligned)
        const bool wide = sizeof(R) == 8 && p.light_bvh == 0 && !p.sc.mat_tex &&
                          !(p.sc.n_quads || p.sc.n_boxes || p.sc.lref || p.sc.emissive) &&
                          rtw::block_waves(true) == rtw::kWavesWide;
        const uint32_t block_waves = rtw::block_waves(wide);
        const size_t tree_lds = rtw::traversal_lds<R>(bin_stack, p.light_bvh != 0, block_waves) +
                                (wide ? 32 + (RTW_WIDE_SPH64 ? 2 : 1) * (size_t)p.sc.n_sph * sizeof(rtw::R4<double>) : 0) +
                                (size_t)p.sc.n_nodes * sizeof(rtw::BvhNode<float>) +
                                (size_t)p.sc.n_sph * sizeof(rtw::R4<float>) +
                                (size_t)((p.sc.n_sph + 7u) & ~7u) * sizeof(uint32_t) +
                                (sizeof(R) == 8 ? 32 : 0) +   // (f64: the light list 32-B aligned)
                                (size_t)p.sc.n_lights * sizeof(rtw::R4<R>) +
                                // f32: the light pairs of the packed light test; f64: the
                                // lights rounded to f32 for the pre-pass (16 B each)
                                (sizeof(R) == 4 ? (size_t)((p.sc.n_lights + 1u) & ~1u) * sizeof(rtw::R4<R>)
                                                : (size_t)p.sc.n_lights * sizeof(rtw::R4<float>));
        if (c->bvh_kind == 2 && p.sc.bvh4_stack + 1 <= rtw::kBvhStack) {
            world = rtw::kWorldBvh4;       // 4-wide, when its stack bound fits
            p.stack = std::max(p.sc.bvh4_stack + 1, min_stack);
            bvh_width = 4;
        } else if (p.sc.bvh_depth <= rtw::kBvhStack && min_stack <= rtw::kWalkStashMax) {
            // the tree bounds the traversal stack; the light grid's walk may ask
            // for a larger per-lane area (its LDS stash + piece slots)
            p.stack = bin_stack;
            bvh_width = 2;
            // (4-wave workgroups: four copies per CU; wide: one workgroup per CU, which may
            // take all of its 160 KiB -- the C2 scene needs 110, ~900 spheres fit)
            const size_t lds_max = c->bvh_lds_max ? c->bvh_lds_max
                                                  : (sizeof(R) == 4 ? 36 * 1024 : (wide ? kLdsLimit : 52 * 1024));
            if (c->bvh_kind == 3 && tree_lds <= lds_max) {
                world = rtw::kWorldBvhLds;
                launch_lds = tree_lds;
            } else {
                world = c->bvh_kind ? rtw::kWorldBvhWW : rtw::kWorldBvh;
            }
        } else {
            return fail(c, RTW_E_UNSUPPORTED, "BVH deeper than the kernel's traversal stack");
        }
    }
    // textured scenes have kernels for the brute-force and binary while-while worlds only
    if (p.sc.mat_tex && (world == rtw::kWorldBvh4 || world == rtw::kWorldBvh)) {
        world = rtw::kWorldBvhWW;
        bvh_width = 2;
        // Textured kernels carry kOptPrims, so their light-grid walk is the
        // per-lane one (no cooperative walk, no stash or piece slots): only the
        // light BVH's walk uses the per-lane stack
        p.stack = std::max(p.sc.bvh_depth, p.light_bvh == 1 ? p.sc.lbvh_depth + 1 : 1u);
        if (p.stack > rtw::kBvhStack) return fail(c, RTW_E_UNSUPPORTED, "BVH deeper than the kernel's traversal stack");
    }
    // f64 hit points: the f32 kernels of sphere + plane scenes (the launch
    // routes textured / quad / cuboid scenes to kernels without them)
    p.hit64 = c->hit64 ? 1u : 0u;
    // auto: walks that cross the whole grid in few pieces give the wave little to
    // share, short ones pay each piece's setup: f32, a fourteenth of the grid's
    // widest side, 4..16 cells (at the default 1/2 cell per light: C3, ~16 cells
    // wide: 4; C5, 158 wide: 11); f64, whose pieces also carry the list-order
    // merge, a seventh, 4..24 (C3 4, C5 22: C5 3249 -> 3133 ms, C3 unchanged;
    // profiles/r04_w_grid_piece_sweep.jsonl)
    const uint32_t grid_w = std::max(p.sc.lg_n[0], std::max(p.sc.lg_n[1], p.sc.lg_n[2]));
    // r05: the f64 walk runs in f32 too, but each piece also keeps and merges
    // candidate list indices: 16..24 cells, the longest a trip may cut (pieces
    // are sized per trip below it: C3 16 vs 11: 554 -> 546 ms at half spp; C5
    // 22; profiles/r05_piece_sweep.jsonl, r05_piece_sweep_final.jsonl)
    p.grid_piece = c->grid_piece != rtw_ctx::kGridPieceAuto
                       ? c->grid_piece
                       : (sizeof(R) == 8 ? std::max(16u, std::min(24u, grid_w / 7u))
                                         : std::max(4u, std::min(16u, grid_w / 14u)));
    p.task_table = nullptr;
    p.tile_cost = nullptr;
    p.cost_spp = 0;
    p.cost_time = 0;
    // Reordering the tiles scatters the tiles in flight over the image: a tree
    // larger than an XCD's L2 (4 MiB) loses its locality (C5, 1M spheres,
    // ~100 MB: +8 %), so by default only worlds held in LDS or small enough
    // for L2 take it (C2: -4 %, C3 (10k spheres): -4 %).
    const bool on_chip = world == rtw::kWorldBvhLds || world == rtw::kWorldLds || c->tree_bytes <= (4u << 20);
    if ((c->lpt == 2 || (c->lpt == 1 && on_chip)) && need_out && p.spp >= std::max(c->lpt_min_spp, 1u) &&
        p.max_depth && p.n_local_tiles > 1 && p.n_chunks < (1u << 20)) {
        const bool same = (c->lpt_valid || c->lpt_pending) && c->lpt_serial == c->scene_serial &&
                          c->lpt_rank == rank && c->lpt_nranks == nranks && c->lpt_prec == (uint32_t)sizeof(R) &&
                          c->lpt_split == sid && memcmp(&c->lpt_cam, cam, sizeof *cam) == 0;
        const bool dbg = getenv("RTW_DEBUG_LPT") != nullptr;   // cold-render cost breakdown (stderr)
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto t0 = now();
        auto keep_key = [&] {
            c->lpt_cam = *cam;
            c->lpt_serial = c->scene_serial;
            c->lpt_rank = rank;
            c->lpt_nranks = nranks;
            c->lpt_prec = (uint32_t)sizeof(R);
            c->lpt_split = sid;
        };
        if (!same && split && !c->split_cost.empty()) {
            // a split dealt by tile costs: those costs order this rank's tasks (no counting)
            c->lpt_pending = false;
            c->lpt_tab_valid = false;
            c->h_lpt_cost.resize(p.n_local_tiles);
            for (uint32_t k = 0; k < p.n_local_tiles; ++k) c->h_lpt_cost[k] = c->split_cost[c->h_tile_map[k]];
            c->lpt_valid = true;
            keep_key();
        } else if (!same && c->lpt_inline) {
            // this render counts its tiles' costs on the way (plain tile order);
            // the key is kept and the counts marked pending only once lpt_ev is
            // recorded after the launch (below), so a failed launch leaves no
            // pending state behind
            c->lpt_valid = c->lpt_pending = false;
            c->lpt_tab_valid = false;
            const uint32_t nt = p.n_local_tiles;
            // a counting render of an earlier key may still run on another stream:
            // the counters are reused only after it
            if (c->lpt_ev) HIP_TRY(c, hipStreamWaitEvent(stream, c->lpt_ev, 0));
            rc = ensure(c, &c->d_lpt, &c->lpt_cap, align_up((size_t)nt, 64) * sizeof(uint32_t));
            if (rc) return rc;
            HIP_TRY(c, hipMemsetAsync(c->d_lpt, 0, (size_t)nt * sizeof(uint32_t), stream));
            p.tile_cost = reinterpret_cast<uint32_t*>(c->d_lpt);
            p.cost_spp = std::min(p.spp, std::max(c->lpt_pilot_spp, 1u));
            p.cost_time = c->cost_time;
        } else if (!same) {
            c->lpt_valid = c->lpt_pending = false;
            c->lpt_tab_valid = false;
            rc = lpt_pilot(c, p, world, launch_lds, stream);
            if (dbg) fprintf(stderr, "lpt pilot %.3f ms (%u tiles)\n",
                             std::chrono::duration<double, std::milli>(now() - t0).count(), p.n_local_tiles);
            t0 = now();
            if (rc) return rc;
            c->lpt_valid = true;
            keep_key();
            HIP_TRY(c, hipMemsetAsync(c->d_counters, 0, rtw_ctx::kCounters * sizeof(unsigned long long), stream));
        } else if (c->lpt_pending) {
            // the counts of the render before (waits for it: once per key)
            rc = lpt_readback(c, p.n_local_tiles);
            if (rc) return rc;
            if (dbg) fprintf(stderr, "lpt counts read back %.3f ms (%u tiles)\n",
                             std::chrono::duration<double, std::milli>(now() - t0).count(), p.n_local_tiles);
            t0 = now();
        }
        const uint64_t target = c->target_tasks ? c->target_tasks : kAutoTasks;
        if (c->lpt_valid && (!c->lpt_tab_valid || c->lpt_tab_chunks != p.n_chunks || c->lpt_tab_group != c->group ||
            c->lpt_tab_target != target)) {
            c->lpt_tab_valid = false;
            rc = lpt_tasks(c, p, c->group ? p.group : 0u, target, stream);
            if (rc) return rc;
            if (dbg) fprintf(stderr, "lpt tasks %.3f ms (%zu tasks)\n",
                             std::chrono::duration<double, std::milli>(now() - t0).count(), c->h_lpt_tasks.size() / 2);
            c->lpt_tab_valid = true;
            c->lpt_tab_chunks = p.n_chunks;
            c->lpt_tab_group = c->group;
            c->lpt_tab_target = target;
        }
        if (c->lpt_valid) {
            p.task_table = reinterpret_cast<const uint32_t*>(c->d_lpt_tasks);
            p.n_tasks = (uint32_t)(c->h_lpt_tasks.size() / 2);
        }
    }
    hipEvent_t* ev = c->ring[c->n_renders % rtw_ctx::kRing];
    HIP_TRY(c, hipEventRecord(c->ev0, stream));
    HIP_TRY(c, hipEventRecord(ev[0], stream));
    int lrc = 0;
    if (need_out == 0) {
        HIP_TRY(c, hipEventRecord(ev[1], stream));
    } else if (p.spp == 0 || p.max_depth == 0) {
        // depth == 0: every sample is Colour::default() + res = 0 (camera.rs:470-472)
        HIP_TRY(c, hipMemsetAsync(d_out, 0, need_out, stream));
        HIP_TRY(c, hipEventRecord(ev[1], stream));
    } else if constexpr (std::is_same<R, float>::value) {
        lrc = rtw::launch_render_f32(p, world, launch_lds, reinterpret_cast<float*>(d_out), stream, ev[1]);
    } else {
        lrc = rtw::launch_render_f64(p, world, launch_lds, reinterpret_cast<double*>(d_out), stream, ev[1]);
    }
    if (lrc < 0) return fail(c, RTW_E_DEVICE, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    c->last_variant = lrc;
    if (p.tile_cost) {   // the counts are complete after this render
        if (!c->lpt_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->lpt_ev, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->lpt_ev, stream));
        c->lpt_cam = *cam;   // read back by the next render of the same key (after lpt_ev)
        c->lpt_serial = c->scene_serial;
        c->lpt_rank = rank;
        c->lpt_nranks = nranks;
        c->lpt_prec = (uint32_t)sizeof(R);
        c->lpt_split = sid;
        c->lpt_pending = true;
    }
    HIP_TRY(c, hipEventRecord(c->ev1, stream));
    HIP_TRY(c, hipEventRecord(ev[2], stream));
    ++c->n_renders;
    c->last = rtw_stats{};
    c->last.samples = rank_pixels(c, p.W, p.H, rank, nranks) * p.spp;
    c->last.accel = (uint32_t)accel;
    c->last.bvh_width = bvh_width;
    c->last.kernel = (uint32_t)world;
    c->last_n_sph = p.sc.n_sph;
    c->last_light_bvh = p.light_bvh;
    c->last_n_list = p.sc.n_list;
    c->last.chunk = chunk;
    return RTW_OK;
}

}  // namespace

extern "C" {

int rtw_abi_version(void) { return RTW_ABI_VERSION; }

rtw_ctx* rtw_create(int device, int precision) {
    if (precision != RTW_F32 && precision != RTW_F64) return nullptr;
    rtw_ctx* c = new (std::nothrow) rtw_ctx();
    if (!c) return nullptr;
    c->device = device;
    c->precision = precision;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&c->d_counters), rtw_ctx::kCounters * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_counters, 0, rtw_ctx::kCounters * sizeof(unsigned long long)) != hipSuccess) {
        rtw_destroy(c);
        return nullptr;
    }
    for (auto& tri : c->ring)
        for (auto& e : tri)
            if (hipEventCreate(&e) != hipSuccess) {
                rtw_destroy(c);
                return nullptr;
            }
    return c;
}

int rtw_visible_devices(void) {
    int visible = 0;
    return hipGetDeviceCount(&visible) == hipSuccess ? visible : RTW_E_DEVICE;
}

// the rank contexts of a multi-device context (devices[0] = rank 0 = the
// returned context) plus the events that order consecutive gathers
static int create_ranks(const int* devices, uint32_t n, int precision, rtw_ctx** out) {
    rtw_ctx* c = rtw_create(devices[0], precision);
    if (!c) return RTW_E_DEVICE;
    c->multi = true;
    for (uint32_t k = 1; k < n; ++k) {
        rtw_ctx* pk = rtw_create(devices[k], precision);
        if (!pk) {
            rtw_destroy(c);
            return RTW_E_DEVICE;
        }
        c->peers.push_back(pk);
        hipEvent_t e = nullptr;
        if (hipSetDevice(devices[k]) != hipSuccess || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            rtw_destroy(c);
            return RTW_E_DEVICE;
        }
        c->peer_ev.push_back(e);
    }
    if (hipSetDevice(devices[0]) != hipSuccess ||
        hipEventCreateWithFlags(&c->gather_ev, hipEventDisableTiming) != hipSuccess) {
        rtw_destroy(c);
        return RTW_E_DEVICE;
    }
    *out = c;
    return RTW_OK;
}

int rtw_create_devices(const int* devices, uint32_t n_devices, int precision, rtw_ctx** out) {
    if (!out) return RTW_E_INVALID;
    *out = nullptr;
    if (!devices || n_devices == 0 || (precision != RTW_F32 && precision != RTW_F64)) return RTW_E_INVALID;
    // the device list is checked before any HIP call: no negative or repeated
    // device (one rank per GPU: a repeated device would render its tiles twice
    // and RCCL rejects a clique with a duplicate device)
    for (uint32_t a = 0; a < n_devices; ++a) {
        if (devices[a] < 0) return RTW_E_INVALID;
        for (uint32_t b = 0; b < a; ++b)
            if (devices[a] == devices[b]) return RTW_E_INVALID;
    }
    const int visible = rtw_visible_devices();
    if (visible < 0) return RTW_E_DEVICE;
    for (uint32_t a = 0; a < n_devices; ++a)
        if (devices[a] >= visible) return RTW_E_INVALID;
    const RcclApi& api = rccl_api();
    if (!api.ok) return RTW_E_DEVICE;
    rtw_ctx* c = nullptr;
    const int rc = create_ranks(devices, n_devices, precision, &c);
    if (rc) return rc;
    c->comms.assign(n_devices, nullptr);
    const std::vector<int> list(devices, devices + n_devices);
    if (api.comm_init_all(c->comms.data(), (int)n_devices, list.data()) != ncclSuccess) {
        c->comms.clear();
        rtw_destroy(c);
        return RTW_E_DEVICE;
    }
    (void)hipSetDevice(devices[0]);
    *out = c;
    return RTW_OK;
}

int rtw_create_virtual(int device, uint32_t n_ranks, int precision, rtw_ctx** out) {
    if (!out) return RTW_E_INVALID;
    *out = nullptr;
    if (device < 0 || n_ranks == 0 || n_ranks > 64 || (precision != RTW_F32 && precision != RTW_F64))
        return RTW_E_INVALID;
    const int visible = rtw_visible_devices();
    if (visible < 0) return RTW_E_DEVICE;
    if (device >= visible) return RTW_E_INVALID;
    const std::vector<int> list(n_ranks, device);
    rtw_ctx* c = nullptr;
    const int rc = create_ranks(list.data(), n_ranks, precision, &c);
    if (rc) return rc;
    c->virt = true;
    *out = c;
    return RTW_OK;
}

int rtw_create_mask_ex(uint64_t device_mask, int precision, rtw_ctx** out) {
    if (!out) return RTW_E_INVALID;
    *out = nullptr;
    std::vector<int> list;
    for (int k = 0; k < 64; ++k)
        if ((device_mask >> k) & 1u) list.push_back(k);
    if (list.empty()) return RTW_E_INVALID;
    return rtw_create_devices(list.data(), (uint32_t)list.size(), precision, out);
}

rtw_ctx* rtw_create_mask(uint64_t device_mask, int precision) {
    rtw_ctx* c = nullptr;
    return rtw_create_mask_ex(device_mask, precision, &c) == RTW_OK ? c : nullptr;
}

uint32_t rtw_device_count(const rtw_ctx* c) { return c ? 1u + (uint32_t)c->peers.size() : 0u; }

rtw_ctx* rtw_device_ctx(rtw_ctx* c, uint32_t k) {
    if (!c) return nullptr;
    if (k == 0) return c;
    return k <= c->peers.size() ? c->peers[k - 1] : nullptr;
}

int rtw_device_of(const rtw_ctx* c) { return c ? c->device : RTW_E_INVALID; }

void rtw_destroy(rtw_ctx* c) {
    if (!c) return;
    if (!c->comms.empty()) {
        // the gathers may still run on any rank's stream (rank 0's is the caller's)
        for (uint32_t k = 0; k < rtw_device_count(c); ++k) {
            (void)hipSetDevice(rtw_device_ctx(c, k)->device);
            (void)hipDeviceSynchronize();
        }
        const RcclApi& api = rccl_api();
        for (ncclComm_t m : c->comms)
            if (m && api.comm_destroy) (void)api.comm_destroy(m);
        c->comms.clear();
    }
    if (c->virt)   // the device copies of the last gather read the peers' buffers on rank 0's device
        for (uint32_t k = 0; k < rtw_device_count(c); ++k) {
            (void)hipSetDevice(rtw_device_ctx(c, k)->device);
            (void)hipDeviceSynchronize();
        }
    for (size_t k = 0; k < c->peer_ev.size(); ++k) {
        (void)hipSetDevice(c->peers[k]->device);
        if (c->peer_ev[k]) (void)hipEventDestroy(c->peer_ev[k]);
    }
    c->peer_ev.clear();
    for (rtw_ctx* pk : c->peers) rtw_destroy(pk);
    c->peers.clear();
    (void)hipSetDevice(c->device);
    if (c->gather_ev) (void)hipEventDestroy(c->gather_ev);
    if (c->d_gather) (void)hipFree(c->d_gather);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_scene) (void)hipFree(c->d_scene);
    if (c->d_partial) (void)hipFree(c->d_partial);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->d_img) (void)hipFree(c->d_img);
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->d_lpt) (void)hipFree(c->d_lpt);
    if (c->d_lpt_tasks) (void)hipFree(c->d_lpt_tasks);
    if (c->d_tile_map) (void)hipFree(c->d_tile_map);
    if (c->d_tile_slot) (void)hipFree(c->d_tile_slot);
    if (c->lpt_ev) (void)hipEventDestroy(c->lpt_ev);
    for (auto& tri : c->ring)
        for (auto& e : tri)
            if (e) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rtw_last_error(const rtw_ctx* c) { return c ? c->err.c_str() : "null context"; }
int rtw_precision(const rtw_ctx* c) { return c ? c->precision : -1; }

int rtw_set_chunk(rtw_ctx* c, uint32_t chunk) {
    if (!c) return RTW_E_INVALID;
    c->chunk = chunk;
    for (rtw_ctx* pk : c->peers) pk->chunk = chunk;   // (multi-device: every rank alike)
    return RTW_OK;
}
int rtw_set_tuning(rtw_ctx* c, const char* key, int64_t value) {
    if (!c || !key) return RTW_E_INVALID;
    for (rtw_ctx* pk : c->peers) {   // multi-device: every rank alike
        const int rc = rtw_set_tuning(pk, key, value);
        if (rc) return fail(c, rc, pk->err);
    }
    const std::string k = key;
    if (value < 0) return fail(c, RTW_E_INVALID, "negative tuning value");
    if (k == "chunk") c->chunk = (uint32_t)value;
    else if (k == "auto_chunk") c->auto_chunk = std::max<uint32_t>(1, (uint32_t)value);
    else if (k == "robust") c->robust = (int)std::min<int64_t>(value, 2);
    else if (k == "bvh_leaf") c->bvh_leaf = (uint32_t)std::min<int64_t>(value, 15);
    else if (k == "light_leaf") c->light_leaf = (uint32_t)std::min<int64_t>(value, 15);
    else if (k == "persist") c->persist = value == 1 ? rtw::kPersistResident : (uint32_t)std::min<int64_t>(value, 1 << 20);
    else if (k == "light_grid") c->light_grid = (uint32_t)std::min<int64_t>(value, 1024);
    else if (k == "item_order") c->item_order = value ? 1u : 0u;
    else if (k == "hit64") c->hit64 = value ? 1u : 0u;
    else if (k == "lpt") c->lpt = (uint32_t)std::min<int64_t>(value, 2);
    else if (k == "lpt_min_spp") c->lpt_min_spp = (uint32_t)std::min<int64_t>(value, 1u << 30);
    else if (k == "lpt_inline") c->lpt_inline = value ? 1u : 0u;
    else if (k == "lpt_pilot_spp") c->lpt_pilot_spp = (uint32_t)std::min<int64_t>(std::max<int64_t>(value, 1), 64);
    else if (k == "lpt_pilot_depth") c->lpt_pilot_depth = (uint32_t)std::min<int64_t>(value, 1u << 20);
    else if (k == "light_bvh_min") c->light_bvh_min = (uint32_t)std::min<int64_t>(value, 1u << 30);
    else if (k == "max_group") { c->max_group = (uint32_t)std::min<int64_t>(std::max<int64_t>(value, 1), 4095); c->lpt_tab_valid = false; }
    else if (k == "grid_piece") c->grid_piece = (uint32_t)std::min<int64_t>(value, 1u << 20);
    else if (k == "partial_max") c->partial_max = std::max<size_t>(1 << 20, (size_t)value);
    else if (k == "group") c->group = (uint32_t)value;
    else if (k == "target_tasks") c->target_tasks = std::max<uint64_t>(1, (uint64_t)value);
    else if (k == "lds") c->world_pref = value ? 1 : 0;
    else if (k == "bvh_ww") c->bvh_kind = value ? 1 : 0;
    else if (k == "bvh_kind") c->bvh_kind = (int)std::min<int64_t>(value, 3);
    else if (k == "bvh_lds_max") c->bvh_lds_max = (size_t)std::min<int64_t>(value, kLdsLimit);
    else if (k == "auto_accel") c->auto_accel = (int)std::min<int64_t>(value, RTW_ACCEL_BVH);
    else if (k == "balance") c->balance = value ? 1u : 0u;
    else if (k == "cost_time") c->cost_time = value ? 1u : 0u;
    else if (k == "guide_div") { c->guide_div = (uint32_t)std::min<int64_t>(value, 1 << 24); c->lpt_tab_valid = false; }
    else if (k == "guide_max") { c->guide_max = (uint32_t)std::min<int64_t>(std::max<int64_t>(value, 1), 4095); c->lpt_tab_valid = false; }
    else if (k == "guide_floor") { c->guide_floor = std::max<uint64_t>(1, (uint64_t)value); c->lpt_tab_valid = false; }
    else return fail(c, RTW_E_INVALID, "unknown tuning key " + k);
    return RTW_OK;
}

int rtw_set_accel(rtw_ctx* c, int accel) {
    if (!c) return RTW_E_INVALID;
    if (accel < RTW_ACCEL_AUTO || accel > RTW_ACCEL_BVH) return fail(c, RTW_E_UNSUPPORTED, "accel not available");
    c->accel = accel;
    for (rtw_ctx* pk : c->peers) pk->accel = accel;
    return RTW_OK;
}

void rtw_camera_builder_default(rtw_camera_builder* b) {
    // CameraBuilder::new(), camera.rs:45-60
    memset(b, 0, sizeof(*b));
    b->samples_per_pixel = 10;
    b->max_depth = 10;
    b->vfov = 90.0;
    b->lookat[2] = -1.0;
    b->vup[1] = 1.0;
    b->defocus_angle = 0.0;
    b->focus_dist = 10.0;
}

static uint32_t round_u32(double x) {
    // f64::round (half away from zero) then `as u32` (saturating, NaN -> 0)
    double r = round(x);
    if (!(r > 0.0)) return 0;
    if (r >= 4294967295.0) return 4294967295u;
    return (uint32_t)r;
}

int rtw_camera_build(const rtw_camera_builder* b, rtw_camera* out) {
    // CameraBuilder::build, camera.rs:114-218
    if (!b || !out) return RTW_E_INVALID;
    struct V { double x, y, z; };
    auto sub = [](V a, V c) { return V{a.x - c.x, a.y - c.y, a.z - c.z}; };
    auto add = [](V a, V c) { return V{a.x + c.x, a.y + c.y, a.z + c.z}; };
    auto mul = [](V a, double s) { return V{a.x * s, a.y * s, a.z * s}; };
    auto dv = [](V a, double s) { return V{a.x / s, a.y / s, a.z / s}; };
    auto dot = [](V a, V c) { return a.x * c.x + a.y * c.y + a.z * c.z; };
    auto cross = [](V a, V c) {
        return V{a.y * c.z - a.z * c.y, a.z * c.x - a.x * c.z, a.x * c.y - a.y * c.x};
    };
    auto norm = [&](V a) { return dv(a, sqrt(dot(a, a))); };
    auto ld = [](const double* p) { return V{p[0], p[1], p[2]}; };
    auto st = [](double* p, V v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; };

    const bool ha = b->has_aspect_ratio, hh = b->has_image_height, hw = b->has_image_width;
    double aspect;
    uint32_t H, W;
    if (!ha && !hh && !hw) { aspect = 1.0; H = 100; W = 100; }
    else if (!ha && !hh && hw) { aspect = 1.0; H = b->image_width; W = b->image_width; }
    else if (!ha && hh && !hw) { aspect = 1.0; H = b->image_height; W = b->image_height; }
    else if (ha && !hh && !hw) { aspect = b->aspect_ratio; H = round_u32(100.0 / b->aspect_ratio); W = 100; }
    else if (!ha && hh && hw) { aspect = (double)b->image_width / (double)b->image_height; H = b->image_height; W = b->image_width; }
    else if (ha && !hh && hw) { aspect = b->aspect_ratio; H = round_u32((double)b->image_width / b->aspect_ratio); W = b->image_width; }
    else if (ha && hh && !hw) { aspect = b->aspect_ratio; H = b->image_height; W = round_u32((double)b->image_height * b->aspect_ratio); }
    else { aspect = b->aspect_ratio; H = b->image_height; W = b->image_width; }

    const double kPi = 3.14159265358979323846;
    V center = ld(b->lookfrom);
    double theta = b->vfov * (kPi / 180.0);   // f64::to_radians
    double h = tan(theta / 2.0);
    double vh = 2.0 * h * b->focus_dist;
    double vw = vh * aspect;
    V w = sub(ld(b->lookfrom), ld(b->lookat));
    V c0 = cross(ld(b->vup), w);
    if (fabs(c0.x) < 1e-8 && fabs(c0.y) < 1e-8 && fabs(c0.z) < 1e-8) w = add(w, V{0.1, 0.0, 0.0});
    w = norm(w);
    V u = norm(cross(ld(b->vup), w));
    V v = cross(w, u);
    V vu = mul(u, vw), vv = mul(v, vh);
    V du = dv(vu, (double)W), dvv = dv(vv, (double)H);
    V ul = sub(sub(sub(center, mul(w, b->focus_dist)), dv(vu, 2.0)), dv(vv, 2.0));
    V p00 = add(ul, dv(add(du, dvv), 2.0));
    double rad = tan(b->defocus_angle / 2.0) * b->focus_dist;
    memset(out, 0, sizeof(*out));
    out->image_width = W;
    out->image_height = H;
    out->samples_per_pixel = b->samples_per_pixel;
    out->max_depth = b->max_depth;
    memcpy(out->background, b->background, sizeof(out->background));
    out->defocus_angle = b->defocus_angle;
    st(out->center, center);
    st(out->pixel00_loc, p00);
    st(out->pixel_delta_u, du);
    st(out->pixel_delta_v, dvv);
    st(out->defocus_disk_u, mul(u, rad));
    st(out->defocus_disk_v, mul(v, rad));
    return RTW_OK;
}

// one device's copy of a staged scene (rtw_set_scene stages once, then
// uploads to every device of the context)
static int upload_scene(rtw_ctx* c, const rtw_scene* s, const std::vector<unsigned char>& blob,
                        rtw::DevScene<float> tmp32, rtw::DevScene<double> tmp64) {
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->scene_bytes < blob.size()) {
        if (c->d_scene) (void)hipFree(c->d_scene);
        c->d_scene = nullptr;
        c->scene_bytes = 0;
        HIP_TRY(c, hipMalloc(&c->d_scene, blob.size()));
        c->scene_bytes = blob.size();
    }
    c->scene_used = blob.size();
    // the closest-hit working set (tree + leaf spheres + ids): what the lpt
    // heuristic weighs against an XCD's L2
    c->tree_bytes = c->precision == RTW_F32
                        ? (size_t)tmp32.n_nodes * sizeof(rtw::BvhNode<float>) + (size_t)tmp32.n_sph * (sizeof(rtw::R4<float>) + 4)
                        : (size_t)tmp64.n_nodes * (sizeof(rtw::BvhNode<double>) + sizeof(rtw::BvhNode<float>)) +
                              (size_t)tmp64.n_sph * (sizeof(rtw::R4<double>) + 4);
    // scale of the scene for the f32 test choice (render_device_t)
    c->scene_extent = 0.0;
    c->min_radius = INFINITY;
    for (uint32_t k = 0; k < s->n_spheres; ++k) {
        const double* q = s->spheres + 4 * k;
        const double r = fabs(q[3]);
        c->scene_extent = std::max(c->scene_extent, std::max(fabs(q[0]), std::max(fabs(q[1]), fabs(q[2]))) + r);
        if (r > 0) c->min_radius = std::min(c->min_radius, r);
    }
    for (uint32_t k = 0; k < s->n_lights; ++k) {
        const double r = fabs(s->lights[4 * k + 3]);
        if (r > 0) c->min_radius = std::min(c->min_radius, r);
    }
    const uintptr_t base = reinterpret_cast<uintptr_t>(c->d_scene);
    auto rebase = [base](auto& ds) {
        auto fix = [base](auto*& ptr) {
            using T = std::remove_reference_t<decltype(ptr)>;
            ptr = reinterpret_cast<T>(reinterpret_cast<uintptr_t>(ptr) + base);
        };
        fix(ds.sph); fix(ds.sph_r); fix(ds.sph_mat); fix(ds.sph_shade); fix(ds.planes); fix(ds.plane_mat);
        fix(ds.mat_type); fix(ds.mat_p); fix(ds.lights); fix(ds.bvh); fix(ds.bsph); fix(ds.bid);
        fix(ds.bvh4); fix(ds.lbvh);
        fix(ds.lsph); fix(ds.lid); fix(ds.lg_start); fix(ds.lg_sph); fix(ds.lg_id); fix(ds.lg_rec);
        fix(ds.quads); fix(ds.quad_mat); fix(ds.lquads); fix(ds.sph64); fix(ds.pl64); fix(ds.mat64);
        if (ds.lref) fix(ds.lref);
        if constexpr (std::is_same<std::decay_t<decltype(ds)>, rtw::DevScene<double>>::value) {
            fix(ds.bvh32);
            fix(ds.bsph32);
            fix(ds.lg_sph32);
        }
        fix(ds.boxes); fix(ds.box_mat);
        if (ds.mat_tex) fix(ds.mat_tex);
        fix(ds.tex_type); fix(ds.tex_p); fix(ds.tex_refs); fix(ds.perlin_vec); fix(ds.perlin_perm);
    };
    static_assert(offsetof(rtw::DevScene<float>, n_sph) == 35 * sizeof(void*),
                  "DevScene gained a pointer: update rebase");
    if (c->precision == RTW_F32) {
        rebase(tmp32);
        c->sc32 = tmp32;
    } else {
        rebase(tmp64);
        c->sc64 = tmp64;
    }
    HIP_TRY(c, hipMemcpy(c->d_scene, blob.data(), blob.size(), hipMemcpyHostToDevice));
    c->has_scene = true;
    ++c->scene_serial;
    return RTW_OK;
}

int rtw_set_scene(rtw_ctx* c, const rtw_scene* s) {
    if (!c) return RTW_E_INVALID;
    int rc = validate_scene(c, s);
    if (rc) return rc;
    // stage once against base 0 (upload_scene rebases the device pointers:
    // EVERY pointer member of DevScene must be listed in its `rebase`)
    rtw::DevScene<float> tmp32{};
    rtw::DevScene<double> tmp64{};
    // auto leaf size: 4; 8 from 100k spheres (C5: +12 %); f64 with a tree too
    // large for LDS (>= 4096 spheres): 2 -- its sphere tests are f64, its node
    // tests f32 (C3 f64 1006 -> 998 ms: 2.8 -> 1.7 sphere tests and 7.2 -> 7.9
    // node visits per segment; 3: 1003; C2's LDS tree and f32 lose with 2,
    // profiles/r06t_ab_leaf_c3_f64.jsonl, r06u_ab_leaf.jsonl)
    const uint32_t leaf = c->bvh_leaf ? c->bvh_leaf
                                      : (s->n_spheres >= 100000 ? 8u
                                         : (c->precision == RTW_F64 && s->n_spheres >= 4096 ? 2u : 4u));
    const uint32_t light_leaf = c->light_leaf ? c->light_leaf : rtw::kLeafMax;
    // the light grid only for light lists long enough to skip the linear loop
    const double grid = s->n_lights >= c->light_bvh_min ? c->light_grid / 16.0 : 0.0;
    std::vector<unsigned char> blob = c->precision == RTW_F32
                                          ? stage_scene<float>(s, &tmp32, 0, leaf, light_leaf, grid)
                                          : stage_scene<double>(s, &tmp64, 0, leaf, light_leaf, grid);
    for (uint32_t k = 0; k < rtw_device_count(c); ++k) {   // multi-device: the same scene on every rank
        rtw_ctx* ck = rtw_device_ctx(c, k);
        rc = upload_scene(ck, s, blob, tmp32, tmp64);
        if (rc) {
            // no rank keeps a scene: a partial update must not render one image
            // from tiles of two scenes
            for (uint32_t q = 0; q < rtw_device_count(c); ++q) rtw_device_ctx(c, q)->has_scene = false;
            if (!c->peers.empty()) (void)hipSetDevice(c->device);
            return k ? fail(c, rc, ck->err) : rc;
        }
    }
    if (!c->peers.empty()) HIP_TRY(c, hipSetDevice(c->device));
    return RTW_OK;
}

uint32_t rtw_tile_size(void) { return rtw::kTile; }

uint32_t rtw_tiles_for_rank(uint32_t W, uint32_t H, uint32_t rank, uint32_t nranks) {
    if (nranks == 0 || rank >= nranks) return 0;
    const uint64_t n = (uint64_t)((W + rtw::kTile - 1) / rtw::kTile) * ((H + rtw::kTile - 1) / rtw::kTile);
    return rank < n ? (uint32_t)((n - rank + nranks - 1) / nranks) : 0u;
}

int rtw_split_deal(const uint32_t* tile_cost, uint32_t W, uint32_t H, uint32_t nranks, uint32_t* tile_rank) {
    if (nranks == 0 || nranks > RTW_MAX_RANKS) return RTW_E_INVALID;
    const uint64_t n = n_tiles_of(W, H);
    if (n > 0xFFFFFFFFull / nranks) return RTW_E_UNSUPPORTED;
    if (n && (!tile_cost || !tile_rank)) return RTW_E_INVALID;
    // costliest tiles first (ties: lower index), each to the rank of least dealt
    // cost (ties: lower rank) among those below their round-robin tile count
    std::vector<uint32_t> order(n);
    for (uint64_t T = 0; T < n; ++T) order[T] = (uint32_t)T;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return tile_cost[a] > tile_cost[b]; });
    std::vector<uint64_t> load(nranks, 0);
    std::vector<uint32_t> room(nranks);
    for (uint32_t r = 0; r < nranks; ++r) room[r] = rtw_tiles_for_rank(W, H, r, nranks);
    for (uint32_t T : order) {
        uint32_t best = nranks;
        for (uint32_t r = 0; r < nranks; ++r)
            if (room[r] && (best == nranks || load[r] < load[best])) best = r;
        tile_rank[T] = best;
        load[best] += tile_cost[T];
        --room[best];
    }
    return RTW_OK;
}
}  // extern "C"

namespace {
// the split (and its costs) on one rank context; tile_rank NULL: the round robin
int apply_split(rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks, const uint32_t* tile_rank,
                const uint32_t* tile_cost, bool automatic, const rtw_camera* cam) {
    if (!tile_rank) {
        c->split_rank.clear();
        c->split_cost.clear();
        c->split_W = c->split_H = c->split_n = 0;
        c->split_auto = false;
        return RTW_OK;
    }
    const uint64_t n = n_tiles_of(W, H);
    c->split_rank.assign(tile_rank, tile_rank + n);
    if (tile_cost) c->split_cost.assign(tile_cost, tile_cost + n);
    else c->split_cost.clear();
    c->split_W = W;
    c->split_H = H;
    c->split_n = nranks;
    ++c->split_serial;
    c->split_auto = automatic;
    if (cam) c->split_cam = *cam;
    c->split_scene = c->scene_serial;
    return RTW_OK;
}

int check_split(uint32_t W, uint32_t H, uint32_t nranks, const uint32_t* tile_rank) {
    if (nranks == 0 || nranks > RTW_MAX_RANKS) return RTW_E_INVALID;
    const uint64_t n = n_tiles_of(W, H);
    if (n > 0xFFFFFFFFull / nranks) return RTW_E_UNSUPPORTED;
    if (!tile_rank) return RTW_OK;
    std::vector<uint32_t> cnt(nranks, 0);
    for (uint64_t T = 0; T < n; ++T) {
        if (tile_rank[T] >= nranks) return RTW_E_INVALID;
        ++cnt[tile_rank[T]];
    }
    for (uint32_t r = 0; r < nranks; ++r)
        if (cnt[r] != rtw_tiles_for_rank(W, H, r, nranks)) return RTW_E_INVALID;
    return RTW_OK;
}

// The tile costs the context counted for (cam, rank, nranks) under its split,
// scattered into cost[global tile]; waits for a pending counting render.
int tile_costs_of(rtw_ctx* c, const rtw_camera* cam, uint32_t rank, uint32_t nranks, uint32_t* cost) {
    if (!lpt_has(c, cam, rank, nranks))
        return fail(c, RTW_E_INVALID, "no tile costs for this camera, scene and rank split: render once with "
                                      "tuning lpt on and spp >= lpt_min_spp first");
    HIP_TRY(c, hipSetDevice(c->device));
    const uint32_t W = cam->image_width, H = cam->image_height;
    std::vector<uint32_t> tiles;
    local_tiles(c, W, H, rank, nranks, tiles);
    if (c->lpt_pending) {
        const int rc = lpt_readback(c, (uint32_t)tiles.size());
        if (rc) return rc;
    }
    if (c->h_lpt_cost.size() != tiles.size()) return fail(c, RTW_E_INVALID, "tile cost count mismatch");
    for (size_t k = 0; k < tiles.size(); ++k) cost[tiles[k]] = c->h_lpt_cost[k];
    return RTW_OK;
}
}  // namespace

extern "C" {

int rtw_set_split(rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks, const uint32_t* tile_rank,
                  const uint32_t* tile_cost) {
    if (!c) return RTW_E_INVALID;
    const int rc = check_split(W, H, nranks, tile_rank);
    if (rc) return fail(c, rc, "bad split: every tile needs a rank < nranks, and rank r exactly "
                               "rtw_tiles_for_rank(W, H, r, nranks) tiles");
    for (uint32_t k = 0; k < rtw_device_count(c); ++k)   // multi-device: every rank alike
        apply_split(rtw_device_ctx(c, k), W, H, nranks, tile_rank, tile_cost, false, nullptr);
    return RTW_OK;
}

int rtw_get_split(rtw_ctx* c, uint32_t W, uint32_t H, uint32_t nranks, uint32_t* tile_rank) {
    if (!c || nranks == 0) return RTW_E_INVALID;
    if (!split_active(c, W, H, nranks)) return 0;
    if (tile_rank) memcpy(tile_rank, c->split_rank.data(), c->split_rank.size() * sizeof(uint32_t));
    return c->split_auto ? 2 : 1;
}

int rtw_tile_costs(rtw_ctx* c, const rtw_camera* cam, uint32_t rank, uint32_t nranks, uint32_t* tile_cost) {
    if (!c || !cam || !tile_cost || nranks == 0 || rank >= nranks) return fail(c, RTW_E_INVALID, "bad argument");
    return tile_costs_of(c, cam, rank, nranks, tile_cost);
}

int rtw_assemble_tiles(rtw_ctx* c, const void* d_ranks, size_t rank_stride_bytes, uint32_t nranks, uint32_t W,
                       uint32_t H, void* d_image, void* stream) {
    if (!c || nranks == 0) return fail(c, RTW_E_INVALID, "bad argument");
    const size_t esz = c->precision == RTW_F32 ? sizeof(float) : sizeof(double);
    if ((uint64_t)W * H == 0) return RTW_OK;
    if (!d_ranks || !d_image || rank_stride_bytes % esz)
        return fail(c, RTW_E_INVALID, "bad assemble buffers");
    if (rank_stride_bytes < (size_t)rtw_tiles_for_rank(W, H, 0, nranks) * 64 * 3 * esz)
        return fail(c, RTW_E_INVALID, "rank stride is smaller than tiles_for_rank(rank 0)*64*3");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = resolve_stream(c, stream);
    const size_t stride = rank_stride_bytes / esz;
    // a dealt split: each tile's slot from its map (null: the round robin)
    const uint32_t* slot = nullptr;
    if (split_active(c, W, H, nranks)) {
        const int mrc = ensure_tile_slot(c, W, H, nranks);
        if (mrc) return mrc;
        slot = reinterpret_cast<const uint32_t*>(c->d_tile_slot);
    }
    const int rc = c->precision == RTW_F32
                       ? rtw::launch_assemble_f32(reinterpret_cast<const float*>(d_ranks), stride, nranks, W, H,
                                                  slot, reinterpret_cast<float*>(d_image), s)
                       : rtw::launch_assemble_f64(reinterpret_cast<const double*>(d_ranks), stride, nranks, W, H,
                                                  slot, reinterpret_cast<double*>(d_image), s);
    if (rc) return fail(c, RTW_E_DEVICE, std::string("assemble launch failed: ") + hipGetErrorString(hipGetLastError()));
    return RTW_OK;
}

int rtw_render_device(rtw_ctx* c, const rtw_camera* cam, uint64_t seed, uint32_t rank, uint32_t nranks,
                      void* d_out, size_t out_bytes, void* stream) {
    if (!c || !cam || nranks == 0 || rank >= nranks) return fail(c, RTW_E_INVALID, "bad argument");
    if (!c->has_scene) return fail(c, RTW_E_NO_SCENE, "rtw_set_scene was not called");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = resolve_stream(c, stream);
    // a multi-device context renders on rank 0 only here: its stats are rank 0's
    c->stats_ranks = 1;
    if (c->gather_pending) {
        // the last gather / assembly may still read d_gather (rank 0 renders into it
        // again only through rtw_render_image_device, but d_out may alias it)
        HIP_TRY(c, hipStreamWaitEvent(s, c->gather_ev, 0));
    }
    return c->precision == RTW_F32 ? render_device_t<float>(c, cam, seed, rank, nranks, d_out, out_bytes, s)
                                   : render_device_t<double>(c, cam, seed, rank, nranks, d_out, out_bytes, s);
}

int rtw_render_image_device(rtw_ctx* c, const rtw_camera* cam, uint64_t seed, void* d_image, size_t image_bytes,
                            void* stream) {
    if (!c || !cam) return fail(c, RTW_E_INVALID, "bad argument");
    if (!c->has_scene) return fail(c, RTW_E_NO_SCENE, "rtw_set_scene was not called");
    const uint32_t W = cam->image_width, H = cam->image_height, n = rtw_device_count(c);
    const size_t esz = c->precision == RTW_F32 ? sizeof(float) : sizeof(double);
    const size_t img = (size_t)W * H * 3 * esz;
    if (image_bytes < img || (img && !d_image)) return fail(c, RTW_E_INVALID, "d_image is smaller than W*H*3");
    hipStream_t s0 = resolve_stream(c, stream);
    // rank k renders the tiles T = k (mod n) into a packed buffer of rank 0's
    // size (the most tiles: RCCL gathers equal counts)
    const size_t per = std::max<size_t>((size_t)rtw_tiles_for_rank(W, H, 0, n) * 64 * 3, 1);
    if (!c->multi) {
        // one device, no collective: the packed tiles -> the image
        HIP_TRY(c, hipSetDevice(c->device));
        int rc = ensure(c, &c->d_out, &c->out_cap, per * esz);
        if (rc) return rc;
        rc = rtw_render_device(c, cam, seed, 0, 1, c->d_out, c->out_cap, stream);
        if (rc) return rc;
        return img ? rtw_assemble_tiles(c, c->d_out, c->out_cap, 1, W, H, d_image, stream) : RTW_OK;
    }
    // Balance (tuning "balance"): once every rank has counted its tiles' costs
    // for this camera and scene (the first render of a key counts them), deal
    // the tiles to the ranks by those costs (rtw_split_deal) -- the reference
    // balances its pixels dynamically over the host cores, camera.rs:340-353.
    // The image does not depend on the split (every pixel's samples are its own).
    const bool have = split_active(c, W, H, n);
    if (c->balance && n > 1 && img &&
        (!have || (c->split_auto && (c->split_scene != c->scene_serial ||
                                     memcmp(&c->split_cam, cam, sizeof *cam) != 0)))) {
        bool all = true;
        for (uint32_t k = 0; k < n && all; ++k) all = lpt_has(rtw_device_ctx(c, k), cam, k, n);
        if (all) {
            std::vector<uint32_t> cost(n_tiles_of(W, H), 0), owner(cost.size(), 0);
            for (uint32_t k = 0; k < n; ++k) {
                rtw_ctx* ck = rtw_device_ctx(c, k);
                const int rc = tile_costs_of(ck, cam, k, n, cost.data());
                if (rc) return k ? fail(c, rc, ck->err) : rc;
            }
            int rc = rtw_split_deal(cost.data(), W, H, n, owner.data());
            if (rc) return fail(c, rc, "rtw_split_deal failed");
            for (uint32_t k = 0; k < n; ++k)
                apply_split(rtw_device_ctx(c, k), W, H, n, owner.data(), cost.data(), true, cam);
        }
    }
    HIP_TRY(c, hipSetDevice(c->device));
    // (the previous call's gather + assembly, possibly on another stream: rank
    // 0's render below waits for gather_ev (rtw_render_device), the peers'
    // streams were made to wait for it when it was recorded; a reallocation of
    // d_gather in `ensure` synchronises the device)
    int rc = ensure(c, &c->d_gather, &c->gather_cap, (size_t)n * per * esz);
    if (rc) return rc;
    // launch every rank's share (asynchronous, each device on its own stream);
    // rank 0 renders in place into its slot of the gather target
    for (uint32_t k = 0; k < n; ++k) {
        rtw_ctx* ck = rtw_device_ctx(c, k);
        HIP_TRY(c, hipSetDevice(ck->device));
        void* dst = c->d_gather;
        if (k) {
            rc = ensure(ck, &ck->d_out, &ck->out_cap, per * esz);
            if (rc) return fail(c, rc, ck->err);
            dst = ck->d_out;
        }
        rc = rtw_render_device(ck, cam, seed, k, n, dst, per * esz, k ? (void*)ck->stream : stream);
        if (rc) return k ? fail(c, rc, ck->err) : rc;
    }
    if (c->virt) {
        // test mode (rtw_create_virtual): the gather as device copies on rank 0's
        // stream, each after its rank's render -- the same slots an RCCL gather
        // to root 0 fills
        for (uint32_t k = 1; k < n; ++k) {
            rtw_ctx* ck = rtw_device_ctx(c, k);
            HIP_TRY(c, hipEventRecord(c->peer_ev[k - 1], ck->stream));
            HIP_TRY(c, hipStreamWaitEvent(s0, c->peer_ev[k - 1], 0));
            HIP_TRY(c, hipMemcpyAsync(static_cast<unsigned char*>(c->d_gather) + (size_t)k * per * esz, ck->d_out,
                                      per * esz, hipMemcpyDeviceToDevice, s0));
        }
    } else {
        // ONE gather of the packed tiles to rank 0 (RCCL over xGMI), ordered after
        // each rank's render on that rank's stream
        const RcclApi& api = rccl_api();
        const ncclDataType_t dt = c->precision == RTW_F32 ? ncclFloat32 : ncclFloat64;
        ncclResult_t r = api.group_start();
        if (r != ncclSuccess) return rccl_fail(c, r, "ncclGroupStart");
        for (uint32_t k = 0; k < n; ++k) {
            rtw_ctx* ck = rtw_device_ctx(c, k);
            r = api.gather(k ? ck->d_out : c->d_gather, k ? nullptr : c->d_gather, per, dt, 0, c->comms[k],
                           k ? ck->stream : s0);
            if (r != ncclSuccess) {
                (void)api.group_end();
                return rccl_fail(c, r, "ncclGather");
            }
        }
        r = api.group_end();
        if (r != ncclSuccess) return rccl_fail(c, r, "ncclGroupEnd");
    }
    HIP_TRY(c, hipSetDevice(c->device));
    // rank 0 un-interleaves the n buffers into the image
    rc = img ? rtw_assemble_tiles(c, c->d_gather, per * esz, n, W, H, d_image, stream) : RTW_OK;
    if (rc) return rc;
    // every rank's next render waits for this gather + assembly (a peer's
    // packed tiles are read on s0 in the virtual mode; d_gather always)
    HIP_TRY(c, hipEventRecord(c->gather_ev, s0));
    for (uint32_t k = 1; k < n; ++k) {
        rtw_ctx* ck = rtw_device_ctx(c, k);
        HIP_TRY(c, hipSetDevice(ck->device));
        HIP_TRY(c, hipStreamWaitEvent(ck->stream, c->gather_ev, 0));
    }
    HIP_TRY(c, hipSetDevice(c->device));
    c->gather_pending = true;
    c->stats_ranks = n;
    return RTW_OK;
}

int rtw_last_kernel(const rtw_ctx* c) {
    if (!c) return RTW_E_INVALID;
    return c->last_variant & 0xffff;
}

static int rtw_get_stats_one(rtw_ctx* c, rtw_stats* out);

int rtw_get_stats_rank(rtw_ctx* c, uint32_t k, rtw_stats* out) {
    if (!c || !out) return RTW_E_INVALID;
    rtw_ctx* ck = rtw_device_ctx(c, k);
    if (!ck) return fail(c, RTW_E_INVALID, "no rank " + std::to_string(k));
    const int rc = rtw_get_stats_one(ck, out);
    if (k && rc) c->err = ck->err;
    (void)hipSetDevice(c->device);
    return rc;
}

int rtw_get_stats(rtw_ctx* c, rtw_stats* out) {
    if (!c || !out) return RTW_E_INVALID;
    if (!c->peers.empty() && c->stats_ranks > 1) {
        // multi-device: the counters summed over the ranks of the last render,
        // kernel_ms the slowest rank's; the rest as rank 0 reports it (after a
        // rank-0-only rtw_render_device: rank 0's alone)
        rtw_stats sum{};
        int worst = RTW_OK;
        for (uint32_t k = 0; k < std::min(c->stats_ranks, rtw_device_count(c)); ++k) {
            rtw_ctx* ck = rtw_device_ctx(c, k);
            rtw_stats st{};
            const int rc = rtw_get_stats_one(ck, &st);
            if (rc == RTW_E_DEVICE || rc == RTW_E_INVALID) return k ? fail(c, rc, ck->err) : rc;
            if (rc && !worst) {
                worst = rc;
                if (k) c->err = ck->err;
            }
            if (k == 0) sum = st;
            else {
                sum.samples += st.samples;
                sum.segments += st.segments;
                sum.lambertian += st.lambertian;
                sum.node_visits += st.node_visits;
                sum.sphere_tests += st.sphere_tests;
                sum.panic_plane_uv += st.panic_plane_uv;
                sum.panic_no_lights += st.panic_no_lights;
                sum.light_tests += st.light_tests;
                sum.grid_cells += st.grid_cells;
                sum.kernel_ms = std::max(sum.kernel_ms, st.kernel_ms);
            }
        }
        (void)hipSetDevice(c->device);
        *out = sum;
        return worst;
    }
    return rtw_get_stats_one(c, out);
}

static int rtw_get_stats_one(rtw_ctx* c, rtw_stats* out) {
    if (c->n_renders == 0) return fail(c, RTW_E_INVALID, "no render yet");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipEventSynchronize(c->ev1));
    unsigned long long h[rtw_ctx::kCounters] = {};
    HIP_TRY(c, hipMemcpy(h, c->d_counters, sizeof h, hipMemcpyDeviceToHost));
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->last.segments = h[0];
    c->last.lambertian = h[1];
    c->last.node_visits = h[2];
    // the brute-force sweep tests every sphere on every segment
    c->last.sphere_tests = c->last.accel == RTW_ACCEL_BVH ? h[3] : h[0] * (uint64_t)c->last_n_sph;
    c->last.kernel_ms = ms;
    c->last.panic_plane_uv = h[4];
    c->last.panic_no_lights = h[5];
    // the linear light loop tests every light of the list on every Lambertian
    // bounce (hittable_list.rs:408-412); the light grid / BVH walks count theirs
    c->last.light_tests = c->last_light_bvh ? h[7] : h[1] * (uint64_t)c->last_n_list;
    c->last.grid_cells = h[8];
    *out = c->last;
    if (h[5])
        return fail(c, RTW_E_NO_LIGHTS, std::to_string(h[5]) + " samples drew a light from an empty light list "
                                        "(the reference panics: HittableList shouldn't be empty, hittable_list.rs:417)");
    if (h[4])
        return fail(c, RTW_E_PANIC, std::to_string(h[4]) + " plane tests produced a non-finite UV "
                                    "(the reference panics in Plane::hit, plane.rs:66-69)");
    return RTW_OK;
}

int rtw_get_timings(rtw_ctx* c, float* render_ms, float* total_ms, int max) {
    if (!c || max < 0) return RTW_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->device));
    const int n = (int)std::min<uint64_t>({(uint64_t)max, c->n_renders, (uint64_t)rtw_ctx::kRing});
    for (int k = 0; k < n; ++k) {
        hipEvent_t* ev = c->ring[(c->n_renders - n + k) % rtw_ctx::kRing];
        HIP_TRY(c, hipEventSynchronize(ev[2]));
        float a = 0.f, b = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&a, ev[0], ev[1]));
        HIP_TRY(c, hipEventElapsedTime(&b, ev[0], ev[2]));
        if (render_ms) render_ms[k] = a;
        if (total_ms) total_ms[k] = b;
    }
    return n;
}

int rtw_render(rtw_ctx* c, const rtw_camera* cam, const rtw_scene* scene, uint64_t seed, double* out_sum,
               rtw_stats* stats) {
    if (!c || !cam || !out_sum) return fail(c, RTW_E_INVALID, "bad argument");
    if (scene) {
        int rc = rtw_set_scene(c, scene);
        if (rc) return rc;
    }
    if (!c->has_scene) return fail(c, RTW_E_NO_SCENE, "no scene");
    const size_t esz = c->precision == RTW_F32 ? sizeof(float) : sizeof(double);
    const size_t n = (size_t)cam->image_width * cam->image_height * 3;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = ensure(c, &c->d_img, &c->img_cap, std::max<size_t>(n * esz, 64));
    if (rc) return rc;
    // every device of the context renders its share; the image lands on the first
    rc = rtw_render_image_device(c, cam, seed, c->d_img, c->img_cap, nullptr);
    if (rc) return rc;
    c->h_out.resize(n * esz);
    if (n) HIP_TRY(c, hipMemcpyAsync(c->h_out.data(), c->d_img, n * esz, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->precision == RTW_F32) {
        const float* f = reinterpret_cast<const float*>(c->h_out.data());
        for (size_t k = 0; k < n; ++k) out_sum[k] = (double)f[k];
    } else {
        memcpy(out_sum, c->h_out.data(), n * sizeof(double));
    }
    rtw_stats st{};
    rc = rtw_get_stats(c, &st);
    if (stats) *stats = st;
    return rc;
}

// ------------------------------------------------------------ scenes::simple
struct rtw_world {
    rtw::FlatScene flat;
    rtw_scene view;
    rtw_camera_builder cam;
};

rtw_world* rtw_scene_simple(uint64_t seed, int grid_n) {
    if (grid_n < 0) return nullptr;
    try {
        auto t = rtw::scenes::simple(seed, grid_n);
        rtw_world* w = new rtw_world();
        w->flat = rtw::flatten(std::get<0>(t), std::get<1>(t));
        w->view = w->flat.view();
        w->cam = std::get<2>(t).raw();
        return w;
    } catch (...) {
        return nullptr;
    }
}
const rtw_scene* rtw_world_scene(const rtw_world* w) { return w ? &w->view : nullptr; }
void rtw_world_camera_builder(const rtw_world* w, rtw_camera_builder* out) {
    if (w && out) *out = w->cam;
}
void rtw_world_free(rtw_world* w) { delete w; }

rtw_world* rtw_scene_named(const char* name, uint64_t seed) {
    if (!name) return nullptr;
    const std::string n = name;
    if (n == "simple") return rtw_scene_simple(seed, 11);
    try {
        std::tuple<rtw::HittableList, rtw::HittableList, rtw::CameraBuilder> t;
        if (n == "cornell_box") t = rtw::scenes::cornell_box();
        else if (n == "debug") t = rtw::scenes::debugging_scene(seed);
        else if (n == "checkered_spheres") t = rtw::scenes::checkered_spheres();
        else if (n == "perlin_spheres") t = rtw::scenes::perlin_spheres(seed);
        else if (n == "plane") t = rtw::scenes::plane();
        else if (n == "simple_light") t = rtw::scenes::simple_light(seed);
        else if (n == "simple_transform") t = rtw::scenes::simple_transform(seed);
        else return nullptr;
        rtw_world* w = new rtw_world();
        w->flat = rtw::flatten(std::get<0>(t), std::get<1>(t));
        w->view = w->flat.view();
        w->cam = std::get<2>(t).raw();
        return w;
    } catch (...) {
    }
    return nullptr;
}

int rtw_perlin_generate(uint64_t seed, double* rand_vec, uint32_t* perm) {
    if (!rand_vec || !perm) return RTW_E_INVALID;
    auto p = rtw::Perlin::generate(seed);
    memcpy(rand_vec, p->rand_vec.data(), sizeof(double) * 768);
    memcpy(perm, p->perm.data(), sizeof(uint32_t) * 768);
    return RTW_OK;
}

// ------------------------------------------------------------ output encoding
static uint8_t to_u8(double x) {
    // (256. * x.clamp(0., 1.)) as u8 -- saturating cast, NaN -> 0 (colour.rs:32-34)
    double c = x != x ? x : (x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x));
    double v = 256.0 * c;
    if (!(v > 0.0)) return 0;
    if (v >= 255.0) return 255;
    return (uint8_t)v;
}

}  // extern "C"

namespace {
// write_colour, colour.rs:14-36: scale = (spp as f64).recip(); sqrt(c * scale),
// on the f64 value of each sum (an f32 sum is widened exactly first); rows in
// reverse, main.rs:97-104
template <typename S>
int encode_rgb8(const S* sums, uint32_t W, uint32_t H, uint32_t spp, uint8_t* out) {
    if ((!sums || !out) && W && H) return RTW_E_INVALID;
    const double scale = 1.0 / (double)(int32_t)spp;
    for (uint32_t r = 0; r < H; ++r) {
        const uint32_t j = H - 1 - r;
        for (uint32_t i = 0; i < W; ++i)
            for (int k = 0; k < 3; ++k)
                out[((size_t)r * W + i) * 3 + k] = to_u8(sqrt((double)sums[((size_t)j * W + i) * 3 + k] * scale));
    }
    return RTW_OK;
}

template <typename S>
int write_ppm(const char* path, const S* sums, uint32_t W, uint32_t H, uint32_t spp) {
    if (!path) return RTW_E_INVALID;
    std::vector<uint8_t> rgb((size_t)W * H * 3);
    int rc = encode_rgb8(sums, W, H, spp, rgb.data());
    if (rc) return rc;
    FILE* f = fopen(path, "wb");
    if (!f) return RTW_E_INVALID;
    int n = fprintf(f, "P3\n%u %u\n255\n", W, H);
    for (size_t p = 0; p < (size_t)W * H; ++p)
        n += fprintf(f, "%u %u %u\n", rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2]);
    fclose(f);
    return n;
}
}  // namespace

extern "C" {

int rtw_encode_rgb8(const double* sums, uint32_t W, uint32_t H, uint32_t spp, uint8_t* out) {
    return encode_rgb8(sums, W, H, spp, out);
}
int rtw_encode_rgb8_f32(const float* sums, uint32_t W, uint32_t H, uint32_t spp, uint8_t* out) {
    return encode_rgb8(sums, W, H, spp, out);
}
int rtw_write_ppm(const char* path, const double* sums, uint32_t W, uint32_t H, uint32_t spp) {
    return write_ppm(path, sums, W, H, spp);
}
int rtw_write_ppm_f32(const char* path, const float* sums, uint32_t W, uint32_t H, uint32_t spp) {
    return write_ppm(path, sums, W, H, spp);
}

}  // extern "C"
