// rtw_host.hpp -- C++ host mirror of the reference's interface for the hot
// path: the types a caller of Camera::render builds (world + lights lists,
// materials, CameraBuilder) and the scenes::simple generator, flattened to the
// C-ABI's SoA rtw_scene and rendered by the gfx950 kernels through rtw.h.
//
// Mirrors (paths relative to N9199/ray_tracing_weekend):
//   CameraBuilder / Camera        shared/src/camera.rs:28-261
//   Camera::render(world, lights) shared/src/camera.rs:295-297
//   HittableList::add             shared/src/hittable_collections/hittable_list.rs:270-294
//   Sphere / Plane                shared/src/entities/sphere.rs:24-47, plane.rs:20-38
//   Lambertian/Metal/Dialectric/Invisible   shared/src/material.rs:321-488
//   SampledColour (+ Display)     shared/src/colour.rs:14-36, 136-148
//   SolidColour / CheckerTexture / NoiseTexture   shared/src/texture.rs:15-102
//   Perlin::new                   shared/src/perlin.rs:27-58
//   BoundedVolumeHierarchy::from  shared/src/hittable_collections/bvh.rs:106-143 (as a list flag)
//   the scene generators          scenes/src/lib.rs:40-653
#pragma once

#include <stdint.h>

#include <array>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../../include/rtw.h"

namespace rtw {

struct Vec3 {
    double x = 0, y = 0, z = 0;
};
using Point3 = Vec3;
using Colour = Vec3;

// Perlin::new (perlin.rs:46-58) from the build's seeded RNG (the reference
// draws the tables from thread_rng): rand_vec = 256 UnitSphere samples, then
// perm_x, perm_y, perm_z, each the identity shuffled by j = Uniform::new(i, 256).
struct Perlin {
    std::array<double, 768> rand_vec{};
    std::array<uint32_t, 768> perm{};   // perm_x, perm_y, perm_z
    static std::shared_ptr<const Perlin> generate(uint64_t seed);
};

// Arc<dyn Texture>: SolidColour, CheckerTexture (even / odd textures and
// inv_scale = scale.recip()), NoiseTexture (scale + its own Perlin).
struct Texture {
    uint32_t kind = RTW_TEX_SOLID;
    Colour colour{};
    double scale = 1.0;                 // checker: inv_scale; noise: scale
    std::shared_ptr<const Texture> even, odd;
    std::shared_ptr<const Perlin> perlin;
    static std::shared_ptr<const Texture> solid(Colour c);
    static std::shared_ptr<const Texture> checker(std::shared_ptr<const Texture> even,
                                                  std::shared_ptr<const Texture> odd, double scale);
    static std::shared_ptr<const Texture> checker(Colour even, Colour odd, double scale);   // new_with_colours
    static std::shared_ptr<const Texture> noise(double scale, uint64_t perlin_seed);
};

// One material record.  DynMaterial in the reference is a pointer to a trait
// object; here it is a small value type with the parameters the kernels read.
// `texture` (Lambertian, DiffuseLight) null = SolidColour(albedo).
struct Material {
    uint32_t type = RTW_INVISIBLE;
    Colour albedo{};
    double fuzz = 0.0;
    double ior = 0.0;
    std::shared_ptr<const Texture> texture;

    static Material lambertian(Colour albedo) { return {RTW_LAMBERTIAN, albedo, 0.0, 0.0, nullptr}; }
    static Material lambertian_tex(std::shared_ptr<const Texture> t) { return {RTW_LAMBERTIAN, {}, 0.0, 0.0, t}; }
    static Material metal(Colour albedo, double fuzz) { return {RTW_METAL, albedo, fuzz, 0.0, nullptr}; }
    static Material dialectric(double ior) { return {RTW_DIELECTRIC, {1, 1, 1}, 0.0, ior, nullptr}; }
    static Material invisible() { return {RTW_INVISIBLE, {0, 0, 0}, 0.0, 0.0, nullptr}; }
    static Material diffuse_light(Colour emit) { return {RTW_DIFFUSE_LIGHT, emit, 0.0, 0.0, nullptr}; }
    static Material diffuse_light_tex(std::shared_ptr<const Texture> t) { return {RTW_DIFFUSE_LIGHT, {}, 0.0, 0.0, t}; }
};

struct Sphere {
    Point3 center;
    double radius = 0;
    Material mat;
};

struct Plane {
    Point3 point;
    Vec3 normal;  // normalized at construction, plane.rs:175
    Material mat;
    Plane(Point3 p, Vec3 n, Material m);
};

// Quad::new(Q, u, v, mat), quadrilateral.rs:37-56
struct Quad {
    Point3 q;
    Vec3 u, v;
    Material mat;
};

// geometry::transformations::Transformation (non-euclid build): p -> R p + T;
// then() composes in call order (transformations.rs:97-108).
struct Transformation {
    double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    Vec3 T{};
    Transformation then(const Transformation& b) const;
    static Transformation translation(Vec3 t);
    static Transformation rotation(double angle_deg, int axis);   // axis 0/1/2 = X/Y/Z
};

// Cuboid::new(p, q, mat) (cuboid.rs:26-47), optionally .transform()ed
struct Cuboid {
    Point3 p, q;
    Material mat;
    Transformation xform{};
    Cuboid transform(const Transformation& t) const {
        Cuboid c = *this;
        c.xform = xform.then(t);
        return c;
    }
};

// A world or light list.  The primitives this build renders: Sphere, Plane,
// Quad, (transformed) Cuboid; Triangle is outside it.  Insertion order is
// kept: it is the light list's order (pdf sum, uniform pick).
class HittableList {
   public:
    enum Kind : uint8_t { kSphere, kPlane, kQuad, kCuboid };
    void add(const Sphere& s) { order_.push_back({kSphere, spheres_.size()}); spheres_.push_back(s); }
    void add(const Plane& p) { order_.push_back({kPlane, planes_.size()}); planes_.push_back(p); }
    void add(const Quad& q) { order_.push_back({kQuad, quads_.size()}); quads_.push_back(q); }
    void add(const Cuboid& c) { order_.push_back({kCuboid, cuboids_.size()}); cuboids_.push_back(c); }
    const std::vector<Cuboid>& cuboids() const { return cuboids_; }
    size_t len() const { return order_.size(); }
    bool is_empty() const { return len() == 0; }
    const std::vector<Sphere>& spheres() const { return spheres_; }
    const std::vector<Plane>& planes() const { return planes_; }
    const std::vector<Quad>& quads() const { return quads_; }
    const std::vector<std::pair<Kind, size_t>>& order() const { return order_; }
    // BoundedVolumeHierarchy::from(list) (bvh.rs:106-143): the same closest
    // hit as the list; as a light list its pdf_value is (sum / n * n) / n
    // (a leaf, n <= 5; deeper BVH light lists are outside this build)
    HittableList into_bvh() const {
        HittableList h = *this;
        h.bvh_ = true;
        return h;
    }
    bool is_bvh() const { return bvh_; }

   private:
    bool bvh_ = false;
    std::vector<Sphere> spheres_;
    std::vector<Plane> planes_;
    std::vector<Quad> quads_;
    std::vector<Cuboid> cuboids_;
    std::vector<std::pair<Kind, size_t>> order_;
};

// Flattened (SoA) world + lights; owns the arrays an rtw_scene points into.
struct FlatScene {
    std::vector<double> spheres, planes, quads, mat_params, lights, light_quads, boxes;
    std::vector<uint32_t> sphere_mat, plane_mat, quad_mat, mat_type, light_kinds, box_mat;
    std::vector<uint32_t> mat_tex, tex_type, tex_refs, perlin_perm;
    std::vector<double> tex_params, perlin_vec;
    uint32_t n_light_other = 0, light_flags = 0;
    bool textured = false;
    rtw_scene view() const;
};
// world's spheres/planes/quads with one material record each; lights
// contribute their geometry only, in list order (their material is never
// consulted on the path).
FlatScene flatten(const HittableList& world, const HittableList& lights);

// SampledColour(sum, spp) -- colour.rs:136-148
struct SampledColour {
    Colour sum;
    int32_t spp = 1;
    std::array<uint8_t, 3> rgb8() const;   // write_colour, colour.rs:14-36
    std::string to_string() const;         // Display: "r g b"
};

class Camera;

class CameraBuilder {
   public:
    CameraBuilder();
    CameraBuilder& with_aspect_ratio(double v) { b_.has_aspect_ratio = 1; b_.aspect_ratio = v; return *this; }
    CameraBuilder& with_image_width(uint32_t v) { b_.has_image_width = 1; b_.image_width = v; return *this; }
    CameraBuilder& with_image_height(uint32_t v) { b_.has_image_height = 1; b_.image_height = v; return *this; }
    CameraBuilder& with_samples_per_pixel(uint32_t v) { b_.samples_per_pixel = v; return *this; }
    CameraBuilder& with_max_depth(uint32_t v) { b_.max_depth = v; return *this; }
    CameraBuilder& with_background(Colour c) { b_.background[0] = c.x; b_.background[1] = c.y; b_.background[2] = c.z; return *this; }
    CameraBuilder& with_vfov(double v) { b_.vfov = v; return *this; }
    CameraBuilder& with_lookfrom(Point3 p) { b_.lookfrom[0] = p.x; b_.lookfrom[1] = p.y; b_.lookfrom[2] = p.z; return *this; }
    CameraBuilder& with_lookat(Point3 p) { b_.lookat[0] = p.x; b_.lookat[1] = p.y; b_.lookat[2] = p.z; return *this; }
    CameraBuilder& with_vup(Vec3 v) { b_.vup[0] = v.x; b_.vup[1] = v.y; b_.vup[2] = v.z; return *this; }
    CameraBuilder& with_defocus_angle(double v) { b_.defocus_angle = v; return *this; }
    CameraBuilder& with_focus_dist(double v) { b_.focus_dist = v; return *this; }
    Camera build() const;
    const rtw_camera_builder& raw() const { return b_; }
    explicit CameraBuilder(const rtw_camera_builder& b) : b_(b) {}

   private:
    rtw_camera_builder b_;
};

// Options for the device render that the reference has no equivalent of.
struct RenderOptions {
    uint64_t seed = 0x5EED0001ULL;  // the reference seeds from thread_rng (non-deterministic)
    int device = 0;
    uint64_t device_mask = 0;       // != 0: one rank per set bit (rtw_create_mask), `device` unused
    int precision = RTW_F64;        // the parity mode (the reference's sums); RTW_F32: the speed mode
    int accel = RTW_ACCEL_AUTO;
};

class Camera {
   public:
    explicit Camera(const rtw_camera& c) : c_(c) {}
    // Camera::render -- rows indexed [j][i], j = 0 the bottom row.
    std::vector<std::vector<SampledColour>> render(const HittableList& world,
                                                   const HittableList& lights,
                                                   const RenderOptions& opt = {}) const;
    // render_debug: the reference's sequential debug path; on the GPU it is the
    // same render (there is no sequential mode to emulate).
    std::vector<std::vector<SampledColour>> render_debug(const HittableList& world,
                                                         const HittableList& lights,
                                                         const RenderOptions& opt = {}) const {
        return render(world, lights, opt);
    }
    const rtw_camera& raw() const { return c_; }

   private:
    rtw_camera c_;
};

namespace scenes {
// scenes::simple restated with the build's seeded RNG; grid a, b in [-n, n).
std::tuple<HittableList, HittableList, CameraBuilder> simple(uint64_t seed, int n = 11);
// scenes::cornell_box (scenes/src/lib.rs:292-395)
std::tuple<HittableList, HittableList, CameraBuilder> cornell_box();
// the other generators (scenes/src/lib.rs); `seed` drives the Perlin tables
std::tuple<HittableList, HittableList, CameraBuilder> perlin_spheres(uint64_t seed);     // :40-89
std::tuple<HittableList, HittableList, CameraBuilder> plane();                           // :91-121
std::tuple<HittableList, HittableList, CameraBuilder> checkered_spheres();               // :123-153
std::tuple<HittableList, HittableList, CameraBuilder> simple_light(uint64_t seed);       // :235-290
std::tuple<HittableList, HittableList, CameraBuilder> debugging_scene(uint64_t seed);    // :397-530
std::tuple<HittableList, HittableList, CameraBuilder> simple_transform(uint64_t seed);   // :532-653
}  // namespace scenes

// host RNG used by the scene generator (the same xoshiro256++/splitmix64 and
// rand 0.8.6 distributions as the device path)
class HostRng {
   public:
    explicit HostRng(uint64_t seed);  // SmallRng::seed_from_u64
    uint64_t next();
    double standard();                               // Standard f64
    double uniform_incl(double low, double high);    // Uniform::new_inclusive(low, high).sample
    uint64_t uniform_u64(uint64_t low, uint64_t high);   // Uniform::new(low, high).sample (usize)
    Vec3 unit_sphere();                              // utils.rs:99-122 (shuffle not drawn)

   private:
    uint64_t s_[4];
};

class Error : public std::runtime_error {
   public:
    Error(int code, const std::string& msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }

   private:
    int code_;
};

}  // namespace rtw
