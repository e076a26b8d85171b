// rtw_host.cpp -- implementation of the C++ host mirror (see rtw_host.hpp).
#include "rtw_host.hpp"

#include <math.h>
#include <string.h>

#include <cstdio>

namespace rtw {

namespace {
inline double vdot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3 vnormalize(Vec3 a) {   // vec.rs:86-94
    double l = sqrt(vdot(a, a));
    return {a.x / l, a.y / l, a.z / l};
}
inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline double unit12(uint64_t v) {
    uint64_t b = (v >> 12) | 0x3FF0000000000000ULL;
    double d;
    memcpy(&d, &b, 8);
    return d;
}
}  // namespace

Plane::Plane(Point3 p, Vec3 n, Material m) : point(p), normal(vnormalize(n)), mat(m) {}

// ---------------------------------------------------------------- HostRng
HostRng::HostRng(uint64_t seed) {
    uint64_t k = seed;
    for (int i = 0; i < 4; ++i) {
        k += 0x9E3779B97F4A7C15ULL;
        s_[i] = mix64(k);
    }
}
uint64_t HostRng::next() {
    uint64_t result = ((s_[0] + s_[3]) << 23 | (s_[0] + s_[3]) >> 41) + s_[0];
    uint64_t t = s_[1] << 17;
    s_[2] ^= s_[0];
    s_[3] ^= s_[1];
    s_[1] ^= s_[2];
    s_[0] ^= s_[3];
    s_[2] ^= t;
    s_[3] = (s_[3] << 45) | (s_[3] >> 19);
    return result;
}
double HostRng::standard() { return (1.0 / 9007199254740992.0) * (double)(next() >> 11); }
double HostRng::uniform_incl(double low, double high) {
    // rand 0.8.6 UniformFloat::new_inclusive + sample
    double max_rand = unit12(~0ULL) - 1.0;
    double scale = (high - low) / max_rand;
    while (scale * max_rand + low > high) {
        uint64_t b;
        memcpy(&b, &scale, 8);
        b -= 1;
        memcpy(&scale, &b, 8);
    }
    double v01 = unit12(next()) - 1.0;
    return v01 * scale + low;
}

// ---------------------------------------------------------------- flatten
rtw_scene FlatScene::view() const {
    rtw_scene s;
    s.n_spheres = (uint32_t)sphere_mat.size();
    s.spheres = spheres.data();
    s.sphere_mat = sphere_mat.data();
    s.n_planes = (uint32_t)plane_mat.size();
    s.planes = planes.data();
    s.plane_mat = plane_mat.data();
    s.n_materials = (uint32_t)mat_type.size();
    s.mat_type = mat_type.data();
    s.mat_params = mat_params.data();
    s.n_lights = (uint32_t)(lights.size() / 4);
    s.lights = lights.data();
    s.n_quads = (uint32_t)quad_mat.size();
    s.quads = quads.data();
    s.quad_mat = quad_mat.data();
    s.n_light_quads = (uint32_t)(light_quads.size() / 9);
    s.light_quads = light_quads.data();
    s.light_kinds = light_kinds.empty() ? nullptr : light_kinds.data();
    s.n_boxes = (uint32_t)box_mat.size();
    s.boxes = boxes.data();
    s.box_mat = box_mat.data();
    return s;
}

// ---------------------------------------------------------------- Transformation
Transformation Transformation::then(const Transformation& b) const {
    // apply(b): rotation = b.R * R, translation = b.T + b.R * T
    Transformation out;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out.R[i][j] = b.R[i][0] * R[0][j] + b.R[i][1] * R[1][j] + b.R[i][2] * R[2][j];
    const double rt[3] = {b.R[0][0] * T.x + b.R[0][1] * T.y + b.R[0][2] * T.z,
                          b.R[1][0] * T.x + b.R[1][1] * T.y + b.R[1][2] * T.z,
                          b.R[2][0] * T.x + b.R[2][1] * T.y + b.R[2][2] * T.z};
    out.T = {b.T.x + rt[0], b.T.y + rt[1], b.T.z + rt[2]};
    return out;
}
Transformation Transformation::translation(Vec3 t) {
    Transformation out;
    out.T = t;
    return out;
}
Transformation Transformation::rotation(double angle_deg, int axis) {
    const double a = angle_deg * (3.14159265358979323846 / 180.0);   // f64::to_radians
    const double c = cos(a), s = sin(a);
    Transformation out;
    const double X[3][3] = {{1, 0, 0}, {0, c, -s}, {0, s, c}};
    const double Y[3][3] = {{c, 0, s}, {0, 1, 0}, {-s, 0, c}};
    const double Z[3][3] = {{c, -s, 0}, {s, c, 0}, {0, 0, 1}};
    const double(*M)[3] = axis == 0 ? X : (axis == 1 ? Y : Z);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out.R[i][j] = M[i][j];
    return out;
}

FlatScene flatten(const HittableList& world, const HittableList& lights) {
    FlatScene f;
    auto push_mat = [&](const Material& m) {
        f.mat_type.push_back(m.type);
        f.mat_params.insert(f.mat_params.end(), {m.albedo.x, m.albedo.y, m.albedo.z, m.fuzz, m.ior});
        return (uint32_t)(f.mat_type.size() - 1);
    };
    for (const Plane& p : world.planes()) {
        f.planes.insert(f.planes.end(),
                        {p.point.x, p.point.y, p.point.z, p.normal.x, p.normal.y, p.normal.z});
        f.plane_mat.push_back(push_mat(p.mat));
    }
    for (const Sphere& s : world.spheres()) {
        f.spheres.insert(f.spheres.end(), {s.center.x, s.center.y, s.center.z, s.radius});
        f.sphere_mat.push_back(push_mat(s.mat));
    }
    for (const Quad& q : world.quads()) {
        f.quads.insert(f.quads.end(), {q.q.x, q.q.y, q.q.z, q.u.x, q.u.y, q.u.z, q.v.x, q.v.y, q.v.z});
        f.quad_mat.push_back(push_mat(q.mat));
    }
    for (const Cuboid& c : world.cuboids()) {
        f.boxes.insert(f.boxes.end(), {c.p.x, c.p.y, c.p.z, c.q.x, c.q.y, c.q.z});
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) f.boxes.push_back(c.xform.R[i][j]);
        f.boxes.insert(f.boxes.end(), {c.xform.T.x, c.xform.T.y, c.xform.T.z});
        f.box_mat.push_back(push_mat(c.mat));
    }
    if (!lights.planes().empty() || !lights.cuboids().empty())
        throw Error(RTW_E_UNSUPPORTED, "planes and cuboids as lights are outside this build's scope");
    for (const auto& e : lights.order()) {
        if (e.first == HittableList::kSphere) {
            const Sphere& s = lights.spheres()[e.second];
            f.lights.insert(f.lights.end(), {s.center.x, s.center.y, s.center.z, s.radius});
            f.light_kinds.push_back(0);
        } else {
            const Quad& q = lights.quads()[e.second];
            f.light_quads.insert(f.light_quads.end(),
                                 {q.q.x, q.q.y, q.q.z, q.u.x, q.u.y, q.u.z, q.v.x, q.v.y, q.v.z});
            f.light_kinds.push_back(1);
        }
    }
    return f;
}

// ---------------------------------------------------------------- SampledColour
std::array<uint8_t, 3> SampledColour::rgb8() const {
    std::array<uint8_t, 3> out{};
    double tmp[3] = {sum.x, sum.y, sum.z};
    rtw_encode_rgb8(tmp, 1, 1, (uint32_t)spp, out.data());
    return out;
}
std::string SampledColour::to_string() const {
    auto c = rgb8();
    char buf[32];
    snprintf(buf, sizeof buf, "%u %u %u", c[0], c[1], c[2]);
    return buf;
}

// ---------------------------------------------------------------- Camera
CameraBuilder::CameraBuilder() { rtw_camera_builder_default(&b_); }

Camera CameraBuilder::build() const {
    rtw_camera c;
    int rc = rtw_camera_build(&b_, &c);
    if (rc != RTW_OK) throw Error(rc, "CameraBuilder::build rejected the builder");
    return Camera(c);
}

std::vector<std::vector<SampledColour>> Camera::render(const HittableList& world,
                                                       const HittableList& lights,
                                                       const RenderOptions& opt) const {
    FlatScene flat = flatten(world, lights);
    rtw_scene view = flat.view();
    rtw_ctx* ctx = rtw_create(opt.device, opt.precision);
    if (!ctx) throw Error(RTW_E_DEVICE, "rtw_create failed (no gfx950 device?)");
    rtw_set_accel(ctx, opt.accel);
    const uint32_t W = c_.image_width, H = c_.image_height;
    std::vector<double> sums((size_t)W * H * 3);
    int rc = rtw_render(ctx, &c_, &view, opt.seed, sums.data(), nullptr);
    std::string err = rc ? rtw_last_error(ctx) : "";
    rtw_destroy(ctx);
    if (rc != RTW_OK) throw Error(rc, "rtw_render: " + err);
    std::vector<std::vector<SampledColour>> out(H, std::vector<SampledColour>(W));
    for (uint32_t j = 0; j < H; ++j)
        for (uint32_t i = 0; i < W; ++i) {
            const double* s = &sums[((size_t)j * W + i) * 3];
            out[j][i] = SampledColour{{s[0], s[1], s[2]}, (int32_t)c_.samples_per_pixel};
        }
    return out;
}

// ---------------------------------------------------------------- scenes
namespace scenes {
std::tuple<HittableList, HittableList, CameraBuilder> simple(uint64_t seed, int n) {
    HittableList lights, world;
    world.add(Plane({0, 0, 0}, {0, 1, 0}, Material::lambertian({0.9, 0.9, 0.9})));
    HostRng rng(seed);
    for (int a = -n; a < n; ++a) {
        for (int b = -n; b < n; ++b) {
            double choose_mat = rng.standard();
            double cx = (double)a + 0.9 * rng.standard();
            double cz = (double)b + 0.9 * rng.standard();
            Point3 center{cx, 0.2, cz};
            Vec3 off{center.x - 4.0, center.y - 0.2, center.z - 0.0};
            if (sqrt(vdot(off, off)) > 0.9) {
                Material mat;
                if (choose_mat < 0.8) {
                    double a1 = rng.standard(), a2 = rng.standard(), a3 = rng.standard();
                    double b1 = rng.standard(), b2 = rng.standard(), b3 = rng.standard();
                    mat = Material::lambertian({a1 * b1, a2 * b2, a3 * b3});
                } else if (choose_mat < 0.95) {
                    double r = rng.uniform_incl(0.5, 1.0);
                    double g = rng.uniform_incl(0.5, 1.0);
                    double bb = rng.uniform_incl(0.5, 1.0);
                    double fuzz = 1.0 - rng.uniform_incl(0.5, 1.0);
                    mat = Material::metal({r, g, bb}, fuzz);
                } else {
                    lights.add(Sphere{center, 0.2, Material::invisible()});
                    mat = Material::dialectric(1.5);
                }
                world.add(Sphere{center, 0.2, mat});
            }
        }
    }
    world.add(Sphere{{0, 1, 0}, 1.0, Material::dialectric(1.5)});
    world.add(Sphere{{-4, 1, 0}, 1.0, Material::lambertian({0.4, 0.2, 0.1})});
    world.add(Sphere{{4, 1, 0}, 1.0, Material::metal({0.7, 0.6, 0.5}, 0.0)});
    lights.add(Sphere{{0, 1, 0}, 1.0, Material::invisible()});

    // camera (lib.rs:219-226) + bin/src/main.rs:73's vfov 40; for n > 11 the
    // camera is pulled back proportionally (synthetic C3/C5 fields)
    double k = n > 11 ? (double)n / 11.0 : 1.0;
    Point3 lookfrom{10.0 * k, 5.0 * k, 10.0 * k}, lookat{0, 0, 0};
    Vec3 d{lookfrom.x - lookat.x, lookfrom.y - lookat.y, lookfrom.z - lookat.z};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom)
        .with_lookat(lookat)
        .with_focus_dist(sqrt(vdot(d, d)))
        .with_vfov(40.0)
        .with_background({1, 1, 1});
    return {std::move(world), std::move(lights), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> cornell_box() {
    // scenes/src/lib.rs:292-395
    HittableList world, lights;
    const Material red = Material::lambertian({0.65, 0.05, 0.05});
    const Material white = Material::lambertian({0.73, 0.73, 0.73});
    const Material green = Material::lambertian({0.12, 0.45, 0.15});
    const Material light = Material::diffuse_light({15.0, 15.0, 15.0});
    const Material glass = Material::dialectric(1.5);
    world.add(Quad{{555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green});
    world.add(Quad{{0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red});
    world.add(Quad{{0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white});
    world.add(Quad{{0, 555, 0}, {555, 0, 0}, {0, 0, 555}, white});
    world.add(Quad{{0, 0, 555}, {0, 555, 0}, {555, 0, 0}, white});
    world.add(Cuboid{{0, 0, 0}, {165, 330, 165}, white}
                  .transform(Transformation::translation({265, 0, 295}))
                  .transform(Transformation::rotation(15.0, 1)));
    world.add(Sphere{{190, 90, 190}, 90.0, glass});
    world.add(Quad{{343, 554, 332}, {-130, 0, 0}, {0, 0, -105}, light});
    lights.add(Quad{{343, 554, 332}, {-130, 0, 0}, {0, 0, -105}, light});
    lights.add(Sphere{{190, 90, 190}, 90.0, glass});
    const Point3 lookfrom{277.5, 277.5, -800.0}, lookat{277.5, 277.5, 0.0};
    const Vec3 d{lookfrom.x - lookat.x, lookfrom.y - lookat.y, lookfrom.z - lookat.z};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom).with_lookat(lookat).with_vfov(40.0).with_defocus_angle(0.0).with_focus_dist(
        sqrt(vdot(d, d)));
    return {std::move(world), std::move(lights), cam};
}
}  // namespace scenes

}  // namespace rtw
