// rtw_host.cpp -- implementation of the C++ host mirror (see rtw_host.hpp).
#include "rtw_host.hpp"

#include <math.h>
#include <string.h>

#include <cstdio>
#include <functional>
#include <unordered_map>

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
uint64_t HostRng::uniform_u64(uint64_t low, uint64_t high) {
    // rand 0.8.6 UniformInt<usize>::new(low, high) = new_inclusive(low, high - 1):
    // range = high - low, zone = u64::MAX - (2^64 - range) % range; sample:
    // (hi, lo) = next_u64 * range, accept lo <= zone, return low + hi
    const uint64_t range = high - low;
    const uint64_t reject = (0 - range) % range;   // (u64::MAX - range + 1) % range
    const uint64_t zone = ~0ULL - reject;
    for (;;) {
        const unsigned __int128 m = (unsigned __int128)next() * range;
        if ((uint64_t)m <= zone) return low + (uint64_t)(m >> 64);
    }
}
Vec3 HostRng::unit_sphere() {
    for (;;) {
        const double a = 2.0 * standard() - 1.0, b = 2.0 * standard() - 1.0, c = 2.0 * standard() - 1.0;
        if (a * a + b * b + c * c < 1.0) return {a, b, c};
    }
}

// ---------------------------------------------------------------- textures
std::shared_ptr<const Perlin> Perlin::generate(uint64_t seed) {
    auto p = std::make_shared<Perlin>();
    HostRng rng(seed);
    for (int i = 0; i < 256; ++i) {            // perlin.rs:47-51
        const Vec3 v = rng.unit_sphere();
        p->rand_vec[3 * i] = v.x;
        p->rand_vec[3 * i + 1] = v.y;
        p->rand_vec[3 * i + 2] = v.z;
    }
    for (int axis = 0; axis < 3; ++axis) {     // perlin_generate_perm, perlin.rs:30-44
        uint32_t* perm = p->perm.data() + 256 * axis;
        for (uint32_t i = 0; i < 256; ++i) perm[i] = i;
        for (uint64_t i = 0; i < 255; ++i) {
            const uint64_t j = rng.uniform_u64(i, 256);
            std::swap(perm[i], perm[j]);
        }
    }
    return p;
}
std::shared_ptr<const Texture> Texture::solid(Colour c) {
    auto t = std::make_shared<Texture>();
    t->kind = RTW_TEX_SOLID;
    t->colour = c;
    return t;
}
std::shared_ptr<const Texture> Texture::checker(std::shared_ptr<const Texture> even,
                                                std::shared_ptr<const Texture> odd, double scale) {
    auto t = std::make_shared<Texture>();
    t->kind = RTW_TEX_CHECKER;
    t->scale = 1.0 / scale;                    // inv_scale: scale.recip(), texture.rs:32-38
    t->even = std::move(even);
    t->odd = std::move(odd);
    return t;
}
std::shared_ptr<const Texture> Texture::checker(Colour even, Colour odd, double scale) {
    return checker(solid(even), solid(odd), scale);
}
std::shared_ptr<const Texture> Texture::noise(double scale, uint64_t perlin_seed) {
    auto t = std::make_shared<Texture>();
    t->kind = RTW_TEX_NOISE;
    t->scale = scale;
    t->perlin = Perlin::generate(perlin_seed);
    return t;
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
    s.mat_tex = textured ? mat_tex.data() : nullptr;
    s.n_textures = (uint32_t)tex_type.size();
    s.tex_type = tex_type.data();
    s.tex_params = tex_params.data();
    s.tex_refs = tex_refs.data();
    s.n_perlin = (uint32_t)(perlin_perm.size() / 768);
    s.perlin_vec = perlin_vec.data();
    s.perlin_perm = perlin_perm.data();
    s.n_light_other = n_light_other;
    s.light_flags = light_flags;
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
    // textures and Perlin tables, each shared object once (Arc identity)
    std::unordered_map<const Texture*, uint32_t> tex_ids;
    std::vector<const Perlin*> perlin_ids;
    std::function<uint32_t(const std::shared_ptr<const Texture>&)> push_tex =
        [&](const std::shared_ptr<const Texture>& t) -> uint32_t {
        auto it = tex_ids.find(t.get());
        if (it != tex_ids.end()) return it->second;
        const uint32_t id = (uint32_t)f.tex_type.size();
        tex_ids.emplace(t.get(), id);
        f.tex_type.push_back(t->kind);
        f.tex_params.insert(f.tex_params.end(), {t->colour.x, t->colour.y, t->colour.z, t->scale});
        f.tex_refs.insert(f.tex_refs.end(), {0u, 0u});
        if (t->kind == RTW_TEX_CHECKER) {
            const uint32_t e = push_tex(t->even), o = push_tex(t->odd);
            f.tex_refs[2 * id] = e;
            f.tex_refs[2 * id + 1] = o;
        } else if (t->kind == RTW_TEX_NOISE) {
            uint32_t q = 0;
            while (q < perlin_ids.size() && perlin_ids[q] != t->perlin.get()) ++q;
            if (q == perlin_ids.size()) {
                perlin_ids.push_back(t->perlin.get());
                f.perlin_vec.insert(f.perlin_vec.end(), t->perlin->rand_vec.begin(), t->perlin->rand_vec.end());
                f.perlin_perm.insert(f.perlin_perm.end(), t->perlin->perm.begin(), t->perlin->perm.end());
            }
            f.tex_refs[2 * id] = q;
        }
        return id;
    };
    auto textured = [](const Material& m) {
        return m.texture && (m.type == RTW_LAMBERTIAN || m.type == RTW_DIFFUSE_LIGHT);
    };
    for (const Plane& o : world.planes()) f.textured |= textured(o.mat);
    for (const Sphere& o : world.spheres()) f.textured |= textured(o.mat);
    for (const Quad& o : world.quads()) f.textured |= textured(o.mat);
    for (const Cuboid& o : world.cuboids()) f.textured |= textured(o.mat);
    auto push_mat = [&](const Material& m) {
        f.mat_type.push_back(m.type);
        f.mat_params.insert(f.mat_params.end(), {m.albedo.x, m.albedo.y, m.albedo.z, m.fuzz, m.ior});
        if (f.textured) {
            // a material without a texture gets its SolidColour as one
            if (textured(m)) {
                f.mat_tex.push_back(push_tex(m.texture));
            } else {
                f.mat_tex.push_back((uint32_t)f.tex_type.size());
                f.tex_type.push_back(RTW_TEX_SOLID);
                f.tex_params.insert(f.tex_params.end(), {m.albedo.x, m.albedo.y, m.albedo.z, 0.0});
                f.tex_refs.insert(f.tex_refs.end(), {0u, 0u});
            }
        }
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
    // Planes and Transformed<Cuboid>s have no pdf_value / random of their own:
    // in a light list they are RTW_LIGHT_DEFAULT entries (hittable.rs:175-181)
    for (const auto& e : lights.order()) {
        if (e.first == HittableList::kSphere) {
            const Sphere& s = lights.spheres()[e.second];
            f.lights.insert(f.lights.end(), {s.center.x, s.center.y, s.center.z, s.radius});
            f.light_kinds.push_back(RTW_LIGHT_SPHERE);
        } else if (e.first == HittableList::kQuad) {
            const Quad& q = lights.quads()[e.second];
            f.light_quads.insert(f.light_quads.end(),
                                 {q.q.x, q.q.y, q.q.z, q.u.x, q.u.y, q.u.z, q.v.x, q.v.y, q.v.z});
            f.light_kinds.push_back(RTW_LIGHT_QUAD);
        } else {
            f.light_kinds.push_back(RTW_LIGHT_DEFAULT);
            ++f.n_light_other;
        }
    }
    if (lights.is_bvh()) {
        if (lights.len() > 5)
            throw Error(RTW_E_UNSUPPORTED, "a BVH light list of more than 5 entries (bvh.rs:78-92)");
        f.light_flags |= RTW_LIGHTS_BVH_LEAF;
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
    rtw_ctx* ctx = nullptr;
    if (opt.device_mask) {
        // the mask's error code: RTW_E_INVALID (empty, or a device that is not
        // visible) vs RTW_E_DEVICE (HIP / RCCL) -- both surface, neither narrows the mask
        const int mrc = rtw_create_mask_ex(opt.device_mask, opt.precision, &ctx);
        if (mrc != RTW_OK)
            throw Error(mrc, mrc == RTW_E_INVALID ? "rtw_create_mask_ex: empty mask or a device that is not visible ("
                                                    + std::to_string(rtw_visible_devices()) + " visible)"
                                                  : "rtw_create_mask_ex: HIP / RCCL failure");
    } else {
        ctx = rtw_create(opt.device, opt.precision);
        if (!ctx) throw Error(RTW_E_DEVICE, "rtw_create failed (no gfx950 device?)");
    }
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

namespace {
double dist(Point3 a, Point3 b) {   // (lookfrom - lookat).length()
    const Vec3 d{a.x - b.x, a.y - b.y, a.z - b.z};
    return sqrt(vdot(d, d));
}
// the eight wall quads of debugging_scene / simple_transform (lib.rs:416-466, :549-599)
void add_walls(HittableList& world, const Material& white) {
    const double c[4][2] = {{6, 6}, {-6, 6}, {-6, -6}, {6, -6}};
    for (const auto& xz : c) {
        const double sx = xz[0] > 0 ? -2.0 : 2.0, sz = xz[1] > 0 ? -2.0 : 2.0;
        world.add(Quad{{xz[0], 0, xz[1]}, {0, 2, 0}, {sx, 0, 0}, white});
        world.add(Quad{{xz[0], 0, xz[1]}, {0, 2, 0}, {0, 0, sz}, white});
    }
}
}  // namespace

std::tuple<HittableList, HittableList, CameraBuilder> perlin_spheres(uint64_t seed) {
    HittableList world, lights;
    const Material pertext = Material::lambertian_tex(Texture::noise(4.0, seed));
    world.add(Plane({0, 0, 0}, {0, 1, 0}, pertext));
    world.add(Sphere{{0, 2, 0}, 2.0, pertext});
    world.add(Sphere{{-5, 1, 5}, 1.0, Material::lambertian({1, 0, 0})});
    world.add(Sphere{{-5, 1, -5}, 1.0, Material::lambertian({0, 1, 0})});
    world.add(Sphere{{5, 1, -5}, 1.0, Material::lambertian({0, 0, 1})});
    world.add(Sphere{{5, 1, 5}, 1.0, Material::lambertian({0.5, 0, 0.5})});
    const Point3 lookfrom{0, 30, 0}, lookat{0, 0, 0};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(dist(lookfrom, lookat)).with_vfov(40.0)
        .with_background({1, 1, 1});
    return {std::move(world), std::move(lights), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> plane() {
    HittableList world, lights;
    world.add(Plane({0, 0, 0}, {0, 1, 0},
                    Material::lambertian_tex(Texture::checker(Colour{0.2, 0.3, 0.1}, Colour{0.9, 0.9, 0.9}, 0.32))));
    const Point3 lookfrom{0, 30, 0}, lookat{0, 0, 0};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(dist(lookfrom, lookat)).with_vfov(40.0)
        .with_background({1, 1, 1});
    return {std::move(world), std::move(lights), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> checkered_spheres() {
    HittableList world, lights;
    const Material checker =
        Material::lambertian_tex(Texture::checker(Colour{0.2, 0.3, 0.1}, Colour{0.9, 0.9, 0.9}, 0.01));
    world.add(Sphere{{0, -10, 0}, 10.0, checker});
    world.add(Sphere{{0, 10, 0}, 10.0, checker});
    lights.add(Sphere{{0, 0, 0}, 0.1, checker});
    const Point3 lookfrom{40, 1, 0}, lookat{0, 0, 0};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(dist(lookfrom, lookat)).with_vfov(40.0)
        .with_background({1, 1, 1});
    return {std::move(world), std::move(lights), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> simple_light(uint64_t seed) {
    HittableList world, lights;
    const Material pertext = Material::lambertian_tex(Texture::noise(4.0, seed));
    const Material difflight = Material::diffuse_light({4, 4, 4});
    world.add(Plane({0, 0, 0}, {0, 1, 0}, pertext));
    world.add(Sphere{{0, 2, 0}, 2.0, pertext});
    world.add(Quad{{3, 1, -2}, {2, 0, 0}, {0, 2, 0}, difflight});
    lights.add(Quad{{3, 1, -2}, {2, 0, 0}, {0, 2, 0}, difflight});
    const Point3 lookfrom{26, 3, 6}, lookat{0, 2, 0};
    CameraBuilder cam;
    cam.with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(dist(lookfrom, lookat)).with_vfov(40.0);
    return {std::move(world), std::move(lights), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> debugging_scene(uint64_t seed) {
    HittableList world, lights;
    const Material pertext = Material::lambertian_tex(Texture::noise(4.0, seed));
    world.add(Plane({0, 0, 0}, {0, 1, 0}, pertext));
    world.add(Sphere{{0, 2, 0}, 2.0, pertext});
    add_walls(world, Material::lambertian({0.75, 0.75, 0.75}));
    const Sphere ls[4] = {{{5, 1, 5}, 1.0, Material::diffuse_light({0.5, 0, 0.5})},
                          {{-5, 1, 5}, 1.0, Material::diffuse_light({1, 0, 0})},
                          {{-5, 1, -5}, 1.0, Material::diffuse_light({0, 1, 0})},
                          {{5, 1, -5}, 1.0, Material::diffuse_light({0, 0, 1})}};
    for (const Sphere& s : ls) {
        world.add(s);
        lights.add(s);
    }
    const Point3 lookfrom{0, 20, 0}, lookat{0, 0, 0};
    CameraBuilder cam;
    cam.with_image_width(3).with_image_height(2).with_samples_per_pixel(10).with_max_depth(5)
        .with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(4.0);
    return {world.into_bvh(), lights.into_bvh(), cam};
}

std::tuple<HittableList, HittableList, CameraBuilder> simple_transform(uint64_t seed) {
    HittableList world, lights;
    const Material pertext = Material::lambertian_tex(Texture::noise(4.0, seed));
    world.add(Plane({0, 0, 0}, {0, 1, 0}, pertext));
    add_walls(world, Material::lambertian({0.75, 0.75, 0.75}));
    const Cuboid original{{0, 0, 0}, {1, 1, 1}, Material::diffuse_light({1, 0, 0})};
    const Cuboid boxes[3] = {
        original.transform(Transformation::translation({-0.5, 0, -0.5})),
        original.transform(Transformation::translation({2, 0, 2})),
        original.transform(Transformation::translation({-3, 0, -3})).transform(Transformation::rotation(45.0, 1))};
    for (const Cuboid& c : boxes) {
        world.add(c);
        lights.add(c);
    }
    const Point3 lookfrom{0, 20, 0}, lookat{0, 0, 0};
    CameraBuilder cam;
    cam.with_image_width(3).with_image_height(2).with_samples_per_pixel(10).with_max_depth(5)
        .with_lookfrom(lookfrom).with_lookat(lookat).with_focus_dist(4.0);
    return {world.into_bvh(), lights.into_bvh(), cam};
}
}  // namespace scenes

}  // namespace rtw
