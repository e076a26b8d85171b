// rtw -- the reference's bin/ (bin/src/main.rs:54-105) on the C++ host mirror:
// reads ./Config.toml's [image] table (bin/src/config.rs:3-107), builds the
// scene, applies main.rs:72-79's camera overrides, renders on the GPU and
// writes image.ppm (P3, rows top to bottom).
//
//   rtw <scene> [--debug] [--seed N] [--f64] [--device N | --device-mask M] [--config PATH] [--out PATH]
//
// <scene> is one of clap's ValueEnum names of main.rs:29-38 (cornell-box,
// debug, checkered-spheres, perlin-spheres, plane, simple, simple-light,
// simple-transform; snake_case accepted too).  --seed drives simple's
// generator and the Perlin tables (the reference uses thread_rng).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <string>

#include "host/rtw_host.hpp"

namespace {

std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// A minimal reader for the [image] table of Config.toml.
bool read_config(const std::string& path, std::map<std::string, std::string>* kv) {
    std::ifstream f(path);
    if (!f) return false;
    std::string line, section;
    while (std::getline(f, line)) {
        size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        line = trim(line);
        if (line.empty()) continue;
        if (line.front() == '[') {
            section = trim(line.substr(1, line.find(']') - 1));
            continue;
        }
        size_t eq = line.find('=');
        if (eq == std::string::npos || section != "image") continue;
        (*kv)[trim(line.substr(0, eq))] = trim(line.substr(eq + 1));
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    std::string scene, config = "Config.toml", out = "image.ppm";
    rtw::RenderOptions opt;
    for (int a = 1; a < argc; ++a) {
        std::string s = argv[a];
        if (s == "--debug") continue;  // render_debug == render on the GPU
        else if (s == "--seed" && a + 1 < argc) opt.seed = strtoull(argv[++a], nullptr, 0);
        else if (s == "--f64") opt.precision = RTW_F64;   // (the default)
        else if (s == "--f32") opt.precision = RTW_F32;   // the speed mode
        else if (s == "--device" && a + 1 < argc) opt.device = atoi(argv[++a]);
        else if (s == "--device-mask" && a + 1 < argc) opt.device_mask = strtoull(argv[++a], nullptr, 0);
        else if (s == "--config" && a + 1 < argc) config = argv[++a];
        else if (s == "--out" && a + 1 < argc) out = argv[++a];
        else if (scene.empty()) scene = s;
        else { fprintf(stderr, "unexpected argument %s\n", s.c_str()); return 2; }
    }
    for (char& ch : scene)
        if (ch == '-') ch = '_';
    using Gen = std::function<std::tuple<rtw::HittableList, rtw::HittableList, rtw::CameraBuilder>()>;
    const uint64_t seed = opt.seed;
    const std::map<std::string, Gen> gens = {
        {"cornell_box", [] { return rtw::scenes::cornell_box(); }},
        {"debug", [seed] { return rtw::scenes::debugging_scene(seed); }},
        {"checkered_spheres", [] { return rtw::scenes::checkered_spheres(); }},
        {"perlin_spheres", [seed] { return rtw::scenes::perlin_spheres(seed); }},
        {"plane", [] { return rtw::scenes::plane(); }},
        {"simple", [seed] { return rtw::scenes::simple(seed); }},
        {"simple_light", [seed] { return rtw::scenes::simple_light(seed); }},
        {"simple_transform", [seed] { return rtw::scenes::simple_transform(seed); }},
    };
    if (!gens.count(scene)) {
        fprintf(stderr, "unknown scene '%s' (cornell-box, debug, checkered-spheres, perlin-spheres, plane, "
                        "simple, simple-light, simple-transform)\n", scene.c_str());
        return 2;
    }
    std::map<std::string, std::string> kv;
    if (!read_config(config, &kv)) {
        fprintf(stderr, "cannot read %s\n", config.c_str());
        return 1;
    }
    // PreImage::fix (config.rs:60-98): two of aspect/width/height are needed
    bool ha = kv.count("aspect_ratio"), hw = kv.count("image_width"), hh = kv.count("image_height");
    double aspect = ha ? atof(kv["aspect_ratio"].c_str()) : 0.0;
    uint32_t W = hw ? (uint32_t)atol(kv["image_width"].c_str()) : 0;
    uint32_t H = hh ? (uint32_t)atol(kv["image_height"].c_str()) : 0;
    if ((int)ha + (int)hw + (int)hh < 2) {
        fprintf(stderr, "Config.toml [image] needs two of aspect_ratio/image_width/image_height\n");
        return 1;
    }
    if (!ha) aspect = (double)W / (double)H;
    else if (!hh) H = (uint32_t)((double)W / aspect);
    else if (!hw) W = (uint32_t)((double)H * aspect);
    const uint32_t spp = (uint32_t)atol(kv["samples_per_pixel"].c_str());
    const uint32_t depth = (uint32_t)atol(kv["max_depth"].c_str());

    auto [world, lights, builder] = gens.at(scene)();
    try {
        rtw::Camera cam = builder.with_vfov(40.0)
                              .with_aspect_ratio(aspect)
                              .with_max_depth(depth)
                              .with_image_width(W)
                              .with_image_height(H)
                              .with_samples_per_pixel(spp)
                              .build();
        auto rows = cam.render(world, lights, opt);
        std::vector<double> sums((size_t)W * H * 3);
        for (uint32_t j = 0; j < H; ++j)
            for (uint32_t i = 0; i < W; ++i) {
                double* d = &sums[((size_t)j * W + i) * 3];
                d[0] = rows[j][i].sum.x;
                d[1] = rows[j][i].sum.y;
                d[2] = rows[j][i].sum.z;
            }
        if (rtw_write_ppm(out.c_str(), sums.data(), W, H, spp) < 0) {
            fprintf(stderr, "cannot write %s\n", out.c_str());
            return 1;
        }
    } catch (const rtw::Error& e) {
        fprintf(stderr, "rtw: %s (code %d)\n", e.what(), e.code());
        return 1;
    }
    return 0;
}
