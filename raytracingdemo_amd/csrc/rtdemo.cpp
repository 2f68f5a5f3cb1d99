// rtdemo — the reference runner (src/main.cpp main/runTest) on librtmi355x.
//
// Reproduces what the reference's benchmark sweep writes, through the C ABI
// only (include/rt.h):
//   * sweep order: repetitions x algorithms (std::multimap order,
//     main.cpp:61-83) x models (std::map order, main.cpp:84-86)
//   * one testruns/testrun_<n> directory per runTest (first free n,
//     benchmark.hpp:17-41)
//   * bvh_build_times.csv (10 builds, main.cpp:211-221), render_times.csv
//     (frame time, main.cpp:253-256), shading_times.csv (hit count,
//     main.cpp:258-260) with the reference's header and ostream formatting
//     (benchmark.hpp:45-84)
//   * screen_<k>.ppm per frame (benchmark.hpp:87-117)
// so scripts/validate_data.py and bvh_analysis.py read its output unchanged.
// OpenGL is not used (the reference runs with no_window = true).
//
// Timing semantics: render_times.csv holds the device time of ray
// generation + traversal + resolve + shading of the frame (rt_frame_out.seconds);
// the reference timed calculateScreen on one CPU core.
//
// Multi-GPU: --devices 0,1,...,N-1 uploads the scene to every listed device;
// rt_render_frame then interleaves image rows over them and gathers the frame
// to the first device with RCCL (include/rt.h), unchanged for this caller.
//
// Usage: rtdemo [--objects DIR] [--out DIR] [--reps N] [--algos a-k,...]
//               [--models name,...] [--frames N] [--size W] [--device D]
//               [--devices D0,D1,...]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt.h"

namespace {

void check(int st) {  // status -> the reference's exception types
    if (st == RT_OK) return;
    const std::string m = rt_last_error();
    if (st == RT_ERR_INVALID_ARGUMENT) throw std::invalid_argument(m);
    if (st == RT_ERR_OUT_OF_RANGE) throw std::out_of_range(m);
    throw std::runtime_error(m);
}

struct Camera {  // position / direction as the CSV rows print them
    double pos[3];
    double dir[3];
};

// Benchmark (benchmark.hpp): one directory per test run, appended CSVs, PPMs.
class Benchmark {
   public:
    explicit Benchmark(const std::filesystem::path& root) {
        for (int n = 0;; n++) {
            std::filesystem::path cand = root / ("testrun_" + std::to_string(n));
            std::error_code ec;
            if (!std::filesystem::exists(cand, ec)) {
                std::filesystem::create_directories(cand, ec);
                dir_ = cand;
                break;
            }
        }
    }
    void save_data_frame(const std::string& file, const std::string& model, double scale, const std::string& algo,
                         const Camera& cam, double value) {
        const auto path = dir_ / file;
        const bool exists = std::filesystem::exists(path);
        std::ofstream f(path, std::ios::app);
        if (!exists)
            f << "file_name,model_name,model_scale,algorithm_name,cam_pos_x,cam_pos_y,cam_pos_z,cam_dir_x,cam_dir_y,"
                 "cam_dir_z,time_seconds\n";
        f << file << "," << model << "," << scale << "," << algo << ",";
        f << cam.pos[0] << "," << cam.pos[1] << "," << cam.pos[2] << ",";
        f << cam.dir[0] << "," << cam.dir[1] << "," << cam.dir[2] << ",";
        f << value << "\n";
    }
    void save_screen(const uint8_t* rgb, int W, int H) {  // rows top to bottom, PPM P6
        std::ofstream f(dir_ / ("screen_" + std::to_string(pictures_++) + ".ppm"), std::ios::binary);
        f << "P6\n" << W << " " << H << "\n255\n";
        f.write(reinterpret_cast<const char*>(rgb), (std::streamsize)W * H * 3);
    }
    const std::filesystem::path& dir() const { return dir_; }

   private:
    std::filesystem::path dir_;
    int pictures_ = 0;
};

struct Config {
    std::string objects = "example";
    std::string out = "testruns";
    int reps = 10;
    int frames = 36;
    int size = 500;
    std::vector<int> devices{0};
    std::vector<std::pair<std::string, int>> algos;
    std::vector<std::pair<std::string, double>> models;
};

// main.cpp:61-83 as a std::multimap: keys sorted, equal keys in insertion order
std::vector<std::pair<std::string, int>> reference_algorithms() {
    std::multimap<std::string, int> m = {
        {"bsah", 2}, {"bsah", 4}, {"bsah", 8}, {"bsah", 16}, {"bsah-c", 4}, {"bsah-c", 8}, {"bsah-c", 16},
        {"sah", 2}, {"sah", 4}, {"sah", 8}, {"sah", 16}, {"median", 2}, {"median", 4}, {"median", 8},
        {"median", 16}, {"sah-c", 4}, {"sah-c", 8}, {"sah-c", 16}, {"median-c", 4}, {"median-c", 8},
        {"median-c", 16}};
    return {m.begin(), m.end()};
}

// main.cpp:84-86 as a std::map (name order)
std::vector<std::pair<std::string, double>> reference_models() {
    std::map<std::string, double> m = {
        {"stanford-bunny.obj", 30.0}, {"teapot.obj", 1.0}, {"suzanne.obj", 3.0}, {"armadillo.obj", 0.035}};
    return {m.begin(), m.end()};
}

void run_test(const Config& cfg, const std::string& model, double scale, const std::string& algo, int k) {
    Benchmark bm(cfg.out);
    double* tri = nullptr;
    uint64_t n = 0;
    check(rt_load_obj((std::filesystem::path(cfg.objects) / model).string().c_str(), scale, &tri, &n));
    double center[3];
    check(rt_scene_center(tri, n, center));
    Camera cam{{center[0], center[1], center[2] + 5.0}, {0.0, 0.0, -1.0}};  // main.cpp:123; camera.hpp:21

    const bool collapse = algo.size() > 2 && algo.compare(algo.size() - 2, 2, "-c") == 0;
    const std::string base = collapse ? algo.substr(0, algo.size() - 2) : algo;
    const int id = base == "bsah" ? RT_ALGO_BSAH : base == "sah" ? RT_ALGO_SAH : base == "median" ? RT_ALGO_MEDIAN : -1;
    const std::string full = algo + "-" + std::to_string(k);
    std::printf("Building BVH using %s split...\n", full.c_str());
    rt_scene* scene = nullptr;
    for (int it = 0; it < 10; it++) {  // main.cpp:211-221: ten timed builds
        if (scene) rt_scene_destroy(scene);
        scene = nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        // reference tree on the host, the walk tree on the first device
        check(rt_scene_create_on_device(tri, n, id, k, collapse, cfg.devices.front(), &scene));
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        bm.save_data_frame("bvh_build_times.csv", model, scale, full, cam, s);
        std::printf("Time build BVH using %s Split: %f \n", full.c_str(), s);
    }
    check(rt_scene_upload(scene, cfg.devices.data(), (int)cfg.devices.size()));

    const int W = cfg.size, H = cfg.size;
    std::vector<uint8_t> rgb((size_t)W * H * 3);
    for (int step = 0; step < cfg.frames; step++) {  // main.cpp:237-281
        // CameraPath(camera.getPosition() - (0,0,5), resolution).circularPath(step)
        check(rt_camera_path(center, cfg.frames, step, cam.pos, cam.dir));
        rt_camera c{};
        for (int a = 0; a < 3; a++) {
            c.pos[a] = cam.pos[a];
            c.dir[a] = cam.dir[a];
        }
        c.width = W;
        c.height = H;
        rt_frame_out out{};
        out.rgb = rgb.data();
        check(rt_render_frame(scene, &c, RT_MODE_EXACT, &out));
        bm.save_data_frame("render_times.csv", model, scale, full, cam, out.seconds);
        bm.save_data_frame("shading_times.csv", model, scale, full, cam, static_cast<double>(out.hit_count));
        bm.save_screen(rgb.data(), W, H);
    }
    rt_scene_destroy(scene);
    rt_free(tri);
}

std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> out;
    std::stringstream ss(s);
    for (std::string t; std::getline(ss, t, ',');)
        if (!t.empty()) out.push_back(t);
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    Config cfg;
    cfg.algos = reference_algorithms();
    cfg.models = reference_models();
    for (int a = 1; a < argc; a++) {
        const std::string k = argv[a];
        auto val = [&]() -> std::string {
            if (a + 1 >= argc) throw std::invalid_argument("missing value for " + k);
            return argv[++a];
        };
        if (k == "--objects") cfg.objects = val();
        else if (k == "--out") cfg.out = val();
        else if (k == "--reps") cfg.reps = std::stoi(val());
        else if (k == "--frames") cfg.frames = std::stoi(val());
        else if (k == "--size") cfg.size = std::stoi(val());
        else if (k == "--device") cfg.devices = {std::stoi(val())};
        else if (k == "--devices") {
            cfg.devices.clear();
            for (const auto& t : split(val())) cfg.devices.push_back(std::stoi(t));
        }
        else if (k == "--algos") {
            cfg.algos.clear();
            for (const auto& t : split(val())) {
                const auto p = t.rfind('-');
                cfg.algos.emplace_back(t.substr(0, p), std::stoi(t.substr(p + 1)));
            }
        } else if (k == "--models") {
            const auto all = reference_models();
            cfg.models.clear();
            for (const auto& t : split(val()))
                for (const auto& m : all)
                    if (m.first == t) cfg.models.push_back(m);
        } else {
            std::cerr << "unknown argument " << k << "\n";
            return 2;
        }
    }
    try {
        for (int i = 0; i < cfg.reps; i++)
            for (const auto& [algo, k] : cfg.algos)
                for (const auto& [model, scale] : cfg.models) run_test(cfg, model, scale, algo, k);
    } catch (const std::exception& e) {
        std::cerr << "rtdemo: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
