// ============================================================================
// oracle/ref_driver.cpp  —  TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the REFERENCE's own hot-path headers,
// compiled in place from /root/reference/src by oracle/Makefile into
// oracle/_ref/librtref.so.  Nothing from the reference is copied: this file
// only #includes its headers by path (include dirs set in the Makefile) and
// restates the glue that lives in src/main.cpp (which itself needs GLFW/glad
// and is therefore not built here — see DESIGN.md "oracle").
//
// What it exposes:
//   ref_load_obj      ObjectLoader::loadFromFile   (object_loader.hpp:14)
//   ref_bvh_create    StackBVH::build + collapse   (stack_bvh.hpp:502,574;
//                     partition selection as main.cpp:128-205)
//   ref_bvh_dump      the reference's real tree (private members read via
//                     an access macro) in reference visit order
//   ref_render        calculateScreen + shadeScreen (main.cpp:322-381) with
//                     StackBVH::traverse (stack_bvh.hpp:611) per pixel
//   ref_camera_path   CameraPath::circularPath (camera_path.hpp:18) with the
//                     centre recomputed as runTest does (main.cpp:123,235)
// ============================================================================
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <numbers>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

// Read-only access to StackBVH's tree and Triangle's vertices for the dumps.
#define private public
#include "stack_bvh.hpp"
#include "primitives/triangle.hpp"
#include "utils/object_loader.hpp"
#undef private
#include "camera.hpp"
#include "camera_path.hpp"
#include "color.hpp"

namespace {
thread_local std::string g_err;

using PartFn = std::vector<std::size_t> (*)(const std::vector<Primitive*>::iterator&,
                                             const std::vector<Primitive*>::iterator&, const int);

PartFn pick(int algo, int k) {
    // main.cpp:128-205 (algo 0 median, 1 sah, 2 bsah)
    static const PartFn table[3][4] = {
        {StackBVH::median2Split, StackBVH::median4Split, StackBVH::median8Split, StackBVH::median16Split},
        {StackBVH::sah2Split, StackBVH::sah4Split, StackBVH::sah8Split, StackBVH::sah16Split},
        {StackBVH::binnedSah2Split, StackBVH::binnedSah4Split, StackBVH::binnedSah8Split, StackBVH::binnedSah16Split},
    };
    int col = k == 2 ? 0 : k == 4 ? 1 : k == 8 ? 2 : k == 16 ? 3 : -1;
    if (algo < 0 || algo > 2 || col < 0) return nullptr;
    return table[algo][col];
}
}  // namespace

struct ref_bvh {
    std::vector<Triangle*> owned;  // loader order; Primitive* identity -> index
    std::unordered_map<const Primitive*, long long> index;
    StackBVH bvh;
};

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }

long long ref_load_obj(const char* path, double scale, double** out) {
    try {
        std::vector<Triangle> t = ObjectLoader::loadFromFile(path, scale);
        double* buf = (double*)malloc(sizeof(double) * 9 * (t.size() ? t.size() : 1));
        // Triangle keeps v0..v2 private; recover them through the public
        // interface is impossible, so read the members directly.
        for (size_t i = 0; i < t.size(); i++) {
            const Vector3* v[3] = {&t[i].v0, &t[i].v1, &t[i].v2};
            for (int k = 0; k < 3; k++) {
                buf[i * 9 + k * 3 + 0] = v[k]->getX();
                buf[i * 9 + k * 3 + 1] = v[k]->getY();
                buf[i * 9 + k * 3 + 2] = v[k]->getZ();
            }
        }
        *out = buf;
        return (long long)t.size();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}
void ref_free(void* p) { free(p); }

ref_bvh* ref_bvh_create(const double* tv, long long n, int algo, int k, int collapse) {
    PartFn fn = pick(algo, collapse ? 2 : k);
    if (!fn) { g_err = "Unsupported bvh degree"; return nullptr; }
    std::vector<Primitive*> prims;
    std::vector<Triangle*> owned;
    for (long long i = 0; i < n; i++) {
        const double* p = tv + i * 9;
        Triangle* t = new Triangle(Vector3{p[0], p[1], p[2]}, Vector3{p[3], p[4], p[5]}, Vector3{p[6], p[7], p[8]});
        owned.push_back(t);
        prims.push_back(t);
    }
    try {
        ref_bvh* h = new ref_bvh{owned, {}, StackBVH::build(prims, fn)};
        for (long long i = 0; i < n; i++) h->index[owned[i]] = i;
        int passes = static_cast<int>(std::log2(k)) - 1;
        for (int i = 0; collapse && i < passes; i++) StackBVH::collapse(h->bvh);
        return h;
    } catch (const std::exception& e) {
        g_err = e.what();
        for (auto* t : owned) delete t;
        return nullptr;
    }
}

void ref_bvh_destroy(ref_bvh* h) {
    if (!h) return;
    for (auto* t : h->owned) delete t;
    delete h;
}

long long ref_bvh_node_count(const ref_bvh* h) {
    long long c = 0;
    std::vector<const StackBVH::BVHNode*> st{&h->bvh.root};
    while (!st.empty()) {
        const auto* n = st.back();
        st.pop_back();
        c++;
        for (const auto& ch : n->children) st.push_back(&ch);
    }
    return c;
}

// Same layout as orc_bvh_dump: reference visit order (stack_bvh.hpp:619-641).
void ref_bvh_dump(const ref_bvh* h, double* boxes, long long* meta, long long* order) {
    const auto base = h->bvh.primitives.begin();
    std::vector<const StackBVH::BVHNode*> st{&h->bvh.root};
    long long k = 0;
    while (!st.empty()) {
        const auto* n = st.back();
        st.pop_back();
        const Vector3& mn = n->box.getMin();
        const Vector3& mx = n->box.getMax();
        boxes[k * 6 + 0] = mn.getX(); boxes[k * 6 + 1] = mn.getY(); boxes[k * 6 + 2] = mn.getZ();
        boxes[k * 6 + 3] = mx.getX(); boxes[k * 6 + 4] = mx.getY(); boxes[k * 6 + 5] = mx.getZ();
        meta[k * 3 + 0] = (long long)(n->begin - base);
        meta[k * 3 + 1] = (long long)(n->end - base);
        meta[k * 3 + 2] = (long long)n->children.size();
        k++;
        for (const auto& ch : n->children) st.push_back(&ch);
    }
    for (size_t i = 0; i < h->bvh.primitives.size(); i++) order[i] = h->index.at(h->bvh.primitives[i]);
}

void ref_scene_center(const double* tv, long long n, double out[3]) {
    // main.cpp:118-122 over heap Triangles (getCenter by value)
    Vector3 c{0.0, 0.0, 0.0};
    for (long long i = 0; i < n; i++) {
        const double* p = tv + i * 9;
        Triangle t(Vector3{p[0], p[1], p[2]}, Vector3{p[3], p[4], p[5]}, Vector3{p[6], p[7], p[8]});
        c = c + t.getCenter();
    }
    c = c * (1.0 / static_cast<double>(n));
    out[0] = c.getX(); out[1] = c.getY(); out[2] = c.getZ();
}

void ref_camera_path(const double center[3], int res, int step, double pos[3], double dir[3]) {
    Camera cam{1, 1};
    cam.setPosition(Vector3{center[0], center[1], center[2]} + Vector3{0.0, 0.0, 5.0});
    CameraPath path(cam.getPosition() - Vector3{0.0, 0.0, 5.0}, res);
    Ray r = path.circularPath(step);
    pos[0] = r.getOrigin().getX(); pos[1] = r.getOrigin().getY(); pos[2] = r.getOrigin().getZ();
    dir[0] = r.getDirection().getX(); dir[1] = r.getDirection().getY(); dir[2] = r.getDirection().getZ();
}

// calculateScreen (main.cpp:322-349) for rows [row0,row0+nrows) of W x H,
// then shadeScreen (main.cpp:351-381) and the PPM byte cast
// (benchmark.hpp:105-114).  Outputs row-major ((j-row0)*W+i); any may be NULL.
long long ref_render(const ref_bvh* h, const double cam_pos[3], const double cam_dir[3], int W, int H, int row0,
                     int nrows, int threads, uint8_t* hit, double* hit_pos, double* hit_nrm, uint8_t* rgb) {
    Camera camera{(unsigned)W, (unsigned)H};
    camera.setPosition(Vector3{cam_pos[0], cam_pos[1], cam_pos[2]});
    camera.setDirection(Vector3{cam_dir[0], cam_dir[1], cam_dir[2]});
    const Vector3 camera_pos = camera.getPosition();
    const Vector3 camera_dir = camera.getDirection();
    const Vector3 world_up{0.0, 1.0, 0.0};
    Vector3 right = Vector3::cross(camera_dir, world_up);
    if (right.length() < 1e-8) right = Vector3{0.0, 0.0, 1.0};
    right = right.normalize();
    Vector3 up = Vector3::cross(right, camera_dir).normalize();
    long long hits = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : hits)
#endif
    for (int i = 0; i < W; ++i) {
        const double px = camera.getPixelX(i);
        for (int j = row0; j < row0 + nrows; ++j) {
            const double py = camera.getPixelY(j);
            Vector3 dir = camera_dir + up * py + right * px;
            dir = dir * (1.0 / dir.length());
            Ray ray{camera_pos, dir};
            size_t o = (size_t)(j - row0) * W + i;
            Vector3 P{0.0, 0.0, 0.0}, N{0.0, 0.0, 0.0};
            bool is_hit = false;
            if (const auto hr = StackBVH::traverse(h->bvh, ray)) {
                is_hit = true;
                P = hr->getOrigin();
                N = hr->getDirection();
            }
            if (hit) hit[o] = is_hit;
            if (hit_pos) { hit_pos[o * 3] = P.getX(); hit_pos[o * 3 + 1] = P.getY(); hit_pos[o * 3 + 2] = P.getZ(); }
            if (hit_nrm) { hit_nrm[o * 3] = N.getX(); hit_nrm[o * 3 + 1] = N.getY(); hit_nrm[o * 3 + 2] = N.getZ(); }
            Color c{0.0, 0.0, 0.0};
            if (is_hit) {
                hits++;
                Vector3 Nn = N;
                double nl = Nn.length();
                if (nl > 0.0) Nn = Nn * (1.0 / nl);
                Vector3 L = camera_pos - P;
                double dist = L.length();
                if (dist > 0.0) L = L * (1.0 / dist);
                const double ambient = 0.45;
                double diffuse = std::max(0.0, Vector3::dot(Nn, L)) * 1.35;
                double attenuation = 1.0 / (1.0 + 0.05 * dist * dist);
                double intensity = std::clamp((ambient + diffuse * attenuation) * 1.25, 0.0, 1.0);
                c = Color(0.5 * (Nn.getX() + 1.0) * intensity, 0.5 * (Nn.getY() + 1.0) * intensity,
                          0.5 * (Nn.getZ() + 1.0) * intensity);
            }
            if (rgb) {
                rgb[o * 3 + 0] = static_cast<unsigned char>(std::clamp(c.r() * 255.0, 0.0, 255.0));
                rgb[o * 3 + 1] = static_cast<unsigned char>(std::clamp(c.g() * 255.0, 0.0, 255.0));
                rgb[o * 3 + 2] = static_cast<unsigned char>(std::clamp(c.b() * 255.0, 0.0, 255.0));
            }
        }
    }
    return hits;
}

}  // extern "C"
