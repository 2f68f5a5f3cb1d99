// Ray-generation front end (host side, fp64, reference operation order).
//   pixel plane caches   src/camera.hpp:20-38
//   camera basis         src/main.cpp:325-329
//   circular path        src/camera_path.hpp:18-26 (+ runTest's centre
//                        round trip, src/main.cpp:123,235)
//   scene centre         src/main.cpp:118-122
// The transcendental calls (tan, sin, cos) stay on the host so the device
// never has to reproduce libm; the device receives the cached coefficients.
#include <cmath>
#include <numbers>

#include "rt_internal.h"

namespace rt {
namespace {
inline double len3(double x, double y, double z) { return std::sqrt(x * x + y * y + z * z); }
}  // namespace

// Camera constructor constants (camera.hpp:20-38): 1/W, 1/H, tan(fov/2), W/H.
void pixel_constants(int W, int H, double& iw, double& ih, double& half, double& aspect) {
    const unsigned w = (unsigned)W, h = (unsigned)H;
    const double fov = 90.0 * (std::numbers::pi / 180.0);
    half = std::tan(fov * 0.5);
    aspect = static_cast<double>(w) / h;
    iw = 1.0 / w;
    ih = 1.0 / h;
}

// The camera's pixel caches (camera.hpp:35-37); the kernels evaluate the same
// expressions per pixel (kernels_common.h pixel_x / pixel_y).
void pixel_caches(int W, int H, std::vector<double>& px, std::vector<double>& py) {
    double iw, ih, half, aspect;
    pixel_constants(W, H, iw, ih, half, aspect);
    px.resize((unsigned)W);
    py.resize((unsigned)H);
    for (int x = 0; x < W; ++x) px[x] = (2.0 * (x + 0.5) * iw - 1.0) * half * aspect;
    for (int y = 0; y < H; ++y) py[y] = (1.0 - 2.0 * (y + 0.5) * ih) * half;
}

void camera_basis(const double d[3], double right[3], double up[3]) {
    // right = cross(dir, (0,1,0)); fallback (0,0,1); normalise (divide)
    double rx = d[1] * 0.0 - d[2] * 1.0;
    double ry = d[2] * 0.0 - d[0] * 0.0;
    double rz = d[0] * 1.0 - d[1] * 0.0;
    if (len3(rx, ry, rz) < 1e-8) { rx = 0.0; ry = 0.0; rz = 1.0; }
    double l = len3(rx, ry, rz);
    if (l != 0) { rx = rx / l; ry = ry / l; rz = rz / l; } else { rx = ry = rz = 0; }
    // up = cross(right, dir).normalize()
    double ux = ry * d[2] - rz * d[1];
    double uy = rz * d[0] - rx * d[2];
    double uz = rx * d[1] - ry * d[0];
    double m = len3(ux, uy, uz);
    if (m != 0) { ux = ux / m; uy = uy / m; uz = uz / m; } else { ux = uy = uz = 0; }
    right[0] = rx; right[1] = ry; right[2] = rz;
    up[0] = ux; up[1] = uy; up[2] = uz;
}

void camera_path(const double c[3], int res, int step, double pos[3], double dir[3]) {
    // runTest: camera at c + (0,0,5); the path centre is camera - (0,0,5)
    const double cx = (c[0] + 0.0) - 0.0, cy = (c[1] + 0.0) - 0.0, cz = (c[2] + 5.0) - 5.0;
    const double ang = 2.0 * M_PI * (static_cast<double>(step % res) / res);
    const double x = 0.0 * std::cos(ang) - 5.0 * std::sin(ang);
    const double z = 0.0 * std::sin(ang) + 5.0 * std::cos(ang);
    const double px = cx + x, py = cy + 0.0, pz = cz + z;
    double dx = cx - px, dy = cy - py, dz = cz - pz;
    double l = len3(dx, dy, dz);
    if (l != 0) { dx = dx / l; dy = dy / l; dz = dz / l; } else { dx = dy = dz = 0; }
    pos[0] = px; pos[1] = py; pos[2] = pz;
    dir[0] = dx; dir[1] = dy; dir[2] = dz;
}

void scene_center(const double* v, uint64_t n, double out[3]) {
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (uint64_t i = 0; i < n; i++) {
        const double* p = v + i * 9;
        sx = sx + ((p[0] + p[3]) + p[6]) * (1.0 / 3);
        sy = sy + ((p[1] + p[4]) + p[7]) * (1.0 / 3);
        sz = sz + ((p[2] + p[5]) + p[8]) * (1.0 / 3);
    }
    const double inv = 1.0 / static_cast<double>(n);
    out[0] = sx * inv; out[1] = sy * inv; out[2] = sz * inv;
}

}  // namespace rt
