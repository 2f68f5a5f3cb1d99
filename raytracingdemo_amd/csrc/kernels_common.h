// Device helpers shared by the gfx950 kernels (render.hip): the reference's
// fp64 arithmetic (slab test, Moller-Trumbore, ray generation, shading) in
// exact operation order, the conservative fp32 pre-filter, the ancestor-
// chain re-verification and the LDS traversal stack.  Included by one TU
// compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"

namespace rtk {


struct Ray64 {
    double ox, oy, oz;
    double dx, dy, dz;
    double ix, iy, iz;
};

__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ double sclamp(double v, double lo, double hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

// AABB::hit (aabb.hpp:32-49); b = {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z}
__device__ __forceinline__ bool box_hit64(const double* __restrict__ b, const Ray64& r) {
    double tx1 = (b[0] - r.ox) * r.ix;
    double tx2 = (b[3] - r.ox) * r.ix;
    double tmin = smin(tx1, tx2);
    double tmax = smax(tx1, tx2);
    double ty1 = (b[1] - r.oy) * r.iy;
    double ty2 = (b[4] - r.oy) * r.iy;
    tmin = smax(tmin, smin(ty1, ty2));
    tmax = smin(tmax, smax(ty1, ty2));
    double tz1 = (b[2] - r.oz) * r.iz;
    double tz2 = (b[5] - r.oz) * r.iz;
    tmin = smax(tmin, smin(tz1, tz2));
    tmax = smin(tmax, smax(tz1, tz2));
    return tmax >= tmin;
}

// Triangle::intersect (triangle.hpp:40-62).  T = v0, edge1, edge2 (the
// edges are precomputed with the same subtraction the reference performs).
__device__ __forceinline__ bool mt64(const double* __restrict__ T, const Ray64& r, double& t_out) {
    const double EPS = 1e-8;
    const double e1x = T[3], e1y = T[4], e1z = T[5];
    const double e2x = T[6], e2y = T[7], e2z = T[8];
    const double hx = r.dy * e2z - r.dz * e2y;
    const double hy = r.dz * e2x - r.dx * e2z;
    const double hz = r.dx * e2y - r.dy * e2x;
    const double a = e1x * hx + e1y * hy + e1z * hz;
    if (a > -EPS && a < EPS) return false;
    const double f = 1.0 / a;
    const double sx = r.ox - T[0], sy = r.oy - T[1], sz = r.oz - T[2];
    const double u = f * (sx * hx + sy * hy + sz * hz);
    if (u < 0.0 || u > 1.0) return false;
    const double qx = sy * e1z - sz * e1y;
    const double qy = sz * e1x - sx * e1z;
    const double qz = sx * e1y - sy * e1x;
    const double v = f * (r.dx * qx + r.dy * qy + r.dz * qz);
    if (v < 0.0 || u + v > 1.0) return false;
    const double t = f * (e2x * qx + e2y * qy + e2z * qz);
    if (!(t > EPS)) return false;
    t_out = t;
    return true;
}

// Conservative fp32 pre-filter of Triangle::intersect.  Returns false only
// when the exact fp64 test must reject (u < 0, v < 0, u+v > 1 or t < 0), or
// the hit lies beyond `tcull`.  Record: v0, e1, e2 (fp32, nearest) and, rounded
// up, M1 = max|e1_i|, M2 = max|e2_i|, Cv = max|v0_i|; `co` = max|o_i| rounded up.
// Every computed MT quantity X (a, U = s.h, V = d.q, T = e2.q) is within a
// quarter of its budget errX of the exact real value, with
//   G = 256 Ms + 64 (co + Cv)     (Ms = max|s_i|, s = o - v0 in fp32)
//   errA = 256 u M1 M2, errU = u M2 G, errV = u M1 G, errT = u M1 M2 G
// (u = 2^-24; |d_i| <= 1; each quantity is a 3-term dot of products of inputs
// carrying <= 2u relative rounding, plus the absolute rounding of s).  A
// rejection therefore leaves >= 3/4 of a budget between the real value and the
// decision boundary — far beyond the fp64 test's own rounding (2^-50 scale) —
// so the fp64 test would reject too.  DESIGN.md "exactness" has the details.
__device__ __forceinline__ bool tri_prefilter(const float4 A, const float4 B, const float4 C, float ox, float oy,
                                              float oz, float dx, float dy, float dz, float co, float tcull) {
    const float e1x = A.w, e1y = B.x, e1z = B.y, e2x = B.z, e2y = B.w, e2z = C.x;
    const float M1 = C.y, M2 = C.z, Cv = C.w;
    const float sx = ox - A.x, sy = oy - A.y, sz = oz - A.z;
    const float hx = __builtin_fmaf(dy, e2z, -dz * e2y);
    const float hy = __builtin_fmaf(dz, e2x, -dx * e2z);
    const float hz = __builtin_fmaf(dx, e2y, -dy * e2x);
    const float a = __builtin_fmaf(e1x, hx, __builtin_fmaf(e1y, hy, e1z * hz));
    const float U = __builtin_fmaf(sx, hx, __builtin_fmaf(sy, hy, sz * hz));
    const float qx = __builtin_fmaf(sy, e1z, -sz * e1y);
    const float qy = __builtin_fmaf(sz, e1x, -sx * e1z);
    const float qz = __builtin_fmaf(sx, e1y, -sy * e1x);
    const float V = __builtin_fmaf(dx, qx, __builtin_fmaf(dy, qy, dz * qz));
    const float T = __builtin_fmaf(e2x, qx, __builtin_fmaf(e2y, qy, e2z * qz));
    const float Ms = fmaxf(fmaxf(__builtin_fabsf(sx), __builtin_fabsf(sy)), __builtin_fabsf(sz));
    const float u = 0x1p-24f;
    const float G = __builtin_fmaf(256.f, Ms, 64.f * (co + Cv));
    const float errA = 256.f * u * M1 * M2;
    const float errU = u * M2 * G, errV = u * M1 * G, errT = u * M1 * M2 * G;
    const float aa = __builtin_fabsf(a);
    if (!(aa > errA)) return true;  // sign of the determinant uncertain: let fp64 decide
    const float sg = a > 0.f ? 1.f : -1.f;
    const float Us = sg * U, Vs = sg * V, Ts = sg * T;
    if (Us < -errU || Vs < -errV || Ts < -errT) return false;
    if (Us + Vs > aa + errU + errV + errA) return false;
    if (Ts - errT > tcull * (aa + errA)) return false;  // t > tcull: cannot improve
    return true;
}

// Classifying variant of tri_prefilter for the deferred fp64 resolve.
//   0  the exact fp64 test must reject (or t > tcull)
//   1  borderline: only the fp64 test can decide
//   2  certain: every fp64 decision passes with margin (|a| >= EPS, u, v,
//      u+v, t > EPS all clear their bounds by a full budget, which is >= 3/4
//      budget beyond the real value — far above fp64 rounding), so the true
//      hit parameter is <= tu and tu may tighten the culling distance.
// tl / tu bound the true t = T/a from below / above whenever class != 0.
__device__ __forceinline__ int tri_classify_nest(const float4 A, const float4 B, const float4 C, float ox,
                                                 float oy, float oz, float dx, float dy, float dz, float co,
                                                 float tcull, float& tl, float& tu) {
    const float e1x = A.w, e1y = B.x, e1z = B.y, e2x = B.z, e2y = B.w, e2z = C.x;
    const float M1 = C.y, M2 = C.z, Cv = C.w;
    const float sx = ox - A.x, sy = oy - A.y, sz = oz - A.z;
    const float hx = __builtin_fmaf(dy, e2z, -dz * e2y);
    const float hy = __builtin_fmaf(dz, e2x, -dx * e2z);
    const float hz = __builtin_fmaf(dx, e2y, -dy * e2x);
    const float a = __builtin_fmaf(e1x, hx, __builtin_fmaf(e1y, hy, e1z * hz));
    const float U = __builtin_fmaf(sx, hx, __builtin_fmaf(sy, hy, sz * hz));
    const float qx = __builtin_fmaf(sy, e1z, -sz * e1y);
    const float qy = __builtin_fmaf(sz, e1x, -sx * e1z);
    const float qz = __builtin_fmaf(sx, e1y, -sy * e1x);
    const float V = __builtin_fmaf(dx, qx, __builtin_fmaf(dy, qy, dz * qz));
    const float T = __builtin_fmaf(e2x, qx, __builtin_fmaf(e2y, qy, e2z * qz));
    const float Ms = fmaxf(fmaxf(__builtin_fabsf(sx), __builtin_fabsf(sy)), __builtin_fabsf(sz));
    const float u = 0x1p-24f;
    const float G = __builtin_fmaf(256.f, Ms, 64.f * (co + Cv));
    const float errA = 256.f * u * M1 * M2;
    const float errU = u * M2 * G, errV = u * M1 * G, errT = u * M1 * M2 * G;
    const float aa = __builtin_fabsf(a);
    tl = 0.f;
    tu = __builtin_huge_valf();
    if (!(aa > errA)) return 1;  // sign of the determinant uncertain: let fp64 decide
    const float sg = a > 0.f ? 1.f : -1.f;
    const float Us = sg * U, Vs = sg * V, Ts = sg * T;
    if (Us < -errU || Vs < -errV || Ts < -errT) return 0;
    if (Us + Vs > aa + errU + errV + errA) return 0;
    if (Ts - errT > tcull * (aa + errA)) return 0;  // t > tcull: cannot improve
    // bounds through v_rcp_f32 (<= 1 ulp) and one rounded multiply: the
    // 2^-20 factors cover both roundings with room to spare
    tl = fmaxf((Ts - errT) * __builtin_amdgcn_rcpf(aa + errA), 0.f) * (1.f - 0x1p-20f);
    const float EPS = 1e-8f;
    const bool certain = Us >= errU && Vs >= errV && Us + Vs <= aa - errU - errV - errA && aa - errA >= 2.f * EPS &&
                         Ts - errT >= 2.f * EPS * (aa + errA);
    if (!certain) return 1;
    tu = (Ts + errT) * __builtin_amdgcn_rcpf(aa - errA) * (1.f + 0x1p-20f);
    return 2;
}

// tri_classify with one divergent branch instead of a nest: the same
// expressions and the same class / bounds (every class-1 and class-2 lane
// computes what tri_classify computes for it; a class-0 lane's tl / tu are
// unused).  The rejection tests are evaluated for every lane, the bounds
// only under `any lane survives`; the certain / borderline split is a
// select.  For the packet walk, where a wave skips a triangle as a whole
// only when all 64 rays reject it, each nested level of tri_classify cost
// an exec save, a branch and an exec restore per triangle record.
// RT_REJ_MAX=1: the five rejection tests of tri_classify_flat as one max and
// one compare (fewer scalar mask ORs, more VALU); 0: five compares.
#ifndef RT_REJ_MAX
#define RT_REJ_MAX 0
#endif
__device__ __forceinline__ int tri_classify_flat(const float4 A, const float4 B, const float4 C, float ox, float oy,
                                                 float oz, float dx, float dy, float dz, float co, float tcull,
                                                 float& tl, float& tu) {
    const float e1x = A.w, e1y = B.x, e1z = B.y, e2x = B.z, e2y = B.w, e2z = C.x;
    const float M1 = C.y, M2 = C.z, Cv = C.w;
    const float sx = ox - A.x, sy = oy - A.y, sz = oz - A.z;
    const float hx = __builtin_fmaf(dy, e2z, -dz * e2y);
    const float hy = __builtin_fmaf(dz, e2x, -dx * e2z);
    const float hz = __builtin_fmaf(dx, e2y, -dy * e2x);
    const float a = __builtin_fmaf(e1x, hx, __builtin_fmaf(e1y, hy, e1z * hz));
    const float U = __builtin_fmaf(sx, hx, __builtin_fmaf(sy, hy, sz * hz));
    const float qx = __builtin_fmaf(sy, e1z, -sz * e1y);
    const float qy = __builtin_fmaf(sz, e1x, -sx * e1z);
    const float qz = __builtin_fmaf(sx, e1y, -sy * e1x);
    const float V = __builtin_fmaf(dx, qx, __builtin_fmaf(dy, qy, dz * qz));
    const float T = __builtin_fmaf(e2x, qx, __builtin_fmaf(e2y, qy, e2z * qz));
    const float Ms = fmaxf(fmaxf(__builtin_fabsf(sx), __builtin_fabsf(sy)), __builtin_fabsf(sz));
    const float u = 0x1p-24f;
    const float G = __builtin_fmaf(256.f, Ms, 64.f * (co + Cv));
    const float errA = 256.f * u * M1 * M2;
    const float errU = u * M2 * G, errV = u * M1 * G, errT = u * M1 * M2 * G;
    const float aa = __builtin_fabsf(a);
    const bool sure = aa > errA;  // else the sign of the determinant is uncertain: class 1
    const float sg = a > 0.f ? 1.f : -1.f;
    const float Us = sg * U, Vs = sg * V, Ts = sg * T;
    // (bitwise & and |: no short-circuit branches)
    bool rej;
    if constexpr (RT_REJ_MAX != 0) {
        // the same five tests as one compare: fl(b - a) > 0 exactly when
        // b > a (a rounded difference is 0 only for a == b and keeps the
        // sign otherwise), and a NaN term drops out of the max as its
        // compare drops out of the OR
        const float m = fmaxf(fmaxf(fmaxf(-errU - Us, -errV - Vs), -errT - Ts),
                              fmaxf((Us + Vs) - (aa + errU + errV + errA), (Ts - errT) - tcull * (aa + errA)));
        rej = sure & (m > 0.f);
    } else {
        rej = sure & ((Us < -errU) | (Vs < -errV) | (Ts < -errT) | (Us + Vs > aa + errU + errV + errA) |
                      (Ts - errT > tcull * (aa + errA)));
    }
    tl = 0.f;
    tu = __builtin_huge_valf();
    int cls = rej ? 0 : 1;
    if (sure & !rej) {
        tl = fmaxf((Ts - errT) * __builtin_amdgcn_rcpf(aa + errA), 0.f) * (1.f - 0x1p-20f);
        const float EPS = 1e-8f;
        const bool certain = (Us >= errU) & (Vs >= errV) & (Us + Vs <= aa - errU - errV - errA) &
                             (aa - errA >= 2.f * EPS) & (Ts - errT >= 2.f * EPS * (aa + errA));
        const float tuv = (Ts + errT) * __builtin_amdgcn_rcpf(aa - errA) * (1.f + 0x1p-20f);
        tu = certain ? tuv : tu;
        cls = certain ? 2 : 1;
    }
    return cls;
}

// The per-lane walks' filter (render.hip LaneWalk, path_kernel.h,
// queue_paths.h): tri_classify_flat unless RT_CLASSIFY_FLAT=0 (the nest).
// The packet walk picks its own (packet_kernel.h RT_FLAT_CLASSIFY).
#ifndef RT_CLASSIFY_FLAT
#define RT_CLASSIFY_FLAT 1
#endif
__device__ __forceinline__ int tri_classify(const float4 A, const float4 B, const float4 C, float ox, float oy,
                                            float oz, float dx, float dy, float dz, float co, float tcull, float& tl,
                                            float& tu) {
    if constexpr (RT_CLASSIFY_FLAT != 0)
        return tri_classify_flat(A, B, C, ox, oy, oz, dx, dy, dz, co, tcull, tl, tu);
    else
        return tri_classify_nest(A, B, C, ox, oy, oz, dx, dy, dz, co, tcull, tl, tu);
}

// Pose of sample frame f with its sub-pixel offset: sample q = f mod spp of
// an n x n pattern at ((q mod n) + 0.5) / n, ((q div n) + 0.5) / n — the
// host's expressions (rt_api.cpp frame_params), so the doubles are the same;
// spp = 1: 0.5, the reference's pixel centre (camera.hpp:35-37).
__device__ __forceinline__ RtFrameCam frame_cam_of(const RtPose& p, const RtFrameParams& fp, int f) {
    RtFrameCam c;
    for (int a = 0; a < 3; a++) {
        c.pos[a] = p.pos[a];
        c.dir[a] = p.dir[a];
        c.right[a] = p.right[a];
        c.up[a] = p.up[a];
    }
    c.pad = p.pad;
    c.reserved = 0;
    if (fp.spp_n == 1) {  // (0 + 0.5) / 1, without the divisions
        c.ox = c.oy = 0.5;
        return c;
    }
    const int q = f % fp.spp, g = fp.spp_n;
    c.ox = ((double)(q % g) + 0.5) / (double)g;
    c.oy = ((double)(q / g) + 0.5) / (double)g;
    return c;
}
__device__ __forceinline__ RtFrameCam frame_cam(const RtFrameParams& fp, int f) {
    return frame_cam_of(fp.pose[f / fp.spp], fp, f);
}

// Camera pixel caches (camera.hpp:35-37), evaluated per pixel in the same
// operation order as the host's pixel_caches (no contraction): bit-identical.
// ox / oy: the sample's offset inside the pixel; the reference's pixel centre
// is 0.5 (x + 0.5 exactly as camera.hpp:35-37), stratified samples use
// (k + 0.5) / n.
__device__ __forceinline__ double pixel_x(const RtFrameParams& fp, const RtFrameCam& cam, int x) {
    return (2.0 * ((double)x + cam.ox) * fp.cam_iw - 1.0) * fp.cam_half * fp.cam_aspect;
}
__device__ __forceinline__ double pixel_y(const RtFrameParams& fp, const RtFrameCam& cam, int y) {
    return (1.0 - 2.0 * ((double)y + cam.oy) * fp.cam_ih) * fp.cam_half;
}

// main.cpp:332-337: d = dir + up*py + right*px; d *= 1/|d|; Ray{pos, d}
// INV: also the reciprocal direction (slab tests); k_resolve adds it only
// when it falls back to the chain walk (with_inv).
template <bool INV = true>
__device__ __forceinline__ Ray64 gen_ray(const RtFrameParams& fp, const RtFrameCam& cam, int i, int j) {
    const double px = pixel_x(fp, cam, i), py = pixel_y(fp, cam, j);
    double dx = (cam.dir[0] + cam.up[0] * py) + cam.right[0] * px;
    double dy = (cam.dir[1] + cam.up[1] * py) + cam.right[1] * px;
    double dz = (cam.dir[2] + cam.up[2] * py) + cam.right[2] * px;
    const double s = 1.0 / __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    dx = dx * s;
    dy = dy * s;
    dz = dz * s;
    Ray64 r;
    r.ox = cam.pos[0];
    r.oy = cam.pos[1];
    r.oz = cam.pos[2];
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
    if (INV) {
        const double inf = __builtin_huge_val();
        r.ix = dx != 0.0 ? 1.0 / dx : inf;
        r.iy = dy != 0.0 ? 1.0 / dy : inf;
        r.iz = dz != 0.0 ? 1.0 / dz : inf;
    } else {
        r.ix = r.iy = r.iz = 0.0;
    }
    return r;
}
__device__ __forceinline__ Ray64 with_inv(Ray64 r) {
    const double inf = __builtin_huge_val();
    r.ix = r.dx != 0.0 ? 1.0 / r.dx : inf;
    r.iy = r.dy != 0.0 ? 1.0 / r.dy : inf;
    r.iz = r.dz != 0.0 ? 1.0 / r.dz : inf;
    return r;
}

// Candidate bookkeeping shared by both kernels.
struct Best {
    double dist;
    uint32_t rank;
    int32_t tri;  // BVH-order index, -1 = none
    double px, py, pz;
};

// Distance of a detected hit exactly as stack_bvh.hpp:630-631 computes it.
__device__ __forceinline__ double hit_dist(const Ray64& r, double t, double& px, double& py, double& pz) {
    px = r.ox + r.dx * t;
    py = r.oy + r.dy * t;
    pz = r.oz + r.dz * t;
    const double ex = px - r.ox, ey = py - r.oy, ez = pz - r.oz;
    return __builtin_sqrt(ex * ex + ey * ey + ez * ez);
}

// shadeScreen body (main.cpp:356-377) + PPM byte cast (benchmark.hpp:105-114)
// count_hit: add this pixel's hit to fp.hit_count here (one atomic per wave);
// k_resolve instead reduces per block and k_fixup adds the block sums once.
// Shading inputs of the winner, from its fp64 record (rt_device.h).
struct Shade {
    double nx, ny, nz;
    uint32_t id;
};
__device__ __forceinline__ Shade shade_of(const RtDevScene& sc, int32_t tri) {
    Shade s{0.0, 0.0, 0.0, RT_INVALID_REF};
    if (tri >= 0) {
        const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)tri;
        s.nx = T[RT_T64_NORMAL];
        s.ny = T[RT_T64_NORMAL + 1];
        s.nz = T[RT_T64_NORMAL + 2];
        s.id = reinterpret_cast<const RT_G uint2*>(T + RT_T64_IDLEAF)->x;
    }
    return s;
}
// Output slot of pixel o (row-major in the shard) of frame f of the launch
// (spp = 1: frame = pose).
__device__ __forceinline__ size_t out_index(const RtFrameParams& fp, int f, size_t o) {
    return (size_t)f * ((size_t)fp.W * (size_t)fp.nrows) + o;
}
// shadeScreen's colour of one sample before the byte cast (main.cpp:356-377):
// (0.5 (n + 1)) * I per channel, 0 on a miss.
__device__ __forceinline__ void shade_color(const RtFrameCam& cam, const Best& b, const Shade& sh, double c[3]) {
    c[0] = c[1] = c[2] = 0.0;
    if (b.tri < 0) return;
    // the record holds the normal already normalised as shadeScreen does
    // it (main.cpp:361; bvh_build.cpp flatten, same IEEE operations)
    const double nx = sh.nx, ny = sh.ny, nz = sh.nz;
    double lx = cam.pos[0] - b.px, ly = cam.pos[1] - b.py, lz = cam.pos[2] - b.pz;
    // the light sits at the ray origin, so |light - p| is bit-for-bit the
    // hit distance hit_dist returned ((o - p) = -(p - o) exactly, same
    // sum order): reuse it instead of a second fp64 sqrt
    const double dist = b.dist;
    if (dist > 0.0) {
        const double s = 1.0 / dist;
        lx = lx * s; ly = ly * s; lz = lz * s;
    }
    const double diffuse = smax(0.0, nx * lx + ny * ly + nz * lz) * 1.35;
    const double att = 1.0 / (1.0 + 0.05 * dist * dist);
    const double I = sclamp((0.45 + diffuse * att) * 1.25, 0.0, 1.0);
    c[0] = (0.5 * (nx + 1.0)) * I;
    c[1] = (0.5 * (ny + 1.0)) * I;
    c[2] = (0.5 * (nz + 1.0)) * I;
}
// Output stores.  RT_NT_STORES: the outputs are written once and never read
// by the kernels, so they go out as non-temporal stores (streaming cache
// policy) instead of displacing the scene's nodes and triangles from L2 and
// MALL: a 36-pose launch writes 1.1 GB of outputs against a 75-MB scene.
#ifndef RT_NT_STORES
#define RT_NT_STORES 1
#endif
template <class P, class V>
__device__ __forceinline__ void out_store(P p, V v) {  // (v has the pointee's type)
    if constexpr (RT_NT_STORES != 0)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
// Per-sample outputs (hit id, distance, position) at sample slot `so`.
__device__ __forceinline__ void store_sample(const RtFrameParams& fp, size_t so, const Best& b, const Shade& sh) {
    if (fp.hit_id) out_store(fp.hit_id + so, b.tri >= 0 ? sh.id : (uint32_t)RT_INVALID_REF);
    if (fp.dist) out_store(fp.dist + so, b.tri >= 0 ? b.dist : -1.0);
    if (fp.hit_pos) {
        out_store(fp.hit_pos + 3 * so, b.tri >= 0 ? b.px : 0.0);
        out_store(fp.hit_pos + 3 * so + 1, b.tri >= 0 ? b.py : 0.0);
        out_store(fp.hit_pos + 3 * so + 2, b.tri >= 0 ? b.pz : 0.0);
    }
}
// Pixel colour as PPM bytes (benchmark.hpp:105-114 truncating cast) from the
// sum of its samples' colours (summed in sample order from 0.0): the mean
// c / spp; for spp = 1 that is the reference's c * 255 bit for bit.
__device__ __forceinline__ void store_rgb(const RtFrameParams& fp, size_t po, const double c[3]) {
    if (!fp.rgb) return;
    const double n = (double)fp.spp;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const double m = fp.spp == 1 ? c[k] : c[k] / n;  // (c / 1 == c: skip the division)
        out_store(fp.rgb + 3 * po + k, (uint8_t)sclamp(m * 255.0, 0.0, 255.0));
    }
}
// spp = 1 store of one pixel of frame f: per-sample outputs, colour and (one
// atomic per wave) the frame's hit count.
__device__ __forceinline__ void shade_store(const RtFrameParams& fp, const RtFrameCam& cam, int f, size_t o,
                                            const Best& b, const Shade& sh, bool count_hit = true) {
    o = out_index(fp, f, o);
    double c[3];
    shade_color(cam, b, sh, c);
    store_rgb(fp, o, c);
    store_sample(fp, o, b, sh);
    if (count_hit && fp.hit_count) {  // one atomic per wave (all active lanes reach this)
        const uint64_t hits = __ballot(b.tri >= 0);
        const uint64_t act = __ballot(1);
        if (hits != 0 && (int)(threadIdx.x & 63) == __builtin_ctzll(act))
            atomicAdd(fp.hit_count + f, (unsigned long long)__builtin_popcountll(hits));
    }
}
__device__ __forceinline__ void shade_store(const RtFrameParams& fp, const RtFrameCam& cam, int f,
                                            const RtDevScene& sc, size_t o, const Best& b, bool count_hit = true) {
    shade_store(fp, cam, f, o, b, shade_of(sc, b.tri), count_hit);
}

template <int W>
__device__ __forceinline__ void load_w(float (&d)[W], const float* __restrict__ p) {
    if constexpr (W % 4 == 0) {
#pragma unroll
        for (int c = 0; c < W; c += 4) {
            const float4 v = *reinterpret_cast<const float4*>(p + c);
            d[c] = v.x; d[c + 1] = v.y; d[c + 2] = v.z; d[c + 3] = v.w;
        }
    } else {
        const float2 v = *reinterpret_cast<const float2*>(p);
        d[0] = v.x; d[1] = v.y;
    }
}
template <int W>
__device__ __forceinline__ void load_refs(uint32_t (&d)[W], const uint32_t* __restrict__ p) {
    if constexpr (W % 4 == 0) {
#pragma unroll
        for (int c = 0; c < W; c += 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(p + c);
            d[c] = v.x; d[c + 1] = v.y; d[c + 2] = v.z; d[c + 3] = v.w;
        }
    } else {
        const uint2 v = *reinterpret_cast<const uint2*>(p);
        d[0] = v.x; d[1] = v.y;
    }
}

// fp32 upper bound of a positive double
__device__ __forceinline__ float round_up_f(double x) {
    float f = (float)x;
    if ((double)f < x) f = __uint_as_float(__float_as_uint(f) + 1u);
    return f;
}

// The reference sees a triangle only when every box on its root path passes
// the fp64 slab test; re-check that chain for a would-be winner.
__device__ __forceinline__ bool chain_ok(const RtDevScene& sc, uint32_t leaf, const Ray64& r, uint32_t& loads) {
    int32_t n = (int32_t)leaf;
    while (n >= 0) {
        loads++;
        if (!box_hit64(sc.rbox + 6 * (size_t)n, r)) return false;
        n = sc.rparent[n];
    }
    return true;
}

// Sufficient condition for chain_ok without walking the chain: if the hit
// point p = fl(o + d t) lies inside the (real) leaf box with a margin
// m_a = 2^-48 (|mn_a| + |mx_a| + |o_a| + |p_a|) on every axis and no direction
// component is zero, every fp64 slab test on the root path passes.  Proof
// sketch (DESIGN.md "exactness"): |p_a - (o_a + d_a t)| <= 2^-52(|o_a|+|d_a t|)
// and each computed slab bound is within 2^-51 |mn_a - o_a| / |d_a| of its
// real value, so every computed near bound is < t < every computed far bound;
// ancestor boxes contain the leaf box, so their margins are no smaller.
__device__ __forceinline__ bool chain_fast_ok(const double* __restrict__ b, const Ray64& r, double px, double py,
                                              double pz) {
    if (r.dx == 0.0 || r.dy == 0.0 || r.dz == 0.0) return false;
    const double o[3] = {r.ox, r.oy, r.oz}, p[3] = {px, py, pz};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double m = 0x1p-48 * (__builtin_fabs(b[a]) + __builtin_fabs(b[3 + a]) + __builtin_fabs(o[a]) +
                                    __builtin_fabs(p[a]));
        if (!(p[a] - b[a] >= m && b[3 + a] - p[a] >= m)) return false;
    }
    return true;
}
// The same test on the record's fp32 leaf box, rounded inward (lo up, hi
// down): a point inside it with the margin is inside the real box with more.
// The margin is widened by 2^-20 relative (and 2^-190 absolute) to cover the
// rounding gap between the fp32 and the real bounds in its own terms.
__device__ __forceinline__ bool chain_fast_ok32(const float (&b)[6], const Ray64& r, double px, double py,
                                                double pz) {
    if (r.dx == 0.0 || r.dy == 0.0 || r.dz == 0.0) return false;
    const double o[3] = {r.ox, r.oy, r.oz}, p[3] = {px, py, pz};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double lo = (double)b[a], hi = (double)b[3 + a];
        const double m = 0x1p-48 * ((__builtin_fabs(lo) + __builtin_fabs(hi)) * (1.0 + 0x1p-20) +
                                    __builtin_fabs(o[a]) + __builtin_fabs(p[a])) + 0x1p-190;
        if (!(p[a] - lo >= m && hi - p[a] >= m)) return false;
    }
    return true;
}

// Per-lane traversal stack: the top S entries live in LDS (one column per
// lane: entry e of lane t at lds[e % S][t], conflict-free for ds_read_b64),
// older entries spill to a global buffer interleaved over the lanes of the
// grid (spill entry e of lane g at spill[e * stride + g]), so lanes of a wave
// at the same depth share cache lines instead of each dirtying its own.
// C: columns of the LDS ring (256: one per thread of a 256-thread block; 64:
// one wave's own ring, the packet kernel's exit path).
template <int S, int C = 256>
struct LaneStack {
    static_assert(S > 0 && (S & (S - 1)) == 0, "the LDS ring is indexed modulo S: a power of two");
    uint2 (*lds)[C];
    uint2* spill;     // this lane's column: aux.spill + global lane index
    uint32_t stride;  // lanes of the grid (aux.grid * 256)
    int tid;
    int top;
    __device__ __forceinline__ void attach(uint2 (*l)[C], const RtLaunchAux& aux, int t) {
        static_assert(C == 256, "one column per thread of the block");
        lds = l;
        spill = reinterpret_cast<uint2*>(aux.spill) + ((size_t)blockIdx.x * 256 + (size_t)t);
        stride = (uint32_t)aux.grid * 256u;
        tid = t;
        top = 0;
    }
    // A wave's own ring (C = 64, column = lane) spilling at global lane
    // `lane_g` of a grid of `lanes` lanes.
    __device__ __forceinline__ void attach_wave(uint2 (*l)[C], RT_G uint64_t* sp, uint32_t lane_g, uint32_t lanes,
                                                int lane) {
        lds = l;
        spill = reinterpret_cast<uint2*>(sp) + lane_g;
        stride = lanes;
        tid = lane;
        top = 0;
    }
    __device__ __forceinline__ void push(uint32_t ref, float t) {
        const int slot = top & (S - 1);
        if (top >= S) spill[(size_t)(top - S) * stride] = lds[slot][tid];
        lds[slot][tid] = make_uint2(ref, __float_as_uint(t));
        top++;
    }
    __device__ __forceinline__ uint2 pop() {
        top--;
        const int slot = top & (S - 1);
        const uint2 e = lds[slot][tid];
        if (top >= S) lds[slot][tid] = spill[(size_t)(top - S) * stride];
        return e;
    }
};

}  // namespace rtk
