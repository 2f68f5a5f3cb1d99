// gfx950 primary-ray kernels: fused ray generation + wide-BVH traversal +
// exact fp64 resolve + head-light shading, one frame (or one row shard) per
// launch.
//
// Reference semantics reproduced (bit for bit):
//   ray generation  src/main.cpp:331-337 (+ camera.hpp:35-37 coefficients)
//   Ray reciprocal  src/primitives/ray.hpp:13-19
//   closest hit     src/stack_bvh.hpp:611-644 — min over detected triangles
//                   of |(o + d t) - o| with strict '<' in visit order
//   slab test       src/aabb.hpp:32-49 (fp64, std::min/std::max semantics)
//   Moller-Trumbore src/primitives/triangle.hpp:40-88 (fp64, EPS 1e-8)
//   shading         src/main.cpp:351-381 and the PPM byte cast
//                   src/utils/benchmark.hpp:105-114
//
// Two traversal kernels, both exact:
//   k_trace_exact   persistent waves pull 8x8 pixel tiles from an atomic
//                   queue; fp32 conservative traversal of W-wide nodes
//                   (outward-rounded boxes, per-frame widened slabs, ordered,
//                   distance-culled) with the traversal stack in LDS (ring of
//                   S entries per lane, global spill beyond); exact fp64
//                   Moller-Trumbore on leaf triangles and an fp64
//                   re-verification of the reference ancestor chain before a
//                   candidate may win (the reference only sees a triangle if
//                   every ancestor's fp64 slab test passes).  Distance ties
//                   resolve by the reference visit rank.  See DESIGN.md.
//   k_trace_literal the reference's own traversal (LIFO, no culling, no
//                   ordering) in fp64 on the real tree — a cross-check.
//
// This TU is compiled with -ffp-contract=off: every fp64 expression must
// round exactly like the reference's x86-64 build.  The fp32 traversal uses
// explicit fmaf where contraction is wanted.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"

namespace {

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

// main.cpp:332-337: d = dir + up*py + right*px; d *= 1/|d|; Ray{pos, d}
__device__ __forceinline__ Ray64 gen_ray(const RtFrameParams& fp, int i, int j) {
    const double px = fp.px[i], py = fp.py[j];
    double dx = (fp.dir[0] + fp.up[0] * py) + fp.right[0] * px;
    double dy = (fp.dir[1] + fp.up[1] * py) + fp.right[1] * px;
    double dz = (fp.dir[2] + fp.up[2] * py) + fp.right[2] * px;
    const double s = 1.0 / __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    dx = dx * s;
    dy = dy * s;
    dz = dz * s;
    Ray64 r;
    r.ox = fp.pos[0];
    r.oy = fp.pos[1];
    r.oz = fp.pos[2];
    r.dx = dx;
    r.dy = dy;
    r.dz = dz;
    const double inf = __builtin_huge_val();
    r.ix = dx != 0.0 ? 1.0 / dx : inf;
    r.iy = dy != 0.0 ? 1.0 / dy : inf;
    r.iz = dz != 0.0 ? 1.0 / dz : inf;
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
__device__ __forceinline__ void shade_store(const RtFrameParams& fp, const RtDevScene& sc, size_t o, const Best& b) {
    uint8_t c0 = 0, c1 = 0, c2 = 0;
    if (b.tri >= 0 && fp.rgb) {
        const uint32_t id = sc.tri_id[b.tri];
        double nx = sc.normal[3 * (size_t)id], ny = sc.normal[3 * (size_t)id + 1], nz = sc.normal[3 * (size_t)id + 2];
        const double nl = __builtin_sqrt(nx * nx + ny * ny + nz * nz);
        if (nl > 0.0) {
            const double s = 1.0 / nl;
            nx = nx * s; ny = ny * s; nz = nz * s;
        }
        double lx = fp.pos[0] - b.px, ly = fp.pos[1] - b.py, lz = fp.pos[2] - b.pz;
        const double dist = __builtin_sqrt(lx * lx + ly * ly + lz * lz);
        if (dist > 0.0) {
            const double s = 1.0 / dist;
            lx = lx * s; ly = ly * s; lz = lz * s;
        }
        const double diffuse = smax(0.0, nx * lx + ny * ly + nz * lz) * 1.35;
        const double att = 1.0 / (1.0 + 0.05 * dist * dist);
        const double I = sclamp((0.45 + diffuse * att) * 1.25, 0.0, 1.0);
        c0 = (uint8_t)sclamp((0.5 * (nx + 1.0)) * I * 255.0, 0.0, 255.0);
        c1 = (uint8_t)sclamp((0.5 * (ny + 1.0)) * I * 255.0, 0.0, 255.0);
        c2 = (uint8_t)sclamp((0.5 * (nz + 1.0)) * I * 255.0, 0.0, 255.0);
    }
    if (fp.rgb) {
        fp.rgb[3 * o] = c0;
        fp.rgb[3 * o + 1] = c1;
        fp.rgb[3 * o + 2] = c2;
    }
    if (fp.hit_id) fp.hit_id[o] = b.tri >= 0 ? sc.tri_id[b.tri] : RT_INVALID_REF;
    if (fp.dist) fp.dist[o] = b.tri >= 0 ? b.dist : -1.0;
    if (fp.hit_pos) {
        fp.hit_pos[3 * o] = b.tri >= 0 ? b.px : 0.0;
        fp.hit_pos[3 * o + 1] = b.tri >= 0 ? b.py : 0.0;
        fp.hit_pos[3 * o + 2] = b.tri >= 0 ? b.pz : 0.0;
    }
    if (b.tri >= 0 && fp.hit_count) atomicAdd(fp.hit_count, 1ull);
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

// Per-lane traversal stack: the top S entries live in LDS (one column per
// lane: entry e of lane t at lds[e % S][t], conflict-free for ds_read_b64),
// older entries spill to the lane's slice of a global buffer.
template <int S>
struct LaneStack {
    uint2 (*lds)[256];
    uint2* spill;
    int tid;
    int top;
    __device__ __forceinline__ void push(uint32_t ref, float t) {
        const int slot = top & (S - 1);
        if (top >= S) spill[top - S] = lds[slot][tid];
        lds[slot][tid] = make_uint2(ref, __float_as_uint(t));
        top++;
    }
    __device__ __forceinline__ uint2 pop() {
        top--;
        const int slot = top & (S - 1);
        const uint2 e = lds[slot][tid];
        if (top >= S) lds[slot][tid] = spill[top - S];
        return e;
    }
};

// --------------------------------------------------------------------------
// Fast exact kernel (persistent).
// --------------------------------------------------------------------------
template <int W, int S, bool COUNT>
__device__ __forceinline__ void trace_exact(const RtDevScene& sc, const RtFrameParams& fp, int i, int r,
                                            LaneStack<S>& st) {
    const int j = fp.row0 + r * fp.row_stride;
    const Ray64 ray = gen_ray(fp, i, j);

    // fp32 ray for the conservative box tests; a zero direction component
    // gets a large finite reciprocal (no 0*inf NaNs; same slab semantics).
    const float ox = (float)ray.ox, oy = (float)ray.oy, oz = (float)ray.oz;
    auto inv32 = [](double v) {
        float f = (float)v;
        if (!(__builtin_fabsf(f) <= 1e18f)) f = v < 0 ? -1e18f : 1e18f;
        return f;
    };
    const float ix = inv32(ray.ix), iy = inv32(ray.iy), iz = inv32(ray.iz);
    // Slab planes widened by fp.pad (world units): t = (plane -/+ pad - o)*inv.
    // Near planes use o + pad*sgn(inv), far planes o - pad*sgn(inv); pad bounds
    // every fp32 rounding of o, inv and the fma (DESIGN.md "exactness").
    const float px_ = ix >= 0.f ? fp.pad : -fp.pad, py_ = iy >= 0.f ? fp.pad : -fp.pad,
                pz_ = iz >= 0.f ? fp.pad : -fp.pad;
    const float onx = (ox + px_) * ix, ony = (oy + py_) * iy, onz = (oz + pz_) * iz;  // near offsets
    const float ofx = (ox - px_) * ix, ofy = (oy - py_) * iy, ofz = (oz - pz_) * iz;  // far offsets
    // near/far plane selection by direction sign (ray-constant)
    const int nxo = ix >= 0.f ? 0 : W, fxo = ix >= 0.f ? W : 0;
    const int nyo = iy >= 0.f ? 2 * W : 3 * W, fyo = iy >= 0.f ? 3 * W : 2 * W;
    const int nzo = iz >= 0.f ? 4 * W : 5 * W, fzo = iz >= 0.f ? 5 * W : 4 * W;
    // fp32 direction and origin magnitude for the triangle pre-filter
    const float dx32 = (float)ray.dx, dy32 = (float)ray.dy, dz32 = (float)ray.dz;
    const double omax = __builtin_fmax(__builtin_fmax(__builtin_fabs(ray.ox), __builtin_fabs(ray.oy)),
                                       __builtin_fabs(ray.oz));
    const float co32 = round_up_f(omax + 1e-30);
    // distance -> ray-parameter slack for culling: dist = |fl(o + d t) - o|
    // differs from t by <= 2^-52 |o| + 2^-50 t, covered by tslack + 2^-20 t
    const double tslack = 0x1p-40 * (omax + 1.0);

    Best best;
    uint32_t n_nodes = 0, n_tris = 0, n_chain = 0, n_chain_nodes = 0, n_pre = 0;
    // pass 0: traverse with the ancestor re-verification deferred to the
    //         winner (one check per ray, usually the margin test alone);
    // pass 1: only if that winner is invisible to the reference — traverse
    //         again verifying every would-be winner inline.
    for (int pass = 0; pass < 2; pass++) {
        best.dist = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
        best.rank = 0xFFFFFFFFu;
        best.tri = -1;
        best.px = best.py = best.pz = 0.0;
        float tcull = __builtin_huge_valf();
        uint32_t chain_leaf = 0xFFFFFFFFu;
        bool chain_res = false;
        st.top = 0;

        uint32_t cur = sc.root_ref;
        {
            const float* b = sc.root_box;
            const float tx0 = __builtin_fmaf(ix >= 0.f ? b[0] : b[1], ix, -onx);
            const float tx1 = __builtin_fmaf(ix >= 0.f ? b[1] : b[0], ix, -ofx);
            const float ty0 = __builtin_fmaf(iy >= 0.f ? b[2] : b[3], iy, -ony);
            const float ty1 = __builtin_fmaf(iy >= 0.f ? b[3] : b[2], iy, -ofy);
            const float tz0 = __builtin_fmaf(iz >= 0.f ? b[4] : b[5], iz, -onz);
            const float tz1 = __builtin_fmaf(iz >= 0.f ? b[5] : b[4], iz, -ofz);
            const float tn = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, 0.f));
            const float tf = fminf(fminf(tx1, ty1), tz1);
            if (!(tn <= tf)) cur = RT_INVALID_REF;
        }

        while (cur != RT_INVALID_REF) {
            if (!(cur & RT_LEAF_BIT)) {
                if (COUNT) n_nodes++;
                const float* nb = reinterpret_cast<const float*>(sc.nodes + (size_t)cur * sc.node_bytes);
                float nx[W], fx[W], ny[W], fy[W], nz[W], fz[W];
                uint32_t ref[W];
                load_w<W>(nx, nb + nxo);
                load_w<W>(fx, nb + fxo);
                load_w<W>(ny, nb + nyo);
                load_w<W>(fy, nb + fyo);
                load_w<W>(nz, nb + nzo);
                load_w<W>(fz, nb + fzo);
                load_refs<W>(ref, reinterpret_cast<const uint32_t*>(nb + 6 * W));
                float tn[W];
                uint32_t mask = 0;
#pragma unroll
                for (int c = 0; c < W; c++) {
                    const float a0 = __builtin_fmaf(nx[c], ix, -onx);
                    const float a1 = __builtin_fmaf(fx[c], ix, -ofx);
                    const float b0 = __builtin_fmaf(ny[c], iy, -ony);
                    const float b1 = __builtin_fmaf(fy[c], iy, -ofy);
                    const float c0 = __builtin_fmaf(nz[c], iz, -onz);
                    const float c1 = __builtin_fmaf(fz[c], iz, -ofz);
                    const float t0 = fmaxf(fmaxf(a0, b0), fmaxf(c0, 0.f));
                    const float t1 = fminf(fminf(a1, b1), fminf(c1, tcull));
                    tn[c] = t0;
                    if (t0 <= t1 && ref[c] != RT_INVALID_REF) mask |= 1u << c;
                }
                if (mask) {
                    // push all but the nearest, farthest first
                    while (__builtin_popcount(mask) > 1) {
                        float far_t = -1.f;
                        int far_c = 0;
#pragma unroll
                        for (int c = 0; c < W; c++)
                            if (((mask >> c) & 1u) && tn[c] > far_t) { far_t = tn[c]; far_c = c; }
                        uint32_t far_ref = ref[0];
#pragma unroll
                        for (int c = 1; c < W; c++)
                            if (c == far_c) far_ref = ref[c];
                        st.push(far_ref, far_t);
                        mask &= ~(1u << far_c);
                    }
                    const int c0 = __builtin_ctz(mask);
                    uint32_t nxt = ref[0];
#pragma unroll
                    for (int c = 1; c < W; c++)
                        if (c == c0) nxt = ref[c];
                    cur = nxt;
                    continue;
                }
            } else {
                const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                for (uint32_t q = first; q < first + cnt; q++) {
                    const float4* R = reinterpret_cast<const float4*>(sc.tri32 + 12 * (size_t)q);
                    if (COUNT) n_pre++;
                    if (!tri_prefilter(R[0], R[1], R[2], ox, oy, oz, dx32, dy32, dz32, co32, tcull)) continue;
                    if (COUNT) n_tris++;
                    const double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)q;
                    double t;
                    if (!mt64(T, ray, t)) continue;
                    double hx, hy, hz;
                    const double d = hit_dist(ray, t, hx, hy, hz);
                    const uint2 rl = *reinterpret_cast<const uint2*>(T + 9);  // {rank, leaf}
                    if (!(d < best.dist || (d == best.dist && rl.x < best.rank))) continue;
                    if (pass == 1) {
                        if (rl.y != chain_leaf) {
                            if (COUNT) n_chain++;
                            chain_leaf = rl.y;
                            chain_res = chain_ok(sc, rl.y, ray, n_chain_nodes);
                        }
                        if (!chain_res) continue;
                    }
                    best.dist = d;
                    best.rank = rl.x;
                    best.tri = (int32_t)q;
                    best.px = hx;
                    best.py = hy;
                    best.pz = hz;
                    tcull = round_up_f((d + tslack) * (1.0 + 0x1p-20));
                }
            }
            // pop the next subtree still in front of the current best
            cur = RT_INVALID_REF;
            while (st.top > 0) {
                const uint2 e = st.pop();
                if (__uint_as_float(e.y) <= tcull) {
                    cur = e.x;
                    break;
                }
            }
        }
        if (pass == 1 || best.tri < 0) break;
        // deferred re-verification of the winner's reference ancestor chain
        const uint32_t leaf = reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + 9)->y;
        if (COUNT) n_chain++;
        if (chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, best.px, best.py, best.pz)) break;
        if (chain_ok(sc, leaf, ray, n_chain_nodes)) break;
    }

    const size_t o = (size_t)r * fp.W + i;
    shade_store(fp, sc, o, best);
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[0], 1ull);
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[2], (unsigned long long)n_tris);
        atomicAdd(&fp.counters[3], (unsigned long long)n_chain);
        if (best.tri >= 0) atomicAdd(&fp.counters[4], 1ull);
        atomicAdd(&fp.counters[5], (unsigned long long)n_chain_nodes);
        atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
    }
}

// Persistent waves: each wave pulls 8x8 pixel tiles from `tile_ctr` until the
// shard is exhausted (every wave reaches the exit test each iteration).
template <int W, int S, bool COUNT>
__global__ void __launch_bounds__(256) k_trace_exact(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint2 lds[S][256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int tiles_x = (fp.W + 7) >> 3;
    const int tiles = tiles_x * ((fp.nrows + 7) >> 3);
    LaneStack<S> st;
    st.lds = lds;
    st.spill = reinterpret_cast<uint2*>(aux.spill) + ((size_t)blockIdx.x * 256 + tid) * aux.spill_cap;
    st.tid = tid;
    st.top = 0;
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = (int)atomicAdd(aux.tile_ctr, 1u);
        tile = __shfl(tile, 0);
        if (tile >= tiles) break;
        const int i = (tile % tiles_x) * 8 + (lane & 7);
        const int r = (tile / tiles_x) * 8 + (lane >> 3);
        if (i < fp.W && r < fp.nrows) trace_exact<W, S, COUNT>(sc, fp, i, r, st);
    }
}

// --------------------------------------------------------------------------
// Literal reference traversal (stack_bvh.hpp:611-644) on the real tree.
// --------------------------------------------------------------------------
__device__ __forceinline__ bool lane_pixel(const RtFrameParams& fp, int& i, int& r) {
    const int lane = threadIdx.x & 63;
    const int tiles_x = (fp.W + 7) >> 3;
    const int tiles_y = (fp.nrows + 7) >> 3;
    const int tile = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (tile >= tiles_x * tiles_y) return false;
    i = (tile % tiles_x) * 8 + (lane & 7);
    r = (tile / tiles_x) * 8 + (lane >> 3);
    return i < fp.W && r < fp.nrows;
}

template <int SMAX, bool COUNT>
__global__ void __launch_bounds__(256) k_trace_literal(RtDevScene sc, RtFrameParams fp) {
    int i, r;
    if (!lane_pixel(fp, i, r)) return;
    const int j = fp.row0 + r * fp.row_stride;
    const Ray64 ray = gen_ray(fp, i, j);
    Best best;
    best.dist = 1.7976931348623157e308;
    best.rank = 0;
    best.tri = -1;
    best.px = best.py = best.pz = 0.0;
    uint32_t st[SMAX];
    int sp = 0;
    st[sp++] = 0;
    uint32_t n_nodes = 0, n_tris = 0;
    while (sp > 0) {
        const uint32_t n = st[--sp];
        if (COUNT) n_nodes++;
        if (!box_hit64(sc.rbox + 6 * (size_t)n, ray)) continue;
        const uint32_t k0 = sc.rkid_off[n], k1 = sc.rkid_off[n + 1];
        if (k0 == k1) {
            const uint32_t b = sc.rrange[2 * n], e = sc.rrange[2 * n + 1];
            for (uint32_t q = b; q < e; q++) {
                if (COUNT) n_tris++;
                double t;
                if (!mt64(sc.tri64 + RT_TRI64_DOUBLES * (size_t)q, ray, t)) continue;
                double hx, hy, hz;
                const double d = hit_dist(ray, t, hx, hy, hz);
                if (d < best.dist) {
                    best.dist = d;
                    best.tri = (int32_t)q;
                    best.px = hx;
                    best.py = hy;
                    best.pz = hz;
                }
            }
        }
        for (uint32_t k = k0; k < k1; k++)
            if (sp < SMAX) st[sp++] = sc.rkid[k];
    }
    const size_t o = (size_t)r * fp.W + i;
    shade_store(fp, sc, o, best);
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[0], 1ull);
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[2], (unsigned long long)n_tris);
        if (best.tri >= 0) atomicAdd(&fp.counters[4], 1ull);
    }
}

constexpr int kLdsStack = 16;  // LDS ring entries per lane (8 B each)

template <int W>
hipError_t launch_exact(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, bool count,
                        hipStream_t s) {
    const dim3 grid((unsigned)aux.grid);
    if (count) hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, true>), grid, dim3(256), 0, s, sc, fp, aux);
    else hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, false>), grid, dim3(256), 0, s, sc, fp, aux);
    return hipGetLastError();
}

template <int SMAX>
hipError_t launch_literal_s(const RtDevScene& sc, const RtFrameParams& fp, bool count, dim3 grid, hipStream_t s) {
    if (count) hipLaunchKernelGGL((k_trace_literal<SMAX, true>), grid, dim3(256), 0, s, sc, fp);
    else hipLaunchKernelGGL((k_trace_literal<SMAX, false>), grid, dim3(256), 0, s, sc, fp);
    return hipGetLastError();
}

}  // namespace

namespace rt {

// Blocks per CU the persistent exact kernel is launched with.
int exact_blocks_per_cu(int width) {
    int n = 0;
    hipError_t e = hipSuccess;
    switch (width) {
        case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<2, kLdsStack, false>, 256, 0); break;
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<4, kLdsStack, false>, 256, 0); break;
        case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<8, kLdsStack, false>, 256, 0); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<16, kLdsStack, false>, 256, 0); break;
    }
    if (e != hipSuccess || n < 1) n = 1;
    return n < 8 ? n : 8;
}

int exact_lds_stack() { return kLdsStack; }

// Host entry: validates the launch geometry against what the kernels assume
// and dispatches on node width.  mode 0 = exact fast, 1 = literal.
hipError_t launch_trace(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, int mode, bool count,
                        hipStream_t s, uint32_t literal_stack) {
    if (fp.W <= 0 || fp.nrows <= 0) return hipSuccess;
    if (mode == 1) {
        const long tiles = (long)((fp.W + 7) / 8) * (long)((fp.nrows + 7) / 8);
        const dim3 grid((unsigned)((tiles + 3) / 4));
        if (literal_stack <= 64) return launch_literal_s<64>(sc, fp, count, grid, s);
        if (literal_stack <= 256) return launch_literal_s<256>(sc, fp, count, grid, s);
        if (literal_stack <= 1024) return launch_literal_s<1024>(sc, fp, count, grid, s);
        return hipErrorInvalidValue;
    }
    if (aux.spill_cap + kLdsStack < sc.stack_bound || !aux.tile_ctr || !aux.spill || aux.grid <= 0)
        return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(aux.tile_ctr, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    switch (sc.width) {
        case 2: return launch_exact<2>(sc, fp, aux, count, s);
        case 4: return launch_exact<4>(sc, fp, aux, count, s);
        case 8: return launch_exact<8>(sc, fp, aux, count, s);
        case 16: return launch_exact<16>(sc, fp, aux, count, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rt
