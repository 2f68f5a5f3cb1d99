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
//                   S entries per lane, global spill beyond); leaf triangles
//                   go through a conservative fp32 pre-filter and, if it
//                   cannot reject them, the exact fp64 Moller-Trumbore.  The
//                   winner's reference ancestor chain is re-verified (margin
//                   test, else the fp64 chain walk); if the reference could not
//                   see it, the ray is traversed again verifying inline.
//                   Distance ties resolve by the reference visit rank.
//   k_trace_literal the reference's own traversal (LIFO, no culling, no
//                   ordering) in fp64 on the real tree — a cross-check.
//
// This TU is compiled with -ffp-contract=off: every fp64 expression must
// round exactly like the reference's x86-64 build.  The fp32 traversal uses
// explicit fmaf where contraction is wanted.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels_common.h"
#include "rt_device.h"

namespace {

using namespace rtk;

// Keeps a value opaque to the optimiser so the fp64 ray is rebuilt where it
// is needed instead of being hoisted and held in 18 VGPRs for the whole walk.
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// fp32 view of one ray, everything the traversal loop needs.
struct Ray32 {
    float ox, oy, oz, dx, dy, dz, co;
    float ix, iy, iz;
    float onx, ony, onz, ofx, ofy, ofz;  // near / far plane offsets
};

__device__ __forceinline__ Ray32 make_ray32(const Ray64& ray, float pad) {
    Ray32 q;
    q.ox = (float)ray.ox;
    q.oy = (float)ray.oy;
    q.oz = (float)ray.oz;
    q.dx = (float)ray.dx;
    q.dy = (float)ray.dy;
    q.dz = (float)ray.dz;
    const double omax = __builtin_fmax(__builtin_fmax(__builtin_fabs(ray.ox), __builtin_fabs(ray.oy)),
                                       __builtin_fabs(ray.oz));
    q.co = round_up_f(omax + 1e-30);
    // zero direction components get a large finite reciprocal (no 0*inf NaNs)
    auto inv32 = [](double v) {
        float f = (float)v;
        if (!(__builtin_fabsf(f) <= 1e18f)) f = v < 0 ? -1e18f : 1e18f;
        return f;
    };
    q.ix = inv32(ray.ix);
    q.iy = inv32(ray.iy);
    q.iz = inv32(ray.iz);
    // Slab planes widened by `pad` (world units): near planes use
    // o + pad*sgn(inv), far planes o - pad*sgn(inv); pad bounds every fp32
    // rounding of o, inv and the fma (DESIGN.md "exactness").
    const float px = q.ix >= 0.f ? pad : -pad, py = q.iy >= 0.f ? pad : -pad, pz = q.iz >= 0.f ? pad : -pad;
    q.onx = (q.ox + px) * q.ix;
    q.ony = (q.oy + py) * q.iy;
    q.onz = (q.oz + pz) * q.iz;
    q.ofx = (q.ox - px) * q.ix;
    q.ofy = (q.oy - py) * q.iy;
    q.ofz = (q.oz - pz) * q.iz;
    return q;
}

// Winner of the exact resolve: distance (the reference's key), ray parameter
// (the hit point is rebuilt as fl(o + d t) bit-identically), rank, triangle.
struct Win {
    double dist, t;
    uint32_t rank;
    int32_t tri;
};

// --------------------------------------------------------------------------
// Fast exact kernel (persistent).
// --------------------------------------------------------------------------
template <int W, int S, bool COUNT>
__device__ __forceinline__ void trace_exact(const RtDevScene& sc, const RtFrameParams& fp, int i, int r,
                                            LaneStack<S>& st) {
    constexpr int G = W < 4 ? W : 4;  // children tested per load group
    const int j = fp.row0 + r * fp.row_stride;
    Ray32 q;
    double tslack;
    {
        const Ray64 ray = gen_ray(fp, i, j);
        q = make_ray32(ray, fp.pad);
        // dist = |fl(o + d t) - o| differs from t by <= 2^-52 |o| + 2^-50 t:
        // covered by tslack + the 2^-20 relative margin of tcull
        tslack = 0x1p-40 * ((double)q.co + 1.0);
    }
    // near/far plane selection by direction sign (ray-constant): a negative
    // reciprocal swaps lo and hi
    const bool sx = q.ix < 0.f, sy = q.iy < 0.f, sz = q.iz < 0.f;

    Win best;
    uint32_t n_nodes = 0, n_tris = 0, n_chain = 0, n_chain_nodes = 0, n_pre = 0;
    // pass 0: traverse with the ancestor re-verification deferred to the
    //         winner (one check per ray, usually the margin test alone);
    // pass 1: only if that winner is invisible to the reference — traverse
    //         again verifying every would-be winner inline.
    for (int pass = 0; pass < 2; pass++) {
        best.dist = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
        best.t = 0.0;
        best.rank = 0xFFFFFFFFu;
        best.tri = -1;
        float tcull = __builtin_huge_valf();
        uint32_t chain_leaf = 0xFFFFFFFFu;
        bool chain_res = false;
        st.top = 0;

        uint32_t cur = sc.root_ref;
        {
            const float* b = sc.root_box;
            const float tx0 = __builtin_fmaf(q.ix >= 0.f ? b[0] : b[1], q.ix, -q.onx);
            const float tx1 = __builtin_fmaf(q.ix >= 0.f ? b[1] : b[0], q.ix, -q.ofx);
            const float ty0 = __builtin_fmaf(q.iy >= 0.f ? b[2] : b[3], q.iy, -q.ony);
            const float ty1 = __builtin_fmaf(q.iy >= 0.f ? b[3] : b[2], q.iy, -q.ofy);
            const float tz0 = __builtin_fmaf(q.iz >= 0.f ? b[4] : b[5], q.iz, -q.onz);
            const float tz1 = __builtin_fmaf(q.iz >= 0.f ? b[5] : b[4], q.iz, -q.ofz);
            const float tn = fmaxf(fmaxf(tx0, ty0), fmaxf(tz0, 0.f));
            const float tf = fminf(fminf(tx1, ty1), tz1);
            if (!(tn <= tf)) cur = RT_INVALID_REF;
        }

        while (cur != RT_INVALID_REF) {
            if (!(cur & RT_LEAF_BIT)) {
                if (COUNT) n_nodes++;
                const float4* nb = reinterpret_cast<const float4*>(sc.nodes + (size_t)cur * sc.node_bytes);
                float tn[W];
                uint32_t rb[W];
                uint32_t mask = 0;
#pragma unroll
                for (int g = 0; g < W; g += G) {
                    float4 lo[G], hi[G];  // {lx,hx,ly,hy}, {lz,hz,ref,pad}
#pragma unroll
                    for (int c = 0; c < G; c++) {
                        lo[c] = nb[2 * (g + c)];
                        hi[c] = nb[2 * (g + c) + 1];
                    }
#pragma unroll
                    for (int c = 0; c < G; c++) {
                        const float a0 = __builtin_fmaf(sx ? lo[c].y : lo[c].x, q.ix, -q.onx);
                        const float a1 = __builtin_fmaf(sx ? lo[c].x : lo[c].y, q.ix, -q.ofx);
                        const float b0 = __builtin_fmaf(sy ? lo[c].w : lo[c].z, q.iy, -q.ony);
                        const float b1 = __builtin_fmaf(sy ? lo[c].z : lo[c].w, q.iy, -q.ofy);
                        const float c0 = __builtin_fmaf(sz ? hi[c].y : hi[c].x, q.iz, -q.onz);
                        const float c1 = __builtin_fmaf(sz ? hi[c].x : hi[c].y, q.iz, -q.ofz);
                        const float t0 = fmaxf(fmaxf(a0, b0), fmaxf(c0, 0.f));
                        const float t1 = fminf(fminf(a1, b1), fminf(c1, tcull));
                        const uint32_t ref = __float_as_uint(hi[c].z);
                        tn[g + c] = t0;
                        rb[g + c] = ref;
                        if (t0 <= t1 && ref != RT_INVALID_REF) mask |= 1u << (g + c);
                    }
                }
                if (mask) {
                    // push all hit children but the nearest, farthest first
                    while (__builtin_popcount(mask) > 1) {
                        float far_t = -1.f;
                        int far_c = 0;
#pragma unroll
                        for (int c = 0; c < W; c++)
                            if (((mask >> c) & 1u) && tn[c] > far_t) { far_t = tn[c]; far_c = c; }
                        st.push(rb[far_c], far_t);
                        mask &= ~(1u << far_c);
                    }
                    cur = rb[__builtin_ctz(mask)];
                    continue;
                }
            } else {
                const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                for (uint32_t k = first; k < first + cnt; k++) {
                    const float4* R = reinterpret_cast<const float4*>(sc.tri32 + 12 * (size_t)k);
                    if (COUNT) n_pre++;
                    if (!tri_prefilter(R[0], R[1], R[2], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull)) continue;
                    if (COUNT) n_tris++;
                    const Ray64 ray = gen_ray(fp, opaque(i), j);
                    const double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)k;
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
                    best.t = t;
                    best.rank = rl.x;
                    best.tri = (int32_t)k;
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
        const Ray64 ray = gen_ray(fp, opaque(i), j);
        double hx, hy, hz;
        (void)hit_dist(ray, best.t, hx, hy, hz);
        const uint32_t leaf = reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + 9)->y;
        if (COUNT) n_chain++;
        if (chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, hx, hy, hz)) break;
        if (chain_ok(sc, leaf, ray, n_chain_nodes)) break;
    }

    Best out;
    out.dist = best.dist;
    out.rank = best.rank;
    out.tri = best.tri;
    out.px = out.py = out.pz = 0.0;
    if (best.tri >= 0) {
        const Ray64 ray = gen_ray(fp, opaque(i), j);
        (void)hit_dist(ray, best.t, out.px, out.py, out.pz);
    }
    const size_t o = (size_t)r * fp.W + i;
    shade_store(fp, sc, o, out);
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

// --------------------------------------------------------------------------
// Wave-cooperative ("packet") exact kernel: the 64 rays of one 8x8 tile walk
// the tree together.  The current node is wave-uniform, so its bounds and
// child refs come in through the scalar data path (s_load into SGPRs, once per
// wave) instead of 64 per-lane copies through the vector memory pipe; each
// lane slab-tests its own ray against the W children; `ballot` turns the
// per-lane results into one 64-bit lane mask per child; the wave continues
// into the child nearest to its first active lane and pushes the others
// (ref + lane mask) on a wave-uniform stack in LDS.  Leaves are tested the
// same way: uniform triangle records, per-lane pre-filter, fp64 only for the
// lanes the pre-filter cannot reject.  Exactness machinery as trace_exact.
// --------------------------------------------------------------------------
struct __attribute__((aligned(32))) ChildRec {  // 32-B child record (rt_device.h)
    float lx, hx, ly, hy, lz, hz;
    uint32_t ref, pad;
};
typedef const __attribute__((address_space(4))) float* cfloat_p;
typedef const __attribute__((address_space(4))) ChildRec* cchild_p;

// Field-wise reads through the constant address space: adjacent uniform loads
// merge into one s_load_dwordx8 (child) / dwordx4 runs (triangle record).
__device__ __forceinline__ ChildRec load_child(cchild_p p) {
    ChildRec r;
    r.lx = p->lx;
    r.hx = p->hx;
    r.ly = p->ly;
    r.hy = p->hy;
    r.lz = p->lz;
    r.hz = p->hz;
    r.ref = p->ref;
    r.pad = p->pad;
    return r;
}
__device__ __forceinline__ float4 load_f4(cfloat_p p) { return make_float4(p[0], p[1], p[2], p[3]); }

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}

template <int W, int SP, bool COUNT>
__device__ __forceinline__ void trace_packet(const RtDevScene& sc, const RtFrameParams& fp, int i, int r, bool valid,
                                             uint4* __restrict__ wstack) {
    const int lane = threadIdx.x & 63;
    const uint64_t me = 1ull << lane;
    if (!valid) { i = 0; r = 0; }
    const int j = fp.row0 + r * fp.row_stride;
    Ray32 q;
    double tslack;
    {
        const Ray64 ray = gen_ray(fp, i, j);
        q = make_ray32(ray, fp.pad);
        tslack = 0x1p-40 * ((double)q.co + 1.0);
    }
    // slab offsets for the lo / hi planes (pad moves lo down and hi up)
    const float pd = fp.pad;
    const float olx = (q.ox + pd) * q.ix, ohx = (q.ox - pd) * q.ix;
    const float oly = (q.oy + pd) * q.iy, ohy = (q.oy - pd) * q.iy;
    const float olz = (q.oz + pd) * q.iz, ohz = (q.oz - pd) * q.iz;

    Win best;
    best.dist = 1.7976931348623157e308;
    best.t = 0.0;
    best.rank = 0xFFFFFFFFu;
    best.tri = -1;
    uint32_t n_nodes = 0, n_tris = 0, n_chain = 0, n_chain_nodes = 0, n_pre = 0;
    uint64_t need = uni64(__ballot(valid));
    for (int pass = 0; pass < 2 && need; pass++) {
        const bool mine = (need & me) != 0;
        if (mine) {
            best.dist = 1.7976931348623157e308;
            best.t = 0.0;
            best.rank = 0xFFFFFFFFu;
            best.tri = -1;
        }
        float tcull = __builtin_huge_valf();
        uint32_t chain_leaf = 0xFFFFFFFFu;
        bool chain_res = false;
        bool root_hit = false;
        {
            const float* b = sc.root_box;
            const float t0 = fmaxf(fmaxf(fminf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                         fminf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                                   fmaxf(fminf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)), 0.f));
            const float t1 = fminf(fminf(fmaxf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                         fmaxf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                                   fmaxf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)));
            root_hit = mine && t0 <= t1;
        }
        uint64_t active = uni64(__ballot(root_hit));
        uint32_t cur = sc.root_ref;
        int sp = 0;
        for (;;) {
            if (active != 0 && cur != RT_INVALID_REF) {
                const bool act = (active & me) != 0;
                if (!(cur & RT_LEAF_BIT)) {
                    if (COUNT && act) n_nodes++;
                    const cchild_p nb = (cchild_p)(sc.nodes + (size_t)cur * sc.node_bytes);
                    float key[W];
                    uint64_t m[W];
                    uint32_t rb[W];
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        const ChildRec ch = load_child(nb + c);  // s_load_dwordx8
                        rb[c] = ch.ref;
                        const float tlx = __builtin_fmaf(ch.lx, q.ix, -olx);
                        const float thx = __builtin_fmaf(ch.hx, q.ix, -ohx);
                        const float tly = __builtin_fmaf(ch.ly, q.iy, -oly);
                        const float thy = __builtin_fmaf(ch.hy, q.iy, -ohy);
                        const float tlz = __builtin_fmaf(ch.lz, q.iz, -olz);
                        const float thz = __builtin_fmaf(ch.hz, q.iz, -ohz);
                        const float t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
                        const float t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull));
                        const bool h = act && t0 <= t1;
                        m[c] = ch.ref == RT_INVALID_REF ? 0ull : uni64(__ballot(h));
                        // ordering key: the entry distance seen by the child's first lane
                        key[c] = m[c] ? __uint_as_float((uint32_t)__builtin_amdgcn_readlane(
                                            (int)__float_as_uint(t0), (int)__builtin_ctzll(m[c])))
                                      : __builtin_huge_valf();
                    }
                    // nearest child continues; the others go on the stack, farthest first
                    int nearest = -1;
                    float kn = __builtin_huge_valf();
#pragma unroll
                    for (int c = 0; c < W; c++)
                        if (m[c] && (nearest < 0 || key[c] < kn)) { kn = key[c]; nearest = c; }
                    if (nearest >= 0) {
                        uint32_t left = 0;
#pragma unroll
                        for (int c = 0; c < W; c++)
                            if (m[c] && c != nearest) left |= 1u << c;
                        while (left) {
                            int far_c = 0;
                            float kf = -1.f;
#pragma unroll
                            for (int c = 0; c < W; c++)
                                if (((left >> c) & 1u) && key[c] >= kf) { kf = key[c]; far_c = c; }
                            uint64_t fm = 0;
#pragma unroll
                            for (int c = 0; c < W; c++)
                                if (c == far_c) fm = m[c];
                            if (sp < SP) {
                                if (lane == 0) wstack[sp] = make_uint4(rb[far_c], (uint32_t)fm, (uint32_t)(fm >> 32), 0u);
                                sp++;
                            }
                            left &= ~(1u << far_c);
                        }
                        uint64_t nm = 0;
#pragma unroll
                        for (int c = 0; c < W; c++)
                            if (c == nearest) nm = m[c];
                        cur = rb[nearest];
                        active = nm;
                        continue;
                    }
                } else {
                    const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                    const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                    for (uint32_t k = first; k < first + cnt; k++) {
                        const cfloat_p R = (cfloat_p)(sc.tri32 + 12 * (size_t)k);  // scalar loads
                        const float4 A = load_f4(R), B = load_f4(R + 4), Cc = load_f4(R + 8);
                        if (COUNT && act) n_pre++;
                        const bool pre =
                            act && tri_prefilter(A, B, Cc, q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull);
                        if (__ballot(pre) == 0) continue;
                        if (!pre) continue;
                        if (COUNT) n_tris++;
                        const Ray64 ray = gen_ray(fp, opaque(i), j);
                        const double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)k;
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
                        best.t = t;
                        best.rank = rl.x;
                        best.tri = (int32_t)k;
                        tcull = round_up_f((d + tslack) * (1.0 + 0x1p-20));
                    }
                }
            }
            if (sp == 0) break;
            sp--;
            const uint4 e = wstack[sp];
            cur = uni(e.x);
            active = ((uint64_t)uni(e.z) << 32) | uni(e.y);
        }
        if (pass == 1) break;
        // deferred re-verification of each lane's winner
        bool redo = false;
        if (mine && best.tri >= 0) {
            const Ray64 ray = gen_ray(fp, opaque(i), j);
            double hx, hy, hz;
            (void)hit_dist(ray, best.t, hx, hy, hz);
            const uint32_t leaf =
                reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + 9)->y;
            if (COUNT) n_chain++;
            redo = !chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, hx, hy, hz) &&
                   !chain_ok(sc, leaf, ray, n_chain_nodes);
        }
        need = uni64(__ballot(redo));
    }
    if (!valid) return;
    Best out;
    out.dist = best.dist;
    out.rank = best.rank;
    out.tri = best.tri;
    out.px = out.py = out.pz = 0.0;
    if (best.tri >= 0) {
        const Ray64 ray = gen_ray(fp, opaque(i), j);
        (void)hit_dist(ray, best.t, out.px, out.py, out.pz);
    }
    const size_t o = (size_t)r * fp.W + i;
    shade_store(fp, sc, o, out);
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

template <int W, int SP, bool COUNT>
__global__ void __launch_bounds__(256) k_trace_packet(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint4 stacks[4][SP];
    const int lane = threadIdx.x & 63;
    uint4* wstack = stacks[threadIdx.x >> 6];
    const int tiles_x = (fp.W + 7) >> 3;
    const int tiles = tiles_x * ((fp.nrows + 7) >> 3);
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = (int)atomicAdd(aux.tile_ctr, 1u);
        tile = __shfl(tile, 0);
        if (tile >= tiles) break;
        const int i = (tile % tiles_x) * 8 + (lane & 7);
        const int r = (tile / tiles_x) * 8 + (lane >> 3);
        trace_packet<W, SP, COUNT>(sc, fp, i, r, i < fp.W && r < fp.nrows, wstack);
    }
}

// Persistent waves: each wave pulls 8x8 pixel tiles from `tile_ctr` until the
// shard is exhausted (every wave reaches the exit test each iteration).
template <int W, int S, bool COUNT, int MINW>
__global__ void __launch_bounds__(256, MINW) k_trace_exact(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
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
            for (uint32_t k = b; k < e; k++) {
                if (COUNT) n_tris++;
                double t;
                if (!mt64(sc.tri64 + RT_TRI64_DOUBLES * (size_t)k, ray, t)) continue;
                double hx, hy, hz;
                const double d = hit_dist(ray, t, hx, hy, hz);
                if (d < best.dist) {
                    best.dist = d;
                    best.tri = (int32_t)k;
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

constexpr int kLdsStack = 16;      // per-lane kernel: LDS ring entries per lane (8 B each)
constexpr int kPacketStack = 128;  // packet kernel: wave-uniform stack entries (16 B each)

// Kernel choice: the packet kernel unless its stack cannot hold the tree's
// bound or RT_KERNEL=lane asks for the per-lane kernel.
bool use_packet(uint32_t stack_bound) {
    static const bool lane_forced = [] {
        const char* e = getenv("RT_KERNEL");
        return e && e[0] == 'l';
    }();
    return !lane_forced && stack_bound <= (uint32_t)kPacketStack;
}

template <int W>
hipError_t launch_exact(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, bool count,
                        hipStream_t s) {
    const dim3 grid((unsigned)aux.grid);
    if (use_packet(sc.stack_bound)) {
        if (count) hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, true>), grid, dim3(256), 0, s, sc, fp, aux);
        else hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, false>), grid, dim3(256), 0, s, sc, fp, aux);
    } else {
        if (count) hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, true, 3>), grid, dim3(256), 0, s, sc, fp, aux);
        else hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, false, 3>), grid, dim3(256), 0, s, sc, fp, aux);
    }
    return hipGetLastError();
}

template <int W>
int blocks_per_cu_w(uint32_t stack_bound) {
    int n = 0;
    hipError_t e = use_packet(stack_bound)
                       ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_packet<W, kPacketStack, false>, 256, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<W, kLdsStack, false, 3>, 256, 0);
    return e == hipSuccess ? n : 1;
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
int exact_blocks_per_cu(int width, uint32_t stack_bound) {
    int n = width == 2   ? blocks_per_cu_w<2>(stack_bound)
            : width == 4 ? blocks_per_cu_w<4>(stack_bound)
            : width == 8 ? blocks_per_cu_w<8>(stack_bound)
                         : blocks_per_cu_w<16>(stack_bound);
    if (n < 1) n = 1;
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
