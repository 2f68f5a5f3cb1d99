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

#include <utility>

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

// fp32 reciprocal of a direction component without an fp64 division:
// v_rcp_f32 of the rounded component and one Newton step, within 3 * 2^-24
// relative of 1/d (the rounded fp64 quotient: 2^-24).  The slab pad covers
// it with room to spare: a relative reciprocal error e moves a slab plane by
// at most e (|o|max + |coord|max) in world units, and pad = 2^-19 of that
// (the fp32 roundings of o, the reciprocal and the fma then
// use 6 / 32 of the pad instead of 4 / 32).  Zero and tiny components get
// the same large finite value as the fp64 path (no 0 * inf NaNs).
#ifndef RT_FAST_INV
#define RT_FAST_INV 1
#endif
constexpr bool kFastInv = RT_FAST_INV != 0;
__device__ __forceinline__ float inv32_fast(double v) {
    const float f = (float)v;
    float r = __builtin_amdgcn_rcpf(f);
    r = __builtin_fmaf(r, __builtin_fmaf(-f, r, 1.f), r);
    if (!(__builtin_fabsf(r) <= 1e18f)) r = v < 0 ? -1e18f : 1e18f;
    return r;
}

template <bool FAST = false>
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
    if constexpr (FAST) {
        q.ix = inv32_fast(ray.dx);
        q.iy = inv32_fast(ray.dy);
        q.iz = inv32_fast(ray.dz);
    } else {
        q.ix = inv32(ray.ix);
        q.iy = inv32(ray.iy);
        q.iz = inv32(ray.iz);
    }
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
// Per-lane traversal counters (COUNT builds).
struct LaneCounts {
    uint32_t nodes = 0, tris = 0, chain = 0, chain_nodes = 0, pre = 0;
    // per-lane walks: records fetched once per wave instruction (the lanes
    // of one step that load the same node or triangle record share the
    // fetch), added in the wave's first active lane only
    uint32_t wnodes = 0, wtris = 0;
};

// COUNT builds: the wave-distinct node fetches and triangle records of one
// step of the lanes' walks that are active here (cur: each lane's next node
// or leaf ref).  Added to lc of the first active lane.
__device__ __forceinline__ void wave_step_fetches(uint32_t cur, LaneCounts& lc) {
    const uint64_t act = __ballot(1);
    const bool node = !(cur & RT_LEAF_BIT);
    uint64_t todo = act;
    uint32_t wn = 0, wt = 0;
    while (todo) {
        const int l = (int)__builtin_ctzll(todo);
        const uint32_t k = (uint32_t)__shfl((int)cur, l);
        todo &= ~__ballot(cur == k);
        if (k & RT_LEAF_BIT) wt += ((k >> 27) & 15u) + 1u;
        else wn++;
    }
    (void)node;
    if ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(act)) {
        lc.wnodes += wn;
        lc.wtris += wt;
    }
}

// The exact per-lane traversal of one ray, the reference's closest-hit
// semantics (stack_bvh.hpp:611-644) over the walk tree: ray_of() returns the
// fp64 ray (with reciprocals) — rebuilt on demand rather than held in
// registers — and pad is a slab margin valid for it (frame_pad's bound).
template <int W, int S, bool COUNT, class RayFn, int C>
__device__ __forceinline__ Win trace_core(const RtDevScene& sc, RayFn&& ray_of, float pad, LaneStack<S, C>& st,
                                          int pass0, LaneCounts& lc) {
    constexpr int G = W < 4 ? W : 4;  // children tested per load group
    Ray32 q;
    double tslack;
    {
        const Ray64 ray = ray_of();
        q = make_ray32(ray, pad);
        // dist = |fl(o + d t) - o| differs from t by <= 2^-52 |o| + 2^-50 t:
        // covered by tslack + the 2^-20 relative margin of tcull
        tslack = 0x1p-40 * ((double)q.co + 1.0);
    }
    // near/far plane selection by direction sign (ray-constant): a negative
    // reciprocal swaps lo and hi
    const bool sx = q.ix < 0.f, sy = q.iy < 0.f, sz = q.iz < 0.f;

    Win best;
    uint32_t& n_nodes = lc.nodes;
    uint32_t& n_tris = lc.tris;
    uint32_t& n_chain = lc.chain;
    uint32_t& n_chain_nodes = lc.chain_nodes;
    uint32_t& n_pre = lc.pre;
    // pass 0: traverse with the ancestor re-verification deferred to the
    //         winner (one check per ray, usually the margin test alone);
    // pass 1: only if that winner is invisible to the reference — traverse
    //         again verifying every would-be winner inline.
    for (int pass = pass0; pass < 2; pass++) {
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
                    const Ray64 ray = ray_of();
                    const double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)k;
                    double t;
                    if (!mt64(T, ray, t)) continue;
                    double hx, hy, hz;
                    const double d = hit_dist(ray, t, hx, hy, hz);
                    const uint32_t rank = sc.tri_rank[k];
                    if (!(d < best.dist || (d == best.dist && rank < best.rank))) continue;
                    if (pass == 1) {
                        const uint32_t leaf = reinterpret_cast<const uint2*>(T + RT_T64_IDLEAF)->y;
                        if (leaf != chain_leaf) {
                            if (COUNT) n_chain++;
                            chain_leaf = leaf;
                            chain_res = chain_ok(sc, leaf, ray, n_chain_nodes);
                        }
                        if (!chain_res) continue;
                    }
                    best.dist = d;
                    best.t = t;
                    best.rank = rank;
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
        const Ray64 ray = ray_of();
        double hx, hy, hz;
        (void)hit_dist(ray, best.t, hx, hy, hz);
        const uint32_t leaf =
            reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + RT_T64_IDLEAF)->y;
        if (COUNT) n_chain++;
        if (chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, hx, hy, hz)) break;
        if (chain_ok(sc, leaf, ray, n_chain_nodes)) break;
    }

    return best;
}

// The per-lane traversal with the fp64 work deferred (K candidates per lane,
// cand[c][tid] in LDS): the walk is fp32 only — tri_classify sorts each leaf
// triangle into reject / borderline / certain (a certain hit's upper bound
// tightens the culling distance at once) and appends the survivors — and the
// exact fp64 Moller-Trumbore of the survivors runs after the walk, when the
// wave's lanes do it together instead of one divergent lane at a time inside
// the loop.  The winner is the (distance, visit rank) minimum and its
// reference ancestor chain is re-verified, as in k_resolve.
// A lane whose list overflows (after compaction against the culling
// distance), or whose winner the reference cannot see, falls back to
// trace_core (pass 0 / pass 1): the same answer, the slow way.
//
// lane_walk: the fp32 walk of ray q; on return cand[0..nc) hold the
// survivors ({triangle, bits of t lower bound}), tcull the culling distance,
// and `over` is set if a survivor had to be dropped.
// QN (W = 8): node boxes from the quantised copy sc.qnodes (96 B per node
// instead of 256 B: 6 vector loads per node step instead of 16; the planes
// are 8-bit offsets from a per-node origin in steps of 2^e, each plane's t
// one fma from per-node terms — DESIGN.md §11).
template <int W, int S, int K, bool COUNT, bool QN = false>
struct LaneWalk {
    static_assert(!QN || W == 8, "quantised nodes are 8 wide");
    static constexpr int G = W < 4 ? W : 4;  // children tested per load group
    Ray32 q;
    float tsl;
    float tcull;
    int nc;
    bool over;
    uint32_t cur;  // the node or leaf to visit next; RT_INVALID_REF: the walk is over

    // The root test; the walk starts at the root if the ray enters its box.
    __device__ __forceinline__ void begin(const RtDevScene& sc, const Ray32& q_, float tsl_, LaneStack<S>& st) {
        q = q_;
        tsl = tsl_;
        tcull = __builtin_huge_valf();
        nc = 0;
        over = false;
        st.top = 0;
        cur = sc.root_ref;
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

    // The next subtree still in front of the culling distance, off the stack.
    __device__ __forceinline__ void pop_next(LaneStack<S>& st) {
        cur = RT_INVALID_REF;
        while (st.top > 0) {
            const uint2 e = st.pop();
            if (__uint_as_float(e.y) <= tcull) {
                cur = e.x;
                break;
            }
        }
    }

    // An inner node: descend into its nearest hit child (the others pushed),
    // or pop if no child is hit.
    __device__ __forceinline__ void visit_node(const RtDevScene& sc, LaneStack<S>& st, LaneCounts& lc) {
        const bool sx = q.ix < 0.f, sy = q.iy < 0.f, sz = q.iz < 0.f;
        if (COUNT) lc.nodes++;
        float tn[W];
        uint32_t rb[W];
        uint32_t mask = 0;
        if constexpr (QN) {
            const uint4* qb = reinterpret_cast<const uint4*>(sc.qnodes + (size_t)cur * RT_QNODE_BYTES);
            const uint4 h = qb[0], PX = qb[1], PY = qb[2], PZ = qb[3], R0 = qb[4], R1 = qb[5];
            // t of plane q: q (2^e ix) + (origin ix - o_near/far ix), exactly
            // the fp32 walk's plane with o +- pad (make_ray32)
            const float ox = __uint_as_float(h.x), oy = __uint_as_float(h.y), oz = __uint_as_float(h.z);
            const float ssx = __uint_as_float((h.w & 0xFFu) << 23) * q.ix;
            const float ssy = __uint_as_float(((h.w >> 8) & 0xFFu) << 23) * q.iy;
            const float ssz = __uint_as_float(((h.w >> 16) & 0xFFu) << 23) * q.iz;
            const float anx = __builtin_fmaf(ox, q.ix, -q.onx), afx = __builtin_fmaf(ox, q.ix, -q.ofx);
            const float any_ = __builtin_fmaf(oy, q.iy, -q.ony), afy = __builtin_fmaf(oy, q.iy, -q.ofy);
            const float anz = __builtin_fmaf(oz, q.iz, -q.onz), afz = __builtin_fmaf(oz, q.iz, -q.ofz);
            // near / far plane bytes: lo for a positive direction, hi for a negative one
            const uint32_t nx0 = sx ? PX.z : PX.x, nx1 = sx ? PX.w : PX.y, fx0 = sx ? PX.x : PX.z,
                           fx1 = sx ? PX.y : PX.w;
            const uint32_t ny0 = sy ? PY.z : PY.x, ny1 = sy ? PY.w : PY.y, fy0 = sy ? PY.x : PY.z,
                           fy1 = sy ? PY.y : PY.w;
            const uint32_t nz0 = sz ? PZ.z : PZ.x, nz1 = sz ? PZ.w : PZ.y, fz0 = sz ? PZ.x : PZ.z,
                           fz1 = sz ? PZ.y : PZ.w;
            const uint32_t refs[8] = {R0.x, R0.y, R0.z, R0.w, R1.x, R1.y, R1.z, R1.w};
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const int sh = 8 * (c & 3);
                auto byte = [&](uint32_t w0, uint32_t w1) { return (float)(((c < 4 ? w0 : w1) >> sh) & 0xFFu); };
                const float a0 = __builtin_fmaf(byte(nx0, nx1), ssx, anx);
                const float a1 = __builtin_fmaf(byte(fx0, fx1), ssx, afx);
                const float b0 = __builtin_fmaf(byte(ny0, ny1), ssy, any_);
                const float b1 = __builtin_fmaf(byte(fy0, fy1), ssy, afy);
                const float c0 = __builtin_fmaf(byte(nz0, nz1), ssz, anz);
                const float c1 = __builtin_fmaf(byte(fz0, fz1), ssz, afz);
                const float t0 = fmaxf(fmaxf(a0, b0), fmaxf(c0, 0.f));
                const float t1 = fminf(fminf(a1, b1), fminf(c1, tcull));
                tn[c] = t0;
                rb[c] = refs[c];
                if (t0 <= t1 && refs[c] != RT_INVALID_REF) mask |= 1u << c;
            }
        } else {
        const float4* nb = reinterpret_cast<const float4*>(sc.nodes + (size_t)cur * sc.node_bytes);
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
            return;
        }
        pop_next(st);
    }

    // A leaf: its triangles through tri_classify into the candidate list; pop.
    __device__ __forceinline__ void visit_leaf(LaneStack<S>& st, const RtDevScene& sc, uint2 (*cand)[256],
                                               LaneCounts& lc) {
        const int tid = st.tid;
        const uint32_t first = cur & RT_LEAF_FIRST_MASK;
        const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
        for (uint32_t k = first; k < first + cnt; k++) {
            const float4* R = reinterpret_cast<const float4*>(sc.tri32 + 12 * (size_t)k);
            if (COUNT) lc.pre++;
            float tl, tu;
            const int cls = tri_classify(R[0], R[1], R[2], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull, tl, tu);
            if (cls == 0) continue;
            // dist of a certain hit <= (tu + slack)(1 + 2^-20)
            if (cls == 2) tcull = fminf(tcull, (tu + tsl) * (1.f + 0x1p-20f));
            if (nc == K) {
                int m = 0;
                for (int c = 0; c < K; c++) {
                    const uint2 e = cand[c][tid];
                    if (__uint_as_float(e.y) <= tcull) cand[m++][tid] = e;
                }
                nc = m;
            }
            if (nc < K) {
                cand[nc][tid] = make_uint2(k, __float_as_uint(tl));
                nc++;
            } else {
                over = true;
            }
        }
        pop_next(st);
    }

    // One step of the walk (cur valid): one node or leaf visit.
    __device__ __forceinline__ void step(const RtDevScene& sc, LaneStack<S>& st, uint2 (*cand)[256], LaneCounts& lc) {
        if (!(cur & RT_LEAF_BIT))
            visit_node(sc, st, lc);
        else
            visit_leaf(st, sc, cand, lc);
    }
};

// lane_walk: the fp32 walk of ray q to its end (LaneWalk::begin, then steps).
template <int W, int S, int K, bool COUNT, bool QN = false>
__device__ __forceinline__ void lane_walk(const RtDevScene& sc, const Ray32& q, float tsl, LaneStack<S>& st,
                                          uint2 (*cand)[256], LaneCounts& lc, float& tcull_out, int& nc_out,
                                          bool& over_out) {
    LaneWalk<W, S, K, COUNT, QN> w;
    w.begin(sc, q, tsl, st);
    while (w.cur != RT_INVALID_REF) {
        if constexpr (COUNT) wave_step_fetches(w.cur, lc);
        w.step(sc, st, cand, lc);
    }
    tcull_out = w.tcull;
    nc_out = w.nc;
    over_out = w.over;
}

// Exact resolve of a candidate list (k_resolve's selection): the (distance,
// visit rank) minimum of the fp64 hits among get(0 .. nc-1) whose t lower
// bound is within tcull.  Returns 0 with the winner in best (tri < 0: none),
// or 1 if the reference cannot see the winner (its ancestor chain fails).
template <bool COUNT, class GetFn>
__device__ __forceinline__ int resolve_cands(const RtDevScene& sc, const Ray64& ray, GetFn&& get, int nc, float tcull,
                                             Win& best, LaneCounts& lc) {
    best.dist = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
    best.t = 0.0;
    best.rank = 0xFFFFFFFFu;
    best.tri = -1;
    for (int c = 0; c < nc; c++) {
        const uint2 e = get(c);
        if (__uint_as_float(e.y) > tcull) continue;  // cannot beat a certain hit
        if (COUNT) lc.tris++;
        const double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)e.x;
        double t;
        if (!mt64(T, ray, t)) continue;
        double hx, hy, hz;
        const double d = hit_dist(ray, t, hx, hy, hz);
        bool take = d < best.dist;
        if (!take && d == best.dist) {  // tie: the reference keeps the earlier visit
            if (best.rank == 0xFFFFFFFFu) best.rank = sc.tri_rank[best.tri];
            const uint32_t rank = sc.tri_rank[e.x];
            take = rank < best.rank;
            if (take) best.rank = rank;
        } else if (take) {
            best.rank = 0xFFFFFFFFu;  // visit ranks are loaded on a tie only
        }
        if (take) {
            best.dist = d;
            best.t = t;
            best.tri = (int32_t)e.x;
        }
    }
    if (best.tri < 0) return 0;
    if (best.rank == 0xFFFFFFFFu) best.rank = sc.tri_rank[best.tri];
    // the reference must see the winner: re-verify its ancestor chain
    double hx, hy, hz;
    (void)hit_dist(ray, best.t, hx, hy, hz);
    const uint32_t leaf =
        reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + RT_T64_IDLEAF)->y;
    if (COUNT) lc.chain++;
    if (chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, hx, hy, hz)) return 0;
    if (chain_ok(sc, leaf, ray, lc.chain_nodes)) return 0;
    return 1;
}

template <int W, int S, int K, bool COUNT, bool QN = false, class RayFn>
__device__ __forceinline__ Win trace_deferred(const RtDevScene& sc, RayFn&& ray_of, float pad, LaneStack<S>& st,
                                              uint2 (*cand)[256], LaneCounts& lc) {
    Ray32 q;
    float tsl;  // distance slack (trace_core's tslack), fp32 rounded up
    {
        const Ray64 ray = ray_of();
        q = make_ray32(ray, pad);
        tsl = round_up_f(0x1p-40 * ((double)q.co + 1.0));
    }
    float tcull;
    int nc;
    bool over;
    lane_walk<W, S, K, COUNT, QN>(sc, q, tsl, st, cand, lc, tcull, nc, over);
    if (over) return trace_core<W, S, COUNT>(sc, ray_of, pad, st, 0, lc);
    Win best;
    const int tid = st.tid;
    if (resolve_cands<COUNT>(sc, ray_of(), [&](int c) { return cand[c][tid]; }, nc, tcull, best, lc) == 0)
        return best;
    return trace_core<W, S, COUNT>(sc, ray_of, pad, st, 1, lc);
}

// Exact per-lane traversal of the primary ray of pixel (i, r) of the sample
// frame whose camera is `cam`.
template <int W, int S, bool COUNT, int C>
__device__ __forceinline__ Best trace_exact_cam(const RtDevScene& sc, const RtFrameParams& fp, const RtFrameCam& cam,
                                                int i, int r, LaneStack<S, C>& st, int pass0 = 0, bool fixup = false) {
    const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, r);
    auto ray_of = [&]() { return gen_ray(fp, cam, opaque(i), j); };
    LaneCounts lc;
    const Win best = trace_core<W, S, COUNT>(sc, ray_of, cam.pad, st, pass0, lc);
    const uint32_t n_nodes = lc.nodes, n_tris = lc.tris, n_chain = lc.chain, n_chain_nodes = lc.chain_nodes,
                   n_pre = lc.pre;
    Best out;
    out.dist = best.dist;
    out.rank = best.rank;
    out.tri = best.tri;
    out.px = out.py = out.pz = 0.0;
    if (best.tri >= 0) {
        const Ray64 ray = ray_of();
        (void)hit_dist(ray, best.t, out.px, out.py, out.pz);
    }
    if (COUNT && fp.counters) {
        if (!fixup) atomicAdd(&fp.counters[0], 1ull);  // a fixed-up ray was counted by the packet kernel
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[2], (unsigned long long)n_tris);
        atomicAdd(&fp.counters[3], (unsigned long long)n_chain);
        if (best.tri >= 0) atomicAdd(&fp.counters[4], 1ull);
        atomicAdd(&fp.counters[5], (unsigned long long)n_chain_nodes);
        atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
    }
    return out;
}
// ... of frame f of the launch.
template <int W, int S, bool COUNT, int C>
__device__ __forceinline__ Best trace_exact(const RtDevScene& sc, const RtFrameParams& fp, int f, int i, int r,
                                            LaneStack<S, C>& st, int pass0 = 0, bool fixup = false) {
    return trace_exact_cam<W, S, COUNT>(sc, fp, frame_cam(fp, f), i, r, st, pass0, fixup);
}

// Adds each active lane's v (< 2^BITS) to *p with one atomic per wave.
template <int BITS = 5>
__device__ __forceinline__ void wave_add(RT_G unsigned long long* p, uint32_t v) {
    uint32_t sum = 0;
#pragma unroll
    for (int b = 0; b < BITS; b++) sum += (uint32_t)__builtin_popcountll(__ballot((v >> b) & 1u)) << b;
    const uint64_t act = __ballot(1);
    if (p && sum != 0 && (int)(threadIdx.x & 63) == __builtin_ctzll(act)) atomicAdd(p, (unsigned long long)sum);
}

// Adds each active lane's v (< 2^BITS) to base[key] with one atomic per
// distinct key of the wave: the lanes of a fix-up wave take redo-list entries
// of different poses of the launch, whose hit counts are separate counters.
template <int BITS = 6>
__device__ __forceinline__ void wave_add_keyed(RT_G unsigned long long* base, int key, uint32_t v) {
    uint64_t todo = __ballot(1);
    const int lane = (int)(threadIdx.x & 63);
    while (todo) {
        const int leader = (int)__builtin_ctzll(todo);
        const int k = __shfl(key, leader);
        const bool mine = key == k;
        uint32_t sum = 0;
#pragma unroll
        for (int b = 0; b < BITS; b++) sum += (uint32_t)__builtin_popcountll(__ballot(mine && ((v >> b) & 1u))) << b;
        if (base && sum != 0 && lane == leader) atomicAdd(base + k, (unsigned long long)sum);
        todo &= ~__ballot(mine);
    }
}

// All spp samples of pixel (i, r) of pose p, whose camera is `pose`, with the
// per-lane exact kernel: per-sample outputs and the averaged colour; returns
// the samples hit.  (The pose comes in by itself so that a caller holding
// the launch parameters in registers never indexes their pose array with a
// lane-varying p: that array would go to the private segment.)
template <int W, int S, bool COUNT, int C>
__device__ __forceinline__ uint32_t trace_pixel_at(const RtDevScene& sc, const RtFrameParams& fp, const RtPose& pose,
                                                   int p, int i, int r, LaneStack<S, C>& st, int pass0 = 0,
                                                   bool fixup = false) {
    const size_t po = out_index(fp, p, (size_t)r * fp.W + i);
    double acc[3] = {0.0, 0.0, 0.0};
    uint32_t hits = 0;
    for (int k = 0; k < fp.spp; k++) {
        const RtFrameCam cam = frame_cam_of(pose, fp, p * fp.spp + k);
        const Best b = trace_exact_cam<W, S, COUNT>(sc, fp, cam, i, r, st, pass0, fixup);
        const Shade sh = shade_of(sc, b.tri);
        store_sample(fp, po * (size_t)fp.spp + k, b, sh);
        double c[3];
        shade_color(cam, b, sh, c);
        acc[0] = acc[0] + c[0];
        acc[1] = acc[1] + c[1];
        acc[2] = acc[2] + c[2];
        hits += b.tri >= 0;
    }
    store_rgb(fp, po, acc);
    return hits;
}
// ... with the pose's hit count added (the lanes of a wave may hold pixels of
// different poses).
template <int W, int S, bool COUNT, int C>
__device__ __forceinline__ void trace_pixel(const RtDevScene& sc, const RtFrameParams& fp, int p, int i, int r,
                                            LaneStack<S, C>& st, int pass0 = 0, bool fixup = false) {
    const uint32_t hits = trace_pixel_at<W, S, COUNT>(sc, fp, fp.pose[p], p, i, r, st, pass0, fixup);
    wave_add_keyed(fp.hit_count, p, hits);
}

#include "packet_kernel.h"
#include "path_kernel.h"
#include "queue_paths.h"

// Finishes the pixels the packet pipeline handed over (redo list, count in
// tile_ctr[RT_REDO_COUNT]) with the per-lane exact kernel: from pass 0 after a
// candidate overflow, straight into the inline-verifying pass 1 when the
// winner's ancestor chain failed.  The list holds redo_cap entries (a fixed
// pool, not one per pixel); a count past it means entries were not stored, and
// the launch is retried whole here: every pose pixel of the launch goes through
// the exact per-lane path (from pass 0, which ends in pass 1 when needed) and
// the walk kernel's hit-count partials are discarded, since every pixel is
// counted again.  Grid-stride; every thread reaches the exit test.  It also leaves the launch's work-queue block zeroed for the next
// launch: block 0 folds the per-frame hit-count partials into the caller's
// counters and clears them, the tile queues and the pool counter (nothing
// else reads them now); the last block to have read the redo count clears it.
template <int W, int S, bool COUNT>
__global__ void __launch_bounds__(256) k_fixup(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint2 lds[S][256];
    __shared__ unsigned long long frame_sum[RT_MAX_BATCH];
    __shared__ uint32_t n_sh;
    const int tid = threadIdx.x;
    if (tid == 0) {
        n_sh = *(volatile uint32_t*)(aux.tile_ctr + RT_REDO_COUNT);
        // the launch's redo count to the host (it sizes the slot's list and
        // the fix-up grid of the next launches by it; a vector store)
        if (blockIdx.x == 0 && aux.redo_seen)
            __hip_atomic_store(aux.redo_seen, n_sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence();
        if (atomicAdd(aux.tile_ctr + RT_FIXUP_DONE, 1u) == gridDim.x - 1) {
            aux.tile_ctr[RT_REDO_COUNT] = 0;
            aux.tile_ctr[RT_FIXUP_DONE] = 0;
        }
    }
    if (blockIdx.x == 0) {
        if (tid < RT_MAX_BATCH) frame_sum[tid] = 0;
        __syncthreads();
        const bool retry = n_sh > aux.redo_cap;  // (n_sh is set: tid 0 wrote it before the barrier)
        const int poses = fp.nframes / fp.spp;
        for (int k = tid; k < poses * RT_HIT_SLOTS; k += 256) {
            RT_G uint32_t* const slot = aux.tile_ctr + RT_HIT_BASE + k * RT_QUEUE_STRIDE;
            const uint32_t v = *slot;
            if (v) {
                atomicAdd(&frame_sum[k / RT_HIT_SLOTS], (unsigned long long)v);
                *slot = 0;
            }
        }
        if (tid < RT_QUEUES) aux.tile_ctr[tid * RT_QUEUE_STRIDE] = 0;
        if (tid == 0) aux.tile_ctr[RT_POOL_COUNT] = 0;
        if (tid < RT_QUEUES) aux.tile_ctr[RT_COPY_BASE + tid * RT_QUEUE_STRIDE] = 0;
        __syncthreads();
        if (!retry && fp.hit_count && tid < poses && frame_sum[tid]) atomicAdd(fp.hit_count + tid, frame_sum[tid]);
    }
    __syncthreads();
    const uint32_t npix = (uint32_t)fp.W * (uint32_t)fp.nrows;
    const bool retry = n_sh > aux.redo_cap;
    // the redo list, or (retry) every pose pixel of the launch
    const uint32_t n = retry ? npix * (uint32_t)(fp.nframes / fp.spp) : n_sh;
    if (n == 0) return;
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    // (grid-stride over the redo list; every thread reaches the exit test)
    for (uint32_t e = blockIdx.x * 256u + (uint32_t)tid; e < n; e += gridDim.x * 256u) {
        // (each entry taken is left kRedoEmpty for the next launch)
        if (retry && e < n_sh && e < aux.redo_cap) aux.redo[e] = kRedoEmpty;
        const uint32_t v = retry ? e : atomicExch(aux.redo + e, kRedoEmpty);
        const uint32_t ob = v & ~kRedoPass1;  // pixel of the batch: pose * npix + pixel
        const int p = (int)(ob / npix);
        const uint32_t o = ob - (uint32_t)p * npix;
        const int i = (int)(o % (uint32_t)fp.W), r = (int)(o / (uint32_t)fp.W);
        // (a retry re-traces pixels the walk counted already: no fetch counts)
        if (COUNT && !retry)
            trace_pixel<W, S, true>(sc, fp, p, i, r, st, (v & kRedoPass1) ? 1 : 0, true);
        else
            trace_pixel<W, S, false>(sc, fp, p, i, r, st, (v & kRedoPass1) ? 1 : 0, true);
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
    st.attach(lds, aux, tid);
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = (int)atomicAdd(aux.tile_ctr, 1u);
        tile = __shfl(tile, 0);
        if (tile >= tiles) break;
        const int i = (tile % tiles_x) * 8 + (lane & 7);
        const int r = (tile / tiles_x) * 8 + (lane >> 3);
        if (i < fp.W && r < fp.nrows) trace_pixel<W, S, COUNT>(sc, fp, 0, i, r, st);
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
__device__ __forceinline__ Best trace_literal(const RtDevScene& sc, const Ray64& ray, uint32_t& n_nodes,
                                              uint32_t& n_tris) {
    Best best;
    best.dist = 1.7976931348623157e308;
    best.rank = 0;
    best.tri = -1;
    best.px = best.py = best.pz = 0.0;
    uint32_t st[SMAX];
    int sp = 0;
    st[sp++] = 0;
    while (sp > 0) {
        const uint32_t n = st[--sp];
        if (COUNT) n_nodes++;
        if (!box_hit64(sc.rbox + 6 * (size_t)n, ray)) continue;
        const uint32_t k0 = sc.rkid_off[n], k1 = sc.rkid_off[n + 1];
        if (k0 == k1) {
            const uint32_t b = sc.rrange[2 * n], e = sc.rrange[2 * n + 1];
            for (uint32_t kr = b; kr < e; kr++) {
                const uint32_t k = sc.ref2walk[kr];  // triangle records are in walk (BVH) order
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
    return best;
}

// One pose (spp samples per pixel) per launch.
template <int SMAX, bool COUNT>
__global__ void __launch_bounds__(256) k_trace_literal(RtDevScene sc, RtFrameParams fp) {
    int i, r;
    if (!lane_pixel(fp, i, r)) return;
    const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, r);
    const size_t po = (size_t)r * fp.W + i;
    uint32_t n_nodes = 0, n_tris = 0, hits = 0;
    double acc[3] = {0.0, 0.0, 0.0};
    for (int k = 0; k < fp.spp; k++) {
        const RtFrameCam cam = frame_cam(fp, k);
        const Ray64 ray = gen_ray(fp, cam, i, j);
        const Best best = trace_literal<SMAX, COUNT>(sc, ray, n_nodes, n_tris);
        const Shade sh = shade_of(sc, best.tri);
        store_sample(fp, po * (size_t)fp.spp + k, best, sh);
        double c[3];
        shade_color(cam, best, sh, c);
        acc[0] = acc[0] + c[0];
        acc[1] = acc[1] + c[1];
        acc[2] = acc[2] + c[2];
        hits += best.tri >= 0;
    }
    store_rgb(fp, po, acc);
    wave_add(fp.hit_count, hits);
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[0], (unsigned long long)fp.spp);
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[2], (unsigned long long)n_tris);
        if (hits) atomicAdd(&fp.counters[4], (unsigned long long)hits);
    }
}

constexpr int kLdsStack = 16;      // per-lane kernel: LDS ring entries per lane (8 B each)
#ifndef RT_PATHS_STACK
#define RT_PATHS_STACK 8  // 24 KB LDS per block with the candidates: 5 waves/SIMD fit
#endif
constexpr int kPathStack = RT_PATHS_STACK;  // path kernel: LDS ring entries per lane
constexpr int kPacketStack = 128;  // packet kernel: wave-uniform stack entries (4 B each)
constexpr int kCandidates = RT_CAND_LDS;  // packet kernel: LDS candidate list entries per lane (8 B each)
// k_fixup blocks: the redo list is short (~0 entries on the sponza proxy), and
// 32 blocks (32 KB of LDS each) start on the first CUs the launch frees, while
// the next launch on the other stream fills the rest (256 blocks: -1.2% at
// the per-GPU size of 8 GPUs)
constexpr int kFixupGrid = 32;

// Rays per lane of the spp = 1 packet kernel: 1 (8x8 tiles, k_trace_packet)
// or 2 (16x8 tiles, k_trace_packet_r).  RT_PACKET_RAYS, read per call.
int packet_rays() {
    const char* e = getenv("RT_PACKET_RAYS");
    return e && e[0] == '2' ? 2 : 1;
}
template <int W>
int packet_blocks_per_cu_w();
// Resident workgroups per CU of k_trace_packet_r (its own register count).
int packet_r_blocks_per_cu() {
    static const int n = [] {
        int m = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &m, k_trace_packet_r<8, kPacketStack, kCandidates / 2, 2, false>, 64 * kPacketWaves, 0) != hipSuccess)
            m = 1;
        return m < 1 ? 1 : m;
    }();
    return n;
}

// Kernel choice: the packet kernel unless its stack cannot hold the tree's
// bound or RT_KERNEL=lane asks for the per-lane kernel.
bool use_packet(uint32_t stack_bound) {
    static const bool lane_forced = [] {
        const char* e = getenv("RT_KERNEL");
        return e && e[0] == 'l';
    }();
    return !lane_forced && stack_bound <= (uint32_t)kPacketStack;
}

// Pose p of a batch (its spp sample frames) as a one-pose launch (kernels
// that run per pose).
RtFrameParams single_pose(const RtFrameParams& fp, int p) {
    RtFrameParams o = fp;
    const size_t off = (size_t)p * (size_t)fp.W * (size_t)fp.nrows;  // pixels before pose p
    const size_t soff = off * (size_t)fp.spp;                         // samples before pose p
    o.nframes = fp.spp;
    o.pose[0] = fp.pose[p];
    if (o.hit_id) o.hit_id += soff;
    if (o.dist) o.dist += soff;
    if (o.hit_pos) o.hit_pos += 3 * soff;
    if (o.rgb) o.rgb += 3 * off;
    if (o.hit_count) o.hit_count += p;
    return o;
}

// Resolve placement of the packet pipeline for spp = 1: fused into the walk
// kernel's tile epilogue (default) or, with RT_RESOLVE=split, the separate
// k_resolve pass over candidate lists in HBM (the spp > 1 path; kept for
// A/B measurement).  Read per call (tests switch it in-process).
// RT_RESOLVE=split: the walk hands candidate lists to k_resolve through HBM
// (the A/B reference for the fused resolve), for any spp
bool split_resolve(int spp) {
    (void)spp;
    const char* e = getenv("RT_RESOLVE");
    return e && e[0] == 's';
}
// the packet pipeline needs the candidate buffers: the split resolve's lists,
// or spp > 1 with the fused resolve (each sample's colour and status)
// (pack: spp 4 and 16 on an 8-wide walk tree with the fused resolve — a wave
// sums a pixel's samples across its lanes, nothing goes through HBM; the
// host's fp.pack, rt_api.cpp pack_samples)
bool needs_cand(int spp, bool pack) { return (spp > 1 && !pack) || split_resolve(spp); }

template <int W>
hipError_t launch_exact(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux_in, bool count,
                        hipStream_t s, const hipEvent_t* ev) {
    const dim3 grid((unsigned)aux_in.grid), blk(256), pgrid((unsigned)aux_in.pgrid), pblk(64 * kPacketWaves);
    // aux.self_fix (the host's offer: the redo list holds every pixel of the
    // launch and the spill the packet grid's lanes) is taken by the fused
    // packet kernel when it resolves every sample itself — spp = 1 or packed
    // samples, one ray per lane: its own waves then finish the redo list and
    // the bookkeeping (packet_exit) and no k_fixup follows, so the launch
    // ends with its traversal kernel
    RtLaunchAux aux = aux_in;
    // The kernel of the launch, chosen once (every launch below follows it):
    // the fused k_trace_packet<FUSED> of spp = 1 or of packed samples is the
    // one that calls packet_exit; RT_SELF_FIX goes to that kernel only, so a
    // kernel without packet_exit (split resolve, k_trace_packet_r, the
    // per-lane kernel) always gets its trailing k_fixup.
    const bool packet = use_packet(sc.stack_bound);
    const bool packet_r = W == 8 && packet && fp.spp == 1 && !fp.pack && !aux_in.job_src && packet_rays() == 2;
    const bool fused_exit = packet && !split_resolve(fp.spp) && (fp.spp == 1 || fp.pack) && !packet_r;
    aux.self_fix = (aux_in.self_fix & RT_SELF_FIX) && fused_exit ? (aux_in.self_fix & (RT_SELF_FIX | RT_SELF_STORE)) : 0;
    // RT_SELF_STORE asked for where the kernel cannot store the counts: zero
    // them first (the launch's poses' counters, nothing else adds to them)
    if ((aux_in.self_fix & RT_SELF_STORE) && !(aux.self_fix & RT_SELF_STORE) && fp.hit_count) {
        const hipError_t e = hipMemsetAsync(fp.hit_count, 0, sizeof(unsigned long long) * (size_t)(fp.nframes / fp.spp), s);
        if (e != hipSuccess) return e;
    }
    // RT_FLAG_TIMING: two markers bracket the traversal kernel only (the
    // rest of the pipeline is timed as frame minus traversal by the caller)
    if (ev) (void)hipEventRecord(ev[0], s);
    if (packet) {
        // (aux.fgrid: the host saw this slot's redo list overflow, so a
        // retry of the whole launch is likely: the full grid)
        int fg = aux.fgrid > 0 ? aux.fgrid : kFixupGrid;
        if (const char* e = getenv("RT_FIXUP_GRID")) fg = atoi(e) > 0 ? atoi(e) : fg;  // tuning hook, read per call
        const dim3 fgrid((unsigned)(aux.grid < fg ? aux.grid : fg));
        if (!split_resolve(fp.spp)) {
            // packed samples (fp.pack, 8-wide walk trees) in their own
            // instantiation: its epilogue's registers stay out of spp = 1's
            bool packed = false;
            if constexpr (W == 8) {
                if (aux.job_src) {  // (packet_takes_job: fused, not counting, 8 x 8 tiles or packed samples)
                    packed = true;
                    if (fp.pack)
                        hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, false, true, true, true>),
                                           pgrid, pblk, 0, s, PacketArgs{sc, fp, aux});
                    else
                        hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, false, true, false, true>),
                                           pgrid, pblk, 0, s, PacketArgs{sc, fp, aux});
                } else if (fp.pack) {
                    packed = true;
                    if (count)
                        hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, true, true, true>), pgrid,
                                           pblk, 0, s, PacketArgs{sc, fp, aux});
                    else
                        hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, false, true, true>), pgrid,
                                           pblk, 0, s, PacketArgs{sc, fp, aux});
                }
            }
            if constexpr (W == 8) {
                // spp = 1: R rays per lane (RT_PACKET_RAYS, read per call)
                if (!packed && fp.spp == 1 && packet_rays() == 2) {
                    packed = true;  // (launched here)
                    const dim3 g2((unsigned)(aux.pgrid / packet_blocks_per_cu_w<8>() * packet_r_blocks_per_cu()));
                    if (count)
                        hipLaunchKernelGGL((k_trace_packet_r<8, kPacketStack, kCandidates / 2, 2, true>), g2, pblk, 0,
                                           s, PacketArgs{sc, fp, aux});
                    else
                        hipLaunchKernelGGL((k_trace_packet_r<8, kPacketStack, kCandidates / 2, 2, false>), g2, pblk,
                                           0, s, PacketArgs{sc, fp, aux});
                }
            }
            if (packed) {
            } else if (count)
                hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, true, true>), pgrid, pblk, 0, s,
                                   PacketArgs{sc, fp, aux});
            else
                hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, false, true>), pgrid, pblk, 0, s,
                                   PacketArgs{sc, fp, aux});
            if (ev) (void)hipEventRecord(ev[1], s);
            if (fp.spp > 1 && !packed) {
                const uint64_t bpf = ((uint64_t)fp.W * (uint64_t)fp.nrows + 255) / 256;
                hipLaunchKernelGGL(k_average, dim3((unsigned)(bpf * (uint64_t)(fp.nframes / fp.spp))), blk, 0, s, fp,
                                   aux);
            }
        } else {
            // k_resolve: one block per 16x16 tile, 8 XCD bands of T8 tiles per pose
            const uint64_t rt8 = (((uint64_t)(fp.W + 15) / 16) * ((uint64_t)(fp.nrows + 15) / 16) + 7) / 8;
            const dim3 rgrid((unsigned)(8 * rt8 * (uint64_t)(fp.nframes / fp.spp)));
            if (count)
                hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, true, false>), pgrid, pblk, 0, s,
                                   PacketArgs{sc, fp, aux});
            else
                hipLaunchKernelGGL((k_trace_packet<W, kPacketStack, kCandidates, false, false>), pgrid, pblk, 0, s,
                                   PacketArgs{sc, fp, aux});
            if (ev) (void)hipEventRecord(ev[1], s);
            if (count) hipLaunchKernelGGL((k_resolve<true>), rgrid, blk, 0, s, sc, fp, aux);
            else hipLaunchKernelGGL((k_resolve<false>), rgrid, blk, 0, s, sc, fp, aux);
        }
        if (aux.self_fix) {
        } else if (count)
            hipLaunchKernelGGL((k_fixup<W, kLdsStack, true>), fgrid, blk, 0, s, sc, fp, aux);
        else
            hipLaunchKernelGGL((k_fixup<W, kLdsStack, false>), fgrid, blk, 0, s, sc, fp, aux);
    } else {
        // per-lane kernel (trees deeper than the packet stack): one launch
        // per frame of the batch, each on a zeroed work queue
        for (int f = 0; f < fp.nframes / fp.spp; f++) {
            const RtFrameParams f1 = single_pose(fp, f);
            if (f > 0) {
                hipError_t e = hipMemsetAsync(aux.tile_ctr, 0, RT_QUEUE_WORDS * sizeof(uint32_t), s);
                if (e != hipSuccess) return e;
            }
            if (count) hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, true, 3>), grid, blk, 0, s, sc, f1, aux);
            else hipLaunchKernelGGL((k_trace_exact<W, kLdsStack, false, 3>), grid, blk, 0, s, sc, f1, aux);
        }
        if (ev) (void)hipEventRecord(ev[1], s);
    }
    return hipGetLastError();
}

// Resident 256-thread workgroups per CU of the per-lane persistent kernels
// (exact traversal, fix-up, paths): the larger of their occupancies.
template <int W>
int blocks_per_cu_w(uint32_t stack_bound) {
    int n = 0, m = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_trace_exact<W, kLdsStack, false, 3>, 256, 0) != hipSuccess)
        n = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, k_paths<W, kPathStack>, 256, 0) != hipSuccess) m = 1;
    int q = 0;  // (the queued segment kernel's persistent grid shares the spill columns)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, k_q_segment<W, RT_Q_STACK, RT_Q_K, false, true>, 256, 0) !=
        hipSuccess)
        q = 1;
    (void)stack_bound;
    n = n > m ? n : m;
    return n > q ? n : q;
}
template <int W>
int packet_blocks_per_cu_w() {
    int n = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &n, k_trace_packet<W, kPacketStack, kCandidates, false, true>, 64 * kPacketWaves, 0);
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
hipError_t launch_job(const RtLaunchAux& a, hipStream_t s);

// Blocks per CU the persistent exact kernel is launched with.
int exact_blocks_per_cu(int width, uint32_t stack_bound) {
    int n = width == 2   ? blocks_per_cu_w<2>(stack_bound)
            : width == 4 ? blocks_per_cu_w<4>(stack_bound)
            : width == 8 ? blocks_per_cu_w<8>(stack_bound)
                         : blocks_per_cu_w<16>(stack_bound);
    if (n < 1) n = 1;
    return n < 8 ? n : 8;
}

// Workgroups per CU of the packet kernel (64 * kPacketWaves threads each).
int packet_blocks_per_cu(int width) {
    int n = width == 2   ? packet_blocks_per_cu_w<2>()
            : width == 4 ? packet_blocks_per_cu_w<4>()
            : width == 8 ? packet_blocks_per_cu_w<8>()
                         : packet_blocks_per_cu_w<16>();
    return n < 1 ? 1 : n;
}

// the smallest LDS ring of the per-lane kernels (spill sizing)
int exact_lds_stack() {
    int a = kLdsStack < kPathStack ? kLdsStack : kPathStack;
    return a < RT_Q_STACK ? a : RT_Q_STACK;
}
int packet_threads() { return 64 * kPacketWaves; }  // threads per packet workgroup (spill columns per block)
int packet_candidates() { return RT_CAND_LDS; }  // candidate entries per pixel (spp > 1 lists; packet_exit's ring)
bool packet_split(int spp, bool pack) { return needs_cand(spp, pack); }
uint32_t params_bytes() { return (uint32_t)sizeof(RtFrameParams); }

// Host entry: validates the launch geometry against what the kernels assume
// and dispatches on node width.  mode 0 = exact fast, 1 = literal.
// ev (optional, 2 events): recorded around the traversal kernel on `s`
// (RT_FLAG_TIMING).
// fresh: the work-queue block is known to be zero (no memset needed);
// *fresh_after: whether it will be zero again once this launch completes
// (the packet pipeline clears it itself; the per-lane kernel does not).
hipError_t launch_trace_core(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, int mode,
                             bool count, hipStream_t s, uint32_t literal_stack, const hipEvent_t* ev, bool fresh,
                             bool* fresh_after);

// The kernels that take the side job (aux.job_*) themselves: the fused
// packet kernel on 8-wide trees, 8x8 tiles or packed samples, outside the
// counting pass (k_trace_packet<..., JOB = true>).  Otherwise it runs after
// the pipeline as k_deinterleave.
bool packet_takes_job(const RtDevScene& sc, const RtFrameParams& fp, int mode, bool count) {
    if (mode == 1 || count || !use_packet(sc.stack_bound) || sc.width != 8 || split_resolve(fp.spp)) return false;
    if (fp.pack) return true;
    return fp.spp == 1 && packet_rays() == 1;
}

hipError_t launch_trace(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, int mode, bool count,
                        hipStream_t s, uint32_t literal_stack, const hipEvent_t* ev, bool fresh, bool* fresh_after) {
    const bool empty = fp.W <= 0 || fp.nrows <= 0 || fp.nframes <= 0;
    const bool own = aux.job_src && (empty || !packet_takes_job(sc, fp, mode, count));
    RtLaunchAux a = aux;
    if (own) a.job_src = nullptr;
    hipError_t e = launch_trace_core(sc, fp, a, mode, count, s, literal_stack, ev, fresh, fresh_after);
    if (e == hipSuccess && own) e = launch_job(aux, s);
    return e;
}

hipError_t launch_trace_core(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, int mode,
                             bool count, hipStream_t s, uint32_t literal_stack, const hipEvent_t* ev, bool fresh,
                             bool* fresh_after) {
    *fresh_after = fresh;
    if (fp.W <= 0 || fp.nrows <= 0 || fp.nframes <= 0) return hipSuccess;
    if (fp.nframes > RT_MAX_BATCH || fp.spp < 1 || fp.nframes % fp.spp != 0 ||
        (uint64_t)fp.W * (uint64_t)fp.nrows * (uint64_t)fp.nframes >= (1ull << 31))
        return hipErrorInvalidValue;
    if (mode == 1) {
        const long tiles = (long)((fp.W + 7) / 8) * (long)((fp.nrows + 7) / 8);
        const dim3 grid((unsigned)((tiles + 3) / 4));
        if (literal_stack > 1024) return hipErrorInvalidValue;
        hipError_t e = hipSuccess;
        if ((aux.self_fix & RT_SELF_STORE) && fp.hit_count)  // (the literal kernel adds: zeroed first)
            e = hipMemsetAsync(fp.hit_count, 0, sizeof(unsigned long long) * (size_t)(fp.nframes / fp.spp), s);
        if (e != hipSuccess) return e;
        if (ev) (void)hipEventRecord(ev[0], s);
        for (int f = 0; f < fp.nframes / fp.spp && e == hipSuccess; f++) {
            const RtFrameParams f1 = single_pose(fp, f);
            e = literal_stack <= 64    ? launch_literal_s<64>(sc, f1, count, grid, s)
                : literal_stack <= 256 ? launch_literal_s<256>(sc, f1, count, grid, s)
                                       : launch_literal_s<1024>(sc, f1, count, grid, s);
        }
        if (ev) (void)hipEventRecord(ev[1], s);
        return e;
    }
    if (aux.spill_cap + kLdsStack < sc.stack_bound || !aux.tile_ctr || !aux.spill || aux.grid <= 0)
        return hipErrorInvalidValue;
    // the redo list is a fixed pool (k_fixup retries the launch whole past
    // it); the split resolve needs candidate lists for every pixel of the batch
    const uint64_t bpix = (uint64_t)fp.W * (uint64_t)fp.nrows * (uint64_t)fp.nframes;  // pixels of the batch
    if (use_packet(sc.stack_bound) && (!aux.redo || aux.redo_cap < 1 || !aux.pool || aux.pgrid <= 0))
        return hipErrorInvalidValue;
    if (use_packet(sc.stack_bound) && needs_cand(fp.spp, fp.pack && sc.width == 8) &&
        (!aux.cand || !aux.cand_cnt || !aux.cand_drop || !aux.cand_ovf || aux.cand_cap < bpix))
        return hipErrorInvalidValue;
    const bool packet = use_packet(sc.stack_bound);
    if (!fresh || !packet) {
        hipError_t e = hipMemsetAsync(aux.tile_ctr, 0, RT_QUEUE_WORDS * sizeof(uint32_t), s);  // queues, counts
        if (e != hipSuccess) return e;
    }
    *fresh_after = packet;
    switch (sc.width) {
        case 2: return launch_exact<2>(sc, fp, aux, count, s, ev);
        case 4: return launch_exact<4>(sc, fp, aux, count, s, ev);
        case 8: return launch_exact<8>(sc, fp, aux, count, s, ev);
        case 16: return launch_exact<16>(sc, fp, aux, count, s, ev);
        default: return hipErrorInvalidValue;
    }
}

// Multi-device frames: the shards gathered to the first device ([G][block]
// bytes) become full frames.  One block per image row of a frame copies the
// row's W * eb bytes from its shard (rt_gathered_row), in words when both
// sides allow it.
__global__ void __launch_bounds__(256) k_deinterleave(RtLaunchAux a) {
    const int H = a.job_H;
    const int f = (int)(blockIdx.x / (unsigned)H), j = (int)(blockIdx.x % (unsigned)H);
    if (f >= a.job_F) return;
    const uint64_t n = (uint64_t)a.job_W * a.job_eb;
    const uint8_t* src = a.job_src + rt_job_src_row(a, j, f);
    uint8_t* d = a.job_dst + ((uint64_t)f * H + j) * n;
    if (((uintptr_t)src | (uintptr_t)d | n) % 4 == 0) {
        const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
        uint32_t* d4 = reinterpret_cast<uint32_t*>(d);
        for (uint64_t k = threadIdx.x; k < n / 4; k += blockDim.x) d4[k] = s4[k];
    } else {
        for (uint64_t k = threadIdx.x; k < n; k += blockDim.x) d[k] = src[k];
    }
}

// The overlap gate (rt_api.cpp launch): one wave that asks for 32 VGPRs per
// lane and does nothing.  Issued on a stream right before a persistent
// traversal grid while another stream's grid may still hold the device, it
// cannot start until a wave of that grid has exited (7 traversal waves per
// SIMD leave 8 of the 512 VGPRs free), so the new grid is dispatched into the
// other one's tail instead of beside all of it (two whole
// persistent grids resident at once on two queues slowed the device 4-70x in
// most runs).
__global__ void __launch_bounds__(64) k_gate() { asm volatile("v_mov_b32 v31, 0" ::: "v31"); }

// Per-frame hit counts of the G shards (u64 [F] at cnt_off of each block) added
// to the caller's counters (store: written over them, RT_FLAG_COUNTS_STORE).
__global__ void k_sum_counts(const uint8_t* __restrict__ gather, uint64_t block, uint64_t cnt_off, int G, int F,
                             unsigned long long* __restrict__ out, int store) {
    const int f = (int)threadIdx.x;
    if (f >= F) return;
    unsigned long long t = 0;
    for (int g = 0; g < G; g++) t += reinterpret_cast<const unsigned long long*>(gather + g * block + cnt_off)[f];
    out[f] = store ? t : out[f] + t;
}

hipError_t launch_deinterleave(const void* gather, uint64_t block, uint64_t sec_off, int G, int F, int H, int W,
                               int eb, void* dst, hipStream_t s) {
    RtLaunchAux a{};
    a.job_src = (decltype(a.job_src))gather;
    a.job_dst = (decltype(a.job_dst))dst;
    a.job_block = block;
    a.job_sec = sec_off;
    a.job_G = G;
    a.job_F = F;
    a.job_H = H;
    a.job_W = W;
    a.job_eb = eb;
    a.job_rows = 0;
    return launch_job(a, s);
}

// A side job on its own (the pipelines whose kernel does not take it).
hipError_t launch_job(const RtLaunchAux& a, hipStream_t s) {
    if (!a.job_src || a.job_F <= 0 || a.job_H <= 0 || a.job_W <= 0 || a.job_G <= 0 || a.job_eb <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_deinterleave, dim3((unsigned)((uint64_t)a.job_F * a.job_H)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gate(hipStream_t s) {
    hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s);
    return hipGetLastError();
}

hipError_t launch_sum_counts(const void* gather, uint64_t block, uint64_t cnt_off, int G, int F,
                             unsigned long long* out, bool store, hipStream_t s) {
    if (F <= 0 || F > 1024) return F <= 0 ? hipSuccess : hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sum_counts, dim3(1), dim3(1024), 0, s, static_cast<const uint8_t*>(gather), block, cnt_off,
                       G, F, out, store ? 1 : 0);
    return hipGetLastError();
}

// Packed primary path segments through the wave walk: 8-wide trees whose
// stack bound fits a wave's 128-entry stack (RT_PATHS_PRIMARY=0: per lane;
// read per call).
bool paths_primary_wave(const RtDevScene& sc) {
    const char* e = getenv("RT_PATHS_PRIMARY");
    if (e && e[0] == '0') return false;
    return RT_PATHS_PRIM && RT_PATHS_DEFER && sc.width == 8 && sc.stack_bound <= (uint32_t)kPacketStack;
}

// Diffuse path tracing of one pose (path_kernel.h): spp paths per pixel of
// 1 + bounces segments each, on a zeroed work queue; leaves it dirty.
// shadow: occlusion rays toward the head-light at the bounce vertices.
template <int W, bool COUNT = false, bool PACK = false, bool PRIM = false>
void launch_k_paths(dim3 grid, dim3 blk, hipStream_t s, const RtDevScene& sc, const RtFrameParams& fp,
                    const RtLaunchAux& aux, uint32_t frame, int bounces, bool shadow) {
    if (shadow)
        hipLaunchKernelGGL((k_paths<W, kPathStack, COUNT, PACK, PRIM, true>), grid, blk, 0, s, sc, fp, aux, frame,
                           bounces);
    else
        hipLaunchKernelGGL((k_paths<W, kPathStack, COUNT, PACK, PRIM, false>), grid, blk, 0, s, sc, fp, aux, frame,
                           bounces);
}
hipError_t launch_paths(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, uint32_t frame,
                        int bounces, bool shadow, hipStream_t s, const hipEvent_t* ev) {
    if (fp.W <= 0 || fp.nrows <= 0) return hipSuccess;
    if (fp.nframes != 1 || fp.spp < 1 || bounces < 0 || bounces > 64 || !aux.tile_ctr || !aux.spill || aux.grid <= 0 ||
        aux.spill_cap + kPathStack < sc.stack_bound)
        return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(aux.tile_ctr, 0, RT_QUEUE_WORDS * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)aux.grid), blk(256);
    if (ev) (void)hipEventRecord(ev[0], s);
    switch (sc.width) {
        case 2: launch_k_paths<2>(grid, blk, s, sc, fp, aux, frame, bounces, shadow); break;
        case 4: launch_k_paths<4>(grid, blk, s, sc, fp, aux, frame, bounces, shadow); break;
        case 8:
            // (fp.pack: a wave holds every sample of 64 / spp pixels)
            if (fp.pack && paths_primary_wave(sc)) {  // primary segments by the wave walk (path_kernel.h)
                if (fp.counters)
                    launch_k_paths<8, true, true, true>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
                else
                    launch_k_paths<8, false, true, true>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
            } else if (fp.counters && fp.pack)  // the counting pass: fetch counts too
                launch_k_paths<8, true, true>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
            else if (fp.counters)
                launch_k_paths<8, true>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
            else if (fp.pack)
                launch_k_paths<8, false, true>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
            else
                launch_k_paths<8>(grid, blk, s, sc, fp, aux, frame, bounces, shadow);
            break;
        case 16: launch_k_paths<16>(grid, blk, s, sc, fp, aux, frame, bounces, shadow); break;
        default: return hipErrorInvalidValue;
    }
    if (ev) (void)hipEventRecord(ev[1], s);
    return hipGetLastError();
}

// Queued path tracing of one pose (queue_paths.h): the primary segments of
// every path, then per bounce segment the compacted queue and its fall-back
// list, then the pixel sums.  The control words are zeroed here.
// A persistent grid of `kernel` (256-thread workgroups) filling every CU to
// its occupancy (the query, once per process per kernel: every device of a
// run is a gfx950).
template <class K>
dim3 occupancy_grid(K kernel) {
    int dev = 0, cus = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, 256, 0) != hipSuccess || n < 1) n = 1;
    return dim3((unsigned)(cus * n));
}
template <int W, bool COUNT, int SH>
void launch_q_segment(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, const PathQs& qs,
                      uint32_t frame, int b, int bounces, hipStream_t s) {
    const dim3 grid((unsigned)aux.grid), blk(256), fgrid(64);
    hipLaunchKernelGGL((k_q_segment<W, RT_Q_STACK, RT_Q_K, COUNT, SH>), grid, blk, 0, s, sc, fp, aux, qs, frame, b,
                       bounces);
    hipLaunchKernelGGL((k_q_fallback<W, kLdsStack, COUNT, SH>), fgrid, blk, 0, s, sc, fp, aux, qs, frame, b, bounces);
    if constexpr (SH == 3)  // the records in emission order, per lane
        hipLaunchKernelGGL((k_sh_lane<W, RT_Q_STACK, COUNT>), grid, blk, 0, s, sc, fp, aux, qs, b);
    if constexpr (SH == 2) {
        // the segment's occlusion records: binned by direction from the light,
        // then walked 64 at a time by the wave-cooperative any-hit walk
        // (RT_SH_BITS bits per pass, lowest digit first; ping-pong between
        // the two pair arrays)
        constexpr int passes = (RT_SH_KEY_BITS + RT_SH_BITS - 1) / RT_SH_BITS;
        for (int pass = 0; pass < passes; pass++) {
            const int shift = pass * RT_SH_BITS;
            hipLaunchKernelGGL(k_sh_hist<RT_SH_BITS>, dim3(RT_SH_BLOCKS), dim3(1024), 0, s, qs, b, pass, shift);
            hipLaunchKernelGGL(k_sh_scan<RT_SH_BITS>, dim3(1), dim3(1024), 0, s, qs);
            hipLaunchKernelGGL(k_sh_scatter<RT_SH_BITS>, dim3(RT_SH_BLOCKS), dim3(1024), 0, s, qs, b, pass, shift);
        }
        static const dim3 wgrid = occupancy_grid(k_sh_walk<W, COUNT>);
        hipLaunchKernelGGL((k_sh_walk<W, COUNT>), wgrid, blk, 0, s, sc, fp, aux, qs, b, (passes - 1) & 1);
    }
}
// sh: 0 no occlusion rays, 1 per lane in the segment kernel, 2 queued and binned
template <int W>
void launch_q_segments(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, const PathQs& qs,
                       uint32_t frame, int bounces, int sh, bool count, hipStream_t s) {
    // the primary segments' fall-back rays (segment 0; no occlusion rays there)
    if (W == 8 && count)
        hipLaunchKernelGGL((k_q_fallback<W, kLdsStack, true, 0>), dim3(64), dim3(256), 0, s, sc, fp, aux, qs, frame, 0,
                           bounces);
    else
        hipLaunchKernelGGL((k_q_fallback<W, kLdsStack, false, 0>), dim3(64), dim3(256), 0, s, sc, fp, aux, qs, frame, 0,
                           bounces);
    for (int b = 1; b <= bounces; b++) {
        if (W == 8 && count) {
            if (sh == 3) launch_q_segment<W, true, 3>(sc, fp, aux, qs, frame, b, bounces, s);
            else if (sh == 2) launch_q_segment<W, true, 2>(sc, fp, aux, qs, frame, b, bounces, s);
            else if (sh == 1) launch_q_segment<W, true, 1>(sc, fp, aux, qs, frame, b, bounces, s);
            else launch_q_segment<W, true, 0>(sc, fp, aux, qs, frame, b, bounces, s);
        } else {
            if (sh == 3) launch_q_segment<W, false, 3>(sc, fp, aux, qs, frame, b, bounces, s);
            else if (sh == 2) launch_q_segment<W, false, 2>(sc, fp, aux, qs, frame, b, bounces, s);
            else if (sh == 1) launch_q_segment<W, false, 1>(sc, fp, aux, qs, frame, b, bounces, s);
            else launch_q_segment<W, false, 0>(sc, fp, aux, qs, frame, b, bounces, s);
        }
    }
}

// Occlusion rays of the queued pipeline (RT_SHADOW_RAYS, read per call):
// "bin" (default): queued, sorted by direction from the light and walked by
// the wave (k_sh_walk; its wave stack holds kPacketStack entries, deeper
// trees stay per lane); "lane": walked per lane inside the segment kernel
// where the vertex is shaded; "rec": queued as records, walked per lane in
// emission order by k_sh_lane.  Config c5 with partitioned counters: 201.0 /
// 220.5 / 216.7 ms per pose (round 4, one counter per queue: 266 / 233 / 237).
// A queued record names its destination in one word (q_light: bit 31, the
// queue in bit 30, the slot in bits 0-29), so pools of 2^30 paths or more
// stay per lane too.
int queued_shadow_mode(const RtDevScene& sc, bool shadow, uint64_t paths) {
    if (!shadow) return 0;
    const char* e = getenv("RT_SHADOW_RAYS");
    if (paths >= (1ull << 30)) return 1;
    if (e && e[0] == 'r') return 3;
    if (e && e[0] == 'l') return 1;
    return sc.stack_bound > (uint32_t)kPacketStack ? 1 : 2;
}

// Packed primary segments of the queued pipeline through the packet kernel
// (RT_QP_PACKET=0: k_q_primary's wave walk; read per call): every sample of
// a pose fits one launch (spp <= RT_MAX_BATCH) and the launch state is there.
bool packet_primaries(const RtFrameParams& fp, const RtLaunchAux& aux) {
    const char* e = getenv("RT_QP_PACKET");
    if (e && e[0] == '0') return false;
    // (the packed tile is (8 / n) x (8 / n) pixels of spp = n x n samples)
    const bool square = fp.spp == 4 || fp.spp == 16;
    return square && fp.spp <= RT_MAX_BATCH && aux.tile_ctr && aux.pool && aux.pgrid > 0;
}

hipError_t launch_paths_q(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, const PathQs& qs_,
                          uint32_t frame, int bounces, bool shadow, hipStream_t s, const hipEvent_t* ev) {
    if (fp.W <= 0 || fp.nrows <= 0) return hipSuccess;
    // one partition, or RT_QPARTS when the packet kernel deals the primaries
    // (its tiles' XCD queues: PathQs)
    PathQs qs = qs_;
    qs.parts = 1;
    qs.pcap = qs.cap;
    qs.ptile = qs.ptiles_x = 1;
    const bool qpacket = sc.width == 8 && fp.pack && paths_primary_wave(sc) && packet_primaries(fp, aux);
    if (qpacket) {
        const RtQParts p = rt_qparts(fp.W, fp.nrows, fp.spp);
        if (p.entries > qs.cap) return hipErrorInvalidValue;
        qs.parts = RT_QPARTS;
        qs.pcap = p.pcap;
        qs.ptile = p.ptile;
        qs.ptiles_x = p.ptiles_x;
    }
    const uint64_t paths = (uint64_t)fp.W * (uint64_t)fp.nrows * (uint64_t)fp.spp;
    if (fp.nframes != 1 || fp.spp < 1 || bounces < 0 || bounces > 64 || !aux.spill || aux.grid <= 0 || !qs.ctl ||
        paths > qs.cap || aux.spill_cap + RT_Q_STACK < sc.stack_bound || aux.spill_cap + kPathStack < sc.stack_bound ||
        aux.spill_cap + kLdsStack < sc.stack_bound)
        return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(qs.ctl, 0, RT_QC_WORDS(bounces) * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const bool count = fp.counters != nullptr;
    // (a queued record's destination names a queue slot: < parts * pcap)
    const int sh = queued_shadow_mode(sc, shadow, std::max(paths, (uint64_t)qs.parts * qs.pcap));
    if (sh == 2 && (!qs.srec || !qs.bhist || aux.pgrid <= 0)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)aux.grid), blk(256), agrid((unsigned)((fp.W * (uint64_t)fp.nrows + 255) / 256));
    // the wave-walked primary kernel uses no per-lane stack (no spill
    // columns): its own occupancy's grid
    static const dim3 pgrid = occupancy_grid(k_q_primary<8, 1, false, true, true>);
    if (ev) (void)hipEventRecord(ev[0], s);
    switch (sc.width) {
        case 2:
            hipLaunchKernelGGL((k_q_primary<2, kPathStack, false, false, false>), grid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            launch_q_segments<2>(sc, fp, aux, qs, frame, bounces, sh, false, s);
            break;
        case 4:
            hipLaunchKernelGGL((k_q_primary<4, kPathStack, false, false, false>), grid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            launch_q_segments<4>(sc, fp, aux, qs, frame, bounces, sh, false, s);
            break;
        case 8:
            if (qpacket) {
                // the packed packet walk (k_trace_packet<…, PATHS>): the
                // headline kernel's walk and resolve, the path's primary
                // vertex as its epilogue (queue_paths.h q_primary_vertex);
                // one pose of spp sample frames, its work-queue block zeroed
                // here and left zeroed by the kernel's exit (packet_exit)
                RtFrameParams fq = fp;
                fq.nframes = fp.spp;
                fq.spp_n = fp.spp == 16 ? 4 : 2;
                RtLaunchAux aq = aux;
                aq.self_fix = 1;
                aq.job_src = nullptr;
                e = hipMemsetAsync(aux.tile_ctr, 0, RT_QUEUE_WORDS * sizeof(uint32_t), s);
                if (e != hipSuccess) return e;
                const dim3 qgrid((unsigned)aux.pgrid), qblk(64 * kPacketWaves);
                if (count)
                    hipLaunchKernelGGL((k_trace_packet<8, kPacketStack, kCandidates, true, true, true, false, true>), qgrid,
                                       qblk, 0, s, PacketArgs{sc, fq, aq, qs, frame, bounces});
                else
                    hipLaunchKernelGGL((k_trace_packet<8, kPacketStack, kCandidates, false, true, true, false, true>),
                                       qgrid, qblk, 0, s, PacketArgs{sc, fq, aq, qs, frame, bounces});
            } else if (fp.pack && paths_primary_wave(sc)) {
                if (count)
                    hipLaunchKernelGGL((k_q_primary<8, 1, true, true, true>), pgrid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
                else
                    hipLaunchKernelGGL((k_q_primary<8, 1, false, true, true>), pgrid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            } else if (paths_primary_wave(sc)) {
                if (count)
                    hipLaunchKernelGGL((k_q_primary<8, 1, true, false, true>), pgrid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
                else
                    hipLaunchKernelGGL((k_q_primary<8, 1, false, false, true>), pgrid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            } else if (fp.pack) {
                hipLaunchKernelGGL((k_q_primary<8, kPathStack, false, true, false>), grid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            } else {
                hipLaunchKernelGGL((k_q_primary<8, kPathStack, false, false, false>), grid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            }
            launch_q_segments<8>(sc, fp, aux, qs, frame, bounces, sh, count, s);
            break;
        case 16:
            hipLaunchKernelGGL((k_q_primary<16, kPathStack, false, false, false>), grid, blk, 0, s, sc, fp, aux, qs, frame, bounces);
            launch_q_segments<16>(sc, fp, aux, qs, frame, bounces, sh, false, s);
            break;
        default:
            return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k_q_accum, agrid, blk, 0, s, fp, qs);
    if (ev) (void)hipEventRecord(ev[1], s);
    return hipGetLastError();
}

}  // namespace rt
