// Wave-cooperative ("packet") exact traversal kernel for gfx950.
// Included by render.hip inside its anonymous namespace (uses Ray32, Win,
// make_ray32 and the rtk helpers).
//
// The 64 rays of one 8x8 pixel tile walk the tree together.  The current
// node is wave-uniform, so its child records come in through the scalar data
// path (s_load_dwordx8 per 32-B child, once per wave) instead of 64 per-lane
// copies through the vector memory pipe; every lane slab-tests its own ray
// against each child and `ballot` says whether any lane needs the child.  The
// wave continues into the hit child nearest to the first lane that hit it and
// pushes the others on a wave-uniform stack of node refs in LDS.
//
// No per-child lane masks are kept: all lanes of a wave execute every child
// test anyway, and a lane that missed a parent box misses its children too
// (real child boxes lie inside the parent box and outward rounding to fp32 is
// monotone), so re-testing with every lane returns the same answers.  Lanes
// that take no part in a pass carry tcull = -1, which fails every test.
//
// Leaves: uniform triangle records, a conservative per-lane fp32 pre-filter,
// the exact fp64 Moller-Trumbore only for lanes it cannot reject.  Each lane's
// fp64 ray (o, d, 1/d) lives in LDS.  Exactness machinery as trace_exact.
#pragma once

struct __attribute__((aligned(32))) ChildRec {  // 32-B child record (rt_device.h)
    float lx, hx, ly, hy, lz, hz;
    uint32_t ref, pad;
};
typedef const __attribute__((address_space(4))) float* cfloat_p;
typedef const __attribute__((address_space(4))) ChildRec* cchild_p;

// Field-wise reads through the constant address space: adjacent uniform loads
// merge into one s_load_dwordx8 (child) / s_load_dwordx4 runs (triangle).
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

// Per-lane fp64 ray in LDS: component k of lane l at ray[k * 64 + l]
// (consecutive lanes -> consecutive 8-B words, conflict-free ds_read_b64).
__device__ __forceinline__ void store_ray(double* __restrict__ ray_lds, int lane, const Ray64& r) {
    ray_lds[0 * 64 + lane] = r.ox;
    ray_lds[1 * 64 + lane] = r.oy;
    ray_lds[2 * 64 + lane] = r.oz;
    ray_lds[3 * 64 + lane] = r.dx;
    ray_lds[4 * 64 + lane] = r.dy;
    ray_lds[5 * 64 + lane] = r.dz;
    ray_lds[6 * 64 + lane] = r.ix;
    ray_lds[7 * 64 + lane] = r.iy;
    ray_lds[8 * 64 + lane] = r.iz;
}
__device__ __forceinline__ Ray64 load_ray(const double* __restrict__ ray_lds, int lane) {
    lane = opaque(lane);  // no store-to-load forwarding: the ray must stay in LDS, not VGPRs
    Ray64 r;
    r.ox = ray_lds[0 * 64 + lane];
    r.oy = ray_lds[1 * 64 + lane];
    r.oz = ray_lds[2 * 64 + lane];
    r.dx = ray_lds[3 * 64 + lane];
    r.dy = ray_lds[4 * 64 + lane];
    r.dz = ray_lds[5 * 64 + lane];
    r.ix = ray_lds[6 * 64 + lane];
    r.iy = ray_lds[7 * 64 + lane];
    r.iz = ray_lds[8 * 64 + lane];
    return r;
}

template <int W, int SP, bool COUNT>
__device__ __forceinline__ void trace_packet(const RtDevScene& sc, const RtFrameParams& fp, int i, int r, bool valid,
                                             uint32_t* __restrict__ wstack, double* __restrict__ ray_lds) {
    constexpr int G = W < 4 ? W : 4;  // children per scalar load group
    const int lane = threadIdx.x & 63;
    if (!valid) { i = 0; r = 0; }
    const int j = fp.row0 + r * fp.row_stride;
    Ray32 q;
    double tslack;
    {
        const Ray64 ray = gen_ray(fp, i, j);
        store_ray(ray_lds, lane, ray);
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
    uint32_t w_nodes = 0, w_leaves = 0;  // wave-level visits (COUNT only)
    bool mine = valid;                   // this lane takes part in the pass
    for (int pass = 0; pass < 2; pass++) {
        if (__ballot(mine) == 0) break;
        if (mine) {
            best.dist = 1.7976931348623157e308;
            best.t = 0.0;
            best.rank = 0xFFFFFFFFu;
            best.tri = -1;
        }
        float tcull = mine ? __builtin_huge_valf() : -1.f;
        uint32_t chain_leaf = 0xFFFFFFFFu;
        bool chain_res = false;
        uint32_t cur = sc.root_ref;
        {
            const float* b = sc.root_box;
            const float t0 = fmaxf(fmaxf(fminf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                         fminf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                                   fmaxf(fminf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)), 0.f));
            const float t1 = fminf(fminf(fmaxf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                         fmaxf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                                   fminf(fmaxf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)), tcull));
            if (__ballot(t0 <= t1) == 0) cur = RT_INVALID_REF;
        }
        int sp = 0;
        for (;;) {
            if (cur != RT_INVALID_REF) {
                if (!(cur & RT_LEAF_BIT)) {
                    if (COUNT) {
                        w_nodes++;
                        n_nodes += mine;
                    }
                    const cchild_p nb = (cchild_p)(sc.nodes + (size_t)cur * (32 * W));
                    uint32_t near_ref = RT_INVALID_REF, near_key = 0xFFFFFFFFu;
#pragma unroll
                    for (int g = 0; g < W; g += G) {
                        __builtin_amdgcn_sched_barrier(0);  // bound the SGPRs of in-flight child records
#pragma unroll
                        for (int c = g; c < g + G; c++) {
                            const ChildRec ch = load_child(nb + c);
                            const float tlx = __builtin_fmaf(ch.lx, q.ix, -olx);
                            const float thx = __builtin_fmaf(ch.hx, q.ix, -ohx);
                            const float tly = __builtin_fmaf(ch.ly, q.iy, -oly);
                            const float thy = __builtin_fmaf(ch.hy, q.iy, -ohy);
                            const float tlz = __builtin_fmaf(ch.lz, q.iz, -olz);
                            const float thz = __builtin_fmaf(ch.hz, q.iz, -ohz);
                            const float t0 =
                                fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
                            const float t1 =
                                fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull));
                            const uint64_t hm = __ballot(t0 <= t1);
                            if (hm != 0 && ch.ref != RT_INVALID_REF) {
                                // entry distance (>= 0, so its bits order like the
                                // value) of the first lane that hit the child
                                const uint32_t key = (uint32_t)__builtin_amdgcn_readlane(
                                    (int)__float_as_uint(t0), (int)__builtin_ctzll(hm));
                                uint32_t push = ch.ref;
                                if (key < near_key) {
                                    push = near_ref;
                                    near_ref = ch.ref;
                                    near_key = key;
                                }
                                if (push != RT_INVALID_REF) {
                                    if (lane == 0) wstack[sp] = push;
                                    sp++;
                                }
                            }
                        }
                    }
                    if (near_ref != RT_INVALID_REF) {
                        cur = near_ref;
                        continue;
                    }
                } else {
                    const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                    const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                    if (COUNT) w_leaves++;
                    for (uint32_t k = first; k < first + cnt; k++) {
                        const cfloat_p R = (cfloat_p)(sc.tri32 + 12 * (size_t)k);  // scalar loads
                        const float4 A = load_f4(R), B = load_f4(R + 4), Cc = load_f4(R + 8);
                        if (COUNT) n_pre += mine;
                        const bool pre =
                            mine && tri_prefilter(A, B, Cc, q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull);
                        if (__ballot(pre) == 0) continue;
                        if (!pre) continue;
                        if (COUNT) n_tris++;
                        const Ray64 ray = load_ray(ray_lds, lane);
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
            cur = uni(wstack[sp]);
        }
        if (pass == 1) break;
        // deferred re-verification of each lane's winner
        bool redo = false;
        if (mine && best.tri >= 0) {
            const Ray64 ray = load_ray(ray_lds, lane);
            double hx, hy, hz;
            (void)hit_dist(ray, best.t, hx, hy, hz);
            const uint32_t leaf =
                reinterpret_cast<const uint2*>(sc.tri64 + RT_TRI64_DOUBLES * (size_t)best.tri + 9)->y;
            if (COUNT) n_chain++;
            redo = !chain_fast_ok(sc.rbox + 6 * (size_t)leaf, ray, hx, hy, hz) &&
                   !chain_ok(sc, leaf, ray, n_chain_nodes);
        }
        mine = redo;
    }
    if (COUNT && fp.counters && lane == 0) {
        atomicAdd(&fp.counters[7], (unsigned long long)w_nodes);
        atomicAdd(&fp.counters[8], (unsigned long long)w_leaves);
        atomicAdd(&fp.counters[9], 1ull);
    }
    if (!valid) return;
    Best out;
    out.dist = best.dist;
    out.rank = best.rank;
    out.tri = best.tri;
    out.px = out.py = out.pz = 0.0;
    if (best.tri >= 0) {
        const Ray64 ray = load_ray(ray_lds, lane);
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

// Persistent waves over 8x8 tiles; the stack bound of the tree must fit SP
// (the host falls back to the per-lane kernel otherwise), so no push can drop.
template <int W, int SP, bool COUNT>
__global__ void __launch_bounds__(256) k_trace_packet(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint32_t stacks[4][SP];
    __shared__ double rays[4][9 * 64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int tiles_x = (fp.W + 7) >> 3;
    const int tiles = tiles_x * ((fp.nrows + 7) >> 3);
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = (int)atomicAdd(aux.tile_ctr, 1u);
        tile = __shfl(tile, 0);
        if (tile >= tiles) break;
        const int i = (tile % tiles_x) * 8 + (lane & 7);
        const int r = (tile / tiles_x) * 8 + (lane >> 3);
        trace_packet<W, SP, COUNT>(sc, fp, i, r, i < fp.W && r < fp.nrows, stacks[wv], rays[wv]);
    }
}
