// Wavefront diffuse path tracing (config c5): the path model of
// path_kernel.h, one kernel per stage instead of one
// megakernel, so the divergent stages stop sharing registers and waves.
// Included by render.hip after path_kernel.h.
//
// Per pose, for sample s = 0 .. spp-1 in order, and segment b = 0 .. bounces:
//   k_pw_walk   persistent waves take rays 64 at a time from the segment's
//               queue (b = 0: every pixel's primary ray, generated in-kernel);
//               each lane walks its ray in fp32 only (lane_walk: ~75 VGPRs,
//               7 waves/SIMD where the megakernel holds 4) and hands its
//               surviving candidates to HBM ({triangle, t bound} x <= K at
//               cand[c * P + slot], count at cand_cnt[slot], 0xFF = overflow);
//   k_pw_shade  one ray per lane: the exact fp64 resolve of the candidates
//               (resolve_cands, the reference's closest hit; overflow or an
//               invisible winner: trace_core, as in trace_deferred), the
//               primary segment's per-sample outputs, the vertex colour added
//               to the path's radiance L, and — for a hit with bounces left —
//               the bounce ray appended to the next segment's queue
//               (compacted: one atomic per wave, finished paths drop out);
//   k_pw_accum  acc += L per pixel (sample order), the colour at the last sample.
// Every fp64 expression is the megakernel's, in the same order, so the
// outputs are bit-identical to k_paths and to the oracle (orc_render_paths).
#pragma once

#ifndef RT_PW_K
#define RT_PW_K 8  // LDS candidates per lane in k_pw_walk
#endif
#ifndef RT_PW_STACK
#define RT_PW_STACK 8  // LDS stack ring entries per lane in k_pw_walk
#endif

// Sample s's primary ray of shard pixel idx (k_paths' ray, path_kernel.h).
__device__ __forceinline__ Ray64 pw_primary(const RtFrameParams& fp, uint32_t frame, uint32_t idx, uint32_t s,
                                            uint32_t& seed) {
    const int i = (int)(idx % (uint32_t)fp.W), r = (int)(idx / (uint32_t)fp.W);
    const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, r);
    seed = path_seed(frame, (uint32_t)j * (uint32_t)fp.W + (uint32_t)i, s);
    RtFrameCam c1 = frame_cam(fp, 0);
    c1.ox = path_u(seed, 0);
    c1.oy = path_u(seed, 1);
    return gen_ray<false>(fp, c1, i, j);
}

// Segment b's ray in queue slot idx, and the path (shard pixel) it belongs to.
__device__ __forceinline__ Ray64 pw_ray(const RtFrameParams& fp, const PathWs& ws, uint32_t frame, int b, uint32_t s,
                                        uint32_t idx, uint32_t& path) {
    if (b == 0) {
        uint32_t seed;
        path = idx;
        return pw_primary(fp, frame, idx, s, seed);
    }
    const RT_G double* e = ws.qray[b & 1] + 8 * (size_t)idx;
    Ray64 r;
    r.ox = e[0];
    r.oy = e[1];
    r.oz = e[2];
    r.dx = e[3];
    r.dy = e[4];
    r.dz = e[5];
    r.ix = r.iy = r.iz = 0.0;
    path = (uint32_t)__double_as_longlong(e[6]);
    return r;
}

template <int W, int S, int K>
__global__ void __launch_bounds__(256) k_pw_walk(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, PathWs ws, int b,
                                                 uint32_t s, uint32_t frame) {
    __shared__ uint2 lds[S][256];
    __shared__ uint2 cand[K][256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // the next stage's queue count (walk b and shade b - 1 are done with it)
    if (blockIdx.x == 0 && tid == 0) ws.ctl[(b + 1) & 1] = 0;
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const uint32_t n = b == 0 ? ws.P : ws.ctl[b & 1];
    const size_t P = ws.P;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(ws.ctl + 2, 64u);
        base = (uint32_t)__shfl((int)base, 0);
        if (base >= n) break;
        const uint32_t idx = base + (uint32_t)lane;
        if (idx >= n) continue;
        uint32_t path;
        const Ray64 ray = with_inv(pw_ray(fp, ws, frame, b, s, idx, path));
        const Ray32 q = make_ray32(ray, ray_pad(sc, ray));
        const float tsl = round_up_f(0x1p-40 * ((double)q.co + 1.0));
        LaneCounts lc;
        float tcull;
        int nc;
        bool over;
        lane_walk<W, S, K, false, W == 8 && RT_QNODES>(sc, q, tsl, st, cand, lc, tcull, nc, over);
        uint32_t m = 0;
        if (!over) {
            for (int c = 0; c < nc; c++) {
                const uint2 e = cand[c][tid];
                if (__uint_as_float(e.y) > tcull) continue;  // cannot beat a certain hit
                reinterpret_cast<RT_G uint2*>(aux.cand)[(size_t)m * P + idx] = e;
                m++;
            }
        }
        aux.cand_cnt[idx] = over ? (uint8_t)0xFF : (uint8_t)m;
    }
}

template <int W, int S>
__global__ void __launch_bounds__(256) k_pw_shade(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, PathWs ws, int b,
                                                  int bounces, uint32_t s, uint32_t frame) {
    __shared__ uint2 lds[S][256];  // trace_core's stack (fallback only)
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // walk b + 1 starts its cursor from zero (walk b is done with it)
    if (blockIdx.x == 0 && tid == 0) ws.ctl[2] = 0;
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const uint32_t n = b == 0 ? ws.P : ws.ctl[b & 1];
    const size_t P = ws.P;
    const RtFrameCam cam = frame_cam(fp, 0);
    const double w = __builtin_ldexp(1.0, -b);  // 0.5^b: k_paths' repeated halving, exactly
    const uint32_t stride = gridDim.x * 256u;
    // every lane of a wave runs the same number of iterations (ballots below)
    const uint32_t iters = (n + stride - 1) / stride;
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t idx = it * stride + blockIdx.x * 256u + (uint32_t)tid;
        const bool act = idx < n;
        bool emit = false;
        double nox = 0.0, noy = 0.0, noz = 0.0, ndx = 0.0, ndy = 0.0, ndz = 0.0;
        uint32_t path = 0;
        bool hit = false;
        if (act) {
            const Ray64 ray = pw_ray(fp, ws, frame, b, s, idx, path);
            auto ray_of = [&]() { return with_inv(ray); };
            const uint32_t cnt = aux.cand_cnt[idx];
            LaneCounts lc;
            Win win;
            if (cnt == 0xFFu) {
                win = trace_core<W, S, false>(sc, ray_of, ray_pad(sc, ray), st, 0, lc);
            } else if (resolve_cands<false>(
                           sc, ray_of(),
                           [&](int c) { return reinterpret_cast<const RT_G uint2*>(aux.cand)[(size_t)c * P + idx]; },
                           (int)cnt, __builtin_huge_valf(), win, lc) != 0) {
                win = trace_core<W, S, false>(sc, ray_of, ray_pad(sc, ray), st, 1, lc);
            }
            Best hb;
            hb.dist = win.dist;
            hb.rank = win.rank;
            hb.tri = win.tri;
            hb.px = hb.py = hb.pz = 0.0;
            if (win.tri >= 0) (void)hit_dist(ray, win.t, hb.px, hb.py, hb.pz);  // (uses o, d only)
            const Shade sh = shade_of(sc, win.tri);
            hit = win.tri >= 0;
            if (b == 0) store_sample(fp, (size_t)path * (size_t)fp.spp + s, hb, sh);  // path = shard pixel
            RT_G double* Lp = ws.L + 3 * (size_t)path;
            if (hit) {
                double c[3];
                shade_at(cam, hb.px, hb.py, hb.pz, sh.nx, sh.ny, sh.nz, c);
                const double l0 = b == 0 ? 0.0 : Lp[0], l1 = b == 0 ? 0.0 : Lp[1], l2 = b == 0 ? 0.0 : Lp[2];
                Lp[0] = l0 + w * c[0];
                Lp[1] = l1 + w * c[1];
                Lp[2] = l2 + w * c[2];
                if (b < bounces) {
                    uint32_t seed;
                    (void)pw_primary(fp, frame, path, s, seed);  // the path's hash seed (folds to the seed)
                    bounce_dir(sh.nx, sh.ny, sh.nz, ray.dx, ray.dy, ray.dz, path_u(seed, 2u + 2u * (uint32_t)b),
                               path_u(seed, 3u + 2u * (uint32_t)b), ndx, ndy, ndz);
                    nox = hb.px;
                    noy = hb.py;
                    noz = hb.pz;
                    emit = true;
                }
            } else if (b == 0) {
                Lp[0] = 0.0;
                Lp[1] = 0.0;
                Lp[2] = 0.0;
            }
        }
        // append the bounce rays to the next queue: one atomic per wave
        const uint64_t em = __ballot(emit);
        if (emit) {
            const int leader = __builtin_ctzll(em);
            uint32_t qb = 0;
            if (lane == leader) qb = atomicAdd(ws.ctl + ((b + 1) & 1), (uint32_t)__builtin_popcountll(em));
            qb = (uint32_t)__builtin_amdgcn_readlane((int)qb, leader);
            const uint32_t slot = qb + (uint32_t)__builtin_popcountll(em & ((1ull << lane) - 1ull));
            RT_G double* e = ws.qray[(b + 1) & 1] + 8 * (size_t)slot;
            e[0] = nox;
            e[1] = noy;
            e[2] = noz;
            e[3] = ndx;
            e[4] = ndy;
            e[5] = ndz;
            e[6] = __longlong_as_double((long long)path);
        }
        if (b == 0) wave_add<1>(fp.hit_count, hit ? 1u : 0u);
        if (fp.counters) wave_add<1>(fp.counters, act ? 1u : 0u);
    }
}

// acc = acc + L per pixel in sample order (k_paths' sum from 0.0); the pixel
// colour after the last sample.
__global__ void __launch_bounds__(256) k_pw_accum(RtFrameParams fp, PathWs ws, uint32_t s) {
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    if (idx >= ws.P) return;
    RT_G double* a = ws.acc + 3 * (size_t)idx;
    const RT_G double* L = ws.L + 3 * (size_t)idx;
    double c[3];
#pragma unroll
    for (int k = 0; k < 3; k++) c[k] = (s == 0 ? 0.0 : a[k]) + L[k];
    if (s + 1 == (uint32_t)fp.spp) {
        store_rgb(fp, idx, c);
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) a[k] = c[k];
    }
}
