// Diffuse path tracing of primary + secondary rays (SURVEY.md §8(f) item 3,
// BASELINE config c5: "16 spp + 4-bounce secondary rays").  Included by
// render.hip after trace_core (uses Ray64, Win, LaneStack, trace_core).
//
// The reference has no secondary rays, so the path model is build-defined
//  and restated operation for operation by the oracle
// (oracle/rt_oracle.cpp orc_render_paths); every *segment* is traced with
// the reference's own closest-hit semantics (stack_bvh.hpp:611-644) by the
// exact per-lane traversal, so a path's vertices are the reference's hits.
//
//   sample s of pixel (i, j), frame F:   seed = h(h(h(0x5EED + F) + j*W + i) + s)
//   draw n:                              u_n = (h(seed + n * 0x9E3779B9) >> 8) * 2^-24
//   primary ray:                         camera.hpp:35-37 with offsets (u_0, u_1)
//                                        in place of the pixel centre 0.5
//   vertex k (k = 0 .. bounces):         c_k = shadeScreen's colour at the hit
//                                        (light at the camera, main.cpp:356-377)
//   radiance:                            L = sum_k 0.5^k c_k   (until a miss)
//   bounce k -> k+1:                     cosine-weighted direction about the
//                                        hit normal facing the ray, draws
//                                        u_{2+2k}, u_{3+2k}
//   pixel colour:                        (sum_s L_s) / spp, cast as saveScreen
//
// Every fp64 expression keeps the oracle's operation order (-ffp-contract=off);
// sin/cos come from the fixed polynomial below, not from a libm, so the CPU
// and the GPU compute the same bits.
#pragma once

// lowbias32 integer hash
__device__ __forceinline__ uint32_t h32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t path_seed(uint32_t frame, uint32_t px, uint32_t s) {
    return h32(h32(h32(0x5EEDu + frame) + px) + s);
}
__device__ __forceinline__ double path_u(uint32_t seed, uint32_t n) {
    return (double)(h32(seed + n * 0x9E3779B9u) >> 8) * 0x1p-24;
}

// sin and cos of 2 pi f, f in [0, 1): octant k = floor(8 f), x = (8 f - k) pi/4
// in [0, pi/4) (8 f is exact), Taylor polynomials to x^17 / x^18 (truncation
// below 2^-60 there), then the octant's rotation.
__device__ __forceinline__ void spec_sincos(double f, double& sn, double& cs) {
    const double f8 = f * 8.0;
    const int k = (int)f8;
    const double x = (f8 - (double)k) * 0x1.921fb54442d18p-1;  // pi / 4
    const double x2 = x * x;
    const double sx = x * (1.0 + x2 * (-0x1.5555555555555p-3 + x2 * (0x1.1111111111111p-7 + x2 * (-0x1.a01a01a01a01ap-13 + x2 * (0x1.71de3a556c734p-19 + x2 * (-0x1.ae64567f544e4p-26 + x2 * (0x1.6124613a86d09p-33 + x2 * (-0x1.ae7f3e733b81fp-41 + x2 * 0x1.952c77030ad4ap-49))))))));
    const double cx = 1.0 + x2 * (-0x1.0000000000000p-1 + x2 * (0x1.5555555555555p-5 + x2 * (-0x1.6c16c16c16c17p-10 + x2 * (0x1.a01a01a01a01ap-16 + x2 * (-0x1.27e4fb7789f5cp-22 + x2 * (0x1.1eed8eff8d898p-29 + x2 * (-0x1.93974a8c07c9dp-37 + x2 * (0x1.ae7f3e733b81fp-45 + x2 * -0x1.6827863b97d97p-53))))))));
    const double r = 0x1.6a09e667f3bcdp-1;  // sqrt(2) / 2
    // the octant's sin / cos (selects, no indexed table: it would live in scratch)
    const double sa = (k == 1 || k == 3) ? r : (k == 5 || k == 7) ? -r : k == 2 ? 1.0 : k == 6 ? -1.0 : 0.0;
    const double ca = (k == 1 || k == 7) ? r : (k == 3 || k == 5) ? -r : k == 0 ? 1.0 : k == 4 ? -1.0 : 0.0;
    sn = sa * cx + ca * sx;
    cs = ca * cx - sa * sx;
}

// Cosine-weighted direction about n (flipped to face against din), from the
// orthonormal basis of Duff et al. (2017); normalised by division by the
// length as Vector3::normalize (vector3.hpp:91-95).
__device__ __forceinline__ void bounce_dir(double nx, double ny, double nz, double dx, double dy, double dz,
                                           double u1, double u2, double& ox, double& oy, double& oz) {
    if (nx * dx + ny * dy + nz * dz > 0.0) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
    }
    const double sign = nz >= 0.0 ? 1.0 : -1.0;
    const double a = -1.0 / (sign + nz);
    const double b = nx * ny * a;
    const double tx = 1.0 + sign * nx * nx * a, ty = sign * b, tz = -sign * nx;
    const double bx = b, by = sign + ny * ny * a, bz = -ny;
    const double rr = __builtin_sqrt(u1);
    double sphi, cphi;
    spec_sincos(u2, sphi, cphi);
    const double x = rr * cphi, y = rr * sphi, z = __builtin_sqrt(1.0 - u1);
    double ex = (tx * x + bx * y) + nx * z;
    double ey = (ty * x + by * y) + ny * z;
    double ez = (tz * x + bz * y) + nz * z;
    const double len = __builtin_sqrt(ex * ex + ey * ey + ez * ez);
    if (len > 0.0) {
        ex = ex / len;
        ey = ey / len;
        ez = ez / len;
    }
    ox = ex;
    oy = ey;
    oz = ez;
}

// shadeScreen's colour of a vertex at p with unit normal n, light at the
// camera (main.cpp:356-377; the primary vertex gives shade_color's value).
__device__ __forceinline__ void shade_at(const RtFrameCam& cam, double px, double py, double pz, double nx, double ny,
                                         double nz, double c[3]) {
    double lx = cam.pos[0] - px, ly = cam.pos[1] - py, lz = cam.pos[2] - pz;
    const double dist = __builtin_sqrt(lx * lx + ly * ly + lz * lz);
    if (dist > 0.0) {
        const double s = 1.0 / dist;
        lx = lx * s;
        ly = ly * s;
        lz = lz * s;
    }
    const double diffuse = smax(0.0, nx * lx + ny * ly + nz * lz) * 1.35;
    const double att = 1.0 / (1.0 + 0.05 * dist * dist);
    const double I = sclamp((0.45 + diffuse * att) * 1.25, 0.0, 1.0);
    c[0] = (0.5 * (nx + 1.0)) * I;
    c[1] = (0.5 * (ny + 1.0)) * I;
    c[2] = (0.5 * (nz + 1.0)) * I;
}

// World-space slab margin valid for a ray from o (frame_pad's bound,
// rt_api.cpp: 2^-19 (|o|max + |coordinate|max), rounded up to fp32).
__device__ __forceinline__ float ray_pad(const RtDevScene& sc, const Ray64& r) {
    const double om = __builtin_fmax(__builtin_fmax(__builtin_fabs(r.ox), __builtin_fabs(r.oy)), __builtin_fabs(r.oz));
    return round_up_f(__builtin_ldexp(om + sc.coord_max + 1e-30, -19));
}

// The primary segment of a packed wave (PACK: every sample of 2x2 pixels at
// 16 spp, one per lane) through the wave-cooperative walk of the packet
// kernel (packet_kernel.h: the 64 rays share one camera origin and a 2x2
// pixel footprint, so a node's W child records come once per wave through
// scalar loads, every lane slab-tests them and `ballot` picks the children
// any ray enters) instead of 64 per-lane walks of the quantised nodes.  The
// outputs are lane_walk's: per lane the survivors of the fp32 triangle
// filter in cand[0 .. nc)[tid] ({triangle, t lower bound}), the culling
// distance, and `over` when more than K survive (the lane then takes the
// exact per-lane path).  wstack: this wave's u32 stack (>= stack bound
// entries).  COUNT: the wave's node steps and triangle records (counters 7
// and 12, as the packet kernel's), the lane's pre-filter tests in lc.pre.
template <int W, int K, bool COUNT>
__device__ __forceinline__ void wave_walk(const RtDevScene& sc, const RtFrameParams& fp, const Ray32& q, float pd,
                                          float tsl, bool valid, uint32_t* __restrict__ wstack,
                                          uint2 (*cand)[256], int tid, LaneCounts& lc, float& tcull_out, int& nc_out,
                                          bool& over_out) {
    const int lane = tid & 63;
    const uint32_t lsg = (q.ix < 0.f ? 1u : 0u) | (q.iy < 0.f ? 2u : 0u) | (q.iz < 0.f ? 4u : 0u);
    const uint32_t dsg = uni(lsg);
    const int oct = __ballot(valid && lsg != dsg) == 0 ? (int)dsg : 8;
    const f2 nox{-(q.ox + pd) * q.ix, -(q.ox - pd) * q.ix};
    const f2 noy{-(q.oy + pd) * q.iy, -(q.oy - pd) * q.iy};
    const f2 noz{-(q.oz + pd) * q.iz, -(q.oz - pd) * q.iz};
    float tcull = valid ? __builtin_huge_valf() : -1.f;
    int nc = 0;
    bool over = false;
    uint32_t w_nodes = 0, w_tris = 0;
    uint32_t cur = sc.root_ref;
    if (!(cur & RT_LEAF_BIT)) cur |= sc.root_meta << 24;
    {
        float b[1][6];
        for (int a = 0; a < 6; a++) b[0][a] = sc.root_box[a];
        uint64_t h[1];
        child_hits<1, -1>(b, q, nox, noy, noz, tcull, h);
        if (h[0] == 0) cur = RT_INVALID_REF;
    }
    int sp = 0;
    const RT_G uint8_t* const nodes = sc.nodes;
    const RT_G float* const tri32 = sc.tri32;
    auto walk = [&]<int OCT>() __attribute__((always_inline)) {
        if (cur == RT_INVALID_REF) return;
        for (;;) {
            if (!(cur & RT_LEAF_BIT)) {
                if (COUNT) w_nodes++;
                float bx[W][6];
                uint32_t rs[W];
                const uint32_t meta = cur >> 24;
                uint64_t hm[W];
                {
                    const cchild_p nb = (cchild_p)(nodes + (size_t)(cur & 0x00FFFFFFu) * (32 * W));
                    ChildRec ch[W];
#pragma unroll
                    for (int c = 0; c < W; c++) ch[c] = load_child(nb + c);
                    // all 8 words of every record loaded (4 s_load_dwordx16),
                    // not the ~24 narrow loads of the words used
#pragma unroll
                    for (int c = 0; c < W; c++) pin_rec(ch[c]);
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        bx[c][0] = ch[c].lx; bx[c][1] = ch[c].hx; bx[c][2] = ch[c].ly;
                        bx[c][3] = ch[c].hy; bx[c][4] = ch[c].lz; bx[c][5] = ch[c].hz;
                    }
#pragma unroll
                    for (int c = 0; c < W; c++) rs[c] = ch[c].pad;  // ref | meta << 24 (bvh_build.cpp flatten)
                    child_hits<W, OCT>(bx, q, nox, noy, noz, tcull, hm);
                }
                const uint32_t mask = any_mask<W>(hm) & ((1u << (meta >> 2)) - 1u);
                if (mask != 0) {
                    const bool rev = (dsg >> (meta & 3u)) & 1u;
                    const int near_c = rev ? 31 - __builtin_clz(mask) : __builtin_ctz(mask);
                    const uint32_t pm = mask & ~(1u << near_c);
                    if (pm != 0) {
                        const uint32_t refv = lanes_of<W>(rs);
                        const uint32_t lid = mbcnt_lo(~0u);
                        const uint32_t below = mbcnt_lo(pm);
                        const uint32_t mine = (pm >> (lid & 31u)) & 1u;
                        const uint32_t above = (uint32_t)__builtin_popcount(pm) - below - mine;
                        const int slot = (int)(rev ? below : above);
                        if (mine & (lid < (uint32_t)W)) wstack[sp + slot] = refv;
                        sp += __builtin_popcount(pm);
                    }
                    uint32_t nr = rs[0];
#pragma unroll
                    for (int c = 1; c < W; c++) nr = near_c == c ? rs[c] : nr;
                    cur = nr;
                    continue;
                }
            } else {
                const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                if (COUNT) w_tris += cnt;
                const uint32_t end = first + cnt;
                for (uint32_t k0 = first; k0 < end; k0 += kLeafChunk) {
                    const cfloat_p R = (cfloat_p)(tri32 + 12 * (size_t)k0);
                    float4 TA[kLeafChunk], TB[kLeafChunk], TC[kLeafChunk];
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) {
                        TA[t] = load_f4(R + 12 * t);
                        TB[t] = load_f4(R + 12 * t + 4);
                        TC[t] = load_f4(R + 12 * t + 8);
                    }
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) pin_s(TA[t], TB[t], TC[t]);
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) {
                        const uint32_t k = k0 + t;
                        if (k >= end) break;
                        if (COUNT) lc.pre += valid;
                        float tl, tu;
                        // (an invalid lane's class is computed and dropped by a
                        // select; no `continue` in the unrolled chunk loop)
                        int cls = tri_classify(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull,
                                               tl, tu);
                        cls = valid ? cls : 0;
                        if (cls != 0) {
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
                    }
                }
            }
            if (sp == 0) break;
            sp--;
            cur = uni(wstack[sp]);
        }
    };
    switch (oct) {
        case 0: walk.template operator()<0>(); break;
        case 1: walk.template operator()<1>(); break;
        case 2: walk.template operator()<2>(); break;
        case 3: walk.template operator()<3>(); break;
        case 4: walk.template operator()<4>(); break;
        case 5: walk.template operator()<5>(); break;
        case 6: walk.template operator()<6>(); break;
        case 7: walk.template operator()<7>(); break;
        default: walk.template operator()<-1>(); break;
    }
    if (COUNT && fp.counters && lane == 0) {
        atomicAdd(&fp.counters[7], (unsigned long long)w_nodes);
        atomicAdd(&fp.counters[12], (unsigned long long)w_tris);
    }
    tcull_out = tcull;
    nc_out = nc;
    over_out = over;
}

// Head-light occlusion of a bounce vertex p (the oracle's occluded(),
// oracle/rt_oracle.cpp): the ray from the light at the camera C
// toward p, o = C, d = e / |e| (e = p - C, Vector3::normalize's divisions),
// is occluded iff some triangle passes the reference's Moller-Trumbore test
// (triangle.hpp:40-62) with t < |e| (1 - 2^-12) — over all triangles, so any
// tree that finds every candidate gives the same answer.  The fp32 walk of the
// walk tree (slabs widened by the pad, interval clipped to the fp32 bound of
// tmax) keeps every triangle the fp64 test could pass; tri_classify's certain
// class with an upper bound below 0.999 tmax is an occluder outright, any
// other survivor whose lower bound is within the interval gets the fp64 test.
// The first occluder ends the walk (any hit, no order needed).  The margin
// 2^-12 is far wider than the fp32 filter's error budget, so p's own triangle
// (t = |e| up to rounding) is rejected in fp32 and costs no fp64 test.
constexpr double kShadowScale = 1.0 - 0x1p-12;
// COUNT: the walk's node steps and triangle records go to oc->nodes / oc->pre.
template <int W, int S, bool QN, bool COUNT = false>
__device__ __forceinline__ bool lane_occluded(const RtDevScene& sc, const RtFrameCam& cam, double px, double py,
                                              double pz, LaneStack<S>& st, LaneCounts* oc = nullptr) {
    // the fp64 ray, built again for the rare fp64 test rather than held
    // (12 VGPRs) through the walk
    auto ray_of = [&](double& len) {
        const double ex = px - cam.pos[0], ey = py - cam.pos[1], ez = pz - cam.pos[2];
        len = __builtin_sqrt(ex * ex + ey * ey + ez * ez);
        Ray64 r;
        r.ox = cam.pos[0];
        r.oy = cam.pos[1];
        r.oz = cam.pos[2];
        r.dx = ex / len;
        r.dy = ey / len;
        r.dz = ez / len;
        r.ix = r.iy = r.iz = 0.0;
        return r;
    };
    double len;
    Ray32 q;
    {
        const Ray64 r = ray_of(len);
        if (!(len > 0.0)) return false;
        q = make_ray32<true>(r, ray_pad(sc, r));
    }
    const double tmax = len * kShadowScale;
    const float tcert = (float)(tmax * 0.999);
    LaneCounts lc;
    LaneWalk<W, S, 1, COUNT, QN> w;
    w.begin(sc, q, 0.f, st);
    w.tcull = round_up_f(tmax);
    bool occ = false;
    while (w.cur != RT_INVALID_REF) {
        if constexpr (COUNT) wave_step_fetches(w.cur, lc);
        if (!(w.cur & RT_LEAF_BIT)) {
            w.visit_node(sc, st, lc);
            continue;
        }
        const uint32_t first = w.cur & RT_LEAF_FIRST_MASK;
        const uint32_t cnt = ((w.cur >> 27) & 15u) + 1u;
        for (uint32_t k = first; k < first + cnt; k++) {
            const float4* R = reinterpret_cast<const float4*>(sc.tri32 + 12 * (size_t)k);
            float tl, tu;
            if (COUNT) lc.pre++;
            const int cls = tri_classify(R[0], R[1], R[2], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, w.tcull, tl, tu);
            if (cls == 2 && tu < tcert) {
                occ = true;
                break;
            }
            if (cls != 0) {
                double t, l2;
                if (mt64(sc.tri64 + RT_TRI64_DOUBLES * (size_t)k, ray_of(l2), t) && t < tmax) {
                    occ = true;
                    break;
                }
            }
        }
        if (occ) break;
        w.pop_next(st);
    }
    if (COUNT) {
        oc->nodes += lc.nodes;
        oc->pre += lc.pre;
        oc->wnodes += lc.wnodes;
        oc->wtris += lc.wtris;
    }
    return occ;
}

// Primary segments through wave_walk (PRIM, PACK on 8-wide trees whose stack
// bound fits 128 entries): RT_PATHS_PRIMARY=0 walks them per lane.
#ifndef RT_PATHS_PRIM
#define RT_PATHS_PRIM 1
#endif

// Persistent waves over 8x8 pixel tiles of one pose; every lane traces all
// spp paths of its pixel (segments in order), so the pixel's sum is formed in
// sample order.  frame: the hash's frame number.
#ifndef RT_PATHS_WPE
#define RT_PATHS_WPE 5  // with the 8-entry LDS ring (RT_PATHS_STACK): 3.54 vs 3.37 G at 4 waves (128 VGPRs)
#endif
#if RT_PATHS_WPE > 0
#define RT_PATHS_ATTR __attribute__((amdgpu_waves_per_eu(RT_PATHS_WPE)))
#else
#define RT_PATHS_ATTR
#endif
// Segments through trace_deferred (fp64 after the walk, RT_PATHS_K LDS
// candidates per lane) or trace_core (fp64 inside the walk): 1 / 0.
#ifndef RT_PATHS_DEFER
#define RT_PATHS_DEFER 1
#endif
#ifndef RT_PATHS_K
#define RT_PATHS_K 4
#endif
// W = 8 paths walk the quantised node copy (lane_walk QN)
#ifndef RT_QNODES
#define RT_QNODES 1
#endif
// COUNT (the counting pass, RT_FLAG_COUNT, W = 8 only): per-lane node steps,
// triangle pre-filter and fp64 tests summed into the fetch counters for the
// roofline's algorithmic bytes (bench.py --paths).
// PACK (fp.pack, 64 % spp == 0): a wave takes all spp samples of 64 / spp
// pixels, one sample path per lane (lane = pixel * spp + sample; the pixels a
// tw x th block), and the pixel's radiance is summed across its lanes in
// sample order — the same additions as the per-lane sample loop.
// SHADOW: a bounce vertex adds its colour only if the light sees it
// (lane_occluded, one occlusion ray per vertex k >= 1; the primary vertex is
// the camera ray's own closest hit, which the light at the camera sees).
template <int W, int S, bool COUNT = false, bool PACK = false, bool PRIM = false, bool SHADOW = false>
__global__ void __launch_bounds__(256) RT_PATHS_ATTR k_paths(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, uint32_t frame,
                                               int bounces) {
    static_assert(!PRIM || (PACK && W == 8 && RT_PATHS_DEFER), "wave-walked primaries: packed 8-wide deferred paths");
    __shared__ uint2 lds[S][256];
#if RT_PATHS_DEFER
    __shared__ uint2 pcand[RT_PATHS_K][256];
#endif
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int spp = fp.spp;
    int tw = 8, th = 8;  // pixels per tile
    if constexpr (PACK) {
        const int P = 64 / spp;
        tw = 1;
        while (tw * tw < P) tw <<= 1;
        th = P / tw;
    }
    const int tiles_x = (fp.W + tw - 1) / tw;
    const int tiles = tiles_x * ((fp.nrows + th - 1) / th);
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const RtFrameCam cam = frame_cam(fp, 0);
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = (int)atomicAdd(aux.tile_ctr, 1u);
        tile = __shfl(tile, 0);
        if (tile >= tiles) break;
        int i, r, s0 = 0, s1 = spp;  // the lane's pixel and samples [s0, s1)
        if constexpr (PACK) {
            const int pl = lane / spp;
            s0 = lane & (spp - 1);
            s1 = s0 + 1;
            i = (tile % tiles_x) * tw + pl % tw;
            r = (tile / tiles_x) * th + pl / tw;
        } else {
            i = (tile % tiles_x) * 8 + (lane & 7);
            r = (tile / tiles_x) * 8 + (lane >> 3);
        }
        uint32_t hits = 0, segs = 0;  // segs: ray segments traced (RT_FLAG_COUNT)
        uint32_t sh_cast = 0, sh_occ = 0;  // SHADOW: occlusion rays cast / occluded
        LaneCounts tot;               // COUNT: the lane's fetch counts over its paths
        LaneCounts shc;               // COUNT: ... of its occlusion walks
        // PRIM: the primary segment of every lane of the wave (one sample per
        // lane) walked together, before the lanes go their own ways
        float p_tcull = 0.f;
        int p_nc = 0;
        bool p_over = false;
        if constexpr (PRIM) {
            const bool valid = i < fp.W && r < fp.nrows;
            const int iv = valid ? i : 0, jv = rt_image_row(fp.row0, fp.row_stride, fp.band, valid ? r : 0);
            const uint32_t seed = path_seed(frame, (uint32_t)jv * (uint32_t)fp.W + (uint32_t)iv, (uint32_t)s0);
            RtFrameCam c1 = cam;
            c1.ox = path_u(seed, 0);
            c1.oy = path_u(seed, 1);
            const Ray64 ray0 = gen_ray<false>(fp, c1, iv, jv);
            const float pd = ray_pad(sc, ray0);
            const Ray32 q0 = make_ray32<true>(ray0, pd);
            const float tsl = round_up_f(0x1p-40 * ((double)q0.co + 1.0));
            uint32_t* wstack = reinterpret_cast<uint32_t*>(&lds[0][tid & ~63]);  // 128 u32 of this wave's row
            wave_walk<W, RT_PATHS_K, COUNT>(sc, fp, q0, pd, tsl, valid, wstack, pcand, tid, tot, p_tcull, p_nc,
                                            p_over);
        }
        if (i < fp.W && r < fp.nrows) {
            const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, r);
            const size_t pix = (size_t)r * fp.W + i;
            double acc[3] = {0.0, 0.0, 0.0};
            for (int s = s0; s < s1; s++) {
                const uint32_t seed = path_seed(frame, (uint32_t)j * (uint32_t)fp.W + (uint32_t)i, (uint32_t)s);
                // primary ray through (i + u0, j + u1): gen_ray with the sample's offsets
                RtFrameCam c1 = cam;
                c1.ox = path_u(seed, 0);
                c1.oy = path_u(seed, 1);
                // the segment's ray without reciprocals (6 doubles live across the
                // walk); ray_of() adds them where the traversal needs them
                Ray64 ray = gen_ray<false>(fp, c1, i, j);
                double L[3] = {0.0, 0.0, 0.0};
                double w = 1.0;
                for (int b = 0; b <= bounces; b++) {
                    LaneCounts lc;
#if RT_PATHS_DEFER
                    Win win;
                    if (PRIM && b == 0) {
                        // the wave walk's list: trace_deferred's resolve and fall-backs
                        auto ray_of = [&]() { return with_inv(ray); };
                        if (p_over) {
                            win = trace_core<W, S, COUNT>(sc, ray_of, ray_pad(sc, ray), st, 0, lc);
                        } else if (resolve_cands<COUNT>(sc, ray_of(), [&](int c) { return pcand[c][tid]; }, p_nc,
                                                        p_tcull, win, lc) != 0) {
                            win = trace_core<W, S, COUNT>(sc, ray_of, ray_pad(sc, ray), st, 1, lc);
                        }
                    } else {
                        win = trace_deferred<W, S, RT_PATHS_K, COUNT, W == 8 && RT_QNODES>(
                            sc, [&]() { return with_inv(ray); }, ray_pad(sc, ray), st, pcand, lc);
                    }
#else
                    const Win win =
                        trace_core<W, S, COUNT>(sc, [&]() { return with_inv(ray); }, ray_pad(sc, ray), st, 0, lc);
#endif
                    segs++;
                    if (COUNT) {
                        tot.nodes += lc.nodes;
                        tot.wnodes += lc.wnodes;
                        tot.wtris += lc.wtris;
                        tot.pre += lc.pre;
                        tot.tris += lc.tris;
                        tot.chain += lc.chain;
                    }
                    Best hb;
                    hb.dist = win.dist;
                    hb.rank = win.rank;
                    hb.tri = win.tri;
                    hb.px = hb.py = hb.pz = 0.0;
                    if (win.tri >= 0) (void)hit_dist(ray, win.t, hb.px, hb.py, hb.pz);  // (uses o, d only)
                    const Shade sh = shade_of(sc, win.tri);
                    if (b == 0) {  // the primary segment's per-sample outputs
                        store_sample(fp, pix * (size_t)fp.spp + s, hb, sh);
                        hits += win.tri >= 0;
                    }
                    if (win.tri < 0) break;
                    bool lit = true;
                    if constexpr (SHADOW) {
                        if (b > 0) {
                            lit = !lane_occluded<W, S, W == 8 && RT_QNODES, COUNT>(sc, cam, hb.px, hb.py, hb.pz, st, &shc);
                            sh_cast++;
                            sh_occ += !lit;
                        }
                    }
                    if (lit) {
                        double c[3];
                        shade_at(cam, hb.px, hb.py, hb.pz, sh.nx, sh.ny, sh.nz, c);
                        L[0] = L[0] + w * c[0];
                        L[1] = L[1] + w * c[1];
                        L[2] = L[2] + w * c[2];
                    }
                    w = w * 0.5;
                    if (b == bounces) break;
                    double nx, ny, nz;
                    bounce_dir(sh.nx, sh.ny, sh.nz, ray.dx, ray.dy, ray.dz, path_u(seed, 2u + 2u * (uint32_t)b),
                               path_u(seed, 3u + 2u * (uint32_t)b), nx, ny, nz);
                    ray.ox = hb.px;
                    ray.oy = hb.py;
                    ray.oz = hb.pz;
                    ray.dx = nx;
                    ray.dy = ny;
                    ray.dz = nz;
                }
                acc[0] = acc[0] + L[0];
                acc[1] = acc[1] + L[1];
                acc[2] = acc[2] + L[2];
            }
            if constexpr (PACK) {
                // the pixel's samples are lanes base .. base + spp - 1
                const int base = lane & ~(spp - 1);
                double sum[3] = {0.0, 0.0, 0.0};
                for (int k = 0; k < spp; k++) {
                    sum[0] = sum[0] + __shfl(acc[0], base + k);
                    sum[1] = sum[1] + __shfl(acc[1], base + k);
                    sum[2] = sum[2] + __shfl(acc[2], base + k);
                }
                if (lane == base) store_rgb(fp, pix, sum);
            } else {
                store_rgb(fp, pix, acc);
            }
        }
        wave_add<13>(fp.hit_count, hits);
        if (fp.counters) wave_add<20>(fp.counters, segs);
        if (SHADOW && fp.counters) {
            wave_add<20>(fp.counters + 24, sh_cast);
            wave_add<20>(fp.counters + 25, sh_occ);
            if (COUNT) {
                wave_add<28>(fp.counters + 28, shc.nodes);
                wave_add<28>(fp.counters + 30, shc.wnodes);
                wave_add<28>(fp.counters + 31, shc.wtris);
                wave_add<28>(fp.counters + 29, shc.pre);
            }
        }
        if (COUNT && fp.counters) {
            wave_add<24>(fp.counters + 1, tot.nodes);
            wave_add<28>(fp.counters + 30, tot.wnodes);
            wave_add<28>(fp.counters + 31, tot.wtris);
            wave_add<24>(fp.counters + 6, tot.pre);
            wave_add<24>(fp.counters + 2, tot.tris);
            wave_add<24>(fp.counters + 3, tot.chain);
        }
    }
}
