// Queued diffuse path tracing (config c5; SURVEY.md §8(f) item 3: a
// wavefront path tracer with compacted bounce queues and occlusion rays).
// Included by render.hip after path_kernel.h.  The path model is
// path_kernel.h's, bit for bit: every fp64 expression is the
// megakernel's in the same order, so the outputs equal k_paths' and the
// oracle's (orc_render_paths).
//
// A pose is traced segment by segment over ALL its paths (W x rows x spp of
// them, up to 132.7 M at config c5: the state of every path of the pose lives
// in HBM, 80 B per queued ray, sized for MI355X's 288 GB):
//   k_q_primary   persistent waves over packed tiles (every sample of 64 / spp
//                 pixels, or 8 x 8 pixels of one sample): the wave-cooperative
//                 walk of the 64 primary rays (path_kernel.h wave_walk), the
//                 exact resolve per lane, the per-sample outputs, the primary
//                 vertex's colour, and the first bounce ray appended to queue
//                 0 — compacted: one atomic per wave, paths that missed drop out;
//   k_q_segment   segment b = 1 .. bounces: persistent waves pull 64 queued
//                 rays at a time; per lane the fp32 walk of the quantised
//                 nodes (lane_walk), the exact fp64 resolve, the occlusion ray
//                 toward the head-light (SHADOW, lane_occluded), the vertex
//                 colour added to the path's radiance, and the next bounce ray
//                 appended to the other queue (compacted again).  A lane whose
//                 candidate list overflowed, or whose winner the reference
//                 tree cannot see, goes on the segment's fall-back list;
//   k_q_fallback  those rays through the exact per-lane traversal (trace_core)
//                 and the same epilogue (kept out of k_q_segment, whose
//                 registers it would raise for ~1e-4 of the rays);
//   k_q_accum     per pixel the paths' final radiance summed in sample order,
//                 the colour cast as saveScreen.
// The path state a ray carries (its radiance so far) travels in its queue
// entry; a path that ends (miss, or its last segment) leaves its radiance in
// Lfin.  Kernel ordering on the stream replaces every device-wide barrier; the
// control words (queue counts, pull cursors, fall-back counts: one per segment,
// each on its own 64-B line) are zeroed once per pose by the host.
#pragma once

#ifndef RT_Q_WPE
#define RT_Q_WPE 6  // waves per SIMD of k_q_segment (80 VGPRs): c5 234 vs 243 ms per pose at 5 (96 VGPRs)
#endif
#ifndef RT_Q_K
#define RT_Q_K 5  // LDS candidates per lane in k_q_segment (26 KB of LDS per block: 6 blocks per CU); c5 232.5 vs 233.9 ms at 4
#endif
#ifndef RT_Q_STACK
#define RT_Q_STACK 8  // LDS stack ring entries per lane in k_q_segment
#endif

// Control words (u32, RT_QC_STRIDE apart): per segment b = 0 .. bounces,
//   emit(b, x)  rays segment b appended to partition x of queue b & 1
//               (segment b + 1's input)
//   pull(b, x)  pull cursor of segment b's kernel in partition x (k_q_primary:
//               its tile cursor)
//   sh(b, x)    occlusion records segment b appended to partition x of the
//               record array (queued shadows)
//   shpull(b,x) the occlusion kernels' pull cursor in part x of their input
//   fb(b)       fall-back entries segment b listed
#define RT_QC_STRIDE 16
__device__ __forceinline__ RT_G uint32_t* qc_emit(const PathQs& q, int b, int x) {
    return q.ctl + (RT_QC_LINES * b + x) * RT_QC_STRIDE;
}
__device__ __forceinline__ RT_G uint32_t* qc_pull(const PathQs& q, int b, int x) {
    return q.ctl + (RT_QC_LINES * b + RT_QPARTS + x) * RT_QC_STRIDE;
}
__device__ __forceinline__ RT_G uint32_t* qc_sh(const PathQs& q, int b, int x) {
    return q.ctl + (RT_QC_LINES * b + 2 * RT_QPARTS + x) * RT_QC_STRIDE;
}
__device__ __forceinline__ RT_G uint32_t* qc_shpull(const PathQs& q, int b, int x) {
    return q.ctl + (RT_QC_LINES * b + 3 * RT_QPARTS + x) * RT_QC_STRIDE;
}
__device__ __forceinline__ RT_G uint32_t* qc_fb(const PathQs& q, int b) {
    return q.ctl + (RT_QC_LINES * b + 4 * RT_QPARTS) * RT_QC_STRIDE;
}
// Occlusion records of segment b: partition x holds entries [x pcap, x pcap +
// *qc_sh(b, x)) of srec as appended; sorted (binned mode) their pairs are one
// run of sh_total records.
__device__ __forceinline__ uint32_t sh_total(const PathQs& q, int b) {
    uint32_t n = 0;
    for (int x = 0; x < (int)q.parts; x++) n += *qc_sh(q, b, x);
    return n;
}
// Range [lo, hi) of part x of `parts` over an input of records: partitioned
// (the appended records: partition x) or one run of n (sorted: its x-th
// slice).
__device__ __forceinline__ void sh_part(const PathQs& q, int b, int x, bool sorted, uint32_t n, uint32_t& lo,
                                        uint32_t& hi) {
    if (sorted) {
        lo = (uint32_t)((uint64_t)n * (uint32_t)x / q.parts);
        hi = (uint32_t)((uint64_t)n * (uint32_t)(x + 1) / q.parts);
    } else {
        lo = (uint32_t)x * q.pcap;
        hi = lo + *qc_sh(q, b, x);
    }
}
// A wave's next 64 records of an occlusion kernel's input: from its part x
// (its XCD's: blocks are dealt round-robin), then the others in turn; false
// when every part is drained.  e0: the first record of the 64, hi: the end of
// its part.
struct ShPull {
    int x, left;
    uint32_t lo, hi;
};
__device__ __forceinline__ void sh_pull_begin(const PathQs& q, int b, bool sorted, uint32_t n, ShPull& p) {
    p.x = (int)(blockIdx.x % q.parts);
    p.left = (int)q.parts;
    sh_part(q, b, p.x, sorted, n, p.lo, p.hi);
}
__device__ __forceinline__ bool sh_pull(const PathQs& q, int b, bool sorted, uint32_t n, ShPull& p, uint32_t& e0) {
    const int lane = (int)(threadIdx.x & 63);
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(qc_shpull(q, b, p.x), 64u);
        base = (uint32_t)__shfl((int)base, 0);
        if (p.lo + base < p.hi) {
            e0 = p.lo + base;
            return true;
        }
        if (--p.left == 0) return false;
        p.x = p.x + 1 == (int)q.parts ? 0 : p.x + 1;
        sh_part(q, b, p.x, sorted, n, p.lo, p.hi);
    }
}

// Queue entry e of queue k: 10 doubles {o, d, L, path | pad}.
constexpr int kQDoubles = 10;
__device__ __forceinline__ RT_G double* q_entry(const PathQs& q, int k, uint32_t e) {
    return q.q[k] + (size_t)kQDoubles * e;
}
__device__ __forceinline__ void q_load(const PathQs& q, int k, uint32_t e, Ray64& r, double L[3], uint32_t& path) {
    const RT_G double* p = q_entry(q, k, e);
    r.ox = p[0];
    r.oy = p[1];
    r.oz = p[2];
    r.dx = p[3];
    r.dy = p[4];
    r.dz = p[5];
    r.ix = r.iy = r.iz = 0.0;
    L[0] = p[6];
    L[1] = p[7];
    L[2] = p[8];
    path = (uint32_t)__double_as_longlong(p[9]);
}

// Appends each emitting lane's bounce ray (origin, direction, path) to
// partition x of queue k (segment b's counter) with one atomic per wave (the
// compaction: lanes whose paths ended append nothing) and returns the lane's
// entry (an index into the whole queue); the radiance is written after the
// occlusion test (q_light).  Every lane of the wave calls it, with one x.
__device__ __forceinline__ uint32_t q_append(const PathQs& q, int k, int x, int b, bool emit, const Ray64& nr,
                                             uint32_t path) {
    const uint64_t em = __ballot(emit);
    if (em == 0) return 0;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __builtin_ctzll(em);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(qc_emit(q, b, x), (uint32_t)__builtin_popcountll(em));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader) + (uint32_t)x * q.pcap;
    const uint32_t slot = base + (uint32_t)__builtin_popcountll(em & ((1ull << lane) - 1ull));
    if (emit) {
        RT_G double* p = q_entry(q, k, slot);
        p[0] = nr.ox;
        p[1] = nr.oy;
        p[2] = nr.oz;
        p[3] = nr.dx;
        p[4] = nr.dy;
        p[5] = nr.dz;
        p[9] = __longlong_as_double((long long)path);
    }
    return slot;
}

// RT_Q_NR_LDS (k_q_segment): the bounce ray's vertex and direction cross
// q_append's atomic in the lane's LDS ring (entries 0-5) rather than in
// registers; q_append_ring<true> writes the entry from there.
#ifndef RT_Q_NR_LDS
#define RT_Q_NR_LDS 1
#endif
static_assert(RT_Q_NR_LDS == 0 || RT_Q_STACK >= 6, "the bounce stash takes entries 0-5 of the LDS ring");
__device__ __forceinline__ uint2 dbits(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return make_uint2((uint32_t)u, (uint32_t)(u >> 32));
}
__device__ __forceinline__ double bitsd(uint2 v) {
    return __longlong_as_double((long long)(((unsigned long long)v.y << 32) | v.x));
}
// (ends the live ranges of values already stashed: nothing is carried in
// registers across the barrier the compiler could not see through)
__device__ __forceinline__ void opaque_regs() { asm volatile("" ::: "memory"); }
template <bool RING>
__device__ __forceinline__ uint32_t q_append_ring(const PathQs& q, int k, int x, int b, bool emit, const Ray64& nr,
                                                  uint32_t path, uint2 (*ring)[256], int tid) {
    if constexpr (!RING) {
        return q_append(q, k, x, b, emit, nr, path);
    } else {
        const uint64_t em = __ballot(emit);
        if (em == 0) return 0;
        const int lane = (int)(threadIdx.x & 63);
        const int leader = __builtin_ctzll(em);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(qc_emit(q, b, x), (uint32_t)__builtin_popcountll(em));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader) + (uint32_t)x * q.pcap;
        const uint32_t slot = base + (uint32_t)__builtin_popcountll(em & ((1ull << lane) - 1ull));
        if (emit) {
            RT_G double* p = q_entry(q, k, slot);
#pragma unroll
            for (int c = 0; c < 6; c++) p[c] = bitsd(ring[c][tid]);
            p[9] = __longlong_as_double((long long)path);
        }
        return slot;
    }
}

// q_append for one lane (the fall-back kernel: lanes of a wave append to
// different partitions, ~1e-4 of the rays).
__device__ __forceinline__ uint32_t q_append_lane(const PathQs& q, int k, int x, int b, bool emit, const Ray64& nr,
                                                  uint32_t path) {
    if (!emit) return 0;
    const uint32_t slot = atomicAdd(qc_emit(q, b, x), 1u) + (uint32_t)x * q.pcap;
    RT_G double* p = q_entry(q, k, slot);
    p[0] = nr.ox;
    p[1] = nr.oy;
    p[2] = nr.oz;
    p[3] = nr.dx;
    p[4] = nr.dy;
    p[5] = nr.dz;
    p[9] = __longlong_as_double((long long)path);
    return slot;
}

// The partition of a primary path (parts > 1: its tile's XCD queue,
// k_trace_packet's tiles of ptile x ptile pixels dealt to queue
// (t / RT_TILE_RUN) % parts).
__device__ __forceinline__ int q_primary_part(const PathQs& q, const RtFrameParams& fp, uint32_t path) {
    if (q.parts <= 1) return 0;
    const uint32_t pix = path / (uint32_t)fp.spp;
    const uint32_t i = pix % (uint32_t)fp.W, r = pix / (uint32_t)fp.W;
    return (int)((((r / q.ptile) * q.ptiles_x + i / q.ptile) / RT_TILE_RUN) % q.parts);
}

// Sample index of a path -> its pixel's image coordinates and the hash seed.
__device__ __forceinline__ uint32_t q_seed(const RtFrameParams& fp, uint32_t frame, uint32_t path) {
    const uint32_t spp = (uint32_t)fp.spp;
    const uint32_t pix = path / spp, s = path - pix * spp;
    const int i = (int)(pix % (uint32_t)fp.W), r = (int)(pix / (uint32_t)fp.W);
    const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, r);
    return path_seed(frame, (uint32_t)j * (uint32_t)fp.W + (uint32_t)i, s);
}

// A segment's vertex, first half (k_paths' loop body after the trace): the
// hit point and, with bounces left, the next bounce ray (emit).  ray: the
// segment's ray (o, d); win: its exact closest hit (tri >= 0).
__device__ __forceinline__ void q_bounce(const RtDevScene& sc, const RtFrameParams& fp, uint32_t frame, int b,
                                         int bounces, const Ray64& ray, const Win& win, uint32_t path, double& px,
                                         double& py, double& pz, bool& emit, Ray64& nr) {
    (void)hit_dist(ray, win.t, px, py, pz);
    emit = b < bounces;
    if (!emit) return;
    const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)win.tri;
    const uint32_t seed = q_seed(fp, frame, path);
    bounce_dir(T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], ray.dx, ray.dy, ray.dz,
               path_u(seed, 2u + 2u * (uint32_t)b), path_u(seed, 3u + 2u * (uint32_t)b), nr.dx, nr.dy, nr.dz);
    nr.ox = px;
    nr.oy = py;
    nr.oz = pz;
}

// q_bounce with RING: the hit point goes to the lane's LDS ring (entries 0-2)
// as soon as it is known and the bounce direction after it (3-5), for
// q_append_ring<true>; px, py, pz are reloaded from the ring by the caller.
template <bool RING>
__device__ __forceinline__ void q_bounce_ring(const RtDevScene& sc, const RtFrameParams& fp, uint32_t frame, int b,
                                              int bounces, const Ray64& ray, const Win& win, uint32_t path,
                                              double& px, double& py, double& pz, bool& emit, Ray64& nr,
                                              uint2 (*ring)[256], int tid) {
    if constexpr (!RING) {
        q_bounce(sc, fp, frame, b, bounces, ray, win, path, px, py, pz, emit, nr);
    } else {
        double hx, hy, hz;
        (void)hit_dist(ray, win.t, hx, hy, hz);
        ring[0][tid] = dbits(hx);
        ring[1][tid] = dbits(hy);
        ring[2][tid] = dbits(hz);
        emit = b < bounces;
        if (!emit) return;
        const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)win.tri;
        const uint32_t seed = q_seed(fp, frame, path);
        double dx, dy, dz;
        bounce_dir(T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], ray.dx, ray.dy, ray.dz,
                   path_u(seed, 2u + 2u * (uint32_t)b), path_u(seed, 3u + 2u * (uint32_t)b), dx, dy, dz);
        ring[3][tid] = dbits(dx);
        ring[4][tid] = dbits(dy);
        ring[5][tid] = dbits(dz);
    }
}

// Second half: the vertex adds 0.5^b of its shadeScreen colour to the path's
// radiance L if the light sees it (SHADOW, b > 0: lane_occluded; vertex 0
// always), and the radiance goes to the bounce ray's entry (emit: queue kout,
// entry slot) or, when the path ends here, to Lfin.  tri < 0: a miss, the
// path ends with L as it is.  L is read from the segment's own queue entry
// (primary: zero), so nothing of the path is held in registers across the
// walks.
// SH: 0 no occlusion rays, 1 the occlusion ray walked here (per lane), 2
// queued: the radiance without this vertex goes to its destination now and
// the occlusion record is returned in `queue` (q_shadow_append; the binned
// occlusion pass adds the colour if the light sees the vertex).
// COUNT (SH 1): the occlusion walk's fetch counts go to *shc.
template <int W, int S, int SH, bool COUNT = false>
__device__ __forceinline__ void q_light(const RtDevScene& sc, const PathQs& qs, const RtFrameCam& cam, int b,
                                        const RT_G double* Lin, int32_t tri, double px, double py, double pz,
                                        bool emit, int kout, uint32_t slot, uint32_t path, LaneStack<S>& st,
                                        uint32_t& sh_cast, uint32_t& sh_occ, bool& queue, uint32_t& dst,
                                        LaneCounts* shc = nullptr) {
    bool lit = tri >= 0;
    queue = false;
    dst = emit ? (0x80000000u | ((uint32_t)kout << 30) | slot) : path;
    if (SH == 1 && lit && b > 0) {
        lit = !lane_occluded<W, S, W == 8 && RT_QNODES, COUNT>(sc, cam, px, py, pz, st, shc);
        sh_cast++;
        sh_occ += !lit;
    }
    if (SH >= 2 && lit && b > 0) {
        queue = true;
        lit = false;
    }
    double L[3] = {0.0, 0.0, 0.0};
    if (Lin) {
        L[0] = Lin[0];
        L[1] = Lin[1];
        L[2] = Lin[2];
    }
    if (lit) {
        const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)tri;
        const double w = __builtin_ldexp(1.0, -b);  // 0.5^b: k_paths' repeated halving, exactly
        double c[3];
        shade_at(cam, px, py, pz, T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], c);
        L[0] = L[0] + w * c[0];
        L[1] = L[1] + w * c[1];
        L[2] = L[2] + w * c[2];
    }
    RT_G double* f = emit ? q_entry(qs, kout, slot) + 6 : qs.Lfin + 3 * (size_t)path;
    f[0] = L[0];
    f[1] = L[1];
    f[2] = L[2];
}

// Radiance destination of a queued occlusion record: a queue entry's L
// (bit 31, queue in bit 30, entry below) or the path's Lfin.
__device__ __forceinline__ RT_G double* q_dst(const PathQs& qs, uint32_t dst) {
    if (dst & 0x80000000u) return q_entry(qs, (dst >> 30) & 1u, dst & 0x3FFFFFFFu) + 6;
    return qs.Lfin + 3 * (size_t)dst;
}

// Sort key of an occlusion ray: the cube-map cell of its direction from the
// light — face (3 bits) over the Morton code of the cell (u, v) on the face
// (RT_SH_CELLS^2 cells, 0.35 degrees).  Only the order of the occlusion pass
// depends on it, never a result.
__device__ __forceinline__ uint32_t morton_spread(uint32_t x) {  // up to 16 bits spread to the even bits
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
__device__ __forceinline__ uint32_t sh_key(const RtFrameCam& cam, double px, double py, double pz) {
    const float dx = (float)(px - cam.pos[0]), dy = (float)(py - cam.pos[1]), dz = (float)(pz - cam.pos[2]);
    const float ax = __builtin_fabsf(dx), ay = __builtin_fabsf(dy), az = __builtin_fabsf(dz);
    uint32_t face;
    float u, v, m;
    if (ax >= ay && ax >= az) {
        face = dx < 0.f ? 1u : 0u;
        m = ax; u = dy; v = dz;
    } else if (ay >= az) {
        face = dy < 0.f ? 3u : 2u;
        m = ay; u = dx; v = dz;
    } else {
        face = dz < 0.f ? 5u : 4u;
        m = az; u = dx; v = dy;
    }
    const float s = m > 0.f ? 0.5f * (float)RT_SH_CELLS / m : 0.f;
    int iu = (int)((u + m) * s), iv = (int)((v + m) * s);
    iu = iu < 0 ? 0 : iu >= RT_SH_CELLS ? RT_SH_CELLS - 1 : iu;
    iv = iv < 0 ? 0 : iv >= RT_SH_CELLS ? RT_SH_CELLS - 1 : iv;
    return (face << (2 * RT_SH_CELL_BITS)) | morton_spread((uint32_t)iu) | (morton_spread((uint32_t)iv) << 1);
}

// Occlusion record k {p, tri, dst} and its sort key.
__device__ __forceinline__ void q_shadow_store(const PathQs& qs, const RtFrameCam& cam, uint32_t k, double px,
                                               double py, double pz, int32_t tri, uint32_t dst) {
    RT_G double* r = qs.srec + 4 * (size_t)k;
    r[0] = px;
    r[1] = py;
    r[2] = pz;
    r[3] = __longlong_as_double((long long)(((uint64_t)dst << 32) | (uint32_t)tri));
    rt_q_skey(qs)[k] = sh_key(cam, px, py, pz);
}
// Appends the lanes' occlusion records to partition x of srec (the partition
// of the segment's input ray: its capacity covers them; one atomic per wave);
// every lane of the wave calls it, with one x.
__device__ __forceinline__ void q_shadow_append(const PathQs& qs, const RtFrameCam& cam, int b, int x, bool queue,
                                                double px, double py, double pz, int32_t tri, uint32_t dst) {
    const uint64_t em = __ballot(queue);
    if (em == 0) return;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __builtin_ctzll(em);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(qc_sh(qs, b, x), (uint32_t)__builtin_popcountll(em));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader) + (uint32_t)x * qs.pcap;
    if (!queue) return;
    q_shadow_store(qs, cam, base + (uint32_t)__builtin_popcountll(em & ((1ull << lane) - 1ull)), px, py, pz, tri,
                   dst);
}
// ... for one lane (the fall-back kernel's lanes append to their own rays'
// partitions).
__device__ __forceinline__ void q_shadow_append_lane(const PathQs& qs, const RtFrameCam& cam, int b, int x,
                                                     bool queue, double px, double py, double pz, int32_t tri,
                                                     uint32_t dst) {
    if (!queue) return;
    q_shadow_store(qs, cam, atomicAdd(qc_sh(qs, b, x), 1u) + (uint32_t)x * qs.pcap, px, py, pz, tri, dst);
}

// Counting-sort pass over segment b's occlusion records, digit (key >> shift)
// mod 2^BITS: pass 0 reads the appended records' keys (skey) and writes
// (key, record) pairs to spair[0], pass p > 0 reorders spair[(p - 1) & 1]
// into spair[p & 1];
// per-block LDS histograms, one scan, then each block scatters its pairs
// (their order inside a block is the LDS atomics', so a pass is stable only
// up to a block's range).  The passes (lowest digit first) order the
// records by key up to that fuzz: neighbouring pairs are rays of nearly the
// same direction from the light.  Only 4-8 B move per record and pass; the
// occlusion walk gathers the 32-B records through the pairs.
// Block k of RT_SH_BLOCKS takes its share of partition k % parts of the
// appended records (pass 0: RT_SH_BLOCKS / parts blocks per partition), or
// pairs [k n / NB, (k+1) n / NB) of the sorted run (pass 1).
__device__ __forceinline__ void sh_range(const PathQs& qs, int b, int pass, uint32_t k, uint32_t& lo, uint32_t& hi) {
    if (pass == 0) {
        const uint32_t x = k % qs.parts, j = k / qs.parts, nb = RT_SH_BLOCKS / qs.parts;
        const uint32_t n = *qc_sh(qs, b, (int)x);
        lo = x * qs.pcap + (uint32_t)((uint64_t)n * j / nb);
        hi = x * qs.pcap + (uint32_t)((uint64_t)n * (j + 1) / nb);
        return;
    }
    const uint32_t n = sh_total(qs, b);
    lo = (uint32_t)((uint64_t)n * k / RT_SH_BLOCKS);
    hi = (uint32_t)((uint64_t)n * (k + 1) / RT_SH_BLOCKS);
}
// Sorted pairs {key, record} of pass p.
__device__ __forceinline__ RT_G uint2* sh_pairs(const PathQs& qs, int p) {
    return reinterpret_cast<RT_G uint2*>(rt_q_spair(qs, p));
}
// The pass's input element e: its key and record.
__device__ __forceinline__ uint2 sh_input(const PathQs& qs, int pass, uint32_t e) {
    return pass == 0 ? make_uint2(rt_q_skey(qs)[e], e) : sh_pairs(qs, (pass - 1) & 1)[e];
}
template <int BITS>
__global__ void __launch_bounds__(1024) k_sh_hist(PathQs qs, int b, int pass, int shift) {
    constexpr uint32_t BINS = 1u << BITS;
    __shared__ uint32_t h[BINS];
    for (uint32_t i = threadIdx.x; i < BINS; i += 1024) h[i] = 0;
    __syncthreads();
    uint32_t lo, hi;
    sh_range(qs, b, pass, blockIdx.x, lo, hi);
    for (uint32_t e = lo + threadIdx.x; e < hi; e += 1024)
        atomicAdd(&h[(sh_input(qs, pass, e).x >> shift) & (BINS - 1)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < BINS; i += 1024) qs.bhist[(size_t)i * RT_SH_BLOCKS + blockIdx.x] = h[i];
}
// Exclusive scan of bhist in place, bin-major (one block: each thread scans a
// contiguous run, then the runs' totals are scanned in LDS).
template <int BITS>
__global__ void __launch_bounds__(1024) k_sh_scan(PathQs qs) {
    constexpr uint32_t N = (1u << BITS) * RT_SH_BLOCKS, R = N / 1024;
    static_assert(N % 1024 == 0 && R % 4 == 0, "scan runs of whole uint4s");
    __shared__ uint32_t part[1024];
    RT_G uint4* run = reinterpret_cast<RT_G uint4*>(qs.bhist + (size_t)threadIdx.x * R);
    uint32_t sum = 0;
    for (uint32_t k = 0; k < R / 4; k++) {
        const uint4 v = run[k];
        sum += v.x + v.y + v.z + v.w;
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan of the run totals
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t acc = part[threadIdx.x] - sum;
    for (uint32_t k = 0; k < R / 4; k++) {
        uint4 v = run[k];
        const uint32_t a = acc, b2 = a + v.x, c = b2 + v.y, d = c + v.z;
        acc = d + v.w;
        v.x = a;
        v.y = b2;
        v.z = c;
        v.w = d;
        run[k] = v;
    }
}
template <int BITS>
__global__ void __launch_bounds__(1024) k_sh_scatter(PathQs qs, int b, int pass, int shift) {
    constexpr uint32_t BINS = 1u << BITS;
    __shared__ uint32_t cur[BINS];
    for (uint32_t i = threadIdx.x; i < BINS; i += 1024) cur[i] = qs.bhist[(size_t)i * RT_SH_BLOCKS + blockIdx.x];
    __syncthreads();
    uint32_t lo, hi;
    sh_range(qs, b, pass, blockIdx.x, lo, hi);
    RT_G uint2* const out = sh_pairs(qs, pass & 1);
    for (uint32_t e = lo + threadIdx.x; e < hi; e += 1024) {
        const uint2 v = sh_input(qs, pass, e);
        out[atomicAdd(&cur[(v.x >> shift) & (BINS - 1)], 1u)] = v;
    }
}

// The wave-cooperative any-hit walk of 64 occlusion rays that share the light
// as origin (one bin's worth of directions): wave_walk's loop with the
// scalar child records and `ballot`, each lane's interval [0, tmax]; a lane
// stops (its interval emptied) at its first occluder: tri_classify's certain
// class with an upper bound below 0.999 tmax, or the fp64 test of any other
// survivor (lane_occluded's rule, same answer).  The walk ends when every
// lane has stopped or the stack is empty.  Returns the lane's occlusion.
template <int W, bool COUNT>
__device__ __forceinline__ bool wave_anyhit(const RtDevScene& sc, const RtFrameCam& cam, double px, double py,
                                            double pz, bool valid, uint32_t* __restrict__ wstack, uint32_t& w_nodes,
                                            uint32_t& w_tris) {
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
    double len = 0.0;
    Ray32 q;
    float pd;
    {
        const Ray64 r = ray_of(len);
        valid = valid && len > 0.0;
        pd = ray_pad(sc, r);
        q = make_ray32<true>(r, pd);
    }
    const double tmax = len * kShadowScale;
    const float tcert = (float)(tmax * 0.999);
    float tcull = valid ? round_up_f(tmax) : -1.f;
    bool occ = false;
    const uint32_t lsg = (q.ix < 0.f ? 1u : 0u) | (q.iy < 0.f ? 2u : 0u) | (q.iz < 0.f ? 4u : 0u);
    const uint32_t dsg = uni(lsg);
    const int oct = __ballot(valid && lsg != dsg) == 0 ? (int)dsg : 8;
    const f2 nox{-(q.ox + pd) * q.ix, -(q.ox - pd) * q.ix};
    const f2 noy{-(q.oy + pd) * q.iy, -(q.oy - pd) * q.iy};
    const f2 noz{-(q.oz + pd) * q.iz, -(q.oz - pd) * q.iz};
    uint32_t cur = sc.root_ref;
    if (!(cur & RT_LEAF_BIT)) cur |= sc.root_meta << 24;
    {
        float bb[1][6];
        for (int a = 0; a < 6; a++) bb[0][a] = sc.root_box[a];
        uint64_t h[1];
        child_hits<1, -1>(bb, q, nox, noy, noz, tcull, h);
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
                const uint32_t end = first + cnt;
                if (COUNT) w_tris += cnt;
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
                        float tl, tu;
                        // (an occluded lane's class is computed and dropped by
                        // a select; no `continue` in the unrolled chunk loop)
                        int cls = tri_classify(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co, tcull,
                                               tl, tu);
                        cls = tcull >= 0.f ? cls : 0;
                        if (cls != 0) {
                            bool hit = cls == 2 && tu < tcert;
                            if (!hit) {
                                double t, l2;
                                hit = mt64(sc.tri64 + RT_TRI64_DOUBLES * (size_t)k, ray_of(l2), t) && t < tmax;
                            }
                            if (hit) {
                                occ = true;
                                tcull = -1.f;  // this lane enters no box from now on
                            }
                        }
                    }
                }
                if (__ballot(tcull >= 0.f) == 0) break;  // every ray is occluded (or was never valid)
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
    return occ;
}

// Segment b's binned occlusion records, 64 per wave through wave_anyhit; a
// vertex the light sees adds 0.5^b of its colour to its destination's
// radiance (the segment kernel wrote the radiance before this vertex there).
#ifndef RT_SH_WPE
#define RT_SH_WPE 5  // waves per SIMD of k_sh_walk (96 VGPRs): c5 190.3 / 190.4 vs 193.9 / 193.8 ms per pose at 6, 4: 189.9 / 190.4
#endif
template <int W, bool COUNT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_SH_WPE))) k_sh_walk(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, PathQs qs, int b, int src) {
    __shared__ uint32_t wst[4][128];  // one 128-entry node stack per wave
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t n = sh_total(qs, b);
    const RtFrameCam cam = frame_cam(fp, 0);
    uint32_t* wstack = wst[tid >> 6];
    uint32_t occl = 0, cast = 0, w_nodes = 0, w_tris = 0;
    ShPull pl;
    sh_pull_begin(qs, b, true, n, pl);
    uint32_t e0;
    while (sh_pull(qs, b, true, n, pl, e0)) {
        const uint32_t e = e0 + (uint32_t)lane;
        const bool act = e < pl.hi;
        double px = 0.0, py = 0.0, pz = 0.0;
        uint64_t td = 0;
        if (act) {
            const RT_G double* r = qs.srec + 4 * (size_t)sh_pairs(qs, src)[e].y;  // (the sorted pairs' record)
            px = r[0];
            py = r[1];
            pz = r[2];
            td = (uint64_t)__double_as_longlong(r[3]);
        }
        const bool occ = wave_anyhit<W, COUNT>(sc, cam, px, py, pz, act, wstack, w_nodes, w_tris);
        if (act) {
            cast++;
            occl += occ;
        }
        if (act && !occ) {
            const uint32_t tri = (uint32_t)td, dst = (uint32_t)(td >> 32);
            const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)tri;
            const double w = __builtin_ldexp(1.0, -b);
            double c[3];
            shade_at(cam, px, py, pz, T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], c);
            RT_G double* L = q_dst(qs, dst);
            L[0] = L[0] + w * c[0];
            L[1] = L[1] + w * c[1];
            L[2] = L[2] + w * c[2];
        }
    }
    if (fp.counters) {
        wave_add<24>(fp.counters + 24, cast);
        wave_add<24>(fp.counters + 25, occl);
        if (COUNT && lane == 0) {  // (wave-uniform: the walk's node steps and triangle records, once per wave)
            atomicAdd(&fp.counters[26], (unsigned long long)w_nodes);
            atomicAdd(&fp.counters[27], (unsigned long long)w_tris);
        }
    }
}

// Fall-back entries: the queue slot (segment 0: the path) | kQFromPass0 when
// the walk's list overflowed (trace_core from pass 0), alone when the winner
// was invisible (from pass 1).
constexpr uint32_t kQFromPass0 = 0x80000000u;

// Primary segments.  PACK (64 % spp == 0): a unit is every sample of 64 / spp
// pixels (lane = pixel * spp + sample); else a unit is 8 x 8 pixels of one
// sample (unit = sample * tiles + tile).  PRIM: the wave-cooperative walk
// (8-wide trees whose stack bound fits 128 entries), else per lane.
// (PRIM: the per-lane stack is not used; S = 1 leaves the LDS to the wave
// stacks (row 0) and the candidate lists, 10 KB per block)
#ifndef RT_QP_WPE
#define RT_QP_WPE 6  // waves per SIMD of k_q_primary (wave-walked)
#endif
#ifndef RT_QP_CLAIM
#define RT_QP_CLAIM 1  // units claimed per atomic by k_q_primary
#endif
// Phase timing builds (never shipped; results are wrong): 1 = the primary
// kernel stops after the walk, 2 = after the exact resolve (its tcull /
// winner go to hit_id so the work stays live).
#ifndef RT_QP_DIAG
#define RT_QP_DIAG 0
#endif
template <int W, int S, bool COUNT, bool PACK, bool PRIM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PRIM ? RT_QP_WPE : RT_PATHS_WPE))) k_q_primary(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux,
                                                                 PathQs qs, uint32_t frame, int bounces) {
    static_assert(!PRIM || (W == 8 && RT_PATHS_DEFER), "wave-walked primaries: 8-wide deferred paths");
    __shared__ uint2 lds[S][256];
    __shared__ uint2 pcand[RT_PATHS_K][256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int spp = fp.spp;
    int tw = 8, th = 8;
    if constexpr (PACK) {
        const int P = 64 / spp;
        tw = 1;
        while (tw * tw < P) tw <<= 1;
        th = P / tw;
    }
    const int tiles_x = (fp.W + tw - 1) / tw;
    const int tiles = tiles_x * ((fp.nrows + th - 1) / th);
    const int units = PACK ? tiles : tiles * spp;
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const RtFrameCam cam = frame_cam(fp, 0);
    for (;;) {
        // RT_QP_CLAIM consecutive units per claim (one atomic on the shared
        // counter per claim, not per unit)
        int u0 = 0;
        if (lane == 0) u0 = (int)atomicAdd(qc_pull(qs, 0, 0), (uint32_t)RT_QP_CLAIM);
        u0 = __shfl(u0, 0);
        if (u0 >= units) break;
        const int u1 = u0 + RT_QP_CLAIM < units ? u0 + RT_QP_CLAIM : units;
        for (int unit = u0; unit < u1; unit++) {
        int i, r, s;
        if constexpr (PACK) {
            const int pl = lane / spp;
            s = lane & (spp - 1);
            i = (unit % tiles_x) * tw + pl % tw;
            r = (unit / tiles_x) * th + pl / tw;
        } else {
            s = unit / tiles;
            const int t = unit - s * tiles;
            i = (t % tiles_x) * 8 + (lane & 7);
            r = (t / tiles_x) * 8 + (lane >> 3);
        }
        const bool valid = i < fp.W && r < fp.nrows;
        const int iv = valid ? i : 0, rv = valid ? r : 0;
        const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, rv);
        const uint32_t seed = path_seed(frame, (uint32_t)j * (uint32_t)fp.W + (uint32_t)iv, (uint32_t)s);
        RtFrameCam c1 = cam;
        c1.ox = path_u(seed, 0);
        c1.oy = path_u(seed, 1);
        const Ray64 ray = gen_ray<false>(fp, c1, iv, j);
        LaneCounts lc;
        Win win;
        // the primary ray's walk: wave-cooperative (PRIM) or per lane; a lane
        // whose list overflowed or whose winner the reference cannot see goes
        // to k_q_fallback (segment 0) with its ray
        float tcull;
        int nc;
        bool over;
        {
            const float pd = ray_pad(sc, ray);
            const Ray32 q0 = make_ray32<true>(ray, pd);
            const float tsl = round_up_f(0x1p-40 * ((double)q0.co + 1.0));
            if constexpr (PRIM) {
                uint32_t* wstack = reinterpret_cast<uint32_t*>(&lds[0][tid & ~63]);  // 128 u32 of this wave's row
                wave_walk<W, RT_PATHS_K, COUNT>(sc, fp, q0, pd, tsl, valid, wstack, pcand, tid, lc, tcull, nc, over);
            } else if (valid) {
                lane_walk<W, S, RT_PATHS_K, COUNT, W == 8 && RT_QNODES>(sc, q0, tsl, st, pcand, lc, tcull, nc, over);
            }
        }
        if constexpr (RT_QP_DIAG == 1) {
            if (valid && fp.hit_id)
                fp.hit_id[((uint32_t)rv * (uint32_t)fp.W + (uint32_t)iv) * (uint32_t)spp + (uint32_t)s] =
                    __float_as_uint(tcull) + (uint32_t)nc + (over ? 1u : 0u);
            continue;
        }
        bool fall = false;
        if (valid) {
            fall = over;
            if (!over)
                fall = resolve_cands<COUNT>(sc, with_inv(ray), [&](int c) { return pcand[c][tid]; }, nc, tcull, win,
                                            lc) != 0;
        }
        const uint32_t path = ((uint32_t)rv * (uint32_t)fp.W + (uint32_t)iv) * (uint32_t)spp + (uint32_t)s;
        if constexpr (RT_QP_DIAG == 2) {
            if (valid && fp.hit_id) fp.hit_id[path] = (uint32_t)win.tri + (fall ? 1u : 0u);
            continue;
        }
        if (fall) {  // the ray to the fall-back list: q[1] (free until segment 1) holds it
            RT_G double* p = q_entry(qs, 1, atomicAdd(qc_fb(qs, 0), 1u));
            p[0] = ray.ox;
            p[1] = ray.oy;
            p[2] = ray.oz;
            p[3] = ray.dx;
            p[4] = ray.dy;
            p[5] = ray.dz;
            p[9] = __longlong_as_double((long long)(path | (over ? kQFromPass0 : 0u)));
        }
        bool emit = false;
        Ray64 nr;
        double px = 0.0, py = 0.0, pz = 0.0;
        uint32_t hit = 0, sc0 = 0, so0 = 0;
        if (valid && !fall) {
            if (win.tri >= 0) q_bounce(sc, fp, frame, 0, bounces, ray, win, path, px, py, pz, emit, nr);
            Best hb;
            hb.dist = win.dist;
            hb.rank = win.rank;
            hb.tri = win.tri;
            hb.px = px;
            hb.py = py;
            hb.pz = pz;
            store_sample(fp, path, hb, shade_of(sc, win.tri));
            hit = win.tri >= 0;
        }
        const uint32_t slot = q_append(qs, 0, 0, 0, emit, nr, path);  // (one partition: qs.parts = 1)
        if (valid && !fall) {
            bool qd;
            uint32_t dst;
            q_light<W, S, 0>(sc, qs, cam, 0, nullptr, win.tri, px, py, pz, emit, 0, slot, path, st, sc0, so0, qd, dst);
        }
        wave_add<13>(fp.hit_count, hit);
        if (fp.counters) wave_add<1>(fp.counters, valid ? 1u : 0u);
        if (COUNT && fp.counters) {
            wave_add<24>(fp.counters + 1, lc.nodes);
            wave_add<24>(fp.counters + 6, lc.pre);
            wave_add<24>(fp.counters + 2, lc.tris);
            wave_add<24>(fp.counters + 3, lc.chain);
        }
        }
    }
}

// The packed packet walk (k_trace_packet<…, PATHS = true>, packet_kernel.h)
// as the primary segment: sample s of pixel (i, r) takes the jittered
// sub-pixel offset of k_q_primary — draws 0 and 1 of the path's hash.
template <int W>
__device__ void q_primary_offset(args_p A, int s, int i, int r, double& ox, double& oy) {
    A = launder(A);
    const int Wd = kword(&A->fp.W);
    const int j = rt_image_row(kword(&A->fp.row0), kword(&A->fp.row_stride), kword(&A->fp.band), r);
    const uint32_t seed = path_seed(kword(&A->frame), (uint32_t)j * (uint32_t)Wd + (uint32_t)i, (uint32_t)s);
    ox = path_u(seed, 0);
    oy = path_u(seed, 1);
}

// Its primary vertex, k_q_primary's epilogue operation for operation: the
// sample's outputs, the first bounce ray appended to queue 0 (compacted, one
// atomic per wave) with the vertex colour as its radiance, or — when the
// exact resolve could not certify the lane's winner (redo: 1 a list
// overflow, 2 a winner the reference tree cannot see) — the ray on segment
// 0's fall-back list for k_q_fallback.  out: the exact winner with its hit
// point fl(o + d t); pre: the fp64 ray (o, d).  Every lane of the wave that
// traced a valid sample calls it (q_append is wave-wide).  Returns 1 for a
// hit resolved here (the pose's hit count).
template <int W, bool COUNT>
__device__ uint32_t q_primary_vertex(args_p A, int s, int i, int r, bool valid, uint32_t redo, const Best& out,
                                     const Ray64& pre) {
    A = launder(A);
    const PathQs qs = kload(&A->qs);
    const int Wd = kword(&A->fp.W), spp = kword(&A->fp.spp);
    const uint32_t path = ((uint32_t)r * (uint32_t)Wd + (uint32_t)i) * (uint32_t)spp + (uint32_t)s;
    const bool fall = valid && redo != 0;
    if (fall) {  // the ray to the fall-back list: q[1] (free until segment 1) holds it
        RT_G double* p = q_entry(qs, 1, atomicAdd(qc_fb(qs, 0), 1u));
        p[0] = pre.ox;
        p[1] = pre.oy;
        p[2] = pre.oz;
        p[3] = pre.dx;
        p[4] = pre.dy;
        p[5] = pre.dz;
        p[9] = __longlong_as_double((long long)(path | (redo == 1 ? kQFromPass0 : 0u)));
    }
    const bool done = valid && !fall;
    bool emit = false;
    Ray64 nr{};
    const RtDevScene sc = kload(&launder(A)->sc);
    if (done && out.tri >= 0) {  // q_bounce with the hit point the resolve computed
        emit = 0 < kword(&A->bounces);
        if (emit) {
            const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)out.tri;
            const int j = rt_image_row(kword(&A->fp.row0), kword(&A->fp.row_stride), kword(&A->fp.band), r);
            const uint32_t seed = path_seed(kword(&A->frame), (uint32_t)j * (uint32_t)Wd + (uint32_t)i, (uint32_t)s);
            bounce_dir(T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], pre.dx, pre.dy, pre.dz,
                       path_u(seed, 2u), path_u(seed, 3u), nr.dx, nr.dy, nr.dz);
            nr.ox = out.px;
            nr.oy = out.py;
            nr.oz = out.pz;
        }
    }
    if (done) store_sample(kload(&launder(A)->fp), path, out, shade_of(sc, out.tri));
    // the partition of the tile's XCD queue (k_trace_packet: xq = block % RT_QUEUES)
    const uint32_t slot = q_append(qs, 0, (int)(blockIdx.x % (uint32_t)qs.parts), 0, emit, nr, path);
    if (done) {  // q_light of vertex 0: its colour always counts (no occlusion ray)
        double L[3] = {0.0, 0.0, 0.0};
        if (out.tri >= 0) {
            const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)out.tri;
            const double w = __builtin_ldexp(1.0, 0);
            double c[3];
            shade_at(frame_cam(kload(&launder(A)->fp), 0), out.px, out.py, out.pz, T[RT_T64_NORMAL],
                     T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], c);
            L[0] = L[0] + w * c[0];
            L[1] = L[1] + w * c[1];
            L[2] = L[2] + w * c[2];
        }
        RT_G double* f = emit ? q_entry(qs, 0, slot) + 6 : qs.Lfin + 3 * (size_t)path;
        f[0] = L[0];
        f[1] = L[1];
        f[2] = L[2];
    }
    return done && out.tri >= 0 ? 1u : 0u;
}

// Segment b (1 .. bounces) over queue (b - 1) & 1.  Fall-back entries: the
// queue slot | 0x80000000 when the walk's list overflowed (trace_core from
// pass 0), the slot alone when the winner was invisible (from pass 1).
#if RT_Q_WPE > 0
#define RT_Q_ATTR __attribute__((amdgpu_waves_per_eu(RT_Q_WPE)))
#else
#define RT_Q_ATTR
#endif
// Phase timing builds of the segment kernel (never shipped; results are
// wrong, and later segments see empty queues): 1 = each ray stops after its
// walk, 2 = after the exact resolve.
#ifndef RT_QS_DIAG
#define RT_QS_DIAG 0
#endif
template <int W, int S, int K, bool COUNT, int SH>
__global__ void __launch_bounds__(256) RT_Q_ATTR k_q_segment(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux,
                                                             PathQs qs, uint32_t frame, int b, int bounces) {
    __shared__ uint2 lds[S][256];
    __shared__ uint2 cand[K][256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int qin = (b - 1) & 1, qout = b & 1;
    // the wave's partition: its XCD's (blocks are dealt to the XCDs round-
    // robin), then, once that is drained, the others in turn (their counters
    // then see a few cross-XCD atomics at the segment's tail)
    const int parts = (int)qs.parts;
    int x = (int)(blockIdx.x % (uint32_t)parts), left = parts;
    uint32_t n = *qc_emit(qs, b - 1, x);
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const RtFrameCam cam = frame_cam(fp, 0);
    uint32_t segs = 0, sh_cast = 0, sh_occ = 0;
    LaneCounts shc;  // COUNT, SH 1: the occlusion walks' fetches
    LaneCounts tot;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(qc_pull(qs, b, x), 64u);
        base = (uint32_t)__shfl((int)base, 0);
        if (base >= n) {
            if (--left == 0) break;
            x = x + 1 == parts ? 0 : x + 1;
            n = *qc_emit(qs, b - 1, x);
            continue;
        }
        const uint32_t e = (uint32_t)x * qs.pcap + base + (uint32_t)lane;
        const bool act = base + (uint32_t)lane < n;
        bool emit = false, fall = false;
        Ray64 nr;
        Win win;
        win.tri = -1;
        double px = 0.0, py = 0.0, pz = 0.0;
        uint32_t path = 0;
        if (act) {
            float tcull;
            int nc;
            bool over;
            {
                // only the fp32 view of the ray lives through the walk
                Ray64 ray;
                double L[3];
                q_load(qs, qin, e, ray, L, path);
                const float pd = ray_pad(sc, ray);
                const Ray32 q = make_ray32<true>(ray, pd);
                const float tsl = round_up_f(0x1p-40 * ((double)q.co + 1.0));
                LaneCounts lc;
                lane_walk<W, S, K, COUNT, W == 8 && RT_QNODES>(sc, q, tsl, st, cand, lc, tcull, nc, over);
                if (COUNT) {
                    tot.nodes += lc.nodes;
                    tot.wnodes += lc.wnodes;
                    tot.wtris += lc.wtris;
                    tot.pre += lc.pre;
                }
            }
            if constexpr (RT_QS_DIAG == 1) {  // phase timing: the walk alone
                qs.Lfin[3 * (size_t)e] = (double)tcull + nc + (over ? 1.0 : 0.0);
                continue;
            }
            Ray64 ray;
            double L[3];
            q_load(qs, qin, e, ray, L, path);  // (the entry again: L1 / L2)
            uint32_t fe = e | kQFromPass0;
            fall = over;
            if (!over) {
                fe = e;
                LaneCounts lc;
                fall = resolve_cands<COUNT>(sc, with_inv(ray), [&](int c) { return cand[c][tid]; }, nc, tcull, win,
                                            lc) != 0;
                if (COUNT) {
                    tot.tris += lc.tris;
                    tot.chain += lc.chain;
                }
            }
            segs++;
            if constexpr (RT_QS_DIAG == 2) {  // phase timing: the walk and the exact resolve
                qs.Lfin[3 * (size_t)e] = win.t + win.tri + (fall ? 1.0 : 0.0);
                continue;
            }
            if constexpr (RT_Q_NR_LDS != 0) {
                // the vertex (and below, the bounce direction) wait out the
                // bounce direction's divisions and q_append's atomic in the
                // lane's LDS stack ring (free once the walk is over: entries
                // 0-5 of its column) instead of in registers — at 80 VGPRs the
                // compiler spilled them to scratch there, once per ray
                lds[0][tid] = dbits(0.0);
                lds[1][tid] = dbits(0.0);
                lds[2][tid] = dbits(0.0);
            }
            if (fall) {
                qs.fb[qin * (size_t)qs.cap + atomicAdd(qc_fb(qs, b), 1u)] = fe;
            } else if (win.tri >= 0) {
                q_bounce_ring<RT_Q_NR_LDS != 0>(sc, fp, frame, b, bounces, ray, win, path, px, py, pz, emit, nr, lds,
                                                tid);
            }
        }
        if constexpr (RT_Q_NR_LDS != 0) opaque_regs();
        const uint32_t slot = q_append_ring<RT_Q_NR_LDS != 0>(qs, qout, x, b, emit, nr, path, lds, tid);
        if constexpr (RT_Q_NR_LDS != 0) {
            if (act) {
                px = bitsd(lds[0][tid]);
                py = bitsd(lds[1][tid]);
                pz = bitsd(lds[2][tid]);
            }
        }
        bool qd = false;
        uint32_t dst = 0;
        if (act && !fall)
            q_light<W, S, SH, COUNT>(sc, qs, cam, b, q_entry(qs, qin, e) + 6, win.tri, px, py, pz, emit, qout, slot, path, st,
                              sh_cast, sh_occ, qd, dst, &shc);
        if constexpr (SH >= 2) q_shadow_append(qs, cam, b, x, qd, px, py, pz, win.tri, dst);
    }
    if (fp.counters) {
        wave_add<24>(fp.counters, segs);
        if (SH == 1) {
            wave_add<24>(fp.counters + 24, sh_cast);
            wave_add<24>(fp.counters + 25, sh_occ);
            if (COUNT) {
                wave_add<28>(fp.counters + 28, shc.nodes);
                wave_add<28>(fp.counters + 30, shc.wnodes);
                wave_add<28>(fp.counters + 31, shc.wtris);
                wave_add<28>(fp.counters + 29, shc.pre);
            }
        }
        if (COUNT) {
            wave_add<28>(fp.counters + 1, tot.nodes);
            wave_add<28>(fp.counters + 30, tot.wnodes);
            wave_add<28>(fp.counters + 31, tot.wtris);
            wave_add<28>(fp.counters + 6, tot.pre);
            wave_add<28>(fp.counters + 2, tot.tris);
            wave_add<28>(fp.counters + 3, tot.chain);
        }
    }
}

// Queued occlusion records walked per lane, in the order the segment kernel
// appended them (RT_SHADOW_RAYS=rec: no binning): lane_occluded in a lean
// kernel of its own.
#ifndef RT_SL_WPE
#define RT_SL_WPE 6
#endif
template <int W, int S, bool COUNT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_SL_WPE)))
k_sh_lane(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, PathQs qs, int b) {
    __shared__ uint2 lds[S][256];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const RtFrameCam cam = frame_cam(fp, 0);
    uint32_t occl = 0, cast = 0;
    LaneCounts shc;
    ShPull pl;
    sh_pull_begin(qs, b, false, 0, pl);
    uint32_t e0;
    while (sh_pull(qs, b, false, 0, pl, e0)) {
        const uint32_t e = e0 + (uint32_t)lane;
        if (e >= pl.hi) continue;
        const RT_G double* r = qs.srec + 4 * (size_t)e;
        const double px = r[0], py = r[1], pz = r[2];
        const bool occ = lane_occluded<W, S, W == 8 && RT_QNODES, COUNT>(sc, cam, px, py, pz, st, &shc);
        cast++;
        occl += occ;
        if (!occ) {
            const uint64_t td = (uint64_t)__double_as_longlong(r[3]);
            const uint32_t tri = (uint32_t)td, dst = (uint32_t)(td >> 32);
            const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)tri;
            const double w = __builtin_ldexp(1.0, -b);
            double c[3];
            shade_at(cam, px, py, pz, T[RT_T64_NORMAL], T[RT_T64_NORMAL + 1], T[RT_T64_NORMAL + 2], c);
            RT_G double* L = q_dst(qs, dst);
            L[0] = L[0] + w * c[0];
            L[1] = L[1] + w * c[1];
            L[2] = L[2] + w * c[2];
        }
    }
    if (fp.counters) {
        wave_add<24>(fp.counters + 24, cast);
        wave_add<24>(fp.counters + 25, occl);
        if (COUNT) {
            wave_add<28>(fp.counters + 28, shc.nodes);
            wave_add<28>(fp.counters + 30, shc.wnodes);
            wave_add<28>(fp.counters + 31, shc.wtris);
            wave_add<28>(fp.counters + 29, shc.pre);
        }
    }
}

// Segment b's fall-back list: trace_core, then the same vertex epilogue.
// Grid-stride with the same trip count for every lane of a wave (the append
// ballots).
template <int W, int S, bool COUNT, int SH>
__global__ void __launch_bounds__(256) k_q_fallback(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux, PathQs qs,
                                                    uint32_t frame, int b, int bounces) {
    __shared__ uint2 lds[S][256];
    const int tid = threadIdx.x;
    // segment 0: the primary rays k_q_primary left in q[1]; segment b > 0:
    // the listed entries of queue (b - 1) & 1
    const int qin = b == 0 ? 1 : (b - 1) & 1, qout = b & 1;
    const uint32_t n = *qc_fb(qs, b);
    LaneStack<S> st;
    st.attach(lds, aux, tid);
    const RtFrameCam cam = frame_cam(fp, 0);
    const uint32_t stride = gridDim.x * 256u;
    const uint32_t iters = (n + stride - 1) / stride;
    uint32_t sh_cast = 0, sh_occ = 0;
    LaneCounts tot, shc;
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t k = it * stride + blockIdx.x * 256u + (uint32_t)tid;
        bool emit = false;
        Ray64 nr;
        Win win;
        win.tri = -1;
        double px = 0.0, py = 0.0, pz = 0.0;
        uint32_t path = 0, e = 0, hit = 0;
        if (k < n) {
            Ray64 ray;
            double L[3];
            bool pass0;
            if (b == 0) {
                e = k;
                q_load(qs, qin, e, ray, L, path);
                pass0 = (path & kQFromPass0) != 0;
                path &= ~kQFromPass0;
            } else {
                const uint32_t fe = qs.fb[qin * (size_t)qs.cap + k];
                e = fe & ~kQFromPass0;
                pass0 = (fe & kQFromPass0) != 0;
                q_load(qs, qin, e, ray, L, path);
            }
            auto ray_of = [&]() { return with_inv(ray); };
            win = trace_core<W, S, COUNT>(sc, ray_of, ray_pad(sc, ray), st, pass0 ? 0 : 1, tot);
            if (win.tri >= 0) q_bounce(sc, fp, frame, b, bounces, ray, win, path, px, py, pz, emit, nr);
            if (b == 0) {  // the primary segment's per-sample outputs
                Best hb;
                hb.dist = win.dist;
                hb.rank = win.rank;
                hb.tri = win.tri;
                hb.px = px;
                hb.py = py;
                hb.pz = pz;
                store_sample(fp, path, hb, shade_of(sc, win.tri));
                hit = win.tri >= 0;
            }
        }
        // (into the partition the ray came from: its capacity covers it)
        const int x = k >= n ? 0 : b == 0 ? q_primary_part(qs, fp, path) : (int)(e / qs.pcap);
        const uint32_t slot = q_append_lane(qs, qout, x, b, emit, nr, path);
        if (b == 0) wave_add<1>(fp.hit_count, hit);
        bool qd = false;
        uint32_t dst = 0;
        if (k < n)
            q_light<W, S, SH, COUNT>(sc, qs, cam, b, b == 0 ? nullptr : q_entry(qs, qin, e) + 6, win.tri, px, py, pz, emit,
                              qout, slot, path, st, sh_cast, sh_occ, qd, dst, &shc);
        if constexpr (SH >= 2) q_shadow_append_lane(qs, cam, b, x, qd, px, py, pz, win.tri, dst);
    }
    if (fp.counters) {
        if (SH == 1) {
            wave_add<24>(fp.counters + 24, sh_cast);
            wave_add<24>(fp.counters + 25, sh_occ);
            if (COUNT) {
                wave_add<28>(fp.counters + 28, shc.nodes);
                wave_add<28>(fp.counters + 30, shc.wnodes);
                wave_add<28>(fp.counters + 31, shc.wtris);
                wave_add<28>(fp.counters + 29, shc.pre);
            }
        }
        if (COUNT) {
            wave_add<28>(fp.counters + 1, tot.nodes);
            wave_add<28>(fp.counters + 30, tot.wnodes);
            wave_add<28>(fp.counters + 31, tot.wtris);
            wave_add<28>(fp.counters + 2, tot.tris);
            wave_add<28>(fp.counters + 3, tot.chain);
        }
    }
}

// Pixel colours: the paths' final radiance summed in sample order from 0.0
// (k_paths' acc), then saveScreen's cast of the mean.
__global__ void __launch_bounds__(256) k_q_accum(RtFrameParams fp, PathQs qs) {
    const uint32_t pix = blockIdx.x * 256u + threadIdx.x;
    if (pix >= (uint32_t)fp.W * (uint32_t)fp.nrows) return;
    double acc[3] = {0.0, 0.0, 0.0};
    const RT_G double* f = qs.Lfin + 3 * (size_t)pix * (size_t)fp.spp;
    for (int s = 0; s < fp.spp; s++) {
        acc[0] = acc[0] + f[3 * s];
        acc[1] = acc[1] + f[3 * s + 1];
        acc[2] = acc[2] + f[3 * s + 2];
    }
    store_rgb(fp, pix, acc);
}
