// Wave-cooperative ("packet") exact traversal kernel for gfx950.
// Included by render.hip inside its anonymous namespace (uses Ray32, Win,
// make_ray32, trace_exact and the rtk helpers).
//
// The 64 rays of one 8x8 pixel tile walk the tree together.  The current
// node is wave-uniform, so its child records come in through the scalar data
// path (s_load_dwordx8 per 32-B child, once per wave) instead of 64 per-lane
// copies through the vector memory pipe; every lane slab-tests its own ray
// against each child and `ballot` says whether any lane needs the child.  The
// wave continues into the hit child nearest along the node's sort axis and
// pushes the others on a wave-uniform stack of node refs in LDS.
//
// No per-child lane masks are kept: all lanes of a wave execute every child
// test anyway, and a lane that missed a parent box misses its children too
// (real child boxes lie inside the parent box and outward rounding to fp32 is
// monotone), so re-testing with every lane returns the same answers.  Lanes
// outside the image carry tcull = -1, which fails every test.
//
// The walk itself is fp32 only.  Leaf triangles go through tri_classify:
// rejected, "certain" (the fp64 test provably passes and its t is bounded
// above, so the culling distance tightens at once) or "borderline".  Both
// kinds of survivor are appended to the lane's candidate list in LDS (index +
// lower bound of t); past K entries they go to a chunk of a shared overflow
// pool in HBM (allocated on first need, one atomic per overflowing lane).
//
// After the walk the tile's own lanes resolve their lists in place (FUSED):
// the exact fp64 Moller-Trumbore of each survivor, the (distance,
// visit rank) minimum, the re-verification of the winner's reference
// ancestor chain, shading and the output stores — one pass, no candidate
// lists through HBM.  With spp > 1 each sample is resolved the same way and
// k_average forms the pixels from the samples' colours.  A
// pixel whose list overflowed past its pool chunk, or whose winner the
// reference could not see, is appended to the redo list and finished by
// k_fixup (the per-lane kernel).
#pragma once

struct __attribute__((aligned(32))) ChildRec {  // 32-B child record (rt_device.h)
    float lx, hx, ly, hy, lz, hz;
    uint32_t ref, pad;
};
typedef const __attribute__((address_space(4))) float* cfloat_p;
typedef float f2 __attribute__((ext_vector_type(2)));
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

// v_writelane_b32: lane L of `v` := uniform `x`
template <int L>
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(L));
    return v;
}

// Bit c set iff any lane of hm[c] is set: two SALU per child, SCC = (mask !=
// 0) then m = 2m + SCC (children from the last down, so child c lands in bit
// c); the compiler would otherwise route each uniform bool through a VGPR.
template <int W>
__device__ __forceinline__ uint32_t any_mask(const uint64_t (&hm)[W]) {
    uint32_t m = 0;
#pragma unroll
    for (int c = W - 1; c >= 0; c--)
        asm("s_cmp_lg_u64 %1, 0\n\ts_addc_u32 %0, %0, %0" : "+s"(m) : "s"(hm[c]) : "scc");
    return m;
}

// Lane c of the result: child c's ref (eight v_writelane from the scalar
// records: measured faster than one vector load of the refs).
template <int W>
__device__ __forceinline__ uint32_t lanes_of(const uint32_t (&ref)[W]) {
    uint32_t v = 0;
    [&]<int... L>(std::integer_sequence<int, L...>) { ((v = writelane<L>(v, ref[L])), ...); }(
        std::make_integer_sequence<int, W>{});
    return v;
}

constexpr uint32_t kRedoPass1 = 0x80000000u;  // redo entry: start directly with the inline-verifying pass
// An empty redo-list entry.  The list is all kRedoEmpty between launches
// (whoever takes an entry resets it), so a wave that takes entries inside
// the launch (packet_exit) can tell one whose store has not landed yet; no
// entry is kRedoEmpty (launch pixels < 2^31).  Entries are swapped in and out
// with device-scope atomics, performed at the memory side, so a reader on
// another XCD sees them while the launch runs.
constexpr uint32_t kRedoEmpty = 0xFFFFFFFFu;
__device__ __forceinline__ void redo_put(const RtLaunchAux& aux, uint32_t v) {
    const uint32_t slot = atomicAdd(aux.tile_ctr + RT_REDO_COUNT, 1u);
    if (slot < aux.redo_cap) (void)atomicExch(aux.redo + slot, v);
}
// triangle records fetched per scalar round trip (walk-tree leaves hold ~2:
// 2 measured 2% faster than 4)
constexpr int kLeafChunk = 2;
constexpr uint32_t kCandDropped = 0x80;  // cand_cnt flag: candidates were dropped (bound in cand_drop)
constexpr uint32_t kCandSpilled = 0x40;  // cand_cnt flag: entries in an overflow pool chunk (cand_ovf)
constexpr uint32_t kCandCount = 0x3F;    // cand_cnt: entries in slots [0, count)
// spp > 1 with the fused resolve: cand_cnt holds each sample's status for
// k_average (bit 0: a hit; kSampRedo: not resolved, the pixel goes to k_fixup)
// and cand the sample's colour (3 doubles at 3 * sample pixel)
constexpr uint32_t kSampRedo = 0x80;
constexpr uint32_t kNoChunk = 0xFFFFFFFFu;   // lane has no overflow chunk (yet)
constexpr uint32_t kPoolDry = 0xFFFFFFFEu;   // the pool ran out: drop with a certified bound
static_assert(kLeafChunk <= RT_TRI32_PAD, "tri32 padding must cover a leaf chunk");
static_assert((RT_MAX_TRIS + (uint64_t)RT_TRI32_PAD) * 48u < (1ull << 32), "tri32 byte offsets are 32-bit");

// Forces uniform values to be materialised (their loads waited on) here, so
// a chunk's loads are all in flight before the first use.
__device__ __forceinline__ void pin_s(const float4& a, const float4& b, const float4& c) {
    asm volatile("" ::"s"(a.x), "s"(a.y), "s"(a.z), "s"(a.w), "s"(b.x), "s"(b.y), "s"(b.z), "s"(b.w), "s"(c.x),
                 "s"(c.y), "s"(c.z), "s"(c.w));
}

// RT_PROFILE=1 (a measurement build, never shipped): the timed kernel adds
// shader-clock cycles per phase of each tile to the counters (18: ray set-up,
// 19: node steps, 20: leaf steps, 21: resolve and stores, 22: tiles, 23:
// whole tiles; tools/phase_profile.py reads them with rt_diag_raw).  The
// s_memtime reads cost some overlap; the proportions are what it is for.
#ifndef RT_PROFILE
#define RT_PROFILE 0
#endif
constexpr bool kProfile = RT_PROFILE != 0;
__device__ __forceinline__ uint64_t prof_clock() {
    if constexpr (kProfile) return (uint64_t)__builtin_amdgcn_s_memtime();
    return 0;
}

// Keep the tile set-up's fp64 ray direction (6 VGPRs) through the walk for
// the resolve instead of generating it again there (a square root and a
// division per ray).
#ifndef RT_KEEP_DIR
#define RT_KEEP_DIR 1
#endif
constexpr bool kKeepDir = RT_KEEP_DIR != 0;

// Load entry 0's shading fields with its Moller-Trumbore part (resolve_list).
#ifndef RT_SPEC_WIN
#define RT_SPEC_WIN 0
#endif
constexpr bool kSpecWin = RT_SPEC_WIN != 0;


#ifndef RT_PIN_REC
#define RT_PIN_REC 1
#endif
// Wave priority (s_setprio) outside the walk: a wave's tile epilogue (the
// fp64 resolve, shading, stores), the next tile's claim and its ray set-up
// run at RT_EPI_PRIO, the walk at 0, so the SIMD's arbiter issues those
// phases ahead of the other waves' node steps.  One box, two pairs: 17.09 /
// 17.10 vs 16.65 / 16.71 Grays/s (+2.5%); the resolve alone raised (to the
// next tile's start): +1.4% at levels 1-3; the walk raised instead: -3.7%
// (DESIGN.md §7).  0: off.
#ifndef RT_EPI_PRIO
#define RT_EPI_PRIO 2
#endif
// ... and the walk's leaf visits (the triangle records' loads and the fp32
// filter of every lane) at RT_LEAF_PRIO, its node steps at 0: 17.48 / 17.57
// vs 17.01 / 16.99 Grays/s (+3.1%, two pairs on one box).
#ifndef RT_LEAF_PRIO
#define RT_LEAF_PRIO 1
#endif
__device__ __forceinline__ void pin_rec(const ChildRec& r) {
    if constexpr (RT_PIN_REC)
        asm volatile("" ::"s"(r.lx), "s"(r.hx), "s"(r.ly), "s"(r.hy), "s"(r.lz), "s"(r.hz), "s"(r.ref), "s"(r.pad));
}

// Lane-private candidate list: entry c of lane l at cand[c * 64 + l]
// ({triangle, bits of t lower bound}; consecutive lanes -> consecutive 8-B
// words, conflict-free ds_read/write_b64).
// List full after compaction: keep the K entries with the smallest t lower
// bound among the list and the new candidate; returns the bound dropped.
template <int K>
__device__ __forceinline__ float keep_nearest(uint2* __restrict__ cand, int lane, uint32_t k, float tl) {
    int far_c = 0;
    float far_t = __uint_as_float(cand[lane].y);
    for (int c = 1; c < K; c++) {
        const float t = __uint_as_float(cand[c * 64 + lane].y);
        if (t > far_t) { far_t = t; far_c = c; }
    }
    if (tl >= far_t) return tl;
    cand[far_c * 64 + lane] = make_uint2(k, __float_as_uint(tl));
    return far_t;
}

template <int K>
__device__ __forceinline__ int compact_candidates(uint2* __restrict__ cand, int lane, float tcull) {
    int m = 0;
    for (int c = 0; c < K; c++) {
        const uint2 e = cand[c * 64 + lane];
        if (__uint_as_float(e.y) <= tcull) {
            cand[m * 64 + lane] = e;
            m++;
        }
    }
    return m;
}

// Kernel arguments.  Each workgroup copies the argument block from the
// kernarg segment into LDS once; copies of the parameter structs are then
// taken from a laundered LDS pointer right where they are needed (ray
// set-up, resolve), so the compiler can neither keep ~60 SGPRs of frame and
// scene constants alive across the walk (the walk needs the SGPRs for the
// child records of a whole node in flight) nor re-read the kernarg segment
// (host-coherent memory, far slower) per tile.
// Unpacked tiles: RT_TILE_W x (64 / RT_TILE_W) pixels of one frame per wave
// (tuning knob; 8 x 8 by default).
#ifndef RT_TILE_W
#define RT_TILE_W 8
#endif
static_assert(RT_TILE_W >= 1 && RT_TILE_W <= 64 && (RT_TILE_W & (RT_TILE_W - 1)) == 0, "tile width: a power of two");
struct PacketArgs {
    RtDevScene sc;
    RtFrameParams fp;
    RtLaunchAux aux;
    // PATHS (queue_paths.h): the queued path tracer's workspace, the hash's
    // frame number and the bounce segments per path
    PathQs qs;
    uint32_t frame;
    int32_t bounces;
};
static_assert(sizeof(PacketArgs) % 4 == 0, "argument block is copied as words");
// Measured (round 5): 16 B more of PathQs (4,336-B block) made
// launches under rocprofv3 stall for 0.3-2 s with no waves resident (the
// dispatch waiting, not the kernel); the round-4 size and below run clean.
static_assert(sizeof(PacketArgs) <= 4320, "kernel argument block grew past the measured-clean size");
typedef const __attribute__((address_space(3))) PacketArgs* args_p;

// PATHS: the packed packet walk traces the primary segments of the queued
// path tracer (config c5).  Defined in queue_paths.h: the sample's jittered
// sub-pixel offset, and the primary vertex (outputs, first bounce appended,
// radiance, or the fall-back list); returns 1 for a resolved hit.
template <int W>
__device__ void q_primary_offset(args_p A, int s, int i, int r, double& ox, double& oy);
template <int W, bool COUNT>
__device__ uint32_t q_primary_vertex(args_p A, int s, int i, int r, bool valid, uint32_t redo, const Best& out,
                                     const Ray64& pre);

__device__ __forceinline__ args_p launder(args_p p) {
    asm volatile("" : "+s"(p));
    return p;
}

// Word-wise uniform copy out of the LDS argument block (unused words fold away).
template <class T>
__device__ __forceinline__ T kload(const __attribute__((address_space(3))) T* p) {
    static_assert(sizeof(T) % 4 == 0, "argument structs are word-sized");
    T out;
    const __attribute__((address_space(3))) uint32_t* src = (const __attribute__((address_space(3))) uint32_t*)p;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
    for (unsigned w = 0; w < sizeof(T) / 4; w++) dst[w] = uni(src[w]);
    return out;
}
template <class T>
__device__ __forceinline__ T kword(const __attribute__((address_space(3))) T* p) {
    static_assert(sizeof(T) == 4, "one word");
    return __builtin_bit_cast(T, uni(*(const __attribute__((address_space(3))) uint32_t*)p));
}

// Slab test of one node's W children for every lane's ray (fp32, outward
// planes).  OCT >= 0: all rays share the direction signs OCT (bit a set =
// negative along axis a), so each axis's near plane is the hi plane for a
// negative direction and the lo plane otherwise — exactly what the per-axis
// min/max of the general test (OCT = -1) selects, since t(lo) <= t(hi) for a
// positive reciprocal and t(hi) <= t(lo) for a negative one.
//
// RT_PK_SLAB=1 (a tuning build): the two planes of an axis in one
// v_pk_fma_f32 — the record's {lo, hi} pair is an aligned SGPR pair, the
// reciprocal goes to both halves and the offsets are the {lo, hi} pair nox —
// so a child costs 3 packed fmas instead of 6 and a node step 65 VALU
// instead of 89 (each half rounds once, as fmaf: the same bits).  Measured
// slower (round 6, one box, three interleaved 20-step pairs): 17.15 / 17.52
// / 17.19 vs 17.88 / 17.93 / 17.96 Grays/s (−3.5%); round 1's plane pairs
// measured ±0.  Fewer VALU per node step do not shorten it.
#ifndef RT_PK_SLAB
#define RT_PK_SLAB 0
#endif
template <int W, int OCT>
__device__ __forceinline__ void child_hits(const float (&bx)[W][6], const Ray32& q, const f2 nox, const f2 noy,
                                           const f2 noz, float tcull, uint64_t (&hm)[W]) {
    const f2 ix2{q.ix, q.ix}, iy2{q.iy, q.iy}, iz2{q.iz, q.iz};
#pragma unroll
    for (int c = 0; c < W; c++) {
        float tlx, thx, tly, thy, tlz, thz;
        if constexpr (RT_PK_SLAB != 0) {
            const f2 tx = __builtin_elementwise_fma(f2{bx[c][0], bx[c][1]}, ix2, nox);
            const f2 ty = __builtin_elementwise_fma(f2{bx[c][2], bx[c][3]}, iy2, noy);
            const f2 tz = __builtin_elementwise_fma(f2{bx[c][4], bx[c][5]}, iz2, noz);
            tlx = tx.x; thx = tx.y; tly = ty.x; thy = ty.y; tlz = tz.x; thz = tz.y;
        } else {
            tlx = __builtin_fmaf(bx[c][0], q.ix, nox.x); thx = __builtin_fmaf(bx[c][1], q.ix, nox.y);
            tly = __builtin_fmaf(bx[c][2], q.iy, noy.x); thy = __builtin_fmaf(bx[c][3], q.iy, noy.y);
            tlz = __builtin_fmaf(bx[c][4], q.iz, noz.x); thz = __builtin_fmaf(bx[c][5], q.iz, noz.y);
        }
        float t0, t1;
        if constexpr (OCT < 0) {
            t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
            t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull));
        } else {
            const float nx = (OCT & 1) ? thx : tlx, fx = (OCT & 1) ? tlx : thx;
            const float ny = (OCT & 2) ? thy : tly, fy = (OCT & 2) ? tly : thy;
            const float nz = (OCT & 4) ? thz : tlz, fz = (OCT & 4) ? tlz : thz;
            t0 = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
            t1 = fminf(fminf(fx, fy), fminf(fz, tcull));
        }
        hm[c] = __ballot(t0 <= t1);
    }
}

// Which of a node's nv valid children (a prefix of the W slots) any lane's
// ray enters, as a bit mask.  The wide nodes of the walk tree hold 4.1 valid
// children on average: for W = 8 the slots are tested in groups (RT_SLOT_GROUP
// slots each) and a group past nv is skipped with a uniform branch.  The
// records stay loaded unconditionally (no value flows out of a branch but
// the mask), so the skipped VALU costs no register copies.
#ifndef RT_SLOT_GROUP
#define RT_SLOT_GROUP 8
#endif
// Empty child slots are inverted boxes (bvh_build.cpp alloc_node): the
// per-octant node tests skip the valid-slot mask.  0: mask anyway.
#ifndef RT_EMPTY_INVERTED
#define RT_EMPTY_INVERTED 1
#endif
// The leaf filter as tri_classify_flat (kernels_common.h: one divergent
// branch per triangle record instead of a nest of five).  0: the nest.
#ifndef RT_FLAT_CLASSIFY
#define RT_FLAT_CLASSIFY 1
#endif
template <int W, int OCT>
__device__ __forceinline__ uint32_t node_mask(const float (&bx)[W][6], const Ray32& q, const f2 nox, const f2 noy,
                                              const f2 noz, float tcull, uint32_t nv) {
    constexpr int G = (W == 8 && RT_SLOT_GROUP < 8) ? RT_SLOT_GROUP : W;
    uint32_t mask = 0;
#pragma unroll
    for (int g0 = 0; g0 < W; g0 += G) {
        if (g0 > 0 && nv <= (uint32_t)g0) break;  // (nv >= 1: group 0 is always tested)
        float b[G][6];
#pragma unroll
        for (int c = 0; c < G; c++)
#pragma unroll
            for (int a = 0; a < 6; a++) b[c][a] = bx[g0 + c][a];
        uint64_t hm[G];
        child_hits<G, OCT>(b, q, nox, noy, noz, tcull, hm);
        mask |= any_mask<G>(hm) << g0;
    }
    // (per-octant tests: empty slots hold inverted boxes, which fail for every
    // ray — bvh_build.cpp alloc_node — so only the general test masks them)
    if constexpr (OCT >= 0 && RT_EMPTY_INVERTED) return mask;
    return mask & ((1u << nv) - 1u);
}

// RT_NEAR_ASM (default): the near child's index and the tile's direction
// along the node's sort axis in one inline-asm block (node step); 0: C.
#ifndef RT_NEAR_ASM
#define RT_NEAR_ASM 1
#endif
// RT_NEAR_TREE (default): the near child's ref picked by a select tree on
// the index bits instead of a compare-and-select chain; 0: the chain.
// Round 6, three interleaved 20-step pairs on one box (the compiler's own
// tree, 13 SALU instead of 14 + 1): 17.81 / 17.92 / 17.92 vs 17.73 / 17.78 /
// 17.83 Grays/s (+0.6%).
#ifndef RT_NEAR_TREE
#define RT_NEAR_TREE 1
#endif

// Per-lane counters of the counting pass (RT_FLAG_COUNT).
struct ResolveCounts {
    uint32_t tris = 0, chain = 0, chain_nodes = 0;
};

// Exact resolve of one sample's candidate list (the reference's closest hit,
// stack_bvh.hpp:611-644): for each candidate the fp64 Moller-Trumbore and hit
// distance (triangle.hpp:40-88, stack_bvh.hpp:630-631); the winner is the
// minimum (distance, reference visit rank) — the reference keeps the first
// strictly closer hit in its LIFO order (stack_bvh.hpp:633) — and its
// reference ancestor chain is re-verified.
//   e0, get(c)  list entries 0 and 1 .. nlist-1 (LDS or HBM)
//   chunk       the overflow pool chunk (entries until a ~0 triangle or
//               RT_POOL_CHUNK), or null
//   drop        if dropped: the smallest t lower bound of a dropped candidate
// Returns 0 (out / sh hold the winner, tri < 0: a miss), 1 (a dropped
// candidate could win) or 2 (the reference cannot see the winner).
template <bool COUNT, class GetFn>
__device__ __forceinline__ uint32_t resolve_list(const RtDevScene& sc, const RtFrameParams& fp, const RtFrameCam& cam,
                                                 int i, int j, uint32_t nlist, const uint2 e0, GetFn&& get,
                                                 const RT_G uint2* chunk, bool dropped, float drop, Best& out,
                                                 Shade& sh, ResolveCounts& rc, const Ray64* pre = nullptr) {
    out.dist = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
    out.rank = 0xFFFFFFFFu;
    out.tri = -1;
    out.px = out.py = out.pz = 0.0;
    sh = Shade{0.0, 0.0, 0.0, RT_INVALID_REF};
    if (nlist == 0 && !chunk && !dropped) return 0;
    // Moller-Trumbore part of entry 0's 128-B record (v0, e1, e2) requested
    // as soon as its index is known; the fp64 ray is built while it is in
    // flight.  The winner's shading fields are loaded once, after the list.
    double R0[9];
    // kSpecWin: entry 0's shading fields too (normal, {id, leaf}, leaf box:
    // the rest of its record), requested with its MT part — entry 0 is the
    // winner of most pixels, whose resolve then makes one memory round trip
    // instead of two
    double N0[3] = {0.0, 0.0, 0.0};
    uint2 IL0 = make_uint2(0u, 0u);
    float4 B0a = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 B0b = make_float2(0.f, 0.f);
    if (nlist > 0) {
        const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)e0.x;
#pragma unroll
        for (int k = 0; k < 9; k++) R0[k] = T[k];
        if constexpr (kSpecWin) {
            N0[0] = T[RT_T64_NORMAL];
            N0[1] = T[RT_T64_NORMAL + 1];
            N0[2] = T[RT_T64_NORMAL + 2];
            IL0 = *reinterpret_cast<const RT_G uint2*>(T + RT_T64_IDLEAF);
            B0a = *reinterpret_cast<const RT_G float4*>(T + RT_T64_BOX);
            B0b = *reinterpret_cast<const RT_G float2*>(T + RT_T64_BOX + 2);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the ray's fp64 set-up
    }
    // the pixel's fp64 ray: the walk's own (pre, kept from the tile set-up)
    // or generated again (the same expressions, so the same bits)
    const Ray64 ray = pre ? *pre : gen_ray<false>(fp, cam, i, j);
    double best_t = 0.0;
    // exact test of candidate e (MT part T: global or a register copy), kept
    // if it is the (distance, visit rank) minimum
    auto consider_rec = [&](const uint2 e, const auto* T) {
        if (COUNT) rc.tris++;
        double t;
        if (!mt64(T, ray, t)) return;
        double hx, hy, hz;
        const double d = hit_dist(ray, t, hx, hy, hz);
        bool take = d < out.dist;
        if (!take && d == out.dist) {  // tie: the reference keeps the earlier visit
            if (out.tri < 0) {
                take = true;
            } else {
                if (out.rank == 0xFFFFFFFFu) out.rank = sc.tri_rank[out.tri];
                const uint32_t rank = sc.tri_rank[e.x];
                take = rank < out.rank;
                if (take) out.rank = rank;
            }
        } else if (take) {
            out.rank = 0xFFFFFFFFu;  // visit ranks are loaded on a tie only
        }
        if (take) {
            out.dist = d;
            out.tri = (int32_t)e.x;
            best_t = t;
        }
    };
    auto consider = [&](const uint2 e) { consider_rec(e, sc.tri64 + RT_TRI64_DOUBLES * (size_t)e.x); };
    if (nlist > 0) consider_rec(e0, R0);
    for (uint32_t c = 1; c < nlist; c++) consider(get(c));
    if (chunk) {
        for (uint32_t c = 0; c < (uint32_t)RT_POOL_CHUNK; c++) {
            const uint2 e = chunk[c];
            if (e.x == ~0u) break;
            consider(e);
        }
    }
    if (dropped) {
        // every dropped candidate has t >= drop, so its distance is at least
        // drop (1 - 2^-20) - slack: the winner must be strictly nearer than
        // that, else only the exact per-lane path can decide
        const double omax = __builtin_fmax(__builtin_fmax(__builtin_fabs(ray.ox), __builtin_fabs(ray.oy)),
                                           __builtin_fabs(ray.oz));
        const double bound = (double)drop * (1.0 - 0x1p-20) - 0x1p-40 * (omax + 1.0);
        if (!(out.tri >= 0 && out.dist < bound)) return 1;
    }
    if (out.tri < 0) return 0;
    // the winner's shading fields: unit normal, {loader id, real leaf}, leaf
    // box (6 floats rounded inward) — the rest of its record
    uint2 il;
    float lb[6];
    if (kSpecWin && nlist > 0 && out.tri == (int32_t)e0.x) {  // entry 0 won: its fields are here
        sh.nx = N0[0];
        sh.ny = N0[1];
        sh.nz = N0[2];
        il = IL0;
        lb[0] = B0a.x; lb[1] = B0a.y; lb[2] = B0a.z; lb[3] = B0a.w; lb[4] = B0b.x; lb[5] = B0b.y;
    } else {
        const RT_G double* T = sc.tri64 + RT_TRI64_DOUBLES * (size_t)out.tri;
        sh.nx = T[RT_T64_NORMAL];
        sh.ny = T[RT_T64_NORMAL + 1];
        sh.nz = T[RT_T64_NORMAL + 2];
        il = *reinterpret_cast<const RT_G uint2*>(T + RT_T64_IDLEAF);
        const float4 b0 = *reinterpret_cast<const RT_G float4*>(T + RT_T64_BOX);
        const float2 b1 = *reinterpret_cast<const RT_G float2*>(T + RT_T64_BOX + 2);
        lb[0] = b0.x; lb[1] = b0.y; lb[2] = b0.z; lb[3] = b0.w; lb[4] = b1.x; lb[5] = b1.y;
    }
    sh.id = il.x;
    (void)hit_dist(ray, best_t, out.px, out.py, out.pz);
    // the reference must see the winner: re-verify its ancestor chain
    if (COUNT) rc.chain++;
    if (!chain_fast_ok32(lb, ray, out.px, out.py, out.pz) && !chain_ok(sc, il.y, with_inv(ray), rc.chain_nodes))
        return 2;
    return 0;
}

// Counting pass only: distinct values over the wave's active lanes, lane l
// contributing get(0) .. get(n - 1) (n <= 32).  The fused resolve fetches the
// fp64 record of every candidate a lane tests; neighbouring rays test the
// same triangles, so a record read by several lanes of the wave is one fetch
// — the per-wave convention the walk's node and triangle records are counted
// in (bench.py roofline).
template <class GetFn>
__device__ uint32_t wave_distinct(uint32_t n, GetFn&& get) {
    uint32_t done = 0, count = 0;
    for (;;) {
        uint32_t mine = 0;
        bool have = false;
        for (uint32_t c = 0; c < n; c++)
            if (!((done >> c) & 1u)) {
                mine = get(c);
                have = true;
                break;
            }
        const uint64_t act = __ballot(have);
        if (act == 0) break;
        const uint32_t u = (uint32_t)__shfl((int)mine, (int)__builtin_ctzll(act));
        count++;
        for (uint32_t c = 0; c < n; c++)
            if (!((done >> c) & 1u) && get(c) == u) done |= 1u << c;
    }
    return count;
}

// Outcome of one tile for the caller's per-frame hit count (FUSED).
struct TileOut {
    bool hit;       // the lane's pixel is resolved here and hit
    uint32_t hits;  // fp.pack: on a pixel's first-sample lane, its samples hit
};

template <int W, int SP, int K, bool COUNT, bool FUSED, bool PACK, bool PATHS = false>
__device__ __forceinline__ TileOut trace_packet(args_p A, int f, int i, int r, bool valid,
                                                uint32_t* __restrict__ wstack, uint2* __restrict__ cand) {
    const int lane = threadIdx.x & 63;
    const uint64_t p0 = prof_clock();
    uint64_t p_node = 0, p_leaf = 0, p_prev = 0;  // RT_PROFILE only
    bool prev_node = false;
    if (!valid) { i = 0; r = 0; }
    Ray32 q;
    float tsl;  // distance slack (see trace_exact), fp32 rounded up
    float pd;
    uint32_t ob;
    double kd[3];  // kKeepDir: the fp64 direction, kept for the resolve
    {
        const RtFrameParams fp = kload(&A->fp);
        // (the pose of sample frame f: a uniform branch skips the integer
        // division at 1 spp)
        int pose = f;
        if (fp.spp != 1) pose = f / fp.spp;
        RtFrameCam cam = frame_cam_of(kload(&A->fp.pose[pose]), fp, f);  // this tile's frame
#if !defined(RT_QPV_DIAG) || RT_QPV_DIAG < 2
        if constexpr (PATHS) q_primary_offset<W>(A, f, i, r, cam.ox, cam.oy);  // the path sample's jitter
#endif
        // kFastInv: the fp32 reciprocals straight from the fp32 direction
        // (v_rcp_f32 + a Newton step: no fp64 divisions in the set-up)
        const Ray64 ray = gen_ray<!kFastInv>(fp, cam, i, rt_image_row(fp.row0, fp.row_stride, fp.band, r));
        kd[0] = ray.dx;
        kd[1] = ray.dy;
        kd[2] = ray.dz;
        q = make_ray32<kFastInv>(ray, cam.pad);
        tsl = round_up_f(0x1p-40 * ((double)q.co + 1.0));
        pd = cam.pad;
        // the lane's pixel in the batch (< 2^31, host-checked)
        ob = (uint32_t)out_index(fp, f, (size_t)r * fp.W + i);
    }
    // direction sign bits (x, y, z) of lane 0's ray: the tile's ordering key
    const uint32_t lsg = (q.ix < 0.f ? 1u : 0u) | (q.iy < 0.f ? 2u : 0u) | (q.iz < 0.f ? 4u : 0u);
    const uint32_t dsg = uni(lsg);
    // the tile's octant if every ray that takes part shares lane 0's signs, else 8
    const int oct = __ballot(valid && lsg != dsg) == 0 ? (int)dsg : 8;
    const RT_G uint8_t* const nodes = kload(&A->sc.nodes);
    const RT_G float* const tri32 = kload(&A->sc.tri32);
    // slab offsets for the lo / hi planes (pad moves lo down and hi up)
    const float olx = (q.ox + pd) * q.ix, ohx = (q.ox - pd) * q.ix;
    const float oly = (q.oy + pd) * q.iy, ohy = (q.oy - pd) * q.iy;
    const float olz = (q.oz + pd) * q.iz, ohz = (q.oz - pd) * q.iz;
    const f2 nox{-olx, -ohx}, noy{-oly, -ohy}, noz{-olz, -ohz};

    uint32_t n_nodes = 0, n_pre = 0, w_nodes = 0, w_leaves = 0, w_tris = 0, w_empty = 0;  // COUNT only
    float tcull = valid ? __builtin_huge_valf() : -1.f;
    int nc = 0;                          // candidates in the lane's LDS list
    int nsp = 0;                         // candidates in the lane's overflow chunk
    uint32_t chunk = kNoChunk;           // the lane's overflow pool chunk
    float drop = __builtin_huge_valf();  // smallest t lower bound of a dropped candidate
    // node refs carry the node's meta (sort axis | valid slots << 2, from the
    // parent's record; bvh_build.cpp flatten) in bits 24-30
    uint32_t cur = kword(&A->sc.root_ref);
    if (!(cur & RT_LEAF_BIT)) cur |= kword(&A->sc.root_meta) << 24;
    {
        float b[6];
        for (int a = 0; a < 6; a++) b[a] = kword(&A->sc.root_box[a]);
        const float t0 = fmaxf(fmaxf(fminf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                     fminf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                               fmaxf(fminf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)), 0.f));
        const float t1 = fminf(fminf(fmaxf(__builtin_fmaf(b[0], q.ix, -olx), __builtin_fmaf(b[1], q.ix, -ohx)),
                                     fmaxf(__builtin_fmaf(b[2], q.iy, -oly), __builtin_fmaf(b[3], q.iy, -ohy))),
                               fminf(fmaxf(__builtin_fmaf(b[4], q.iz, -olz), __builtin_fmaf(b[5], q.iz, -ohz)), tcull));
        if (__ballot(t0 <= t1) == 0) cur = RT_INVALID_REF;
    }
    int sp = 0;
    // The walk, specialised on the tile's octant (one dispatch per tile, not
    // per node step: 9 copies of the loop).  Every popped ref is a real node
    // or leaf, so only the root can be invalid: tested once, not per step.
    const uint64_t p1 = prof_clock();
    p_prev = p1;
    auto walk = [&]<int OCT>() __attribute__((always_inline)) {
        if (cur == RT_INVALID_REF) return;
        for (;;) {
            if constexpr (kProfile) {  // the previous step's cycles to its bucket
                const uint64_t now = prof_clock();
                (prev_node ? p_node : p_leaf) += now - p_prev;
                p_prev = now;
                prev_node = !(cur & RT_LEAF_BIT);
            }
            if (!(cur & RT_LEAF_BIT)) {
                if (COUNT) {
                    w_nodes++;
                    n_nodes += valid;
                }
                float bx[W][6];  // child boxes {lx, hx, ly, hy, lz, hz}
                uint32_t rs[W];  // the children's refs (scalars), their nodes' meta in bits 24-30
                const uint32_t meta = cur >> 24;  // sort axis | valid slots << 2
                const uint32_t nv = meta >> 2;    // valid slots (a prefix)
                uint32_t mask;   // bit c: some lane's ray enters child c
                {
                    // all W records are loaded before any test so their loads
                    // are in flight together
                    const cchild_p nb = (cchild_p)(nodes + (size_t)(cur & 0x00FFFFFFu) * (32 * W));
                    ChildRec ch[W];
#pragma unroll
                    for (int c = 0; c < W; c++) ch[c] = load_child(nb + c);
                    // every record is materialised here: the compiler would
                    // otherwise sink the loads of skipped slot groups into
                    // their branches (a second round trip per node step)
#pragma unroll
                    for (int c = 0; c < W; c++) pin_rec(ch[c]);
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        bx[c][0] = ch[c].lx; bx[c][1] = ch[c].hx; bx[c][2] = ch[c].ly;
                        bx[c][3] = ch[c].hy; bx[c][4] = ch[c].lz; bx[c][5] = ch[c].hz;
                    }
                    // the ref words come with the boxes (same scalar loads);
                    // an inner child's ref gets its node's meta (leaf pads are 0)
#pragma unroll
                    for (int c = 0; c < W; c++) rs[c] = ch[c].pad;  // ref | meta << 24 (bvh_build.cpp flatten)
                    mask = node_mask<W, OCT>(bx, q, nox, noy, noz, tcull, nv);
#if defined(RT_DBL_NODE) && RT_DBL_NODE
                    {   // (measurement build: the child test twice, the second on an
                        // opaque copy of tcull so it is not merged; its cost is the
                        // node test's dynamic instruction count, tools/phase_counts.py)
                        // (opaque copies of every lane input: no part of the
                        // second test can be shared with the first)
                        float t2 = tcull;
                        Ray32 q2 = q;
                        f2 nx2 = nox, ny2 = noy, nz2 = noz;
                        asm volatile("" : "+v"(t2), "+v"(q2.ix), "+v"(q2.iy), "+v"(q2.iz), "+v"(nx2), "+v"(ny2),
                                     "+v"(nz2));
                        const uint32_t m2 = node_mask<W, OCT>(bx, q2, nx2, ny2, nz2, t2, nv);
                        asm volatile("" ::"s"(m2));
                    }
#endif
                }
                if (COUNT) w_empty += mask == 0;
                if (mask != 0) {
                    // children are sorted along `axis`: walk them front to back
                    // for the tile's direction (lowest index first when the
                    // tile looks along +axis)
                    int near_c;
                    uint64_t revm;  // all ones when the tile looks along -axis (RT_NEAR_ASM)
                    bool rev = false;
                    if constexpr (RT_NEAR_ASM != 0) {
                        // the near index and the direction as one SCC: 7
                        // scalar instructions instead of 10 (the compiler's
                        // form re-tests the bit and ANDs the lane mask with exec)
                        // (a per-octant walk's direction bits are OCT itself:
                        // an inline constant, no register)
                        uint32_t n, l, ax;
#define RT_NEAR_ASM_BODY                                      \
    "s_ff1_i32_b32 %[n], %[m]\n\t"                             \
    "s_flbit_i32_b32 %[l], %[m]\n\t"                           \
    "s_sub_u32 %[l], 31, %[l]\n\t"                             \
    "s_bfe_u32 %[ax], %[cur], 0x20018\n\t" /* meta & 3 */      \
    "s_bitcmp1_b32 %[d], %[ax]\n\t"                            \
    "s_cselect_b64 %[rv], -1, 0\n\t"                           \
    "s_cselect_b32 %[n], %[l], %[n]"
                        if constexpr (OCT >= 0)
                            asm(RT_NEAR_ASM_BODY
                                : [n] "=&s"(n), [l] "=&s"(l), [ax] "=&s"(ax), [rv] "=&s"(revm)
                                : [m] "s"(mask), [cur] "s"(cur), [d] "i"(OCT)
                                : "scc");
                        else
                            asm(RT_NEAR_ASM_BODY
                                : [n] "=&s"(n), [l] "=&s"(l), [ax] "=&s"(ax), [rv] "=&s"(revm)
                                : [m] "s"(mask), [cur] "s"(cur), [d] "s"(dsg)
                                : "scc");
#undef RT_NEAR_ASM_BODY
                        near_c = (int)n;
                    } else {
                        rev = (dsg >> (meta & 3u)) & 1u;
                        near_c = rev ? 31 - __builtin_clz(mask) : __builtin_ctz(mask);
                        revm = 0;
                    }
                    const uint32_t pm = mask & ~(1u << near_c);
                    if (pm != 0) {
                        // lane c: child c's ref (built only for nodes that push)
                        const uint32_t refv = lanes_of<W>(rs);
                        // the rest go on the stack so that they pop in order:
                        // lane c < W holds child c; `below` counts pm's bits
                        // under it (v_mbcnt), the 64-bit shift is 0 for every
                        // lane >= W (pm < 2^W), so no lane-range mask
                        const uint32_t np = (uint32_t)__builtin_popcount(pm);
                        const uint32_t below = __builtin_amdgcn_mbcnt_lo(pm, 0u);
                        int slot;
                        if constexpr (RT_NEAR_ASM != 0)
                            asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(slot) : "v"(np - 1u - below), "v"(below),
                                "s"(revm));
                        else
                            slot = (int)(rev ? below : np - 1u - below);
                        if (((uint64_t)pm >> lane) & 1u) wstack[sp + slot] = refv;
                        sp += np;
                    }
                    // the near child's ref, picked on the scalar unit (a
                    // readlane from the lanes measured 0.5% slower, a scalar
                    // reload of the record's word +-0)
                    uint32_t nr = rs[0];
                    if constexpr (RT_NEAR_TREE != 0 && W == 8) {
                        // a 3-level select on the index bits: 3 s_bitcmp1 + 7
                        // s_cselect instead of 7 compares + 7 selects (the
                        // compiler's own select tree took 3 s_and + 3 s_cmp)
                        uint32_t a, b, c, d;
                        asm("s_bitcmp1_b32 %[n], 0\n\t"
                            "s_cselect_b32 %[a], %[r1], %[r0]\n\t"
                            "s_cselect_b32 %[b], %[r3], %[r2]\n\t"
                            "s_cselect_b32 %[c], %[r5], %[r4]\n\t"
                            "s_cselect_b32 %[d], %[r7], %[r6]\n\t"
                            "s_bitcmp1_b32 %[n], 1\n\t"
                            "s_cselect_b32 %[a], %[b], %[a]\n\t"
                            "s_cselect_b32 %[c], %[d], %[c]\n\t"
                            "s_bitcmp1_b32 %[n], 2\n\t"
                            "s_cselect_b32 %[a], %[c], %[a]"
                            : [a] "=&s"(a), [b] "=&s"(b), [c] "=&s"(c), [d] "=&s"(d)
                            : [n] "s"((uint32_t)near_c), [r0] "s"(rs[0]), [r1] "s"(rs[1]), [r2] "s"(rs[2]),
                              [r3] "s"(rs[3]), [r4] "s"(rs[4]), [r5] "s"(rs[5]), [r6] "s"(rs[6]), [r7] "s"(rs[7])
                            : "scc");
                        nr = a;
                    } else {
#pragma unroll
                        for (int c = 1; c < W; c++) nr = near_c == c ? rs[c] : nr;
                    }
                    cur = nr;
                    continue;
                }
            } else {
                if constexpr (RT_LEAF_PRIO > 0) __builtin_amdgcn_s_setprio(RT_LEAF_PRIO);
                const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                if (COUNT) {
                    w_leaves++;
                    w_tris += cnt;
                }
                // triangles come in chunks of kLeafChunk records: all their
                // scalar loads are issued, then waited on once (tri32 carries
                // padding records, so reading past a leaf is safe)
                const uint32_t end = first + cnt;
                // (a leaf holds >= 1 record: a do-while; the records' byte
                // offset is 32-bit — the host caps the scene at 2^32 / 48
                // records, rt_api.cpp — so the loads take it as an SGPR
                // offset, with no 64-bit address arithmetic per chunk)
                uint32_t k0 = first, kb = first * 48u;
                do {
                    __builtin_assume(kb < 0xFFFFFFF0u);
                    const cfloat_p R = (cfloat_p)(tri32 + (size_t)(kb >> 2));
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
                        if (t > 0 && k >= end) break;  // (record k0 < end: the do-while)
                        if (COUNT) n_pre += valid;
                        float tl, tu;
                        int cls;
                        if constexpr (RT_FLAT_CLASSIFY != 0) {
                            // (an invalid lane holds pixel 0's finite ray: its
                            // class is computed and dropped by a select, not
                            // branched around)
                            cls = tri_classify_flat(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co,
                                                    tcull, tl, tu);
                            cls = valid ? cls : 0;
                        } else
                            cls = valid ? tri_classify_nest(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz,
                                                            q.co, tcull, tl, tu)
                                        : 0;
#if defined(RT_DBL_LEAF) && RT_DBL_LEAF
                        {   // (measurement build: the triangle filter twice, tools/phase_counts.py)
                            float t2 = tcull, tl2 = 0.f, tu2 = 0.f;
                            float ox2 = q.ox, oy2 = q.oy, oz2 = q.oz, dx2 = q.dx, dy2 = q.dy, dz2 = q.dz, co2 = q.co;
                            asm volatile("" : "+v"(t2), "+v"(ox2), "+v"(oy2), "+v"(oz2), "+v"(dx2), "+v"(dy2), "+v"(dz2),
                                         "+v"(co2));
                            const int c2 = valid ? tri_classify(TA[t], TB[t], TC[t], ox2, oy2, oz2, dx2, dy2, dz2, co2,
                                                                t2, tl2, tu2)
                                                 : 0;
                            asm volatile("" ::"v"(c2), "v"(tl2), "v"(tu2));
                        }
#endif
                        // (no `continue`: in the unrolled chunk loop each one
                        // cost the structurizer a flow variable and its tests)
                        if (cls != 0) {
                            // dist of a certain hit <= (tu + slack)(1 + 2^-20)
                            if (cls == 2) tcull = fminf(tcull, (tu + tsl) * (1.f + 0x1p-20f));
                            if (nc == K) nc = compact_candidates<K>(cand, lane, tcull);
                            if (nc < K) {
                                cand[nc * 64 + lane] = make_uint2(k, __float_as_uint(tl));
                                nc++;
                            } else {
                                // LDS list full: append to the lane's overflow
                                // chunk, taking one from the pool on first need
                                const args_p A2 = launder(A);  // (A itself stays uniform)
                                if (chunk == kNoChunk) {
                                    const uint32_t c = atomicAdd(kload(&A2->aux.tile_ctr) + RT_POOL_COUNT, 1u);
                                    chunk = c < kword(&A2->aux.pool_chunks) ? c : kPoolDry;
                                }
                                if (chunk != kPoolDry && nsp < RT_POOL_CHUNK) {
                                    RT_G uint2* const pool = reinterpret_cast<RT_G uint2*>(kload(&A2->aux.pool));
                                    pool[(size_t)chunk * RT_POOL_CHUNK + nsp] = make_uint2(k, __float_as_uint(tl));
                                    nsp++;
                                } else {
                                    // full: keep the K smallest lower bounds, remember
                                    // the smallest bound dropped (the resolve certifies
                                    // the winner against it, else the pixel is redone
                                    // exactly)
                                    drop = fminf(drop, keep_nearest<K>(cand, lane, k, tl));
                                }
                            }
                        }
                    }
                    k0 += kLeafChunk;
                    kb += 48u * kLeafChunk;
                } while (k0 < end);
            }
            if constexpr (RT_LEAF_PRIO > 0) __builtin_amdgcn_s_setprio(0);
            if (sp == 0) break;
            sp--;
            cur = uni(wstack[sp]);
        }
    };
    if constexpr (RT_EPI_PRIO > 0) __builtin_amdgcn_s_setprio(0);  // the walk at the lowest priority
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
    if constexpr (RT_EPI_PRIO > 0) __builtin_amdgcn_s_setprio(RT_EPI_PRIO);  // epilogue, claim, next set-up
    uint64_t p2 = 0;
    if constexpr (kProfile) {
        p2 = prof_clock();
        (prev_node ? p_node : p_leaf) += p2 - p_prev;
    }
    A = launder(A);
    const RtFrameParams fp = kload(&A->fp);
    if (COUNT && fp.counters && lane == 0) {
        atomicAdd(&fp.counters[7], (unsigned long long)w_nodes);
        atomicAdd(&fp.counters[8], (unsigned long long)w_leaves);
        atomicAdd(&fp.counters[9], 1ull);
        atomicAdd(&fp.counters[12], (unsigned long long)w_tris);
        atomicAdd(&fp.counters[15], (unsigned long long)w_empty);
    }
    TileOut res{false, 0u};
    auto prof_out = [&]() __attribute__((always_inline)) {
        if constexpr (kProfile) {
            const uint64_t p3 = prof_clock();
            if (fp.counters && lane == (int)__builtin_ctzll(__ballot(true))) {
                atomicAdd(&fp.counters[18], (unsigned long long)(p1 - p0));
                atomicAdd(&fp.counters[19], (unsigned long long)p_node);
                atomicAdd(&fp.counters[20], (unsigned long long)p_leaf);
                atomicAdd(&fp.counters[21], (unsigned long long)(p3 - p2));
                atomicAdd(&fp.counters[22], 1ull);
                atomicAdd(&fp.counters[23], (unsigned long long)(p3 - p0));
            }
        }
    };
    if (!valid) {
        if (__ballot(true) == ~0ull) prof_out();  // (a wholly invalid tile)
        return res;
    }
    const RtLaunchAux aux = kload(&A->aux);
    const bool dropped = drop < __builtin_huge_valf() && drop <= tcull;  // a dropped candidate could still win
    if (chunk != kNoChunk && chunk != kPoolDry && nsp < RT_POOL_CHUNK)  // terminate the chunk
        reinterpret_cast<RT_G uint2*>(aux.pool)[(size_t)chunk * RT_POOL_CHUNK + nsp] = make_uint2(~0u, 0u);
    const bool spilled = chunk != kNoChunk && chunk != kPoolDry && nsp > 0;
    if constexpr (FUSED) {
        // the tile's own lanes resolve their lists (frame f = sample f % spp
        // of pose f / spp), compacted against the final culling distance
        // first (an entry beyond it cannot beat a certain hit)
        uint32_t nl = 0;
        for (int c = 0; c < nc; c++) {
            const uint2 e = cand[c * 64 + lane];
            if (__uint_as_float(e.y) <= tcull) cand[nl++ * 64 + lane] = e;
        }
        const RtDevScene sc = kload(&A->sc);
        const int spp = fp.spp;
        const int pose = f / spp;
        const RtFrameCam cam = frame_cam_of(kload(&A->fp.pose[pose]), fp, f);
        Best out;
        Shade sh;
        ResolveCounts rc;
        const RT_G uint2* ch = spilled ? reinterpret_cast<const RT_G uint2*>(aux.pool) + (size_t)chunk * RT_POOL_CHUNK
                                       : nullptr;
        Ray64 pre;
        if constexpr (kKeepDir) {
            pre.ox = cam.pos[0];
            pre.oy = cam.pos[1];
            pre.oz = cam.pos[2];
            pre.dx = kd[0];
            pre.dy = kd[1];
            pre.dz = kd[2];
            pre.ix = pre.iy = pre.iz = 0.0;
        }
        const uint32_t redo = resolve_list<COUNT>(
            sc, fp, cam, i, rt_image_row(fp.row0, fp.row_stride, fp.band, r), nl, nl ? cand[lane] : make_uint2(0u, 0u),
            [&](uint32_t c) { return cand[c * 64 + lane]; }, ch, dropped, drop, out, sh, rc,
            kKeepDir ? &pre : nullptr);
        const bool hit_s = !redo && out.tri >= 0;
        if constexpr (PATHS) {
            // the path's primary vertex (queue_paths.h; the sample's
            // outputs, its first bounce ray appended, or the fall-back list)
            static_assert(PACK && kKeepDir, "path primaries: packed samples, the kept fp64 direction");
#if defined(RT_QPV_DIAG) && RT_QPV_DIAG > 0
            res.hits = out.tri >= 0;  // timing build: no path vertex (wrong results)
#else
            res.hits = q_primary_vertex<W, COUNT>(A, f - pose * spp, i, r, true, redo, out, pre);
#endif
        } else if (spp == 1) {
            if (redo) {
                // k_fixup redoes the pixel with the exact per-lane path
                redo_put(aux, ob | (redo == 2u ? kRedoPass1 : 0u));
            } else {
                store_sample(fp, ob, out, sh);
                double c[3];
                shade_color(cam, out, sh, c);
                store_rgb(fp, ob, c);
                res.hit = hit_s;
            }
        } else if constexpr (PACK) {
            // the pixel's spp samples are lanes base .. base + spp - 1 of this
            // wave (sample k in lane base + k): each lane stores its sample's
            // outputs, the colours are summed in sample order across the lanes
            // (k_average's order), and the first lane stores the pixel or, if
            // a sample is unresolved, sends the pixel to k_fixup whole
            const int base = lane & ~(spp - 1);
            const uint64_t gm = (spp == 64 ? ~0ull : ((1ull << spp) - 1ull)) << base;
            const uint64_t bad = __ballot(redo != 0) & gm;
            const uint64_t hm = __ballot(hit_s) & gm;
            const size_t fpix = (size_t)fp.W * (size_t)fp.nrows;
            const size_t po = (size_t)ob - (size_t)f * fpix;
            double c[3] = {0.0, 0.0, 0.0};
            if (!redo) {
                store_sample(fp, out_index(fp, pose, po) * (size_t)spp + (size_t)(f - pose * spp), out, sh);
                shade_color(cam, out, sh, c);
            }
            double acc[3] = {0.0, 0.0, 0.0};
            for (int k = 0; k < spp; k++) {
                acc[0] = acc[0] + __shfl(c[0], base + k);
                acc[1] = acc[1] + __shfl(c[1], base + k);
                acc[2] = acc[2] + __shfl(c[2], base + k);
            }
            if (lane == base) {
                const size_t pix = out_index(fp, pose, po);
                if (bad) {
                    redo_put(aux, (uint32_t)pix);
                } else {
                    store_rgb(fp, pix, acc);
                    res.hits = (uint32_t)__builtin_popcountll(hm);
                }
            }
        } else {
            // one sample of a pixel: its outputs at sample index pix * spp + k
            // (k_resolve's layout), its colour and status for k_average,
            // which sums the pixel's samples in order and counts its hits
            if (redo) {
                aux.cand_cnt[ob] = (uint8_t)kSampRedo;
            } else {
                const size_t fpix = (size_t)fp.W * (size_t)fp.nrows;
                const size_t po = (size_t)ob - (size_t)f * fpix;
                store_sample(fp, out_index(fp, pose, po) * (size_t)spp + (size_t)(f - pose * spp), out, sh);
                double c[3];
                shade_color(cam, out, sh, c);
                RT_G double* const col = reinterpret_cast<RT_G double*>(aux.cand) + (size_t)ob * 3;
                col[0] = c[0];
                col[1] = c[1];
                col[2] = c[2];
                aux.cand_cnt[ob] = (uint8_t)(hit_s ? 1u : 0u);
            }
        }
        if (COUNT && fp.counters) {
            // wave-distinct fp64 records: the candidates' Moller-Trumbore parts
            // and the winners' shading parts (one wave-level fetch each)
            static_assert(K + RT_POOL_CHUNK <= 32, "one bit per list entry");
            uint32_t nch = 0;
            if (ch)
                while (nch < (uint32_t)RT_POOL_CHUNK && ch[nch].x != ~0u) nch++;
            const uint32_t u_tests = wave_distinct(nl + nch, [&](uint32_t c) {
                return c < nl ? cand[c * 64 + lane].x : ch[c - nl].x;
            });
            const uint32_t u_win = wave_distinct(out.tri >= 0 ? 1u : 0u, [&](uint32_t) { return (uint32_t)out.tri; });
            if (lane == (int)__builtin_ctzll(__ballot(true))) {
                atomicAdd(&fp.counters[16], (unsigned long long)u_tests);
                atomicAdd(&fp.counters[17], (unsigned long long)u_win);
            }
            atomicAdd(&fp.counters[0], 1ull);
            // (PATHS: node_fetches are the per-lane bounce walks' counter)
            if constexpr (!PATHS) atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
            atomicAdd(&fp.counters[2], (unsigned long long)rc.tris);
            atomicAdd(&fp.counters[3], (unsigned long long)rc.chain);
            if (hit_s) atomicAdd(&fp.counters[4], 1ull);
            atomicAdd(&fp.counters[5], (unsigned long long)rc.chain_nodes);
            atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
            if (!PATHS && redo == 1) atomicAdd(&fp.counters[10], 1ull);
            if (!PATHS && redo == 2) atomicAdd(&fp.counters[11], 1ull);
            if (spilled) atomicAdd(&fp.counters[13], 1ull);
            if (dropped) atomicAdd(&fp.counters[14], 1ull);
        }
        prof_out();
    } else {
        // hand the lane's surviving candidates to k_resolve: count per
        // pixel, entry c of batch pixel o at cand[c * npix + o] (coalesced
        // across a row; frame f's pixels follow frame f-1's)
        const size_t o = ob;
        const size_t npix = (size_t)fp.W * fp.nrows * fp.nframes;
        uint32_t m = 0;
        for (int c = 0; c < nc; c++) {
            const uint2 e = cand[c * 64 + lane];
            if (__uint_as_float(e.y) > tcull) continue;  // cannot beat a certain hit
            reinterpret_cast<RT_G uint2*>(aux.cand)[(size_t)m * npix + o] = e;
            m++;
        }
        if (dropped) aux.cand_drop[o] = drop;
        if (spilled) aux.cand_ovf[o] = chunk;
        aux.cand_cnt[o] = (uint8_t)(m | (dropped ? kCandDropped : 0u) | (spilled ? kCandSpilled : 0u));
        if (COUNT && fp.counters) {
            atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
            atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
            if (spilled) atomicAdd(&fp.counters[13], 1ull);
            if (dropped) atomicAdd(&fp.counters[14], 1ull);
        }
    }
    return res;
}

// Exact resolve of the packet kernel's candidate lists for spp > 1, one pixel
// per lane over all spp samples of its pose (each sample's list in its own
// sample frame); one block per 16x16 tile of one pose.  The pixel colour is
// the samples' shadeScreen colours summed in sample order, divided by spp.
template <bool COUNT>
__global__ void __launch_bounds__(256) k_resolve(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint32_t wave_hits[4];
    // One block = one 16x16 pixel tile.  Blocks are dealt to the 8 XCDs
    // round-robin (block b on XCD b % 8), so block b = 8k + x takes logical
    // tile x * T8 + k: each XCD resolves one horizontal band of the pose.
    // Blocks never straddle poses: pose p owns blocks [p * bpf, (p + 1) * bpf).
    const uint32_t fpix = (uint32_t)fp.W * (uint32_t)fp.nrows;
    const uint32_t tx = ((uint32_t)fp.W + 15u) >> 4, ty = ((uint32_t)fp.nrows + 15u) >> 4;
    const uint32_t T8 = (tx * ty + 7u) >> 3;             // tiles per XCD band
    const uint32_t bpf = 8u * T8;
    const int p = (int)(blockIdx.x / bpf);
    const uint32_t fb = blockIdx.x - (uint32_t)p * bpf;  // block within the pose
    const uint32_t lt = (fb & 7u) * T8 + (fb >> 3);       // logical tile (raster order)
    const int i = (int)((lt % tx) * 16u + (threadIdx.x & 15u));
    const int r = (int)((lt / tx) * 16u + (threadIdx.x >> 4));
    const bool active = lt < tx * ty && i < fp.W && r < fp.nrows;
    const size_t po = active ? (size_t)r * fp.W + i : 0;  // pixel within the frame
    const size_t npix = (size_t)fpix * fp.nframes;       // candidate-list stride
    const size_t pix = out_index(fp, p, po);             // pixel of the pose outputs
    const RT_G uint2* const cl = reinterpret_cast<const RT_G uint2*>(aux.cand);
    uint32_t redo_any = 0, hits = 0, n_redo[3] = {0, 0, 0};
    ResolveCounts rc;
    double acc[3] = {0.0, 0.0, 0.0};
    const int spp = fp.spp;
    for (int k = 0; k < spp; k++) {
        const int f = p * spp + k;
        const size_t o = out_index(fp, f, po);
        uint32_t cnt = 0u;
        uint2 e0 = make_uint2(0u, 0u);
        if (active) {
            cnt = aux.cand_cnt[o];  // entry 0 is loaded alongside the count
            e0 = cl[o];
        }
        const uint32_t nlist = cnt & kCandCount;
        const RT_G uint2* ch = (cnt & kCandSpilled)
                                   ? reinterpret_cast<const RT_G uint2*>(aux.pool) + (size_t)aux.cand_ovf[o] * RT_POOL_CHUNK
                                   : nullptr;
        const bool dropped = (cnt & kCandDropped) != 0;
        Best out;
        Shade sh;
        const uint32_t redo = resolve_list<COUNT>(
            sc, fp, frame_cam(fp, f), i, rt_image_row(fp.row0, fp.row_stride, fp.band, r), nlist, e0,
            [&](uint32_t c) { return cl[(size_t)c * npix + o]; }, ch, dropped, dropped ? aux.cand_drop[o] : 0.f, out,
            sh, rc);
        if (COUNT) n_redo[redo]++;
        redo_any = redo_any > redo ? redo_any : redo;
        if (active && !redo) {
            store_sample(fp, pix * (size_t)spp + k, out, sh);
            double c[3];
            shade_color(frame_cam(fp, f), out, sh, c);
            acc[0] = acc[0] + c[0];
            acc[1] = acc[1] + c[1];
            acc[2] = acc[2] + c[2];
            hits += out.tri >= 0;
        }
    }
    if (active) {
        if (redo_any) {
            // k_fixup redoes every sample of the pixel with the exact per-lane path
            redo_put(aux, (uint32_t)pix);
            hits = 0;
        } else {
            store_rgb(fp, pix, acc);
        }
    }
    // hit count (samples hit): block sums spread over RT_HIT_SLOTS counters
    // per pose (k_fixup adds them up) instead of same-address device atomics
    uint32_t wsum = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) wsum += (uint32_t)__builtin_popcountll(__ballot((hits >> b) & 1u)) << b;
    if ((threadIdx.x & 63) == 0) wave_hits[threadIdx.x >> 6] = wsum;
    __syncthreads();
    if (threadIdx.x == 0 && fp.hit_count) {
        const uint32_t sum = wave_hits[0] + wave_hits[1] + wave_hits[2] + wave_hits[3];
        if (sum) atomicAdd(aux.tile_ctr + RT_HIT_BASE + (p * RT_HIT_SLOTS + fb % RT_HIT_SLOTS) * RT_QUEUE_STRIDE, sum);
    }
    if (!active) return;
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[0], (unsigned long long)spp);
        atomicAdd(&fp.counters[2], (unsigned long long)rc.tris);
        atomicAdd(&fp.counters[3], (unsigned long long)rc.chain);
        if (hits) atomicAdd(&fp.counters[4], (unsigned long long)hits);
        atomicAdd(&fp.counters[5], (unsigned long long)rc.chain_nodes);
        if (n_redo[1]) atomicAdd(&fp.counters[10], (unsigned long long)n_redo[1]);
        if (n_redo[2]) atomicAdd(&fp.counters[11], (unsigned long long)n_redo[2]);
    }
}

// spp > 1 behind the fused walk: one thread per pixel of a pose sums its
// samples' colours in sample order (k_resolve's order, so the bytes are the
// same), stores the PPM bytes and counts the samples hit; a pixel with a
// sample the walk kernel could not resolve goes to k_fixup whole (its hits are
// counted there).  Blocks never straddle poses.
__global__ void __launch_bounds__(256) k_average(RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint32_t wave_hits[4];
    const uint32_t fpix = (uint32_t)fp.W * (uint32_t)fp.nrows;
    const uint32_t bpf = (fpix + 255u) >> 8;  // blocks per pose
    const int p = (int)(blockIdx.x / bpf);
    const uint32_t fb = blockIdx.x - (uint32_t)p * bpf;
    const uint32_t po = fb * 256u + threadIdx.x;
    const int spp = fp.spp;
    uint32_t hits = 0;
    if (po < fpix) {
        bool redo = false;
        double acc[3] = {0.0, 0.0, 0.0};
        for (int k = 0; k < spp; k++) {
            const size_t o = out_index(fp, p * spp + k, po);
            const uint32_t st = aux.cand_cnt[o];
            if (st & kSampRedo) {
                redo = true;
                continue;
            }
            const RT_G double* const col = reinterpret_cast<const RT_G double*>(aux.cand) + o * 3;
            acc[0] = acc[0] + col[0];
            acc[1] = acc[1] + col[1];
            acc[2] = acc[2] + col[2];
            hits += st & 1u;
        }
        const size_t pix = out_index(fp, p, po);
        if (redo) {
            redo_put(aux, (uint32_t)pix);
            hits = 0;
        } else {
            store_rgb(fp, pix, acc);
        }
    }
    uint32_t wsum = 0;
#pragma unroll
    for (int b = 0; b < 7; b++) wsum += (uint32_t)__builtin_popcountll(__ballot((hits >> b) & 1u)) << b;
    if ((threadIdx.x & 63) == 0) wave_hits[threadIdx.x >> 6] = wsum;
    __syncthreads();
    if (threadIdx.x == 0 && fp.hit_count) {
        const uint32_t sum = wave_hits[0] + wave_hits[1] + wave_hits[2] + wave_hits[3];
        if (sum) atomicAdd(aux.tile_ctr + RT_HIT_BASE + (p * RT_HIT_SLOTS + fb % RT_HIT_SLOTS) * RT_QUEUE_STRIDE, sum);
    }
}

// Persistent waves over 8x8 tiles; the stack bound of the tree must fit SP
// (the host falls back to the per-lane kernel otherwise), so no push can drop.
// FUSED: each tile is resolved, shaded and stored by its own wave (spp > 1:
// each sample; k_average then forms the pixels).
// Waves per workgroup of the packet kernel (4: seven workgroups per CU at 7
// waves/SIMD).  7-wave workgroups (4 per CU, the LDS argument block shared by
// 7 waves) measured 5% slower: a workgroup's waves land unevenly on the 4
// SIMDs.
#ifndef RT_PACKET_WAVES
#define RT_PACKET_WAVES 4
#endif
constexpr int kPacketWaves = RT_PACKET_WAVES;

// Occupancy target of the packet kernel in waves per SIMD (0: the compiler's
// choice).  The fused resolve's fp64 set-up raises the kernel's VGPR peak
// above the walk's (91 VGPRs, 5 waves); 7 waves (72 VGPRs, 28 B of spills
// per lane in the resolve) measured fastest: 14.48 vs 14.23 (6 waves) and
// 13.64 Grays/s (compiler's choice) on the sponza-proxy orbit.
#ifndef RT_PACKET_WPE
#define RT_PACKET_WPE 7
#endif
#if RT_PACKET_WPE > 0
#define RT_PACKET_ATTR __attribute__((amdgpu_waves_per_eu(RT_PACKET_WPE)))
#else
#define RT_PACKET_ATTR
#endif

// One row of the launch's side de-interleave job (RtLaunchAux::job_*, rank 0
// of a one-process-per-GPU driver: the previous step's gathered shards into
// full frames): row c of the [F][H] frames, 16 B per lane per access when
// both sides allow it.  The copy is memory-bound and the walk is not, so a
// wave that takes a row after a tile (and the waves whose tiles have run
// out) move the frames while the other waves trace, in place of a separate
// kernel that would wait for the persistent grid to drain.
__device__ __forceinline__ void side_copy_row(const RtLaunchAux& a, uint32_t c, int lane) {
    const uint32_t f = c / (uint32_t)a.job_H, j = c - f * (uint32_t)a.job_H;
    const uint64_t n = (uint64_t)a.job_W * (uint64_t)a.job_eb;
    const RT_G uint8_t* src = a.job_src + rt_job_src_row(a, (int)j, (int)f);
    RT_G uint8_t* dst = a.job_dst + ((uint64_t)f * (uint64_t)a.job_H + j) * n;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if ((((uintptr_t)src | (uintptr_t)dst | n) & 15u) == 0) {
        const RT_G u32x4* s4 = reinterpret_cast<const RT_G u32x4*>(src);
        RT_G u32x4* d4 = reinterpret_cast<RT_G u32x4*>(dst);
        const uint32_t n16 = (uint32_t)(n / 16);
        // (6 x 1 KB per round trip: a 1920-pixel rgb row in one)
        for (uint32_t k0 = 0; k0 < n16; k0 += 6 * 64) {
            u32x4 v[6];
#pragma unroll
            for (int u = 0; u < 6; u++) {
                const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
                v[u] = k < n16 ? s4[k] : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < 6; u++) {
                const uint32_t k = k0 + (uint32_t)(u * 64 + lane);
                if (k < n16) out_store(d4 + k, v[u]);
            }
        }
    } else {
        for (uint64_t k = (uint64_t)lane; k < n; k += 64) out_store(dst + k, src[k]);
    }
}
// Claims and copies one row of the side job from the wave's XCD queue xq
// (rows xq, xq + RT_QUEUES, ...); false once the queue's rows are taken.
__device__ __forceinline__ bool side_copy(args_p A, int lane, uint32_t xq) {
    A = launder(A);
    const RtLaunchAux a = kload(&A->aux);
    uint32_t c = 0;
    if (lane == 0) c = xq + RT_QUEUES * atomicAdd(a.tile_ctr + RT_COPY_BASE + xq * RT_QUEUE_STRIDE, 1u);
    c = __builtin_amdgcn_readfirstlane(c);
    if (c >= (uint32_t)a.job_F * (uint32_t)a.job_H) return false;
    side_copy_row(a, c, lane);
    return true;
}

// Sum of a u32 over the wave's active lanes, in every lane.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// The end of a packet launch without a trailing kernel (aux.self_fix; the
// host sets it when the redo list holds an entry for every pixel of the
// launch, so the launch never needs a whole retry).  A trailing k_fixup
// could only start once the next launch's persistent grid, issued on the
// other stream, had drained — it holds every CU's wave slots, SGPRs and LDS
// — so a launch ended one launch late.  Instead every wave,
// once out of tiles:
//  1. waits for its own hit-partial atomics (`s_waitcnt vmcnt(0)`: a
//     device-scope atomic counts as complete once performed), so they are in
//     before its exit ticket;
//  2. takes redo-list entries while untaken ones exist, up to 64 at a time,
//     by a compare-and-swap that never moves the claim counter past the
//     count — an entry is taken only after its append, and the wave that
//     appended it runs this loop afterwards, so every entry is taken — and
//     finishes those pixels with k_fixup's per-lane exact path (its LDS ring
//     is the wave's candidate list, its spill the slot's stack buffer);
//  3. takes an exit ticket.  The wave with the last ticket (every other wave
//     is past steps 1 and 2) folds the per-pose hit partials into the
//     caller's counters, reports the redo count to the host and clears the
//     work-queue block for the next launch — k_fixup's bookkeeping.
// Step 2 out of line, so the kernel body's registers stay as they are
// (inlined, the per-lane exact path raised the fused kernel's spills from
// 36 B to 4 KB of scratch per lane).
template <int W, int K, bool COUNT>
#ifndef RT_REDO_INLINE
#define RT_REDO_INLINE 0
#endif
#if RT_REDO_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
void packet_redo(args_p A, uint2* ring, int lane) {
    // (a call's arguments arrive in VGPRs: the argument block's address made
    // uniform again)
    A = (args_p)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)A);
    A = launder(A);
    const RtLaunchAux aux = kload(&A->aux);
    RT_G uint32_t* const ctr = aux.tile_ctr;
    const uint32_t cap = aux.redo_cap < 0xFFFFFFFFull ? (uint32_t)aux.redo_cap : 0xFFFFFFFFu;
    LaneStack<K, 64> st;
    st.attach_wave(reinterpret_cast<uint2(*)[64]>(ring), aux.spill,
                   blockIdx.x * (64u * kPacketWaves) + threadIdx.x, gridDim.x * (64u * kPacketWaves), lane);
    for (;;) {
        uint32_t lo = 0, hi = 0;
        if (lane == 0) {
            const uint32_t n = __builtin_elementwise_min(atomicAdd(ctr + RT_REDO_COUNT, 0u), cap);
            uint32_t c = atomicAdd(ctr + RT_REDO_CLAIM, 0u);
            while (c < n) {
                const uint32_t e = __builtin_elementwise_min(n, c + 64u);
                const uint32_t prev = atomicCAS(ctr + RT_REDO_CLAIM, c, e);
                if (prev == c) {
                    lo = c;
                    hi = e;
                    break;
                }
                c = prev;
            }
        }
        lo = uni(lo);
        hi = uni(hi);
        if (lo >= hi) break;
        uint32_t v = kRedoEmpty;
        if ((uint32_t)lane < hi - lo) {
            // (the append's count came first: its entry lands within a round
            // trip; a spin past 2^22 sleeps means the all-kRedoEmpty
            // invariant is broken: the lane gives the entry up and the launch
            // reports it to the host, which fails the next call on the slot —
            // rt_api.cpp launch — instead of hanging the GPU)
            uint32_t spins = 0;
            while ((v = atomicExch(aux.redo + lo + (uint32_t)lane, kRedoEmpty)) == kRedoEmpty) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins == (1u << 22)) break;
            }
            if (v == kRedoEmpty) (void)atomicOr(ctr + RT_EXIT_ERROR, 1u);
        }
        if (v != kRedoEmpty) {
            const RtDevScene sc = kload(&A->sc);
            const RtFrameParams fp = kload(&A->fp);  // (its pose array is never indexed here)
            const uint32_t npix = (uint32_t)fp.W * (uint32_t)fp.nrows;
            const uint32_t ob = v & ~kRedoPass1;  // pixel of the batch: pose * npix + pixel
            const int p = (int)(ob / npix);
            const uint32_t o = ob - (uint32_t)p * npix;
            // the lane's pose, read out of the LDS argument block by the lane
            // itself (lanes may hold different poses)
            RtPose pose;
            {
                const __attribute__((address_space(3))) uint32_t* src =
                    (const __attribute__((address_space(3))) uint32_t*)&A->fp.pose[p];
                uint32_t* dst = reinterpret_cast<uint32_t*>(&pose);
#pragma unroll
                for (unsigned w = 0; w < sizeof(RtPose) / 4; w++) dst[w] = src[w];
            }
            const uint32_t hits = trace_pixel_at<W, K, COUNT>(sc, fp, pose, p, (int)(o % (uint32_t)fp.W),
                                                              (int)(o / (uint32_t)fp.W), st,
                                                              (v & kRedoPass1) ? 1 : 0, true);
            // into the pose's partials, which the last wave folds (or stores)
            if (hits) atomicAdd(ctr + RT_HIT_BASE + (p * RT_HIT_SLOTS + lane) * RT_QUEUE_STRIDE, hits);
        }
    }
}

template <int W, int K, bool COUNT>
__device__ __forceinline__ void packet_exit(args_p A, uint2* ring, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    A = launder(A);
    RT_G uint32_t* const ctr = kload(&A->aux.tile_ctr);
    // (a cheap check first: the call only when entries are waiting)
    uint32_t pending = 0;
    if (lane == 0) pending = atomicAdd(ctr + RT_REDO_COUNT, 0u) > atomicAdd(ctr + RT_REDO_CLAIM, 0u);
    // (RT_NO_REDO=1: a measurement build without the redo call — and its
    // callee frame in the private segment; wrong results if any pixel needs
    // a redo, never shipped)
#if !defined(RT_NO_REDO) || !RT_NO_REDO
    if (uni(pending)) packet_redo<W, K, COUNT>(A, ring, lane);
#else
    (void)pending;
#endif
    // Ordering of the partials before the exit ticket.  Every value the
    // waves exchange here (hit partials, redo entries, claim and ticket
    // counters) is written and read by device-scope atomic RMWs, which
    // gfx950 performs at the memory side, past the XCDs' L2s; a wave's
    // `s_waitcnt vmcnt(0)` before its ticket waits until its own atomics are
    // performed, so the last ticket holder's atomicExch reads see them all.
    // The HIP memory model would ask for a release ticket and an acquire in
    // the last wave; at agent scope those compile to an L2 write-back per
    // exiting wave (7,168 per launch) and an L2 invalidate, and measured
    // (RT_EXIT_FENCE=1, round 6, one box, 20-step runs): 16.96 / 17.38 G in
    // the good runs but 3.7 and 0.76 Grays/s in two of six — sporadic
    // whole-launch stalls — against 17.08-17.14 in every run without them.
    uint32_t tk = 0;
#if defined(RT_EXIT_FENCE) && RT_EXIT_FENCE
    if (lane == 0)
        tk = __hip_atomic_fetch_add(ctr + RT_EXIT_COUNT, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
#else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) tk = atomicAdd(ctr + RT_EXIT_COUNT, 1u) + 1u;
#endif
    if (uni(tk) != gridDim.x * (uint32_t)kPacketWaves) return;
#if defined(RT_EXIT_FENCE) && RT_EXIT_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    // the last wave: per pose, the 64 spread partials (one per lane) summed,
    // then added to the caller's counter or (RT_SELF_STORE) stored in it
    A = launder(A);
    const int poses = kword(&A->fp.nframes) / kword(&A->fp.spp);
    RT_G unsigned long long* const hc = kload(&A->fp.hit_count);
#if !defined(RT_STORE_COUNTS) || RT_STORE_COUNTS
    const bool store = (kword(&A->aux.self_fix) & RT_SELF_STORE) != 0;
#else
    const bool store = false;  // (bisection build: always add)
#endif
    // (poses in groups of 12, each group's exchanges in flight together:
    // three round trips for 36 poses, 12 registers — an unrolled 36-entry
    // array went to the private segment, 144 B per lane)
#ifndef RT_FOLD_GROUP
#define RT_FOLD_GROUP 12
#endif
    constexpr int kFold = RT_FOLD_GROUP;
    for (int m0 = 0; m0 < poses; m0 += kFold) {
        uint32_t part[kFold];
#pragma unroll
        for (int k = 0; k < kFold; k++)
            part[k] = m0 + k < poses
                          ? atomicExch(ctr + RT_HIT_BASE + ((m0 + k) * RT_HIT_SLOTS + lane) * RT_QUEUE_STRIDE, 0u)
                          : 0u;
#pragma unroll
        for (int k = 0; k < kFold; k++) {
            const uint32_t s = wave_sum_u32(part[k]);
            if (m0 + k < poses && lane == 0 && hc) {
                if (store)
                    __hip_atomic_store(hc + m0 + k, (unsigned long long)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (s)
                    atomicAdd(hc + m0 + k, (unsigned long long)s);
            }
        }
    }
    if (lane < RT_QUEUES) {
        (void)atomicExch(ctr + lane * RT_QUEUE_STRIDE, 0u);
        (void)atomicExch(ctr + RT_COPY_BASE + lane * RT_QUEUE_STRIDE, 0u);
    }
    if (lane == 0) {
        // the redo count to the host (RT_SEEN_ERROR: an entry was given up)
        const uint32_t n = atomicExch(ctr + RT_REDO_COUNT, 0u);
        const uint32_t err = atomicExch(ctr + RT_EXIT_ERROR, 0u);
        uint32_t* const seen = kload(&A->aux.redo_seen);
        if (seen) __hip_atomic_store(seen, n | (err ? RT_SEEN_ERROR : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        (void)atomicExch(ctr + RT_POOL_COUNT, 0u);
        (void)atomicExch(ctr + RT_REDO_CLAIM, 0u);
        (void)atomicExch(ctr + RT_EXIT_COUNT, 0u);
    }
}

#ifndef RT_SCRATCH_PAD
#define RT_SCRATCH_PAD 4096
#endif

// The launch's tile geometry, computed once per block into LDS (RT_TILE_GEOM,
// default): the per-tile claim then divides by the tiles per frame and per
// tile row with a multiply-high and a shift instead of two runtime integer
// divisions (a float-reciprocal sequence each, ~50 scalar instructions per
// tile with the signed divisions by constants).
#ifndef RT_TILE_GEOM
#define RT_TILE_GEOM 1
#endif
struct TileGeom {
    uint32_t tiles_x, tiles_f, tiles, claim;
    uint32_t mf, sf, mx, sx;  // n / tiles_f = (n * mf) >> sf, n / tiles_x = (n * mx) >> sx, for n < 2^31
};
// m = ceil(2^(31+l) / d), l = ceil(log2 d): for n < 2^31, floor(n m / 2^(31+l))
// = floor(n / d), since m d - 2^(31+l) < d <= 2^l and n < 2^31 (m < 2^32)
__device__ __forceinline__ void div_magic(uint32_t d, uint32_t& m, uint32_t& sh) {
    const uint32_t l = d > 1u ? 32u - (uint32_t)__builtin_clz(d - 1u) : 0u;
    const uint64_t P = 1ull << (31u + l);
    // (an fp64 quotient within one of P / d, then the exact ceiling by
    // multiplies: no 64-bit integer division)
    uint32_t q = (uint32_t)fmin((double)P / (double)d, 4294967295.0);
    while ((uint64_t)q * d < P) q++;
    while (q > 1u && (uint64_t)(q - 1u) * d >= P) q--;
    m = q;
    sh = 31u + l;
}
__device__ __forceinline__ uint32_t div_by(uint32_t n, uint32_t m, uint32_t sh) {
    return (uint32_t)(((uint64_t)n * m) >> sh);
}

// JOB: the launch carries a side de-interleave job (RtLaunchAux::job_*; its
// own instantiation, so the kernels without one keep their registers).
template <int W, int SP, int K, bool COUNT, bool FUSED, bool PACK = false, bool JOB = false, bool PATHS = false>
__global__ void __launch_bounds__(64 * kPacketWaves) RT_PACKET_ATTR k_trace_packet(PacketArgs args) {
    __shared__ uint32_t stacks[kPacketWaves][SP];
    __shared__ uint2 cands[kPacketWaves][K * 64];
    __shared__ PacketArgs s_args;
    __shared__ TileGeom s_geom;
    constexpr bool pack = FUSED && PACK;  // (launched only when fp.pack)
    {
        const __attribute__((address_space(4))) uint32_t* src =
            (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
        uint32_t* dst = reinterpret_cast<uint32_t*>(&s_args);
        for (unsigned w = threadIdx.x; w < sizeof(PacketArgs) / 4; w += blockDim.x) dst[w] = src[w];
        if constexpr (RT_TILE_GEOM != 0) {
            __syncthreads();
            if (threadIdx.x == 0) {
                // fp.pack: a tile is ts x ts pixels of one pose with all spp
                // samples (ts = 8 / n), else 8 x 8 pixels of one sample frame
                // (from the LDS copy: the kernel argument itself stays unread)
                const RtFrameParams& f = s_args.fp;
                const uint32_t ts = pack ? 8u / (uint32_t)f.spp_n : (uint32_t)RT_TILE_W;
                const uint32_t th = pack ? ts : 64u / RT_TILE_W;
                TileGeom g;
                g.tiles_x = ((uint32_t)f.W + ts - 1u) / ts;
                g.tiles_f = g.tiles_x * (((uint32_t)f.nrows + th - 1u) / th);  // tiles per frame (pose when packed)
                g.tiles = g.tiles_f * (uint32_t)(pack ? f.nframes / f.spp : f.nframes);
                g.claim = g.tiles >= 64u * gridDim.x * kPacketWaves ? 2u : 1u;
                div_magic(g.tiles_f, g.mf, g.sf);
                div_magic(g.tiles_x, g.mx, g.sx);
                s_geom = g;
            }
        }
        __syncthreads();
    }
    args_p A = (args_p)&s_args;
    typedef const __attribute__((address_space(3))) TileGeom* geom_p;
    geom_p G = (geom_p)&s_geom;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    // tile scheduling: one queue per XCD (blocks are dealt to the 8 XCDs
    // round-robin, so block b's XCD is b % 8): slot s of queue x is tile
    // queue_tile(x, s) — runs of RT_TILE_RUN consecutive tiles, every 8th
    // run; every queue is drained by the blocks b = x mod 8.
    const uint32_t xq = blockIdx.x % RT_QUEUES;
    bool first = true;
    // one atomic claims `claim` consecutive slots of the queue: 2 when there
    // are many tiles per wave (the orbit at full size: +1.2%), else 1 (at the
    // size of an 8-GPU shard a second slot per claim lengthens the tail: -1.6%)
    int pend = -1, pend_n = 0;  // the claim's next tile, slots used of it
    int claim = 1;
    // FUSED: hits of the wave's tiles of frame hf, added to one of the
    // frame's spread counters when the wave moves on to another frame
    uint32_t hacc = 0;
    int hf = -1;
    const uint32_t hslot = (blockIdx.x * kPacketWaves + (uint32_t)wv) % RT_HIT_SLOTS;
    bool job = JOB;  // rows of the side job may be left
    for (;;) {
        A = launder(A);
        // (laundered like A: the geometry is re-read per tile, not held in
        // SGPRs across the walk)
        asm volatile("" : "+s"(G));
        const int W_ = kword(&A->fp.W), nrows = kword(&A->fp.nrows);
        // fp.pack: a tile is ts x ts pixels of one pose with all spp samples
        // (ts = 8 / n), else 8 x 8 pixels of one sample frame
        const int spp = kword(&A->fp.spp);
        const int ts = pack ? 8 / kword(&A->fp.spp_n) : RT_TILE_W;
        int tiles_x, tiles_f, tiles;
        if constexpr (RT_TILE_GEOM != 0) {
            tiles_x = (int)kword(&G->tiles_x);
            tiles_f = (int)kword(&G->tiles_f);
            tiles = (int)kword(&G->tiles);
            claim = (int)kword(&G->claim);
        } else {
            const int th = pack ? ts : 64 / RT_TILE_W;
            tiles_x = (W_ + ts - 1) / ts;
            tiles_f = tiles_x * ((nrows + th - 1) / th);  // tiles per frame (pose when packed)
            tiles = tiles_f * (pack ? kword(&A->fp.nframes) / spp : kword(&A->fp.nframes));
            claim = tiles >= 64 * (int)(gridDim.x * kPacketWaves) ? 2 : 1;
        }
        int s = 0;
        bool claimed = false;
        if (pend >= 0) {  // the rest of the last claim
            s = pend;
            pend = (++pend_n < claim) ? pend + 1 : -1;
        } else if (first) {
            // a wave's first tile is its own slot in the queue (no atomic: the
            // whole grid starting at once would serialise on the 8 counters
            // for ~10 us); the counter hands out the slots after the XCD's waves
            first = false;
            s = (int)((blockIdx.x / RT_QUEUES) * kPacketWaves + wv);
        } else {
            claimed = true;
            if (lane == 0) {
                const uint32_t nwq = kPacketWaves * ((gridDim.x + RT_QUEUES - 1 - xq) / RT_QUEUES);  // waves of queue xq
                s = (int)(nwq + (uint32_t)claim * atomicAdd(kload(&A->aux.tile_ctr) + xq * RT_QUEUE_STRIDE, 1u));
            }
        }
        const int slot = __builtin_amdgcn_readlane(s, 0);  // wave-uniform: a uniform loop exit
        if (claimed && claim > 1) {  // the claim's further slots
            pend = slot + 1;
            pend_n = 1;
        }
        // (increasing with the slot: the first tile past the end ends the queue)
        // (slot >= 0: unsigned arithmetic, shifts for the constant divisors)
        const int tile = (int)((((uint32_t)slot / RT_TILE_RUN) * RT_QUEUES + xq) * RT_TILE_RUN +
                               (uint32_t)slot % RT_TILE_RUN);
        if (tile >= tiles) {
            if constexpr (JOB)
                while (job) job = side_copy(A, lane, xq);  // the job's rows the tiles left
            break;
        }
        int fr, ft, ty, tx;
        if constexpr (RT_TILE_GEOM != 0) {  // (tile < tiles < 2^31)
            fr = (int)div_by((uint32_t)tile, kword(&G->mf), kword(&G->sf));  // frame of the batch (pose when packed)
            ft = tile - fr * tiles_f;
            ty = (int)div_by((uint32_t)ft, kword(&G->mx), kword(&G->sx));
            tx = ft - ty * tiles_x;
        } else {
            fr = tile / tiles_f;  // frame of the batch (pose when packed)
            ft = tile - fr * tiles_f;
            ty = ft / tiles_x;
            tx = ft - ty * tiles_x;
        }
        int f = fr, i, r;
        if constexpr (pack) {  // lane = pixel * spp + sample
            const int pl = lane / spp;
            f = fr * spp + (lane & (spp - 1));
            i = tx * ts + pl % ts;
            r = ty * ts + pl / ts;
        } else {
            i = tx * RT_TILE_W + (lane & (RT_TILE_W - 1));
            r = ty * (64 / RT_TILE_W) + lane / RT_TILE_W;
        }
        const TileOut o =
            trace_packet<W, SP, K, COUNT, FUSED, PACK, PATHS>(A, f, i, r, i < W_ && r < nrows, stacks[wv], cands[wv]);
        if constexpr (FUSED) {
            uint32_t h = (uint32_t)__builtin_popcountll(__ballot(o.hit));
            if constexpr (pack) {  // samples hit per pixel (<= 64) summed over the wave
                h = 0;
#pragma unroll
                for (int b = 0; b < 7; b++) h += (uint32_t)__builtin_popcountll(__ballot((o.hits >> b) & 1u)) << b;
            }
            if (fr != hf) {
                if (hacc != 0 && lane == 0)
                    atomicAdd(kload(&A->aux.tile_ctr) + RT_HIT_BASE + (hf * RT_HIT_SLOTS + hslot) * RT_QUEUE_STRIDE,
                              hacc);
                hacc = 0;
                hf = fr;
            }
            hacc += h;
        }
        if constexpr (JOB)
            if (job) job = side_copy(A, lane, xq);  // one row of the side job per tile
    }
    if (FUSED && hacc != 0 && lane == 0)
        atomicAdd(kload(&launder(A)->aux.tile_ctr) + RT_HIT_BASE + (hf * RT_HIT_SLOTS + hslot) * RT_QUEUE_STRIDE,
                  hacc);
    if constexpr (FUSED)
        if (kword(&launder(A)->aux.self_fix)) packet_exit<W, K, COUNT>(A, cands[wv], lane);
#if RT_SCRATCH_PAD > 0
    // RT_SCRATCH_PAD bytes of private segment per lane, touched only on a
    // path no launch takes.  The HIP runtime manages a dispatch's scratch by
    // its size: with the kernel's own 408 B (or 20 B in a 6-wave build) two
    // streams' overlapped launches slowed the device 4-70x in most runs (31
    // of 37, round 6); with 4.5 KB per lane — round 5's frame size, which
    // round 5 had by accident — 6 of 6 ran at full speed, with or without
    // a zero fill between launches.  Never read or written in
    // a real launch: the cost is the runtime's scratch reservation only.
    if (kword(&launder(A)->fp.W) == -12345) {
        volatile uint32_t pad[RT_SCRATCH_PAD / 4];
        pad[lane % (RT_SCRATCH_PAD / 4)] = (uint32_t)lane;
        pad[(lane * 7) % (RT_SCRATCH_PAD / 4)] += 1u;
    }
#endif
}

// v_mbcnt_lo_u32_b32: bits of m set below this lane (lanes 0-31; m = ~0: the
// lane id).  volatile: recomputed at each use rather than held across a loop.
__device__ __forceinline__ uint32_t mbcnt_lo(uint32_t m) {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, %1, 0" : "=v"(v) : "s"(m));
    return v;
}

// --------------------------------------------------------------------------
// R rays per lane (spp = 1, fused resolve): a wave walks an (8 R) x 8 pixel
// tile, lane l holding the R horizontally adjacent pixels (8 R tx + R (l & 7)
// + k, 8 ty + (l >> 3)), k < R.  Node steps per tile grow far slower than the
// tile (the tree's depth sets most of them: 8x8 tiles 12.36 per tile, 4x4
// pixels of packed samples 11.47), while a node step's scalar work — the
// child-record loads and their round trip, the any-lane mask, the near-child
// pick, the pushes and pops — is paid once per wave however many rays test
// the children.  With R = 2 each step serves 128 rays.
//
// Each ray keeps K LDS candidates (entry c of ray k of lane l at
// cand[(c R + k) 64 + l]: R K entries per lane, the same LDS as the
// one-ray kernel's K R); past them the K nearest lower bounds are kept and
// the smallest dropped bound certifies the winner (else the pixel is redone
// by k_fixup) — no overflow pool.  The resolve runs ray by ray.
// Returns the lane's hits (bit k: ray k resolved here and hit).
template <int W, int SP, int K, int R, bool COUNT>
__device__ __forceinline__ uint32_t trace_packet_r(args_p A, int f, int i0, int r, const bool (&valid)[R],
                                                   uint32_t* __restrict__ wstack, uint2* __restrict__ cand) {
    const int lane = threadIdx.x & 63;
    Ray32 q[R];
    float tsl, pd;
    uint32_t ob0;  // the lane's first pixel in the batch (ray k: ob0 + k)
    {
        const RtFrameParams fp = kload(&A->fp);
        const RtFrameCam cam = frame_cam_of(kload(&A->fp.pose[f]), fp, f);
        const int j = rt_image_row(fp.row0, fp.row_stride, fp.band, valid[0] ? r : 0);
#pragma unroll
        for (int k = 0; k < R; k++) {
            const Ray64 ray = gen_ray(fp, cam, valid[k] ? i0 + k : 0, j);
            q[k] = make_ray32(ray, cam.pad);
        }
        tsl = round_up_f(0x1p-40 * ((double)q[0].co + 1.0));
        pd = cam.pad;
        ob0 = (uint32_t)out_index(fp, f, (size_t)(valid[0] ? r : 0) * fp.W + (valid[0] ? i0 : 0));
    }
    // the tile's octant: lane 0's first ray's direction signs, if every ray
    // that takes part shares them (else 8, the general slab test)
    uint32_t lsg[R];
    bool mixed = false;
#pragma unroll
    for (int k = 0; k < R; k++) {
        lsg[k] = (q[k].ix < 0.f ? 1u : 0u) | (q[k].iy < 0.f ? 2u : 0u) | (q[k].iz < 0.f ? 4u : 0u);
    }
    const uint32_t dsg = uni(lsg[0]);
#pragma unroll
    for (int k = 0; k < R; k++) mixed |= valid[k] && lsg[k] != dsg;
    const int oct = __ballot(mixed) == 0 ? (int)dsg : 8;
    const RT_G uint8_t* const nodes = kload(&A->sc.nodes);
    const RT_G float* const tri32 = kload(&A->sc.tri32);
    f2 nox[R], noy[R], noz[R];
    float tcull[R], drop[R];
    int nc[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
        nox[k] = f2{-(q[k].ox + pd) * q[k].ix, -(q[k].ox - pd) * q[k].ix};
        noy[k] = f2{-(q[k].oy + pd) * q[k].iy, -(q[k].oy - pd) * q[k].iy};
        noz[k] = f2{-(q[k].oz + pd) * q[k].iz, -(q[k].oz - pd) * q[k].iz};
        tcull[k] = valid[k] ? __builtin_huge_valf() : -1.f;
        drop[k] = __builtin_huge_valf();
        nc[k] = 0;
    }
    uint32_t n_nodes = 0, n_pre = 0, w_nodes = 0, w_leaves = 0, w_tris = 0, w_empty = 0;  // COUNT only
    uint32_t cur = kword(&A->sc.root_ref);
    if (!(cur & RT_LEAF_BIT)) cur |= kword(&A->sc.root_meta) << 24;
    {
        float b[1][6];
        for (int a = 0; a < 6; a++) b[0][a] = kword(&A->sc.root_box[a]);
        uint64_t any = 0;
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint64_t h[1];
            child_hits<1, -1>(b, q[k], nox[k], noy[k], noz[k], tcull[k], h);
            any |= h[0];
        }
        if (any == 0) cur = RT_INVALID_REF;
    }
    int sp = 0;
    // candidate list of ray k: entry c at cand[(c * R + k) * 64 + lane]
    auto entry = [&](int c, int k) -> uint2& { return cand[(c * R + k) * 64 + lane]; };
    auto walk = [&]<int OCT>() __attribute__((always_inline)) {
        if (cur == RT_INVALID_REF) return;
        for (;;) {
            if (!(cur & RT_LEAF_BIT)) {
                if (COUNT) w_nodes++;
                float bx[W][6];
                uint32_t rs[W];
                const uint32_t meta = cur >> 24;
                const uint32_t nv = meta >> 2;
                uint64_t hm[W];
                {
                    const cchild_p nb = (cchild_p)(nodes + (size_t)(cur & 0x00FFFFFFu) * (32 * W));
                    ChildRec ch[W];
#pragma unroll
                    for (int c = 0; c < W; c++) ch[c] = load_child(nb + c);
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        bx[c][0] = ch[c].lx; bx[c][1] = ch[c].hx; bx[c][2] = ch[c].ly;
                        bx[c][3] = ch[c].hy; bx[c][4] = ch[c].lz; bx[c][5] = ch[c].hz;
                    }
#pragma unroll
                    for (int c = 0; c < W; c++) rs[c] = ch[c].pad;  // ref | meta << 24 (bvh_build.cpp flatten)
                    // child c is needed if any ray of any lane enters it
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        bool in = false;
#pragma unroll
                        for (int k = 0; k < R; k++) {
                            const float (&bc)[6] = bx[c];
                            const float tlx = __builtin_fmaf(bc[0], q[k].ix, nox[k].x),
                                        thx = __builtin_fmaf(bc[1], q[k].ix, nox[k].y);
                            const float tly = __builtin_fmaf(bc[2], q[k].iy, noy[k].x),
                                        thy = __builtin_fmaf(bc[3], q[k].iy, noy[k].y);
                            const float tlz = __builtin_fmaf(bc[4], q[k].iz, noz[k].x),
                                        thz = __builtin_fmaf(bc[5], q[k].iz, noz[k].y);
                            float t0, t1;
                            if constexpr (OCT < 0) {
                                t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
                                t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull[k]));
                            } else {
                                const float nx = (OCT & 1) ? thx : tlx, fx = (OCT & 1) ? tlx : thx;
                                const float ny = (OCT & 2) ? thy : tly, fy = (OCT & 2) ? tly : thy;
                                const float nz = (OCT & 4) ? thz : tlz, fz = (OCT & 4) ? tlz : thz;
                                t0 = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
                                t1 = fminf(fminf(fx, fy), fminf(fz, tcull[k]));
                            }
                            in |= t0 <= t1;
                        }
                        hm[c] = __ballot(in);
                    }
                }
                const uint32_t mask = any_mask<W>(hm) & ((1u << nv) - 1u);
                if (COUNT) w_empty += mask == 0;
                if (mask != 0) {
                    const bool rev = (dsg >> (meta & 3u)) & 1u;
                    const int near_c = rev ? 31 - __builtin_clz(mask) : __builtin_ctz(mask);
                    const uint32_t pm = mask & ~(1u << near_c);
                    if (pm != 0) {
                        const uint32_t refv = lanes_of<W>(rs);
                        // the slot from the lane's own position in pm, with the
                        // lane id made here (v_mbcnt) instead of kept live across
                        // the walk: no register, no spill reload on the push path
                        const uint32_t lid = mbcnt_lo(~0u);  // lane id (lanes < 32)
                        const uint32_t below = mbcnt_lo(pm);  // pm's bits below the lane
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
                if (COUNT) {
                    w_leaves++;
                    w_tris += cnt;
                }
                const uint32_t end = first + cnt;
                for (uint32_t k0 = first; k0 < end; k0 += kLeafChunk) {
                    const cfloat_p Rp = (cfloat_p)(tri32 + 12 * (size_t)k0);
                    float4 TA[kLeafChunk], TB[kLeafChunk], TC[kLeafChunk];
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) {
                        TA[t] = load_f4(Rp + 12 * t);
                        TB[t] = load_f4(Rp + 12 * t + 4);
                        TC[t] = load_f4(Rp + 12 * t + 8);
                    }
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) pin_s(TA[t], TB[t], TC[t]);
#pragma unroll
                    for (int t = 0; t < kLeafChunk; t++) {
                        const uint32_t tri = k0 + t;
                        if (tri >= end) break;
                        int cls[R];
                        float tl[R], tu[R];
                        bool anyc = false;
#pragma unroll
                        for (int k = 0; k < R; k++) {
                            if (COUNT) n_pre += valid[k];
                            cls[k] = valid[k] ? tri_classify(TA[t], TB[t], TC[t], q[k].ox, q[k].oy, q[k].oz, q[k].dx,
                                                             q[k].dy, q[k].dz, q[k].co, tcull[k], tl[k], tu[k])
                                              : 0;
                            anyc |= cls[k] != 0;
                        }
                        if (__ballot(anyc) == 0) continue;
#pragma unroll
                        for (int k = 0; k < R; k++) {
                            if (cls[k] == 0) continue;
                            if (cls[k] == 2) tcull[k] = fminf(tcull[k], (tu[k] + tsl) * (1.f + 0x1p-20f));
                            if (nc[k] == K) {  // full: compact against the culling distance
                                int m = 0;
                                for (int c = 0; c < K; c++) {
                                    const uint2 e = entry(c, k);
                                    if (__uint_as_float(e.y) <= tcull[k]) entry(m++, k) = e;
                                }
                                nc[k] = m;
                            }
                            if (nc[k] < K) {
                                entry(nc[k], k) = make_uint2(tri, __float_as_uint(tl[k]));
                                nc[k]++;
                            } else {
                                // keep the K smallest lower bounds; the smallest
                                // dropped bound certifies the winner
                                int far_c = 0;
                                float far_t = __uint_as_float(entry(0, k).y);
                                for (int c = 1; c < K; c++) {
                                    const float tt = __uint_as_float(entry(c, k).y);
                                    if (tt > far_t) { far_t = tt; far_c = c; }
                                }
                                if (tl[k] >= far_t) {
                                    drop[k] = fminf(drop[k], tl[k]);
                                } else {
                                    entry(far_c, k) = make_uint2(tri, __float_as_uint(tl[k]));
                                    drop[k] = fminf(drop[k], far_t);
                                }
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
    A = launder(A);
    const RtFrameParams fp = kload(&A->fp);
    if (COUNT && fp.counters && lane == 0) {
        atomicAdd(&fp.counters[7], (unsigned long long)w_nodes);
        atomicAdd(&fp.counters[8], (unsigned long long)w_leaves);
        atomicAdd(&fp.counters[9], 1ull);
        atomicAdd(&fp.counters[12], (unsigned long long)w_tris);
        atomicAdd(&fp.counters[15], (unsigned long long)w_empty);
    }
    if (COUNT) {
#pragma unroll
        for (int k = 0; k < R; k++) n_nodes += valid[k] ? w_nodes : 0u;
    }
    uint32_t hits = 0;
    const RtLaunchAux aux = kload(&A->aux);
    const RtDevScene sc = kload(&A->sc);
    const RtFrameCam cam = frame_cam_of(kload(&A->fp.pose[f]), fp, f);
    uint32_t u_tests = 0, u_win = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
        // ray k's list compacted against its final culling distance
        uint32_t nl = 0;
        for (int c = 0; c < nc[k]; c++) {
            const uint2 e = entry(c, k);
            if (__uint_as_float(e.y) <= tcull[k]) entry(nl++, k) = e;
        }
        if (!valid[k]) nl = 0;
        const bool dropped = valid[k] && drop[k] < __builtin_huge_valf() && drop[k] <= tcull[k];
        Best out;
        Shade sh;
        ResolveCounts rc;
        uint32_t redo = 0;
        if (valid[k]) {
            redo = resolve_list<COUNT>(
                sc, fp, cam, i0 + k, rt_image_row(fp.row0, fp.row_stride, fp.band, r), nl,
                nl ? entry(0, k) : make_uint2(0u, 0u), [&](uint32_t c) { return entry(c, k); }, nullptr, dropped,
                drop[k], out, sh, rc);
            const uint32_t ob = ob0 + (uint32_t)k;
            if (redo) {
                redo_put(aux, ob | (redo == 2u ? kRedoPass1 : 0u));
            } else {
                store_sample(fp, ob, out, sh);
                double c[3];
                shade_color(cam, out, sh, c);
                store_rgb(fp, ob, c);
                if (out.tri >= 0) hits |= 1u << k;
            }
        } else {
            out.tri = -1;
        }
        if (COUNT && fp.counters) {
            u_tests += wave_distinct(nl, [&](uint32_t c) { return entry(c, k).x; });
            u_win += wave_distinct(valid[k] && out.tri >= 0 ? 1u : 0u, [&](uint32_t) { return (uint32_t)out.tri; });
            if (valid[k]) {
                atomicAdd(&fp.counters[0], 1ull);
                atomicAdd(&fp.counters[2], (unsigned long long)rc.tris);
                atomicAdd(&fp.counters[3], (unsigned long long)rc.chain);
                if (!redo && out.tri >= 0) atomicAdd(&fp.counters[4], 1ull);
                atomicAdd(&fp.counters[5], (unsigned long long)rc.chain_nodes);
                if (redo == 1) atomicAdd(&fp.counters[10], 1ull);
                if (redo == 2) atomicAdd(&fp.counters[11], 1ull);
                if (dropped) atomicAdd(&fp.counters[14], 1ull);
            }
        }
    }
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
        if (lane == 0) {
            atomicAdd(&fp.counters[16], (unsigned long long)u_tests);
            atomicAdd(&fp.counters[17], (unsigned long long)u_win);
        }
    }
    return hits;
}

// Persistent waves over (8 R) x 8 tiles, spp = 1 with the fused resolve
// (k_trace_packet's queues, claims and hit-count partials).
template <int W, int SP, int K, int R, bool COUNT>
__global__ void __launch_bounds__(64 * kPacketWaves) RT_PACKET_ATTR k_trace_packet_r(PacketArgs args) {
    __shared__ uint32_t stacks[kPacketWaves][SP];
    __shared__ uint2 cands[kPacketWaves][K * R * 64];
    __shared__ PacketArgs s_args;
    {
        const __attribute__((address_space(4))) uint32_t* src =
            (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
        uint32_t* dst = reinterpret_cast<uint32_t*>(&s_args);
        for (unsigned w = threadIdx.x; w < sizeof(PacketArgs) / 4; w += blockDim.x) dst[w] = src[w];
        __syncthreads();
    }
    args_p A = (args_p)&s_args;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const uint32_t xq = blockIdx.x % RT_QUEUES;
    bool first = true;
    int pend = -1, pend_n = 0;
    int claim = 1;
    uint32_t hacc = 0;
    int hf = -1;
    const uint32_t hslot = (blockIdx.x * kPacketWaves + (uint32_t)wv) % RT_HIT_SLOTS;
    for (;;) {
        A = launder(A);
        const int W_ = kword(&A->fp.W), nrows = kword(&A->fp.nrows);
        const int tiles_x = (W_ + 8 * R - 1) / (8 * R);
        const int tiles_f = tiles_x * ((nrows + 7) / 8);
        const int tiles = tiles_f * kword(&A->fp.nframes);
        claim = tiles >= 64 * (int)(gridDim.x * kPacketWaves) ? 2 : 1;
        int t = 0;
        bool claimed = false;
        if (pend >= 0) {
            t = pend;
            pend = (++pend_n < claim) ? pend + RT_QUEUES : -1;
        } else if (first) {
            first = false;
            t = (int)(xq + RT_QUEUES * ((blockIdx.x / RT_QUEUES) * kPacketWaves + wv));
        } else {
            claimed = true;
            if (lane == 0) {
                const uint32_t nwq = kPacketWaves * ((gridDim.x + RT_QUEUES - 1 - xq) / RT_QUEUES);
                t = (int)(xq + RT_QUEUES * (nwq + (uint32_t)claim * atomicAdd(kload(&A->aux.tile_ctr) +
                                                                                  xq * RT_QUEUE_STRIDE, 1u)));
            }
        }
        const int tile = __builtin_amdgcn_readlane(t, 0);
        if (claimed && claim > 1) {
            pend = tile + RT_QUEUES;
            pend_n = 1;
        }
        if (tile >= tiles) break;
        const int fr = tile / tiles_f;
        const int ft = tile - fr * tiles_f;
        const int ty = ft / tiles_x, tx = ft - ty * tiles_x;
        const int i0 = tx * 8 * R + (lane & 7) * R, r = ty * 8 + (lane >> 3);
        bool valid[R];
#pragma unroll
        for (int k = 0; k < R; k++) valid[k] = i0 + k < W_ && r < nrows;
        const uint32_t hits = trace_packet_r<W, SP, K, R, COUNT>(A, fr, i0, r, valid, stacks[wv], cands[wv]);
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < R; k++) h += (uint32_t)__builtin_popcountll(__ballot((hits >> k) & 1u));
        if (fr != hf) {
            if (hacc != 0 && lane == 0)
                atomicAdd(kload(&A->aux.tile_ctr) + RT_HIT_BASE + (hf * RT_HIT_SLOTS + hslot) * RT_QUEUE_STRIDE, hacc);
            hacc = 0;
            hf = fr;
        }
        hacc += h;
    }
    if (hacc != 0 && lane == 0)
        atomicAdd(kload(&launder(A)->aux.tile_ctr) + RT_HIT_BASE + (hf * RT_HIT_SLOTS + hslot) * RT_QUEUE_STRIDE,
                  hacc);
}
