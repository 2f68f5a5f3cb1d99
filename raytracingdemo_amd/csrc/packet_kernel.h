// Wave-cooperative ("packet") exact traversal kernel for gfx950.
// Included by render.hip inside its anonymous namespace (uses Ray32, Win,
// make_ray32, trace_exact and the rtk helpers).
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
// outside the image carry tcull = -1, which fails every test.
//
// The walk itself is fp32 only.  Leaf triangles go through tri_classify:
// rejected, "certain" (the fp64 test provably passes and its t is bounded
// above, so the culling distance tightens at once) or "borderline".  Both
// kinds of survivor are appended to the lane's candidate list in LDS (index +
// lower bound of t).  After the walk the survivors that can still win go to
// HBM, and k_resolve (one pixel per lane, full occupancy) runs the exact fp64
// Moller-Trumbore, picks the (distance, visit rank) minimum and re-verifies
// the winner's reference ancestor chain.  A pixel whose list overflowed, or
// whose winner the reference could not see, is appended to the redo list and
// finished by k_fixup (the per-lane kernel).  Keeping fp64 out of
// the walk keeps it at < 64 VGPRs.
#pragma once

// Tile scheduling of the packet kernel: 0 one device-wide queue, 1 one queue
// per XCD over interleaved tile columns (default), 2 static round-robin
// (diagnostic), 3 one queue per XCD over a contiguous band of tile rows (the
// XCD's L2 holds its band's subtrees), stealing from the other bands once
// its own is drained.  4 = 1 with the tile index scattered by a
// multiplicative permutation (t * P mod tiles): the tiles in flight at any
// moment are spread over the whole image instead of a band of ~30 tile rows.
#ifndef RT_TILE_SCHED
#define RT_TILE_SCHED 1
#endif

// Cycle-split diagnostic (RT_DIAG_TIMING builds only): per-wave s_memtime
// deltas accumulated over the whole persistent loop and flushed once per wave
// into aux.diag[0..7]: node-load wait, node work, leaves, stack pops, ray
// set-up, exact resolve, output stores, tile fetch.
#if defined(RT_DIAG_TILECOST) && RT_DIAG_TILECOST >= 2 && !defined(RT_DIAG_TIMING)
#define RT_DIAG_TIMING 1  // per-tile cycle split (tools/tile_costs.py)
#endif
#ifdef RT_DIAG_TIMING
#define RT_TSTAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define RT_TACC(slot, t0) (tacc[slot] += __builtin_amdgcn_s_memtime() - (t0))
#else
#define RT_TSTAMP(v)
#define RT_TACC(slot, t0)
#endif

#ifdef RT_DIAG_TILECOST
#define RT_DIAG_WAVE_STATS 1
#else
#define RT_DIAG_WAVE_STATS 0
#endif

// Diagnostic accumulators (aux.diag): [0..7] cycle split, then RT_DIAG_SLOTS
// spread slots of 8 words from RT_DIAG_SPREAD.
#define RT_DIAG_SPREAD 16
#define RT_DIAG_SLOTS 64

// Work stealing between the per-XCD tile queues (RT_TILE_SCHED 1); measured
// slower (9528 vs 9850 Mrays/s) with no change in wave busy fraction, so off.
#ifndef RT_STEAL
#define RT_STEAL 0
#endif

// Packed (lo, hi) slab fma (measured: no gain over scalar fma); next-tile
// prefetch (measured: slower, a reserved tile lengthens the tail).
#ifndef RT_PK_SLAB
#define RT_PK_SLAB 0
#endif
#ifndef RT_TILE_PREFETCH
#define RT_TILE_PREFETCH 0
#endif

// L2 prefetch of pushed children (their records are fetched when popped,
// many steps later): 0 off, 1 first 128-B line, 2 both lines.  One vector
// load per pushed child whose value is consumed at the next push, so its
// wait lands a whole step later.  (A no-return atomic add of 0 as the
// prefetch measured 3.6x slower.)
#ifndef RT_PREFETCH
#define RT_PREFETCH 0
#endif

// Tail shortening: a wave that has spent RT_PRIO_STEPS loop steps on its tile
// raises its issue priority (s_setprio 1, 2 at twice, 3 at three times
// that), so the long tiles that set the kernel's end get the SIMD first and
// the cheap tiles fill in around them.  0 = off.
#ifndef RT_PRIO_STEPS
#define RT_PRIO_STEPS 0
#endif

// Child refs of the scalar node path: 1 one vector load (lane c: child c),
// 0 eight v_writelane from the scalar records (measured faster: 131 vs 134
// us per 1080p frame; the any-mask s_addc chain gains 1.5%).
#ifndef RT_REF_VLOAD
#define RT_REF_VLOAD 0
#endif

// Pop-time culling: every pushed child's box goes on the wave stack beside
// its ref (lane c loads child c's record with one vector load alongside the
// scalar loads); a popped entry is re-tested against every lane's current
// culling distance and skipped, without loading its children, when no lane
// can still enter it (20% of node steps pop a node no lane enters).
// Measured: node visits 14.27 -> 12.97 per tile but no faster (the per-step
// record loads and the pop test cost what the skipped steps save; with K = 8
// LDS candidates the box stack costs a block per CU: -12%), so off.
#ifndef RT_POP_CULL
#define RT_POP_CULL 0
#endif

// Octant dispatch of the child test: 1 bit-test tree, 0 switch (measured
// equal: 12.16-12.31 vs 12.15-12.21 Grays/s over three runs each).
#ifndef RT_OCT_TREE
#define RT_OCT_TREE 0
#endif

// Octant dispatch hoisted out of the walk: the whole node loop is
// specialised per tile octant (9 copies), instead of a per-step dispatch.
#ifndef RT_OCT_HOIST
#define RT_OCT_HOIST 1
#endif

// Stack pushes without exec-mask branches (spare slot per lane; measured
// equal: 1.413-1.419 vs 1.417-1.421 ms per launch, 2: 1.423-1.441): 0 off,
// 1 on, 2 also without the branch on "anything to push".
#ifndef RT_PUSH_FLAT
#define RT_PUSH_FLAT 0
#endif
#if RT_PUSH_FLAT && (RT_POP_CULL || RT_PREFETCH)
#error "RT_PUSH_FLAT pushes refs only"
#endif

// W = 8 walk on the fp16-step node copy (sc.hnodes, 144 B per node instead
// of 256 B: 3 scalar loads and 36 SGPRs per node step instead of 8 and 64;
// each plane's t is one v_fma_mix_f32 of its fp16 step count).  Measured
// slower (1.535 vs 1.398 ms per launch, parity green): 9 more VALU per node
// step and looser boxes cost more than the scalar loads save — off.
#ifndef RT_HNODES
#define RT_HNODES 0
#endif

// Scalar-cache prefetch of the stack top's node at each leaf (the pop that
// follows a leaf then hits the scalar cache): 1 on, 0 off.  Measured slower
// (1.437-1.445 vs 1.416-1.418 ms per launch): the stack-top LDS read it
// needs sits in front of the leaf's own loads.
#ifndef RT_POP_PREFETCH
#define RT_POP_PREFETCH 0
#endif

// Leaf triangle filter without early exits (tri_classify_nb): 1 on, 0 off.
// Measured slower: 76 VGPRs (6 waves/SIMD) 1.483 ms, held to 72 (7 waves,
// spills) 1.444 ms, against 1.411-1.421 ms with the exits — the exits skip
// the rest of the test for triangles no lane of the tile can hit.
#ifndef RT_TRI_NB
#define RT_TRI_NB 0
#endif

// Node record fetch: 0 scalar loads (default), 1 uniform vector loads.
#ifndef RT_NODE_FETCH
#define RT_NODE_FETCH 0
#endif

// Child test of the walk: 0 every lane slab-tests its own ray against each
// of the W children (records through scalar loads), 1 group interval test:
// lane l tests child l % W against the interval of the rays of lane group
// l / W (W lanes), all W x 64/W pairs in one pass (records through one
// vector load per lane; see group_hits).
#ifndef RT_GROUP_TEST
#define RT_GROUP_TEST 0
#endif

// Occupancy target of the packet kernel (waves per SIMD); 0 = compiler's choice.
#ifndef RT_PACKET_WPE
#define RT_PACKET_WPE 0
#endif
#if RT_PACKET_WPE > 0
#define RT_PACKET_ATTR __attribute__((amdgpu_waves_per_eu(RT_PACKET_WPE)))
#elif defined(RT_PACKET_SGPRS)
#define RT_PACKET_ATTR __attribute__((amdgpu_num_sgpr(RT_PACKET_SGPRS)))
#else
#define RT_PACKET_ATTR
#endif

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
// BIT if any lane is set in the wave mask, else 0 — two SALU instructions
// (the compiler otherwise routes the uniform bool through a VGPR).
template <uint32_t BIT>
__device__ __forceinline__ uint32_t any_bit(uint64_t m) {
    uint32_t r;
    asm("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, %2, 0" : "=s"(r) : "s"(m), "i"(BIT) : "scc");
    return r;
}

// Bit c set iff any lane of hm[c] is set.
#ifndef RT_ANY_ADDC
#define RT_ANY_ADDC 1
#endif
template <int W>
__device__ __forceinline__ uint32_t any_mask(const uint64_t (&hm)[W]) {
    uint32_t m = 0;
#if RT_ANY_ADDC == 2
    if constexpr (W == 8) {
        // one asm block: no hazard padding between the children's pairs
        asm("s_cmp_lg_u64 %1, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %2, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %3, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %4, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %5, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %6, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %7, 0\n\ts_addc_u32 %0, %0, %0\n\t"
            "s_cmp_lg_u64 %8, 0\n\ts_addc_u32 %0, %0, %0"
            : "+s"(m)
            : "s"(hm[7]), "s"(hm[6]), "s"(hm[5]), "s"(hm[4]), "s"(hm[3]), "s"(hm[2]), "s"(hm[1]), "s"(hm[0])
            : "scc");
        return m;
    }
#endif
#if RT_ANY_ADDC
    // two SALU per child: SCC = (mask != 0), then m = 2m + SCC (children
    // from the last down, so child c lands in bit c)
#pragma unroll
    for (int c = W - 1; c >= 0; c--)
        asm("s_cmp_lg_u64 %1, 0\n\ts_addc_u32 %0, %0, %0" : "+s"(m) : "s"(hm[c]) : "scc");
#else
    [&]<int... C>(std::integer_sequence<int, C...>) { ((m |= any_bit<1u << C>(hm[C])), ...); }(
        std::make_integer_sequence<int, W>{});
#endif
    return m;
}

// A zero the compiler must treat as per-lane (forces vector-memory loads).
__device__ __forceinline__ int vzero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

template <int W>
__device__ __forceinline__ uint32_t lanes_of(const ChildRec (&ch)[W]) {
    uint32_t v = 0;
    [&]<int... L>(std::integer_sequence<int, L...>) { ((v = writelane<L>(v, ch[L].ref)), ...); }(
        std::make_integer_sequence<int, W>{});
    return v;
}

constexpr uint32_t kRedoPass1 = 0x80000000u;
#ifndef RT_LEAF_CHUNK
#define RT_LEAF_CHUNK 2
#endif
// triangle records fetched per scalar round trip (walk-tree leaves hold ~2:
// 2 measured 2% faster than 4)
constexpr int kLeafChunk = RT_LEAF_CHUNK;
constexpr uint32_t kCandDropped = 0x80;  // cand_cnt flag: candidates were dropped (bound in cand_drop)
constexpr uint32_t kCandSpilled = 0x40;  // cand_cnt flag: entries in the HBM overflow slots
constexpr uint32_t kCandCount = 0x3F;    // cand_cnt: entries in slots [0, count)
// A lane whose LDS list (K entries) is full appends further candidates
// straight to its pixel's HBM overflow slots [K, K + kCandSpill) (terminated
// by a tri = ~0 entry when not full); only past those is a candidate dropped
// (certified by the dropped bound, else the pixel is redone exactly).
constexpr int kCandSpill = RT_CAND_SLOTS - RT_CAND_LDS;
static_assert(kLeafChunk <= RT_TRI32_PAD, "tri32 padding must cover a leaf chunk");

// Forces uniform values to be materialised (their loads waited on) here, so
// a chunk's loads are all in flight before the first use.
__device__ __forceinline__ void pin_s(const float4& a, const float4& b, const float4& c) {
    asm volatile("" ::"s"(a.x), "s"(a.y), "s"(a.z), "s"(a.w), "s"(b.x), "s"(b.y), "s"(b.z), "s"(b.w), "s"(c.x),
                 "s"(c.y), "s"(c.z), "s"(c.w));
}  // redo entry: start directly with the inline-verifying pass

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
struct PacketArgs {
    RtDevScene sc;
    RtFrameParams fp;
    RtLaunchAux aux;
};
static_assert(sizeof(PacketArgs) % 4 == 0, "argument block is copied as words");
typedef const __attribute__((address_space(3))) PacketArgs* args_p;

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

typedef const __attribute__((address_space(4))) uint32_t* cuint_p;

// v_fma_mix_f32: fp16 half `hi` of uniform word w (an integer step count,
// exact) times b plus c, fused in fp32 with one rounding.
__device__ __forceinline__ float fma_h(uint32_t w, float b, float c, bool hi) {
    float d;
    if (hi)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "s"(w), "v"(b), "v"(c));
    else
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "s"(w), "v"(b), "v"(c));
    return d;
}

// child_hits on an fp16-step node (walk_tree.cpp quantize_wide8_f16): plane
// q of axis a lies at origin + q 2^e exactly, so its t is
// q (2^e i) + (origin i - o_lo/hi i) — the same slab value as the fp32
// record's fma, from a box that contains the record's box.
template <int OCT>
__device__ __forceinline__ void child_hits_h(const uint32_t (&hw)[36], const Ray32& q, const f2 nox, const f2 noy,
                                             const f2 noz, float tcull, uint64_t (&hm)[8]) {
    const float sx = __uint_as_float((hw[3] & 0xFFu) << 23) * q.ix;
    const float sy = __uint_as_float(((hw[3] >> 8) & 0xFFu) << 23) * q.iy;
    const float sz = __uint_as_float(((hw[3] >> 16) & 0xFFu) << 23) * q.iz;
    const float ox = __uint_as_float(hw[0]), oy = __uint_as_float(hw[1]), oz = __uint_as_float(hw[2]);
    const float alx = __builtin_fmaf(ox, q.ix, nox.x), ahx = __builtin_fmaf(ox, q.ix, nox.y);
    const float aly = __builtin_fmaf(oy, q.iy, noy.x), ahy = __builtin_fmaf(oy, q.iy, noy.y);
    const float alz = __builtin_fmaf(oz, q.iz, noz.x), ahz = __builtin_fmaf(oz, q.iz, noz.y);
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const bool h = c & 1;
        const int k = c >> 1;
        const float tlx = fma_h(hw[4 + k], sx, alx, h), thx = fma_h(hw[8 + k], sx, ahx, h);
        const float tly = fma_h(hw[12 + k], sy, aly, h), thy = fma_h(hw[16 + k], sy, ahy, h);
        const float tlz = fma_h(hw[20 + k], sz, alz, h), thz = fma_h(hw[24 + k], sz, ahz, h);
        float t0, t1;
        if constexpr (OCT < 0) {
            t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
            t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull));
        } else {
            const float nx = (OCT & 1) ? thx : tlx, fx = (OCT & 1) ? tlx : thx;
            const float ny = (OCT & 2) ? thy : tly, fy = (OCT & 2) ? tly : thy;
            const float nz = (OCT & 4) ? thz : tlz, fz = (OCT & 4) ? tlz : thz;
            // min/max in asm: the compiler would canonicalise each asm result first
            float m0, m1;
            asm("v_max_f32 %0, 0, %1" : "=v"(m0) : "v"(nz));
            asm("v_max3_f32 %0, %1, %2, %3" : "=v"(t0) : "v"(nx), "v"(ny), "v"(m0));
            asm("v_min_f32 %0, %1, %2" : "=v"(m1) : "v"(fz), "v"(tcull));
            asm("v_min3_f32 %0, %1, %2, %3" : "=v"(t1) : "v"(fx), "v"(fy), "v"(m1));
        }
        hm[c] = __ballot(t0 <= t1);
    }
}

// Slab test of one node's W children for every lane's ray (fp32, outward
// planes).  OCT >= 0: all rays share the direction signs OCT (bit a set =
// negative along axis a), so each axis's near plane is the hi plane for a
// negative direction and the lo plane otherwise — exactly what the per-axis
// min/max of the general test (OCT = -1) selects, since t(lo) <= t(hi) for a
// positive reciprocal and t(hi) <= t(lo) for a negative one.
template <int W, int OCT>
__device__ __forceinline__ void child_hits(const float (&bx)[W][6], const Ray32& q, const f2 nox, const f2 noy,
                                           const f2 noz, float tcull, uint64_t (&hm)[W]) {
    // fresh copies per specialisation: stops the compiler from hoisting the
    // (identical) plane fmas of every switch case above the switch
    float ix = q.ix, iy = q.iy, iz = q.iz;
#if !RT_OCT_HOIST
    asm volatile("" : "+v"(ix), "+v"(iy), "+v"(iz));
#endif
#pragma unroll
    for (int c = 0; c < W; c++) {
#if RT_PK_SLAB
        // (lo, hi) plane pairs in one v_pk_fma_f32 each
        const f2 tx = __builtin_elementwise_fma(f2{bx[c][0], bx[c][1]}, f2{ix, ix}, nox);
        const f2 ty = __builtin_elementwise_fma(f2{bx[c][2], bx[c][3]}, f2{iy, iy}, noy);
        const f2 tz = __builtin_elementwise_fma(f2{bx[c][4], bx[c][5]}, f2{iz, iz}, noz);
        const float tlx = tx.x, thx = tx.y, tly = ty.x, thy = ty.y, tlz = tz.x, thz = tz.y;
#else
        const float tlx = __builtin_fmaf(bx[c][0], ix, nox.x), thx = __builtin_fmaf(bx[c][1], ix, nox.y);
        const float tly = __builtin_fmaf(bx[c][2], iy, noy.x), thy = __builtin_fmaf(bx[c][3], iy, noy.y);
        const float tlz = __builtin_fmaf(bx[c][4], iz, noz.x), thz = __builtin_fmaf(bx[c][5], iz, noz.y);
#endif
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

// Lane-group reductions over groups of G consecutive lanes (G <= 32, a
// power of 2): ds_swizzle in xor mode (and_mask 0x1F, xor_mask s).
template <int S>
__device__ __forceinline__ float swz_xor(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (S << 10) | 0x1F));
}
template <int G>
__device__ __forceinline__ float group_min(float v) {
    if constexpr (G > 1) v = fminf(v, swz_xor<1>(v));
    if constexpr (G > 2) v = fminf(v, swz_xor<2>(v));
    if constexpr (G > 4) v = fminf(v, swz_xor<4>(v));
    if constexpr (G > 8) v = fminf(v, swz_xor<8>(v));
    static_assert(G <= 16, "groups of up to 16 lanes");
    return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
    if constexpr (G > 1) v = fmaxf(v, swz_xor<1>(v));
    if constexpr (G > 2) v = fmaxf(v, swz_xor<2>(v));
    if constexpr (G > 4) v = fmaxf(v, swz_xor<4>(v));
    if constexpr (G > 8) v = fmaxf(v, swz_xor<8>(v));
    return v;
}

// Ray interval of a lane group (RT_GROUP_TEST): the group's rays share the
// origin o (primary rays: the camera position, kernels_common.h gen_ray) and
// their fp32 reciprocals lie in [i0, i1] per axis.  al / ah = o + 2 pad and
// o - 2 pad: the lo / hi plane offsets, padded twice as far as the per-lane
// test's (o + pad, o - pad).
struct GroupIv {
    float ix0, ix1, iy0, iy1, iz0, iz1;  // per lane (its group's interval)
    float alx, ahx, aly, ahy, alz, ahz;  // uniform
};

// Group interval test of child (lane % W) for ray group (lane / W).  For one
// axis and a plane at offset d = p - a from the origin, t = d * i is linear
// in the reciprocal i, so over i in [i0, i1] it lies between d * i0 and
// d * i1 whatever the signs (a group whose rays straddle the axis plane has
// i0 < 0 < i1 and simply gets a wide interval).  A ray's near value
// min(t_lo, t_hi) is therefore >= the least of the four products and its far
// value <= the greatest, so the test below passes whenever any ray of the
// group passes the per-lane test: a superset, never a miss.  Rounding: the
// fp32 errors here are below 2^-23 (|p| + |o|) |i| <= pad |i| / 16 (pad =
// 2^-19 (|o|max + |coord|max), rt_api.cpp frame_pad), and the extra pad of
// the offsets moves every bound by pad |i|, so the computed test contains the
// per-lane computed test (which contains the fp64 reference test).
__device__ __forceinline__ bool group_hits(const float4 ra, const float2 rb, const GroupIv& g, float tg) {
    const float dlx = ra.x - g.alx, dhx = ra.y - g.ahx;
    const float dly = ra.z - g.aly, dhy = ra.w - g.ahy;
    const float dlz = rb.x - g.alz, dhz = rb.y - g.ahz;
    const float ax = dlx * g.ix0, bx = dlx * g.ix1, cx = dhx * g.ix0, ex = dhx * g.ix1;
    const float ay = dly * g.iy0, by = dly * g.iy1, cy = dhy * g.iy0, ey = dhy * g.iy1;
    const float az = dlz * g.iz0, bz = dlz * g.iz1, cz = dhz * g.iz0, ez = dhz * g.iz1;
    const float nx = fminf(fminf(ax, bx), fminf(cx, ex)), fx = fmaxf(fmaxf(ax, bx), fmaxf(cx, ex));
    const float ny = fminf(fminf(ay, by), fminf(cy, ey)), fy = fmaxf(fmaxf(ay, by), fmaxf(cy, ey));
    const float nz = fminf(fminf(az, bz), fminf(cz, ez)), fz = fmaxf(fmaxf(az, bz), fmaxf(cz, ez));
    const float t0 = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.f));
    const float t1 = fminf(fminf(fx, fy), fminf(fz, tg));
    return t0 <= t1;
}

// Bit c set iff some group's bit c of the ballot is set (groups of W lanes).
template <int W>
__device__ __forceinline__ uint32_t fold_groups(uint64_t m) {
#pragma unroll
    for (int s = 32; s >= W; s >>= 1) m |= m >> s;
    return (uint32_t)m & ((1u << W) - 1u);
}

template <int W, int SP, int K, bool COUNT>
__device__ __forceinline__ void trace_packet(args_p A, int f, int i, int r, bool valid, uint32_t* __restrict__ wstack,
                                             uint2* __restrict__ cand, uint64_t* tacc, float4* __restrict__ wbox4,
                                             float2* __restrict__ wbox2) {
    const int lane = threadIdx.x & 63;
    RT_TSTAMP(t_setup);
    if (!valid) { i = 0; r = 0; }
    Ray32 q;
    float tsl;  // distance slack (see trace_exact), fp32 rounded up
    float pd;
    uint32_t ob;
    {
        const RtFrameParams fp = kload(&A->fp);
        const RtFrameCam cam = kload(&A->fp.cam[f]);  // this tile's frame
        const Ray64 ray = gen_ray(fp, cam, i, fp.row0 + r * fp.row_stride);
        q = make_ray32(ray, cam.pad);
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
    constexpr bool kHN = W == 8 && RT_HNODES && RT_OCT_HOIST && !RT_POP_CULL && RT_NODE_FETCH == 0 && !RT_GROUP_TEST;
    const RT_G uint8_t* const hnodes = kHN ? kload(&A->sc.hnodes) : nullptr;
    const RT_G float* const tri32 = kload(&A->sc.tri32);
    // slab offsets for the lo / hi planes (pad moves lo down and hi up)
    const float olx = (q.ox + pd) * q.ix, ohx = (q.ox - pd) * q.ix;
    const float oly = (q.oy + pd) * q.iy, ohy = (q.oy - pd) * q.iy;
    const float olz = (q.oz + pd) * q.iz, ohz = (q.oz - pd) * q.iz;
    const f2 nox{-olx, -ohx}, noy{-oly, -ohy}, noz{-olz, -ohz};
#if RT_GROUP_TEST
    (void)oct;
    (void)nox;
    (void)noy;
    (void)noz;
    // the lane group's ray interval (lanes outside the image do not widen it;
    // a group with none has an empty interval and tg = -1: it passes no test)
    GroupIv g;
    g.ix0 = group_min<W>(valid ? q.ix : 3e38f);
    g.ix1 = group_max<W>(valid ? q.ix : -3e38f);
    g.iy0 = group_min<W>(valid ? q.iy : 3e38f);
    g.iy1 = group_max<W>(valid ? q.iy : -3e38f);
    g.iz0 = group_min<W>(valid ? q.iz : 3e38f);
    g.iz1 = group_max<W>(valid ? q.iz : -3e38f);
    g.alx = __builtin_bit_cast(float, uni(__float_as_uint(q.ox + 2.f * pd)));
    g.ahx = __builtin_bit_cast(float, uni(__float_as_uint(q.ox - 2.f * pd)));
    g.aly = __builtin_bit_cast(float, uni(__float_as_uint(q.oy + 2.f * pd)));
    g.ahy = __builtin_bit_cast(float, uni(__float_as_uint(q.oy - 2.f * pd)));
    g.alz = __builtin_bit_cast(float, uni(__float_as_uint(q.oz + 2.f * pd)));
    g.ahz = __builtin_bit_cast(float, uni(__float_as_uint(q.oz - 2.f * pd)));
#endif

    uint32_t n_nodes = 0, n_pre = 0, w_nodes = 0, w_leaves = 0, w_tris = 0;  // COUNT only
    uint32_t w_empty = 0;                // COUNT only: node steps where no lane enters any child
    uint32_t w_empty_pop = 0;            // COUNT only: of which the node came off the stack
    uint32_t w_popcull = 0;              // COUNT only: popped entries culled without a node step
    bool popped = false;                 // COUNT only: the current node came off the stack
#if RT_PREFETCH
    uint32_t pf_sink = 0, pf_val = 0, pf_val2 = 0;  // L2 prefetch loads (values unused)
#endif
    float tcull = valid ? __builtin_huge_valf() : -1.f;
#if RT_GROUP_TEST
    float tg = group_max<W>(tcull);  // the group's largest culling distance
#endif
    int nc = 0;         // candidates in the lane's list
    int nsp = 0;        // candidates in the pixel's HBM overflow slots
    float drop = __builtin_huge_valf();  // smallest t lower bound of a dropped candidate
    uint32_t cur = kword(&A->sc.root_ref);
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
    RT_TACC(4, t_setup);
#if RT_PRIO_STEPS
    uint32_t steps = 0;
#endif
#if RT_OCT_HOIST
    // the walk specialised on the tile's octant (one dispatch per tile, not per node step)
    auto walk = [&]<int OCT>() __attribute__((always_inline)) {
#endif
    // (without pop-time culling every popped ref is a real node or leaf, so
    // only the root can be invalid: tested once, not per step)
#if RT_OCT_HOIST
    constexpr bool kRootOnly = !RT_POP_CULL;
    if (kRootOnly && cur == RT_INVALID_REF) return;  // from the walk lambda
#else
    constexpr bool kRootOnly = false;
#endif
    for (;;) {
#if RT_PRIO_STEPS
        steps++;
        if (steps == RT_PRIO_STEPS) __builtin_amdgcn_s_setprio(1);
        if (steps == 2 * RT_PRIO_STEPS) __builtin_amdgcn_s_setprio(2);
        if (steps == 3 * RT_PRIO_STEPS) __builtin_amdgcn_s_setprio(3);
#endif
        if (kRootOnly || cur != RT_INVALID_REF) {
            if (!(cur & RT_LEAF_BIT)) {
                RT_TSTAMP(t_n0);
                if (COUNT || RT_DIAG_WAVE_STATS) {
                    w_nodes++;
                    n_nodes += valid;
                }
#if !RT_GROUP_TEST
                float bx[W][6];  // child boxes {lx, hx, ly, hy, lz, hz}
#endif
                uint32_t refv;   // lane c: child c's ref
#if RT_POP_CULL
                float4 cb4;      // lane c: child c's {lx, hx, ly, hy}
                float2 cb2;      //         and {lz, hz}
#endif
                uint32_t meta;   // slot 0's pad: sort axis | valid slots << 2 (bvh_build.cpp set_meta)
#if RT_GROUP_TEST
                uint32_t mask;
                {
                    // lane l loads child l % W's record (the W records of the
                    // node, 256 B for W = 8, one request per lane group)
                    const RT_G float4* cv =
                        reinterpret_cast<const RT_G float4*>(nodes + (size_t)cur * (32 * W)) + 2 * (lane & (W - 1));
                    const float4 ra = cv[0];
                    const float4 rb = cv[1];
                    refv = __float_as_uint(rb.z);
                    meta = (uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(rb.w), 0);
                    RT_TACC(0, t_n0);
                    mask = fold_groups<W>(__ballot(group_hits(ra, make_float2(rb.x, rb.y), g, tg))) &
                           ((1u << (meta >> 2)) - 1u);
                }
                RT_TSTAMP(t_n1);
#else
#if RT_NODE_FETCH == 0
                uint32_t hw[36];  // kHN: the fp16-step node, in SGPRs
                if constexpr (kHN) {
                    const cuint_p hb = (cuint_p)(hnodes + (size_t)cur * RT_HNODE_BYTES);
#pragma unroll
                    for (int k = 0; k < 36; k++) hw[k] = hb[k];
                    refv = 0;
                    [&]<int... L>(std::integer_sequence<int, L...>) {
                        ((refv = writelane<L>(refv, hw[28 + L])), ...);
                    }(std::make_integer_sequence<int, 8>{});
                    meta = hw[3] >> 24;
                } else
                {
                    // scalar path: all W records are loaded before any branch
                    // so their loads are in flight together
                    const cchild_p nb = (cchild_p)(nodes + (size_t)cur * (32 * W));
                    ChildRec ch[W];
#pragma unroll
                    for (int c = 0; c < W; c++) ch[c] = load_child(nb + c);
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        bx[c][0] = ch[c].lx; bx[c][1] = ch[c].hx; bx[c][2] = ch[c].ly;
                        bx[c][3] = ch[c].hy; bx[c][4] = ch[c].lz; bx[c][5] = ch[c].hz;
                    }
#if RT_POP_CULL
                    // lane c (< W) loads child c's whole record (box for the
                    // stack, ref) with vector loads alongside the scalar loads
                    {
                        const RT_G float4* cv =
                            reinterpret_cast<const RT_G float4*>(nodes + (size_t)cur * (32 * W)) + 2 * (lane & (W - 1));
                        cb4 = cv[0];
                        const float4 c1 = cv[1];
                        cb2 = make_float2(c1.x, c1.y);
                        refv = __float_as_uint(c1.z);
                    }
#elif RT_REF_VLOAD
                    // lane c (< W) loads child c's ref with one vector load
                    // issued alongside the scalar box loads (no writelanes)
                    refv = reinterpret_cast<const RT_G uint32_t*>(nodes + (size_t)cur * (32 * W))
                        [8 * (lane & (W - 1)) + RT_CHILD_REF];
#else
                    // built before any branch so the ref words load with the
                    // boxes, not in a second round trip
                    refv = lanes_of<W>(ch);
#endif
                    meta = ch[0].pad;
                }
#else
                {
                    // vector path: every lane loads the same record words
                    // (one request per wave-instruction through the vector
                    // L1), lane c loads child c's ref
                    const RT_G uint32_t* nw = (const RT_G uint32_t*)(nodes + (size_t)cur * (32 * W)) + vzero();
#pragma unroll
                    for (int c = 0; c < W; c++) {
                        const float4 a = *(const RT_G float4*)(nw + 8 * c);
                        const float2 b = *(const RT_G float2*)(nw + 8 * c + 4);
                        bx[c][0] = a.x; bx[c][1] = a.y; bx[c][2] = a.z; bx[c][3] = a.w;
                        bx[c][4] = b.x; bx[c][5] = b.y;
                    }
                    refv = nw[8 * (lane & (W - 1)) + RT_CHILD_REF];
                    meta = uni(nw[7]);
                }
#endif
#ifdef RT_DIAG_TIMING
                asm volatile("" : "+v"(refv));
#endif
                RT_TACC(0, t_n0);
                RT_TSTAMP(t_n1);
                uint64_t hm[W];  // per child: lanes whose ray enters it
                // all lanes' rays share the tile's direction signs (nearly every
                // tile): the near/far plane of each axis is known, no per-axis
                // min/max; otherwise the general test
#if RT_OCT_HOIST
                if constexpr (kHN) child_hits_h<OCT>(hw, q, nox, noy, noz, tcull, *reinterpret_cast<uint64_t(*)[8]>(hm));
                else child_hits<W, OCT>(bx, q, nox, noy, noz, tcull, hm);
#elif RT_OCT_TREE
                // binary dispatch on the octant bits (3 uniform branches)
                if (oct > 7) {
                    child_hits<W, -1>(bx, q, nox, noy, noz, tcull, hm);
                } else if (oct & 4) {
                    if (oct & 2) {
                        if (oct & 1) child_hits<W, 7>(bx, q, nox, noy, noz, tcull, hm);
                        else child_hits<W, 6>(bx, q, nox, noy, noz, tcull, hm);
                    } else {
                        if (oct & 1) child_hits<W, 5>(bx, q, nox, noy, noz, tcull, hm);
                        else child_hits<W, 4>(bx, q, nox, noy, noz, tcull, hm);
                    }
                } else {
                    if (oct & 2) {
                        if (oct & 1) child_hits<W, 3>(bx, q, nox, noy, noz, tcull, hm);
                        else child_hits<W, 2>(bx, q, nox, noy, noz, tcull, hm);
                    } else {
                        if (oct & 1) child_hits<W, 1>(bx, q, nox, noy, noz, tcull, hm);
                        else child_hits<W, 0>(bx, q, nox, noy, noz, tcull, hm);
                    }
                }
#else
                switch (oct) {
                    case 0: child_hits<W, 0>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 1: child_hits<W, 1>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 2: child_hits<W, 2>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 3: child_hits<W, 3>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 4: child_hits<W, 4>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 5: child_hits<W, 5>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 6: child_hits<W, 6>(bx, q, nox, noy, noz, tcull, hm); break;
                    case 7: child_hits<W, 7>(bx, q, nox, noy, noz, tcull, hm); break;
                    default: child_hits<W, -1>(bx, q, nox, noy, noz, tcull, hm); break;
                }
#endif
                uint32_t mask = any_mask<W>(hm) & ((1u << (meta >> 2)) - 1u);
#endif  // RT_GROUP_TEST
                if (COUNT) {
                    w_empty += mask == 0;
                    w_empty_pop += mask == 0 && popped;
                }
                if (mask != 0) {
                    // children are sorted along `axis`: walk them front to back
                    // for the tile's direction (lowest index first when the
                    // tile looks along +axis)
                    const bool rev = (dsg >> (meta & 3u)) & 1u;
                    const int near_c = rev ? 31 - __builtin_clz(mask) : __builtin_ctz(mask);
                    const uint32_t pm = mask & ~(1u << near_c);
#if RT_PUSH_FLAT
                    // the rest go on the stack so that they pop in order; a
                    // lane with nothing to push writes its own spare slot
                    // (no exec-mask branch; flat 2: no branch on pm either)
                    if (RT_PUSH_FLAT == 2 || pm != 0) {
                        const uint32_t below = pm & ((1u << (lane & 31)) - 1u);
                        const uint32_t above = (pm >> (lane & 31)) >> 1;
                        const int slot = (int)__builtin_popcount(rev ? below : above);
                        const bool push = ((pm >> (lane & 31)) & 1u) && lane < W;
                        wstack[push ? sp + slot : SP + lane] = refv;
                        sp += __builtin_popcount(pm);
                    }
#else
                    if (pm != 0) {
                        // the rest go on the stack so that they pop in order
                        const uint32_t below = pm & ((1u << (lane & 31)) - 1u);
                        const uint32_t above = (pm >> (lane & 31)) >> 1;
                        const int slot = (int)__builtin_popcount(rev ? below : above);
                        if ((pm >> (lane & 31)) & 1u & (lane < W)) {
                            wstack[sp + slot] = refv;
#if RT_POP_CULL
                            wbox4[sp + slot] = cb4;
                            wbox2[sp + slot] = cb2;
#endif
#if RT_PREFETCH
                            const RT_G uint8_t* pa =
                                (refv & RT_LEAF_BIT)
                                    ? (const RT_G uint8_t*)(tri32 + 12 * (size_t)(refv & RT_LEAF_FIRST_MASK))
                                    : nodes + (size_t)refv * (32 * W);
                            // consume the previous push's prefetch (long returned), issue this one
                            pf_sink ^= pf_val ^ pf_val2;
                            pf_val = *(const RT_G uint32_t*)pa;
                            if (RT_PREFETCH >= 2) pf_val2 = *(const RT_G uint32_t*)(pa + 128);
#endif
                        }
                        sp += __builtin_popcount(pm);
                    }
#endif
                    cur = (uint32_t)__builtin_amdgcn_readlane((int)refv, near_c);
                    if (COUNT) popped = false;
                    RT_TACC(1, t_n1);
                    continue;
                }
                RT_TACC(1, t_n1);
            } else {
                RT_TSTAMP(t_l0);
                const uint32_t first = cur & RT_LEAF_FIRST_MASK;
                const uint32_t cnt = ((cur >> 27) & 15u) + 1u;
                if (COUNT || RT_DIAG_WAVE_STATS) {
                    w_leaves++;
                    w_tris += cnt;
                }
#if RT_POP_PREFETCH
                // a leaf is followed by a pop: touch the stack top's node (one
                // word per 64-B line) so its records are in the scalar cache
                // when the pop loads them; the words are consumed after the
                // leaf, whose own waits cover them
                // (straight-line: an invalid target reads the root node instead)
                const uint32_t nxt = uni(wstack[sp > 0 ? sp - 1 : 0]);
                const uint32_t pnode = (sp > 0 && !(nxt & RT_LEAF_BIT)) ? nxt : 0u;
                const cuint_p pfp = (cuint_p)(nodes + (size_t)pnode * (32 * W));
                const uint32_t pf0 = pfp[0], pf1 = pfp[16], pf2 = pfp[32], pf3 = pfp[48];
#endif
                // triangles come in chunks of kLeafChunk records: all their
                // scalar loads are issued, then waited on once (tri32 carries
                // kLeafChunk padding records, so reading past a leaf is safe)
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
                        if (COUNT) n_pre += valid;
                        float tl, tu;
#if RT_TRI_NB
                        int cls = tri_classify_nb(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz, q.co,
                                                  tcull, tl, tu);
                        cls = valid ? cls : 0;
#else
                        const int cls = valid ? tri_classify(TA[t], TB[t], TC[t], q.ox, q.oy, q.oz, q.dx, q.dy, q.dz,
                                                             q.co, tcull, tl, tu)
                                              : 0;
#endif
                        if (__ballot(cls != 0) == 0) continue;
                        if (cls != 0) {
                            // dist of a certain hit <= (tu + slack)(1 + 2^-20)
                            if (cls == 2) tcull = fminf(tcull, (tu + tsl) * (1.f + 0x1p-20f));
                            if (nc == K) nc = compact_candidates<K>(cand, lane, tcull);
                            if (nc < K) {
                                cand[nc * 64 + lane] = make_uint2(k, __float_as_uint(tl));
                                nc++;
                            } else if (nsp < kCandSpill) {
                                // LDS list full: append to the pixel's HBM overflow slots
                                const args_p A2 = launder(A);  // (A itself stays uniform)
                                const size_t np = (size_t)kword(&A2->fp.W) * kword(&A2->fp.nrows) *
                                                  kword(&A2->fp.nframes);
                                RT_G uint2* const hc = reinterpret_cast<RT_G uint2*>(kload(&A2->aux.cand));
                                hc[(size_t)(K + nsp) * np + ob] = make_uint2(k, __float_as_uint(tl));
                                nsp++;
                            } else {
                                // full: keep the K smallest lower bounds, remember the
                                // smallest bound dropped (k_resolve certifies the winner
                                // against it, else the pixel is redone exactly)
                                drop = fminf(drop, keep_nearest<K>(cand, lane, k, tl));
                            }
                        }
                    }
                }
#if RT_GROUP_TEST
                tg = group_max<W>(tcull);
#endif
#if RT_POP_PREFETCH
                asm volatile("" ::"s"(pf0), "s"(pf1), "s"(pf2), "s"(pf3));
#endif
                RT_TACC(2, t_l0);
            }
        }
        RT_TSTAMP(t_p0);
        if (sp == 0) {
#if RT_PRIO_STEPS
            if (steps >= RT_PRIO_STEPS) __builtin_amdgcn_s_setprio(0);
#endif
            break;
        }
        sp--;
        cur = uni(wstack[sp]);
        if (COUNT) popped = true;
#if RT_POP_CULL
        {
            // re-test the popped entry's box for every lane (general slab test)
            const float4 b4 = wbox4[sp];
            const float2 b2 = wbox2[sp];
            const float tlx = __builtin_fmaf(b4.x, q.ix, nox.x), thx = __builtin_fmaf(b4.y, q.ix, nox.y);
            const float tly = __builtin_fmaf(b4.z, q.iy, noy.x), thy = __builtin_fmaf(b4.w, q.iy, noy.y);
            const float tlz = __builtin_fmaf(b2.x, q.iz, noz.x), thz = __builtin_fmaf(b2.y, q.iz, noz.y);
            const float t0 = fmaxf(fmaxf(fminf(tlx, thx), fminf(tly, thy)), fmaxf(fminf(tlz, thz), 0.f));
            const float t1 = fminf(fminf(fmaxf(tlx, thx), fmaxf(tly, thy)), fminf(fmaxf(tlz, thz), tcull));
            if (__ballot(t0 <= t1) == 0) {
                cur = RT_INVALID_REF;  // no lane can enter it any more: pop the next one
                if (COUNT) w_popcull++;
            }
        }
#endif
#ifdef RT_DIAG_TIMING
        asm volatile("" ::"s"(cur));
#endif
        RT_TACC(3, t_p0);
    }
#if RT_OCT_HOIST
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
#endif
    RT_TSTAMP(t_r0);
#if RT_PREFETCH
    asm volatile("" ::"v"(pf_sink ^ pf_val ^ pf_val2));  // keeps the prefetch loads
#endif
    A = launder(A);
    const RtFrameParams fp = kload(&A->fp);
    if (COUNT && fp.counters && lane == 0) {
        atomicAdd(&fp.counters[7], (unsigned long long)w_nodes);
        atomicAdd(&fp.counters[8], (unsigned long long)w_leaves);
        atomicAdd(&fp.counters[9], 1ull);
        atomicAdd(&fp.counters[12], (unsigned long long)w_tris);
        atomicAdd(&fp.counters[15], (unsigned long long)w_empty);
        atomicAdd(&fp.counters[14], (unsigned long long)w_popcull);
        atomicAdd(&fp.counters[13], (unsigned long long)w_empty_pop);
    }
#ifdef RT_DIAG_TILECOST
    {   // wave-level visits of this tile into hit_pos[3 * tile + 1 / + 2]
        RT_G double* hp = fp.hit_pos;
        const int tile = (r >> 3) * ((fp.W + 7) >> 3) + (i >> 3);
        if (hp && (threadIdx.x & 63) == 0) {
            hp[3 * (size_t)tile + 1] = (double)w_nodes + 1e6 * (double)w_leaves;
            hp[3 * (size_t)tile + 2] = (double)w_tris;
        }
    }
#endif
    if (!valid) return;
    // hand the lane's surviving candidates to k_resolve: count per pixel,
    // entry c of batch pixel o at cand[c * npix + o] (coalesced across a row;
    // frame f's pixels follow frame f-1's)
    const RtLaunchAux aux = kload(&A->aux);
    const size_t o = ob;
    const size_t npix = (size_t)fp.W * fp.nrows * fp.nframes;
    uint32_t m = 0;
    for (int c = 0; c < nc; c++) {
        const uint2 e = cand[c * 64 + lane];
        if (__uint_as_float(e.y) > tcull) continue;  // cannot beat a certain hit
        reinterpret_cast<RT_G uint2*>(aux.cand)[(size_t)m * npix + o] = e;
        m++;
    }
    const bool dropped = drop < __builtin_huge_valf() && drop <= tcull;  // a dropped candidate could still win
    if (dropped) aux.cand_drop[o] = drop;
    if (nsp > 0 && nsp < kCandSpill)  // terminate the overflow slots
        reinterpret_cast<RT_G uint2*>(aux.cand)[(size_t)(K + nsp) * npix + o] = make_uint2(~0u, 0u);
    aux.cand_cnt[o] = (uint8_t)(m | (dropped ? kCandDropped : 0u) | (nsp > 0 ? kCandSpilled : 0u));
    RT_TACC(5, t_r0);
    if (COUNT && fp.counters) {
        atomicAdd(&fp.counters[1], (unsigned long long)n_nodes);
        atomicAdd(&fp.counters[6], (unsigned long long)n_pre);
    }
}

// Exact resolve of the packet kernel's candidate lists, one pixel per lane
// (full occupancy: the dependent fp64 loads of many pixels overlap).  For
// each candidate the reference's fp64 Moller-Trumbore and hit distance
// (triangle.hpp:40-88, stack_bvh.hpp:630-631); the winner is the minimum
// (distance, reference visit rank) — the reference keeps the first strictly
// closer hit in its LIFO order (stack_bvh.hpp:633).  The winner's ancestor
// chain is re-verified (the reference must see the triangle); a failure or
// a candidate-list overflow sends the pixel to k_fixup.
#ifndef RT_RESOLVE_PRELOAD
#define RT_RESOLVE_PRELOAD 1
#endif
#ifndef RT_RESOLVE_SPEC
#define RT_RESOLVE_SPEC 1
#endif
#ifndef RT_RESOLVE_WPE
#define RT_RESOLVE_WPE 0
#endif
#if RT_RESOLVE_WPE > 0
#define RT_RESOLVE_ATTR __attribute__((amdgpu_waves_per_eu(RT_RESOLVE_WPE)))
#else
#define RT_RESOLVE_ATTR
#endif
// Exact resolve of one sample (frame f of the launch, pixel (i, r), batch
// pixel index o of the candidate lists): the winner, its shading inputs, and
// whether the pixel must be redone (1: a dropped candidate could win, 2: the
// reference cannot see the winner).
template <bool COUNT>
__device__ __forceinline__ void resolve_sample(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux,
                                               int f, int i, int r, size_t o, size_t npix, bool active, Best& out,
                                               Shade& sh, uint32_t& redo, uint32_t& n_tris, uint32_t& n_chain,
                                               uint32_t& n_chain_nodes) {
    const RtFrameCam& cam = fp.cam[f];
    const RT_G uint2* const cl = reinterpret_cast<const RT_G uint2*>(aux.cand);
    uint32_t cnt = 0u;
#if RT_RESOLVE_SPEC
    // entry 0 is loaded alongside the count (one dependent round trip less)
    uint2 e0 = make_uint2(0u, 0u);
    if (active) {
        cnt = aux.cand_cnt[o];
        e0 = cl[o];
    }
#else
    if (active) cnt = aux.cand_cnt[o];
#endif
    out.dist = 1.7976931348623157e308;  // std::numeric_limits<double>::max()
    out.rank = 0xFFFFFFFFu;
    out.tri = -1;
    out.px = out.py = out.pz = 0.0;
    sh = Shade{0.0, 0.0, 0.0, RT_INVALID_REF};
    redo = 0;
    const uint32_t nlist = cnt & kCandCount;
#if RT_RESOLVE_PRELOAD
    // the whole 128-B record of entry 0 is requested as soon as its index
    // arrives, and the fp64 ray is built while it is in flight (one
    // dependent round trip instead of three: MT part, v0, shading fields)
    double R0[RT_TRI64_DOUBLES];
    // the record array's base in SGPRs before the count arrives (else its
    // kernel-argument load sits between the index and the record loads)
    const RT_G double* tri64 = sc.tri64;
    asm volatile("" : "+s"(tri64));
    if (cnt != 0) {
        const RT_G double2* T2 = reinterpret_cast<const RT_G double2*>(tri64 + RT_TRI64_DOUBLES * (size_t)e0.x);
#pragma unroll
        for (int k = 0; k < RT_TRI64_DOUBLES / 2; k++) {
            const double2 v = T2[k];
            R0[2 * k] = v.x;
            R0[2 * k + 1] = v.y;
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the ray's fp64 set-up
    }
#endif
    if (cnt != 0) {
        const Ray64 ray = gen_ray<false>(fp, cam, i, fp.row0 + r * fp.row_stride);
        double best_t = 0.0;
        uint32_t leaf = 0;
        float lb[6];
        // exact test of candidate e (record T: global or a register copy),
        // kept if it is the (distance, visit rank) minimum
        auto consider_rec = [&](const uint2 e, const auto* T) {
            if (COUNT) n_tris++;
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
                sh.nx = T[RT_T64_NORMAL];
                sh.ny = T[RT_T64_NORMAL + 1];
                sh.nz = T[RT_T64_NORMAL + 2];
                const uint64_t il = __builtin_bit_cast(uint64_t, (double)T[RT_T64_IDLEAF]);
                sh.id = (uint32_t)il;
                leaf = (uint32_t)(il >> 32);
#pragma unroll
                for (int a = 0; a < 3; a++) {
                    const uint64_t bb = __builtin_bit_cast(uint64_t, (double)T[RT_T64_BOX + a]);
                    lb[2 * a] = __uint_as_float((uint32_t)bb);
                    lb[2 * a + 1] = __uint_as_float((uint32_t)(bb >> 32));
                }
            }
        };
        // one 128-B record per candidate: triangle, normal, id, leaf and its box
        auto consider = [&](const uint2 e) { consider_rec(e, sc.tri64 + RT_TRI64_DOUBLES * (size_t)e.x); };
#if RT_RESOLVE_PRELOAD
        if (nlist > 0) consider_rec(e0, R0);
        for (uint32_t c = 1; c < nlist; c++) consider(cl[(size_t)c * npix + o]);
#elif RT_RESOLVE_SPEC
        if (nlist > 0) consider(e0);
        for (uint32_t c = 1; c < nlist; c++) consider(cl[(size_t)c * npix + o]);
#else
        for (uint32_t c = 0; c < nlist; c++) consider(cl[(size_t)c * npix + o]);
#endif
        if (cnt & kCandSpilled) {
            for (uint32_t c = RT_CAND_LDS; c < (uint32_t)RT_CAND_SLOTS; c++) {
                const uint2 e = cl[(size_t)c * npix + o];
                if (e.x == ~0u) break;
                consider(e);
            }
        }
        if (cnt & kCandDropped) {
            // every dropped candidate has t >= drop, so its distance is at
            // least drop (1 - 2^-20) - slack: the winner must be strictly
            // nearer than that, else only the exact per-lane path can decide
            const double omax = __builtin_fmax(__builtin_fmax(__builtin_fabs(ray.ox), __builtin_fabs(ray.oy)),
                                               __builtin_fabs(ray.oz));
            const double bound = (double)aux.cand_drop[o] * (1.0 - 0x1p-20) - 0x1p-40 * (omax + 1.0);
            if (!(out.tri >= 0 && out.dist < bound)) redo = 1;
        }
        if (!redo && out.tri >= 0) {
            (void)hit_dist(ray, best_t, out.px, out.py, out.pz);
            // the reference must see the winner: re-verify its ancestor chain
            if (COUNT) n_chain++;
            if (!chain_fast_ok32(lb, ray, out.px, out.py, out.pz) &&
                !chain_ok(sc, leaf, with_inv(ray), n_chain_nodes))
                redo = 2;
        }
    }
}

// One pixel per lane over all spp samples of its pose; one block per 16x16
// tile of one pose.  MULTI = false: spp == 1, the straight-line reference
// path (no sample loop, 76 instead of 105 VGPRs).
template <bool COUNT, bool MULTI>
__global__ void __launch_bounds__(256) RT_RESOLVE_ATTR k_resolve(RtDevScene sc, RtFrameParams fp, RtLaunchAux aux) {
    __shared__ uint32_t wave_hits[4];
    // the traversal kernel is done with the tile queues: clear them for the
    // next launch (the packet pipeline needs no memset)
    if (blockIdx.x == 0 && threadIdx.x < RT_QUEUES) aux.tile_ctr[threadIdx.x * RT_QUEUE_STRIDE] = 0;
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
    uint32_t redo_any = 0, hits = 0, n_tris = 0, n_chain = 0, n_chain_nodes = 0, n_redo[3] = {0, 0, 0};
    double acc[3] = {0.0, 0.0, 0.0};
    const int spp = MULTI ? fp.spp : 1;
    for (int k = 0; k < spp; k++) {
        const int f = p * spp + k;
        Best out;
        Shade sh;
        uint32_t redo;
        resolve_sample<COUNT>(sc, fp, aux, f, i, r, out_index(fp, f, po), npix, active, out, sh, redo, n_tris,
                              n_chain, n_chain_nodes);
        if (COUNT) n_redo[redo]++;
        redo_any = redo_any > redo ? redo_any : redo;
        if (active && !redo) {
            store_sample(fp, pix * (size_t)spp + k, out, sh);
            if (MULTI) {
                double c[3];
                shade_color(fp.cam[f], out, sh, c);
                acc[0] = acc[0] + c[0];
                acc[1] = acc[1] + c[1];
                acc[2] = acc[2] + c[2];
            } else {
                shade_color(fp.cam[f], out, sh, acc);  // the sample's colour is the pixel's
            }
            hits += out.tri >= 0;
        }
    }
    if (active) {
        if (redo_any) {
            // k_fixup redoes every sample of the pixel with the exact per-lane path
            const uint32_t slot = atomicAdd(aux.tile_ctr + RT_REDO_COUNT, 1u);
            aux.redo[slot] = (uint32_t)pix | (redo_any == 2u && !MULTI ? kRedoPass1 : 0u);
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
        atomicAdd(&fp.counters[2], (unsigned long long)n_tris);
        atomicAdd(&fp.counters[3], (unsigned long long)n_chain);
        if (hits) atomicAdd(&fp.counters[4], (unsigned long long)hits);
        atomicAdd(&fp.counters[5], (unsigned long long)n_chain_nodes);
        if (n_redo[1]) atomicAdd(&fp.counters[10], (unsigned long long)n_redo[1]);
        if (n_redo[2]) atomicAdd(&fp.counters[11], (unsigned long long)n_redo[2]);
    }
}

// Persistent waves over 8x8 tiles; the stack bound of the tree must fit SP
// (the host falls back to the per-lane kernel otherwise), so no push can drop.
template <int W, int SP, int K, bool COUNT>
__global__ void __launch_bounds__(256) RT_PACKET_ATTR k_trace_packet(PacketArgs args) {
    __shared__ uint32_t stacks[4][SP + (RT_PUSH_FLAT ? 64 : 0)];  // + a spare slot per lane
    __shared__ uint2 cands[4][K * 64];
#if RT_POP_CULL
    __shared__ float4 sbox4[4][SP];
    __shared__ float2 sbox2[4][SP];
#endif
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
    if (blockIdx.x == 0) {
        // self-reset for this launch's k_resolve / k_fixup (the previous
        // launch's fix-up has completed: stream order)
        RT_G uint32_t* const q = kload(&A->aux.tile_ctr);
        if (threadIdx.x == 0) q[RT_REDO_COUNT] = 0;
        const int nslots = kword(&A->fp.nframes) * RT_HIT_SLOTS;
        for (int k = threadIdx.x; k < nslots; k += blockDim.x) q[RT_HIT_BASE + k * RT_QUEUE_STRIDE] = 0;
    }
    uint64_t tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)tacc;
#if defined(RT_DIAG_TIMING) || defined(RT_DIAG_LIFE) || defined(RT_DIAG_WAVES)
    const uint64_t t_life = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
    uint32_t n_tiles = 0;
#endif
    // tile scheduling: one queue per XCD (blocks are dealt to the 8 XCDs
    // round-robin, so block b's XCD is b % 8): queue x hands out tiles
    // x, x + 8, x + 16, ...; every queue is drained by the blocks b = x mod 8.
    const uint32_t xq = blockIdx.x % RT_QUEUES;
    bool first = true;
    uint32_t hop = 0;  // queues (after the own one) this wave found drained
    (void)hop;
    // waves drained through queue xq: 4 per block b = xq (mod 8)
    const uint32_t nwx = 4u * ((gridDim.x + RT_QUEUES - 1 - xq) / RT_QUEUES);
    (void)first;
    (void)nwx;
#if RT_TILE_SCHED == 2
    uint32_t iter = 0;  // diagnostic: static round-robin, no atomics
#elif RT_TILE_SCHED == 3
    uint32_t drained = 0;  // bands this wave found empty (bit per queue)
#endif
    // The next tile index is fetched one tile ahead, so the queue atomic's
    // round trip overlaps the current tile's walk.
    auto fetch = [&]() -> int {
        int t = 0;
#if RT_TILE_SCHED == 0
        if (lane == 0) t = (int)atomicAdd(kload(&A->aux.tile_ctr), 1u);
#elif RT_TILE_SCHED == 1 || RT_TILE_SCHED == 4 || RT_TILE_SCHED == 5
        // a wave's first tile is its own slot in the queue (no atomic: the
        // whole grid starting at once would serialise on the 8 counters for
        // ~10 us); the counter hands out the slots after the XCD's waves
        if (first) {
            first = false;
            t = (int)(xq + RT_QUEUES * ((blockIdx.x / RT_QUEUES) * 4 + wv));
        } else if (lane == 0) {
            // own queue first; once it is drained, steal from the next
            // queues in turn (a drained queue stays drained), so no XCD
            // idles while another still has tiles
            const int W_ = kword(&A->fp.W), nrows = kword(&A->fp.nrows);
            const int all = ((W_ + 7) >> 3) * ((nrows + 7) >> 3) * kword(&A->fp.nframes);
            RT_G uint32_t* const ctr = kload(&A->aux.tile_ctr);
            for (;;) {
                const uint32_t qx = (xq + hop) & (RT_QUEUES - 1);
                const uint32_t nwq = 4u * ((gridDim.x + RT_QUEUES - 1 - qx) / RT_QUEUES);
                t = (int)(qx + RT_QUEUES * (nwq + atomicAdd(ctr + qx * RT_QUEUE_STRIDE, 1u)));
                if (!RT_STEAL || t < all || hop == RT_QUEUES - 1) break;
                hop++;
            }
        }
#elif RT_TILE_SCHED == 3
        {
            const int W_ = kword(&A->fp.W), nrows = kword(&A->fp.nrows);
            const uint32_t tiles = (uint32_t)(((W_ + 7) >> 3) * ((nrows + 7) >> 3) * kword(&A->fp.nframes));
            t = (int)tiles;
            for (uint32_t k = 0; k < RT_QUEUES; k++) {
                const uint32_t x = (xq + k) & (RT_QUEUES - 1);
                if ((drained >> x) & 1u) continue;
                const uint32_t b0 = (uint32_t)((uint64_t)tiles * x / RT_QUEUES);
                const uint32_t b1 = (uint32_t)((uint64_t)tiles * (x + 1) / RT_QUEUES);
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(kload(&A->aux.tile_ctr) + x * RT_QUEUE_STRIDE, 1u);
                c = (uint32_t)__shfl((int)c, 0);
                if (b0 + c < b1) {
                    t = (int)(b0 + c);
                    break;
                }
                drained |= 1u << x;
            }
        }
#else
        t = (int)((blockIdx.x * 4 + wv) + iter++ * gridDim.x * 4);
#endif
        return t;
    };
    int next = RT_TILE_PREFETCH ? fetch() : 0;
    for (;;) {
        A = launder(A);
        const int W_ = kword(&A->fp.W), nrows = kword(&A->fp.nrows);
        const int tiles_x = (W_ + 7) >> 3;
        const int tiles_f = tiles_x * ((nrows + 7) >> 3);  // tiles per frame
        const int tiles = tiles_f * kword(&A->fp.nframes);
        RT_TSTAMP(t_q0);
        if (!RT_TILE_PREFETCH) next = fetch();
        int tile = __shfl(next, 0);
#if RT_TILE_SCHED == 5
        if (tile < tiles) tile = tiles - 1 - tile;  // diagnostic: bottom rows first
#endif
#if RT_TILE_SCHED == 4
        if (tile < tiles) {
            const uint32_t P = (tiles % 7919) ? 7919u : 7927u;  // primes: coprime to tiles
            tile = (int)(((uint64_t)(uint32_t)tile * P) % (uint32_t)tiles);
        }
#endif
#ifdef RT_DIAG_TIMING
        asm volatile("" ::"v"(tile));
#endif
        RT_TACC(7, t_q0);
        if (tile >= tiles) break;
#if defined(RT_DIAG_TIMING) || defined(RT_DIAG_LIFE) || defined(RT_DIAG_WAVES)
        n_tiles++;
#endif
        if (RT_TILE_PREFETCH) next = fetch();
        const int f = tile / tiles_f;  // frame of the batch
        const int ft = tile - f * tiles_f;
        const int i = (ft % tiles_x) * 8 + (lane & 7);
        const int r = (ft / tiles_x) * 8 + (lane >> 3);
#if defined(RT_DIAG_HIST) || defined(RT_DIAG_TILECOST)
        const uint64_t th0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef RT_DIAG_TILECOST
        uint64_t tb[6];
        for (int k = 0; k < 6; k++) tb[k] = tacc[k];
#endif
#if RT_POP_CULL
        trace_packet<W, SP, K, COUNT>(A, f, i, r, i < W_ && r < nrows, stacks[wv], cands[wv], tacc, sbox4[wv],
                                      sbox2[wv]);
#else
        trace_packet<W, SP, K, COUNT>(A, f, i, r, i < W_ && r < nrows, stacks[wv], cands[wv], tacc, nullptr, nullptr);
#endif
#ifdef RT_DIAG_TILECOST
        {   // per-tile duration (10-ns ticks) into hit_pos[3 * tile] (diagnostic build:
            // shade_store leaves hit_pos alone), and the tile's cycle split
            // (s_memtime) into hit_pos[3 * tiles + 8 * tile + k]
            const uint64_t dt = __builtin_amdgcn_s_memrealtime() - th0;
            RT_G double* hp = kload(&A->fp.hit_pos);
            if (hp && lane == 0) {
                hp[3 * (size_t)tile] = (double)dt;
                for (int k = 0; k < 6; k++) hp[3 * (size_t)tiles + 8 * (size_t)tile + k] = (double)(tacc[k] - tb[k]);
                hp[3 * (size_t)tiles + 8 * (size_t)tile + 6] = (double)th0;  // start (10-ns ticks)
            }
        }
#endif
#ifdef RT_DIAG_HIST
        {   // per-tile duration histogram: 64 bins of 2 us (10-ns ticks)
            const uint64_t dt = __builtin_amdgcn_s_memrealtime() - th0;
            RT_G unsigned long long* const dg = kload(&A->aux.diag);
            const uint32_t bin = dt / 200 < 63 ? (uint32_t)(dt / 200) : 63u;
            if (dg && lane == 0) atomicAdd(dg + RT_DIAG_SPREAD + bin * 8 + 4, 1ull);
            // and where it was: rows of tiles, 64 bands, summed duration
            const uint32_t band = (uint32_t)(tile / tiles_x) * 64u / (uint32_t)((nrows + 7) >> 3);
            if (dg && lane == 0) atomicAdd(dg + RT_DIAG_SPREAD + (band & 63) * 8 + 5, dt);
            const uint32_t cband = (uint32_t)(tile % tiles_x) * 64u / (uint32_t)tiles_x;
            if (dg && lane == 0) atomicAdd(dg + RT_DIAG_SPREAD + (cband & 63) * 8 + 6, dt);
        }
#endif
    }
#ifdef RT_DIAG_WAVES
    {   // per-wave start / end (10-ns ticks) and tile count into hit_pos[3 * wave + k]
        // (diagnostic build: shade_store leaves hit_pos alone; tools/wave_life.py)
        RT_G double* hp = kload(&A->fp.hit_pos);
        const size_t wid = (size_t)blockIdx.x * 4 + wv;
        if (hp && lane == 0) {
            hp[3 * wid] = (double)t_life;
            hp[3 * wid + 1] = (double)__builtin_amdgcn_s_memrealtime();
            hp[3 * wid + 2] = (double)n_tiles;
        }
    }
#endif
#if defined(RT_DIAG_TIMING) || defined(RT_DIAG_LIFE) || defined(RT_DIAG_WAVES)
    RT_G unsigned long long* const diag = kload(&A->aux.diag);
    if (diag && lane == 0) {
#ifdef RT_DIAG_TIMING
        for (int q = 0; q < 8; q++) atomicAdd(diag + q, (unsigned long long)tacc[q]);
#endif
        // tail: wave lifetimes (10-ns ticks) and tiles per wave, accumulated
        // over RT_DIAG_SLOTS cache lines (one hot address would serialise)
        const unsigned long long life = __builtin_amdgcn_s_memrealtime() - t_life;
        RT_G unsigned long long* slot = diag + RT_DIAG_SPREAD + (blockIdx.x % RT_DIAG_SLOTS) * 8;
        atomicAdd(slot + 0, life);
        atomicMax(slot + 1, life);
        atomicAdd(slot + 2, 1ull);
        atomicMax(slot + 3, (unsigned long long)n_tiles);
    }
#endif
}
