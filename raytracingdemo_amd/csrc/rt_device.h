// Layouts shared by the host flattener and the gfx950 kernels.
//
// HBM layout of one scene replica (see DESIGN.md §Data layout):
//   wide nodes   W child records of 32 B: fp32 lo.x hi.x lo.y hi.y lo.z hi.z,
//                u32 ref, u32 meta of the child node (its children's sort
//                axis | valid slots << 2; 0 for leaves) — one s_load_dwordx8 per child in the packet
//                kernel, two dwordx4 in the per-lane kernel; node_bytes(W) =
//                32*W (W=8: 256 B, four 64-B lines).  Bounds are the
//                reference's fp64 boxes rounded outward to fp32 (a
//                conservative superset); the kernels widen every slab by a
//                per-frame margin (RtFrameParams.pad).
//   tri32        BVH order, fp32 v0,e1,e2 + pad (48 B)   — fp32 pre-filter
//   tri64        BVH order, fp64 v0,e1,e2 + u32 visit rank + u32 real leaf
//                (80 B)                                  — exact reference MT
//   tri_id/rank/leaf  BVH order u32: loader index, reference visit rank,
//                real leaf node (for the ancestor re-verification)
//   rbox/rparent real reference nodes: fp64 box (48 B) + parent
//   normal       loader order fp64 normal (24 B), read once per hit pixel
#pragma once
#include <stdint.h>

#define RT_LEAF_BIT 0x80000000u
#define RT_INVALID_REF 0xFFFFFFFFu
#define RT_LEAF_FIRST_MASK 0x07FFFFFFu
#define RT_LEAF_MAX_FIRST 0x07FFFFFFu
// scene triangle cap: the packet walk addresses tri32 records (48 B) with
// 32-bit byte offsets (packet_kernel.h leaf loop), padding included
#define RT_MAX_TRIS 0x05000000u
#define RT_CHILD_REF 6       // u32 slot of the child ref in a 32-B child record
// fp64 triangle record, one 128-B line in BVH order: everything k_resolve
// needs for a candidate in one round trip.
//   [0..8]   v0, e1, e2 (doubles)         Moller-Trumbore (triangle.hpp:42)
//   [9..11]  unit normal (triangle.hpp:17, normalised as main.cpp:361 does)
//   [12]     {u32 loader id, u32 real leaf}
//   [13..15] leaf box as 6 floats rounded inward (chain_fast_ok32)
// The visit rank (ties only) stays in RtDevScene::tri_rank.
#define RT_TRI64_DOUBLES 16
#define RT_T64_NORMAL 9
#define RT_T64_IDLEAF 12
#define RT_T64_BOX 13
// Work-queue block (RtLaunchAux::tile_ctr, RT_QUEUE_WORDS u32, zeroed per
// launch): RT_QUEUES tile queues RT_QUEUE_STRIDE words apart (one per XCD,
// separate cache lines), the redo-list length, and the hit-count partials.
#ifndef RT_QUEUES
#define RT_QUEUES 8
#endif
#define RT_QUEUE_STRIDE 16
#define RT_REDO_COUNT (RT_QUEUES * RT_QUEUE_STRIDE)
// chunks of the candidate overflow pool handed out so far
#define RT_POOL_COUNT (RT_REDO_COUNT + RT_QUEUE_STRIDE)
// k_fixup blocks that have read the redo count (the last one clears it)
#define RT_FIXUP_DONE (RT_REDO_COUNT + 2 * RT_QUEUE_STRIDE)
// redo-list entries taken so far by the packet kernel's own waves, and its
// exit tickets (RtLaunchAux::self_fix: the launch ends without k_fixup)
#define RT_REDO_CLAIM (RT_REDO_COUNT + 3 * RT_QUEUE_STRIDE)
#define RT_EXIT_COUNT (RT_REDO_COUNT + 4 * RT_QUEUE_STRIDE)
// nonzero: a wave of the packet kernel's own redo pass gave an entry up (the
// list's all-empty invariant was broken); reported to the host through
// RtLaunchAux::redo_seen as RT_SEEN_ERROR (launch pixels < 2^31, so the bit
// is free)
#define RT_EXIT_ERROR (RT_REDO_COUNT + 5 * RT_QUEUE_STRIDE)
#define RT_SEEN_ERROR 0x80000000u
// rows of the side de-interleave job (RtLaunchAux::job_*) claimed so far,
// one counter per XCD queue (queue x takes rows x, x + RT_QUEUES, ...: a
// counter shared by all XCDs would serialise on cross-XCD atomics)
#define RT_COPY_BASE 256
// then, per frame of the launch, RT_HIT_SLOTS hit-count partial sums
// RT_QUEUE_STRIDE words apart (frame f's slot s at RT_HIT_BASE + (f *
// RT_HIT_SLOTS + s) * RT_QUEUE_STRIDE)
#define RT_HIT_SLOTS 64
#define RT_HIT_BASE 1024
// Frames per launch: one launch of the packet pipeline renders up to
// RT_MAX_BATCH frames (camera poses) of the same geometry, so the persistent
// traversal kernel's ramp-up and tail, and the launch gaps, are paid once per
// batch instead of once per frame.
#ifndef RT_MAX_BATCH
#define RT_MAX_BATCH 36
#endif
#define RT_QUEUE_WORDS (RT_HIT_BASE + RT_MAX_BATCH * RT_HIT_SLOTS * RT_QUEUE_STRIDE)
// Candidate lists of the packet walk, per pixel: RT_CAND_LDS entries kept in
// LDS ({triangle, t lower bound}, 8 B each); past them a lane takes one chunk
// of RT_POOL_CHUNK entries from a shared overflow pool in HBM (allocated with
// one atomic, sized by the host; a dry pool falls back to the certified
// dropped bound).  With spp > 1 the LDS entries go to HBM for k_resolve
// ([RT_CAND_LDS][pixels] + count byte + dropped bound + chunk index).
#ifndef RT_CAND_LDS
#define RT_CAND_LDS 8
#endif
#define RT_POOL_CHUNK 24
// Quantised W = 8 node for the per-lane walk (walk_tree.cpp quantize_wide8):
// origin, exponents, SoA 8-bit planes, refs.
#ifndef RT_QNODE_BYTES
#define RT_QNODE_BYTES 96
#endif
// tri32 is followed by this many zero records (chunked leaf fetches may read past the end)
#define RT_TRI32_PAD 4

#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif
// Image shards for multi-GPU frames: bands of RT_SHARD_BAND
// rows (one row of 8x8 tiles) interleaved over the shards — band b of a frame
// goes to shard b mod G, so every shard keeps whole, coherent tiles and the
// depth-complexity gradient is still spread evenly.  (Single interleaved rows,
// the round-1 layout, turn a shard's 8x8 tile into 8 columns spread over 64
// image rows: one GPU's rate on 1/8 of a frame fell to 48% of its full-frame
// rate.)  A shard's rows, in shard order, are its bands back to back; image
// row of shard row r: rt_image_row(g, G, RT_SHARD_BAND, r).
#define RT_SHARD_BAND 8
static inline RT_HD int rt_image_row(int row0, int row_stride, int band, int r) {
    return band <= 1 ? row0 + r * row_stride : (row0 + (r / band) * row_stride) * band + r % band;
}
static inline RT_HD int rt_shard_rows(int H, int G, int g) {
    const int nb = (H + RT_SHARD_BAND - 1) / RT_SHARD_BAND;  // bands, the last one possibly partial
    if (g >= nb) return 0;
    const int bands = (nb - 1 - g) / G + 1;
    const int last = H - (nb - 1) * RT_SHARD_BAND;  // rows of the last band
    return bands * RT_SHARD_BAND - ((nb - 1) % G == g ? RT_SHARD_BAND - last : 0);
}
// rows every shard's block is sized for
static inline RT_HD int rt_shard_pad(int H, int G) {
    return ((H + RT_SHARD_BAND - 1) / RT_SHARD_BAND + G - 1) / G * RT_SHARD_BAND;
}
// Byte offset of image row j of frame f in the gathered [G][block] buffer:
// shard g's block holds at sec_off its frames back to back ([F][rows_g][W]
// elements of eb bytes, as its shard render wrote them).
static inline RT_HD uint64_t rt_gathered_row(int j, int f, int G, int H, int W, int eb, uint64_t block,
                                             uint64_t sec_off) {
    const int b = j / RT_SHARD_BAND, g = b % G;
    const int r = (b / G) * RT_SHARD_BAND + j % RT_SHARD_BAND;  // row within the shard
    return (uint64_t)g * block + sec_off + ((uint64_t)f * (uint64_t)rt_shard_rows(H, G, g) + (uint64_t)r) *
                                               (uint64_t)W * (uint64_t)eb;
}

#ifdef __cplusplus
static inline constexpr uint32_t rt_node_bytes(int W) { return (uint32_t)(32 * W); }
static inline constexpr uint32_t rt_make_leaf(uint32_t first, uint32_t count) {
    return RT_LEAF_BIT | ((count - 1u) << 27) | first;
}
#endif

// Device passes see every pointer member as a global-memory pointer, so
// kernels that read these structs out of the kernarg block (not only as
// kernel parameters) still emit global_* rather than flat_* accesses.  The
// layout is the same on host and device.
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_G __attribute__((address_space(1)))
#else
#define RT_G
#endif

struct RtDevScene {
    const RT_G uint8_t* nodes;
    const RT_G float* tri32;      // 12 floats per triangle: v0,e1,e2, max|e1|,max|e2|,max|v0|
    const RT_G double* tri64;     // RT_TRI64_DOUBLES per triangle (layout above)
    const RT_G uint32_t* tri_id;
    const RT_G uint32_t* tri_rank;
    const RT_G uint32_t* tri_leaf;
    const RT_G double* rbox;      // 6 per real node
    const RT_G int32_t* rparent;
    const RT_G double* normal;    // loader order, 3 per triangle
    const RT_G uint32_t* rkid_off;// real tree CSR (literal reference-order mode)
    const RT_G uint32_t* rkid;
    const RT_G uint32_t* rrange;  // real node primitive range [begin, end) (reference order)
    const RT_G uint32_t* ref2walk;// reference-order position -> BVH-order triangle index
    const RT_G uint8_t* qnodes;   // W = 8: quantised copy of `nodes` (RT_QNODE_BYTES each), else null
    uint32_t root_ref;
    float root_box[6];
    uint32_t n_tris;
    uint32_t node_bytes;
    int32_t width;
    uint32_t stack_bound;
    double coord_max;             // max |coordinate| of the scene (slab margins of arbitrary rays)
    uint32_t n_wide;              // wide nodes
    uint32_t root_meta;           // the root's sort axis | valid slots << 2 (each child record's pad
                                  // word holds its child node's; bvh_build.cpp flatten)
};

// RtLaunchAux::self_fix bits
#define RT_SELF_FIX 1
#define RT_SELF_STORE 2

// Per-launch resources of the persistent exact kernel.
struct RtLaunchAux {
    RT_G uint32_t* tile_ctr;   // work-queue block (RT_QUEUE_WORDS words), zeroed before every launch
    RT_G uint64_t* spill;      // traversal-stack spill: spill_cap entries per lane
    uint32_t spill_cap;
    int32_t grid;         // persistent blocks (CUs x resident blocks per CU)
    RT_G uint32_t* redo;       // packet kernel -> k_fixup: pixel index | start-pass bit (kRedoEmpty: none)
    uint64_t redo_cap;    // entries (a fixed pool: past it k_fixup retries the whole launch)
    uint32_t* redo_seen;  // host-mapped word: k_fixup reports the launch's redo count there (or null);
                          // the host grows the slot's list for its next launches from it
    int32_t fgrid;        // k_fixup blocks (0: the default kFixupGrid)
    int32_t self_fix;     // RT_SELF_FIX: the fused packet kernel's own waves finish the redo list
                          // and the bookkeeping (packet_exit), no k_fixup (redo_cap >= the launch's
                          // pixels; spill sized for the packet grid); | RT_SELF_STORE: its last wave
                          // stores the per-pose hit counts instead of adding them (RT_FLAG_COUNTS_STORE)
    RT_G uint64_t* pool;       // candidate overflow pool: pool_chunks x RT_POOL_CHUNK entries
    uint32_t pool_chunks;
    int32_t pgrid;             // workgroups of the packet kernel (64 * kPacketWaves threads each)
    // spp > 1 (packet kernel -> k_resolve) and the wavefront path tracer:
    RT_G uint64_t* cand;       // {tri, t lower bound} per entry, [K][pixels]
    RT_G uint8_t* cand_cnt;    // entries per pixel | kCandSpilled | kCandDropped (wavefront: 0xFF = overflow)
    uint64_t cand_cap;         // pixels the candidate buffers hold
    RT_G float* cand_drop;     // per pixel: smallest t bound of a dropped candidate (if flagged)
    RT_G uint32_t* cand_ovf;   // per pixel: its overflow pool chunk (if flagged)
    // A de-interleave done on the side (include/rt.h rt_deinterleave_job):
    // the packet kernel's waves copy its rows between and after their tiles.
    // Row j of frame f comes from shard g = (j / RT_SHARD_BAND) % job_G of
    // the gathered [job_G][job_block] buffer (job_rows rows per frame in each
    // block, 0: rt_shard_rows, the library's own group layout).  job_src NULL:
    // no job.
    RT_G const uint8_t* job_src;
    RT_G uint8_t* job_dst;
    uint64_t job_block, job_sec;
    int32_t job_G, job_F, job_H, job_W, job_eb, job_rows;
};
// Byte offsets of row j of frame f of a side job: in the gathered buffer and
// in the frames [F][H][W][eb].
static inline RT_HD uint64_t rt_job_src_row(const RtLaunchAux& a, int j, int f) {
    if (a.job_rows <= 0) return rt_gathered_row(j, f, a.job_G, a.job_H, a.job_W, a.job_eb, a.job_block, a.job_sec);
    const int b = j / RT_SHARD_BAND, g = b % a.job_G;
    const int r = (b / a.job_G) * RT_SHARD_BAND + j % RT_SHARD_BAND;
    return (uint64_t)g * a.job_block + a.job_sec +
           ((uint64_t)f * (uint64_t)a.job_rows + (uint64_t)r) * (uint64_t)a.job_W * (uint64_t)a.job_eb;
}

// One camera pose of a launch (Camera, camera.hpp:20-38: position, view
// direction and the basis main.cpp:325-329 derives from it).
struct RtPose {
    double pos[3], dir[3], right[3], up[3];
    float pad;                     // world-space slab margin of the fp32 traversal (per pose)
    uint32_t reserved;
};
// A pose with the sub-pixel offset of one sample (kernel side: frame_cam).
struct RtFrameCam {
    double pos[3], dir[3], right[3], up[3];
    float pad;
    uint32_t reserved;
    double ox, oy;                 // sub-pixel sample offset (0.5, 0.5 = the reference's pixel centre)
};

// One launch: `nframes` sample frames of the same image geometry and row
// shard, poses pose[0 .. nframes / spp - 1].  With spp samples per pixel a
// pose is spp consecutive frames (sample s of pose p = frame p * spp + s, its
// own sub-pixel offset, computed in-kernel: frame_cam); outputs are per pose: per-sample values (hit_id, dist,
// hit_pos) of pose p, pixel o, sample s at (p * W * nrows + o) * spp + s, the
// averaged colour (rgb) at p * W * nrows + o, the hit counter (samples hit)
// at hit_count[p].  spp = 1 is the reference's one ray per pixel centre.
struct RtFrameParams {
    double cam_iw, cam_ih;        // 1/W, 1/H            (camera.hpp:33-34)
    double cam_half, cam_aspect;  // tan(fov/2), W/H      (camera.hpp:29-30)
    int32_t W, H;
    int32_t row0, row_stride, nrows;  // shard row r is image row rt_image_row(row0, row_stride, band, r)
    int32_t nframes;              // 1..RT_MAX_BATCH, a multiple of spp
    int32_t spp;                  // samples per pixel (n x n stratified), >= 1
    int32_t band;                 // 1: rows (row0, row_stride in rows); RT_SHARD_BAND: banded shard (in bands)
    int32_t spp_n;                // n of the n x n sample pattern (spp = n * n)
    int32_t pack;                 // 1: a packet wave takes all spp samples of (8/n)^2 pixels (64 % spp == 0)
    RT_G uint32_t* hit_id;
    RT_G double* dist;
    RT_G double* hit_pos;
    RT_G uint8_t* rgb;
    RT_G unsigned long long* hit_count;
    RT_G unsigned long long* counters;  // [rays, node_fetches, tri_tests, chain_checks, hits, chain_nodes] or NULL
    RtPose pose[RT_MAX_BATCH];    // pose f / spp of sample frame f (104 B each: 36 fit the LDS copy)
};

// Workspace of the queued path tracer (queue_paths.h), per replica: every
// path of a pose at once.
struct PathQs {
    RT_G double* q[2];     // segment queues, 10 doubles per entry {o, d, L, path}
    RT_G double* Lfin;     // 3 per path (pixel * spp + sample): radiance when the path ended
    RT_G uint32_t* fb;     // fall-back lists, [2][cap]: queue slots for the exact per-lane traversal
    RT_G uint32_t* ctl;    // control words (queue_paths.h qc_*), zeroed per pose
    uint32_t cap;          // paths (entries per queue)
    // Each queue is `parts` partitions of `pcap` entries (parts * pcap <=
    // cap), each with its own append and pull counters: partition x holds
    // the rays of the primary tiles of XCD queue x and everything they
    // bounce into, so no counter is shared by the whole chip (one word takes
    // ~88 atomics per us: 2.07 M primary tiles on one counter alone took
    // 23.7 ms per pose).  parts = 1: one queue (k_q_primary's primaries).
    uint32_t parts, pcap;
    uint32_t ptile, ptiles_x;  // parts > 1: the primary tiles' edge in pixels and tiles per row
    // occlusion-ray queue (queued shadows): records {p (3 doubles), tri | dst}
    // as the segment kernel appends them, each with its sort key (skey: the
    // direction from the light, queue_paths.h sh_key); the binning passes
    // order (key, record) pairs (spair[0] after the low digit, spair[1] after
    // the high one) with per-block bin counts bhist, and the occlusion walk
    // reads the records through the sorted pairs
    // (one base pointer: srec's records, then per record slot the two pair
    // arrays and the keys — rt_q_spair / rt_q_skey; the argument block of the
    // packet kernel, which carries PathQs, keeps its size)
    RT_G double* srec;
    RT_G uint32_t* bhist;  // [bins][sh_blocks]
    uint32_t sh_blocks;
};
// The sort arrays behind the occlusion records (cap record slots): pairs
// {key, record} (two u32) after pass p at spair(p & 1), the keys at skey.
static inline RT_HD RT_G uint64_t* rt_q_spair(const PathQs& q, int k) {
    return reinterpret_cast<RT_G uint64_t*>(reinterpret_cast<RT_G char*>(q.srec) + (uint64_t)q.cap * (32u + 8u * (uint32_t)k));
}
static inline RT_HD RT_G uint32_t* rt_q_skey(const PathQs& q) {
    return reinterpret_cast<RT_G uint32_t*>(reinterpret_cast<RT_G char*>(q.srec) + (uint64_t)q.cap * 48u);
}
#define RT_QPARTS RT_QUEUES
// k_trace_packet deals its tiles to the XCD queues in runs of RT_TILE_RUN
// consecutive tiles (tile t to queue (t / RUN) % RT_QUEUES).  Tuning knob:
// runs of 4 (a run's 8-pixel tile rows = 96 B of rgb, three whole 32-B
// sectors from one XCD) measured 1.49 GB of writes per headline launch
// against 1.38 with runs of 1, and 1.69 with cached (not non-temporal)
// outputs, at the same 4.16-4.21 ms.
#ifndef RT_TILE_RUN
#define RT_TILE_RUN 1
#endif
#define RT_QC_LINES (4 * RT_QPARTS + 1)
#define RT_QC_WORDS(bounces) (RT_QC_LINES * ((bounces) + 1) * 16)
// The partitioned layout of a pose of W x nrows pixels at spp = n x n samples
// (n = 2 or 4): the packed primary tiles (8 / n pixels square, 64 samples)
// dealt in runs of RT_TILE_RUN round-robin to the RT_QPARTS partitions, each
// with room for its tiles' samples; `entries` = the queue length it needs
// (>= the paths).
struct RtQParts {
    uint32_t pcap, ptile, ptiles_x;
    uint64_t entries;
};
static inline RT_HD RtQParts rt_qparts(int W, int nrows, int spp) {
    RtQParts p{};
    p.ptile = spp == 16 ? 2u : 4u;
    p.ptiles_x = ((uint32_t)W + p.ptile - 1) / p.ptile;
    const uint64_t T = (uint64_t)p.ptiles_x * (((uint32_t)nrows + p.ptile - 1) / p.ptile);
    const uint64_t runs = (T + RT_TILE_RUN - 1) / RT_TILE_RUN;
    p.pcap = (uint32_t)((runs + RT_QPARTS - 1) / RT_QPARTS * RT_TILE_RUN * 64);
    p.entries = (uint64_t)p.pcap * RT_QPARTS;
    return p;
}
// occlusion-ray order: a cube map around the light, 2^RT_SH_CELL_BITS squared
// cells per face in Morton order (19-bit keys), counting-sorted in passes of RT_SH_BITS
// bits (per-block counts of RT_SH_BLOCKS blocks; RT_SH_HBINS bins)
#ifndef RT_SH_CELL_BITS
#define RT_SH_CELL_BITS 8  // 256 x 256 cells per face: c5 187.1 / 187.3 vs 189.2 / 189.4 ms per pose at 512^2, 190.7 at 128^2
#endif
#define RT_SH_CELLS (1 << RT_SH_CELL_BITS)
#define RT_SH_KEY_BITS (3 + 2 * RT_SH_CELL_BITS)
#ifndef RT_SH_BITS
#define RT_SH_BITS 7
#endif
#define RT_SH_HBINS (1 << RT_SH_BITS)
#define RT_SH_BLOCKS 256

