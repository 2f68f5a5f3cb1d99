/*
 * rt.h — C ABI of librtmi355x.so, the MI355X-native primary-ray tracer.
 *
 * The reference (insomnick/raytracingdemo) has no FFI; its natural seam is
 * one whole frame, `calculateScreen(StackBVH&, Camera&)` (src/main.cpp:322),
 * which the caller `runTest` times (src/main.cpp:253-257) and follows with
 * `shadeScreen` (src/main.cpp:351-381).  This ABI replaces that frame call
 * and the objects it needs; each entry point names the reference interface it
 * stands in for.  Plain pointers and sizes only; caller owns host buffers,
 * the library owns device memory unless an *_device entry point is used.
 *
 * Semantics are the reference's, bit for bit: per-pixel hit-IDs (loader
 * order), hit positions (fp64 o + d*t) and PPM bytes are identical to
 * StackBVH::traverse + shadeScreen on the same tree.
 *
 * Errors: every int-returning call returns RT_OK (0) or a status below; the
 * message is in rt_last_error() (thread-local).  Where the reference throws
 * (stack_bvh.hpp:543,550 std::out_of_range; main.cpp:159,180,201
 * std::invalid_argument "Unsupported bvh degree"; main.cpp:204
 * std::out_of_range "Unknown algorithm"; object_loader.hpp:17
 * std::runtime_error "Failed to load OBJ file") the same message text is
 * returned with the matching status.  Nothing crosses the ABI as an exception.
 *
 * Threading: a scene's geometry is immutable after rt_scene_create.  Any
 * number of host threads may call the render and stats entry points on one
 * scene; the scene's lock serialises the host side of the calls (a caller
 * stream still runs its launches asynchronously).
 * Device ordering follows the caller's streams: launches issued on one
 * stream run in order; launches issued on two different streams may run
 * concurrently on the device (each device replica keeps two sets of launch
 * state and alternates them), so a caller that issues consecutive batches on
 * two streams overlaps one batch's tail with the next one's start.  Ordering
 * between streams that read each other's outputs is the caller's, as for any
 * HIP work.  Counting passes (RT_FLAG_COUNT) and the modes that use the
 * replica-wide candidate lists are ordered after every earlier launch.
 * rt_scene_destroy must not race with other calls on the same scene.
 *
 * Deviations from the boundary SURVEY.md §8(b) sketched (deliberate):
 *  - rt_render_frame_cpu is absent.  The library has no CPU render path of
 *    any kind, so nothing can fall back to one; the CPU baseline is the
 *    reference's own traversal compiled -O3 from its headers (oracle/_ref,
 *    test and bench infrastructure only).
 *  - Samples per pixel and the seed are not rt_camera fields.  spp travels as
 *    an argument of the entry points that take samples
 *    (rt_render_batch_spp_device, rt_render_shard_device,
 *    rt_render_batch_multi, rt_render_paths_device); stratified samples need
 *    no seed, and the path tracer's hash seed is the `frame` argument.
 *    rt_camera keeps the reference's Camera fields (camera.hpp:20-38) plus
 *    the image size.
 *  - SURVEY's mode PARITY_FP64 | FAST_FP32 maps to RT_MODE_FP64 (fp64
 *    traversal of the reference tree throughout) | RT_MODE_EXACT (fp32
 *    conservative traversal with the fp64 reference tests at the leaves).
 *    Both return the reference's results bit for bit; FAST_FP32 in the survey
 *    allowed a tolerance this library does not need.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6

/* status codes */
#define RT_OK 0
#define RT_ERR_INVALID_ARGUMENT 1 /* std::invalid_argument in the reference */
#define RT_ERR_OUT_OF_RANGE 2     /* std::out_of_range in the reference    */
#define RT_ERR_RUNTIME 3          /* std::runtime_error (OBJ load failure)  */
#define RT_ERR_HIP 4              /* HIP runtime failure                    */
#define RT_ERR_NO_DEVICE 5        /* no gfx950 device / scene not uploaded  */

/* BVH partition algorithms (main.cpp:128-205; stack_bvh.hpp:453-499) */
#define RT_ALGO_MEDIAN 0
#define RT_ALGO_SAH 1
#define RT_ALGO_BSAH 2

/* traversal modes: both are exact (identical results); they differ in speed
 * (SURVEY.md §8(b)'s FAST_FP32 / PARITY_FP64) */
#define RT_MODE_EXACT 0 /* fp32 conservative traversal + fp64 reference leaf tests */
#define RT_MODE_FP64 1  /* fp64 traversal throughout (simple, slower)          */

/* render flags */
#define RT_FLAG_COUNT 1u  /* also count node/triangle fetches (rt_frame_stats) */
#define RT_FLAG_TIMING 2u /* time the pipeline kernels with HIP events on the
                             launching stream (rt_frame_stats)              */
#define RT_FLAG_SHADOW 4u /* rt_render_paths_device: one occlusion ray toward the
                             head-light from every bounce vertex            */
#define RT_FLAG_SIDE_SLOT 8u /* primary-ray renders: the persistent traversal
                             grid leaves one workgroup slot per CU free, so a
                             kernel on another stream — a collective shipping
                             the previous step's frames — runs beside the
                             render instead of after it (one-process-per-GPU
                             drivers)                         */
#define RT_FLAG_COUNTS_STORE 16u /* batch / shard / paths renders: hit_count[f]
                             is SET to the call's count instead of being added
                             to, so the caller need not zero it before every
                             render (runTest's per-frame shadeScreen return,
                             main.cpp:260-262).  The fused packet kernel
                             stores the counts from its last wave; where a
                             pipeline cannot, the library zeroes the counters
                             on the stream first (same result).             */

#define RT_MISS 0xFFFFFFFFu

typedef struct rt_scene rt_scene;

/* A camera pose plus image geometry.  pos/dir as produced by
 * rt_camera_path (CameraPath::circularPath, camera_path.hpp:18-26). */
typedef struct {
    double pos[3];
    double dir[3];
    int32_t width, height; /* the reference hard-codes 500x500 (main.cpp:36-37) */
} rt_camera;

/* Host-side frame outputs (any pointer may be NULL).  Pixel (i, j) — i the
 * column (left->right), j the row (top->bottom) as in main.cpp:331-334 — is
 * stored row-major at j*width + i (the reference stores idx=j+i*H, a layout
 * choice; PPM order is row-major, benchmark.hpp:105-114). */
typedef struct {
    uint32_t *hit_id;   /* W*H, loader-order triangle index, RT_MISS = none  */
    double *dist;       /* W*H, |hit - o| (stack_bvh.hpp:631), -1 on a miss */
    double *pos;        /* 3*W*H, hit position o + d*t (triangle.hpp:86)      */
    uint8_t *rgb;       /* 3*W*H, shadeScreen colour as PPM bytes             */
    uint64_t hit_count; /* out: shadeScreen's return value (main.cpp:380)    */
    double seconds;     /* out: device time of ray generation + traversal   */
} rt_frame_out;

/* Device-side outputs for rt_render_rows_device (pointers on the scene's
 * device; any may be NULL).  Row r of the shard is image row
 * row0 + r*row_stride; its pixels are at r*width + i. */
typedef struct {
    uint32_t *hit_id;
    double *dist;
    double *pos;
    uint8_t *rgb;
    unsigned long long *hit_count; /* one counter, atomically incremented */
} rt_device_out;

typedef struct {
    uint64_t triangles;
    uint64_t real_nodes, real_inner, real_leaves;
    uint32_t depth, max_children, max_leaf_size;
    uint32_t wide_width;      /* W of the device node format (2/4/8/16) */
    uint64_t wide_nodes;      /* device wide nodes (incl. virtual ones) */
    uint64_t device_bytes;    /* scene bytes resident per device        */
    uint32_t stack_bound;     /* worst-case traversal stack entries     */
    double node_bytes;        /* bytes of one wide node                 */
    uint32_t walk_tree;       /* 1: device nodes from the rebuilt SAH walk tree
                                 (results unchanged), 0: from the
                                 reference tree itself (RT_WALK=reference) */
    uint64_t layout_digest;   /* 64-bit FNV-style digest of the device scene
                                 sections (host copy): equal digests = the same
                                 device scene, byte for byte (build tests) */
} rt_scene_stats_t;

typedef struct {
    uint64_t rays;
    uint64_t node_fetches;  /* wide nodes loaded                     */
    uint64_t tri_tests;     /* fp64 Moller-Trumbore tests             */
    uint64_t chain_checks;  /* fp64 ancestor-chain re-verifications  */
    uint64_t hits;
    uint64_t chain_nodes;   /* fp64 ancestor boxes loaded by those checks */
    uint64_t tri_prefilter; /* fp32 conservative triangle pre-tests     */
    uint64_t wave_nodes;    /* packet kernel: inner-node visits per wave */
    uint64_t wave_leaves;   /* packet kernel: leaf visits per wave       */
    uint64_t wave_tiles;    /* packet kernel: 8x8 tiles traced           */
    uint64_t wave_tris;     /* packet kernel: triangle records fetched per wave */
    uint64_t redo_rays;     /* rays finished by the fix-up kernel (exact per-lane path) */
    uint64_t redo_chain;    /*   of which: winner invisible to the reference (chain check) */
    uint64_t spilled_rays;  /* packet kernel: rays whose candidate list overflowed
                               LDS into a pool chunk in HBM                */
    uint64_t dropped_rays;  /*   of which: the chunk filled too, a candidate was
                               dropped (certified bound, else fix-up)      */
    uint64_t empty_node_steps; /* packet kernel: node steps where no lane entered
                                  any child                                */
    uint64_t wave_tri_tests; /* packet kernel, fused resolve: fp64 triangle records
                                tested, counted once per wave (distinct over its
                                lanes; tri_tests counts them per lane)     */
    uint64_t wave_winners;   /*   winners' shading records, once per wave  */
    uint64_t shadow_rays;    /* paths with RT_FLAG_SHADOW: occlusion rays cast  */
    uint64_t shadow_occluded;/*   of which occluded                            */
    uint64_t side_jobs_fused;  /* rt_deinterleave_job: done by the traversal kernel */
    uint64_t side_jobs_kernel; /*   done by a de-interleave kernel after the render */
    uint64_t shadow_wave_nodes;/* queued occlusion rays: wave node steps of the any-hit walk */
    uint64_t shadow_wave_tris; /*   and triangle records it fetched, once per wave      */
    uint64_t shadow_lane_nodes;/* per-lane occlusion walks: quantised node steps, per lane */
    uint64_t shadow_lane_tris; /*   and fp32 triangle records they tested                  */
    uint64_t timed_launches; /* RT_FLAG_TIMING launches since the last reset */
    double trace_ms;         /*   summed traversal-kernel time (HIP events
                                  recorded around it on the launch stream) */
    uint64_t lane_wave_nodes;/* per-lane walks (paths, occlusion rays): node fetches
                                counted once per wave instruction (lanes of one
                                step loading the same node share the fetch) */
    uint64_t lane_wave_tris; /*   and fp32 triangle records, the same way  */
} rt_frame_stats_t;

/* Host time of each stage of rt_scene_create (std::chrono, ms).  With the
 * walk tree built on a device (rt_scene_create_on_device) the two trees are
 * built at the same time (the reference tree on host threads), so their times
 * overlap: total_ms = soup + max(reference tree, walk tree) + flatten. */
typedef struct {
    double soup_ms;           /* triangle set-up (triangle.hpp:14-19)                 */
    double reference_tree_ms; /* StackBVH::build + collapse (stack_bvh.hpp:502-608)   */
    double walk_tree_ms;      /* the SAH walk tree: host, or device build + copy back */
    double flatten_ms;        /* wide nodes, records, ranks and chains                */
    int32_t walk_device;      /* device that built the walk tree, -1 = host           */
    int32_t reserved;
    double total_ms;          /* wall time of the whole rt_scene_create               */
} rt_build_times_t;

/* objl::Loader + ObjectLoader::loadFromFile (object_loader.hpp:14-70,
 * lib/OBJ_Loader.h:431-713): N*9 doubles (v0,v1,v2), loader order, each
 * coordinate double(float) * scale.  *tris is malloc'd; free with rt_free. */
int rt_load_obj(const char *path, double scale, double **tris, uint64_t *n_tris);
void rt_free(void *p);

/* rt_load_obj through a binary scene cache: the
 * loader's output is kept in cache_dir under the FNV-1a digest of the OBJ
 * bytes and the scale; a valid entry is returned as is (bit-identical to
 * rt_load_obj), anything else is parsed and the entry (re)written.
 * *from_cache (may be NULL) = 1 on a cache hit. */
int rt_load_obj_cached(const char *path, double scale, const char *cache_dir, double **tris, uint64_t *n_tris,
                       int *from_cache);

/* runTest's scene centre (main.cpp:118-122). */
int rt_scene_center(const double *tri_v, uint64_t n_tris, double center[3]);

/* CameraPath(centre, resolution).circularPath(step) with the path centre
 * recomputed as runTest does (main.cpp:123,235; camera_path.hpp:18-26). */
int rt_camera_path(const double scene_center[3], int resolution, int step, double pos[3], double dir[3]);

/* StackBVH::build(prims, partitionFn) (+ collapse passes for the "-c"
 * variants: 2-way partition then log2(k)-1 collapse passes, main.cpp:208,
 * 219-221).  algo = RT_ALGO_*, k in {2,4,8,16}.  The tree is identical to the
 * reference's.  The scene is host-only until rt_scene_upload.  At most
 * 83,886,080 triangles (the packet walk's 32-bit record offsets): more is
 * RT_ERR_INVALID_ARGUMENT "too many triangles". */
int rt_scene_create(const double *tri_v, uint64_t n_tris, int algo, int k, int collapse, rt_scene **out);

/* rt_scene_create with the walk tree (the SAH tree the device traverses,
 * DESIGN.md §3) built on HIP device `device` (the
 * reference times StackBVH::build as its dynamic-scene metric,
 * scripts/bvh_analysis.py:62,543).  The splits are the host builder's; only
 * the order of triangles inside a node may differ, which never changes a
 * result.  The reference tree itself stays a host build: it fixes the tie
 * ranks and ancestor chains and its libstdc++ partition order. */
int rt_scene_create_on_device(const double *tri_v, uint64_t n_tris, int algo, int k, int collapse, int device,
                              rt_scene **out);

/* Stage times of the scene's creation. */
int rt_scene_build_times(const rt_scene *s, rt_build_times_t *out);

/* Replicate the flattened scene on each listed HIP device (ordinal).  With
 * more than one device, the first rt_render_frame / rt_render_batch_multi
 * creates an RCCL communicator over them (ncclCommInitAll, one rank per device
 * in this process; rank g = the g-th uploaded device); uploading itself never
 * needs RCCL. */
int rt_scene_upload(rt_scene *s, const int *devices, int n_devices);

/* One whole frame, blocking; replaces calculateScreen + shadeScreen
 * (main.cpp:253-262).  On one device it renders there; on G uploaded devices
 * image rows are sharded in bands of 8 (band b on the (b mod G)-th device; as
 * rt_render_shard_device), each device
 * renders its shard, and the shards (hit-id + dist + pos + rgb as requested,
 * hit counts) are gathered to the first device with RCCL and de-interleaved
 * there before the copy to the host (shards as
 * rt_render_shard_device's).  seconds: device time
 * of the frame on the first device's stream (renders to gather). */
int rt_render_frame(rt_scene *s, const rt_camera *cam, int mode, rt_frame_out *out);

/* Shard `shard` of `nshards` of every pose's frame (the multi-GPU partition,
 * SURVEY.md §8(e)): bands of 8 image rows (one row of 8x8 tiles) interleaved
 * over the shards, band b on shard b mod nshards, so each shard keeps whole
 * tiles.  Outputs as rt_render_batch_spp_device's with nrows =
 * rt_shard_height(height, nshards, shard) rows per frame, the shard's rows in
 * image order.  This is the call of a one-process-per-GPU driver (bench.py);
 * rt_render_batch_multi uses the same layout inside the library. */
int rt_render_shard_device(rt_scene *s, int device, const rt_camera *cams, int nframes, int spp, int mode, int shard,
                           int nshards, const rt_device_out *out, void *stream, uint32_t flags);

/* A de-interleave of gathered shards into full frames, done by the traversal
 * kernel of a render on the side (rank 0 of a one-process-per-GPU driver:
 * the previous step's gathered framebuffers, while this step renders).
 * `gathered` holds `shards` blocks of block_bytes; image row j of frame f
 * comes from shard g = (j / 8) % shards, row r = ((j / 8) / shards) * 8 + j % 8
 * of it, at g * block_bytes + section_offset + (f * rows + r) * width *
 * elem_bytes, rows = frame_rows, or rt_shard_height(height, shards, g) when
 * frame_rows is 0 (rt_render_batch_multi's own layout).  Writes
 * frames_out[frames][height][width] elements of elem_bytes.  The caller
 * orders the gather that fills `gathered` before the render, and keeps both
 * buffers alive until the render is done. */
typedef struct rt_deinterleave_job {
    const void *gathered;
    uint64_t block_bytes;
    uint64_t section_offset;
    int shards, frames, height, width, elem_bytes;
    int frame_rows;
    void *frames_out;
} rt_deinterleave_job;

/* rt_render_shard_device plus a de-interleave job (NULL: none) that the
 * render's persistent traversal waves carry out between and after their
 * tiles — memory-bound copies beside the latency-bound walk — instead of a
 * separate kernel that waits for the render's grid to drain.
 * Pipelines whose kernel does not take the job run it after the render. */
int rt_render_shard_device_job(rt_scene *s, int device, const rt_camera *cams, int nframes, int spp, int mode,
                               int shard, int nshards, const rt_device_out *out, const rt_deinterleave_job *job,
                               void *stream, uint32_t flags);

/* Rows of shard `shard` of `nshards` of an image `height` rows high (-1 on bad
 * arguments). */
int rt_shard_height(int height, int nshards, int shard);

/* rt_render_batch_spp_device over every uploaded device: nframes poses of full
 * frames (row0 = 0, stride 1, nrows = height) into device buffers `out` on the
 * FIRST uploaded device, asynchronous on `stream` (a stream of that device).
 * With G > 1 devices the frames are sharded as rt_render_shard_device's, each device
 * renders its rows of every pose, and one RCCL gather per call brings the
 * shards to the first device, which de-interleaves them; hit_count[f] adds
 * all shards.  Results are identical to a one-device render.  (Test hooks:
 * RT_VIRTUAL_SHARDS=N shards a one-device scene into N row shards on that
 * device, gathered with device copies; RT_GROUP_RCCL=1 sends a one-device
 * scene through the RCCL gather with a one-rank communicator.) */
int rt_render_batch_multi(rt_scene *s, const rt_camera *cams, int nframes, int spp, int mode, const rt_device_out *out,
                          void *stream, uint32_t flags);

/* The de-interleave of rt_render_batch_multi on the host (the same index
 * arithmetic as the device kernel; for tests and host-side gathers):
 * `gathered` holds `shards` blocks of block_bytes; shard g's block holds at
 * section_offset its frames back to back, [frames][rows_g][width] elements
 * of elem_bytes, rows_g = rt_shard_height(height, shards, g) rows in the
 * layout of rt_render_shard_device; writes frames_out[frames][height][width]
 * elements. */
int rt_deinterleave_rows(const void *gathered, uint64_t block_bytes, uint64_t section_offset, int shards, int frames,
                         int height, int width, int elem_bytes, void *frames_out);

/* Asynchronous shard render into caller device buffers on a caller stream
 * (hipStream_t passed as void*; NULL = the null stream).  Used by the
 * multi-GPU driver (one process per GPU, RCCL gather of the shards).
 * flags: RT_FLAG_COUNT accumulates into the scene's per-device counters. */
int rt_render_rows_device(rt_scene *s, int device, const rt_camera *cam, int mode, int row0, int row_stride,
                          int nrows, const rt_device_out *out, void *stream, uint32_t flags);

/* A batch of nframes camera poses of one image geometry (all cams share
 * width/height), rendered as rt_render_rows_device would render each of them
 * in turn (the reference's runTest loop over its camera path, main.cpp:234-281,
 * with calculateScreen + shadeScreen per pose, main.cpp:253-262).  Frame f's
 * outputs start f * width * nrows pixels into every buffer of `out` (rgb and
 * pos: 3 values per pixel), and its hit counter is out->hit_count[f].  The
 * library launches up to 36 frames at a time (one persistent traversal launch
 * with the resolve fused in, one fix-up launch), so per-launch ramp-up, tail and
 * launch gaps are paid once per batch.  Results are identical to per-frame
 * calls. */
int rt_render_batch_device(rt_scene *s, int device, const rt_camera *cams, int nframes, int mode, int row0,
                           int row_stride, int nrows, const rt_device_out *out, void *stream, uint32_t flags);

/* rt_render_batch_device with spp samples per pixel (spp = n*n: 1, 4, 9 or
 * 16), stratified: sample s of a pixel is shot through sub-pixel offset
 * (((s % n) + 0.5) / n, ((s / n) + 0.5) / n) in place of the reference's
 * pixel centre (0.5, 0.5) (camera.hpp:35-37; SURVEY.md §8(d) config c4 uses
 * the 2x2 pattern).  Per-sample outputs (hit_id, dist, pos) of pose f, pixel
 * o, sample s are at (f * width * nrows + o) * spp + s; the colour (rgb) of
 * pixel o is shadeScreen's colour (main.cpp:356-377) summed over the samples
 * in order from 0.0, divided by spp, then cast as Benchmark::saveScreen does
 * (benchmark.hpp:105-114); hit_count[f] counts the samples that hit.  spp = 1
 * is rt_render_batch_device exactly. */
int rt_render_batch_spp_device(rt_scene *s, int device, const rt_camera *cams, int nframes, int spp, int mode,
                               int row0, int row_stride, int nrows, const rt_device_out *out, void *stream,
                               uint32_t flags);

/* Diffuse path tracing of one pose (BASELINE config
 * c5 "16 spp + 4-bounce secondary rays").  The reference has no secondary
 * rays: the path model is build-defined and every segment is
 * traced with the reference's closest-hit semantics (stack_bvh.hpp:611-644).
 * Per pixel (i, j) and sample s: hash-seeded sub-pixel offset (frame, pixel,
 * sample), 1 + bounces segments, cosine-weighted bounces, radiance
 * sum_k 0.5^k * shadeScreen colour of vertex k (light at the camera); the
 * pixel colour is the mean over samples cast as saveScreen does.
 * RT_FLAG_SHADOW: vertex k >= 1 adds its colour only if no triangle passes the
 * reference's Moller-Trumbore test on the segment from the light (the camera
 * position C) to the vertex p, at t < |p - C| (1 - 2^-12) along the unit
 * direction (p - C) / |p - C| — one occlusion ray per bounce vertex; the
 * primary vertex is the camera ray's own hit and casts none.  Outputs:
 * rgb per pixel; hit_id / dist / pos of the primary segment per sample at
 * (row * width + i) * spp + s; hit_count += samples whose primary ray hit.
 * Row shard as rt_render_rows_device; asynchronous on `stream`.  flags:
 * RT_FLAG_COUNT adds the ray segments traced to rt_frame_stats' rays,
 * RT_FLAG_TIMING times the kernel (trace_ms).  Pipeline (same results
 * either way): with RT_FLAG_SHADOW the queued tracer (every path of the pose
 * in HBM queues, one kernel per bounce segment, 256 B of workspace per
 * path), without it the megakernel; the environment variable RT_PATHS=queue
 * or RT_PATHS=mega (read per call) overrides, and RT_SHADOW_RAYS=lane|rec|bin
 * picks how the queued tracer walks its occlusion rays. */
int rt_render_paths_device(rt_scene *s, int device, const rt_camera *cam, int frame, int spp, int bounces, int row0,
                           int row_stride, int nrows, const rt_device_out *out, void *stream, uint32_t flags);

/* Read (and optionally reset) the per-device counters filled by
 * RT_FLAG_COUNT renders (synchronises the device). */
int rt_frame_stats(rt_scene *s, int device, int reset, rt_frame_stats_t *out);

int rt_scene_stats(const rt_scene *s, rt_scene_stats_t *out);

/* Diagnostics: copy up to n (<= 16) words of the device's raw counter block
 * (the rt_frame_stats counters).  Waits for the scene's launches on it. */
int rt_diag_raw(rt_scene *s, int device, uint64_t *out, size_t n);

/* Reference visit order rank of every triangle (loader index -> rank) and
 * the real tree in reference visit order, for tree-parity tests:
 * boxes[6*nodes], meta[3*nodes] = (begin, end, nchildren), order[n_tris]
 * (the BVH's owned primitive vector as loader indices). */
int rt_scene_tree_dump(const rt_scene *s, double *boxes, int64_t *meta, int64_t *order);

void rt_scene_destroy(rt_scene *s);

const char *rt_last_error(void);
int rt_abi_version(void);
/* device name of ordinal `device` (for reports); "" when unavailable */
const char *rt_device_name(int device);
/* Diagnostics: opens RCCL as the first multi-device render does — the copy
 * the process has mapped already (PyTorch's), else ROCm's, never a second
 * one — and returns the path of the mapped file (NULL: none, see
 * rt_last_error). */
const char *rt_rccl_path(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
