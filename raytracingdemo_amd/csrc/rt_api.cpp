// extern "C" surface of librtmi355x.so (include/rt.h).  Host C++ around the
// gfx950 kernels in render.hip: scene ownership, device replicas, the frame
// call that replaces calculateScreen + shadeScreen (src/main.cpp:253-262).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <exception>
#include <mutex>
#include <system_error>
#include <thread>
#include <string>
#include <array>
#include <vector>

#include "rt_internal.h"

namespace rt {
hipError_t launch_trace(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, int mode, bool count,
                        hipStream_t s, uint32_t literal_stack, const hipEvent_t* ev, bool fresh, bool* fresh_after);
int exact_blocks_per_cu(int width, uint32_t stack_bound);
int packet_blocks_per_cu(int width);
hipError_t launch_paths(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, uint32_t frame,
                        int bounces, bool shadow, hipStream_t s, const hipEvent_t* ev);
hipError_t launch_paths_q(const RtDevScene& sc, const RtFrameParams& fp, const RtLaunchAux& aux, const PathQs& qs,
                          uint32_t frame, int bounces, bool shadow, hipStream_t s, const hipEvent_t* ev);
int packet_candidates();
int packet_threads();
bool packet_takes_job(const RtDevScene& sc, const RtFrameParams& fp, int mode, bool count);
bool packet_split(int spp, bool pack);
uint32_t params_bytes();
int exact_lds_stack();
hipError_t launch_deinterleave(const void* gather, uint64_t block, uint64_t sec_off, int G, int F, int H, int W,
                               int eb, void* dst, hipStream_t s);
hipError_t launch_sum_counts(const void* gather, uint64_t block, uint64_t cnt_off, int G, int F,
                             unsigned long long* out, bool store, hipStream_t s);
hipError_t launch_job(const RtLaunchAux& a, hipStream_t s);
hipError_t launch_gate(hipStream_t s);
}

namespace {

thread_local std::string g_err;

int fail(int status, const std::string& msg) {
    g_err = msg;
    return status;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) throw rt::Error{RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
    } while (0)

struct DevGuard {  // restores the caller's current device
    int prev = -1;
    explicit DevGuard(int dev) {
        hipGetDevice(&prev);
        if (prev != dev) HIP_TRY(hipSetDevice(dev));
    }
    ~DevGuard() {
        int now = -1;
        hipGetDevice(&now);
        if (prev >= 0 && now != prev) hipSetDevice(prev);
    }
};

template <class T>
size_t align_up(size_t x) {
    return (x + 255) & ~size_t(255);
}

// d_counters: RT_FLAG_COUNT counters (rt_frame_stats)
constexpr size_t kCounterWords = 32;  // 18-23: RT_PROFILE builds (packet_kernel.h); 24-29: occlusion rays; 30-31: per-lane walks, wave-distinct fetches
#if defined(RT_PROFILE) && RT_PROFILE
constexpr bool RT_PROFILE_BUILD = true;  // every timed launch writes the counters
#else
constexpr bool RT_PROFILE_BUILD = false;
#endif
// Candidate overflow pool: chunks of RT_POOL_CHUNK entries, one per lane whose
// LDS list overflows in a launch (a dry pool falls back to the certified
// dropped bound, so the size trades memory against fix-up work only).
constexpr uint32_t kPoolChunks = 1u << 17;  // 24 MiB

// One set of the device state a batch launch works in: the work-queue block
// (tile queues, hit-count slots, redo count), the fix-up's redo list, the
// candidate overflow pool and the per-lane kernels' stack spill.  A replica
// holds kSlots of them and its launches take them in turn, so a launch waits
// only for the earlier launch that used the same slot: launches the caller
// issues on different streams run concurrently (the next launch's waves fill
// the CUs the last one's tail leaves idle), launches on one
// stream stay in order.
constexpr int kSlots = 2;
struct Slot {
    uint32_t* d_tiles = nullptr;
    uint64_t* d_spill = nullptr;
    uint32_t* d_redo = nullptr;  // packet pipeline -> fix-up kernel pixel list
    uint64_t redo_cap = 0;
    uint32_t* h_seen = nullptr;  // host-mapped: the redo count k_fixup saw in the slot's last launch
    uint64_t* d_pool = nullptr;  // candidate overflow pool (pool_chunks x RT_POOL_CHUNK entries)
    hipStream_t last = nullptr;  // the stream of the slot's last launch
    bool used = false;
    bool fresh = true;  // work-queue block known to be zero (packet pipeline self-resets it)
    hipEvent_t ev = nullptr;
};

// Host-mapped words for k_fixup's redo counts (Slot::h_seen): one pinned
// page for the process, handed out and taken back, never freed — a scene
// destroyed at interpreter shutdown returns its words without a HIP call.
std::mutex g_seen_mu;
uint32_t* g_seen_page = nullptr;
auto& g_seen_free = *new std::vector<uint32_t*>();  // (never destroyed: no static-destructor order at exit)
uint32_t* seen_word_alloc() {
    std::lock_guard<std::mutex> lk(g_seen_mu);
    if (g_seen_free.empty()) {
        constexpr size_t kWords = 4096 / sizeof(uint32_t);
        void* p = nullptr;
        HIP_TRY(hipHostMalloc(&p, kWords * sizeof(uint32_t), hipHostMallocMapped));
        g_seen_page = static_cast<uint32_t*>(p);
        for (size_t k = 0; k < kWords; k += 16) g_seen_free.push_back(g_seen_page + k);  // one 64-B line each
    }
    uint32_t* w = g_seen_free.back();
    g_seen_free.pop_back();
    __atomic_store_n(w, 0u, __ATOMIC_RELAXED);
    return w;
}
void seen_word_free(uint32_t* w) {
    std::lock_guard<std::mutex> lk(g_seen_mu);
    g_seen_free.push_back(w);
}

struct Replica {
    int device = -1;
    void* blob = nullptr;       // one allocation for the whole scene
    size_t blob_bytes = 0;
    RtDevScene dev{};

    unsigned long long* d_counters = nullptr;  // RT_FLAG_COUNT counters
    // staging for the host-output frame call
    void* frame = nullptr;
    size_t frame_bytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // persistent-kernel resources, per launch slot (above)
    Slot slot[kSlots];
    int next_slot = 0;
    uint32_t spill_cap = 0;
    // stack spill words per slot: the per-lane kernels' (grid * 256 lanes x
    // spill_cap) or the packet kernel's exit path (pgrid * 256 lanes x the
    // stack bound past its LDS ring), whichever is larger
    size_t spill_words = 0;
    int grid = 0;                // per-lane kernels: 256-thread workgroups
    int pgrid = 0;               // packet kernel: 64 * kPacketWaves-thread workgroups
    int cus = 0;                 // compute units of the device
    uint32_t pool_chunks = 0;
    void* d_cand = nullptr;      // spp > 1 / wavefront paths: candidate lists in HBM
    uint64_t cand_cap = 0;       // pixels
    void* d_pq = nullptr;        // queued path tracer workspace (PathQs), pq_cap paths
    uint64_t pq_cap = 0;
    // RT_FLAG_TIMING: events around the traversal kernel per timed launch,
    // read and recycled by rt_frame_stats
    std::vector<std::array<hipEvent_t, 2>> tev;
    size_t tev_used = 0;
    hipEvent_t ev_out = nullptr;
    // side de-interleave jobs run by the traversal kernel itself / as their own kernel
    uint64_t jobs_fused = 0, jobs_kernel = 0;
};

}  // namespace

// Multi-device frames (rt_render_batch_multi): per shard a staging block on
// its device, the gathered blocks on the first device, and the RCCL
// communicator over the uploaded devices (one rank per device, this process).
struct Group {
    std::vector<void*> stage;      // shard g's block (on its shard's device)
    std::vector<int> stage_dev;
    uint64_t block = 0;            // bytes per block (grown, never shrunk)
    void* gather = nullptr;        // [G][block] on the first device
    uint64_t gather_bytes = 0;
    std::vector<ncclComm_t> comms; // comms[g]: rank g = reps[g] (distinct devices only)
    hipEvent_t ev_in = nullptr, ev_out = nullptr, ev0 = nullptr, ev1 = nullptr;  // on the first device
    std::vector<hipEvent_t> ev_shard;  // per shard: its render is done (copy transport)
};

struct rt_scene {
    rt::Soup soup;
    rt::Tree tree;
    rt::Flat flat;
    std::vector<std::unique_ptr<Replica>> reps;  // stable addresses: a replica outlives the lock
    std::mutex mu;
    uint32_t literal_stack = 0;  // stack bound of the literal (reference-order) traversal
    Group grp;
    rt_build_times_t times{};    // rt_scene_build_times
};

namespace {

// RCCL, opened on the first multi-device render (dlopen, so single-device
// users never initialise it).  One copy per process: the one already mapped
// (PyTorch's: torch/lib/librccl.so, soname librccl.so.1 — the Python binding
// imports torch before a multi-device upload when torch is installed), else
// ROCm's, opened RTLD_LOCAL.  Never RTLD_GLOBAL: an RCCL mapped globally ahead
// of torch interposes its symbols on torch's libraries, and objects shared
// that way were destroyed twice at exit ("double free or corruption", round
// 4; tests/test_host.py pins both import orders).
struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) throw rt::Error{RT_ERR_RUNTIME, std::string("RCCL not found: ") + dlerror()};
        x.init_all = (decltype(x.init_all))dlsym(h, "ncclCommInitAll");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.gather = (decltype(x.gather))dlsym(h, "ncclGather");
        x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        if (!x.init_all || !x.destroy || !x.gather || !x.group_start || !x.group_end || !x.error_string)
            throw rt::Error{RT_ERR_RUNTIME, "RCCL lacks ncclCommInitAll / ncclGather / group calls"};
        return x;
    }();
    return r;
}
#define NCCL_TRY(expr)                                                                               \
    do {                                                                                             \
        ncclResult_t e_ = (expr);                                                                    \
        if (e_ != ncclSuccess) throw rt::Error{RT_ERR_HIP, std::string(#expr) + ": " + rccl().error_string(e_)}; \
    } while (0)

void free_group(rt_scene* s) {
    Group& g = s->grp;
    int prev = -1;
    hipGetDevice(&prev);
    for (size_t k = 0; k < g.stage.size(); k++)
        if (g.stage[k]) {
            hipSetDevice(g.stage_dev[k]);
            hipFree(g.stage[k]);
        }
    g.stage.clear();
    g.stage_dev.clear();
    g.block = 0;
    if (!s->reps.empty()) hipSetDevice(s->reps.front()->device);
    if (g.gather) hipFree(g.gather);
    g.gather = nullptr;
    g.gather_bytes = 0;
    for (hipEvent_t e : {g.ev_in, g.ev_out, g.ev0, g.ev1})
        if (e) hipEventDestroy(e);
    g.ev_in = g.ev_out = g.ev0 = g.ev1 = nullptr;
    for (hipEvent_t e : g.ev_shard)
        if (e) hipEventDestroy(e);
    g.ev_shard.clear();
    for (ncclComm_t c : g.comms) rccl().destroy(c);
    g.comms.clear();
    if (prev >= 0) hipSetDevice(prev);
}

void free_replica(Replica& r) {
    if (r.device < 0) return;
    int prev = -1;
    hipGetDevice(&prev);
    hipSetDevice(r.device);
    if (r.blob) hipFree(r.blob);
    if (r.d_counters) hipFree(r.d_counters);
    if (r.frame) hipFree(r.frame);
    for (Slot& q : r.slot) {
        if (q.d_tiles) hipFree(q.d_tiles);
        if (q.d_spill) hipFree(q.d_spill);
        if (q.d_redo) hipFree(q.d_redo);
        if (q.h_seen) seen_word_free(q.h_seen);
        if (q.d_pool) hipFree(q.d_pool);
        if (q.ev) hipEventDestroy(q.ev);
    }
    if (r.d_cand) hipFree(r.d_cand);
    if (r.d_pq) hipFree(r.d_pq);
    for (auto& a : r.tev)
        for (hipEvent_t e : a) hipEventDestroy(e);
    if (r.ev_out) hipEventDestroy(r.ev_out);
    if (r.ev0) hipEventDestroy(r.ev0);
    if (r.ev1) hipEventDestroy(r.ev1);
    if (r.stream) hipStreamDestroy(r.stream);
    if (prev >= 0) hipSetDevice(prev);
    r = Replica{};
}

Replica& replica_for(rt_scene* s, int device) {
    for (auto& r : s->reps)
        if (r->device == device) return *r;
    throw rt::Error{RT_ERR_NO_DEVICE, "scene not uploaded to device " + std::to_string(device)};
}

// The launch state of one slot (work-queue block, stack spill, candidate
// pool, redo-count word; the redo list is sized per launch by ensure_redo).
void alloc_slot(Replica& r, Slot& q) {
    if (q.d_tiles) return;
    HIP_TRY(hipMalloc(&q.d_tiles, RT_QUEUE_WORDS * sizeof(uint32_t)));
    HIP_TRY(hipMemset(q.d_tiles, 0, RT_QUEUE_WORDS * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&q.d_spill, r.spill_words * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&q.d_pool, (size_t)r.pool_chunks * RT_POOL_CHUNK * sizeof(uint64_t)));
    HIP_TRY(hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
    q.h_seen = seen_word_alloc();
}

void upload_one(rt_scene* s, int device) {
    DevGuard g(device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw rt::Error{RT_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950"};
    if (rt::params_bytes() != sizeof(RtFrameParams))  // host and device built with one RT_MAX_BATCH
        throw rt::Error{RT_ERR_RUNTIME, "library built inconsistently (RtFrameParams layout differs)"};
    const rt::Flat& f = s->flat;
    auto rp = std::make_unique<Replica>();
    Replica& r = *rp;
    r.device = device;
    // carve one allocation (256-B aligned sections)
    struct Sec { const void* src; size_t bytes; size_t off; };
    // W = 8: the per-lane walk's quantised node copy (walk_tree.cpp)
    const std::vector<uint8_t> qn = f.width == 8 ? rt::quantize_wide8(f.wide.data(), f.n_wide) : std::vector<uint8_t>{};
    std::vector<Sec> secs = {
        {f.wide.data(), f.wide.size(), 0},
        {f.tri32.data(), f.tri32.size() * sizeof(float), 0},
        {f.tri64.data(), f.tri64.size() * sizeof(double), 0},
        {f.tri_id.data(), f.tri_id.size() * sizeof(uint32_t), 0},
        {f.tri_rank.data(), f.tri_rank.size() * sizeof(uint32_t), 0},
        {f.tri_leaf.data(), f.tri_leaf.size() * sizeof(uint32_t), 0},
        {f.rbox.data(), f.rbox.size() * sizeof(double), 0},
        {f.rparent.data(), f.rparent.size() * sizeof(int32_t), 0},
        {s->soup.normal.data(), s->soup.normal.size() * sizeof(double), 0},
        {f.rkid_off.data(), f.rkid_off.size() * sizeof(uint32_t), 0},
        {f.rkid.data(), f.rkid.size() * sizeof(uint32_t), 0},
        {f.rrange.data(), f.rrange.size() * sizeof(uint32_t), 0},
        {f.ref2walk.data(), f.ref2walk.size() * sizeof(uint32_t), 0},
        {qn.data(), qn.size(), 0},
    };
    size_t off = 0;
    for (auto& sc : secs) {
        sc.off = off;
        off += align_up<char>(std::max<size_t>(sc.bytes, 1));
    }
    r.blob_bytes = off;
    HIP_TRY(hipMalloc(&r.blob, off));
    for (auto& sc : secs)  // straight from the flat arrays: no host staging copy
        if (sc.bytes) HIP_TRY(hipMemcpy(static_cast<uint8_t*>(r.blob) + sc.off, sc.src, sc.bytes, hipMemcpyHostToDevice));
    auto at = [&](int k) { return static_cast<uint8_t*>(r.blob) + secs[k].off; };
    RtDevScene& d = r.dev;
    d.nodes = at(0);
    d.tri32 = reinterpret_cast<const float*>(at(1));
    d.tri64 = reinterpret_cast<const double*>(at(2));
    d.tri_id = reinterpret_cast<const uint32_t*>(at(3));
    d.tri_rank = reinterpret_cast<const uint32_t*>(at(4));
    d.tri_leaf = reinterpret_cast<const uint32_t*>(at(5));
    d.rbox = reinterpret_cast<const double*>(at(6));
    d.rparent = reinterpret_cast<const int32_t*>(at(7));
    d.normal = reinterpret_cast<const double*>(at(8));
    d.rkid_off = reinterpret_cast<const uint32_t*>(at(9));
    d.rkid = reinterpret_cast<const uint32_t*>(at(10));
    d.rrange = reinterpret_cast<const uint32_t*>(at(11));
    d.ref2walk = reinterpret_cast<const uint32_t*>(at(12));
    d.qnodes = qn.empty() ? nullptr : at(13);
    d.root_ref = f.root_ref;
    d.root_meta = f.root_meta;
    std::memcpy(d.root_box, f.root_box, sizeof d.root_box);
    d.n_tris = (uint32_t)s->soup.n;
    d.node_bytes = rt_node_bytes(f.width);
    d.width = f.width;
    d.stack_bound = f.stack_bound;
    d.coord_max = f.coord_max;
    d.n_wide = (uint32_t)f.n_wide;
    HIP_TRY(hipMalloc(&r.d_counters, kCounterWords * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(r.d_counters, 0, kCounterWords * sizeof(unsigned long long)));
    HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&r.ev0));
    HIP_TRY(hipEventCreate(&r.ev1));
    HIP_TRY(hipEventCreateWithFlags(&r.ev_out, hipEventDisableTiming));
    int bpc = rt::exact_blocks_per_cu(f.width, f.stack_bound);
    if (const char* e = std::getenv("RT_BLOCKS_PER_CU")) {  // diagnostic: lower the persistent grid
        const int v = std::atoi(e);
        if (v >= 1 && v < bpc) bpc = v;
    }
    r.grid = prop.multiProcessorCount * bpc;
    int pbpc = rt::packet_blocks_per_cu(f.width);
    if (const char* e = std::getenv("RT_PACKET_BLOCKS_PER_CU")) {  // diagnostic: leave block slots free per CU
        const int v = std::atoi(e);
        if (v >= 1 && v < pbpc) pbpc = v;
    }
    r.pgrid = prop.multiProcessorCount * pbpc;
    r.cus = prop.multiProcessorCount;
    const int S = rt::exact_lds_stack();
    r.spill_cap = f.stack_bound > (uint32_t)S ? f.stack_bound - (uint32_t)S : 1u;
    const uint32_t K = (uint32_t)rt::packet_candidates();  // packet_exit's LDS ring (render.hip)
    // (packet_redo spills at lane blockIdx * packet_threads + threadIdx of a
    // grid of pgrid * packet_threads lanes)
    r.spill_words = std::max((size_t)r.grid * 256 * r.spill_cap,
                             (size_t)r.pgrid * (size_t)rt::packet_threads() * (f.stack_bound > K ? f.stack_bound - K : 1u));
    r.pool_chunks = kPoolChunks;
    if (const char* e = std::getenv("RT_POOL_CHUNKS")) {  // test hook: a small pool runs dry
        const long v = std::atol(e);
        if (v >= 1 && v <= (long)kPoolChunks) r.pool_chunks = (uint32_t)v;
    }
    alloc_slot(r, r.slot[0]);  // (the second slot on the first launch from another stream: take_slot)
    s->reps.push_back(std::move(rp));
}

// Waits for every launch issued on a slot so far (before its buffers are
// replaced): only the slot's last stream, not the whole device.
void quiesce_slot(Slot& q) {
    if (!q.used) return;
    HIP_TRY(hipEventRecord(q.ev, q.last));
    HIP_TRY(hipEventSynchronize(q.ev));
}
// ... and on every slot of the replica.
void quiesce(Replica& r) {
    for (Slot& q : r.slot) quiesce_slot(q);
}

// Redo list: one entry per pose pixel of a launch (4 B each: 298 MB for
// the 36-pose 1080p orbit), so no launch can overflow it and the fused packet
// kernel finishes the list itself (aux.self_fix, packet_exit) instead of a
// trailing k_fixup that would start only after the next launch's
// persistent grid.  On the sponza proxy ~0 pixels are redone.
// If that allocation fails the list is a fixed pool of kRedoEntries and
// k_fixup runs after every launch: a launch whose redo count passes the pool
// is retried whole there; k_fixup reports each launch's count to a
// host-mapped word of the slot, and a slot that overflowed gets a longer list
// (twice the count, up to kRedoGrow entries) and, while its launches still
// overflow, the full fix-up grid for the retry.  RT_REDO_CAP (read per call;
// a test hook) lowers the entries a launch may use, which forces the k_fixup
// path.  Entries are kRedoEmpty between launches (packet_kernel.h).
constexpr uint64_t kRedoEntries = 1u << 20;  // 4 MiB
constexpr uint64_t kRedoGrow = 1u << 26;     // 256 MiB
uint64_t redo_limit() {
    const char* e = std::getenv("RT_REDO_CAP");
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (uint64_t)v : UINT64_MAX;
}

// Redo list of a slot for a launch of `pixels` pose pixels (grown, never
// shrunk): every pixel, or past a failed allocation at most `most`.
void ensure_redo(Slot& q, uint64_t pixels, uint64_t most = kRedoEntries) {
    pixels = std::max<uint64_t>(pixels, 1);
    if (q.redo_cap >= pixels) return;
    quiesce_slot(q);
    const uint64_t had = q.redo_cap;
    if (q.d_redo) HIP_TRY(hipFree(q.d_redo));
    q.d_redo = nullptr;
    q.redo_cap = 0;
    uint64_t n = pixels;
    if (hipMalloc(&q.d_redo, n * sizeof(uint32_t)) != hipSuccess) {
        (void)hipGetLastError();
        n = std::min<uint64_t>(pixels, std::max<uint64_t>(most, had));
        HIP_TRY(hipMalloc(&q.d_redo, n * sizeof(uint32_t)));
    }
    HIP_TRY(hipMemset(q.d_redo, 0xFF, n * sizeof(uint32_t)));  // kRedoEmpty
    q.redo_cap = n;
}

// Candidate lists in HBM for `pixels` sample pixels (spp > 1 resolve, the
// wavefront path tracer; grown, never shrunk):
// [K][pixels] entries | [pixels] f32 drop bounds | [pixels] u32 chunks | [pixels] counts
constexpr uint64_t kCandBytesPerPixel = 8 * RT_CAND_LDS + 4 + 4 + 1;
void ensure_cand(Replica& r, uint64_t pixels) {
    if (r.cand_cap >= pixels) return;
    quiesce(r);
    if (r.d_cand) HIP_TRY(hipFree(r.d_cand));
    r.d_cand = nullptr;
    r.cand_cap = 0;
    HIP_TRY(hipMalloc(&r.d_cand, pixels * kCandBytesPerPixel));
    r.cand_cap = pixels;
}

// Queued path-tracer workspace for P paths (grown, never shrunk): two
// segment queues (80 B per entry), the final radiance (24 B per path), two
// fall-back lists (4 B per path each) and the control words.
// (+ the occlusion records, 32 B twice)
constexpr uint64_t kPqBytesPerPath = 2 * 80 + 24 + 2 * 4 + 2 * 32;
PathQs ensure_pq(Replica& r, uint64_t P) {
    if (r.pq_cap < P) {
        quiesce(r);  // earlier launches may still use it
        if (r.d_pq) HIP_TRY(hipFree(r.d_pq));
        r.d_pq = nullptr;
        r.pq_cap = 0;
        HIP_TRY(hipMalloc(&r.d_pq, P * kPqBytesPerPath + RT_QC_WORDS(64) * sizeof(uint32_t) +
                                       (uint64_t)RT_SH_HBINS * RT_SH_BLOCKS * sizeof(uint32_t) + 2048));
        r.pq_cap = P;
    }
    uint8_t* base = static_cast<uint8_t*>(r.d_pq);
    const uint64_t c = r.pq_cap;
    PathQs qs{};
    qs.q[0] = reinterpret_cast<double*>(base);
    qs.q[1] = reinterpret_cast<double*>(base + c * 80);
    qs.Lfin = reinterpret_cast<double*>(base + c * 160);
    qs.fb = reinterpret_cast<uint32_t*>(base + c * 184);
    // (and behind the records, 32 B per path: two arrays of sort pairs and
    // the keys, rt_device.h rt_q_spair / rt_q_skey)
    qs.srec = reinterpret_cast<double*>(base + align_up<char>(c * 192));
    const uint64_t o_ctl = align_up<char>(align_up<char>(c * 192) + c * 64);
    qs.ctl = reinterpret_cast<uint32_t*>(base + o_ctl);
    const uint64_t o_bh = align_up<char>(o_ctl + RT_QC_WORDS(64) * sizeof(uint32_t));
    qs.bhist = reinterpret_cast<uint32_t*>(base + o_bh);
    qs.sh_blocks = RT_SH_BLOCKS;
    qs.cap = (uint32_t)c;
    return qs;
}

// Path pipeline (RT_PATHS, read per call: tests switch it in-process):
// "queue" — the queued tracer (queue_paths.h: compacted segment queues, lean
// per-segment kernels); "mega" — the megakernel (path_kernel.h k_paths).
// Unset: the faster of the two — the queued tracer with occlusion rays
// (config c5: 201 vs 250 ms per pose), and without them wherever its primary
// segments go through the packet kernel (an 8-wide tree, spp 4 or 16: c5
// 143.9 vs 157.0 ms), else the megakernel.  (The round-2
// wavefront tracer, 1.45x slower than either, was removed in round 5.)
enum class PathPipe { mega, queue };
bool path_pipe_forced() {
    const char* e = std::getenv("RT_PATHS");
    return e && (e[0] == 'q' || e[0] == 'm');
}
PathPipe path_pipe(bool shadow, int width, int spp) {
    const char* e = std::getenv("RT_PATHS");
    if (e && e[0] == 'q') return PathPipe::queue;
    if (e && e[0] == 'm') return PathPipe::mega;
    return shadow || (width == 8 && (spp == 4 || spp == 16)) ? PathPipe::queue : PathPipe::mega;
}

void check_camera(const rt_scene* s, const rt_camera* c) {
    if (!c) throw rt::Error{RT_ERR_INVALID_ARGUMENT, "camera is NULL"};
    if (c->width <= 0 || c->height <= 0 || c->width > 65536 || c->height > 65536 ||
        (int64_t)c->width * c->height >= (int64_t(1) << 31))
        throw rt::Error{RT_ERR_INVALID_ARGUMENT, "bad image size"};
    for (int a = 0; a < 3; a++)
        if (!std::isfinite(c->pos[a]) || !std::isfinite(c->dir[a]))
            throw rt::Error{RT_ERR_INVALID_ARGUMENT, "camera position/direction must be finite"};
    (void)s;
}

// World-space margin added to every fp32 slab plane: 2^-19 * (|o|_max +
// |coordinate|_max) dominates the fp32 rounding of the origin, the reciprocal
// and the fma (each <= 2^-24 relative) by >= 8x (DESIGN.md "exactness").
// n of an n x n stratified pattern (spp = n * n, checked by the caller)
int spp_grid(int spp) {
    int g = 1;
    while ((g + 1) * (g + 1) <= spp) g++;
    return g;
}

float frame_pad(const rt_scene* s, const rt_camera* c) {
    double om = std::max({std::fabs(c->pos[0]), std::fabs(c->pos[1]), std::fabs(c->pos[2])});
    double p = std::ldexp(om + s->flat.coord_max + 1e-30, -19);
    float f = (float)p;
    if ((double)f < p) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

// Launch parameters for poses c[0..n-1] (n * spp <= RT_MAX_BATCH) of one
// image geometry: per-pose camera basis (main.cpp:325-329) and slab margin,
// and per sample frame its stratified sub-pixel offset: sample s of an
// n x n pattern sits at ((s % n) + 0.5) / n, ((s / n) + 0.5) / n (spp = 1:
// the reference's pixel centre 0.5, camera.hpp:35-37).
// The fused packet walk takes a pixel's samples in one wave when they divide
// it (spp 4, 16) and the walk tree is 8 wide; RT_SPP_PACK=0 keeps one sample
// frame per tile (packet_kernel.h).
bool pack_samples(const rt_scene* s, int spp) {
    const char* pk = std::getenv("RT_SPP_PACK");
    return spp > 1 && 64 % spp == 0 && s->flat.width == 8 && !(pk && pk[0] == '0');
}

RtFrameParams frame_params(const rt_scene* s, const rt_camera* c, int n, int row0, int row_stride, int nrows,
                           int spp = 1, int band = 1) {
    RtFrameParams fp{};
    fp.band = band;
    fp.nframes = n * spp;
    fp.spp = spp;
    // sample q of each pose sits at ((q % g) + 0.5) / g, ((q / g) + 0.5) / g
    // (computed in-kernel by frame_cam with these same expressions)
    fp.spp_n = spp_grid(spp);
    fp.pack = pack_samples(s, spp);
    for (int p = 0; p < n; p++) {
        RtPose k{};
        k.pad = frame_pad(s, &c[p]);
        for (int a = 0; a < 3; a++) {
            k.pos[a] = c[p].pos[a];
            k.dir[a] = c[p].dir[a];
        }
        rt::camera_basis(c[p].dir, k.right, k.up);
        fp.pose[p] = k;
    }
    rt::pixel_constants(c->width, c->height, fp.cam_iw, fp.cam_ih, fp.cam_half, fp.cam_aspect);
    fp.W = c->width;
    fp.H = c->height;
    fp.row0 = row0;
    fp.row_stride = row_stride;
    fp.nrows = nrows;
    return fp;
}

// Sample frames per launch of a batch: 18 (36-frame orbits in two launches:
// 13.3 vs 13.1 Grays/s with 12), or RT_BATCH (1..RT_MAX_BATCH) for A/B runs.
int batch_frames() {
    static const int b = [] {
        const char* e = std::getenv("RT_BATCH");
        const int v = e ? std::atoi(e) : RT_MAX_BATCH;
        return v >= 1 && v <= RT_MAX_BATCH ? v : RT_MAX_BATCH;
    }();
    return b;
}

// The next launch slot of the replica for a launch on stream st, ordered
// after the slot's earlier launches (a wait only when they were issued on
// another stream).  shared: the launch also uses the replica-wide buffers
// (HBM candidate lists, the wavefront workspace, the counting pass's
// counters), so it follows the launches of every slot.
Slot& take_slot(Replica& r, hipStream_t st, bool shared) {
    // one caller stream: slot 0 only (launches on one stream are ordered
    // anyway); the second slot is allocated when a launch comes from another
    // stream than slot 0's last one
    if (!r.slot[1].d_tiles) {
        if (!r.slot[0].used || r.slot[0].last == st) r.next_slot = 0;
        else alloc_slot(r, r.slot[1]);
    }
    Slot& q = r.slot[r.next_slot];
    r.next_slot = (r.next_slot + 1) % kSlots;
    auto follow = [&](Slot& o) {
        if (o.used && o.last != st) {
            HIP_TRY(hipEventRecord(o.ev, o.last));
            HIP_TRY(hipStreamWaitEvent(st, o.ev, 0));
        }
    };
    if (shared) {
        for (Slot& o : r.slot) follow(o);
    } else {
        follow(q);
    }
    q.last = st;
    q.used = true;
    return q;
}

// Runs the pipeline and tracks whether its work-queue block is left zeroed.
// store: RT_FLAG_COUNTS_STORE (the launch sets its poses' hit counts).
void launch(const rt_scene* s, Replica& r, Slot& q, const RtFrameParams& fp, int mode, bool count, hipStream_t st,
            const hipEvent_t* tev, const rt_deinterleave_job* job = nullptr, bool side_slot = false,
            bool store = false);

// A side de-interleave job (include/rt.h) in the launch's aux block.
void set_job(RtLaunchAux& a, const rt_deinterleave_job* j) {
    if (!j || j->frames <= 0) return;
    a.job_src = static_cast<const uint8_t*>(j->gathered);
    a.job_dst = static_cast<uint8_t*>(j->frames_out);
    a.job_block = j->block_bytes;
    a.job_sec = j->section_offset;
    a.job_G = j->shards;
    a.job_F = j->frames;
    a.job_H = j->height;
    a.job_W = j->width;
    a.job_eb = j->elem_bytes;
    a.job_rows = j->frame_rows;
}

RtLaunchAux aux_of(Replica& r, const Slot& q) {
    RtLaunchAux a{};
    a.tile_ctr = q.d_tiles;
    a.spill = q.d_spill;
    a.spill_cap = r.spill_cap;
    a.grid = r.grid;
    a.pgrid = r.pgrid;
    a.redo = q.d_redo;
    a.redo_cap = std::min<uint64_t>(q.redo_cap, redo_limit());
    a.pool = q.d_pool;
    a.pool_chunks = r.pool_chunks;
    a.cand = static_cast<uint64_t*>(r.d_cand);
    if (r.d_cand) {
        uint8_t* base = static_cast<uint8_t*>(r.d_cand);
        const uint64_t k = (uint64_t)rt::packet_candidates();
        a.cand_drop = reinterpret_cast<float*>(base + r.cand_cap * 8 * k);
        a.cand_ovf = reinterpret_cast<uint32_t*>(base + r.cand_cap * (8 * k + 4));
        a.cand_cnt = base + r.cand_cap * (8 * k + 8);
    }
    a.cand_cap = r.cand_cap;
    return a;
}

uint32_t literal_stack_bound(const rt_scene* s) {
    // literal traversal pushes every child of a visited node
    uint32_t best = 1;
    struct It { int32_t n; uint32_t sb; };
    std::vector<It> st{{0, 1}};
    while (!st.empty()) {
        It it = st.back();
        st.pop_back();
        const auto& n = s->tree.nodes[it.n];
        best = std::max(best, it.sb);
        for (int32_t k : n.kids) st.push_back({k, it.sb + (uint32_t)n.kids.size() - 1});
    }
    return best + 1;
}

void launch(const rt_scene* s, Replica& r, Slot& q, const RtFrameParams& fp, int mode, bool count, hipStream_t st,
            const hipEvent_t* tev, const rt_deinterleave_job* job, bool side_slot, bool store) {
    bool fresh_after = false;
    // a slot whose last launch overflowed its redo list (the count k_fixup
    // reported, possibly from a launch still running: a sizing hint only)
    const uint32_t seen = __atomic_load_n(q.h_seen, __ATOMIC_RELAXED);
    if (seen & RT_SEEN_ERROR) {
        // a wave of an earlier launch on the slot gave a redo entry up
        // (packet_kernel.h packet_redo): its pixel was not finished
        __atomic_store_n(q.h_seen, 0u, __ATOMIC_RELAXED);
        throw rt::Error{RT_ERR_RUNTIME, "redo list invariant broken: an earlier launch left a pixel unfinished"};
    }
    const uint64_t lpix = (uint64_t)fp.W * (uint64_t)fp.nrows * (uint64_t)(fp.nframes / std::max(fp.spp, 1));
    if (seen > q.redo_cap && q.redo_cap < std::min(lpix, kRedoGrow))
        ensure_redo(q, std::min<uint64_t>(2ull * seen, lpix), kRedoGrow);
    RtLaunchAux a = aux_of(r, q);
    a.redo_seen = q.h_seen;
    if (seen > a.redo_cap) a.fgrid = r.grid;
    // the packet kernel may end the launch itself: no retry is possible
    a.self_fix = (a.redo_cap >= lpix ? RT_SELF_FIX : 0) | (store ? RT_SELF_STORE : 0);
    // RT_FLAG_SIDE_SLOT: one workgroup slot per CU left to other streams
    if (side_slot && r.pgrid > r.cus) a.pgrid = r.pgrid - r.cus;
    set_job(a, job);
    // The overlap gate: when the replica's other slot last launched on
    // another stream, its persistent grid may still hold every CU; a gate
    // kernel on this stream first lets this launch's grid start only in that
    // grid's tail (render.hip k_gate).  RT_OVERLAP_GATE=0
    // (read per call) turns it off.
    {
        const Slot& other = &q == &r.slot[0] ? r.slot[1] : r.slot[0];
        const char* g = std::getenv("RT_OVERLAP_GATE");
        if (other.used && other.last != st && !(g && g[0] == '0')) HIP_TRY(rt::launch_gate(st));
    }
    if (a.job_src) {
        const bool empty = fp.W <= 0 || fp.nrows <= 0 || fp.nframes <= 0;
        (!empty && rt::packet_takes_job(r.dev, fp, mode, count) ? r.jobs_fused : r.jobs_kernel)++;
    }
    const hipError_t e = rt::launch_trace(r.dev, fp, a, mode, count, st, s->literal_stack, tev, q.fresh, &fresh_after);
    q.fresh = e == hipSuccess && fresh_after;
    HIP_TRY(e);
}

// Poses cams[0..nframes) of one row shard on replica r, into device buffers
// `out`, on stream st (scene lock held, r's device current): up to
// batch_frames() sample frames per launch.
void render_batch_locked(rt_scene* s, Replica& rr, const rt_camera* cams, int nframes, int spp, int mode, int row0,
                         int row_stride, int nrows, const rt_device_out* out, hipStream_t st, uint32_t flags,
                         int band = 1, const rt_deinterleave_job* job = nullptr) {
    Replica* r = &rr;
    const rt_camera* cam = &cams[0];
    const uint64_t fpix = (uint64_t)cam->width * (uint64_t)nrows;  // pixels per frame
    // poses per launch: the batch's sample-frame limit, and batch pixels
    // < 2^31 (redo-list entries)
    int per = std::max(1, batch_frames() / spp);
    while (per > 1 && fpix * (uint64_t)(per * spp) >= (1ull << 31)) per--;
    if (fpix * (uint64_t)spp >= (1ull << 31)) throw rt::Error{RT_ERR_INVALID_ARGUMENT, "image too large for spp"};
    const bool split = mode == RT_MODE_EXACT && rt::packet_split(spp, pack_samples(s, spp));
    if (split) {
        // candidate lists in HBM (73 B per sample pixel): at most half of
        // the device memory that is free (or already ours), fewer poses
        // per launch otherwise
        size_t mfree = 0, mtotal = 0;
        HIP_TRY(hipMemGetInfo(&mfree, &mtotal));
        const uint64_t avail = (uint64_t)mfree + r->cand_cap * kCandBytesPerPixel;
        while (per > 1 && fpix * (uint64_t)(per * spp) * kCandBytesPerPixel > avail / 2) per--;
        ensure_cand(*r, fpix * (uint64_t)(std::min(per, nframes) * spp));
    }
    const bool count = (flags & RT_FLAG_COUNT) != 0;
    for (int f0 = 0; f0 < nframes; f0 += per) {
        // each launch in the next slot (a batch of more poses than one launch
        // takes alternates slots too)
        Slot& q = take_slot(*r, st, split || count || RT_PROFILE_BUILD);
        ensure_redo(q, fpix * (uint64_t)std::min(per, nframes));
        const int n = std::min(per, nframes - f0);
        RtFrameParams fp = frame_params(s, cams + f0, n, row0, row_stride, nrows, spp, band);
        const uint64_t off = (uint64_t)f0 * fpix, soff = off * (uint64_t)spp;
        fp.hit_id = out->hit_id ? out->hit_id + soff : nullptr;
        fp.dist = out->dist ? out->dist + soff : nullptr;
        fp.hit_pos = out->pos ? out->pos + 3 * soff : nullptr;
        fp.rgb = out->rgb ? out->rgb + 3 * off : nullptr;
        fp.hit_count = out->hit_count ? out->hit_count + f0 : nullptr;
#if defined(RT_PROFILE) && RT_PROFILE
        fp.counters = r->d_counters;  // (a phase-profiling build: the timed kernel writes counters 18-23)
#else
        fp.counters = (flags & RT_FLAG_COUNT) ? r->d_counters : nullptr;
#endif
        const hipEvent_t* tev = nullptr;
        if (flags & RT_FLAG_TIMING) {
            if (r->tev_used == r->tev.size()) {
                std::array<hipEvent_t, 2> a{};
                for (auto& e : a) HIP_TRY(hipEventCreate(&e));
                r->tev.push_back(a);
            }
            tev = r->tev[r->tev_used++].data();
        }
        launch(s, *r, q, fp, mode, count, st, tev, f0 == 0 ? job : nullptr,  // (the job rides the first launch)
               (flags & RT_FLAG_SIDE_SLOT) != 0, (flags & RT_FLAG_COUNTS_STORE) != 0);
    }
}

// RT_GROUP_RCCL=1 (test hook, read per call): a one-device scene takes the
// multi-device path with its real transport — a one-rank RCCL communicator
// over that device, ncclGroupStart / ncclGather / ncclGroupEnd into the root
// buffer, then the de-interleave — so the RCCL branch runs on a one-GPU box.
bool rccl_self(const rt_scene* s) {
    if (s->reps.size() != 1) return false;
    const char* e = std::getenv("RT_GROUP_RCCL");
    return e && e[0] == '1';
}

// Shards of a multi-device frame: RT_VIRTUAL_SHARDS=N (test hook, read per
// call) splits a one-device scene into N shards on that device, gathered by
// device copies instead of RCCL.
int group_shards(const rt_scene* s) {
    if (s->reps.size() > 1) return (int)s->reps.size();
    if (rccl_self(s)) return 1;
    const char* e = std::getenv("RT_VIRTUAL_SHARDS");
    const int v = e ? std::atoi(e) : 1;
    return v >= 1 && v <= 64 ? v : 1;
}

// The multi-device path (render_group) is taken for more than one shard, or
// for the one-rank RCCL hook.
bool use_group(const rt_scene* s) { return group_shards(s) > 1 || rccl_self(s); }

// The RCCL communicator over the uploaded devices (rank g = the g-th
// replica), created on the first group render that needs it: uploading to
// several devices does not need RCCL, and per-device entry points never
// touch it.  Built into a local vector and kept only on success, so a failed
// init leaves no null handles behind and the next call retries.
void ensure_comms(rt_scene* s) {
    Group& gp = s->grp;
    if (gp.comms.size() == s->reps.size()) return;
    for (auto& r : s->reps) quiesce(*r);
    for (ncclComm_t c : gp.comms) rccl().destroy(c);
    gp.comms.clear();
    std::vector<int> devs;
    for (auto& r : s->reps) devs.push_back(r->device);
    std::vector<ncclComm_t> comms(devs.size(), nullptr);
    NCCL_TRY(rccl().init_all(comms.data(), (int)devs.size(), devs.data()));
    gp.comms = std::move(comms);
}

// Block layout of one shard (256-B aligned sections): per-sample hit ids,
// distances and positions, per-pixel rgb, per-pose hit counts — only the
// outputs the caller asked for.
struct ShardLayout {
    uint64_t id = 0, dist = 0, pos = 0, rgb = 0, cnt = 0, bytes = 0;
};
ShardLayout shard_layout(const rt_device_out* out, int F, int R, int W, int spp) {
    ShardLayout L;
    const uint64_t px = (uint64_t)F * R * W;
    uint64_t off = 0;
    auto sec = [&](bool want, uint64_t bytes) {
        const uint64_t o = off;
        if (want) off += align_up<char>(bytes);
        return o;
    };
    L.id = sec(out->hit_id, px * spp * 4);
    L.dist = sec(out->dist, px * spp * 8);
    L.pos = sec(out->pos, px * spp * 24);
    L.rgb = sec(out->rgb, px * 3);
    L.cnt = sec(true, (uint64_t)F * 8);
    L.bytes = off;
    return L;
}

// All poses over every shard (row g of every G-th row on the g-th device),
// gathered to the first device and de-interleaved there into full frames
// `out` (device pointers on the first device), asynchronous on st0 (a stream
// of the first device).  Scene lock held.
void render_group(rt_scene* s, const rt_camera* cams, int nframes, int spp, int mode, const rt_device_out* out,
                  hipStream_t st0, uint32_t flags) {
    Group& gp = s->grp;
    const int G = group_shards(s);
    const int W = cams[0].width, H = cams[0].height, R = rt_shard_pad(H, G);
    const bool virt = s->reps.size() == 1 && !rccl_self(s);
    Replica& r0 = *s->reps.front();
    const ShardLayout L = shard_layout(out, nframes, R, W, spp);
    if (!virt) ensure_comms(s);
    // buffers (grown, never shrunk; earlier groups finished first)
    if (gp.block < L.bytes || (int)gp.stage.size() != G) {
        for (auto& r : s->reps) quiesce(*r);
        for (size_t k = 0; k < gp.stage.size(); k++) {
            DevGuard dg(gp.stage_dev[k]);
            HIP_TRY(hipFree(gp.stage[k]));
        }
        gp.stage.assign(G, nullptr);
        gp.stage_dev.assign(G, r0.device);
        for (int g = 0; g < G; g++) {
            gp.stage_dev[g] = virt ? r0.device : s->reps[g]->device;
            DevGuard dg(gp.stage_dev[g]);
            HIP_TRY(hipMalloc(&gp.stage[g], L.bytes));
        }
        gp.block = L.bytes;
    }
    const uint64_t block = gp.block;
    DevGuard d0(r0.device);
    if (gp.gather_bytes < block * G) {
        quiesce(r0);
        if (gp.gather) HIP_TRY(hipFree(gp.gather));
        gp.gather = nullptr;
        HIP_TRY(hipMalloc(&gp.gather, block * G));
        gp.gather_bytes = block * G;
    }
    if (!gp.ev_in) {
        for (hipEvent_t* e : {&gp.ev_in, &gp.ev_out}) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
        for (hipEvent_t* e : {&gp.ev0, &gp.ev1}) HIP_TRY(hipEventCreate(e));
    }
    HIP_TRY(hipEventRecord(gp.ev_in, st0));
    HIP_TRY(hipEventRecord(gp.ev0, r0.stream));
    // every shard renders its rows of every pose into its block
    for (int g = 0; g < G; g++) {
        Replica& r = virt ? r0 : *s->reps[g];
        DevGuard dg(r.device);
        HIP_TRY(hipStreamWaitEvent(r.stream, gp.ev_in, 0));
        uint8_t* b = static_cast<uint8_t*>(gp.stage[g]);
        rt_device_out so{};
        so.hit_id = out->hit_id ? reinterpret_cast<uint32_t*>(b + L.id) : nullptr;
        so.dist = out->dist ? reinterpret_cast<double*>(b + L.dist) : nullptr;
        so.pos = out->pos ? reinterpret_cast<double*>(b + L.pos) : nullptr;
        so.rgb = out->rgb ? b + L.rgb : nullptr;
        so.hit_count = reinterpret_cast<unsigned long long*>(b + L.cnt);
        const int nrows = rt_shard_rows(H, G, g);
        if (nrows > 0) {  // (the shard's counts stored into its block: no zeroing)
            render_batch_locked(s, r, cams, nframes, spp, mode, g, G, nrows, &so, r.stream,
                                flags | RT_FLAG_COUNTS_STORE, RT_SHARD_BAND);
        } else {
            HIP_TRY(hipMemsetAsync(b + L.cnt, 0, (size_t)nframes * 8, r.stream));
        }
    }
    // gather to the first device: RCCL between distinct devices (one group of
    // ncclGather calls, each on its shard's stream), device copies otherwise
    if (!virt) {
        NCCL_TRY(rccl().group_start());
        for (int g = 0; g < G; g++) {
            DevGuard dg(s->reps[g]->device);
            NCCL_TRY(rccl().gather(gp.stage[g], g == 0 ? gp.gather : nullptr, block, ncclUint8, 0, gp.comms[g],
                                   s->reps[g]->stream));
        }
        NCCL_TRY(rccl().group_end());
    } else {
        for (int g = 0; g < G; g++)
            HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(gp.gather) + (uint64_t)g * block, gp.stage[g], block,
                                   hipMemcpyDeviceToDevice, r0.stream));
    }
    // de-interleave on the first device (its stream follows its gather)
    const int ssz = spp;
    if (out->hit_id)
        HIP_TRY(rt::launch_deinterleave(gp.gather, block, L.id, G, nframes, H, W, 4 * ssz, out->hit_id, r0.stream));
    if (out->dist)
        HIP_TRY(rt::launch_deinterleave(gp.gather, block, L.dist, G, nframes, H, W, 8 * ssz, out->dist, r0.stream));
    if (out->pos)
        HIP_TRY(rt::launch_deinterleave(gp.gather, block, L.pos, G, nframes, H, W, 24 * ssz, out->pos, r0.stream));
    if (out->rgb) HIP_TRY(rt::launch_deinterleave(gp.gather, block, L.rgb, G, nframes, H, W, 3, out->rgb, r0.stream));
    if (out->hit_count)
        HIP_TRY(rt::launch_sum_counts(gp.gather, block, L.cnt, G, nframes, out->hit_count,
                                      (flags & RT_FLAG_COUNTS_STORE) != 0, r0.stream));
    HIP_TRY(hipEventRecord(gp.ev1, r0.stream));
    HIP_TRY(hipEventRecord(gp.ev_out, r0.stream));
    HIP_TRY(hipStreamWaitEvent(st0, gp.ev_out, 0));
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_err.c_str(); }
void rt_free(void* p) { std::free(p); }

const char* rt_rccl_path(void) {
    static std::string path;
    try {
        Dl_info info{};
        if (!dladdr(reinterpret_cast<void*>(rccl().gather), &info) || !info.dli_fname) {
            fail(RT_ERR_RUNTIME, "RCCL mapped but its file is unknown");
            return nullptr;
        }
        path = info.dli_fname;
        return path.c_str();
    } catch (const rt::Error& e) {
        fail(e.status, e.msg);
        return nullptr;
    }
}

const char* rt_device_name(int device) {
    static thread_local std::string name;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return "";
    name = std::string(prop.name) + " (" + prop.gcnArchName + ")";
    return name.c_str();
}

int rt_load_obj(const char* path, double scale, double** tris, uint64_t* n_tris) {
    if (!path || !tris || !n_tris) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    try {
        std::vector<double> v = rt::load_obj(path, scale);
        double* buf = (double*)std::malloc(std::max<size_t>(v.size(), 1) * sizeof(double));
        if (!buf) return fail(RT_ERR_RUNTIME, "out of memory");
        if (!v.empty()) std::memcpy(buf, v.data(), v.size() * sizeof(double));
        *tris = buf;
        *n_tris = v.size() / 9;
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_load_obj_cached(const char* path, double scale, const char* cache_dir, double** tris, uint64_t* n_tris,
                       int* from_cache) {
    if (!path || !cache_dir || !tris || !n_tris) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    try {
        bool hit = false;
        std::vector<double> v = rt::load_obj_cached(path, scale, cache_dir, &hit);
        double* buf = (double*)std::malloc(std::max<size_t>(v.size(), 1) * sizeof(double));
        if (!buf) return fail(RT_ERR_RUNTIME, "out of memory");
        if (!v.empty()) std::memcpy(buf, v.data(), v.size() * sizeof(double));
        *tris = buf;
        *n_tris = v.size() / 9;
        if (from_cache) *from_cache = hit ? 1 : 0;
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_scene_center(const double* tri_v, uint64_t n, double center[3]) {
    if (!tri_v || !center || n == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty scene");
    rt::scene_center(tri_v, n, center);
    return RT_OK;
}

int rt_camera_path(const double c[3], int res, int step, double pos[3], double dir[3]) {
    if (!c || !pos || !dir || res <= 0) return fail(RT_ERR_INVALID_ARGUMENT, "bad camera path arguments");
    rt::camera_path(c, res, step, pos, dir);
    return RT_OK;
}

// rt_scene_create / rt_scene_create_on_device: walk_device < 0 builds the
// walk tree on the host (walk_tree.cpp), else on that HIP device (walk_build.hip).
static int scene_create(const double* tri_v, uint64_t n, int algo, int k, int collapse, int walk_device,
                        rt_scene** out) {
    if (!out || (n && !tri_v)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = nullptr;
    if (algo < 0 || algo > 2) return fail(RT_ERR_OUT_OF_RANGE, "Unknown algorithm");
    if (!(k == 2 || k == 4 || k == 8 || k == 16)) return fail(RT_ERR_INVALID_ARGUMENT, "Unsupported bvh degree");
    if (n > RT_LEAF_MAX_FIRST || n > RT_MAX_TRIS) return fail(RT_ERR_INVALID_ARGUMENT, "too many triangles");
    try {
        using clk = std::chrono::steady_clock;
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::unique_ptr<rt_scene> s(new rt_scene);
        const auto t0 = clk::now();
        s->soup = rt::make_soup(tri_v, n);
        const auto t1 = clk::now();
        // the device walks a rebuilt SAH tree (walk_tree.cpp) unless
        // RT_WALK=reference asks for the reference tree's own nodes
        const char* wk = std::getenv("RT_WALK");
        s->times.walk_device = -1;
        auto t2 = t1, t3 = t1;
        if (wk && wk[0] == 'r') {
            s->tree = rt::build_tree(s->soup, algo, k, collapse);
            t2 = t3 = clk::now();
            s->flat = rt::flatten(s->soup, s->tree, 0);
        } else {
            if (walk_device >= 0) {
                int count = 0;
                if (hipGetDeviceCount(&count) != hipSuccess || walk_device >= count)
                    return fail(RT_ERR_NO_DEVICE, "bad device ordinal for the walk-tree build");
            }
            rt::WalkTree wt;
            if (walk_device >= 0) {
                // the two trees are independent (both read only the soup): the
                // reference tree builds on host threads while this thread
                // drives the device build of the walk tree (mostly waiting)
                std::exception_ptr tree_err;
                auto ref_tree = [&] {
                    try {
                        s->tree = rt::build_tree(s->soup, algo, k, collapse);
                    } catch (...) { tree_err = std::current_exception(); }
                    t2 = clk::now();
                };
                // spawn-or-run-inline: a host that cannot start a thread
                // builds the reference tree on this one first
                std::thread ref;
                try {
                    ref = std::thread(ref_tree);
                } catch (const std::system_error&) {
                    ref_tree();
                }
                try {
                    wt = rt::build_walk_tree_device(s->soup, walk_device, rt::walk_max_leaf(), rt::walk_node_cost());
                    rt::restructure_treelets(wt, rt::walk_treelet_passes());
                    rt::plan_wide_collapse(wt, 8);
                } catch (...) {
                    if (ref.joinable()) ref.join();
                    throw;
                }
                s->times.walk_device = walk_device;
                t3 = clk::now();
                if (ref.joinable()) ref.join();
                if (tree_err) std::rethrow_exception(tree_err);
            } else {
                // host walk build: one after the other (both want the host's
                // cores and memory bandwidth)
                s->tree = rt::build_tree(s->soup, algo, k, collapse);
                t2 = clk::now();
                wt = rt::build_walk_tree(s->soup);
                rt::restructure_treelets(wt, rt::walk_treelet_passes());
                rt::plan_wide_collapse(wt, 8);
                t3 = clk::now();
            }
            s->flat = rt::flatten(s->soup, s->tree, 0, &wt);
        }
        const auto t4 = clk::now();
        s->literal_stack = literal_stack_bound(s.get());
        s->times.soup_ms = ms(t0, t1);
        s->times.reference_tree_ms = ms(t1, t2);
        s->times.walk_tree_ms = walk_device >= 0 ? ms(t1, t3) : ms(t2, t3);
        s->times.flatten_ms = ms(std::max(t2, t3), t4);
        s->times.total_ms = ms(t0, t4);
        *out = s.release();
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::bad_alloc&) {
        return fail(RT_ERR_RUNTIME, "out of memory");
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_scene_create(const double* tri_v, uint64_t n, int algo, int k, int collapse, rt_scene** out) {
    return scene_create(tri_v, n, algo, k, collapse, -1, out);
}

int rt_scene_create_on_device(const double* tri_v, uint64_t n, int algo, int k, int collapse, int device,
                              rt_scene** out) {
    if (device < 0) return fail(RT_ERR_NO_DEVICE, "bad device ordinal for the walk-tree build");
    return scene_create(tri_v, n, algo, k, collapse, device, out);
}

int rt_scene_build_times(const rt_scene* s, rt_build_times_t* out) {
    if (!s || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = s->times;
    return RT_OK;
}

int rt_scene_upload(rt_scene* s, const int* devices, int n_devices) {
    if (!s || (n_devices > 0 && !devices)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n_devices < 0) return fail(RT_ERR_INVALID_ARGUMENT, "negative device count");
    // the list is rank order of the RCCL communicator a multi-device render
    // builds (ncclCommInitAll): every ordinal once, checked before any device
    // or RCCL call
    for (int q = 0; q < n_devices; q++) {
        if (devices[q] < 0) return fail(RT_ERR_INVALID_ARGUMENT, "negative device ordinal");
        for (int p = 0; p < q; p++)
            if (devices[p] == devices[q]) return fail(RT_ERR_INVALID_ARGUMENT, "device ordinal listed twice");
    }
    std::lock_guard<std::mutex> lk(s->mu);
    try {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device");
        for (int q = 0; q < n_devices; q++)
            if (devices[q] >= count) return fail(RT_ERR_INVALID_ARGUMENT, "device ordinal out of range");
        for (int q = 0; q < n_devices; q++) {
            bool have = false;
            for (auto& r : s->reps) have |= r->device == devices[q];
            if (!have) upload_one(s, devices[q]);
        }
        // (the RCCL communicator over several devices is created by the first
        // multi-device render, ensure_comms)
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_render_batch_spp_device(rt_scene* s, int device, const rt_camera* cams, int nframes, int spp, int mode,
                               int row0, int row_stride, int nrows, const rt_device_out* out, void* stream,
                               uint32_t flags) {
    if (!s || !out || (nframes > 0 && !cams)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (nframes < 0) return fail(RT_ERR_INVALID_ARGUMENT, "negative frame count");
    if (spp < 1 || spp > RT_MAX_BATCH || spp_grid(spp) * spp_grid(spp) != spp)
        return fail(RT_ERR_INVALID_ARGUMENT, "spp must be n*n samples (1, 4, 9 or 16)");
    if (mode != RT_MODE_EXACT && mode != RT_MODE_FP64) return fail(RT_ERR_INVALID_ARGUMENT, "bad mode");
    try {
        for (int f = 0; f < nframes; f++) {
            check_camera(s, &cams[f]);
            if (cams[f].width != cams[0].width || cams[f].height != cams[0].height)
                return fail(RT_ERR_INVALID_ARGUMENT, "frames of a batch must share the image size");
        }
        if (nframes == 0) return RT_OK;
        const rt_camera* cam = &cams[0];
        if (row0 < 0 || row_stride < 1 || nrows < 0 || (nrows > 0 && row0 + (int64_t)(nrows - 1) * row_stride >= cam->height))
            return fail(RT_ERR_INVALID_ARGUMENT, "row shard outside the image");
        // one caller at a time per scene: launches on a replica share its
        // work-queue block, redo list and pool
        std::lock_guard<std::mutex> lk(s->mu);
        Replica* r = &replica_for(s, device);
        DevGuard g(device);
        render_batch_locked(s, *r, cams, nframes, spp, mode, row0, row_stride, nrows, out, (hipStream_t)stream, flags);
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_render_batch_multi(rt_scene* s, const rt_camera* cams, int nframes, int spp, int mode, const rt_device_out* out,
                          void* stream, uint32_t flags) {
    if (!s || !out || (nframes > 0 && !cams)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (nframes < 0) return fail(RT_ERR_INVALID_ARGUMENT, "negative frame count");
    if (nframes > 1024) return fail(RT_ERR_INVALID_ARGUMENT, "at most 1024 poses per call");
    if (spp < 1 || spp > RT_MAX_BATCH || spp_grid(spp) * spp_grid(spp) != spp)
        return fail(RT_ERR_INVALID_ARGUMENT, "spp must be n*n samples (1, 4, 9 or 16)");
    if (mode != RT_MODE_EXACT && mode != RT_MODE_FP64) return fail(RT_ERR_INVALID_ARGUMENT, "bad mode");
    try {
        for (int f = 0; f < nframes; f++) {
            check_camera(s, &cams[f]);
            if (cams[f].width != cams[0].width || cams[f].height != cams[0].height)
                return fail(RT_ERR_INVALID_ARGUMENT, "frames of a batch must share the image size");
        }
        if (nframes == 0) return RT_OK;
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->reps.empty()) return fail(RT_ERR_NO_DEVICE, "scene not uploaded");
        Replica& r0 = *s->reps.front();
        DevGuard g(r0.device);
        if (!use_group(s))
            render_batch_locked(s, r0, cams, nframes, spp, mode, 0, 1, cams[0].height, out, (hipStream_t)stream, flags);
        else
            render_group(s, cams, nframes, spp, mode, out, (hipStream_t)stream, flags);
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_render_shard_device(rt_scene* s, int device, const rt_camera* cams, int nframes, int spp, int mode, int shard,
                           int nshards, const rt_device_out* out, void* stream, uint32_t flags) {
    return rt_render_shard_device_job(s, device, cams, nframes, spp, mode, shard, nshards, out, nullptr, stream, flags);
}

int rt_render_shard_device_job(rt_scene* s, int device, const rt_camera* cams, int nframes, int spp, int mode,
                               int shard, int nshards, const rt_device_out* out, const rt_deinterleave_job* job,
                               void* stream, uint32_t flags) {
    if (job && job->frames > 0 &&
        (!job->gathered || !job->frames_out || job->shards < 1 || job->height < 1 || job->width < 1 ||
         job->elem_bytes < 1 || job->frame_rows < 0 ||
         (job->frame_rows > 0 && job->frame_rows < rt_shard_rows(job->height, job->shards, 0)) ||
         (uint64_t)job->frames * (uint64_t)job->height >= (1ull << 32) ||
         // every shard's section must lie inside its block (the tallest
         // shard's rows: frame_rows, or rt_shard_rows of shard 0)
         job->section_offset + (uint64_t)job->frames *
                 (uint64_t)(job->frame_rows > 0 ? job->frame_rows : rt_shard_rows(job->height, job->shards, 0)) *
                 (uint64_t)job->width * (uint64_t)job->elem_bytes > job->block_bytes))
        return fail(RT_ERR_INVALID_ARGUMENT, "bad de-interleave job");
    if (!s || !out || (nframes > 0 && !cams)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (nframes < 0) return fail(RT_ERR_INVALID_ARGUMENT, "negative frame count");
    if (spp < 1 || spp > RT_MAX_BATCH || spp_grid(spp) * spp_grid(spp) != spp)
        return fail(RT_ERR_INVALID_ARGUMENT, "spp must be n*n samples (1, 4, 9 or 16)");
    if (mode != RT_MODE_EXACT && mode != RT_MODE_FP64) return fail(RT_ERR_INVALID_ARGUMENT, "bad mode");
    if (nshards < 1 || shard < 0 || shard >= nshards) return fail(RT_ERR_INVALID_ARGUMENT, "bad shard");
    try {
        for (int f = 0; f < nframes; f++) {
            check_camera(s, &cams[f]);
            if (cams[f].width != cams[0].width || cams[f].height != cams[0].height)
                return fail(RT_ERR_INVALID_ARGUMENT, "frames of a batch must share the image size");
        }
        const int nrows = nframes > 0 ? rt_shard_rows(cams[0].height, nshards, shard) : 0;
        std::lock_guard<std::mutex> lk(s->mu);
        Replica* r = &replica_for(s, device);
        DevGuard g(device);
        if (nframes == 0 || nrows == 0) {  // nothing to render: the job on its own
            if (job && job->frames > 0) {
                RtLaunchAux a{};
                set_job(a, job);
                HIP_TRY(rt::launch_job(a, (hipStream_t)stream));
            }
            return RT_OK;
        }
        render_batch_locked(s, *r, cams, nframes, spp, mode, shard, nshards, nrows, out, (hipStream_t)stream, flags,
                            RT_SHARD_BAND, job);
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_shard_height(int height, int nshards, int shard) {
    if (height < 0 || nshards < 1 || shard < 0 || shard >= nshards) return -1;
    return rt_shard_rows(height, nshards, shard);
}

int rt_render_batch_device(rt_scene* s, int device, const rt_camera* cams, int nframes, int mode, int row0,
                           int row_stride, int nrows, const rt_device_out* out, void* stream, uint32_t flags) {
    return rt_render_batch_spp_device(s, device, cams, nframes, 1, mode, row0, row_stride, nrows, out, stream, flags);
}

int rt_render_paths_device(rt_scene* s, int device, const rt_camera* cam, int frame, int spp, int bounces, int row0,
                           int row_stride, int nrows, const rt_device_out* out, void* stream, uint32_t flags) {
    if (!s || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (spp < 1 || spp > 4096) return fail(RT_ERR_INVALID_ARGUMENT, "spp must be 1..4096");
    if (bounces < 0 || bounces > 64) return fail(RT_ERR_INVALID_ARGUMENT, "bounces must be 0..64");
    try {
        check_camera(s, cam);
        if (row0 < 0 || row_stride < 1 || nrows < 0 || (nrows > 0 && row0 + (int64_t)(nrows - 1) * row_stride >= cam->height))
            return fail(RT_ERR_INVALID_ARGUMENT, "row shard outside the image");
        if ((uint64_t)cam->width * (uint64_t)nrows * (uint64_t)spp >= (1ull << 31))
            return fail(RT_ERR_INVALID_ARGUMENT, "image too large for spp");
        std::lock_guard<std::mutex> lk(s->mu);
        Replica* r = &replica_for(s, device);
        DevGuard g(device);
        hipStream_t st = (hipStream_t)stream;
        RtFrameParams fp = frame_params(s, cam, 1, row0, row_stride, nrows);
        fp.spp = spp;  // samples per pixel of the paths (one frame: offsets come from the hash)
        {
            // a wave takes every sample of 64 / spp pixels, one path per lane
            // (8-wide walk trees; RT_PATHS_PACK=0: one pixel per lane)
            const char* e = std::getenv("RT_PATHS_PACK");
            fp.pack = spp > 1 && 64 % spp == 0 && s->flat.width == 8 && !(e && e[0] == '0');
        }
        fp.counters = (flags & RT_FLAG_COUNT) ? r->d_counters : nullptr;  // [0] += ray segments traced
        fp.hit_id = out->hit_id;
        fp.dist = out->dist;
        fp.hit_pos = out->pos;
        fp.rgb = out->rgb;
        fp.hit_count = out->hit_count;
        // (the path kernels add their hits: a stored count is zeroed first)
        if ((flags & RT_FLAG_COUNTS_STORE) && out->hit_count)
            HIP_TRY(hipMemsetAsync(out->hit_count, 0, sizeof(unsigned long long), st));
        const hipEvent_t* tev = nullptr;
        if (flags & RT_FLAG_TIMING) {
            if (r->tev_used == r->tev.size()) {
                std::array<hipEvent_t, 2> a{};
                for (auto& e : a) HIP_TRY(hipEventCreate(&e));
                r->tev.push_back(a);
            }
            tev = r->tev[r->tev_used++].data();
        }
        hipError_t e;
        PathPipe pipe = path_pipe((flags & RT_FLAG_SHADOW) != 0, (int)r->dev.width, spp);
        PathQs qs{};
        if (pipe == PathPipe::queue) {
            // the queued workspace (256 B per path: 34 GB for a c5 pose);
            // when the library chose the queue itself and the workspace
            // cannot be had, the megakernel renders the same bits with none
            uint64_t P = (uint64_t)cam->width * (uint64_t)nrows * (uint64_t)spp;
            if (spp == 4 || spp == 16)  // (room for the partitioned layout of the packet primaries)
                P = std::max(P, rt_qparts(cam->width, nrows, spp).entries);
            try {
                qs = ensure_pq(*r, P);
            } catch (const rt::Error&) {
                if (path_pipe_forced()) throw;
                (void)hipGetLastError();
                pipe = PathPipe::mega;
            }
        }
        if (pipe == PathPipe::queue) {
            Slot& q = take_slot(*r, st, true);  // (the replica-wide workspace: after every slot's launches)
            e = rt::launch_paths_q(r->dev, fp, aux_of(*r, q), qs, (uint32_t)frame, bounces,
                                   (flags & RT_FLAG_SHADOW) != 0, st, tev);
        } else {
            Slot& q = take_slot(*r, st, (flags & RT_FLAG_COUNT) != 0);
            e = rt::launch_paths(r->dev, fp, aux_of(*r, q), (uint32_t)frame, bounces, (flags & RT_FLAG_SHADOW) != 0,
                                 st, tev);
            q.fresh = false;
        }
        HIP_TRY(e);
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_render_rows_device(rt_scene* s, int device, const rt_camera* cam, int mode, int row0, int row_stride,
                          int nrows, const rt_device_out* out, void* stream, uint32_t flags) {
    if (!cam) return fail(RT_ERR_INVALID_ARGUMENT, "camera is NULL");
    return rt_render_batch_device(s, device, cam, 1, mode, row0, row_stride, nrows, out, stream, flags);
}

int rt_render_frame(rt_scene* s, const rt_camera* cam, int mode, rt_frame_out* out) {
    if (!s || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    try {
        check_camera(s, cam);
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->reps.empty()) return fail(RT_ERR_NO_DEVICE, "scene not uploaded");
        Replica& r = *s->reps.front();
        DevGuard g(r.device);
        const size_t npx = (size_t)cam->width * cam->height;
        // staging: hit_id u32 | dist f64 | pos 3xf64 | rgb 3xu8 | hit counter
        const size_t o_id = 0, o_dist = align_up<char>(npx * 4), o_pos = o_dist + align_up<char>(npx * 8),
                     o_rgb = o_pos + align_up<char>(npx * 24), o_cnt = o_rgb + align_up<char>(npx * 3),
                     total = o_cnt + 256;
        if (r.frame_bytes < total) {
            if (r.frame) HIP_TRY(hipFree(r.frame));
            r.frame = nullptr;
            HIP_TRY(hipMalloc(&r.frame, total));
            r.frame_bytes = total;
        }
        uint8_t* base = static_cast<uint8_t*>(r.frame);
        rt_device_out d{};
        d.hit_id = out->hit_id ? reinterpret_cast<uint32_t*>(base + o_id) : nullptr;
        d.dist = out->dist ? reinterpret_cast<double*>(base + o_dist) : nullptr;
        d.pos = out->pos ? reinterpret_cast<double*>(base + o_pos) : nullptr;
        d.rgb = reinterpret_cast<uint8_t*>(base + o_rgb);  // always shaded (shadeScreen)
        d.hit_count = reinterpret_cast<unsigned long long*>(base + o_cnt);
        RtFrameParams fp = frame_params(s, cam, 1, 0, 1, cam->height);
        fp.hit_id = d.hit_id;
        fp.dist = d.dist;
        fp.hit_pos = d.pos;
        fp.rgb = d.rgb;
        fp.hit_count = d.hit_count;
        hipEvent_t e0 = r.ev0, e1 = r.ev1;
        if (use_group(s)) {
            // every uploaded device renders its interleaved rows; the frame
            // is gathered and de-interleaved on the first device (the device
            // time is the group's, first device's stream: renders to gather)
            render_group(s, cam, 1, 1, mode, &d, r.stream, RT_FLAG_COUNTS_STORE);
            e0 = s->grp.ev0;
            e1 = s->grp.ev1;
        } else {
            const bool split = mode == RT_MODE_EXACT && rt::packet_split(1, false);
            if (split) ensure_cand(r, npx);
            Slot& q = take_slot(r, r.stream, split);
            ensure_redo(q, npx);
            HIP_TRY(hipEventRecord(r.ev0, r.stream));
            launch(s, r, q, fp, mode, false, r.stream, nullptr, nullptr, false, true);  // (counts stored)
            HIP_TRY(hipEventRecord(r.ev1, r.stream));
        }
        if (out->hit_id) HIP_TRY(hipMemcpyAsync(out->hit_id, d.hit_id, npx * 4, hipMemcpyDeviceToHost, r.stream));
        if (out->dist) HIP_TRY(hipMemcpyAsync(out->dist, d.dist, npx * 8, hipMemcpyDeviceToHost, r.stream));
        if (out->pos) HIP_TRY(hipMemcpyAsync(out->pos, d.pos, npx * 24, hipMemcpyDeviceToHost, r.stream));
        if (out->rgb) HIP_TRY(hipMemcpyAsync(out->rgb, d.rgb, npx * 3, hipMemcpyDeviceToHost, r.stream));
        unsigned long long hc = 0;
        HIP_TRY(hipMemcpyAsync(&hc, d.hit_count, 8, hipMemcpyDeviceToHost, r.stream));
        HIP_TRY(hipStreamSynchronize(r.stream));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        out->hit_count = hc;
        out->seconds = ms * 1e-3;
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_deinterleave_rows(const void* gathered, uint64_t block_bytes, uint64_t section_offset, int shards, int frames,
                         int height, int width, int elem_bytes, void* frames_out) {
    if (!gathered || !frames_out || shards < 1 || frames < 0 || height < 0 || width < 0 || elem_bytes < 1)
        return fail(RT_ERR_INVALID_ARGUMENT, "bad de-interleave arguments");
    const uint64_t n = (uint64_t)width * elem_bytes;
    for (int f = 0; f < frames; f++)
        for (int j = 0; j < height; j++)
            std::memcpy(static_cast<uint8_t*>(frames_out) + ((uint64_t)f * height + j) * n,
                        static_cast<const uint8_t*>(gathered) +
                            rt_gathered_row(j, f, shards, height, width, elem_bytes, block_bytes, section_offset),
                        n);
    return RT_OK;
}

int rt_diag_raw(rt_scene* s, int device, uint64_t* out, size_t n) {
    if (!s || (!out && n)) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    try {
        std::lock_guard<std::mutex> lk(s->mu);
        Replica& r = replica_for(s, device);
        DevGuard g(device);
        quiesce(r);
        HIP_TRY(hipMemcpy(out, r.d_counters, std::min(n, kCounterWords) * sizeof(uint64_t), hipMemcpyDeviceToHost));
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_frame_stats(rt_scene* s, int device, int reset, rt_frame_stats_t* out) {
    if (!s || !out) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    try {
        std::lock_guard<std::mutex> lk(s->mu);
        Replica& r = replica_for(s, device);
        DevGuard g(device);
        quiesce(r);
        std::vector<unsigned long long> cv(kCounterWords);
        HIP_TRY(hipMemcpy(cv.data(), r.d_counters, cv.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const unsigned long long* c = cv.data();
        out->rays = c[0];
        out->node_fetches = c[1];
        out->tri_tests = c[2];
        out->chain_checks = c[3];
        out->hits = c[4];
        out->chain_nodes = c[5];
        out->tri_prefilter = c[6];
        out->wave_nodes = c[7];
        out->wave_leaves = c[8];
        out->wave_tiles = c[9];
        out->wave_tris = c[12];
        out->redo_rays = c[10] + c[11];
        out->redo_chain = c[11];
        out->spilled_rays = c[13];
        out->dropped_rays = c[14];
        out->empty_node_steps = c[15];
        out->wave_tri_tests = c[16];
        out->wave_winners = c[17];
        out->shadow_rays = c[24];
        out->shadow_occluded = c[25];
        out->shadow_wave_nodes = c[26];
        out->shadow_wave_tris = c[27];
        out->shadow_lane_nodes = c[28];
        out->shadow_lane_tris = c[29];
        out->lane_wave_nodes = c[30];
        out->lane_wave_tris = c[31];
        out->side_jobs_fused = r.jobs_fused;
        out->side_jobs_kernel = r.jobs_kernel;
        if (reset) r.jobs_fused = r.jobs_kernel = 0;
        out->timed_launches = r.tev_used;
        out->trace_ms = 0.0;
        for (size_t k = 0; k < r.tev_used; k++) {
            float a = 0;
            HIP_TRY(hipEventElapsedTime(&a, r.tev[k][0], r.tev[k][1]));
            out->trace_ms += a;
        }
        if (reset) r.tev_used = 0;
        if (reset) HIP_TRY(hipMemset(r.d_counters, 0, cv.size() * sizeof(unsigned long long)));
        return RT_OK;
    } catch (const rt::Error& e) {
        return fail(e.status, e.msg);
    } catch (const std::exception& e) {
        return fail(RT_ERR_RUNTIME, e.what());
    }
}

int rt_scene_stats(const rt_scene* s, rt_scene_stats_t* o) {
    if (!s || !o) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    const rt::Flat& f = s->flat;
    o->triangles = s->soup.n;
    o->real_inner = f.real_inner;
    o->real_leaves = f.real_leaves;
    o->real_nodes = f.real_inner + f.real_leaves;
    o->depth = f.depth;
    o->max_children = f.max_children;
    o->max_leaf_size = f.max_leaf;
    o->wide_width = (uint32_t)f.width;
    o->wide_nodes = f.n_wide;
    o->node_bytes = rt_node_bytes(f.width);
    o->stack_bound = f.stack_bound;
    o->walk_tree = f.walk ? 1u : 0u;
    o->device_bytes = f.wide.size() + f.tri32.size() * 4 + f.tri64.size() * 8 + f.tri_id.size() * 12 +
                      f.rbox.size() * 8 + f.rparent.size() * 4 + s->soup.normal.size() * 8 +
                      (f.rkid_off.size() + f.rkid.size() + f.rrange.size() + f.ref2walk.size()) * 4;
    uint64_t h = 0xcbf29ce484222325ull;
    auto mix = [&](const void* p, size_t bytes) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        h = (h ^ bytes) * 0x100000001b3ull;
        size_t i = 0;
        for (; i + 8 <= bytes; i += 8) {
            uint64_t w;
            std::memcpy(&w, b + i, 8);
            h = (h ^ w) * 0x100000001b3ull;
        }
        for (; i < bytes; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    };
    auto vec = [&](const auto& v) { mix(v.data(), v.size() * sizeof(v[0])); };
    vec(f.wide); vec(f.tri32); vec(f.tri64); vec(f.tri_id); vec(f.tri_rank); vec(f.tri_leaf); vec(f.rbox);
    vec(f.rparent); vec(f.rkid_off); vec(f.rkid); vec(f.rrange); vec(f.ref2walk);
    mix(&f.root_ref, sizeof f.root_ref);
    mix(&f.root_meta, sizeof f.root_meta);
    mix(f.root_box, sizeof f.root_box);
    mix(&f.stack_bound, sizeof f.stack_bound);
    o->layout_digest = h;
    return RT_OK;
}

int rt_scene_tree_dump(const rt_scene* s, double* boxes, int64_t* meta, int64_t* order) {
    if (!s || !boxes || !meta || !order) return fail(RT_ERR_INVALID_ARGUMENT, "NULL argument");
    std::vector<int32_t> st{0};
    int64_t k = 0;
    while (!st.empty()) {
        const rt::RNode& n = s->tree.nodes[st.back()];
        st.pop_back();
        for (int a = 0; a < 3; a++) { boxes[k * 6 + a] = n.mn[a]; boxes[k * 6 + 3 + a] = n.mx[a]; }
        meta[k * 3] = n.begin;
        meta[k * 3 + 1] = n.end;
        meta[k * 3 + 2] = (int64_t)n.kids.size();
        k++;
        for (int32_t c : n.kids) st.push_back(c);
    }
    for (size_t i = 0; i < s->tree.order.size(); i++) order[i] = s->tree.order[i];
    return RT_OK;
}

void rt_scene_destroy(rt_scene* s) {
    if (!s) return;
    free_group(s);
    for (auto& r : s->reps) free_replica(*r);
    delete s;
}

}  // extern "C"
