// The walk tree built on the device: the binned-SAH
// binary tree of walk_tree.cpp (32 centroid bins over the three axes, leaves
// of at most RT_WALK_LEAF triangles, the same cost rule), built breadth-first
// on a gfx950 device, then collapsed and flattened on the host as before.
//
// The splits are the host builder's, operation for operation in fp64: the same
// centroids 0.5 (lo + hi), bin index, suffix/prefix box areas and cost
// expression, the first strictly smaller cost over axes 0..2 and bins 1..31.
// A node's triangle SET therefore equals the host's; only the order inside a
// node differs (a stable device partition instead of std::partition), which
// matters only where the host splits by position (a split that leaves one
// side empty, or coincident centroids) and for the order inside a leaf.
// Which walk tree is walked never changes a result (walk_tree.cpp).
//
// Device work per level (every node of the level with more than kSmall
// triangles is one task; its triangles are a contiguous range of `idx`):
//   k_bounds    node box and centroid box (wave-reduced fp64 min / max through
//               order-preserving u64 keys, then atomics)
//   k_bin       3 x 32 bins per task: counts and boxes (LDS-privatised when a
//               block lies inside one task, else global atomics)
//   k_split     one thread per task: best split, node box, child sizes
//   scan        child numbering (hipcub exclusive scan over tasks)
//   k_children  child node ids, next-level tasks, small subtrees
//   k_flags     side of every triangle; scan; k_scatter: stable partition
// Subtrees of at most kSmall triangles are finished by k_small, one thread
// per subtree running the host algorithm in place.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdlib>
#include <vector>

#include "rt_internal.h"

namespace {

#ifndef RT_WALK_BINS
#define RT_WALK_BINS 32  // centroid bins per axis (host and device builds must agree)
#endif
constexpr int kBins = RT_WALK_BINS;
constexpr uint32_t kSmall = 16;  // a subtree of at most this many triangles: one thread (16: 64 measured 13 ms in k_small)

static_assert(sizeof(rt::WalkNode) == 64, "device nodes are copied straight into WalkNode");

struct DNode {  // = rt::WalkNode
    double mn[3], mx[3];
    int32_t left, right;
    uint32_t first, count;
};

// order-preserving u64 key of a double (no NaNs): min / max of keys = of values
__device__ __forceinline__ uint64_t okey(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double odec(uint64_t k) {
    const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}
constexpr uint64_t kKeyPosInf = 0xFFF0000000000000ull;  // okey(+inf)
constexpr uint64_t kKeyNegInf = 0x000FFFFFFFFFFFFFull;  // okey(-inf)

// walk_tree.cpp BBox::area
__device__ __forceinline__ double area(const double mn[3], const double mx[3]) {
    if (!(mx[0] >= mn[0])) return 0.0;
    const double ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
    return 2.0 * (ex * ey + ey * ez + ez * ex);
}

__device__ __forceinline__ int bin_of(double c, double lo, double scale) {
    int k = (int)((c - lo) * scale);
    return k < 0 ? 0 : (k > kBins - 1 ? kBins - 1 : k);
}

struct Tri {  // SoA triangle boxes and centroids
    const double* lo[3];
    const double* hi[3];
    double* cen[3];
};

__global__ void k_init(Tri t, uint32_t n, uint32_t* idx, int32_t* seg) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        for (int a = 0; a < 3; a++) t.cen[a][i] = 0.5 * (t.lo[a][i] + t.hi[a][i]);  // walk_tree.cpp:93
        idx[i] = i;
        seg[i] = 0;
    }
}

// box (6 keys) and centroid box (6 keys) of each task: lo as min keys, hi as max keys
__global__ void k_task_reset(uint32_t T, uint64_t* box, uint64_t* cbox, uint32_t* bin_cnt, uint64_t* bin_box) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    for (int a = 0; a < 3; a++) {
        box[6 * t + a] = kKeyPosInf;
        box[6 * t + 3 + a] = kKeyNegInf;
        cbox[6 * t + a] = kKeyPosInf;
        cbox[6 * t + 3 + a] = kKeyNegInf;
    }
    for (int k = 0; k < 3 * kBins; k++) {
        bin_cnt[(size_t)t * 3 * kBins + k] = 0;
        uint64_t* b = bin_box + ((size_t)t * 3 * kBins + k) * 6;
        for (int a = 0; a < 3; a++) {
            b[a] = kKeyPosInf;
            b[3 + a] = kKeyNegInf;
        }
    }
}

__device__ __forceinline__ uint64_t wmin(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wmax(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

__global__ void __launch_bounds__(256) k_bounds(Tri tr, uint32_t n, const uint32_t* idx, const int32_t* seg,
                                                uint64_t* box, uint64_t* cbox) {
    const uint32_t stride = gridDim.x * blockDim.x;
    // every lane iterates the same number of times (wave-level reductions)
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint32_t p = base + threadIdx.x;
        const int32_t t = p < n ? seg[p] : -1;
        uint64_t k[12];
        if (t >= 0) {
            const uint32_t i = idx[p];
            for (int a = 0; a < 3; a++) {
                k[a] = okey(tr.lo[a][i]);
                k[3 + a] = okey(tr.hi[a][i]);
                k[6 + a] = okey(tr.cen[a][i]);
                k[9 + a] = k[6 + a];
            }
        } else {
            for (int a = 0; a < 3; a++) {
                k[a] = k[6 + a] = kKeyPosInf;
                k[3 + a] = k[9 + a] = kKeyNegInf;
            }
        }
        const uint64_t valid = __ballot(t >= 0);
        if (valid == 0) continue;
        const int32_t tw = __shfl(t, __ffsll((unsigned long long)valid) - 1);  // the first valid lane's task
        if (__all(t == tw || t < 0)) {
            // the wave's triangles are in one task: reduce first, one atomic per key
            for (int a = 0; a < 3; a++) {
                k[a] = wmin(k[a]);
                k[3 + a] = wmax(k[3 + a]);
                k[6 + a] = wmin(k[6 + a]);
                k[9 + a] = wmax(k[9 + a]);
            }
            if ((threadIdx.x & 63) == 0) {
                for (int a = 0; a < 3; a++) {
                    atomicMin((unsigned long long*)&box[6 * tw + a], (unsigned long long)k[a]);
                    atomicMax((unsigned long long*)&box[6 * tw + 3 + a], (unsigned long long)k[3 + a]);
                    atomicMin((unsigned long long*)&cbox[6 * tw + a], (unsigned long long)k[6 + a]);
                    atomicMax((unsigned long long*)&cbox[6 * tw + 3 + a], (unsigned long long)k[9 + a]);
                }
            }
        } else if (t >= 0) {
            for (int a = 0; a < 3; a++) {
                atomicMin((unsigned long long*)&box[6 * t + a], (unsigned long long)k[a]);
                atomicMax((unsigned long long*)&box[6 * t + 3 + a], (unsigned long long)k[3 + a]);
                atomicMin((unsigned long long*)&cbox[6 * t + a], (unsigned long long)k[6 + a]);
                atomicMax((unsigned long long*)&cbox[6 * t + 3 + a], (unsigned long long)k[9 + a]);
            }
        }
    }
}

// Binning of every task's triangles: 3 axes x kBins (count, box).  A block
// whose 256 positions all belong to one task accumulates in LDS first.
__global__ void __launch_bounds__(256) k_bin(Tri tr, uint32_t n, const uint32_t* idx, const int32_t* seg,
                                             const uint64_t* cbox, uint32_t* bin_cnt, uint64_t* bin_box) {
    __shared__ uint32_t s_cnt[3 * kBins];
    __shared__ unsigned long long s_box[3 * kBins * 6];
    __shared__ int32_t s_task;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint32_t p = base + threadIdx.x;
        const int32_t t = p < n ? seg[p] : -1;
        if (threadIdx.x == 0) s_task = t;
        __syncthreads();
        const int32_t tb = s_task;
        const bool priv = __syncthreads_and(t == tb || p >= n) && tb >= 0;
        if (priv) {
            for (int k = threadIdx.x; k < 3 * kBins; k += blockDim.x) {
                s_cnt[k] = 0;
                for (int a = 0; a < 3; a++) {
                    s_box[6 * k + a] = kKeyPosInf;
                    s_box[6 * k + 3 + a] = kKeyNegInf;
                }
            }
            __syncthreads();
        }
        if (t >= 0) {
            const uint32_t i = idx[p];
            uint64_t kb[6];
            for (int a = 0; a < 3; a++) {
                kb[a] = okey(tr.lo[a][i]);
                kb[3 + a] = okey(tr.hi[a][i]);
            }
            for (int a = 0; a < 3; a++) {
                const double lo = odec(cbox[6 * t + a]), ext = odec(cbox[6 * t + 3 + a]) - lo;
                if (!(ext > 0.0)) continue;
                const int k = a * kBins + bin_of(tr.cen[a][i], lo, kBins / ext);
                if (priv) {
                    atomicAdd(&s_cnt[k], 1u);
                    for (int q = 0; q < 3; q++) {
                        atomicMin(&s_box[6 * k + q], (unsigned long long)kb[q]);
                        atomicMax(&s_box[6 * k + 3 + q], (unsigned long long)kb[3 + q]);
                    }
                } else {
                    const size_t g = (size_t)t * 3 * kBins + k;
                    atomicAdd(&bin_cnt[g], 1u);
                    for (int q = 0; q < 3; q++) {
                        atomicMin((unsigned long long*)&bin_box[6 * g + q], (unsigned long long)kb[q]);
                        atomicMax((unsigned long long*)&bin_box[6 * g + 3 + q], (unsigned long long)kb[3 + q]);
                    }
                }
            }
        }
        if (priv) {
            __syncthreads();
            for (int k = threadIdx.x; k < 3 * kBins; k += blockDim.x) {
                if (s_cnt[k] == 0) continue;
                const size_t g = (size_t)tb * 3 * kBins + k;
                atomicAdd(&bin_cnt[g], s_cnt[k]);
                for (int q = 0; q < 3; q++) {
                    atomicMin((unsigned long long*)&bin_box[6 * g + q], s_box[6 * k + q]);
                    atomicMax((unsigned long long*)&bin_box[6 * g + 3 + q], s_box[6 * k + 3 + q]);
                }
            }
        }
        __syncthreads();
    }
}

struct Split {
    int32_t axis;     // -1: positional split at mid
    int32_t bin;      // triangles with bin < bin go left
    uint32_t nleft;
    uint32_t leaf;    // 1: the task becomes a leaf
};

// Per task of a level: 1 if it becomes an inner node, its children of more
// than kSmall triangles (next level's tasks) and of at most kSmall (k_small's
// subtrees); an exclusive scan over the tasks numbers them.  Three full u32
// fields: a level of up to n / (kSmall + 1) tasks cannot overflow them.
struct Cnt3 {
    uint32_t inner, big, small;
};
struct Cnt3Sum {
    __host__ __device__ Cnt3 operator()(const Cnt3& a, const Cnt3& b) const {
        return Cnt3{a.inner + b.inner, a.big + b.big, a.small + b.small};
    }
};

// walk_tree.cpp:117-167 for one task (all big tasks have > kSmall >= LMAX
// triangles, so the leaf rule never applies here, but it is kept for symmetry)
__global__ void k_split(uint32_t T, const uint32_t* task_node, const uint32_t* task_b, const uint32_t* task_e,
                        const uint64_t* box, const uint64_t* cbox, const uint32_t* bin_cnt, const uint64_t* bin_box,
                        int lmax, double node_cost, DNode* nodes, Split* split, Cnt3* pack) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    double mn[3], mx[3];
    for (int a = 0; a < 3; a++) {
        mn[a] = odec(box[6 * t + a]);
        mx[a] = odec(box[6 * t + 3 + a]);
    }
    DNode& nd = nodes[task_node[t]];
    for (int a = 0; a < 3; a++) {
        nd.mn[a] = mn[a];
        nd.mx[a] = mx[a];
    }
    const uint32_t cnt = task_e[t] - task_b[t];
    const double A = area(mn, mx);
    double best = __builtin_huge_val();
    int best_axis = -1, best_bin = 0;
    for (int a = 0; a < 3; a++) {
        const double lo = odec(cbox[6 * t + a]), ext = odec(cbox[6 * t + 3 + a]) - lo;
        if (!(ext > 0.0)) continue;
        const uint32_t* bc = bin_cnt + ((size_t)t * 3 + a) * kBins;
        const uint64_t* bb = bin_box + ((size_t)t * 3 + a) * kBins * 6;
        double ra[kBins];
        uint32_t rc[kBins];
        double amn[3], amx[3];
        for (int q = 0; q < 3; q++) {
            amn[q] = __builtin_huge_val();
            amx[q] = -__builtin_huge_val();
        }
        uint32_t c = 0;
        for (int k = kBins - 1; k > 0; k--) {
            for (int q = 0; q < 3; q++) {
                amn[q] = fmin(amn[q], odec(bb[6 * k + q]));
                amx[q] = fmax(amx[q], odec(bb[6 * k + 3 + q]));
            }
            c += bc[k];
            ra[k] = area(amn, amx);
            rc[k] = c;
        }
        for (int q = 0; q < 3; q++) {
            amn[q] = __builtin_huge_val();
            amx[q] = -__builtin_huge_val();
        }
        uint32_t lc = 0;
        for (int k = 1; k < kBins; k++) {
            for (int q = 0; q < 3; q++) {
                amn[q] = fmin(amn[q], odec(bb[6 * (k - 1) + q]));
                amx[q] = fmax(amx[q], odec(bb[6 * (k - 1) + 3 + q]));
            }
            lc += bc[k - 1];
            if (lc == 0 || rc[k] == 0) continue;
            const double cost = (area(amn, amx) * lc + ra[k] * rc[k]) / (A > 0 ? A : 1.0);
            if (cost < best) {
                best = cost;
                best_axis = a;
                best_bin = k;
            }
        }
    }
    Split s{best_axis, best_bin, 0, 0};
    if (cnt <= 1 || (cnt <= (uint32_t)lmax && (best_axis < 0 || (double)cnt <= node_cost + best))) {
        s.leaf = 1;
        nd.left = nd.right = -1;
        nd.first = task_b[t];
        nd.count = cnt;
        split[t] = s;
        pack[t] = Cnt3{0u, 0u, 0u};
        return;
    }
    if (best_axis >= 0) {
        const uint32_t* bc = bin_cnt + ((size_t)t * 3 + best_axis) * kBins;
        for (int k = 0; k < best_bin; k++) s.nleft += bc[k];
        if (s.nleft == 0 || s.nleft == cnt) s.axis = -1;  // the host's mid == b || mid == e case
    }
    if (s.axis < 0) s.nleft = cnt / 2;
    split[t] = s;
    const uint32_t nl = s.nleft, nr = cnt - s.nleft;
    const uint32_t big = (nl > kSmall) + (nr > kSmall), small = 2 - big;
    pack[t] = Cnt3{1u, big, small};  // inner, big children, small children
}

struct Small {
    uint32_t node, b, e;
};

__global__ void k_children(uint32_t T, const uint32_t* task_node, const uint32_t* task_b, const uint32_t* task_e,
                           const Split* split, const Cnt3* off, uint32_t node_base, uint32_t small_base,
                           DNode* nodes, uint32_t* nx_node, uint32_t* nx_b, uint32_t* nx_e, Small* small,
                           int32_t* child_task) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const Split s = split[t];
    child_task[2 * t] = child_task[2 * t + 1] = -1;
    if (s.leaf) return;
    const Cnt3 o = off[t];
    const uint32_t q = o.inner, qb = o.big, qs = o.small;
    const uint32_t b = task_b[t], e = task_e[t];
    const uint32_t cb[2] = {b, b + s.nleft}, ce[2] = {b + s.nleft, e};
    DNode& nd = nodes[task_node[t]];
    nd.left = (int32_t)(node_base + 2 * q);
    nd.right = (int32_t)(node_base + 2 * q + 1);
    nd.first = 0;
    nd.count = 0;
    uint32_t nb = 0, ns = 0;
    for (int c = 0; c < 2; c++) {
        const uint32_t id = node_base + 2 * q + c;
        if (ce[c] - cb[c] > kSmall) {
            const uint32_t k = qb + nb++;
            nx_node[k] = id;
            nx_b[k] = cb[c];
            nx_e[k] = ce[c];
            child_task[2 * t + c] = (int32_t)k;
        } else {
            small[small_base + qs + ns++] = Small{id, cb[c], ce[c]};
        }
    }
}

__global__ void k_flags(Tri tr, uint32_t n, const uint32_t* idx, const int32_t* seg, const uint32_t* task_b,
                        const uint64_t* cbox, const Split* split, uint32_t* flag) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const int32_t t = seg[p];
        uint32_t f = 0;
        if (t >= 0 && !split[t].leaf) {
            const Split s = split[t];
            if (s.axis < 0) {
                f = p - task_b[t] < s.nleft;
            } else {
                const double lo = odec(cbox[6 * t + s.axis]), ext = odec(cbox[6 * t + 3 + s.axis]) - lo;
                f = bin_of(tr.cen[s.axis][idx[p]], lo, kBins / ext) < s.bin;
            }
        }
        flag[p] = f;
    }
}

// stable partition of every inner task's range by the flags (scan = exclusive
// prefix sum of the flags); elements of leaves and small subtrees keep their
// place and leave the level loop (seg -1)
__global__ void k_scatter(uint32_t n, const uint32_t* idx, const int32_t* seg, const uint32_t* task_b,
                          const uint32_t* task_e, const Split* split, const uint32_t* flag, const uint32_t* scan,
                          const int32_t* child_task, uint32_t* idx2, int32_t* seg2) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const int32_t t = seg[p];
        if (t < 0 || split[t].leaf) {
            idx2[p] = idx[p];
            seg2[p] = -1;
            continue;
        }
        const uint32_t b = task_b[t];
        const uint32_t lb = scan[p] - scan[b];  // left elements before p in the task
        const int c = flag[p] ? 0 : 1;
        // (the left count from the flags themselves: every position stays in
        // the task's range even if it disagreed with the bins' count)
        const uint32_t nl = scan[task_e[t]] - scan[b];
        const uint32_t np = c == 0 ? b + lb : b + nl + (p - b - lb);
        idx2[np] = idx[p];
        seg2[np] = child_task[2 * t + c];
    }
}

// One thread per small subtree: walk_tree.cpp's loop (binned SAH, leaf rule,
// in-place partition) over its range; node ids from a global counter.
__global__ void k_small(Tri tr, uint32_t nsmall, const Small* small, uint32_t* idx, DNode* nodes,
                        uint32_t* node_ctr, int lmax, double node_cost) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsmall) return;
    struct Job { uint32_t node, b, e; };
    Job st[2 * kSmall];
    int sp = 0;
    st[sp++] = Job{small[s].node, small[s].b, small[s].e};
    while (sp > 0) {
        const Job j = st[--sp];
        double mn[3], mx[3], cmn[3], cmx[3];
        for (int a = 0; a < 3; a++) {
            mn[a] = cmn[a] = __builtin_huge_val();
            mx[a] = cmx[a] = -__builtin_huge_val();
        }
        for (uint32_t p = j.b; p < j.e; p++) {
            const uint32_t i = idx[p];
            for (int a = 0; a < 3; a++) {
                mn[a] = fmin(mn[a], tr.lo[a][i]);
                mx[a] = fmax(mx[a], tr.hi[a][i]);
                cmn[a] = fmin(cmn[a], tr.cen[a][i]);
                cmx[a] = fmax(cmx[a], tr.cen[a][i]);
            }
        }
        DNode& nd = nodes[j.node];
        for (int a = 0; a < 3; a++) {
            nd.mn[a] = mn[a];
            nd.mx[a] = mx[a];
        }
        const uint32_t cnt = j.e - j.b;
        nd.left = nd.right = -1;
        nd.first = j.b;
        nd.count = cnt;
        if (cnt <= 1) continue;
        const double A = area(mn, mx);
        double best = __builtin_huge_val();
        int best_axis = -1, best_bin = 0;
        for (int a = 0; a < 3; a++) {
            const double lo = cmn[a], ext = cmx[a] - cmn[a];
            if (!(ext > 0.0)) continue;
            const double scale = kBins / ext;
            double bmn[kBins][3], bmx[kBins][3];
            uint32_t bc[kBins];
            for (int k = 0; k < kBins; k++) {
                bc[k] = 0;
                for (int q = 0; q < 3; q++) {
                    bmn[k][q] = __builtin_huge_val();
                    bmx[k][q] = -__builtin_huge_val();
                }
            }
            for (uint32_t p = j.b; p < j.e; p++) {
                const uint32_t i = idx[p];
                const int k = bin_of(tr.cen[a][i], lo, scale);
                bc[k]++;
                for (int q = 0; q < 3; q++) {
                    bmn[k][q] = fmin(bmn[k][q], tr.lo[q][i]);
                    bmx[k][q] = fmax(bmx[k][q], tr.hi[q][i]);
                }
            }
            double ra[kBins];
            uint32_t rc[kBins];
            double amn[3], amx[3];
            for (int q = 0; q < 3; q++) {
                amn[q] = __builtin_huge_val();
                amx[q] = -__builtin_huge_val();
            }
            uint32_t c = 0;
            for (int k = kBins - 1; k > 0; k--) {
                for (int q = 0; q < 3; q++) {
                    amn[q] = fmin(amn[q], bmn[k][q]);
                    amx[q] = fmax(amx[q], bmx[k][q]);
                }
                c += bc[k];
                ra[k] = area(amn, amx);
                rc[k] = c;
            }
            for (int q = 0; q < 3; q++) {
                amn[q] = __builtin_huge_val();
                amx[q] = -__builtin_huge_val();
            }
            uint32_t lc = 0;
            for (int k = 1; k < kBins; k++) {
                for (int q = 0; q < 3; q++) {
                    amn[q] = fmin(amn[q], bmn[k - 1][q]);
                    amx[q] = fmax(amx[q], bmx[k - 1][q]);
                }
                lc += bc[k - 1];
                if (lc == 0 || rc[k] == 0) continue;
                const double cost = (area(amn, amx) * lc + ra[k] * rc[k]) / (A > 0 ? A : 1.0);
                if (cost < best) {
                    best = cost;
                    best_axis = a;
                    best_bin = k;
                }
            }
        }
        if (cnt <= (uint32_t)lmax && (best_axis < 0 || (double)cnt <= node_cost + best)) continue;  // leaf
        uint32_t mid;
        if (best_axis < 0) {
            mid = j.b + cnt / 2;
        } else {
            const double lo = cmn[best_axis], scale = kBins / (cmx[best_axis] - cmn[best_axis]);
            uint32_t w = j.b;  // in-place partition (order inside a side is free)
            for (uint32_t p = j.b; p < j.e; p++) {
                const uint32_t i = idx[p];
                if (bin_of(tr.cen[best_axis][i], lo, scale) < best_bin) {
                    idx[p] = idx[w];
                    idx[w] = i;
                    w++;
                }
            }
            mid = w;
            if (mid == j.b || mid == j.e) mid = j.b + cnt / 2;
        }
        const uint32_t l = atomicAdd(node_ctr, 2u);
        nd.left = (int32_t)l;
        nd.right = (int32_t)l + 1;
        nd.first = 0;
        nd.count = 0;
        st[sp++] = Job{l + 1, mid, j.e};
        st[sp++] = Job{l, j.b, mid};
    }
}

#define HT(expr)                                                                                    \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) throw rt::Error{RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
    } while (0)

// device allocations of one build, freed on every exit
struct Pool {
    std::vector<void*> ptrs;
    template <class T>
    T* get(size_t count) {
        void* p = nullptr;
        HT(hipMalloc(&p, count * sizeof(T) + 16));
        ptrs.push_back(p);
        return static_cast<T*>(p);
    }
    ~Pool() {
        for (void* p : ptrs) (void)hipFree(p);
    }
};

}  // namespace

namespace rt {

WalkTree build_walk_tree_device(const Soup& s, int device, int lmax, double node_cost) {
    const uint32_t n = (uint32_t)s.n;
    if (n <= 1) return build_walk_tree(s);
    int prev = -1;
    HT(hipGetDevice(&prev));
    HT(hipSetDevice(device));
    struct Restore {
        int d;
        ~Restore() {
            if (d >= 0) (void)hipSetDevice(d);
        }
    } restore{prev};
    hipStream_t st = nullptr;
    HT(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct SDel {
        hipStream_t s;
        ~SDel() { (void)hipStreamDestroy(s); }
    } sdel{st};
    Pool P;
    Tri tr;
    double* dlo = P.get<double>(6 * (size_t)n);
    double* dcen = P.get<double>(3 * (size_t)n);
    for (int a = 0; a < 3; a++) {
        tr.lo[a] = dlo + (size_t)a * n;
        tr.hi[a] = dlo + (size_t)(3 + a) * n;
        tr.cen[a] = dcen + (size_t)a * n;
        HT(hipMemcpyAsync((void*)tr.lo[a], s.lo[a].data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        HT(hipMemcpyAsync((void*)tr.hi[a], s.hi[a].data(), n * sizeof(double), hipMemcpyHostToDevice, st));
    }
    uint32_t* idx = P.get<uint32_t>(n);
    uint32_t* idx2 = P.get<uint32_t>(n);
    int32_t* seg = P.get<int32_t>(n);
    int32_t* seg2 = P.get<int32_t>(n);
    uint32_t* flag = P.get<uint32_t>(n + 1);
    uint32_t* scan = P.get<uint32_t>(n + 1);
    const uint32_t tcap = n / (kSmall + 1) + 2;  // big tasks hold > kSmall triangles each
    uint32_t* tnode[2] = {P.get<uint32_t>(tcap), P.get<uint32_t>(tcap)};
    uint32_t* tb[2] = {P.get<uint32_t>(tcap), P.get<uint32_t>(tcap)};
    uint32_t* te[2] = {P.get<uint32_t>(tcap), P.get<uint32_t>(tcap)};
    uint64_t* box = P.get<uint64_t>(6 * (size_t)tcap);
    uint64_t* cbox = P.get<uint64_t>(6 * (size_t)tcap);
    uint32_t* bin_cnt = P.get<uint32_t>((size_t)tcap * 3 * kBins);
    uint64_t* bin_box = P.get<uint64_t>((size_t)tcap * 3 * kBins * 6);
    Split* split = P.get<Split>(tcap);
    Cnt3* pack = P.get<Cnt3>(tcap + 1);
    Cnt3* off = P.get<Cnt3>(tcap + 1);
    int32_t* child_task = P.get<int32_t>(2 * (size_t)tcap);
    Small* small = P.get<Small>(n);
    DNode* nodes = P.get<DNode>(2 * (size_t)n);
    uint32_t* node_ctr = P.get<uint32_t>(1);
    // hipcub scan workspaces (the larger of the two scans)
    size_t ws_a = 0, ws_b = 0;
    HT(hipcub::DeviceScan::ExclusiveSum(nullptr, ws_a, flag, scan, n + 1, st));
    HT(hipcub::DeviceScan::ExclusiveScan(nullptr, ws_b, pack, off, Cnt3Sum{}, Cnt3{0u, 0u, 0u}, tcap + 1, st));
    void* ws = P.get<uint8_t>(std::max(ws_a, ws_b));
    const size_t ws_bytes = std::max(ws_a, ws_b);

    const dim3 blk(256);
    const unsigned egrid = std::min<unsigned>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_init, dim3(egrid), blk, 0, st, tr, n, idx, seg);
    uint32_t T = 0, node_base = 1, nsmall = 0;
    int cur = 0;
    if (n > kSmall) {
        const uint32_t h[3] = {0u, 0u, n};
        HT(hipMemcpyAsync(tnode[0], &h[0], 4, hipMemcpyHostToDevice, st));
        HT(hipMemcpyAsync(tb[0], &h[1], 4, hipMemcpyHostToDevice, st));
        HT(hipMemcpyAsync(te[0], &h[2], 4, hipMemcpyHostToDevice, st));
        T = 1;
    } else {
        const Small root{0u, 0u, n};
        HT(hipMemcpyAsync(small, &root, sizeof root, hipMemcpyHostToDevice, st));
        nsmall = 1;
    }
    while (T > 0) {
        const unsigned tg = (T + 255) / 256;
        hipLaunchKernelGGL(k_task_reset, dim3(tg), blk, 0, st, T, box, cbox, bin_cnt, bin_box);
        hipLaunchKernelGGL(k_bounds, dim3(egrid), blk, 0, st, tr, n, idx, seg, box, cbox);
        hipLaunchKernelGGL(k_bin, dim3(egrid), blk, 0, st, tr, n, idx, seg, cbox, bin_cnt, bin_box);
        hipLaunchKernelGGL(k_split, dim3(tg), blk, 0, st, T, tnode[cur], tb[cur], te[cur], box, cbox, bin_cnt,
                           bin_box, lmax, node_cost, nodes, split, pack);
        HT(hipMemsetAsync(pack + T, 0, sizeof(Cnt3), st));
        size_t wsb = ws_bytes;
        HT(hipcub::DeviceScan::ExclusiveScan(ws, wsb, pack, off, Cnt3Sum{}, Cnt3{0u, 0u, 0u}, T + 1, st));
        Cnt3 tot{0u, 0u, 0u};
        HT(hipMemcpyAsync(&tot, off + T, sizeof tot, hipMemcpyDeviceToHost, st));
        hipLaunchKernelGGL(k_children, dim3(tg), blk, 0, st, T, tnode[cur], tb[cur], te[cur], split, off, node_base,
                           nsmall, nodes, tnode[cur ^ 1], tb[cur ^ 1], te[cur ^ 1], small, child_task);
        hipLaunchKernelGGL(k_flags, dim3(egrid), blk, 0, st, tr, n, idx, seg, tb[cur], cbox, split, flag);
        HT(hipMemsetAsync(flag + n, 0, sizeof(uint32_t), st));
        wsb = ws_bytes;
        HT(hipcub::DeviceScan::ExclusiveSum(ws, wsb, flag, scan, n + 1, st));
        hipLaunchKernelGGL(k_scatter, dim3(egrid), blk, 0, st, n, idx, seg, tb[cur], te[cur], split, flag, scan,
                           child_task, idx2, seg2);
        HT(hipGetLastError());
        HT(hipStreamSynchronize(st));  // tot: this level's inner / big / small children
        std::swap(idx, idx2);
        std::swap(seg, seg2);
        const uint32_t inner = tot.inner, big = tot.big, sm = tot.small;
        node_base += 2 * inner;
        nsmall += sm;
        T = big;
        cur ^= 1;
    }
    HT(hipMemcpyAsync(node_ctr, &node_base, sizeof node_base, hipMemcpyHostToDevice, st));
    if (nsmall > 0)
        hipLaunchKernelGGL(k_small, dim3((nsmall + 63) / 64), dim3(64), 0, st, tr, nsmall, small, idx, nodes, node_ctr,
                           lmax, node_cost);
    HT(hipGetLastError());
    uint32_t nn = 0;
    HT(hipMemcpyAsync(&nn, node_ctr, sizeof nn, hipMemcpyDeviceToHost, st));
    HT(hipStreamSynchronize(st));
    WalkTree w;
    w.nodes.resize(nn);
    w.order.resize(n);
    HT(hipMemcpyAsync(w.nodes.data(), nodes, (size_t)nn * sizeof(DNode), hipMemcpyDeviceToHost, st));
    HT(hipMemcpyAsync(w.order.data(), idx, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HT(hipStreamSynchronize(st));
    return w;
}

}  // namespace rt
