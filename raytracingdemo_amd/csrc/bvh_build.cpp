// Host BVH feeder: rebuilds the reference's StackBVH tree exactly
// (src/stack_bvh.hpp:26-608) and flattens it into the device format.
//
// The tree has to be *the same tree* as the reference's, not merely a good
// one: the reference only reports a triangle if every ancestor's fp64 slab
// test passes (stack_bvh.hpp:623), so exact parity on grazing rays depends on
// the ancestor boxes.  The partition arithmetic below therefore keeps the
// reference's operation order, and the sorts use libstdc++'s std::sort /
// std::nth_element with the same comparator on the same input sequence, which
// yields the same permutation as sorting the reference's Primitive* vector.
// Compiled with -ffp-contract=off (the reference's x86-64 -O0 build had no FMA).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>
#include <cstdlib>
#include <exception>
#include <system_error>
#include <thread>

#include "rt_internal.h"

namespace rt {
namespace {

constexpr double DMAX = std::numeric_limits<double>::max();
constexpr double DLOW = std::numeric_limits<double>::lowest();

inline double smin(double a, double b) { return (b < a) ? b : a; }  // std::min
inline double smax(double a, double b) { return (a < b) ? b : a; }  // std::max

struct Box {
    double mn[3] = {DMAX, DMAX, DMAX};
    double mx[3] = {DLOW, DLOW, DLOW};
    void grow(const Box& o) {
        for (int a = 0; a < 3; a++) { mn[a] = smin(mn[a], o.mn[a]); mx[a] = smax(mx[a], o.mx[a]); }
    }
};
// calculateSurfaceArea (stack_bvh.hpp:65-69)
inline double area(const Box& b) {
    double ex = b.mx[0] - b.mn[0], ey = b.mx[1] - b.mn[1], ez = b.mx[2] - b.mn[2];
    return 2.0 * (ex * ey + ey * ez + ez * ex);
}

// Threads alive in the builders at once, over every spawn site (subtrees
// and the sorts inside them nest): past the budget work runs inline.
std::atomic<int> g_live_threads{0};
int thread_budget() {
    static const int b = (int)std::max(2u, std::min(32u, std::thread::hardware_concurrency()));
    return b;
}

// Runs f on a new thread kept in `th`, or here when the thread budget is
// spent or no thread can be made (the result is the same either way).
template <class F>
void spawn(std::vector<std::thread>& th, F&& f) {
    if (g_live_threads.fetch_add(1) >= thread_budget()) {
        g_live_threads.fetch_sub(1);
        f();
        return;
    }
    try {
        th.emplace_back([f]() mutable {
            f();
            g_live_threads.fetch_sub(1);
        });
    } catch (const std::system_error&) {
        g_live_threads.fetch_sub(1);
        f();
    }
}

struct Builder {
    const Soup& s;
    std::vector<uint32_t> order;

    explicit Builder(const Soup& soup) : s(soup) {}

    Box tri_box(uint32_t t) const {
        Box b;
        for (int a = 0; a < 3; a++) { b.mn[a] = s.lo[a][t]; b.mx[a] = s.hi[a][t]; }
        return b;
    }
    // findBounds (stack_bvh.hpp:26-52): the per-axis min/max chain; an empty
    // range is the zero box.
    Box bounds(int64_t lo, int64_t hi) const {
        Box b;
        if (lo == hi) { for (int a = 0; a < 3; a++) b.mn[a] = b.mx[a] = 0.0; return b; }
        for (int64_t i = lo; i < hi; i++) {
            uint32_t t = order[i];
            for (int a = 0; a < 3; a++) { b.mn[a] = smin(b.mn[a], s.lo[a][t]); b.mx[a] = smax(b.mx[a], s.hi[a][t]); }
        }
        return b;
    }
    // std::sort of the range by centre.  Large ranges run the same introsort
    // with the right side of the top partitions on threads (par_introsort):
    // the permutation is std::sort's, ties included.
    bool threads = true;
    void sort_range(int64_t lo, int64_t hi, int axis) {
        const double* c = s.c[axis].data();
        auto less = [c](uint32_t p, uint32_t q) { return c[p] < c[q]; };
        auto first = order.begin() + lo, last = order.begin() + hi;
        if (!threads || hi - lo < 65536) { std::sort(first, last, less); return; }
        const int64_t n = hi - lo;
        par_introsort(first, last, 2 * (63 - __builtin_clzll((uint64_t)n)), less, std::max<int64_t>(16384, n / 32));
        // std::sort's closing pass: insertion sort of the whole range (every
        // element is at most 16 places from home, inside its partition)
        for (auto i = first + 1; i < last; ++i) {
            const uint32_t v = *i;
            auto j = i;
            for (; j > first && less(v, *(j - 1)); --j) *j = *(j - 1);
            *j = v;
        }
    }
    // The introsort loop of libstdc++'s std::sort (bits/stl_algo.h:
    // median-of-three of first + 1, middle, last - 1 moved to first, Hoare
    // partition about it, recursion on the right side, loop on the left, heap
    // sort past 2 log2(n) levels, stop at 16 elements).  The two sides of a
    // partition are disjoint and each is processed the same way wherever it
    // runs, so right sides of at least par_min elements go to threads.
    template <class It, class C>
    static void par_introsort(It first, It last, int depth, C less, int64_t par_min) {
        std::vector<std::thread> th;
        while (last - first > 16) {
            if (depth == 0) { std::partial_sort(first, last, last, less); break; }
            --depth;
            It a = first + 1, b = first + (last - first) / 2, c = last - 1;
            It med = less(*a, *b) ? (less(*b, *c) ? b : (less(*a, *c) ? c : a))
                                  : (less(*a, *c) ? a : (less(*b, *c) ? c : b));
            std::iter_swap(first, med);
            It lo = first + 1, hi = last;
            for (;;) {
                while (less(*lo, *first)) ++lo;
                --hi;
                while (less(*first, *hi)) --hi;
                if (!(lo < hi)) break;
                std::iter_swap(lo, hi);
                ++lo;
            }
            if (last - lo >= par_min) spawn(th, [=] { par_introsort(lo, last, depth, less, par_min); });
            else par_introsort(lo, last, depth, less, par_min);
            last = lo;
        }
        for (auto& x : th) x.join();
    }
    static bool leaf(int64_t n, int k) { return n <= (int64_t)k || k < 2; }  // isLeaf :71-76

    // medianSplit (:79-100)
    std::vector<size_t> median(int64_t lo, int64_t hi, int axis, int k) {
        const int64_t n = hi - lo;
        if (leaf(n, k)) return {};
        std::vector<size_t> sp;
        for (int i = 1; i < k; ++i) {
            size_t x = (size_t)(n * i) / k;
            if (x == 0 || x >= (size_t)n) break;
            sp.push_back(x);
        }
        const double* c = s.c[axis].data();
        auto base = order.begin() + lo;
        auto from = base;
        for (size_t x : sp) {
            std::nth_element(from, base + (std::ptrdiff_t)x, order.begin() + hi,
                             [c](uint32_t p, uint32_t q) { return c[p] < c[q]; });
            from = base + x + 1;
        }
        return sp;
    }

    // Greedy "split the most expensive segment" over `cells` (:153-236 and
    // :342-438).  cost(seg) = area(bounds of cells) * count(cells); the split
    // minimises left area*count + right area*count over cell boundaries.
    template <bool BINNED>
    std::vector<size_t> greedy(const std::vector<Box>& cell, const std::vector<int>& cnt, int k) {
        struct Seg { size_t b, e; };
        std::vector<Seg> segs{{0, cell.size()}};
        auto seg_cost = [&](const Seg& g) {
            Box b;
            int64_t n = 0;
            for (size_t i = g.b; i < g.e; ++i) b.grow(cell[i]);
            if (BINNED) { for (size_t i = g.b; i < g.e; ++i) n += cnt[i]; }
            else n = (int64_t)(g.e - g.b);
            return area(b) * (double)n;
        };
        std::vector<size_t> splits;
        std::vector<Box> pre, suf;
        while (segs.size() < (size_t)k) {
            size_t pick = SIZE_MAX;
            double worst = -1.0;
            for (size_t i = 0; i < segs.size(); ++i) {
                if (segs[i].e - segs[i].b < 2) continue;
                double c = seg_cost(segs[i]);
                if (c > worst) { worst = c; pick = i; }
            }
            if (pick == SIZE_MAX) break;
            const Seg g = segs[pick];
            const size_t m = g.e - g.b;
            pre.assign(m, Box{});
            suf.assign(m, Box{});
            pre[0] = cell[g.b];
            for (size_t q = 1; q < m; ++q) { pre[q] = pre[q - 1]; pre[q].grow(cell[g.b + q]); }
            suf[m - 1] = cell[g.e - 1];
            for (size_t q = m - 1; q-- > 0;) { suf[q] = suf[q + 1]; suf[q].grow(cell[g.b + q]); }
            size_t best_at = 1;
            double best = DMAX;
            if (BINNED) {
                int left = 0, right = 0;
                for (size_t q = 0; q < m; ++q) right += cnt[g.b + q];
                for (size_t x = 1; x < m; ++x) {
                    left += cnt[g.b + x - 1];
                    right -= cnt[g.b + x - 1];
                    double c = area(pre[x - 1]) * left + area(suf[x]) * right;
                    if (c < best) { best = c; best_at = x; }
                }
                size_t prims = 0;  // primitives in cells [0, g.b + best_at)
                for (size_t q = 0; q < g.b + best_at; ++q) prims += (size_t)cnt[q];
                splits.push_back(prims);
            } else {
                for (size_t x = 1; x < m; ++x) {
                    double c = area(pre[x - 1]) * x + area(suf[x]) * (m - x);
                    if (c < best) { best = c; best_at = x; }
                }
                splits.push_back(g.b + best_at);
            }
            segs.erase(segs.begin() + pick);
            segs.push_back({g.b, g.b + best_at});
            segs.push_back({g.b + best_at, g.e});
        }
        return splits;
    }

    // sahSplit (:103-239): cells are the sorted primitives.
    std::vector<size_t> sah(int64_t lo, int64_t hi, int axis, int k) {
        if (leaf(hi - lo, k)) return {};
        sort_range(lo, hi, axis);
        std::vector<Box> cell((size_t)(hi - lo));
        for (int64_t i = lo; i < hi; i++) cell[i - lo] = tri_box(order[i]);
        return greedy<false>(cell, {}, k);
    }

    // binnedSahSplit (:241-449): 16 centre bins on `axis`.
    std::vector<size_t> binned(int64_t lo, int64_t hi, int axis, int k) {
        constexpr int NB = 16;
        if (leaf(hi - lo, k)) return {};
        sort_range(lo, hi, axis);
        const double* c = s.c[axis].data();
        double cmin = DMAX, cmax = DLOW;
        for (int64_t i = lo; i < hi; ++i) { cmin = smin(cmin, c[order[i]]); cmax = smax(cmax, c[order[i]]); }
        double range = cmax - cmin;
        if (range < 1e-10) range = 1.0;
        std::vector<Box> bin(NB);
        std::vector<int> cnt(NB, 0);
        for (int64_t i = lo; i < hi; ++i) {
            uint32_t t = order[i];
            int b = static_cast<int>(((c[t] - cmin) / range) * NB);
            b = std::clamp(b, 0, NB - 1);
            bin[b].grow(tri_box(t));
            cnt[b]++;
        }
        std::vector<size_t> sp = greedy<true>(bin, cnt, k);
        std::sort(sp.begin(), sp.end());
        sp.erase(std::unique(sp.begin(), sp.end()), sp.end());
        return sp;
    }
};

// calculateLongestAxis (:54-63)
int longest_axis(const double mn[3], const double mx[3]) {
    double ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
    if (ey > ex && ey >= ez) return 1;
    if (ez > ex && ez >= ey) return 2;
    return 0;
}

// Runs fn(lo, hi) over [0, n) in contiguous chunks on up to 16 threads (each
// chunk writes only its own outputs, so the result does not depend on the
// split).  Small ranges run inline.
template <class F>
void parallel_for(uint64_t n, F fn) {
    const uint64_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint64_t T = std::min<uint64_t>(hw, n / 16384);
    if (T <= 1) { fn(uint64_t(0), n); return; }
    std::vector<std::thread> th;
    const uint64_t per = (n + T - 1) / T;
    for (uint64_t c = 1; c < T; c++) {
        const uint64_t a = std::min(n, c * per), b = std::min(n, (c + 1) * per);
        spawn(th, [&fn, a, b] { fn(a, b); });
    }
    fn(uint64_t(0), std::min(n, per));
    for (auto& x : th) x.join();
}

}  // namespace

Soup make_soup(const double* tri_v, uint64_t n) {
    Soup s;
    s.n = n;
    s.v.resize(n * 9);
    for (int a = 0; a < 3; a++) { s.c[a].resize(n); s.lo[a].resize(n); s.hi[a].resize(n); }
    s.normal.resize(n * 3);
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
    std::memcpy(s.v.data() + lo * 9, tri_v + lo * 9, (hi - lo) * 9 * sizeof(double));
    for (uint64_t i = lo; i < hi; i++) {
        const double* p = tri_v + i * 9;
        for (int a = 0; a < 3; a++) {
            double x0 = p[a], x1 = p[3 + a], x2 = p[6 + a];
            // centre = (v0 + v1 + v2) * (1.0/3)  (triangle.hpp:18)
            s.c[a][i] = ((x0 + x1) + x2) * (1.0 / 3);
            // std::min({..}) / std::max({..}): first extreme wins
            double m = x0; if (x1 < m) m = x1; if (x2 < m) m = x2;
            double M = x0; if (M < x1) M = x1; if (M < x2) M = x2;
            s.lo[a][i] = m;
            s.hi[a][i] = M;
        }
        // normal = cross(v1 - v0, v2 - v0).normalize()  (triangle.hpp:17)
        double ax = p[3] - p[0], ay = p[4] - p[1], az = p[5] - p[2];
        double bx = p[6] - p[0], by = p[7] - p[1], bz = p[8] - p[2];
        double nx = ay * bz - az * by, ny = az * bx - ax * bz, nz = ax * by - ay * bx;
        double len = std::sqrt(nx * nx + ny * ny + nz * nz);
        if (len == 0) { nx = ny = nz = 0; } else { nx = nx / len; ny = ny / len; nz = nz / len; }
        s.normal[i * 3] = nx; s.normal[i * 3 + 1] = ny; s.normal[i * 3 + 2] = nz;
    }
    });
    return s;
}

namespace {

// Splits node n (index ni of its vector) with the reference's partition and
// returns its children (:520-568): bounds per child range, parent = ni.  An
// empty result is a leaf.
std::vector<RNode> split_node(Builder& B, int algo, int pk, const RNode& n, int32_t ni) {
    const int64_t lo = n.begin, hi = n.end;
    if (hi - lo <= 1) return {};
    const int axis = longest_axis(n.mn, n.mx);
    std::vector<size_t> sp = algo == RT_ALGO_MEDIAN ? B.median(lo, hi, axis, pk)
                             : algo == RT_ALGO_SAH  ? B.sah(lo, hi, axis, pk)
                                                     : B.binned(lo, hi, axis, pk);
    if (sp.empty()) return {};
    std::sort(sp.begin(), sp.end());
    std::vector<RNode> kids;
    int64_t from = lo;
    auto add_child = [&](int64_t a, int64_t b) {
        RNode c;
        c.begin = a;
        c.end = b;
        c.parent = ni;
        Box bx = B.bounds(a, b);
        std::memcpy(c.mn, bx.mn, sizeof bx.mn);
        std::memcpy(c.mx, bx.mx, sizeof bx.mx);
        kids.push_back(std::move(c));
    };
    for (size_t x : sp) {
        if (x == 0 || x >= (size_t)(hi - lo)) throw Error{RT_ERR_OUT_OF_RANGE, "invalid split position"};
        int64_t to = lo + (int64_t)x;
        if (from >= to) throw Error{RT_ERR_OUT_OF_RANGE, "Invalid iterator range"};
        add_child(from, to);
        from = to;
    }
    add_child(from, hi);
    return kids;
}

// The reference's build loop (work stack, :520-568) below nodes[0].  Node ids
// follow its numbering: a node's children are appended when it is split, and
// the stack is LIFO, so the descendants of a node's last child come next,
// then those of the child before it, and so on.
void grow(Builder& B, int algo, int pk, std::vector<RNode>& nodes) {
    std::vector<int32_t> work{0};
    while (!work.empty()) {
        int32_t ni = work.back();
        work.pop_back();
        std::vector<RNode> kids = split_node(B, algo, pk, nodes[ni], ni);
        for (RNode& c : kids) {
            nodes[ni].kids.push_back((int32_t)nodes.size());
            nodes.push_back(std::move(c));
        }
        for (int32_t c : nodes[ni].kids) work.push_back(c);
    }
}

// The same tree with the subtrees of large nodes built on threads.  Every
// split reads and permutes only its own range of B.order, so subtrees are
// independent; the numbering above makes the descendants of child j one
// contiguous id range, so the subtrees built apart (each numbered from its own
// root = 0) are spliced in with an offset: children at 1..k, then child k's
// descendants, then child k-1's, ...  The result equals grow()'s node for node.
std::vector<RNode> grow_parallel(Builder& B, int algo, int pk, RNode root, int64_t par_min) {
    std::vector<RNode> out;
    if (root.end - root.begin < par_min) {
        out.push_back(std::move(root));
        grow(B, algo, pk, out);
        return out;
    }
    std::vector<RNode> kids = split_node(B, algo, pk, root, 0);
    const size_t k = kids.size();
    std::vector<std::vector<RNode>> sub(k);
    std::vector<std::exception_ptr> err(k);
    std::vector<std::thread> th;
    auto run = [&](size_t j) {
        try {
            RNode c = kids[j];
            c.parent = -1;
            sub[j] = grow_parallel(B, algo, pk, std::move(c), par_min);
        } catch (...) { err[j] = std::current_exception(); }
    };
    for (size_t j = 0; j + 1 < k; j++) spawn(th, [&run, j] { run(j); });
    if (k) run(k - 1);
    for (auto& x : th) x.join();
    for (auto& e : err) if (e) std::rethrow_exception(e);
    // splice: base[j] = id of child j's first descendant
    std::vector<int32_t> base(k);
    int32_t next = (int32_t)(1 + k);
    for (size_t j = k; j-- > 0;) { base[j] = next; next += (int32_t)sub[j].size() - 1; }
    out.reserve((size_t)next);
    out.push_back(std::move(root));
    for (size_t j = 0; j < k; j++) out[0].kids.push_back((int32_t)(1 + j));
    auto remap = [&](size_t j, int32_t x) { return x == 0 ? (int32_t)(1 + j) : base[j] + x - 1; };
    for (size_t j = 0; j < k; j++) {  // the children themselves (ids 1..k)
        RNode c = std::move(sub[j][0]);
        c.parent = 0;
        for (int32_t& q : c.kids) q = remap(j, q);
        out.push_back(std::move(c));
    }
    for (size_t j = k; j-- > 0;)
        for (size_t x = 1; x < sub[j].size(); x++) {
            RNode c = std::move(sub[j][x]);
            c.parent = remap(j, c.parent);
            for (int32_t& q : c.kids) q = remap(j, q);
            out.push_back(std::move(c));
        }
    return out;
}

}  // namespace

Tree build_tree(const Soup& s, int algo, int k, int collapse) {
    if (algo < 0 || algo > 2) throw Error{RT_ERR_OUT_OF_RANGE, "Unknown algorithm"};
    if (!(k == 2 || k == 4 || k == 8 || k == 16)) throw Error{RT_ERR_INVALID_ARGUMENT, "Unsupported bvh degree"};
    const int pk = collapse ? 2 : k;  // the -c variants partition 2-way (main.cpp:128-139)
    Builder B(s);
    B.order.resize(s.n);
    std::iota(B.order.begin(), B.order.end(), 0u);
    Tree t;
    RNode root;
    root.begin = 0;
    root.end = (int64_t)s.n;
    if (s.n == 0) {
        for (int a = 0; a < 3; a++) root.mn[a] = root.mx[a] = 0.0;
        t.nodes.push_back(root);
        return t;
    }
    {
        Box b = B.bounds(0, root.end);
        std::memcpy(root.mn, b.mn, sizeof b.mn);
        std::memcpy(root.mx, b.mx, sizeof b.mx);
    }
    // subtrees of at least par_min primitives go to threads (RT_BUILD_THREADS=1:
    // the serial loop, for A/B)
    const char* bt = std::getenv("RT_BUILD_THREADS");
    const bool serial = bt && std::atoi(bt) == 1;
    B.threads = !serial;
    const int64_t par_min = std::max<int64_t>(4096, (int64_t)s.n / 256);
    t.nodes = serial ? std::vector<RNode>{root} : grow_parallel(B, algo, pk, root, par_min);
    if (serial) grow(B, algo, pk, t.nodes);
    if (collapse) {
        // collapse (:574-608), log2(k)-1 passes (main.cpp:208)
        const int passes = static_cast<int>(std::log2(k)) - 1;
        for (int p = 0; p < passes; p++) {
            std::vector<int32_t> st{0};
            while (!st.empty()) {
                int32_t ni = st.back();
                st.pop_back();
                if (t.nodes[ni].kids.empty()) continue;
                std::vector<int32_t> nk;
                for (int32_t c : t.nodes[ni].kids) {
                    if (!t.nodes[c].kids.empty()) nk.insert(nk.end(), t.nodes[c].kids.begin(), t.nodes[c].kids.end());
                    else nk.push_back(c);
                }
                t.nodes[ni].kids = nk;
                for (int32_t c : nk) { t.nodes[c].parent = ni; st.push_back(c); }
            }
        }
    }
    t.order = std::move(B.order);
    return t;
}

// ------------------------------------------------------------------ flatten
namespace {

inline float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}
inline float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

struct Flattener {
    const Soup& s;
    const Tree& t;
    Flat& f;
    int W;
    uint32_t nb;
    uint32_t wide_depth = 0;             // max wide nodes on a root-leaf path

    Flattener(const Soup& s_, const Tree& t_, Flat& f_) : s(s_), t(t_), f(f_), W(f_.width), nb(rt_node_bytes(f_.width)) {}

    // fp32 conservative (outward-rounded) box of a real node; the kernel adds a
    // per-frame margin to the planes (render.hip, "pad")
    void box32(const double mn[3], const double mx[3], float out[6]) const {
        for (int a = 0; a < 3; a++) {
            out[2 * a] = round_down(mn[a]);
            out[2 * a + 1] = round_up(mx[a]);
        }
    }

    uint32_t alloc_node() {
        uint32_t id = (uint32_t)f.n_wide++;
        f.wide.resize(f.n_wide * nb, 0);
        // empty slot: an inverted box (lo = +inf, hi = -inf on every axis)
        // and ref RT_INVALID_REF.  A slab test that takes each axis's near
        // plane by the ray's direction sign (the packet walks' per-octant
        // tests) fails it for every ray, so those walks need not mask the
        // slots past the node's valid count; the general test and the
        // per-lane walks still check the count or the ref
        uint32_t* p = reinterpret_cast<uint32_t*>(f.wide.data() + (size_t)id * nb);
        for (int c = 0; c < W; c++) {
            float* b = reinterpret_cast<float*>(p + 8 * c);
            for (int a = 0; a < 3; a++) {
                b[2 * a] = std::numeric_limits<float>::infinity();
                b[2 * a + 1] = -std::numeric_limits<float>::infinity();
            }
            p[8 * c + RT_CHILD_REF] = RT_INVALID_REF;
        }
        return id;
    }
    // one 32-B child record: lo.x hi.x lo.y hi.y lo.z hi.z ref pad
    void set_slot(uint32_t node, int c, const float b6[6], uint32_t ref) {
        float* b = reinterpret_cast<float*>(f.wide.data() + (size_t)node * nb) + 8 * c;
        for (int k = 0; k < 6; k++) b[k] = b6[k];
        reinterpret_cast<uint32_t*>(b)[RT_CHILD_REF] = ref;
        reinterpret_cast<uint32_t*>(b)[7] = 0;
    }

    // reference of a real node as a child slot value
    uint32_t ref_of(int32_t ni, uint32_t depth) {
        const RNode& n = t.nodes[ni];
        if (n.kids.empty()) {
            uint64_t cnt = (uint64_t)(n.end - n.begin);
            if (cnt == 0) return RT_INVALID_REF;  // only the empty scene's root
            if (cnt > 16) throw Error{RT_ERR_INVALID_ARGUMENT, "leaf larger than 16 primitives"};
            if ((uint64_t)n.begin > RT_LEAF_MAX_FIRST) throw Error{RT_ERR_INVALID_ARGUMENT, "scene too large"};
            return rt_make_leaf((uint32_t)n.begin, (uint32_t)cnt);
        }
        return emit_inner(n.kids, depth);
    }

    // Emits one wide node for a list of real children.  When a real node has
    // more children than W (collapsed trees reach 16..256), the children are
    // grouped under virtual wide nodes whose slot box is the union of the
    // group's boxes (a conservative superset; the exact ancestor chain used by
    // the fp64 re-verification only contains real nodes).
    // Slot 0's pad word carries the node's ordering hint for the packet
    // kernel: bits 0-1 the axis its children are sorted along (the builder's
    // partition axis: longest axis of the node box, main k-way order), bits
    // 2-6 the number of valid slots (valid slots come first).
    void set_meta(uint32_t node, const std::vector<int32_t>& kids, uint32_t nvalid) {
        double mn[3], mx[3];
        for (int a = 0; a < 3; a++) {
            mn[a] = std::numeric_limits<double>::infinity();
            mx[a] = -std::numeric_limits<double>::infinity();
        }
        for (int32_t k : kids)
            for (int a = 0; a < 3; a++) {
                mn[a] = std::min(mn[a], t.nodes[k].mn[a]);
                mx[a] = std::max(mx[a], t.nodes[k].mx[a]);
            }
        uint32_t* p = reinterpret_cast<uint32_t*>(f.wide.data() + (size_t)node * nb);
        p[7] = (uint32_t)longest_axis(mn, mx) | (nvalid << 2);
    }

    // walk-tree child reference: a leaf range or a new wide node whose slots
    // are the collapsed children, sorted by centre along the node's longest
    // axis (the packet kernel walks them front to back along it)
    uint32_t walk_ref(const WalkTree& w, int32_t b, uint32_t depth) {
        const WalkNode& n = w.nodes[b];
        if (n.left < 0) {
            if (n.count == 0) return RT_INVALID_REF;
            if (n.count > 16) throw Error{RT_ERR_INVALID_ARGUMENT, "leaf larger than 16 primitives"};
            if (n.first > RT_LEAF_MAX_FIRST) throw Error{RT_ERR_INVALID_ARGUMENT, "scene too large"};
            return rt_make_leaf(n.first, n.count);
        }
        const uint32_t id = alloc_node();
        walk_fill(w, b, id, depth);
        return id;
    }

    // Fills wide node `id` from walk node b.  The wide nodes of its inner
    // children are allocated together before any of their subtrees, so
    // siblings are adjacent and the top levels form a prefix of the array
    // (the root is node 0, its inner children nodes 1..k).
    void walk_fill(const WalkTree& w, int32_t b, uint32_t id, uint32_t depth) {
        const WalkNode& n = w.nodes[b];
        std::vector<int32_t> kids = collapse_children(w, b, W);
        const int axis = longest_axis(n.mn, n.mx);
        std::stable_sort(kids.begin(), kids.end(), [&](int32_t x, int32_t y) {
            return w.nodes[x].mn[axis] + w.nodes[x].mx[axis] < w.nodes[y].mn[axis] + w.nodes[y].mx[axis];
        });
        wide_depth = std::max(wide_depth, depth + 1);
        std::vector<uint32_t> refs(kids.size());
        for (size_t c = 0; c < kids.size(); c++)
            refs[c] = w.nodes[kids[c]].left < 0 ? walk_ref(w, kids[c], depth + 1) : alloc_node();
        for (size_t c = 0; c < kids.size(); c++) {
            float b6[6];
            box32(w.nodes[kids[c]].mn, w.nodes[kids[c]].mx, b6);
            set_slot(id, (int)c, b6, refs[c]);
        }
        uint32_t* p = reinterpret_cast<uint32_t*>(f.wide.data() + (size_t)id * nb);
        p[7] = (uint32_t)axis | ((uint32_t)kids.size() << 2);
        for (size_t c = 0; c < kids.size(); c++)
            if (w.nodes[kids[c]].left >= 0) walk_fill(w, kids[c], refs[c], depth + 1);
    }

    // walk_ref(w, 0, 0) for an inner root, with the subtrees of the root's
    // inner children filled on threads.  walk_fill numbers depth first: the
    // root 0, its inner children 1..m, then child 1's descendants, child 2's,
    // ... — each a contiguous id range.  Every child's subtree is filled into
    // a Flat of its own (the child = local node 0) and copied to its range,
    // inner-node refs shifted; the array equals the serial fill byte for byte.
    uint32_t walk_root(const WalkTree& w) {
        const uint32_t id = alloc_node();
        std::vector<int32_t> kids = collapse_children(w, 0, W);
        const WalkNode& n = w.nodes[0];
        const int axis = longest_axis(n.mn, n.mx);
        std::stable_sort(kids.begin(), kids.end(), [&](int32_t x, int32_t y) {
            return w.nodes[x].mn[axis] + w.nodes[x].mx[axis] < w.nodes[y].mn[axis] + w.nodes[y].mx[axis];
        });
        wide_depth = std::max(wide_depth, 1u);
        std::vector<uint32_t> refs(kids.size());
        std::vector<size_t> inner;
        for (size_t c = 0; c < kids.size(); c++) {
            if (w.nodes[kids[c]].left < 0) refs[c] = walk_ref(w, kids[c], 1);
            else { refs[c] = alloc_node(); inner.push_back(c); }
        }
        for (size_t c = 0; c < kids.size(); c++) {
            float b6[6];
            box32(w.nodes[kids[c]].mn, w.nodes[kids[c]].mx, b6);
            set_slot(id, (int)c, b6, refs[c]);
        }
        uint32_t* p = reinterpret_cast<uint32_t*>(f.wide.data() + (size_t)id * nb);
        p[7] = (uint32_t)axis | ((uint32_t)kids.size() << 2);
        const size_t m = inner.size();
        std::vector<Flat> sub(m);
        std::vector<uint32_t> sub_depth(m, 0);
        std::vector<std::exception_ptr> err(m);
        auto run = [&](size_t j) {
            try {
                sub[j].width = W;
                Flattener L(s, t, sub[j]);
                const uint32_t root = L.alloc_node();
                L.walk_fill(w, kids[inner[j]], root, 1);
                sub_depth[j] = L.wide_depth;
            } catch (...) { err[j] = std::current_exception(); }
        };
        std::vector<std::thread> th;
        for (size_t j = 0; j + 1 < m; j++) spawn(th, [&run, j] { run(j); });
        if (m) run(m - 1);
        for (auto& x : th) x.join();
        for (auto& e : err) if (e) std::rethrow_exception(e);
        uint64_t total = f.n_wide;
        std::vector<uint64_t> base(m);
        for (size_t j = 0; j < m; j++) { base[j] = total; total += sub[j].n_wide - 1; }
        f.wide.resize(total * nb, 0);
        for (size_t j = 0; j < m; j++) {
            wide_depth = std::max(wide_depth, sub_depth[j]);
            const uint32_t self = refs[inner[j]];
            auto remap = [&](uint32_t r) -> uint32_t {
                if (r == RT_INVALID_REF || (r & RT_LEAF_BIT)) return r;
                return r == 0 ? self : (uint32_t)(base[j] + r - 1);
            };
            for (uint64_t x = 0; x < sub[j].n_wide; x++) {
                const uint64_t g = x == 0 ? self : base[j] + x - 1;
                uint8_t* dst = f.wide.data() + g * nb;
                std::memcpy(dst, sub[j].wide.data() + x * nb, nb);
                uint32_t* q = reinterpret_cast<uint32_t*>(dst);
                for (int c = 0; c < W; c++) q[8 * c + RT_CHILD_REF] = remap(q[8 * c + RT_CHILD_REF]);
            }
        }
        f.n_wide = total;
        return id;
    }

    uint32_t emit_inner(const std::vector<int32_t>& kids, uint32_t depth) {
        uint32_t id = alloc_node();
        wide_depth = std::max(wide_depth, depth + 1);
        if ((int)kids.size() <= W) {
            for (size_t c = 0; c < kids.size(); c++) {
                float b6[6];
                box32(t.nodes[kids[c]].mn, t.nodes[kids[c]].mx, b6);
                uint32_t r = ref_of(kids[c], depth + 1);
                set_slot(id, (int)c, b6, r);
            }
            set_meta(id, kids, (uint32_t)kids.size());
            return id;
        }
        size_t groups = std::min<size_t>((size_t)W, (kids.size() + W - 1) / W);
        size_t per = (kids.size() + groups - 1) / groups;
        uint32_t nslots = 0;
        for (size_t g = 0; g < groups; g++) {
            size_t a = g * per, b = std::min(kids.size(), a + per);
            if (a >= b) break;
            std::vector<int32_t> sub(kids.begin() + a, kids.begin() + b);
            float b6[6] = {std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                           std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                           std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity()};
            for (int32_t k : sub) {
                float c6[6];
                box32(t.nodes[k].mn, t.nodes[k].mx, c6);
                for (int q = 0; q < 3; q++) {
                    b6[2 * q] = std::min(b6[2 * q], c6[2 * q]);
                    b6[2 * q + 1] = std::max(b6[2 * q + 1], c6[2 * q + 1]);
                }
            }
            uint32_t r = sub.size() == 1 ? ref_of(sub[0], depth + 1) : emit_inner(sub, depth + 1);
            set_slot(id, (int)g, b6, r);
            nslots++;
        }
        set_meta(id, kids, nslots);
        return id;
    }
};

}  // namespace

Flat flatten(const Soup& s, const Tree& t, int width_hint, const WalkTree* walk) {
    Flat f;
    // --- tree statistics
    uint32_t maxk = 0, maxleaf = 0, depth = 0, stack_bound = 1;
    {
        struct It { int32_t n; uint32_t d; uint32_t sb; };
        std::vector<It> st{{0, 0, 1}};
        while (!st.empty()) {
            It it = st.back();
            st.pop_back();
            const RNode& n = t.nodes[it.n];
            depth = std::max(depth, it.d);
            if (n.kids.empty()) {
                f.real_leaves++;
                maxleaf = std::max<uint32_t>(maxleaf, (uint32_t)(n.end - n.begin));
                stack_bound = std::max(stack_bound, it.sb);
            } else {
                f.real_inner++;
                maxk = std::max<uint32_t>(maxk, (uint32_t)n.kids.size());
                for (int32_t c : n.kids) st.push_back({c, it.d + 1, it.sb + (uint32_t)n.kids.size() - 1});
            }
        }
    }
    f.depth = depth;
    f.max_children = maxk;
    f.max_leaf = maxleaf;
    int W = width_hint;
    if (walk) W = 8;
    f.walk = walk != nullptr;
    if (W <= 0) {
        W = 2;
        while (W < (int)maxk && W < 16) W *= 2;
    }
    if (!(W == 2 || W == 4 || W == 8 || W == 16)) throw Error{RT_ERR_INVALID_ARGUMENT, "wide node width must be 2/4/8/16"};
    f.width = W;
    (void)stack_bound;  // real-tree bound: used by the literal kernel (rt_api.cpp)

    // --- scene coordinate magnitude: sizes the per-frame plane margin of the
    // fp32 traversal (rt_api.cpp frame_params, DESIGN.md "exactness")
    double cm = 0;
    for (double x : s.v) cm = std::max(cm, std::fabs(x));
    f.coord_max = cm;
    f.pad = 0;

    // --- per-triangle data in BVH (walk) order
    const uint64_t n = s.n;
    const std::vector<uint32_t>& worder = walk ? walk->order : t.order;
    f.tri64.resize(n * RT_TRI64_DOUBLES);
    f.tri32.resize((n + RT_TRI32_PAD) * 12);  // + zeroed padding records (packet kernel leaf chunks)
    std::fill(f.tri32.begin() + (ptrdiff_t)(n * 12), f.tri32.end(), 0.0f);
    f.tri_id.resize(n);
    f.tri_rank.resize(n);
    f.tri_leaf.resize(n);
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; i++) {
        uint32_t id = worder[i];
        const double* p = s.v.data() + (size_t)id * 9;
        double* q = f.tri64.data() + i * RT_TRI64_DOUBLES;
        q[0] = p[0]; q[1] = p[1]; q[2] = p[2];
        q[3] = p[3] - p[0]; q[4] = p[4] - p[1]; q[5] = p[5] - p[2];  // edge1 = v1 - v0 (triangle.hpp:42)
        q[6] = p[6] - p[0]; q[7] = p[7] - p[1]; q[8] = p[8] - p[2];  // edge2 = v2 - v0
        // fp32 pre-filter record: v0, e1, e2 rounded to nearest, then the
        // magnitudes its error bounds need, rounded up: max|e1_i|, max|e2_i|,
        // max|v0_i| (render.hip tri_prefilter)
        float* r = f.tri32.data() + i * 12;
        for (int k = 0; k < 9; k++) r[k] = (float)q[k];
        auto up = [](double x) {
            float v = (float)x;
            if ((double)v < x) v = std::nextafter(v, std::numeric_limits<float>::infinity());
            return v;
        };
        r[9] = up(std::max({std::fabs(q[3]), std::fabs(q[4]), std::fabs(q[5])}));
        r[10] = up(std::max({std::fabs(q[6]), std::fabs(q[7]), std::fabs(q[8])}));
        r[11] = up(std::max({std::fabs(q[0]), std::fabs(q[1]), std::fabs(q[2])}));
        f.tri_id[i] = id;
    }
    });
    // --- real nodes (fp64 box + parent) and reference visit ranks
    const size_t R = t.nodes.size();
    f.rbox.resize(R * 6);
    f.rparent.resize(R);
    for (size_t i = 0; i < R; i++) {
        for (int a = 0; a < 3; a++) { f.rbox[i * 6 + a] = t.nodes[i].mn[a]; f.rbox[i * 6 + 3 + a] = t.nodes[i].mx[a]; }
        f.rparent[i] = t.nodes[i].parent;
    }
    f.rkid_off.assign(R + 1, 0);
    f.rrange.resize(R * 2);
    for (size_t i = 0; i < R; i++) {
        f.rkid_off[i + 1] = f.rkid_off[i] + (uint32_t)t.nodes[i].kids.size();
        f.rrange[i * 2] = (uint32_t)t.nodes[i].begin;
        f.rrange[i * 2 + 1] = (uint32_t)t.nodes[i].end;
    }
    f.rkid.reserve(f.rkid_off[R]);
    for (size_t i = 0; i < R; i++) for (int32_t c : t.nodes[i].kids) f.rkid.push_back((uint32_t)c);
    {
        // visit order of StackBVH::traverse (stack_bvh.hpp:619-641): LIFO,
        // children pushed 0..n-1 so the last child is visited first.
        // (computed per reference-order position, then placed at each
        // triangle's walk-order index)
        std::vector<uint32_t> rrank(n), rleaf(n), wpos(n);
        uint32_t rank = 0;
        std::vector<int32_t> st{0};
        while (!st.empty()) {
            int32_t ni = st.back();
            st.pop_back();
            const RNode& nd = t.nodes[ni];
            if (nd.kids.empty())
                for (int64_t i = nd.begin; i < nd.end; i++) { rrank[i] = rank++; rleaf[i] = (uint32_t)ni; }
            for (int32_t c : nd.kids) st.push_back(c);
        }
        for (uint64_t i = 0; i < n; i++) wpos[worder[i]] = (uint32_t)i;
        f.ref2walk.resize(n);
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t w = wpos[t.order[i]];
            f.ref2walk[i] = w;
            f.tri_rank[w] = rrank[i];
            f.tri_leaf[w] = rleaf[i];
        }
    }
    // normal, loader id, leaf and the leaf box (fp32, rounded inward) complete
    // the 128-B fp64 record (rt_device.h)
    auto down = [](double x) {
        float v = (float)x;
        if ((double)v > x) v = std::nextafter(v, -std::numeric_limits<float>::infinity());
        return v;
    };
    auto up = [](double x) {
        float v = (float)x;
        if ((double)v < x) v = std::nextafter(v, std::numeric_limits<float>::infinity());
        return v;
    };
    parallel_for(n, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; i++) {
        double* q = f.tri64.data() + i * RT_TRI64_DOUBLES;
        const uint32_t id = f.tri_id[i], leaf = f.tri_leaf[i];
        // shadeScreen's normal.normalize() (main.cpp:361, vector3.hpp), done
        // once here with the same IEEE operations the kernel would run
        double nx = s.normal[(size_t)id * 3], ny = s.normal[(size_t)id * 3 + 1], nz = s.normal[(size_t)id * 3 + 2];
        const double nl = std::sqrt(nx * nx + ny * ny + nz * nz);
        if (nl > 0.0) {
            const double inv = 1.0 / nl;
            nx = nx * inv; ny = ny * inv; nz = nz * inv;
        }
        q[RT_T64_NORMAL] = nx; q[RT_T64_NORMAL + 1] = ny; q[RT_T64_NORMAL + 2] = nz;
        uint32_t* w = reinterpret_cast<uint32_t*>(q + RT_T64_IDLEAF);
        w[0] = id;
        w[1] = leaf;
        float* b = reinterpret_cast<float*>(q + RT_T64_BOX);
        for (int a = 0; a < 3; a++) {
            b[a] = up(f.rbox[(size_t)leaf * 6 + a]);
            b[3 + a] = down(f.rbox[(size_t)leaf * 6 + 3 + a]);
        }
    }
    });
    // --- wide nodes
    Flattener F(s, t, f);
    F.box32(t.nodes[0].mn, t.nodes[0].mx, f.root_box);
    if (walk && n > 0) {
        F.box32(walk->nodes[0].mn, walk->nodes[0].mx, f.root_box);
        const char* bt = std::getenv("RT_BUILD_THREADS");  // 1: the serial fill (A/B, tests)
        const bool serial = (bt && std::atoi(bt) == 1) || walk->nodes[0].left < 0;
        f.root_ref = serial ? F.walk_ref(*walk, 0, 0) : F.walk_root(*walk);
        if (f.n_wide == 0) F.alloc_node();
    } else if (n == 0) {
        f.root_ref = RT_INVALID_REF;
        F.alloc_node();
    } else {
        f.root_ref = F.ref_of(0, 0);
        if (f.n_wide == 0) F.alloc_node();  // root is a leaf: keep a valid node array
    }
    // Each child record's pad word carries the child's ref with the CHILD
    // node's ordering meta (sort axis | valid slots << 2; slot 0's pad held
    // the node's own meta until here) in bits 24-30 — node ids stay below
    // 2^24 — so the wave walks (packet_kernel.h, path_kernel.h wave_walk,
    // queue_paths.h k_sh_walk) take a node's next ref from one word, with
    // its valid slots known before the node is loaded, and no scalar
    // instructions combine ref and meta in every node step (16 SALU per step
    // of 8 children in round 4).  Leaf slots hold the leaf ref there, empty
    // slots RT_INVALID_REF; the ref word stays the plain ref for the per-lane
    // walks.  The root's meta is root_meta.
    if (f.n_wide >= (1u << 24)) throw Error{RT_ERR_INVALID_ARGUMENT, "scene too large (wide nodes)"};
    {
        const uint64_t nb = rt_node_bytes(W);
        std::vector<uint32_t> meta(f.n_wide);
        for (uint64_t x = 0; x < f.n_wide; x++) meta[x] = reinterpret_cast<const uint32_t*>(f.wide.data() + x * nb)[7];
        for (uint64_t x = 0; x < f.n_wide; x++) {
            uint32_t* p = reinterpret_cast<uint32_t*>(f.wide.data() + x * nb);
            for (int c = 0; c < W; c++) {
                const uint32_t r = p[8 * c + RT_CHILD_REF];
                p[8 * c + 7] = (r != RT_INVALID_REF && !(r & RT_LEAF_BIT)) ? (r | meta[r] << 24) : r;
            }
        }
        f.root_meta = (f.root_ref != RT_INVALID_REF && !(f.root_ref & RT_LEAF_BIT)) ? meta[f.root_ref] : 0u;
    }
    // ordered traversal pushes at most W-1 siblings per wide level
    f.stack_bound = F.wide_depth * (uint32_t)(W - 1) + 1;
    return f;
}

}  // namespace rt
