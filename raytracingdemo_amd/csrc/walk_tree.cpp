// Walk tree: the acceleration structure the gfx950 traversal actually walks.
//
// Results never depend on it.  The reference (src/stack_bvh.hpp:611-644)
// reports, among the triangles whose fp64 Moller-Trumbore test passes and
// whose every ancestor box in *its* tree passes the fp64 slab test, the
// nearest one (first in its LIFO visit order on ties).  The device pipeline
// finds every triangle the fp32 filters cannot rule out, whatever tree it
// walks, and takes the ancestor chain (rbox/rparent) and the visit ranks
// (tri_rank) from the reference's own tree.  So the walk tree
// is free to be a better tree than the reference's.
//
// The reference's k-way "bsah" partition splits a node into up to k slabs
// along one axis from 16 bins (stack_bvh.hpp:241-449): long thin children
// that overlap a tile's rays far more than needed.  This builder makes a
// binary SAH tree over all three axes (32 centroid bins, leaves of at most
// RT_WALK_LEAF triangles), then collapses it into W-wide nodes by a dynamic
// programme over the SAH cost (plan_wide_collapse; the greedy collapse, which
// repeatedly opens the child of largest surface area, with
// RT_WALK_COLLAPSE=greedy).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <system_error>
#include <thread>

#include "rt_internal.h"

namespace rt {
namespace {

#ifndef RT_WALK_BINS
#define RT_WALK_BINS 32  // centroid bins per axis (host and device builds must agree)
#endif
constexpr int kBins = RT_WALK_BINS;

struct BBox {
    double mn[3], mx[3];
    BBox() {
        for (int a = 0; a < 3; a++) {
            mn[a] = std::numeric_limits<double>::infinity();
            mx[a] = -std::numeric_limits<double>::infinity();
        }
    }
    void grow(const BBox& o) {
        for (int a = 0; a < 3; a++) {
            mn[a] = std::min(mn[a], o.mn[a]);
            mx[a] = std::max(mx[a], o.mx[a]);
        }
    }
    void grow(const double p[3]) {
        for (int a = 0; a < 3; a++) {
            mn[a] = std::min(mn[a], p[a]);
            mx[a] = std::max(mx[a], p[a]);
        }
    }
    double area() const {
        if (!(mx[0] >= mn[0])) return 0.0;
        const double ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
        return 2.0 * (ex * ey + ey * ez + ez * ex);
    }
};

// (read at every scene build, so a process can build trees of both kinds)
int max_leaf() {
    const char* e = std::getenv("RT_WALK_LEAF");
    const int v = e ? std::atoi(e) : 4;
    return v >= 1 && v <= 16 ? v : 4;
}

// SAH cost of one inner-node visit relative to one triangle test (the packet
// kernel's 8-child step and a triangle test cost about the same: DESIGN.md §7)
double node_cost() {
    const char* e = std::getenv("RT_WALK_CT");
    const double v = e ? std::atof(e) : 1.0;
    return v > 0.0 && v < 100.0 ? v : 1.0;
}

}  // namespace

int walk_max_leaf() { return max_leaf(); }
double walk_node_cost() { return node_cost(); }

WalkTree build_walk_tree(const Soup& s) {
    WalkTree w;
    const uint32_t n = (uint32_t)s.n;
    w.order.resize(n);
    for (uint32_t i = 0; i < n; i++) w.order[i] = i;
    if (n == 0) return w;
    const int LMAX = max_leaf();
    const double CT = node_cost();
    std::vector<BBox> tb(n);
    std::vector<double> cen(3 * (size_t)n);
    for (uint32_t i = 0; i < n; i++) {
        for (int a = 0; a < 3; a++) {
            tb[i].mn[a] = s.lo[a][i];
            tb[i].mx[a] = s.hi[a][i];
            cen[3 * (size_t)i + a] = 0.5 * (s.lo[a][i] + s.hi[a][i]);
        }
    }
    struct Job { int32_t node; uint32_t b, e; };
    w.nodes.push_back(WalkNode{});
    std::vector<Job> jobs{{0, 0, n}};
    uint32_t* idx = w.order.data();
    while (!jobs.empty()) {
        const Job j = jobs.back();
        jobs.pop_back();
        BBox box, cb;
        for (uint32_t i = j.b; i < j.e; i++) {
            box.grow(tb[idx[i]]);
            cb.grow(&cen[3 * (size_t)idx[i]]);
        }
        WalkNode& nd = w.nodes[j.node];
        for (int a = 0; a < 3; a++) { nd.mn[a] = box.mn[a]; nd.mx[a] = box.mx[a]; }
        const uint32_t cnt = j.e - j.b;
        auto make_leaf = [&]() {
            WalkNode& m = w.nodes[j.node];
            m.first = j.b;
            m.count = cnt;
        };
        if (cnt <= 1) { make_leaf(); continue; }
        // binned SAH over the three axes (cost in units of one box / triangle test)
        const double A = box.area();
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_bin = 0;
        for (int a = 0; a < 3; a++) {
            const double lo = cb.mn[a], ext = cb.mx[a] - cb.mn[a];
            if (!(ext > 0.0)) continue;
            const double scale = kBins / ext;
            BBox bb[kBins];
            uint32_t bc[kBins] = {};
            for (uint32_t i = j.b; i < j.e; i++) {
                int k = (int)((cen[3 * (size_t)idx[i] + a] - lo) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                bc[k]++;
                bb[k].grow(tb[idx[i]]);
            }
            double ra[kBins];
            uint32_t rc[kBins];
            BBox acc;
            uint32_t c = 0;
            for (int k = kBins - 1; k > 0; k--) {
                acc.grow(bb[k]);
                c += bc[k];
                ra[k] = acc.area();
                rc[k] = c;
            }
            BBox lacc;
            uint32_t lc = 0;
            for (int k = 1; k < kBins; k++) {
                lacc.grow(bb[k - 1]);
                lc += bc[k - 1];
                if (lc == 0 || rc[k] == 0) continue;
                const double cost = (lacc.area() * lc + ra[k] * rc[k]) / (A > 0 ? A : 1.0);
                if (cost < best) { best = cost; best_axis = a; best_bin = k; }
            }
        }
        // a leaf costs cnt triangle tests; an inner node one more box test
        if (cnt <= (uint32_t)LMAX && (best_axis < 0 || (double)cnt <= CT + best)) { make_leaf(); continue; }
        uint32_t mid;
        if (best_axis < 0) {
            mid = j.b + cnt / 2;  // coincident centroids: split the range in half
        } else {
            const double lo = cb.mn[best_axis], scale = kBins / (cb.mx[best_axis] - cb.mn[best_axis]);
            uint32_t* p = std::partition(idx + j.b, idx + j.e, [&](uint32_t t) {
                int k = (int)((cen[3 * (size_t)t + best_axis] - lo) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                return k < best_bin;
            });
            mid = (uint32_t)(p - idx);
            if (mid == j.b || mid == j.e) mid = j.b + cnt / 2;
        }
        const int32_t l = (int32_t)w.nodes.size();
        w.nodes.push_back(WalkNode{});
        w.nodes.push_back(WalkNode{});
        w.nodes[j.node].left = l;
        w.nodes[j.node].right = l + 1;
        jobs.push_back({l + 1, mid, j.e});
        jobs.push_back({l, j.b, mid});
    }
    return w;
}

namespace {

double env_cost(const char* name, double dflt) {
    const char* e = std::getenv(name);
    const double v = e ? std::atof(e) : dflt;
    return v >= 0.0 && v < 100.0 ? v : dflt;
}

}  // namespace

// Treelet restructuring of the binary walk tree (Karras and Aila, "Fast
// parallel construction of high-quality bounding volume hierarchies", HPG
// 2013), before the wide collapse: for every inner node r, children before
// parents, the treelet of up to 7 leaves grown from r by opening its largest
// inner member is rebuilt with the SAH-optimal binary topology over those
// leaves (a dynamic programme over the 2^7 leaf subsets), reusing the
// treelet's inner nodes.  Cost model: inner A * RT_WALK_CT, leaf A * count.
// Triangles never move between leaves, so the result is still a tree over
// every triangle once; the leaves' ranges are then laid out again depth
// first, so every subtree is a contiguous range of `order` for the collapse.
void restructure_treelets(WalkTree& w, int passes) {
    const size_t N = w.nodes.size();
    if (N < 3 || w.nodes[0].left < 0 || passes < 1) return;
    const double CI = node_cost();
    auto box_of = [&](int32_t b) {
        BBox bb;
        for (int a = 0; a < 3; a++) { bb.mn[a] = w.nodes[b].mn[a]; bb.mx[a] = w.nodes[b].mx[a]; }
        return bb;
    };
    std::vector<double> C(N, 0.0);
    std::vector<int32_t> post;
    post.reserve(N);
    constexpr int TL = 7, NS = 1 << TL;
    for (int pass = 0; pass < passes; pass++) {
        // post-order of the current shape, taken again every pass: within a
        // pass a restructured treelet's root keeps its id and its other
        // members were visited before it, but a pass renumbers inner nodes,
        // so the next pass's children-before-parents order (and the costs C
        // of finished children it relies on) must come from the new shape
        post.clear();
        {
            std::vector<std::pair<int32_t, bool>> st{{0, false}};
            while (!st.empty()) {
                auto [b, done] = st.back();
                st.pop_back();
                if (done || w.nodes[b].left < 0) { post.push_back(b); continue; }
                st.push_back({b, true});
                st.push_back({w.nodes[b].right, false});
                st.push_back({w.nodes[b].left, false});
            }
        }
        for (int32_t r : post) {
            WalkNode& nr = w.nodes[r];
            if (nr.left < 0) { C[r] = box_of(r).area() * nr.count; continue; }
            int32_t leaf[TL], inner[TL];
            int nl = 2, ni = 1;
            leaf[0] = nr.left;
            leaf[1] = nr.right;
            inner[0] = r;
            while (nl < TL) {
                int pick = -1;
                double pa = -1.0;
                for (int i = 0; i < nl; i++)
                    if (w.nodes[leaf[i]].left >= 0) {
                        const double a = box_of(leaf[i]).area();
                        if (a > pa) { pa = a; pick = i; }
                    }
                if (pick < 0) break;
                const int32_t m = leaf[pick];
                inner[ni++] = m;
                leaf[pick] = w.nodes[m].left;
                leaf[nl++] = w.nodes[m].right;
            }
            // current cost of r (its children's C are final)
            const double cur = box_of(r).area() * CI + C[nr.left] + C[nr.right];
            if (nl < 3) { C[r] = cur; continue; }
            const int full = (1 << nl) - 1;
            BBox sb[NS];
            double cost[NS], area[NS];
            int part[NS];
            for (int S = 1; S <= full; S++) {
                const int low = S & -S;
                if (S == low) {
                    const int i = __builtin_ctz((unsigned)S);
                    sb[S] = box_of(leaf[i]);
                    cost[S] = C[leaf[i]];
                } else {
                    sb[S] = sb[S ^ low];
                    sb[S].grow(sb[low]);
                }
                area[S] = sb[S].area();
            }
            for (int S = 1; S <= full; S++) {
                if ((S & (S - 1)) == 0) continue;  // (one leaf: its subtree's cost)
                // subsets in increasing value: every proper subset of S is smaller
                double best = std::numeric_limits<double>::infinity();
                int bp = 0;
                const int low = S & -S;
                for (int P = (S - 1) & S; P > 0; P = (P - 1) & S) {
                    if (!(P & low)) continue;  // each split once: P holds S's lowest leaf
                    const double v = cost[P] + cost[S ^ P];
                    if (v < best) { best = v; bp = P; }
                }
                cost[S] = area[S] * CI + best;
                part[S] = bp;
            }
            if (!(cost[full] < cur * (1.0 - 1e-9))) { C[r] = cur; continue; }
            // rebuild: subset S -> node id (r for the whole set, then the
            // treelet's other inner nodes in turn)
            int next_inner = 1;
            auto build = [&](auto&& self, int S) -> int32_t {
                if ((S & (S - 1)) == 0) return leaf[__builtin_ctz((unsigned)S)];
                const int32_t id = S == full ? r : inner[next_inner++];
                const int32_t a = self(self, part[S]);
                const int32_t b = self(self, S ^ part[S]);
                WalkNode& m = w.nodes[id];
                m.left = a;
                m.right = b;
                m.first = m.count = 0;
                for (int k = 0; k < 3; k++) { m.mn[k] = sb[S].mn[k]; m.mx[k] = sb[S].mx[k]; }
                C[id] = cost[S];
                return id;
            };
            build(build, full);
        }
    }
    // leaves' ranges depth first: subtrees contiguous again
    std::vector<uint32_t> order(w.order.size());
    uint32_t at = 0;
    std::vector<int32_t> st{0};
    while (!st.empty()) {
        const int32_t b = st.back();
        st.pop_back();
        WalkNode& n = w.nodes[b];
        if (n.left < 0) {
            for (uint32_t i = 0; i < n.count; i++) order[at + i] = w.order[n.first + i];
            n.first = at;
            at += n.count;
            continue;
        }
        st.push_back(n.right);
        st.push_back(n.left);
    }
    if (at != order.size()) throw Error{RT_ERR_RUNTIME, "treelet restructuring lost triangles"};
    w.order.swap(order);
}
int walk_treelet_passes() {
    const char* e = std::getenv("RT_WALK_TREELET");
    const int v = e ? std::atoi(e) : 0;
    return v >= 0 && v <= 8 ? v : 0;
}

// The collapse as a dynamic programme (the SAH-optimal wide-BVH conversion of
// Ylitie, Karras and Laine, HPG 2017), costs in the packet kernel's units:
//   leaf(n)        = A(n) (c_leaf + c_tri cnt(n))        cnt(n) <= P
//   inner(n)       = A(n) c_node + split(n, W)
//   split(n, i)    = min_k  C(left, k) + C(right, i - k)
//   C(n, 1)        = min(leaf(n), inner(n))
//   C(n, i > 1)    = min(C(n, i - 1), split(n, i))
// C(n, i) is the cheapest way to stand for n's subtree with at most i slots of
// a parent wide node.  Any subtree of the binary tree is a contiguous range
// of `order`, so "this subtree is one leaf" only relabels the node.
void plan_wide_collapse(WalkTree& w, int W) {
    w.wide_off.clear();
    w.wide_cnt.clear();
    w.wide_kids.clear();
    const char* mode = std::getenv("RT_WALK_COLLAPSE");
    if (mode && mode[0] == 'g') return;
    const size_t N = w.nodes.size();
    if (N < 3 || w.nodes[0].left < 0 || W < 2 || W > 16) return;
    const double cN = env_cost("RT_WALK_CN", 1.0);
    const double cL = env_cost("RT_WALK_CLV", 0.25);
    const double cT = env_cost("RT_WALK_CTRI", 0.5);
    const uint32_t P = (uint32_t)std::min(16.0, std::max(1.0, env_cost("RT_WALK_PMAX", 8.0)));

    const int S = W + 1;
    uvector<double> C(N * S);        // every row is written before it is read
    uvector<uint8_t> pick(N * S);    // [0] inner split k; [1] leaf flag; [i] split k or 0 (= C(n, i-1))
    uvector<uint32_t> rb(N), re(N);  // the subtree's range of `order`
    // one row of the programme; the children's rows are complete
    auto row = [&](int32_t b) {
        const WalkNode& n = w.nodes[b];
        BBox bb;
        for (int a = 0; a < 3; a++) { bb.mn[a] = n.mn[a]; bb.mx[a] = n.mx[a]; }
        const double A = bb.area();
        double* c = &C[(size_t)b * S];
        uint8_t* p = &pick[(size_t)b * S];
        if (n.left < 0) {
            rb[b] = n.first;
            re[b] = n.first + n.count;
            const double leaf = A * (cL + cT * n.count);
            for (int i = 0; i <= W; i++) { c[i] = leaf; p[i] = 0; }
            p[1] = 1;
            return;
        }
        const int32_t l = n.left, r = n.right;
        bool contiguous = true;
        if (re[l] == rb[r]) { rb[b] = rb[l]; re[b] = re[r]; }
        else if (re[r] == rb[l]) { rb[b] = rb[r]; re[b] = re[l]; }
        else { rb[b] = std::min(rb[l], rb[r]); re[b] = std::max(re[l], re[r]); contiguous = false; }
        const double* cl = &C[(size_t)l * S];
        const double* cr = &C[(size_t)r * S];
        double dist[17];
        uint8_t dk[17];
        for (int i = 2; i <= W; i++) {
            double best = std::numeric_limits<double>::infinity();
            int bk = 1;
            for (int k = 1; k < i; k++) {
                const double v = cl[k] + cr[i - k];
                if (v < best) { best = v; bk = k; }
            }
            dist[i] = best;
            dk[i] = (uint8_t)bk;
        }
        const double inner = A * cN + dist[W];
        p[0] = dk[W];
        const uint32_t cnt = re[b] - rb[b];
        const double leaf = contiguous && cnt <= P && b != 0 ? A * (cL + cT * cnt) : std::numeric_limits<double>::infinity();
        if (leaf <= inner) { c[1] = leaf; p[1] = 1; }
        else { c[1] = inner; p[1] = 0; }
        for (int i = 2; i <= W; i++) {
            if (dist[i] < c[i - 1]) { c[i] = dist[i]; p[i] = dk[i]; }
            else { c[i] = c[i - 1]; p[i] = 0; }
        }
    };
    // rows of one subtree, children before parents (explicit post-order)
    auto subtree = [&](int32_t root) {
        std::vector<std::pair<int32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [b, done] = st.back();
            st.pop_back();
            const WalkNode& n = w.nodes[b];
            if (done || n.left < 0) { row(b); continue; }
            st.push_back({b, true});
            st.push_back({n.right, false});
            st.push_back({n.left, false});
        }
    };
    // The top levels breadth-first until there are enough subtrees for the
    // threads; the subtrees run on threads, then the top levels bottom-up.
    std::vector<int32_t> top, front{0};
    for (int level = 0; level < 7 && !front.empty(); level++) {
        std::vector<int32_t> next;
        for (int32_t b : front) {
            const WalkNode& n = w.nodes[b];
            top.push_back(b);
            if (n.left >= 0) { next.push_back(n.left); next.push_back(n.right); }
        }
        front.swap(next);
    }
    {
        std::atomic<size_t> take{0};
        auto work = [&] {
            for (size_t t; (t = take.fetch_add(1)) < front.size();) subtree(front[t]);
        };
        std::vector<std::thread> th;
        const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        for (unsigned t = 1; t < hw && t < front.size(); t++) {
            try { th.emplace_back(work); } catch (const std::system_error&) { break; }
        }
        work();
        for (auto& x : th) x.join();
    }
    for (size_t t = top.size(); t-- > 0;) row(top[t]);

    // top-down: the slots of each wide node; slots that chose "leaf" become leaves
    w.wide_off.assign(N, UINT32_MAX);
    w.wide_cnt.assign(N, 0);
    std::vector<int32_t> slots;
    auto expand = [&](auto&& self, int32_t m, int i) -> void {
        const WalkNode& n = w.nodes[m];
        while (i > 1 && n.left >= 0 && pick[(size_t)m * S + i] == 0) i--;
        if (i == 1 || n.left < 0) { slots.push_back(m); return; }
        const int k = pick[(size_t)m * S + i];
        self(self, n.left, k);
        self(self, n.right, i - k);
    };
    std::vector<int32_t> todo{0};
    while (!todo.empty()) {
        const int32_t b = todo.back();
        todo.pop_back();
        slots.clear();
        const int k = pick[(size_t)b * S];
        expand(expand, w.nodes[b].left, k);
        expand(expand, w.nodes[b].right, W - k);
        w.wide_off[b] = (uint32_t)w.wide_kids.size();
        w.wide_cnt[b] = (uint8_t)slots.size();
        for (int32_t m : slots) {
            w.wide_kids.push_back(m);
            WalkNode& n = w.nodes[m];
            if (n.left < 0) continue;
            if (pick[(size_t)m * S + 1]) {
                n.left = n.right = -1;
                n.first = rb[m];
                n.count = re[m] - rb[m];
            } else {
                todo.push_back(m);
            }
        }
    }
}

// Children of binary node b for one W-wide node: the planned slots
// (plan_wide_collapse), or greedily: open the inner child of largest surface
// area until W children (or only leaves) remain.
std::vector<int32_t> collapse_children(const WalkTree& w, int32_t b, int W) {
    if (!w.wide_off.empty() && w.wide_off[b] != UINT32_MAX) {
        const int32_t* k = w.wide_kids.data() + w.wide_off[b];
        return std::vector<int32_t>(k, k + w.wide_cnt[b]);
    }
    std::vector<int32_t> kids{w.nodes[b].left, w.nodes[b].right};
    while ((int)kids.size() < W) {
        int pick = -1;
        double pa = -1.0;
        for (int c = 0; c < (int)kids.size(); c++) {
            const WalkNode& k = w.nodes[kids[c]];
            if (k.left < 0) continue;
            BBox bb;
            for (int a = 0; a < 3; a++) { bb.mn[a] = k.mn[a]; bb.mx[a] = k.mx[a]; }
            const double ar = bb.area();
            if (ar > pa) { pa = ar; pick = c; }
        }
        if (pick < 0) break;
        const WalkNode& k = w.nodes[kids[pick]];
        const int32_t l = k.left, r = k.right;
        kids[pick] = l;
        kids.push_back(r);
    }
    return kids;
}

// Quantised copy of W = 8 wide nodes for the per-lane walk (render.hip
// lane_walk, QN): RT_QNODE_BYTES per node —
//   dwords 0-2   origin x, y, z (fp32)
//   dword 3      exponents e_x, e_y, e_z as bytes (biased by 127)
//   dwords 4-15  8-bit planes, SoA: lo.x[8] hi.x[8] lo.y[8] hi.y[8] lo.z[8] hi.z[8]
//   dwords 16-23 the 8 child refs (as in the 32-B records)
// Plane q of axis a stands for origin[a] + q 2^e[a], exactly: the origin is
// an fp32 multiple of 2^e (|origin / 2^e| < 2^24), lo planes are rounded down
// and hi planes up in exact (double) arithmetic, so every quantised box
// contains its fp32 record box — a superset, which the exact traversal
// allows.  Empty slots get lo = 255, hi = 0 and the invalid ref.
std::vector<uint8_t> quantize_wide8(const uint8_t* wide, uint64_t n_nodes) {
    std::vector<uint8_t> out(n_nodes * RT_QNODE_BYTES, 0);
    for (uint64_t n = 0; n < n_nodes; n++) {
        const float* rec = reinterpret_cast<const float*>(wide + n * 256);
        uint32_t* q = reinterpret_cast<uint32_t*>(out.data() + n * RT_QNODE_BYTES);
        uint8_t* planes = reinterpret_cast<uint8_t*>(q + 4);
        bool valid[8];
        double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
        bool any = false;
        for (int c = 0; c < 8; c++) {
            const uint32_t ref = reinterpret_cast<const uint32_t*>(rec + 8 * c)[RT_CHILD_REF];
            q[16 + c] = ref;
            valid[c] = ref != RT_INVALID_REF;
            if (!valid[c]) continue;
            for (int a = 0; a < 3; a++) {
                const double l = rec[8 * c + 2 * a], h = rec[8 * c + 2 * a + 1];
                lo[a] = any ? std::min(lo[a], l) : l;
                hi[a] = any ? std::max(hi[a], h) : h;
            }
            any = true;
        }
        uint32_t exps = 0;
        for (int a = 0; a < 3; a++) {
            const double ext = hi[a] - lo[a];
            int e = ext > 0 ? (int)std::ceil(std::log2(ext / 255.0)) : -100;
            e = std::max(e, -100);
            double org = 0, sc = 0;
            for (;; e++) {
                sc = std::ldexp(1.0, e);
                org = std::floor(lo[a] / sc) * sc;
                if (std::fabs(org) / sc < 16777216.0 && (hi[a] - org) / sc <= 255.0) break;
            }
            if (e > 127) throw Error{RT_ERR_INVALID_ARGUMENT, "scene extent too large to quantise"};
            reinterpret_cast<float*>(q)[a] = (float)org;  // exact: an fp32 multiple of 2^e
            exps |= (uint32_t)(e + 127) << (8 * a);
            for (int c = 0; c < 8; c++) {
                uint8_t ql = 255, qh = 0;
                if (valid[c]) {
                    const double l = rec[8 * c + 2 * a], h = rec[8 * c + 2 * a + 1];
                    const double fl = std::floor((l - org) / sc), ch = std::ceil((h - org) / sc);
                    if (fl < 0 || ch > 255 || org + fl * sc > l || org + ch * sc < h)
                        throw Error{RT_ERR_RUNTIME, "node quantisation out of range"};
                    ql = (uint8_t)fl;
                    qh = (uint8_t)ch;
                }
                planes[16 * a + c] = ql;      // lo[a] array
                planes[16 * a + 8 + c] = qh;  // hi[a] array
            }
        }
        q[3] = exps;
    }
    return out;
}


}  // namespace rt
