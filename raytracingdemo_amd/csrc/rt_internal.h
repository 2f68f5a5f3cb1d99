// Host-side internals of librtmi355x.so (not part of the ABI).
#pragma once
#include <cstdint>
#include <string>
#include <memory>
#include <utility>
#include <vector>

#include "rt_device.h"
#include "../../include/rt.h"

namespace rt {

// Status + message, thrown inside the library and converted at the ABI.
struct Error {
    int status;
    std::string msg;
};

// std::vector storage whose resize() leaves elements uninitialised: arrays
// that a parallel loop fills completely are first touched by the threads that
// write them, not zero-filled by one thread beforehand.
template <class T>
struct UninitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = UninitAlloc<U>; };
    UninitAlloc() = default;
    template <class U> UninitAlloc(const UninitAlloc<U>&) noexcept {}
    template <class U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <class T>
using uvector = std::vector<T, UninitAlloc<T>>;

// Triangle soup in loader order with the per-triangle values the reference
// precomputes (triangle.hpp:14-19, getMin/getMax :27-38), stored SoA.
struct Soup {
    uint64_t n = 0;
    uvector<double> v;               // n*9: v0, v1, v2
    uvector<double> c[3];            // centre per axis
    uvector<double> lo[3], hi[3];    // per-triangle box
    uvector<double> normal;          // n*3
};
Soup make_soup(const double* tri_v, uint64_t n);

// One node of the reference tree (stack_bvh.hpp:13-18): a contiguous range of
// the owned primitive vector and its children.
struct RNode {
    double mn[3], mx[3];
    int64_t begin, end;
    std::vector<int32_t> kids;
    int32_t parent = -1;
};

struct Tree {
    std::vector<RNode> nodes;     // nodes[0] = root
    std::vector<uint32_t> order;  // owned primitive vector (loader indices)
};

// StackBVH::build + partition fn + collapse (stack_bvh.hpp:26-608).
Tree build_tree(const Soup& s, int algo, int k, int collapse);

// Walk tree (walk_tree.cpp): the binary SAH tree the device traversal walks
// after collapsing it into W-wide nodes.  Leaves are [first, first + count)
// ranges of `order` (loader indices).
struct WalkNode {
    double mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    int32_t left = -1, right = -1;  // inner node: both >= 0
    uint32_t first = 0, count = 0;  // leaf
};
struct WalkTree {
    std::vector<WalkNode> nodes;  // nodes[0] = root
    std::vector<uint32_t> order;  // triangle (loader) index per walk position
    // Planned W-wide collapse (plan_wide_collapse): for a binary node that
    // becomes a wide node, its slots are wide_kids[wide_off[b] ..
    // wide_off[b] + wide_cnt[b]); empty = the greedy collapse.
    std::vector<uint32_t> wide_off;
    std::vector<uint8_t> wide_cnt;
    std::vector<int32_t> wide_kids;
};
WalkTree build_walk_tree(const Soup& s);
// SAH-optimal W-wide collapse of the binary walk tree (dynamic programme over
// slot counts; subtrees of <= RT_WALK_PMAX triangles may become one leaf).
// Rewrites the chosen subtrees as leaves in place and records the slots of
// every wide node.  RT_WALK_COLLAPSE=greedy leaves the tree untouched.
void plan_wide_collapse(WalkTree& w, int W);
// Treelet restructuring of the binary walk tree (RT_WALK_TREELET = passes,
// 0 = off; walk_tree.cpp), before plan_wide_collapse.
void restructure_treelets(WalkTree& w, int passes);
int walk_treelet_passes();
// The same binned-SAH tree built on a gfx950 device (walk_build.hip): equal
// splits, device-stable order inside nodes.
WalkTree build_walk_tree_device(const Soup& s, int device, int lmax, double node_cost);
int walk_max_leaf();       // RT_WALK_LEAF (leaf size bound of the walk tree)
double walk_node_cost();   // RT_WALK_CT (SAH cost of a node visit)
std::vector<int32_t> collapse_children(const WalkTree& w, int32_t b, int W);
// 8-bit quantised copy of W = 8 wide nodes (RT_QNODE_BYTES each; walk_tree.cpp).
std::vector<uint8_t> quantize_wide8(const uint8_t* wide, uint64_t n_nodes);

// Device-format scene (wide fp32 nodes + fp64 leaf data), built from Tree.
struct Flat {
    int width = 8;                        // W
    uint32_t root_ref = 0;
    uint32_t root_meta = 0;               // the root's sort axis | valid slots << 2 (child records carry their node's)
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    double pad = 0, coord_max = 0;        // max |coordinate| (sizes the per-frame margin)
    std::vector<uint8_t> wide;            // wide nodes, node_bytes(W) each
    uint64_t n_wide = 0;
    uvector<double> tri64;                // BVH order: v0, e1, e2 (9 doubles)
    uvector<float> tri32;                 // BVH order: v0, e1, e2 (fp32, 12 floats padded)
    uvector<uint32_t> tri_id, tri_rank, tri_leaf;
    std::vector<double> rbox;             // real nodes: 6 doubles
    std::vector<int32_t> rparent;         // real nodes: parent
    std::vector<uint32_t> rkid_off, rkid, rrange;  // real tree in CSR form
    std::vector<uint32_t> ref2walk;       // reference-order position -> walk-order (BVH-order) index
    bool walk = false;                    // wide nodes come from the walk tree (not the reference tree)
    uint32_t stack_bound = 0;
    uint32_t depth = 0, max_children = 0, max_leaf = 0;
    uint64_t real_inner = 0, real_leaves = 0;
};
// walk: when non-null, the wide nodes and the per-triangle order come from
// the walk tree (W = 8); the reference tree still supplies ranks and chains.
Flat flatten(const Soup& s, const Tree& t, int width_hint, const WalkTree* walk = nullptr);

// Camera helpers (camera.hpp:20-38, main.cpp:325-329, camera_path.hpp:18-26)
void pixel_constants(int W, int H, double& iw, double& ih, double& half, double& aspect);
void pixel_caches(int W, int H, std::vector<double>& px, std::vector<double>& py);
void camera_basis(const double dir[3], double right[3], double up[3]);
void camera_path(const double center[3], int res, int step, double pos[3], double dir[3]);
void scene_center(const double* tri_v, uint64_t n, double out[3]);

// OBJ ingestion with objl semantics (lib/OBJ_Loader.h:431-1003).
std::vector<double> load_obj(const std::string& path, double scale);
// The same through the binary scene cache in cache_dir (scene_cache.cpp);
// *hit: the entry was valid and used.
std::vector<double> load_obj_cached(const std::string& path, double scale, const std::string& cache_dir, bool* hit);

}  // namespace rt
