// ============================================================================
// oracle/rt_oracle.cpp  —  TEST INFRASTRUCTURE ONLY (the parity checker).
//
// A plain, single-purpose CPU restatement of insomnick/raytracingdemo's
// primary-ray path, written from the reference's behaviour (not copied):
//   OBJ ingestion  (lib/OBJ_Loader.h:321-394, 431-713, 727-1003;
//                   src/utils/object_loader.hpp:14-70)
//   Triangle       (src/primitives/triangle.hpp:14-88)
//   StackBVH       (src/stack_bvh.hpp:26-608 build/partition/collapse,
//                   :611-644 traverse — literal: no culling, no ordering)
//   AABB::hit      (src/aabb.hpp:32-49)
//   Camera / path  (src/camera.hpp:20-38, src/camera_path.hpp:18-26)
//   calculateScreen / shadeScreen (src/main.cpp:322-381)
//   PPM encoding   (src/utils/benchmark.hpp:87-117)
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this library.  The product (raytracingdemo_amd/) never links it.
//
// Pinning: tests/test_oracle.py checks this restatement against the
// reference's own published goldens (testruns_final/ PPM digests and
// shading_times.csv hit counts, committed under tests/golden/) and against
// oracle/_ref (the reference headers compiled by oracle/Makefile) when built.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fopenmp).  FP
// contraction is disabled: the reference ran on x86-64 without FMA.
// ============================================================================
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <numbers>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ---------------------------------------------------------------- Vector3
// src/primitives/vector3.hpp:41-95.  Every op keeps the reference's order.
struct V3 {
    double x = 0, y = 0, z = 0;
};
inline V3 add(const V3& a, const V3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(const V3& a, const V3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(const V3& a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(const V3& a, const V3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double length(const V3& a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline V3 normalize(const V3& a) {  // vector3.hpp:91-95 — divides by length
    double len = length(a);
    if (len == 0) return {0, 0, 0};
    return {a.x / len, a.y / len, a.z / len};
}
inline double axis_of(const V3& a, int axis) { return axis == 0 ? a.x : (axis == 1 ? a.y : a.z); }
// std::min / std::max (two-argument) semantics, incl. NaN behaviour
inline double smin(double a, double b) { return (b < a) ? b : a; }
inline double smax(double a, double b) { return (a < b) ? b : a; }

// ---------------------------------------------------------------- Triangle
// src/primitives/triangle.hpp:14-19 (ctor), :27-38 (min/max of 3 via
// initializer-list min/max: first-smallest / first-largest).
struct Tri {
    V3 v0, v1, v2, normal, center, bmin, bmax;
};
inline double min3(double a, double b, double c) { double m = a; if (b < m) m = b; if (c < m) m = c; return m; }
inline double max3(double a, double b, double c) { double m = a; if (m < b) m = b; if (m < c) m = c; return m; }
Tri make_tri(const V3& a, const V3& b, const V3& c) {
    Tri t;
    t.v0 = a; t.v1 = b; t.v2 = c;
    t.normal = normalize(cross(sub(b, a), sub(c, a)));
    t.center = mul(add(add(a, b), c), 1.0 / 3);
    t.bmin = {min3(a.x, b.x, c.x), min3(a.y, b.y, c.y), min3(a.z, b.z, c.z)};
    t.bmax = {max3(a.x, b.x, c.x), max3(a.y, b.y, c.y), max3(a.z, b.z, c.z)};
    return t;
}

// ---------------------------------------------------------------- Ray
// src/primitives/ray.hpp:13-19: +inf reciprocal for an exactly-zero component.
struct Ray {
    V3 o, d, inv;
};
inline Ray make_ray(const V3& o, const V3& d) {
    const double inf = std::numeric_limits<double>::infinity();
    return {o, d, {d.x != 0.0 ? 1.0 / d.x : inf, d.y != 0.0 ? 1.0 / d.y : inf, d.z != 0.0 ? 1.0 / d.z : inf}};
}

// AABB::hit, src/aabb.hpp:32-49 — slab test, interval not clipped to [0,inf).
inline bool box_hit(const V3& mn, const V3& mx, const Ray& r) {
    double tx1 = (mn.x - r.o.x) * r.inv.x;
    double tx2 = (mx.x - r.o.x) * r.inv.x;
    double tmin = smin(tx1, tx2);
    double tmax = smax(tx1, tx2);
    double ty1 = (mn.y - r.o.y) * r.inv.y;
    double ty2 = (mx.y - r.o.y) * r.inv.y;
    tmin = smax(tmin, smin(ty1, ty2));
    tmax = smin(tmax, smax(ty1, ty2));
    double tz1 = (mn.z - r.o.z) * r.inv.z;
    double tz2 = (mx.z - r.o.z) * r.inv.z;
    tmin = smax(tmin, smin(tz1, tz2));
    tmax = smin(tmax, smax(tz1, tz2));
    return tmax >= tmin;
}

// Möller–Trumbore, src/primitives/triangle.hpp:40-62 (+ :64-88 which repeats
// the same arithmetic and returns o + d*t).  Returns t or -1 on a miss.
inline bool tri_hit(const Tri& T, const Ray& r, double& t_out) {
    const double EPS = 1e-8;
    V3 e1 = sub(T.v1, T.v0);
    V3 e2 = sub(T.v2, T.v0);
    V3 h = cross(r.d, e2);
    double a = dot(e1, h);
    if (a > -EPS && a < EPS) return false;
    double f = 1.0 / a;
    V3 s = sub(r.o, T.v0);
    double u = f * dot(s, h);
    if (u < 0.0 || u > 1.0) return false;
    V3 q = cross(s, e1);
    double v = f * dot(r.d, q);
    if (v < 0.0 || u + v > 1.0) return false;
    double t = f * dot(e2, q);
    if (!(t > EPS)) return false;
    t_out = t;
    return true;
}

// ---------------------------------------------------------------- OBJ
// Restatement of objl::Loader (lib/OBJ_Loader.h, vendored Bly7/OBJ-Loader)
// as used by ObjectLoader::loadFromFile (src/utils/object_loader.hpp:14-70).
struct F3 {
    float X = 0, Y = 0, Z = 0;
};
inline bool feq(const F3& a, const F3& b) { return a.X == b.X && a.Y == b.Y && a.Z == b.Z; }
inline F3 fsub(const F3& a, const F3& b) { return {a.X - b.X, a.Y - b.Y, a.Z - b.Z}; }
inline F3 fcross(const F3& a, const F3& b) {
    return {a.Y * b.Z - a.Z * b.Y, a.Z * b.X - a.X * b.Z, a.X * b.Y - a.Y * b.X};
}
inline float fdot(const F3& a, const F3& b) { return (a.X * b.X) + (a.Y * b.Y) + (a.Z * b.Z); }
inline float fmag(const F3& a) { return sqrtf(powf(a.X, 2) + powf(a.Y, 2) + powf(a.Z, 2)); }

// OBJ_Loader.h:321-357 — the library's peculiar splitter (empty fields kept)
void objl_split(const std::string& in, std::vector<std::string>& out, const std::string& tok) {
    out.clear();
    std::string temp;
    for (int i = 0; i < int(in.size()); i++) {
        std::string test = in.substr(i, tok.size());
        if (test == tok) {
            if (!temp.empty()) {
                out.push_back(temp);
                temp.clear();
                i += (int)tok.size() - 1;
            } else {
                out.push_back("");
            }
        } else if (i + tok.size() >= in.size()) {
            temp += in.substr(i, tok.size());
            out.push_back(temp);
            break;
        } else {
            temp += in[i];
        }
    }
}
// OBJ_Loader.h:360-375
std::string objl_tail(const std::string& in) {
    size_t a = in.find_first_not_of(" \t");
    size_t sp = in.find_first_of(" \t", a);
    size_t b = in.find_first_not_of(" \t", sp);
    size_t e = in.find_last_not_of(" \t");
    if (b != std::string::npos && e != std::string::npos) return in.substr(b, e - b + 1);
    if (b != std::string::npos) return in.substr(b);
    return "";
}
// OBJ_Loader.h:378-394
std::string objl_first(const std::string& in) {
    if (in.empty()) return "";
    size_t a = in.find_first_not_of(" \t");
    size_t e = in.find_first_of(" \t", a);
    if (a != std::string::npos && e != std::string::npos) return in.substr(a, e - a);
    if (a != std::string::npos) return in.substr(a);
    return "";
}
struct LoadError {
    std::string msg;
};
float parse_f(const std::string& s) {  // std::stof
    errno = 0;
    const char* c = s.c_str();
    char* end = nullptr;
    float v = strtof(c, &end);
    if (end == c) throw LoadError{"stof: no conversion"};
    if (errno == ERANGE) throw LoadError{"stof: out of range"};
    return v;
}
int parse_i(const std::string& s) {  // std::stoi
    errno = 0;
    const char* c = s.c_str();
    char* end = nullptr;
    long v = strtol(c, &end, 10);
    if (end == c) throw LoadError{"stoi: no conversion"};
    if (errno == ERANGE || v < INT32_MIN || v > INT32_MAX) throw LoadError{"stoi: out of range"};
    return (int)v;
}
// OBJ_Loader.h:398-406 (1-based; negative = relative to the end)
const F3& objl_elem(const std::vector<F3>& v, const std::string& s) {
    int idx = parse_i(s);
    if (idx < 0) idx = int(v.size()) + idx; else idx--;
    if (idx < 0 || idx >= int(v.size())) throw LoadError{"face index out of range"};
    return v[idx];
}
// OBJ_Loader.h:273-318
bool same_side(const F3& p1, const F3& p2, const F3& a, const F3& b) {
    F3 cp1 = fcross(fsub(b, a), fsub(p1, a));
    F3 cp2 = fcross(fsub(b, a), fsub(p2, a));
    return fdot(cp1, cp2) >= 0;
}
bool in_triangle(const F3& p, const F3& t1, const F3& t2, const F3& t3) {
    bool prism = same_side(p, t1, t2, t3) && same_side(p, t2, t1, t3) && same_side(p, t3, t1, t2);
    if (!prism) return false;
    F3 n = fcross(fsub(t2, t1), fsub(t3, t1));
    float m = fmag(n);
    F3 bn = {n.X / m, n.Y / m, n.Z / m};
    float d = fdot(p, bn);
    F3 proj = {bn.X * d, bn.Y * d, bn.Z * d};
    return fmag(proj) == 0;
}
// OBJ_Loader.h:838-1003 — ear clipping that emits indices by *position
// equality* against the face's vertex list, in ascending list order.
void objl_triangulate(std::vector<unsigned>& out, const std::vector<F3>& iv) {
    if (iv.size() < 3) return;
    if (iv.size() == 3) { out.push_back(0); out.push_back(1); out.push_back(2); return; }
    std::vector<F3> tv = iv;
    auto emit3 = [&](const F3& a, const F3& b, const F3& c, size_t upto) {
        for (size_t j = 0; j < upto; j++) {
            if (feq(iv[j], a)) out.push_back((unsigned)j);
            if (feq(iv[j], b)) out.push_back((unsigned)j);
            if (feq(iv[j], c)) out.push_back((unsigned)j);
        }
    };
    while (true) {
        for (int i = 0; i < int(tv.size()); i++) {
            F3 prev = (i == 0) ? tv[tv.size() - 1] : tv[i - 1];
            F3 cur = tv[i];
            F3 next = (i == int(tv.size()) - 1) ? tv[0] : tv[i + 1];
            if (tv.size() == 3) {  // last triangle: scans only tv.size() entries of iv
                emit3(cur, prev, next, tv.size());
                tv.clear();
                break;
            }
            if (tv.size() == 4) {
                emit3(cur, prev, next, iv.size());
                F3 other;
                for (size_t j = 0; j < tv.size(); j++) {
                    if (!feq(tv[j], cur) && !feq(tv[j], prev) && !feq(tv[j], next)) { other = tv[j]; break; }
                }
                for (size_t j = 0; j < iv.size(); j++) {
                    if (feq(iv[j], prev)) out.push_back((unsigned)j);
                    if (feq(iv[j], next)) out.push_back((unsigned)j);
                    if (feq(iv[j], other)) out.push_back((unsigned)j);
                }
                tv.clear();
                break;
            }
            // (the library's angle test `angle <= 0 && angle >= 180` never fires)
            bool inside = false;
            for (size_t j = 0; j < iv.size(); j++) {
                if (in_triangle(iv[j], prev, cur, next) && !feq(iv[j], prev) && !feq(iv[j], cur) &&
                    !feq(iv[j], next)) { inside = true; break; }
            }
            if (inside) continue;
            emit3(cur, prev, next, iv.size());
            for (size_t j = 0; j < tv.size(); j++) {
                if (feq(tv[j], cur)) { tv.erase(tv.begin() + j); break; }
            }
            i = -1;
        }
        if (out.empty()) break;
        if (tv.empty()) break;
    }
}

struct Mesh {
    std::vector<F3> verts;  // only positions matter downstream
    std::vector<unsigned> idx;
};

// OBJ_Loader.h:431-713 (positions only) + ObjectLoader (object_loader.hpp:14-70)
std::vector<Tri> load_obj(const std::string& path, double scale) {
    if (path.size() < 4 || path.substr(path.size() - 4, 4) != ".obj") throw LoadError{"not an .obj path"};
    std::ifstream f(path);
    if (!f.is_open()) throw LoadError{"cannot open " + path};
    std::vector<F3> pos;
    std::vector<Mesh> meshes;
    Mesh cur;
    bool listening = false;
    size_t loaded_vertices = 0;
    std::string line;
    std::vector<std::string> parts, sv;
    while (std::getline(f, line)) {
        std::string ft = objl_first(line);
        if (ft == "o" || ft == "g" || (!line.empty() && line[0] == 'g')) {
            if (!listening) {
                listening = true;
            } else if (!cur.idx.empty() && !cur.verts.empty()) {
                meshes.push_back(cur);
                cur = Mesh{};
            }
        }
        if (ft == "v") {
            objl_split(objl_tail(line), parts, " ");
            if (parts.size() < 3) throw LoadError{"short v line"};
            F3 p;
            p.X = parse_f(parts[0]);
            p.Y = parse_f(parts[1]);
            p.Z = parse_f(parts[2]);
            pos.push_back(p);
        }
        if (ft == "f") {
            objl_split(objl_tail(line), parts, " ");
            std::vector<F3> fv;
            for (auto& s : parts) {
                objl_split(s, sv, "/");
                if (sv.size() < 1 || sv.size() > 3) continue;  // library: vtype undefined -> skip
                fv.push_back(objl_elem(pos, sv[0]));
            }
            size_t base = cur.verts.size();
            for (auto& v : fv) cur.verts.push_back(v);
            loaded_vertices += fv.size();
            std::vector<unsigned> tri_idx;
            objl_triangulate(tri_idx, fv);
            for (unsigned k : tri_idx) cur.idx.push_back((unsigned)base + k);
        }
        if (ft == "usemtl") {
            if (!cur.idx.empty() && !cur.verts.empty()) {
                meshes.push_back(cur);
                cur = Mesh{};
            }
        }
    }
    if (!cur.idx.empty() && !cur.verts.empty()) meshes.push_back(cur);
    if (meshes.empty() && loaded_vertices == 0) throw LoadError{"Failed to load OBJ file: " + path};
    std::vector<Tri> tris;
    for (const Mesh& m : meshes) {
        for (size_t i = 0; i + 2 < m.idx.size(); i += 3) {
            unsigned a = m.idx[i], b = m.idx[i + 1], c = m.idx[i + 2];
            if (a >= m.verts.size() || b >= m.verts.size() || c >= m.verts.size()) continue;
            V3 A{(double)m.verts[a].X, (double)m.verts[a].Y, (double)m.verts[a].Z};
            V3 B{(double)m.verts[b].X, (double)m.verts[b].Y, (double)m.verts[b].Z};
            V3 C{(double)m.verts[c].X, (double)m.verts[c].Y, (double)m.verts[c].Z};
            tris.push_back(make_tri(mul(A, scale), mul(B, scale), mul(C, scale)));
        }
    }
    return tris;
}

// ---------------------------------------------------------------- StackBVH
// src/stack_bvh.hpp.  Tree nodes hold a contiguous range of `order`
// (the BVH's owned primitive vector, :21/:506) and child node indices.
struct Node {
    V3 mn, mx;
    int begin = 0, end = 0;
    std::vector<int> kids;
};
struct BVH {
    std::vector<Tri> tris;   // loader order
    std::vector<int> order;  // owned primitive vector (indices into tris)
    std::vector<Node> nodes; // nodes[0] = root
};

// :26-52
void find_bounds(const BVH& b, int lo, int hi, V3& mn, V3& mx) {
    if (lo == hi) { mn = {0, 0, 0}; mx = {0, 0, 0}; return; }
    double ax = std::numeric_limits<double>::max(), ay = ax, az = ax;
    double bx = std::numeric_limits<double>::lowest(), by = bx, bz = bx;
    for (int i = lo; i < hi; i++) {
        const Tri& t = b.tris[b.order[i]];
        ax = smin(ax, t.bmin.x); ay = smin(ay, t.bmin.y); az = smin(az, t.bmin.z);
        bx = smax(bx, t.bmax.x); by = smax(by, t.bmax.y); bz = smax(bz, t.bmax.z);
    }
    mn = {ax, ay, az};
    mx = {bx, by, bz};
}
// :54-63
int longest_axis(const V3& mn, const V3& mx) {
    V3 e = sub(mx, mn);
    if (e.y > e.x && e.y >= e.z) return 1;
    if (e.z > e.x && e.z >= e.y) return 2;
    return 0;
}
// :65-69, :118-122, :263-267
inline double area(const V3& mn, const V3& mx) {
    V3 e = sub(mx, mn);
    return 2.0 * (e.x * e.y + e.y * e.z + e.z * e.x);
}
// :71-76
inline bool is_leaf(size_t n, int k) { return n <= (size_t)k || k < 2; }

struct ByCenter {
    const BVH* b;
    int axis;
    bool operator()(int p, int q) const {
        return axis_of(b->tris[p].center, axis) < axis_of(b->tris[q].center, axis);
    }
};

// :79-100
std::vector<size_t> split_median(BVH& b, int lo, int hi, int axis, int k) {
    const long n = hi - lo;
    if (is_leaf((size_t)n, k)) return {};
    std::vector<size_t> s;
    for (int i = 1; i < k; ++i) {
        size_t sp = (size_t)(n * i) / k;
        if (sp == 0 || sp >= (size_t)n) break;
        s.push_back(sp);
    }
    auto first = b.order.begin() + lo;
    auto rb = first;
    for (size_t sp : s) {
        std::nth_element(rb, first + (std::ptrdiff_t)sp, b.order.begin() + hi, ByCenter{&b, axis});
        rb = first + sp + 1;
    }
    return s;
}

// :103-239
std::vector<size_t> split_sah(BVH& b, int lo, int hi, int axis, int k) {
    const long range = hi - lo;
    if (is_leaf((size_t)range, k)) return {};
    std::sort(b.order.begin() + lo, b.order.begin() + hi, ByCenter{&b, axis});
    auto prim = [&](size_t i) -> const Tri& { return b.tris[b.order[lo + i]]; };
    struct Seg { size_t b, e; };
    std::vector<Seg> segs{{0, (size_t)range}};
    auto seg_cost = [&](const Seg& s) {
        double ax = std::numeric_limits<double>::max(), ay = ax, az = ax;
        double bx = std::numeric_limits<double>::lowest(), by = bx, bz = bx;
        for (size_t i = s.b; i < s.e; ++i) {
            const Tri& t = prim(i);
            ax = smin(ax, t.bmin.x); bx = smax(bx, t.bmax.x);
            ay = smin(ay, t.bmin.y); by = smax(by, t.bmax.y);
            az = smin(az, t.bmin.z); bz = smax(bz, t.bmax.z);
        }
        return area({ax, ay, az}, {bx, by, bz}) * (double)(s.e - s.b);
    };
    std::vector<size_t> splits;
    while (segs.size() < (size_t)k) {
        size_t pick = SIZE_MAX;
        double worst = -1.0;
        for (size_t i = 0; i < segs.size(); ++i) {
            if (segs[i].e - segs[i].b < 2) continue;
            double c = seg_cost(segs[i]);
            if (c > worst) { worst = c; pick = i; }
        }
        if (pick == SIZE_MAX) break;
        Seg sg = segs[pick];
        size_t cnt = sg.e - sg.b;
        std::vector<V3> pmn(cnt), pmx(cnt), smn(cnt), smx(cnt);
        for (size_t q = 0; q < cnt; ++q) {
            const Tri& t = prim(sg.b + q);
            if (q == 0) { pmn[q] = t.bmin; pmx[q] = t.bmax; continue; }
            pmn[q] = {smin(pmn[q - 1].x, t.bmin.x), smin(pmn[q - 1].y, t.bmin.y), smin(pmn[q - 1].z, t.bmin.z)};
            pmx[q] = {smax(pmx[q - 1].x, t.bmax.x), smax(pmx[q - 1].y, t.bmax.y), smax(pmx[q - 1].z, t.bmax.z)};
        }
        for (size_t q = cnt; q-- > 0;) {
            const Tri& t = prim(sg.b + q);
            if (q == cnt - 1) { smn[q] = t.bmin; smx[q] = t.bmax; continue; }
            smn[q] = {smin(smn[q + 1].x, t.bmin.x), smin(smn[q + 1].y, t.bmin.y), smin(smn[q + 1].z, t.bmin.z)};
            smx[q] = {smax(smx[q + 1].x, t.bmax.x), smax(smx[q + 1].y, t.bmax.y), smax(smx[q + 1].z, t.bmax.z)};
        }
        size_t best_off = 1;
        double best = std::numeric_limits<double>::max();
        for (size_t sp = 1; sp < cnt; ++sp) {
            double c = area(pmn[sp - 1], pmx[sp - 1]) * sp + area(smn[sp], smx[sp]) * (cnt - sp);
            if (c < best) { best = c; best_off = sp; }
        }
        size_t abs_split = sg.b + best_off;
        splits.push_back(abs_split);
        segs.erase(segs.begin() + pick);
        segs.push_back({sg.b, abs_split});
        segs.push_back({abs_split, sg.e});
    }
    return splits;
}

// :241-449 — 16 bins over the centre range on `axis`.
std::vector<size_t> split_binned(BVH& b, int lo, int hi, int axis, int k) {
    const int NB = 16;
    const long range = hi - lo;
    if (is_leaf((size_t)range, k)) return {};
    std::sort(b.order.begin() + lo, b.order.begin() + hi, ByCenter{&b, axis});
    struct Bin {
        int count = 0;
        V3 mn{std::numeric_limits<double>::max(), std::numeric_limits<double>::max(), std::numeric_limits<double>::max()};
        V3 mx{std::numeric_limits<double>::lowest(), std::numeric_limits<double>::lowest(), std::numeric_limits<double>::lowest()};
    };
    double cmin = std::numeric_limits<double>::max();
    double cmax = std::numeric_limits<double>::lowest();
    for (int i = lo; i < hi; ++i) {
        double c = axis_of(b.tris[b.order[i]].center, axis);
        cmin = smin(cmin, c);
        cmax = smax(cmax, c);
    }
    double br = cmax - cmin;
    if (br < 1e-10) br = 1.0;
    std::vector<Bin> bins(NB);
    for (int i = lo; i < hi; ++i) {
        const Tri& t = b.tris[b.order[i]];
        int bi = static_cast<int>(((axis_of(t.center, axis) - cmin) / br) * NB);
        bi = std::clamp(bi, 0, NB - 1);
        Bin& B = bins[bi];
        B.mn = {smin(B.mn.x, t.bmin.x), smin(B.mn.y, t.bmin.y), smin(B.mn.z, t.bmin.z)};
        B.mx = {smax(B.mx.x, t.bmax.x), smax(B.mx.y, t.bmax.y), smax(B.mx.z, t.bmax.z)};
        B.count++;
    }
    struct Seg { size_t b, e; };
    std::vector<Seg> segs{{0, (size_t)NB}};
    auto seg_cost = [&](const Seg& s) {
        double ax = std::numeric_limits<double>::max(), ay = ax, az = ax;
        double bx = std::numeric_limits<double>::lowest(), by = bx, bz = bx;
        int n = 0;
        for (size_t i = s.b; i < s.e; ++i) {
            ax = smin(ax, bins[i].mn.x); bx = smax(bx, bins[i].mx.x);
            ay = smin(ay, bins[i].mn.y); by = smax(by, bins[i].mx.y);
            az = smin(az, bins[i].mn.z); bz = smax(bz, bins[i].mx.z);
        }
        for (size_t i = s.b; i < s.e; ++i) n += bins[i].count;
        return area({ax, ay, az}, {bx, by, bz}) * (double)n;
    };
    std::vector<size_t> splits;
    while (segs.size() < (size_t)k) {
        size_t pick = SIZE_MAX;
        double worst = -1.0;
        for (size_t i = 0; i < segs.size(); ++i) {
            if (segs[i].e - segs[i].b < 2) continue;
            double c = seg_cost(segs[i]);
            if (c > worst) { worst = c; pick = i; }
        }
        if (pick == SIZE_MAX) break;
        Seg sg = segs[pick];
        size_t cnt = sg.e - sg.b;
        std::vector<V3> pmn(cnt), pmx(cnt), smn(cnt), smx(cnt);
        for (size_t q = 0; q < cnt; ++q) {
            const Bin& B = bins[sg.b + q];
            if (q == 0) { pmn[q] = B.mn; pmx[q] = B.mx; continue; }
            pmn[q] = {smin(pmn[q - 1].x, B.mn.x), smin(pmn[q - 1].y, B.mn.y), smin(pmn[q - 1].z, B.mn.z)};
            pmx[q] = {smax(pmx[q - 1].x, B.mx.x), smax(pmx[q - 1].y, B.mx.y), smax(pmx[q - 1].z, B.mx.z)};
        }
        for (size_t q = cnt; q-- > 0;) {
            const Bin& B = bins[sg.b + q];
            if (q == cnt - 1) { smn[q] = B.mn; smx[q] = B.mx; continue; }
            smn[q] = {smin(smn[q + 1].x, B.mn.x), smin(smn[q + 1].y, B.mn.y), smin(smn[q + 1].z, B.mn.z)};
            smx[q] = {smax(smx[q + 1].x, B.mx.x), smax(smx[q + 1].y, B.mx.y), smax(smx[q + 1].z, B.mx.z)};
        }
        size_t best_sp = 1;
        int left = 0, right = 0;
        for (size_t q = 0; q < cnt; ++q) right += bins[sg.b + q].count;
        double best = std::numeric_limits<double>::max();
        for (size_t sp = 1; sp < cnt; ++sp) {
            left += bins[sg.b + sp - 1].count;
            right -= bins[sg.b + sp - 1].count;
            double c = area(pmn[sp - 1], pmx[sp - 1]) * left + area(smn[sp], smx[sp]) * right;
            if (c < best) { best = c; best_sp = sp; }
        }
        size_t prim_split = 0;  // prims in bins [0, seg.b + best_sp)
        for (size_t q = 0; q < sg.b + best_sp; ++q) prim_split += bins[q].count;
        splits.push_back(prim_split);
        segs.erase(segs.begin() + pick);
        segs.push_back({sg.b, sg.b + best_sp});
        segs.push_back({sg.b + best_sp, sg.e});
    }
    std::sort(splits.begin(), splits.end());
    splits.erase(std::unique(splits.begin(), splits.end()), splits.end());
    return splits;
}

enum { ALGO_MEDIAN = 0, ALGO_SAH = 1, ALGO_BSAH = 2 };

struct BuildError {
    std::string msg;
};

// :502-571
void build(BVH& b, int algo, int k) {
    b.order.resize(b.tris.size());
    for (size_t i = 0; i < b.tris.size(); i++) b.order[i] = (int)i;
    b.nodes.clear();
    Node root;
    root.begin = 0;
    root.end = (int)b.tris.size();
    if (b.tris.empty()) { b.nodes.push_back(root); return; }
    find_bounds(b, 0, root.end, root.mn, root.mx);
    b.nodes.push_back(root);
    std::vector<int> work{0};
    while (!work.empty()) {
        int ni = work.back();
        work.pop_back();
        int lo = b.nodes[ni].begin, hi = b.nodes[ni].end;
        if (hi - lo <= 1) continue;
        int axis = longest_axis(b.nodes[ni].mn, b.nodes[ni].mx);
        std::vector<size_t> s;
        if (algo == ALGO_MEDIAN) s = split_median(b, lo, hi, axis, k);
        else if (algo == ALGO_SAH) s = split_sah(b, lo, hi, axis, k);
        else s = split_binned(b, lo, hi, axis, k);
        if (s.empty()) continue;
        std::sort(s.begin(), s.end());
        int rb = lo;
        std::vector<int> kids;
        for (size_t sp : s) {
            if (sp == 0 || sp >= (size_t)(hi - lo)) throw BuildError{"invalid split position"};
            int re = lo + (int)sp;
            if (rb >= re) throw BuildError{"Invalid iterator range"};
            Node c;
            c.begin = rb; c.end = re;
            find_bounds(b, rb, re, c.mn, c.mx);
            kids.push_back((int)b.nodes.size());
            b.nodes.push_back(c);
            rb = re;
        }
        Node c;
        c.begin = rb; c.end = hi;
        find_bounds(b, rb, hi, c.mn, c.mx);
        kids.push_back((int)b.nodes.size());
        b.nodes.push_back(c);
        b.nodes[ni].kids = kids;
        for (int kx : kids) work.push_back(kx);
    }
}

// :574-608 — one pass: every visited node adopts its grandchildren.
void collapse_once(BVH& b) {
    std::vector<int> st{0};
    while (!st.empty()) {
        int ni = st.back();
        st.pop_back();
        if (b.nodes[ni].kids.empty()) continue;
        std::vector<int> nk;
        for (int c : b.nodes[ni].kids) {
            if (!b.nodes[c].kids.empty()) for (int g : b.nodes[c].kids) nk.push_back(g);
            else nk.push_back(c);
        }
        b.nodes[ni].kids = nk;
        for (int c : nk) st.push_back(c);
    }
}

// :611-644 — literal closest-hit traversal.  Returns loader index or -1.
struct TravStats {
    uint64_t box_tests = 0, box_hits = 0, tri_tests = 0;
};
int traverse(const BVH& b, const Ray& r, V3& hit_pos, double& hit_dist, std::vector<int>& st, TravStats& ts) {
    st.clear();
    st.push_back(0);
    int best = -1;
    double bestd = std::numeric_limits<double>::max();
    while (!st.empty()) {
        const Node& n = b.nodes[st.back()];
        st.pop_back();
        ts.box_tests++;
        if (!box_hit(n.mn, n.mx, r)) continue;
        ts.box_hits++;
        if (n.kids.empty()) {
            for (int i = n.begin; i < n.end; ++i) {
                int p = b.order[i];
                double t;
                ts.tri_tests++;
                if (!tri_hit(b.tris[p], r, t)) continue;
                V3 pos = add(r.o, mul(r.d, t));
                double d = length(sub(pos, r.o));
                if (d < bestd) { bestd = d; best = p; hit_pos = pos; }
            }
        }
        for (int c : n.kids) st.push_back(c);
    }
    hit_dist = bestd;
    return best;
}

// camera.hpp:20-38 pixel plane caches
void pixel_caches(unsigned W, unsigned H, std::vector<double>& px, std::vector<double>& py) {
    const double fov = 90.0 * (std::numbers::pi / 180.0);
    const double th = std::tan(fov * 0.5);
    const double aspect = static_cast<double>(W) / H;
    px.resize(W);
    py.resize(H);
    const double iw = 1.0 / W, ih = 1.0 / H;
    for (unsigned x = 0; x < W; ++x) px[x] = (2.0 * (x + 0.5) * iw - 1.0) * th * aspect;
    for (unsigned y = 0; y < H; ++y) py[y] = (1.0 - 2.0 * (y + 0.5) * ih) * th;
}

// main.cpp:325-329 camera basis
void basis(const V3& dir, V3& right, V3& up) {
    right = cross(dir, V3{0.0, 1.0, 0.0});
    if (length(right) < 1e-8) right = V3{0.0, 0.0, 1.0};
    right = normalize(right);
    up = normalize(cross(right, dir));
}

// main.cpp:351-381 shading of one pixel
void shade(bool hit, const V3& pos, const V3& nrm, const V3& cam, double rgb[3]) {
    if (!hit) { rgb[0] = rgb[1] = rgb[2] = 0.0; return; }
    V3 N = nrm;
    double nl = length(N);
    if (nl > 0.0) N = mul(N, 1.0 / nl);
    V3 L = sub(cam, pos);
    double dist = length(L);
    if (dist > 0.0) L = mul(L, 1.0 / dist);
    const double ambient = 0.45;
    double diffuse = smax(0.0, dot(N, L)) * 1.35;
    double att = 1.0 / (1.0 + 0.05 * dist * dist);
    double I = std::clamp((ambient + diffuse * att) * 1.25, 0.0, 1.0);
    rgb[0] = (0.5 * (N.x + 1.0)) * I;
    rgb[1] = (0.5 * (N.y + 1.0)) * I;
    rgb[2] = (0.5 * (N.z + 1.0)) * I;
}
// benchmark.hpp:105-114 byte conversion (truncating cast)
inline uint8_t to_byte(double c) { return static_cast<unsigned char>(std::clamp(c * 255.0, 0.0, 255.0)); }

thread_local std::string g_err;

}  // namespace

// ============================================================================
// extern "C" surface (ctypes).  All outputs are caller-owned.  Pixel layout of
// every per-pixel array is row-major (j*W + i); the reference's own storage is
// column-major (main.cpp:339) — that is a layout choice, not a semantic one.
// ============================================================================
extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

// Loads an OBJ into a malloc'd N*9 double array (v0,v1,v2 per triangle,
// loader order, scaled).  Returns N, or -1 on error.
long long orc_load_obj(const char* path, double scale, double** out) {
    try {
        std::vector<Tri> t = load_obj(path, scale);
        double* buf = (double*)malloc(sizeof(double) * 9 * (t.size() ? t.size() : 1));
        for (size_t i = 0; i < t.size(); i++) {
            const V3* v[3] = {&t[i].v0, &t[i].v1, &t[i].v2};
            for (int k = 0; k < 3; k++) {
                buf[i * 9 + k * 3 + 0] = v[k]->x;
                buf[i * 9 + k * 3 + 1] = v[k]->y;
                buf[i * 9 + k * 3 + 2] = v[k]->z;
            }
        }
        *out = buf;
        return (long long)t.size();
    } catch (const LoadError& e) {
        g_err = e.msg;
        return -1;
    }
}
void orc_free(void* p) { free(p); }

// main.cpp:118-122 — mean of triangle centres (sequential sum, then *1/n)
void orc_scene_center(const double* tv, long long n, double out[3]) {
    V3 c{0, 0, 0};
    for (long long i = 0; i < n; i++) {
        Tri t = make_tri({tv[i * 9], tv[i * 9 + 1], tv[i * 9 + 2]}, {tv[i * 9 + 3], tv[i * 9 + 4], tv[i * 9 + 5]},
                         {tv[i * 9 + 6], tv[i * 9 + 7], tv[i * 9 + 8]});
        c = add(c, t.center);
    }
    c = mul(c, 1.0 / static_cast<double>(n));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}

// main.cpp:123,235 + camera_path.hpp:18-26.  `center` is the scene centre;
// the path centre is recomputed exactly as runTest does.
void orc_camera_path(const double center[3], int res, int step, double pos[3], double dir[3]) {
    V3 cam = add(V3{center[0], center[1], center[2]}, V3{0.0, 0.0, 5.0});
    V3 pc = sub(cam, V3{0.0, 0.0, 5.0});
    const double ang = 2.0 * M_PI * (static_cast<double>(step % res) / res);
    const double x = 0.0 * std::cos(ang) - 5.0 * std::sin(ang);
    const double z = 0.0 * std::sin(ang) + 5.0 * std::cos(ang);
    V3 p = add(pc, V3{x, 0.0, z});
    V3 d = normalize(sub(pc, p));
    pos[0] = p.x; pos[1] = p.y; pos[2] = p.z;
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

struct orc_bvh {
    BVH b;
};

// algo: 0 median, 1 sah, 2 binned sah; collapse != 0 => the "-c" variants
// (2-way partition, log2(k)-1 collapse passes; main.cpp:128-139,208,219-221).
orc_bvh* orc_bvh_create(const double* tv, long long n, int algo, int k, int collapse) {
    orc_bvh* h = new orc_bvh;
    h->b.tris.reserve(n);
    for (long long i = 0; i < n; i++)
        h->b.tris.push_back(make_tri({tv[i * 9], tv[i * 9 + 1], tv[i * 9 + 2]},
                                     {tv[i * 9 + 3], tv[i * 9 + 4], tv[i * 9 + 5]},
                                     {tv[i * 9 + 6], tv[i * 9 + 7], tv[i * 9 + 8]}));
    try {
        build(h->b, algo, collapse ? 2 : k);
        if (collapse) {
            int passes = static_cast<int>(std::log2(k)) - 1;
            for (int i = 0; i < passes; i++) collapse_once(h->b);
        }
    } catch (const BuildError& e) {
        g_err = e.msg;
        delete h;
        return nullptr;
    }
    return h;
}
void orc_bvh_destroy(orc_bvh* h) { delete h; }

// Tree statistics: [reachable nodes, inner, leaves, max depth, max children]
void orc_bvh_stats(const orc_bvh* h, long long out[5]) {
    long long nodes = 0, inner = 0, leaves = 0, depth = 0, maxk = 0;
    std::vector<std::pair<int, int>> st{{0, 0}};
    while (!st.empty()) {
        auto [ni, d] = st.back();
        st.pop_back();
        const Node& n = h->b.nodes[ni];
        nodes++;
        depth = std::max<long long>(depth, d);
        if (n.kids.empty()) leaves++;
        else { inner++; maxk = std::max<long long>(maxk, (long long)n.kids.size()); }
        for (int c : n.kids) st.push_back({c, d + 1});
    }
    out[0] = nodes; out[1] = inner; out[2] = leaves; out[3] = depth; out[4] = maxk;
}

// Reference-visit-order dump (pre-order, children visited last-first, as the
// traversal stack of stack_bvh.hpp:639-641 does).  Per reachable node:
// box[6] -> boxes, (begin, end, nkids) -> meta.  `order` gets the owned
// primitive vector.  Arrays sized by orc_bvh_stats()[0] and n.
void orc_bvh_dump(const orc_bvh* h, double* boxes, long long* meta, long long* order) {
    std::vector<int> st{0};
    long long k = 0;
    while (!st.empty()) {
        const Node& n = h->b.nodes[st.back()];
        st.pop_back();
        boxes[k * 6 + 0] = n.mn.x; boxes[k * 6 + 1] = n.mn.y; boxes[k * 6 + 2] = n.mn.z;
        boxes[k * 6 + 3] = n.mx.x; boxes[k * 6 + 4] = n.mx.y; boxes[k * 6 + 5] = n.mx.z;
        meta[k * 3 + 0] = n.begin; meta[k * 3 + 1] = n.end; meta[k * 3 + 2] = (long long)n.kids.size();
        k++;
        for (int c : n.kids) st.push_back(c);
    }
    for (size_t i = 0; i < h->b.order.size(); i++) order[i] = h->b.order[i];
}

// One frame of calculateScreen + shadeScreen (main.cpp:322-381).
// Rows [row0, row0+nrows) of a W x H image are rendered (the timed bounded
// sample of bench.py uses a row band).  Any output pointer may be NULL.
// Outputs are indexed (j-row0)*W + i.  Returns the hit count, or -1.
long long orc_render(const orc_bvh* h, const double cam_pos[3], const double cam_dir[3], int W, int H,
                     int row0, int nrows, int threads, int32_t* hit_id, double* hit_pos, double* hit_nrm,
                     double* hit_dist, uint8_t* rgb, unsigned long long counters[3]) {
    if (W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) { g_err = "bad frame geometry"; return -1; }
    std::vector<double> px, py;
    pixel_caches((unsigned)W, (unsigned)H, px, py);
    const V3 cp{cam_pos[0], cam_pos[1], cam_pos[2]};
    const V3 cd{cam_dir[0], cam_dir[1], cam_dir[2]};
    V3 right, up;
    basis(cd, right, up);
    long long hits = 0;
    unsigned long long c0 = 0, c1 = 0, c2 = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : hits, c0, c1, c2)
#endif
    for (int i = 0; i < W; ++i) {  // column-major loop as main.cpp:331-333
        std::vector<int> st;
        st.reserve(64);
        TravStats ts;
        for (int j = row0; j < row0 + nrows; ++j) {
            V3 d = add(add(cd, mul(up, py[j])), mul(right, px[i]));
            d = mul(d, 1.0 / length(d));
            Ray r = make_ray(cp, d);
            V3 pos;
            double dist;
            int id = traverse(h->b, r, pos, dist, st, ts);
            size_t o = (size_t)(j - row0) * W + i;
            if (hit_id) hit_id[o] = id;
            V3 nrm{0, 0, 0};
            if (id >= 0) { nrm = h->b.tris[id].normal; hits++; }
            if (hit_pos) { hit_pos[o * 3] = pos.x; hit_pos[o * 3 + 1] = pos.y; hit_pos[o * 3 + 2] = pos.z; }
            if (hit_nrm) { hit_nrm[o * 3] = nrm.x; hit_nrm[o * 3 + 1] = nrm.y; hit_nrm[o * 3 + 2] = nrm.z; }
            if (hit_dist) hit_dist[o] = id >= 0 ? dist : -1.0;
            if (rgb) {
                double c[3];
                shade(id >= 0, pos, nrm, cp, c);
                rgb[o * 3] = to_byte(c[0]); rgb[o * 3 + 1] = to_byte(c[1]); rgb[o * 3 + 2] = to_byte(c[2]);
            }
        }
        c0 += ts.box_tests; c1 += ts.box_hits; c2 += ts.tri_tests;
    }
    if (counters) { counters[0] = c0; counters[1] = c1; counters[2] = c2; }
    return hits;
}

// Stratified multi-sample frame (build-defined extension, SURVEY.md §8(d)
// config c4; include/rt.h rt_render_batch_spp_device): spp = n*n samples per
// pixel at sub-pixel offsets (((s % n) + 0.5) / n, ((s / n) + 0.5) / n) in
// place of camera.hpp:35-37's 0.5; per-sample outputs at
// ((j-row0)*W + i)*spp + s; the pixel colour is the samples' shadeScreen
// colours summed in sample order from 0.0, divided by spp, then cast.
// Returns the number of samples that hit, or -1.
long long orc_render_spp(const orc_bvh* h, const double cam_pos[3], const double cam_dir[3], int W, int H,
                         int row0, int nrows, int spp, int threads, int32_t* hit_id, double* hit_pos,
                         double* hit_dist, uint8_t* rgb) {
    if (W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) { g_err = "bad frame geometry"; return -1; }
    int g = 1;
    while ((g + 1) * (g + 1) <= spp) g++;
    if (spp < 1 || g * g != spp) { g_err = "spp must be n*n"; return -1; }
    const double fov = 90.0 * (std::numbers::pi / 180.0);
    const double th = std::tan(fov * 0.5);
    const double aspect = static_cast<double>(W) / H;
    const double iw = 1.0 / W, ih = 1.0 / H;
    const V3 cp{cam_pos[0], cam_pos[1], cam_pos[2]};
    const V3 cd{cam_dir[0], cam_dir[1], cam_dir[2]};
    V3 right, up;
    basis(cd, right, up);
    long long hits = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : hits)
#endif
    for (int i = 0; i < W; ++i) {
        std::vector<int> st;
        st.reserve(64);
        TravStats ts;
        for (int j = row0; j < row0 + nrows; ++j) {
            const size_t o = (size_t)(j - row0) * W + i;
            double acc[3] = {0.0, 0.0, 0.0};
            for (int s = 0; s < spp; ++s) {
                const double ox = ((double)(s % g) + 0.5) / (double)g, oy = ((double)(s / g) + 0.5) / (double)g;
                const double px = (2.0 * (i + ox) * iw - 1.0) * th * aspect;
                const double py = (1.0 - 2.0 * (j + oy) * ih) * th;
                V3 d = add(add(cd, mul(up, py)), mul(right, px));
                d = mul(d, 1.0 / length(d));
                Ray r = make_ray(cp, d);
                V3 pos;
                double dist;
                const int id = traverse(h->b, r, pos, dist, st, ts);
                const size_t so = o * spp + s;
                if (hit_id) hit_id[so] = id;
                if (hit_pos) { hit_pos[so * 3] = pos.x; hit_pos[so * 3 + 1] = pos.y; hit_pos[so * 3 + 2] = pos.z; }
                if (hit_dist) hit_dist[so] = id >= 0 ? dist : -1.0;
                V3 nrm{0, 0, 0};
                if (id >= 0) { nrm = h->b.tris[id].normal; hits++; }
                double c[3];
                shade(id >= 0, pos, nrm, cp, c);
                acc[0] = acc[0] + c[0];
                acc[1] = acc[1] + c[1];
                acc[2] = acc[2] + c[2];
            }
            if (rgb)
                for (int k = 0; k < 3; k++) rgb[o * 3 + k] = to_byte(acc[k] / (double)spp);
        }
    }
    return hits;
}

// ---------------------------------------------------------------- paths
// Diffuse path tracing (build-defined extension, SURVEY.md §8(f) item 3 /
// config c5; GPU: raytracingdemo_amd/csrc/path_kernel.h).
// Every segment is traverse() above, the reference's closest hit.  All fp64
// expressions in the GPU's operation order (this TU: -ffp-contract=off).
}  // extern "C"
namespace {
inline uint32_t h32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
inline uint32_t path_seed(uint32_t frame, uint32_t px, uint32_t s) { return h32(h32(h32(0x5EEDu + frame) + px) + s); }
inline double path_u(uint32_t seed, uint32_t n) { return (double)(h32(seed + n * 0x9E3779B9u) >> 8) * 0x1p-24; }
// sin / cos of 2 pi f by octant + Taylor polynomials (no libm: same bits as the GPU)
void spec_sincos(double f, double& sn, double& cs) {
    const double f8 = f * 8.0;
    const int k = (int)f8;
    const double x = (f8 - (double)k) * 0x1.921fb54442d18p-1;
    const double x2 = x * x;
    const double S[8] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
                         -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49};
    const double Cc[9] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10,
                          0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29,
                          -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53};
    double ps = x2 * S[7];
    for (int q = 6; q >= 0; q--) ps = x2 * (S[q] + ps);
    const double sx = x * (1.0 + ps);
    double pc = x2 * Cc[8];
    for (int q = 7; q >= 0; q--) pc = x2 * (Cc[q] + pc);
    const double cx = 1.0 + pc;
    const double r = 0x1.6a09e667f3bcdp-1;
    static const double SA[8] = {0.0, r, 1.0, r, 0.0, -r, -1.0, -r};
    static const double CA[8] = {1.0, r, 0.0, -r, -1.0, -r, 0.0, r};
    sn = SA[k] * cx + CA[k] * sx;
    cs = CA[k] * cx - SA[k] * sx;
}
// cosine-weighted bounce about n facing against din (Duff et al. 2017 basis),
// normalised by division as Vector3::normalize
V3 bounce_dir(V3 n, const V3& din, double u1, double u2) {
    if (n.x * din.x + n.y * din.y + n.z * din.z > 0.0) n = {-n.x, -n.y, -n.z};
    const double sign = n.z >= 0.0 ? 1.0 : -1.0;
    const double a = -1.0 / (sign + n.z);
    const double b = n.x * n.y * a;
    const V3 t{1.0 + sign * n.x * n.x * a, sign * b, -sign * n.x};
    const V3 bt{b, sign + n.y * n.y * a, -n.y};
    const double rr = std::sqrt(u1);
    double sphi, cphi;
    spec_sincos(u2, sphi, cphi);
    const double x = rr * cphi, y = rr * sphi, z = std::sqrt(1.0 - u1);
    V3 e{(t.x * x + bt.x * y) + n.x * z, (t.y * x + bt.y * y) + n.y * z, (t.z * x + bt.z * y) + n.z * z};
    const double len = std::sqrt(e.x * e.x + e.y * e.y + e.z * e.z);
    if (len > 0.0) e = {e.x / len, e.y / len, e.z / len};
    return e;
}

// Head-light occlusion ray of a bounce vertex p (build-defined):
// the segment from the light (at the camera C, main.cpp:356-377) to p — ray
// o = C, d = e / |e| with e = p - C (Vector3::normalize's division,
// vector3.hpp:91-95), length len = |e|.  Occluded iff some triangle of the
// scene passes the reference's Moller-Trumbore test (triangle.hpp:40-62,
// EPS 1e-8) with t < len * (1 - 2^-12) — any triangle, whatever the tree: the
// test is tree-independent (no ancestor-box semantics), and the 2^-12 margin
// keeps p's own triangle (t = len up to rounding) and its neighbours through p
// out.  The traversal only prunes: boxes widened by wpad (far above any fp64
// rounding of a passing test), interval unclipped.  len = 0: lit.
constexpr double kShadowScale = 1.0 - 0x1p-12;
inline bool box_hit_wide(const V3& mn, const V3& mx, const Ray& r, double w) {
    return box_hit(V3{mn.x - w, mn.y - w, mn.z - w}, V3{mx.x + w, mx.y + w, mx.z + w}, r);
}
bool occluded(const BVH& b, const V3& C, const V3& p, double wpad, std::vector<int>& st) {
    const V3 e = sub(p, C);
    const double len = length(e);
    if (!(len > 0.0)) return false;
    const Ray r = make_ray(C, V3{e.x / len, e.y / len, e.z / len});
    const double tmax = len * kShadowScale;
    st.clear();
    st.push_back(0);
    while (!st.empty()) {
        const Node& n = b.nodes[st.back()];
        st.pop_back();
        if (!box_hit_wide(n.mn, n.mx, r, wpad)) continue;
        for (int i = n.begin; n.kids.empty() && i < n.end; ++i) {
            double t;
            if (tri_hit(b.tris[b.order[i]], r, t) && t < tmax) return true;
        }
        for (int c : n.kids) st.push_back(c);
    }
    return false;
}
}  // namespace
extern "C" {

// One pose: spp paths per pixel of 1 + bounces segments; rgb per pixel,
// primary-segment id / pos / dist per sample at ((j-row0)*W + i)*spp + s.
// shadow != 0: a bounce vertex (k >= 1) adds its colour only if the light
// sees it (occluded() above); the primary vertex is the camera ray's own
// closest hit, seen from the light at the camera by definition, and casts none.
// shadow_counts (may be NULL): [occlusion rays cast, of which occluded].
// Returns the number of samples whose primary ray hit, or -1.
long long orc_render_paths(const orc_bvh* h, const double cam_pos[3], const double cam_dir[3], int W, int H,
                           int row0, int nrows, int frame, int spp, int bounces, int shadow, int threads,
                           int32_t* hit_id, double* hit_pos, double* hit_dist, uint8_t* rgb,
                           long long* shadow_counts) {
    if (W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H || spp < 1 || bounces < 0) {
        g_err = "bad path geometry";
        return -1;
    }
    // occlusion box margin: 2^-30 of the scene's coordinate range
    const Node& root = h->b.nodes[0];
    const double cmax = std::max({std::fabs(root.mn.x), std::fabs(root.mn.y), std::fabs(root.mn.z),
                                  std::fabs(root.mx.x), std::fabs(root.mx.y), std::fabs(root.mx.z),
                                  std::fabs(cam_pos[0]), std::fabs(cam_pos[1]), std::fabs(cam_pos[2])});
    const double wpad = std::ldexp(cmax + 1.0, -30);
    long long s_cast = 0, s_occ = 0;
    const double fov = 90.0 * (std::numbers::pi / 180.0);
    const double th = std::tan(fov * 0.5);
    const double aspect = static_cast<double>(W) / H;
    const double iw = 1.0 / W, ih = 1.0 / H;
    const V3 cp{cam_pos[0], cam_pos[1], cam_pos[2]};
    const V3 cd{cam_dir[0], cam_dir[1], cam_dir[2]};
    V3 right, up;
    basis(cd, right, up);
    long long hits = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : hits, s_cast, s_occ)
#endif
    for (int i = 0; i < W; ++i) {
        std::vector<int> st;
        st.reserve(64);
        TravStats ts;
        for (int j = row0; j < row0 + nrows; ++j) {
            const size_t o = (size_t)(j - row0) * W + i;
            double acc[3] = {0.0, 0.0, 0.0};
            for (int s = 0; s < spp; ++s) {
                const uint32_t seed = path_seed((uint32_t)frame, (uint32_t)j * (uint32_t)W + (uint32_t)i, (uint32_t)s);
                const double ox = path_u(seed, 0), oy = path_u(seed, 1);
                const double px = (2.0 * (i + ox) * iw - 1.0) * th * aspect;
                const double py = (1.0 - 2.0 * (j + oy) * ih) * th;
                V3 d = add(add(cd, mul(up, py)), mul(right, px));
                d = mul(d, 1.0 / length(d));
                Ray r = make_ray(cp, d);
                double L[3] = {0.0, 0.0, 0.0};
                double w = 1.0;
                for (int b = 0; b <= bounces; ++b) {
                    V3 pos{0, 0, 0};
                    double dist;
                    const int id = traverse(h->b, r, pos, dist, st, ts);
                    if (b == 0) {
                        const size_t so = o * spp + s;
                        if (hit_id) hit_id[so] = id;
                        if (hit_pos) { hit_pos[so * 3] = pos.x; hit_pos[so * 3 + 1] = pos.y; hit_pos[so * 3 + 2] = pos.z; }
                        if (hit_dist) hit_dist[so] = id >= 0 ? dist : -1.0;
                        if (id >= 0) hits++;
                    }
                    if (id < 0) break;
                    const V3 nrm = h->b.tris[id].normal;
                    bool lit = true;
                    if (shadow && b > 0) {
                        s_cast++;
                        lit = !occluded(h->b, cp, pos, wpad, st);
                        s_occ += !lit;
                    }
                    if (lit) {
                        double c[3];
                        shade(true, pos, nrm, cp, c);
                        L[0] = L[0] + w * c[0];
                        L[1] = L[1] + w * c[1];
                        L[2] = L[2] + w * c[2];
                    }
                    w = w * 0.5;
                    if (b == bounces) break;
                    V3 N = nrm;  // the unit normal shade() uses (normalised once more)
                    const double nl = length(N);
                    if (nl > 0.0) N = mul(N, 1.0 / nl);
                    const V3 nd = bounce_dir(N, r.d, path_u(seed, 2u + 2u * (uint32_t)b), path_u(seed, 3u + 2u * (uint32_t)b));
                    r = make_ray(pos, nd);
                }
                acc[0] = acc[0] + L[0];
                acc[1] = acc[1] + L[1];
                acc[2] = acc[2] + L[2];
            }
            if (rgb)
                for (int k = 0; k < 3; k++) rgb[o * 3 + k] = to_byte(spp == 1 ? acc[k] : acc[k] / (double)spp);
        }
    }
    if (shadow_counts) {
        shadow_counts[0] = s_cast;
        shadow_counts[1] = s_occ;
    }
    return hits;
}

int orc_max_threads() {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

}  // extern "C"
