// Scene ingestion with the reference's loader semantics.
//
// The reference loads scenes through the vendored Bly7/OBJ-Loader
// (lib/OBJ_Loader.h) wrapped by ObjectLoader::loadFromFile
// (src/utils/object_loader.hpp:14-70).  The triangle ORDER it produces is the
// hit-ID contract and its VALUES are float-parsed coordinates widened to
// double and multiplied by the scale, so this loader reproduces:
//   * line classification by first token (OBJ_Loader.h:486-667), including
//     mesh breaks on o/g/usemtl which regroup the index stream per mesh;
//   * the library's splitter, which keeps empty fields (OBJ_Loader.h:321-357);
//   * std::stof / std::stoi parsing and 1-based / negative face indices
//     (OBJ_Loader.h:398-406, 545-547);
//   * polygon triangulation by ear clipping that emits indices by position
//     equality in ascending vertex order (OBJ_Loader.h:838-1003) — e.g. a
//     quad (0,1,2,3) becomes (0,1,3),(1,2,3).
// The file is read in one go and scanned without per-line allocation.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string_view>

#include "rt_internal.h"

namespace rt {
namespace {

struct P3 {
    float x, y, z;
    bool operator==(const P3& o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(const P3& o) const { return !(*this == o); }
    P3 operator-(const P3& o) const { return {x - o.x, y - o.y, z - o.z}; }
};
inline P3 pcross(const P3& a, const P3& b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float pdot(const P3& a, const P3& b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
inline float pmag(const P3& a) { return sqrtf(powf(a.x, 2) + powf(a.y, 2) + powf(a.z, 2)); }

// OBJ_Loader.h:273-318 (float arithmetic as the library does it)
bool same_side(const P3& p1, const P3& p2, const P3& a, const P3& b) {
    return pdot(pcross(b - a, p1 - a), pcross(b - a, p2 - a)) >= 0;
}
bool inside_tri(const P3& p, const P3& a, const P3& b, const P3& c) {
    if (!(same_side(p, a, b, c) && same_side(p, b, a, c) && same_side(p, c, a, b))) return false;
    P3 n = pcross(b - a, c - a);
    float m = pmag(n);
    P3 u{n.x / m, n.y / m, n.z / m};
    float d = pdot(p, u);
    P3 pr{u.x * d, u.y * d, u.z * d};
    return pmag(pr) == 0;
}

// Ear clipping of one face (OBJ_Loader.h:838-1003); indices are positions in
// `v` found by equality scans.
void triangulate(const std::vector<P3>& v, std::vector<uint32_t>& out) {
    const size_t n = v.size();
    if (n < 3) return;
    if (n == 3) { out.insert(out.end(), {0u, 1u, 2u}); return; }
    auto scan = [&](const P3& a, const P3& b, const P3& c, size_t limit) {
        for (size_t j = 0; j < limit; j++) {
            if (v[j] == a) out.push_back((uint32_t)j);
            if (v[j] == b) out.push_back((uint32_t)j);
            if (v[j] == c) out.push_back((uint32_t)j);
        }
    };
    std::vector<P3> ring = v;
    const size_t emitted0 = out.size();
    for (;;) {
        for (long i = 0; i < (long)ring.size(); i++) {
            const size_t m = ring.size();
            const P3 prev = ring[i == 0 ? m - 1 : (size_t)i - 1];
            const P3 cur = ring[(size_t)i];
            const P3 next = ring[(size_t)i == m - 1 ? 0 : (size_t)i + 1];
            if (m == 3) {  // the library scans only the first ring.size() vertices here
                scan(cur, prev, next, m);
                ring.clear();
                break;
            }
            if (m == 4) {
                scan(cur, prev, next, n);
                P3 rest{0, 0, 0};
                for (const P3& q : ring)
                    if (q != cur && q != prev && q != next) { rest = q; break; }
                for (size_t j = 0; j < n; j++) {
                    if (v[j] == prev) out.push_back((uint32_t)j);
                    if (v[j] == next) out.push_back((uint32_t)j);
                    if (v[j] == rest) out.push_back((uint32_t)j);
                }
                ring.clear();
                break;
            }
            bool blocked = false;
            for (size_t j = 0; j < n && !blocked; j++)
                blocked = inside_tri(v[j], prev, cur, next) && v[j] != prev && v[j] != cur && v[j] != next;
            if (blocked) continue;
            scan(cur, prev, next, n);
            for (size_t j = 0; j < ring.size(); j++)
                if (ring[j] == cur) { ring.erase(ring.begin() + (long)j); break; }
            i = -1;
        }
        if (out.size() == emitted0) break;
        if (ring.empty()) break;
    }
}

// The library's splitter on single-character tokens: every separator ends a
// field, so runs of separators yield empty fields; a separator at the very end
// of a non-empty field does not add one (OBJ_Loader.h:321-357).
template <class F>
void split_fields(std::string_view s, char sep, F&& emit) {
    size_t start = 0;
    bool pending = false;
    for (size_t i = 0; i < s.size(); i++) {
        if (s[i] == sep) {
            emit(s.substr(start, i - start));
            start = i + 1;
            pending = false;
        } else {
            pending = true;
        }
    }
    if (pending) emit(s.substr(start));
}

inline bool is_ws(char c) { return c == ' ' || c == '\t'; }

// algorithm::firstToken / algorithm::tail (OBJ_Loader.h:360-394)
std::string_view first_token(std::string_view l) {
    size_t a = 0;
    while (a < l.size() && is_ws(l[a])) a++;
    size_t e = a;
    while (e < l.size() && !is_ws(l[e])) e++;
    return l.substr(a, e - a);
}
std::string_view tail(std::string_view l) {
    size_t a = 0;
    while (a < l.size() && is_ws(l[a])) a++;
    while (a < l.size() && !is_ws(l[a])) a++;
    while (a < l.size() && is_ws(l[a])) a++;
    size_t e = l.size();
    while (e > a && is_ws(l[e - 1])) e--;
    return l.substr(a, e - a);
}

float to_float(std::string_view f) {  // std::stof
    char buf[128];
    if (f.size() >= sizeof buf) throw Error{RT_ERR_RUNTIME, "stof: field too long"};
    std::memcpy(buf, f.data(), f.size());
    buf[f.size()] = 0;
    errno = 0;
    char* end = nullptr;
    float v = std::strtof(buf, &end);
    if (end == buf) throw Error{RT_ERR_INVALID_ARGUMENT, "stof"};
    if (errno == ERANGE) throw Error{RT_ERR_OUT_OF_RANGE, "stof"};
    return v;
}
int to_int(std::string_view f) {  // std::stoi
    char buf[64];
    if (f.size() >= sizeof buf) throw Error{RT_ERR_RUNTIME, "stoi: field too long"};
    std::memcpy(buf, f.data(), f.size());
    buf[f.size()] = 0;
    errno = 0;
    char* end = nullptr;
    long v = std::strtol(buf, &end, 10);
    if (end == buf) throw Error{RT_ERR_INVALID_ARGUMENT, "stoi"};
    if (errno == ERANGE || v > 2147483647L || v < -2147483648L) throw Error{RT_ERR_OUT_OF_RANGE, "stoi"};
    return (int)v;
}

}  // namespace

std::vector<double> load_obj(const std::string& path, double scale) {
    const std::string fail = "Failed to load OBJ file: " + path;  // object_loader.hpp:17
    if (path.size() < 4 || path.compare(path.size() - 4, 4, ".obj") != 0) throw Error{RT_ERR_RUNTIME, fail};
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) throw Error{RT_ERR_RUNTIME, fail};
    std::string data;
    {
        std::fseek(fp, 0, SEEK_END);
        long sz = std::ftell(fp);
        std::fseek(fp, 0, SEEK_SET);
        data.resize(sz > 0 ? (size_t)sz : 0);
        if (sz > 0 && std::fread(data.data(), 1, (size_t)sz, fp) != (size_t)sz) { std::fclose(fp); throw Error{RT_ERR_RUNTIME, fail}; }
        std::fclose(fp);
    }
    std::vector<P3> pos;
    std::vector<P3> mesh_v;         // current mesh's face vertices
    std::vector<uint32_t> mesh_i;   // current mesh's indices
    std::vector<double> tris;
    bool listening = false;
    uint64_t face_vertices = 0;
    size_t meshes = 0;
    std::vector<P3> face;
    std::vector<uint32_t> local;

    auto flush_mesh = [&]() {  // ObjectLoader's per-mesh triples (object_loader.hpp:53-67)
        meshes++;
        for (size_t i = 0; i + 2 < mesh_i.size(); i += 3) {
            uint32_t a = mesh_i[i], b = mesh_i[i + 1], c = mesh_i[i + 2];
            if (a >= mesh_v.size() || b >= mesh_v.size() || c >= mesh_v.size()) continue;
            for (uint32_t k : {a, b, c}) {
                tris.push_back((double)mesh_v[k].x * scale);
                tris.push_back((double)mesh_v[k].y * scale);
                tris.push_back((double)mesh_v[k].z * scale);
            }
        }
        mesh_v.clear();
        mesh_i.clear();
    };

    size_t p = 0;
    const size_t N = data.size();
    while (p < N) {
        size_t e = p;
        while (e < N && data[e] != '\n') e++;
        std::string_view line(data.data() + p, e - p);
        p = e + 1;
        const std::string_view ft = first_token(line);
        if (ft == "o" || ft == "g" || (!line.empty() && line[0] == 'g')) {
            if (!listening) listening = true;
            else if (!mesh_i.empty() && !mesh_v.empty()) flush_mesh();
        }
        if (ft == "v") {
            float c[3];
            int k = 0;
            split_fields(tail(line), ' ', [&](std::string_view f) {
                if (k < 3) c[k] = to_float(f);
                k++;
            });
            if (k < 3) throw Error{RT_ERR_RUNTIME, fail};
            pos.push_back({c[0], c[1], c[2]});
        } else if (ft == "f") {
            face.clear();
            split_fields(tail(line), ' ', [&](std::string_view f) {
                int nf = 0;
                std::string_view f0;
                split_fields(f, '/', [&](std::string_view g) {
                    if (nf == 0) f0 = g;
                    nf++;
                });
                if (nf < 1 || nf > 3) return;  // the library leaves the vertex type undefined
                int idx = to_int(f0);
                idx = idx < 0 ? (int)pos.size() + idx : idx - 1;
                if (idx < 0 || idx >= (int)pos.size()) throw Error{RT_ERR_OUT_OF_RANGE, "face index out of range"};
                face.push_back(pos[(size_t)idx]);
            });
            const uint32_t base = (uint32_t)mesh_v.size();
            mesh_v.insert(mesh_v.end(), face.begin(), face.end());
            face_vertices += face.size();
            local.clear();
            triangulate(face, local);
            for (uint32_t k : local) mesh_i.push_back(base + k);
        } else if (ft == "usemtl") {
            if (!mesh_i.empty() && !mesh_v.empty()) flush_mesh();
        }
    }
    if (!mesh_i.empty() && !mesh_v.empty()) flush_mesh();
    if (meshes == 0 && face_vertices == 0) throw Error{RT_ERR_RUNTIME, fail};
    return tris;
}

}  // namespace rt
