// Scene ingestion cache: the loader's output for an
// OBJ file, stored as a binary file keyed by the OBJ bytes' digest and the
// scale, so repeated runs skip the text parse.  The cached payload is the
// loader's triangle array verbatim (loader order = the hit-ID contract,
// object_loader.hpp:14-70), so a cache hit returns exactly what rt_load_obj
// would.  Any mismatch (version, digest, scale, size, payload checksum) falls
// back to parsing and rewrites the entry.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

constexpr uint32_t kMagic = 0x43535452u;  // "RTSC"
constexpr uint32_t kVersion = 1;

struct Header {
    uint32_t magic, version;
    uint64_t digest;  // FNV-1a 64 of the OBJ bytes
    double scale;
    uint64_t n;       // triangles
    uint64_t sum;     // FNV-1a 64 of the payload
};

uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; i++) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

bool read_file(const std::string& path, std::string& out) {
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) return false;
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    out.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = sz >= 0 && (sz == 0 || std::fread(out.data(), 1, (size_t)sz, fp) == (size_t)sz);
    std::fclose(fp);
    return ok;
}

}  // namespace

std::vector<double> load_obj_cached(const std::string& path, double scale, const std::string& cache_dir,
                                    bool* hit) {
    *hit = false;
    std::string obj;
    if (path.size() < 4 || path.compare(path.size() - 4, 4, ".obj") != 0 || !read_file(path, obj))
        throw Error{RT_ERR_RUNTIME, "Failed to load OBJ file: " + path};  // object_loader.hpp:17
    const uint64_t digest = fnv1a(obj.data(), obj.size());
    char name[64];
    std::snprintf(name, sizeof name, "/%016llx.rtsc", (unsigned long long)digest);
    const std::string cpath = cache_dir + name;
    {
        std::string c;
        if (read_file(cpath, c) && c.size() >= sizeof(Header)) {
            Header h;
            std::memcpy(&h, c.data(), sizeof h);
            const size_t bytes = c.size() - sizeof h;
            if (h.magic == kMagic && h.version == kVersion && h.digest == digest &&
                std::memcmp(&h.scale, &scale, sizeof scale) == 0 && bytes == h.n * 9 * sizeof(double) &&
                fnv1a(c.data() + sizeof h, bytes) == h.sum) {
                std::vector<double> v(h.n * 9);
                if (bytes) std::memcpy(v.data(), c.data() + sizeof h, bytes);
                *hit = true;
                return v;
            }
        }
    }
    std::vector<double> v = load_obj(path, scale);
    Header h{kMagic, kVersion, digest, scale, v.size() / 9, fnv1a(v.data(), v.size() * sizeof(double))};
    // write to a temporary name, then rename: a reader never sees a partial entry
    const std::string tmp = cpath + ".tmp";
    if (FILE* fp = std::fopen(tmp.c_str(), "wb")) {
        bool ok = std::fwrite(&h, sizeof h, 1, fp) == 1 &&
                  (v.empty() || std::fwrite(v.data(), sizeof(double), v.size(), fp) == v.size());
        ok = std::fclose(fp) == 0 && ok;
        if (!ok || std::rename(tmp.c_str(), cpath.c_str()) != 0) std::remove(tmp.c_str());
    }
    return v;
}

}  // namespace rt
