// Memory-latency probe for the traversal design (diagnostic tool, not part
// of the library).  Pointer-chases through a buffer of 256-B "nodes" in a
// random cyclic order and reports clock ticks (s_memtime) per dependent hop:
//   scalar  s_load of the next index (wave-uniform address)
//   vector  global_load of the next index, every lane the same address
// once with a single wave on the chip and once with every CU busy (W waves
// per SIMD), for working sets that fit L2, MALL and neither.
// Build: hipcc -O3 --offload-arch=gfx950 tools/latency_probe.hip -o /tmp/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

typedef const __attribute__((address_space(4))) uint32_t* cu32;

__global__ void chase_scalar(const uint32_t* __restrict__ next, int hops, unsigned long long* out) {
    uint32_t i = (blockIdx.x * 977u + (threadIdx.x >> 6) * 131u) % 1024u;  // per-wave start
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int h = 0; h < hops; h++) i = ((cu32)next)[(size_t)i * 64];
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, (unsigned long long)(t1 - t0));
        atomicAdd(out + 1, (unsigned long long)i);  // keep the chain live
    }
}

__device__ __forceinline__ int vzero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

__global__ void chase_vector(const uint32_t* __restrict__ next, int hops, unsigned long long* out) {
    uint32_t i = (blockIdx.x * 977u + (threadIdx.x >> 6) * 131u) % 1024u;
    const int z = vzero();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int h = 0; h < hops; h++) i = __builtin_amdgcn_readfirstlane(next[(size_t)i * 64 + z]);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, (unsigned long long)(t1 - t0));
        atomicAdd(out + 1, (unsigned long long)i);
    }
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipSetDevice(dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    unsigned long long* d_out;
    CHECK(hipMalloc(&d_out, 16));
    const size_t sizes_mb[] = {1, 4, 32, 1024};
    const int hops = 2000;
    std::printf("CUs %d; ticks per dependent hop (s_memtime)\n", cus);
    for (size_t mb : sizes_mb) {
        const size_t nodes = mb * 1024 * 1024 / 256;
        std::vector<uint32_t> perm(nodes);
        std::iota(perm.begin(), perm.end(), 0u);
        std::mt19937 rng(1234);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<uint32_t> h(nodes * 64, 0);
        for (size_t k = 0; k < nodes; k++) h[(size_t)perm[k] * 64] = perm[(k + 1) % nodes];
        uint32_t* d;
        CHECK(hipMalloc(&d, h.size() * 4));
        CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        for (int kind = 0; kind < 2; kind++) {
            for (int load = 0; load < 3; load++) {
                const int blocks = load == 0 ? 1 : cus * (load == 1 ? 1 : 5);  // 1 wave / 4 / 20 waves per CU
                const int threads = load == 0 ? 64 : 256;
                const int waves = blocks * threads / 64;
                CHECK(hipMemset(d_out, 0, 16));
                if (kind == 0) hipLaunchKernelGGL(chase_scalar, dim3(blocks), dim3(threads), 0, 0, d, hops, d_out);
                else hipLaunchKernelGGL(chase_vector, dim3(blocks), dim3(threads), 0, 0, d, hops, d_out);
                CHECK(hipDeviceSynchronize());
                unsigned long long r[2];
                CHECK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
                std::printf("%5zu MB %-6s waves %6d : %8.1f ticks/hop\n", mb, kind == 0 ? "scalar" : "vector", waves,
                            (double)r[0] / waves / hops);
            }
        }
        CHECK(hipFree(d));
    }
    return 0;
}
