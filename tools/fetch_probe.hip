// Calibration of rocprofv3's FETCH_SIZE for the read types of the headline
// kernel (k_trace_packet): a known number of bytes is read from HBM by each
// access pattern, and tools/fetch_calib.py divides FETCH_SIZE (and
// TCC_EA0_RDREQ) of each dispatch by it.  MI355X_MICROARCH.md ("HBM")
// calibrates only wide 16-B/lane coalesced reads (FETCH_SIZE = half the
// bytes); the headline kernel reads wide-node child records with uniform
// (scalar) 32-B loads and fp64 triangle records with per-lane gathers.
//
//   k_uniform32  every wave reads its own contiguous slice as 32-B uniform
//                records, 8 per step (a 256-B wide node per step)
//   k_gather8    8 B per lane, lanes permuted inside each 512-B block
//   k_rec72      lane l reads the first 72 B of its own 128-B record (the
//                resolve's Moller-Trumbore part of a tri64 record); known
//                bytes = whole 128-B records (both 64-B halves are touched)
//   k_wide16     16 B per lane, coalesced (the guide's calibrated case)
//   k_store4/8/3 4-B, 8-B and 3 x 1-B stores per lane, coalesced (the hit
//                id, distance and colour outputs), 2 GiB each (store3: 3 * (2 GiB / 3))
//   k_flush      streams a separate buffer between probes so that no probe
//                starts with its data in the 256-MiB Infinity Cache
//
// Every probe reads 2 GiB once (8x the Infinity Cache).  Only loads are
// issued through the scalar path; results leave through vector stores.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_probe.hip -o tools/fetch_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

struct __attribute__((aligned(32))) Rec32 {
    uint32_t w[8];
};
typedef const __attribute__((address_space(4))) Rec32* crec_p;

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// one wave per 64-thread block; wave w reads records [w * per, (w + 1) * per)
__global__ void __launch_bounds__(64) k_uniform32(const Rec32* buf, uint32_t per, uint32_t* out) {
    const uint32_t w = uni(blockIdx.x);
    const crec_p p = (crec_p)(buf + (size_t)w * per);
    uint32_t acc = 0;
    for (uint32_t i = 0; i < per; i += 8) {
        Rec32 r[8];
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int k = 0; k < 8; k++) r[c].w[k] = p[i + c].w[k];
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int k = 0; k < 8; k++) acc = acc * 33u + r[c].w[k];
    }
    out[(size_t)w * 64 + threadIdx.x] = acc + threadIdx.x;
}

__global__ void __launch_bounds__(256) k_gather8(const uint2* buf, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x; b < n; b += stride) {
        const uint64_t base = b & ~63ull;  // (blockDim 256: b is a multiple of 64)
        const uint2 v = buf[base + ((threadIdx.x * 37u) & 63u) + (threadIdx.x & ~63u)];
        acc = acc * 33u + v.x + v.y;
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k_rec72(const double* buf, uint64_t nrec, uint32_t* out) {
    double acc = 0.0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrec; r += stride) {
        // lanes of a wave take records 37 apart modulo 64 (scattered, like
        // the candidates of neighbouring rays)
        const uint64_t rr = (r & ~63ull) | ((r * 37u) & 63u);
        const double* T = buf + rr * 16;
#pragma unroll
        for (int k = 0; k < 9; k++) acc += T[k];
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(acc != 0.0);
}

__global__ void __launch_bounds__(256) k_wide16(const uint4* buf, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4 v = buf[i];
        acc = acc * 33u + v.x + v.y + v.z + v.w;
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// stores: the headline kernel's outputs are a u32 hit id (4 B per lane), an
// fp64 distance (8 B per lane) and 3 colour bytes per lane, coalesced
__global__ void __launch_bounds__(256) k_store4(uint32_t* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = (uint32_t)i;
}
__global__ void __launch_bounds__(256) k_store8(double* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = (double)i;
}
__global__ void __launch_bounds__(256) k_store3(uint8_t* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        buf[3 * i] = (uint8_t)i;
        buf[3 * i + 1] = (uint8_t)(i >> 8);
        buf[3 * i + 2] = (uint8_t)(i >> 16);
    }
}

__global__ void __launch_bounds__(256) k_flush(const uint4* buf, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc ^= buf[i].x;
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint4* buf, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 7) | 1u, 3u, 5u);
}

int main() {
    const uint64_t bytes = 2ull << 30;       // 2 GiB per probe
    const uint64_t flush_bytes = 1ull << 30; // 1 GiB between probes
    void *buf = nullptr, *fl = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&out, 64ull << 20));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint4*)buf, bytes / 16);
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (uint4*)fl, flush_bytes / 16);
    auto flush = [&] { hipLaunchKernelGGL(k_flush, dim3(8192), dim3(256), 0, 0, (const uint4*)fl, flush_bytes / 16, out); };
    const int grid = 8192;
    // uniform 32-B records: 2 GiB over 65536 waves
    const uint32_t waves = 65536;
    const uint32_t per = (uint32_t)(bytes / 32 / waves);
    flush();
    hipLaunchKernelGGL(k_uniform32, dim3(waves), dim3(64), 0, 0, (const Rec32*)buf, per, out);
    flush();
    hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(256), 0, 0, (const uint2*)buf, bytes / 8, out);
    flush();
    hipLaunchKernelGGL(k_rec72, dim3(grid), dim3(256), 0, 0, (const double*)buf, bytes / 128, out);
    flush();
    hipLaunchKernelGGL(k_wide16, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
    flush();
    hipLaunchKernelGGL(k_store4, dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, bytes / 4);
    flush();
    hipLaunchKernelGGL(k_store8, dim3(grid), dim3(256), 0, 0, (double*)buf, bytes / 8);
    flush();
    hipLaunchKernelGGL(k_store3, dim3(grid), dim3(256), 0, 0, (uint8_t*)buf, bytes / 3);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::printf("{\"known_bytes_per_probe\": %llu, \"probes\": [\"k_uniform32\", \"k_gather8\", \"k_rec72\", \"k_wide16\", "
                "\"k_store4\", \"k_store8\", \"k_store3\"]}\n",
                (unsigned long long)bytes);
    CK(hipFree(buf));
    CK(hipFree(fl));
    CK(hipFree(out));
    return 0;
}
