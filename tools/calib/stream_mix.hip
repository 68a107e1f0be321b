// stream_mix.hip — the HBM ceiling for bt_parse_filter_main's C2 data movement.
//
// C2 reads 64 B and writes 96 B per packet (16M packets: 1 GiB in, 1.5 GiB out, the
// records tiled as six 1-KiB slabs per 64-packet tile). These kernels move exactly
// those bytes with no parsing, so the gap between them and the real kernel is the
// cost of the parse itself, and the gap between them and 8 TB/s is the memory
// system's. Timed with hipEvents, best and median of 15 launches.
//   copy      : 1 GiB -> 1 GiB, 16 B per lane, grid-stride (the guide's float4 copy)
//   read      : 1 GiB read only
//   write     : 1.5 GiB write only (nt stores)
//   mix       : the C2 shape: per wave tile, 4 x 1-KiB loads, 6 x 1-KiB stores,
//               persistent grid of G blocks x 4 waves; nt / default stores
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ in, size_t n16, unsigned* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ out, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const u32x4 x = {(uint32_t)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + i));
    }
}

template <bool NT, int SLABS = 6>
__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ in, uint4* __restrict__ rec, uint32_t ntiles) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u;
    for (uint32_t t = blockIdx.x * 4u + wid; t < ntiles; t += W) {
        const uint4* src = in + (size_t)t * 256;   // 4 KiB
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = src[j * 64 + lane];
        uint4* dst = rec + (size_t)t * 384;        // 6 KiB
#pragma unroll
        for (int k = 0; k < SLABS; ++k) {
            const uint4 a = v[k & 3];
            const u32x4 x = {a.x ^ (uint32_t)k, a.y, a.z, a.w};
            if (NT) __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(dst + k * 64 + lane));
            else dst[k * 64 + lane] = make_uint4(x.x, x.y, x.z, x.w);
        }
    }
}

template <class F>
void timeit(const char* name, double bytes, F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> ms;
    for (int i = 0; i < 15; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float x;
        CK(hipEventElapsedTime(&x, a, b));
        ms.push_back(x);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-28s best %.4f ms (%.2f TB/s)  median %.4f ms (%.2f TB/s)\n", name, ms[0], bytes / ms[0] / 1e9,
           ms[7], bytes / ms[7] / 1e9);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const size_t n = 1u << 24;                  // packets
    const size_t in_bytes = n * 64, rec_bytes = n * 96;
    uint4 *in, *rec;
    unsigned* sink;
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&rec, rec_bytes));
    CK(hipMalloc(&sink, 16));
    CK(hipMemset(in, 1, in_bytes));
    CK(hipMemset(rec, 0, rec_bytes));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s, %d CUs\n", p.name, cus);
    const size_t n16 = in_bytes / 16;
    timeit("copy 1GiB->1GiB", 2.0 * in_bytes, [&] { hipLaunchKernelGGL(k_copy, dim3(cus * 8), dim3(256), 0, 0, in, rec, n16); });
    timeit("read 1GiB", 1.0 * in_bytes, [&] { hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, in, n16, sink); });
    timeit("write 1.5GiB nt", 1.0 * rec_bytes, [&] { hipLaunchKernelGGL(k_write, dim3(cus * 8), dim3(256), 0, 0, rec, rec_bytes / 16); });
    const uint32_t ntiles = (uint32_t)(n / 64);
    for (int per_cu : {4, 6, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "mix nt  %2d blocks/CU", per_cu);
        timeit(nm, 160.0 * n, [&] { hipLaunchKernelGGL(k_mix<true>, dim3(cus * per_cu), dim3(256), 0, 0, in, rec, ntiles); });
        snprintf(nm, sizeof nm, "mix def %2d blocks/CU", per_cu);
        timeit(nm, 160.0 * n, [&] { hipLaunchKernelGGL(k_mix<false>, dim3(cus * per_cu), dim3(256), 0, 0, in, rec, ntiles); });
    }
    timeit("mix nt 4 slabs (64 B rec)", 128.0 * n, [&] { hipLaunchKernelGGL((k_mix<true, 4>), dim3(cus * 4), dim3(256), 0, 0, in, rec, ntiles); });
    timeit("mix nt 5 slabs (80 B rec)", 144.0 * n, [&] { hipLaunchKernelGGL((k_mix<true, 5>), dim3(cus * 4), dim3(256), 0, 0, in, rec, ntiles); });
    timeit("mix nt  1 tile/wave", 160.0 * n, [&] { hipLaunchKernelGGL(k_mix<true>, dim3(ntiles / 4), dim3(256), 0, 0, in, rec, ntiles); });
    return 0;
}
