// gather_mix.hip — the HBM ceiling for C3's data movement (IMIX, descriptor mode).
//
// C3 (16M packets, IMIX 64/512/1500 B at 7:4:1, frames packed at 64-B-aligned offsets)
// moves per packet: an 8-B descriptor, the first 64 B of the frame (one 128-B line at
// most), a 64-B packed record (4 slabs, tiled), a decision byte and 1/8 verdict byte.
// These kernels move exactly those bytes with no parsing, on the main kernel's grid
// shape (persistent, 64-packet tiles per wave, 4 lanes x 16 B per packet window), so
// the gap to bt_parse_filter_main is the cost of the parse and filter themselves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT_LOAD>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ base, const uint64_t* __restrict__ desc,
                                                uint4* __restrict__ rec, uint8_t* __restrict__ dec,
                                                uint64_t* __restrict__ ver, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u, ntiles = (n + 63) / 64;
    for (uint32_t t = blockIdx.x * 4u + wid; t < ntiles; t += W) {
        const uint32_t my = t * 64 + lane;
        const uint64_t d = my < n ? desc[my] : 0;
        const uint64_t off = d & 0xFFFFFFFFFFFFull;
        uint4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {   // packet j*16 + lane/4, chunk lane%4
            const uint32_t q = j * 16 + (lane >> 2);
            const uint64_t qo = ((uint64_t)(uint32_t)__shfl((int)(off >> 32), (int)q) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)off, (int)q);
            const uint8_t* p = base + (qo & ~15ull) + 16 * (lane & 3);
            if (NT_LOAD) {
                const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
                v[j] = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                v[j] = *reinterpret_cast<const uint4*>(p);
            }
        }
        uint32_t acc = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w;
        uint4* tile = rec + (size_t)t * 384;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 x = {acc ^ (uint32_t)k, v[k].y, v[k].z, v[k].w};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(tile + k * 64 + lane));
        }
        const uint64_t pass = __ballot(acc & 1u);
        if (my < n) dec[my] = (uint8_t)acc;
        if (lane == 0) ver[t] = pass;
    }
}

int main() {
    const uint32_t n = 1u << 24;
    // C3's layout: lengths 64/512/1500 at 7:4:1 (hashed), frames at 64-B-aligned offsets
    std::vector<uint64_t> desc(n);
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t h = (i * 2654435761u) >> 8;
        const uint32_t r = h % 12;
        const uint32_t len = r < 7 ? 64 : r < 11 ? 512 : 1500;
        desc[i] = off | ((uint64_t)len << 48);
        off += (len + 63) & ~63u;
    }
    uint8_t *base, *dec;
    uint64_t *d_desc, *ver;
    uint4* rec;
    CK(hipMalloc(&base, off + 256));
    CK(hipMalloc(&d_desc, (size_t)n * 8));
    CK(hipMalloc(&rec, (size_t)(n / 64) * 6144));
    CK(hipMalloc(&dec, n));
    CK(hipMalloc(&ver, (size_t)(n / 64) * 8));
    CK(hipMemset(base, 7, off + 256));
    CK(hipMemcpy(d_desc, desc.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double bytes = (double)n * (8 + 64 + 64 + 1 + 0.125);
    printf("C3 layout: %u packets, %.2f GB of frames; per-packet bytes moved %.3f\n", n, off / 1e9, bytes / n);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int nt = 0; nt < 2; ++nt) {
        for (int per_cu : {2, 3, 4, 8}) {
            auto launch = [&] {
                if (nt) hipLaunchKernelGGL(k_gather<true>, dim3(cus * per_cu), dim3(256), 0, 0, base, d_desc, rec, dec, ver, n);
                else hipLaunchKernelGGL(k_gather<false>, dim3(cus * per_cu), dim3(256), 0, 0, base, d_desc, rec, dec, ver, n);
            };
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
            printf("gather %s loads, %d blocks/CU: best %.4f ms  median %.4f ms  (%.2f TB/s of algorithmic bytes)\n",
                   nt ? "nt " : "def", per_cu, ms[0], ms[7], bytes / ms[7] / 1e9);
        }
    }
    return 0;
}
