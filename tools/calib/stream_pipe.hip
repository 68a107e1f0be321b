// stream_pipe.hip — c2f's data movement with and without counted memory waits.
//
// c2f (the headline: 16M x 64-B frames, fixed stride, parse + filter) moves per packet
// 64 B of frame, 48 B of packed record (3 tiled 1-KiB slabs per 64-packet tile), one
// decision byte, and per tile one verdict word and one pass count. These kernels move
// exactly those bytes with no parse, on the main kernel's persistent grid of 64-packet
// wave tiles. They differ only in how a wave overlaps the next tile's loads with this
// tile's stores:
//   D0  load tile t, use it, store: every iteration waits for its own stores (the
//       vmcnt counter retires loads and stores in issue order), the shape of
//       bt_parse_filter_main's fixed-stride loop today (its loop top is vmcnt(0));
//   D1  the loads of tile t+1 issued before tile t's stores, every store unconditional,
//       so the wait for tile t+1 is vmcnt(#stores of tile t): stores retire behind it;
//   D2  two tiles ahead.
// Timed with hipEvents, best and median of 15 launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld(const uint4* p, bool nt) {
    if (nt) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return *p;
}

__device__ __forceinline__ void st(uint4* p, uint4 v) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}

template <int AHEAD, bool NTL>
__global__ __launch_bounds__(256) void k_pipe(const uint4* __restrict__ in, uint4* __restrict__ rec,
                                              uint8_t* __restrict__ dec, uint64_t* __restrict__ ver,
                                              uint32_t* __restrict__ cnt, uint32_t ntiles) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u;
    uint32_t t = blockIdx.x * 4u + wid;
    constexpr int D = AHEAD > 0 ? AHEAD + 1 : 1;
    uint4 v[D][4];
    const auto rv = __builtin_amdgcn_make_buffer_rsrc(ver, (short)0, (int)(ntiles * 8u), 0x00020000);
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(cnt, (short)0, (int)(ntiles * 4u), 0x00020000);
    // prologue: tiles t .. t + AHEAD*W in flight (clamped to the last tile: the loads
    // of a wave past the end re-read its last tile and are never used)
    auto issue = [&](uint4 (&dst)[4], uint32_t tt) {
        const uint4* src = in + (size_t)min(tt, ntiles - 1) * 256;
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j] = ld(src + j * 64 + lane, NTL);
    };
    if (t >= ntiles) return;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue(v[k], t + (uint32_t)k * W);
    for (int it = 0; t < ntiles; t += W, ++it) {
        uint4 cur[4];
        if (AHEAD == 0) {
            issue(cur, t);
        } else {
            issue(v[D - 1], t + (uint32_t)(D - 1) * W);
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[j] = v[0][j];
#pragma unroll
            for (int k = 0; k < D - 1; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) v[k][j] = v[k + 1][j];
        }
        // "parse": a packet is 4 lanes' chunks; every lane folds its chunks into record dwords
        const uint32_t a = cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w ^ cur[0].y ^ cur[1].z ^ cur[2].w ^ cur[3].x;
        uint4* tile = rec + (size_t)t * 192;   // 3 KiB
#pragma unroll
        for (int k = 0; k < 3; ++k)
            st(tile + k * 64 + lane, make_uint4(a ^ cur[k].x, cur[k].y ^ cur[3].y, cur[k].z ^ cur[3].z, cur[k].w ^ cur[3].w));
        const bool pass = (a & 3u) == 1u;
        dec[(size_t)t * 64 + lane] = (uint8_t)a;
        const uint64_t b = __ballot(pass);
        // lane 0 stores the tile's verdict word and count; the other lanes' buffer stores
        // fall outside the range and are dropped, so every path issues the same stores
        const uint32_t o = lane == 0 ? 0u : 0x80000000u;
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 bw = {(uint32_t)b, (uint32_t)(b >> 32)};
        __builtin_amdgcn_raw_buffer_store_b64(bw, rv, (int)(t * 8u + o), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((uint32_t)__popcll(b), rc, (int)(t * 4u + o), 0, 0);
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
    printf("%-34s best %.4f ms (%.2f TB/s)  median %.4f ms (%.2f TB/s)\n", name, ms[0], bytes / ms[0] / 1e9,
           ms[7], bytes / ms[7] / 1e9);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const size_t n = 1u << 24;
    const uint32_t ntiles = (uint32_t)(n / 64);
    uint4 *in, *rec;
    uint8_t* dec;
    uint64_t* ver;
    uint32_t* cnt;
    CK(hipMalloc(&in, n * 64));
    CK(hipMalloc(&rec, n * 48));
    CK(hipMalloc(&dec, n));
    CK(hipMalloc(&ver, ntiles * 8ull));
    CK(hipMalloc(&cnt, ntiles * 4ull));
    CK(hipMemset(in, 1, n * 64));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s, %d CUs; bytes/packet 64 + 48 + 1 + 12/64\n", p.name, cus);
    const double bytes = (64.0 + 48.0 + 1.0 + 12.0 / 64.0) * n;
    for (int per_cu : {2, 3, 4, 6, 8}) {
        char nm[64];
        const dim3 g(cus * per_cu), blk(256);
        snprintf(nm, sizeof nm, "D0 %d blocks/CU", per_cu);
        timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_pipe<0, false>), g, blk, 0, 0, in, rec, dec, ver, cnt, ntiles); });
        snprintf(nm, sizeof nm, "D0 nt-load %d blocks/CU", per_cu);
        timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_pipe<0, true>), g, blk, 0, 0, in, rec, dec, ver, cnt, ntiles); });
        snprintf(nm, sizeof nm, "D1 %d blocks/CU", per_cu);
        timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_pipe<1, false>), g, blk, 0, 0, in, rec, dec, ver, cnt, ntiles); });
        snprintf(nm, sizeof nm, "D1 nt-load %d blocks/CU", per_cu);
        timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_pipe<1, true>), g, blk, 0, 0, in, rec, dec, ver, cnt, ntiles); });
        snprintf(nm, sizeof nm, "D2 %d blocks/CU", per_cu);
        timeit(nm, bytes, [&] { hipLaunchKernelGGL((k_pipe<2, false>), g, blk, 0, 0, in, rec, dec, ver, cnt, ntiles); });
    }
    return 0;
}
