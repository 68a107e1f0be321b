// gather_c4.hip — the HBM ceiling for C4's data movement ("close C4's line-rate
// gap or document why it cannot close").
//
// C4 (16M frames: QinQ / 802.1Q / untagged, IPv6 or IPv4 with IHL 5..15, TCP with options,
// 2-mod-4 frame starts; bench.py's capture, libbt_synth cfg 4) moves per packet an 8-B
// descriptor, the 128-B lines of the frame bytes the walk reads ([off, off + need), need =
// the kernel's header_end with its 38-B floor, at most the frame), a packed record (R slabs
// of 16 B, tiled), a decision byte and a verdict bit. These kernels move exactly those lines
// and bytes with no parsing, on bt_parse_filter_pipe's shape (persistent grid at 2 blocks/CU,
// a 64-packet tile per wave, 4 lanes x 16 B per packet window, need carried in the
// descriptor's length field):
//   one-round  every 16-B chunk of [a0, off + need) in one round of loads (two groups of
//              four chunks, both issued before either is used): the bytes without the
//              dependency;
//   two-round  the kernel's wide form: chunks up to the end of the window's first 128-B line,
//              waited, then the rest, whose addresses depend on the first round's data (an
//              opaque zero from it, as the walk's EtherTypes / IHL decide round B).
// Each prints ms per launch (median of 15) and the algorithmic rate; bt_parse_filter_pipe's
// C4 main kernel is bench.py --config c4's roofline.kernel_ms. The same box runs both
// (tools/gpu_r04.sh c4-ceiling).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

extern "C" uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc);
extern "C" int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads);

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ uint4 g_zero[8];

template <int MODE>   // 0 one-round, 1 two-round (dependent)
__global__ __launch_bounds__(256) void k_c4(const uint8_t* __restrict__ base, const uint64_t* __restrict__ desc,
                                            uint4* __restrict__ rec, uint8_t* __restrict__ dec,
                                            uint64_t* __restrict__ ver, uint32_t n, uint32_t slabs, uint32_t opaque) {
    __shared__ uint4 img[4][64][9];
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u, ntiles = (n + 63) / 64;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero);
    for (uint32_t t = blockIdx.x * 4u + wid; t < ntiles; t += W) {
        const uint32_t my = t * 64 + lane;
        const uint64_t d = my < n ? desc[my] : 0;
        const uint64_t off = d & 0xFFFFFFFFFFFFull;
        const uint32_t need = (uint32_t)(d >> 48);
        uint4 v[8];
        uint32_t acc = 0;
        uint64_t qa[4];
        uint32_t qe[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t q = j * 16 + (lane >> 2);
            const uint64_t qo = ((uint64_t)(uint32_t)__shfl((int)(off >> 32), (int)q) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)off, (int)q);
            const uint32_t qn = (uint32_t)__shfl((int)need, (int)q);
            qa[j] = qo & ~15ull;
            const uint32_t e = (uint32_t)(qo & 15u) + qn;                     // bytes from a0 the walk reads
            const uint32_t line_end = 128u - (uint32_t)(qa[j] & 127u);        // end of a0's first line
            qe[j] = e;
            const uint32_t c = lane & 3u;
            const uint32_t lim_a = MODE == 1 ? min(qe[j], line_end) : qe[j];
            v[j] = *reinterpret_cast<const uint4*>(16u * c < lim_a ? base + qa[j] + 16u * c : zero);
            if (MODE != 1) v[4 + j] = *reinterpret_cast<const uint4*>(16u * (c + 4u) < lim_a ? base + qa[j] + 16u * (c + 4u) : zero);
        }
        if (MODE == 1) {   // round B: after round A's data is in (the walk reads it first)
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) img[wid][j * 16 + (lane >> 2)][lane & 3u] = v[j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t dep = img[wid][lane][0].x & opaque;   // 0, but not to the compiler
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t c = lane & 3u;
                const uint32_t line_end = 128u - (uint32_t)(qa[j] & 127u);
                const uint32_t lo = (min(qe[j], line_end) + 15u) / 16u;   // first chunk round A did not read
                const uint32_t c0 = lo + c, c1 = lo + c + 4u;
                v[4 + j] = *reinterpret_cast<const uint4*>(c0 < 8u && 16u * c0 < qe[j] ? base + qa[j] + 16u * c0 + dep : zero);
                const uint4 w = *reinterpret_cast<const uint4*>(c1 < 8u && 16u * c1 < qe[j] ? base + qa[j] + 16u * c1 + dep
                                                                                                : zero);
                acc ^= w.x;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].w;
        uint4* tile = rec + (size_t)t * 384;
        for (uint32_t k = 0; k < slabs; ++k) {
            const u32x4 x = {acc ^ k, acc, acc + k, acc};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(tile + k * 64 + lane));
        }
        const uint64_t pass = __ballot(acc & 1u);
        if (my < n) dec[my] = (uint8_t)acc;
        if (lane == 0) ver[t] = pass;
    }
}

// The kernel's header_end (bt_kernels.hip) with its 38-B floor, at most the frame.
static uint32_t need_of(const uint8_t* f, uint32_t len) {
    auto be16 = [&](uint32_t i) { return i + 1 < len ? ((uint32_t)f[i] << 8) | f[i + 1] : 0u; };
    auto vlan = [](uint32_t et) { return et == 0x8100u || et == 0x88A8u; };
    const uint32_t et0 = be16(12), et1 = be16(16), et2 = be16(20);
    const bool t0 = vlan(et0), t1 = t0 && vlan(et1);
    const uint32_t o3 = 14u + (t0 ? 4u : 0u) + (t1 ? 4u : 0u);
    const uint32_t et = t1 ? et2 : t0 ? et1 : et0;
    const uint32_t ib = o3 < len ? f[o3] : 0u;
    const uint32_t ihl = ib & 0x0Fu;
    const uint32_t v4end = o3 + 40u + (ihl > 5u ? 4u * ihl - 20u : 0u);
    uint32_t end = et == 0x0800u ? v4end : et == 0x86DDu ? o3 + 60u : o3;
    end = std::max(end, 38u);
    return std::min(end, len);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u << 24;
    const uint64_t seed = 0x5EED0004ull;   // beatrice_amd/synth.py SEEDS[C4], bench.py's capture
    std::vector<uint64_t> desc(n);
    const uint64_t bytes = bt_synth_layout(4, n, seed, desc.data());
    std::vector<uint8_t> data(bytes + 256);
    bt_synth_fill(4, n, seed, desc.data(), data.data(), 16);
    // need in the length field; the line floor of what the walk reads
    double lines = 0, need_sum = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = desc[i] & 0xFFFFFFFFFFFFull;
        const uint32_t len = (uint32_t)(desc[i] >> 48);
        const uint32_t need = need_of(data.data() + off, len);
        desc[i] = off | ((uint64_t)need << 48);
        need_sum += need;
        lines += need ? (double)((off + need - 1) / 128 - off / 128 + 1) : 0.0;
    }
    uint8_t *d_base, *dec;
    uint64_t *d_desc, *ver;
    uint4* rec;
    CK(hipMalloc(&d_base, bytes + 256));
    CK(hipMalloc(&d_desc, (size_t)n * 8));
    CK(hipMalloc(&rec, (size_t)((n + 63) / 64) * 6144));
    CK(hipMalloc(&dec, n));
    CK(hipMalloc(&ver, (size_t)((n + 63) / 64) * 8));
    CK(hipMemcpy(d_base, data.data(), bytes + 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_desc, desc.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const uint32_t slabs = 5;   // C4's packed records average 76 B (4.75 slabs); 5 slab stores per tile
    const double alg = (double)n * 212.0;   // C4's algorithmic bytes per packet
    const double moved = lines * 128.0 + (double)n * (8 + 16.0 * slabs + 1 + 0.125);
    printf("C4 layout: %u packets, %.2f GB of frames, need %.1f B/packet, %.3f lines/packet; line-floor traffic %.1f B/packet\n",
           n, bytes / 1e9, need_sum / n, lines / n, moved / n);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[2] = {"one-round", "two-round"};
    for (int mode = 0; mode < 2; ++mode) {
        for (int per_cu : {2, 3}) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(k_c4<0>, dim3(cus * per_cu), dim3(256), 0, 0, d_base, d_desc, rec, dec, ver, n, slabs, 0u);
                else hipLaunchKernelGGL(k_c4<1>, dim3(cus * per_cu), dim3(256), 0, 0, d_base, d_desc, rec, dec, ver, n, slabs, 0u);
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
            printf("%-10s %d blocks/CU: best %.4f ms  median %.4f ms  (%.2f TB/s of C4's algorithmic bytes, %.2f TB/s of its line floor)\n",
                   names[mode], per_cu, ms[0], ms[7], alg / ms[7] / 1e9, moved / ms[7] / 1e9);
        }
    }
    return 0;
}
