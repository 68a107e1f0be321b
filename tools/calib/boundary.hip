// boundary.hip — what a kernel boundary costs between back-to-back launches on one stream.
//
// The main parse+filter kernel shows a 5-10 us gap before and after it in rocprofv3
// traces, where the guide measures ~1.7-1.9 us between streaming
// kernels. This separates the candidate causes: the kernel-argument size (the main
// kernel takes MainArgs + DevProgram by value, 2424 B), the bytes the predecessor wrote,
// and the static LDS of the persistent grid. Each case: N back-to-back launches between
// one event pair; gap per boundary = (span - N x the single-launch median) / N.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct BigArg {            // the size of MainArgs + DevProgram
    uint32_t w[600];
};

__global__ void k_tiny(uint32_t* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1;
}
__global__ void k_tiny_big(uint32_t* out, BigArg a) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += a.w[7];
}

// c2f-shaped mover (stream_pipe.hip's D0 with nt loads)
template <int LDS_DW>
__device__ __forceinline__ void mover(const uint4* __restrict__ in, uint4* __restrict__ rec, uint32_t ntiles, uint32_t salt) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u;
    __shared__ uint32_t lds[LDS_DW > 0 ? LDS_DW : 1];
    for (uint32_t t = blockIdx.x * 4u + wid; t < ntiles; t += W) {
        const uint4* src = in + (size_t)t * 256;
        uint4 cur[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + j * 64 + lane));
            cur[j] = make_uint4(x.x, x.y, x.z, x.w);
        }
        uint32_t a = cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w ^ salt;
        if (LDS_DW > 0) {
            lds[(wid * 64 + lane) % LDS_DW] = a;
            __builtin_amdgcn_wave_barrier();
            a ^= lds[(wid * 64 + (lane ^ 1)) % LDS_DW];
        }
        uint4* tile = rec + (size_t)t * 192;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 x = {a ^ cur[k].x, cur[k].y, cur[k].z, cur[k].w};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(tile + k * 64 + lane));
        }
    }
}
__global__ __launch_bounds__(256) void k_mover(const uint4* in, uint4* rec, uint32_t ntiles) { mover<0>(in, rec, ntiles, 0); }
__global__ __launch_bounds__(256) void k_mover_big(const uint4* in, uint4* rec, uint32_t ntiles, BigArg a) {
    mover<0>(in, rec, ntiles, a.w[5]);
}
__global__ __launch_bounds__(256) void k_mover_lds(const uint4* in, uint4* rec, uint32_t ntiles) { mover<4480>(in, rec, ntiles, 0); }

template <class F>
void boundary(const char* name, int N, F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> one;
    for (int i = 0; i < 9; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float x;
        CK(hipEventElapsedTime(&x, a, b));
        one.push_back(x);
    }
    std::sort(one.begin(), one.end());
    std::vector<float> span;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float x;
        CK(hipEventElapsedTime(&x, a, b));
        span.push_back(x);
    }
    std::sort(span.begin(), span.end());
    const double per = span[2] / N;
    printf("%-40s single %.2f us  back-to-back %.2f us/launch  -> %.2f us per boundary\n", name, one[4] * 1e3,
           per * 1e3, (per - one[4]) * 1e3);
    fflush(stdout);
}

int main() {
    const size_t n = 1u << 24;
    const uint32_t ntiles = (uint32_t)(n / 64);
    uint4 *in, *rec;
    uint32_t* cnt;
    CK(hipMalloc(&in, n * 64));
    CK(hipMalloc(&rec, n * 48));
    CK(hipMalloc(&cnt, 64));
    CK(hipMemset(in, 1, n * 64));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    BigArg big{};
    for (int i = 0; i < 600; ++i) big.w[i] = i;
    boundary("tiny, 8-B args", 50, [&] { hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, cnt); });
    boundary("tiny, 2.4-KB args", 50, [&] { hipLaunchKernelGGL(k_tiny_big, dim3(1), dim3(64), 0, 0, cnt, big); });
    boundary("tiny 1024 blocks, 8-B args", 50, [&] { hipLaunchKernelGGL(k_tiny, dim3(1024), dim3(256), 0, 0, cnt); });
    for (int per_cu : {2, 3}) {
        char nm[64];
        const dim3 g(cus * per_cu), blk(256);
        snprintf(nm, sizeof nm, "mover %d/CU, 8-B args", per_cu);
        boundary(nm, 20, [&] { hipLaunchKernelGGL(k_mover, g, blk, 0, 0, in, rec, ntiles); });
        snprintf(nm, sizeof nm, "mover %d/CU, 2.4-KB args", per_cu);
        boundary(nm, 20, [&] { hipLaunchKernelGGL(k_mover_big, g, blk, 0, 0, in, rec, ntiles, big); });
        snprintf(nm, sizeof nm, "mover %d/CU, 17.5-KB LDS", per_cu);
        boundary(nm, 20, [&] { hipLaunchKernelGGL(k_mover_lds, g, blk, 0, 0, in, rec, ntiles); });
    }
    // the runtime's timed launches: events recorded by the kernel's own dispatch
    // (hipExtLaunchKernelGGL), a fresh pair per launch as bt_time_device_ex does
    std::vector<hipEvent_t> ev(64);
    for (auto& evk : ev) CK(hipEventCreate(&evk));
    int k = 0;
    const dim3 g3(cus * 3), blk(256);
    boundary("mover 3/CU, ext launch with e0+e1", 20, [&] {
        hipExtLaunchKernelGGL(k_mover_big, g3, blk, 0, 0, ev[k % 64], ev[(k + 1) % 64], 0, in, rec, ntiles, big);
        k += 2;
    });
    boundary("mover 3/CU, ext launch with e1 only", 20, [&] {
        hipExtLaunchKernelGGL(k_mover_big, g3, blk, 0, 0, nullptr, ev[k % 64], 0, in, rec, ntiles, big);
        k += 1;
    });
    boundary("mover 3/CU, ext launch, no events", 20, [&] {
        hipExtLaunchKernelGGL(k_mover_big, g3, blk, 0, 0, nullptr, nullptr, 0, in, rec, ntiles, big);
    });
    boundary("mover 3/CU + hipEventRecord after", 20, [&] {
        hipLaunchKernelGGL(k_mover_big, g3, blk, 0, 0, in, rec, ntiles, big);
        CK(hipEventRecord(ev[k % 64], 0));
        k += 1;
    });
    // a small follow-on kernel on the same stream (the compaction's shape)
    boundary("mover 3/CU then tiny 1024 blocks", 20, [&] {
        hipLaunchKernelGGL(k_mover_big, g3, blk, 0, 0, in, rec, ntiles, big);
        hipLaunchKernelGGL(k_tiny, dim3(1024), dim3(256), 0, 0, cnt);
    });
    return 0;
}
