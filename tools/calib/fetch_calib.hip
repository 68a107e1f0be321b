// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE / TCC_EA0_RDREQ on gfx950 for the
// access shapes bt_parse_filter_main uses (MI355X_MICROARCH.md §HBM: "calibrate on a
// known byte count in your own access pattern before trusting an absolute").
//
// Each pattern kernel reads a known set of bytes exactly once (1 GiB-class footprint,
// past the 256 MiB Infinity Cache) and writes one word per wave. Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and divide the counter by the printed byte counts.
//   P0 stream   : contiguous, 16 B per lane (1 KiB per wave instruction)
//   P1 seg64    : 64 B at the start of every 512-B record, 4 lanes per record (64-B aligned)
//   P2 seg64u   : 64 B at a 16-B-aligned offset inside every 512-B record (crosses lines)
//   P3 seg112u  : 112 B at a 16-B-aligned offset inside every 1024-B record
//   P4 desc8    : 8 B per lane, contiguous (descriptor reads)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void p_stream(const uint4* __restrict__ in, size_t n16, unsigned* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// rec_bytes-stride records; read `chunks` 16-B chunks starting at chunk `first(rec)`
template <int CHUNKS, int REC, bool UNALIGNED>
__global__ void p_seg(const uint8_t* __restrict__ in, size_t nrec, unsigned* out) {
    uint32_t acc = 0;
    const size_t lanes = (size_t)gridDim.x * blockDim.x;
    for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < nrec * CHUNKS; g += lanes) {
        const size_t r = g / CHUNKS;
        const uint32_t c = (uint32_t)(g % CHUNKS);
        uint32_t first = 0;
        if (UNALIGNED) first = (uint32_t)((r * 2654435761u) >> 7) % (REC / 16 - CHUNKS);   // 16-B aligned
        uint4 v = *reinterpret_cast<const uint4*>(in + r * REC + (first + c) * 16u);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void p_desc8(const uint64_t* __restrict__ in, size_t n, unsigned* out) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= in[i];
    if (acc == 0x12345678u) out[0] = (unsigned)acc;
}

int main() {
    const size_t bytes = (size_t)1 << 30;   // 1 GiB per pattern buffer
    uint8_t* buf;
    unsigned* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, bytes));
    CK(hipDeviceSynchronize());
    const int grid = 2048, block = 256;
    const size_t rec512 = bytes / 512, rec1024 = bytes / 1024;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(p_stream, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, bytes / 16, out);
        hipLaunchKernelGGL((p_seg<4, 512, false>), dim3(grid), dim3(block), 0, 0, buf, rec512, out);
        hipLaunchKernelGGL((p_seg<4, 512, true>), dim3(grid), dim3(block), 0, 0, buf, rec512, out);
        hipLaunchKernelGGL((p_seg<7, 1024, true>), dim3(grid), dim3(block), 0, 0, buf, rec1024, out);
        hipLaunchKernelGGL(p_desc8, dim3(grid), dim3(block), 0, 0, (const uint64_t*)buf, bytes / 8, out);
        CK(hipDeviceSynchronize());
    }
    printf("{\"p_stream\": %zu, \"p_seg4_512_aligned\": %zu, \"p_seg4_512_unaligned\": %zu, "
           "\"p_seg7_1024_unaligned\": %zu, \"p_desc8\": %zu}\n",
           bytes, rec512 * 64, rec512 * 64, rec1024 * 112, bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
