// bt_extract.hip — gfx950 field extraction for user-defined protocol tables.
//
// The reference's ProtocolParser is a generic, table-driven extractor: for one buffer and
// one ProtocolDefinition, parsePacketInternal (src/parser/ProtocolParser.cpp:238-284) gates
// on getTotalLength(), then extractField / extractValue<T> (:286-433) copy and decode each
// field at its fixed offset. bt_extract_tile does that for a whole batch: one packet per
// lane, one 64-packet tile per wavefront, persistent grid.
//   LOAD   the first `window` (<= 256) bytes of each packet, the span of the table, are
//          staged into a per-wave LDS image with coalesced 16-B loads, four lanes per
//          packet and 16 packets per wave instruction (the main kernel's round A);
//   DECODE each lane walks the table (kernel argument, scalar loads) over its own row:
//          the extractValue<T> bits of every numeric field go to a field-major u64 column,
//          so a wave's store for one field is 512 contiguous bytes;
//   IMAGE  the wave writes its tile's packets' [0, span) bytes as one contiguous region,
//          64 lanes per store, from which the host materialises rawHex and byte fields.
// Fields that end past the staged window (span > 256) read their bytes from memory
// directly. Both forms give identical results; tests check both (tests/test_gpu_extract.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "bt_device.h"

namespace bt {
namespace {

constexpr uint32_t kExRow = kExWindow / 4 + 4 + 1;   // dwords per packet row: window + misalignment + pad

__device__ __forceinline__ uint4 ld16_plain(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

// Byte b (< span) of the packet in row `row` (byte 0 at row byte s), or from memory when
// past the staged window.
__device__ __forceinline__ uint32_t byte_at(const uint8_t* rowb, uint32_t s, uint32_t b, uint32_t window,
                                            const uint8_t* frame) {
    return b < window ? (uint32_t)rowb[s + b] : (uint32_t)frame[b];
}

// extractValue<T> (src/parser/ProtocolParser.cpp:385-433) for one field of one packet.
__device__ __forceinline__ uint64_t decode_field(const ExField& f, const uint8_t* rowb, uint32_t s, uint32_t window,
                                                 const uint8_t* frame) {
    const uint32_t type = f.ctl & 0xFFu;
    const bool le = ((f.ctl >> 8) & 0xFFu) == BT_ENDIAN_LITTLE;
    const uint32_t o = f.offset, L = f.length;
    switch (type) {
    case BT_FT_FLOAT32:
    case BT_FT_FLOAT64: {   // the raw bits when the length matches the type, else T{}
        const uint32_t want = type == BT_FT_FLOAT32 ? 4u : 8u;
        if (L != want) return 0;
        uint64_t v = 0;
        for (uint32_t i = 0; i < want; ++i) {
            const uint64_t b = byte_at(rowb, s, o + (le ? i : want - 1u - i), window, frame);
            v |= b << (8u * i);
        }
        return v;
    }
    case BT_FT_BOOLEAN: return byte_at(rowb, s, o, window, frame) != 0u ? 1u : 0u;   // fieldData[0] != 0
    case BT_FT_BYTES: case BT_FT_STRING: case BT_FT_MAC: case BT_FT_IPV4: case BT_FT_IPV6: case BT_FT_CUSTOM:
        return 0;   // the bytes themselves (image)
    default: {
        // integer types and TIMESTAMP: byte i (from the field's low end) ORed in at
        // (8 i) mod the shift width, then cut to the type's width
        const bool wide = type == BT_FT_UINT64 || type == BT_FT_INT64 || type == BT_FT_TIMESTAMP;
        const uint32_t m = wide ? 63u : 31u;
        const uint32_t w = (type == BT_FT_UINT8 || type == BT_FT_INT8) ? 8u
                         : (type == BT_FT_UINT16 || type == BT_FT_INT16) ? 16u
                         : (type == BT_FT_UINT32 || type == BT_FT_INT32) ? 32u : 64u;
        uint64_t v = 0;
        for (uint32_t i = 0; i < L; ++i) {
            const uint32_t sh = (8u * i) & m;
            if (sh >= w) continue;   // lands past the type's width: cut anyway
            const uint64_t b = byte_at(rowb, s, o + (le ? i : L - 1u - i), window, frame);
            v |= b << sh;
        }
        return w == 64u ? v : (v & ((1ull << w) - 1ull));
    }
    }
}

__global__ __launch_bounds__(kBlock) void bt_extract_tile(ExArgs a, ExTable tab) {
    __shared__ uint32_t lds_all[kWavesPerBlock * (kWave * kExRow + 3 * kWave) + 32];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* img = lds_all + wid * (kWave * kExRow + 3 * kWave);
    uint32_t* meta = img + kWave * kExRow;          // per packet: s | ok << 8
    uint64_t* offs = reinterpret_cast<uint64_t*>(meta + kWave);   // per packet: frame offset
    const uint8_t* rowb = reinterpret_cast<const uint8_t*>(img + lane * kExRow);

    const uint32_t window = tab.window, span = tab.span;
    const uint32_t groups = (window + 15u + 63u) / 64u;   // 4 chunks of 16 B per group
    const uint32_t total_waves = gridDim.x * kWavesPerBlock;
    for (uint32_t t = blockIdx.x * kWavesPerBlock + wid; t < a.ntiles; t += total_waves) {
        const uint32_t p0 = t * 64u;
        const uint32_t my = p0 + lane;
        const bool live = my < a.n;
        uint64_t off = 0;
        uint32_t len = 0;
        if (live) {
            if (!a.desc) {
                off = (uint64_t)my * a.stride;
                len = a.stride;
            } else if (a.desc_words == 1) {
                const uint64_t d = a.desc[my];
                off = d & 0xFFFFFFFFFFFFull;
                len = (uint32_t)(d >> 48);
            } else {
                const uint4 d = *reinterpret_cast<const uint4*>(a.desc + 2ull * my);
                off = ((uint64_t)d.y << 32) | d.x;
                len = d.z > 0xFFFFu ? 0xFFFFu : d.z;
            }
        }
        const bool ok = live && len >= span;
        const uint32_t s = (uint32_t)off & 15u;
        // ---- LOAD: [a0, off + min(len, window)) of every packet, 4 lanes per packet ----
        const uint32_t wl = len < window ? len : window;
        const uint32_t off_lo = (uint32_t)off, off_hi = (uint32_t)(off >> 32);
        for (uint32_t g = 0; g < groups; ++g) {
            uint4 v[4];
            uint32_t dst[4];
            bool keep[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t q = j * 16u + (lane >> 2);
                const uint64_t qo = ((uint64_t)(uint32_t)__shfl((int)off_hi, (int)q) << 32) |
                                    (uint32_t)__shfl((int)off_lo, (int)q);
                const uint32_t qe = (uint32_t)__shfl((int)((uint32_t)off & 15u) + (int)wl, (int)q);   // s + wl of q
                const uint32_t c = 4u * g + (lane & 3u);
                const uint64_t addr = (qo & ~15ull) + 16ull * c;
                const bool want = 16u * c < qe && addr + 16ull <= a.bytes;
                v[j] = want ? ld16_plain(a.base + addr) : make_uint4(0, 0, 0, 0);
                dst[j] = q * kExRow + 4u * c;
                keep[j] = want;   // 16 c < s + wl <= 15 + window: inside the row
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                if (!keep[j]) continue;
                uint32_t* d = img + dst[j];
                d[0] = v[j].x; d[1] = v[j].y; d[2] = v[j].z; d[3] = v[j].w;
            }
        }
        meta[lane] = s | (ok ? 0x100u : 0u);
        offs[lane] = off;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- DECODE: one u64 per numeric field per packet, field-major ----
        const uint8_t* frame = a.base + off;
        if (a.values && live) {
            for (uint32_t f = 0; f < tab.n; ++f) {
                const uint64_t v = ok ? decode_field(tab.f[f], rowb, s, window, frame) : 0ull;
                a.values[(uint64_t)f * a.n_cap + my] = v;
            }
        }
        if (a.status && live) a.status[my] = ok ? 0u : 9u;   // ParseStatus SUCCESS / PACKET_TOO_SHORT

        // ---- IMAGE: the tile's packets' [0, span) bytes as one contiguous region ----
        if (a.image && span) {
            const uint32_t cnt = min(64u, a.n - p0);
            const uint32_t total = cnt * span;
            uint8_t* out = a.image + (uint64_t)p0 * span;
            const float inv = 1.0f / (float)span;
            for (uint32_t q = lane; q < total; q += 64u) {
                uint32_t j = (uint32_t)((float)q * inv);
                if (j * span > q) --j;                     // float rounding: one step either way
                else if ((j + 1u) * span <= q) ++j;
                const uint32_t b = q - j * span;
                const uint32_t m = meta[j];
                uint32_t val = 0;
                if (m & 0x100u) {
                    const uint8_t* rj = reinterpret_cast<const uint8_t*>(img + j * kExRow);
                    val = b < window ? (uint32_t)rj[(m & 15u) + b] : (uint32_t)a.base[offs[j] + b];
                }
                out[q] = (uint8_t)val;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace

int launch_extract(const ExArgs& a, const ExTable& tab, void* stream) {
    if (a.ntiles == 0) return BT_OK;
    static int per_cu = 0, cus = 0;
    static std::once_flag once;
    std::call_once(once, [] {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bt_extract_tile, kBlock, 0) != hipSuccess) per_cu = 1;
        if (cus <= 0) cus = 256;
        if (per_cu <= 0) per_cu = 1;
    });
    const uint32_t needed = (a.ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t grid = std::min<uint32_t>(needed, (uint32_t)(cus * per_cu));
    hipLaunchKernelGGL(bt_extract_tile, dim3(grid), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream), a, tab);
    return hipGetLastError() == hipSuccess ? BT_OK : BT_E_INTERNAL;
}

}  // namespace bt
