// bt_extract.hip — gfx950 field extraction for user-defined protocol tables.
//
// The reference's ProtocolParser is a generic, table-driven extractor: for one buffer and
// one ProtocolDefinition, parsePacketInternal (src/parser/ProtocolParser.cpp:238-284) gates
// on getTotalLength(), then extractField / extractValue<T> (:286-433) copy and decode each
// field at its fixed offset. bt_extract_tile does that for a whole batch: one packet per
// lane, one 64-packet tile per wavefront, persistent grid.
//   LOAD   the first `window` (<= 256) bytes of each packet, the span of the table, are
//          staged into a per-wave LDS image with coalesced 16-B loads, four lanes per
//          packet and 16 packets per wave instruction (the main kernel's round A). The
//          rows are sized from the table (dynamic LDS: 11 dwords for a 17-byte span, 71
//          for 256), so a small table leaves the occupancy to the registers;
//   DECODE each lane walks the table (kernel argument, scalar loads) over its own row:
//          the extractValue<T> bits of every numeric field go to a field-major u64 column,
//          so a wave's store for one field is 512 contiguous bytes. A field no longer than
//          its type is one unaligned 8-byte window (two alignbytes over three dwords) and,
//          for the network byte orders, a byte reversal; longer fields keep the byte loop
//          of the reference's masked shifts;
//   IMAGE  the wave writes its tile's packets' [0, span) bytes as one contiguous region,
//          4 bytes per lane and 256 bytes per store instruction, from which the host
//          materialises rawHex and byte fields.
// Fields that end past the staged window (span > 256) read their bytes from memory
// directly, and so does the image then (a byte per lane and store). Both forms give
// identical results; tests check both (tests/test_gpu_extract.py).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "bt_device.h"

namespace bt {

// BT_DEBUG_BOUNDS: this module's log of failed bounds checks (bt_bounds.h)
__device__ BoundsLog g_bounds_extract;

namespace {

// Header loads and the value / image stores are non-temporal: nothing re-reads them, and
// with the default policy c1 took 0.383-0.386 ms against 0.362 (nt loads alone 0.392-0.394,
// nt stores alone 0.374-0.377; profiles/r02/ab/extract_policy.txt).
typedef unsigned int ex_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const uint8_t* p) {
    const ex_u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const ex_u32x4*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}
template <class T>
__device__ __forceinline__ void st_nt(T* p, T v) { __builtin_nontemporal_store(v, p); }

// Byte b (< span) of the packet in row `rowb` (byte 0 at row byte s), or from memory when
// past the staged window. `room` = the bytes readable from the frame's start (the batch's
// bytes minus its offset): a descriptor whose length runs past the buffer reads zeros
// there, never past it.
__device__ __forceinline__ uint32_t byte_at(const uint8_t* rowb, uint32_t s, uint32_t b, uint32_t window,
                                            const uint8_t* frame, uint64_t room) {
    return b < window ? (uint32_t)rowb[s + b] : b < room ? (uint32_t)frame[b] : 0u;
}

// The 4 bytes at row byte x (any alignment), low byte first.
__device__ __forceinline__ uint32_t row_word(const uint32_t* row, uint32_t x) {
    return __builtin_amdgcn_alignbyte(row[(x >> 2) + 1], row[x >> 2], x & 3u);
}

__device__ __forceinline__ uint32_t type_bits(uint32_t type) {
    return (type == BT_FT_UINT8 || type == BT_FT_INT8) ? 8u
         : (type == BT_FT_UINT16 || type == BT_FT_INT16) ? 16u
         : (type == BT_FT_UINT32 || type == BT_FT_INT32 || type == BT_FT_FLOAT32) ? 32u : 64u;
}

// extractValue<T> (src/parser/ProtocolParser.cpp:385-433) for one field of one packet.
__device__ __forceinline__ uint64_t decode_field(const ExField& f, const uint32_t* row, uint32_t s, uint32_t window,
                                                 const uint8_t* frame, uint64_t room) {
    const uint8_t* rowb = reinterpret_cast<const uint8_t*>(row);
    const uint32_t type = f.ctl & 0xFFu;   // every test on the table below is wave-uniform
    const bool le = ((f.ctl >> 8) & 0xFFu) == BT_ENDIAN_LITTLE;
    const uint32_t o = f.offset, L = f.length;
    switch (type) {
    case BT_FT_BOOLEAN: return byte_at(rowb, s, o, window, frame, room) != 0u ? 1u : 0u;   // fieldData[0] != 0
    case BT_FT_BYTES: case BT_FT_STRING: case BT_FT_MAC: case BT_FT_IPV4: case BT_FT_IPV6: case BT_FT_CUSTOM:
        return 0;   // the bytes themselves (image)
    default: break;
    }
    const uint32_t w = type_bits(type);
    if ((type == BT_FT_FLOAT32 || type == BT_FT_FLOAT64) && L * 8u != w) return 0;   // T{}: raw bits only at the width
    if (L * 8u <= w && o + L <= window) {
        // within the type and the staged window: the L bytes as one 8-byte window, low
        // byte first; the network orders put the field's first byte highest
        if (L == 0) return 0;
        const uint32_t x = s + o;
        const uint64_t v = ((uint64_t)row_word(row, x + 4u) << 32) | row_word(row, x);
        if (le) return L >= 8u ? v : v & ((1ull << (8u * L)) - 1ull);
        const uint64_t r = ((uint64_t)__builtin_bswap32((uint32_t)v) << 32) | __builtin_bswap32((uint32_t)(v >> 32));
        return r >> (64u - 8u * L);
    }
    // byte i (from the field's low end) ORed in at (8 i) mod the shift width, then cut to
    // the type's width
    const uint32_t m = w == 64u ? 63u : 31u;
    uint64_t v = 0;
    for (uint32_t i = 0; i < L; ++i) {
        const uint32_t sh = (8u * i) & m;
        if (sh >= w) continue;   // lands past the type's width: cut anyway
        const uint64_t b = byte_at(rowb, s, o + (le ? i : L - 1u - i), window, frame, room);
        v |= b << sh;
    }
    return w == 64u ? v : (v & ((1ull << w) - 1ull));
}

// Packet j of the tile for byte q of its image (q / span, by float reciprocal and one fix).
__device__ __forceinline__ uint32_t packet_of(uint32_t q, uint32_t span, float inv) {
    uint32_t j = (uint32_t)((float)q * inv);
    if (j * span > q) --j;
    else if ((j + 1u) * span <= q) ++j;
    return j;
}

__global__ __launch_bounds__(kBlock) void bt_extract_tile(ExArgs a, ExTable tab) {
    extern __shared__ uint32_t lds_dyn[];
    const uint32_t row_dw = tab.row_dw;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* img = lds_dyn + wid * (kWave * row_dw + 3u * kWave);
    uint32_t* meta = img + kWave * row_dw;                          // per packet: s | ok << 8
    uint64_t* offs = reinterpret_cast<uint64_t*>(meta + kWave);     // per packet: frame offset
    const uint32_t* row = img + lane * row_dw;

    const uint32_t window = tab.window, span = tab.span;
    const uint32_t groups = (window + 15u + 63u) / 64u;   // 4 chunks of 16 B per group
    const uint32_t total_waves = gridDim.x * kWavesPerBlock;
    // the image as dwords: every byte staged (span <= window), a dword holds bytes of at
    // most two packets (span >= 4), and the output is 4-byte aligned (all uniform)
    const bool img_words = a.image && span >= 4u && span <= window && ((uintptr_t)a.image & 3u) == 0u;
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
                const bool want = 16u * c < qe && addr + 16ull <= a.bytes &&
                                  BT_IN(&g_bounds_extract, kSiteExLoad, addr + 15u, a.bytes);
                v[j] = want ? ld16_nt(a.base + addr) : make_uint4(0, 0, 0, 0);
                dst[j] = q * row_dw + 4u * c;
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
        const uint64_t room = off < a.bytes ? a.bytes - off : 0u;
        if (a.values && live) {
            for (uint32_t f = 0; f < tab.n; ++f) {
                const uint64_t v = ok ? decode_field(tab.f[f], row, s, window, frame, room) : 0ull;
                if (BT_IN(&g_bounds_extract, kSiteExValue, (uint64_t)f * a.n_cap + my, (uint64_t)tab.n * a.n_cap))
                    st_nt(a.values + (uint64_t)f * a.n_cap + my, v);
            }
        }
        if (a.status && live && BT_IN(&g_bounds_extract, kSiteExStatus, my, a.n))
            a.status[my] = ok ? 0u : 9u;   // ParseStatus SUCCESS / PACKET_TOO_SHORT

        // ---- IMAGE: the tile's packets' [0, span) bytes as one contiguous region ----
        if (a.image && span) {
            const uint32_t cnt = min(64u, a.n - p0);
            const uint32_t total = cnt * span;
            uint8_t* out = a.image + (uint64_t)p0 * span;
            const float inv = 1.0f / (float)span;
            uint32_t q0 = 0;   // bytes below q0 went out as dwords
            if (img_words) {
                // dword d = bytes 4d..4d+3: packet j from byte b and, when fewer than 4 of
                // its bytes remain, the first bytes of packet j + 1 (which exists: the
                // dword ends inside the tile's image)
                const uint32_t nd = total >> 2;
                for (uint32_t d = lane; d < nd; d += 64u) {
                    const uint32_t q = 4u * d;
                    const uint32_t j = packet_of(q, span, inv);
                    const uint32_t b = q - j * span;
                    const uint32_t mj = meta[j];
                    uint32_t word = (mj & 0x100u) ? row_word(img + j * row_dw, (mj & 15u) + b) : 0u;
                    const uint32_t k = span - b;   // bytes of packet j in this dword
                    if (k < 4u) {
                        const uint32_t mn = meta[j + 1u];
                        const uint32_t nx = (mn & 0x100u) ? row_word(img + (j + 1u) * row_dw, mn & 15u) : 0u;
                        word = (word & ((1u << (8u * k)) - 1u)) | (nx << (8u * k));
                    }
                    if (BT_IN(&g_bounds_extract, kSiteExImage, (uint64_t)p0 * span + q + 3u, (uint64_t)a.n * span))
                        st_nt(reinterpret_cast<uint32_t*>(out + q), word);
                }
                q0 = nd * 4u;
            }
            const uint8_t* rows8 = reinterpret_cast<const uint8_t*>(img);
            for (uint32_t q = q0 + lane; q < total; q += 64u) {   // the tail, or every byte
                const uint32_t j = packet_of(q, span, inv);
                const uint32_t b = q - j * span;
                const uint32_t m = meta[j];
                uint32_t val = 0;
                if (m & 0x100u)
                    val = b < window ? (uint32_t)rows8[4u * j * row_dw + (m & 15u) + b]
                        : offs[j] + b < a.bytes ? (uint32_t)a.base[offs[j] + b] : 0u;
                if (BT_IN(&g_bounds_extract, kSiteExImage, (uint64_t)p0 * span + q, (uint64_t)a.n * span))
                    out[q] = (uint8_t)val;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace

uint32_t bounds_take_extract(void* stream, BoundsLog* first) {
#ifdef BT_DEBUG_BOUNDS
    if (hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return 0;
    BoundsLog log{};
    if (hipMemcpyFromSymbol(&log, HIP_SYMBOL(g_bounds_extract), sizeof(log)) != hipSuccess) return 0;
    if (log.count) {
        const BoundsLog zero{};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_extract), &zero, sizeof(zero));
        if (first) *first = log;
    }
    return log.count;
#else
    (void)stream;
    (void)first;
    return 0;
#endif
}

#ifndef BT_EX_BLOCKS_PER_CU
#define BT_EX_BLOCKS_PER_CU 4   // grid cap (blocks per CU), a build knob for A/B
#endif
int launch_extract(const ExArgs& a, const ExTable& tab_in, void* stream, void* timing_start, void* timing_stop) {
    if (a.ntiles == 0) return BT_OK;
    ExTable tab = tab_in;
    // a row holds the 16-B chunks [a0, a0 + s + window) plus two dwords for the 8-byte
    // windows read at its end; odd, so the per-lane reads spread over the banks
    tab.row_dw = 4u * ((tab.window + 15u + 15u) / 16u) + 3u;
    const uint32_t dyn = (uint32_t)sizeof(uint32_t) * kWavesPerBlock * (kWave * tab.row_dw + 3u * kWave);
    static int cus = 0;
    static std::map<uint32_t, int> per_cu_of;   // resident blocks per CU, by LDS size
    static std::mutex mu;
    int per_cu = 1;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!cus) {
            int dev = 0;
            hipDeviceProp_t prop;
            if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                cus = prop.multiProcessorCount;
            if (cus <= 0) cus = 256;
        }
        auto it = per_cu_of.find(dyn);
        if (it == per_cu_of.end()) {
            // the widest window (256 B) needs 74 KiB per block: past the 64-KiB default
            if (dyn > 65536u &&
                hipFuncSetAttribute(reinterpret_cast<const void*>(&bt_extract_tile),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn) != hipSuccess)
                return BT_E_INTERNAL;
            int r = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&r, bt_extract_tile, kBlock, dyn) != hipSuccess || r <= 0)
                r = 1;
            it = per_cu_of.emplace(dyn, r).first;
        }
        per_cu = it->second;
    }
    // With the non-temporal policy, at most 4 blocks (16 waves) per CU: c1 0.333-0.355 ms
    // against 0.351-0.360 at 5 and 0.380-0.385 at 3 (profiles/r02/ab/extract_policy.txt).
    // Before it, at most 5: with parser_example's table the residency is 8,
    // and fewer concurrent read/write streams suit HBM better (c1, 16M packets: 0.432 ms
    // at 8 blocks/CU, 0.383-0.393 at 4, 0.383-0.385 at 5, 0.387-0.389 at 6, 0.425-0.437
    // at 3, 0.529-0.541 at 2; alternating processes, profiles/r02/ab/c1_grid.txt).
    per_cu = std::min(per_cu, BT_EX_BLOCKS_PER_CU);
    const uint32_t needed = (a.ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t grid = std::min<uint32_t>(needed, (uint32_t)(cus * per_cu));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipEvent_t e0 = reinterpret_cast<hipEvent_t>(timing_start), e1 = reinterpret_cast<hipEvent_t>(timing_stop);
    if (e0 || e1)   // timed from the kernel's own dispatch packet (as launch_main)
        hipExtLaunchKernelGGL(bt_extract_tile, dim3(grid), dim3(kBlock), dyn, st, e0, e1, 0, a, tab);
    else
        hipLaunchKernelGGL(bt_extract_tile, dim3(grid), dim3(kBlock), dyn, st, a, tab);
    return hipGetLastError() == hipSuccess ? BT_OK : BT_E_INTERNAL;
}

}  // namespace bt
