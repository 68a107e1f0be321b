// bt_device.h — shared between the host runtime and the gfx950 kernels.
#pragma once

#include <stdint.h>

#include "beatrice_gpu.h"
#include "bt_bounds.h"

namespace bt {

// Compiled filter slot as the device sees it (32 B; kernel-argument resident).
// kind / a / b: the bt_filter_slot fields (PAYLOAD: a = blob offset, b = blob size).
// mask / lo / span / ctl: the same slot as one uniform predicate over the packet's
// features (to_device_program), so a program without PAYLOAD slots is evaluated with
// no per-kind branching:
//   x1, x2 = the feature pair ctl&3 selects: 0 (src, dst IPv4), 1 (sport, dport),
//            2 (proto, proto), 3 (pbit, pbit) with pbit = tcp | udp<<1 | icmp<<2
//   pred   = ((x1 & mask) - lo) <= span  ||  ((x2 & mask) - lo) <= span   (unsigned)
//   gate   = ctl>>2 & 3: 0 none, 1 IPv4 gate (len >= 34, EtherType 0x0800),
//            2 IPv4 gate and the TCP/UDP length gate of the port filter
//   result = !gate ? 0 : ctl>>4 & 3: 0 pred, 1 throw (2), 2 host (3)
struct DevFilter {
    uint32_t kind, a, b, ctl;
    uint32_t mask, lo, span, pad;
};
constexpr uint32_t kSelIp = 0, kSelPort = 1, kSelProto = 2, kSelPbit = 3;
constexpr uint32_t kGateNone = 0, kGateIpv4 = 1, kGateL4 = 2;
constexpr uint32_t kResPred = 0, kResThrow = 1, kResHost = 2;

struct DevProgram {
    uint32_t n;
    uint32_t pad[3];
    DevFilter f[BT_MAX_FILTERS];
};

// Everything the main kernel needs (passed by value as a kernel argument).
struct MainArgs {
    const uint8_t* base;
    const uint64_t* desc;      // nullptr: fixed stride
    uint32_t desc_words;       // descriptor stride in u64 words: 1 packed, 2 xdp_desc
    uint64_t bytes;            // read limit from base: round_up(base + bytes, 16) - base (read_limit)
    uint32_t stride;
    uint32_t n;
    uint32_t ntiles;           // ceil(n / 64): one wavefront tile = 64 packets
    uint32_t n_cap;            // record plane stride (records)
    uint8_t* records;          // plane-major (or AoS when the AOS variant is launched)
    uint8_t* decide;
    uint64_t* verdict;         // per-tile pass words (also the compaction's input)
    uint32_t blocked;          // tile order: 0 cyclic, 1 one contiguous range per wavefront
    uint32_t nt;               // bit0 non-temporal record stores, bit1 non-temporal header loads,
                               // bit2 / bit3 force two-round / wide loads (A/B)
    const uint8_t* dfa;        // PAYLOAD DFA pool (device), copied to dynamic LDS per block
    uint32_t dfa_bytes;        // 0: the program has no BT_K_PAYLOAD slot
    uint32_t prefixes;         // BT_BATCH_PREFIXES: base holds header prefixes only
    uint32_t lean;             // descriptor mode: bytes of a frame round A reads at most (0xFFFF:
                               // its first 64-B window); 38 for host-resident frames (kLeanPcie)
    uint32_t lean_lo;          // ... and the first of them it needs: round A skips the 16-B chunks
                               // that end at or before it (0; 12 for lean calls: nothing in a
                               // filter-only call reads the MAC addresses)
};
// Frames read over PCIe (registered host memory) by a filter-only call: round A reads only
// the 16-B chunks holding bytes 12..37 of a frame (every filter gate and the detector column)
// instead of the whole 64-B window (DESIGN.md §9.2 has the A/Bs: round 3's first 46 B, round
// 4's [12, 38): C4 +3..7 %, the others level).
constexpr uint32_t kLeanPcie = 38;
constexpr uint32_t kLeanLo = 12;

constexpr uint32_t kDfaPoolMax = 16384;   // bytes of DFA tables per program (LDS budget)

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kRowDwords = 33;                    // 128 B header window + 4 B pad (bank spread)
constexpr int kChunkTiles = 256;                  // compaction chunk = 16Ki packets (one tile per thread)
constexpr uint32_t kNeedParse = 102;              // 14 + 2*4 + 60 (IPv4 max) + 20 (TCP fields)
constexpr uint32_t kNeedFilter = 38;              // PacketFilter reads bytes 12..37

// Launch wrappers (bt_kernels.hip). All are asynchronous on `stream`.
enum RecLayout { kRecNone = 0, kRecPlanes = 1, kRecAoS = 2, kRecTiled = 3 };
// timing_start / timing_stop (hipEvent_t, may be null): recorded by the kernel's own
// dispatch (hipExtLaunchKernelGGL), so timing a launch adds no packets to the stream.
int launch_main(const MainArgs& a, const DevProgram& prog, int rec_layout, bool filter,
                int grid_blocks, bool prefetch, void* stream, void* timing_start = nullptr,
                void* timing_stop = nullptr);
// The ordered compaction of an n-packet batch: pass_idx = the indices of the set verdict
// bits, ascending; n_pass = their count. chunk_sums: ceil(ceil(n / 64) / kChunkTiles) words
// of workspace.
int launch_compact(const uint64_t* verdict, uint32_t n, uint32_t* chunk_sums, uint32_t* pass_idx,
                   uint32_t* n_pass, void* stream);
int device_grid_blocks(int device);

// The limit the kernels' 16-B chunk reads are checked against: chunks sit at 16-B offsets
// from base, and a chunk may pass the buffer's last byte, but never the end of the
// 16-B-aligned (absolute address) granule that holds it, so never another page.
inline uint64_t read_limit(const void* base, uint64_t bytes) {
    const uint64_t b = (uint64_t)(uintptr_t)base;
    return bytes ? ((b + bytes + 15u) & ~15ull) - b : 0u;
}

// BT_DEBUG_BOUNDS builds (bt_bounds.h): wait for `stream`, then read and clear the
// module's log; returns the number of failed checks since the last call (*first = the
// first one). Release builds return 0 without touching the device.
uint32_t bounds_take_main(void* stream, BoundsLog* first);
uint32_t bounds_take_extract(void* stream, BoundsLog* first);

// ---- TPACKET_V3 frame-chain walk on the GPU (bt_ring_walk.hip) ----
struct RingBlock {                    // one taken block, from its header (read by the host)
    uint32_t block;                   // ring block index
    uint32_t n;                       // num_pkts
    uint32_t start;                   // index of its first descriptor
    uint32_t first_off;               // offset_to_first_pkt
};
struct RingWalkArgs {
    const uint8_t* ring;              // device-visible ring (bt_host_register alias)
    uint64_t block_size;
    const RingBlock* blocks;          // pinned host memory, read by the kernel
    uint32_t count;
    bt_pkt_desc* desc;                // device memory, cap entries
    uint32_t cap;
    uint32_t* bad;                    // optional: max(block + 1) of the malformed blocks
};
int launch_ring_walk(const RingWalkArgs& a, void* stream);
uint32_t bounds_take_ring(void* stream, BoundsLog* first);

// ---- user-defined protocol extraction (bt_extract.hip) ----
constexpr uint32_t kExWindow = 256;   // bytes of each packet staged in LDS; fields past it read memory
struct ExField {                      // one bt_field_def as the kernel sees it
    uint32_t offset, length;          // both < 65536 once the table's span is
    uint32_t ctl;                     // type | endianness << 8
    uint32_t pad;
};
struct ExTable {                      // kernel argument
    uint32_t n;                       // fields
    uint32_t span;                    // getTotalLength()
    uint32_t window;                  // min(span, kExWindow)
    uint32_t row_dw;                  // LDS dwords per staged packet (set by launch_extract)
    ExField f[BT_FIELD_MAX];
};
struct ExArgs {
    const uint8_t* base;
    const uint64_t* desc;             // nullptr: fixed stride
    uint32_t desc_words;
    uint64_t bytes;                   // read limit from base (read_limit)
    uint32_t stride, n, ntiles;
    uint8_t* status;
    uint64_t* values;
    uint8_t* image;
    uint32_t n_cap;
};
int launch_extract(const ExArgs& a, const ExTable& tab, void* stream, void* timing_start = nullptr,
                   void* timing_stop = nullptr);

// Host filter compiler (bt_filter_compile.cpp): pure C++, no device needed.
int compile_filters(const bt_filter_desc* f, uint32_t n, bt_filter_slot* out, uint32_t cap,
                    uint32_t* n_slots, char* err, size_t errlen);
void to_device_program(const bt_filter_slot* s, uint32_t n, DevProgram* p);

}  // namespace bt
