// bt_ring.cpp — capture-ring ingest for the parse+filter stage: the AF_PACKET
// TPACKET_V3 block walker (include/beatrice_gpu.h, "capture-ring ingest").
//
// It replaces the reference's AF_PacketBackend::packetProcessingLoop
// (src/AF_PacketBackend.cpp:318-363): one recv() into a 64 KiB buffer, a heap copy
// and a locked queue push per packet, then a 100 us sleep. With a PACKET_RX_RING the
// kernel writes frames into shared blocks; this file only produces descriptors
// pointing into those blocks, so the GPU reads the frames in place.
//
// Block layout (linux/if_packet.h; net/packet/af_packet.c, prb_* helpers):
//   tpacket_block_desc { version, offset_to_priv, hdr.bh1 { block_status, num_pkts,
//                        offset_to_first_pkt, blk_len, seq_num, ts_first, ts_last } }
//   frame j at offset_to_first_pkt + sum(tp_next_offset of frames < j):
//   tpacket3_hdr { tp_next_offset, tp_sec, tp_nsec, tp_snaplen, tp_len, tp_status,
//                  tp_mac, tp_net, ... }, MAC header at frame + tp_mac.
// num_pkts is in the block header, so a prefix over the taken blocks places every
// block's descriptors before any frame is read and the blocks are walked in parallel.
#include <emmintrin.h>
#include <linux/if_packet.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "bt_host.h"

namespace {

constexpr uint32_t kDescLenMax = 0xFFFF;

inline const tpacket_block_desc* block_at(const bt_tpv3_ring* r, uint32_t b) {
    return reinterpret_cast<const tpacket_block_desc*>(static_cast<const uint8_t*>(r->base) +
                                                       (uint64_t)b * r->block_size);
}

inline uint32_t status_acquire(const tpacket_block_desc* bd) {
    return __atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE);
}

// Walks the frame chains of `count` blocks in lock-step. Each chain is a dependent
// load sequence (the next header's offset is in the current header), so one chain per
// thread is bound by memory / TLB latency per frame; advancing kChains chains round-
// robin, with the next header prefetched as soon as its offset is known, keeps that
// many misses in flight per thread. Chain g starts g * kStagger rounds late: blocks are
// block_size-aligned, so chains that advance in phase sit at equal offsets in their
// blocks and collide in the same cache sets (measured: C3 with 1 MiB blocks stopped
// scaling past one thread without it). Returns the first malformed block, or -1.
#ifndef BT_RING_CHAINS
#define BT_RING_CHAINS 16   // a build knob for A/B
#endif
constexpr int kChains = BT_RING_CHAINS;
constexpr uint32_t kStagger = 4;

struct Chain {
    const uint8_t* blk;
    uint64_t base_off, off;
    uint32_t j, n, delay;
    bt_pkt_desc* out;
    bt_pkt_desc* rout;         // dense gather: the frames' ring descriptors too (optional)
    int64_t block;
    uint64_t first;            // global index of the block's first frame (slot numbering)
    const uint8_t* pend;       // gather: frame whose prefix is copied on the next visit
    uint32_t pend_len;
    uint8_t* pend_slot;
    uint8_t* line;             // dense gather: the 64-B line being filled, and its
    uint32_t fill;             //   16-B chunks so far (staged in `stage`)
    __m128i stage[4];
};

// What the walk does with each frame besides its descriptor.
enum WalkMode { kWalkOnly, kGatherSlots, kGatherDense, kGatherLean };

// Lean gather (filter-only batches): each frame's bytes [kLeanFrom, kLeanFrom + 32), the 16-B
// chunk pair holding what every filter gate reads (12..37), packed like the dense gather
// after a 16-B pad at the block's first slot; a descriptor points kLeanFrom bytes before its
// frame's chunks.
constexpr uint32_t kLeanFrom = 12;
constexpr bool packs(WalkMode m) { return m == kGatherDense || m == kGatherLean; }

inline uint8_t* dense_at(const Chain& ch) { return ch.line + 16u * ch.fill; }

inline void push16(Chain& ch, __m128i v) {
    ch.stage[ch.fill++] = v;
    if (ch.fill == 4) {
        __m128i* d = reinterpret_cast<__m128i*>(ch.line);
        _mm_stream_si128(d, ch.stage[0]);
        _mm_stream_si128(d + 1, ch.stage[1]);
        _mm_stream_si128(d + 2, ch.stage[2]);
        _mm_stream_si128(d + 3, ch.stage[3]);
        ch.line += 64;
        ch.fill = 0;
    }
}

inline void flush_stage(Chain& ch) {
    for (uint32_t i = 0; i < ch.fill; ++i) _mm_stream_si128(reinterpret_cast<__m128i*>(ch.line) + i, ch.stage[i]);
}

inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

// The bytes the layer walk and the built-in filters read (the kernel's header_end,
// bt_kernels.hip): EtherTypes at 12/16/20, IHL at L3, at least 38 (filter gates and the
// detector), rounded up to 16 and capped at the frame.
inline uint32_t prefix_len(const uint8_t* f, uint32_t len) {
    uint32_t end = 38;
    if (len >= 24) {
        uint32_t o3 = 14, et = be16(f + 12);
        if (et == 0x8100u || et == 0x88A8u) {
            o3 = 18;
            et = be16(f + 16);
            if (et == 0x8100u || et == 0x88A8u) { o3 = 22; et = be16(f + 20); }
        }
        if (et == 0x0800u && len > o3) {
            const uint32_t ihl = f[o3] & 0x0Fu;
            end = o3 + 20u + (ihl > 5 ? 4u * ihl - 20u : 0u) + 20u;
        } else if (et == 0x86DDu) {
            end = o3 + 60u;
        }
        end = end > 38u ? end : 38u;
    }
    end = (end + 15u) & ~15u;
    if (end > BT_PREFIX_SLOT) end = BT_PREFIX_SLOT;
    return end < len ? end : len;
}

// Slots: non-temporal 16-B stores into the (16-B-aligned) slot: the slot lines are not
// read for ownership first, and they do not evict the ring lines the chains still walk.
// Dense: each chain writes its block's prefixes back to back; 16 chains per thread are more
// open lines than the write-combining buffers hold, so the chunks are staged per chain and
// streamed as whole lines.
template <WalkMode MODE>
inline void copy_prefix(Chain& ch) {
    if (MODE == kGatherLean) {   // two chunks, zero past the frame (whose end may end the mapping)
        const uint32_t len = ch.pend_len;
        if (len >= kLeanFrom + 32u) {
            push16(ch, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ch.pend + kLeanFrom)));
            push16(ch, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ch.pend + kLeanFrom + 16)));
        } else {
            alignas(16) uint8_t t[32] = {};
            if (len > kLeanFrom) std::memcpy(t, ch.pend + kLeanFrom, len - kLeanFrom);
            push16(ch, _mm_load_si128(reinterpret_cast<const __m128i*>(t)));
            push16(ch, _mm_load_si128(reinterpret_cast<const __m128i*>(t + 16)));
        }
        ch.pend = nullptr;
        return;
    }
    const uint32_t m = prefix_len(ch.pend, ch.pend_len);
    if (MODE == kGatherDense) {
        const uint32_t full = m & ~15u;
        uint32_t k = 0;
        for (; k < full; k += 16) push16(ch, _mm_loadu_si128(reinterpret_cast<const __m128i*>(ch.pend + k)));
        if (k < m) {
            alignas(16) uint8_t tail[16] = {};
            std::memcpy(tail, ch.pend + k, m - k);
            push16(ch, _mm_load_si128(reinterpret_cast<const __m128i*>(tail)));
        }
        ch.pend = nullptr;
        return;
    }
    if (((uintptr_t)ch.pend_slot & 15u) == 0) {
        // whole 16-B chunks of the frame with vector loads; the last partial chunk with
        // memcpy into a zeroed chunk, so no load reads past the frame (whose end may be
        // the end of the ring mapping)
        const uint32_t full = std::min(m, ch.pend_len) & ~15u;
        uint32_t k = 0;
        for (; k < full; k += 16) {
            const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(ch.pend + k));
            _mm_stream_si128(reinterpret_cast<__m128i*>(ch.pend_slot + k), v);
        }
        if (k < m) {
            alignas(16) uint8_t tail[16] = {};
            std::memcpy(tail, ch.pend + k, std::min<uint32_t>(16u, ch.pend_len - std::min(ch.pend_len, k)));
            _mm_stream_si128(reinterpret_cast<__m128i*>(ch.pend_slot + k),
                             _mm_load_si128(reinterpret_cast<const __m128i*>(tail)));
        }
    } else {
        std::memcpy(ch.pend_slot, ch.pend, m);
    }
    ch.pend = nullptr;
}

template <WalkMode MODE>
int64_t walk_blocks(const bt_tpv3_ring* r, const uint32_t* blocks, const uint32_t* start, uint32_t count,
                    bt_pkt_desc* desc, uint8_t* slots, bt_pkt_desc* ring_desc) {
    const uint64_t bs = r->block_size;
    for (uint32_t g0 = 0; g0 < count; g0 += kChains) {
        Chain c[kChains];
        int live = 0;
        for (uint32_t k = g0; k < std::min(count, g0 + kChains); ++k) {
            const uint32_t b = blocks[k];
            Chain& ch = c[live];
            ch.blk = static_cast<const uint8_t*>(r->base) + (uint64_t)b * bs;
            ch.base_off = (uint64_t)b * bs;
            const tpacket_block_desc* bd = reinterpret_cast<const tpacket_block_desc*>(ch.blk);
            ch.off = bd->hdr.bh1.offset_to_first_pkt;
            ch.n = bd->hdr.bh1.num_pkts;
            ch.j = 0;
            ch.out = desc + start[k];
            ch.rout = ring_desc ? ring_desc + start[k] : nullptr;
            ch.block = b;
            ch.first = start[k];
            ch.pend = nullptr;
            ch.line = slots ? slots + (uint64_t)start[k] * BT_PREFIX_SLOT + (MODE == kGatherLean ? 16u : 0u) : nullptr;
            ch.fill = 0;
            if (ch.n) {
                __builtin_prefetch(ch.blk + ch.off);
                ++live;
            }
        }
        for (int g = 0; g < live; ++g) c[g].delay = (uint32_t)g * kStagger;
        while (live) {
            for (int g = 0; g < live;) {
                Chain& ch = c[g];
                if (ch.delay) {
                    --ch.delay;
                    ++g;
                    continue;
                }
                if (MODE != kWalkOnly && ch.pend) copy_prefix<MODE>(ch);   // its lines were prefetched a round ago
                if (ch.off + sizeof(tpacket3_hdr) > bs) return ch.block;
                const tpacket3_hdr* h = reinterpret_cast<const tpacket3_hdr*>(ch.blk + ch.off);
                const uint64_t mac = ch.off + h->tp_mac;
                const uint32_t snap = h->tp_snaplen, next = h->tp_next_offset;
                if (mac + snap > bs) return ch.block;
                if (MODE != kWalkOnly) {
                    const uint64_t i = ch.first + ch.j;
                    ch.pend_slot = packs(MODE) ? dense_at(ch) : slots + i * BT_PREFIX_SLOT;
                    ch.out[ch.j] = BT_DESC((uint64_t)(ch.pend_slot - slots) - (MODE == kGatherLean ? kLeanFrom : 0u),
                                           std::min<uint32_t>(snap, kDescLenMax));
                    if (ch.rout) ch.rout[ch.j] = BT_DESC(ch.base_off + mac, std::min<uint32_t>(snap, kDescLenMax));
                    ch.pend = ch.blk + mac;
                    ch.pend_len = snap;
                    __builtin_prefetch(ch.pend);
                    __builtin_prefetch(ch.pend + 63);
                } else {
                    ch.out[ch.j] = BT_DESC(ch.base_off + mac, std::min<uint32_t>(snap, kDescLenMax));
                }
                if (++ch.j == ch.n) {          // chain done: swap in the last live one
                    if (MODE != kWalkOnly && ch.pend) copy_prefix<MODE>(ch);
                    if (packs(MODE)) flush_stage(ch);
                    c[g] = c[--live];
                    continue;
                }
                if (next < sizeof(tpacket3_hdr)) return ch.block;
                ch.off += next;
                __builtin_prefetch(ch.blk + ch.off);
                ++g;
            }
        }
    }
    return -1;
}

}  // namespace

extern "C" {

namespace {

int ring_walk(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks, uint8_t* slots,
              WalkMode mode, bt_pkt_desc* desc, bt_pkt_desc* ring_desc, uint32_t cap, uint32_t* n_desc,
              uint32_t* n_blocks_taken) {
    if (!ring || !ring->base || !n_desc || !n_blocks_taken || (cap && !desc))
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3: null argument");
    if (!ring->n_blocks || ring->block_size < sizeof(tpacket_block_desc) || first_block >= ring->n_blocks)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3: bad ring geometry");
    *n_desc = 0;
    *n_blocks_taken = 0;
    // 1. which blocks are ready, and where each one's descriptors go
    const uint32_t lim = std::min(max_blocks, ring->n_blocks);
    std::vector<uint32_t> blocks, start;
    uint64_t total = 0;
    for (uint32_t k = 0; k < lim; ++k) {
        const uint32_t b = (first_block + k) % ring->n_blocks;
        const tpacket_block_desc* bd = block_at(ring, b);
        if (!(status_acquire(bd) & TP_STATUS_USER)) break;
        const uint32_t np = bd->hdr.bh1.num_pkts;
        if (total + np > cap) break;
        if (np && bd->hdr.bh1.offset_to_first_pkt >= ring->block_size)
            return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3: block %u: first frame outside block", b);
        blocks.push_back(b);
        start.push_back((uint32_t)total);
        total += np;
    }
    // 2. walk the taken blocks in parallel: contiguous runs of blocks per worker, each
    //    worker interleaving up to kChains block chains
    const uint32_t nb = (uint32_t)blocks.size();
    std::atomic<int64_t> bad{-1};
    auto work = [&](unsigned w, unsigned T) {
        const uint32_t a = (uint32_t)((uint64_t)nb * w / T), b = (uint32_t)((uint64_t)nb * (w + 1) / T);
        if (a >= b) return;
        const uint32_t* bl = blocks.data() + a;
        const uint32_t* st = start.data() + a;
        const int64_t e = mode == kWalkOnly ? walk_blocks<kWalkOnly>(ring, bl, st, b - a, desc, nullptr, nullptr)
                        : mode == kGatherDense ? walk_blocks<kGatherDense>(ring, bl, st, b - a, desc, slots, ring_desc)
                        : mode == kGatherLean ? walk_blocks<kGatherLean>(ring, bl, st, b - a, desc, slots, ring_desc)
                                              : walk_blocks<kGatherSlots>(ring, bl, st, b - a, desc, slots, nullptr);
        if (slots) _mm_sfence();   // this worker's streaming stores land before the join
        if (e >= 0) bad.store(e);
    };
    if (total >= 4096 && nb > 1) bt::host_parallel(ctx, work);
    else work(0, 1);
    if (bad.load() >= 0)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3: block %lld: frame chain leaves the block",
                             (long long)bad.load());
    *n_desc = (uint32_t)total;
    *n_blocks_taken = nb;
    return BT_OK;
}

}  // namespace

int bt_ring_walk_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                      bt_pkt_desc* desc, uint32_t cap, uint32_t* n_desc, uint32_t* n_blocks_taken) {
    return ring_walk(ctx, ring, first_block, max_blocks, nullptr, kWalkOnly, desc, nullptr, cap, n_desc, n_blocks_taken);
}

int bt_ring_gather_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                        uint8_t* slots, bt_pkt_desc* desc, uint32_t cap, uint32_t* n_desc,
                        uint32_t* n_blocks_taken) {
    if (!slots && cap) return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_gather_tpv3: null slots");
    return ring_walk(ctx, ring, first_block, max_blocks, slots, kGatherSlots, desc, nullptr, cap, n_desc, n_blocks_taken);
}

int bt_ring_gather_dense_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                              uint8_t* slots, bt_pkt_desc* desc, bt_pkt_desc* ring_desc, uint32_t cap,
                              uint32_t* n_desc, uint32_t* n_blocks_taken) {
    if (!slots && cap) return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_gather_dense_tpv3: null slots");
    if ((uintptr_t)slots & 15u)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_gather_dense_tpv3: slots not 16-B aligned");
    return ring_walk(ctx, ring, first_block, max_blocks, slots, kGatherDense, desc, ring_desc, cap, n_desc, n_blocks_taken);
}

int bt_ring_gather_lean_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                             uint8_t* slots, bt_pkt_desc* desc, bt_pkt_desc* ring_desc, uint32_t cap,
                             uint32_t* n_desc, uint32_t* n_blocks_taken) {
    if (!slots && cap) return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_gather_lean_tpv3: null slots");
    if ((uintptr_t)slots & 15u)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_gather_lean_tpv3: slots not 16-B aligned");
    return ring_walk(ctx, ring, first_block, max_blocks, slots, kGatherLean, desc, ring_desc, cap, n_desc, n_blocks_taken);
}

int bt_ring_release_tpv3(const bt_tpv3_ring* ring, uint32_t first_block, uint32_t count) {
    if (!ring || !ring->base || !ring->n_blocks || first_block >= ring->n_blocks || count > ring->n_blocks)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_release_tpv3: bad arguments");
    for (uint32_t k = 0; k < count; ++k) {
        tpacket_block_desc* bd = reinterpret_cast<tpacket_block_desc*>(
            static_cast<uint8_t*>(ring->base) + (uint64_t)((first_block + k) % ring->n_blocks) * ring->block_size);
        __atomic_store_n(&bd->hdr.bh1.block_status, (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE);
    }
    return BT_OK;
}

}  // extern "C"
