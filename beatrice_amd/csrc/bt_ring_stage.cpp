// bt_ring_stage.cpp — bt_ring_stage_tpv3: a run of ready TPACKET_V3 ring blocks through the
// GPU filter, the host's walk of each batch of blocks overlapping the device's kernels over
// the batch before it.
//
// The reference's AF_PacketBackend::packetProcessingLoop (src/AF_PacketBackend.cpp:318-363)
// receives one frame per recv(), copies it to the heap and pushes it onto a queue that the
// plugins' PacketFilter::applyFilters then walks packet by packet. Here the ring is the batch:
// the walker (bt_ring_walk_tpv3) turns a batch of blocks into descriptors relative to the
// registered ring, the main kernel reads each frame's header bytes over PCIe in place, and
// only the decision bytes come back. With `gather`, batches instead have each frame's bytes
// 12..43 packed into registered slots on the host (bt_ring_gather_lean_tpv3), which the
// kernels read as one contiguous run; with `in_place_every` = k, every k-th batch is still
// read in place, sharing the work between the host's copies and the GPU's PCIe reads
// (DESIGN.md §9.2); with `in_place_blocks` = m, every batch has its last m blocks read in
// place and the rest gathered.
//
// Batch k's descriptors (and slots) are written while batch k-1's kernels run on the
// context's stream: the kernels are launched asynchronously, the walk of the next batch
// follows at once, and the call waits for the stream only after the last batch. The verdict
// words and the pass count are built from the decisions on the context's host threads at the
// end (a batch starts at any packet, so its tiles do not line up with the words).
#include <algorithm>
#include <atomic>
#include <cstring>

#include "bt_host.h"

extern "C" int bt_ring_stage_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t n_blocks,
                                  const bt_ring_stage_opts* opts, bt_pkt_desc* desc, uint8_t* slots, uint8_t* decide,
                                  uint64_t* verdict, uint32_t cap, uint32_t* n_desc, uint32_t* n_pass) {
    if (!ctx || !ring || !ring->base || !desc || !decide || !n_desc)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_stage_tpv3: null argument");
    if (!ring->n_blocks || first_block >= ring->n_blocks || n_blocks > ring->n_blocks)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_stage_tpv3: block range outside the ring");
    const bt_ring_stage_opts o = opts ? *opts : bt_ring_stage_opts{};
    const uint32_t per = o.batch_blocks ? o.batch_blocks : 128u;
    if (o.gather && !slots) return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_stage_tpv3: gather needs slots");
    if (slots && ((uintptr_t)slots & 15u))
        return bt::set_error(BT_E_INVALID_ARGUMENT, "bt_ring_stage_tpv3: slots not 16-B aligned");
    const int dev = bt::ctx_device(ctx);
    const uint64_t ring_bytes = ring->block_size * ring->n_blocks;
    // every buffer the kernels read or write must be registered (bt_host_register)
    uint8_t *a_ring = nullptr, *a_desc = nullptr, *a_slots = nullptr, *a_dec = nullptr;
    if (bt::pin_alias(ring->base, ring_bytes, dev, &a_ring) || bt::pin_alias(desc, (uint64_t)cap * 8u, dev, &a_desc) ||
        bt::pin_alias(decide, cap, dev, &a_dec) ||
        (o.gather && bt::pin_alias(slots, (uint64_t)cap * BT_PREFIX_SLOT, dev, &a_slots)))
        return bt::set_error(BT_E_INVALID_ARGUMENT,
                             "bt_ring_stage_tpv3: the ring, desc, decide%s must be registered with the context "
                             "(bt_host_register)", o.gather ? " and slots" : "");
    // with gather and in_place_blocks: each batch is two launches, its first blocks gathered and
    // its last in_place_blocks read in place, so the host's copies and the device's PCIe reads
    // share every batch instead of alternating between batches
    const uint32_t split = o.gather == 1u && o.in_place_blocks ? std::min(o.in_place_blocks, per) : 0u;
    // gather == 2 (adaptive): a batch is gathered when the device is still busy with the batches
    // before it (the device is the bound: the host takes on the copies) and read in place when
    // the device has caught up (the host is the bound: it only walks)
    const bool adaptive = o.gather == 2u;
    uint32_t start = 0, done_blocks = 0, k = 0;
    while (done_blocks < n_blocks) {
        const uint32_t part = split ? (k & 1u) : 0u;   // split: even parts gathered, odd in place
        const bool gathered = adaptive ? (k == 0u || bt::ctx_stream_busy(ctx))
                            : split ? part == 0u
                                    : o.gather && !(o.in_place_every && k % o.in_place_every == o.in_place_every - 1);
        const uint32_t fb = (first_block + done_blocks) % ring->n_blocks;
        const uint32_t nb = std::min(split ? (part ? split : per - split) : per, n_blocks - done_blocks);
        uint32_t cnt = 0, taken = 0;
        const int rc = gathered
            ? bt_ring_gather_lean_tpv3(ctx, ring, fb, nb, slots + (uint64_t)start * BT_PREFIX_SLOT, desc + start,
                                       nullptr, cap - start, &cnt, &taken)
            : bt_ring_walk_tpv3(ctx, ring, fb, nb, desc + start, cap - start, &cnt, &taken);
        if (rc) return rc;
        if (!taken) break;   // a block the kernel still owns, or more frames than cap
        if (cnt) {
            bt_batch b{};
            b.base = gathered ? a_slots + (uint64_t)start * BT_PREFIX_SLOT : a_ring;
            b.desc = a_desc + (uint64_t)start * 8u;
            b.n = cnt;
            b.bytes = gathered ? (uint64_t)cnt * BT_PREFIX_SLOT : ring_bytes;
            b.desc_format = BT_DESC_PACKED;
            b.flags = gathered ? (BT_BATCH_PREFIXES | BT_BATCH_LEAN) : 0u;
            bt_outputs out{};
            out.n_cap = cnt;
            out.decide = a_dec + start;
            if (int e = bt_parse_filter_device(ctx, &b, &out, nullptr)) return e;   // async on ctx's stream
        }
        start += cnt;
        done_blocks += taken;
        ++k;
    }
    if (int e = bt_synchronize(ctx)) return e;
    *n_desc = start;
    // verdict words and the pass count from the decisions
    if (verdict || n_pass) {
        const uint32_t words = (start + 63u) / 64u;
        std::atomic<uint64_t> passed{0};
        bt::host_parallel(ctx, [&](unsigned w, unsigned T) {
            const uint32_t a = (uint32_t)((uint64_t)words * w / T), e = (uint32_t)((uint64_t)words * (w + 1) / T);
            uint64_t mine = 0;
            for (uint32_t j = a; j < e; ++j) {
                uint64_t bits = 0;
                const uint32_t hi = std::min(64u, start - 64u * j);
                const uint8_t* d = decide + 64ull * j;
                for (uint32_t i = 0; i < hi; ++i) bits |= (uint64_t)((d[i] >> 6) == 0u) << i;
                if (verdict) verdict[j] = bits;
                mine += (uint64_t)__builtin_popcountll(bits);
            }
            passed.fetch_add(mine);
        });
        if (n_pass) *n_pass = (uint32_t)passed.load();
    }
    return BT_OK;
}
