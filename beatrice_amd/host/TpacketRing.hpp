// TpacketRing.hpp — an AF_PACKET TPACKET_V3 receive ring.
//
// The reference's AF_PacketBackend reads one packet per recv() into a 64 KiB buffer,
// copies it to the heap and sleeps 100 us (src/AF_PacketBackend.cpp:318-363). Here
// the socket gets a PACKET_RX_RING instead: the kernel fills shared blocks of frames
// and the consumer takes whole blocks (bt_ring_walk_tpv3), reads the frames where
// they lie — on the host or, once the ring is registered with bt_host_register, from
// the GPU — and hands the blocks back (bt_ring_release_tpv3).
//
// Socket creation, interface lookup and bind fail with the reference's messages
// (createSocket :261-269, bindToInterface :271-297).
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <vector>

#include "beatrice/Error.hpp"
#include "beatrice_gpu.h"

namespace beatrice {
namespace gpu {

class TpacketV3Ring {
public:
    struct Options {
        std::string interface;
        uint32_t blockSize = 1u << 22;     // bytes per block (page multiple); frames up to
                                           // blockSize - 130 B are captured whole
        uint32_t numBlocks = 64;
        uint32_t retireTimeoutMs = 2;      // a partly filled block is handed over after this
        bool promiscuous = true;
        int fanoutGroup = -1;              // >= 0: PACKET_FANOUT_HASH group (one ring per worker)
    };
    struct Stats {
        uint64_t packets = 0, drops = 0, freezes = 0;   // PACKET_STATISTICS (tpacket_stats_v3)
    };

    TpacketV3Ring() = default;
    ~TpacketV3Ring();
    TpacketV3Ring(const TpacketV3Ring&) = delete;
    TpacketV3Ring& operator=(const TpacketV3Ring&) = delete;

    Result<void> open(const Options& opts);
    // Adopts an existing ring image (blockSize x numBlocks bytes at `mem`, e.g. a ring
    // shared by another process or a saved kernel-written ring being replayed): no
    // socket; waitReady only checks block status. The memory stays the caller's.
    Result<void> attach(void* mem, uint32_t blockSize, uint32_t numBlocks);
    void close();
    bool isOpen() const { return map_ != nullptr; }

    // ring geometry for the C-ABI (base = host address of the mapping)
    bt_tpv3_ring ring() const { return bt_tpv3_ring{map_, opts_.blockSize, opts_.numBlocks, 0}; }
    uint64_t bytes() const { return (uint64_t)opts_.blockSize * opts_.numBlocks; }
    uint32_t cursor() const { return cursor_; }
    int fd() const { return fd_; }

    // true once the block at the cursor belongs to user space (polls the socket)
    bool waitReady(std::chrono::milliseconds timeout);
    // walks up to maxBlocks ready blocks from the cursor (bt_ring_walk_tpv3 on ctx's
    // host pool; ctx may be null); desc receives ring-relative descriptors
    Result<uint32_t> take(bt_ctx* ctx, uint32_t maxBlocks, bt_pkt_desc* desc, uint32_t cap, uint32_t* n);
    // the same walk, with each frame's header prefix packed into `slots` (bt_ring_gather_dense_tpv3:
    // slotDesc points into slots, ringDesc at the frames); lean: only frame bytes 12..43 for
    // filter-only batches (bt_ring_gather_lean_tpv3, run with BT_BATCH_LEAN)
    Result<uint32_t> takeGathered(bt_ctx* ctx, uint32_t maxBlocks, uint8_t* slots, bt_pkt_desc* slotDesc,
                                  bt_pkt_desc* ringDesc, uint32_t cap, uint32_t* n, bool lean = false);
    // hands `blocks` blocks back to the kernel starting at the cursor and advances it
    void release(uint32_t blocks);
    Stats statistics();
    const std::string& lastError() const { return err_; }

private:
    Options opts_;
    int fd_ = -1;
    void* map_ = nullptr;
    bool owned_ = false;      // map_ is our mmap of the socket's ring
    uint32_t cursor_ = 0;
    std::string err_;
};

}  // namespace gpu
}  // namespace beatrice
