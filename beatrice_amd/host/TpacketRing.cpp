// TpacketRing.cpp — see TpacketRing.hpp.
#include "TpacketRing.hpp"

#include <arpa/inet.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <net/if.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

namespace beatrice {
namespace gpu {

namespace {
std::string errstr() { return std::string(strerror(errno)); }
}  // namespace

TpacketV3Ring::~TpacketV3Ring() { close(); }

Result<void> TpacketV3Ring::open(const Options& o) {
    close();
    opts_ = o;
    const long page = sysconf(_SC_PAGESIZE);
    if (o.interface.empty() || o.interface.size() >= IFNAMSIZ)
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT, err_ = "Invalid interface: " + o.interface);
    if (!o.numBlocks || !o.blockSize || o.blockSize % page)
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT,
                                   err_ = "ring block size must be a non-zero multiple of the page size");
    fd_ = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
    if (fd_ < 0)
        return Result<void>::error(ErrorCode::INITIALIZATION_FAILED,
                                   err_ = "Failed to create AF_PACKET socket: " + errstr());
    auto fail = [&](const std::string& what) {
        err_ = what + ": " + errstr();
        close();
        return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, err_);
    };
    int v = TPACKET_V3;
    if (setsockopt(fd_, SOL_PACKET, PACKET_VERSION, &v, sizeof(v)) < 0) return fail("PACKET_VERSION");
    tpacket_req3 req{};
    req.tp_block_size = o.blockSize;
    req.tp_block_nr = o.numBlocks;
    req.tp_frame_size = 2048;   // V3 packs variable-size frames; the kernel only checks the geometry
    req.tp_frame_nr = (uint32_t)((uint64_t)o.blockSize * o.numBlocks / req.tp_frame_size);
    req.tp_retire_blk_tov = o.retireTimeoutMs;
    if (setsockopt(fd_, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req)) < 0) return fail("PACKET_RX_RING");
    map_ = mmap(nullptr, bytes(), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, 0);
    if (map_ == MAP_FAILED) {
        map_ = nullptr;
        return fail("mmap of the RX ring");
    }
    owned_ = true;
    ifreq ifr{};
    std::strncpy(ifr.ifr_name, o.interface.c_str(), IFNAMSIZ - 1);
    if (ioctl(fd_, SIOCGIFINDEX, &ifr) < 0) return fail("Failed to get interface index");
    sockaddr_ll addr{};
    addr.sll_family = AF_PACKET;
    addr.sll_protocol = htons(ETH_P_ALL);
    addr.sll_ifindex = ifr.ifr_ifindex;
    if (bind(fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0) return fail("Failed to bind to interface");
    if (o.promiscuous) {
        packet_mreq mr{};
        mr.mr_ifindex = ifr.ifr_ifindex;
        mr.mr_type = PACKET_MR_PROMISC;
        if (setsockopt(fd_, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof(mr)) < 0) return fail("PACKET_MR_PROMISC");
    }
    if (o.fanoutGroup >= 0) {
        int arg = (o.fanoutGroup & 0xFFFF) | (PACKET_FANOUT_HASH << 16);
        if (setsockopt(fd_, SOL_PACKET, PACKET_FANOUT, &arg, sizeof(arg)) < 0) return fail("PACKET_FANOUT");
    }
    cursor_ = 0;
    err_.clear();
    return Result<void>::success();
}

Result<void> TpacketV3Ring::attach(void* mem, uint32_t blockSize, uint32_t numBlocks) {
    close();
    if (!mem || !blockSize || !numBlocks)
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT, err_ = "attach: empty ring");
    opts_ = Options{};
    opts_.blockSize = blockSize;
    opts_.numBlocks = numBlocks;
    map_ = mem;
    owned_ = false;
    cursor_ = 0;
    return Result<void>::success();
}

void TpacketV3Ring::close() {
    if (map_ && owned_) munmap(map_, bytes());
    owned_ = false;
    map_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
}

bool TpacketV3Ring::waitReady(std::chrono::milliseconds timeout) {
    if (!map_) return false;
    const auto* bd = reinterpret_cast<const tpacket_block_desc*>(static_cast<const uint8_t*>(map_) +
                                                                 (uint64_t)cursor_ * opts_.blockSize);
    if (__atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE) & TP_STATUS_USER) return true;
    if (fd_ < 0) return false;   // attached image: nothing will arrive
    pollfd p{fd_, POLLIN | POLLERR, 0};
    (void)poll(&p, 1, (int)timeout.count());
    return __atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE) & TP_STATUS_USER;
}

Result<uint32_t> TpacketV3Ring::take(bt_ctx* ctx, uint32_t maxBlocks, bt_pkt_desc* desc, uint32_t cap,
                                     uint32_t* n) {
    const bt_tpv3_ring r = ring();
    uint32_t blocks = 0;
    *n = 0;
    if (bt_ring_walk_tpv3(ctx, &r, cursor_, maxBlocks, desc, cap, n, &blocks) != BT_OK)
        return Result<uint32_t>::error(ErrorCode::INVALID_ARGUMENT, err_ = bt_last_error());
    return Result<uint32_t>::success(blocks);
}

Result<uint32_t> TpacketV3Ring::takeGathered(bt_ctx* ctx, uint32_t maxBlocks, uint8_t* slots, bt_pkt_desc* slotDesc,
                                             bt_pkt_desc* ringDesc, uint32_t cap, uint32_t* n, bool lean) {
    const bt_tpv3_ring r = ring();
    uint32_t blocks = 0;
    *n = 0;
    auto gather = lean ? bt_ring_gather_lean_tpv3 : bt_ring_gather_dense_tpv3;
    if (gather(ctx, &r, cursor_, maxBlocks, slots, slotDesc, ringDesc, cap, n, &blocks) != BT_OK)
        return Result<uint32_t>::error(ErrorCode::INVALID_ARGUMENT, err_ = bt_last_error());
    return Result<uint32_t>::success(blocks);
}

void TpacketV3Ring::release(uint32_t blocks) {
    if (!blocks) return;
    const bt_tpv3_ring r = ring();
    (void)bt_ring_release_tpv3(&r, cursor_, blocks);
    cursor_ = (cursor_ + blocks) % opts_.numBlocks;
}

TpacketV3Ring::Stats TpacketV3Ring::statistics() {
    Stats s;
    tpacket_stats_v3 st{};
    socklen_t l = sizeof(st);
    if (fd_ >= 0 && getsockopt(fd_, SOL_PACKET, PACKET_STATISTICS, &st, &l) == 0) {   // read-and-clear
        s.packets = st.tp_packets;
        s.drops = st.tp_drops;
        s.freezes = st.tp_freeze_q_cnt;
    }
    return s;
}

}  // namespace gpu
}  // namespace beatrice
