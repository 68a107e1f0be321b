// GpuCapture.hpp — capture-ring ingest in front of the MI355X parse+filter stage
// ("AF_PACKET TPACKET_V3 ring ingest replacing per-packet recv() +
// copy"; the north star: the path starts and ends in host ring buffers).
//
//   GpuAfPacketBackend  drop-in for the reference's AF_PacketBackend
//                       (include/beatrice/AF_PacketBackend.hpp, src/AF_PacketBackend.cpp):
//                       the same ICaptureBackend interface and queue / callback
//                       semantics, fed from a TPACKET_V3 ring (whole blocks per wake-up)
//                       instead of one recv() + copy + 100 us sleep per packet.
//   GpuTpacketStage     the zero-copy path: the ring is registered with the GPU once,
//                       ready blocks become descriptors (bt_ring_walk_tpv3) and the
//                       parse+filter kernels read the frames in place over PCIe; the
//                       decisions / verdict bitmap / records land in registered host
//                       memory. Nothing is copied on the host.
//
// Both live in libbeatrice_gpu_capture.so; Packet's out-of-line members resolve
// against beatrice_core in the process that loads it, as for the plugin.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <new>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "GpuPacketFilter.hpp"
#include "TpacketRing.hpp"
#include "beatrice/ICaptureBackend.hpp"

namespace beatrice {

namespace gpu {

// Page-aligned, page-padded storage for the buffers a stage registers with the devices:
// registration is in whole pages (include/beatrice_gpu.h, bt_host_register), so two such
// buffers must never share a page, as std::vector's heap blocks can.
template <class T>
struct PageAllocator {
    using value_type = T;
    PageAllocator() = default;
    template <class U>
    PageAllocator(const PageAllocator<U>&) {}
    T* allocate(size_t n) {
        const size_t bytes = std::max<size_t>((n * sizeof(T) + 4095) & ~size_t(4095), 4096);
        void* p = nullptr;
        if (posix_memalign(&p, 4096, bytes) != 0) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { free(p); }
    template <class U>
    bool operator==(const PageAllocator<U>&) const { return true; }
    template <class U>
    bool operator!=(const PageAllocator<U>&) const { return false; }
};
template <class T>
using PageVector = std::vector<T, PageAllocator<T>>;

class GpuAfPacketBackend : public ICaptureBackend {
public:
    GpuAfPacketBackend();
    ~GpuAfPacketBackend() override;

    Result<void> initialize(const Config& config) override;
    Result<void> start() override;
    Result<void> stop() override;
    bool isRunning() const noexcept override;
    std::optional<Packet> nextPacket(std::chrono::milliseconds timeout = std::chrono::milliseconds(1000)) override;
    std::vector<Packet> getPackets(size_t maxPackets = 64,
                                   std::chrono::milliseconds timeout = std::chrono::milliseconds(1000)) override;
    void setPacketCallback(std::function<void(Packet)> callback) override;
    void removePacketCallback() override;
    Statistics getStatistics() const override;
    void resetStatistics() override;
    std::string getName() const override;
    std::string getVersion() const override;
    std::vector<std::string> getSupportedFeatures() const override;
    bool isFeatureSupported(const std::string& feature) const override;
    Config getConfig() const override;
    Result<void> updateConfig(const Config& config) override;
    std::string getLastError() const override;
    bool isHealthy() const override;
    Result<void> healthCheck() override;

    bool isZeroCopyEnabled() const override;
    bool isDMAAccessEnabled() const override;
    Result<void> enableZeroCopy(bool enabled) override;
    Result<void> enableDMAAccess(bool enabled, const std::string& device = "") override;
    Result<void> setDMABufferSize(size_t size) override;
    size_t getDMABufferSize() const override;
    std::string getDMADevice() const override;
    Result<void> allocateDMABuffers(size_t count) override;
    Result<void> freeDMABuffers() override;

    // ring geometry used by initialize(): the reference's buffer budget
    // (bufferSize x numBuffers), in blocks of blockBytes
    static TpacketV3Ring::Options ringOptions(const Config& config);

private:
    void captureLoop();
    void setError(const std::string& e);

    Config config_;
    bool initialized_ = false;
    std::atomic<bool> running_{false};
    TpacketV3Ring ring_;
    std::thread thread_;
    std::queue<Packet> queue_;
    std::mutex queueMutex_;
    std::condition_variable queueCv_;
    std::function<void(Packet)> callback_;
    std::mutex callbackMutex_;
    Statistics stats_;
    mutable std::mutex statsMutex_;
    std::string lastError_;
    mutable std::mutex errorMutex_;
    bool zeroCopy_ = true, dma_ = false;
    std::string dmaDevice_;
    size_t dmaBufferSize_ = 0;
};

class GpuTpacketStage {
public:
    struct Options {
        uint32_t maxBlocks = 64;        // blocks per batch (upper bound; more blocks = more
                                        // frame chains walked in parallel)
        uint32_t maxPackets = 1u << 20; // descriptors per batch (upper bound)
        bool records = false;           // also write bt_rec records (device tiled layout)
        // Header gather (bt_ring_gather_dense_tpv3): the walker packs each frame's header
        // prefix into registered slots and the kernels read those instead of the ring over
        // PCIe. inPlaceEvery = k > 0: every k-th batch is still read in
        // place, sharing the work between the host's copy and the GPU's PCIe reads. The
        // default since round 6 (gather, every other batch in place, lean prefixes for
        // filter-only batches): bench.py's ring entry, C2 / C3 frames, 516 / 429 Mpps against
        // 328 / 299 reading every batch in place (profiles/r06/bench_default_a.json).
        bool gather = true;
        uint32_t inPlaceEvery = 2;
        // Gathered batches that ask for no records pack only frame bytes 12..43
        // (bt_ring_gather_lean_tpv3, BT_BATCH_LEAN): the ring's e2e verdicts +17..45 % over the
        // full prefixes with inPlaceEvery = 2. false: the full prefixes.
        bool lean = true;
    };
    // One batch of ring blocks, owned by the caller until release().
    struct Batch {
        uint32_t n = 0, blocks = 0;
        const bt_pkt_desc* desc = nullptr;   // ring-relative
        const uint8_t* decide = nullptr;     // (code << 6) | slot, host-side slots resolved
        const uint64_t* verdict = nullptr;   // bit i = packet i passed
        const void* records = nullptr;       // tiled (include/beatrice_gpu.h); records == true only
        std::vector<uint32_t> pass;          // ascending
        bool gathered = false;               // the kernels read packed header prefixes
    };

    // The filter supplies the devices and the compiled program: the ring and the stage's
    // buffers are registered with every device of the filter, and each batch is split across
    // them, every device reading its range of the ring over its own PCIe link. The ring must
    // stay open for the stage's lifetime. Throws std::runtime_error when the ring cannot be
    // mapped into the devices.
    GpuTpacketStage(GpuPacketFilter& filter, TpacketV3Ring& ring, Options opts);
    GpuTpacketStage(GpuPacketFilter& filter, TpacketV3Ring& ring) : GpuTpacketStage(filter, ring, Options()) {}
    ~GpuTpacketStage();
    GpuTpacketStage(const GpuTpacketStage&) = delete;
    GpuTpacketStage& operator=(const GpuTpacketStage&) = delete;

    // Waits up to `timeout` for a ready block, takes the ready blocks from the ring
    // cursor and runs them through the GPU. An empty batch (n == 0, blocks == 0) means
    // nothing arrived. Throws what GpuPacketFilter::applyFilters throws.
    const Batch& poll(std::chrono::milliseconds timeout);
    // Hands the last batch's blocks back to the kernel.
    void release();

    const uint8_t* frame(uint32_t i) const { return ringBase_ + BT_DESC_OFF(batch_.desc[i]); }
    uint32_t length(uint32_t i) const { return BT_DESC_LEN(batch_.desc[i]); }
    bt_rec record(uint32_t i) const;

private:
    GpuPacketFilter& filter_;
    TpacketV3Ring& ring_;
    Options opts_;
    uint8_t* ringBase_ = nullptr;
    // registered host buffers: descriptors in, decisions / verdicts / records out
    PageVector<bt_pkt_desc> desc_;
    PageVector<uint8_t> decide_;
    PageVector<uint64_t> verdict_;
    PageVector<uint8_t> records_;
    // header gather: packed prefixes and their descriptors (registered)
    PageVector<uint8_t> slots_;
    PageVector<bt_pkt_desc> slotDesc_;
    std::vector<void*> registered_;   // with the filter's group
    uint64_t polls_ = 0;
    Batch batch_;
};

}  // namespace gpu
}  // namespace beatrice
