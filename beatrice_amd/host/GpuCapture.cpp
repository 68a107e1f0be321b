// GpuCapture.cpp — see GpuCapture.hpp.
#include "GpuCapture.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace beatrice {
namespace gpu {

namespace {
constexpr uint32_t kBlockBytes = 1u << 20;   // 1 MiB blocks: any frame <= 65535 B fits whole
constexpr uint32_t kMinBlocks = 4;
}  // namespace

// ---------------------------------------------------------------------------------
// GpuAfPacketBackend
// ---------------------------------------------------------------------------------

GpuAfPacketBackend::GpuAfPacketBackend() = default;

GpuAfPacketBackend::~GpuAfPacketBackend() {
    (void)stop();
    ring_.close();
}

TpacketV3Ring::Options GpuAfPacketBackend::ringOptions(const Config& c) {
    TpacketV3Ring::Options o;
    o.interface = c.interface;
    o.blockSize = kBlockBytes;
    const uint64_t budget = (uint64_t)c.bufferSize * c.numBuffers;
    o.numBlocks = (uint32_t)std::max<uint64_t>(kMinBlocks, (budget + kBlockBytes - 1) / kBlockBytes);
    o.retireTimeoutMs = 2;
    o.promiscuous = c.promiscuous;
    return o;
}

Result<void> GpuAfPacketBackend::initialize(const Config& config) {   // reference :47-73
    if (initialized_) return Result<void>::success();
    config_ = config;
    if (config_.interface.empty() || config_.interface.length() >= 16)   // validateInterface :255-259
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Invalid interface: " + config_.interface);
    auto r = ring_.open(ringOptions(config_));
    if (r.isError()) {
        setError(ring_.lastError());
        const std::string& e = ring_.lastError();
        if (e.rfind("Failed to create AF_PACKET socket", 0) == 0)
            return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "Failed to create AF_PACKET socket");
        if (e.rfind("Failed to get interface index", 0) == 0 || e.rfind("Failed to bind", 0) == 0)
            return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "Failed to bind to interface");
        return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "Failed to set socket options");
    }
    initialized_ = true;
    return Result<void>::success();
}

Result<void> GpuAfPacketBackend::start() {   // :75-88
    if (!initialized_)
        return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "AF_PACKET backend not initialized");
    if (running_) return Result<void>::success();
    running_ = true;
    thread_ = std::thread(&GpuAfPacketBackend::captureLoop, this);
    return Result<void>::success();
}

Result<void> GpuAfPacketBackend::stop() {   // :90-103
    if (!running_) return Result<void>::success();
    running_ = false;
    queueCv_.notify_all();
    if (thread_.joinable()) thread_.join();
    return Result<void>::success();
}

bool GpuAfPacketBackend::isRunning() const noexcept { return running_; }

void GpuAfPacketBackend::captureLoop() {
    // One wake-up per ready block run instead of one recv() + 100 us sleep per packet
    // (reference :318-363). Each frame is still copied into its own Packet, as the
    // queue / callback contract hands Packets out past the block's lifetime.
    std::vector<bt_pkt_desc> desc;
    const bt_tpv3_ring geom = ring_.ring();
    const uint8_t* base = static_cast<const uint8_t*>(geom.base);
    while (running_) {
        if (!ring_.waitReady(std::chrono::milliseconds(100))) continue;
        const uint32_t cap = (uint32_t)(geom.block_size / 96 + 1) * geom.n_blocks;
        if (desc.size() < cap) desc.resize(cap);
        uint32_t n = 0;
        auto taken = ring_.take(nullptr, geom.n_blocks, desc.data(), cap, &n);
        if (taken.isError()) {
            setError("Error reading from ring: " + taken.getErrorMessage());
            break;
        }
        std::vector<Packet> batch;
        batch.reserve(n);
        uint64_t bytes = 0;
        const auto now = std::chrono::steady_clock::now();
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t len = BT_DESC_LEN(desc[i]);
            std::shared_ptr<uint8_t[]> data(new uint8_t[len]);
            std::memcpy(data.get(), base + BT_DESC_OFF(desc[i]), len);
            batch.emplace_back(data, len, now);
            bytes += len;
        }
        ring_.release(taken.getValue());
        const TpacketV3Ring::Stats ks = ring_.statistics();
        {
            std::lock_guard<std::mutex> lock(statsMutex_);
            stats_.packetsCaptured += n;
            stats_.bytesCaptured += bytes;
            stats_.packetsDropped += ks.drops;
            stats_.lastUpdate = now;
        }
        {
            std::lock_guard<std::mutex> lock(queueMutex_);
            for (const Packet& p : batch) queue_.push(p);
        }
        queueCv_.notify_all();
        std::lock_guard<std::mutex> lock(callbackMutex_);
        if (callback_)
            for (const Packet& p : batch) callback_(p);
    }
}

std::optional<Packet> GpuAfPacketBackend::nextPacket(std::chrono::milliseconds timeout) {   // :110-122
    std::unique_lock<std::mutex> lock(queueMutex_);
    if (queueCv_.wait_for(lock, timeout, [this] { return !queue_.empty(); })) {
        Packet p = queue_.front();
        queue_.pop();
        return p;
    }
    return std::nullopt;
}

std::vector<Packet> GpuAfPacketBackend::getPackets(size_t maxPackets, std::chrono::milliseconds timeout) {   // :124-137
    std::vector<Packet> out;
    std::unique_lock<std::mutex> lock(queueMutex_);
    if (queueCv_.wait_for(lock, timeout, [this] { return !queue_.empty(); })) {
        while (!queue_.empty() && out.size() < maxPackets) {
            out.push_back(queue_.front());
            queue_.pop();
        }
    }
    return out;
}

void GpuAfPacketBackend::setPacketCallback(std::function<void(Packet)> callback) {
    std::lock_guard<std::mutex> lock(callbackMutex_);
    callback_ = std::move(callback);
}

void GpuAfPacketBackend::removePacketCallback() {
    std::lock_guard<std::mutex> lock(callbackMutex_);
    callback_ = nullptr;
}

ICaptureBackend::Statistics GpuAfPacketBackend::getStatistics() const {
    std::lock_guard<std::mutex> lock(statsMutex_);
    return stats_;
}

void GpuAfPacketBackend::resetStatistics() {
    std::lock_guard<std::mutex> lock(statsMutex_);
    stats_ = Statistics{};
}

std::string GpuAfPacketBackend::getName() const { return "AF_PACKET Backend"; }
std::string GpuAfPacketBackend::getVersion() const { return "AF_PACKET TPACKET_V3 Backend v1.0.0 (MI355X stage)"; }

std::vector<std::string> GpuAfPacketBackend::getSupportedFeatures() const {
    return {"Raw packet capture", "Promiscuous mode", "Configurable buffer size", "Real-time packet processing",
            "TPACKET_V3 ring", "Zero-copy GPU ingest"};
}

bool GpuAfPacketBackend::isFeatureSupported(const std::string& feature) const {
    const auto f = getSupportedFeatures();
    return std::find(f.begin(), f.end(), feature) != f.end();
}

ICaptureBackend::Config GpuAfPacketBackend::getConfig() const { return config_; }

Result<void> GpuAfPacketBackend::updateConfig(const Config& config) {
    if (running_) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Cannot update config while running");
    config_ = config;
    return Result<void>::success();
}

std::string GpuAfPacketBackend::getLastError() const {
    std::lock_guard<std::mutex> lock(errorMutex_);
    return lastError_;
}

void GpuAfPacketBackend::setError(const std::string& e) {
    std::lock_guard<std::mutex> lock(errorMutex_);
    lastError_ = e;
}

bool GpuAfPacketBackend::isHealthy() const { return initialized_ && ring_.isOpen(); }

Result<void> GpuAfPacketBackend::healthCheck() {
    if (!initialized_) return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "Backend not initialized");
    if (!ring_.isOpen()) return Result<void>::error(ErrorCode::INITIALIZATION_FAILED, "Socket not valid");
    return Result<void>::success();
}

// The ring is shared memory by construction: "zero copy" is always on for the ring
// itself; the DMA-buffer knobs of the interface are kept as settings only.
bool GpuAfPacketBackend::isZeroCopyEnabled() const { return zeroCopy_; }
bool GpuAfPacketBackend::isDMAAccessEnabled() const { return dma_; }

Result<void> GpuAfPacketBackend::enableZeroCopy(bool enabled) {
    if (running_) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Cannot change zero-copy mode while running");
    zeroCopy_ = enabled;
    return Result<void>::success();
}

Result<void> GpuAfPacketBackend::enableDMAAccess(bool enabled, const std::string& device) {
    if (running_) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Cannot change DMA access while running");
    dma_ = enabled && !device.empty();
    dmaDevice_ = dma_ ? device : std::string();
    return Result<void>::success();
}

Result<void> GpuAfPacketBackend::setDMABufferSize(size_t size) {
    if (running_)
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Cannot change DMA buffer size while running");
    dmaBufferSize_ = size ? size : kBlockBytes;
    return Result<void>::success();
}

size_t GpuAfPacketBackend::getDMABufferSize() const { return dmaBufferSize_; }
std::string GpuAfPacketBackend::getDMADevice() const { return dmaDevice_; }

Result<void> GpuAfPacketBackend::allocateDMABuffers(size_t) {
    if (!dma_) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "DMA access not enabled");
    return Result<void>::error(ErrorCode::NOT_IMPLEMENTED,
                               "the TPACKET_V3 ring is the capture buffer; register it with GpuTpacketStage");
}

Result<void> GpuAfPacketBackend::freeDMABuffers() { return Result<void>::success(); }

// ---------------------------------------------------------------------------------
// GpuTpacketStage
// ---------------------------------------------------------------------------------

GpuTpacketStage::GpuTpacketStage(GpuPacketFilter& filter, TpacketV3Ring& ring, Options opts)
    : filter_(filter), ring_(ring), opts_(opts) {
    if (!ring_.isOpen()) throw std::runtime_error("GpuTpacketStage: ring is not open");
    const bt_tpv3_ring g = ring_.ring();
    ringBase_ = static_cast<uint8_t*>(g.base);
    const uint32_t cap = opts_.maxPackets;
    const uint32_t tiles = (cap + 63) / 64;
    desc_.resize(cap);
    decide_.resize((size_t)tiles * 64);
    verdict_.resize(tiles);
    if (opts_.records) records_.resize((size_t)tiles * 64 * BT_REC_BYTES);
    if (opts_.gather) {
        slots_.resize((size_t)cap * BT_PREFIX_SLOT + 64);
        slotDesc_.resize(cap);
    }
    // registered once with every device of the filter: each reads its range of a batch in
    // place over its own PCIe link (bt_group_parse_filter_mapped)
    try {
        for (auto [p, bytes] : {std::pair<void*, size_t>{ringBase_, ring_.bytes()},
                                {desc_.data(), desc_.size() * sizeof(bt_pkt_desc)},
                                {decide_.data(), decide_.size()},
                                {verdict_.data(), verdict_.size() * 8},
                                {records_.data(), records_.size()},
                                {slots_.data(), slots_.size()},
                                {slotDesc_.data(), slotDesc_.size() * sizeof(bt_pkt_desc)}}) {
            if (!p || !bytes) continue;
            filter_.registerHost(p, bytes);
            registered_.push_back(p);
        }
    } catch (...) {
        for (void* p : registered_) (void)bt_group_host_unregister(filter_.group(), p);
        throw;
    }
}

GpuTpacketStage::~GpuTpacketStage() {
    for (void* p : registered_) (void)bt_group_host_unregister(filter_.group(), p);
}

const GpuTpacketStage::Batch& GpuTpacketStage::poll(std::chrono::milliseconds timeout) {
    batch_ = Batch{};
    if (!ring_.waitReady(timeout)) return batch_;
    uint32_t n = 0;
    const bool gathered = opts_.gather && !(opts_.inPlaceEvery && polls_ % opts_.inPlaceEvery == opts_.inPlaceEvery - 1);
    ++polls_;
    const bool lean = gathered && opts_.lean && !opts_.records;
    auto taken = gathered ? ring_.takeGathered(filter_.context(), opts_.maxBlocks, slots_.data(), slotDesc_.data(),
                                               desc_.data(), opts_.maxPackets, &n, lean)
                          : ring_.take(filter_.context(), opts_.maxBlocks, desc_.data(), opts_.maxPackets, &n);
    if (taken.isError()) throw std::runtime_error("GpuTpacketStage: " + taken.getErrorMessage());
    batch_.blocks = taken.getValue();
    if (batch_.blocks == 0)   // a single ready block with more frames than maxPackets
        throw std::runtime_error("GpuTpacketStage: a ring block holds more than maxPackets frames");
    batch_.n = n;
    batch_.desc = desc_.data();
    batch_.decide = decide_.data();
    batch_.verdict = verdict_.data();
    batch_.records = opts_.records ? records_.data() : nullptr;
    batch_.gathered = gathered;
    bt_batch b{};   // host addresses: the filter's group maps them per device
    b.base = gathered ? slots_.data() : ringBase_;
    b.desc = gathered ? slotDesc_.data() : desc_.data();
    b.n = n;
    b.bytes = gathered ? slots_.size() : ring_.bytes();
    b.desc_format = BT_DESC_PACKED;
    b.flags = (gathered ? BT_BATCH_PREFIXES : 0u) | (lean ? BT_BATCH_LEAN : 0u);   // PAYLOAD: on the host, from the frame
    bt_outputs o{};
    o.records = opts_.records ? records_.data() : nullptr;
    o.n_cap = opts_.maxPackets;
    o.verdict = verdict_.data();
    o.decide = decide_.data();
    batch_.pass = filter_.classifyMapped(b, o, [this](uint32_t i) {
        const uint32_t len = length(i);
        std::shared_ptr<uint8_t[]> data(new uint8_t[len]);
        std::memcpy(data.get(), frame(i), len);
        return Packet(data, len);
    });
    return batch_;
}

void GpuTpacketStage::release() {
    ring_.release(batch_.blocks);
    batch_ = Batch{};
}

bt_rec GpuTpacketStage::record(uint32_t i) const {
    bt_rec r;
    if (!opts_.records) throw std::logic_error("GpuTpacketStage: records were not requested");
    bt_record_gather(records_.data(), opts_.maxPackets, i, &r);
    return r;
}

}  // namespace gpu
}  // namespace beatrice
