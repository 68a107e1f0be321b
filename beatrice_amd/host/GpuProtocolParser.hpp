// GpuProtocolParser.hpp — batch front end of the MI355X parse stage for callers of
// beatrice::parser::ProtocolParser (reference include/parser/ProtocolParser.hpp:67).
//
// parseBatch() runs the whole layer walk (Ethernet, up to two VLAN tags, IPv4/IPv6,
// TCP/UDP/ICMP — DESIGN.md "R-WALK") for every packet on the GPU and keeps the 96-B
// bt_rec per packet. layer(i, k) materialises, on demand, the reference ParseResult of
// the k-th walked layer of packet i: identical to
//     ProtocolParser(cfg with enablePerformanceMetrics=false)
//         .parsePacket(std::vector<uint8_t>(frame + offset, frame + len), name)
// in every member except the wall-clock timings (parseTime / totalParseTime = 0).
//
// detect(i) / detectMultiple(i) / is(i, BT_IS_*) answer the reference's static
// ProtocolDetector (include/parser/ProtocolRegistry.hpp:83-108) for the whole frame
// from the record's detector column, which the same kernel pass fills: equal to
// ProtocolDetector::detectProtocol(frame) etc. except `confidence` of a non-Ethernet
// frame, which the reference leaves uninitialised (ProtocolRegistry.cpp:355) and this
// layer reports as 0.0.
//
// User-defined protocols (the rest of include/parser/ProtocolParser.hpp:56-93):
// registerProtocol / unregisterProtocol / hasProtocol / getSupportedProtocols,
// parsePacket(packet, name), parsePacket(packet, ProtocolDefinition),
// parsePacketMultipleProtocols and validatePacket, with the reference's results, stats
// and protocol iteration order; and the batch forms parseBatch(packets, name | definition)
// / parseBatchMultipleProtocols, whose GpuFieldBatch holds the GPU's extracted columns
// (bt_extract, beatrice_amd/csrc/bt_extract.hip) and materialises each packet's
// ParseResult on demand. Differences, all where the reference is undefined: a TIMESTAMP
// that localtime() cannot convert formats as "" (the reference crashes in put_time); a
// BOOLEAN field of length 0 throws std::invalid_argument (the reference reads past an
// empty vector); parsePacket(packet, "") with no protocol registered throws
// std::out_of_range (the reference indexes an empty vector); a failed first parse does not
// raise SIGFPE in the stats (the reference divides by successfulParses).
#pragma once

#include <atomic>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <type_traits>
#include <utility>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "beatrice/Packet.hpp"
#include "beatrice_gpu.h"
#include "parser/ParserResult.hpp"
#include "parser/ProtocolParser.hpp"
#include "parser/ProtocolRegistry.hpp"

namespace beatrice {
namespace gpu {

// std::allocator that leaves trivially constructible elements uninitialised on resize():
// the records are written by the device pass right after, so zeroing them first only
// doubled the host's memory traffic.
template <class T>
struct UninitAllocator : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = UninitAllocator<U>;
    };
    UninitAllocator() = default;
    template <class U>
    UninitAllocator(const UninitAllocator<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible_v<U>) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... Args>
    void construct(U* p, Args&&... args) {
        ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
    }
};

struct WalkedLayer {
    std::string name;   // "ethernet", "vlan", "ipv4", "ipv6", "tcp", "udp", "icmp"
    size_t offset;      // slice start in the frame
    int tag;            // VLAN tag index (0/1), -1 otherwise
};

namespace detail {
// What a destroyed GpuParsedBatch hands back to the parser that made it: its arrays, whose
// pages are already in, for the next parseBatch (a fresh 96-B record per packet faulted in
// during every call, and each packet's reference released on one thread at destruction, were
// most of a large call's time); the references are released on the parser's host threads
// while the parser lives (ctx is null once it is gone).
struct BatchStore {
    using Recs = std::vector<bt_rec, UninitAllocator<bt_rec>>;
    using Bytes = std::vector<uint8_t, UninitAllocator<uint8_t>>;
    using Words = std::vector<uint64_t, UninitAllocator<uint64_t>>;
    using Keep = std::vector<std::shared_ptr<const uint8_t[]>>;
    static constexpr size_t kSets = 2;   // sets of arrays kept for reuse
    std::mutex mu;
    bt_ctx* ctx = nullptr;
    std::vector<Recs> recs;
    std::vector<std::vector<const uint8_t*>> frames;
    std::vector<std::vector<uint32_t>> lens;
    std::vector<Keep> keep;
    std::vector<Bytes> bytes;   // a field batch's status and image columns
    std::vector<Words> words;   // its value columns
    BatchStore() {   // a destructor hands arrays back without allocating
        recs.reserve(kSets);
        frames.reserve(kSets);
        lens.reserve(kSets);
        keep.reserve(kSets);
        bytes.reserve(2 * kSets);
        words.reserve(kSets);
    }
    // A destroyed batch's arrays: the frames' references released (on the parser's host
    // threads for a large batch while the parser lives), the arrays kept for reuse.
    void give(std::vector<const uint8_t*>& f, std::vector<uint32_t>& l, Keep& k);
};
}  // namespace detail

class GpuParsedBatch {
public:
    GpuParsedBatch() = default;
    GpuParsedBatch(const GpuParsedBatch&) = default;
    GpuParsedBatch(GpuParsedBatch&&) noexcept = default;
    GpuParsedBatch& operator=(const GpuParsedBatch&) = default;
    GpuParsedBatch& operator=(GpuParsedBatch&&) noexcept = default;
    ~GpuParsedBatch();

    size_t size() const { return recs_.size(); }
    const bt_rec& record(size_t i) const { return recs_[i]; }
    std::vector<WalkedLayer> layers(size_t i) const;
    parser::ParseResult layer(size_t i, size_t k) const;
    // first walked layer called `name` (PROTOCOL_NOT_FOUND result when absent)
    parser::ParseResult layer(size_t i, const std::string& name) const;

    using DetectionResult = parser::ProtocolDetector::DetectionResult;
    DetectionResult detect(size_t i) const;                     // detectProtocol (:353-388)
    std::vector<DetectionResult> detectMultiple(size_t i) const; // detectMultipleProtocols (:390-416)
    // isEthernet .. isDNS as BT_IS_* bits; isARP as BT_IS2_ARP via isARP()
    bool is(size_t i, uint32_t bt_is_bit) const { return (recs_.at(i).detect_is & bt_is_bit) != 0; }
    bool isARP(size_t i) const { return (recs_.at(i).detect_is2 & BT_IS2_ARP) != 0; }

    // Text of layer(i, k).toJsonString() / toXmlString() / toCsvString() /
    // toHumanReadableString() (fmt = BT_FMT_*) for every walked layer, each followed by
    // '\n', straight from the records (bt_format_records): packet i, or the whole batch
    // on the context's host threads.
    std::string format(size_t i, uint32_t fmt) const;
    std::string format(uint32_t fmt) const;

private:
    friend class GpuProtocolParser;
    std::vector<bt_rec, UninitAllocator<bt_rec>> recs_;
    std::vector<const uint8_t*> frames_;
    std::vector<uint32_t> lens_;
    std::vector<std::shared_ptr<const uint8_t[]>> keep_;   // the frames of a vector<Packet> batch
    bt_ctx* ctx_ = nullptr;      // host pool for format(); owned by the GpuProtocolParser
    std::shared_ptr<detail::BatchStore> store_;   // where the arrays go when the batch is destroyed
};

// One user protocol over a batch: the GPU's columns (status, extractValue<T> bits per
// numeric field, the [0, span) bytes of each packet) and ParseResult on demand.
class GpuFieldBatch {
public:
    GpuFieldBatch() = default;
    GpuFieldBatch(const GpuFieldBatch&) = default;
    GpuFieldBatch(GpuFieldBatch&&) noexcept = default;
    GpuFieldBatch& operator=(const GpuFieldBatch&) = default;
    GpuFieldBatch& operator=(GpuFieldBatch&&) noexcept = default;
    ~GpuFieldBatch();

    size_t size() const { return lens_.size(); }
    const parser::ProtocolDefinition& protocol() const {
        static const parser::ProtocolDefinition kNone{};   // a default-constructed batch
        return def_ ? *def_ : kNone;
    }
    parser::ParseStatus status(size_t i) const { return static_cast<parser::ParseStatus>(status_.at(i)); }
    bool isSuccess(size_t i) const { return status_.at(i) == 0; }
    // extractValue<T> bits of field k (0 for byte-typed fields and packets that did not parse)
    uint64_t raw(size_t i, size_t k) const { return values_.at(k * size() + i); }
    template <class T>
    T value(size_t i, size_t k) const {
        const uint64_t b = raw(i, k);
        T v;
        std::memcpy(&v, &b, sizeof(T));
        return v;
    }
    // the field's bytes (empty when the packet did not parse)
    std::vector<uint8_t> bytes(size_t i, size_t k) const;
    // == ProtocolParser(config).parsePacket(packet_i, protocol()) but for wall-clock times (0)
    parser::ParseResult result(size_t i) const;

private:
    friend class GpuProtocolParser;
    std::shared_ptr<const parser::ProtocolDefinition> def_;   // the registered definition, shared
    bool validate_ = true;
    uint64_t span_ = 0;
    detail::BatchStore::Bytes status_;
    detail::BatchStore::Words values_;   // field-major, column stride size()
    detail::BatchStore::Bytes image_;    // size() x span_
    std::vector<const uint8_t*> frames_;
    std::vector<uint32_t> lens_;
    std::vector<std::shared_ptr<const uint8_t[]>> keep_;
    std::shared_ptr<detail::BatchStore> store_;   // where the arrays go when the batch is destroyed
};

class GpuProtocolParser {
public:
    explicit GpuProtocolParser(int device = 0, const bt_opts* opts = nullptr);
    explicit GpuProtocolParser(const parser::ProtocolParser::ParserConfig& config, int device = 0,
                               const bt_opts* opts = nullptr);
    ~GpuProtocolParser();
    GpuProtocolParser(const GpuProtocolParser&) = delete;
    GpuProtocolParser& operator=(const GpuProtocolParser&) = delete;

    // ---- factories (ProtocolParser.hpp:56-58, ProtocolParser.cpp:10-29) ----
    static std::unique_ptr<GpuProtocolParser> create(
        const parser::ProtocolParser::ParserConfig& config = parser::ProtocolParser::ParserConfig{}, int device = 0,
        const bt_opts* opts = nullptr);
    // Registers each named protocol the registry holds, skipping the others, as the
    // reference does with its ProtocolRegistry singleton: pass
    // parser::ProtocolRegistry::getInstance() (or anything with hasProtocol / getProtocol).
    template <class Registry>
    static std::unique_ptr<GpuProtocolParser> createWithProtocols(const std::vector<std::string>& protocolNames,
                                                                  const parser::ProtocolParser::ParserConfig& config,
                                                                  Registry& registry, int device = 0,
                                                                  const bt_opts* opts = nullptr) {
        auto p = create(config, device, opts);
        for (const auto& name : protocolNames)
            if (registry.hasProtocol(name))
                if (const parser::ProtocolDefinition* def = registry.getProtocol(name)) p->registerProtocol(*def);
        return p;
    }

    // ---- builtin layer walk (Ethernet / VLAN / IPv4 / IPv6 / TCP / UDP / ICMP) ----
    GpuParsedBatch parseBatch(const std::vector<Packet>& packets);
    // borrows `base` for the lifetime of the returned batch
    GpuParsedBatch parseBatch(const uint8_t* base, const bt_pkt_desc* desc, uint32_t n);

    // ---- user-defined protocols (ProtocolParser.hpp:63-72; ProtocolParser.cpp:41-143) ----
    bool registerProtocol(const parser::ProtocolDefinition& protocol);
    bool unregisterProtocol(const std::string& name);
    bool hasProtocol(const std::string& name) const;
    std::vector<std::string> getSupportedProtocols() const;
    parser::ParseResult parsePacket(const std::vector<uint8_t>& packet, const std::string& protocolName = "");
    parser::ParseResult parsePacket(const std::vector<uint8_t>& packet, const parser::ProtocolDefinition& protocol);
    std::vector<parser::ParseResult> parsePacketMultipleProtocols(const std::vector<uint8_t>& packet);
    bool validatePacket(const std::vector<uint8_t>& packet, const std::string& protocolName);
    bool validatePacket(const std::vector<uint8_t>& packet, const parser::ProtocolDefinition& protocol);
    void setConfig(const parser::ProtocolParser::ParserConfig& config);
    const parser::ProtocolParser::ParserConfig& getConfig() const { return config_; }
    // parsePacket / parsePacketMultipleProtocols and batches of fewer than hostBatchBelow()
    // packets extract on the calling thread (bt_extract_host: the kernel's extractValue<T>
    // decode) instead of paying a device round trip (~0.1 ms per bt_extract call). Default
    // BEATRICE_GPU_HOST_BELOW, else kHostBelowDefault; 0 sends every call to the device.
    static constexpr size_t kHostBelowDefault = 512;
    void setHostBatchBelow(size_t n) { hostBelow_ = n; }
    size_t hostBatchBelow() const { return hostBelow_; }

    // ---- text and bytes of a ParseResult (ProtocolParser.hpp:74-75, 84-89) ----
    // formatPacket: the reference's ParseResult::toJsonString / toXmlString / toCsvString /
    // toHumanReadableString for "json" / "xml" / "csv" / "human", json for anything else,
    // for any ParseResult (a GpuParsedBatch layer, a GpuFieldBatch result, one of the
    // caller's). serializePacket: its rawData.
    std::string formatPacket(const parser::ParseResult& result, const std::string& format = "json");
    std::vector<uint8_t> serializePacket(const parser::ParseResult& result);
    std::vector<std::string> getSupportedFormats() const;
    // false unless the protocol is registered; kept, and (as in the reference) not called
    bool addCustomValidator(const std::string& protocolName,
                            std::function<bool(const std::vector<uint8_t>&, const parser::ParseResult&)> validator);
    bool addCustomFormatter(const std::string& protocolName,
                            std::function<std::string(const parser::ParseResult&)> formatter);
    void clearCache() {}   // the GPU path keeps no field cache
    void enableProfiling(bool enable) { profiling_ = enable; }
    bool isProfilingEnabled() const { return profiling_; }
    std::string bytesToHex(const std::vector<uint8_t>& bytes) const;
    std::string formatMacAddress(const std::vector<uint8_t>& bytes) const;
    std::string formatIPv4Address(const std::vector<uint8_t>& bytes) const;
    std::string formatIPv6Address(const std::vector<uint8_t>& bytes) const;
    std::string formatTimestamp(uint64_t timestamp) const;

    // batch forms: one GPU pass per protocol over the whole batch
    GpuFieldBatch parseBatch(const std::vector<Packet>& packets, const parser::ProtocolDefinition& protocol);
    // PROTOCOL_NOT_FOUND has no batch form: throws std::out_of_range for an unknown name
    GpuFieldBatch parseBatch(const std::vector<Packet>& packets, const std::string& protocolName);
    // one batch per registered protocol, in the order parsePacketMultipleProtocols uses
    std::vector<GpuFieldBatch> parseBatchMultipleProtocols(const std::vector<Packet>& packets);

    // ProtocolParser::getStats / resetStats (include/parser/ProtocolParser.hpp:40-54,
    // src/parser/ProtocolParser.cpp:174-182, updateStats :482-506): every walked layer of
    // every batch counts as one parsePacket call, with the same totalPacketsParsed /
    // successfulParses / failedParses / protocolUsageCount. Times are the batch's wall
    // time spread evenly over its layers, in whole microseconds as the reference keeps
    // them. The reference divides by successfulParses and raises SIGFPE when the first
    // parse on an instance fails; here the averages stay 0 until a parse succeeds.
    parser::ProtocolParser::ParserStats getStats() const;
    void resetStats();

private:
    template <class Batch>
    static void adopt(bt_ctx* ctx, const std::vector<Packet>& packets, Batch& b);
    void newBatch(GpuParsedBatch& b);   // arrays from the store, ready for reuse
    void newBatch(GpuFieldBatch& b);
    void run(GpuParsedBatch& b);
    void extract(GpuFieldBatch& b);
    using DefPtr = std::shared_ptr<const parser::ProtocolDefinition>;
    GpuFieldBatch batchOf(const std::vector<Packet>& packets, DefPtr def);
    parser::ParseResult parseOne(const std::vector<uint8_t>& packet, DefPtr def);
    DefPtr findProtocol(const std::string& name) const;   // nullptr when not registered
    std::vector<DefPtr> allProtocols() const;             // the reference's iteration order
    void countParses(const std::string& protocol, uint64_t ok, uint64_t bad, double us);
    bt_ctx* ctx_ = nullptr;
    std::shared_ptr<detail::BatchStore> store_ = std::make_shared<detail::BatchStore>();
    size_t hostBelow_ = kHostBelowDefault;
    parser::ProtocolParser::ParserConfig config_;
    // as the reference's protocols_; each definition immutable and shared, so a call takes a
    // reference under the lock instead of copying the field table (parsePacket copied it twice)
    std::unordered_map<std::string, DefPtr> protocols_;
    std::unordered_map<std::string, std::function<bool(const std::vector<uint8_t>&, const parser::ParseResult&)>>
        customValidators_;
    std::unordered_map<std::string, std::function<std::string(const parser::ParseResult&)>> customFormatters_;
    std::atomic<bool> profiling_{false};
    mutable std::shared_mutex protocols_mu_;
    mutable std::mutex stats_mu_;
    parser::ProtocolParser::ParserStats stats_;
    double time_carry_us_ = 0.0;   // sub-microsecond remainder of the amortised time
};

// ParserBuilder (include/parser/ProtocolParser.hpp:141-166) building a GpuProtocolParser.
class GpuParserBuilder {
public:
    GpuParserBuilder& withValidation(bool enable);
    GpuParserBuilder& withChecksumValidation(bool enable);
    GpuParserBuilder& withFieldConstraints(bool enable);
    GpuParserBuilder& withCustomValidators(bool enable);
    GpuParserBuilder& withPerformanceMetrics(bool enable);
    GpuParserBuilder& withFieldCaching(bool enable);
    GpuParserBuilder& withMaxFieldCacheSize(size_t size);
    GpuParserBuilder& withMaxValidationErrors(size_t max);
    GpuParserBuilder& withMaxParseTime(std::chrono::microseconds time);
    GpuParserBuilder& withErrorCallback(std::function<void(const std::string&)> callback);
    GpuParserBuilder& withWarningCallback(std::function<void(const std::string&)> callback);
    GpuParserBuilder& withInfoCallback(std::function<void(const std::string&)> callback);
    GpuParserBuilder& withProtocol(const parser::ProtocolDefinition& protocol);
    GpuParserBuilder& withProtocols(const std::vector<parser::ProtocolDefinition>& protocols);
    // every protocol the registry holds, in its iteration order (ProtocolParser.cpp:716-728):
    // pass parser::ProtocolRegistry::getInstance()
    template <class Registry>
    GpuParserBuilder& withBuiltinProtocols(Registry& registry) {
        for (const auto& name : registry.getRegisteredProtocols())
            if (const parser::ProtocolDefinition* def = registry.getProtocol(name)) protocols_.push_back(*def);
        return *this;
    }
    std::unique_ptr<GpuProtocolParser> build(int device = 0, const bt_opts* opts = nullptr);

private:
    parser::ProtocolParser::ParserConfig config_;
    std::vector<parser::ProtocolDefinition> protocols_;
};

}  // namespace gpu
}  // namespace beatrice
