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
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "beatrice/Packet.hpp"
#include "beatrice_gpu.h"
#include "parser/ParserResult.hpp"
#include "parser/ProtocolParser.hpp"
#include "parser/ProtocolRegistry.hpp"

namespace beatrice {
namespace gpu {

struct WalkedLayer {
    std::string name;   // "ethernet", "vlan", "ipv4", "ipv6", "tcp", "udp", "icmp"
    size_t offset;      // slice start in the frame
    int tag;            // VLAN tag index (0/1), -1 otherwise
};

class GpuParsedBatch {
public:
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
    std::vector<bt_rec> recs_;
    std::vector<const uint8_t*> frames_;
    std::vector<uint32_t> lens_;
    std::vector<Packet> keep_;   // owns the frames of a vector<Packet> batch
    bt_ctx* ctx_ = nullptr;      // host pool for format(); owned by the GpuProtocolParser
};

class GpuProtocolParser {
public:
    explicit GpuProtocolParser(int device = 0, const bt_opts* opts = nullptr);
    ~GpuProtocolParser();
    GpuProtocolParser(const GpuProtocolParser&) = delete;
    GpuProtocolParser& operator=(const GpuProtocolParser&) = delete;

    GpuParsedBatch parseBatch(const std::vector<Packet>& packets);
    // borrows `base` for the lifetime of the returned batch
    GpuParsedBatch parseBatch(const uint8_t* base, const bt_pkt_desc* desc, uint32_t n);

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
    void run(GpuParsedBatch& b);
    bt_ctx* ctx_ = nullptr;
    mutable std::mutex stats_mu_;
    parser::ProtocolParser::ParserStats stats_;
    double time_carry_us_ = 0.0;   // sub-microsecond remainder of the amortised time
};

}  // namespace gpu
}  // namespace beatrice
