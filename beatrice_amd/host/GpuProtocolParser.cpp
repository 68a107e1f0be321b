// GpuProtocolParser.cpp — see GpuProtocolParser.hpp. The per-protocol field lists
// (names, order, types) follow the reference builtin tables
// src/parser/ProtocolRegistry.cpp:150-234/289-297; FieldValue contents follow
// src/parser/ProtocolParser.cpp:286-383 (rawHex, formatted addresses) and the
// ParseResult header fields :238-284.
#include "GpuProtocolParser.hpp"

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <type_traits>

namespace beatrice {
namespace gpu {

using parser::FieldValue;
using parser::FieldValueType;
using parser::ParseResult;
using parser::ParseStatus;

namespace {

enum Kind { U8, U16, U32, BYTES, IPV4, IPV6 };

struct Field {
    const char* name;
    Kind kind;
    uint32_t rec_off;   // position in bt_rec
    uint32_t len;       // field length (bytes)
};

struct Table {
    const char* name;
    const char* version;
    uint32_t total;     // ProtocolDefinition::getTotalLength()
    std::vector<Field> fields;
};

const Table kEth{"ethernet", "2.0", 14,
                 {{"destination_mac", BYTES, 0, 6}, {"source_mac", BYTES, 6, 6}, {"ethertype", U16, 12, 2}}};
const Table kVlan{"vlan", "1.0", 4, {{"tpid", U16, 16, 2}, {"tci", U16, 20, 2}}};
const Table kIpv4{"ipv4", "4.0", 20,
                  {{"version", U8, 28, 1}, {"ihl", U8, 29, 1}, {"tos", U8, 30, 1}, {"total_length", U16, 34, 2},
                   {"identification", U16, 36, 2}, {"flags", U16, 38, 2}, {"ttl", U8, 31, 1},
                   {"protocol", U8, 32, 1}, {"checksum", U16, 40, 2}, {"source_ip", IPV4, 44, 4},
                   {"destination_ip", IPV4, 48, 4}}};
const Table kIpv6{"ipv6", "6.0", 40,
                  {{"version_traffic_class_flow_label", U32, 28, 4}, {"payload_length", U16, 32, 2},
                   {"next_header", U8, 34, 1}, {"hop_limit", U8, 35, 1}, {"source_ip", IPV6, 36, 16},
                   {"destination_ip", IPV6, 52, 16}}};
const Table kTcp{"tcp", "1.0", 20,
                 {{"source_port", U16, 68, 2}, {"destination_port", U16, 70, 2}, {"sequence_number", U32, 72, 4},
                  {"acknowledgment_number", U32, 76, 4}, {"data_offset", U8, 80, 1}, {"flags", U8, 81, 1},
                  {"window_size", U16, 82, 2}, {"checksum", U16, 84, 2}, {"urgent_pointer", U16, 86, 2}}};
const Table kUdp{"udp", "1.0", 8,
                 {{"source_port", U16, 68, 2}, {"destination_port", U16, 70, 2}, {"length", U16, 72, 2},
                  {"checksum", U16, 74, 2}}};
const Table kIcmp{"icmp", "1.0", 8,
                  {{"type", U8, 68, 1}, {"code", U8, 69, 1}, {"checksum", U16, 70, 2}, {"identifier", U16, 72, 2},
                   {"sequence_number", U16, 74, 2}}};

std::string hex(const uint8_t* b, size_t n) {   // ProtocolParser::bytesToHex (:591-597)
    static const char* d = "0123456789abcdef";
    std::string s(2 * n, '0');
    for (size_t i = 0; i < n; ++i) {
        s[2 * i] = d[b[i] >> 4];
        s[2 * i + 1] = d[b[i] & 15];
    }
    return s;
}

std::string fmt_ipv4(const uint8_t* b) {        // :610-619
    char buf[16];
    const int n = std::snprintf(buf, sizeof(buf), "%u.%u.%u.%u", b[0], b[1], b[2], b[3]);
    return std::string(buf, (size_t)n);
}

std::string fmt_ipv6(const uint8_t* b) {        // :621-631
    std::stringstream ss;
    for (size_t i = 0; i < 16; i += 2) {
        if (i > 0) ss << ":";
        uint16_t v = (uint16_t)((b[i] << 8) | b[i + 1]);
        ss << std::hex << v;
    }
    return ss.str();
}

FieldValue make_field(const bt_rec& r, const Field& f, uint32_t bias) {
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(&r) + f.rec_off + bias;
    FieldValue v;
    v.valid = true;
    uint8_t wire[16];
    switch (f.kind) {
    case U8:
        v.type = FieldValueType::UINT8;
        v.value = rb[0];
        wire[0] = rb[0];
        break;
    case U16: {
        uint16_t x;
        std::memcpy(&x, rb, 2);
        v.type = FieldValueType::UINT16;
        v.value = x;
        wire[0] = (uint8_t)(x >> 8);
        wire[1] = (uint8_t)x;
        break;
    }
    case U32: {
        uint32_t x;
        std::memcpy(&x, rb, 4);
        v.type = FieldValueType::UINT32;
        v.value = x;
        for (int k = 0; k < 4; ++k) wire[k] = (uint8_t)(x >> (24 - 8 * k));
        break;
    }
    case BYTES:
        v.type = FieldValueType::BYTES;
        v.value = std::vector<uint8_t>(rb, rb + f.len);
        std::memcpy(wire, rb, f.len);
        break;
    case IPV4:
        v.type = FieldValueType::IPV4_ADDRESS;
        v.value = std::vector<uint8_t>(rb, rb + 4);
        v.formatted = fmt_ipv4(rb);
        std::memcpy(wire, rb, 4);
        break;
    case IPV6:
        v.type = FieldValueType::IPV6_ADDRESS;
        v.value = std::vector<uint8_t>(rb, rb + 16);
        v.formatted = fmt_ipv6(rb);
        std::memcpy(wire, rb, 16);
        break;
    }
    v.rawHex = hex(wire, f.len);
    return v;
}



}  // namespace

namespace {

// One walked layer as the record states it (the walk, DESIGN.md R-WALK): its table, slice
// offset, VLAN tag index and `present` / `ok` bit.
struct Walked {
    const Table* table;
    uint32_t offset;
    int tag;
    uint32_t bit;
};

uint32_t walk_of(const bt_rec& r, Walked* out) {
    uint32_t k = 0;
    out[k++] = {&kEth, 0, -1, BT_L_ETH};
    if (r.present & BT_L_VLAN0) out[k++] = {&kVlan, 12, 0, BT_L_VLAN0};
    if (r.present & BT_L_VLAN1) out[k++] = {&kVlan, 16, 1, BT_L_VLAN1};
    if (r.present & BT_L_IPV4) out[k++] = {&kIpv4, r.l3_off, -1, BT_L_IPV4};
    if (r.present & BT_L_IPV6) out[k++] = {&kIpv6, r.l3_off, -1, BT_L_IPV6};
    if (r.present & BT_L_TCP) out[k++] = {&kTcp, r.l4_off, -1, BT_L_TCP};
    if (r.present & BT_L_UDP) out[k++] = {&kUdp, r.l4_off, -1, BT_L_UDP};
    if (r.present & BT_L_ICMP) out[k++] = {&kIcmp, r.l4_off, -1, BT_L_ICMP};
    return k;
}

}  // namespace

std::vector<WalkedLayer> GpuParsedBatch::layers(size_t i) const {
    Walked w[8];
    const uint32_t k = walk_of(recs_.at(i), w);
    std::vector<WalkedLayer> out;
    out.reserve(k);
    for (uint32_t j = 0; j < k; ++j) out.push_back({w[j].table->name, w[j].offset, w[j].tag});
    return out;
}

ParseResult GpuParsedBatch::layer(size_t i, size_t k) const {
    Walked w[8];
    const bt_rec& r = recs_.at(i);
    if (k >= walk_of(r, w)) throw std::out_of_range("GpuParsedBatch::layer: no walked layer " + std::to_string(k));
    const Walked& L = w[k];
    const Table& t = *L.table;
    const uint8_t* f = frames_[i];
    const size_t len = lens_[i];
    ParseResult res;   // parsePacketInternal (:238-284)
    res.protocolName = t.name;
    res.protocolVersion = t.version;
    res.rawData.assign(f + L.offset, f + len);
    res.packetLength = len - L.offset;
    res.parsedBytes = 0;
    if (!(r.ok & L.bit)) {
        res.status = ParseStatus::PACKET_TOO_SHORT;
        res.errorMessage = "Packet too short for protocol";
        return res;
    }
    const uint32_t bias = L.tag == 1 ? 2u : 0u;
    // inserted one by one in table order, as the reference's result.fields[name] = value, so
    // the map's iteration order (which the formatters print in) is the reference's
    for (const Field& fd : t.fields) res.fields.emplace(fd.name, make_field(r, fd, bias));
    res.parsedBytes = t.total;
    return res;
}

ParseResult GpuParsedBatch::layer(size_t i, const std::string& name) const {
    const auto ls = layers(i);
    for (size_t k = 0; k < ls.size(); ++k)
        if (ls[k].name == name) return layer(i, k);
    ParseResult res;   // parsePacket with an unknown / absent protocol (:76-81)
    res.status = ParseStatus::PROTOCOL_NOT_FOUND;
    res.errorMessage = "Protocol not found: " + name;
    return res;
}

GpuParsedBatch::DetectionResult GpuParsedBatch::detect(size_t i) const {
    // names, confidences and reasons of ProtocolDetector::detectProtocol (:353-388)
    static const struct { const char* name; double conf; const char* reason; } kDet[] = {
        {"unknown", 0.0, "Packet too short"},        {"", 0.0, ""},
        {"ethernet", 0.95, "Valid Ethernet frame"},  {"tcp", 0.98, "Ethernet + IPv4 + TCP"},
        {"udp", 0.98, "Ethernet + IPv4 + UDP"},      {"icmp", 0.98, "Ethernet + IPv4 + ICMP"}};
    const uint8_t c = recs_.at(i).detect_code;
    if (c > BT_DET_ICMP) throw std::logic_error("GpuParsedBatch::detect: bad detector code");
    DetectionResult r;
    r.protocolName = kDet[c].name;
    r.confidence = kDet[c].conf;
    r.reason = kDet[c].reason;
    r.detectionTime = std::chrono::microseconds(0);
    return r;
}

std::vector<GpuParsedBatch::DetectionResult> GpuParsedBatch::detectMultiple(size_t i) const {
    std::vector<DetectionResult> out{detect(i)};
    const uint8_t x = recs_[i].detect_is2;
    if (x & (BT_IS2_MULTI_TCP | BT_IS2_MULTI_UDP)) {   // :395-413
        DetectionResult r;
        const bool tcp = (x & BT_IS2_MULTI_TCP) != 0;
        r.protocolName = tcp ? "tcp" : "udp";
        r.confidence = 0.98;
        r.reason = tcp ? "TCP over IPv4" : "UDP over IPv4";
        r.detectionTime = std::chrono::microseconds(0);
        out.push_back(r);
    }
    return out;
}

namespace {
std::string format_recs(bt_ctx* ctx, const bt_rec* r, uint32_t n, uint32_t fmt) {
    // formatted once (bt_format_records_to), placed straight into the string
    std::string s;
    uint64_t need = 0;
    auto dest = [](void* user, uint64_t bytes) -> char* {
        auto* str = static_cast<std::string*>(user);
        str->resize(bytes);
        return bytes ? &(*str)[0] : nullptr;
    };
    if (bt_format_records_to(ctx, r, n, fmt, dest, &s, &need, nullptr) != BT_OK)
        throw std::invalid_argument(std::string("GpuParsedBatch::format: ") + bt_last_error());
    return s;
}
}  // namespace

std::string GpuParsedBatch::format(size_t i, uint32_t fmt) const { return format_recs(nullptr, &recs_.at(i), 1, fmt); }

std::string GpuParsedBatch::format(uint32_t fmt) const {
    return format_recs(ctx_, recs_.data(), (uint32_t)recs_.size(), fmt);
}

void detail::BatchStore::give(std::vector<const uint8_t*>& f, std::vector<uint32_t>& l, Keep& k) {
    // under mu (the caller's lock); the parser's destructor waits for it
    if (k.size() >= 65536 && ctx) {   // release the frames' references on the host threads
        auto release = [](void* x, uint32_t w, uint32_t T) {
            auto& v = *static_cast<Keep*>(x);
            for (size_t i = v.size() * w / T; i < v.size() * (w + 1) / T; ++i) v[i].reset();
        };
        if (bt_host_parallel(ctx, release, &k) != BT_OK) k.clear();
    }
    k.clear();
    f.clear();
    l.clear();
    auto keep_for_reuse = [](auto& pool, auto& v, size_t cap) {
        if (v.capacity() && pool.size() < cap) pool.push_back(std::move(v));
    };
    keep_for_reuse(frames, f, kSets);
    keep_for_reuse(lens, l, kSets);
    keep_for_reuse(keep, k, kSets);
}

GpuParsedBatch::~GpuParsedBatch() {
    if (!store_) return;
    std::lock_guard<std::mutex> lk(store_->mu);
    store_->give(frames_, lens_, keep_);
    recs_.clear();
    if (recs_.capacity() && store_->recs.size() < detail::BatchStore::kSets) store_->recs.push_back(std::move(recs_));
}

GpuFieldBatch::~GpuFieldBatch() {
    if (!store_) return;
    std::lock_guard<std::mutex> lk(store_->mu);
    store_->give(frames_, lens_, keep_);
    for (auto* v : {&status_, &image_}) {
        v->clear();
        if (v->capacity() && store_->bytes.size() < 2 * detail::BatchStore::kSets) store_->bytes.push_back(std::move(*v));
    }
    values_.clear();
    if (values_.capacity() && store_->words.size() < detail::BatchStore::kSets) store_->words.push_back(std::move(values_));
}

namespace {
// The largest array of `pool` for a batch about to be filled (empty if none).
template <class V>
V take_from(std::vector<V>& pool) {
    if (pool.empty()) return V{};
    auto it = std::max_element(pool.begin(), pool.end(),
                               [](const V& a, const V& b) { return a.capacity() < b.capacity(); });
    V v = std::move(*it);
    pool.erase(it);
    return v;
}
}  // namespace

void GpuProtocolParser::newBatch(GpuParsedBatch& b) {
    b.store_ = store_;
    std::lock_guard<std::mutex> lk(store_->mu);
    b.recs_ = take_from(store_->recs);
    b.frames_ = take_from(store_->frames);
    b.lens_ = take_from(store_->lens);
    b.keep_ = take_from(store_->keep);
}

void GpuProtocolParser::newBatch(GpuFieldBatch& b) {
    b.store_ = store_;
    std::lock_guard<std::mutex> lk(store_->mu);
    b.image_ = take_from(store_->bytes);   // the larger byte column first
    b.status_ = take_from(store_->bytes);
    b.values_ = take_from(store_->words);
    b.frames_ = take_from(store_->frames);
    b.lens_ = take_from(store_->lens);
    b.keep_ = take_from(store_->keep);
}

GpuProtocolParser::GpuProtocolParser(int device, const bt_opts* opts)
    : GpuProtocolParser(parser::ProtocolParser::ParserConfig{}, device, opts) {}

GpuProtocolParser::GpuProtocolParser(const parser::ProtocolParser::ParserConfig& config, int device,
                                     const bt_opts* opts)
    : config_(config) {
    if (bt_create(device, opts, &ctx_) != BT_OK)
        throw std::runtime_error(std::string("GpuProtocolParser: ") + bt_last_error());
    if (config_.enablePerformanceMetrics) profiling_ = true;   // :31-35
    if (const char* e = std::getenv("BEATRICE_GPU_HOST_BELOW")) hostBelow_ = std::strtoull(e, nullptr, 10);
    store_->ctx = ctx_;
}

GpuProtocolParser::~GpuProtocolParser() {
    {   // batches that outlive the parser release their references on their own thread
        std::lock_guard<std::mutex> lk(store_->mu);
        store_->ctx = nullptr;
    }
    bt_destroy(ctx_);
}

void GpuProtocolParser::run(GpuParsedBatch& b) {
    const uint32_t n = (uint32_t)b.frames_.size();
    b.recs_.resize(n);
    b.ctx_ = ctx_;
    const auto t0 = std::chrono::steady_clock::now();
    if (n && bt_parse_filter_ptrs(ctx_, b.frames_.data(), b.lens_.data(), n, b.recs_.data(), nullptr, nullptr,
                                  nullptr, nullptr) != BT_OK)
        throw std::runtime_error(std::string("GpuProtocolParser: ") + bt_last_error());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    // updateStats (src/parser/ProtocolParser.cpp:482-506) for every walked layer
    static const char* kName[8] = {"ethernet", "vlan", "vlan", "ipv4", "ipv6", "tcp", "udp", "icmp"};
    // per-layer counts of the batch, tallied on the host threads (a 96-B record per packet)
    struct Tally {
        uint64_t ok = 0, bad = 0, per[8] = {};
        char pad[64];   // one cache line apart
    };
    std::vector<Tally> parts(n >= 65536 ? 16 : 1);
    struct U {
        const bt_rec* recs;
        size_t n;
        std::vector<Tally>* parts;
    } u{b.recs_.data(), n, &parts};
    auto tally = [](void* x, uint32_t w, uint32_t T) {
        auto* u = static_cast<U*>(x);
        const uint32_t P = (uint32_t)u->parts->size();
        for (uint32_t part = w; part < P; part += T) {
            Tally& t = (*u->parts)[part];
            for (size_t i = u->n * part / P; i < u->n * (part + 1) / P; ++i) {
                const bt_rec& r = u->recs[i];
                for (int k = 0; k < 8; ++k) {
                    if (!(r.present & (1u << k))) continue;
                    ++t.per[k];
                    if (r.ok & (1u << k)) ++t.ok; else ++t.bad;
                }
            }
        }
    };
    if (parts.size() == 1 || bt_host_parallel(ctx_, tally, &u) != BT_OK) tally(&u, 0, 1);
    uint64_t ok = 0, bad = 0, per[8] = {};
    for (const Tally& t : parts) {
        ok += t.ok;
        bad += t.bad;
        for (int k = 0; k < 8; ++k) per[k] += t.per[k];
    }
    std::lock_guard<std::mutex> lk(stats_mu_);
    const uint64_t layers = ok + bad;
    if (!layers) return;
    auto& st = stats_;
    st.totalPacketsParsed += layers;
    st.successfulParses += ok;
    st.failedParses += bad;
    const double each = us / (double)layers;
    time_carry_us_ += us;
    const auto total = std::chrono::microseconds((int64_t)time_carry_us_);
    st.totalParseTime += total;
    time_carry_us_ -= (double)total.count();
    const auto per_layer = std::chrono::microseconds((int64_t)each);
    if (per_layer < st.minParseTime) st.minParseTime = per_layer;
    if (per_layer > st.maxParseTime) st.maxParseTime = per_layer;
    if (st.successfulParses) st.averageParseTime = std::chrono::microseconds(st.totalParseTime.count() / st.successfulParses);
    for (int k = 0; k < 8; ++k)
        if (per[k]) st.protocolUsageCount[kName[k]] += per[k];
}

parser::ProtocolParser::ParserStats GpuProtocolParser::getStats() const {
    std::lock_guard<std::mutex> lk(stats_mu_);
    return stats_;
}

void GpuProtocolParser::resetStats() {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_ = parser::ProtocolParser::ParserStats{};
    time_carry_us_ = 0.0;
}

// A batch keeps each packet's bytes alive through a reference to them (Packet::getData, 16 B)
// rather than a copy of the Packet (216 B, its Metadata strings included, which cost more to
// copy and destroy than the GPU pass took), and lists frames and lengths; large batches are
// filled on the context's host threads.
template <class Batch>
void GpuProtocolParser::adopt(bt_ctx* ctx, const std::vector<Packet>& packets, Batch& b) {
    const size_t n = packets.size();
    b.keep_.resize(n);
    b.frames_.resize(n);
    b.lens_.resize(n);
    struct U {
        const std::vector<Packet>* packets;
        Batch* b;
        size_t n;
    } u{&packets, &b, n};
    auto fill = [](void* x, uint32_t w, uint32_t T) {
        auto* u = static_cast<U*>(x);
        for (size_t i = u->n * w / T; i < u->n * (w + 1) / T; ++i) {
            const Packet& p = (*u->packets)[i];
            u->b->keep_[i] = p.getData();
            u->b->frames_[i] = p.data();
            u->b->lens_[i] = (uint32_t)p.length();
        }
    };
    if (n < 8192 || bt_host_parallel(ctx, fill, &u) != BT_OK) fill(&u, 0, 1);
}

GpuParsedBatch GpuProtocolParser::parseBatch(const std::vector<Packet>& packets) {
    GpuParsedBatch b;
    newBatch(b);
    adopt(ctx_, packets, b);
    run(b);
    return b;
}

GpuParsedBatch GpuProtocolParser::parseBatch(const uint8_t* base, const bt_pkt_desc* desc, uint32_t n) {
    GpuParsedBatch b;
    newBatch(b);
    b.frames_.resize(n);
    b.lens_.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        b.frames_[i] = base + BT_DESC_OFF(desc[i]);
        b.lens_[i] = BT_DESC_LEN(desc[i]);
    }
    run(b);
    return b;
}

// ---- user-defined protocols ------------------------------------------------------------

namespace {

// ProtocolParser::formatMacAddress / formatIPv4Address / formatIPv6Address / formatTimestamp
// (src/parser/ProtocolParser.cpp:599-640), the same standard-library calls.
std::string fmt_mac(const std::vector<uint8_t>& b) {
    if (b.size() != 6) return "invalid";
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < 6; ++i) {
        if (i) s += ':';
        s += d[b[i] >> 4];
        s += d[b[i] & 15];
    }
    return s;
}

std::string fmt_ts(uint64_t ts) {
    const auto tp = std::chrono::system_clock::from_time_t(ts);
    const auto t = std::chrono::system_clock::to_time_t(tp);
    const std::tm* tm = std::localtime(&t);
    if (!tm) return "";   // the reference passes NULL to put_time here (and crashes)
    std::stringstream ss;
    ss << std::put_time(tm, "%Y-%m-%d %H:%M:%S");
    return ss.str();
}

// ProtocolParser::validateField (:435-475): value constraints apply to the unsigned types,
// pattern constraints to FieldValue::toString() (src/parser/ParserResult.cpp:9-48).
std::string to_string_of(const FieldValue& v) {
    if (!v.valid) return "INVALID";
    switch (v.type) {
    case FieldValueType::UINT8: return std::to_string(std::get<uint8_t>(v.value));
    case FieldValueType::UINT16: return std::to_string(std::get<uint16_t>(v.value));
    case FieldValueType::UINT32: return std::to_string(std::get<uint32_t>(v.value));
    case FieldValueType::UINT64: return std::to_string(std::get<uint64_t>(v.value));
    case FieldValueType::INT8: return std::to_string(std::get<int8_t>(v.value));
    case FieldValueType::INT16: return std::to_string(std::get<int16_t>(v.value));
    case FieldValueType::INT32: return std::to_string(std::get<int32_t>(v.value));
    case FieldValueType::INT64: return std::to_string(std::get<int64_t>(v.value));
    case FieldValueType::FLOAT32: return std::to_string(std::get<float>(v.value));
    case FieldValueType::FLOAT64: return std::to_string(std::get<double>(v.value));
    case FieldValueType::BYTES: return "[" + std::to_string(std::get<std::vector<uint8_t>>(v.value).size()) + " bytes]";
    case FieldValueType::STRING: return std::get<std::string>(v.value);
    case FieldValueType::BOOLEAN: return std::get<bool>(v.value) ? "true" : "false";
    case FieldValueType::MAC_ADDRESS: case FieldValueType::IPV4_ADDRESS: case FieldValueType::IPV6_ADDRESS:
    case FieldValueType::TIMESTAMP: case FieldValueType::CUSTOM:
        return v.formatted.empty() ? "formatted" : v.formatted;
    default: return "unknown";
    }
}

// ---- the reference's ParseResult text, for any ParseResult ---------------------------
// FieldValue::toHexString / toJsonString (src/parser/ParserResult.cpp:50-108) and
// ParseResult::toJsonString / toXmlString / toCsvString / toHumanReadableString (:214-349),
// restated on an appender: what ProtocolParser::formatPacket returns (ProtocolParser.cpp:
// 145-157). bt_format_records writes the same text straight from GPU records for the
// builtin walk; this one takes whatever ParseResult the caller holds (a user table's,
// one the caller built or edited).
struct Text {
    std::string s;
    Text& operator<<(const std::string& x) { s += x; return *this; }
    Text& operator<<(const char* x) { s += x; return *this; }
    Text& operator<<(char c) { s += c; return *this; }
    template <class I, class = std::enable_if_t<std::is_integral_v<I>>>
    Text& operator<<(I v) { s += std::to_string(v); return *this; }
};

std::string hex_string_of(const FieldValue& v) {   // toHexString (:50-64)
    if (!v.valid) return "INVALID";
    if (v.type != FieldValueType::BYTES) return v.rawHex;
    const auto& b = std::get<std::vector<uint8_t>>(v.value);
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < std::min(b.size(), size_t(16)); ++i) {
        s += d[b[i] >> 4];
        s += d[b[i] & 15];
        s += ' ';
    }
    if (b.size() > 16) s += "...";
    return s;
}

void value_json(const FieldValue& v, Text& o) {   // toJsonString (:66-108)
    if (!v.valid) {
        o << "null";
        return;
    }
    o << "{\"type\":\"" << (int)v.type << "\",\"value\":";
    switch (v.type) {
    case FieldValueType::UINT8: case FieldValueType::UINT16: case FieldValueType::UINT32: case FieldValueType::UINT64:
    case FieldValueType::INT8: case FieldValueType::INT16: case FieldValueType::INT32: case FieldValueType::INT64:
    case FieldValueType::FLOAT32: case FieldValueType::FLOAT64: case FieldValueType::BOOLEAN:
        o << to_string_of(v);
        break;
    case FieldValueType::STRING: o << '"' << std::get<std::string>(v.value) << '"'; break;
    case FieldValueType::BYTES: o << '"' << hex_string_of(v) << '"'; break;
    default: o << '"' << to_string_of(v) << '"'; break;
    }
    if (!v.rawHex.empty()) o << ",\"raw_hex\":\"" << v.rawHex << '"';
    if (!v.formatted.empty()) o << ",\"formatted\":\"" << v.formatted << '"';
    o << ",\"parse_time\":" << (long long)v.parseTime.count() << '}';
}

std::string result_text(const ParseResult& r, uint32_t fmt) {
    Text o;
    switch (fmt) {
    case BT_FMT_JSON: {
        o << "{\"status\":" << (int)r.status << ",\"protocol_name\":\"" << r.protocolName
          << "\",\"protocol_version\":\"" << r.protocolVersion << "\",\"packet_length\":" << r.packetLength
          << ",\"parsed_bytes\":" << r.parsedBytes << ",\"total_parse_time\":" << (long long)r.totalParseTime.count()
          << ",\"total_validation_time\":" << (long long)r.totalValidationTime.count() << ",\"fields\":{";
        bool first = true;
        for (const auto& [name, v] : r.fields) {
            if (!first) o << ',';
            first = false;
            o << '"' << name << "\":";
            value_json(v, o);
        }
        o << "},\"validation_results\":[";
        first = true;
        for (const auto& vr : r.validationResults) {
            if (!first) o << ',';
            first = false;
            o << "{\"field_name\":\"" << vr.fieldName << "\",\"valid\":" << (vr.valid ? "true" : "false")
              << ",\"error_message\":\"" << vr.errorMessage << "\",\"validation_time\":"
              << (long long)vr.validationTime.count() << '}';
        }
        o << ']';
        if (!r.errorMessage.empty()) o << ",\"error_message\":\"" << r.errorMessage << '"';
        o << '}';
        break;
    }
    case BT_FMT_XML:
        o << "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<parse_result>\n  <status>" << (int)r.status
          << "</status>\n  <protocol_name>" << r.protocolName << "</protocol_name>\n  <protocol_version>"
          << r.protocolVersion << "</protocol_version>\n  <packet_length>" << r.packetLength
          << "</packet_length>\n  <parsed_bytes>" << r.parsedBytes << "</parsed_bytes>\n  <total_parse_time>"
          << (long long)r.totalParseTime.count() << "</total_parse_time>\n  <total_validation_time>"
          << (long long)r.totalValidationTime.count() << "</total_validation_time>\n  <fields>\n";
        for (const auto& [name, v] : r.fields) {
            o << "    <field name=\"" << name << "\">\n      <value>" << to_string_of(v) << "</value>\n      <type>"
              << (int)v.type << "</type>\n";
            if (!v.rawHex.empty()) o << "      <raw_hex>" << v.rawHex << "</raw_hex>\n";
            o << "    </field>\n";
        }
        o << "  </fields>\n";
        if (!r.validationResults.empty()) {
            o << "  <validation_results>\n";
            for (const auto& vr : r.validationResults) {
                o << "    <result field=\"" << vr.fieldName << "\" valid=\"" << (vr.valid ? "true" : "false") << "\">\n";
                if (!vr.errorMessage.empty()) o << "      <error>" << vr.errorMessage << "</error>\n";
                o << "    </result>\n";
            }
            o << "  </validation_results>\n";
        }
        if (!r.errorMessage.empty()) o << "  <error_message>" << r.errorMessage << "</error_message>\n";
        o << "</parse_result>";
        break;
    case BT_FMT_CSV:
        o << "Field,Value,Type,Valid,ParseTime\n";
        for (const auto& [name, v] : r.fields)
            o << name << ',' << to_string_of(v) << ',' << (int)v.type << ',' << (v.valid ? "true" : "false") << ','
              << (long long)v.parseTime.count() << '\n';
        break;
    default:   // human
        o << "Protocol: " << r.protocolName << " v" << r.protocolVersion << "\nStatus: "
          << (r.isSuccess() ? "SUCCESS" : "FAILED") << "\nPacket Length: " << r.packetLength
          << " bytes\nParsed Bytes: " << r.parsedBytes << " bytes\nParse Time: " << (long long)r.totalParseTime.count()
          << " \xce\xbcs\nValidation Time: " << (long long)r.totalValidationTime.count() << " \xce\xbcs\n\nFields:\n";
        for (const auto& [name, v] : r.fields) {
            o << "  " << name << ": " << to_string_of(v);
            if (!v.formatted.empty()) o << " (" << v.formatted << ')';
            o << '\n';
        }
        if (!r.validationResults.empty()) {
            o << "\nValidation Results:\n";
            for (const auto& vr : r.validationResults) {
                o << "  " << vr.fieldName << ": " << (vr.valid ? "PASS" : "FAIL");
                if (!vr.errorMessage.empty()) o << " - " << vr.errorMessage;
                o << '\n';
            }
        }
        if (!r.errorMessage.empty()) o << "\nError: " << r.errorMessage << '\n';
        break;
    }
    return std::move(o.s);
}

bool validate_field(const FieldValue& v, const parser::FieldDefinition& f) {
    if (!v.valid) return false;
    if (!f.constraint) return true;
    const auto& c = f.constraint.value();
    if (c.minValue.index() != std::variant_npos && c.maxValue.index() != std::variant_npos) {
        if (v.type == FieldValueType::UINT8 || v.type == FieldValueType::UINT16 || v.type == FieldValueType::UINT32 ||
            v.type == FieldValueType::UINT64) {
            const uint64_t x = std::visit([](const auto& y) -> uint64_t {
                if constexpr (std::is_arithmetic_v<std::decay_t<decltype(y)>>) return static_cast<uint64_t>(y);
                return 0;
            }, v.value);
            if (c.minValue.index() == 1 && x < std::get<uint64_t>(c.minValue)) return false;
            if (c.maxValue.index() == 1 && x > std::get<uint64_t>(c.maxValue)) return false;
        }
    }
    if (!c.pattern.empty() && to_string_of(v).find(c.pattern) == std::string::npos) return false;
    return true;
}

// extractField (:286-383) from the GPU's value bits and the field's bytes.
FieldValue field_value(const parser::FieldDefinition& f, uint64_t bits, const uint8_t* b) {
    FieldValue v;
    v.valid = true;
    v.rawHex = hex(b, f.length);
    std::vector<uint8_t> data(b, b + f.length);
    auto as = [&](auto t) {
        decltype(t) x;
        std::memcpy(&x, &bits, sizeof(x));
        return x;
    };
    using parser::FieldType;
    switch (f.type) {
    case FieldType::UINT8: v.type = FieldValueType::UINT8; v.value = as(uint8_t{}); break;
    case FieldType::UINT16: v.type = FieldValueType::UINT16; v.value = as(uint16_t{}); break;
    case FieldType::UINT32: v.type = FieldValueType::UINT32; v.value = as(uint32_t{}); break;
    case FieldType::UINT64: v.type = FieldValueType::UINT64; v.value = as(uint64_t{}); break;
    case FieldType::INT8: v.type = FieldValueType::INT8; v.value = as(int8_t{}); break;
    case FieldType::INT16: v.type = FieldValueType::INT16; v.value = as(int16_t{}); break;
    case FieldType::INT32: v.type = FieldValueType::INT32; v.value = as(int32_t{}); break;
    case FieldType::INT64: v.type = FieldValueType::INT64; v.value = as(int64_t{}); break;
    case FieldType::FLOAT32: v.type = FieldValueType::FLOAT32; v.value = as(float{}); break;
    case FieldType::FLOAT64: v.type = FieldValueType::FLOAT64; v.value = as(double{}); break;
    case FieldType::BYTES: v.type = FieldValueType::BYTES; v.value = data; break;
    case FieldType::STRING: v.type = FieldValueType::STRING; v.value = std::string(data.begin(), data.end()); break;
    case FieldType::BOOLEAN: v.type = FieldValueType::BOOLEAN; v.value = bits != 0; break;
    case FieldType::MAC_ADDRESS:
        v.type = FieldValueType::MAC_ADDRESS;
        v.formatted = fmt_mac(data);
        v.value = data;
        break;
    case FieldType::IPV4_ADDRESS:
        v.type = FieldValueType::IPV4_ADDRESS;
        v.formatted = data.size() == 4 ? fmt_ipv4(b) : "invalid";
        v.value = data;
        break;
    case FieldType::IPV6_ADDRESS:
        v.type = FieldValueType::IPV6_ADDRESS;
        v.formatted = data.size() == 16 ? fmt_ipv6(b) : "invalid";
        v.value = data;
        break;
    case FieldType::TIMESTAMP:
        v.type = FieldValueType::TIMESTAMP;
        v.value = bits;
        v.formatted = fmt_ts(bits);
        break;
    case FieldType::CUSTOM:
        v.type = FieldValueType::CUSTOM;
        v.value = data;
        if (f.formatter) v.formatted = f.formatter(data);
        break;
    }
    return v;
}

std::vector<bt_field_def> table_of_def(const parser::ProtocolDefinition& d) {
    std::vector<bt_field_def> t;
    for (const auto& f : d.fields)
        t.push_back(bt_field_def{(uint64_t)f.offset, (uint64_t)f.length, (uint32_t)f.type, (uint32_t)f.endianness});
    return t;
}

}  // namespace

std::vector<uint8_t> GpuFieldBatch::bytes(size_t i, size_t k) const {
    const auto& f = def_->fields.at(k);
    if (!isSuccess(i)) return {};
    const uint8_t* b = image_.data() + i * span_ + f.offset;
    return std::vector<uint8_t>(b, b + f.length);
}

ParseResult GpuFieldBatch::result(size_t i) const {   // parsePacketInternal (:238-284)
    ParseResult r;
    const uint32_t len = lens_.at(i);
    r.protocolName = def_->name;
    r.protocolVersion = def_->version;
    r.rawData.assign(frames_[i], frames_[i] + len);
    r.packetLength = len;
    r.parsedBytes = 0;
    if (!isSuccess(i)) {
        r.status = ParseStatus::PACKET_TOO_SHORT;
        r.errorMessage = "Packet too short for protocol";
        return r;
    }
    size_t parsed = 0;
    const uint8_t* img = image_.data() + i * span_;
    for (size_t k = 0; k < def_->fields.size(); ++k) {
        const auto& f = def_->fields[k];
        if (f.offset + f.length > len) continue;   // :252-254 (never once len >= span)
        FieldValue v = field_value(f, raw(i, k), img + f.offset);
        r.fields[f.name] = v;   // ParseResult::addField (ParserResult.cpp:351-353)
        if (validate_ && !validate_field(v, f)) {
            parser::ValidationResult vr;
            vr.fieldName = f.name;
            vr.valid = false;
            vr.errorMessage = "Field validation failed";
            r.validationResults.push_back(vr);
        }
        parsed = std::max(parsed, f.offset + f.length);
    }
    r.parsedBytes = parsed;   // validateChecksum is always true (:477-480)
    return r;
}

void GpuProtocolParser::countParses(const std::string& protocol, uint64_t ok, uint64_t bad, double us) {
    if (!config_.enablePerformanceMetrics) return;   // parsePacket updates stats only then (:89-92)
    std::lock_guard<std::mutex> lk(stats_mu_);
    const uint64_t n = ok + bad;
    if (!n) return;
    auto& st = stats_;
    st.totalPacketsParsed += n;
    st.successfulParses += ok;
    st.failedParses += bad;
    time_carry_us_ += us;
    const auto total = std::chrono::microseconds((int64_t)time_carry_us_);
    st.totalParseTime += total;
    time_carry_us_ -= (double)total.count();
    const auto each = std::chrono::microseconds((int64_t)(us / (double)n));
    if (each < st.minParseTime) st.minParseTime = each;
    if (each > st.maxParseTime) st.maxParseTime = each;
    if (st.successfulParses) {
        st.averageParseTime = std::chrono::microseconds(st.totalParseTime.count() / st.successfulParses);
        st.averageValidationTime = std::chrono::microseconds(st.totalValidationTime.count() / st.successfulParses);
    }
    st.protocolUsageCount[protocol] += n;
}

void GpuProtocolParser::extract(GpuFieldBatch& b) {
    const auto table = table_of_def(*b.def_);
    for (const auto& f : table)
        if (f.type == BT_FT_BOOLEAN && f.length == 0)
            throw std::invalid_argument("GpuProtocolParser: BOOLEAN field of length 0 (undefined in the reference)");
    uint64_t span = 0;
    if (bt_proto_span(table.data(), (uint32_t)table.size(), &span) != BT_OK)
        throw std::invalid_argument(std::string("GpuProtocolParser: ") + bt_last_error());
    const uint32_t n = (uint32_t)b.frames_.size();
    b.span_ = span > 0xFFFFu ? 0 : span;
    b.validate_ = config_.enableValidation;
    // bt_extract writes every status, value and image byte; bt_extract_host gets zeroed columns
    const bool on_host = n && n < hostBelow_;
    b.status_.resize(n);
    b.values_.resize((size_t)table.size() * n);
    b.image_.resize((size_t)n * b.span_);
    if (on_host) {
        std::fill(b.status_.begin(), b.status_.end(), 0);
        std::fill(b.values_.begin(), b.values_.end(), 0);
        std::fill(b.image_.begin(), b.image_.end(), 0);
    }
    const auto t0 = std::chrono::steady_clock::now();
    // a small batch (parsePacket's one packet) on this thread: the device's round trip costs more
    int rc = BT_OK;
    if (on_host)
        rc = bt_extract_host(b.frames_.data(), b.lens_.data(), n, table.data(), (uint32_t)table.size(), b.status_.data(),
                             table.empty() ? nullptr : b.values_.data(), b.span_ ? b.image_.data() : nullptr);
    else if (n)
        rc = bt_extract(ctx_, b.frames_.data(), b.lens_.data(), n, table.data(), (uint32_t)table.size(),
                        b.status_.data(), table.empty() ? nullptr : b.values_.data(), b.span_ ? b.image_.data() : nullptr);
    if (rc != BT_OK) throw std::runtime_error(std::string("GpuProtocolParser: ") + bt_last_error());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const uint64_t ok = (uint64_t)std::count(b.status_.begin(), b.status_.end(), (uint8_t)0);
    countParses(b.def_->name, ok, n - ok, us);
}

bool GpuProtocolParser::registerProtocol(const parser::ProtocolDefinition& protocol) {   // :41-50
    std::unique_lock<std::shared_mutex> lk(protocols_mu_);
    if (protocols_.find(protocol.name) != protocols_.end()) return false;
    protocols_[protocol.name] = std::make_shared<const parser::ProtocolDefinition>(protocol);
    return true;
}

bool GpuProtocolParser::unregisterProtocol(const std::string& name) {   // :52-62
    std::unique_lock<std::shared_mutex> lk(protocols_mu_);
    auto it = protocols_.find(name);
    if (it == protocols_.end()) return false;
    protocols_.erase(it);
    return true;
}

bool GpuProtocolParser::hasProtocol(const std::string& name) const {
    std::shared_lock<std::shared_mutex> lk(protocols_mu_);
    return protocols_.find(name) != protocols_.end();
}

std::vector<std::string> GpuProtocolParser::getSupportedProtocols() const {   // :193-204
    std::shared_lock<std::shared_mutex> lk(protocols_mu_);
    std::vector<std::string> names;
    names.reserve(protocols_.size());
    for (const auto& kv : protocols_) names.push_back(kv.first);
    return names;
}

void GpuProtocolParser::setConfig(const parser::ProtocolParser::ParserConfig& config) {   // :163-168
    config_ = config;
    if (config_.enablePerformanceMetrics) profiling_ = true;
}

GpuProtocolParser::DefPtr GpuProtocolParser::findProtocol(const std::string& name) const {
    std::shared_lock<std::shared_mutex> lk(protocols_mu_);
    auto it = protocols_.find(name);
    return it == protocols_.end() ? nullptr : it->second;
}

std::vector<GpuProtocolParser::DefPtr> GpuProtocolParser::allProtocols() const {
    std::shared_lock<std::shared_mutex> lk(protocols_mu_);
    std::vector<DefPtr> defs;
    defs.reserve(protocols_.size());
    for (const auto& kv : protocols_) defs.push_back(kv.second);   // the reference's iteration order (:117)
    return defs;
}

GpuFieldBatch GpuProtocolParser::batchOf(const std::vector<Packet>& packets, DefPtr def) {
    GpuFieldBatch b;
    newBatch(b);
    b.def_ = std::move(def);
    adopt(ctx_, packets, b);
    extract(b);
    return b;
}

GpuFieldBatch GpuProtocolParser::parseBatch(const std::vector<Packet>& packets,
                                           const parser::ProtocolDefinition& protocol) {
    return batchOf(packets, std::make_shared<const parser::ProtocolDefinition>(protocol));
}

GpuFieldBatch GpuProtocolParser::parseBatch(const std::vector<Packet>& packets, const std::string& protocolName) {
    DefPtr def = findProtocol(protocolName);
    if (!def) throw std::out_of_range("GpuProtocolParser: protocol not found: " + protocolName);
    return batchOf(packets, std::move(def));
}

std::vector<GpuFieldBatch> GpuProtocolParser::parseBatchMultipleProtocols(const std::vector<Packet>& packets) {
    std::vector<GpuFieldBatch> out;
    for (auto& d : allProtocols()) out.push_back(batchOf(packets, std::move(d)));
    return out;
}

ParseResult GpuProtocolParser::parseOne(const std::vector<uint8_t>& packet, DefPtr def) {
    GpuFieldBatch b;   // :97-110; a batch of one, borrowing the caller's vector for the call
    b.def_ = std::move(def);
    b.frames_.push_back(packet.data());
    b.lens_.push_back((uint32_t)packet.size());
    extract(b);
    return b.result(0);
}

ParseResult GpuProtocolParser::parsePacket(const std::vector<uint8_t>& packet, const parser::ProtocolDefinition& protocol) {
    return parseOne(packet, std::make_shared<const parser::ProtocolDefinition>(protocol));
}

ParseResult GpuProtocolParser::parsePacket(const std::vector<uint8_t>& packet, const std::string& protocolName) {
    if (protocolName.empty()) {   // :70-72
        auto all = parsePacketMultipleProtocols(packet);
        if (all.empty()) throw std::out_of_range("GpuProtocolParser::parsePacket: no protocol registered");
        return all[0];
    }
    DefPtr def = findProtocol(protocolName);
    if (!def) {   // :76-81: no stats update
        ParseResult r;
        r.status = ParseStatus::PROTOCOL_NOT_FOUND;
        r.errorMessage = "Protocol not found: " + protocolName;
        return r;
    }
    return parseOne(packet, std::move(def));
}

std::vector<ParseResult> GpuProtocolParser::parsePacketMultipleProtocols(const std::vector<uint8_t>& packet) {
    std::vector<ParseResult> out;
    for (auto& d : allProtocols()) out.push_back(parseOne(packet, std::move(d)));
    return out;
}

bool GpuProtocolParser::validatePacket(const std::vector<uint8_t>& packet, const std::string& protocolName) {
    return parsePacket(packet, protocolName).isSuccess();
}

bool GpuProtocolParser::validatePacket(const std::vector<uint8_t>& packet, const parser::ProtocolDefinition& protocol) {
    return parsePacket(packet, protocol).isSuccess();
}

// ---- the rest of ProtocolParser's surface (include/parser/ProtocolParser.hpp:56-93) ----

std::unique_ptr<GpuProtocolParser> GpuProtocolParser::create(const parser::ProtocolParser::ParserConfig& config,
                                                             int device, const bt_opts* opts) {   // :10-12
    return std::make_unique<GpuProtocolParser>(config, device, opts);
}

std::string GpuProtocolParser::formatPacket(const ParseResult& result, const std::string& format) {   // :145-157
    const uint32_t fmt = format == "xml" ? BT_FMT_XML : format == "csv" ? BT_FMT_CSV
                       : format == "human" ? BT_FMT_HUMAN : BT_FMT_JSON;   // anything else: json
    return result_text(result, fmt);
}

std::vector<uint8_t> GpuProtocolParser::serializePacket(const ParseResult& result) { return result.rawData; }   // :159-161

std::vector<std::string> GpuProtocolParser::getSupportedFormats() const { return {"json", "xml", "csv", "human"}; }

// :205-228. Like the reference, the callbacks are kept for the registered protocol and
// nothing calls them (formatPacket does not consult them).
bool GpuProtocolParser::addCustomValidator(const std::string& protocolName,
                                           std::function<bool(const std::vector<uint8_t>&, const ParseResult&)> validator) {
    std::unique_lock<std::shared_mutex> lk(protocols_mu_);
    if (protocols_.find(protocolName) == protocols_.end()) return false;
    customValidators_[protocolName] = std::move(validator);
    return true;
}

bool GpuProtocolParser::addCustomFormatter(const std::string& protocolName,
                                           std::function<std::string(const ParseResult&)> formatter) {
    std::unique_lock<std::shared_mutex> lk(protocols_mu_);
    if (protocols_.find(protocolName) == protocols_.end()) return false;
    customFormatters_[protocolName] = std::move(formatter);
    return true;
}

// ProtocolParser::bytesToHex / formatMacAddress / formatIPv4Address / formatIPv6Address /
// formatTimestamp (:591-640)
std::string GpuProtocolParser::bytesToHex(const std::vector<uint8_t>& bytes) const { return hex(bytes.data(), bytes.size()); }
std::string GpuProtocolParser::formatMacAddress(const std::vector<uint8_t>& bytes) const { return fmt_mac(bytes); }
std::string GpuProtocolParser::formatIPv4Address(const std::vector<uint8_t>& bytes) const {
    return bytes.size() == 4 ? fmt_ipv4(bytes.data()) : "invalid";
}
std::string GpuProtocolParser::formatIPv6Address(const std::vector<uint8_t>& bytes) const {
    return bytes.size() == 16 ? fmt_ipv6(bytes.data()) : "invalid";
}
std::string GpuProtocolParser::formatTimestamp(uint64_t timestamp) const { return fmt_ts(timestamp); }

// ParserBuilder (:642-738)
GpuParserBuilder& GpuParserBuilder::withValidation(bool e) { config_.enableValidation = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withChecksumValidation(bool e) { config_.enableChecksumValidation = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withFieldConstraints(bool e) { config_.enableFieldConstraints = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withCustomValidators(bool e) { config_.enableCustomValidators = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withPerformanceMetrics(bool e) { config_.enablePerformanceMetrics = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withFieldCaching(bool e) { config_.enableFieldCaching = e; return *this; }
GpuParserBuilder& GpuParserBuilder::withMaxFieldCacheSize(size_t n) { config_.maxFieldCacheSize = n; return *this; }
GpuParserBuilder& GpuParserBuilder::withMaxValidationErrors(size_t n) { config_.maxValidationErrors = n; return *this; }
GpuParserBuilder& GpuParserBuilder::withMaxParseTime(std::chrono::microseconds t) { config_.maxParseTime = t; return *this; }
GpuParserBuilder& GpuParserBuilder::withErrorCallback(std::function<void(const std::string&)> cb) {
    config_.errorCallback = std::move(cb);
    return *this;
}
GpuParserBuilder& GpuParserBuilder::withWarningCallback(std::function<void(const std::string&)> cb) {
    config_.warningCallback = std::move(cb);
    return *this;
}
GpuParserBuilder& GpuParserBuilder::withInfoCallback(std::function<void(const std::string&)> cb) {
    config_.infoCallback = std::move(cb);
    return *this;
}
GpuParserBuilder& GpuParserBuilder::withProtocol(const parser::ProtocolDefinition& p) {
    protocols_.push_back(p);
    return *this;
}
GpuParserBuilder& GpuParserBuilder::withProtocols(const std::vector<parser::ProtocolDefinition>& ps) {
    protocols_.insert(protocols_.end(), ps.begin(), ps.end());
    return *this;
}
std::unique_ptr<GpuProtocolParser> GpuParserBuilder::build(int device, const bt_opts* opts) {
    auto p = std::make_unique<GpuProtocolParser>(config_, device, opts);
    for (const auto& proto : protocols_) p->registerProtocol(proto);   // duplicates: the first stays
    return p;
}

}  // namespace gpu
}  // namespace beatrice
