// ref_harness.cpp — drives the COMPILED REFERENCE (oracle/_ref, built by
// oracle/Makefile from the unmodified sources under /root/reference) over a batch
// of frames. TEST INFRASTRUCTURE ONLY: used to generate the golden fixtures in
// tests/golden/ and, in bench.py's cpu_baseline leg, to time the reference's own
// parser + PacketFilter on the host cores.
//
// Layer walk: the build-defined walk of DESIGN.md ("R-WALK"); each layer record is
// exactly ProtocolParser(enablePerformanceMetrics=false).parsePacket(slice, name)
// (reference src/parser/ProtocolParser.cpp:69-95) written into the bt_rec layout.
// The walk decisions (EtherType, IHL, protocol, next header) are read from the
// reference's own ParseResults.
#include "parser/ProtocolParser.hpp"
#include "parser/ProtocolRegistry.hpp"
#include "beatrice/PacketFilter.hpp"
#include "beatrice/Packet.hpp"

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <variant>
#include <type_traits>

using beatrice::Packet;
using beatrice::PacketFilter;
using namespace beatrice::parser;

namespace {

struct Walker {
    std::unique_ptr<ProtocolParser> parser;
    Walker() {
        ProtocolParser::ParserConfig cfg;
        cfg.enablePerformanceMetrics = false;   // updateStats divides by successfulParses (SIGFPE)
        parser = std::make_unique<ProtocolParser>(cfg);
        parser->registerProtocol(BuiltinProtocols::createEthernetProtocol());
        parser->registerProtocol(BuiltinProtocols::createVLANProtocol());
        parser->registerProtocol(BuiltinProtocols::createIPv4Protocol());
        parser->registerProtocol(BuiltinProtocols::createIPv6Protocol());
        parser->registerProtocol(BuiltinProtocols::createTCPProtocol());
        parser->registerProtocol(BuiltinProtocols::createUDPProtocol());
        parser->registerProtocol(BuiltinProtocols::createICMPProtocol());
    }

    ParseResult layer(const uint8_t* f, uint32_t len, uint32_t off, const char* name) {
        std::vector<uint8_t> slice(f + off, f + len);
        return parser->parsePacket(slice, name);
    }
};

template <class T> void put(uint8_t* rec, int off, T v) { std::memcpy(rec + off, &v, sizeof(T)); }

template <class T> T fv(const ParseResult& r, const char* n) { return std::get<T>(r.fields.at(n).value); }

void put_bytes(uint8_t* rec, int off, const ParseResult& r, const char* n) {
    const auto& b = std::get<std::vector<uint8_t>>(r.fields.at(n).value);
    std::memcpy(rec + off, b.data(), b.size());
}

// returns false when the reference gave a status other than SUCCESS / PACKET_TOO_SHORT
bool status_ok(const ParseResult& r, bool* ok) {
    if (r.status == ParseStatus::SUCCESS) { *ok = true; return true; }
    if (r.status == ParseStatus::PACKET_TOO_SHORT && r.fields.empty()) { *ok = false; return true; }
    return false;
}

// bt_rec bytes 88..90 from the reference's own ProtocolDetector over the whole frame
void detect(const uint8_t* f, uint32_t len, uint8_t* out) {
    const std::vector<uint8_t> v(f, f + len);
    const auto d = ProtocolDetector::detectProtocol(v);
    const std::string& nm = d.protocolName;
    out[0] = nm == "unknown" ? 0 : nm.empty() ? 1 : nm == "ethernet" ? 2 : nm == "tcp" ? 3 : nm == "udp" ? 4
           : nm == "icmp" ? 5 : 0xFF;
    out[1] = (uint8_t)(ProtocolDetector::isEthernet(v) | ProtocolDetector::isIPv4(v) << 1 |
                       ProtocolDetector::isIPv6(v) << 2 | ProtocolDetector::isTCP(v) << 3 |
                       ProtocolDetector::isUDP(v) << 4 | ProtocolDetector::isICMP(v) << 5 |
                       ProtocolDetector::isHTTP(v) << 6 | ProtocolDetector::isDNS(v) << 7);
    const auto m = ProtocolDetector::detectMultipleProtocols(v);
    uint8_t extra = 0;
    if (m.size() > 1) extra = m[1].protocolName == "tcp" ? 0x02 : m[1].protocolName == "udp" ? 0x04 : 0x80;
    out[2] = (uint8_t)(ProtocolDetector::isARP(v) | extra | (m.size() > 2 ? 0x80 : 0));
}

// `results`, when given, receives every walked layer's ParseResult in walk order.
int walk(Walker& w, const uint8_t* f, uint32_t len, uint8_t* rec, std::vector<ParseResult>* results = nullptr) {
    auto layer = [&](const uint8_t* fr, uint32_t l, uint32_t off, const char* name) {
        ParseResult r = w.layer(fr, l, off, name);
        if (results) results->push_back(r);
        return r;
    };
    std::memset(rec, 0, 96);
    put<uint16_t>(rec, 14, (uint16_t)(len > 0xFFFF ? 0xFFFF : len));
    uint8_t present = 0x01, okb = 0;
    bool ok;
    int err = 0;
    do {
        ParseResult eth = layer(f, len, 0, "ethernet");
        if (!status_ok(eth, &ok)) { err = 1; break; }
        if (!ok) break;
        okb |= 0x01;
        put_bytes(rec, 0, eth, "destination_mac");
        put_bytes(rec, 6, eth, "source_mac");
        uint16_t et = fv<uint16_t>(eth, "ethertype");
        put<uint16_t>(rec, 12, et);

        int k = 0;
        bool stop = false;
        while (k < 2 && (et == 0x8100 || et == 0x88A8)) {
            uint32_t vo = 12 + 4 * k;
            present |= (uint8_t)(0x02 << k);
            ParseResult v = layer(f, len, vo, "vlan");
            if (!status_ok(v, &ok)) { err = 1; stop = true; break; }
            if (!ok) { stop = true; break; }
            okb |= (uint8_t)(0x02 << k);
            put<uint16_t>(rec, 16 + 2 * k, fv<uint16_t>(v, "tpid"));
            put<uint16_t>(rec, 20 + 2 * k, fv<uint16_t>(v, "tci"));
            if (len < vo + 6) { stop = true; break; }
            et = (uint16_t)((f[vo + 4] << 8) | f[vo + 5]);
            ++k;
        }
        if (stop) break;

        uint32_t o3 = 14 + 4 * k, o4 = 0;
        uint8_t l4 = 0;
        if (et == 0x0800) {
            present |= 0x08;
            rec[26] = (uint8_t)o3;
            ParseResult ip = layer(f, len, o3, "ipv4");
            if (!status_ok(ip, &ok)) { err = 1; break; }
            if (!ok) break;
            okb |= 0x08;
            put<uint8_t>(rec, 28, fv<uint8_t>(ip, "version"));
            put<uint8_t>(rec, 29, fv<uint8_t>(ip, "ihl"));
            put<uint8_t>(rec, 30, fv<uint8_t>(ip, "tos"));
            put<uint8_t>(rec, 31, fv<uint8_t>(ip, "ttl"));
            put<uint8_t>(rec, 32, fv<uint8_t>(ip, "protocol"));
            put<uint16_t>(rec, 34, fv<uint16_t>(ip, "total_length"));
            put<uint16_t>(rec, 36, fv<uint16_t>(ip, "identification"));
            put<uint16_t>(rec, 38, fv<uint16_t>(ip, "flags"));
            put<uint16_t>(rec, 40, fv<uint16_t>(ip, "checksum"));
            put_bytes(rec, 44, ip, "source_ip");
            put_bytes(rec, 48, ip, "destination_ip");
            uint8_t ihl = fv<uint8_t>(ip, "ihl") & 0x0F, proto = fv<uint8_t>(ip, "protocol");
            o4 = o3 + 4u * ihl;
            l4 = proto == 6 ? 0x20 : proto == 17 ? 0x40 : proto == 1 ? 0x80 : 0;
            if (!l4 || o4 > len) break;
        } else if (et == 0x86DD) {
            present |= 0x10;
            rec[26] = (uint8_t)o3;
            ParseResult ip = layer(f, len, o3, "ipv6");
            if (!status_ok(ip, &ok)) { err = 1; break; }
            if (!ok) break;
            okb |= 0x10;
            put<uint32_t>(rec, 28, fv<uint32_t>(ip, "version_traffic_class_flow_label"));
            put<uint16_t>(rec, 32, fv<uint16_t>(ip, "payload_length"));
            put<uint8_t>(rec, 34, fv<uint8_t>(ip, "next_header"));
            put<uint8_t>(rec, 35, fv<uint8_t>(ip, "hop_limit"));
            put_bytes(rec, 36, ip, "source_ip");
            put_bytes(rec, 52, ip, "destination_ip");
            uint8_t nh = fv<uint8_t>(ip, "next_header");
            o4 = o3 + 40;
            l4 = nh == 6 ? 0x20 : nh == 17 ? 0x40 : 0;
            if (!l4) break;
        } else {
            break;
        }

        present |= l4;
        rec[27] = (uint8_t)o4;
        const char* name = l4 == 0x20 ? "tcp" : l4 == 0x40 ? "udp" : "icmp";
        ParseResult t = layer(f, len, o4, name);
        if (!status_ok(t, &ok)) { err = 1; break; }
        if (!ok) break;
        okb |= l4;
        if (l4 == 0x20) {
            put<uint16_t>(rec, 68, fv<uint16_t>(t, "source_port"));
            put<uint16_t>(rec, 70, fv<uint16_t>(t, "destination_port"));
            put<uint32_t>(rec, 72, fv<uint32_t>(t, "sequence_number"));
            put<uint32_t>(rec, 76, fv<uint32_t>(t, "acknowledgment_number"));
            put<uint8_t>(rec, 80, fv<uint8_t>(t, "data_offset"));
            put<uint8_t>(rec, 81, fv<uint8_t>(t, "flags"));
            put<uint16_t>(rec, 82, fv<uint16_t>(t, "window_size"));
            put<uint16_t>(rec, 84, fv<uint16_t>(t, "checksum"));
            put<uint16_t>(rec, 86, fv<uint16_t>(t, "urgent_pointer"));
        } else if (l4 == 0x40) {
            put<uint16_t>(rec, 68, fv<uint16_t>(t, "source_port"));
            put<uint16_t>(rec, 70, fv<uint16_t>(t, "destination_port"));
            put<uint16_t>(rec, 72, fv<uint16_t>(t, "length"));
            put<uint16_t>(rec, 74, fv<uint16_t>(t, "checksum"));
        } else {
            put<uint8_t>(rec, 68, fv<uint8_t>(t, "type"));
            put<uint8_t>(rec, 69, fv<uint8_t>(t, "code"));
            put<uint16_t>(rec, 70, fv<uint16_t>(t, "checksum"));
            put<uint16_t>(rec, 72, fv<uint16_t>(t, "identifier"));
            put<uint16_t>(rec, 74, fv<uint16_t>(t, "sequence_number"));
        }
    } while (false);
    rec[24] = present;
    rec[25] = okb;
    return err;
}

struct FilterSpec {
    int32_t type;
    const char* expression;
    int32_t enabled;
    int32_t priority;
    int32_t custom_id;   // 0 = no std::function installed
};

// Custom callbacks the golden tests can name by id (host-side CUSTOM filter parity).
bool custom_fn(int id, const Packet& p) {
    switch (id) {
    case 1: return p.length() % 3 != 0;
    case 2: return p.length() >= 100;
    default: return true;
    }
}

std::unique_ptr<PacketFilter> make_filter(const FilterSpec* fs, uint32_t nf) {
    auto pf = std::make_unique<PacketFilter>();
    for (uint32_t i = 0; i < nf; ++i) {
        PacketFilter::FilterConfig c;
        c.type = static_cast<PacketFilter::FilterType>(fs[i].type);
        c.expression = fs[i].expression ? fs[i].expression : "";
        c.enabled = fs[i].enabled != 0;
        c.priority = fs[i].priority;
        std::string name = "f" + std::to_string(i);
        pf->addFilter(name, c);
        if (fs[i].custom_id) {
            int id = fs[i].custom_id;
            pf->setCustomFilter(name, [id](const Packet& p) { return custom_fn(id, p); });
        }
    }
    return pf;
}

const uint8_t* frame_at(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t i,
                        uint32_t* len) {
    if (desc) {
        *len = (uint32_t)(desc[i] >> 48);
        return base + (desc[i] & 0xFFFFFFFFFFFFull);
    }
    *len = stride;
    return base + (uint64_t)i * stride;
}

Packet make_packet(const uint8_t* f, uint32_t len) {
    // zero-copy view: the batch owns the bytes for the duration of the call
    return Packet(std::shared_ptr<const uint8_t[]>(f, [](const uint8_t*) {}), len);
}

}  // namespace

extern "C" {

// Per-packet bt_rec (AoS, 96 B) from the reference parser, bytes 88..90 from the
// reference ProtocolDetector (the CPU baseline, ref_bench, times the parser only). Returns the number of
// packets whose layers produced an unexpected ParseStatus (must be 0).
int ref_parse(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n, uint8_t* records) {
    Walker w;
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len;
        const uint8_t* f = frame_at(base, desc, stride, i, &len);
        bad += walk(w, f, len, records + (uint64_t)i * 96);
        detect(f, len, records + (uint64_t)i * 96 + 88);
    }
    return bad;
}

// The reference's own ParseResult formatters (src/parser/ParserResult.cpp:214-349) over
// every walked layer of every packet, each text followed by '\n': fmt 0 toJsonString,
// 1 toXmlString, 2 toCsvString, 3 toHumanReadableString. Each field's parseTime is a
// wall-clock duration_cast<microseconds> of one extractField call (ProtocolParser.cpp:256-261),
// so it is set to 0 before formatting. Returns the bytes needed; writes when they fit `cap`.
uint64_t ref_format(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n, int fmt, char* out,
                    uint64_t cap) {
    Walker w;
    std::string all;
    uint8_t rec[96];
    std::vector<ParseResult> rs;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len;
        const uint8_t* f = frame_at(base, desc, stride, i, &len);
        rs.clear();
        walk(w, f, len, rec, &rs);
        for (auto& r : rs) {
            for (auto& kv : r.fields) kv.second.parseTime = std::chrono::microseconds(0);
            all += fmt == 0 ? r.toJsonString() : fmt == 1 ? r.toXmlString() : fmt == 2 ? r.toCsvString()
                                                                              : r.toHumanReadableString();
            all += '\n';
        }
    }
    if (out && all.size() <= cap) std::memcpy(out, all.data(), all.size());
    return all.size();
}

// Per-packet PacketFilter::applyFilters(const Packet&) outcome:
//   code[i] = 0 passed, 1 rejected, 2 threw std::invalid_argument, 3 threw std::out_of_range,
//             4 threw something else
//   src[i]  = index of FilterResult::filterName ("f<idx>"), 255 when empty or on throw
int ref_filter(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
               const FilterSpec* fs, uint32_t nf, uint8_t* code, uint8_t* src) {
    auto pf = make_filter(fs, nf);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len;
        const uint8_t* f = frame_at(base, desc, stride, i, &len);
        Packet p = make_packet(f, len);
        try {
            auto r = pf->applyFilters(p);
            code[i] = r.passed ? 0 : 1;
            src[i] = r.filterName.empty() ? 255 : (uint8_t)std::stoi(r.filterName.substr(1));
        } catch (const std::invalid_argument&) {
            code[i] = 2; src[i] = 255;
        } catch (const std::out_of_range&) {
            code[i] = 3; src[i] = 255;
        } catch (...) {
            code[i] = 4; src[i] = 255;
        }
    }
    return 0;
}

// Batch overload PacketFilter::applyFilters(const std::vector<Packet>&): returns
// 0 and fills passed/src when no exception escaped, else 1 (+kind in *what).
int ref_filter_batch(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                     const FilterSpec* fs, uint32_t nf, uint8_t* passed, uint8_t* src, int* what) {
    auto pf = make_filter(fs, nf);
    std::vector<Packet> pk;
    pk.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len;
        const uint8_t* f = frame_at(base, desc, stride, i, &len);
        pk.push_back(make_packet(f, len));
    }
    try {
        auto rs = pf->applyFilters(pk);
        for (uint32_t i = 0; i < n; ++i) {
            passed[i] = rs[i].passed;
            src[i] = rs[i].filterName.empty() ? 255 : (uint8_t)std::stoi(rs[i].filterName.substr(1));
        }
        *what = 0;
        return 0;
    } catch (const std::invalid_argument&) {
        *what = 2;
    } catch (const std::out_of_range&) {
        *what = 3;
    }
    return 1;
}

// ProtocolParser::parsePacket(frame, ProtocolDefinition) (reference
// src/parser/ProtocolParser.cpp:97-110 -> parsePacketInternal :238-284) with a user field
// table, over every frame: fields[4k..4k+3] = {offset, length, FieldType, Endianness}.
// Outputs per packet: status (ParseStatus), per field the bits of the alternative the
// FieldValue variant holds (arithmetic types memcpy'd into a zeroed u64, bool 0/1,
// vectors / strings 0) at values[k * n + i], and the field's bytes decoded from its
// rawHex, concatenated in table order at fb + i * fb_stride (zeros for a packet that did
// not parse). Metrics are off (updateStats divides by successfulParses). Returns the
// number of packets whose result has a field count other than 0 or nf.
int ref_extract(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n, const uint64_t* fields,
                uint32_t nf, uint8_t* status, uint64_t* values, uint8_t* fb, uint64_t fb_stride) {
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    ProtocolParser parser(cfg);
    ProtocolDefinition def("USER", "1.0");
    for (uint32_t k = 0; k < nf; ++k)
        def.addField(FieldDefinition("f" + std::to_string(k), (size_t)fields[4 * k], (size_t)fields[4 * k + 1],
                                     static_cast<FieldType>(fields[4 * k + 2]),
                                     static_cast<Endianness>(fields[4 * k + 3])));
    int odd = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len;
        const uint8_t* f = frame_at(base, desc, stride, i, &len);
        const ParseResult r = parser.parsePacket(std::vector<uint8_t>(f, f + len), def);
        status[i] = static_cast<uint8_t>(r.status);
        if (r.fields.size() != 0 && r.fields.size() != nf) ++odd;
        uint8_t* out = fb + (uint64_t)i * fb_stride;
        std::memset(out, 0, fb_stride);
        uint64_t at = 0;
        for (uint32_t k = 0; k < nf; ++k) {
            uint64_t bits = 0;
            auto it = r.fields.find("f" + std::to_string(k));
            if (it != r.fields.end()) {
                std::visit([&](const auto& v) {
                    using V = std::decay_t<decltype(v)>;
                    if constexpr (std::is_same_v<V, bool>) bits = v ? 1u : 0u;
                    else if constexpr (std::is_arithmetic_v<V>) std::memcpy(&bits, &v, sizeof(V));
                }, it->second.value);
                const std::string& hx = it->second.rawHex;
                for (size_t b = 0; 2 * b + 1 < hx.size(); ++b)
                    out[at + b] = (uint8_t)std::stoi(hx.substr(2 * b, 2), nullptr, 16);
            }
            values[(uint64_t)k * n + i] = bits;
            at += fields[4 * k + 1];
        }
    }
    return odd;
}

// CPU baseline: the reference parser (one parsePacket per walked layer) and the
// reference PacketFilter, nthreads std::threads with per-thread instances on
// disjoint shards, repeated over the batch until `seconds` of wall time pass.
// Returns packets processed; *elapsed gets the wall seconds.
uint64_t ref_bench(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                   const FilterSpec* fs, uint32_t nf, int do_parse, int nthreads, double seconds,
                   double* elapsed) {
    std::atomic<uint64_t> total{0};
    std::atomic<bool> stop{false};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([&, t] {
            Walker w;
            auto pf = make_filter(fs, nf);
            uint32_t lo = (uint32_t)((uint64_t)n * t / nthreads), hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
            uint8_t rec[96];
            uint64_t done = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                for (uint32_t i = lo; i < hi; ++i) {
                    uint32_t len;
                    const uint8_t* f = frame_at(base, desc, stride, i, &len);
                    if (do_parse) walk(w, f, len, rec);
                    if (nf) {
                        Packet p = make_packet(f, len);
                        try { (void)pf->applyFilters(p); } catch (...) {}
                    }
                    ++done;
                    if ((done & 255) == 0) {
                        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                        if (s >= seconds) stop = true;
                        if (stop.load(std::memory_order_relaxed)) break;
                    }
                }
            }
            total += done;
        });
    }
    for (auto& x : th) x.join();
    *elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return total.load();
}

// CPU baseline of the user-protocol path: ProtocolParser::parsePacket(frame,
// ProtocolDefinition) (src/parser/ProtocolParser.cpp:97-110) with metrics off, nthreads
// std::threads with per-thread parser + definition on disjoint shards, repeated until
// `seconds` of wall time pass. Returns packets parsed; *elapsed gets the wall seconds.
uint64_t ref_bench_extract(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                           const uint64_t* fields, uint32_t nf, int nthreads, double seconds, double* elapsed) {
    std::atomic<uint64_t> total{0};
    std::atomic<bool> stop{false};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([&, t] {
            ProtocolParser::ParserConfig cfg;
            cfg.enablePerformanceMetrics = false;
            ProtocolParser parser(cfg);
            ProtocolDefinition def("USER", "1.0");
            for (uint32_t k = 0; k < nf; ++k)
                def.addField(FieldDefinition("f" + std::to_string(k), (size_t)fields[4 * k], (size_t)fields[4 * k + 1],
                                             static_cast<FieldType>(fields[4 * k + 2]),
                                             static_cast<Endianness>(fields[4 * k + 3])));
            uint32_t lo = (uint32_t)((uint64_t)n * t / nthreads), hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
            uint64_t done = 0, sink = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                for (uint32_t i = lo; i < hi; ++i) {
                    uint32_t len;
                    const uint8_t* f = frame_at(base, desc, stride, i, &len);
                    const ParseResult r = parser.parsePacket(std::vector<uint8_t>(f, f + len), def);
                    sink += r.fields.size();
                    ++done;
                    if ((done & 255) == 0) {
                        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                        if (s >= seconds) stop = true;
                        if (stop.load(std::memory_order_relaxed)) break;
                    }
                }
            }
            total += done + (sink == ~0ull);   // keep the results live
        });
    }
    for (auto& x : th) x.join();
    *elapsed = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return total.load();
}

}  // extern "C"
