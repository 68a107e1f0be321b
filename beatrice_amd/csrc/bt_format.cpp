// bt_format.cpp — text output of parsed records: the reference's ParseResult
// formatters (src/parser/ParserResult.cpp:9-108 FieldValue::toString / toHexString /
// toJsonString, :214-349 ParseResult::toJsonString / toXmlString / toCsvString /
// toHumanReadableString) produced straight from bt_rec, without building a
// ParseResult per layer. Host-only code (no device needed); the context's host pool
// splits the batch.
//
// Each walked layer (DESIGN.md "R-WALK"; GpuParsedBatch::layers) is the ParseResult
// ProtocolParser::parsePacket(slice, name) returns (ProtocolParser.cpp:69-95,
// 238-284): SUCCESS with every field of the builtin table, or PACKET_TOO_SHORT with
// no fields. Wall-clock values are 0: totalParseTime / totalValidationTime are never
// set by parsePacket (ParseResult() initialises them to 0), and each field's
// parseTime is a duration_cast<microseconds> of one extractField call.
//
// `fields` is an std::unordered_map, so the reference prints fields in that map's
// iteration order. The order is a property of the insertion sequence (table order,
// ParseResult::addField :351-353) and of the standard library's hash and bucket
// policy, so it is taken from an std::unordered_map filled the same way, once.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "beatrice_gpu.h"
#include "bt_host.h"

namespace bt {
namespace {

// FieldValueType values (include/parser/ParserResult.hpp:29-48) of the builtin fields
enum Kind { K_U8 = 0, K_U16 = 1, K_U32 = 2, K_BYTES = 10, K_IPV4 = 14, K_IPV6 = 15 };

struct FieldDef {
    const char* name;
    Kind kind;
    uint32_t rec_off;   // position in bt_rec (tag 1 of a VLAN adds 2)
    uint32_t len;
};

struct Table {
    const char* name;
    const char* version;
    uint32_t total;                 // ProtocolDefinition::getTotalLength()
    std::vector<FieldDef> fields;   // table order (ProtocolRegistry.cpp)
    std::vector<int> order;         // the reference's unordered_map iteration order
};

// reference src/parser/ProtocolRegistry.cpp:150-234, 289-297
Table kTables[] = {
    {"ethernet", "2.0", 14, {{"destination_mac", K_BYTES, 0, 6}, {"source_mac", K_BYTES, 6, 6},
                             {"ethertype", K_U16, 12, 2}}, {}},
    {"vlan", "1.0", 4, {{"tpid", K_U16, 16, 2}, {"tci", K_U16, 20, 2}}, {}},
    {"ipv4", "4.0", 20, {{"version", K_U8, 28, 1}, {"ihl", K_U8, 29, 1}, {"tos", K_U8, 30, 1},
                         {"total_length", K_U16, 34, 2}, {"identification", K_U16, 36, 2},
                         {"flags", K_U16, 38, 2}, {"ttl", K_U8, 31, 1}, {"protocol", K_U8, 32, 1},
                         {"checksum", K_U16, 40, 2}, {"source_ip", K_IPV4, 44, 4},
                         {"destination_ip", K_IPV4, 48, 4}}, {}},
    {"ipv6", "6.0", 40, {{"version_traffic_class_flow_label", K_U32, 28, 4}, {"payload_length", K_U16, 32, 2},
                         {"next_header", K_U8, 34, 1}, {"hop_limit", K_U8, 35, 1},
                         {"source_ip", K_IPV6, 36, 16}, {"destination_ip", K_IPV6, 52, 16}}, {}},
    {"tcp", "1.0", 20, {{"source_port", K_U16, 68, 2}, {"destination_port", K_U16, 70, 2},
                        {"sequence_number", K_U32, 72, 4}, {"acknowledgment_number", K_U32, 76, 4},
                        {"data_offset", K_U8, 80, 1}, {"flags", K_U8, 81, 1}, {"window_size", K_U16, 82, 2},
                        {"checksum", K_U16, 84, 2}, {"urgent_pointer", K_U16, 86, 2}}, {}},
    {"udp", "1.0", 8, {{"source_port", K_U16, 68, 2}, {"destination_port", K_U16, 70, 2},
                       {"length", K_U16, 72, 2}, {"checksum", K_U16, 74, 2}}, {}},
    {"icmp", "1.0", 8, {{"type", K_U8, 68, 1}, {"code", K_U8, 69, 1}, {"checksum", K_U16, 70, 2},
                        {"identifier", K_U16, 72, 2}, {"sequence_number", K_U16, 74, 2}}, {}},
};
enum { T_ETH, T_VLAN, T_IPV4, T_IPV6, T_TCP, T_UDP, T_ICMP };

std::once_flag g_order_once;

void init_orders() {
    for (Table& t : kTables) {
        std::unordered_map<std::string, int> m;   // ParseResult::fields, filled by addField
        for (size_t i = 0; i < t.fields.size(); ++i) m[t.fields[i].name] = (int)i;
        const std::unordered_map<std::string, int> built(m);   // ParseResultBuilder::build() copies
        t.order.clear();
        for (const auto& kv : built) t.order.push_back(kv.second);
    }
}

// ---- a small appender (no iostreams) -----------------------------------------------
struct Out {
    std::string s;
    void put(const char* x) { s.append(x); }
    void put(const char* x, size_t n) { s.append(x, n); }
    void put(const std::string& x) { s.append(x); }
    void ch(char c) { s.push_back(c); }
    void u64(uint64_t v) {
        char b[24];
        int k = 0;
        do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (k) s.push_back(b[--k]);
    }
};

const char kHex[] = "0123456789abcdef";

struct Value {          // one FieldValue, as the reference's extractField fills it (:286-383)
    Kind kind;
    uint64_t num;       // integer fields
    const uint8_t* raw; // BYTES / address fields: the raw bytes in the record
    uint32_t len;
};

void hex_of(const Value& v, Out& o) {   // rawHex = bytesToHex(wire bytes) (:591-597)
    if (v.kind == K_BYTES || v.kind == K_IPV4 || v.kind == K_IPV6) {
        for (uint32_t i = 0; i < v.len; ++i) { o.ch(kHex[v.raw[i] >> 4]); o.ch(kHex[v.raw[i] & 15]); }
    } else {
        for (int i = (int)v.len - 1; i >= 0; --i) {   // big-endian wire order of the decoded value
            const uint32_t b = (uint32_t)(v.num >> (8 * i)) & 0xFFu;
            o.ch(kHex[b >> 4]);
            o.ch(kHex[b & 15]);
        }
    }
}

void formatted_of(const Value& v, Out& o) {   // formatIPv4Address / formatIPv6Address (:610-631)
    if (v.kind == K_IPV4) {
        for (int i = 0; i < 4; ++i) { if (i) o.ch('.'); o.u64(v.raw[i]); }
    } else if (v.kind == K_IPV6) {
        for (int i = 0; i < 16; i += 2) {
            if (i) o.ch(':');
            const uint32_t g = ((uint32_t)v.raw[i] << 8) | v.raw[i + 1];   // std::hex, no padding
            bool lead = true;
            for (int sh = 12; sh >= 0; sh -= 4) {
                const uint32_t d = (g >> sh) & 15u;
                if (lead && d == 0 && sh) continue;
                lead = false;
                o.ch(kHex[d]);
            }
        }
    }
}
bool has_formatted(const Value& v) { return v.kind == K_IPV4 || v.kind == K_IPV6; }

void to_string(const Value& v, Out& o) {   // FieldValue::toString (:9-48)
    if (v.kind == K_BYTES) { o.ch('['); o.u64(v.len); o.put(" bytes]"); }
    else if (has_formatted(v)) formatted_of(v, o);
    else o.u64(v.num);
}

void value_json(const Value& v, Out& o) {   // FieldValue::toJsonString (:66-108)
    o.put("{\"type\":\"");
    o.u64((uint64_t)v.kind);
    o.put("\",\"value\":");
    if (v.kind == K_BYTES) {   // "\"" + toHexString() + "\"": "%02x " per byte, <= 16 bytes (:50-64)
        o.ch('"');
        for (uint32_t i = 0; i < std::min<uint32_t>(v.len, 16); ++i) {
            o.ch(kHex[v.raw[i] >> 4]); o.ch(kHex[v.raw[i] & 15]); o.ch(' ');
        }
        if (v.len > 16) o.put("...");
        o.ch('"');
    } else if (has_formatted(v)) {
        o.ch('"'); formatted_of(v, o); o.ch('"');
    } else {
        o.u64(v.num);
    }
    o.put(",\"raw_hex\":\"");
    hex_of(v, o);
    o.ch('"');
    if (has_formatted(v)) { o.put(",\"formatted\":\""); formatted_of(v, o); o.ch('"'); }
    o.put(",\"parse_time\":0}");
}

Value field_value(const bt_rec& r, const FieldDef& f, uint32_t bias) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&r) + f.rec_off + bias;
    Value v{f.kind, 0, p, f.len};
    if (f.kind == K_U8) v.num = p[0];
    else if (f.kind == K_U16) { uint16_t x; std::memcpy(&x, p, 2); v.num = x; }
    else if (f.kind == K_U32) { uint32_t x; std::memcpy(&x, p, 4); v.num = x; }
    return v;
}

struct Layer {
    int table;
    uint32_t offset;
    int tag;
    bool ok;
};

int walked_layers(const bt_rec& r, Layer* L) {   // GpuParsedBatch::layers()
    int n = 0;
    L[n++] = {T_ETH, 0, -1, (r.ok & BT_L_ETH) != 0};
    if (r.present & BT_L_VLAN0) L[n++] = {T_VLAN, 12, 0, (r.ok & BT_L_VLAN0) != 0};
    if (r.present & BT_L_VLAN1) L[n++] = {T_VLAN, 16, 1, (r.ok & BT_L_VLAN1) != 0};
    if (r.present & BT_L_IPV4) L[n++] = {T_IPV4, r.l3_off, -1, (r.ok & BT_L_IPV4) != 0};
    if (r.present & BT_L_IPV6) L[n++] = {T_IPV6, r.l3_off, -1, (r.ok & BT_L_IPV6) != 0};
    if (r.present & BT_L_TCP) L[n++] = {T_TCP, r.l4_off, -1, (r.ok & BT_L_TCP) != 0};
    if (r.present & BT_L_UDP) L[n++] = {T_UDP, r.l4_off, -1, (r.ok & BT_L_UDP) != 0};
    if (r.present & BT_L_ICMP) L[n++] = {T_ICMP, r.l4_off, -1, (r.ok & BT_L_ICMP) != 0};
    return n;
}

const char kTooShort[] = "Packet too short for protocol";   // ProtocolParser.cpp:245

void format_layer(const bt_rec& r, const Layer& L, uint32_t fmt, Out& o) {
    const Table& t = kTables[L.table];
    const uint64_t plen = r.pkt_len >= L.offset ? r.pkt_len - L.offset : 0;
    const uint64_t parsed = L.ok ? t.total : 0;
    const uint32_t status = L.ok ? 0u : 9u;   // SUCCESS / PACKET_TOO_SHORT
    const uint32_t bias = L.tag == 1 ? 2u : 0u;
    switch (fmt) {
    case BT_FMT_JSON:   // :214-254
        o.put("{\"status\":"); o.u64(status);
        o.put(",\"protocol_name\":\""); o.put(t.name);
        o.put("\",\"protocol_version\":\""); o.put(t.version);
        o.put("\",\"packet_length\":"); o.u64(plen);
        o.put(",\"parsed_bytes\":"); o.u64(parsed);
        o.put(",\"total_parse_time\":0,\"total_validation_time\":0,\"fields\":{");
        if (L.ok) {
            bool first = true;
            for (int k : t.order) {
                if (!first) o.ch(',');
                first = false;
                o.ch('"'); o.put(t.fields[k].name); o.put("\":");
                value_json(field_value(r, t.fields[k], bias), o);
            }
        }
        o.put("},\"validation_results\":[]");
        if (!L.ok) { o.put(",\"error_message\":\""); o.put(kTooShort); o.ch('"'); }
        o.ch('}');
        break;
    case BT_FMT_XML:    // :256-298
        o.put("<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<parse_result>\n  <status>"); o.u64(status);
        o.put("</status>\n  <protocol_name>"); o.put(t.name);
        o.put("</protocol_name>\n  <protocol_version>"); o.put(t.version);
        o.put("</protocol_version>\n  <packet_length>"); o.u64(plen);
        o.put("</packet_length>\n  <parsed_bytes>"); o.u64(parsed);
        o.put("</parsed_bytes>\n  <total_parse_time>0</total_parse_time>\n"
              "  <total_validation_time>0</total_validation_time>\n  <fields>\n");
        if (L.ok) {
            for (int k : t.order) {
                const Value v = field_value(r, t.fields[k], bias);
                o.put("    <field name=\""); o.put(t.fields[k].name); o.put("\">\n      <value>");
                to_string(v, o);
                o.put("</value>\n      <type>"); o.u64((uint64_t)v.kind);
                o.put("</type>\n      <raw_hex>"); hex_of(v, o);
                o.put("</raw_hex>\n    </field>\n");
            }
        }
        o.put("  </fields>\n");
        if (!L.ok) { o.put("  <error_message>"); o.put(kTooShort); o.put("</error_message>\n"); }
        o.put("</parse_result>");
        break;
    case BT_FMT_CSV:    // :300-313
        o.put("Field,Value,Type,Valid,ParseTime\n");
        if (L.ok) {
            for (int k : t.order) {
                const Value v = field_value(r, t.fields[k], bias);
                o.put(t.fields[k].name); o.ch(',');
                to_string(v, o); o.ch(',');
                o.u64((uint64_t)v.kind); o.put(",true,0\n");
            }
        }
        break;
    default:            // BT_FMT_HUMAN :315-349
        o.put("Protocol: "); o.put(t.name); o.put(" v"); o.put(t.version);
        o.put(L.ok ? "\nStatus: SUCCESS\nPacket Length: " : "\nStatus: FAILED\nPacket Length: "); o.u64(plen);
        o.put(" bytes\nParsed Bytes: "); o.u64(parsed);
        o.put(" bytes\nParse Time: 0 \xce\xbcs\nValidation Time: 0 \xce\xbcs\n\nFields:\n");
        if (L.ok) {
            for (int k : t.order) {
                const Value v = field_value(r, t.fields[k], bias);
                o.put("  "); o.put(t.fields[k].name); o.put(": ");
                to_string(v, o);
                if (has_formatted(v)) { o.put(" ("); formatted_of(v, o); o.ch(')'); }
                o.ch('\n');
            }
        }
        if (!L.ok) { o.put("\nError: "); o.put(kTooShort); o.ch('\n'); }
        break;
    }
    o.ch('\n');
}

}  // namespace
}  // namespace bt

using namespace bt;

namespace {

// Formats records [0, n) into at most 64 slices on packet boundaries (each worker its own
// slices, in its own buffer); base[s] = slice s's offset in the whole text, base[n_slices] =
// its size; pkt_off (n + 1 entries) each packet's offset.
struct Formatted {
    std::vector<Out> parts;
    std::vector<uint64_t> base;
};

Formatted format_slices(bt_ctx* ctx, const bt_rec* recs, uint32_t n, uint32_t format, uint64_t* pkt_off) {
    std::call_once(g_order_once, init_orders);
    const uint32_t n_slices = std::max<uint32_t>(1, std::min<uint32_t>(64, (n + 4095) / 4096));
    Formatted f;
    f.parts.resize(n_slices);
    std::vector<std::vector<uint64_t>> offs(pkt_off ? n_slices : 0);
    host_parallel(ctx, [&](unsigned w, unsigned T) {
        for (uint32_t s = w; s < n_slices; s += T) {
            const uint32_t lo = (uint32_t)((uint64_t)n * s / n_slices), hi = (uint32_t)((uint64_t)n * (s + 1) / n_slices);
            Out& o = f.parts[s];
            o.s.reserve((size_t)(hi - lo) * (format == BT_FMT_CSV ? 400 : 1200));
            if (pkt_off) offs[s].resize(hi - lo);
            Layer L[8];
            for (uint32_t i = lo; i < hi; ++i) {
                if (pkt_off) offs[s][i - lo] = o.s.size();
                const int nl = walked_layers(recs[i], L);
                for (int k = 0; k < nl; ++k) format_layer(recs[i], L[k], format, o);
            }
        }
    });
    f.base.assign(n_slices + 1, 0);
    for (uint32_t s = 0; s < n_slices; ++s) f.base[s + 1] = f.base[s] + f.parts[s].s.size();
    if (pkt_off) {
        for (uint32_t s = 0; s < n_slices; ++s) {
            const uint32_t lo = (uint32_t)((uint64_t)n * s / n_slices);
            for (size_t j = 0; j < offs[s].size(); ++j) pkt_off[lo + j] = f.base[s] + offs[s][j];
        }
        pkt_off[n] = f.base[n_slices];
    }
    return f;
}

void place(bt_ctx* ctx, const Formatted& f, char* out) {
    const uint32_t n_slices = (uint32_t)f.parts.size();
    host_parallel(ctx, [&](unsigned w, unsigned T) {
        for (uint32_t s = w; s < n_slices; s += T) std::memcpy(out + f.base[s], f.parts[s].s.data(), f.parts[s].s.size());
    });
}

}  // namespace

extern "C" int bt_format_records(bt_ctx* ctx, const bt_rec* recs, uint32_t n, uint32_t format, char* out,
                                 uint64_t cap, uint64_t* out_len, uint64_t* pkt_off) {
    if ((!recs && n) || !out_len || format > BT_FMT_HUMAN)
        return set_error(BT_E_INVALID_ARGUMENT, "bt_format_records: null argument or unknown format %u", format);
    const Formatted f = format_slices(ctx, recs, n, format, pkt_off);
    *out_len = f.base.back();
    if (!out) return BT_OK;   // size query
    if (cap < f.base.back())
        return set_error(BT_E_INVALID_ARGUMENT, "bt_format_records: %llu bytes needed, buffer holds %llu",
                         (unsigned long long)f.base.back(), (unsigned long long)cap);
    place(ctx, f, out);
    return BT_OK;
}

extern "C" int bt_format_records_to(bt_ctx* ctx, const bt_rec* recs, uint32_t n, uint32_t format,
                                    char* (*dest)(void* user, uint64_t bytes), void* user, uint64_t* out_len,
                                    uint64_t* pkt_off) {
    if ((!recs && n) || !out_len || !dest || format > BT_FMT_HUMAN)
        return set_error(BT_E_INVALID_ARGUMENT, "bt_format_records_to: null argument or unknown format %u", format);
    const Formatted f = format_slices(ctx, recs, n, format, pkt_off);
    *out_len = f.base.back();
    char* out = dest(user, f.base.back());
    if (!out && f.base.back())
        return set_error(BT_E_INVALID_ARGUMENT, "bt_format_records_to: no destination for %llu bytes",
                         (unsigned long long)f.base.back());
    if (out) place(ctx, f, out);
    return BT_OK;
}
