// bt_filter_compile.cpp — host-side compiler from PacketFilter expressions to the
// POD program the gfx950 kernel evaluates.
//
// The reference re-parses every expression string for every packet inside
// applyFilters (src/PacketFilter.cpp:168-372, std::stoi / std::getline /
// std::regex per call). The result of that parsing depends only on the string, so
// it is done once here, with the very same libstdc++ calls, and the per-packet
// work left for the device is integer compares. Where the reference would throw
// from std::stoi, the slot records which exception and the gates after which it
// fires; where the reference needs std::regex or a user std::function, the slot
// is BT_K_HOST and the host adapter finishes those packets.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <regex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "bt_device.h"

namespace bt {
namespace {

// PacketFilter::parseIPAddress (src/PacketFilter.cpp:330-340), same calls.
std::vector<uint8_t> parse_ip(const std::string& s) {
    std::vector<uint8_t> r;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, '.')) r.push_back(static_cast<uint8_t>(std::stoi(tok)));
    return r;
}

uint32_t be_addr(const std::vector<uint8_t>& v) {
    return ((uint32_t)v[0] << 24) | ((uint32_t)v[1] << 16) | ((uint32_t)v[2] << 8) | v[3];
}

// One slot from one FilterConfig. Throws std::invalid_argument / std::out_of_range
// exactly where the reference's isIPInRange / isPortInRange would.
void compile_ip(const std::string& range, bt_filter_slot* s) {
    // isIPInRange (:342-360)
    size_t pos = range.find('/');
    if (pos != std::string::npos) {
        int prefix = std::stoi(range.substr(pos + 1));
        auto net = parse_ip(range.substr(0, pos));
        if (net.size() != 4) { s->kind = BT_K_FALSE; return; }
        // `0xFFFFFFFF << (32 - prefixLen)` on x86-64: SHL masks the count to 5 bits,
        // so /0 behaves as /32 and /33 as /1 (pinned by tests/golden quirk fixtures).
        uint32_t mask = 0xFFFFFFFFu << ((uint32_t)(32 - (int64_t)prefix) & 31u);
        s->kind = BT_K_IP_MASK;
        s->a = be_addr(net) & mask;
        s->b = mask;
        return;
    }
    auto ip = parse_ip(range);
    if (ip.size() != 4) { s->kind = BT_K_FALSE; return; }   // vector equality never holds
    s->kind = BT_K_IP_MASK;
    s->a = be_addr(ip);
    s->b = 0xFFFFFFFFu;
}

void compile_port(const std::string& range, bt_filter_slot* s) {
    // isPortInRange (:362-372)
    size_t pos = range.find('-');
    uint16_t lo, hi;
    if (pos != std::string::npos) {
        lo = static_cast<uint16_t>(std::stoi(range.substr(0, pos)));
        hi = static_cast<uint16_t>(std::stoi(range.substr(pos + 1)));
    } else {
        lo = hi = static_cast<uint16_t>(std::stoi(range));
    }
    s->kind = BT_K_PORT;
    s->a = lo;
    s->b = hi;
}

void compile_one(const bt_filter_desc& f, bt_filter_slot* s) {
    const std::string e = f.expression ? f.expression : "";
    s->kind = BT_K_TRUE;
    s->a = s->b = 0;
    s->throw_kind = 0;
    switch (f.type) {
    case BT_FILTER_BPF: {   // applyBPFFilter (:168-191): substring keywords
        if (e.empty()) return;
        uint32_t m = (e.find("tcp") != std::string::npos ? 1u : 0u) |
                     (e.find("udp") != std::string::npos ? 2u : 0u) |
                     (e.find("icmp") != std::string::npos ? 4u : 0u);
        s->kind = m ? BT_K_BPF : BT_K_FALSE;
        s->a = m;
        return;
    }
    case BT_FILTER_PROTOCOL:   // applyProtocolFilter (:193-217): exact names
        if (e.empty()) return;
        if (e == "tcp") { s->kind = BT_K_PROTO_EQ; s->a = 6; }
        else if (e == "udp") { s->kind = BT_K_PROTO_EQ; s->a = 17; }
        else if (e == "icmp") { s->kind = BT_K_PROTO_EQ; s->a = 1; }
        else if (e == "ip") { s->kind = BT_K_PROTO_NZ; }
        else s->kind = BT_K_FALSE;
        return;
    case BT_FILTER_IP_RANGE:   // applyIPRangeFilter (:219-247)
        if (e.empty()) return;
        try {
            compile_ip(e, s);
        } catch (const std::invalid_argument&) {
            s->kind = BT_K_IP_THROW; s->throw_kind = 1;
        } catch (const std::out_of_range&) {
            s->kind = BT_K_IP_THROW; s->throw_kind = 2;
        }
        return;
    case BT_FILTER_PORT_RANGE:   // applyPortRangeFilter (:249-286)
        if (e.empty()) return;
        try {
            compile_port(e, s);
            if (s->a > s->b) { s->kind = BT_K_FALSE; s->a = s->b = 0; }
        } catch (const std::invalid_argument&) {
            s->kind = BT_K_PORT_THROW; s->throw_kind = 1;
        } catch (const std::out_of_range&) {
            s->kind = BT_K_PORT_THROW; s->throw_kind = 2;
        }
        return;
    case BT_FILTER_PAYLOAD:   // applyPayloadFilter (:288-321): regex_error -> false
        if (e.empty()) return;
        try {
            std::regex probe(e);
            s->kind = BT_K_HOST;
        } catch (const std::regex_error&) {
            s->kind = BT_K_FALSE;
        }
        return;
    case BT_FILTER_CUSTOM:   // applyCustomFilter (:323-328): no function -> true
        s->kind = f.has_custom_func ? BT_K_HOST : BT_K_TRUE;
        return;
    default:   // a FilterType outside the enum matches no case: filterResult stays false (:80)
        s->kind = BT_K_FALSE;
        return;
    }
}

}  // namespace

int compile_filters(const bt_filter_desc* f, uint32_t n, bt_filter_slot* out, uint32_t cap,
                    uint32_t* n_slots, char* err, size_t errlen) {
    std::vector<uint32_t> ord;
    for (uint32_t i = 0; i < n; ++i)
        if (f[i].enabled) ord.push_back(i);
    // applyFilters sorts by priority, higher first (:70-73). Stable here: ties keep
    // the caller's order (the C++ adapter feeds the reference's own order).
    std::stable_sort(ord.begin(), ord.end(),
                     [&](uint32_t x, uint32_t y) { return f[x].priority > f[y].priority; });
    if (ord.size() > BT_MAX_FILTERS || ord.size() > cap) {
        if (err) snprintf(err, errlen, "too many enabled filters: %zu (max %d)", ord.size(), BT_MAX_FILTERS);
        return BT_E_INVALID_ARGUMENT;
    }
    for (size_t k = 0; k < ord.size(); ++k) {
        compile_one(f[ord[k]], &out[k]);
        out[k].source_index = ord[k];
    }
    *n_slots = (uint32_t)ord.size();
    return BT_OK;
}

// The uniform-predicate form of one slot (bt_device.h DevFilter): every built-in kind
// is a masked range test over a feature pair, behind one of three gates.
void uniform_form(const bt_filter_slot& s, DevFilter* d) {
    auto set = [&](uint32_t sel, uint32_t gate, uint32_t res, uint32_t mask, uint32_t lo, uint32_t span) {
        d->ctl = sel | (gate << 2) | (res << 4);
        d->mask = mask;
        d->lo = lo;
        d->span = span;
    };
    switch (s.kind) {
    case BT_K_TRUE: set(kSelProto, kGateNone, kResPred, 0u, 0u, ~0u); break;            // 0 - 0 <= ~0
    case BT_K_BPF: set(kSelPbit, kGateIpv4, kResPred, s.a, 1u, 6u); break;              // pbit & a in 1..7
    case BT_K_PROTO_EQ: set(kSelProto, kGateIpv4, kResPred, 0xFFu, s.a, 0u); break;     // proto == a
    case BT_K_PROTO_NZ: set(kSelProto, kGateIpv4, kResPred, 0xFFu, 1u, 254u); break;    // proto in 1..255
    case BT_K_IP_MASK: set(kSelIp, kGateIpv4, kResPred, s.b, s.a, 0u); break;           // (ip & b) == a
    case BT_K_PORT: set(kSelPort, kGateL4, kResPred, 0xFFFFu, s.a, s.b - s.a); break;   // a <= port <= b
    case BT_K_IP_THROW: set(kSelProto, kGateIpv4, kResThrow, 0u, 0u, 0u); break;
    case BT_K_PORT_THROW: set(kSelProto, kGateL4, kResThrow, 0u, 0u, 0u); break;
    case BT_K_HOST: case BT_K_PAYLOAD: set(kSelProto, kGateNone, kResHost, 0u, 0u, 0u); break;
    default: set(kSelProto, kGateNone, kResPred, 0u, 1u, 0u); break;                    // FALSE: 0 - 1 > 0
    }
}

void to_device_program(const bt_filter_slot* s, uint32_t n, DevProgram* p) {
    std::memset(p, 0, sizeof(*p));
    p->n = n;
    for (uint32_t i = 0; i < n && i < BT_MAX_FILTERS; ++i) {
        p->f[i].kind = s[i].kind;
        p->f[i].a = s[i].a;
        p->f[i].b = s[i].b;
        // compile_one turns an empty port range (a > b) into FALSE, so span never wraps
        uniform_form(s[i], &p->f[i]);
    }
}

}  // namespace bt
