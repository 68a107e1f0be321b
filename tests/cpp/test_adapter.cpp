// test_adapter.cpp — GPU parity of the C++ drop-in layer against the reference itself.
//
// Links the reference's own parser + PacketFilter objects (oracle/_ref/obj, compiled
// from the unmodified sources by oracle/Makefile — test infrastructure) next to
// libbeatrice_gpu_host.so, and runs both on the same synthetic captures:
//   filters  GpuPacketFilter vs beatrice::PacketFilter: every FilterResult (passed,
//            filterName, reason), the stats, getActiveFilters, the exception thrown —
//            including equal-priority ties, PAYLOAD regex, CUSTOM callbacks, removal.
//   parser   GpuProtocolParser::layer(i, k) vs ProtocolParser::parsePacket(slice, name)
//            for every walked layer: every ParseResult member but the wall-clock times,
//            field iteration order included.
//   surface  formatPacket (every format, builtin and user-table results, validation results),
//            serializePacket, getSupportedFormats, addCustomFormatter / Validator, the
//            address / hex / timestamp utilities, create / createWithProtocols / ParserBuilder
//            over the reference's own ProtocolRegistry singleton.
//   plugin   dlopen of libgpu_parse_filter_plugin.so through createPlugin(), the
//            IPacketPlugin lifecycle, pass count vs the reference.
// Prints one line per check; exit status 0 = all passed.
#include <optional>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <variant>
#include <type_traits>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "beatrice/IPacketPlugin.hpp"
#include "beatrice/PacketFilter.hpp"
#include "parser/ProtocolParser.hpp"
#include "parser/ProtocolRegistry.hpp"
#include "../../beatrice_amd/host/GpuPacketFilter.hpp"
#include "../../beatrice_amd/host/GpuProtocolParser.hpp"

extern "C" uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc);
extern "C" int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads);

using beatrice::Packet;
using beatrice::PacketFilter;
using beatrice::gpu::GpuPacketFilter;

static int g_fail = 0;
#define CHECK(cond, ...)                                                  \
    do {                                                                  \
        if (!(cond)) {                                                    \
            ++g_fail;                                                     \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__);              \
            std::printf(__VA_ARGS__);                                     \
            std::printf("\n");                                            \
            return false;                                                 \
        }                                                                 \
    } while (0)

struct Capture {
    std::vector<uint8_t> data;
    std::vector<uint64_t> desc;
    std::vector<Packet> packets;
};

static Capture capture(int cfg, uint32_t n, uint64_t seed) {
    Capture c;
    c.desc.resize(n);
    c.data.resize(bt_synth_layout(cfg, n, seed, c.desc.data()));
    bt_synth_fill(cfg, n, seed, c.desc.data(), c.data.data(), 8);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = c.data.data() + (c.desc[i] & 0xFFFFFFFFFFFFull);
        c.packets.emplace_back(std::shared_ptr<const uint8_t[]>(f, [](const uint8_t*) {}), (size_t)(c.desc[i] >> 48));
    }
    return c;
}

struct Spec {
    std::string name;
    PacketFilter::FilterType type;
    std::string expr;
    int priority;
    bool enabled;
    int custom;   // 0 none, 1 len % 3 != 0, 2 len >= 100, 3 throws
};

static std::function<bool(const Packet&)> custom_fn(int id) {
    switch (id) {
    case 1: return [](const Packet& p) { return p.length() % 3 != 0; };
    case 2: return [](const Packet& p) { return p.length() >= 100; };
    default: return [](const Packet& p) -> bool {
        if (p.length() == 777) throw std::runtime_error("custom boom");
        return true;
    };
    }
}

template <class F>
static void install(F& f, const std::vector<Spec>& specs) {
    for (const auto& s : specs) {
        PacketFilter::FilterConfig c;
        c.type = s.type;
        c.expression = s.expr;
        c.priority = s.priority;
        c.enabled = s.enabled;
        f.addFilter(s.name, c);
        if (s.custom) f.setCustomFilter(s.name, custom_fn(s.custom));
    }
}

static std::string what_kind(const std::exception_ptr& e) {
    try {
        std::rethrow_exception(e);
    } catch (const std::invalid_argument& x) {
        return std::string("invalid_argument:") + x.what();
    } catch (const std::out_of_range& x) {
        return std::string("out_of_range:") + x.what();
    } catch (const std::exception& x) {
        return std::string("exception:") + x.what();
    }
}

// members > 1: the filter drives a group of that many contexts on device 0 (a device list,
// as BEATRICE_GPU_DEVICES gives; BT_OPT_GROUP_SHARED_DEVICE lets one GPU stand in for several)
static bt_opts shared_device_opts() {
    bt_opts o{};
    o.flags = BT_OPT_GROUP_SHARED_DEVICE;
    return o;
}

static bool filter_case(const char* label, const Capture& cap, const std::vector<Spec>& specs,
                        const std::vector<std::string>& remove = {}, int members = 1) {
    PacketFilter ref;
    const bt_opts shared = shared_device_opts();
    GpuPacketFilter gpu(std::vector<int>(members, 0), members > 1 ? &shared : nullptr);
    install(ref, specs);
    install(gpu, specs);
    for (const auto& r : remove) {
        ref.removeFilter(r);
        gpu.removeFilter(r);
    }
    CHECK(ref.getActiveFilters() == gpu.getActiveFilters(), "%s: active filter lists differ", label);
    std::vector<PacketFilter::FilterResult> a, b;
    std::exception_ptr ea, eb;
    try { a = ref.applyFilters(cap.packets); } catch (...) { ea = std::current_exception(); }
    try { b = gpu.applyFilters(cap.packets); } catch (...) { eb = std::current_exception(); }
    CHECK((bool)ea == (bool)eb, "%s: exception mismatch ref=%d gpu=%d", label, (bool)ea, (bool)eb);
    if (ea) {
        CHECK(what_kind(ea) == what_kind(eb), "%s: %s vs %s", label, what_kind(ea).c_str(), what_kind(eb).c_str());
    } else {
        CHECK(a.size() == b.size(), "%s: result counts", label);
        for (size_t i = 0; i < a.size(); ++i) {
            CHECK(a[i].passed == b[i].passed && a[i].filterName == b[i].filterName && a[i].reason == b[i].reason,
                  "%s: packet %zu ref=(%d,%s,%s) gpu=(%d,%s,%s)", label, i, a[i].passed, a[i].filterName.c_str(),
                  a[i].reason.c_str(), b[i].passed, b[i].filterName.c_str(), b[i].reason.c_str());
        }
    }
    {   // classify / classifyPerPacket on their own filter: the same passes (and throw)
        GpuPacketFilter g2(0);
        install(g2, specs);
        for (const auto& r : remove) g2.removeFilter(r);
        std::exception_ptr ec;
        GpuPacketFilter::Verdicts v;
        try { v = g2.classify(cap.packets); } catch (...) { ec = std::current_exception(); }
        CHECK((bool)ea == (bool)ec, "%s: classify exception mismatch", label);
        if (ec) {
            CHECK(what_kind(ea) == what_kind(ec), "%s: classify threw %s", label, what_kind(ec).c_str());
        } else {
            std::vector<uint32_t> want;
            for (size_t i = 0; i < a.size(); ++i)
                if (a[i].passed) want.push_back((uint32_t)i);
            CHECK(v.pass_idx == want, "%s: classify pass list (%zu vs %zu)", label, v.pass_idx.size(), want.size());
            const auto w = g2.classifyPerPacket(cap.packets);
            CHECK(w.pass_idx == want && w.error_idx.empty(), "%s: classifyPerPacket pass list", label);
        }
    }
    auto sa = ref.getStats(), sb = gpu.getStats();
    CHECK(sa.packetsProcessed == sb.packetsProcessed && sa.packetsPassed == sb.packetsPassed &&
              sa.packetsDropped == sb.packetsDropped && sa.filterCounts == sb.filterCounts,
          "%s: stats differ (processed %lu/%lu passed %lu/%lu)", label, (unsigned long)sa.packetsProcessed,
          (unsigned long)sb.packetsProcessed, (unsigned long)sa.packetsPassed, (unsigned long)sb.packetsPassed);
    std::printf("ok   filters %-22s %zu packets, %lu passed%s\n", label, cap.packets.size(),
                (unsigned long)sa.packetsPassed, ea ? (" (threw " + what_kind(ea) + ")").c_str() : "");
    return true;
}

// Several threads calling one GpuPacketFilter at once (each on its own shard, in chunks),
// while another thread keeps re-enabling a filter (a recompile between their calls): every
// result and the summed stats equal the reference's over the whole capture.
// lanes > 1: device 0 listed that many times (concurrent calls routed whole to the least busy
// lane); chunk0: the first thread's call size (small calls take the host branch, §1)
static bool concurrent_case(const char* label, const Capture& cap, const std::vector<Spec>& specs, int threads,
                            int lanes = 1, size_t chunk0 = 700) {
    PacketFilter ref;
    GpuPacketFilter gpu(std::vector<int>(lanes, 0));
    install(ref, specs);
    install(gpu, specs);
    const std::vector<PacketFilter::FilterResult> want = ref.applyFilters(cap.packets);
    std::vector<PacketFilter::FilterResult> got(cap.packets.size());
    std::vector<uint8_t> classified(cap.packets.size(), 2);
    std::atomic<bool> done{false};
    std::atomic<int> errors{0};
    std::thread mutator([&] {
        while (!done.load()) {
            gpu.setFilterEnabled(specs.front().name, true);
            std::this_thread::sleep_for(std::chrono::microseconds(300));
        }
    });
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            const size_t lo = cap.packets.size() * t / threads, hi = cap.packets.size() * (t + 1) / threads;
            size_t chunk = chunk0 + 311 * (size_t)t;
            for (size_t at = lo; at < hi; at += chunk) {
                const std::vector<Packet> part(cap.packets.begin() + at, cap.packets.begin() + std::min(hi, at + chunk));
                try {
                    if ((at / chunk) % 2) {   // half the chunks through classify
                        const auto v = gpu.classify(part);
                        for (size_t i = 0; i < part.size(); ++i) classified[at + i] = (v.decide[i] >> 6) == BT_DECIDE_PASS;
                        std::vector<PacketFilter::FilterResult> r = gpu.applyFilters(part);
                        for (size_t i = 0; i < r.size(); ++i) got[at + i] = std::move(r[i]);
                    } else {
                        std::vector<PacketFilter::FilterResult> r = gpu.applyFilters(part);
                        for (size_t i = 0; i < r.size(); ++i) got[at + i] = std::move(r[i]);
                    }
                } catch (...) {
                    ++errors;
                }
            }
        });
    for (auto& x : th) x.join();
    done = true;
    mutator.join();
    CHECK(errors == 0, "%s: %d calls threw", label, errors.load());
    for (size_t i = 0; i < want.size(); ++i) {
        CHECK(want[i].passed == got[i].passed && want[i].filterName == got[i].filterName && want[i].reason == got[i].reason,
              "%s: packet %zu ref=(%d,%s) gpu=(%d,%s)", label, i, want[i].passed, want[i].filterName.c_str(), got[i].passed,
              got[i].filterName.c_str());
        CHECK(classified[i] == 2 || classified[i] == (uint8_t)want[i].passed, "%s: classify packet %zu", label, i);
    }
    // classified chunks were counted twice (classify + applyFilters)
    uint64_t twice = 0, twice_passed = 0;
    for (size_t i = 0; i < want.size(); ++i)
        if (classified[i] != 2) {
            ++twice;
            twice_passed += want[i].passed;
        }
    const auto sa = ref.getStats(), sb = gpu.getStats();
    CHECK(sb.packetsProcessed == sa.packetsProcessed + twice && sb.packetsPassed == sa.packetsPassed + twice_passed,
          "%s: stats processed %lu (want %lu) passed %lu (want %lu)", label, (unsigned long)sb.packetsProcessed,
          (unsigned long)(sa.packetsProcessed + twice), (unsigned long)sb.packetsPassed,
          (unsigned long)(sa.packetsPassed + twice_passed));
    std::printf("ok   concurrent %-19s %zu packets on %d threads (%d lane(s), calls of %zu+) + a recompiling thread, "
                "%lu passed\n", label, cap.packets.size(), threads, lanes, chunk0, (unsigned long)sa.packetsPassed);
    return true;
}

static bool same_field(const beatrice::parser::FieldValue& x, const beatrice::parser::FieldValue& y) {
    return x.value == y.value && x.type == y.type && x.rawHex == y.rawHex && x.formatted == y.formatted &&
           x.valid == y.valid && x.errorMessage == y.errorMessage;
}

static bool parser_case(const char* label, const Capture& cap) {
    using namespace beatrice::parser;
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    ProtocolParser ref(cfg);
    for (auto p : {BuiltinProtocols::createEthernetProtocol(), BuiltinProtocols::createVLANProtocol(),
                   BuiltinProtocols::createIPv4Protocol(), BuiltinProtocols::createIPv6Protocol(),
                   BuiltinProtocols::createTCPProtocol(), BuiltinProtocols::createUDPProtocol(),
                   BuiltinProtocols::createICMPProtocol()})
        ref.registerProtocol(p);
    beatrice::gpu::GpuProtocolParser gpu(0);
    auto batch = gpu.parseBatch(cap.packets);
    size_t nlayers = 0;
    for (size_t i = 0; i < cap.packets.size(); ++i) {
        const uint8_t* f = cap.packets[i].data();
        const size_t len = cap.packets[i].length();
        auto ls = batch.layers(i);
        for (size_t k = 0; k < ls.size(); ++k) {
            ParseResult want = ref.parsePacket(std::vector<uint8_t>(f + ls[k].offset, f + len), ls[k].name);
            ParseResult got = batch.layer(i, k);
            ++nlayers;
            CHECK(want.status == got.status && want.protocolName == got.protocolName &&
                      want.protocolVersion == got.protocolVersion && want.errorMessage == got.errorMessage &&
                      want.packetLength == got.packetLength && want.parsedBytes == got.parsedBytes &&
                      want.rawData == got.rawData && want.validationResults.size() == got.validationResults.size(),
                  "%s: packet %zu layer %s header differs (status %d/%d)", label, i, ls[k].name.c_str(),
                  (int)want.status, (int)got.status);
            std::vector<std::string> ka, kb;
            for (const auto& [n, v] : want.fields) ka.push_back(n);
            for (const auto& [n, v] : got.fields) kb.push_back(n);
            CHECK(ka == kb, "%s: packet %zu layer %s field order differs", label, i, ls[k].name.c_str());
            for (const auto& [n, v] : want.fields)
                CHECK(same_field(v, got.fields.at(n)), "%s: packet %zu %s.%s differs", label, i, ls[k].name.c_str(),
                      n.c_str());
        }
    }
    // the reference's formatters over the materialised layers == bt_format_records text
    // (wall-clock field parse times zeroed; ParserResult.cpp:214-349)
    for (uint32_t fmt = BT_FMT_JSON; fmt <= BT_FMT_HUMAN; ++fmt) {
        std::string want;
        for (size_t i = 0; i < cap.packets.size() && i < 2000; ++i) {
            const uint8_t* f = cap.packets[i].data();
            const size_t len = cap.packets[i].length();
            for (const auto& L : batch.layers(i)) {
                ParseResult r = ref.parsePacket(std::vector<uint8_t>(f + L.offset, f + len), L.name);
                for (auto& kv : r.fields) kv.second.parseTime = std::chrono::microseconds(0);
                want += fmt == BT_FMT_JSON ? r.toJsonString() : fmt == BT_FMT_XML ? r.toXmlString()
                      : fmt == BT_FMT_CSV ? r.toCsvString() : r.toHumanReadableString();
                want += '\n';
            }
            const std::string one = batch.format(i, fmt);
            CHECK(want.size() >= one.size() && want.compare(want.size() - one.size(), one.size(), one) == 0,
                  "%s: packet %zu format %u differs", label, i, fmt);
        }
        const std::string all = batch.format(fmt);
        CHECK(all.compare(0, want.size(), want) == 0, "%s: batch text (format %u) differs", label, fmt);
    }
    // ProtocolDetector over the whole frame (ProtocolRegistry.cpp:353-487)
    for (size_t i = 0; i < cap.packets.size(); ++i) {
        const std::vector<uint8_t> v(cap.packets[i].data(), cap.packets[i].data() + cap.packets[i].length());
        const auto want = ProtocolDetector::detectMultipleProtocols(v);
        const auto got = batch.detectMultiple(i);
        const auto d = batch.detect(i);
        CHECK(want.size() == got.size() && d.protocolName == got[0].protocolName, "%s: packet %zu detector entries",
              label, i);
        for (size_t k = 0; k < want.size() && k < got.size(); ++k) {
            // the reference leaves confidence uninitialised for a non-Ethernet frame (name "")
            const bool conf_defined = !want[k].protocolName.empty();
            CHECK(want[k].protocolName == got[k].protocolName && want[k].reason == got[k].reason &&
                      (!conf_defined || want[k].confidence == got[k].confidence) &&
                      want[k].detectionTime == got[k].detectionTime,
                  "%s: packet %zu detector entry %zu: %s/%s", label, i, k, want[k].protocolName.c_str(),
                  got[k].protocolName.c_str());
        }
        const bool is_ref[8] = {ProtocolDetector::isEthernet(v), ProtocolDetector::isIPv4(v), ProtocolDetector::isIPv6(v),
                                ProtocolDetector::isTCP(v),      ProtocolDetector::isUDP(v),  ProtocolDetector::isICMP(v),
                                ProtocolDetector::isHTTP(v),     ProtocolDetector::isDNS(v)};
        for (int b = 0; b < 8; ++b)
            CHECK(is_ref[b] == batch.is(i, 1u << b), "%s: packet %zu predicate bit %d", label, i, b);
        CHECK(ProtocolDetector::isARP(v) == batch.isARP(i), "%s: packet %zu isARP", label, i);
    }
    // getStats: a reference parser with performance metrics on (its default), fed the same
    // layers, counts the same (times are wall clock: not compared)
    {
        ProtocolParser counted;   // default ParserConfig: enablePerformanceMetrics = true
        for (auto p : {BuiltinProtocols::createEthernetProtocol(), BuiltinProtocols::createVLANProtocol(),
                       BuiltinProtocols::createIPv4Protocol(), BuiltinProtocols::createIPv6Protocol(),
                       BuiltinProtocols::createTCPProtocol(), BuiltinProtocols::createUDPProtocol(),
                       BuiltinProtocols::createICMPProtocol()})
            counted.registerProtocol(p);
        gpu.resetStats();
        auto b2 = gpu.parseBatch(cap.packets);
        // a failed first parse makes the reference divide by zero (SIGFPE): compare only
        // captures whose first frame holds an Ethernet header
        const bool first_ok = !cap.packets.empty() && cap.packets[0].length() >= 14;
        for (size_t i = 0; first_ok && i < cap.packets.size(); ++i) {
            const uint8_t* f = cap.packets[i].data();
            const size_t len = cap.packets[i].length();
            for (const auto& L : b2.layers(i)) (void)counted.parsePacket(std::vector<uint8_t>(f + L.offset, f + len), L.name);
        }
        const auto want = counted.getStats();
        const auto got = gpu.getStats();
        CHECK(!first_ok || (want.totalPacketsParsed == got.totalPacketsParsed && want.successfulParses == got.successfulParses &&
                  want.failedParses == got.failedParses && want.protocolUsageCount == got.protocolUsageCount),
              "%s: parser stats differ: total %lu/%lu ok %lu/%lu failed %lu/%lu", label,
              (unsigned long)want.totalPacketsParsed, (unsigned long)got.totalPacketsParsed,
              (unsigned long)want.successfulParses, (unsigned long)got.successfulParses,
              (unsigned long)want.failedParses, (unsigned long)got.failedParses);
    }
    // GpuParsedBatch hands its arrays back to the parser when destroyed (and releases a large
    // batch's packet references on the parser's host threads): batches made from recycled
    // arrays hold the same records, at a size past the parallel-release threshold too, and a
    // batch that outlives its parser stays readable
    if (!cap.packets.empty()) {
        std::vector<Packet> big;
        while (big.size() < 70000) big.insert(big.end(), cap.packets.begin(), cap.packets.end());
        auto same = [&](const beatrice::gpu::GpuParsedBatch& b, const std::vector<Packet>& pk) {
            if (b.size() != pk.size()) return false;
            for (size_t i = 0; i < b.size(); ++i)
                if (std::memcmp(&b.record(i), &batch.record(i % cap.packets.size()), sizeof(bt_rec))) return false;
            return true;
        };
        for (int r = 0; r < 3; ++r) {
            auto b3 = gpu.parseBatch(r == 1 ? cap.packets : big);
            CHECK(same(b3, r == 1 ? cap.packets : big), "%s: records from recycled arrays differ (round %d)", label, r);
        }
        std::optional<beatrice::gpu::GpuParsedBatch> late;
        {
            beatrice::gpu::GpuProtocolParser p2(0);
            late = p2.parseBatch(big);
            (void)p2.parseBatch(big);
        }
        CHECK(same(*late, big), "%s: a batch outliving its parser", label);
        late.reset();
    }
    std::printf("ok   parser  %-22s %zu packets, %zu layer results, detector, stats, recycled arrays\n", label,
                cap.packets.size(), nlayers);
    return true;
}

// ---- user-defined protocols: GpuProtocolParser vs ProtocolParser with the same tables ----
static bool same_value(const beatrice::parser::FieldValue& x, const beatrice::parser::FieldValue& y) {
    if (x.value.index() != y.value.index()) return false;
    return std::visit([&](const auto& a) {
        using V = std::decay_t<decltype(a)>;
        const V& b = std::get<V>(y.value);
        if constexpr (std::is_arithmetic_v<V>) return std::memcmp(&a, &b, sizeof(V)) == 0;   // NaN payloads too
        else return a == b;
    }, x.value);
}

static bool same_fv(const beatrice::parser::FieldValue& x, const beatrice::parser::FieldValue& y) {
    return same_value(x, y) && x.type == y.type && x.rawHex == y.rawHex && x.formatted == y.formatted &&
           x.valid == y.valid && x.errorMessage == y.errorMessage;
}

static bool same_result(const char* label, size_t i, const beatrice::parser::ParseResult& want,
                        const beatrice::parser::ParseResult& got) {
    CHECK(want.status == got.status && want.protocolName == got.protocolName &&
              want.protocolVersion == got.protocolVersion && want.errorMessage == got.errorMessage &&
              want.packetLength == got.packetLength && want.parsedBytes == got.parsedBytes && want.rawData == got.rawData,
          "%s: packet %zu result header differs (status %d/%d)", label, i, (int)want.status, (int)got.status);
    std::vector<std::string> ka, kb;
    for (const auto& kv : want.fields) ka.push_back(kv.first);
    for (const auto& kv : got.fields) kb.push_back(kv.first);
    CHECK(ka == kb, "%s: packet %zu field order differs", label, i);
    for (const auto& kv : want.fields)
        CHECK(same_fv(kv.second, got.fields.at(kv.first)), "%s: packet %zu field %s differs (raw %s/%s fmt %s/%s)", label,
              i, kv.first.c_str(), kv.second.rawHex.c_str(), got.fields.at(kv.first).rawHex.c_str(),
              kv.second.formatted.c_str(), got.fields.at(kv.first).formatted.c_str());
    CHECK(want.validationResults.size() == got.validationResults.size(), "%s: packet %zu validation count %zu/%zu", label,
          i, want.validationResults.size(), got.validationResults.size());
    for (size_t k = 0; k < want.validationResults.size(); ++k)
        CHECK(want.validationResults[k].fieldName == got.validationResults[k].fieldName &&
                  want.validationResults[k].valid == got.validationResults[k].valid &&
                  want.validationResults[k].errorMessage == got.validationResults[k].errorMessage,
              "%s: packet %zu validation result %zu differs", label, i, k);
    return true;
}

static beatrice::parser::ProtocolDefinition parser_example_protocol() {   // examples/parser_example.cpp:18-22
    using namespace beatrice::parser;
    ProtocolDefinition p("CUSTOM_PROTO", "1.0");
    p.addField(FieldFactory::createUInt32Field("header", 0, Endianness::NETWORK, true, "Protocol header"));
    p.addField(FieldFactory::createUInt8Field("version", 4, true, "Protocol version"));
    p.addField(FieldFactory::createUInt16Field("length", 5, Endianness::NETWORK, true, "Data length"));
    p.addField(FieldFactory::createBytesField("data", 7, 10, "Payload data"));
    return p;
}

static beatrice::parser::ProtocolDefinition random_protocol(std::mt19937& rng, int k) {
    using namespace beatrice::parser;
    ProtocolDefinition p("USER_" + std::to_string(k), std::to_string(k % 3) + ".0");
    const int nf = 1 + (int)(rng() % 10);
    static const size_t natural[18] = {1, 2, 4, 8, 1, 2, 4, 8, 4, 8, 0, 0, 1, 6, 4, 16, 8, 0};
    for (int f = 0; f < nf; ++f) {
        const auto t = static_cast<FieldType>(rng() % 18);
        size_t len = (natural[(int)t] && rng() % 10 < 6) ? natural[(int)t] : rng() % 21;
        if (t == FieldType::TIMESTAMP) len = rng() % 6;   // localtime() range (the reference crashes past it)
        if (t == FieldType::BOOLEAN && len == 0) len = 1;
        const size_t off = (k % 4 == 3 && rng() % 2) ? 200 + rng() % 100 : rng() % 80;
        FieldDefinition fd("f" + std::to_string(f) + (rng() % 7 == 0 ? "" : "_" + std::to_string(rng() % 100)), off, len, t,
                           static_cast<Endianness>(rng() % 4));
        if (rng() % 5 == 0) {   // value / pattern constraints (validateField, ProtocolParser.cpp:435-475)
            FieldConstraint c;
            if (rng() % 2) { c.minValue = (uint64_t)(rng() % 64); c.maxValue = (uint64_t)(64 + rng() % 200); }
            static const char* pats[] = {"", "1", "invalid", "bytes]", "true", ":", "0"};
            c.pattern = pats[rng() % 7];
            fd.constraint = c;
        }
        if (t == FieldType::CUSTOM && rng() % 2)
            fd.formatter = [](const std::vector<uint8_t>& b) {
                return "n=" + std::to_string(b.size()) + (b.empty() ? "" : "/" + std::to_string(b[0]));
            };
        p.addField(fd);
    }
    return p;
}

static bool user_proto_case(const char* label, const Capture& cap) {
    using namespace beatrice::parser;
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    ProtocolParser ref(cfg);
    beatrice::gpu::GpuProtocolParser gpu(cfg, 0);
    std::mt19937 rng(0xB1A5);
    std::vector<ProtocolDefinition> defs{parser_example_protocol(), ProtocolDefinition("EMPTY", "0")};
    for (int k = 0; k < 24; ++k) defs.push_back(random_protocol(rng, k));
    size_t nres = 0;
    for (const auto& d : defs) {
        CHECK(ref.registerProtocol(d) == gpu.registerProtocol(d), "%s: registerProtocol(%s)", label, d.name.c_str());
        auto b = gpu.parseBatch(cap.packets, d);
        for (size_t i = 0; i < cap.packets.size(); ++i) {
            const uint8_t* f = cap.packets[i].data();
            const std::vector<uint8_t> v(f, f + cap.packets[i].length());
            ParseResult want = ref.parsePacket(v, d);
            if (!same_result(label, i, want, b.result(i))) return false;
            ++nres;
        }
    }
    CHECK(ref.registerProtocol(defs[0]) == gpu.registerProtocol(defs[0]), "%s: duplicate registerProtocol", label);
    CHECK(ref.getSupportedProtocols() == gpu.getSupportedProtocols(), "%s: getSupportedProtocols order", label);
    // parser_example's own calls (examples/parser_example.cpp:31-83): by name, and its JSON
    const std::vector<uint8_t> kat = {0x12, 0x34, 0x56, 0x78, 0x01, 0x00, 0x0A, 0xAA, 0xBB,
                                      0xCC, 0xDD, 0xEE, 0xFF, 0x11, 0x22, 0x33, 0x44};
    ParseResult want = ref.parsePacket(kat, "CUSTOM_PROTO"), got = gpu.parsePacket(kat, "CUSTOM_PROTO");
    if (!same_result("parser_example", 0, want, got)) return false;
    for (auto& kv : want.fields) kv.second.parseTime = std::chrono::microseconds(0);
    CHECK(want.toJsonString() == got.toJsonString(), "parser_example: JSON differs");
    CHECK(got.getFieldUInt("header") == 0x12345678u && got.getFieldUInt("version") == 1 &&
              got.getFieldUInt("length") == 10 && got.getFieldBytes("data").size() == 10,
          "parser_example: known answer (header 0x12345678, version 1, length 10, 10 data bytes)");
    // by name, unknown name, all protocols, validatePacket
    for (size_t i = 0; i < cap.packets.size() && i < 200; ++i) {
        const std::vector<uint8_t> v(cap.packets[i].data(), cap.packets[i].data() + cap.packets[i].length());
        auto w = ref.parsePacketMultipleProtocols(v), g = gpu.parsePacketMultipleProtocols(v);
        CHECK(w.size() == g.size(), "%s: parsePacketMultipleProtocols size", label);
        for (size_t k = 0; k < w.size(); ++k)
            if (!same_result(label, i, w[k], g[k])) return false;
        if (!same_result(label, i, ref.parsePacket(v, "USER_3"), gpu.parsePacket(v, "USER_3"))) return false;
        if (!same_result(label, i, ref.parsePacket(v, "NO_SUCH"), gpu.parsePacket(v, "NO_SUCH"))) return false;
        if (!same_result(label, i, ref.parsePacket(v, ""), gpu.parsePacket(v, ""))) return false;
        CHECK(ref.validatePacket(v, "USER_5") == gpu.validatePacket(v, "USER_5"), "%s: validatePacket", label);
    }
    CHECK(ref.unregisterProtocol("USER_2") == gpu.unregisterProtocol("USER_2") &&
              ref.unregisterProtocol("USER_2") == gpu.unregisterProtocol("USER_2") &&
              ref.hasProtocol("USER_2") == gpu.hasProtocol("USER_2"),
          "%s: unregisterProtocol / hasProtocol", label);
    // stats with metrics on (the reference's default): the first parse must succeed there
    {
        ProtocolParser counted;
        beatrice::gpu::GpuProtocolParser gcount(ProtocolParser::ParserConfig{}, 0);
        (void)counted.parsePacket(kat, defs[0]);
        (void)gcount.parsePacket(kat, defs[0]);
        for (size_t k = 1; k < 6; ++k) {
            (void)gcount.parseBatch(cap.packets, defs[k]);
            for (const auto& p : cap.packets)
                (void)counted.parsePacket(std::vector<uint8_t>(p.data(), p.data() + p.length()), defs[k]);
        }
        const auto w = counted.getStats(), g = gcount.getStats();
        CHECK(w.totalPacketsParsed == g.totalPacketsParsed && w.successfulParses == g.successfulParses &&
                  w.failedParses == g.failedParses && w.protocolUsageCount == g.protocolUsageCount,
              "%s: user-protocol stats differ: total %lu/%lu ok %lu/%lu", label, (unsigned long)w.totalPacketsParsed,
              (unsigned long)g.totalPacketsParsed, (unsigned long)w.successfulParses, (unsigned long)g.successfulParses);
    }
    std::printf("ok   proto   %-22s %zu packets x %zu tables (parser_example + random, constraints, CUSTOM "
                "formatters): %zu ParseResults, by-name / multiple / unknown / stats\n",
                label, cap.packets.size(), defs.size(), nres);
    return true;
}

// ---- the rest of ProtocolParser's surface: formatPacket / serializePacket /
// getSupportedFormats / addCustom* / utilities / create / createWithProtocols / ParserBuilder
static bool surface_case(const char* label, const Capture& cap) {
    using namespace beatrice::parser;
    using beatrice::gpu::GpuProtocolParser;
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    ProtocolParser ref(cfg);
    GpuProtocolParser gpu(cfg, 0);
    for (auto p : {BuiltinProtocols::createEthernetProtocol(), BuiltinProtocols::createVLANProtocol(),
                   BuiltinProtocols::createIPv4Protocol(), BuiltinProtocols::createIPv6Protocol(),
                   BuiltinProtocols::createTCPProtocol(), BuiltinProtocols::createUDPProtocol(),
                   BuiltinProtocols::createICMPProtocol()})
        ref.registerProtocol(p);
    const char* formats[] = {"json", "xml", "csv", "human", "yaml"};   // unknown: json
    CHECK(ref.getSupportedFormats() == gpu.getSupportedFormats(), "%s: getSupportedFormats", label);
    size_t ntext = 0;
    // builtin walk: the GPU layer's text == the reference's text of its own result
    auto batch = gpu.parseBatch(cap.packets);
    for (size_t i = 0; i < cap.packets.size() && i < 3000; ++i) {
        const uint8_t* f = cap.packets[i].data();
        const size_t len = cap.packets[i].length();
        const auto ls = batch.layers(i);
        for (size_t k = 0; k < ls.size(); ++k) {
            ParseResult want = ref.parsePacket(std::vector<uint8_t>(f + ls[k].offset, f + len), ls[k].name);
            const ParseResult got = batch.layer(i, k);
            for (const char* fm : formats) {
                // the formatter restated over the reference's own result (wall-clock times included)
                CHECK(ref.formatPacket(want, fm) == gpu.formatPacket(want, fm), "%s: packet %zu %s: formatPacket(%s) of "
                      "the reference's result differs", label, i, ls[k].name.c_str(), fm);
            }
            for (auto& kv : want.fields) kv.second.parseTime = std::chrono::microseconds(0);
            for (const char* fm : formats) {
                CHECK(ref.formatPacket(want, fm) == gpu.formatPacket(got, fm), "%s: packet %zu %s: formatPacket(%s) "
                      "of the GPU's result differs", label, i, ls[k].name.c_str(), fm);
                ++ntext;
            }
            CHECK(ref.serializePacket(want) == gpu.serializePacket(got), "%s: packet %zu serializePacket", label, i);
        }
    }
    // user tables with constraints (validation results and their messages in the text)
    std::mt19937 rng(0x5FAC);
    std::vector<ProtocolDefinition> defs{parser_example_protocol()};
    for (int k = 0; k < 8; ++k) defs.push_back(random_protocol(rng, 100 + k));
    ProtocolParser vref;   // validation and constraints on (the default config), metrics on
    GpuProtocolParser vgpu(ProtocolParser::ParserConfig{}, 0);
    for (const auto& d : defs) {
        vref.registerProtocol(d);
        vgpu.registerProtocol(d);
        auto b = vgpu.parseBatch(cap.packets, d);
        for (size_t i = 0; i < cap.packets.size() && i < 500; ++i) {
            const std::vector<uint8_t> v(cap.packets[i].data(), cap.packets[i].data() + cap.packets[i].length());
            ParseResult want = vref.parsePacket(v, d);
            const ParseResult got = b.result(i);
            for (const char* fm : formats)
                CHECK(vref.formatPacket(want, fm) == vgpu.formatPacket(want, fm), "%s: %s packet %zu: formatPacket(%s) "
                      "of the reference's result differs", label, d.name.c_str(), i, fm);
            want.totalParseTime = want.totalValidationTime = std::chrono::microseconds(0);
            for (auto& kv : want.fields) kv.second.parseTime = std::chrono::microseconds(0);
            for (auto& vr : want.validationResults) vr.validationTime = std::chrono::microseconds(0);
            for (const char* fm : formats) {
                CHECK(vref.formatPacket(want, fm) == vgpu.formatPacket(got, fm), "%s: %s packet %zu: formatPacket(%s) "
                      "of the GPU's result differs", label, d.name.c_str(), i, fm);
                ++ntext;
            }
            CHECK(vref.serializePacket(want) == vgpu.serializePacket(got), "%s: %s serializePacket", label,
                  d.name.c_str());
        }
    }
    // custom validators / formatters: registered protocols only (neither is ever called)
    auto fmt_cb = [](const ParseResult& r) { return r.protocolName; };
    auto val_cb = [](const std::vector<uint8_t>&, const ParseResult&) { return false; };
    CHECK(vref.addCustomFormatter("NOPE", fmt_cb) == vgpu.addCustomFormatter("NOPE", fmt_cb) &&
              vref.addCustomFormatter(defs[1].name, fmt_cb) == vgpu.addCustomFormatter(defs[1].name, fmt_cb) &&
              vref.addCustomValidator("NOPE", val_cb) == vgpu.addCustomValidator("NOPE", val_cb) &&
              vref.addCustomValidator(defs[2].name, val_cb) == vgpu.addCustomValidator(defs[2].name, val_cb),
          "%s: addCustomFormatter / addCustomValidator", label);
    CHECK(vref.isProfilingEnabled() == vgpu.isProfilingEnabled() && ref.isProfilingEnabled() == gpu.isProfilingEnabled(),
          "%s: isProfilingEnabled", label);
    vref.enableProfiling(false);
    vgpu.enableProfiling(false);
    CHECK(vref.isProfilingEnabled() == vgpu.isProfilingEnabled(), "%s: enableProfiling", label);
    // the utility methods
    for (size_t len : {0, 4, 5, 6, 16, 17}) {
        std::vector<uint8_t> b(len);
        for (auto& x : b) x = (uint8_t)rng();
        CHECK(ref.bytesToHex(b) == gpu.bytesToHex(b) && ref.formatMacAddress(b) == gpu.formatMacAddress(b) &&
                  ref.formatIPv4Address(b) == gpu.formatIPv4Address(b) &&
                  ref.formatIPv6Address(b) == gpu.formatIPv6Address(b),
              "%s: address/hex utilities, %zu bytes", label, len);
    }
    for (uint64_t ts : {0ull, 1ull, 1700000000ull, 4102444800ull})
        CHECK(ref.formatTimestamp(ts) == gpu.formatTimestamp(ts), "%s: formatTimestamp(%llu)", label,
              (unsigned long long)ts);
    // factories and the builder, over the reference's registry singleton
    auto& registry = ProtocolRegistry::getInstance();
    registry.loadBuiltinProtocols();
    registry.registerProtocol(parser_example_protocol());
    const std::vector<std::string> names = {"ethernet", "ipv4", "no_such", "udp", "CUSTOM_PROTO"};
    auto r1 = ProtocolParser::createWithProtocols(names, cfg);
    auto g1 = GpuProtocolParser::createWithProtocols(names, cfg, registry, 0);
    CHECK(r1->getSupportedProtocols() == g1->getSupportedProtocols(), "%s: createWithProtocols protocols", label);
    auto r2 = ProtocolParser::create(cfg);
    auto g2 = GpuProtocolParser::create(cfg, 0);
    CHECK(r2->getSupportedProtocols().empty() && g2->getSupportedProtocols().empty() &&
              r2->isProfilingEnabled() == g2->isProfilingEnabled() &&
              r2->getConfig().enablePerformanceMetrics == g2->getConfig().enablePerformanceMetrics,
          "%s: create", label);
    auto r3 = ParserBuilder().withValidation(false).withPerformanceMetrics(false).withMaxFieldCacheSize(7)
                  .withProtocol(random_protocol(rng, 200)).withBuiltinProtocols().build();
    CHECK(r3->getConfig().maxFieldCacheSize == 7, "builder config");
    auto g3 = beatrice::gpu::GpuParserBuilder().withValidation(false).withPerformanceMetrics(false)
                  .withMaxFieldCacheSize(7).withProtocols(std::vector<ProtocolDefinition>{})
                  .withBuiltinProtocols(registry).build(0);
    // the builder's protocols: the same registry walk (r3 also holds the random table)
    std::vector<std::string> pr = r3->getSupportedProtocols(), pg = g3->getSupportedProtocols();
    for (const auto& n : pg) CHECK(r3->hasProtocol(n), "%s: builder protocol %s", label, n.c_str());
    CHECK(pr.size() == pg.size() + 1 && g3->getConfig().maxFieldCacheSize == 7 &&
              g3->getConfig().enableValidation == r3->getConfig().enableValidation &&
              g3->isProfilingEnabled() == r3->isProfilingEnabled(),
          "%s: ParserBuilder (%zu / %zu protocols)", label, pr.size(), pg.size());
    size_t nparse = 0;
    for (size_t i = 0; i < cap.packets.size() && i < 200; ++i) {
        const std::vector<uint8_t> v(cap.packets[i].data(), cap.packets[i].data() + cap.packets[i].length());
        for (const char* n : {"ethernet", "ipv4", "udp", "CUSTOM_PROTO", "no_such"}) {
            if (!same_result(label, i, r1->parsePacket(v, n), g1->parsePacket(v, n))) return false;
            if (!same_result(label, i, r3->parsePacket(v, n), g3->parsePacket(v, n))) return false;
            nparse += 2;
        }
    }
    std::printf("ok   surface %-22s formatPacket x5 formats (%zu texts, builtin + user tables with validation), "
                "serializePacket, formats, addCustom*, utilities, create / createWithProtocols / ParserBuilder "
                "(%zu ParseResults)\n", label, ntext, nparse);
    return true;
}

static bool plugin_case(const Capture& cap, const char* so) {
    setenv("BEATRICE_GPU_FILTERS", "proto|PROTOCOL|3|udp;net|IP_RANGE|2|10.0.0.0/8;ports|PORT_RANGE|1|1000-2000", 1);
    setenv("BEATRICE_GPU_BATCH", "4096", 1);
    setenv("BEATRICE_GPU_FLUSH_US", "100000000", 1);
    void* h = dlopen(so, RTLD_LAZY);   // PluginManager::loadPlugin (src/PluginManager.cpp:57-79)
    CHECK(h, "dlopen %s: %s", so, dlerror());
    using CreateFunc = beatrice::IPacketPlugin* (*)();
    auto create = reinterpret_cast<CreateFunc>(dlsym(h, "createPlugin"));
    auto flush = reinterpret_cast<void (*)(beatrice::IPacketPlugin*)>(dlsym(h, "gpu_plugin_flush"));
    auto passed = reinterpret_cast<uint64_t (*)(const beatrice::IPacketPlugin*)>(dlsym(h, "gpu_plugin_passed"));
    CHECK(create && flush && passed, "plugin symbols missing");
    std::unique_ptr<beatrice::IPacketPlugin> p(create());
    p->onStart();
    // four context threads call onPacket at once (src/BeatriceContext.cpp:215-278)
    {
        std::vector<std::thread> th;
        for (int w = 0; w < 4; ++w)
            th.emplace_back([&, w] {
                for (size_t i = w; i < cap.packets.size(); i += 4) p->onPacket(const_cast<Packet&>(cap.packets[i]));
            });
        for (auto& x : th) x.join();
    }
    flush(p.get());
    PacketFilter ref;
    install(ref, {{"proto", PacketFilter::FilterType::PROTOCOL, "udp", 3, true, 0},
                  {"net", PacketFilter::FilterType::IP_RANGE, "10.0.0.0/8", 2, true, 0},
                  {"ports", PacketFilter::FilterType::PORT_RANGE, "1000-2000", 1, true, 0}});
    uint64_t want = 0;
    for (const auto& pk : cap.packets) want += ref.applyFilters(pk).passed;
    CHECK(p->getProcessedPacketCount() == cap.packets.size(), "plugin processed %lu",
          (unsigned long)p->getProcessedPacketCount());
    CHECK(passed(p.get()) == want, "plugin passed %lu, reference %lu", (unsigned long)passed(p.get()),
          (unsigned long)want);
    CHECK(p->getName() == "gpu_parse_filter" && p->getErrorCount() == 0, "plugin identity/errors");
    p->onStop();
    p.reset();
    dlclose(h);
    std::printf("ok   plugin  createPlugin/onStart/onPacket x%zu on 4 threads/onStop, %lu passed\n", cap.packets.size(),
                (unsigned long)want);
    return true;
}

// ---- small calls: a single packet / a small batch is decided (parsed) on the host -------
// GpuPacketFilter::applyFilters(const Packet&) and batches below hostBatchBelow() run the
// compiled program on the calling thread; GpuProtocolParser::parsePacket extracts on it.
// Both branches (host, and the device with setHostBatchBelow(0)) against the reference.
static Capture load_capture(const char* path) {   // u64 n, n x u64 desc, u64 bytes, data
    Capture c;
    FILE* f = std::fopen(path, "rb");
    if (!f) return c;
    uint64_t n = 0, nb = 0;
    if (std::fread(&n, 8, 1, f) == 1) {
        c.desc.resize(n);
        if (std::fread(c.desc.data(), 8, n, f) == n && std::fread(&nb, 8, 1, f) == 1) {
            c.data.resize(nb + 64);
            if (std::fread(c.data.data(), 1, nb, f) != nb) c.desc.clear();
        }
    }
    std::fclose(f);
    for (uint64_t d : c.desc) {
        const uint8_t* fr = c.data.data() + (d & 0xFFFFFFFFFFFFull);
        c.packets.emplace_back(std::shared_ptr<const uint8_t[]>(fr, [](const uint8_t*) {}), (size_t)(d >> 48));
    }
    return c;
}

static bool small_filter_case(const char* label, const Capture& cap, const std::vector<Spec>& specs) {
    PacketFilter ref;
    GpuPacketFilter host(0), dev(0);   // host: default threshold; dev: every call on the device
    dev.setHostBatchBelow(0);
    install(ref, specs);
    install(host, specs);
    install(dev, specs);
    CHECK(host.hostBatchBelow() > 100, "%s: host threshold %zu", label, host.hostBatchBelow());
    size_t threw = 0;
    for (size_t i = 0; i < cap.packets.size(); ++i) {   // one packet per call
        PacketFilter::FilterResult a, b, c;
        std::exception_ptr ea, eb, ec;
        try { a = ref.applyFilters(cap.packets[i]); } catch (...) { ea = std::current_exception(); }
        try { b = host.applyFilters(cap.packets[i]); } catch (...) { eb = std::current_exception(); }
        if (i % 7 == 0) {   // the device branch is a round trip per packet: a sample
            try { c = dev.applyFilters(cap.packets[i]); } catch (...) { ec = std::current_exception(); }
            CHECK((bool)ea == (bool)ec && (!ea || what_kind(ea) == what_kind(ec)) &&
                      (ea || (a.passed == c.passed && a.filterName == c.filterName && a.reason == c.reason)),
                  "%s: device branch, packet %zu", label, i);
        }
        CHECK((bool)ea == (bool)eb, "%s: packet %zu exception ref=%d host=%d", label, i, (bool)ea, (bool)eb);
        if (ea) {
            CHECK(what_kind(ea) == what_kind(eb), "%s: packet %zu %s vs %s", label, i, what_kind(ea).c_str(),
                  what_kind(eb).c_str());
            ++threw;
            continue;
        }
        CHECK(a.passed == b.passed && a.filterName == b.filterName && a.reason == b.reason,
              "%s: packet %zu ref=(%d,%s) host=(%d,%s)", label, i, a.passed, a.filterName.c_str(), b.passed,
              b.filterName.c_str());
    }
    auto sa = ref.getStats(), sb = host.getStats();
    CHECK(sa.packetsProcessed == sb.packetsProcessed && sa.packetsPassed == sb.packetsPassed &&
              sa.packetsDropped == sb.packetsDropped && sa.filterCounts == sb.filterCounts,
          "%s: per-packet stats differ (processed %lu/%lu)", label, (unsigned long)sa.packetsProcessed,
          (unsigned long)sb.packetsProcessed);
    // small batches (host) and the same batches on the device; classify on filters of their own
    GpuPacketFilter hostc(0), devc(0);
    devc.setHostBatchBelow(0);
    install(hostc, specs);
    install(devc, specs);
    for (size_t lo = 0; lo < cap.packets.size(); lo += 100) {
        const std::vector<Packet> part(cap.packets.begin() + lo,
                                       cap.packets.begin() + std::min(cap.packets.size(), lo + 100));
        std::vector<PacketFilter::FilterResult> a, b, c;
        std::exception_ptr ea, eb, ec;
        try { a = ref.applyFilters(part); } catch (...) { ea = std::current_exception(); }
        try { b = host.applyFilters(part); } catch (...) { eb = std::current_exception(); }
        try { c = dev.applyFilters(part); } catch (...) { ec = std::current_exception(); }
        CHECK((bool)ea == (bool)eb && (bool)ea == (bool)ec, "%s: batch at %zu exceptions", label, lo);
        if (ea) {
            CHECK(what_kind(ea) == what_kind(eb) && what_kind(ea) == what_kind(ec), "%s: batch at %zu exception kind",
                  label, lo);
            continue;
        }
        for (size_t i = 0; i < a.size(); ++i)
            CHECK(a[i].passed == b[i].passed && a[i].filterName == b[i].filterName && a[i].passed == c[i].passed &&
                      a[i].filterName == c[i].filterName,
                  "%s: batch at %zu packet %zu", label, lo, i);
        GpuPacketFilter::Verdicts v = hostc.classify(part), w = devc.classify(part);
        CHECK(v.decide == w.decide && v.pass_idx == w.pass_idx, "%s: classify host/device at %zu", label, lo);
    }
    sa = ref.getStats();
    sb = host.getStats();
    CHECK(sa.packetsProcessed == sb.packetsProcessed && sa.packetsPassed == sb.packetsPassed &&
              sa.filterCounts == sb.filterCounts,
          "%s: stats after batches differ", label);
    std::printf("ok   small   %-22s %zu single-packet calls (%zu threw), batches of 100 on host and device\n", label,
                cap.packets.size(), threw);
    return true;
}

static bool small_parser_case(const char* label, const Capture& cap) {
    using namespace beatrice::parser;
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    ProtocolParser ref(cfg);
    beatrice::gpu::GpuProtocolParser host(cfg, 0), dev(cfg, 0);
    dev.setHostBatchBelow(0);
    for (auto p : {BuiltinProtocols::createEthernetProtocol(), BuiltinProtocols::createVLANProtocol(),
                   BuiltinProtocols::createIPv4Protocol(), BuiltinProtocols::createIPv6Protocol(),
                   BuiltinProtocols::createTCPProtocol(), BuiltinProtocols::createUDPProtocol(),
                   BuiltinProtocols::createICMPProtocol()}) {
        ref.registerProtocol(p);
        host.registerProtocol(p);
        dev.registerProtocol(p);
    }
    auto walk = host.parseBatch(cap.packets);
    size_t nres = 0;
    for (size_t i = 0; i < cap.packets.size(); ++i) {
        const uint8_t* f = cap.packets[i].data();
        const size_t len = cap.packets[i].length();
        for (const auto& L : walk.layers(i)) {   // parsePacket(slice, name) per walked layer
            const std::vector<uint8_t> v(f + L.offset, f + len);
            if (!same_result(label, i, ref.parsePacket(v, L.name), host.parsePacket(v, L.name))) return false;
            if (i % 5 == 0 && !same_result(label, i, ref.parsePacket(v, L.name), dev.parsePacket(v, L.name))) return false;
            ++nres;
        }
        const std::vector<uint8_t> v(f, f + len);   // every protocol over the whole frame (too-short ones too)
        auto w = ref.parsePacketMultipleProtocols(v), g = host.parsePacketMultipleProtocols(v);
        CHECK(w.size() == g.size(), "%s: multiple size", label);
        for (size_t k = 0; k < w.size(); ++k)
            if (!same_result(label, i, w[k], g[k])) return false;
    }
    std::printf("ok   small   parser %-15s %zu parsePacket(slice, name) calls on the host, a fifth on the device\n",
                label, nres);
    return true;
}

// A crash names where it happened (the test's stdout is a pipe, so its buffered lines are lost).
static void on_fatal(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    dprintf(2, "test_adapter: signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(frames, n, 2);
    _exit(128 + sig);
}

// A randomized round for `test_adapter fuzz`: one program on one capture through a fresh
// GpuPacketFilter (members contexts on device 0, a 4,096-packet staging chunk so batches span
// chunks) against the reference PacketFilter: the vector form (results, exception kind), the
// single-packet form on the first packets, classify's pass list, and the stats.
static bool fuzz_case(const char* label, const Capture& cap, const std::vector<Spec>& specs, int members) {
    PacketFilter ref;
    bt_opts o{};
    o.flags = members > 1 ? BT_OPT_GROUP_SHARED_DEVICE : 0u;
    o.host_chunk_packets = 4096;
    GpuPacketFilter gpu(std::vector<int>(members, 0), &o);
    install(ref, specs);
    install(gpu, specs);
    std::vector<PacketFilter::FilterResult> a, b;
    std::exception_ptr ea, eb;
    try { a = ref.applyFilters(cap.packets); } catch (...) { ea = std::current_exception(); }
    try { b = gpu.applyFilters(cap.packets); } catch (...) { eb = std::current_exception(); }
    CHECK((bool)ea == (bool)eb, "%s: exception mismatch ref=%d gpu=%d", label, (bool)ea, (bool)eb);
    if (ea) {
        CHECK(what_kind(ea) == what_kind(eb), "%s: %s vs %s", label, what_kind(ea).c_str(), what_kind(eb).c_str());
    } else {
        for (size_t i = 0; i < a.size(); ++i)
            CHECK(a[i].passed == b[i].passed && a[i].filterName == b[i].filterName && a[i].reason == b[i].reason,
                  "%s: packet %zu ref=(%d,%s) gpu=(%d,%s)", label, i, a[i].passed, a[i].filterName.c_str(), b[i].passed,
                  b[i].filterName.c_str());
        std::vector<uint32_t> want;
        for (size_t i = 0; i < a.size(); ++i)
            if (a[i].passed) want.push_back((uint32_t)i);
        const GpuPacketFilter::Verdicts v = gpu.classify(cap.packets);
        CHECK(v.pass_idx == want, "%s: classify pass list (%zu vs %zu)", label, v.pass_idx.size(), want.size());
        ref.applyFilters(cap.packets);   // the reference's stats count classify's packets too
    }
    for (size_t i = 0; i < std::min<size_t>(cap.packets.size(), 300); ++i) {
        PacketFilter::FilterResult x, y;
        std::exception_ptr ex, ey;
        try { x = ref.applyFilters(cap.packets[i]); } catch (...) { ex = std::current_exception(); }
        try { y = gpu.applyFilters(cap.packets[i]); } catch (...) { ey = std::current_exception(); }
        CHECK((bool)ex == (bool)ey && (!ex || what_kind(ex) == what_kind(ey)) &&
                  (ex || (x.passed == y.passed && x.filterName == y.filterName && x.reason == y.reason)),
              "%s: single packet %zu", label, i);
    }
    if (!ea) {
        const auto sa = ref.getStats(), sb = gpu.getStats();
        CHECK(sa.packetsProcessed == sb.packetsProcessed && sa.packetsPassed == sb.packetsPassed &&
                  sa.packetsDropped == sb.packetsDropped && sa.filterCounts == sb.filterCounts,
              "%s: stats differ (processed %lu/%lu passed %lu/%lu)", label, (unsigned long)sa.packetsProcessed,
              (unsigned long)sb.packetsProcessed, (unsigned long)sa.packetsPassed, (unsigned long)sb.packetsPassed);
    }
    return true;
}

static int fuzz_main(double seconds, uint64_t seed) {
    using T = PacketFilter::FilterType;
    std::mt19937_64 rng(seed);
    auto pick = [&](size_t n) { return (size_t)(rng() % n); };
    const std::vector<std::pair<T, std::vector<std::string>>> pools = {
        {T::BPF, {"", "tcp", "udp", "icmp", "not udp", "UDP", "tcp or udp", "ip", "xyz"}},
        {T::PROTOCOL, {"tcp", "udp", "icmp", "ip", "UDP", "", "foo"}},
        {T::IP_RANGE, {"10.0.0.0/8", "192.168.0.0/16", "0.0.0.0/0", "10.1.2.3", "10.0.0.0/33", "10.0.0.0/-1",
                       "266.0.0.0/8", "10.0.0", " 10.0.0.0/8", "abc", "10.0.0.0/x"}},
        {T::PORT_RANGE, {"1000-2000", "53", "0-65535", "2000-1000", "66770", "-5", "80-80", "abc", "1000-", "0-1023"}},
        {T::PAYLOAD, {"GET", "[\\x00-\\x1f][a-z]", "^..?\\d", "a|b", "\\d\\d", "(ab|cd)e", "x*y", ".", "[A-Z][a-z]+"}},
        {T::CUSTOM, {""}}};
    const char* names[] = {"a", "zeta", "m7", "q", "beta", "k2", "proto", "net", "ports", "x1", "hi", "c"};
    std::printf("fuzz seed %#llx, %.0f s\n", (unsigned long long)seed, seconds);
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
    int rounds = 0;
    while (std::chrono::steady_clock::now() < t_end || rounds < 4) {
        const int cfg = (int[]){3, 4, 9}[pick(3)];
        const uint32_t n = (uint32_t[]){1, 2047, 2048, 2049, 4097, (uint32_t)(1 + pick(6000))}[pick(6)];
        const Capture cap = capture(cfg, n, rng());
        std::vector<Spec> specs;
        const size_t m = 1 + pick(6);
        std::vector<size_t> used;
        for (size_t k = 0; k < m; ++k) {
            size_t ni = pick(12);
            while (std::find(used.begin(), used.end(), ni) != used.end()) ni = (ni + 1) % 12;
            used.push_back(ni);
            const auto& pool = pools[pick(pools.size())];
            Spec sp{names[ni], pool.first, pool.second[pick(pool.second.size())], (int)pick(6), pick(10) != 0, 0};
            if (sp.type == T::CUSTOM) sp.custom = 1 + (int)pick(3);
            specs.push_back(sp);
        }
        const int members = 1 + (int)pick(2);
        char label[96];
        std::snprintf(label, sizeof(label), "fuzz#%d cfg%d n%u m%zu g%d", rounds, cfg, n, m, members);
        // every 4th round with a capture of up to 1,500 packets: the parser's batch, layers,
        // formatters and detector on it against the reference's ProtocolParser
        if (rounds % 4 == 0 && n <= 1500 && !parser_case(label, cap)) break;
        if (!fuzz_case(label, cap, specs, members)) {
            for (const auto& sp : specs)
                std::printf("  spec %s type %d expr '%s' prio %d enabled %d custom %d\n", sp.name.c_str(), (int)sp.type,
                            sp.expr.c_str(), sp.priority, sp.enabled, sp.custom);
            break;
        }
        ++rounds;
        if (rounds % 25 == 0) std::printf("ok   fuzz %d rounds\n", rounds);
    }
    std::printf("%s: %d rounds (%d failures)\n", g_fail ? "FAILED" : "ALL OK", rounds, g_fail);
    return g_fail ? 1 : 0;
}

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);
    signal(SIGSEGV, on_fatal);
    signal(SIGABRT, on_fatal);
    using T = PacketFilter::FilterType;
    if (argc > 1 && std::string(argv[1]) == "fuzz")   // test_adapter fuzz [seconds] [seed]
        return fuzz_main(argc > 2 ? std::atof(argv[2]) : 10.0,
                         argc > 3 ? std::strtoull(argv[3], nullptr, 0) : (uint64_t)std::random_device{}());
    if (argc > 2 && std::string(argv[1]) == "small") {   // test_adapter small <capture.bin> <label>
        const Capture cap = load_capture(argv[2]);
        const char* label = argc > 3 ? argv[3] : argv[2];
        if (cap.packets.empty()) {
            std::printf("FAILED: cannot read %s\n", argv[2]);
            return 1;
        }
        const std::vector<Spec> sets[] = {
            {{"proto", T::PROTOCOL, "udp", 3, true, 0}, {"net", T::IP_RANGE, "10.0.0.0/8", 2, true, 0},
             {"ports", T::PORT_RANGE, "1000-2000", 1, true, 0}},
            {{"tcp", T::PROTOCOL, "tcp", 3, true, 0}, {"get", T::PAYLOAD, "GET|HTTP", 2, true, 0},
             {"cust", T::CUSTOM, "", 2, true, 1}, {"ports", T::PORT_RANGE, "0-2047", 1, true, 0}},
            {{"a", T::PORT_RANGE, "0-1023", 1, true, 0}, {"zeta", T::BPF, "tcp", 1, true, 0},
             {"q", T::PROTOCOL, "ip", 1, true, 0}, {"hi", T::BPF, "udp tcp", 5, true, 0}},
            {{"udp", T::BPF, "udp", 2, true, 0}, {"bad", T::IP_RANGE, "10.0.0.0/x", 1, true, 0}},
            {{"c", T::CUSTOM, "", 1, true, 3}, {"re", T::PAYLOAD, "(a|b)+c\\d", 2, true, 0}},
            {}};
        const char* names[] = {"headline", "payload+custom", "ties", "throw", "custom-throw+dfa", "none"};
        bool ok = true;
        for (int k = 0; k < 6; ++k) ok &= small_filter_case((std::string(label) + "/" + names[k]).c_str(), cap, sets[k]);
        ok &= small_parser_case(label, cap);
        std::printf("%s (%d failures)\n", ok && !g_fail ? "ALL OK" : "FAILED", g_fail);
        return ok && !g_fail ? 0 : 1;
    }
    const char* plugin_so = argc > 1 ? argv[1] : "beatrice_amd/libgpu_parse_filter_plugin.so";
    Capture c3 = capture(3, 20000, 0x5EED0003), c4 = capture(4, 12000, 0x5EED0004), fz = capture(9, 30000, 0x5EED0009);
    const std::vector<Spec> headline = {{"proto", T::PROTOCOL, "udp", 3, true, 0},
                                        {"net", T::IP_RANGE, "10.0.0.0/8", 2, true, 0},
                                        {"ports", T::PORT_RANGE, "1000-2000", 1, true, 0}};
    // equal priorities: the order comes from unordered_map iteration + std::sort
    const std::vector<Spec> ties = {{"a", T::PORT_RANGE, "0-1023", 1, true, 0},
                                    {"zeta", T::BPF, "tcp", 1, true, 0},
                                    {"m7", T::IP_RANGE, "10.0.0.0/9", 1, true, 0},
                                    {"q", T::PROTOCOL, "ip", 1, true, 0},
                                    {"beta", T::IP_RANGE, "192.168.0.0/17", 1, true, 0},
                                    {"k2", T::PORT_RANGE, "0-30000", 1, true, 0},
                                    {"off", T::BPF, "udp", 1, false, 0},
                                    {"hi", T::BPF, "udp tcp", 5, true, 0}};
    const std::vector<Spec> host_side = {{"tcp", T::PROTOCOL, "tcp", 3, true, 0},
                                         {"get", T::PAYLOAD, "GET|HTTP", 2, true, 0},
                                         {"cust", T::CUSTOM, "", 2, true, 1},
                                         {"ports", T::PORT_RANGE, "0-2047", 1, true, 0},
                                         {"nofn", T::CUSTOM, "x", 0, true, 0}};
    const std::vector<Spec> throws = {{"udp", T::BPF, "udp", 2, true, 0}, {"bad", T::IP_RANGE, "10.0.0.0/x", 1, true, 0}};
    const std::vector<Spec> throws_late = {{"tcp", T::PROTOCOL, "tcp", 9, true, 0},
                                           {"p", T::PORT_RANGE, "1000-2000", 5, true, 0},
                                           {"oor", T::PORT_RANGE, "99999999999", 1, true, 0}};
    const std::vector<Spec> custom_throw = {{"c", T::CUSTOM, "", 1, true, 3}};
    bool ok = true;
    ok &= filter_case("c3/headline", c3, headline);
    ok &= filter_case("c4/headline", c4, headline);
    ok &= filter_case("fuzz/headline", fz, headline);
    ok &= filter_case("fuzz/ties", fz, ties);
    ok &= filter_case("c3/ties-removed", c3, ties, {"m7", "q"});
    ok &= filter_case("fuzz/payload+custom", fz, host_side);
    ok &= filter_case("c4/payload+custom", c4, host_side);
    ok &= filter_case("fuzz/throw", fz, throws);
    ok &= filter_case("c3/throw-late", c3, throws_late);
    ok &= filter_case("c4/custom-throw", c4, custom_throw);
    ok &= filter_case("c3/no-filters", c3, {});
    // batches of >= 65536 packets take the parallel decision scan (a HOST code falls back to
    // the serial one; a throw stops the tally at the first throwing packet)
    {
        Capture big = capture(3, 300000, 0x5EED0033);
        ok &= filter_case("big/headline", big, headline);
        ok &= filter_case("big/throw-late", big, throws_late);
        ok &= filter_case("big/payload+custom", big, host_side);
        // a three-member group (one device standing in for three): split, merged, same results
        ok &= filter_case("group3/big/headline", big, headline, {}, 3);
        ok &= filter_case("group3/big/throw-late", big, throws_late, {}, 3);
        ok &= filter_case("group2/fuzz/payload+custom", fz, host_side, {}, 2);
    }
    ok &= concurrent_case("c3/headline", c3, headline, 8);
    ok &= concurrent_case("fuzz/payload+custom", fz, host_side, 6);
    // device-branch calls (>= 4096 packets) from 8 threads over two lanes on one device
    {
        Capture c3b = capture(3, 160000, 0x5EED0035), fzb = capture(9, 120000, 0x5EED0036);
        ok &= concurrent_case("c3/headline/lanes", c3b, headline, 8, 2, 4096);
        ok &= concurrent_case("fuzz/host-side/lanes", fzb, host_side, 6, 2, 4096);
    }
    ok &= parser_case("c3", c3);
    ok &= parser_case("c4", c4);
    ok &= parser_case("fuzz", fz);
    ok &= user_proto_case("fuzz", fz);
    ok &= user_proto_case("c3", c3);
    ok &= surface_case("c4", c4);
    ok &= surface_case("fuzz", fz);
    ok &= plugin_case(c3, plugin_so);
    std::printf("%s (%d failures)\n", ok && !g_fail ? "ALL OK" : "FAILED", g_fail);
    return ok && !g_fail ? 0 : 1;
}
