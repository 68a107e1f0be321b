// surface_bench.cpp — what an integrator gets from the drop-in C++ surfaces, timed next
// to the reference's own PacketFilter on the same host CPUs (VERDICT r02 "time what an
// integrator calls").
//
//   surface_bench [all|filter|ref|mt|parser|usertable|sizes|single|group|plugin|plugin-hot] [--packets N] [--seconds S] [--threads T]
//                 [--plugin SO] [--chunks 16384,65536] [--members 1,2,4] [--data-node none|auto|N]
//
// For C2 (64-B Eth/IPv4/UDP) and C3 (IMIX) frames held as std::vector<beatrice::Packet>
// (the reference's batch type, include/beatrice/Packet.hpp) and C3's 5-tuple filter set:
//   ref       beatrice::PacketFilter::applyFilters(const std::vector<Packet>&) — the
//             reference's batch entry (src/PacketFilter.cpp:121-130), compiled from its
//             own sources — on T threads, one PacketFilter per thread on its own shard
//             (and on 1 thread);
//   apply     GpuPacketFilter::applyFilters(const std::vector<Packet>&) -> vector<FilterResult>,
//             whole capture per call, with the split of the call into the device pass
//             (host gather -> H2D -> kernels -> D2H) and the host's FilterResult / stats work;
//   classify  GpuPacketFilter::classify(const std::vector<Packet>&) (decisions + pass list);
//   mt        the same two from T threads at once on ONE shared GpuPacketFilter, each thread
//             on its own shard in chunks (the reference's pattern above, one instance);
//   parser    ProtocolParser::parsePacket per walked layer against GpuProtocolParser::parseBatch
//             (records, ParseResults on demand, JSON text): bench_parser below;
//   usertable parser_example's user protocol table (BASELINE configs[0]) over the C2 frames:
//             parsePacket(frame, definition) against parseBatch(packets, definition);
//   single    one packet per call (applyFilters(const Packet&), parsePacket(slice, name)) and small
//             classify() batches, host branch against device branch: bench_single below;
//   group     one GpuPacketFilter over a device group of 1 / 2 / 4 members: bench_group below;
//   plugin-hot  the plugin fed by producers that copy each frame into a fresh buffer just
//             before onPacket (a capture backend's just-received frames);
//   plugin    libgpu_parse_filter_plugin.so through createPlugin(): onPacket from 1 and from
//             T threads (PluginManager::processPacket's per-packet call), until the verdict
//             sink has seen every packet.
// --data-node auto (or a node number) sets this process's memory policy to prefer the NUMA node
// nearest device 0 (bt_context_placement) before the captures are built, so the frames, the
// Packets and their control blocks sit where the host gather's pinned threads run
// (tools/e2e.py --data-node does the same for its buffers); default none: first touch.
// One JSON object per line. The parity of every surface is tests/cpp/test_adapter.cpp's
// and test_plugin.cpp's job; this tool only times them.
#include <dlfcn.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../beatrice_amd/host/GpuPacketFilter.hpp"
#include "../../beatrice_amd/host/GpuProtocolParser.hpp"
#include "parser/ProtocolParser.hpp"
#include "parser/ProtocolRegistry.hpp"
#include "beatrice/IPacketPlugin.hpp"
#include "beatrice/PacketFilter.hpp"
#include "beatrice_gpu_plugin.h"

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

extern "C" uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc);
extern "C" int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads);

using beatrice::Packet;
using beatrice::PacketFilter;
using beatrice::gpu::GpuPacketFilter;
using Clock = std::chrono::steady_clock;

namespace {

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// CPUs this process may use: the affinity set bounded by the cgroup v2 CPU quota.
int usable_cpus() {
    cpu_set_t set;
    int aff = 1;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) aff = CPU_COUNT(&set);
    std::ifstream f("/sys/fs/cgroup/cpu.max");
    std::string q, p;
    if (f >> q >> p && q != "max") {
        const int quota = (int)(std::stod(q) / std::stod(p));
        if (quota >= 1) return std::min(aff, quota);
    }
    return aff;
}

struct Capture {
    const char* name;
    std::vector<uint8_t> data;
    std::vector<uint64_t> desc;
    std::vector<Packet> packets;
};

Capture capture(const char* name, int cfg, uint32_t n, uint64_t seed) {
    Capture c;
    c.name = name;
    c.desc.resize(n);
    c.data.resize(bt_synth_layout(cfg, n, seed, c.desc.data()));
    bt_synth_fill(cfg, n, seed, c.desc.data(), c.data.data(), 16);
    c.packets.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = c.data.data() + (c.desc[i] & 0xFFFFFFFFFFFFull);
        c.packets.emplace_back(std::shared_ptr<const uint8_t[]>(f, [](const uint8_t*) {}), (size_t)(c.desc[i] >> 48));
    }
    return c;
}

const std::vector<std::tuple<std::string, int, int, std::string>> kC3Set = {
    {"proto", 1, 3, "udp"}, {"net", 2, 2, "10.0.0.0/8"}, {"ports", 3, 1, "1000-2000"}};

template <class F>
void add_set(F& f) {
    for (auto& [name, type, prio, expr] : kC3Set) {
        PacketFilter::FilterConfig c;
        c.type = static_cast<PacketFilter::FilterType>(type);
        c.priority = prio;
        c.expression = expr;
        f.addFilter(name, c);
    }
}

void line(const char* surface, const Capture& c, int threads, double pps, const std::string& extra = "") {
    std::printf("{\"surface\": \"%s\", \"config\": \"%s\", \"threads\": %d, \"mpps\": %.4f, \"packets\": %zu%s%s}\n",
                surface, c.name, threads, pps / 1e6, c.packets.size(), extra.empty() ? "" : ", ", extra.c_str());
    std::fflush(stdout);
}

// The reference's batch entry on T threads, each with its own PacketFilter and shard.
void bench_ref(const Capture& c, int threads, double seconds) {
    std::atomic<uint64_t> done{0};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    const auto t0 = Clock::now();
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            PacketFilter pf;
            add_set(pf);
            const size_t lo = c.packets.size() * t / threads, hi = c.packets.size() * (t + 1) / threads;
            const std::vector<Packet> shard(c.packets.begin() + lo, c.packets.begin() + hi);
            const size_t chunk = 4096;
            std::vector<Packet> part;
            for (size_t at = 0; !stop.load(std::memory_order_relaxed); at = (at + chunk) % shard.size()) {
                part.assign(shard.begin() + at, shard.begin() + std::min(shard.size(), at + chunk));
                auto r = pf.applyFilters(part);
                done += r.size();
                if (t == 0 && secs(t0, Clock::now()) > seconds) stop = true;
            }
        });
    for (auto& x : th) x.join();
    const double el = secs(t0, Clock::now());
    line("ref PacketFilter::applyFilters(vector<Packet>)", c, threads, done / el,
         "\"seconds\": " + std::to_string(el));
}

void bench_gpu_filter(const Capture& c, double seconds, const char* which) {
    GpuPacketFilter f;
    add_set(f);
    const bool apply = std::strcmp(which, "apply") == 0;
    // warm-up: device init, program compile, staging allocation
    if (apply) (void)f.applyFilters(c.packets);
    else (void)f.classify(c.packets);
    uint64_t done = 0, passed = 0;
    double dev_s = 0, host_s = 0;
    const auto t0 = Clock::now();
    while (secs(t0, Clock::now()) < seconds) {
        if (apply) {
            auto r = f.applyFilters(c.packets);
            done += r.size();
            passed += r.empty() ? 0 : r[0].passed;
        } else {
            auto v = f.classify(c.packets);
            done += v.decide.size();
            passed += v.pass_idx.size();
        }
        const auto tm = f.lastBatchTiming();
        dev_s += tm.device_s;
        host_s += tm.host_s;
    }
    const double el = secs(t0, Clock::now());
    char extra[256];
    std::snprintf(extra, sizeof(extra), "\"devices\": %u, \"device_pass_s\": %.4f, \"host_post_s\": %.4f, "
                  "\"seconds\": %.3f", f.deviceCount(), dev_s, host_s, el);
    line(apply ? "GpuPacketFilter::applyFilters(vector<Packet>) -> vector<FilterResult>"
               : "GpuPacketFilter::classify(vector<Packet>)",
         c, 0, done / el, extra);
    (void)passed;
}

// One GpuPacketFilter called from T threads at once, each on its own shard in chunks of
// `chunk` packets: the reference's multi-threaded pattern (bench_ref) against one shared
// filter instead of T private ones. Results are consumed and destroyed on the calling
// thread, as a caller's would be.
void bench_gpu_filter_mt(const Capture& c, int threads, size_t chunk, double seconds, const char* which) {
    GpuPacketFilter f;
    add_set(f);
    const bool apply = std::strcmp(which, "apply") == 0;
    (void)f.classify(std::vector<Packet>(c.packets.begin(), c.packets.begin() + std::min(c.packets.size(), chunk)));
    std::atomic<uint64_t> done{0};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    const auto t0 = Clock::now();
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            const size_t lo = c.packets.size() * t / threads, hi = c.packets.size() * (t + 1) / threads;
            const std::vector<Packet> shard(c.packets.begin() + lo, c.packets.begin() + hi);
            std::vector<Packet> part;
            uint64_t mine = 0;
            for (size_t at = 0; !stop.load(std::memory_order_relaxed); at = (at + chunk) % shard.size()) {
                part.assign(shard.begin() + at, shard.begin() + std::min(shard.size(), at + chunk));
                if (apply) mine += f.applyFilters(part).size();
                else mine += f.classify(part).decide.size();
                if (t == 0 && secs(t0, Clock::now()) > seconds) stop = true;
            }
            done += mine;
        });
    for (auto& x : th) x.join();
    const double el = secs(t0, Clock::now());
    char extra[160];
    std::snprintf(extra, sizeof(extra), "\"chunk\": %zu, \"shared_instance\": true, \"seconds\": %.3f", chunk, el);
    line(apply ? "GpuPacketFilter::applyFilters(vector<Packet>) -> vector<FilterResult>, T callers"
               : "GpuPacketFilter::classify(vector<Packet>), T callers",
         c, threads, done / el, extra);
}

// One caller, classify() over batches of growing size: the per-call time splits into a fixed
// cost (host gather start, copies, launch, the wait) and a per-packet cost.
void bench_call_sizes(const Capture& c, double seconds) {
    GpuPacketFilter f;
    add_set(f);
    for (size_t n : {1024u, 4096u, 16384u, 65536u, 262144u}) {
        if (n > c.packets.size()) break;
        const std::vector<Packet> part(c.packets.begin(), c.packets.begin() + n);
        (void)f.classify(part);
        uint64_t calls = 0;
        double dev = 0;
        const auto t0 = Clock::now();
        while (secs(t0, Clock::now()) < seconds / 5) {
            (void)f.classify(part);
            dev += f.lastBatchTiming().device_s;
            ++calls;
        }
        const double el = secs(t0, Clock::now());
        char extra[160];
        std::snprintf(extra, sizeof(extra), "\"batch\": %zu, \"us_per_call\": %.1f, \"device_pass_us\": %.1f", n,
                      el / calls * 1e6, dev / calls * 1e6);
        line("GpuPacketFilter::classify(vector<Packet>) by batch size", c, 1, (double)calls * n / el, extra);
    }
}

// The floor of any applyFilters(vector) -> vector<FilterResult>: constructing n results,
// filling them from per-slot strings (on T threads) and destroying them, with no filtering.
void bench_result_floor(const Capture& c, int threads, double seconds) {
    const std::string pass = "Packet passed all filters", rej = "Filter proto rejected packet", name = "ports";
    uint64_t done = 0;
    double build_s = 0, fill_s = 0, free_s = 0;
    const auto t0 = Clock::now();
    while (secs(t0, Clock::now()) < seconds) {
        const auto a = Clock::now();
        std::vector<PacketFilter::FilterResult> r(c.packets.size());
        const auto b = Clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                for (size_t i = r.size() * t / threads; i < r.size() * (t + 1) / threads; ++i) {
                    r[i].passed = i & 1;
                    r[i].filterName = name;
                    r[i].reason = (i & 1) ? pass : rej;
                }
            });
        for (auto& x : th) x.join();
        const auto d = Clock::now();
        { std::vector<PacketFilter::FilterResult> gone; gone.swap(r); }
        const auto e = Clock::now();
        build_s += secs(a, b);
        fill_s += secs(b, d);
        free_s += secs(d, e);
        done += c.packets.size();
    }
    const double el = secs(t0, Clock::now());
    char extra[200];
    std::snprintf(extra, sizeof(extra), "\"construct_s\": %.4f, \"fill_s\": %.4f, \"destroy_s\": %.4f, \"seconds\": %.3f",
                  build_s, fill_s, free_s, el);
    line("floor: vector<FilterResult>(n) + fill + destroy (no filtering)", c, threads, done / el, extra);
}

// The parser side. The reference's parse of a batch is ProtocolParser::parsePacket(slice,
// name) per walked layer (the bench's cpu_baseline, oracle/ref_harness.cpp), on T threads
// with a parser each; against it:
//   parseBatch         GpuProtocolParser::parseBatch(vector<Packet>): every packet's layer
//                      walk on the GPU, its bt_rec back on the host (records are the product)
//   parseBatch+layer   the same, then layer(i, k) -> the reference's ParseResult for every
//                      walked layer of every packet, on T threads (what a caller that wants
//                      ParseResult objects pays)
//   parseBatch+json    the same, then format(BT_FMT_JSON): the reference's toJsonString text
//                      of every walked layer of the batch
// The walk (layer names and offsets) the reference threads follow is taken from one GPU pass
// before their timing starts: their time is the parsePacket calls alone.
void bench_parser(const Capture& c, int threads, double seconds) {
    using namespace beatrice::parser;
    beatrice::gpu::GpuProtocolParser gp;
    const size_t n = std::min<size_t>(c.packets.size(), 1u << 20);
    const std::vector<Packet> pk(c.packets.begin(), c.packets.begin() + n);
    (void)gp.parseBatch(pk);   // warm-up: device init, staging
    struct Walk {
        uint32_t off;
        const char* name;
    };
    std::vector<std::vector<Walk>> walks(n);
    {
        const auto b = gp.parseBatch(pk);
        static const char* names[] = {"ethernet", "vlan", "ipv4", "ipv6", "tcp", "udp", "icmp"};
        for (size_t i = 0; i < n; ++i)
            for (const auto& l : b.layers(i))
                for (const char* nm : names)
                    if (l.name == nm) walks[i].push_back({(uint32_t)l.offset, nm});
    }
    size_t n_layers = 0;
    for (const auto& w : walks) n_layers += w.size();
    {   // the reference, T threads, one ProtocolParser each (metrics off, as the harness)
        std::atomic<uint64_t> done{0};
        std::atomic<bool> stop{false};
        std::vector<std::thread> th;
        const auto t0 = Clock::now();
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                ProtocolParser::ParserConfig cfg;
                cfg.enablePerformanceMetrics = false;
                ProtocolParser rp(cfg);
                rp.registerProtocol(BuiltinProtocols::createEthernetProtocol());
                rp.registerProtocol(BuiltinProtocols::createVLANProtocol());
                rp.registerProtocol(BuiltinProtocols::createIPv4Protocol());
                rp.registerProtocol(BuiltinProtocols::createIPv6Protocol());
                rp.registerProtocol(BuiltinProtocols::createTCPProtocol());
                rp.registerProtocol(BuiltinProtocols::createUDPProtocol());
                rp.registerProtocol(BuiltinProtocols::createICMPProtocol());
                const size_t lo = n * t / threads, hi = n * (t + 1) / threads;
                uint64_t mine = 0;
                for (size_t i = lo; !stop.load(std::memory_order_relaxed); i = i + 1 < hi ? i + 1 : lo) {
                    const uint8_t* f = pk[i].data();
                    const size_t len = pk[i].length();
                    for (const Walk& w : walks[i]) {
                        const std::vector<uint8_t> slice(f + w.off, f + len);
                        const ParseResult r = rp.parsePacket(slice, w.name);
                        (void)r;
                    }
                    ++mine;
                    if (t == 0 && (mine & 1023) == 0 && secs(t0, Clock::now()) > seconds) stop = true;
                }
                done += mine;
            });
        for (auto& x : th) x.join();
        const double el = secs(t0, Clock::now());
        char extra[128];
        std::snprintf(extra, sizeof(extra), "\"layers_per_packet\": %.3f, \"seconds\": %.3f", (double)n_layers / n, el);
        line("ref ProtocolParser::parsePacket per walked layer", c, threads, done / el, extra);
    }
    auto timed = [&](const char* what, int mode) {
        uint64_t done = 0;
        double dev_s = 0, post_s = 0;
        const auto t0 = Clock::now();
        while (secs(t0, Clock::now()) < seconds) {
            const auto a = Clock::now();
            const auto b = gp.parseBatch(pk);
            const auto m = Clock::now();
            if (mode == 1) {
                std::vector<std::thread> th;
                for (int t = 0; t < threads; ++t)
                    th.emplace_back([&, t] {
                        for (size_t i = n * t / threads; i < n * (t + 1) / threads; ++i) {
                            const size_t k = walks[i].size();
                            for (size_t j = 0; j < k; ++j) {
                                const ParseResult r = b.layer(i, j);
                                (void)r;
                            }
                        }
                    });
                for (auto& x : th) x.join();
            } else if (mode == 2) {
                const std::string text = b.format(BT_FMT_JSON);
                if (text.empty()) std::abort();
            }
            dev_s += secs(a, m);
            post_s += secs(m, Clock::now());
            done += n;
        }
        const double el = secs(t0, Clock::now());
        char extra[160];
        std::snprintf(extra, sizeof(extra), "\"parse_batch_s\": %.4f, \"host_post_s\": %.4f, \"seconds\": %.3f", dev_s,
                      post_s, el);
        line(what, c, mode == 1 ? threads : 0, done / el, extra);
    };
    timed("GpuProtocolParser::parseBatch(vector<Packet>) -> records", 0);
    timed("GpuProtocolParser::parseBatch + layer(i,k) ParseResult for every walked layer", 1);
    timed("GpuProtocolParser::parseBatch + format(BT_FMT_JSON) of the batch", 2);
}

// BASELINE configs[0]'s path through the C++ API: parser_example's CUSTOM_PROTO table
// (examples/parser_example.cpp:18-22: header u32 @0, version u8 @4, length u16 @5, data
// BYTES[10] @7) over every frame. The reference: ProtocolParser::parsePacket(frame, definition)
// per packet on T threads, a parser each (metrics off, as oracle/ref_harness.cpp); against it
// GpuProtocolParser::parseBatch(packets, definition) (the GPU's status / value / byte columns),
// alone and with result(i) — the reference's ParseResult — for every packet on T threads.
void bench_usertable(const Capture& c, int threads, double seconds) {
    using namespace beatrice::parser;
    ProtocolDefinition def("CUSTOM_PROTO", "1.0");
    def.addField(FieldFactory::createUInt32Field("header", 0, Endianness::NETWORK, true, "Protocol header"));
    def.addField(FieldFactory::createUInt8Field("version", 4, true, "Protocol version"));
    def.addField(FieldFactory::createUInt16Field("length", 5, Endianness::NETWORK, true, "Data length"));
    def.addField(FieldFactory::createBytesField("data", 7, 10, "Payload data"));
    const size_t n = std::min<size_t>(c.packets.size(), 1u << 20);
    const std::vector<Packet> pk(c.packets.begin(), c.packets.begin() + n);
    {
        std::atomic<uint64_t> done{0};
        std::atomic<bool> stop{false};
        std::vector<std::thread> th;
        const auto t0 = Clock::now();
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                ProtocolParser::ParserConfig cfg;
                cfg.enablePerformanceMetrics = false;
                ProtocolParser rp(cfg);
                const size_t lo = n * t / threads, hi = n * (t + 1) / threads;
                uint64_t mine = 0;
                for (size_t i = lo; !stop.load(std::memory_order_relaxed); i = i + 1 < hi ? i + 1 : lo) {
                    const std::vector<uint8_t> frame(pk[i].data(), pk[i].data() + pk[i].length());
                    const ParseResult r = rp.parsePacket(frame, def);
                    (void)r;
                    ++mine;
                    if (t == 0 && (mine & 1023) == 0 && secs(t0, Clock::now()) > seconds) stop = true;
                }
                done += mine;
            });
        for (auto& x : th) x.join();
        const double el = secs(t0, Clock::now());
        char extra[64];
        std::snprintf(extra, sizeof(extra), "\"seconds\": %.3f", el);
        line("ref ProtocolParser::parsePacket(frame, CUSTOM_PROTO definition)", c, threads, done / el, extra);
    }
    ProtocolParser::ParserConfig cfg;
    cfg.enablePerformanceMetrics = false;
    beatrice::gpu::GpuProtocolParser gp(cfg, 0);
    (void)gp.parseBatch(pk, def);   // warm-up
    for (int mode = 0; mode < 2; ++mode) {
        uint64_t done = 0;
        double dev_s = 0, post_s = 0;
        const auto t0 = Clock::now();
        while (secs(t0, Clock::now()) < seconds) {
            const auto a = Clock::now();
            const auto b = gp.parseBatch(pk, def);
            const auto m = Clock::now();
            if (mode == 1) {
                std::vector<std::thread> th;
                for (int t = 0; t < threads; ++t)
                    th.emplace_back([&, t] {
                        for (size_t i = n * t / threads; i < n * (t + 1) / threads; ++i) {
                            const ParseResult r = b.result(i);
                            (void)r;
                        }
                    });
                for (auto& x : th) x.join();
            }
            dev_s += secs(a, m);
            post_s += secs(m, Clock::now());
            done += n;
        }
        const double el = secs(t0, Clock::now());
        char extra[160];
        std::snprintf(extra, sizeof(extra), "\"parse_batch_s\": %.4f, \"host_post_s\": %.4f, \"seconds\": %.3f", dev_s,
                      post_s, el);
        line(mode ? "GpuProtocolParser::parseBatch(packets, CUSTOM_PROTO) + result(i) ParseResult for every packet"
                  : "GpuProtocolParser::parseBatch(packets, CUSTOM_PROTO) -> status / value / byte columns",
             c, mode ? threads : 0, done / el, extra);
    }
}

// Single-packet calls and small batches (VERDICT r03 "stop charging single-packet callers a
// device round trip"): the reference's per-packet entries on one thread against the drop-in's
// host branch (the compiled program / extractor on the calling thread) and its device branch
// (setHostBatchBelow(0): one device round trip per call); then classify() by batch size on
// both branches, which places the default threshold (kHostBelowDefault).
void bench_single(const Capture& c, double seconds) {
    using namespace beatrice::parser;
    const size_t n = std::min<size_t>(c.packets.size(), 1u << 16);
    auto per_packet = [&](const char* what, auto&& call, size_t limit) {
        uint64_t done = 0;
        (void)call(c.packets[0]);
        const auto t0 = Clock::now();
        for (size_t i = 0; secs(t0, Clock::now()) < seconds; i = (i + 1) % std::min(n, limit)) {
            call(c.packets[i]);
            ++done;
        }
        const double el = secs(t0, Clock::now());
        char extra[96];
        std::snprintf(extra, sizeof(extra), "\"us_per_call\": %.3f, \"seconds\": %.3f", el / done * 1e6, el);
        line(what, c, 1, done / el, extra);
    };
    {
        PacketFilter ref;
        add_set(ref);
        per_packet("ref PacketFilter::applyFilters(const Packet&)", [&](const Packet& p) { return ref.applyFilters(p).passed; },
                   n);
        GpuPacketFilter host, dev;
        add_set(host);
        add_set(dev);
        dev.setHostBatchBelow(0);
        per_packet("GpuPacketFilter::applyFilters(const Packet&), host branch",
                   [&](const Packet& p) { return host.applyFilters(p).passed; }, n);
        per_packet("GpuPacketFilter::applyFilters(const Packet&), device round trip",
                   [&](const Packet& p) { return dev.applyFilters(p).passed; }, n);
        for (size_t b : {1u, 4u, 16u, 64u, 256u, 512u, 1024u, 4096u}) {
            const std::vector<Packet> part(c.packets.begin(), c.packets.begin() + std::min(n, (size_t)b));
            for (int branch = 0; branch < 2; ++branch) {
                GpuPacketFilter& f = branch ? dev : host;
                (void)f.classify(part);
                uint64_t calls = 0;
                const auto t0 = Clock::now();
                while (secs(t0, Clock::now()) < seconds / 8) {
                    (void)f.classify(part);
                    ++calls;
                }
                const double el = secs(t0, Clock::now());
                char extra[128];
                std::snprintf(extra, sizeof(extra), "\"batch\": %zu, \"branch\": \"%s\", \"us_per_call\": %.2f", part.size(),
                              branch ? "device" : "host", el / calls * 1e6);
                line("GpuPacketFilter::classify(vector<Packet>) small batch", c, 1, (double)calls * part.size() / el,
                     extra);
            }
        }
    }
    {   // parsePacket(slice, name) per walked layer: the reference, the host branch, the device
        ProtocolParser::ParserConfig cfg;
        cfg.enablePerformanceMetrics = false;
        ProtocolParser rp(cfg);
        beatrice::gpu::GpuProtocolParser hp(cfg, 0), dp(cfg, 0);
        dp.setHostBatchBelow(0);
        for (auto pr : {BuiltinProtocols::createEthernetProtocol(), BuiltinProtocols::createVLANProtocol(),
                        BuiltinProtocols::createIPv4Protocol(), BuiltinProtocols::createIPv6Protocol(),
                        BuiltinProtocols::createTCPProtocol(), BuiltinProtocols::createUDPProtocol(),
                        BuiltinProtocols::createICMPProtocol()}) {
            rp.registerProtocol(pr);
            hp.registerProtocol(pr);
            dp.registerProtocol(pr);
        }
        const std::vector<Packet> pk(c.packets.begin(), c.packets.begin() + n);
        const auto b = hp.parseBatch(pk);
        std::vector<std::pair<std::vector<uint8_t>, std::string>> slices;
        for (size_t i = 0; i < n && slices.size() < 200000; ++i)
            for (const auto& l : b.layers(i))
                slices.emplace_back(std::vector<uint8_t>(pk[i].data() + l.offset, pk[i].data() + pk[i].length()), l.name);
        auto per_layer = [&](const char* what, auto&& parse, size_t limit) {
            uint64_t done = 0;
            const auto t0 = Clock::now();
            for (size_t i = 0; secs(t0, Clock::now()) < seconds; i = (i + 1) % std::min(slices.size(), limit)) {
                const ParseResult r = parse(slices[i].first, slices[i].second);
                (void)r;
                ++done;
            }
            const double el = secs(t0, Clock::now());
            char extra[96];
            std::snprintf(extra, sizeof(extra), "\"us_per_layer\": %.3f, \"seconds\": %.3f", el / done * 1e6, el);
            line(what, c, 1, done / el, extra);   // mpps here = M layers / s
        };
        per_layer("ref ProtocolParser::parsePacket(slice, name), layers",
                  [&](const std::vector<uint8_t>& v, const std::string& nm) { return rp.parsePacket(v, nm); }, slices.size());
        per_layer("GpuProtocolParser::parsePacket(slice, name), host branch, layers",
                  [&](const std::vector<uint8_t>& v, const std::string& nm) { return hp.parsePacket(v, nm); }, slices.size());
        per_layer("GpuProtocolParser::parsePacket(slice, name), device round trip, layers",
                  [&](const std::vector<uint8_t>& v, const std::string& nm) { return dp.parsePacket(v, nm); }, slices.size());
    }
}

// An in-process device group (bt_group) behind one GpuPacketFilter: classify() of the whole
// capture from one caller and from T callers, for groups of `members` contexts (on device 0 when
// the box has fewer GPUs: "shared_device"), with the process's CPU time per million packets.
void bench_group(const Capture& c, int threads, double seconds, const std::vector<int>& member_counts) {
    int ndev = 0;
    (void)bt_device_count(&ndev);
    for (int m : member_counts) {
        const bool shared = ndev < m;
        std::vector<int> devs;
        for (int k = 0; k < m; ++k) devs.push_back(shared ? 0 : k);
        bt_opts o{};
        if (shared) o.flags = BT_OPT_GROUP_SHARED_DEVICE;
        GpuPacketFilter f(devs, &o);
        add_set(f);
        (void)f.classify(c.packets);
        for (int callers : {1, threads}) {
            std::atomic<uint64_t> done{0};
            std::atomic<bool> stop{false};
            const double cpu0 = (double)std::clock() / CLOCKS_PER_SEC;
            const auto t0 = Clock::now();
            std::vector<std::thread> th;
            const size_t chunk = callers == 1 ? c.packets.size() : 65536;
            for (int t = 0; t < callers; ++t)
                th.emplace_back([&, t] {
                    const size_t lo = c.packets.size() * t / callers, hi = c.packets.size() * (t + 1) / callers;
                    const std::vector<Packet> shard(c.packets.begin() + lo, c.packets.begin() + hi);
                    std::vector<Packet> part;
                    uint64_t mine = 0;
                    for (size_t at = 0; !stop.load(std::memory_order_relaxed); at = (at + chunk) % shard.size()) {
                        if (chunk >= shard.size()) {   // one call over the whole shard: no copy of it per call
                            mine += f.classify(shard).decide.size();
                        } else {
                            part.assign(shard.begin() + at, shard.begin() + std::min(shard.size(), at + chunk));
                            mine += f.classify(part).decide.size();
                        }
                        if (t == 0 && secs(t0, Clock::now()) > seconds) stop = true;
                    }
                    done += mine;
                });
            for (auto& x : th) x.join();
            const double el = secs(t0, Clock::now());
            const double cpu = (double)std::clock() / CLOCKS_PER_SEC - cpu0;
            char extra[200];
            std::snprintf(extra, sizeof(extra),
                          "\"members\": %d, \"shared_device\": %s, \"chunk\": %zu, \"host_cpu_s_per_mpkt\": %.4f, "
                          "\"seconds\": %.3f", m, shared ? "true" : "false", chunk, cpu / (done / 1e6), el);
            line("GpuPacketFilter(group)::classify(vector<Packet>)", c, callers, done / el, extra);
        }
    }
}

// hot: each producer copies the frame into a fresh heap buffer right before onPacket, as a
// capture backend hands over a just-received frame (the reference's AF_PacketBackend: recv()
// + a heap copy per packet, src/AF_PacketBackend.cpp:318-363; GpuAfPacketBackend copies each
// frame into its own Packet the same way): the frame's bytes are in the producer's cache when
// the plugin sees them, which is what BEATRICE_GPU_PACK (copying the prefix at onPacket) needs.
// the job cgroup's throttled time (cgroup v2 cpu.stat), -1 when not readable
long long cgroup_throttled_usec() {
    FILE* f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
    if (!f) return -1;
    char key[64];
    long long v, out = -1;
    while (std::fscanf(f, "%63s %lld", key, &v) == 2)
        if (!std::strcmp(key, "throttled_usec")) out = v;
    std::fclose(f);
    return out;
}

void bench_plugin(const Capture& c, int threads, double seconds, const char* so, bool hot = false) {
    void* h = dlopen(so, RTLD_LAZY);
    if (!h) {
        std::fprintf(stderr, "dlopen %s: %s\n", so, dlerror());
        std::exit(3);
    }
    auto create = reinterpret_cast<beatrice::IPacketPlugin* (*)()>(dlsym(h, "createPlugin"));
    auto set_sink = reinterpret_cast<void (*)(gpu_plugin*, gpu_verdict_sink_fn, void*)>(dlsym(h, "gpu_plugin_set_sink"));
    auto flush = reinterpret_cast<void (*)(gpu_plugin*)>(dlsym(h, "gpu_plugin_flush"));
    setenv("BEATRICE_GPU_FILTERS", "proto|PROTOCOL|3|udp;net|IP_RANGE|2|10.0.0.0/8;ports|PORT_RANGE|1|1000-2000;", 1);
    if (!getenv("BEATRICE_GPU_BATCH")) setenv("BEATRICE_GPU_BATCH", "65536", 1);
    beatrice::IPacketPlugin* p = create();
    p->onStart();
    std::atomic<uint64_t> seen{0};
    set_sink(p, [](void* u, const gpu_verdict_batch* b) { *static_cast<std::atomic<uint64_t>*>(u) += b->n; }, &seen);
    auto feed = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            if (hot) {
                const size_t len = c.packets[i].length();
                std::shared_ptr<uint8_t[]> b(new uint8_t[len]);
                std::memcpy(b.get(), c.packets[i].data(), len);
                Packet pk(std::shared_ptr<const uint8_t[]>(std::move(b)), len);
                try {
                    p->onPacket(pk);
                } catch (const std::exception&) {
                }
                continue;
            }
            Packet pk = c.packets[i];
            try {
                p->onPacket(pk);   // PluginManager::processPacket (src/PluginManager.cpp:158-171)
            } catch (const std::exception&) {
            }
        }
    };
    feed(0, std::min<size_t>(c.packets.size(), 70000));   // warm-up: device init
    flush(p);
    while (seen < std::min<size_t>(c.packets.size(), 70000)) std::this_thread::yield();
    seen = 0;
    // every thread feeds its shard over and over for `seconds` (steady state: the pending
    // shards have grown, the device pass is warm), then the last partial batches are flushed
    std::atomic<uint64_t> fed{0};
    std::atomic<bool> stop{false};
    struct rusage ru0, ru1;
    getrusage(RUSAGE_SELF, &ru0);
    const long long thr0 = cgroup_throttled_usec();
    const auto t0 = Clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            const size_t lo = c.packets.size() * t / threads, hi = c.packets.size() * (t + 1) / threads;
            const size_t step = 16384;
            uint64_t mine = 0;
            for (size_t at = lo; !stop.load(std::memory_order_relaxed); at = at + step < hi ? at + step : lo) {
                const size_t e = std::min(hi, at + step);
                feed(at, e);
                mine += e - at;
                if (t == 0 && secs(t0, Clock::now()) > seconds) stop = true;
            }
            fed += mine;
        });
    for (auto& x : th) x.join();
    const auto t_fed = Clock::now();
    flush(p);
    while (seen < fed) std::this_thread::yield();
    const auto t1 = Clock::now();
    getrusage(RUSAGE_SELF, &ru1);
    const long long thr1 = cgroup_throttled_usec();
    auto tv = [](const timeval& a) { return a.tv_sec + a.tv_usec * 1e-6; };
    const double cpu_s = tv(ru1.ru_utime) - tv(ru0.ru_utime) + tv(ru1.ru_stime) - tv(ru0.ru_stime);
    char extra[400];
    std::snprintf(extra, sizeof(extra), "\"onPacket_s\": %.4f, \"seconds\": %.4f, \"fed\": %llu, \"batch\": %s, "
                  "\"hot_frames\": %s, \"pack\": \"%s\", \"cpu_s\": %.3f, \"sys_s\": %.3f, \"minflt\": %ld, "
                  "\"cgroup_throttled_ms\": %.1f, \"plugin\": \"%s\"", secs(t0, t_fed), secs(t0, t1), (unsigned long long)fed.load(),
                  getenv("BEATRICE_GPU_BATCH"), hot ? "true" : "false", getenv("BEATRICE_GPU_PACK") ? getenv("BEATRICE_GPU_PACK") : "0",
                  cpu_s, tv(ru1.ru_stime) - tv(ru0.ru_stime), ru1.ru_minflt - ru0.ru_minflt,
                  thr0 >= 0 && thr1 >= 0 ? (thr1 - thr0) / 1e3 : -1.0, so);
    line(hot ? "plugin onPacket (hot frames: heap copy per packet) -> verdict sink" : "plugin onPacket -> verdict sink", c,
         threads, fed / secs(t0, t1), extra);
    p->onStop();
    set_sink(p, nullptr, nullptr);
    delete p;
}

}  // namespace

int main(int argc, char** argv) {
    std::string what = argc > 1 ? argv[1] : "all";
    uint32_t n2 = 1u << 22, n3 = 1u << 21;
    double seconds = 3.0;
    int threads = usable_cpus();
    const char* so = "beatrice_amd/libgpu_parse_filter_plugin.so";
    std::vector<size_t> chunks = {16384, 65536};
    std::vector<int> members = {1, 2, 4};
    std::string data_node = "none";
    int node = -1;
    for (int i = 2; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--packets")) n2 = n3 = (uint32_t)std::atol(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--seconds")) seconds = std::atof(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--threads")) threads = std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--plugin")) so = argv[i + 1];
        else if (!std::strcmp(argv[i], "--data-node")) {
            data_node = argv[i + 1];
            if (data_node != "auto" && data_node != "none") node = std::atoi(argv[i + 1]);
        }
        else if (!std::strcmp(argv[i], "--members")) {   // comma-separated group sizes of "group"
            members.clear();
            for (const char* q = argv[i + 1]; *q;) {
                members.push_back(std::atoi(q));
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
        else if (!std::strcmp(argv[i], "--chunks")) {   // comma-separated chunk sizes of the T-caller runs
            chunks.clear();
            for (const char* q = argv[i + 1]; *q;) {
                chunks.push_back((size_t)std::atol(q));
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
    }
    if (data_node == "auto") {
        bt_ctx* ctx = nullptr;
        bt_placement pl{};
        node = bt_create(0, nullptr, &ctx) == BT_OK && bt_context_placement(ctx, &pl) == BT_OK ? pl.numa_node : -1;
        bt_destroy(ctx);
    }
    if (node >= 0 && node < 64) {   // MPOL_PREFERRED: allocations go to `node` while it has room
        const unsigned long mask = 1ul << node;
        if (syscall(SYS_set_mempolicy, 1, &mask, 64) != 0) node = -1;
    }
    std::fprintf(stderr, "surface_bench: %d usable CPUs, data node %d\n", threads, node);
    const Capture caps[2] = {capture("c2", 2, n2, 0xC2), capture("c3", 3, n3, 0xC3)};
    for (const Capture& c : caps) {
        if (what == "all" || what == "filter" || what == "ref") {
            bench_ref(c, 1, seconds);
            bench_ref(c, threads, seconds);
        }
        if (what == "all" || what == "filter") {
            bench_result_floor(c, std::min(threads, 8), seconds);
            bench_gpu_filter(c, seconds, "apply");
            bench_gpu_filter(c, seconds, "classify");
        }
        if (what == "all" || what == "filter" || what == "mt") {
            for (size_t ch : chunks) {
                bench_gpu_filter_mt(c, threads, ch, seconds, "apply");
                bench_gpu_filter_mt(c, threads, ch, seconds, "classify");
            }
        }
        if (what == "all" || what == "parser") bench_parser(c, threads, seconds);
        if ((what == "all" || what == "usertable") && c.name == std::string("c2")) bench_usertable(c, threads, seconds);
        if (what == "all" || what == "sizes") bench_call_sizes(c, seconds);
        if (what == "all" || what == "single") bench_single(c, seconds);
        if (what == "all" || what == "group") bench_group(c, threads, seconds, members);
        if (what == "plugin-hot") {   // 1 / 8 / 16 producers writing each frame right before onPacket
            bench_plugin(c, 1, seconds, so, true);
            if (threads >= 8) bench_plugin(c, 8, seconds, so, true);
            bench_plugin(c, threads, seconds, so, true);
        }
        if (what == "all" || what == "plugin") {
            bench_plugin(c, 1, seconds, so);
            if (threads >= 4) bench_plugin(c, threads / 2, seconds, so);   // producers leave CPUs to the plugin
            bench_plugin(c, threads, seconds, so);
        }
    }
    return 0;
}
