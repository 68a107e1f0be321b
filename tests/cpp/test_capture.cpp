// test_capture.cpp — the TPACKET_V3 capture layer (beatrice_amd/host/GpuCapture.*,
// TpacketRing.*) against the reference.
//
//   test_capture backend
//       CPU, needs CAP_NET_RAW. GpuAfPacketBackend (ICaptureBackend drop-in):
//       the reference AF_PacketBackend's initialize / start error results, then a live
//       capture on `lo` — every datagram sent arrives through getPackets with its
//       bytes intact, the callback sees every packet, the statistics count them.
//   test_capture stage <ring.bin> <block_size> <n_blocks>
//       GPU. A ring image (tests/golden/ring_lo.npz, written by the kernel) attached to
//       a TpacketV3Ring and drained by GpuTpacketStage one block at a time; for each
//       batch the decisions, pass indices and verdict bits equal the reference
//       PacketFilter::applyFilters on the same frames (PAYLOAD, CUSTOM and a throwing
//       filter set included), the stats equal the reference's, and every block is handed
//       back to the kernel.
//   test_capture stage-synth
//       GPU. The same on a 300k-frame C3 capture packed into a ring (bt_synth_tpv3_pack).
// Prints one line per check; exit status 0 = all passed.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "beatrice/PacketFilter.hpp"
#include "../../beatrice_amd/host/GpuCapture.hpp"

extern "C" uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc);
extern "C" int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads);
extern "C" uint64_t bt_synth_tpv3_pack(const uint8_t* data, const uint64_t* desc, uint64_t n, uint64_t block_size,
                                       uint8_t* ring, uint64_t ring_blocks, uint64_t* ring_desc, uint64_t* blocks_used);

using beatrice::ErrorCode;
using beatrice::Packet;
using beatrice::PacketFilter;
using beatrice::gpu::GpuAfPacketBackend;
using beatrice::gpu::GpuPacketFilter;
using beatrice::gpu::GpuTpacketStage;
using beatrice::gpu::TpacketV3Ring;

static std::atomic<int> g_fail{0};
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

// ------------------------------------------------------------------ backend (CPU)

static bool backend_errors() {
    GpuAfPacketBackend b;
    auto r = b.start();
    CHECK(r.isError() && r.getErrorCode() == ErrorCode::INITIALIZATION_FAILED &&
              r.getErrorMessage() == "AF_PACKET backend not initialized",
          "start before initialize: %s", r.getErrorMessage().c_str());
    GpuAfPacketBackend::Config c;
    c.interface = "";
    r = b.initialize(c);
    CHECK(r.isError() && r.getErrorCode() == ErrorCode::INVALID_ARGUMENT && r.getErrorMessage() == "Invalid interface: ",
          "empty interface: %s", r.getErrorMessage().c_str());
    c.interface = "bt-no-such0";
    r = b.initialize(c);
    CHECK(r.isError() && r.getErrorCode() == ErrorCode::INITIALIZATION_FAILED &&
              r.getErrorMessage() == "Failed to bind to interface",
          "missing interface: %s", r.getErrorMessage().c_str());
    CHECK(b.getLastError().rfind("Failed to get interface index", 0) == 0, "lastError: %s", b.getLastError().c_str());
    CHECK(!b.isHealthy() && b.healthCheck().isError(), "health of an uninitialised backend");
    std::printf("ok   backend errors          start/initialize results match the reference\n");
    return true;
}

static bool backend_loopback() {
    GpuAfPacketBackend b;
    GpuAfPacketBackend::Config c;
    c.interface = "lo";
    auto r = b.initialize(c);
    CHECK(r.isSuccess(), "initialize(lo): %s / %s", r.getErrorMessage().c_str(), b.getLastError().c_str());
    std::atomic<uint64_t> seen{0};
    b.setPacketCallback([&](Packet) { seen++; });
    CHECK(b.start().isSuccess() && b.isRunning(), "start");
    const int kSend = 400;
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    sockaddr_in to{};
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    std::set<std::string> want;
    for (int i = 0; i < kSend; ++i) {
        char mark[32];
        std::snprintf(mark, sizeof(mark), "btcap-%05d", i);
        std::string payload;
        for (int k = 0; k <= i % 9; ++k) payload += mark;
        to.sin_port = htons((uint16_t)(6000 + i % 50));
        sendto(s, payload.data(), payload.size(), 0, reinterpret_cast<sockaddr*>(&to), sizeof(to));
        want.insert(mark);
    }
    close(s);
    uint64_t got = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (!want.empty() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
        for (const Packet& p : b.getPackets(64, std::chrono::milliseconds(200))) {
            ++got;
            const std::string body(reinterpret_cast<const char*>(p.data()), p.length());
            const size_t at = body.find("btcap-");
            if (at != std::string::npos && at + 11 <= body.size()) {
                // the UDP payload is intact: it repeats its own marker 1 + i % 9 times
                const std::string mark = body.substr(at, 11);
                const int i = std::atoi(mark.c_str() + 6);
                std::string expect;
                for (int k = 0; k <= i % 9; ++k) expect += mark;
                CHECK(body.compare(at, std::string::npos, expect) == 0, "payload of %s damaged", mark.c_str());
                CHECK(p.length() == at + expect.size(), "frame length of %s: %zu vs %zu", mark.c_str(), p.length(), at + expect.size());
                want.erase(mark);
            }
        }
    }
    CHECK(want.empty(), "%zu of %d datagrams never arrived", want.size(), kSend);
    CHECK(b.stop().isSuccess() && !b.isRunning(), "stop");
    const auto st = b.getStatistics();
    CHECK(st.packetsCaptured >= (uint64_t)kSend && seen.load() == st.packetsCaptured,
          "stats: captured %lu callback %lu", (unsigned long)st.packetsCaptured, (unsigned long)seen.load());
    CHECK(got <= st.packetsCaptured, "queue handed out more than captured");
    std::printf("ok   backend loopback        %d datagrams via getPackets, %lu frames captured, callback saw all\n",
                kSend, (unsigned long)st.packetsCaptured);
    return true;
}

// ------------------------------------------------------------------ stage (GPU)

struct Spec {
    std::string name;
    PacketFilter::FilterType type;
    std::string expr;
    int priority;
    int custom;   // 0 none, 1 len % 3 != 0
};

template <class F>
static void install(F& f, const std::vector<Spec>& specs) {
    for (const auto& s : specs) {
        PacketFilter::FilterConfig c;
        c.type = s.type;
        c.expression = s.expr;
        c.priority = s.priority;
        f.addFilter(s.name, c);
        if (s.custom) f.setCustomFilter(s.name, [](const Packet& p) { return p.length() % 3 != 0; });
    }
}

static std::string kind_of(const std::exception_ptr& e) {
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

static const std::vector<Spec> kHeadline = {{"proto", PacketFilter::FilterType::PROTOCOL, "udp", 3, 0},
                                            {"net", PacketFilter::FilterType::IP_RANGE, "10.0.0.0/8", 2, 0},
                                            {"ports", PacketFilter::FilterType::PORT_RANGE, "1000-2000", 1, 0}};
static const std::vector<Spec> kLoopback = {{"bpf", PacketFilter::FilterType::BPF, "udp", 4, 0},
                                            {"lo", PacketFilter::FilterType::IP_RANGE, "127.0.0.0/8", 3, 0},
                                            {"pay", PacketFilter::FilterType::PAYLOAD, "v6|btc|\\x01", 2, 0},
                                            {"odd", PacketFilter::FilterType::CUSTOM, "", 1, 1}};
static const std::vector<Spec> kHost = {{"tcp", PacketFilter::FilterType::BPF, "tcp", 3, 0},
                                        {"get", PacketFilter::FilterType::PAYLOAD, "GET|HTTP", 2, 0},
                                        {"len", PacketFilter::FilterType::CUSTOM, "", 1, 1}};
static const std::vector<Spec> kThrow = {{"udp", PacketFilter::FilterType::PROTOCOL, "udp", 2, 0},
                                         {"bad", PacketFilter::FilterType::PORT_RANGE, "1000-", 1, 0}};

// A filter over `members` contexts of device 0 (a group sharing the one GPU of the test box:
// each member still has its own streams and host threads and reads its range of every batch).
static bt_opts shared_opts() {
    bt_opts o{};
    o.flags = BT_OPT_GROUP_SHARED_DEVICE;
    return o;
}

static bool stage_case(const char* label, uint8_t* ring_mem, uint32_t bs, uint32_t nb, const std::vector<Spec>& specs,
                       uint32_t maxBlocks, bool records, bool gather = false, uint32_t inPlaceEvery = 0,
                       uint32_t members = 1) {
    // fresh copy of the image: the stage hands blocks back (status -> kernel)
    std::vector<uint8_t> mem(ring_mem, ring_mem + (size_t)bs * nb);
    TpacketV3Ring ring;
    CHECK(ring.attach(mem.data(), bs, nb).isSuccess(), "%s: attach", label);
    const bt_opts so = shared_opts();
    GpuPacketFilter gpu(std::vector<int>(members, 0), &so);
    CHECK(gpu.deviceCount() == members, "%s: %u members", label, gpu.deviceCount());
    PacketFilter ref;
    install(gpu, specs);
    install(ref, specs);
    const auto order = gpu.evaluationOrder();
    GpuTpacketStage::Options o;
    o.maxBlocks = maxBlocks;
    o.maxPackets = 1u << 20;
    o.records = records;
    o.gather = gather;
    o.inPlaceEvery = inPlaceEvery;
    GpuTpacketStage stage(gpu, ring, o);
    uint64_t total = 0, passed = 0;
    uint32_t batches = 0, gathered = 0;
    for (;;) {
        std::vector<Packet> pk;
        std::exception_ptr eg, er;
        const GpuTpacketStage::Batch* b = nullptr;
        try {
            b = &stage.poll(std::chrono::milliseconds(0));
        } catch (...) {
            eg = std::current_exception();
        }
        if (eg) {
            // the reference throws the same on the same frames: rebuild them from the ring
            uint32_t n = 0;
            std::vector<bt_pkt_desc> d(1u << 20);
            const bt_tpv3_ring g = ring.ring();
            uint32_t taken = 0;
            bt_ring_walk_tpv3(nullptr, &g, ring.cursor(), maxBlocks, d.data(), (uint32_t)d.size(), &n, &taken);
            for (uint32_t i = 0; i < n; ++i)
                pk.emplace_back(std::shared_ptr<const uint8_t[]>(mem.data() + BT_DESC_OFF(d[i]), [](const uint8_t*) {}),
                                (size_t)BT_DESC_LEN(d[i]));
            try { ref.applyFilters(pk); } catch (...) { er = std::current_exception(); }
            CHECK(er && kind_of(er) == kind_of(eg), "%s: gpu threw %s, reference %s", label, kind_of(eg).c_str(),
                  er ? kind_of(er).c_str() : "nothing");
            std::printf("ok   stage %-20s threw %s like the reference\n", label, kind_of(eg).c_str());
            return true;
        }
        if (b->n == 0 && b->blocks == 0) break;
        ++batches;
        gathered += b->gathered;
        CHECK(b->gathered == (gather && !(inPlaceEvery && batches % inPlaceEvery == 0)), "%s: batch %u gathered=%d",
              label, batches, b->gathered);
        for (uint32_t i = 0; i < b->n; ++i)
            pk.emplace_back(std::shared_ptr<const uint8_t[]>(stage.frame(i), [](const uint8_t*) {}),
                            (size_t)stage.length(i));
        std::vector<PacketFilter::FilterResult> a;
        try { a = ref.applyFilters(pk); } catch (...) { er = std::current_exception(); }
        CHECK(!er, "%s: reference threw %s but the stage did not", label, kind_of(er).c_str());
        size_t k = 0;
        for (uint32_t i = 0; i < b->n; ++i) {
            const uint32_t code = b->decide[i] >> 6, slot = b->decide[i] & 63u;
            const bool pass = code == BT_DECIDE_PASS;
            const std::string name = order.empty() ? "" : (pass ? order.back() : order[slot]);
            CHECK(a[i].passed == pass && a[i].filterName == name, "%s: frame %u ref=(%d,%s) gpu=(%d,%s)", label, i,
                  a[i].passed, a[i].filterName.c_str(), pass, name.c_str());
            CHECK((((b->verdict[i / 64] >> (i % 64)) & 1) != 0) == pass, "%s: verdict bit %u", label, i);
            if (pass) {
                CHECK(k < b->pass.size() && b->pass[k] == i, "%s: pass index %zu", label, k);
                ++k;
            }
        }
        CHECK(k == b->pass.size(), "%s: pass list length", label);
        if (records) {   // records equal a direct host-path run of the same frames
            std::vector<const uint8_t*> ptr(b->n);
            std::vector<uint32_t> len(b->n);
            for (uint32_t i = 0; i < b->n; ++i) {
                ptr[i] = stage.frame(i);
                len[i] = stage.length(i);
            }
            std::vector<bt_rec> direct(b->n);
            CHECK(bt_parse_filter_ptrs(gpu.context(), ptr.data(), len.data(), b->n, direct.data(), nullptr, nullptr,
                                       nullptr, nullptr) == BT_OK, "%s: direct run", label);
            for (uint32_t i = 0; i < b->n; ++i) {
                const bt_rec r = stage.record(i);
                CHECK(std::memcmp(&r, &direct[i], sizeof(r)) == 0, "%s: record %u differs", label, i);
            }
        }
        total += b->n;
        passed += b->pass.size();
        stage.release();
    }
    const bt_tpv3_ring g = ring.ring();
    for (uint32_t blk = 0; blk < nb; ++blk) {
        const auto* bd = reinterpret_cast<const uint32_t*>(static_cast<uint8_t*>(g.base) + (size_t)blk * bs);
        CHECK(bd[2] == 0, "%s: block %u not handed back (status %u)", label, blk, bd[2]);
    }
    const auto sa = ref.getStats(), sb = gpu.getStats();
    CHECK(sa.packetsProcessed == sb.packetsProcessed && sa.packetsPassed == sb.packetsPassed &&
              sa.packetsDropped == sb.packetsDropped && sa.filterCounts == sb.filterCounts,
          "%s: stats differ (processed %lu/%lu passed %lu/%lu)", label, (unsigned long)sa.packetsProcessed,
          (unsigned long)sb.packetsProcessed, (unsigned long)sa.packetsPassed, (unsigned long)sb.packetsPassed);
    CHECK(total > 0, "%s: nothing drained", label);
    CHECK(!gather || gathered > 0, "%s: no batch was gathered", label);
    std::printf("ok   stage %-24s %lu frames in %u batches (%u gathered), %lu passed%s, %u device(s)\n", label,
                (unsigned long)total, batches, gathered, (unsigned long)passed, records ? ", records equal" : "",
                members);
    return true;
}

// Per-GPU ring sharding: PACKET_FANOUT_HASH gives each GPU worker its own ring, a
// flow always landing in the same one. Here a capture is split by the kernel's flow hash
// stand-in (the 5-tuple's symmetric sum) into `rings` ring images, each drained by its own
// filter + GpuTpacketStage on its own thread (its own context on the test box's one GPU),
// and every ring's decisions are checked against the reference PacketFilter; together the
// rings must see every frame once.
static uint32_t flow_of(const uint8_t* f, uint32_t len) {
    if (len < 38 || f[12] != 0x08 || f[13] != 0x00) return 0;
    uint32_t h = (uint32_t)f[23];
    for (int i = 26; i < 34; ++i) h += f[i];
    for (int i = 34; i < 38; ++i) h += f[i];
    return h * 2654435761u;
}

static bool stage_fanout(uint32_t rings) {
    const uint32_t n = 200000, bs = 1u << 20;
    std::vector<uint64_t> desc(n);
    std::vector<uint8_t> data(bt_synth_layout(3, n, 91, desc.data()));
    bt_synth_fill(3, n, 91, desc.data(), data.data(), 8);
    // per ring: the frames of its flows, packed in capture order
    std::vector<std::vector<uint64_t>> part(rings);
    std::vector<std::vector<uint8_t>> bytes(rings);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = data.data() + BT_DESC_OFF(desc[i]);
        const uint32_t len = (uint32_t)BT_DESC_LEN(desc[i]);
        const uint32_t r = flow_of(f, len) % rings;
        part[r].push_back(BT_DESC(bytes[r].size(), len));
        bytes[r].insert(bytes[r].end(), f, f + len);
    }
    std::vector<std::vector<uint8_t>> ringmem(rings);
    std::vector<uint64_t> used(rings, 0);
    for (uint32_t r = 0; r < rings; ++r) {
        bt_synth_tpv3_pack(bytes[r].data(), part[r].data(), part[r].size(), bs, nullptr, 1ull << 40, nullptr, &used[r]);
        ringmem[r].resize(used[r] * bs);
        CHECK(bt_synth_tpv3_pack(bytes[r].data(), part[r].data(), part[r].size(), bs, ringmem[r].data(), used[r], nullptr,
                                 &used[r]) == part[r].size(), "fanout: ring %u packing", r);
    }
    std::vector<int> ok(rings, 0);
    std::vector<std::thread> th;
    for (uint32_t r = 0; r < rings; ++r)
        th.emplace_back([&, r] {
            char label[64];
            std::snprintf(label, sizeof(label), "fanout %u/%u", r, rings);
            ok[r] = stage_case(label, ringmem[r].data(), bs, (uint32_t)used[r], kHeadline, 8, r == 0);
        });
    for (auto& t : th) t.join();
    size_t total = 0;
    for (uint32_t r = 0; r < rings; ++r) total += part[r].size();
    CHECK(total == n, "fanout: %zu frames over the rings, %u captured", total, n);
    for (uint32_t r = 0; r < rings; ++r) CHECK(ok[r], "fanout: ring %u", r);
    std::printf("ok   fanout  %u rings, one stage + context each, %u frames once each\n", rings, n);
    return true;
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "backend") {
        backend_errors();
        backend_loopback();
    } else if (mode == "stage" && argc == 5) {
        std::ifstream in(argv[2], std::ios::binary);
        std::vector<uint8_t> img((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        const uint32_t bs = (uint32_t)std::stoul(argv[3]), nb = (uint32_t)std::stoul(argv[4]);
        if (img.size() != (size_t)bs * nb) {
            std::printf("FAIL ring image is %zu bytes, expected %u x %u\n", img.size(), bs, nb);
            return 1;
        }
        stage_case("lo/headline", img.data(), bs, nb, kHeadline, 1, true);
        stage_case("lo/payload+custom", img.data(), bs, nb, kLoopback, 2, false);
        stage_case("lo/host-slots", img.data(), bs, nb, kHost, 16, false);
        stage_case("lo/throws", img.data(), bs, nb, kThrow, 1, false);
        stage_case("lo/no-filters", img.data(), bs, nb, {}, 3, false);
        stage_case("lo/headline gathered", img.data(), bs, nb, kHeadline, 1, true, true);
        stage_case("lo/payload+custom g", img.data(), bs, nb, kLoopback, 2, false, true, 2);
        stage_case("lo/throws gathered", img.data(), bs, nb, kThrow, 1, false, true);
        stage_case("lo/headline 2 dev", img.data(), bs, nb, kHeadline, 4, true, false, 0, 2);
        stage_case("lo/payload+custom 3 dev", img.data(), bs, nb, kLoopback, 4, false, false, 0, 3);
        stage_case("lo/throws 2 dev", img.data(), bs, nb, kThrow, 4, false, false, 0, 2);
        stage_case("lo/headline g 3 dev", img.data(), bs, nb, kHeadline, 4, true, true, 2, 3);
    } else if (mode == "stage-fanout") {
        stage_fanout(2);
        stage_fanout(3);
    } else if (mode == "stage-synth") {
        const uint32_t n = 300000, bs = 1u << 20;
        std::vector<uint64_t> desc(n);
        std::vector<uint8_t> data(bt_synth_layout(3, n, 77, desc.data()));
        bt_synth_fill(3, n, 77, desc.data(), data.data(), 8);
        uint64_t used = 0;
        bt_synth_tpv3_pack(data.data(), desc.data(), n, bs, nullptr, 1ull << 40, nullptr, &used);
        std::vector<uint8_t> ring(used * bs);
        const uint64_t packed = bt_synth_tpv3_pack(data.data(), desc.data(), n, bs, ring.data(), used, nullptr, &used);
        if (packed != n) {
            std::printf("FAIL packed %lu of %u\n", (unsigned long)packed, n);
            return 1;
        }
        stage_case("c3/headline", ring.data(), bs, (uint32_t)used, kHeadline, 8, true);
        stage_case("c3/host-slots", ring.data(), bs, (uint32_t)used, kHost, 32, false);
        stage_case("c3/headline gathered", ring.data(), bs, (uint32_t)used, kHeadline, 8, true, true);
        stage_case("c3/host-slots mixed", ring.data(), bs, (uint32_t)used, kHost, 8, false, true, 3);
        stage_case("c3/headline 2 dev", ring.data(), bs, (uint32_t)used, kHeadline, 8, true, false, 0, 2);
        stage_case("c3/headline 3 dev", ring.data(), bs, (uint32_t)used, kHeadline, 16, true, false, 0, 3);
        stage_case("c3/host-slots 2 dev", ring.data(), bs, (uint32_t)used, kHost, 32, false, false, 0, 2);
        stage_case("c3/headline g 2 dev", ring.data(), bs, (uint32_t)used, kHeadline, 8, true, true, 2, 2);
    } else {
        std::printf("usage: test_capture backend | stage <ring.bin> <block_size> <n_blocks> | stage-synth | "
                    "stage-fanout\n");
        return 2;
    }
    if (g_fail) {
        std::printf("%d FAILED\n", g_fail.load());
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
