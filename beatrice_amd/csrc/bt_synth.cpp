// bt_synth.cpp — deterministic synthetic captures for the BASELINE.json configs.
//
// Stand-in for a capture backend's batch (reference ICaptureBackend::getPackets,
// include/beatrice/ICaptureBackend.hpp:49-50): frames packed into one buffer plus
// one bt_pkt_desc per frame. Used by bench.py (16M-packet batches), the GPU parity
// tests and the golden-fixture script. Generation is split into 64Ki-packet blocks,
// each with its own std::mt19937_64 seeded from (seed, block), so it is parallel and
// bit-reproducible.
//
//   cfg 2  C1/C2: fixed 64 B Eth/IPv4/UDP (SURVEY.md §8(d) "C2 inputs")
//   cfg 3  C3: IMIX 64/512/1500 (7:4:1), 25 % 802.1Q, TCP/UDP 50/50, IHL 5
//   cfg 4  C4: 50 % QinQ / 25 % 802.1Q / 25 % untagged, IPv6 or IPv4 with IHL 5..15,
//              TCP data offset 5..15, lengths 64..1500, frames at 2-mod-4 offsets
//   cfg 9  fuzz: short/odd frames, random EtherTypes/IHL/protocols, byte mutations
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <sys/socket.h>
#include <linux/if_packet.h>
#include <random>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kBlock = 65536;

uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Rng {
    std::mt19937_64 g;
    Rng(uint64_t seed, uint64_t block, uint64_t stream) : g(splitmix(seed ^ splitmix(block * 4 + stream))) {}
    uint64_t u64() { return g(); }
    uint32_t below(uint32_t n) { return (uint32_t)(((g() >> 32) * (uint64_t)n) >> 32); }
    uint32_t range(uint32_t lo, uint32_t hi) { return lo + below(hi - lo + 1); }  // inclusive
};

uint32_t align_of(int cfg) {
    switch (cfg) {
    case 2: return 64;
    case 3: return 64;
    case 4: return 4;    // then +2: AF_PACKET-style 2-mod-4 frame starts
    default: return 1;
    }
}

// Structural choices of frame i (tags, L3/L4 kinds, IHL, data offset), drawn from a
// per-frame hash so the layout pass can clamp lengths to the header size.
struct Shape {
    uint32_t nv = 0, tp0 = 0x8100, tp1 = 0x8100, tp2 = 0x8100;
    uint32_t l3 = 0x0800, l4 = 17, ihl = 5, doff = 5;
};

Shape shape_of(int cfg, uint64_t seed, uint64_t i) {
    Shape s;
    uint64_t h = splitmix(seed * 0x2545F4914F6CDD1Dull + i * 0x9E3779B97F4A7C15ull + 12345);
    auto take = [&](uint32_t n) { uint32_t v = (uint32_t)(h % n); h /= n; return v; };
    if (cfg == 3) {
        s.nv = take(4) == 0 ? 1 : 0;
        s.l4 = take(2) ? 6 : 17;
    } else if (cfg == 4) {
        uint32_t x = take(4);
        s.nv = x < 2 ? 2 : x == 2 ? 1 : 0;
        if (s.nv == 2) s.tp0 = 0x88A8;
        s.l3 = take(2) ? 0x86DD : 0x0800;
        s.l4 = take(2) ? 6 : 17;
        s.ihl = 5 + take(11);
        s.doff = 5 + take(11);
    } else if (cfg == 9) {
        static const uint32_t ets[] = {0x0800, 0x0800, 0x0800, 0x86DD, 0x86DD, 0x8100, 0x88A8, 0x0806, 0x0000, 0xFFFF};
        uint32_t e = ets[take(10)];
        while ((e == 0x8100 || e == 0x88A8) && s.nv < 3) {
            uint32_t tp = take(2) ? 0x8100 : 0x88A8;
            (s.nv == 0 ? s.tp0 : s.nv == 1 ? s.tp1 : s.tp2) = tp;
            ++s.nv;
            e = ets[take(10)];
        }
        s.l3 = e;
        static const uint32_t ps[] = {6, 6, 17, 17, 1, 0, 58, 255};
        s.l4 = ps[take(8)];
        s.ihl = take(4) == 0 ? take(16) : 5;
        s.doff = take(16);
    }
    return s;
}

uint32_t header_len(const Shape& s) {
    uint32_t o3 = 14 + 4 * s.nv;
    if (s.l3 == 0x0800) {
        uint32_t o4 = o3 + 4 * std::max<uint32_t>(s.ihl, 5);
        return o4 + (s.l4 == 6 ? 4 * std::max<uint32_t>(s.doff, 5) : 8);
    }
    if (s.l3 == 0x86DD) return o3 + 40 + (s.l4 == 6 ? 4 * std::max<uint32_t>(s.doff, 5) : 8);
    return o3;
}

uint32_t frame_len(int cfg, Rng& r, const Shape& s) {
    switch (cfg) {
    case 2: return 64;
    case 3: { uint32_t x = r.below(12); return x < 7 ? 64 : x < 11 ? 512 : 1500; }
    case 4: return std::max(r.range(64, 1500), header_len(s));
    default: {
        uint32_t x = r.below(10);
        if (x < 5) return r.range(0, 80);
        if (x < 8) return r.range(81, 200);
        return r.range(201, 1600);
    }
    }
}

void be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
void be32(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; }
void rnd(uint8_t* p, uint32_t n, Rng& r) { for (uint32_t i = 0; i < n; i += 8) { uint64_t v = r.u64(); std::memcpy(p + i, &v, std::min<uint32_t>(8, n - i)); } }

void ipv4_csum(uint8_t* ip, uint32_t hlen) {
    ip[10] = ip[11] = 0;
    uint32_t s = 0;
    for (uint32_t i = 0; i < hlen; i += 2) s += ((uint32_t)ip[i] << 8) | ip[i + 1];
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    be16(ip + 10, ~s & 0xFFFF);
}

const uint8_t* pattern() {
    static uint8_t pat[4096 + 256];
    static bool init = [] {
        for (int i = 0; i < (int)sizeof(pat); ++i) pat[i] = (uint8_t)(i * 131 + 7);
        return true;
    }();
    (void)init;
    return pat;
}

// Builds one frame of `len` bytes at p (len may be < the header size: truncated).
void build(int cfg, const Shape& s, uint8_t* p, uint32_t len, uint64_t idx, Rng& r) {
    uint8_t h[256];
    std::memset(h, 0, sizeof(h));
    uint32_t hl = 0;
    rnd(h, 12, r);                                   // dst/src MAC
    uint32_t nv = s.nv, et_pos = 12;
    uint32_t l3 = s.l3, l4 = s.l4, ihl = s.ihl, doff = s.doff;
    bool fuzz = cfg == 9;
    for (uint32_t k = 0; k < nv; ++k) {
        uint32_t tp = k == 0 ? s.tp0 : k == 1 ? s.tp1 : s.tp2;
        be16(h + et_pos, tp);
        be16(h + et_pos + 2, (uint32_t)r.u64() & 0xFFFF);
        et_pos += 4;
    }
    be16(h + et_pos, l3);
    uint32_t o3 = et_pos + 2, o4 = o3;
    if (l3 == 0x0800) {
        uint8_t* ip = h + o3;
        ip[0] = (uint8_t)(0x40 | ihl);
        ip[1] = fuzz ? (uint8_t)r.u64() : 0;
        be16(ip + 2, len > o3 ? len - o3 : 0);
        be16(ip + 4, (uint32_t)r.u64() & 0xFFFF);
        be16(ip + 6, 0x4000);
        ip[8] = 64;
        ip[9] = (uint8_t)l4;
        be32(ip + 12, 0x0A000000u | ((uint32_t)r.u64() & 0xFFFFFF));   // 10.0.0.0/8
        be32(ip + 16, 0xC0A80000u | ((uint32_t)r.u64() & 0xFFFF));     // 192.168.0.0/16
        if (fuzz && r.below(3) == 0) { be32(ip + 12, (uint32_t)r.u64()); be32(ip + 16, (uint32_t)r.u64()); }
        uint32_t ihb = std::max<uint32_t>(ihl, 5) * 4;
        if (ihb > 20) rnd(ip + 20, ihb - 20, r);   // options
        ipv4_csum(ip, ihb);
        o4 = o3 + ihl * 4;
        hl = o3 + ihb;
    } else if (l3 == 0x86DD) {
        uint8_t* ip = h + o3;
        be32(ip, 0x60000000u | ((uint32_t)r.u64() & 0x0FFFFFFF));
        be16(ip + 4, len > o3 + 40 ? len - o3 - 40 : 0);
        ip[6] = (uint8_t)l4;
        ip[7] = 64;
        rnd(ip + 8, 32, r);
        o4 = o3 + 40;
        hl = o4;
    } else {
        rnd(h + o3, 40, r);
        hl = o3 + 40;
        l4 = 0;
    }
    if (l4 == 6 || l4 == 17 || l4 == 1) {
        uint8_t* t = h + o4;
        uint32_t sport = (uint32_t)r.u64() & 0xFFFF, dport = r.below(4096);
        if (fuzz && r.below(2)) dport = (uint32_t)r.u64() & 0xFFFF;
        if (l4 == 6) {
            be16(t, sport); be16(t + 2, dport);
            be32(t + 4, (uint32_t)r.u64()); be32(t + 8, (uint32_t)r.u64());
            t[12] = (uint8_t)(doff << 4);
            t[13] = (uint8_t)r.u64();
            be16(t + 14, (uint32_t)r.u64() & 0xFFFF);
            be16(t + 16, (uint32_t)r.u64() & 0xFFFF);
            be16(t + 18, 0);
            uint32_t db = std::max<uint32_t>(doff, 5) * 4;
            if (db > 20) rnd(t + 20, db - 20, r);
            hl = o4 + db;
        } else if (l4 == 17) {
            be16(t, sport); be16(t + 2, dport);
            be16(t + 4, len > o4 ? len - o4 : 0);
            be16(t + 6, 0);
            hl = o4 + 8;
        } else {
            t[0] = (uint8_t)r.below(20); t[1] = 0;
            be16(t + 2, (uint32_t)r.u64() & 0xFFFF);
            be16(t + 4, (uint32_t)r.u64() & 0xFFFF);
            be16(t + 6, (uint32_t)r.u64() & 0xFFFF);
            hl = o4 + 8;
        }
    }
    if (fuzz) {   // a few byte mutations anywhere in the first 64 bytes
        uint32_t m = r.below(4);
        for (uint32_t k = 0; k < m; ++k) h[r.below(64)] = (uint8_t)r.u64();
        if (hl < 64) hl = 64;
    }
    uint32_t nh = std::min<uint32_t>(hl, len);
    std::memcpy(p, h, nh);
    if (len > nh) {   // payload: cheap deterministic pattern; some frames carry HTTP text
        const uint8_t* pat = pattern();
        uint32_t pl = len - nh, o = (uint32_t)(idx & 255);
        static const char http[] = "GET /index.html HTTP/1.1\r\nHost: beatrice\r\n";
        uint32_t done = 0;
        if ((fuzz || cfg == 4) && (idx % 8) == 3) {
            done = std::min<uint32_t>(pl, sizeof(http) - 1);
            std::memcpy(p + nh, http, done);
        }
        while (done < pl) {
            uint32_t c = std::min<uint32_t>(pl - done, 4096);
            std::memcpy(p + nh + done, pat + o, c);
            done += c;
        }
    }
}

}  // namespace

extern "C" {

// Lengths and offsets for n frames; fills desc (n entries) when non-NULL and returns
// the data-buffer size in bytes (rounded up to 256).
uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc) {
    uint64_t off = 0;
    uint32_t a = align_of(cfg);
    uint64_t nb = (n + kBlock - 1) / kBlock;
    for (uint64_t b = 0; b < nb; ++b) {
        Rng r(seed, b, 0);
        uint64_t lo = b * kBlock, hi = std::min(n, lo + kBlock);
        for (uint64_t i = lo; i < hi; ++i) {
            uint32_t len = frame_len(cfg, r, shape_of(cfg, seed, i));
            uint64_t start = off + (cfg == 4 ? 2 : 0);
            if (desc) desc[i] = start | ((uint64_t)len << 48);
            uint64_t end = start + len;
            off = (end + a - 1) / a * a;
        }
    }
    return (off + 255) / 256 * 256;
}

// Fills frames [lo, hi) of the capture described by desc; frame i goes to
// data + (offset_i - data_off). lo must be a multiple of the 65536-frame RNG block, so a
// capture filled range by range is identical to one filled at once (bench.py streams
// large captures to the device this way instead of holding them whole on the host).
int bt_synth_fill_range(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint64_t lo, uint64_t hi,
                        uint8_t* data, uint64_t data_off, int nthreads) {
    if (lo % kBlock || hi > n || lo > hi) return 1;
    const uint64_t b0 = lo / kBlock, b1 = (hi + kBlock - 1) / kBlock;
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([=] {
            for (uint64_t b = b0 + (uint64_t)t; b < b1; b += (uint64_t)nthreads) {
                Rng r(seed, b, 1);
                const uint64_t a = b * kBlock, e = std::min(hi, a + kBlock);
                for (uint64_t i = a; i < e; ++i) {
                    const uint64_t d = desc[i];
                    build(cfg, shape_of(cfg, seed, i), data + ((d & 0xFFFFFFFFFFFFull) - data_off), (uint32_t)(d >> 48),
                          i, r);
                }
            }
        });
    }
    for (auto& x : th) x.join();
    return 0;
}

// Fills the frames described by desc into data (nthreads threads).
int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads) {
    return bt_synth_fill_range(cfg, n, seed, desc, 0, n, data, 0, nthreads);
}

// Packs a capture into an AF_PACKET TPACKET_V3 RX-ring image the way the kernel lays
// one out (net/packet/af_packet.c, tpacket_rcv / prb_* with tp_reserve 0, no block
// private area): 48-B block header, frames 8-B aligned, each a tpacket3_hdr + sockaddr_ll
// with the MAC header at tp_mac = 82, snaplen clamped to the block's max frame length,
// and the last frame of a block with tp_next_offset 0. Frames are packed until
// ring_blocks blocks are full. ring == NULL only counts. ring_desc (optional) gets
// BT_DESC(ring offset of the MAC header, snaplen) per packed frame. Returns the number
// of frames packed; *blocks_used the blocks written (all marked TP_STATUS_USER).
uint64_t bt_synth_tpv3_pack(const uint8_t* data, const uint64_t* desc, uint64_t n, uint64_t block_size,
                            uint8_t* ring, uint64_t ring_blocks, uint64_t* ring_desc, uint64_t* blocks_used) {
    const uint32_t kBlkHdr = 48, kMacOff = 82, kAlign = 8;
    const uint64_t max_frame = block_size - kBlkHdr;
    uint64_t blk = 0, off = kBlkHdr, packed = 0, seq = 1;
    uint32_t in_blk = 0;
    uint8_t* prev = nullptr;
    auto close_block = [&]() {
        if (!in_blk) return;
        if (ring) {
            tpacket_block_desc* bd = reinterpret_cast<tpacket_block_desc*>(ring + blk * block_size);
            bd->version = TPACKET_V3;
            bd->offset_to_priv = kBlkHdr;
            bd->hdr.bh1.num_pkts = in_blk;
            bd->hdr.bh1.offset_to_first_pkt = kBlkHdr;
            bd->hdr.bh1.blk_len = (uint32_t)off;
            bd->hdr.bh1.seq_num = seq;
            bd->hdr.bh1.block_status = TP_STATUS_USER;
            reinterpret_cast<tpacket3_hdr*>(prev)->tp_next_offset = 0;
        }
        ++seq;
        ++blk;
        off = kBlkHdr;
        in_blk = 0;
    };
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t src = desc[i] & 0xFFFFFFFFFFFFull;
        const uint32_t len = (uint32_t)(desc[i] >> 48);
        const uint32_t snap = (uint32_t)std::min<uint64_t>(len, max_frame - kMacOff);
        const uint64_t need = (kMacOff + snap + kAlign - 1) & ~(uint64_t)(kAlign - 1);
        if (off + need > block_size) close_block();
        if (blk >= ring_blocks) break;
        if (ring) {
            uint8_t* f = ring + blk * block_size + off;
            std::memset(f, 0, kMacOff);
            tpacket3_hdr* h = reinterpret_cast<tpacket3_hdr*>(f);
            h->tp_next_offset = (uint32_t)need;
            h->tp_sec = (uint32_t)(i / 1000000);
            h->tp_nsec = (uint32_t)(i % 1000000) * 1000;
            h->tp_snaplen = snap;
            h->tp_len = len;
            h->tp_status = TP_STATUS_USER;
            h->tp_mac = kMacOff;
            h->tp_net = kMacOff + 14;
            sockaddr_ll* sll = reinterpret_cast<sockaddr_ll*>(f + 48);
            sll->sll_family = AF_PACKET;
            sll->sll_ifindex = 1;
            sll->sll_halen = 6;
            if (snap) std::memcpy(f + kMacOff, data + src, snap);
            prev = f;
        }
        if (ring_desc) ring_desc[packed] = ((uint64_t)snap << 48) | (blk * block_size + off + kMacOff);
        off += need;
        ++in_blk;
        ++packed;
    }
    if (blk < ring_blocks) close_block();
    if (blocks_used) *blocks_used = blk;
    return packed;
}

}  // extern "C"
