// bt_kernels.hip — gfx950 kernels for the Beatrice parse+filter stage.
//
// bt_parse_filter_main / bt_parse_filter_pipe: one packet per lane, one 64-packet tile
// per wavefront, persistent grid-stride over tiles. Per tile:
//   1. LOAD   — the wave fetches the 64 header windows (16-B aligned chunks) with
//               coalesced 16-B loads: in descriptor mode round A reads the first 64 B
//               of every window with 4 lanes per packet (16 packets per instruction),
//               round B only the further chunks the walked headers need; in
//               fixed-stride mode the tile is one contiguous span (1 KiB per
//               instruction). Chunks go into a per-wave LDS image, one row per packet
//               (33 dwords in descriptor mode: the odd stride spreads the per-lane reads
//               over the banks).
//   2. PARSE  — each lane walks its own row: Ethernet, up to two 802.1Q/802.1ad tags,
//               IPv4/IPv6, TCP/UDP/ICMP (DESIGN.md "R-WALK"). Unaligned header windows
//               are rebuilt from aligned ds_read_b32 pairs with v_alignbyte_b32. The
//               record is assembled in registers: the packed device form (2-6 16-B
//               slabs, tiled per 64-packet tile, include/beatrice_gpu.h) or the 96-B
//               bt_rec (AoS, host copies).
//   3. FILTER — the compiled PacketFilter program (kernel argument, scalar loads) is
//               evaluated wave-uniformly slot by slot with early exit once every lane
//               has decided; the verdict is a wavefront __ballot word and the per-tile
//               pass count feeds the ordered compaction kernels below.
// bt_parse_filter_pipe is the descriptor-mode form with counted memory waits (see the
// comment above it); bt_parse_filter_main serves fixed stride and the other layouts.
// Replaces the per-packet work of reference src/parser/ProtocolParser.cpp:238-433 and
// src/PacketFilter.cpp:57-372 (see DESIGN.md for the line-by-line mapping).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "bt_device.h"
#include "bt_slot_eval.h"

namespace bt {

// BT_DEBUG_BOUNDS: this module's log of failed bounds checks (bt_bounds.h)
__device__ BoundsLog g_bounds_main;

namespace {

__device__ __forceinline__ uint32_t byte_of(const uint32_t* w, int i) {
    return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
}
__device__ __forceinline__ uint32_t be16_of(const uint32_t* w, int i) {
    return (byte_of(w, i) << 8) | byte_of(w, i + 1);
}
__device__ __forceinline__ uint32_t be32_of(const uint32_t* w, int i) {
    return (byte_of(w, i) << 24) | (byte_of(w, i + 1) << 16) | (byte_of(w, i + 2) << 8) | byte_of(w, i + 3);
}

// K little-endian dwords starting at byte `a` of the LDS image (any alignment).
template <int K>
__device__ __forceinline__ void window(const uint32_t* lds, uint32_t a, uint32_t* out) {
    const uint32_t d = a >> 2, sh = a & 3u;
    uint32_t prev = lds[d];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t next = lds[d + k + 1];
        out[k] = __builtin_amdgcn_alignbyte(next, prev, sh);
        prev = next;
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    // Lanes of one wavefront hand rows to each other through LDS: keep the compiler
    // from moving LDS accesses across this point and drain the LDS queue.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool is_vlan(uint32_t et) { return et == 0x8100u || et == 0x88A8u; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-B global load / store; `nt` selects the non-temporal (streaming) cache policy.
__device__ __forceinline__ uint4 ld16(const uint8_t* p, bool nt) {
    if (nt) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void st16(uint4* p, uint4 v, bool nt) {
    if (nt) {
        const u32x4 x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
    } else {
        *p = v;
    }
}

struct Parsed {
    uint32_t r[24];   // bt_rec as 24 little-endian dwords
};

// ProtocolDetector column (bt_rec bytes 88..90) from the first 38 frame bytes:
// detectProtocol (reference src/parser/ProtocolRegistry.cpp:353-388), the is*
// predicates (:418-487) and detectMultipleProtocols' second entry (:390-416). Every
// byte it reads is gated by the reference's own length checks, so bytes past the
// frame end (another frame's, in the LDS image) never decide anything.
__device__ __forceinline__ uint32_t detect_word(const uint32_t* w0, uint32_t len) {
    const uint32_t et = be16_of(w0, 12), b0 = byte_of(w0, 0), pr = byte_of(w0, 23);
    const uint32_t ports = be16_of(w0, 34) | (be16_of(w0, 36) << 16);
    // bitwise & / | throughout: short-circuit forms became exec-mask branches
    const bool eth = (len >= 14) & ((et == 0x0800u) | (et == 0x86DDu) | (et == 0x0806u));
    const bool l34 = len >= 34;
    const uint32_t code0 = len < 14 ? BT_DET_UNKNOWN : eth ? BT_DET_ETHERNET : BT_DET_NONE;
    const uint32_t l4code = pr == 6 ? BT_DET_TCP : pr == 17 ? BT_DET_UDP : pr == 1 ? BT_DET_ICMP : 0u;
    const uint32_t code = (eth & l34 & (l4code != 0u)) ? l4code : code0;
    const bool v4 = l34 & ((b0 >> 4) == 4u);
    const bool tcp = v4 & (pr == 6), udp = v4 & (pr == 17);
    const bool p80 = ((ports & 0xFFFFu) == 80u) | ((ports >> 16) == 80u);
    const bool p53 = ((ports & 0xFFFFu) == 53u) | ((ports >> 16) == 53u);
    const uint32_t is = (eth ? BT_IS_ETHERNET : 0u) | (v4 ? BT_IS_IPV4 : 0u) |
                        (((len >= 54) & ((b0 >> 4) == 6u)) ? BT_IS_IPV6 : 0u) | (tcp ? BT_IS_TCP : 0u) |
                        (udp ? BT_IS_UDP : 0u) | ((v4 & (pr == 1)) ? BT_IS_ICMP : 0u) |
                        ((tcp & (len >= 54) & p80) ? BT_IS_HTTP : 0u) | ((udp & (len >= 42) & p53) ? BT_IS_DNS : 0u);
    const uint32_t is2 = (((len >= 28) & (et == 0x0806u)) ? BT_IS2_ARP : 0u) |
                         ((l34 & (pr == 6)) ? BT_IS2_MULTI_TCP : 0u) | ((l34 & (pr == 17)) ? BT_IS2_MULTI_UDP : 0u);
    return code | (is << 8) | (is2 << 16);
}

// The layer walk + field extraction for one packet whose byte 0 sits at byte `s` of
// the lane's LDS row. Field semantics: ProtocolRegistry.cpp tables, extractValue<T>
// big-endian decode, all-or-nothing per layer (ProtocolParser.cpp:244-247).
// PACKED = false: p.r is the 96-B bt_rec (host AoS path); returns 6.
// PACKED = true:  p.r is the packed device record (include/beatrice_gpu.h): the fields
// of the layers that parsed, each right after the previous, so an Eth/IPv4/UDP packet
// fills 3 slabs instead of 6; returns the slab count (2..6). Dwords past it are 0, because
// every field of a layer that did not parse is 0. Both forms come from the same
// branch-free selects, so the packed form costs no registers beyond bt_rec's.
template <bool PACKED>
__device__ __forceinline__ uint32_t parse_packet(const uint32_t* row, uint32_t s, uint32_t len,
                                                 const uint32_t* w0, Parsed& p) {
    const uint32_t pl = len > 0xFFFFu ? 0xFFFFu : len;
    // Ethernet (ProtocolRegistry.cpp:150-159): total length 14
    const bool eth_ok = len >= 14;
    const uint32_t et0 = be16_of(w0, 12);
    p.r[0] = eth_ok ? w0[0] : 0;
    p.r[1] = eth_ok ? w0[1] : 0;
    p.r[2] = eth_ok ? w0[2] : 0;
    p.r[3] = (eth_ok ? et0 : 0u) | (pl << 16);

    // VLAN tags (ProtocolRegistry.cpp:289-297): slice k at 12+4k, total length 4
    const bool v0 = eth_ok && is_vlan(et0);
    const bool v0ok = v0 && len >= 16;
    const bool has_et1 = v0ok && len >= 18;
    const uint32_t et1 = be16_of(w0, 16);
    const bool v1 = has_et1 && is_vlan(et1);
    const bool v1ok = v1 && len >= 20;
    const bool has_et2 = v1ok && len >= 22;
    const uint32_t et2 = be16_of(w0, 20);
    const uint32_t tp0 = v0ok ? et0 : 0u, tp1 = v1ok ? et1 : 0u;
    const uint32_t tc0 = v0ok ? be16_of(w0, 14) : 0u, tc1 = v1ok ? be16_of(w0, 18) : 0u;

    bool have_et;
    uint32_t l3et, o3;
    if (!v0) { have_et = eth_ok; l3et = et0; o3 = 14; }
    else if (!v1) { have_et = has_et1; l3et = et1; o3 = 18; }
    else { have_et = has_et2; l3et = et2; o3 = 22; }
    const bool is4 = have_et && l3et == 0x0800u;
    const bool is6 = have_et && l3et == 0x86DDu;
    const bool v4ok = is4 && len >= o3 + 20;
    const bool v6ok = is6 && len >= o3 + 40;

    uint32_t w3[10];
    window<10>(row, s + o3, w3);
    const uint32_t b0 = byte_of(w3, 0);
    const uint32_t proto = byte_of(w3, 9), nh = byte_of(w3, 6);
    uint32_t o4 = is4 ? o3 + 4u * (b0 & 0x0Fu) : o3 + 40u;
    const uint32_t l4v4 = proto == 6 ? BT_L_TCP : proto == 17 ? BT_L_UDP : proto == 1 ? BT_L_ICMP : 0u;
    const uint32_t l4v6 = nh == 6 ? BT_L_TCP : nh == 17 ? BT_L_UDP : 0u;
    const uint32_t l4 = v6ok ? l4v6 : (v4ok & (o4 <= len)) ? l4v4 : 0u;

    // L4 fields (bt_rec dwords 17..21): TCP :194-209, UDP :211-221, ICMP :223-234
    uint32_t w4[5];
    window<5>(row, s + (l4 ? o4 : 0u), w4);
    const bool tcp_ok = l4 == BT_L_TCP && len >= o4 + 20;
    const bool udp_ok = l4 == BT_L_UDP && len >= o4 + 8;
    const bool icmp_ok = l4 == BT_L_ICMP && len >= o4 + 8;
    uint32_t l4v[5];
    {
        const uint32_t ports = be16_of(w4, 0) | (be16_of(w4, 2) << 16);
        const uint32_t icmp0 = byte_of(w4, 0) | (byte_of(w4, 1) << 8) | (be16_of(w4, 2) << 16);
        const uint32_t pair45 = be16_of(w4, 4) | (be16_of(w4, 6) << 16);
        l4v[0] = tcp_ok || udp_ok ? ports : (icmp_ok ? icmp0 : 0u);
        l4v[1] = tcp_ok ? be32_of(w4, 4) : (udp_ok || icmp_ok ? pair45 : 0u);
        l4v[2] = tcp_ok ? be32_of(w4, 8) : 0u;
        l4v[3] = tcp_ok ? byte_of(w4, 12) | (byte_of(w4, 13) << 8) | (be16_of(w4, 14) << 16) : 0u;
        l4v[4] = tcp_ok ? be16_of(w4, 16) | (be16_of(w4, 18) << 16) : 0u;
    }

    const uint32_t l3bit = is4 ? BT_L_IPV4 : is6 ? BT_L_IPV6 : 0u;
    const uint32_t present = BT_L_ETH | (v0 ? BT_L_VLAN0 : 0u) | (v1 ? BT_L_VLAN1 : 0u) | l3bit | l4;
    const uint32_t okbits = (eth_ok ? BT_L_ETH : 0u) | (v0ok ? BT_L_VLAN0 : 0u) | (v1ok ? BT_L_VLAN1 : 0u) |
                            (v4ok ? BT_L_IPV4 : 0u) | (v6ok ? BT_L_IPV6 : 0u) |
                            (tcp_ok ? BT_L_TCP : 0u) | (udp_ok ? BT_L_UDP : 0u) | (icmp_ok ? BT_L_ICMP : 0u);
    const uint32_t meta = present | (okbits << 8) | ((l3bit ? o3 : 0u) << 16) | ((l4 ? o4 : 0u) << 24);
    const uint32_t det = detect_word(w0, len);
    // IPv6 (ProtocolRegistry.cpp:180-192) is stored the same way in both forms
    const uint32_t v6[10] = {be32_of(w3, 0), be16_of(w3, 4) | (nh << 16) | (byte_of(w3, 7) << 24),
                             w3[2], w3[3], w3[4], w3[5], w3[6], w3[7], w3[8], w3[9]};
    p.r[23] = 0;
    if constexpr (!PACKED) {
        p.r[4] = tp0 | (tp1 << 16);
        p.r[5] = tc0 | (tc1 << 16);
        p.r[6] = meta;
        // IPv4 (ProtocolRegistry.cpp:161-178) in bt_rec's padded layout: L3 union at 28
        const uint32_t v4[10] = {b0 | (b0 << 8) | (byte_of(w3, 1) << 16) | (byte_of(w3, 8) << 24),
                                 proto | (be16_of(w3, 2) << 16), be16_of(w3, 4) | (be16_of(w3, 6) << 16),
                                 be16_of(w3, 10), w3[3], w3[4], 0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 10; ++k) p.r[7 + k] = v4ok ? v4[k] : (v6ok ? v6[k] : 0u);
#pragma unroll
        for (int k = 0; k < 5; ++k) p.r[17 + k] = l4v[k];
        p.r[22] = det;
        return BT_REC_SLABS;
    } else {
        // present | ok | detector (3 + 8 + 3 bits); l3_off / l4_off follow from present
        // and the IPv4 IHL, so they are not stored
        p.r[4] = present | (okbits << 8) | ((det & 7u) << 16) | (((det >> 8) & 0xFFu) << 19) |
                 (((det >> 16) & 7u) << 27);
        // VLAN extension, one dword per tag that parsed (tpid0 is the ethertype)
        const uint32_t ne = (v0ok ? 1u : 0u) + (v1ok ? 1u : 0u);
        const uint32_t x0 = tc0 | (tp1 << 16), x1 = tc1;
        // L3 then L4: IPv4 without bt_rec's pads and its duplicate version byte (5 dwords)
        // or IPv6 (10), then TCP (5) or UDP / ICMP (2)
        const uint32_t v4[5] = {b0 | (byte_of(w3, 1) << 8) | (byte_of(w3, 8) << 16) | (proto << 24),
                                be16_of(w3, 2) | (be16_of(w3, 4) << 16), be16_of(w3, 6) | (be16_of(w3, 10) << 16),
                                w3[3], w3[4]};
#ifndef BT_NO_SIMPLE_WAVES
        // Wave-uniform fast path: no lane of the wave parsed IPv6 or a second tag (every
        // C2/C3 wave). Then ne <= 1 and L is IPv4 + L4 or nothing: one select per dword
        // instead of three.
        if (__ballot(v6ok || v1ok) == 0ull) {
            // l4v is 0 unless v4ok here, so only the IPv4 dwords need the v4ok select
            uint32_t Ls[11];
#pragma unroll
            for (int j = 0; j < 5; ++j) Ls[j] = v4ok ? v4[j] : 0u;
#pragma unroll
            for (int j = 0; j < 5; ++j) Ls[5 + j] = l4v[j];
            Ls[10] = 0u;
#pragma unroll
            for (int j = 0; j < 19; ++j)
                p.r[5 + j] = j > 10 ? 0u : v0ok ? (j == 0 ? x0 : Ls[j > 0 ? j - 1 : 0]) : Ls[j <= 10 ? j : 0];
            const uint32_t nd = 5u + ne + (v4ok ? 5u : 0u) + (tcp_ok ? 5u : (udp_ok || icmp_ok) ? 2u : 0u);
            return (nd + 3u) >> 2;
        }
#endif
        uint32_t L[15];
#pragma unroll
        for (int j = 0; j < 15; ++j)
            L[j] = v4ok ? (j < 5 ? v4[j] : j < 10 ? l4v[j - 5] : 0u) : v6ok ? (j < 10 ? v6[j] : l4v[j - 10]) : 0u;
#pragma unroll
        for (int j = 0; j < 19; ++j) {
            const uint32_t e0 = j < 15 ? L[j] : 0u;
            const uint32_t e1 = j == 0 ? x0 : (j - 1 < 15 ? L[j - 1] : 0u);
            const uint32_t e2 = j == 0 ? x0 : j == 1 ? x1 : (j - 2 < 15 ? L[j - 2] : 0u);
            p.r[5 + j] = ne == 0u ? e0 : ne == 1u ? e1 : e2;
        }
        const uint32_t nd = 5u + ne + (v4ok ? 5u : v6ok ? 10u : 0u) + (tcp_ok ? 5u : (udp_ok || icmp_ok) ? 2u : 0u);
        return (nd + 3u) >> 2;
    }
}

// One filter slot on one packet: FilterIn / eval_slot (bt_slot_eval.h), the same functions the
// C++ drop-in layer evaluates single packets and host continuations with.

// PAYLOAD filter on the GPU (BT_K_PAYLOAD): applyPayloadFilter's window
// (src/PacketFilter.cpp:293-309: IPv4 only, bytes [14 + 4*IHL, +min(len - that, 100)))
// run through the host-compiled byte DFA (bt_regex_dfa.cpp; blob layout there) that
// sits in this block's dynamic LDS. The window lies beyond the header image, so the
// lane stages it into its own LDS row first (the row is the lane's alone once PARSE
// is done): <= 8 16-B loads, 4 in flight at a time (all 8 would cost the variant a
// wave of occupancy). The walk is one dependent LDS read per byte (C == 256) or two
// (byte classes); the sinks K (match) / K+1 (none possible) end it early.

__device__ uint4 g_zero16[8];                    // source of the loads that read nothing

// applyPayloadFilter's window of a frame (eval_payload's gates): its start offset in the
// frame (po) and length L; L = 0 when the filter returns false without a search.
__device__ __forceinline__ uint32_t payload_window(uint32_t len, const uint32_t* w0, uint32_t& po) {
    po = 14u + (byte_of(w0, 14) & 15u) * 4u;
    if (!(len >= 34u && be16_of(w0, 12) == 0x0800u) || len <= po) return 0u;
    return min(len - po, 100u);
}

// The bit-parallel form (bt_regex_dfa.cpp "AST -> bit-parallel form"; blob layout there): an
// extended Shift-And over the position set D. The loop takes four window bytes per turn
// from the lane's LDS row (where eval_payload put the window) and runs until every lane of
// the wave has matched or passed its window (wave-uniform exit, no divergence inside); the
// row dwords two turns ahead and the table entries of the next four bytes are read before
// this turn's state steps, which are then only shift / or / and on registers. Entries are 1,
// 2, 4 or 8 bytes (the positions rounded up), so a small pattern's 256-entry table spans
// few distinct dwords per LDS bank (1-byte entries: at most 2 per bank, 4-byte: 8). A byte
// past the window (pos >= L) gets an empty mask: the partial matches of a SIMPLE pattern end
// there, and the others hold D ($ reads D at the window's end). Returns regex_search's answer
// over the L bytes.
template <typename E, bool SIMPLE>
__device__ __forceinline__ uint32_t bitpar_walk(const uint8_t* blob, const uint32_t* row, uint32_t staged_sh,
                                                uint32_t L, uint32_t rdw) {
    using T = typename std::conditional<sizeof(E) == 8, uint64_t, uint32_t>::type;
    const uint64_t* mk = reinterpret_cast<const uint64_t*>(blob + 16);
    const T Iall = (T)mk[0], F = (T)mk[5];
    const E* B = reinterpret_cast<const E*>(blob + 80);
    const uint32_t* r = row + (staged_sh >> 2);
    const uint32_t sh = staged_sh & 3u, rmax = rdw - 2u - (staged_sh >> 2);   // r[] stays inside the row
    // the general form's masks (SIMPLE: none of them is used)
    const T I0 = SIMPLE ? (T)0 : (T)mk[1], S = SIMPLE ? (T)0 : (T)mk[2], A = SIMPLE ? (T)0 : (T)mk[3];
    const T NF = SIMPLE ? ~(T)0 : (T)mk[4], Fe = SIMPLE ? (T)0 : (T)mk[6];
    const uint32_t R = SIMPLE ? 0u : blob[7];
    const bool anchored_all = !SIMPLE && (*reinterpret_cast<const uint32_t*>(blob + 8) & 4u) != 0u;
    T D = 0, hit = 0, inj = Iall | I0;
    auto step = [&](T b, uint32_t pos) {
        if constexpr (SIMPLE) {
            D = ((D << 1) | Iall) & (pos < L ? b : (T)0);
            hit |= D & F;
        } else {
            T n = (((D << 1) & NF) | inj | (D & S)) & b;
            inj = Iall;
            for (uint32_t k = 0; k < R; ++k) n |= (n << 1) & A;
            D = pos < L ? n : D;
            hit |= D & F;
        }
    };
    uint32_t t0 = r[0], t1 = r[1];
    uint32_t w = __builtin_amdgcn_alignbyte(t1, t0, sh);
    t0 = t1;
    t1 = r[2];
    T b0 = B[w & 0xFFu], b1 = B[(w >> 8) & 0xFFu], b2 = B[(w >> 16) & 0xFFu], b3 = B[w >> 24];
    for (uint32_t i = 0;; i += 4u) {
        // the next turn's bytes and entries, ahead of this turn's steps
        const uint32_t wn = __builtin_amdgcn_alignbyte(t1, t0, sh);
        t0 = t1;
        t1 = r[min((i >> 2) + 3u, rmax)];
        const T n0 = B[wn & 0xFFu], n1 = B[(wn >> 8) & 0xFFu], n2 = B[(wn >> 16) & 0xFFu], n3 = B[wn >> 24];
        step(b0, i);
        step(b1, i + 1u);
        step(b2, i + 2u);
        step(b3, i + 3u);
        if (__ballot(!hit && i + 4u < L && (SIMPLE || D || !anchored_all)) == 0ull) break;
        b0 = n0; b1 = n1; b2 = n2; b3 = n3;
    }
    return (hit || (D & Fe)) ? 1u : 0u;
}

// A SIMPLE pattern with a byte z that no class holds (the compiler records it): the window's
// bytes past its end are overwritten with z in the row, so every byte the wave's walk reads
// past a lane's window empties that lane's D and no position needs a bound check. The steps
// are then ((D << 1) | I) & B[c] and an OR of the states (H; a match ended where H & F is
// set): about 4 VALU per byte against 8 with the bound checks, which made the walk VALU-bound
// (C3 /GET|POST/ first: 123 k VALU per wave of the 129 k the walk added, SQ counters).
// Reading the window one LDS byte per byte instead (no alignbyte / extraction; the compiler
// merges the reads into unaligned 8-byte LDS reads and adds with byte selects) was slower
// filter-only, 0.708-0.718 against 0.663-0.670 ms (profiles/r06/payload/libs_bytes_wpe4.log).
template <typename E>
__device__ __forceinline__ uint32_t bitpar_fast(const uint8_t* blob, const uint32_t* row, uint32_t staged_sh,
                                                uint32_t L, uint32_t rdw) {
    const uint64_t* mk = reinterpret_cast<const uint64_t*>(blob + 16);
    const uint32_t Iall = (uint32_t)mk[0], F = (uint32_t)mk[5];
    const E* B = reinterpret_cast<const E*>(blob + 80);
    const uint32_t* r = row + (staged_sh >> 2);
    const uint32_t sh = staged_sh & 3u, rmax = rdw - 2u - (staged_sh >> 2);   // the row's last padded dword
    uint32_t t0 = r[0], t1 = r[1], t2 = r[2];
    uint32_t D = 0, H = 0;
    for (uint32_t i = 0;; i += 8u) {
        uint32_t b[8];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(t1, t0, sh), w1 = __builtin_amdgcn_alignbyte(t2, t1, sh);
        t0 = t2;
        t1 = r[min((i >> 2) + 3u, rmax)];
        t2 = r[min((i >> 2) + 4u, rmax)];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            b[k] = B[(w0 >> (8 * k)) & 0xFFu];
            b[4 + k] = B[(w1 >> (8 * k)) & 0xFFu];
        }
        const uint32_t d0 = ((D << 1) | Iall) & b[0], d1 = ((d0 << 1) | Iall) & b[1];
        const uint32_t d2 = ((d1 << 1) | Iall) & b[2], d3 = ((d2 << 1) | Iall) & b[3];
        const uint32_t d4 = ((d3 << 1) | Iall) & b[4], d5 = ((d4 << 1) | Iall) & b[5];
        const uint32_t d6 = ((d5 << 1) | Iall) & b[6];
        D = ((d6 << 1) | Iall) & b[7];
        H |= d0 | d1 | d2 | d3 | d4 | d5 | d6 | D;
        if (__ballot(!(H & F) && i + 8u < L) == 0ull) break;
    }
    return (H & F) ? 1u : 0u;
}

// `reuse`: the 16-B chunks of the frame's header window (from its 16-B-aligned start) that round
// A left in the row (4 in descriptor mode with whole 64-B windows, else 0). The window's chunks
// among them are moved down the row instead of read again: their lines were read a tile ago and
// are often gone from L2 by now (C3 with /GET|POST/ first: 209 B read per packet against a
// 131-B line floor).
//
// `rdw`: the row's dwords (row_dw: 33 in descriptor mode, 17 for 64-B fixed strides). The window,
// its padding and the walks' reads stay inside the lane's own row: the padding written past
// a 17-dword row once overwrote the next lane's staged window (64-B fixed-stride batches,
// tests/test_gpu_payload.py::test_fixed_stride_payload).
__device__ __forceinline__ uint32_t eval_payload(const MainArgs& a, const uint8_t* blob, uint32_t* row,
                                                 uint64_t frame_off, uint32_t len, const uint32_t* w0,
                                                 uint32_t& staged_sh, uint32_t reuse, uint32_t rdw) {
    uint32_t po;
    const uint32_t L = payload_window(len, w0, po);
    if (!L) return 0u;
    const uint32_t K = *reinterpret_cast<const uint16_t*>(blob);
    if (K == 0xFFFFu && blob[6] != 1u) return blob[6] == 2u ? 1u : 0u;   // bit-parallel: always / never
    if (staged_sh == ~0u) {
        const uint64_t start = frame_off + po;
        const uint64_t al = start & ~15ull;
        staged_sh = (uint32_t)(start & 15ull);
        // <= 8: 128 B of the 132-B row; a 64-B fixed-stride frame's window ends by row byte 32
        const uint32_t nch = min((staged_sh + L + 15u) >> 4, (rdw - 1u) >> 2);
        // window chunk k = header chunk d + k: those still in the row move down (d >= 2)
        const uint32_t d = (uint32_t)((al - (frame_off & ~15ull)) >> 4);
        const uint32_t kept = reuse > d ? min(reuse - d, nch) : 0u;
        for (uint32_t k = 0; k < kept; ++k) {
            uint32_t* dst = row + 4u * k;
            const uint32_t* src = row + 4u * (k + d);
            dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2]; dst[3] = src[3];
        }
#pragma unroll
        for (uint32_t h = 0; h < 8u; h += 4u) {
            if (h < nch && h + 4u > kept) {
                uint4 v[4];
#pragma unroll
                for (uint32_t k = 0; k < 4u; ++k) {
                    const uint64_t g = al + 16ull * (h + k);
                    v[k] = (h + k >= kept && h + k < nch && g + 16ull <= a.bytes) ? ld16(a.base + g, a.nt & 2u)
                                                                                 : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (uint32_t k = 0; k < 4u; ++k)
                    if (h + k >= kept) {
                        uint32_t* q = row + 4u * (h + k);
                        q[0] = v[k].x; q[1] = v[k].y; q[2] = v[k].z; q[3] = v[k].w;
                    }
            }
        }
    }
    if (K == 0xFFFFu) {   // the bit-parallel form (wave-uniform: the slot's blob)
        const uint32_t W = *reinterpret_cast<const uint16_t*>(blob + 2);
        const bool simple = *reinterpret_cast<const uint32_t*>(blob + 8) == 0u && blob[7] == 0u;
        const uint32_t z = blob[12];   // 1 + a byte no class holds, 0: none
        if (simple && z && W <= 32u) {
            // the row past the window: z in every byte (the dword the window ends in keeps
            // the window's bytes below the end)
            const uint32_t end = staged_sh + L, q = end >> 2, zz = (z - 1u) * 0x01010101u;
            const uint32_t keep = (end & 3u) ? (1u << (8u * (end & 3u))) - 1u : 0u;
            row[q] = (row[q] & keep) | (zz & ~keep);
            for (uint32_t k = q + 1u; k < rdw; ++k) row[k] = zz;
            return W == 8 ? bitpar_fast<uint8_t>(blob, row, staged_sh, L, rdw)
                 : W == 16 ? bitpar_fast<uint16_t>(blob, row, staged_sh, L, rdw)
                           : bitpar_fast<uint32_t>(blob, row, staged_sh, L, rdw);
        }
        switch (W) {
        case 8: return simple ? bitpar_walk<uint8_t, true>(blob, row, staged_sh, L, rdw)
                              : bitpar_walk<uint8_t, false>(blob, row, staged_sh, L, rdw);
        case 16: return simple ? bitpar_walk<uint16_t, true>(blob, row, staged_sh, L, rdw)
                               : bitpar_walk<uint16_t, false>(blob, row, staged_sh, L, rdw);
        case 32: return simple ? bitpar_walk<uint32_t, true>(blob, row, staged_sh, L, rdw)
                               : bitpar_walk<uint32_t, false>(blob, row, staged_sh, L, rdw);
        default: return bitpar_walk<uint64_t, false>(blob, row, staged_sh, L, rdw);
        }
    }
    const uint32_t C = *reinterpret_cast<const uint16_t*>(blob + 2);
    uint32_t q = blob[4];
    if (q >= K) return q == K ? 1u : 0u;
    const uint8_t* endacc = blob + 8;
    const uint8_t* cls = endacc + ((K + 3u) & ~3u);
    const uint8_t* next = C == 256u ? cls : cls + 256;
    const uint32_t dw = staged_sh >> 2, sh8 = (staged_sh & 3u) * 8u;
    uint32_t i = 0;
    if (blob[6]) {
        // Two-byte table: the classes of four bytes are independent of q and issued
        // first, then two dependent reads cover them (half the chain of one per byte).
        const uint32_t P = blob[7];
        const uint8_t* clsp = blob + ((((uint32_t)(next - blob) + K * C) + 3u) & ~3u);
        const uint8_t* pair = clsp + 256;
        for (; i + 4u <= L; i += 4u) {
            const uint32_t lo = row[dw + (i >> 2)], hi = row[dw + (i >> 2) + 1u];
            const uint32_t w = sh8 ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh8) : lo;
            const uint32_t c0 = clsp[w & 0xFFu], c1 = clsp[(w >> 8) & 0xFFu];
            const uint32_t c2 = clsp[(w >> 16) & 0xFFu], c3 = clsp[w >> 24];
            q = pair[(q * P + c0) * P + c1];
            if (q >= K) return q == K ? 1u : 0u;
            q = pair[(q * P + c2) * P + c3];
            if (q >= K) return q == K ? 1u : 0u;
        }
        // the last 1..3 bytes: one more pair if two remain, then the one-byte table
        if (i + 2u <= L) {
            const uint32_t lo = row[dw + (i >> 2)], hi = row[dw + (i >> 2) + 1u];
            const uint32_t w = sh8 ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh8) : lo;
            q = pair[(q * P + clsp[w & 0xFFu]) * P + clsp[(w >> 8) & 0xFFu]];
            if (q >= K) return q == K ? 1u : 0u;
            i += 2u;
        }
        if (i < L) {   // one byte left: payload byte i sits at row byte staged_sh + i
            const uint32_t at = staged_sh + i;
            const uint32_t b = (row[at >> 2] >> (8u * (at & 3u))) & 0xFFu;
            q = next[q * C + (C == 256u ? b : (uint32_t)cls[b])];
            if (q >= K) return q == K ? 1u : 0u;
        }
        return endacc[q];
    }
    for (; i < L; i += 4u) {
        // four payload bytes from two aligned row dwords (independent of q: issued early)
        const uint32_t lo = row[dw + (i >> 2)], hi = row[dw + (i >> 2) + 1u];
        const uint32_t w = sh8 ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh8) : lo;
        const uint32_t m = min(4u, L - i);
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
            if (k < m) {
                const uint32_t b = (w >> (8u * k)) & 0xFFu;
                q = next[q * C + (C == 256u ? b : (uint32_t)cls[b])];
                if (q >= K) return q == K ? 1u : 0u;
            }
        }
    }
    return endacc[q];
}

// The compiled PacketFilter program on this lane's packet: the reference's AND chain in
// priority order with early exit (src/PacketFilter.cpp:57-119), wave-uniform slot by slot
// until every lane has decided. Returns the decision code (BT_DECIDE_*) and the deciding
// slot. `lrow` = the lane's LDS row, reused to stage a PAYLOAD window after the parse.
// F = 1: no PAYLOAD slot in the program: every slot is evaluated in its uniform-predicate
// form (bt_device.h DevFilter), one straight-line sequence with no per-kind branches.
// F = 2: the per-kind evaluator and the GPU DFA for PAYLOAD slots.
// The first kHotSlots slots of the program, read from the kernel arguments once per wave
// before the tile loop and kept in registers. The slot loop used to read each slot with
// a scalar load from the kernel-argument segment and wait for it, once per slot and tile:
// a memory round trip on the parse's critical path (c2f at 2 blocks/CU: 0.391 ms with
// the filter evaluated, 0.333 without; tools/gpu_ab_libs_grid.sh).
#ifndef BT_HOT_SLOTS
#define BT_HOT_SLOTS 4
#endif
constexpr uint32_t kHotSlots = BT_HOT_SLOTS;
struct HotProgram {
    uint32_t n;
    DevFilter f[kHotSlots ? kHotSlots : 1u];
};
__device__ __forceinline__ HotProgram hot_program(const DevProgram& prog) {
    HotProgram h;
    h.n = prog.n;
#pragma unroll
    for (uint32_t k = 0; k < (kHotSlots ? kHotSlots : 1u); ++k) h.f[k] = prog.f[k];
    return h;
}

template <int F>
__device__ __forceinline__ uint32_t filter_packet(const MainArgs& a, const DevProgram& prog, const HotProgram& hot,
                                                  const uint8_t* dfa_lds, uint32_t* lrow, uint32_t rdw,
                                                  uint64_t my_off, uint32_t len, const uint32_t* w0, bool live,
                                                  uint32_t& slot, uint32_t reuse = 0u) {
    const FilterIn x = filter_in([w0](uint32_t i) { return byte_of(w0, (int)i); }, len);
    uint32_t code = BT_DECIDE_PASS;
    slot = prog.n ? prog.n - 1u : 0u;
    bool open = live;
    if constexpr (F == 1) {
        const uint32_t pbit = (x.proto == 6 ? 1u : 0u) | (x.proto == 17 ? 2u : 0u) | (x.proto == 1 ? 4u : 0u);
        const bool g4 = x.gate & x.l4_ok;
        // slot f's result on this packet: 1 pass, 0 reject, 2 throw, 3 host
        auto result = [&](const DevFilter& d) -> uint32_t {
            const uint32_t sel = d.ctl & 3u, gm = (d.ctl >> 2) & 3u, rm = (d.ctl >> 4) & 3u;   // uniform
            const uint32_t x1 = sel == kSelIp ? x.src : sel == kSelPort ? x.sport : sel == kSelProto ? x.proto : pbit;
            const uint32_t x2 = sel == kSelIp ? x.dst : sel == kSelPort ? x.dport : sel == kSelProto ? x.proto : pbit;
            const bool pred = (((x1 & d.mask) - d.lo) <= d.span) | (((x2 & d.mask) - d.lo) <= d.span);
            const bool g = gm == kGateNone ? true : gm == kGateIpv4 ? x.gate : g4;
            return !g ? 0u : rm == kResPred ? (pred ? 1u : 0u) : rm == kResThrow ? 2u : 3u;
        };
        auto decide = [](uint32_t r) {
            return r == 0u ? BT_DECIDE_REJECT : r == 2u ? BT_DECIDE_THROW : BT_DECIDE_HOST;
        };
        // The hot slots side by side: their results are independent, so they are computed
        // without the early exit's branches (which made one long dependent chain of
        // compares, lane-mask and branch instructions per slot, which two waves per SIMD
        // could not hide), then the first slot that did not pass decides (AND chain order).
        if constexpr (kHotSlots > 0) {
            uint32_t r[kHotSlots ? kHotSlots : 1u];
#pragma unroll
            for (uint32_t f = 0; f < kHotSlots; ++f) r[f] = f < hot.n ? result(hot.f[f]) : 1u;
#pragma unroll
            for (int f = (int)kHotSlots - 1; f >= 0; --f)
                if (r[f] != 1u) { code = decide(r[f]); slot = (uint32_t)f; }
            if (!live) { code = BT_DECIDE_PASS; slot = prog.n ? prog.n - 1u : 0u; }
            open = live && code == BT_DECIDE_PASS;
        }
        for (uint32_t f = kHotSlots; f < prog.n; ++f) {   // longer programs: the rest from memory
            if (__ballot(open) == 0ull) break;
            const uint32_t rf = result(prog.f[f]);
            if (open && rf != 1u) {
                code = decide(rf);
                slot = f;
                open = false;
            }
        }
        return code;
    }
    uint32_t staged_sh = ~0u;   // payload window not staged yet
    for (uint32_t f = 0; f < prog.n; ++f) {
        if (__ballot(open) == 0ull) break;
        uint32_t r;
        if (prog.f[f].kind == BT_K_PAYLOAD)   // wave-uniform
            r = a.prefixes ? 3u   // the payload is not in a prefix batch: host
              : open ? eval_payload(a, dfa_lds + prog.f[f].a, lrow, my_off, len, w0, staged_sh, reuse, rdw) : 0u;
        else
            r = eval_slot(prog.f[f].kind, prog.f[f].a, prog.f[f].b, x);
        if (open && r != 1u) {
            code = r == 0u ? BT_DECIDE_REJECT : r == 2u ? BT_DECIDE_THROW : BT_DECIDE_HOST;
            slot = f;
            open = false;
        }
    }
    return code;
}


// Header windows of one 64-packet tile in flight in registers (LOAD stage).
//  fixed stride: the tile is one contiguous span, cpp 16-B chunks per packet;
//  descriptors:  round A = the first 64 B (chunks 0..3) of every packet's 16-B-aligned
//                window, 4 lanes per packet, 16 packets per wave instruction.
//                "wide" (wave-adaptive): chunks 4..7 in the same round, for waves whose
//                previous tile mostly needed them (QinQ / IPv6 / IP options): one round
//                trip, and no second fetch of lines L2 evicted between two rounds.
template <int FIXED_LOG2>
struct Stage {
    static constexpr int kV = FIXED_LOG2 >= 0 ? (1 << (FIXED_LOG2 >= 0 ? FIXED_LOG2 : 0)) : 8;
    uint4 v[kV];
    uint64_t qa0[FIXED_LOG2 >= 0 ? 1 : 4];   // aligned window base of packet j*16 + lane/4
    uint64_t off;                             // this lane's own packet
    uint32_t len;
    bool wide;
};

// Round A of a wide tile reads the packet's window [a0, a0 + sq + min(len, need_max))
// only up to the end of a0's 128-B line: the line is then fetched once, and round B reads
// the next line's chunks only if the walked headers reach them. (Reading the whole window
// up front, the first version, fetched the second line for 1.78 instead of 1.60 lines per
// C4 packet.)
__device__ __forceinline__ uint32_t round_a_end_wide(uint64_t a0, uint32_t sq, uint32_t len, uint32_t need_max) {
    const uint32_t line_rem = 128u - ((uint32_t)a0 & 127u);
    const uint32_t want = sq + (len < need_max ? len : need_max);
    return want < line_rem ? want : line_rem;
}

// LATE (fixed stride, bt_parse_filter_main's late issue): every lane loads, the zero line
// past n, always non-temporal, so every path issues the same four loads and the loop top
// can wait for each with a counted vmcnt.
template <int FIXED_LOG2, bool LATE = false>
__device__ __forceinline__ void issue_loads(const MainArgs& a, uint32_t t, uint32_t lane, Stage<FIXED_LOG2>& st,
                                            bool wide, uint32_t need_max) {
    const uint32_t p0 = t * 64u;
    const uint32_t my = p0 + lane;
    const bool live = my < a.n;
    if constexpr (FIXED_LOG2 >= 0) {
        constexpr int kL = FIXED_LOG2 >= 0 ? FIXED_LOG2 : 0;
        constexpr uint32_t cpp = 1u << kL;
        st.off = (uint64_t)my * a.stride;
        st.len = a.stride;
        const uint8_t* span = a.base + (uint64_t)p0 * a.stride;
#pragma unroll
        for (uint32_t j = 0; j < cpp; ++j) {
            const uint32_t g = j * 64u + lane;
            const bool ok = p0 + (g >> kL) < a.n &&
                            BT_IN(&g_bounds_main, kSiteFixedLoad, (uint64_t)p0 * a.stride + g * 16u + 15u, a.bytes);
            if (LATE)
                st.v[j] = ld16(ok ? span + (uint64_t)g * 16u : reinterpret_cast<const uint8_t*>(g_zero16), true);
            else
                st.v[j] = ok ? ld16(span + (uint64_t)g * 16u, a.nt & 2u) : make_uint4(0, 0, 0, 0);
        }
    } else {
        if (a.desc) {
            if (a.desc_words == 1) {   // bt_pkt_desc
                const uint64_t d = live ? a.desc[my] : 0ull;
                st.off = d & 0xFFFFFFFFFFFFull;
                st.len = (uint32_t)(d >> 48);
            } else {                   // xdp_desc {u64 addr; u32 len; u32 options}
                const uint4 d = live ? *reinterpret_cast<const uint4*>(a.desc + 2ull * my) : make_uint4(0, 0, 0, 0);
                st.off = ((uint64_t)d.y << 32) | d.x;
                st.len = d.z > 0xFFFFu ? 0xFFFFu : d.z;
            }
        } else {
            st.off = live ? (uint64_t)my * a.stride : 0ull;
            st.len = live ? a.stride : 0u;
        }
        const uint32_t off_lo = (uint32_t)st.off, off_hi = (uint32_t)(st.off >> 32);
        const uint32_t c = lane & 3u;
        st.wide = wide;
        // Non-temporal header loads pay off in two-round-free tiles (C3: 0.595 -> 0.564 ms),
        // but in wide tiles they raised C4's read traffic from the exact-line 214 to 235 B
        // per packet (rocprofv3 FETCH_SIZE, tools/gpu_fetch_modes.sh); wide tiles and
        // round B use the default policy.
        const bool ntl = (a.nt & 2u) && !wide;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t q = j * 16u + (lane >> 2);
            const uint64_t qo = ((uint64_t)(uint32_t)__shfl((int)off_hi, (int)q) << 32) |
                                (uint32_t)__shfl((int)off_lo, (int)q);
            const uint32_t ql = (uint32_t)__shfl((int)st.len, (int)q);
            const uint64_t a0 = qo & ~15ull;
            const uint64_t addr = a0 + 16u * c;
            const uint32_t sq = (uint32_t)qo & 15u;
            st.qa0[j] = a0;
            const bool live_q = p0 + q < a.n;
            // bytes from a0 this round may read: the frame; when wide, only up to the end
            // of a0's 128-B line (round B takes the next line, and only what is needed)
            const uint32_t a_end = wide ? round_a_end_wide(a0, sq, ql, need_max) : sq + min(ql, a.lean);
            const uint32_t a_lo = wide ? 0u : sq + a.lean_lo;   // chunks ending at or before it: unread
            const bool ok = live_q && (16u * c < a_end) && (16u * c + 16u > a_lo) && (addr + 16u <= a.bytes);
            st.v[j] = ok ? ld16(a.base + addr, ntl) : make_uint4(0, 0, 0, 0);
            if (wide) {   // chunks 4..7 of the same line
                const bool okb = live_q && (16u * (c + 4u) < a_end) && (addr + 64u + 16u <= a.bytes);
                st.v[4 + j] = okb ? ld16(a.base + addr + 64u, false) : make_uint4(0, 0, 0, 0);
            }
        }
    }
}

// LDS row (dwords) of one packet: the 128-B header window + 1 pad dword in descriptor
// mode; in fixed-stride mode the whole frame (stride <= 64 B) + 1 pad dword. An odd row
// stride spreads the per-lane reads over the banks. The smaller rows of the 16/32/64-B
// strides cut a block's LDS (C2: 33.8 -> 17.4 KB), so the VGPR budget, not LDS, sets
// the residency. Reads past a short frame's row land in the next row (or the block's
// tail pad) and are never used: every field the walk keeps is gated by len.
template <int FIXED_LOG2>
__device__ constexpr uint32_t row_dw() {
    return FIXED_LOG2 >= 0 && FIXED_LOG2 < 3 ? (4u << (FIXED_LOG2 >= 0 ? FIXED_LOG2 : 0)) + 1u : (uint32_t)kRowDwords;
}

template <int FIXED_LOG2>
__device__ __forceinline__ void stage_to_lds(const Stage<FIXED_LOG2>& st, uint32_t* img, uint32_t lane) {
    if constexpr (FIXED_LOG2 >= 0) {
        constexpr int kL = FIXED_LOG2 >= 0 ? FIXED_LOG2 : 0;
        constexpr uint32_t cpp = 1u << kL;
#pragma unroll
        for (uint32_t j = 0; j < cpp; ++j) {
            const uint32_t g = j * 64u + lane;
            uint32_t* dst = img + (g >> kL) * row_dw<FIXED_LOG2>() + (g & (cpp - 1u)) * 4u;
            dst[0] = st.v[j].x; dst[1] = st.v[j].y; dst[2] = st.v[j].z; dst[3] = st.v[j].w;
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            uint32_t* dst = img + (j * 16u + (lane >> 2)) * row_dw<FIXED_LOG2>() + (lane & 3u) * 4u;
            dst[0] = st.v[j].x; dst[1] = st.v[j].y; dst[2] = st.v[j].z; dst[3] = st.v[j].w;
        }
        if (st.wide) {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                uint32_t* dst = img + (j * 16u + (lane >> 2)) * row_dw<FIXED_LOG2>() + 16u + (lane & 3u) * 4u;
                dst[0] = st.v[4 + j].x; dst[1] = st.v[4 + j].y; dst[2] = st.v[4 + j].z; dst[3] = st.v[4 + j].w;
            }
        }
    }
}

// Upper bound of the frame bytes the walk + filters will read, from round A's 64 B
// (everything it looks at — EtherTypes at 12/16/20, IHL at L3+0 — sits below byte 49).
// `w0` = the packet's first 40 bytes (window<10> at its start); only bytes < 28 are used.
__device__ __forceinline__ uint32_t header_end(const uint32_t* w0, uint32_t len, uint32_t floor_) {
    // branch-free: the walk's tag / EtherType / IHL choice as selects
    const uint32_t et0 = be16_of(w0, 12), et1 = be16_of(w0, 16), et2 = be16_of(w0, 20);
    const bool t0 = is_vlan(et0), t1 = t0 & is_vlan(et1);
    const uint32_t o3 = 14u + (t0 ? 4u : 0u) + (t1 ? 4u : 0u);
    const uint32_t et = t1 ? et2 : t0 ? et1 : et0;
    const uint32_t ihl = (t1 ? byte_of(w0, 22) : t0 ? byte_of(w0, 18) : byte_of(w0, 14)) & 0x0Fu;
    const uint32_t v4end = o3 + 40u + (ihl > 5u ? 4u * ihl - 20u : 0u);
    uint32_t end = et == 0x0800u ? v4end : et == 0x86DDu ? o3 + 60u : o3;
    end = end > floor_ ? end : floor_;
    return end < len ? end : len;
}

// Round B: the chunks [lo, hi) of each packet's window that round A did not read and
// the walk needs (my_b = lo | hi << 8, in chunks / bytes from a0; hi = 0: none). Lane
// (lane & 3) of a packet's four takes chunks lo + (lane & 3) and, when `second`, + 4.
template <int FIXED_LOG2>
__device__ __forceinline__ void load_round_b(const MainArgs& a, uint32_t t, uint32_t lane, const uint64_t* qa0,
                                             uint32_t my_b, uint32_t* img, bool second) {
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        if (k == 1 && !second) break;
        uint4 v[4];
        uint32_t cs[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t q = j * 16u + (lane >> 2);
            const uint32_t qb = (uint32_t)__shfl((int)my_b, (int)q);
            const uint32_t c = (qb & 0xFFu) + (lane & 3u) + 4u * k;
            const uint64_t addr = qa0[j] + 16u * c;
            const bool want = c < 8u && (16u * c < (qb >> 8));   // never overwrite round A's chunks
            cs[j] = want ? c : 8u;
            const bool ok = want && (t * 64u + q < a.n) && (addr + 16u <= a.bytes);
            v[j] = ok ? ld16(a.base + addr, false) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            if (cs[j] < 8u) {
                uint32_t* dst = img + (j * 16u + (lane >> 2)) * row_dw<FIXED_LOG2>() + cs[j] * 4u;
                dst[0] = v[j].x; dst[1] = v[j].y; dst[2] = v[j].z; dst[3] = v[j].w;
            }
        }
    }
}

// Descriptor mode after round A: where this lane's walked headers end (header_end, with
// a floor of 38 B for the PacketFilter gates and the detector column), round B for the
// chunks round A did not read (wave-uniform: only if some lane needs it; then the row
// and `w0` are refreshed), and the wave's load mode for its next tile (wide when most
// packets needed more than 64 B; nt bits 2/3 force it, A/B). Returns that mode.
__device__ __forceinline__ bool round_b(const MainArgs& a, uint32_t t, uint32_t lane, const uint64_t* qa0,
                                       uint32_t* img, const uint32_t* row, uint32_t s, uint64_t my_off,
                                       uint32_t my_len, bool live, bool this_wide, uint32_t need_max,
                                       uint32_t* w0) {
    // bytes from a0 that round A read, and whether they hold what header_end reads
    const uint32_t a_end = this_wide ? round_a_end_wide(my_off & ~15ull, s, my_len, need_max)
                                     : min(64u, s + min(my_len, a.lean));
    const bool cov = a_end >= s + min(my_len, 28u);
    const uint32_t end = !live ? 0u
                       : cov ? s + header_end(w0, my_len, kNeedFilter)
                             : s + min(my_len, need_max);
    const uint32_t lo = (a_end + 15u) >> 4;   // first chunk round A did not read
    const bool my_nb = end > 16u * lo;
    if (__ballot(my_nb) != 0ull) {
        const bool second = __ballot(my_nb && lo < 4u && end > 16u * (lo + 4u)) != 0ull;
        load_round_b<-1>(a, t, lane, qa0, my_nb ? (lo | (end << 8)) : 0u, img, second);
        wave_lds_sync();
        window<10>(row, s, w0);
    }
    bool wide = __popcll(__ballot(end > 64u)) > 32;
    if (a.nt & 12u) wide = (a.nt & 8u) != 0u;
    return wide;
}

constexpr uint32_t kOob = 0x80000000u;           // buffer offset past every range: dropped / reads 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Whether bt_parse_filter_main issues the next tile's loads after the record stores (see
// the kernel); launch_t sizes the grid by it.
constexpr bool late_issue(int fixed_log2, int rec, int filter, bool prefetch) {
    return fixed_log2 >= 0 && !prefetch && rec != kRecAoS && filter == 1;
}

// Waves per SIMD the compiler must fit bt_parse_filter_main into (1: no constraint). PAYLOAD
// programs in descriptor mode: 4, the LDS residency (4 blocks/CU), so that the register budget
// (128 VGPRs) does not hold the kernel at 3 and the window loads and the walk have a fourth
// wave to hide behind (C3 with /GET|POST/ first, records: 0.818-0.836 against 0.908-0.917 ms,
// with /GET|POST/ last 0.773-0.777 against 0.912-0.916; tools/gpu_payload_libs.sh,
// profiles/r06/payload/libs_wpe4.log). launch_t runs those programs without the next-tile
// prefetch, whose registers would spill at 128 (as would AoS records').
constexpr int main_waves_per_eu(int fixed_log2, int rec, int filter, bool prefetch) {
    return fixed_log2 < 0 && filter == 2 && !prefetch && rec != kRecAoS ? 4 : 1;
}

template <int FIXED_LOG2, int REC, int FILTER, bool PREFETCH>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(main_waves_per_eu(FIXED_LOG2, REC, FILTER, PREFETCH))))
void bt_parse_filter_main(MainArgs a, DevProgram prog) {
    // Per-wave LDS image: 64 rows x 33 dwords.
    constexpr uint32_t kRow = row_dw<FIXED_LOG2>();
    // a wave's image; with AoS records at least the tile's 6 KiB of bt_rec (staged below)
    constexpr uint32_t kImg = REC == kRecAoS && kRow < BT_REC_BYTES / 4 ? kWave * (BT_REC_BYTES / 4) : kWave * kRow;
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[kWavesPerBlock * kImg + 32];   // + tail pad
    extern __shared__ uint4 dyn_lds[];   // PAYLOAD DFA pool (a.dfa_bytes), else empty
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform
    uint32_t* img = lds_all + wid * kImg;
    const uint32_t* row = img + lane * kRow;
    if (FILTER == 2 && a.dfa_bytes) {   // uniform: the whole block copies the pool once
        const uint4* src = reinterpret_cast<const uint4*>(a.dfa);
        for (uint32_t k = threadIdx.x; k < (a.dfa_bytes + 15u) / 16u && BT_IN(&g_bounds_main, kSitePayload, 16u * k, kDfaPoolMax); k += kBlock)
            dyn_lds[k] = src[k];
        __syncthreads();
    }
    const uint8_t* dfa_lds = reinterpret_cast<const uint8_t*>(dyn_lds);

    const uint32_t total_waves = gridDim.x * kWavesPerBlock;

    // Tile order: cyclic (wave w takes w, w+W, ...) or blocked (wave w takes one
    // contiguous range, so concurrent accesses spread over the whole buffer).
    const uint32_t gw = blockIdx.x * kWavesPerBlock + wid;
    uint32_t t, t_end, step;
    if (a.blocked) {
        const uint32_t per = (a.ntiles + total_waves - 1) / total_waves;
        t = gw * per;
        t_end = min(a.ntiles, t + per);
        step = 1;
    } else {
        t = gw;
        t_end = a.ntiles;
        step = total_waves;
    }
    const uint32_t need_max = REC != kRecNone ? kNeedParse : kNeedFilter;
    const HotProgram hot = hot_program(prog);
    bool wide = false;   // wave-uniform: previous tile mostly needed chunks 4..7
    Stage<FIXED_LOG2> st;
    // Fixed stride (not AoS): the next tile's loads are issued right after this tile's
    // record stores, so they are in flight while the filter runs; only the decision and
    // verdict stores (two unconditional buffer stores) follow them, and the loop top waits
    // with vmcnt(2..5) instead of draining every store. The filter's dependent chain is
    // then no longer added to each tile's load latency, and the 64-B parse+filter runs at
    // 2 blocks/CU like the parse alone (c2f kernel 0.327 against 0.343-0.350 ms at 3
    // blocks/CU without it; profiles/r02/ab/c2f_late_issue.txt). Not with PAYLOAD slots,
    // whose staging loads would have to wait behind the next tile's loads, and not
    // parse-only (nothing to overlap: C2 0.321 against 0.319 ms). Its header loads are
    // always non-temporal (BT_OPT_CACHE_DEFAULT keeps the default policy for the rest).
    constexpr bool LATE = late_issue(FIXED_LOG2, REC, FILTER, PREFETCH);
    if ((PREFETCH || LATE) && t < t_end) issue_loads<FIXED_LOG2, LATE>(a, t, lane, st, wide, need_max);
    if (LATE && FILTER && t < t_end) {
        // stand-ins for a tile's decision / verdict stores (an empty range: dropped), so
        // the loop top's wait counts the same operations on the first iteration as later
        const auto r = rsrc_of(g_zero16, 0u);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, r, 0, 0, 0);
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 z = {0u, 0u};
        __builtin_amdgcn_raw_buffer_store_b64(z, r, 16, 0, 0);
    }
    for (; t < t_end; t += step) {
        const uint32_t p0 = t * 64u;
        const uint32_t my = p0 + lane;
        const bool live = my < a.n;

        // ---- 1. LOAD (this tile's windows -> LDS; next tile's loads go in flight) ----
        if (!PREFETCH && !LATE) issue_loads<FIXED_LOG2>(a, t, lane, st, wide, need_max);
        stage_to_lds<FIXED_LOG2>(st, img, lane);
        const uint64_t my_off = st.off;
        const uint32_t my_len = st.len;
        uint64_t qa0[FIXED_LOG2 >= 0 ? 1 : 4];
#pragma unroll
        for (int j = 0; j < (FIXED_LOG2 >= 0 ? 1 : 4); ++j) qa0[j] = st.qa0[j];
        wave_lds_sync();
        const bool this_wide = FIXED_LOG2 < 0 && st.wide;
        if (PREFETCH && t + step < t_end) issue_loads<FIXED_LOG2>(a, t + step, lane, st, wide, need_max);
        // the packet's first 40 bytes; read once here (round A's chunks hold them) and
        // again only if round B rewrote the row
        const uint32_t s = (FIXED_LOG2 >= 0) ? 0u : ((uint32_t)my_off & 15u);
        uint32_t w0[10];
        window<10>(row, s, w0);
        if constexpr (FIXED_LOG2 < 0) {
            if (REC != kRecNone)   // filter-only needs <= 38 B: round A always suffices
                wide = round_b(a, t, lane, qa0, img, row, s, my_off, my_len, live, this_wide, need_max, w0);
        }

        // ---- 2. PARSE -------------------------------------------------------
        const uint32_t len = live ? my_len : 0u;

        if (REC != kRecNone && live) {
            Parsed p;
            if (REC == kRecPlanes || REC == kRecTiled) {
                // packed device record: its first `ns` slabs (2..6) hold every parsed field
                const uint32_t ns = parse_packet<true>(row, s, len, w0, p);
                if (REC == kRecTiled) {
                    // [tile][slab][slot]: slabs 0 and 1 at the lane's slot; slab k >= 2 only
                    // for the lanes that need it, packed to the front of the tile's slab-k
                    // region in lane order, so the stores fill whole 128-B lines except the
                    // last one of each region.
                    uint4* tile = reinterpret_cast<uint4*>(a.records) + (uint64_t)t * (BT_REC_SLABS * 64);
                    const uint64_t below = (1ull << lane) - 1ull;
                    const bool rec_in = BT_IN(&g_bounds_main, kSiteRecord, t, (a.n_cap + 63u) / 64u);
#pragma unroll
                    for (uint32_t k = 0; k < BT_REC_SLABS; ++k) {
                        const uint64_t mk = __ballot(k < ns);
                        if (mk == 0ull) break;   // ns only falls: no lane needs a later slab
                        if (k < ns && rec_in)
                            st16(tile + k * 64 + (k < 2u ? lane : (uint32_t)__popcll(mk & below)),
                                 make_uint4(p.r[4 * k], p.r[4 * k + 1], p.r[4 * k + 2], p.r[4 * k + 3]), a.nt & 1u);
                    }
                } else {
                    // plane-major: slab k is stored by the whole wave when any lane needs it
                    // (the other lanes' dwords there are 0)
                    uint4* dst = reinterpret_cast<uint4*>(a.records) + (uint64_t)my;
#pragma unroll
                    for (uint32_t k = 0; k < BT_REC_SLABS; ++k)
                        if ((k < 2u || __ballot(k < ns) != 0ull) && BT_IN(&g_bounds_main, kSiteRecord, my, a.n_cap))
                            st16(dst + (uint64_t)k * a.n_cap,
                                 make_uint4(p.r[4 * k], p.r[4 * k + 1], p.r[4 * k + 2], p.r[4 * k + 3]), a.nt & 1u);
                }
            }
        }
        Parsed aos;   // AoS: the 96-B bt_rec, stored after the filter through LDS (below)
        if (REC == kRecAoS) {
            parse_packet<false>(row, s, len, w0, aos);
            if (!live)
#pragma unroll
                for (int k = 0; k < 24; ++k) aos.r[k] = 0u;
        }

        if (REC == kRecTiled && !live) {
            // the last tile's unused slots: a zero slab 1 reads as a 2-slab record, so a
            // reader can rebuild the slab-k packing of the tile without knowing n
            uint4* tile = reinterpret_cast<uint4*>(a.records) + (uint64_t)t * (BT_REC_SLABS * 64);
            if (BT_IN(&g_bounds_main, kSiteRecord, t, (a.n_cap + 63u) / 64u)) {
                st16(tile + lane, make_uint4(0, 0, 0, 0), a.nt & 1u);
                st16(tile + 64 + lane, make_uint4(0, 0, 0, 0), a.nt & 1u);
            }
        }

        if (LATE && t + step < t_end) issue_loads<FIXED_LOG2, LATE>(a, t + step, lane, st, wide, need_max);
        // ---- 3. FILTER ------------------------------------------------------
        if (FILTER) {
            uint32_t slot;
            // round A's 64-B window (descriptor mode, whole windows, not a wide tile, whose
            // line-bounded round A may stop short of it) is still in the row for PAYLOAD slots
            const uint32_t reuse = FIXED_LOG2 < 0 && a.lean == 0xFFFFu && !this_wide ? 4u : 0u;
            const uint32_t code = filter_packet<FILTER>(a, prog, hot, dfa_lds, img + lane * kRow, kRow, my_off, len, w0, live,
                                                        slot, reuse);
            const uint64_t pass = __ballot(live && code == BT_DECIDE_PASS);
            if (LATE) {   // unconditional buffer stores: a static count behind the next loads
                const uint32_t cnt = min(64u, a.n - p0);
                const auto rd = rsrc_of(a.decide ? a.decide + p0 : nullptr, a.decide ? cnt : 0u);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((code << 6) | slot), rd, (int)lane, 0, 0);
                const bool v_in = BT_IN(&g_bounds_main, kSiteVerdict, t, a.ntiles);
                const auto rv = rsrc_of(a.verdict ? a.verdict + t : nullptr, a.verdict && v_in ? 8u : 0u);
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 pv = {(uint32_t)pass, (uint32_t)(pass >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(pv, rv, lane == 0 ? 0 : (int)kOob, 0, 0);
            } else {
                if (a.decide && live && BT_IN(&g_bounds_main, kSiteDecide, my, a.n)) a.decide[my] = (uint8_t)((code << 6) | slot);
                if (lane == 0 && a.verdict && BT_IN(&g_bounds_main, kSiteVerdict, t, a.ntiles))
                    a.verdict[t] = pass;   // also the compaction's input
            }
        }
        // ---- 4. AoS records: the tile's 64 bt_rec are one contiguous 6-KiB range. Each
        // lane's 96 B are written to the wave's LDS image (the row is free once the filter
        // has run) and the wave stores the range 1 KiB per instruction, so every store is
        // a whole-line, fully coalesced write instead of 64 segments 96 B apart (C3:
        // 0.90 ms with per-lane stores).
        if (REC == kRecAoS) {
            wave_lds_sync();   // the filter's row reads (PAYLOAD staging) are done
            uint4* lrec = reinterpret_cast<uint4*>(img);   // 6 KiB: the image, or kImg's extension
#pragma unroll
            for (uint32_t k = 0; k < BT_REC_SLABS; ++k)
                lrec[lane * BT_REC_SLABS + k] = make_uint4(aos.r[4 * k], aos.r[4 * k + 1], aos.r[4 * k + 2], aos.r[4 * k + 3]);
            wave_lds_sync();
            const uint32_t q_end = min(64u, a.n - p0) * BT_REC_SLABS;   // live records only
            uint4* dst = reinterpret_cast<uint4*>(a.records + (uint64_t)p0 * BT_REC_BYTES);
#pragma unroll
            for (uint32_t i = 0; i < BT_REC_SLABS; ++i) {
                const uint32_t q = i * 64u + lane;
                if (q < q_end && BT_IN(&g_bounds_main, kSiteRecord, (uint64_t)p0 * BT_REC_SLABS + q,
                                       (uint64_t)a.n_cap * BT_REC_SLABS))
                    st16(dst + q, lrec[q], a.nt & 1u);
            }
        }
        wave_lds_sync();   // the next tile overwrites this wave's image
    }
}

// ---- descriptor-mode pipeline with counted waits ------------------------------
// gfx950 has one vmcnt counter for loads AND stores, retired in issue order. In
// bt_parse_filter_main the loop top waits for the prefetched header loads, and because
// some paths between the prefetch and that wait issue fewer stores (exec-skipped
// blocks, the early `break` of the slab loop, null outputs), the compiler can only
// emit vmcnt(0) there: every tile waited for its predecessor's record stores to be
// acknowledged, and for the next tile's descriptor load right after. Here every store
// of a tile is an unconditional buffer store (lanes that must not write get an
// offset past the descriptor's range, which the hardware drops), the header loads of
// lanes with nothing to read load a zero line instead of being skipped, and the
// descriptors are loaded one tile ahead. Every path then issues the same operations,
// so the wait for the next tile's headers is vmcnt(K) with K = this tile's stores:
// the stores retire in the background.


// The descriptors of tile t as the wave needs them: `me` = this lane's packet (the
// parse), q[j] = packet j*16 + lane/4 (round A: four lanes per packet). Both are buffer
// loads of the same 512-B tile slice (the q loads hit the lines the `me` load brings
// in), zero past n or when !valid; loading q directly replaces three ds_bpermute
// shuffles per round-A instruction. DW = descriptor words (1 bt_pkt_desc, 2 xdp_desc), a
// template argument so that no register is written on one format's path and loaded on
// the other's.
// Cache policy of the descriptor loads (buffer-load aux bits; 2 = nt). A lane's own
// descriptor load keeps the default policy and the four round-A loads, which re-read the
// lines it brings in, are non-temporal: C3 kernel 0.470-0.474 against 0.475-0.488 ms on
// one box, 0.5 % on another, C4 level; both non-temporal made C3 0.504-0.508
// (profiles/r02/ab/desc_policy.txt).
#ifndef BT_DESC_AUX
#define BT_DESC_AUX 0
#endif
#ifndef BT_DESC_AUX_Q
#define BT_DESC_AUX_Q 2
#endif
template <int DW>
struct TileDesc {
    uint32_t me[DW + 1];
    uint32_t q[4][DW + 1];
};

template <int DW>
__device__ __forceinline__ void load_desc_pipe(const MainArgs& a, uint32_t t, bool valid, uint32_t lane,
                                               TileDesc<DW>& d) {
    const uint32_t p0 = t * 64u;
    const uint32_t cnt = valid && p0 < a.n ? min(64u, a.n - p0) : 0u;
    const auto r = rsrc_of(a.desc + (valid ? (uint64_t)DW * p0 : 0ull), cnt * 8u * DW);
    const uint32_t qoff = (lane >> 2) * 8u * DW;
    if constexpr (DW == 1) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(lane * 8u), 0, BT_DESC_AUX);
        d.me[0] = v.x; d.me[1] = v.y;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(qoff + j * 128u), 0, BT_DESC_AUX_Q);
            d.q[j][0] = w.x; d.q[j][1] = w.y;
        }
    } else {
        typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
        const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)(lane * 16u), 0, BT_DESC_AUX);
        d.me[0] = v.x; d.me[1] = v.y; d.me[2] = v.z;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(r, (int)(qoff + j * 256u), 0, BT_DESC_AUX_Q);
            d.q[j][0] = w.x; d.q[j][1] = w.y; d.q[j][2] = w.z;
        }
    }
}

template <int DW>
__device__ __forceinline__ void decode_desc(const uint32_t (&w)[DW + 1], uint64_t& off, uint32_t& len) {
    if constexpr (DW == 1) {   // bt_pkt_desc: off in bits 0..47, len in 48..63
        off = ((uint64_t)(w[1] & 0xFFFFu) << 32) | w[0];
        len = w[1] >> 16;
    } else {                   // xdp_desc {u64 addr; u32 len; u32 options}
        off = ((uint64_t)w[1] << 32) | w[0];
        len = w[2] > 0xFFFFu ? 0xFFFFu : w[2];
    }
}

// Round A of tile t from descriptors already in registers (issue_loads' loads, with the
// zero line standing in for the skipped ones). A packet past n has an all-zero
// descriptor: off = len = 0, so nothing of it is read.
template <int DW>
__device__ __forceinline__ void issue_round_a_pipe(const MainArgs& a, uint32_t lane, const TileDesc<DW>& d,
                                                   Stage<-1>& st, bool wide, uint32_t need_max) {
    decode_desc<DW>(d.me, st.off, st.len);
    const uint32_t c = lane & 3u;
    st.wide = wide;
    const bool ntl = (a.nt & 2u) && !wide;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero16);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        uint64_t qo;
        uint32_t ql;
        decode_desc<DW>(d.q[j], qo, ql);
        const uint64_t a0 = qo & ~15ull;
        const uint64_t addr = a0 + 16u * c;
        const uint32_t sq = (uint32_t)qo & 15u;
        st.qa0[j] = a0;
        // bitwise & keeps the conditions branch-free (&& made exec-mask branches)
        const uint32_t a_end = wide ? round_a_end_wide(a0, sq, ql, need_max) : sq + min(ql, a.lean);
        const uint32_t a_lo = wide ? 0u : sq + a.lean_lo;   // chunks ending at or before it: unread
        const bool ok = (16u * c < a_end) & (16u * c + 16u > a_lo) & (addr + 16u <= a.bytes);
        st.v[j] = ld16(ok ? a.base + addr : zero, ntl);
        if (wide) {
            const bool okb = (16u * (c + 4u) < a_end) & (addr + 64u + 16u <= a.bytes);
            st.v[4 + j] = ld16(okb ? a.base + addr + 64u : zero, false);
        }
    }
}

// The stores of one tile, all unconditional (see above): K = 6 slab stores (tiled
// records) + 3 filter outputs. Record stores are always non-temporal here (a runtime
// choice of policy would be a branch, and a path that skips both stores).
template <bool NT>
__device__ __forceinline__ void st_b128(const __amdgpu_buffer_rsrc_t& r, uint32_t off, uint4 v) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)off, 0, NT ? 2 : 0);
}

template <int REC, int FILTER>
__device__ __forceinline__ void pad_stores() {   // the prologue's stand-ins for a tile's stores
    const auto r = rsrc_of(g_zero16, 0u);
    const u32x4 z = {0u, 0u, 0u, 0u};
    // distinct offsets, or the compiler merges them (the range is empty: all are dropped)
    if (REC == kRecTiled)
#pragma unroll
        for (int k = 0; k < BT_REC_SLABS; ++k) __builtin_amdgcn_raw_buffer_store_b128(z, r, 16 * k, 0, 0);
    if (FILTER)
#pragma unroll
        for (int k = 0; k < 3; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, r, 256 + 16 * k, 0, 0);
}

// Descriptor mode only. A fixed-stride form (contiguous 1-KiB loads, prefetched) was
// measured slower on C2 (0.369 against 0.340 ms for bt_parse_filter_main without
// prefetch, at 1-4 blocks/CU): there, a wave's loads in flight during its record stores
// cost more HBM efficiency than the hidden latency gains.
template <int REC, int FILTER, int DW>
__global__ __launch_bounds__(kBlock) void bt_parse_filter_pipe(MainArgs a, DevProgram prog) {
    static_assert(REC == kRecTiled || REC == kRecNone, "pipe variant: tiled records or none");
    constexpr uint32_t kRow = kRowDwords;
    __shared__ uint32_t lds_all[kWavesPerBlock * kWave * kRow + 32];   // + tail pad for over-reads
    extern __shared__ uint4 dyn_lds[];   // PAYLOAD DFA pool (a.dfa_bytes), else empty
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably wave-uniform
    uint32_t* img = lds_all + wid * (kWave * kRow);
    const uint32_t* row = img + lane * kRow;
    if (FILTER == 2 && a.dfa_bytes) {
        const uint4* src = reinterpret_cast<const uint4*>(a.dfa);
        for (uint32_t k = threadIdx.x; k < (a.dfa_bytes + 15u) / 16u && BT_IN(&g_bounds_main, kSitePayload, 16u * k, kDfaPoolMax); k += kBlock)
            dyn_lds[k] = src[k];
        __syncthreads();
    }
    const uint8_t* dfa_lds = reinterpret_cast<const uint8_t*>(dyn_lds);

    const uint32_t total_waves = gridDim.x * kWavesPerBlock;
    const uint32_t gw = blockIdx.x * kWavesPerBlock + wid;
    uint32_t t, t_end, step;
    if (a.blocked) {
        const uint32_t per = (a.ntiles + total_waves - 1) / total_waves;
        t = gw * per;
        t_end = min(a.ntiles, t + per);
        step = 1;
    } else {
        t = gw;
        t_end = a.ntiles;
        step = total_waves;
    }
    if (t >= t_end) return;   // wave-uniform; no block barrier follows
    const uint32_t need_max = REC != kRecNone ? kNeedParse : kNeedFilter;
    const HotProgram hot = hot_program(prog);
    bool wide = false;

    // prologue: descriptors of t and t + step, round A of t (waited), then stand-ins for
    // a tile's stores so the first iteration's waits count like every later one's
    Stage<-1> st;
    TileDesc<DW> dn;
    load_desc_pipe<DW>(a, t, true, lane, dn);
    issue_round_a_pipe<DW>(a, lane, dn, st, wide, need_max);
    load_desc_pipe<DW>(a, t + step, t + step < t_end, lane, dn);
    pad_stores<REC, FILTER>();
    stage_to_lds<-1>(st, img, lane);
    wave_lds_sync();

    for (;;) {
        const uint32_t p0 = t * 64u;
        const uint32_t my = p0 + lane;
        const bool live = my < a.n;
        const uint64_t my_off = st.off;
        const uint32_t my_len = st.len;
        const uint32_t s = (uint32_t)my_off & 15u;
        uint32_t w0[10];
        window<10>(row, s, w0);
        if (REC != kRecNone)   // round B, before the next tile's loads
            wide = round_b(a, t, lane, st.qa0, img, row, s, my_off, my_len, live, st.wide, need_max, w0);

        // next tile: round A from the descriptors loaded one tile ago, then the
        // descriptors of the tile after it
        const uint32_t tn = t + step;
        const bool more = tn < t_end;
        issue_round_a_pipe<DW>(a, lane, dn, st, wide, need_max);
        load_desc_pipe<DW>(a, tn + step, more && tn + step < t_end, lane, dn);

        // ---- PARSE + tiled record stores ----
        const uint32_t len = live ? my_len : 0u;
        if (REC == kRecTiled) {
            Parsed p;
            uint32_t ns = parse_packet<true>(row, s, len, w0, p);
            if (!live) {   // the last tile's unused slots: zero slabs 0-1 (a 2-slab record)
                ns = 2u;
#pragma unroll
                for (int k = 0; k < 8; ++k) p.r[k] = 0u;
            }
            const bool rec_in = BT_IN(&g_bounds_main, kSiteRecord, t, (a.n_cap + 63u) / 64u);
            const auto r = rsrc_of(a.records + (uint64_t)t * (BT_REC_SLABS * 64 * 16), rec_in ? BT_REC_SLABS * 64 * 16 : 0u);
            const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
            for (uint32_t k = 0; k < BT_REC_SLABS; ++k) {
                const uint64_t mk = __ballot(k < ns);
                const uint32_t off = k < 2u ? (k * 64u + lane) * 16u
                                   : k < ns ? (k * 64u + (uint32_t)__popcll(mk & below)) * 16u : kOob;
                st_b128<true>(r, off, make_uint4(p.r[4 * k], p.r[4 * k + 1], p.r[4 * k + 2], p.r[4 * k + 3]));
            }
        }

        // ---- FILTER ----
        if (FILTER) {
            uint32_t slot;
            const uint32_t code = filter_packet<FILTER>(a, prog, hot, dfa_lds, img + lane * kRow, kRow, my_off, len, w0, live, slot);
            const uint64_t pass = __ballot(live && code == BT_DECIDE_PASS);
            const uint32_t cnt = min(64u, a.n - p0);
            const auto rd = rsrc_of(a.decide ? a.decide + p0 : nullptr, a.decide ? cnt : 0u);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((code << 6) | slot), rd, (int)lane, 0, 0);
            const bool v_in = BT_IN(&g_bounds_main, kSiteVerdict, t, a.ntiles);
            const auto rv = rsrc_of(a.verdict ? a.verdict + t : nullptr, a.verdict && v_in ? 8u : 0u);
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 pv = {(uint32_t)pass, (uint32_t)(pass >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(pv, rv, lane == 0 ? 0 : (int)kOob, 0, 0);
        }

        wave_lds_sync();   // this tile's LDS reads are done
        if (!more) break;
        stage_to_lds<-1>(st, img, lane);
        wave_lds_sync();
        t = tn;
    }
}

// ---- ordered compaction of passing packet indices ---------------------------------
// K2: chunk_sums[c] = the passing packets of chunk c (kChunkTiles = 256 tiles, one per
// thread): the popcounts of the tiles' verdict words.
__global__ __launch_bounds__(256) void bt_chunk_sums(const uint64_t* verdict, uint32_t ntiles,
                                                     uint32_t* chunk_sums, uint32_t nchunks) {
    static_assert(kChunkTiles == 256, "one tile per thread");
    __shared__ uint32_t red[4];
    const uint32_t t = blockIdx.x * kChunkTiles + threadIdx.x;
    uint32_t s = t < ntiles ? (uint32_t)__popcll(verdict[t]) : 0u;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0 && BT_IN(&g_bounds_main, kSiteChunkSums, blockIdx.x, nchunks))
        chunk_sums[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// K3: block c scans its chunk's 256 tile counts, adds the prefix of earlier chunks and
// writes the indices of passing packets in ascending order. Thread tid owns tile tid
// (its count and verdict word go to LDS in one coalesced pass); wave w then scatters
// tiles 64w..64w+63, so each wave's stores run forward through one contiguous range
// of pass_idx, and the set lanes of one verdict word store to consecutive slots. Four
// tiles per step keep the LDS reads of the next tiles in flight behind the stores.
// (The first version had 1024-tile chunks, i.e. 256 blocks = one per CU, and a
// strided one-tile loop: 34 us on C3.)
__global__ __launch_bounds__(256) void bt_compact(const uint64_t* verdict, const uint32_t* chunk_sums,
                                                  uint32_t nchunks, uint32_t ntiles, uint32_t n, uint32_t* pass_idx,
                                                  uint32_t* n_pass) {
    __shared__ uint32_t tile_off[kChunkTiles];
    __shared__ uint64_t words[kChunkTiles];
    __shared__ uint32_t red[4];
    __shared__ uint32_t wsum[4];
    const uint32_t c = blockIdx.x;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t t = c * kChunkTiles + tid;
    const uint64_t word = t < ntiles ? verdict[t] : 0ull;   // issued before the prefix loop

    // prefix of earlier chunks (and the grand total for n_pass)
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = tid; i < nchunks; i += 256) {
        const uint32_t x = chunk_sums[i];
        tot += x;
        if (i < c) pre += x;
    }
    for (int o = 32; o > 0; o >>= 1) { pre += __shfl_xor(pre, o); tot += __shfl_xor(tot, o); }
    if (lane == 0) { red[wid] = pre; wsum[wid] = tot; }
    __syncthreads();
    const uint32_t base = red[0] + red[1] + red[2] + red[3];
    if (c == 0 && tid == 0 && n_pass) *n_pass = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (!pass_idx) return;   // count only
    __syncthreads();

    const uint32_t v = (uint32_t)__popcll(word);   // the tile's passing packets
    uint32_t incl = v;   // inclusive wave scan of the tile counts
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) red[wid] = incl;
    words[tid] = word;
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t w = 0; w < wid; ++w) wpre += red[w];
    tile_off[tid] = base + wpre + incl - v;
    __syncthreads();

    const uint64_t below_mask = (1ull << lane) - 1ull;
    const uint32_t first = wid * 64u;
    for (uint32_t i = 0; i < 64u; i += 4u) {
        uint64_t w4[4];
        uint32_t o4[4];
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) { w4[k] = words[first + i + k]; o4[k] = tile_off[first + i + k]; }
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k)
            if (((w4[k] >> lane) & 1ull) &&
                BT_IN(&g_bounds_main, kSitePassIdx, o4[k] + (uint32_t)__popcll(w4[k] & below_mask), n))
                pass_idx[o4[k] + (uint32_t)__popcll(w4[k] & below_mask)] = (c * kChunkTiles + first + i + k) * 64u + lane;
    }
}

int cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        hipDeviceProp_t prop;
        cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                  ? prop.multiProcessorCount : 256;
    }
    return cus;
}

// One residency wave of blocks: the persistent grid-stride loop then has no tail of
// late blocks (measured: 2x residency cost C3 11 %). Cached per kernel instantiation
// (the template argument), and for PAYLOAD programs per dynamic-LDS size.
template <auto Kernel>
int resident_grid(uint32_t dyn) {
    static int blocks = 0;
    static uint32_t last_dyn = ~0u;
    static int last_blocks = 0;
    static std::mutex mu;
    auto query = [&](uint32_t bytes) {
        int dev = 0, per_cu = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, Kernel, kBlock, bytes) != hipSuccess || per_cu < 1)
            return 1024;
        return prop.multiProcessorCount * per_cu;
    };
    std::lock_guard<std::mutex> lk(mu);
    if (dyn) {   // a PAYLOAD program: occupancy depends on its DFA pool size
        if (dyn != last_dyn) {
            last_blocks = query(dyn);
            last_dyn = dyn;
        }
        return last_blocks;
    }
    if (!blocks) blocks = query(0);
    return blocks;
}

// The counted-wait pipeline (bt_parse_filter_pipe) serves descriptor mode with tiled
// records or none; BT_NO_PIPE=1 in the environment selects bt_parse_filter_main
// instead (A/B).
bool use_pipe() {
    static const bool on = [] {
        const char* e = getenv("BT_NO_PIPE");
        return !(e && *e && *e != '0');
    }();
    return on;
}

template <int FL, int REC, int F>
void launch_t(const MainArgs& a, const DevProgram& prog, int grid, bool pf, hipStream_t st, hipEvent_t e0,
              hipEvent_t e1) {
    const uint32_t needed = (a.ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t dyn = F == 2 ? (a.dfa_bytes + 15u) & ~15u : 0u;
    auto go = [&](auto kernel, int resident) {
        int g = grid > 0 ? grid : resident;
        // Fixed stride: two blocks (8 waves) per CU parse-only, three with a filter. C2
        // measured 0.416 ms at the residency (7 blocks/CU), 0.403 at 3, 0.387 at 2, 0.56
        // at 1 (4 processes each): fewer concurrent read and write streams suit HBM
        // better; with the final kernels 0.338-0.341 at 2 against 0.353-0.356 at 3. With
        // the filter (its decision / verdict stores and the slot loop per tile) the 64-B
        // parse+filter headline needs more waves: 0.366-0.368 ms at 3 blocks/CU against
        // 0.378-0.379 at 4 and 0.420-0.426 at 2 (round 2, alternating processes, 3
        // passes each; round 1's code was best at 4).
        // With the late issue (bt_parse_filter_main) the filter no longer needs the third
        // block: c2f 0.327 ms at 2 blocks/CU against 0.343-0.350 at 3 without it.
        if (FL >= 0 && grid <= 0) g = std::min(g, (F && !late_issue(FL, REC, F, false) ? 3 : 2) * cu_count());
        if ((uint32_t)g > needed) g = (int)(needed ? needed : 1);
        if (e0 || e1)
            hipExtLaunchKernelGGL(kernel, dim3(g), dim3(kBlock), dyn, st, e0, e1, 0, a, prog);
        else
            hipLaunchKernelGGL(kernel, dim3(g), dim3(kBlock), dyn, st, a, prog);
    };
    // Not for PAYLOAD programs (F == 2): bt_parse_filter_main at its residency hides the window
    // loads and the walk better than the pipe at 2 blocks/CU (C3 with /GET|POST/ first 0.885
    // against 0.98 ms, filter-only 0.60 against 0.87; tools/payload_ab.py with BT_NO_PIPE).
    if constexpr (FL < 0 && F != 2 && (REC == kRecTiled || REC == kRecNone)) {
        if (pf && a.desc && (a.nt & 1u) && use_pipe()) {
            // At most 2 blocks/CU (the residency is 3): with the filter slots evaluated side
            // by side, C3 0.491 against 0.498 ms and C4 0.915 against 0.948 at the residency
            // (profiles/r02/ab/pipe_grid.txt; before that change the residency was level or
            // better).
            const int cap2 = 2 * cu_count();
            if (a.desc_words == 1)
                go(bt_parse_filter_pipe<REC, F, 1>,
                   grid > 0 ? 0 : std::min(cap2, resident_grid<bt_parse_filter_pipe<REC, F, 1>>(dyn)));
            else
                go(bt_parse_filter_pipe<REC, F, 2>,
                   grid > 0 ? 0 : std::min(cap2, resident_grid<bt_parse_filter_pipe<REC, F, 2>>(dyn)));
            return;
        }
    }
    static const bool fixed_pf = [] {   // A/B: next-tile prefetch in fixed-stride mode
        const char* e = getenv("BT_FIXED_PREFETCH");
        return e && *e && *e != '0';
    }();
    // PAYLOAD programs in descriptor mode: no next-tile prefetch (main_waves_per_eu)
    if (FL < 0 && F == 2) pf = false;
    // PAYLOAD programs in descriptor mode run one block per 12 tiles (three per wave), not one
    // residency wave of blocks: without the prefetch there is nothing for a persistent block to
    // carry from tile to tile, and a residency grid that fills every CU leaves none for the
    // previous step's compaction, so that some of its blocks start only when others end (C3 with
    // /GET|POST/ first, pipelined steps: 0.771-0.775 ms at one tile per wave against 1.080-1.142
    // at the residency and 0.892-0.895 at 3 blocks/CU; two / three / four / eight / sixteen tiles
    // per wave 0.775-0.778 / 0.753 / 0.756-0.759 / 0.764-0.767 / 0.803 ms; tools/gpu_payload_grid.sh,
    // profiles/r06/payload/grid/).
    // BT_PAYLOAD_GRID (A/B): blocks per CU instead, 0 = the residency, -k = one block per 4k tiles.
    static const int pay_grid = [] {
        const char* e = getenv("BT_PAYLOAD_GRID");
        return e && *e ? atoi(e) : -3;
    }();
    if (pf && (FL < 0 || fixed_pf)) go(bt_parse_filter_main<FL, REC, F, true>, grid > 0 ? 0 : resident_grid<bt_parse_filter_main<FL, REC, F, true>>(dyn));
    else if (FL < 0 && F == 2 && grid <= 0 && pay_grid)
        go(bt_parse_filter_main<FL, REC, F, false>,
           pay_grid < 0 ? (int)((needed + (uint32_t)(-pay_grid) - 1u) / (uint32_t)(-pay_grid))
                        : std::min(pay_grid * cu_count(), resident_grid<bt_parse_filter_main<FL, REC, F, false>>(dyn)));
    else go(bt_parse_filter_main<FL, REC, F, false>, grid > 0 ? 0 : resident_grid<bt_parse_filter_main<FL, REC, F, false>>(dyn));
}

template <int FL>
void launch_fl(const MainArgs& a, const DevProgram& prog, int rec, int f, int grid, bool pf, hipStream_t st,
               hipEvent_t e0, hipEvent_t e1) {
    // f: 0 no filter, 1 built-in slots only (uniform predicates), 2 with PAYLOAD slots
    auto by_f = [&](auto rec_c) {
        constexpr int R = decltype(rec_c)::value;
        if (f == 2) launch_t<FL, R, 2>(a, prog, grid, pf, st, e0, e1);
        else if (f == 1) launch_t<FL, R, 1>(a, prog, grid, pf, st, e0, e1);
        else launch_t<FL, R, 0>(a, prog, grid, pf, st, e0, e1);
    };
    if (rec == kRecPlanes) by_f(std::integral_constant<int, kRecPlanes>{});
    else if (rec == kRecTiled) by_f(std::integral_constant<int, kRecTiled>{});
    else if (rec == kRecAoS) by_f(std::integral_constant<int, kRecAoS>{});
    else if (f == 2) launch_t<FL, kRecNone, 2>(a, prog, grid, pf, st, e0, e1);
    else launch_t<FL, kRecNone, 1>(a, prog, grid, pf, st, e0, e1);
}

}  // namespace

int launch_main(const MainArgs& a, const DevProgram& prog, int rec_layout, bool filter, int grid_blocks,
                bool prefetch, void* stream, void* timing_start, void* timing_stop) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipEvent_t e0 = reinterpret_cast<hipEvent_t>(timing_start), e1 = reinterpret_cast<hipEvent_t>(timing_stop);
    const int grid = grid_blocks;   // <= 0: one residency wave of the chosen variant
    int fl = -1;   // fixed-stride fast path when the stride is 16/32/64/128 B
    if (!a.desc) {
        if (a.stride == 16) fl = 0;
        else if (a.stride == 32) fl = 1;
        else if (a.stride == 64) fl = 2;
        else if (a.stride == 128) fl = 3;
    }
    // Next-tile prefetch: the pipe kernel always prefetches (BT_OPT_NO_PREFETCH selects
    // bt_parse_filter_main without it). In bt_parse_filter_main it pays for descriptor
    // mode (+3 % C3) but not for fixed stride (-16 % C2); launch_t drops it there.
    // the filter variant: none, built-in slots only, or with PAYLOAD DFAs
    const int f = !filter ? 0 : a.dfa_bytes ? 2 : 1;
    switch (fl) {
    case 0: launch_fl<0>(a, prog, rec_layout, f, grid, prefetch, st, e0, e1); break;
    case 1: launch_fl<1>(a, prog, rec_layout, f, grid, prefetch, st, e0, e1); break;
    case 2: launch_fl<2>(a, prog, rec_layout, f, grid, prefetch, st, e0, e1); break;
    case 3: launch_fl<3>(a, prog, rec_layout, f, grid, prefetch, st, e0, e1); break;
    default: launch_fl<-1>(a, prog, rec_layout, f, grid, prefetch, st, e0, e1); break;
    }
    return hipGetLastError() == hipSuccess ? BT_OK : BT_E_INTERNAL;
}

int launch_compact(const uint64_t* verdict, uint32_t n, uint32_t* chunk_sums, uint32_t* pass_idx,
                   uint32_t* n_pass, void* stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint32_t ntiles = (n + 63u) / 64u;
    const uint32_t nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    if (nchunks == 0) return BT_OK;
    hipLaunchKernelGGL(bt_chunk_sums, dim3(nchunks), dim3(256), 0, st, verdict, ntiles, chunk_sums, nchunks);
    hipLaunchKernelGGL(bt_compact, dim3(nchunks), dim3(256), 0, st, verdict, chunk_sums, nchunks, ntiles, n, pass_idx,
                       n_pass);
    return hipGetLastError() == hipSuccess ? BT_OK : BT_E_INTERNAL;
}

uint32_t bounds_take_main(void* stream, BoundsLog* first) {
#ifdef BT_DEBUG_BOUNDS
    if (hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return 0;
    BoundsLog log{};
    if (hipMemcpyFromSymbol(&log, HIP_SYMBOL(g_bounds_main), sizeof(log)) != hipSuccess) return 0;
    if (log.count) {
        const BoundsLog zero{};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_main), &zero, sizeof(zero));
        if (first) *first = log;
    }
    return log.count;
#else
    (void)stream;
    (void)first;
    return 0;
#endif
}

int device_grid_blocks(int device) {
    (void)device;
    return 0;   // auto: one residency wave per kernel variant (resident_grid)
}

}  // namespace bt
