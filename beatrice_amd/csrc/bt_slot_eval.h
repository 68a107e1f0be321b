// bt_slot_eval.h — the built-in PacketFilter slot semantics, one copy for the kernels
// (bt_kernels.hip, the per-kind evaluator of programs with PAYLOAD slots) and the C++ drop-in
// layer (beatrice_amd/host/GpuPacketFilter.cpp: single packets, small batches, and the host
// continuation of a chain the device handed over at a PAYLOAD / CUSTOM slot).
//
// Reference: src/PacketFilter.cpp:168-286 (applyBPFFilter, applyIPFilter, applyPortFilter,
// applyProtocolFilter). Every built-in filter first requires length >= 34 and EtherType
// 0x0800 at frame bytes 12..13 (VLAN / IPv6 frames fail: SURVEY §8(a) R-QUIRK-F); IPs are read
// at the fixed offsets 26 / 30, the protocol at 23 and the ports at 34 / 36 (the port filter
// needs TCP with length >= 54 or UDP with length >= 42, :264-276).
#pragma once

#include <stdint.h>

#include "beatrice_gpu.h"

#if defined(__HIPCC__)
#define BT_SLOT_FN __host__ __device__ __forceinline__
#else
#define BT_SLOT_FN inline
#endif

namespace bt {

// What the built-in filters read of one packet. Fields the gates do not admit are 0, so a
// caller never reads a frame byte past `len`.
struct FilterIn {
    bool gate;          // len >= 34 && frame[12..13] == 0x0800
    bool l4_ok;         // gate && ((proto 6 && len >= 54) || (proto 17 && len >= 42))
    uint32_t proto, src, dst, sport, dport;
};

// `at(i)` returns frame byte i (i < 38); it is called only for bytes the gates admit.
template <class ByteAt>
BT_SLOT_FN FilterIn filter_in(const ByteAt& at, uint32_t len) {
    FilterIn x;
    const uint32_t et = len >= 34u ? (at(12) << 8) | at(13) : 0u;
    x.gate = et == 0x0800u;
    x.proto = x.gate ? at(23) : 0u;
    x.src = x.gate ? (at(26) << 24) | (at(27) << 16) | (at(28) << 8) | at(29) : 0u;
    x.dst = x.gate ? (at(30) << 24) | (at(31) << 16) | (at(32) << 8) | at(33) : 0u;
    x.l4_ok = ((x.proto == 6u) & (len >= 54u)) | ((x.proto == 17u) & (len >= 42u));
    x.sport = x.l4_ok ? (at(34) << 8) | at(35) : 0u;
    x.dport = x.l4_ok ? (at(36) << 8) | at(37) : 0u;
    return x;
}

// One compiled slot (bt_filter_slot kind / a / b) on one packet: 1 pass, 0 reject, 2 throw
// (the reference's std::stoi exception), 3 not built in (PAYLOAD / HOST: the caller's).
// Bitwise & / | throughout: on the device the short-circuit forms became exec-mask branches.
BT_SLOT_FN uint32_t eval_slot(uint32_t kind, uint32_t a, uint32_t b, const FilterIn& x) {
    switch (kind) {
    case BT_K_TRUE: return 1;
    case BT_K_FALSE: return 0;
    case BT_K_BPF:
        return x.gate & ((((a & 1u) != 0u) & (x.proto == 6)) | (((a & 2u) != 0u) & (x.proto == 17)) |
                         (((a & 4u) != 0u) & (x.proto == 1)));
    case BT_K_PROTO_EQ: return x.gate & (x.proto == a);
    case BT_K_PROTO_NZ: return x.gate & (x.proto != 0);
    case BT_K_IP_MASK: return x.gate & (((x.src & b) == a) | ((x.dst & b) == a));
    case BT_K_PORT:
        return x.gate & x.l4_ok & (((x.sport >= a) & (x.sport <= b)) | ((x.dport >= a) & (x.dport <= b)));
    case BT_K_IP_THROW: return x.gate ? 2u : 0u;
    case BT_K_PORT_THROW: return (x.gate & x.l4_ok) ? 2u : 0u;
    default: return 3;   // BT_K_PAYLOAD, BT_K_HOST
    }
}

}  // namespace bt

#undef BT_SLOT_FN
