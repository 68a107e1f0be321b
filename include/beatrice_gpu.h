/*
 * beatrice_gpu.h — C-ABI of the MI355X parse+filter stage.
 *
 * This is the drop-in boundary between Beatrice's C++ host (capture backends,
 * PluginManager, PacketFilter callers) and the hand-written gfx950 kernels in
 * beatrice_amd/csrc/. Plain C types only: pointers, sizes, POD structs. No
 * exception crosses it; every entry point returns an int status
 * (0 = OK, otherwise a beatrice::ErrorCode value, include/beatrice/Error.hpp:11-26
 * of the reference) and bt_last_error() gives the message.
 *
 * What each entry point replaces in the reference (/root/reference, read-only):
 *
 *   bt_filter_compile   PacketFilter::addFilter + the per-packet priority sort and
 *                       per-packet expression re-parsing of applyFilters
 *                       (src/PacketFilter.cpp:19-31, :57-73, :330-372). Expressions
 *                       are parsed ONCE here with the reference's own stoi/getline
 *                       semantics; the device gets a POD program.
 *   bt_parse_filter     PacketFilter::applyFilters(const std::vector<Packet>&)
 *                       (src/PacketFilter.cpp:121-130) fused with the per-layer
 *                       ProtocolParser::parsePacket(slice, name) calls
 *                       (src/parser/ProtocolParser.cpp:69-95, :238-284) over a
 *                       host batch (pinned staging, H2D -> kernels -> D2H).
 *   bt_parse_filter_device  the same over device-resident buffers, async on a
 *                       caller stream (the hot path that bench.py measures).
 *   bt_extract_device / bt_extract
 *                       ProtocolParser::parsePacket(packet, ProtocolDefinition) and the
 *                       by-name form for registered user protocols
 *                       (src/parser/ProtocolParser.cpp:69-110, :238-433) over a batch;
 *                       bt_time_extract_ex times it (bench.py's c1 entry).
 *
 * Record layout (bt_rec, 96 B per packet). Each layer L found by the layer walk
 * (DESIGN.md "R-WALK") has the field values that
 *   ProtocolParser(enablePerformanceMetrics=false).parsePacket(
 *       std::vector<uint8_t>(frame + off_L, frame + len), L)
 * returns, bit for bit: integers are the reference's extractValue<T> results
 * (big-endian wire order decoded, src/parser/ProtocolParser.cpp:418-431) stored
 * little-endian; BYTES / IPV4_ADDRESS / IPV6_ADDRESS fields are the raw bytes.
 * A layer whose slice is shorter than its table's getTotalLength() has status
 * PACKET_TOO_SHORT and no fields (:244-247): its field bytes are zero here.
 * Bytes of absent layers and reserved bytes are zero. Bytes 88..90 hold the
 * ProtocolDetector column of the whole frame (BT_DET_* / BT_IS_* below).
 *
 * On the device the records are PACKED and stored tiled by 64 packets (one wavefront
 * tile), SoA by 16-byte slab inside the tile: slab k (k = 0..5) of packet i lives at
 *     records + ((i / 64) * 6 + k) * 1024 + (i % 64) * 16
 * so each wavefront store instruction writes 1 KiB contiguously. The buffer needs
 * ceil(n / 64) * 6144 bytes. BT_OPT_RECORDS_PLANES selects plane-major slabs instead:
 * (k * n_cap + i) * 16. A packed record holds only the fields of the layers that
 * parsed (bt_rec.ok), each right after the previous one, as 24 little-endian dwords c[]:
 *   c0..c3  = bt_rec bytes 0..15 (Ethernet, pkt_len)
 *   c4      = present | ok << 8 | detect_code << 16 (3 bits) | detect_is << 19 (8 bits)
 *             | detect_is2 << 27 (3 bits); l3_off / l4_off are implied by present (+ IHL)
 *   then, per VLAN tag that parsed: vlan_tci[0] | vlan_tpid[1] << 16, then vlan_tci[1]
 *             (vlan_tpid[0] is the ethertype)
 *   then L3: IPv4 b0 | tos << 8 | ttl << 16 | protocol << 24, total_length | id << 16,
 *            flags | checksum << 16, source_ip, destination_ip (version == ihl == b0);
 *            or IPv6 as bt_rec bytes 28..67
 *   then L4: TCP 5 dwords / UDP, ICMP 2 dwords, as bt_rec bytes 68..
 * A record needs ceil(dwords / 4) slabs (bt_record_slabs): untagged Eth/IPv4/UDP 3,
 * IPv4/TCP or one tag 4, IPv6/TCP + QinQ 6, no IP 2. In the tiled layout, slabs 0 and 1
 * of packet i are at the addresses above; slab k >= 2 is stored only by the packets that
 * need it, packed in packet order to the front of the tile's slab-k region (a packet's
 * slot = its rank among them; the last tile's unused slots hold a zero slab 1). In the
 * plane-major layout slab k is at the packet's slot, written for the whole wavefront
 * when any packet needs it. Bytes no packet needs are left as they were.
 * bt_record_gather() / bt_record_unpack() rebuild the bt_rec, which is the parity unit.
 */
#ifndef BEATRICE_GPU_H
#define BEATRICE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 1 = round 1-3. 2 = round 4: a descriptor batch must state bt_batch.bytes
 * (0 was "unbounded" before and is now BT_E_INVALID_ARGUMENT); bt_group_host_register /
 * bt_group_parse_filter_mapped / bt_group_split_cost / bt_context_placement added. Hosts
 * built against an older header should check bt_abi_version() >= the version they need. */
#define BT_ABI_VERSION 2

/* ---- status codes (values of beatrice::ErrorCode, reference include/beatrice/Error.hpp:11-26) */
#define BT_OK                    0
#define BT_E_INVALID_ARGUMENT    1
#define BT_E_INIT_FAILED         2
#define BT_E_RESOURCE            3
#define BT_E_INTERNAL           10
#define BT_E_NOT_IMPLEMENTED    11

/* ---- packet descriptor: byte offset (48 bits) | length (16 bits) << 48 -------- */
typedef uint64_t bt_pkt_desc;
#define BT_DESC(off, len) ((uint64_t)(off) | ((uint64_t)(len) << 48))
#define BT_DESC_OFF(d)    ((uint64_t)(d) & 0xFFFFFFFFFFFFull)
#define BT_DESC_LEN(d)    ((uint32_t)((uint64_t)(d) >> 48))

/* ---- parsed record --------------------------------------------------------- */
#define BT_REC_BYTES  96
#define BT_REC_SLABS  6

/* bt_rec.present / bt_rec.ok bits: layer attempted by the walk / status SUCCESS */
#define BT_L_ETH   0x01u
#define BT_L_VLAN0 0x02u
#define BT_L_VLAN1 0x04u
#define BT_L_IPV4  0x08u
#define BT_L_IPV6  0x10u
#define BT_L_TCP   0x20u
#define BT_L_UDP   0x40u
#define BT_L_ICMP  0x80u

/* bt_rec.detect_*: reference ProtocolDetector (src/parser/ProtocolRegistry.cpp:353-484)
 * applied to the whole frame. detect_code is detectProtocol(frame).protocolName:
 *   BT_DET_UNKNOWN   "unknown",  confidence 0.0,  reason "Packet too short"   (len < 14)
 *   BT_DET_NONE      "" / "" (the reference leaves confidence uninitialised)  (:356-357)
 *   BT_DET_ETHERNET  "ethernet", 0.95, "Valid Ethernet frame"
 *   BT_DET_TCP/UDP/ICMP  "tcp"/"udp"/"icmp", 0.98, "Ethernet + IPv4 + TCP|UDP|ICMP"
 *                    (frame byte 23 once len >= 34, whatever the EtherType)
 * detect_is: isEthernet, isIPv4, isIPv6, isTCP, isUDP, isICMP, isHTTP, isDNS (:418-480;
 * the IPv4/IPv6 tests read the version nibble of frame byte 0, as the reference does).
 * detect_is2: isARP (:482-487) and the second entry of detectMultipleProtocols (:390-416). */
#define BT_DET_UNKNOWN  0u
#define BT_DET_NONE     1u
#define BT_DET_ETHERNET 2u
#define BT_DET_TCP      3u
#define BT_DET_UDP      4u
#define BT_DET_ICMP     5u
#define BT_IS_ETHERNET  0x01u
#define BT_IS_IPV4      0x02u
#define BT_IS_IPV6      0x04u
#define BT_IS_TCP       0x08u
#define BT_IS_UDP       0x10u
#define BT_IS_ICMP      0x20u
#define BT_IS_HTTP      0x40u
#define BT_IS_DNS       0x80u
#define BT_IS2_ARP       0x01u
#define BT_IS2_MULTI_TCP 0x02u   /* detectMultipleProtocols adds {"tcp", 0.98, "TCP over IPv4"} */
#define BT_IS2_MULTI_UDP 0x04u   /* ... {"udp", 0.98, "UDP over IPv4"}                          */

#pragma pack(push, 1)
typedef struct bt_ipv4_fields {   /* reference src/parser/ProtocolRegistry.cpp:161-178 */
    uint8_t  version;             /* raw byte 0 (quirk: same byte as ihl)              */
    uint8_t  ihl;                 /* raw byte 0                                         */
    uint8_t  tos;
    uint8_t  ttl;
    uint8_t  protocol;
    uint8_t  _pad0;
    uint16_t total_length;
    uint16_t identification;
    uint16_t flags;               /* raw 16-bit flags + fragment offset                 */
    uint16_t checksum;
    uint16_t _pad1;
    uint8_t  source_ip[4];
    uint8_t  destination_ip[4];
    uint8_t  _pad2[16];
} bt_ipv4_fields;                 /* 40 B */

typedef struct bt_ipv6_fields {   /* reference src/parser/ProtocolRegistry.cpp:180-192 */
    uint32_t version_traffic_class_flow_label;
    uint16_t payload_length;
    uint8_t  next_header;
    uint8_t  hop_limit;
    uint8_t  source_ip[16];
    uint8_t  destination_ip[16];
} bt_ipv6_fields;                 /* 40 B */

typedef struct bt_tcp_fields {    /* reference src/parser/ProtocolRegistry.cpp:194-209 */
    uint16_t source_port;
    uint16_t destination_port;
    uint32_t sequence_number;
    uint32_t acknowledgment_number;
    uint8_t  data_offset;         /* raw byte 12 */
    uint8_t  flags;               /* raw byte 13 */
    uint16_t window_size;
    uint16_t checksum;
    uint16_t urgent_pointer;
} bt_tcp_fields;                  /* 20 B */

typedef struct bt_udp_fields {    /* reference src/parser/ProtocolRegistry.cpp:211-221 */
    uint16_t source_port;
    uint16_t destination_port;
    uint16_t length;
    uint16_t checksum;
    uint8_t  _pad[12];
} bt_udp_fields;                  /* 20 B */

typedef struct bt_icmp_fields {   /* reference src/parser/ProtocolRegistry.cpp:223-234 */
    uint8_t  type;
    uint8_t  code;
    uint16_t checksum;
    uint16_t identifier;
    uint16_t sequence_number;
    uint8_t  _pad[12];
} bt_icmp_fields;                 /* 20 B */

typedef struct bt_rec {
    /* slab 0 */
    uint8_t  eth_destination_mac[6];   /* reference ProtocolRegistry.cpp:154 (BYTES) */
    uint8_t  eth_source_mac[6];        /* :155 (BYTES)                               */
    uint16_t eth_ethertype;            /* :156                                       */
    uint16_t pkt_len;                  /* min(frame length, 65535)                   */
    /* slab 1 */
    uint16_t vlan_tpid[2];             /* ProtocolRegistry.cpp:293 per tag           */
    uint16_t vlan_tci[2];              /* :294                                       */
    uint8_t  present;                  /* BT_L_* layers the walk attempted           */
    uint8_t  ok;                       /* BT_L_* layers with ParseStatus::SUCCESS    */
    uint8_t  l3_off;                   /* frame offset of the L3 slice (0 if none)   */
    uint8_t  l4_off;                   /* frame offset of the L4 slice (0 if none)   */
    /* slabs 1..4: L3 union at 28, L4 union at 68 */
    union { bt_ipv4_fields ipv4; bt_ipv6_fields ipv6; } l3;
    union { bt_tcp_fields tcp; bt_udp_fields udp; bt_icmp_fields icmp; } l4;
    /* slab 5 tail: the ProtocolDetector column for the whole frame */
    uint8_t  detect_code;              /* BT_DET_*: detectProtocol(frame)            */
    uint8_t  detect_is;                /* BT_IS_* predicate bits                     */
    uint8_t  detect_is2;               /* BT_IS2_* bits                              */
    uint8_t  _reserved[5];
} bt_rec;
#pragma pack(pop)

/* ---- filters --------------------------------------------------------------- */
/* Same enumerator order as beatrice::PacketFilter::FilterType
 * (reference include/beatrice/PacketFilter.hpp:17-24). */
enum bt_filter_type {
    BT_FILTER_BPF = 0,
    BT_FILTER_PROTOCOL = 1,
    BT_FILTER_IP_RANGE = 2,
    BT_FILTER_PORT_RANGE = 3,
    BT_FILTER_PAYLOAD = 4,
    BT_FILTER_CUSTOM = 5
};

typedef struct bt_filter_desc {       /* mirrors PacketFilter::FilterConfig hpp:26-33 */
    int32_t     type;                  /* enum bt_filter_type                          */
    const char* expression;            /* NUL-terminated; NULL == ""                   */
    int32_t     enabled;
    int32_t     priority;              /* higher = evaluated first                      */
    int32_t     has_custom_func;       /* CUSTOM only: a std::function is installed     */
} bt_filter_desc;

/* compiled filter kinds (device program) */
enum bt_filter_kind {
    BT_K_TRUE = 0,        /* empty expression (every apply*Filter :169,194,220,250,289) or unset CUSTOM */
    BT_K_FALSE = 1,       /* can only ever return false                                           */
    BT_K_BPF = 2,         /* substring keywords tcp/udp/icmp (:168-191)                           */
    BT_K_PROTO_EQ = 3,    /* "tcp"/"udp"/"icmp" (:210-212)                                        */
    BT_K_PROTO_NZ = 4,    /* "ip" (:213)                                                          */
    BT_K_IP_MASK = 5,     /* CIDR or exact dotted quad (:219-247, :342-360)                       */
    BT_K_PORT = 6,        /* inclusive range or exact port (:249-286, :362-372)                   */
    BT_K_IP_THROW = 7,    /* expression makes std::stoi throw once the IPv4 gates pass            */
    BT_K_PORT_THROW = 8,  /* same for the port filter once the TCP/UDP length gates pass          */
    BT_K_HOST = 9,        /* PAYLOAD regex outside the DFA subset / installed CUSTOM callback:    */
                          /* evaluated on the host                                                */
    BT_K_PAYLOAD = 10     /* PAYLOAD regex compiled to a byte DFA (bt_payload_dfa_compile):       */
                          /* a = byte offset of its blob in the context's DFA pool, b = blob size */
};

typedef struct bt_filter_slot {       /* one compiled program slot, in evaluation order */
    uint32_t source_index;            /* index into the bt_filter_desc array            */
    uint32_t kind;                    /* enum bt_filter_kind                            */
    uint32_t a, b;                    /* kind parameters                */
    int32_t  throw_kind;              /* 0 none, 1 std::invalid_argument, 2 std::out_of_range */
} bt_filter_slot;

#define BT_MAX_FILTERS 64

/* Per-packet decision byte: (code << 6) | slot. */
#define BT_DECIDE_PASS   0u   /* every enabled filter returned true (slot = last slot, 0 if none) */
#define BT_DECIDE_REJECT 1u   /* slot = first filter that returned false                           */
#define BT_DECIDE_THROW  2u   /* slot = filter whose expression throws (reference rethrows)        */
#define BT_DECIDE_HOST   3u   /* slot = first host-only filter reached; host continues from there  */
#define BT_DECIDE_CODE(x) ((uint32_t)(x) >> 6)
#define BT_DECIDE_SLOT(x) ((uint32_t)(x) & 63u)

/* ---- context --------------------------------------------------------------- */
typedef struct bt_ctx bt_ctx;

typedef struct bt_opts {
    uint32_t host_chunk_packets;   /* bt_parse_filter pipeline chunk (0 = default 1M)  */
    uint32_t host_chunk_bytes;     /* pinned staging bytes per chunk (0 = default 256 MiB) */
    uint32_t grid_waves;           /* 0 = auto (persistent grid sized to the device)    */
    uint32_t flags;                /* BT_OPT_*                                          */
    uint32_t host_threads;         /* host-path threads (0 = auto: BT_HOST_THREADS, else the
                                      usable CPUs (affinity, cgroup quota)); <= 16; a host
                                      batch uses <= 8 of them while others wait for the context */
    uint32_t reserved[3];
} bt_opts;

#define BT_OPT_NO_PREFETCH 0x1u    /* disable the next-tile load prefetch (A/B only)    */
#define BT_OPT_TILE_BLOCKED 0x2u   /* one contiguous tile range per wavefront           */
#define BT_OPT_RECORDS_AOS 0x4u    /* device records as bt_rec AoS instead of planes    */
#define BT_OPT_GRAPH 0x8u          /* bt_time_device: replay the steps as one hipGraph  */
#define BT_OPT_RECORDS_PLANES 0x10u /* device records plane-major (k * n_cap + i) * 16  */
#define BT_OPT_NT_STORES 0x20u     /* force non-temporal record stores                   */
#define BT_OPT_NT_LOADS 0x40u      /* force non-temporal header loads                    */
#define BT_OPT_CACHE_DEFAULT 0x80u /* default cache policy everywhere (A/B only)         */
#define BT_OPT_SPIN_SYNC 0x100u    /* spin-wait host synchronisation (bench / latency)   */
#define BT_OPT_PAYLOAD_HOST 0x200u /* keep every PAYLOAD filter on the host (std::regex) */
#define BT_OPT_WIDE_NEVER 0x400u   /* descriptor mode: always two-round loads (A/B only)   */
#define BT_OPT_WIDE_ALWAYS 0x800u  /* descriptor mode: always wide round A (A/B only)      */
#define BT_OPT_PIPELINE 0x2000u    /* bt_time_device: steps as bt_parse_filter_device_async */
#define BT_OPT_GROUP_SHARED_DEVICE 0x4000u /* bt_group_create: allow a device listed more than once:
                                      that many lanes (contexts) on it; concurrent host batches
                                      then run whole on the least busy member (groups route a
                                      call that finds another in flight, up to
                                      BT_GROUP_ROUTE_BELOW packets, default 1M, instead of
                                      splitting it) */
#define BT_OPT_NO_LEAN_PCIE 0x8000u /* frames in host memory: read whole 64-B windows (A/B only) */
#define BT_OPT_MAPPED_GATHER_SPARSE 0x10000u /* bt_group_parse_filter_mapped, filter-only calls over
                                      bt_pkt_desc: a member whose frames lie far apart (sampled
                                      mean spacing >= BT_MAPPED_GATHER_ABOVE, default 512 B)
                                      gathers their prefixes on its host threads instead of
                                      reading each frame's window over PCIe */
#define BT_OPT_NO_LEAN_HOST 0x20000u /* host batches, filter-only: stage each frame's first 48 B
                                      instead of bytes 12..43 (A/B only) */
#define BT_OPT_PAYLOAD_DFA 0x40000u /* PAYLOAD slots as byte DFAs even where the bit-parallel
                                      form fits (A/B only) */

/* descriptor formats (bt_batch.desc_format) */
#define BT_DESC_PACKED 0u          /* bt_pkt_desc: u64 offset:48 | length:16            */
#define BT_DESC_XDP    1u          /* struct xdp_desc {u64 addr; u32 len; u32 options} as
                                      an AF_XDP RX ring holds it (linux/if_xdp.h), aligned
                                      chunk mode: addr = byte offset into the UMEM        */

typedef struct bt_batch {          /* input; device memory or host memory mapped with
                                      bt_host_register (zero-copy over PCIe)             */
    const uint8_t* base;           /* packet bytes (e.g. the UMEM)                      */
    const void* desc;              /* one descriptor per packet; NULL = fixed stride    */
    uint32_t stride;               /* fixed-stride mode: packet i = base[i*stride .. +stride) */
    uint32_t n;                    /* packets                                           */
    uint64_t bytes;                /* size of the base buffer (bounds check)            */
    uint32_t desc_format;          /* BT_DESC_PACKED / BT_DESC_XDP                      */
    uint32_t flags;                /* BT_BATCH_*                                        */
} bt_batch;

/* bt_batch.flags */
#define BT_BATCH_PREFIXES 0x1u     /* base holds header prefixes (bt_ring_gather_tpv3), not
                                      whole frames: PAYLOAD slots, which read past the
                                      headers, are left to the host (BT_DECIDE_HOST)     */
#define BT_BATCH_LEAN 0x2u         /* with BT_BATCH_PREFIXES: frame bytes 12..43 only
                                      (bt_ring_gather_lean_tpv3); records refused        */

typedef struct bt_outputs {        /* any pointer may be NULL = not produced            */
    void*     records;             /* ceil(n/64) * 6144 bytes, tiled slabs (see above)  */
    uint32_t  n_cap;               /* records capacity (>= n); plane stride with PLANES */
    uint64_t* verdict;             /* ceil(n/64) words, bit i%64 of word i/64 = passed  */
    uint8_t*  decide;              /* n bytes, BT_DECIDE_*                              */
    uint32_t* pass_idx;            /* n entries: indices of passing packets, ascending  */
    uint32_t* n_pass;              /* 1 word                                            */
} bt_outputs;

int  bt_abi_version(void);
const char* bt_last_error(void);              /* thread-local message of the last failure */

int  bt_create(int device, const bt_opts* opts, bt_ctx** out);
void bt_destroy(bt_ctx* ctx);
int  bt_device_count(int* out);
/* The context's device: its HIP ordinal and PCI bus id ("0000:05:00.0"; cap >= 16), so
 * that processes sharing a node can check they drive distinct GPUs. */
int  bt_context_device(const bt_ctx* ctx, int* device, char* pci_bus_id, uint32_t cap);
/* Where the context's host work runs: the host NUMA node closest to its device (HIP's
 * hipDeviceAttributeHostNumaId, else the PCI function's sysfs numa_node; -1 unknown), how
 * many CPUs of that node (in this process's affinity set) its pool workers are pinned to
 * (0 = not pinned; BT_NUMA_PIN=0 turns pinning off), the pool's size, and the node of the
 * host pipeline's pinned staging (-1 until a host batch allocated it). */
typedef struct bt_placement {
    int32_t  numa_node;
    uint32_t pinned_cpus;
    uint32_t pool_threads;
    int32_t  staging_node;
    uint32_t reserved[4];
} bt_placement;
int  bt_context_placement(bt_ctx* ctx, bt_placement* out);
/* Host-only: the CPUs this process may use (affinity set bounded by the cgroup v2 quota). */
uint32_t bt_usable_cpus(void);

/* Compile the enabled filters: stable sort by priority (descending), parse each
 * expression once. The C++ adapter (beatrice_amd/host) passes filters already in
 * the reference's own evaluation order so ties match libstdc++ exactly. */
int  bt_filter_compile(bt_ctx* ctx, const bt_filter_desc* filters, uint32_t n);
int  bt_filter_program(const bt_ctx* ctx, bt_filter_slot* out, uint32_t cap, uint32_t* n_slots);
/* The compiled program's PAYLOAD DFA tables (BT_K_PAYLOAD slot s: bytes [s.a, s.a + s.b) of
 * the pool, a blob for bt_payload_dfa_eval): *bytes = the pool's size, min(cap, size) bytes
 * copied to out. For hosts that evaluate small batches on the CPU with the same program. */
int  bt_filter_dfa_pool(const bt_ctx* ctx, void* out, uint32_t cap, uint32_t* bytes);

/* Pre-size the device workspace for batches of up to n packets (so later launches
 * never allocate, e.g. under hipGraph capture). */
int  bt_reserve(bt_ctx* ctx, uint32_t n);

/* Device-resident parse+filter, asynchronous on `stream` (a hipStream_t, NULL =
 * the context's own stream). records != NULL selects parsing; the filter
 * outputs are produced when any of verdict/decide/pass_idx/n_pass is set. */
int  bt_parse_filter_device(bt_ctx* ctx, const bt_batch* batch, const bt_outputs* out, void* stream);

/* Pipelined form for a stream of batches. The main kernel runs on `stream` as above
 * (records, decide and verdict are complete in stream order); the ordered compaction
 * (pass_idx, n_pass) runs on the context's own compaction stream once that kernel has
 * finished, and `done_event` (a hipEvent_t, may be NULL) is recorded after it. The next
 * call's main kernel on `stream` does not wait for it, so the compaction of batch i runs
 * beside the parse of batch i + 1. Until done_event completes, the caller must neither
 * read pass_idx / n_pass nor rewrite this call's verdict buffer (the compaction reads
 * it): alternate two output sets. */
int  bt_parse_filter_device_async(bt_ctx* ctx, const bt_batch* batch, const bt_outputs* out, void* stream,
                                  void* done_event);

/* Host batch: borrows base/desc for the call, copies through pinned staging in
 * chunks (H2D, kernels, D2H double-buffered on two streams), fills host outputs,
 * returns when done. Output pointers are host memory (records in bt_rec AoS). Records
 * that lie inside a range registered with bt_host_register on this context are written
 * in place by the D2H copies (no pass through the staging). */
int  bt_parse_filter(bt_ctx* ctx, const uint8_t* base, const bt_pkt_desc* desc, uint32_t n,
                     bt_rec* records, uint64_t* verdict, uint8_t* decide,
                     uint32_t* pass_idx, uint32_t* n_pass);

/* The same over a gather list — one pointer + length per frame, e.g. the buffers of a
 * std::vector<beatrice::Packet> (reference include/beatrice/Packet.hpp:145-211). Only
 * the first min(len, 112) bytes of each frame are staged for the device. */
int  bt_parse_filter_ptrs(bt_ctx* ctx, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                          bt_rec* records, uint64_t* verdict, uint8_t* decide,
                          uint32_t* pass_idx, uint32_t* n_pass);
/* The bytes of each frame the two calls above read (and stage) with the context's current
 * program: at most min(len, *bytes) from the frame's start; 48 for filter-only calls (which
 * read and stage bytes 12..43 of it), 112 with
 * records, 176 when the program has a GPU PAYLOAD slot (with_records: whether the call asks
 * for records). A caller may pass, in place of a frame, a copy of that many of its first
 * bytes with the frame's true length (e.g. prefixes packed when the packet arrived). */
int  bt_host_stage_bytes(const bt_ctx* ctx, int with_records, uint32_t* bytes);

/* Zero-copy ingest: page-lock a host range (an AF_XDP UMEM, an RX descriptor ring,
 * an output array) and map it into the device; *dev_alias is the pointer kernels
 * use (it may be passed as bt_batch.base / .desc or as an output). The kernels then
 * read the header windows straight over PCIe: no host gather, no staging copy.
 * Registration is in whole pages, in one table for the process (contexts and groups
 * alike): the pages that hold [host, host + bytes) are registered once; a range inside
 * pages a live registration already holds shares them (a reference, no second lock); a
 * range that shares only some of its pages with a live registration is refused
 * (BT_E_INVALID_ARGUMENT: register page-aligned buffers, or one range covering both), so no
 * page is ever locked twice and no unregister unlocks a page another registration still
 * covers. A range is registered once per context. bt_host_unregister drops the context's
 * reference; the last one waits for the devices that hold an alias, then unlocks. The pages
 * must stay mapped (not freed or unmapped) while registered. */
int  bt_host_register(bt_ctx* ctx, void* host, uint64_t bytes, void** dev_alias);
int  bt_host_unregister(bt_ctx* ctx, void* host);

/* ---- PAYLOAD filters on the GPU ---------------------------------
 * Replaces the per-packet std::regex construction + regex_search of
 * PacketFilter::applyPayloadFilter (src/PacketFilter.cpp:288-321) for the regular
 * subset of libstdc++'s ECMAScript grammar: bt_filter_compile compiles every PAYLOAD
 * expression it can once (BT_K_PAYLOAD slots, up to 16 KiB of tables per program); the
 * rest stay BT_K_HOST. The compiler itself is in include/beatrice_gpu_bench.h.
 *   bt_payload_dfa_eval  applyPayloadFilter(frame, len) on the host with a compiled slot's
 *                        blob (bt_filter_dfa_pool): the C++ filter's continuation of a
 *                        chain the device handed over */
int  bt_payload_dfa_eval(const void* blob, const uint8_t* frame, uint32_t len);

/* ---- capture-ring ingest: AF_PACKET TPACKET_V3 ---------------
 * Replaces the per-packet recv() + heap copy + queue push of the reference's
 * AF_PacketBackend::packetProcessingLoop (src/AF_PacketBackend.cpp:318-363). A
 * PACKET_RX_RING of n_blocks blocks of block_size bytes (linux/if_packet.h,
 * struct tpacket_req3) is mmap'd once; the kernel fills a block with a chain of
 * tpacket3_hdr frames and flips block_status to TP_STATUS_USER. The walker turns
 * ready blocks into bt_pkt_desc entries whose offsets are relative to the ring base,
 * so the ring itself (registered with bt_host_register, or copied to the device) is
 * the bt_batch.base: the frames are never copied on the host. */
typedef struct bt_tpv3_ring {
    void* base;                    /* host address of the mmap'd ring */
    uint64_t block_size;           /* tpacket_req3.tp_block_size      */
    uint32_t n_blocks;             /* tpacket_req3.tp_block_nr        */
    uint32_t reserved;
} bt_tpv3_ring;

/* Takes the ready blocks first_block, first_block+1, ... (mod n_blocks): at most
 * max_blocks of them, stopping at the first block the kernel still owns or whose
 * packets would overflow `cap` descriptors. Writes one descriptor per frame in ring
 * order, BT_DESC(block * block_size + frame offset + tp_mac, min(tp_snaplen, 65535)),
 * and the counts. Blocks are walked in parallel on ctx's host pool (ctx may be NULL:
 * single-threaded, no GPU needed). A malformed block (a frame chain leaving the block)
 * returns BT_E_INVALID_ARGUMENT and takes nothing. The blocks stay owned by the
 * caller until bt_ring_release_tpv3. */
int  bt_ring_walk_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block,
                       uint32_t max_blocks, bt_pkt_desc* desc, uint32_t cap,
                       uint32_t* n_desc, uint32_t* n_blocks_taken);
#define BT_PREFIX_SLOT 128u
/* Header-prefix gathers: BT_PREFIX_SLOT bytes of `slots` per taken frame (the slot form,
 * bt_ring_gather_tpv3, is in include/beatrice_gpu_bench.h). A batch over `slots`
 * (registered, or copied to the device) runs with flags = BT_BATCH_PREFIXES.
 * The walk with each frame's header prefix packed: the frames of the k-th taken block (whose first
 * descriptor is j_k) go back to back, each 16-B aligned and taking its prefix length rounded
 * up to 16, from byte j_k * BT_PREFIX_SLOT of `slots` (16-B aligned, BT_PREFIX_SLOT * cap
 * bytes, as above); desc[i] = BT_DESC(offset of frame i's prefix, min(tp_snaplen, 65535)),
 * and ring_desc[i] (optional, cap entries) = frame i's ring descriptor as bt_ring_walk_tpv3
 * writes it, for what reads the whole frame (PAYLOAD / CUSTOM slots, forwarding).
 * A block's packets then sit in consecutive bytes (a 42-B UDP header in 48 B), so the
 * kernels' reads of a tile are one contiguous run over PCIe instead of one 128-B slot per
 * packet. Bytes past a prefix belong to the next frame: the batch flag BT_BATCH_PREFIXES
 * (PAYLOAD slots decided on the host) is required as for the slots. */
int  bt_ring_gather_dense_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                               uint8_t* slots, bt_pkt_desc* desc, bt_pkt_desc* ring_desc, uint32_t cap,
                               uint32_t* n_desc, uint32_t* n_blocks_taken);
/* The same walk for filter-only batches: each frame's bytes 12..43 (the 16-B chunk pair
 * holding what every built-in filter reads, zeros past the frame) packed back to back after a
 * 16-B pad at the block's first slot (j_k * BT_PREFIX_SLOT + 16), 32 B per frame;
 * desc[i] = BT_DESC(offset of frame i's 32 B - 12, min(tp_snaplen, 65535)). Run the batch
 * with flags BT_BATCH_PREFIXES | BT_BATCH_LEAN: a call that asks for records is refused. */
int  bt_ring_gather_lean_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                              uint8_t* slots, bt_pkt_desc* desc, bt_pkt_desc* ring_desc, uint32_t cap,
                              uint32_t* n_desc, uint32_t* n_blocks_taken);
/* Hands `count` blocks starting at first_block back to the kernel (TP_STATUS_KERNEL,
 * release-ordered). Call it once the device has finished reading them. */
int  bt_ring_release_tpv3(const bt_tpv3_ring* ring, uint32_t first_block, uint32_t count);

/* The ring stage in one call: up to n_blocks ready blocks from first_block through the
 * context's filter program, in batches of batch_blocks (0 = 128). Each batch is walked on the
 * host (bt_ring_walk_tpv3; with gather, its frames' bytes 12..43 packed into `slots`,
 * bt_ring_gather_lean_tpv3) while the kernels of the batch before it run, so the host walk
 * and the device's PCIe reads overlap. Writes one descriptor (ring-relative in place; slot-
 * relative for gathered batches) and one decision byte per frame in ring order, and, if
 * given, the verdict words and the pass count; stops early at a block the kernel still owns.
 * The ring, desc (cap entries), decide (cap bytes) and, with gather, slots (cap *
 * BT_PREFIX_SLOT bytes, 16-B aligned) must be registered with the context
 * (bt_host_register). Filter-only: the decision bytes are the product (records: the
 * descriptors + bt_parse_filter_device). Replaces the per-frame recv() loop feeding
 * PacketFilter::applyFilters (reference src/AF_PacketBackend.cpp:318-363). */
typedef struct bt_ring_stage_opts {
    uint32_t batch_blocks;        /* blocks per kernel launch (0 = 128)                     */
    uint32_t gather;              /* 1: pack bytes 12..43 of each frame (lean) before launch;
                                     2: adaptive: a batch is gathered while the device is still
                                     busy with earlier batches, read in place once it caught up */
    uint32_t in_place_every;      /* with gather: every k-th batch read in place (0 = none)  */
    uint32_t in_place_blocks;     /* with gather: the last m blocks of every batch read in
                                     place, the rest gathered (0 = whole batches; overrides
                                     in_place_every)                                         */
} bt_ring_stage_opts;
int  bt_ring_stage_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t n_blocks,
                        const bt_ring_stage_opts* opts, bt_pkt_desc* desc, uint8_t* slots, uint8_t* decide,
                        uint64_t* verdict, uint32_t cap, uint32_t* n_desc, uint32_t* n_pass);

/* ---- several devices in one process -------------------------------
 * The reference runs one daemon process whose capture threads feed one plugin set
 * (src/BeatriceContext.cpp:215-278, src/PluginManager.cpp:158-188). A group is one
 * context per device (its own streams, pinned staging and host threads). The filter
 * program is compiled once on the host and installed on every member. A host batch is
 * split into contiguous ranges that start on 64-packet boundaries and balance the bytes
 * each member stages (bt_group_split), every member runs its range concurrently, and the
 * outputs land in the caller's arrays exactly as bt_parse_filter / _ptrs write them for
 * the whole batch (pass indices in ascending order). No data crosses devices. */
typedef struct bt_group bt_group;
int      bt_group_create(const int* devices, uint32_t n_devices, const bt_opts* opts, bt_group** out);
void     bt_group_destroy(bt_group* group);
uint32_t bt_group_size(const bt_group* group);
bt_ctx*  bt_group_member(bt_group* group, uint32_t k);   /* member k's context (device k) */
int      bt_group_filter_compile(bt_group* group, const bt_filter_desc* filters, uint32_t n);
int      bt_group_parse_filter(bt_group* group, const uint8_t* base, const bt_pkt_desc* desc, uint32_t n,
                               bt_rec* records, uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx,
                               uint32_t* n_pass);
int      bt_group_parse_filter_ptrs(bt_group* group, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                                    bt_rec* records, uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx,
                                    uint32_t* n_pass);
/* bt_host_parallel over the whole group's host threads: fn(user, w, workers) runs once for
 * every w in [0, workers), workers = the members' pool sizes summed (member k's pool, on its
 * NUMA node, takes a contiguous range of w); returns when all have. For host-side work on a
 * batch's results (a filter's decision scan, its FilterResults), so that a group spends its
 * whole budget there rather than member 0's share of it. */
int      bt_group_host_parallel(bt_group* group, void (*fn)(void* user, uint32_t worker, uint32_t workers), void* user);

/* Zero-copy over the group (AF_XDP UMEM, TPACKET_V3 ring, output arrays): page-lock a host
 * range once (portable, mapped) and map it into every member's device; each member reads
 * it through its own alias over its own PCIe link. Whole pages, in the same process-wide
 * table as bt_host_register (shared when another registration holds all of the range's
 * pages, refused when it holds only some). A group's ranges must not overlap. The last
 * reference on the pages waits for every device holding an alias, then unlocks. */
int      bt_group_host_register(bt_group* group, void* host, uint64_t bytes);
int      bt_group_host_unregister(bt_group* group, void* host);
/* bt_parse_filter_device over group-registered host memory, split across the members:
 * `batch` and `out` hold HOST addresses. batch.base / batch.desc and out.records /
 * out.verdict / out.decide must lie in ranges registered with bt_group_host_register;
 * out.pass_idx / out.n_pass are written by the host and may be any host memory. The batch
 * is split on 64-packet tiles by bt_group_cost(mapped) and member k runs its range
 * [lo, hi) with its own alias of every buffer: descriptors from desc + lo (fixed stride:
 * base + lo * stride), records at the range's tile (tiled: + lo / 64 * 6144 bytes, n_cap -
 * lo; BT_OPT_RECORDS_AOS: + lo * 96; plane-major records cannot be split and are
 * refused with more than one member), decisions at + lo, verdict words at + lo / 64. The
 * pass list is built from the verdict words on the members' host threads (out.verdict, or
 * the group's own registered words when the caller asked for none), in ascending order.
 * Synchronous: every output is complete on return. */
int      bt_group_parse_filter_mapped(bt_group* group, const bt_batch* batch, const bt_outputs* out);

/* ---- context helpers ------------------------------------------------------------ */
/* Waits for the context's stream and its compaction stream (bt_parse_filter_device_async). */
int  bt_synchronize(bt_ctx* ctx);
/* Runs fn(user, w, workers) once on each of the context's host threads (w = 0 .. workers-1,
 * the caller is worker 0) and returns when all have: the pool that gathers and drains the
 * host-batch pipeline, lent to host-side post-processing of a batch. */
int  bt_host_parallel(bt_ctx* ctx, void (*fn)(void* user, uint32_t worker, uint32_t workers), void* user);
/* Device memory, copies, streams and timing loops for hosts without a HIP toolchain (tests,
 * benchmarks, ctypes): include/beatrice_gpu_bench.h. */

/* ---- user-defined protocols: ProtocolParser with any ProtocolDefinition -------------
 * Replaces ProtocolParser::parsePacketInternal / extractField / extractValue<T>
 * (src/parser/ProtocolParser.cpp:238-433) for a table registered with registerProtocol
 * (include/parser/ProtocolParser.hpp:63-69) or passed as a ProtocolDefinition: one
 * kernel pass extracts every field of every packet of a batch.
 *   span   = ProtocolDefinition::getTotalLength() (src/parser/FieldDefinition.cpp:31-46),
 *            the largest field end; a packet shorter than span is PACKET_TOO_SHORT with no
 *            field (:244-247), a longer one has every field (each ends within span).
 *   values = the result of extractValue<T> for the field's type (:385-433), as the bits
 *            of T zero-extended to 64: integer types and TIMESTAMP assemble the field's
 *            bytes little-endian (LITTLE) or big-endian (BIG / NETWORK / HOST), byte i
 *            shifted by (8 i) mod the width the shift is done in (32 for types narrower
 *            than 64 bits, 64 otherwise) as x86-64 does, then cut to T; FLOAT32 / FLOAT64
 *            are the raw bits when the length is 4 / 8, else 0; BOOLEAN is byte 0 != 0;
 *            byte-typed fields (BYTES, STRING, MAC/IPV4/IPV6_ADDRESS, CUSTOM) are 0.
 *   image  = the packet's bytes [0, span), from which the host materialises rawHex and
 *            the byte-typed fields of the ParseResult.
 * A BOOLEAN field of length 0 is rejected (BT_E_INVALID_ARGUMENT): the reference reads
 * fieldData[0] of an empty vector there. */
#define BT_FIELD_MAX 64u           /* fields per protocol table                          */
enum bt_field_type {               /* FieldType (include/parser/FieldDefinition.hpp:16-35) */
    BT_FT_UINT8 = 0, BT_FT_UINT16, BT_FT_UINT32, BT_FT_UINT64, BT_FT_INT8, BT_FT_INT16, BT_FT_INT32,
    BT_FT_INT64, BT_FT_FLOAT32, BT_FT_FLOAT64, BT_FT_BYTES, BT_FT_STRING, BT_FT_BOOLEAN, BT_FT_MAC,
    BT_FT_IPV4, BT_FT_IPV6, BT_FT_TIMESTAMP, BT_FT_CUSTOM
};
#define BT_ENDIAN_LITTLE 0u        /* Endianness::LITTLE (:37-42); 1..3 all decode big-endian */

typedef struct bt_field_def {      /* FieldDefinition (:61-82): the parts extraction uses */
    uint64_t offset;
    uint64_t length;
    uint32_t type;                 /* bt_field_type                                       */
    uint32_t endianness;           /* Endianness value                                    */
} bt_field_def;

typedef struct bt_extract_out {    /* device-visible; any pointer may be NULL             */
    uint8_t*  status;              /* n bytes: 0 SUCCESS, 9 PACKET_TOO_SHORT (ParseStatus) */
    uint64_t* values;              /* n_fields x n_cap, field-major: values[f * n_cap + i] */
    uint8_t*  image;               /* n x span bytes: packet i at image + i * span, its
                                      bytes [0, span) when SUCCESS, zeros otherwise        */
    uint32_t  n_cap;               /* values column stride (>= n)                         */
    uint32_t  reserved;
} bt_extract_out;

/* getTotalLength() of a field table (0 for no fields). */
int  bt_proto_span(const bt_field_def* fields, uint32_t n_fields, uint64_t* span);
/* Device-resident extraction, asynchronous on `stream` (NULL = the context's stream);
 * the table is copied into the launch, so it need not outlive the call. */
int  bt_extract_device(bt_ctx* ctx, const bt_batch* batch, const bt_field_def* fields, uint32_t n_fields,
                       const bt_extract_out* out, void* stream);
/* Host gather list in (the buffers of a std::vector<Packet>), host outputs back; waits.
 * status: n bytes; values: n_fields x n, values[f * n + i]; image: n x span bytes. Only the
 * [0, span) prefix of each frame is staged for the device. */
int  bt_extract(bt_ctx* ctx, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                const bt_field_def* fields, uint32_t n_fields, uint8_t* status, uint64_t* values,
                uint8_t* image);
/* The same outputs computed on the calling thread, no device: for batches too small to pay
 * for a device round trip (GpuProtocolParser::parsePacket of one packet; ≈ 0.1 ms per
 * bt_extract call). extractValue<T>'s bits exactly as bt_extract_tile decodes them. */
int  bt_extract_host(const uint8_t* const* frames, const uint32_t* lens, uint32_t n, const bt_field_def* fields,
                     uint32_t n_fields, uint8_t* status, uint64_t* values, uint8_t* image);
/* ---- text output --------------------------------------------------------------
 * The text the reference's ParseResult formatters print for every walked layer of
 * records [0, n) (reference src/parser/ParserResult.cpp:214-349; each layer is the
 * ParseResult ProtocolParser::parsePacket(slice, name) returns, wall-clock values 0),
 * each layer's text followed by '\n', packets in order. Replaces a loop of
 * parsePacket(...).toJsonString() etc. (e.g. src/beatrice_cli.cpp:1654-1660).
 * `recs` are host bt_rec (AoS, e.g. from bt_parse_filter or bt_record_gather).
 * out == NULL: size query (*out_len = bytes needed). pkt_off (optional, n + 1
 * entries) receives each packet's start offset and the total. A `cap` below the
 * size returns BT_E_INVALID_ARGUMENT with *out_len set. ctx (optional, may be NULL)
 * lends its host thread pool; no device is used. */
#define BT_FMT_JSON  0u   /* ParseResult::toJsonString          (:214-254) */
#define BT_FMT_XML   1u   /* ParseResult::toXmlString           (:256-298) */
#define BT_FMT_CSV   2u   /* ParseResult::toCsvString           (:300-313) */
#define BT_FMT_HUMAN 3u   /* ParseResult::toHumanReadableString (:315-349) */
int  bt_format_records(bt_ctx* ctx, const bt_rec* recs, uint32_t n, uint32_t format, char* out, uint64_t cap,
                       uint64_t* out_len, uint64_t* pkt_off);
/* The same text in one pass: the records are formatted once, then dest(user, bytes) is called
 * once with the exact size and returns where to put it (NULL only when bytes == 0); the
 * size query plus the call above format everything twice. */
int  bt_format_records_to(bt_ctx* ctx, const bt_rec* recs, uint32_t n, uint32_t format,
                          char* (*dest)(void* user, uint64_t bytes), void* user, uint64_t* out_len,
                          uint64_t* pkt_off);

/* host-side record gather from the device layout (after a D2H copy) */
void bt_record_gather(const void* records, uint32_t n_cap, uint32_t i, bt_rec* out);
/* All n records at once (planes != 0: plane-major), on ctx's host threads (ctx may be
 * NULL); *slabs (optional) gets the total of slabs the device stored. out == NULL with
 * slabs != NULL only counts (reads slab 1 of each record). */
int  bt_record_unpack(bt_ctx* ctx, const void* records, uint32_t n_cap, uint32_t n, uint32_t planes, bt_rec* out,
                      uint64_t* slabs);

#ifdef __cplusplus
}
#endif

#if defined(__cplusplus)
static_assert(sizeof(bt_rec) == BT_REC_BYTES, "bt_rec must be 96 bytes");
static_assert(offsetof(bt_rec, l3) == 28, "L3 union at 28");
static_assert(offsetof(bt_rec, l4) == 68, "L4 union at 68");
static_assert(offsetof(bt_rec, detect_code) == 88, "detector column at 88");
#endif

#endif /* BEATRICE_GPU_H */
