/*
 * bt_oracle.c — CPU restatement of the reference parse+filter hot path.
 *
 * TEST INFRASTRUCTURE ONLY (checker for tests/, smoke() and bench.py's
 * cpu_baseline leg). Nothing under beatrice_amd/ links or loads this file.
 *
 * It deliberately follows the reference's *shape*, not the GPU kernel's:
 *  - the parser is table-driven: per-protocol field tables (name, offset,
 *    length, type) restated from src/parser/ProtocolRegistry.cpp:150-234/289-297,
 *    a getTotalLength() gate (src/parser/FieldDefinition.cpp:31-46,
 *    src/parser/ProtocolParser.cpp:244-247) and extractValue<T>
 *    (src/parser/ProtocolParser.cpp:385-433);
 *  - the filter re-parses every expression string for every packet, exactly as
 *    src/PacketFilter.cpp:168-372 does (std::stoi restated via strtol, the way
 *    libstdc++ implements it; std::getline(ss, tok, '.') restated by hand).
 * The layer walk (which slice is handed to which table) has no reference symbol;
 * it is the build-defined walk of SURVEY.md §8(a) R-WALK / DESIGN.md.
 */
#define _GNU_SOURCE
#include "bt_oracle.h"

#include <errno.h>
#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- field tables */
enum { F_U8, F_U16, F_U32, F_BYTES };   /* BYTES covers BYTES/IPV4_ADDRESS/IPV6_ADDRESS */

typedef struct {
    const char* name;
    uint32_t off, len, type;
    uint32_t rec_off;        /* destination in bt_rec */
} field_def;

/* src/parser/ProtocolRegistry.cpp:150-159 */
static const field_def T_ETH[] = {
    {"destination_mac", 0, 6, F_BYTES, 0},
    {"source_mac", 6, 6, F_BYTES, 6},
    {"ethertype", 12, 2, F_U16, 12},
};
/* :289-297 (rec_off for tag 0; tag 1 adds 2) */
static const field_def T_VLAN[] = {
    {"tpid", 0, 2, F_U16, 16},
    {"tci", 2, 2, F_U16, 20},
};
/* :161-178 */
static const field_def T_IPV4[] = {
    {"version", 0, 1, F_U8, 28},
    {"ihl", 0, 1, F_U8, 29},
    {"tos", 1, 1, F_U8, 30},
    {"total_length", 2, 2, F_U16, 34},
    {"identification", 4, 2, F_U16, 36},
    {"flags", 6, 2, F_U16, 38},
    {"ttl", 8, 1, F_U8, 31},
    {"protocol", 9, 1, F_U8, 32},
    {"checksum", 10, 2, F_U16, 40},
    {"source_ip", 12, 4, F_BYTES, 44},
    {"destination_ip", 16, 4, F_BYTES, 48},
};
/* :180-192 */
static const field_def T_IPV6[] = {
    {"version_traffic_class_flow_label", 0, 4, F_U32, 28},
    {"payload_length", 4, 2, F_U16, 32},
    {"next_header", 6, 1, F_U8, 34},
    {"hop_limit", 7, 1, F_U8, 35},
    {"source_ip", 8, 16, F_BYTES, 36},
    {"destination_ip", 24, 16, F_BYTES, 52},
};
/* :194-209 */
static const field_def T_TCP[] = {
    {"source_port", 0, 2, F_U16, 68},
    {"destination_port", 2, 2, F_U16, 70},
    {"sequence_number", 4, 4, F_U32, 72},
    {"acknowledgment_number", 8, 4, F_U32, 76},
    {"data_offset", 12, 1, F_U8, 80},
    {"flags", 13, 1, F_U8, 81},
    {"window_size", 14, 2, F_U16, 82},
    {"checksum", 16, 2, F_U16, 84},
    {"urgent_pointer", 18, 2, F_U16, 86},
};
/* :211-221 */
static const field_def T_UDP[] = {
    {"source_port", 0, 2, F_U16, 68},
    {"destination_port", 2, 2, F_U16, 70},
    {"length", 4, 2, F_U16, 72},
    {"checksum", 6, 2, F_U16, 74},
};
/* :223-234 */
static const field_def T_ICMP[] = {
    {"type", 0, 1, F_U8, 68},
    {"code", 1, 1, F_U8, 69},
    {"checksum", 2, 2, F_U16, 70},
    {"identifier", 4, 2, F_U16, 72},
    {"sequence_number", 6, 2, F_U16, 74},
};
#define NF(t) ((int)(sizeof(t) / sizeof((t)[0])))

/* ProtocolDefinition::getTotalLength, src/parser/FieldDefinition.cpp:31-46 */
static uint32_t total_length(const field_def* t, int nf)
{
    if (nf == 0) return 0;
    uint32_t max_off = 0, max_len = 0;
    for (int i = 0; i < nf; ++i) {
        uint32_t end = t[i].off + t[i].len;
        if (end > max_off + max_len) { max_off = t[i].off; max_len = t[i].len; }
    }
    return max_off + max_len;
}

/* extractValue<T> for NETWORK endianness (every builtin field is NETWORK):
 * value |= packet[offset + length - 1 - i] << (i*8)  (ProtocolParser.cpp:426-428) */
static uint64_t extract_be(const uint8_t* s, uint32_t off, uint32_t len)
{
    uint64_t v = 0;
    for (uint32_t i = 0; i < len; ++i) v |= (uint64_t)s[off + len - 1 - i] << (i * 8);
    return v;
}

/* parsePacketInternal (ProtocolParser.cpp:238-284): returns 1 on SUCCESS, 0 on
 * PACKET_TOO_SHORT (zero fields). Fields with offset+length > size are skipped
 * (:252-254) — unreachable once the total-length gate passed. */
static int parse_layer(const uint8_t* slice, uint32_t slen, const field_def* t, int nf,
                       uint8_t* rec, uint32_t rec_bias)
{
    if (slen < total_length(t, nf)) return 0;
    for (int i = 0; i < nf; ++i) {
        const field_def* f = &t[i];
        if (f->off + f->len > slen) continue;
        uint8_t* dst = rec + f->rec_off + rec_bias;
        switch (f->type) {
        case F_U8: dst[0] = (uint8_t)extract_be(slice, f->off, 1); break;
        case F_U16: { uint16_t v = (uint16_t)extract_be(slice, f->off, 2); memcpy(dst, &v, 2); } break;
        case F_U32: { uint32_t v = (uint32_t)extract_be(slice, f->off, 4); memcpy(dst, &v, 4); } break;
        default: memcpy(dst, slice + f->off, f->len); break;   /* raw bytes */
        }
    }
    return 1;
}

#define L_ETH 0x01u
#define L_VLAN0 0x02u
#define L_IPV4 0x08u
#define L_IPV6 0x10u
#define L_TCP 0x20u
#define L_UDP 0x40u
#define L_ICMP 0x80u

static uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* ProtocolDetector, src/parser/ProtocolRegistry.cpp:353-487, one predicate per
 * reference function, each over the whole frame. */
static int det_is_ethernet(const uint8_t* p, uint32_t n)   /* :418-423 */
{
    if (n < 14) return 0;
    uint32_t et = be16(p + 12);
    return et == 0x0800 || et == 0x0806 || et == 0x86DD;
}
static int det_is_ipv4(const uint8_t* p, uint32_t n) { return n >= 34 && (p[0] >> 4) == 4; }  /* :425-430 */
static int det_is_ipv6(const uint8_t* p, uint32_t n) { return n >= 54 && (p[0] >> 4) == 6; }  /* :432-437 */
static int det_is_tcp(const uint8_t* p, uint32_t n) { return det_is_ipv4(p, n) && p[23] == 6; }
static int det_is_udp(const uint8_t* p, uint32_t n) { return det_is_ipv4(p, n) && p[23] == 17; }
static int det_is_icmp(const uint8_t* p, uint32_t n) { return det_is_ipv4(p, n) && p[23] == 1; }
static int det_is_http(const uint8_t* p, uint32_t n)      /* :460-469 */
{
    if (!det_is_tcp(p, n) || n < 54) return 0;
    return be16(p + 36) == 80 || be16(p + 34) == 80;
}
static int det_is_dns(const uint8_t* p, uint32_t n)       /* :471-480 */
{
    if (!det_is_udp(p, n) || n < 42) return 0;
    return be16(p + 36) == 53 || be16(p + 34) == 53;
}
static int det_is_arp(const uint8_t* p, uint32_t n) { return n >= 28 && be16(p + 12) == 0x0806; }

static void detect(const uint8_t* p, uint32_t n, uint8_t* out)
{
    uint8_t code;                                          /* detectProtocol :353-388 */
    if (n < 14) code = 0;                                  /* "unknown"  */
    else if (!det_is_ethernet(p, n)) code = 1;             /* ""         */
    else {
        code = 2;                                          /* "ethernet" */
        if (n >= 34) code = p[23] == 6 ? 3 : p[23] == 17 ? 4 : p[23] == 1 ? 5 : code;
    }
    out[0] = code;
    out[1] = (uint8_t)(det_is_ethernet(p, n) | det_is_ipv4(p, n) << 1 | det_is_ipv6(p, n) << 2 |
                       det_is_tcp(p, n) << 3 | det_is_udp(p, n) << 4 | det_is_icmp(p, n) << 5 |
                       det_is_http(p, n) << 6 | det_is_dns(p, n) << 7);
    /* detectMultipleProtocols :390-416 appends tcp/udp when n >= 34 */
    out[2] = (uint8_t)(det_is_arp(p, n) | (n >= 34 && p[23] == 6) << 1 | (n >= 34 && p[23] == 17) << 2);
}

void bto_parse(const uint8_t* frame, uint32_t len, uint8_t rec[96])
{
    memset(rec, 0, 96);
    detect(frame, len, rec + 88);
    uint16_t pl = (uint16_t)(len > 0xFFFF ? 0xFFFF : len);
    memcpy(rec + 14, &pl, 2);
    uint8_t present = L_ETH, ok = 0;

    /* 1. Ethernet at 0 */
    if (parse_layer(frame, len, T_ETH, NF(T_ETH), rec, 0)) ok |= L_ETH;
    else goto done;

    /* 2-3. up to two 802.1Q / 802.1ad tags */
    uint32_t et = be16(frame + 12);
    int k = 0;
    while (k < 2 && (et == 0x8100 || et == 0x88A8)) {
        uint32_t vo = 12 + 4 * (uint32_t)k;
        present |= (uint8_t)(L_VLAN0 << k);
        if (!parse_layer(frame + vo, len - vo, T_VLAN, NF(T_VLAN), rec, 2 * (uint32_t)k)) goto done;
        ok |= (uint8_t)(L_VLAN0 << k);
        if (len < vo + 6) goto done;          /* next EtherType not in the frame */
        et = be16(frame + vo + 4);
        ++k;
    }

    /* 4. L3 */
    uint32_t o3 = 14 + 4 * (uint32_t)k, o4 = 0, l4 = 0;
    if (et == 0x0800) {
        present |= L_IPV4;
        rec[26] = (uint8_t)o3;
        if (!parse_layer(frame + o3, len - o3, T_IPV4, NF(T_IPV4), rec, 0)) goto done;
        ok |= L_IPV4;
        uint32_t ihl = frame[o3] & 0x0F, proto = frame[o3 + 9];
        o4 = o3 + 4 * ihl;
        l4 = proto == 6 ? L_TCP : proto == 17 ? L_UDP : proto == 1 ? L_ICMP : 0;
        if (!l4 || o4 > len) goto done;
    } else if (et == 0x86DD) {
        present |= L_IPV6;
        rec[26] = (uint8_t)o3;
        if (!parse_layer(frame + o3, len - o3, T_IPV6, NF(T_IPV6), rec, 0)) goto done;
        ok |= L_IPV6;
        uint32_t nh = frame[o3 + 6];
        o4 = o3 + 40;
        l4 = nh == 6 ? L_TCP : nh == 17 ? L_UDP : 0;
        if (!l4) goto done;
    } else {
        goto done;
    }

    /* 5. L4 */
    present |= (uint8_t)l4;
    rec[27] = (uint8_t)o4;
    {
        const field_def* t = l4 == L_TCP ? T_TCP : l4 == L_UDP ? T_UDP : T_ICMP;
        int nf = l4 == L_TCP ? NF(T_TCP) : l4 == L_UDP ? NF(T_UDP) : NF(T_ICMP);
        if (parse_layer(frame + o4, len - o4, t, nf, rec, 0)) ok |= (uint8_t)l4;
    }
done:
    rec[24] = present;
    rec[25] = ok;
}

/* ---------------------------------------------------------------- filters */
enum { FT_BPF, FT_PROTOCOL, FT_IP_RANGE, FT_PORT_RANGE, FT_PAYLOAD, FT_CUSTOM };
enum { R_FALSE = 0, R_TRUE = 1, R_THROW = 2, R_HOST = 3 };

/* std::stoi as libstdc++ implements it (__stoa over strtol): no digits ->
 * invalid_argument; ERANGE or outside int -> out_of_range. Returns 0/1/2. */
static int stoi_r(const char* s, size_t n, int* out)
{
    char small[256];
    char* buf = n < sizeof(small) ? small : (char*)malloc(n + 1);
    memcpy(buf, s, n);
    buf[n] = 0;
    char* end;
    errno = 0;
    long v = strtol(buf, &end, 10);
    int rc = 0;
    if (end == buf) rc = 1;
    else if (errno == ERANGE || v < INT_MIN || v > INT_MAX) rc = 2;
    else *out = (int)v;
    if (buf != small) free(buf);
    return rc;
}

/* PacketFilter::parseIPAddress (src/PacketFilter.cpp:330-340): getline on '.', stoi
 * each token, cast to uint8_t. Returns token count (capped at 8) or -1 on throw. */
static int parse_ip(const char* s, size_t n, uint8_t* out)
{
    int cnt = 0;
    size_t pos = 0;
    while (pos < n) {
        size_t e = pos;
        while (e < n && s[e] != '.') ++e;
        int v;
        if (stoi_r(s + pos, e - pos, &v)) return -1;
        if (cnt < 8) out[cnt] = (uint8_t)v;
        ++cnt;
        pos = e < n ? e + 1 : n;
    }
    return cnt > 8 ? 8 : cnt;
}

/* isIPInRange (:342-360); returns R_TRUE/R_FALSE/R_THROW */
static int ip_in_range(const uint8_t ip[4], const char* r)
{
    size_t n = strlen(r);
    const char* slash = memchr(r, '/', n);
    uint8_t oct[8];
    if (slash) {
        size_t pos = (size_t)(slash - r);
        int prefix;
        if (stoi_r(r + pos + 1, n - pos - 1, &prefix)) return R_THROW;
        int cnt = parse_ip(r, pos, oct);
        if (cnt < 0) return R_THROW;
        if (cnt != 4) return R_FALSE;
        uint32_t net = ((uint32_t)oct[0] << 24) | ((uint32_t)oct[1] << 16) | ((uint32_t)oct[2] << 8) | oct[3];
        uint32_t ipa = ((uint32_t)ip[0] << 24) | ((uint32_t)ip[1] << 16) | ((uint32_t)ip[2] << 8) | ip[3];
        /* 0xFFFFFFFF << (32 - prefixLen): x86 SHL masks the count to 5 bits */
        uint32_t sh = (uint32_t)(32u - (uint32_t)prefix) & 31u;
        uint32_t mask = 0xFFFFFFFFu << sh;
        return (net & mask) == (ipa & mask) ? R_TRUE : R_FALSE;
    }
    int cnt = parse_ip(r, n, oct);
    if (cnt < 0) return R_THROW;
    return (cnt == 4 && memcmp(oct, ip, 4) == 0) ? R_TRUE : R_FALSE;
}

/* isPortInRange (:362-372) */
static int port_in_range(uint32_t port, const char* r)
{
    size_t n = strlen(r);
    const char* dash = memchr(r, '-', n);
    int a, b;
    if (dash) {
        size_t pos = (size_t)(dash - r);
        if (stoi_r(r, pos, &a)) return R_THROW;
        if (stoi_r(r + pos + 1, n - pos - 1, &b)) return R_THROW;
        uint32_t lo = (uint16_t)a, hi = (uint16_t)b;
        return (port >= lo && port <= hi) ? R_TRUE : R_FALSE;
    }
    if (stoi_r(r, n, &a)) return R_THROW;
    return port == (uint16_t)a ? R_TRUE : R_FALSE;
}

static int apply_one(const uint8_t* d, uint32_t len, const bto_filter* f)
{
    const char* e = f->expression ? f->expression : "";
    switch (f->type) {
    case FT_BPF:            /* :168-191 */
        if (!*e) return R_TRUE;
        if (len < 14) return R_FALSE;
        if (be16(d + 12) != 0x0800) return R_FALSE;
        if (len < 34) return R_FALSE;
        if (strstr(e, "tcp") && d[23] == 6) return R_TRUE;
        if (strstr(e, "udp") && d[23] == 17) return R_TRUE;
        if (strstr(e, "icmp") && d[23] == 1) return R_TRUE;
        return R_FALSE;
    case FT_PROTOCOL:       /* :193-217 */
        if (!*e) return R_TRUE;
        if (len < 14) return R_FALSE;
        if (be16(d + 12) != 0x0800) return R_FALSE;
        if (len < 34) return R_FALSE;
        if (!strcmp(e, "tcp") && d[23] == 6) return R_TRUE;
        if (!strcmp(e, "udp") && d[23] == 17) return R_TRUE;
        if (!strcmp(e, "icmp") && d[23] == 1) return R_TRUE;
        if (!strcmp(e, "ip") && d[23] != 0) return R_TRUE;
        return R_FALSE;
    case FT_IP_RANGE: {     /* :219-247 */
        if (!*e) return R_TRUE;
        if (len < 34) return R_FALSE;
        if (be16(d + 12) != 0x0800) return R_FALSE;
        int r = ip_in_range(d + 26, e);
        if (r != R_FALSE) return r;
        return ip_in_range(d + 30, e);
    }
    case FT_PORT_RANGE: {   /* :249-286 — L4 at the fixed offset 34 (ignores IHL and VLAN) */
        if (!*e) return R_TRUE;
        if (len < 34) return R_FALSE;
        if (be16(d + 12) != 0x0800) return R_FALSE;
        uint8_t proto = d[23];
        if ((proto == 6 && len >= 54) || (proto == 17 && len >= 42)) {
            int r = port_in_range(be16(d + 34), e);
            if (r != R_FALSE) return r;
            return port_in_range(be16(d + 36), e);
        }
        return R_FALSE;
    }
    case FT_PAYLOAD:        /* :288-321 — std::regex lives on the host */
        return *e ? R_HOST : R_TRUE;
    case FT_CUSTOM:         /* :323-328 */
        return f->has_custom_func ? R_HOST : R_TRUE;
    }
    return R_FALSE;         /* a type outside FilterType matches no case: filterResult stays false (:80) */
}

/* applyFilters(const Packet&) (:57-119): enabled filters, priority-descending
 * (stable here: ties keep input order), AND with early exit. */
static uint32_t sorted_order(const bto_filter* f, uint32_t nf, uint32_t* ord)
{
    uint32_t m = 0;
    for (uint32_t i = 0; i < nf; ++i)
        if (f[i].enabled) ord[m++] = i;
    for (uint32_t i = 1; i < m; ++i) {          /* insertion sort = stable */
        uint32_t x = ord[i], j = i;
        while (j > 0 && f[ord[j - 1]].priority < f[x].priority) { ord[j] = ord[j - 1]; --j; }
        ord[j] = x;
    }
    return m;
}

static uint8_t eval_sorted(const uint8_t* d, uint32_t len, const bto_filter* f,
                           const uint32_t* ord, uint32_t m)
{
    for (uint32_t s = 0; s < m; ++s) {
        int r = apply_one(d, len, &f[ord[s]]);
        if (r == R_FALSE) return (uint8_t)((1u << 6) | s);
        if (r == R_THROW) return (uint8_t)((2u << 6) | s);
        if (r == R_HOST) return (uint8_t)((3u << 6) | s);
    }
    return (uint8_t)(m ? m - 1 : 0);
}

uint8_t bto_filter_eval(const uint8_t* frame, uint32_t len, const bto_filter* f, uint32_t nf)
{
    uint32_t ord[64];
    if (nf > 64) nf = 64;
    uint32_t m = sorted_order(f, nf, ord);
    return eval_sorted(frame, len, f, ord, m);
}

/* ---------------------------------------------------------------- batch driver */
typedef struct {
    const uint8_t* base;
    const uint64_t* desc;
    uint32_t stride, lo, hi;
    const bto_filter* f;
    const uint32_t* ord;
    uint32_t m;
    uint8_t* records;
    uint8_t* decide;
    uint64_t passed;
} shard;

static void* run_shard(void* arg)
{
    shard* s = (shard*)arg;
    uint64_t passed = 0;
    for (uint32_t i = s->lo; i < s->hi; ++i) {
        const uint8_t* fr;
        uint32_t len;
        if (s->desc) {
            fr = s->base + (s->desc[i] & 0xFFFFFFFFFFFFull);
            len = (uint32_t)(s->desc[i] >> 48);
        } else {
            fr = s->base + (uint64_t)i * s->stride;
            len = s->stride;
        }
        if (s->records) bto_parse(fr, len, s->records + (uint64_t)i * 96);
        if (s->decide || s->f) {
            uint8_t dcs = eval_sorted(fr, len, s->f, s->ord, s->m);
            if (s->decide) s->decide[i] = dcs;
            passed += (dcs >> 6) == 0;
        }
    }
    s->passed = passed;
    return NULL;
}

uint64_t bto_run(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                 const bto_filter* f, uint32_t nf, uint8_t* records, uint8_t* decide,
                 int nthreads)
{
    uint32_t ord[64];
    if (nf > 64) nf = 64;
    uint32_t m = sorted_order(f, nf, ord);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    shard sh[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        sh[t] = (shard){base, desc, stride,
                        (uint32_t)((uint64_t)n * t / nthreads),
                        (uint32_t)((uint64_t)n * (t + 1) / nthreads),
                        f, ord, m, records, decide, 0};
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, run_shard, &sh[t]);
    run_shard(&sh[0]);
    uint64_t passed = sh[0].passed;
    for (int t = 1; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        passed += sh[t].passed;
    }
    return passed;
}

/* ------------------------------------------------- user-defined protocol tables */
/* FieldType values (reference include/parser/FieldDefinition.hpp:16-35) */
enum { UT_U8, UT_U16, UT_U32, UT_U64, UT_I8, UT_I16, UT_I32, UT_I64, UT_F32, UT_F64, UT_BYTES, UT_STRING,
       UT_BOOL, UT_MAC, UT_IPV4, UT_IPV6, UT_TIMESTAMP, UT_CUSTOM };

/* ProtocolDefinition::getTotalLength (src/parser/FieldDefinition.cpp:31-46): the end of
 * the first field whose end beats every earlier one. */
static uint64_t user_total_length(const uint64_t* fields, uint32_t nf) {
    uint64_t mo = 0, ml = 0;
    if (!nf) return 0;
    for (uint32_t k = 0; k < nf; ++k) {
        const uint64_t end = fields[4 * k] + fields[4 * k + 1];
        if (end > mo + ml) { mo = fields[4 * k]; ml = fields[4 * k + 1]; }
    }
    return mo + ml;
}

/* extractValue<T> (src/parser/ProtocolParser.cpp:385-433). The integer loop
 * `value |= static_cast<T>(p[...]) << (i * 8)` shifts in int (types narrower than 32 bits
 * are promoted), unsigned or 64-bit arithmetic; a count at or past that width is
 * undefined in C++, and x86-64 takes it modulo the width, which is what the compiled
 * reference does (pinned by the extract golden, lengths up to 20 on every type). */
static uint64_t user_value(const uint8_t* p, uint64_t o, uint64_t L, uint32_t type, uint32_t endian) {
    const int le = endian == 0;
    uint64_t v = 0;
    switch (type) {
    case UT_F32:
    case UT_F64: {
        const uint64_t want = type == UT_F32 ? 4 : 8;
        if (L != want) return 0;
        for (uint64_t i = 0; i < want; ++i) v |= (uint64_t)p[o + (le ? i : want - 1 - i)] << (8 * i);
        return v;
    }
    case UT_BOOL: return p[o] != 0;
    case UT_BYTES: case UT_STRING: case UT_MAC: case UT_IPV4: case UT_IPV6: case UT_CUSTOM: return 0;
    default: {
        const int wide = type == UT_U64 || type == UT_I64 || type == UT_TIMESTAMP;
        const uint32_t width = (type == UT_U8 || type == UT_I8) ? 8 : (type == UT_U16 || type == UT_I16) ? 16
                             : (type == UT_U32 || type == UT_I32) ? 32 : 64;
        for (uint64_t i = 0; i < L; ++i) {
            const uint64_t b = p[o + (le ? i : L - 1 - i)];
            v |= b << ((8 * i) & (wide ? 63 : 31));
        }
        return width == 64 ? v : (v & ((1ull << width) - 1));
    }
    }
}

uint64_t bto_extract(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                     const uint64_t* fields, uint32_t nf, uint8_t* status, uint64_t* values, uint8_t* image) {
    const uint64_t span = user_total_length(fields, nf);
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = desc ? base + (desc[i] & 0xFFFFFFFFFFFFull) : base + (uint64_t)i * stride;
        const uint64_t len = desc ? desc[i] >> 48 : stride;
        const int ok = len >= span;   /* parsePacketInternal :244-247 */
        if (status) status[i] = ok ? 0 : 9;
        for (uint32_t k = 0; values && k < nf; ++k) {
            const uint64_t o = fields[4 * k], L = fields[4 * k + 1];
            /* :251-254: a field past the packet is skipped (never, once len >= span) */
            values[(uint64_t)k * n + i] = ok && o + L <= len
                ? user_value(f, o, L, (uint32_t)fields[4 * k + 2], (uint32_t)fields[4 * k + 3]) : 0;
        }
        if (image && span) {
            uint8_t* out = image + (uint64_t)i * span;
            if (ok) memcpy(out, f, span);
            else memset(out, 0, span);
        }
    }
    return span;
}
