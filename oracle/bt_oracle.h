/*
 * bt_oracle.h — CPU restatement of the reference parse+filter hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product path (beatrice_amd/) never does.
 *
 * Pinned against the compiled reference (oracle/_ref, built from the unmodified
 * /root/reference sources by oracle/Makefile) through the golden fixtures in
 * tests/golden/ (see tests/golden/make_golden.py).
 */
#ifndef BT_ORACLE_H
#define BT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bto_filter {      /* one PacketFilter::FilterConfig (reference PacketFilter.hpp:26-33) */
    int32_t     type;            /* FilterType order: BPF, PROTOCOL, IP_RANGE, PORT_RANGE, PAYLOAD, CUSTOM */
    const char* expression;
    int32_t     enabled;
    int32_t     priority;
    int32_t     has_custom_func;
} bto_filter;

/* Parse one frame into the 96-byte bt_rec layout (include/beatrice_gpu.h). */
void bto_parse(const uint8_t* frame, uint32_t len, uint8_t rec[96]);

/* Evaluate filters (input order; the oracle does its own stable priority sort)
 * on one frame; returns the decision byte (code << 6 | slot). */
uint8_t bto_filter_eval(const uint8_t* frame, uint32_t len, const bto_filter* f, uint32_t nf);

/* Batch driver: desc == NULL selects fixed stride. records (AoS, 96 B each) and/or
 * decide may be NULL. Uses nthreads host threads on disjoint shards. Returns the
 * number of packets that passed (decision code PASS). */
uint64_t bto_run(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                 const bto_filter* f, uint32_t nf, uint8_t* records, uint8_t* decide,
                 int nthreads);

/* User-defined protocol tables: ProtocolParser::parsePacket(frame, ProtocolDefinition)
 * (reference src/parser/ProtocolParser.cpp:238-433). fields[4k..4k+3] = {offset, length,
 * FieldType, Endianness}. status[i] = ParseStatus (0 SUCCESS / 9 PACKET_TOO_SHORT);
 * values[k * n + i] = the bits of extractValue<T> zero-extended (bool 0/1, byte types 0);
 * image + i * span = the frame's bytes [0, span) when SUCCESS, zeros otherwise (any
 * output may be NULL). Returns the table's span (getTotalLength). */
uint64_t bto_extract(const uint8_t* base, const uint64_t* desc, uint32_t stride, uint32_t n,
                     const uint64_t* fields, uint32_t nf, uint8_t* status, uint64_t* values, uint8_t* image);

#ifdef __cplusplus
}
#endif
#endif
