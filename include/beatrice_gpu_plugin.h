/* beatrice_gpu_plugin.h — C hooks of libgpu_parse_filter_plugin.so, the MI355X parse +
 * PacketFilter stage as a Beatrice IPacketPlugin (reference include/beatrice/IPacketPlugin.hpp:9-33,
 * loaded by PluginManager::loadPlugin, src/PluginManager.cpp:38-122).
 *
 * The plugin batches onPacket calls and classifies whole batches on the GPU, so a packet's
 * verdict is known only after its batch ran. Code downstream of PluginManager that wants
 * the verdicts (another plugin, the application) installs a verdict sink on the
 * IPacketPlugin* the manager created: it is called once per classified batch, in arrival
 * order, one batch at a time, on one of the plugin's classifier threads. All pointers are
 * valid for the duration of the call only.
 *
 * With BEATRICE_GPU_RECORDS=1 the same kernel pass also parses every packet, and the sink
 * sees each packet's bt_rec: the fields of every walked layer as the reference's
 * ProtocolParser::parsePacket(slice, name) returns them (include/beatrice_gpu.h). The
 * helpers below turn a record into its walked layers or into the reference's ParseResult
 * text, as PluginManager::processPackets consumers (src/PluginManager.cpp:173-188) would
 * get from calling the parser themselves. */
#ifndef BEATRICE_GPU_PLUGIN_H
#define BEATRICE_GPU_PLUGIN_H

#include <stdint.h>

#include "beatrice_gpu.h"

#ifdef __cplusplus
namespace beatrice { class IPacketPlugin; }
typedef beatrice::IPacketPlugin gpu_plugin;
extern "C" {
#else
typedef struct gpu_plugin gpu_plugin;
#endif

typedef struct gpu_verdict_batch {
    uint64_t seq;                      /* batch number, 0, 1, 2, ... in arrival order       */
    uint32_t n;                        /* packets in the batch                               */
    const uint8_t* const* frames;      /* bytes of packet i (the Packet's own buffer)        */
    const uint32_t* lens;
    const uint8_t* decide;             /* (BT_DECIDE_* << 6) | deciding slot, per packet     */
    const uint32_t* pass_idx;          /* ascending indices of the packets that passed       */
    uint32_t n_pass;
    const uint32_t* error_idx;         /* indices of the packets whose evaluation threw       */
    uint32_t n_error;                  /* (counted in IPacketPlugin::getErrorCount)          */
    const bt_rec* records;             /* BEATRICE_GPU_RECORDS=1: packet i's parse record; else NULL */
} gpu_verdict_batch;

typedef struct gpu_walked_layer {      /* one layer of the walk (DESIGN.md R-WALK)           */
    const char* name;                  /* "ethernet" "vlan" "ipv4" "ipv6" "tcp" "udp" "icmp" */
    uint32_t offset;                   /* the slice's start in the frame                     */
    int32_t tag;                       /* VLAN tag index 0 / 1, -1 for other layers          */
    uint32_t parsed;                   /* 1 SUCCESS, 0 PACKET_TOO_SHORT (no fields)          */
} gpu_walked_layer;

typedef void (*gpu_verdict_sink_fn)(void* user, const gpu_verdict_batch* batch);

/* Installs (fn != NULL) or removes the verdict sink. */
void gpu_plugin_set_sink(gpu_plugin* plugin, gpu_verdict_sink_fn fn, void* user);
/* Classifies the partial batches now and returns once every batch queued so far has reached
 * the sink (the plugin's flush thread queues a partial batch on its own
 * BEATRICE_GPU_FLUSH_US after the batch's first packet). Not from inside the sink, which
 * runs on a classifier thread the call would wait for. */
void gpu_plugin_flush(gpu_plugin* plugin);
/* Packets that passed every filter so far. */
uint64_t gpu_plugin_passed(const gpu_plugin* plugin);
/* Packet i's walked layers (records != NULL): writes min(count, cap) entries, returns the
 * count (0 without records). */
uint32_t gpu_batch_layers(const gpu_verdict_batch* batch, uint32_t i, gpu_walked_layer* out, uint32_t cap);
/* The reference's ParseResult text of every walked layer of packet i (fmt = BT_FMT_*),
 * bt_format_records on its record: out == NULL asks for the size. BT_E_INVALID_ARGUMENT
 * without records or with a short buffer (*out_len = the size needed). */
int gpu_batch_format(const gpu_verdict_batch* batch, uint32_t i, uint32_t fmt, char* out, uint64_t cap,
                     uint64_t* out_len);

#ifdef __cplusplus
}
#endif

#endif /* BEATRICE_GPU_PLUGIN_H */
