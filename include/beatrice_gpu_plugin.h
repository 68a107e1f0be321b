/* beatrice_gpu_plugin.h — C hooks of libgpu_parse_filter_plugin.so, the MI355X parse +
 * PacketFilter stage as a Beatrice IPacketPlugin (reference include/beatrice/IPacketPlugin.hpp:9-33,
 * loaded by PluginManager::loadPlugin, src/PluginManager.cpp:38-122).
 *
 * The plugin batches onPacket calls and classifies whole batches on the GPU, so a packet's
 * verdict is known only after its batch ran. Code downstream of PluginManager that wants
 * the verdicts (another plugin, the application) installs a verdict sink on the
 * IPacketPlugin* the manager created: it is called once per classified batch, in arrival
 * order, on the thread that classified it (an onPacket caller or the plugin's flush
 * thread). All pointers are valid for the duration of the call only. */
#ifndef BEATRICE_GPU_PLUGIN_H
#define BEATRICE_GPU_PLUGIN_H

#include <stdint.h>

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
} gpu_verdict_batch;

typedef void (*gpu_verdict_sink_fn)(void* user, const gpu_verdict_batch* batch);

/* Installs (fn != NULL) or removes the verdict sink. */
void gpu_plugin_set_sink(gpu_plugin* plugin, gpu_verdict_sink_fn fn, void* user);
/* Classifies the partial batch now (the plugin's flush thread does it on its own
 * BEATRICE_GPU_FLUSH_US after the batch's first packet). */
void gpu_plugin_flush(gpu_plugin* plugin);
/* Packets that passed every filter so far. */
uint64_t gpu_plugin_passed(const gpu_plugin* plugin);

#ifdef __cplusplus
}
#endif

#endif /* BEATRICE_GPU_PLUGIN_H */
