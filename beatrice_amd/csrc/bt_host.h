// bt_host.h — runtime services shared by the host-only translation units of
// libbeatrice_gpu.so (bt_ring.cpp, bt_group.cpp): the thread-local error slot behind
// bt_last_error(), the context's host thread pool, and filter programs.
#pragma once

#include <sched.h>

#include <functional>
#include <vector>

#include "beatrice_gpu_bench.h"   // the product header + the harness entry points

namespace bt {

// A compiled PacketFilter program: the slots (bt_filter_compile_host) and the DFA tables
// of its BT_K_PAYLOAD slots. compile_program is host-only; install_program puts it on a
// context's device (bt_filter_compile = both; a group compiles once, installs on each).
struct CompiledProgram {
    std::vector<bt_filter_slot> slots;
    std::vector<uint8_t> dfa_pool;
};
int compile_program(const bt_filter_desc* f, uint32_t n, uint32_t ctx_flags, CompiledProgram* out);
int install_program(bt_ctx* c, const CompiledProgram& p);
uint32_t ctx_flags(const bt_ctx* c);
int ctx_device(const bt_ctx* c);
// Whether the context's stream still has queued work (hipStreamQuery: not ready).
bool ctx_stream_busy(bt_ctx* c);
// The CPUs the context's pool workers are pinned to (its device's NUMA node), or NULL.
const cpu_set_t* ctx_pin(const bt_ctx* c);
// Drops the context's cached "is this batch base host memory" answer (after an unregister).
void ctx_forget_base(bt_ctx* c);
// bt_host_stage_bytes without the C-ABI's checks.
uint32_t stage_bytes_of(bt_ctx* c, bool records);
// Bytes per frame the host pipeline copies to the device (<= stage_bytes_of: a filter-only
// call stages bytes 12..43 only): the host batches' split cost.
uint32_t staged_bytes_of(bt_ctx* c, bool records);
// The same, lock-free: the value the context published when its program was last installed
// (bt_filter_compile on the context itself or through its group), so a group's split never
// waits for a member's host batch in flight.
uint32_t staged_window(const bt_ctx* c, bool records);
// CPUs this process may use: its affinity set bounded by the cgroup v2 CPU quota.
unsigned usable_cpus();
// The CPUs of NUMA node `node` in this process's affinity set (false: none / unknown).
bool node_cpus(int node, cpu_set_t* out);

// The process's registered host pages (bt_pin.h / bt_pin.cpp): every bt_host_register,
// bt_group_host_register and group scratch registration goes through these. acquire takes a
// reference on the whole pages of [host, host + bytes) (registering them, portable + mapped,
// unless a live span holds them all; refused when a live span holds some of them) and writes
// the alias of `host` on each of devices[0..n) to aliases[i]; release drops it (the last one
// waits for the devices that hold an alias, then unregisters). BT_OK or a bt_last_error code.
int pin_acquire(const void* host, uint64_t bytes, const int* devices, uint32_t n_devices, uint8_t** aliases);
int pin_alias(const void* host, uint64_t bytes, int device, uint8_t** alias);
int pin_release(const void* host, uint64_t bytes);
// (lo, hi, refs) of up to cap live spans, ascending; returns how many there are.
uint32_t pin_spans(uint64_t* lo_hi_refs, uint32_t cap);

// Sets bt_last_error() and returns `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Runs fn(worker, n_workers) on every worker of ctx's host pool (the caller is
// worker 0) and waits; with ctx == NULL it runs fn(0, 1) inline.
void host_parallel(bt_ctx* ctx, const std::function<void(unsigned, unsigned)>& fn);
// The size of ctx's host pool (created on first use).
unsigned pool_size(bt_ctx* ctx);

}  // namespace bt
