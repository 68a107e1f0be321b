/* beatrice_gpu_bench.h — the test and benchmark side of libbeatrice_gpu.so.
 *
 * Device memory, copies and streams for hosts without a HIP toolchain (the Python tests
 * through ctypes, bench.py), and the timing loops bench.py measures the kernels with. A
 * Beatrice host integrating the stage needs only include/beatrice_gpu.h (INTEGRATION.md
 * §1); nothing here is part of the drop-in contract of SURVEY §8(b). The symbols live in the
 * same library. */
#ifndef BEATRICE_GPU_BENCH_H
#define BEATRICE_GPU_BENCH_H

#include "beatrice_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- device memory and streams ------------------------------------------------ */
int  bt_dev_malloc(bt_ctx* ctx, uint64_t bytes, void** out);
int  bt_dev_free(bt_ctx* ctx, void* p);
int  bt_memcpy_h2d(bt_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int  bt_memcpy_d2h(bt_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int  bt_memset_d(bt_ctx* ctx, void* dst, int value, uint64_t bytes);
/* Caller-owned streams on the context's device (a hipStream_t, non-blocking) for the
 * `stream` arguments of bt_parse_filter_device / bt_extract_device, for hosts that cannot
 * create one themselves. Destroying a stream waits for its work. */
int  bt_stream_create(bt_ctx* ctx, void** stream);
int  bt_stream_synchronize(bt_ctx* ctx, void* stream);
int  bt_stream_destroy(bt_ctx* ctx, void* stream);
/* Timing of a device-resident run on the context stream: `iters` steps, each = the
 * main kernel between an event pair + the compaction kernels; returns the event span
 * per step and the mean main-kernel time. With BT_OPT_GRAPH the steps are captured
 * once into a hipGraph (first call per (batch, outputs, iters)) and replayed, and
 * main_ms is -1 (HIP does not time events recorded inside a graph). */
int  bt_time_device(bt_ctx* ctx, const bt_batch* batch, const bt_outputs* out,
                    uint32_t iters, float* ms_per_iter, float* main_kernel_ms);
/* The same with a breakdown of where the host's wall time goes (bench.py puts it in its
 * JSON line). The host waits by polling hipEventQuery (no interrupt wake-up): the time
 * until the first event is seen complete and from there until the last one are
 * reported separately, so a late start on the GPU and a late completion notice can be
 * told apart. */
typedef struct bt_timing {
    float span_ms;                 /* GPU: event before the first step -> after the last */
    float main_ms;                 /* mean main-kernel time (its own dispatch events)     */
    float main_min_ms, main_max_ms;
    float lead_ms;                 /* GPU: first event -> first main kernel's start       */
    float gap_ms;                  /* GPU: sum over steps of (next main start - main end) */
    double enqueue_ms;             /* host: all launches enqueued                         */
    double first_seen_ms;          /* host: enqueue done -> first event seen complete     */
    double last_seen_ms;           /* host: first event seen -> last event seen           */
    double query_ms;               /* host: elapsed-time queries                          */
    double wall_ms;                /* host: the whole call                                */
    int32_t spin_rc;               /* hipSetDeviceFlags(spin) result at bt_create, -1 unset */
    uint32_t device_flags;         /* hipGetDeviceFlags after bt_create                   */
    uint32_t reserved[6];
} bt_timing;
int  bt_time_device_ex(bt_ctx* ctx, const bt_batch* batch, const bt_outputs* out, uint32_t iters,
                       bt_timing* timing);
/* The general form. Step i writes output set out[i % n_out]. mode:
 *   BT_TIME_KERNEL_EVENTS  an event pair on every main kernel (main_ms, lead_ms, gap_ms);
 *                          recorded by the kernel's own dispatch, they cost the GPU ~9 us
 *                          per step on gfx950, so a throughput loop leaves them out and
 *                          the kernel is timed in a second call;
 *   BT_TIME_PIPELINED      the steps as bt_parse_filter_device_async (n_out = 2 keeps the
 *                          API's rule that a call's verdict buffer is not rewritten
 *                          before its compaction is done).
 * bt_time_device_ex = mode BT_TIME_KERNEL_EVENTS (| BT_TIME_PIPELINED under
 * BT_OPT_PIPELINE), n_out = 1. Without kernel events main_ms.. are -1, lead/gap 0. */
#define BT_TIME_KERNEL_EVENTS 0x1u
#define BT_TIME_PIPELINED     0x2u
int  bt_time_device2(bt_ctx* ctx, const bt_batch* batch, const bt_outputs* out, uint32_t n_out,
                     uint32_t iters, uint32_t mode, bt_timing* timing);

/* ---- timing of the user-protocol extractor ------------------------------------- */
/* bt_extract_device `iters` times on the context's stream, each launch timed by an event
 * pair from its own dispatch packet (bt_timing.main_* = the extraction kernel). For
 * benchmarks; the outputs are those of the last launch. BT_E_INVALID_ARGUMENT for an empty
 * batch or a table whose span no frame can reach (nothing would launch). */
int  bt_time_extract_ex(bt_ctx* ctx, const bt_batch* batch, const bt_field_def* fields, uint32_t n_fields,
                        const bt_extract_out* out, uint32_t iters, bt_timing* timing);
/* The same with a mode (BT_TIME_KERNEL_EVENTS only; without it main_ms.. are -1). */
int  bt_time_extract2(bt_ctx* ctx, const bt_batch* batch, const bt_field_def* fields, uint32_t n_fields,
                      const bt_extract_out* out, uint32_t iters, uint32_t mode, bt_timing* timing);

/* ---- host helpers the tests, tools and bench use (moved from beatrice_gpu.h: not part of
 * the drop-in contract INTEGRATION.md binds) ---------------------------------------- */
/* Host-only helpers: the CPUs of NUMA node `node` this process may use (*n = 0 if none or
 * unknown; at most cap written), and the CPUs it may use at all (affinity set bounded by
 * the cgroup v2 quota). */
int  bt_node_cpus(int node, int32_t* cpus, uint32_t cap, uint32_t* n);
/* host-only helper: compile without a context (no device needed) */
int  bt_filter_compile_host(const bt_filter_desc* filters, uint32_t n,
                            bt_filter_slot* out, uint32_t cap, uint32_t* n_slots);
/* ---- PAYLOAD filters on the GPU ---------------------------------
 * Replaces the per-packet std::regex construction + regex_search of
 * PacketFilter::applyPayloadFilter (src/PacketFilter.cpp:288-321) for the regular
 * subset of libstdc++'s ECMAScript grammar: the expression is compiled once to a byte
 * DFA that the kernel runs over the same <= 100-byte window after the IPv4 header.
 * bt_filter_compile does this for every PAYLOAD filter it can (BT_K_PAYLOAD slots, up
 * to 16 KiB of tables per program); the rest stay BT_K_HOST. The helpers below expose
 * the compiler and a host executor of the same DFA (tests, other hosts).
 *   bt_payload_dfa_compile  BT_OK (+ blob; blob == NULL: size only),
 *                           BT_E_INVALID_ARGUMENT if std::regex rejects the expression
 *                           (the reference's filter is then always false),
 *                           BT_E_NOT_IMPLEMENTED outside the modelled subset / too big,
 *                           BT_E_RESOURCE if cap is too small.
 *   bt_payload_dfa_search   regex_search(string(s, n), regex(expr)) for a compiled expr
 *   bt_payload_dfa_eval     applyPayloadFilter(frame, len) for a non-empty expression */
int  bt_payload_dfa_compile(const char* expression, void* blob, uint32_t cap, uint32_t* size);
/* The same with options: BT_DFA_NO_PAIRS leaves out the optional two-byte table (the
 * compiler adds it when it is <= 4 KiB; the filter compiler drops it when a program's
 * tables would not fit the 16 KiB pool otherwise). */
#define BT_DFA_NO_PAIRS 0x1u
/* BT_DFA_NO_BITPAR: always the DFA, never the bit-parallel form the compiler prefers for
 * unions of linear class sequences (A/B and tests; blob layouts in bt_regex_dfa.cpp). */
#define BT_DFA_NO_BITPAR 0x2u
int  bt_payload_dfa_compile_ex(const char* expression, uint32_t flags, void* blob, uint32_t cap, uint32_t* size);
int  bt_payload_dfa_search(const void* blob, const uint8_t* s, uint32_t n);
/* The same walk, and each frame's header prefix is also copied into slot i of `slots`
 * (BT_PREFIX_SLOT bytes per frame, slot i at i * BT_PREFIX_SLOT): the bytes the layer walk
 * and the built-in filters read, i.e. max(38, the walked header end) rounded up to 16, at
 * most the frame. desc[i] = BT_DESC(i * BT_PREFIX_SLOT, min(tp_snaplen, 65535)). A batch
 * over `slots` (registered, or copied to the device) with flags = BT_BATCH_PREFIXES then
 * reads one aligned 64-B host line per packet over PCIe for headers up to 64 B, instead
 * of a window straddling the ring's 2-mod-16 frame starts. The walker copies while its
 * chains are in flight, one frame behind each chain's header read. */
int  bt_ring_gather_tpv3(bt_ctx* ctx, const bt_tpv3_ring* ring, uint32_t first_block, uint32_t max_blocks,
                         uint8_t* slots, bt_pkt_desc* desc, uint32_t cap, uint32_t* n_desc,
                         uint32_t* n_blocks_taken);
/* The walk with the frame chains followed on the GPU. The host reads only the taken blocks'
 * headers (block_status, num_pkts, offset_to_first_pkt: one line per block) and a kernel on
 * `stream` walks every chain through ring_dev (the ring's device-visible alias, e.g. from
 * bt_host_register), one lane per block, writing the descriptors (as bt_ring_walk_tpv3
 * does) into desc_dev, device memory of cap entries. *n_desc and *n_blocks_taken are known
 * on return, the descriptors once the stream has run the kernel; batches on the same
 * stream that read desc_dev follow it in order. A chain that leaves its block makes that
 * block's remaining descriptors empty (length 0: nothing of them is read) and stores
 * block + 1 into *bad_dev (device memory, optional; the largest such block wins). */
int  bt_ring_walk_tpv3_gpu(bt_ctx* ctx, const bt_tpv3_ring* ring, const void* ring_dev, uint32_t first_block,
                           uint32_t max_blocks, bt_pkt_desc* desc_dev, uint32_t cap, uint32_t* n_desc,
                           uint32_t* n_blocks_taken, uint32_t* bad_dev, void* stream);
/* The split (host only): bounds[0..parts] with bounds[0] = 0, bounds[parts] = n, every
 * inner bound a multiple of 64, member k taking [bounds[k], bounds[k+1]); balanced by the
 * cost min(len, 128) + 8 + 96 bytes per packet (beatrice_amd/shard.py:shard_bounds). */
int      bt_group_split(const uint32_t* lens, uint32_t n, uint32_t parts, uint32_t* bounds);
/* The same with a cost model: packet cost = round_up(min(len, window), align) + fixed.
 * The group's calls weigh packets by what each call moves (bt_group_cost). */
typedef struct bt_split_cost {
    uint32_t window;               /* bytes of each frame the call reads / stages         */
    uint32_t align;                /* ... rounded up to this (1 = exact)                  */
    uint32_t fixed;                /* per-packet bytes independent of the length          */
    uint32_t reserved;
} bt_split_cost;
int      bt_group_split_cost(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost,
                             uint32_t* bounds);
/* The split the group's calls use: bt_group_split_cost up to 4096 tiles; above, the cost of
 * one tile in every S (~4096 samples) stands for its run of S tiles and the cuts interpolate
 * within a run (an exact pass over 16M descriptors took ~45 ms on one thread before any
 * member started). Same form of bounds. */
int      bt_group_split_plan(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost,
                             uint32_t* bounds);
/* The cost model a group call uses (mapped: bt_group_parse_filter_mapped, else the host
 * batches), for a call that asks for records / filter outputs, with desc_bytes-byte
 * descriptors (8 packed, 16 xdp_desc, 0 fixed stride):
 *   host batches: window = the bytes staged per frame (32: a filter-only call stages frame
 *                 bytes 12..43; 112 with records; 176 with a GPU PAYLOAD slot), align 16,
 *                 fixed = desc_bytes + 96 (records, bt_rec D2H) + 1 (decision D2H)
 *   mapped:       window = 128 with records (the walk's wide window) else 48 (the lean
 *                 first round reads frame bytes 12..37: two or three 16-B chunks by the
 *                 frame's alignment, 32 B + one chunk of slack), align 16, fixed =
 *                 desc_bytes + 64 (records: packed slabs) + 1 (decision) — all of it PCIe
 *                 traffic of the member's link. */
int      bt_group_cost(bt_group* group, int mapped, int records, int filters, uint32_t desc_bytes,
                       bt_split_cost* out);
/* Host threads per member: `requested` (opts.host_threads, else BT_HOST_THREADS; 0 = auto)
 * is the whole group's budget, split evenly (at least 1, at most 16 each); auto gives each
 * member usable / members, at least 1 and at most 16 (one context alone: min(16, usable), the
 * single-context default; a context's host pipeline takes at most 8 of them while other callers
 * wait for the context). Host only; bt_group_create applies it. */
int      bt_group_thread_budget(uint32_t members, uint32_t usable, uint32_t requested, uint32_t* per_member);
void bt_record_gather_planes(const void* planes, uint32_t n_cap, uint32_t i, bt_rec* out);
/* Slabs the packed device form of this record occupies (2..6). */
uint32_t bt_record_slabs(const bt_rec* r);

/* ---- registered host pages (diagnostics) ---------------------------------------
 * bt_host_register and bt_group_host_register keep one process-wide table of the whole
 * pages they registered (beatrice_amd/csrc/bt_pin.h): lo_hi_refs[3 i .. 3 i + 2] = span i's
 * first byte, end (both page-aligned) and reference count, ascending, for up to cap spans;
 * *n = the number of live spans. Host only (no device call). */
int  bt_host_pins(uint64_t* lo_hi_refs, uint32_t cap, uint32_t* n);
/* Device `device`'s alias of [host, host + bytes), which must lie inside one registered span
 * (BT_E_INVALID_ARGUMENT otherwise): what the kernels of a mapped call read it through. */
int  bt_host_alias(const void* host, uint64_t bytes, int device, void** alias);

#ifdef __cplusplus
}
#endif

#endif /* BEATRICE_GPU_BENCH_H */
