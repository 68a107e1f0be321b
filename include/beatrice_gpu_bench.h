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

/* ---- registered host pages (diagnostics) ---------------------------------------
 * bt_host_register and bt_group_host_register keep one process-wide table of the whole
 * pages they registered (beatrice_amd/csrc/bt_pin.h): lo_hi_refs[3 i .. 3 i + 2] = span i's
 * first byte, end (both page-aligned) and reference count, ascending, for up to cap spans;
 * *n = the number of live spans. Host only (no device call). */
int  bt_host_pins(uint64_t* lo_hi_refs, uint32_t cap, uint32_t* n);

#ifdef __cplusplus
}
#endif

#endif /* BEATRICE_GPU_BENCH_H */
