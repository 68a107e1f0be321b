// bt_runtime.cpp — the C-ABI (include/beatrice_gpu.h) over the gfx950 kernels.
//
// Owns per-context HIP resources: a stream for device-resident calls, two streams +
// pinned staging for the host-batch pipeline, the compiled filter program and the
// device workspace for the ordered compaction. Nothing here throws across the ABI:
// failures return a beatrice::ErrorCode value and set a thread-local message.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cctype>
#include <mutex>
#include <string>
#include <vector>

#include "beatrice_gpu_bench.h"
#include "bt_device.h"
#include "bt_hip_util.h"
#include "bt_host_pool.h"
#include "bt_host.h"

using namespace bt;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(x)                                                                       \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) return fail(BT_E_INTERNAL, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

constexpr uint32_t kHostSlot = 112;   // bytes of each frame staged for the device (>= kNeedParse + pad)
// ... and with a GPU PAYLOAD slot in the program: applyPayloadFilter's window ends at most
// at 14 + 60 + 100 = 174 bytes (src/PacketFilter.cpp:293-309), rounded up to 16
constexpr uint32_t kHostSlotPayload = 176;
// ... and for calls that return no records and have no GPU PAYLOAD slot: the filters read
// bytes 12..37 (kNeedFilter) and such calls never take a second round, so 48 B
constexpr uint32_t kHostSlotFilter = 48;
// ... of which a filter-only call stages bytes [kLeanLo, kLeanLo + 32)
constexpr uint32_t kHostLeanWidth = 32;
static_assert(kLeanLo + kHostLeanWidth >= kNeedFilter && kLeanLo + kHostLeanWidth <= kHostSlotFilter, "lean staging");
constexpr uint32_t kGatherAheadDefault = 12;   // frames the host gather prefetches ahead
static_assert(kHostSlotFilter >= kNeedFilter && kHostSlotFilter % 16 == 0, "filter-only staging");

struct HostSlot {                      // one half of the double-buffered host pipeline
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* h_in = nullptr;           // pinned: prefixes then descriptors
    uint8_t* d_in = nullptr;
    uint8_t* h_out = nullptr;          // pinned: records (AoS) | decide | verdict
    uint8_t* d_out = nullptr;
    uint32_t* d_tile = nullptr;
    bool busy = false;
    uint32_t lo = 0, cnt = 0;          // packet range of the chunk in flight
};

using bt::HostPool;   // bt_host_pool.h

}  // namespace

struct bt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bt_opts opts{};
    int grid = 0;
    std::mutex mu;

    std::vector<bt_filter_slot> slots;
    DevProgram prog{};
    std::vector<uint8_t> dfa_pool;     // BT_K_PAYLOAD tables of the current program
    // the host batches' staged bytes per frame without / with records for the installed
    // program (stage_bytes / staged_bytes_of below), published by install_program so that a
    // group's split reads them without this context's lock (a host batch in flight holds it)
    std::atomic<uint32_t> staged_window[2] = {{0u}, {0u}};
    // PAYLOAD DFA pools, double-buffered: a recompile writes the buffer no queued launch
    // uses. Every stream that launched a kernel reading dfa_dev[k] has its own event in
    // dfa_readers[k], recorded right after that launch; a recompile that reuses buffer k
    // waits for all of them (a single event would only cover the last stream).
    uint8_t* dfa_dev[2] = {nullptr, nullptr};
    std::vector<std::pair<hipStream_t, hipEvent_t>> dfa_readers[2];
    std::vector<hipEvent_t> dfa_spare;   // events of cleared reader lists, reused
    int dfa_cur = 0;

    // device workspace of the compaction: chunk sums, and the verdict words when the
    // caller asks for none. Double-buffered (consecutive calls alternate). `last` = the
    // last stream that queued work touching the buffer (compared, never used, unless the
    // context owns it); before another stream touches it, that stream waits for `sync`:
    // recorded right after the work when `last` is a caller's stream (which may be
    // destroyed before the next touch), or at the switch when it is one of the context's
    // own streams (which live as long as the context). Calls that stay on the context's
    // streams queue no extra packets.
    uint32_t ws_cap = 0;
    struct Ws {
        uint32_t* chunk_sums = nullptr;
        uint64_t* verdict = nullptr;
        hipStream_t last = nullptr;
        bool lazy = false;             // sync not recorded yet (last is a context stream)
        hipEvent_t sync = nullptr;
    } ws[2];
    int ws_next = 0;
    // pipelined: main kernel -> compaction stream. A ring, so that an event is re-recorded
    // only long after the wait on its previous record has been consumed (re-recording one
    // of two alternating events cost ~7 us per step, profiles/r02/ab/timing_modes.txt).
    static constexpr int kMainDone = 8;
    hipEvent_t main_done[kMainDone] = {};
    int md_next = 0;
    hipStream_t cstream = nullptr;     // pipelined compaction (bt_parse_filter_device_async)

    // host pipeline
    uint32_t chunk = 0;
    HostSlot hs[2];
    bool host_ready = false;
    std::unique_ptr<HostPool> pool;   // created on first use (pool_of)
    std::atomic<int> waiters{0};      // callers waiting for `mu` to run a host batch (pipeline_share)
    uint64_t last_caller = 0;         // under mu: the last host batch's thread tag (WaitFor::thread_tag)
    uint64_t last_end = 0;            // ... and its end time in us
    bool shared_call = false;         // under mu: another thread used the context just before
    std::once_flag pool_once;
    // placement (place_ctx): the host NUMA node closest to the device and the CPUs of it this
    // process may use; the pool's workers run there when `pinned`
    int numa_node = -1;
    cpu_set_t pin{};
    bool pinned = false;

    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t pipe_done = nullptr;    // BT_OPT_PIPELINE: the last step's compaction
    hipEvent_t pipe_step = nullptr;    // pipelined with one output set: each step's compaction
    std::vector<hipEvent_t> tev;
    // bt_time_device: K steps captured once into one hipGraph, replayed per call
    hipGraphExec_t tgraph = nullptr;
    bt_batch tg_batch{};
    bt_outputs tg_out{};
    uint32_t tg_iters = 0;
    int spin_rc = -1;                  // hipSetDeviceFlags(hipDeviceScheduleSpin) result
    const void* last_base = nullptr;   // host_resident's one-entry cache
    bool last_base_host = false;
    // ranges page-locked through bt_host_register (under mu): a host batch's outputs inside
    // one are copied D2H in place instead of through the pinned staging
    std::vector<std::pair<uintptr_t, uint64_t>> host_regs;
    unsigned device_flags = 0;

    // bt_memcpy_h2d / bt_memcpy_d2h: two pinned chunks, so no copy of the caller's
    // (pageable) memory goes through the runtime's own pageable-copy path
    std::mutex xfer_mu;
    uint8_t* xfer_h[2] = {nullptr, nullptr};
    hipEvent_t xfer_ev[2] = {nullptr, nullptr};
    hipEvent_t xfer_after = nullptr;   // the compaction stream's tail (after_cstream)

    // bt_ring_walk_tpv3_gpu: the taken blocks' headers, in pinned memory the kernel reads;
    // two buffers, each reused once the walk that read it has run
    struct WalkStage {
        RingBlock* h = nullptr;
        uint32_t cap = 0;
        hipEvent_t done = nullptr;
        bool used = false;
    } walk[2];
    int walk_next = 0;

    // bt_extract (host lists): pinned + device staging, grown on demand
    uint8_t* ex_h = nullptr;
    uint8_t* ex_d = nullptr;
    size_t ex_cap = 0;
};

namespace bt {
void publish_staged_window(bt_ctx* c);   // defined with the host pipeline

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// CPUs this process may run on: the affinity set, bounded by the cgroup v2 CPU quota (a GPU
// box's job sees every CPU of the machine in its affinity set but may use 16).
unsigned usable_cpus() {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period) {
            const unsigned long long quota = strtoull(q, nullptr, 10) / period;
            if (quota >= 1 && quota < n) n = (unsigned)quota;
        }
        fclose(f);
    }
    return n;
}

// "0-3,8,10-11" (a sysfs cpulist) -> set; false if unreadable
bool parse_cpulist(const char* s, cpu_set_t* out) {
    CPU_ZERO(out);
    bool any = false;
    while (s && *s) {
        char* e = nullptr;
        const long a = strtol(s, &e, 10);
        if (e == s || a < 0) return false;
        long b = a;
        s = e;
        if (*s == '-') {
            b = strtol(s + 1, &e, 10);
            if (e == s + 1 || b < a) return false;
            s = e;
        }
        for (long i = a; i <= b && i < CPU_SETSIZE; ++i) CPU_SET((int)i, out);
        any = true;
        while (*s == ',' || *s == '\n' || *s == ' ') ++s;
    }
    return any;
}

// The host NUMA node closest to `device`: HIP's attribute, else the PCI function's sysfs
// numa_node (read from its bus id); -1 when the host has no NUMA information.
int device_numa_node(int device) {
    int node = -1;
    if (hipDeviceGetAttribute(&node, hipDeviceAttributeHostNumaId, device) != hipSuccess) {
        (void)hipGetLastError();
        node = -1;
    }
    if (node >= 0) return node;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char* p = bus; *p; ++p) *p = (char)tolower((unsigned char)*p);
    char path[160];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE* f = fopen(path, "r")) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    return node;
}

// The CPUs of NUMA node `node` that this process may run on (its affinity set); false when
// there are none or the node's cpulist is unreadable.
bool node_cpus(int node, cpu_set_t* out) {
    if (node < 0) return false;
    char path[96];
    snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    char buf[4096] = {0};
    FILE* f = fopen(path, "r");
    if (!f) return false;
    const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[got] = 0;
    cpu_set_t nodeset, aff;
    if (!parse_cpulist(buf, &nodeset)) return false;
    if (sched_getaffinity(0, sizeof(aff), &aff) != 0) return false;
    CPU_AND(out, &nodeset, &aff);
    return CPU_COUNT(out) > 0;
}

// Places a context's host work next to its device: the pool's workers (gather, drain, ring
// walk) run on the CPUs of the device's NUMA node. hipHostMalloc without
// hipHostMallocNumaUser allocates the pinned staging near the current device already (HIP
// lets the user's policy decide only with that flag, hip_runtime_api.h), and the staging
// is allocated after hipSetDevice (ensure_host). BT_NUMA_PIN=0 turns the pinning off (A/B).
void place_ctx(bt_ctx* c) {
    c->numa_node = device_numa_node(c->device);
    static const bool off = [] {
        const char* e = getenv("BT_NUMA_PIN");
        return e && atoi(e) == 0;
    }();
    c->pinned = !off && node_cpus(c->numa_node, &c->pin);
}

// The pool's size: opts.host_threads, else BT_HOST_THREADS, else the usable CPUs; at most 16.
// A group sets each member's opts.host_threads from its budget (bt_group.cpp). Round 3 capped
// the default at 8: with callers on all 16 of a GPU box's CPUs (T callers of one
// GpuPacketFilter, the plugin's onPacket threads) a 16-thread pool oversubscribed them
// (profiles/r03/surfaces/ab_pool_threads.jsonl). Now a chunk's gather takes at most 8 of the
// pool while other callers wait (pipeline_share), and a lone caller all of it.
unsigned pool_threads_of(const bt_ctx* c) {
    unsigned nt = c->opts.host_threads;
    if (!nt) {
        const char* e = getenv("BT_HOST_THREADS");
        nt = e && atoi(e) > 0 ? (unsigned)atoi(e) : usable_cpus();
    }
    return std::max(1u, std::min(nt, 16u));
}

HostPool& pool_of(bt_ctx* c) {
    std::call_once(c->pool_once, [c] {
        c->pool = std::make_unique<HostPool>(pool_threads_of(c), c->pinned ? &c->pin : nullptr);
    });
    return *c->pool;
}

unsigned pool_size(bt_ctx* ctx) { return pool_of(ctx).size(); }

void host_parallel(bt_ctx* ctx, const std::function<void(unsigned, unsigned)>& fn) {
    if (!ctx) {
        fn(0, 1);
        return;
    }
    HostPool& pool = pool_of(ctx);
    const unsigned T = pool.size();
    pool.run([&](unsigned w) { fn(w, T); });
}

}  // namespace bt

namespace {

void free_ws(bt_ctx* c) {
    for (auto& w : c->ws) {
        if (w.chunk_sums) (void)hipFree(w.chunk_sums);
        if (w.verdict) (void)hipFree(w.verdict);
        w.chunk_sums = nullptr; w.verdict = nullptr; w.last = nullptr; w.lazy = false;
    }
    c->ws_cap = 0;
}

int ensure_ws(bt_ctx* c, uint32_t n) {
    if (n <= c->ws_cap && c->ws[0].chunk_sums) return BT_OK;
    HIP_TRY(hipSetDevice(c->device));
    // a cached BT_OPT_GRAPH timing graph holds the pointers replaced here
    if (c->tgraph) { (void)hipGraphExecDestroy(c->tgraph); c->tgraph = nullptr; }
    if (c->ws[0].chunk_sums) HIP_TRY(hipDeviceSynchronize());   // launches on any stream may use it
    free_ws(c);
    const uint32_t ntiles = (std::max(n, 1u) + 63) / 64;
    const uint32_t nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    for (auto& w : c->ws) {
        if (!w.sync) HIP_TRY(hipEventCreateWithFlags(&w.sync, hipEventDisableTiming));
        HIP_TRY(hipMalloc(&w.chunk_sums, (size_t)nchunks * 4));
        HIP_TRY(hipMalloc(&w.verdict, (size_t)ntiles * 8));
    }
    for (auto& e : c->main_done)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ws_cap = ntiles * 64;
    return BT_OK;
}

bool ctx_stream(const bt_ctx* c, hipStream_t s) { return s == c->stream || (c->cstream && s == c->cstream); }

// `s` is about to queue work that touches workspace buffer w: if another stream did last,
// s waits for everything that stream had queued on w.
int ws_touch(bt_ctx* c, bt_ctx::Ws* w, hipStream_t s) {
    if (w->last && w->last != s) {
        if (w->lazy) HIP_TRY(hipEventRecord(w->sync, w->last));   // a context stream: alive
        HIP_TRY(hipStreamWaitEvent(s, w->sync, 0));
    }
    (void)c;
    return BT_OK;
}

// `s` has just queued work touching w.
int ws_done(bt_ctx* c, bt_ctx::Ws* w, hipStream_t s) {
    w->last = s;
    w->lazy = ctx_stream(c, s);
    if (!w->lazy) HIP_TRY(hipEventRecord(w->sync, s));   // a caller's stream: record now
    return BT_OK;
}

int ensure_cstream(bt_ctx* c) {
    if (c->cstream) return BT_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    return BT_OK;
}

// Whether a batch's frames sit in host memory the device reads over PCIe (registered or
// pinned). One pointer query per new base (a capture ring or UMEM is one base for its life).
bool host_resident(bt_ctx* c, const void* base) {
    if (base == c->last_base) return c->last_base_host;
    hipPointerAttribute_t attr{};
    bool host = false;
    if (hipPointerGetAttributes(&attr, base) == hipSuccess) host = attr.type == hipMemoryTypeHost;
    else (void)hipGetLastError();
    c->last_base = base;
    c->last_base_host = host;
    static const bool dbg = getenv("BT_DEBUG_LEAN") != nullptr;
    if (dbg) fprintf(stderr, "[bt] batch base %p: %s memory (type %d)\n", base, host ? "host" : "device", (int)attr.type);
    return host;
}

// BT_DEBUG_BOUNDS builds: after a launch, wait and read the kernels' bounds logs
// (bt_bounds.h); a failed check becomes BT_E_INTERNAL naming the first one.
int check_bounds(hipStream_t st, hipStream_t cst, const char* what) {
#ifdef BT_DEBUG_BOUNDS
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return BT_OK;   // graph capture
    BoundsLog f{};
    uint32_t k = bounds_take_main(st, &f);
    if (!k && cst && cst != st) k = bounds_take_main(cst, &f);
    if (!k) k = bounds_take_extract(st, &f);
    if (k) {
        fprintf(stderr, "BT_DEBUG_BOUNDS: %s: %u failed checks, first %s (site %u) block %u thread %u index %llu "
                "limit %llu\n", what, k, bounds_site_name(f.site), f.site, f.block, f.lane,
                (unsigned long long)f.index, (unsigned long long)f.limit);
        return fail(BT_E_INTERNAL, "BT_DEBUG_BOUNDS: %s: %u failed checks, first %s index %llu limit %llu", what, k,
                    bounds_site_name(f.site), (unsigned long long)f.index, (unsigned long long)f.limit);
    }
#else
    (void)st;
    (void)cst;
    (void)what;
#endif
    return BT_OK;
}

// One parse+filter(+compaction) pass on `st`. `cst` = the stream of the compaction
// kernels: st itself, or (pipelined, bt_parse_filter_device_async) the context's
// compaction stream, which waits for this call's main kernel only, so the next call's
// main kernel on st runs beside this call's compaction; `done` (may be null) is
// recorded after the compaction on cst.
int run_device(bt_ctx* c, const bt_batch* b, const bt_outputs* o, hipStream_t st, bool aos,
               hipEvent_t e0, hipEvent_t e1, hipStream_t cst = nullptr, hipEvent_t done = nullptr) {
    if (!b || !o) return fail(BT_E_INVALID_ARGUMENT, "null batch/outputs");
    if (b->n && !b->base) return fail(BT_E_INVALID_ARGUMENT, "null packet buffer");
    if (!b->desc && b->stride == 0 && b->n) return fail(BT_E_INVALID_ARGUMENT, "fixed-stride mode needs stride > 0");
    // the calling thread's current device may be another context's (a group's member threads,
    // a host driving several devices): launches, events and allocations below are this one's
    HIP_TRY(hipSetDevice(c->device));
    if (o->records && o->n_cap < b->n) return fail(BT_E_INVALID_ARGUMENT, "records n_cap %u < n %u", o->n_cap, b->n);
    const bool filter = o->verdict || o->decide || o->pass_idx || o->n_pass;
    const bool compact = o->pass_idx || o->n_pass;
    if (!filter && !o->records) return BT_OK;
    if (!cst) cst = st;
    if (b->n == 0) {
        if (o->n_pass) HIP_TRY(hipMemsetAsync(o->n_pass, 0, 4, st));
        if (done) HIP_TRY(hipEventRecord(done, st));
        return BT_OK;
    }
    bt_ctx::Ws* w = nullptr;
    if (compact) {
        int rc = ensure_ws(c, b->n);
        if (rc) return rc;
        w = &c->ws[c->ws_next];
        c->ws_next ^= 1;
    }
    if (b->desc_format > BT_DESC_XDP) return fail(BT_E_INVALID_ARGUMENT, "unknown desc_format %u", b->desc_format);
    if ((b->flags & BT_BATCH_LEAN) && o->records)
        return fail(BT_E_INVALID_ARGUMENT, "a BT_BATCH_LEAN batch holds frame bytes 12..43 only: no records");
    // The readable range of base is part of the contract: descriptor batches must state it
    // (a descriptor past it then reads zeros instead of arbitrary memory); fixed-stride
    // batches default to n * stride.
    uint64_t bytes = b->bytes;
    if (b->desc) {
        if (!bytes) return fail(BT_E_INVALID_ARGUMENT, "descriptor batch with bytes == 0 (the readable size of base)");
    } else {
        const uint64_t need = (uint64_t)b->n * b->stride;
        if (!bytes) bytes = need;
        else if (bytes < need) return fail(BT_E_INVALID_ARGUMENT, "fixed-stride batch: bytes %llu < n * stride %llu",
                                           (unsigned long long)bytes, (unsigned long long)need);
    }
    MainArgs a{};
    a.base = b->base;
    a.desc = static_cast<const uint64_t*>(b->desc);
    a.desc_words = b->desc_format == BT_DESC_XDP ? 2u : 1u;
    a.prefixes = (b->flags & (BT_BATCH_PREFIXES | BT_BATCH_LEAN)) ? 1u : 0u;
    a.stride = b->stride;
    a.n = b->n;
    a.ntiles = (b->n + 63) / 64;
    a.bytes = read_limit(b->base, bytes);
    a.n_cap = o->records ? o->n_cap : 0;
    a.records = reinterpret_cast<uint8_t*>(o->records);
    a.decide = o->decide;
    a.verdict = o->verdict ? o->verdict : (w ? w->verdict : nullptr);
    if (w && !o->verdict) { int rc = ws_touch(c, w, st); if (rc) return rc; }   // the main kernel writes w->verdict
    a.blocked = (c->opts.flags & BT_OPT_TILE_BLOCKED) ? 1u : 0u;
    // Lean round A for frames read over PCIe, filter-only calls: the filters and the
    // detector read bytes 12..37, so round A reads only the 16-B chunks holding them (A/Bs:
    // round 3's 46-B first round against the 64-B window, profiles/r03/e2e/lean_ab.jsonl:
    // zero-copy verdicts C3 +17 %, C4 +4..10 %, C2 +2..4 %; round 4's [12, 38) against
    // [0, 46), profiles/r04/e2e/ab_lean_lo.jsonl: C4 zero-copy and ring +3..7 %, C2 / C3
    // level). Calls that also parse would need a second round for almost every tile (the
    // walk reads to L3 + 40 B) and lost 28-39 %: not lean.
    a.lean = 0xFFFFu;
    const bool lean = b->desc && !o->records && !(c->opts.flags & BT_OPT_NO_LEAN_PCIE) && host_resident(c, b->base);
    a.dfa = c->dfa_dev[c->dfa_cur];
    a.dfa_bytes = filter ? (uint32_t)c->dfa_pool.size() : 0u;
    // Cache policy (measured): non-temporal record stores everywhere (C2 +3..9 %,
    // profiles/r01) and non-temporal header loads (descriptor mode: C3 +15 %, C4 +8 %,
    // profiles/r01; fixed stride since round 2's kernels: c2f kernel 0.349-0.358 against
    // 0.364-0.365 ms, C2 0.332-0.337 against 0.347-0.348, profiles/r02/ab/nt_loads_fixed.txt).
    // BT_OPT_CACHE_DEFAULT turns both off, BT_OPT_NT_* force them on.
    if (c->opts.flags & BT_OPT_CACHE_DEFAULT) a.nt = 0;
    else a.nt = 3u;
    // A program with a GPU PAYLOAD slot reads each frame's payload window right after its
    // header window: header loads that keep their lines in L2 save those lines a second trip
    // to HBM (C3 with /GET|POST/ first, filter-only: 0.60 against 0.92 ms; a slot that reads
    // no window, 0.33 against 0.70; tools/payload_ab.py *_cache variants)
    if (a.dfa_bytes && !(c->opts.flags & BT_OPT_NT_LOADS)) a.nt &= ~2u;
    if (c->opts.flags & BT_OPT_NT_STORES) a.nt |= 1u;
    if (c->opts.flags & BT_OPT_NT_LOADS) a.nt |= 2u;
    if (c->opts.flags & BT_OPT_WIDE_NEVER) a.nt |= 4u;
    if (c->opts.flags & BT_OPT_WIDE_ALWAYS) a.nt |= 8u;
    a.lean_lo = 0;
    if (lean && !(a.nt & 8u)) {   // frames over PCIe: lean round A, never the wide 128-B mode
        static const uint32_t lean_end = [] {   // A/B knobs: BT_LEAN_END, BT_LEAN_LO
            const char* e = getenv("BT_LEAN_END");
            return e && atoi(e) >= (int)kNeedFilter ? (uint32_t)atoi(e) : kLeanPcie;
        }();
        static const uint32_t lean_lo = [] {
            const char* e = getenv("BT_LEAN_LO");
            return e && atoi(e) >= 0 && atoi(e) <= 12 ? (uint32_t)atoi(e) : kLeanLo;
        }();
        a.lean = lean_end;
        a.lean_lo = lean_lo;
        a.nt |= 4u;
    }
    int rec = kRecNone;
    if (o->records) {
        if (aos || (c->opts.flags & BT_OPT_RECORDS_AOS)) rec = kRecAoS;
        else if (c->opts.flags & BT_OPT_RECORDS_PLANES) rec = kRecPlanes;
        else rec = kRecTiled;
    }
    // e0 / e1 time the main kernel from its own dispatch packet (no marker packets: a
    // pair of hipEventRecord around the launch left the GPU idle ~6 us each, per step)
    const bool piped = compact && cst != st;
    // pipelined: the compaction stream waits for this main kernel's end, signalled by
    // the kernel's own dispatch (e1, or main_done)
    hipEvent_t mend = e1;
    if (piped && !e1) {
        mend = c->main_done[c->md_next];
        c->md_next = (c->md_next + 1) % bt_ctx::kMainDone;
    }
    int rc = launch_main(a, c->prog, rec, filter, c->grid, !(c->opts.flags & BT_OPT_NO_PREFETCH), st, e0, mend);
    if (rc) return fail(rc, "main kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (w && !o->verdict) { if ((rc = ws_done(c, w, st))) return rc; }
    if (a.dfa_bytes) {   // the pool this launch reads stays untouched until it has run
        auto& rd = c->dfa_readers[c->dfa_cur];
        auto it = std::find_if(rd.begin(), rd.end(), [st](const auto& x) { return x.first == st; });
        if (it == rd.end()) {
            hipEvent_t e = nullptr;
            if (!c->dfa_spare.empty()) { e = c->dfa_spare.back(); c->dfa_spare.pop_back(); }
            else HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            rd.emplace_back(st, e);
            it = rd.end() - 1;
        }
        HIP_TRY(hipEventRecord(it->second, st));
    }
    if (compact) {
        if (piped) HIP_TRY(hipStreamWaitEvent(cst, mend, 0));
        if ((rc = ws_touch(c, w, cst))) return rc;
        rc = launch_compact(a.verdict, b->n, w->chunk_sums, o->pass_idx, o->n_pass, cst);
        if (rc) return fail(rc, "compaction launch failed");
        if ((rc = ws_done(c, w, cst))) return rc;
        if (done) HIP_TRY(hipEventRecord(done, cst));
    } else if (done) {
        HIP_TRY(hipEventRecord(done, st));
    }
    return check_bounds(st, cst, "parse+filter");
}

void free_host(bt_ctx* c) {
    for (auto& s : c->hs) {
        if (s.stream) (void)hipStreamDestroy(s.stream);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.h_in) (void)hipHostFree(s.h_in);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.d_in) (void)hipFree(s.d_in);
        if (s.d_out) (void)hipFree(s.d_out);
        if (s.d_tile) (void)hipFree(s.d_tile);
        s = HostSlot{};
    }
    c->host_ready = false;
}

size_t in_bytes(uint32_t chunk) { return (size_t)chunk * kHostSlotPayload + (size_t)chunk * 8; }
size_t out_bytes(uint32_t chunk) { return (size_t)chunk * BT_REC_BYTES + chunk + ((size_t)chunk + 63) / 64 * 8; }

int ensure_host(bt_ctx* c) {
    if (c->host_ready) return BT_OK;
    HIP_TRY(hipSetDevice(c->device));
    static const uint32_t default_chunk = [] {   // BT_HOST_CHUNK: A/B knob for the default
        const char* e = getenv("BT_HOST_CHUNK");
        return e && atoi(e) >= 64 ? (uint32_t)atoi(e) : (1u << 20);
    }();
    uint32_t chunk = c->opts.host_chunk_packets ? c->opts.host_chunk_packets : default_chunk;
    chunk = (chunk + 63) / 64 * 64;
    c->chunk = chunk;
    (void)pool_of(c);
    for (auto& s : c->hs) {
        HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIP_TRY(hipHostMalloc(&s.h_in, in_bytes(chunk), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&s.h_out, out_bytes(chunk), hipHostMallocDefault));
        HIP_TRY(hipMalloc(&s.d_in, in_bytes(chunk)));
        HIP_TRY(hipMalloc(&s.d_out, out_bytes(chunk)));
    }
    c->host_ready = true;
    return BT_OK;
}

// The host pipeline's parallel steps for a chunk of `cnt` packets: on the pool, or for small
// chunks on the calling thread (every w in turn), where waking the pool cost more than the
// work (a 1k-packet classify took ~0.1 ms per call).
// fn(w) for w in [0, T), T = pipeline_share(c).
template <class Fn>
void pipeline_run(bt_ctx* c, uint32_t cnt, unsigned T, Fn&& fn) {
    static const uint32_t below = [] {
        const char* e = getenv("BT_HOST_INLINE_BELOW");   // A/B knob, 0 = always the pool
        return e ? (uint32_t)strtoul(e, nullptr, 10) : 8192u;
    }();
    if (cnt < below) {
        for (unsigned w = 0; w < T; ++w) fn(w);
    } else {
        c->pool->run(fn, T);
    }
}

// How much of the pool one chunk's gather / drain uses: all of it, or, while other callers
// wait for this context, at most kSharedPool threads. A lone caller then gets every pool thread
// (host-gather e2e with 16 of a 16-CPU host's: C4 349-408 -> 515-535 Mpps), while callers on
// every CPU (T callers of one GpuPacketFilter) keep to the share that does not oversubscribe
// them (16 callers lost 10-25 % with a 16-thread pool, profiles/r04/surfaces/ab_pool_8_16.jsonl).
constexpr unsigned kSharedPool = 8;
unsigned pipeline_share(const bt_ctx* c) {
    const unsigned T = c->pool->size();
    const bool shared = c->waiters.load(std::memory_order_relaxed) > 0 || c->shared_call;
    return shared ? std::min(T, kSharedPool) : T;
}

// Counts the caller as waiting for the context until it holds the context's lock, and marks
// the call shared when another thread held the context within the last kSharedWindowUs: callers
// that spend time outside the context between their calls (building FilterResults) are not
// waiting for it at the moment a chunk starts, but they are on the host's CPUs all the same.
constexpr uint64_t kSharedWindowUs = 2000;
struct WaitFor {
    std::unique_lock<std::mutex> lk;
    bt_ctx* c;
    uint64_t me;
    static uint64_t now_us() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    explicit WaitFor(bt_ctx* ctx) : lk(ctx->mu, std::defer_lock), c(ctx) {
        c->waiters.fetch_add(1, std::memory_order_relaxed);
        lk.lock();
        c->waiters.fetch_sub(1, std::memory_order_relaxed);
        me = thread_tag();
        const uint64_t now = now_us();
        c->shared_call = c->last_end && c->last_caller != me && now - c->last_end < kSharedWindowUs;
    }
    ~WaitFor() {
        c->last_caller = me;
        c->last_end = now_us();
    }
    // a process-unique number per thread (a hash of std::thread::id cut to 16 bits let two
    // threads collide and look like one lone caller)
    static uint64_t thread_tag() {
        static std::atomic<uint64_t> next{1};
        thread_local const uint64_t tag = next.fetch_add(1, std::memory_order_relaxed);
        return tag;
    }
};

// One frame's staged prefix: m bytes of src to dst (16-B aligned, its slot rounded up to 16).
// With `nt`, whole 16-B chunks go out as non-temporal stores (no read-for-ownership of the
// staging lines, which only the DMA engine reads next); the tail chunk is assembled from the
// frame's last bytes, never read past them. The caller fences (sfence) before the copy's
// consumer runs.
typedef long long v2i64 __attribute__((vector_size(16)));
inline void stage_prefix(uint8_t* dst, const uint8_t* src, uint32_t m, bool nt) {
    if (!nt) {
        std::memcpy(dst, src, m);
        return;
    }
    uint32_t k = 0;
    for (; k + 16 <= m; k += 16) {
        v2i64 x;
        std::memcpy(&x, src + k, 16);
        __builtin_nontemporal_store(x, reinterpret_cast<v2i64*>(dst + k));
    }
    if (k < m) {
        v2i64 x{};
        std::memcpy(&x, src + k, m - k);
        __builtin_nontemporal_store(x, reinterpret_cast<v2i64*>(dst + k));
    }
}

// Copies one finished chunk from pinned staging into the caller's buffers.
void drain_slot(bt_ctx* c, HostSlot& s, bt_rec* records, uint64_t* verdict, uint8_t* decide) {
    const uint32_t chunk = c->chunk;
    const uint8_t* rec = s.h_out;
    const uint8_t* dec = s.h_out + (size_t)chunk * BT_REC_BYTES;
    const uint64_t* ver = reinterpret_cast<const uint64_t*>(dec + chunk);
    const unsigned T = pipeline_share(c);
    const uint32_t lo = s.lo, cnt = s.cnt;
    static const bool drain_nt = [] {   // A/B knob: BT_DRAIN_NT=1 streams the records out
        const char* e = getenv("BT_DRAIN_NT");
        return e && atoi(e) != 0;
    }();
    pipeline_run(c, cnt, T, [&](unsigned w) {   // split on 64-packet boundaries
        const uint32_t tiles = (cnt + 63) / 64;
        const uint32_t t0 = (uint32_t)((uint64_t)tiles * w / T), t1 = (uint32_t)((uint64_t)tiles * (w + 1) / T);
        const uint32_t a = t0 * 64, b = std::min(cnt, t1 * 64);
        if (a >= b) return;
        if (records) {
            uint8_t* dst = reinterpret_cast<uint8_t*>(records + lo + a);
            const uint8_t* src = rec + (size_t)a * BT_REC_BYTES;
            const size_t bytes = (size_t)(b - a) * BT_REC_BYTES;   // a multiple of 16
            if (drain_nt && ((uintptr_t)dst & 15u) == 0) {   // the caller's records: not read back here
                for (size_t k = 0; k < bytes; k += 16)
                    __builtin_nontemporal_store(*reinterpret_cast<const v2i64*>(src + k), reinterpret_cast<v2i64*>(dst + k));
                __builtin_ia32_sfence();
            } else {
                std::memcpy(dst, src, bytes);
            }
        }
        if (decide) std::memcpy(decide + lo + a, dec + a, b - a);
        if (verdict) std::memcpy(verdict + (lo + a) / 64, ver + a / 64, (size_t)(t1 - t0) * 8);
    });
    s.busy = false;
}

}  // namespace

extern "C" {

int bt_abi_version(void) { return BT_ABI_VERSION; }

const char* bt_last_error(void) { return g_err.c_str(); }

int bt_device_count(int* out) {
    if (!out) return fail(BT_E_INVALID_ARGUMENT, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return BT_OK;
}

int bt_create(int device, const bt_opts* opts, bt_ctx** out) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!out) return fail(BT_E_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(BT_E_INIT_FAILED, "no HIP device visible (the MI355X path needs a GPU)");
    if (device < 0 || device >= n) return fail(BT_E_INVALID_ARGUMENT, "device %d out of range [0,%d)", device, n);
    auto* c = new bt_ctx();
    c->device = device;
    if (opts) c->opts = *opts;
    if (c->opts.flags & BT_OPT_SPIN_SYNC) {
        // host waits spin instead of sleeping: no wake-up latency on a loaded host.
        // Only possible before the process's first HIP context on this device.
        (void)hipSetDevice(device);
        c->spin_rc = (int)hipSetDeviceFlags(hipDeviceScheduleSpin);
        (void)hipGetLastError();   // a refusal (context already active) is reported, not sticky
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(BT_E_INIT_FAILED, "hipSetDevice/hipStreamCreate failed on device %d", device);
    }
    (void)hipGetDeviceFlags(&c->device_flags);
    (void)hipEventCreate(&c->ev0);
    (void)hipEventCreate(&c->ev1);
    c->grid = c->opts.grid_waves ? (int)((c->opts.grid_waves + kWavesPerBlock - 1) / kWavesPerBlock)
                                 : device_grid_blocks(device);
    to_device_program(nullptr, 0, &c->prog);
    bt::publish_staged_window(c);
    place_ctx(c);
    *out = c;
    return BT_OK;
}

int bt_context_device(const bt_ctx* c, int* device, char* pci_bus_id, uint32_t cap) {
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (device) *device = c->device;
    if (pci_bus_id) {
        if (cap < 16) return fail(BT_E_INVALID_ARGUMENT, "pci_bus_id buffer of %u bytes (need >= 16)", cap);
        HIP_TRY(hipDeviceGetPCIBusId(pci_bus_id, (int)cap, c->device));
    }
    return BT_OK;
}

int bt_context_placement(bt_ctx* c, bt_placement* out) {
    if (!c || !out) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    *out = bt_placement{};
    out->numa_node = c->numa_node;
    out->pinned_cpus = c->pinned ? (uint32_t)CPU_COUNT(&c->pin) : 0u;
    out->pool_threads = pool_threads_of(c);
    out->staging_node = -1;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->host_ready && c->hs[0].h_in) {   // where the kernel put the pinned staging's first page
        void* page = c->hs[0].h_in;
        int status = -1;
        if (syscall(SYS_move_pages, 0, 1UL, &page, nullptr, &status, 0) == 0 && status >= 0) out->staging_node = status;
    }
    return BT_OK;
}

int bt_node_cpus(int node, int32_t* cpus, uint32_t cap, uint32_t* n) {
    if (!n || (cap && !cpus)) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    *n = 0;
    cpu_set_t s;
    if (!bt::node_cpus(node, &s)) return BT_OK;
    for (int i = 0; i < CPU_SETSIZE; ++i)
        if (CPU_ISSET(i, &s)) {
            if (*n < cap) cpus[*n] = i;
            ++*n;
        }
    return BT_OK;
}

uint32_t bt_usable_cpus(void) { return bt::usable_cpus(); }

void bt_destroy(bt_ctx* c) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    for (const auto& r : c->host_regs)   // registrations the caller left: this context's references
        (void)bt::pin_release(reinterpret_cast<const void*>(r.first), r.second);
    c->host_regs.clear();
    free_host(c);
    c->pool.reset();
    if (c->tgraph) (void)hipGraphExecDestroy(c->tgraph);
    free_ws(c);
    for (auto& w : c->ws)
        if (w.sync) (void)hipEventDestroy(w.sync);
    for (auto e : c->main_done)
        if (e) (void)hipEventDestroy(e);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    for (int k = 0; k < 2; ++k) {
        if (c->dfa_dev[k]) (void)hipFree(c->dfa_dev[k]);
        for (auto& r : c->dfa_readers[k]) (void)hipEventDestroy(r.second);
    }
    for (auto e : c->dfa_spare) (void)hipEventDestroy(e);
    if (c->pipe_step) (void)hipEventDestroy(c->pipe_step);
    for (auto e : c->tev) (void)hipEventDestroy(e);
    if (c->pipe_done) (void)hipEventDestroy(c->pipe_done);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ex_h) (void)hipHostFree(c->ex_h);
    if (c->ex_d) (void)hipFree(c->ex_d);
    for (int k = 0; k < 2; ++k) {
        if (c->xfer_h[k]) (void)hipHostFree(c->xfer_h[k]);
        if (c->xfer_ev[k]) (void)hipEventDestroy(c->xfer_ev[k]);
    }
    if (c->xfer_after) (void)hipEventDestroy(c->xfer_after);
    for (auto& w : c->walk) {
        if (w.h) (void)hipHostFree(w.h);
        if (w.done) (void)hipEventDestroy(w.done);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int bt_filter_compile_host(const bt_filter_desc* f, uint32_t n, bt_filter_slot* out, uint32_t cap,
                           uint32_t* n_slots) {
    if ((!f && n) || !out || !n_slots) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    char err[256] = {0};
    int rc = compile_filters(f, n, out, cap, n_slots, err, sizeof(err));
    if (rc) return fail(rc, "%s", err);
    return BT_OK;
}

}  // extern "C"

namespace bt {

// The host half of bt_filter_compile: the slots, and the PAYLOAD regexes the DFA compiler
// takes turned into BT_K_PAYLOAD slots with their tables in one pool (copied into each
// block's LDS, so capped at kDfaPoolMax). No device is touched: a group compiles once and
// installs the result on every member.
int compile_program(const bt_filter_desc* f, uint32_t n, uint32_t ctx_flags, CompiledProgram* out) {
    std::vector<bt_filter_slot> slots(BT_MAX_FILTERS);
    uint32_t m = 0;
    int rc = bt_filter_compile_host(f, n, slots.data(), BT_MAX_FILTERS, &m);
    if (rc) return rc;
    slots.resize(m);
    std::vector<uint8_t> pool;
    if (!(ctx_flags & BT_OPT_PAYLOAD_HOST)) {
        for (auto& s : slots) {
            const bt_filter_desc& d = f[s.source_index];
            if (s.kind != BT_K_HOST || d.type != BT_FILTER_PAYLOAD || !d.expression) continue;
            // the compiler's preferred form (bit-parallel where it fits, else the DFA with its
            // two-byte table); when that does not fit the pool, the DFA, then the DFA without
            // the optional table
            const uint32_t base = (ctx_flags & BT_OPT_PAYLOAD_DFA) ? BT_DFA_NO_BITPAR : 0u;
            const uint32_t forms[3] = {base, BT_DFA_NO_BITPAR, BT_DFA_NO_BITPAR | BT_DFA_NO_PAIRS};
            const size_t at = (pool.size() + 15) & ~(size_t)15;
            uint32_t size = 0, fl = 0;
            bool fits = false;
            for (uint32_t k = base ? 1u : 0u; k < 3 && !fits; ++k) {
                fl = forms[k];
                fits = bt_payload_dfa_compile_ex(d.expression, fl, nullptr, 0, &size) == BT_OK && at + size <= kDfaPoolMax;
            }
            if (!fits) continue;
            pool.resize(at + size);
            if (bt_payload_dfa_compile_ex(d.expression, fl, pool.data() + at, size, &size) != BT_OK) {
                pool.resize(at);
                continue;
            }
            s.kind = BT_K_PAYLOAD;
            s.a = (uint32_t)at;
            s.b = size;
        }
    }
    out->slots = std::move(slots);
    out->dfa_pool = std::move(pool);
    return BT_OK;
}

// The device half: the DFA pool into the buffer no queued launch reads (launches on any
// stream that still read it, with the old program, are waited for first), then the slots.
int install_program(bt_ctx* c, const CompiledProgram& p) {
    std::lock_guard<std::mutex> lk(c->mu);
    if (!p.dfa_pool.empty()) {
        HIP_TRY(hipSetDevice(c->device));
        const int k = c->dfa_cur ^ 1;
        if (!c->dfa_dev[k]) HIP_TRY(hipMalloc(&c->dfa_dev[k], kDfaPoolMax));
        for (auto& r : c->dfa_readers[k]) {   // every stream's last launch that read buffer k
            HIP_TRY(hipEventSynchronize(r.second));
            c->dfa_spare.push_back(r.second);
        }
        c->dfa_readers[k].clear();
        if (int rc = bt_memcpy_h2d(c, c->dfa_dev[k], p.dfa_pool.data(), p.dfa_pool.size())) return rc;   // synchronous
        c->dfa_cur = k;
    }
    // a cached BT_OPT_GRAPH timing graph holds the old program: drop it
    if (c->tgraph) { (void)hipGraphExecDestroy(c->tgraph); c->tgraph = nullptr; }
    c->dfa_pool = p.dfa_pool;
    c->slots = p.slots;
    to_device_program(c->slots.data(), (uint32_t)c->slots.size(), &c->prog);
    publish_staged_window(c);
    return BT_OK;
}

uint32_t ctx_flags(const bt_ctx* c) { return c->opts.flags; }
int ctx_device(const bt_ctx* c) { return c->device; }

bool ctx_stream_busy(bt_ctx* c) {
    const bt::DeviceRestore keep_device;
    if (hipSetDevice(c->device) != hipSuccess) return false;
    return hipStreamQuery(c->stream) == hipErrorNotReady;
}
const cpu_set_t* ctx_pin(const bt_ctx* c) { return c->pinned ? &c->pin : nullptr; }
void ctx_forget_base(bt_ctx* c) {
    std::lock_guard<std::mutex> lk(c->mu);
    c->last_base = nullptr;
}
uint32_t stage_bytes_of(bt_ctx* c, bool records);   // defined with the host pipeline
uint32_t staged_window(const bt_ctx* c, bool records) {
    return c->staged_window[records ? 1 : 0].load(std::memory_order_acquire);
}

}  // namespace bt

extern "C" {

int bt_filter_compile(bt_ctx* c, const bt_filter_desc* f, uint32_t n) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    CompiledProgram p;
    if (int rc = compile_program(f, n, c->opts.flags, &p)) return rc;
    return install_program(c, p);
}

int bt_filter_program(const bt_ctx* c, bt_filter_slot* out, uint32_t cap, uint32_t* n_slots) {
    if (!c || !n_slots) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    *n_slots = (uint32_t)c->slots.size();
    for (uint32_t i = 0; i < c->slots.size() && i < cap && out; ++i) out[i] = c->slots[i];
    return BT_OK;
}

int bt_reserve(bt_ctx* c, uint32_t n) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    return ensure_ws(c, n);
}

int bt_parse_filter_device(bt_ctx* c, const bt_batch* b, const bt_outputs* o, void* stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    return run_device(c, b, o, st, false, nullptr, nullptr);
}


int bt_parse_filter_device_async(bt_ctx* c, const bt_batch* b, const bt_outputs* o, void* stream,
                                 void* done_event) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    std::lock_guard<std::mutex> lk(c->mu);
    if (int rc = ensure_cstream(c)) return rc;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    return run_device(c, b, o, st, false, nullptr, nullptr, c->cstream, reinterpret_cast<hipEvent_t>(done_event));
}

// The host side of a timed loop whose launches (K of them, each between the event pair
// c->tev[2i], c->tev[2i+1]) were enqueued on c->stream after c->ev0 at h0, followed by
// c->ev1: wait by polling, then fill the breakdown.
static int finish_timing(bt_ctx* c, uint32_t iters, bool no_kernel_events, std::chrono::steady_clock::time_point h0,
                         bt_timing* t, const char* who) {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    const auto h1 = clk::now();
    // Poll instead of hipEventSynchronize: a blocking wait is woken by an interrupt, whose
    // latency would sit inside the caller's timed region.
    auto poll = [](hipEvent_t e) -> hipError_t {
        for (;;) {
            const hipError_t q = hipEventQuery(e);
            if (q != hipErrorNotReady) return q;
        }
    };
    HIP_TRY(poll(c->ev0));
    const auto h2 = clk::now();
    HIP_TRY(poll(c->ev1));
    const auto h3 = clk::now();
    float tot = 0, k = 0, kmin = 1e30f, kmax = 0, lead = 0, gap = 0;
    HIP_TRY(hipEventElapsedTime(&tot, c->ev0, c->ev1));
    for (uint32_t i = 0; !no_kernel_events && i < iters; ++i) {
        float x = 0;
        HIP_TRY(hipEventElapsedTime(&x, c->tev[2 * i], c->tev[2 * i + 1]));
        k += x;
        kmin = std::min(kmin, x);
        kmax = std::max(kmax, x);
        if (i + 1 < iters) {
            float g = 0;
            HIP_TRY(hipEventElapsedTime(&g, c->tev[2 * i + 1], c->tev[2 * i + 2]));
            gap += g;
        }
    }
    if (!no_kernel_events) HIP_TRY(hipEventElapsedTime(&lead, c->ev0, c->tev[0]));
    const auto h4 = clk::now();
    if (t) {
        *t = bt_timing{};
        t->span_ms = tot;
        t->main_ms = no_kernel_events ? -1.0f : k / iters;
        t->main_min_ms = no_kernel_events ? -1.0f : kmin;
        t->main_max_ms = no_kernel_events ? -1.0f : kmax;
        t->lead_ms = lead;
        t->gap_ms = gap;
        t->enqueue_ms = ms(h0, h1);
        t->first_seen_ms = ms(h1, h2);
        t->last_seen_ms = ms(h2, h3);
        t->query_ms = ms(h3, h4);
        t->wall_ms = ms(h0, h4);
        t->spin_rc = c->spin_rc;
        t->device_flags = c->device_flags;
    }
    static const bool dbg = getenv("BT_DEBUG_TIMING") != nullptr;
    if (dbg)
        fprintf(stderr, "[%s] enqueue %.3f ms, first-seen %.3f ms, last-seen %.3f ms, queries %.3f ms, "
                "gpu span %.3f ms\n", who, ms(h0, h1), ms(h1, h2), ms(h2, h3), ms(h3, h4), tot);
    return BT_OK;
}

static int ensure_timing_events(bt_ctx* c, uint32_t iters) {
    while (c->tev.size() < 2 * (size_t)iters) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->tev.push_back(e);
    }
    return BT_OK;
}

int bt_time_device2(bt_ctx* c, const bt_batch* b, const bt_outputs* outs, uint32_t n_out, uint32_t iters,
                    uint32_t mode, bt_timing* t) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !b || !outs || !n_out || !iters) return fail(BT_E_INVALID_ARGUMENT, "null argument / zero iterations");
    if (mode & ~(uint32_t)(BT_TIME_KERNEL_EVENTS | BT_TIME_PIPELINED)) return fail(BT_E_INVALID_ARGUMENT, "unknown mode");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    const bool kev = (mode & BT_TIME_KERNEL_EVENTS) != 0;
    const bool piped = (mode & BT_TIME_PIPELINED) != 0;
    if (kev) { if (int rc = ensure_timing_events(c, iters)) return rc; }
    // BT_OPT_GRAPH: the K steps replay as one hipGraph (no per-kernel events: HIP cannot
    // time events recorded inside a captured graph), main_ms is then reported as -1.
    const bool use_graph = (c->opts.flags & BT_OPT_GRAPH) != 0 && !piped;
    const bt_outputs* o = outs;
    const bool cached = c->tgraph && c->tg_iters == iters && !std::memcmp(&c->tg_batch, b, sizeof(*b)) &&
                        !std::memcmp(&c->tg_out, o, sizeof(*o));
    if (use_graph && !cached) {
        // Build once (the first call is the caller's untimed warm-up): the main kernel +
        // the compaction kernels, K times, in one graph.
        if (c->tgraph) { (void)hipGraphExecDestroy(c->tgraph); c->tgraph = nullptr; }
        if (o->pass_idx || o->n_pass) { int rc = ensure_ws(c, b->n); if (rc) return rc; }
        hipGraph_t g = nullptr;
        HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
        int rc = BT_OK;
        for (uint32_t i = 0; rc == BT_OK && i < iters; ++i) rc = run_device(c, b, o, c->stream, false, nullptr, nullptr);
        hipError_t ee = hipStreamEndCapture(c->stream, &g);
        if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
        if (ee != hipSuccess || !g) return fail(BT_E_INTERNAL, "graph capture failed: %s", hipGetErrorString(ee));
        hipError_t e = hipGraphInstantiate(&c->tgraph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) { c->tgraph = nullptr; return fail(BT_E_INTERNAL, "hipGraphInstantiate: %s", hipGetErrorString(e)); }
        c->tg_batch = *b;
        c->tg_out = *o;
        c->tg_iters = iters;
    }
    if (piped) {
        if (int rc = ensure_cstream(c)) return rc;
        if (!c->pipe_done) HIP_TRY(hipEventCreateWithFlags(&c->pipe_done, hipEventDisableTiming));
        if (!c->pipe_step) HIP_TRY(hipEventCreateWithFlags(&c->pipe_step, hipEventDisableTiming));
    }
    const auto h0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    if (use_graph) {
        HIP_TRY(hipGraphLaunch(c->tgraph, c->stream));
    } else {
        // Step i uses output set i % n_out. Pipelined (bt_parse_filter_device_async per
        // step): each compaction runs beside the next step's main kernel and the last one
        // joins c->stream before the closing event. The per-kernel event pairs
        // (BT_TIME_KERNEL_EVENTS) are recorded by the main kernel's own dispatch; they cost
        // the GPU ~9 us per launch on gfx950 (tools/calib/boundary.hip), so the bench
        // times its steps without them and measures the kernel in a second pass.
        // With one output set, step i + 1's main kernel would rewrite the verdict words
        // step i's compaction reads: it waits for that compaction (no overlap, no race).
        const bool serial = piped && n_out == 1;
        for (uint32_t i = 0; i < iters; ++i) {
            const bt_outputs* oi = outs + (i % n_out);
            hipEvent_t e0 = kev ? c->tev[2 * i] : nullptr, e1 = kev ? c->tev[2 * i + 1] : nullptr;
            if (serial && i) HIP_TRY(hipStreamWaitEvent(c->stream, c->pipe_step, 0));
            int rc = piped ? run_device(c, b, oi, c->stream, false, e0, e1, c->cstream,
                                        i + 1 == iters ? c->pipe_done : serial ? c->pipe_step : nullptr)
                           : run_device(c, b, oi, c->stream, false, e0, e1);
            if (rc) return rc;
        }
        if (piped) HIP_TRY(hipStreamWaitEvent(c->stream, c->pipe_done, 0));
    }
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    return finish_timing(c, iters, use_graph || !kev, h0, t, "bt_time_device");
}

int bt_time_device_ex(bt_ctx* c, const bt_batch* b, const bt_outputs* o, uint32_t iters, bt_timing* t) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    const uint32_t mode = BT_TIME_KERNEL_EVENTS | ((c && (c->opts.flags & BT_OPT_PIPELINE)) ? BT_TIME_PIPELINED : 0u);
    return bt_time_device2(c, b, o, 1, iters, mode, t);
}

int bt_time_device(bt_ctx* c, const bt_batch* b, const bt_outputs* o, uint32_t iters, float* ms_per_iter,
                   float* main_ms) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    bt_timing t{};
    const int rc = bt_time_device_ex(c, b, o, iters, &t);
    if (rc) return rc;
    if (ms_per_iter) *ms_per_iter = t.span_ms / iters;
    if (main_ms) *main_ms = t.main_ms;
    return BT_OK;
}

}  // extern "C"

namespace {

// Bytes of each frame the host pipeline reads (bt_host_stage_bytes): the walk's 112 with
// records; the filters' 38 B (as 48; bytes 12..43 of them staged) for filter-only calls, whose
// kernels take no second round (staging the walk's 112 B took 2-3x the gather and the copy for IMIX frames); the
// payload window with a GPU PAYLOAD slot (bytes past the staged prefix would be the next
// frame's).
uint32_t stage_bytes(const bt_ctx* c, bool records) {
    return !c->dfa_pool.empty() ? kHostSlotPayload : records ? kHostSlot : kHostSlotFilter;
}

}  // namespace

namespace bt {
uint32_t stage_bytes_of(bt_ctx* c, bool records) {
    std::lock_guard<std::mutex> lk(c->mu);
    return stage_bytes(c, records);
}
uint32_t staged_bytes_locked(const bt_ctx* c, bool records) {
    const uint32_t w = stage_bytes(c, records);
    return w == kHostSlotFilter && !(c->opts.flags & BT_OPT_NO_LEAN_HOST) ? kHostLeanWidth : w;
}
uint32_t staged_bytes_of(bt_ctx* c, bool records) {
    std::lock_guard<std::mutex> lk(c->mu);
    return staged_bytes_locked(c, records);
}
void publish_staged_window(bt_ctx* c) {   // under c->mu, after the program changed
    for (int r = 0; r < 2; ++r) c->staged_window[r].store(staged_bytes_locked(c, r != 0), std::memory_order_release);
}
}  // namespace bt

namespace {

// Host batch pipeline shared by bt_parse_filter (base + descriptors) and
// bt_parse_filter_ptrs (one pointer per frame): frame(i, &len) returns frame i.
template <class FrameFn>
int host_pipeline_run(bt_ctx* c, uint32_t n, FrameFn frame, bt_rec* records, uint64_t* verdict, uint8_t* decide,
                  uint32_t* pass_idx, uint32_t* n_pass) {
    int rc = ensure_host(c);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));   // the calling thread may last have driven another device
    const bool want_filter = verdict || decide || pass_idx || n_pass;
    // pass indices come from the verdict words; keep a private copy when the caller
    // did not ask for them
    std::vector<uint64_t> vtmp;
    uint64_t* ver = verdict;
    if (!ver && (pass_idx || n_pass)) { vtmp.resize(((size_t)n + 63) / 64); ver = vtmp.data(); }

    const uint32_t chunk = c->chunk;
    // Records inside a range registered with bt_host_register are copied D2H in place, each
    // chunk at its offset, and skip the drain (96 B of staging-to-caller copy per packet, most
    // of the host's memory traffic with records: e2e records + verdicts C2 / C3 / C4 +1..17 /
    // +17..22 / +8..15 %, profiles/r05/e2e/ab_registered_outputs.jsonl). Decisions and verdict
    // words keep the staging (the same A/B moved them in place: C2 -3..+32 %, C3 -8..-28 %, C4
    // -4..-7 %).
    auto registered = [c](const void* p, size_t bytes) {
        const uintptr_t a = (uintptr_t)p;
        for (const auto& r : c->host_regs)
            if (a >= r.first && a + bytes <= r.first + r.second) return true;
        return false;
    };
    const bool rec_direct = records && registered(records, (size_t)n * BT_REC_BYTES);
    bt_rec* const rec_drain = rec_direct ? nullptr : records;
    // bytes staged per frame: the header walk's, or with a GPU PAYLOAD slot in the program
    // the payload window's too (bytes past the staged prefix would be the next frame's)
    const uint32_t slot = stage_bytes(c, records != nullptr);
    // Filter-only calls (no records, no GPU PAYLOAD slot) stage only frame bytes [12, 44): the
    // filters read 12..37 and such calls take no second round. Each frame's descriptor then
    // points 12 B before its staged bytes (the buffer starts with a 16-B pad, so no offset is
    // negative); bytes 0..11 of that window are the previous slot's, which nothing reads.
    const bool lean = slot == kHostSlotFilter && !(c->opts.flags & BT_OPT_NO_LEAN_HOST);
    const uint32_t lo = lean ? kLeanLo : 0u;
    const uint32_t width = lean ? kHostLeanWidth : slot;
    const uint32_t pad = lean ? 16u : 0u;
    static const bool prefetch = getenv("BT_NO_GATHER_PREFETCH") == nullptr;   // A/B knobs
    // non-temporal staging stores (BT_GATHER_NT=0: plain copies). Same-box A/B, 5 pairs over
    // two boxes (profiles/r04/e2e/ab_gather_nt*.jsonl): C2 verdicts +2..+34 % in every pair,
    // C4 +8 % on average, C3 level
    static const bool nt = [] {
        const char* e = getenv("BT_GATHER_NT");
        return !e || atoi(e) != 0;
    }();
    static const uint32_t kGatherAhead = [] {
        const char* e = getenv("BT_GATHER_AHEAD");
        return e && atoi(e) > 0 ? (uint32_t)atoi(e) : kGatherAheadDefault;
    }();
    uint32_t next = 0, k = 0;
    while (next < n || c->hs[0].busy || c->hs[1].busy) {
        HostSlot& s = c->hs[k & 1];
        if (s.busy) {   // retire the chunk that used this half
            HIP_TRY(hipEventSynchronize(s.done));
            if (rec_drain || decide || ver) drain_slot(c, s, rec_drain, ver, decide);
            else s.busy = false;
        }
        if (next < n) {
            const uint32_t cnt = std::min(chunk, n - next);
            // gather the header prefixes (<= slot bytes) into pinned staging:
            // per-worker byte counts, exclusive scan, then parallel copies (lean: every frame
            // one 32-B slot, so worker w starts at pad + 32 * its first frame and the counting
            // pass is skipped)
            uint8_t* pre = s.h_in;
            uint64_t* d = reinterpret_cast<uint64_t*>(s.h_in + (size_t)chunk * kHostSlotPayload);
            const unsigned T = pipeline_share(c);
            std::vector<uint64_t> part(T + 1, 0);
            const uint32_t base_i = next;
            if (lean) {
                for (unsigned w = 0; w <= T; ++w) part[w] = pad + (uint64_t)width * (uint32_t)((uint64_t)cnt * w / T);
            } else pipeline_run(c, cnt, T, [&](unsigned w) {
                const uint32_t a = (uint32_t)((uint64_t)cnt * w / T), b = (uint32_t)((uint64_t)cnt * (w + 1) / T);
                uint64_t sum = 0;
                for (uint32_t i = a; i < b; ++i) {
                    uint32_t len = 0;
                    (void)frame(base_i + i, &len);
                    sum += (std::min(len > lo ? len - lo : 0u, width) + 15) & ~15u;
                }
                part[w + 1] = sum;
            });
            if (!lean)
                for (unsigned w = 0; w < T; ++w) part[w + 1] += part[w];
            pipeline_run(c, cnt, T, [&](unsigned w) {
                const uint32_t a = (uint32_t)((uint64_t)cnt * w / T), b = (uint32_t)((uint64_t)cnt * (w + 1) / T);
                uint64_t p = part[w];
                for (uint32_t i = a; i < b; ++i) {
                    if (prefetch && i + kGatherAhead < b) {   // frames far apart: start the miss early
                        uint32_t l2 = 0;
                        const uint8_t* g = frame(base_i + i + kGatherAhead, &l2) + lo;
                        __builtin_prefetch(g);
                        if (((uintptr_t)g & 63u) + std::min(l2 > lo ? l2 - lo : 0u, width) > 64u) __builtin_prefetch(g + 64);
                    }
                    uint32_t len = 0;
                    const uint8_t* f = frame(base_i + i, &len);
                    const uint32_t m = std::min(len > lo ? len - lo : 0u, width);
                    if (m) stage_prefix(pre + p, f + lo, m, nt);
                    d[i] = BT_DESC(p - lo, len);
                    p += lean ? width : (m + 15) & ~15u;
                }
                if (nt) __builtin_ia32_sfence();   // the prefixes are visible before the H2D copy
            });
            const uint64_t pos = part[T];
            const size_t pre_bytes = (pos + 15) & ~15ull;
            if (pre_bytes) HIP_TRY(hipMemcpyAsync(s.d_in, pre, pre_bytes, hipMemcpyHostToDevice, s.stream));
            HIP_TRY(hipMemcpyAsync(s.d_in + (size_t)chunk * kHostSlotPayload, d, (size_t)cnt * 8, hipMemcpyHostToDevice,
                                   s.stream));
            bt_batch b{};
            b.base = s.d_in;
            b.desc = reinterpret_cast<const uint64_t*>(s.d_in + (size_t)chunk * kHostSlotPayload);
            b.n = cnt;
            b.bytes = (uint64_t)chunk * kHostSlotPayload;
            bt_outputs o{};
            uint8_t* drec = s.d_out;
            uint8_t* ddec = s.d_out + (size_t)chunk * BT_REC_BYTES;
            uint64_t* dver = reinterpret_cast<uint64_t*>(ddec + chunk);
            o.records = records ? drec : nullptr;
            o.n_cap = chunk;
            o.decide = want_filter ? ddec : nullptr;
            o.verdict = want_filter ? dver : nullptr;
            rc = run_device(c, &b, &o, s.stream, true, nullptr, nullptr);
            if (rc) return rc;
            if (records)
                HIP_TRY(hipMemcpyAsync(rec_direct ? static_cast<void*>(records + next) : s.h_out, drec,
                                       (size_t)cnt * BT_REC_BYTES, hipMemcpyDeviceToHost, s.stream));
            if (want_filter) {
                if (decide)   // (nothing on the host reads the staged decisions otherwise)
                    HIP_TRY(hipMemcpyAsync(s.h_out + (size_t)chunk * BT_REC_BYTES, ddec, cnt, hipMemcpyDeviceToHost,
                                           s.stream));
                HIP_TRY(hipMemcpyAsync(s.h_out + (size_t)chunk * BT_REC_BYTES + chunk, dver,
                                       ((size_t)cnt + 63) / 64 * 8, hipMemcpyDeviceToHost, s.stream));
            }
            HIP_TRY(hipEventRecord(s.done, s.stream));
            s.busy = true;
            s.lo = next;
            s.cnt = cnt;
            next += cnt;
        }
        ++k;
    }
    if (ver && (pass_idx || n_pass)) {
        uint32_t np = 0;
        for (uint32_t w = 0; w < (n + 63) / 64; ++w) {
            uint64_t x = ver[w];
            if (w == (n - 1) / 64 && (n & 63)) x &= (1ull << (n & 63)) - 1ull;
            while (x) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(x);
                if (pass_idx) pass_idx[np] = w * 64 + bit;
                ++np;
                x &= x - 1;
            }
        }
        if (n_pass) *n_pass = np;
    }
    return BT_OK;
}

template <class FrameFn>
int host_pipeline(bt_ctx* c, uint32_t n, FrameFn frame, bt_rec* records, uint64_t* verdict, uint8_t* decide,
                  uint32_t* pass_idx, uint32_t* n_pass) {
    const int rc = host_pipeline_run(c, n, frame, records, verdict, decide, pass_idx, n_pass);
    if (rc) {   // retire chunks still in flight, so none is drained into a later call's buffers
        for (auto& s : c->hs) {
            if (s.busy) (void)hipEventSynchronize(s.done);
            s.busy = false;
        }
    }
    return rc;
}

}  // namespace

extern "C" {

int bt_parse_filter(bt_ctx* c, const uint8_t* base, const bt_pkt_desc* desc, uint32_t n, bt_rec* records,
                    uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (n && (!base || !desc)) return fail(BT_E_INVALID_ARGUMENT, "null packet buffer/descriptors");
    const WaitFor lk(c);
    return host_pipeline(
        c, n,
        [&](uint32_t i, uint32_t* len) {
            *len = BT_DESC_LEN(desc[i]);
            return base + BT_DESC_OFF(desc[i]);
        },
        records, verdict, decide, pass_idx, n_pass);
}

int bt_parse_filter_ptrs(bt_ctx* c, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                         bt_rec* records, uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (n && (!frames || !lens)) return fail(BT_E_INVALID_ARGUMENT, "null frame pointers/lengths");
    for (uint32_t i = 0; i < n; ++i)
        if (lens[i] > 0xFFFFu) return fail(BT_E_INVALID_ARGUMENT, "frame %u longer than 65535 bytes", i);
    const WaitFor lk(c);
    return host_pipeline(
        c, n,
        [&](uint32_t i, uint32_t* len) {
            *len = lens[i];
            return frames[i];
        },
        records, verdict, decide, pass_idx, n_pass);
}

int bt_host_stage_bytes(const bt_ctx* c, int with_records, uint32_t* bytes) {
    if (!c || !bytes) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> lk(const_cast<bt_ctx*>(c)->mu);
    *bytes = stage_bytes(c, with_records != 0);
    return BT_OK;
}

int bt_host_register(bt_ctx* c, void* host, uint64_t bytes, void** dev_alias) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !host || !dev_alias || !bytes) return fail(BT_E_INVALID_ARGUMENT, "null argument / empty range");
    {
        std::lock_guard<std::mutex> lk(c->mu);
        for (const auto& r : c->host_regs)
            if (r.first == (uintptr_t)host)
                return fail(BT_E_INVALID_ARGUMENT, "%p is already registered on this context", host);
    }
    // whole pages, in the process's one table (bt_pin.h): a range inside pages another
    // registration holds shares them, one that holds only some of them is refused
    uint8_t* alias = nullptr;
    if (int rc = bt::pin_acquire(host, bytes, &c->device, 1, &alias)) return rc;
    *dev_alias = alias;
    std::lock_guard<std::mutex> lk(c->mu);
    c->host_regs.emplace_back((uintptr_t)host, bytes);
    return BT_OK;
}

int bt_host_unregister(bt_ctx* c, void* host) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !host) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    uint64_t bytes = 0;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        for (const auto& r : c->host_regs)
            if (r.first == (uintptr_t)host) bytes = r.second;
    }
    if (!bytes) return fail(BT_E_INVALID_ARGUMENT, "%p is not registered on this context", host);
    // the last reference waits for every device that holds an alias of the pages (queued
    // kernels that read or write them) before they are unregistered
    if (int rc = bt::pin_release(host, bytes)) return rc;
    std::lock_guard<std::mutex> lk(c->mu);   // host_resident's cache (read under mu): the
    c->last_base = nullptr;                   // address may come back as another kind
    auto& r = c->host_regs;
    r.erase(std::remove_if(r.begin(), r.end(), [host](const auto& x) { return x.first == (uintptr_t)host; }), r.end());
    return BT_OK;
}

int bt_dev_malloc(bt_ctx* c, uint64_t bytes, void** out) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !out) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    static const unsigned flags = [] {
        const char* e = getenv("BT_MALLOC_FLAGS");   // experiments: 4 = hipDeviceMallocContiguous
        return e ? (unsigned)strtoul(e, nullptr, 0) : 0u;
    }();
    if (flags) HIP_TRY(hipExtMallocWithFlags(out, bytes ? bytes : 16, flags));
    else HIP_TRY(hipMalloc(out, bytes ? bytes : 16));
    return BT_OK;
}

int bt_dev_free(bt_ctx* c, void* p) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (!p) return BT_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipFree(p));   // implicitly waits for the device: no queued kernel still uses p
    std::lock_guard<std::mutex> lk(c->mu);
    c->last_base = nullptr;   // host_resident's cache (as bt_host_unregister)
    return BT_OK;
}

}  // extern "C"

namespace {

constexpr size_t kXferChunk = size_t(8) << 20;

// The copies run on the context stream; work queued on the compaction stream
// (bt_parse_filter_device_async) is waited for first, so a copy issued after an async call
// sees its pass list. Work on a caller's own stream is the caller's to synchronise.
int after_cstream(bt_ctx* c) {
    if (!c->cstream) return BT_OK;
    if (!c->xfer_after) HIP_TRY(hipEventCreateWithFlags(&c->xfer_after, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->xfer_after, c->cstream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->xfer_after, 0));
    return BT_OK;
}

int ensure_xfer(bt_ctx* c) {
    for (int k = 0; k < 2; ++k) {
        if (!c->xfer_h[k]) HIP_TRY(hipHostMalloc(&c->xfer_h[k], kXferChunk, hipHostMallocDefault));
        if (!c->xfer_ev[k]) HIP_TRY(hipEventCreateWithFlags(&c->xfer_ev[k], hipEventDisableTiming));
    }
    return BT_OK;
}

}  // namespace

extern "C" {

// Both copies go through the context's two pinned chunks (host memcpy of chunk k while the
// DMA of chunk k^1 runs), so no DMA touches the caller's (usually pageable) memory; they
// are ordered after the context's streams (after_cstream) and complete before returning.
int bt_memcpy_h2d(bt_ctx* c, void* dst, const void* src, uint64_t bytes) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (bytes && (!dst || !src)) return fail(BT_E_INVALID_ARGUMENT, "null pointer");
    std::lock_guard<std::mutex> lk(c->xfer_mu);
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = ensure_xfer(c)) return rc;
    if (int rc = after_cstream(c)) return rc;
    bool used[2] = {false, false};
    int k = 0;
    for (uint64_t off = 0; off < bytes; off += kXferChunk, k ^= 1) {
        const size_t n = (size_t)std::min<uint64_t>(kXferChunk, bytes - off);
        if (used[k]) HIP_TRY(hipEventSynchronize(c->xfer_ev[k]));   // its last DMA has read it
        std::memcpy(c->xfer_h[k], static_cast<const uint8_t*>(src) + off, n);
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, c->xfer_h[k], n, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->xfer_ev[k], c->stream));
        used[k] = true;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BT_OK;
}

int bt_memcpy_d2h(bt_ctx* c, void* dst, const void* src, uint64_t bytes) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (bytes && (!dst || !src)) return fail(BT_E_INVALID_ARGUMENT, "null pointer");
    std::lock_guard<std::mutex> lk(c->xfer_mu);
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = ensure_xfer(c)) return rc;
    if (int rc = after_cstream(c)) return rc;
    // chunk i lands in buffer i & 1; chunk i + 1's DMA runs while chunk i is copied out
    auto issue = [&](uint64_t off, int k) -> int {
        const size_t n = (size_t)std::min<uint64_t>(kXferChunk, bytes - off);
        HIP_TRY(hipMemcpyAsync(c->xfer_h[k], static_cast<const uint8_t*>(src) + off, n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipEventRecord(c->xfer_ev[k], c->stream));
        return BT_OK;
    };
    if (bytes) { if (int rc = issue(0, 0)) return rc; }
    int k = 0;
    for (uint64_t off = 0; off < bytes; off += kXferChunk, k ^= 1) {
        if (off + kXferChunk < bytes) { if (int rc = issue(off + kXferChunk, k ^ 1)) return rc; }
        HIP_TRY(hipEventSynchronize(c->xfer_ev[k]));
        std::memcpy(static_cast<uint8_t*>(dst) + off, c->xfer_h[k], (size_t)std::min<uint64_t>(kXferChunk, bytes - off));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BT_OK;
}

int bt_memset_d(bt_ctx* c, void* dst, int value, uint64_t bytes) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = after_cstream(c)) return rc;
    HIP_TRY(hipMemsetAsync(dst, value, bytes, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BT_OK;
}

int bt_ring_walk_tpv3_gpu(bt_ctx* c, const bt_tpv3_ring* ring, const void* ring_dev, uint32_t first_block,
                          uint32_t max_blocks, bt_pkt_desc* desc_dev, uint32_t cap, uint32_t* n_desc,
                          uint32_t* n_blocks_taken, uint32_t* bad_dev, void* stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !ring || !ring->base || !ring_dev || !n_desc || !n_blocks_taken || (cap && !desc_dev))
        return fail(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3_gpu: null argument");
    if (!ring->n_blocks || ring->block_size < 48 || first_block >= ring->n_blocks)
        return fail(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3_gpu: bad ring geometry");
    *n_desc = 0;
    *n_blocks_taken = 0;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    auto& w = c->walk[c->walk_next];
    const uint32_t lim = std::min(max_blocks, ring->n_blocks);
    if (w.used) HIP_TRY(hipEventSynchronize(w.done));   // the walk that last read this buffer has run
    if (w.cap < lim) {
        if (w.h) HIP_TRY(hipHostFree(w.h));
        w.h = nullptr;
        HIP_TRY(hipHostMalloc(&w.h, sizeof(RingBlock) * std::max(lim, 64u), hipHostMallocDefault));
        w.cap = std::max(lim, 64u);
    }
    if (!w.done) HIP_TRY(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    // the ready blocks and where each one's descriptors go (bt_ring.cpp's first phase)
    uint64_t total = 0;
    uint32_t nb = 0;
    for (uint32_t k = 0; k < lim; ++k) {
        const uint32_t b = (first_block + k) % ring->n_blocks;
        const uint8_t* bd = static_cast<const uint8_t*>(ring->base) + (uint64_t)b * ring->block_size;
        // tpacket_block_desc: version, offset_to_priv, then bh1 { block_status, num_pkts,
        // offset_to_first_pkt, ... } (linux/if_packet.h)
        const uint32_t status = __atomic_load_n(reinterpret_cast<const uint32_t*>(bd + 8), __ATOMIC_ACQUIRE);
        if (!(status & 1u)) break;   // TP_STATUS_USER
        const uint32_t np = *reinterpret_cast<const uint32_t*>(bd + 12);
        const uint32_t first = *reinterpret_cast<const uint32_t*>(bd + 16);
        if (total + np > cap) break;
        if (np && first >= ring->block_size)
            return fail(BT_E_INVALID_ARGUMENT, "bt_ring_walk_tpv3_gpu: block %u: first frame outside block", b);
        w.h[nb++] = RingBlock{b, np, (uint32_t)total, first};
        total += np;
    }
    RingWalkArgs a{};
    a.ring = static_cast<const uint8_t*>(ring_dev);
    a.block_size = ring->block_size;
    a.blocks = w.h;
    a.count = nb;
    a.desc = desc_dev;
    a.cap = cap;
    a.bad = bad_dev;
    if (int rc = launch_ring_walk(a, st)) return fail(rc, "ring walk launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(w.done, st));
    w.used = true;
    c->walk_next ^= 1;
    *n_desc = (uint32_t)total;
    *n_blocks_taken = nb;
#ifdef BT_DEBUG_BOUNDS
    BoundsLog f{};
    if (const uint32_t k = bounds_take_ring(st, &f))
        return fail(BT_E_INTERNAL, "BT_DEBUG_BOUNDS: ring walk: %u failed checks, first %s index %llu limit %llu", k,
                    bounds_site_name(f.site), (unsigned long long)f.index, (unsigned long long)f.limit);
#endif
    return BT_OK;
}

int bt_host_parallel(bt_ctx* c, void (*fn)(void*, uint32_t, uint32_t), void* user) {
    if (!c || !fn) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    bt::host_parallel(c, [&](unsigned w, unsigned T) { fn(user, w, T); });
    return BT_OK;
}

int bt_stream_create(bt_ctx* c, void** stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !stream) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return BT_OK;
}

int bt_stream_synchronize(bt_ctx* c, void* stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !stream) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return BT_OK;
}

int bt_stream_destroy(bt_ctx* c, void* stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !stream) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
    return BT_OK;
}

int bt_synchronize(bt_ctx* c) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->cstream) HIP_TRY(hipStreamSynchronize(c->cstream));
    return BT_OK;
}

}  // extern "C"

namespace {

// A bt_field_def table as the kernel takes it (ExTable), with the span and the checks the
// C-ABI promises. span > 65535 can never parse a frame (lengths are 16-bit): *never = true.
int build_table(const bt_field_def* f, uint32_t n, ExTable* t, uint64_t* span_out, bool* never) {
    if (n && !f) return fail(BT_E_INVALID_ARGUMENT, "null field table");
    if (n > BT_FIELD_MAX) return fail(BT_E_INVALID_ARGUMENT, "%u fields (max %u)", n, BT_FIELD_MAX);
    // getTotalLength (src/parser/FieldDefinition.cpp:31-46): the end of the field that ends
    // last (offset + length in size_t arithmetic)
    uint64_t mo = 0, ml = 0;
    for (uint32_t k = 0; k < n; ++k) {
        if (f[k].type > BT_FT_CUSTOM) return fail(BT_E_INVALID_ARGUMENT, "field %u: unknown type %u", k, f[k].type);
        if (f[k].type == BT_FT_BOOLEAN && f[k].length == 0)
            return fail(BT_E_INVALID_ARGUMENT, "field %u: BOOLEAN of length 0 (the reference reads fieldData[0] "
                        "of an empty vector)", k);
        if (f[k].offset + f[k].length < f[k].offset)
            return fail(BT_E_INVALID_ARGUMENT, "field %u: offset + length overflows", k);
        if (f[k].offset + f[k].length > mo + ml) { mo = f[k].offset; ml = f[k].length; }
    }
    const uint64_t span = n ? mo + ml : 0;
    if (span_out) *span_out = span;
    *never = span > 0xFFFFu;
    std::memset(t, 0, sizeof(*t));
    t->n = n;
    t->span = *never ? 0u : (uint32_t)span;
    t->window = std::min<uint32_t>(t->span, kExWindow);
    for (uint32_t k = 0; k < n && !*never; ++k) {
        t->f[k].offset = (uint32_t)f[k].offset;
        t->f[k].length = (uint32_t)f[k].length;
        t->f[k].ctl = f[k].type | ((f[k].endianness & 0xFFu) << 8);
    }
    return BT_OK;
}

int run_extract(bt_ctx* c, const bt_batch* b, const ExTable& t, bool never, const bt_extract_out* o, hipStream_t st,
                hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
    if (!b || !o) return fail(BT_E_INVALID_ARGUMENT, "null batch/outputs");
    if (b->n && !b->base) return fail(BT_E_INVALID_ARGUMENT, "null packet buffer");
    if (!b->desc && b->stride == 0 && b->n) return fail(BT_E_INVALID_ARGUMENT, "fixed-stride mode needs stride > 0");
    if (o->values && o->n_cap < b->n) return fail(BT_E_INVALID_ARGUMENT, "values n_cap %u < n %u", o->n_cap, b->n);
    if (b->desc_format > BT_DESC_XDP) return fail(BT_E_INVALID_ARGUMENT, "unknown desc_format %u", b->desc_format);
    if (b->flags & BT_BATCH_LEAN)
        return fail(BT_E_INVALID_ARGUMENT, "a BT_BATCH_LEAN batch holds frame bytes 12..43 only: no user-table extraction");
    if (!b->n) return BT_OK;
    uint64_t bytes = b->bytes;   // as run_device: mandatory with descriptors
    if (b->desc) {
        if (!bytes) return fail(BT_E_INVALID_ARGUMENT, "descriptor batch with bytes == 0 (the readable size of base)");
    } else {
        const uint64_t need = (uint64_t)b->n * b->stride;
        if (!bytes) bytes = need;
        else if (bytes < need) return fail(BT_E_INVALID_ARGUMENT, "fixed-stride batch: bytes %llu < n * stride %llu",
                                           (unsigned long long)bytes, (unsigned long long)need);
    }
    if (never) {   // no frame reaches the span: every packet PACKET_TOO_SHORT, no field
        if (o->status) HIP_TRY(hipMemsetAsync(o->status, 9, b->n, st));
        if (o->values) for (uint32_t k = 0; k < t.n; ++k)
            HIP_TRY(hipMemsetAsync(o->values + (size_t)k * o->n_cap, 0, (size_t)b->n * 8, st));
        return BT_OK;
    }
    ExArgs a{};
    a.base = b->base;
    a.desc = static_cast<const uint64_t*>(b->desc);
    a.desc_words = b->desc_format == BT_DESC_XDP ? 2u : 1u;
    a.bytes = read_limit(b->base, bytes);
    a.stride = b->stride;
    a.n = b->n;
    a.ntiles = (b->n + 63) / 64;
    a.status = o->status;
    a.values = o->values;
    a.image = o->image;
    a.n_cap = o->n_cap;
    const int rc = launch_extract(a, t, st, e0, e1);
    if (rc) return fail(rc, "extract kernel launch failed: %s", hipGetErrorString(hipGetLastError()));
    return check_bounds(st, nullptr, "extract");
}

}  // namespace

extern "C" {

int bt_proto_span(const bt_field_def* fields, uint32_t n_fields, uint64_t* span) {
    if (!span) return fail(BT_E_INVALID_ARGUMENT, "null span");
    ExTable t;
    bool never = false;
    return build_table(fields, n_fields, &t, span, &never);
}

int bt_extract_device(bt_ctx* c, const bt_batch* b, const bt_field_def* fields, uint32_t n_fields,
                      const bt_extract_out* out, void* stream) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    ExTable t;
    bool never = false;
    int rc = build_table(fields, n_fields, &t, nullptr, &never);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    return run_extract(c, b, t, never, out, stream ? reinterpret_cast<hipStream_t>(stream) : c->stream);
}

int bt_time_extract2(bt_ctx* c, const bt_batch* b, const bt_field_def* fields, uint32_t n_fields,
                     const bt_extract_out* out, uint32_t iters, uint32_t mode, bt_timing* t) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c || !b || !out || !iters) return fail(BT_E_INVALID_ARGUMENT, "null argument / zero iterations");
    if (mode & ~(uint32_t)BT_TIME_KERNEL_EVENTS) return fail(BT_E_INVALID_ARGUMENT, "unknown mode");
    const bool kev = (mode & BT_TIME_KERNEL_EVENTS) != 0;
    ExTable tab;
    bool never = false;
    int rc = build_table(fields, n_fields, &tab, nullptr, &never);
    if (rc) return rc;
    if (never || !b->n) return fail(BT_E_INVALID_ARGUMENT, "nothing to time: empty batch or a span no frame reaches");
    std::lock_guard<std::mutex> lk(c->mu);
    HIP_TRY(hipSetDevice(c->device));
    if (kev && (rc = ensure_timing_events(c, iters))) return rc;
    const auto h0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    for (uint32_t i = 0; i < iters; ++i)
        if ((rc = run_extract(c, b, tab, never, out, c->stream, kev ? c->tev[2 * i] : nullptr,
                              kev ? c->tev[2 * i + 1] : nullptr)))
            return rc;
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    return finish_timing(c, iters, !kev, h0, t, "bt_time_extract");
}

int bt_time_extract_ex(bt_ctx* c, const bt_batch* b, const bt_field_def* fields, uint32_t n_fields,
                       const bt_extract_out* out, uint32_t iters, bt_timing* t) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    return bt_time_extract2(c, b, fields, n_fields, out, iters, BT_TIME_KERNEL_EVENTS, t);
}

// extractValue<T> (src/parser/ProtocolParser.cpp:385-433) on the host for one field of a
// frame at least the table's span long: bt_extract.hip's decode_field byte loop (its one-window
// fast path computes the same bits for fields no longer than their type).
static uint64_t decode_field_host(const ExField& f, const uint8_t* frame) {
    const uint32_t type = f.ctl & 0xFFu;
    const bool le = ((f.ctl >> 8) & 0xFFu) == BT_ENDIAN_LITTLE;
    const uint32_t o = f.offset, L = f.length;
    switch (type) {
    case BT_FT_BOOLEAN: return frame[o] != 0 ? 1u : 0u;
    case BT_FT_BYTES: case BT_FT_STRING: case BT_FT_MAC: case BT_FT_IPV4: case BT_FT_IPV6: case BT_FT_CUSTOM:
        return 0;
    default: break;
    }
    const uint32_t w = (type == BT_FT_UINT8 || type == BT_FT_INT8) ? 8u
                     : (type == BT_FT_UINT16 || type == BT_FT_INT16) ? 16u
                     : (type == BT_FT_UINT32 || type == BT_FT_INT32 || type == BT_FT_FLOAT32) ? 32u : 64u;
    if ((type == BT_FT_FLOAT32 || type == BT_FT_FLOAT64) && L * 8u != w) return 0;
    const uint32_t m = w == 64u ? 63u : 31u;
    uint64_t v = 0;
    for (uint32_t i = 0; i < L; ++i) {
        const uint32_t sh = (8u * i) & m;
        if (sh >= w) continue;
        v |= (uint64_t)frame[o + (le ? i : L - 1u - i)] << sh;
    }
    return w == 64u ? v : (v & ((1ull << w) - 1ull));
}

int bt_extract_host(const uint8_t* const* frames, const uint32_t* lens, uint32_t n, const bt_field_def* fields,
                    uint32_t n_fields, uint8_t* status, uint64_t* values, uint8_t* image) {
    if (n && (!frames || !lens)) return fail(BT_E_INVALID_ARGUMENT, "null frame pointers/lengths");
    ExTable t;
    bool never = false;
    uint64_t span64 = 0;
    int rc = build_table(fields, n_fields, &t, &span64, &never);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        const bool ok = !never && lens[i] >= t.span;
        if (status) status[i] = ok ? 0u : 9u;   // ParseStatus SUCCESS / PACKET_TOO_SHORT
        if (values)
            for (uint32_t k = 0; k < n_fields; ++k) values[(size_t)k * n + i] = ok ? decode_field_host(t.f[k], frames[i]) : 0u;
        if (image && !never && t.span) {
            uint8_t* out = image + (size_t)i * t.span;
            if (ok) std::memcpy(out, frames[i], t.span);
            else std::memset(out, 0, t.span);
        }
    }
    return BT_OK;
}

int bt_filter_dfa_pool(const bt_ctx* c, void* out, uint32_t cap, uint32_t* bytes) {
    if (!c || !bytes || (cap && !out)) return fail(BT_E_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> lk(const_cast<bt_ctx*>(c)->mu);
    *bytes = (uint32_t)c->dfa_pool.size();
    if (out && cap) std::memcpy(out, c->dfa_pool.data(), std::min<size_t>(cap, c->dfa_pool.size()));
    return BT_OK;
}

int bt_extract(bt_ctx* c, const uint8_t* const* frames, const uint32_t* lens, uint32_t n, const bt_field_def* fields,
               uint32_t n_fields, uint8_t* status, uint64_t* values, uint8_t* image) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!c) return fail(BT_E_INVALID_ARGUMENT, "null context");
    if (n && (!frames || !lens)) return fail(BT_E_INVALID_ARGUMENT, "null frame pointers/lengths");
    ExTable t;
    bool never = false;
    uint64_t span64 = 0;
    int rc = build_table(fields, n_fields, &t, &span64, &never);
    if (rc) return rc;
    if (!n) return BT_OK;
    if (never) {
        if (status) std::memset(status, 9, n);
        if (values) std::memset(values, 0, (size_t)n_fields * n * 8);
        return BT_OK;   // image: n x span bytes the caller could not have allocated anyway
    }
    const uint32_t span = t.span;
    const WaitFor lk(c);
    HIP_TRY(hipSetDevice(c->device));
    (void)pool_of(c);
    // chunks of at most 1M packets: [prefixes | descriptors] in, [status | values | image] out.
    // The gather and the drain run on the context's host threads (a serial gather, length
    // check and drain were most of a 1M-packet call). Tables up to 64 B (no frame is shorter
    // than an Ethernet minimum's worth of slot) give every frame one slot of round_up(span, 16)
    // bytes, so the gather needs no prefix pass; wider ones pack each frame's
    // round_up(min(len, span), 16) bytes after a per-worker count and scan.
    const uint32_t chunk = 1u << 20;
    const size_t slot = ((size_t)span + 15u) & ~(size_t)15u;
    const bool fixed = slot <= 64;
    for (uint32_t lo = 0; lo < n; lo += chunk) {
        const uint32_t m = std::min(chunk, n - lo);
        const unsigned T = pipeline_share(c);
        std::vector<uint64_t> part(T + 1, 0);   // packed: each worker's first staging byte
        if (!fixed) {
            pipeline_run(c, m, T, [&](unsigned w) {
                const uint32_t a = (uint32_t)((uint64_t)m * w / T), e = (uint32_t)((uint64_t)m * (w + 1) / T);
                uint64_t sum = 0;
                for (uint32_t i = a; i < e; ++i) sum += (std::min(lens[lo + i], span) + 15u) & ~15u;
                part[w + 1] = sum;
            });
            for (unsigned w = 0; w < T; ++w) part[w + 1] += part[w];
        }
        const size_t pre = (fixed ? (size_t)m * slot : part[T]) + 16, dsc = (size_t)m * 8;
        const size_t st_b = ((size_t)m + 15) & ~(size_t)15, val_b = (size_t)n_fields * m * 8, img_b = (size_t)m * span;
        const size_t in_b = pre + dsc, out_b = st_b + val_b + img_b;
        const size_t need = in_b + out_b + 64;
        if (need > c->ex_cap) {
            if (c->ex_h) (void)hipHostFree(c->ex_h);
            if (c->ex_d) (void)hipFree(c->ex_d);
            c->ex_h = nullptr;
            c->ex_d = nullptr;
            c->ex_cap = 0;
            const size_t cap = std::max(need, (size_t)1 << 20);
            HIP_TRY(hipHostMalloc(&c->ex_h, cap, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&c->ex_d, cap));
            c->ex_cap = cap;
        }
        uint8_t* h = c->ex_h;
        uint64_t* d = reinterpret_cast<uint64_t*>(h + pre);
        std::vector<uint32_t> bad(T, UINT32_MAX);   // per worker: first frame longer than 65535 B
        pipeline_run(c, m, T, [&](unsigned w) {
            const uint32_t a = (uint32_t)((uint64_t)m * w / T), e = (uint32_t)((uint64_t)m * (w + 1) / T);
            uint64_t p = fixed ? (uint64_t)a * slot : part[w];
            for (uint32_t i = a; i < e; ++i) {   // only [0, span) of a frame is ever read
                const uint32_t len = lens[lo + i];
                const uint32_t k = std::min(len, span);
                if (len > 0xFFFFu) bad[w] = std::min(bad[w], lo + i);
                else if (k) std::memcpy(h + p, frames[lo + i], k);
                d[i] = BT_DESC(p, len & 0xFFFFu);
                p += fixed ? slot : (k + 15u) & ~15u;
            }
        });
        const uint32_t first_bad = *std::min_element(bad.begin(), bad.end());
        if (first_bad != UINT32_MAX) return fail(BT_E_INVALID_ARGUMENT, "frame %u longer than 65535 bytes", first_bad);
        HIP_TRY(hipMemcpyAsync(c->ex_d, h, in_b, hipMemcpyHostToDevice, c->stream));
        bt_batch b{};
        b.base = c->ex_d;
        b.desc = c->ex_d + pre;
        b.n = m;
        b.bytes = pre;
        uint8_t* dout = c->ex_d + ((in_b + 15) & ~(size_t)15);
        uint8_t* hout = h + ((in_b + 15) & ~(size_t)15);
        bt_extract_out o{};
        o.status = dout;
        o.values = n_fields ? reinterpret_cast<uint64_t*>(dout + st_b) : nullptr;
        o.image = span ? dout + st_b + val_b : nullptr;
        o.n_cap = m;
        rc = run_extract(c, &b, t, false, &o, c->stream);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(hout, dout, out_b, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        pipeline_run(c, m, T, [&](unsigned w) {
            const uint32_t a = (uint32_t)((uint64_t)m * w / T), e = (uint32_t)((uint64_t)m * (w + 1) / T);
            if (a >= e) return;
            if (status) std::memcpy(status + lo + a, hout + a, e - a);
            for (uint32_t k = 0; values && k < n_fields; ++k)
                std::memcpy(values + (size_t)k * n + lo + a, hout + st_b + ((size_t)k * m + a) * 8, (size_t)(e - a) * 8);
            if (image && span) std::memcpy(image + ((size_t)lo + a) * span, hout + st_b + val_b + (size_t)a * span,
                                           (size_t)(e - a) * span);
        });
    }
    return BT_OK;
}

}  // extern "C"

namespace {

// Unpacks the packed device record (bt_kernels.hip parse_packet<true>; layout in
// beatrice_gpu.h) into a bt_rec. `slab(k)` returns the k-th 16-B slab; all six are read
// (every layout keeps slab k of a record in bounds) and the dwords past the record's own
// are masked off, so the unpack has no data-dependent branches: a capture's random mix
// of tags / L3 / L4 costs no mispredictions.
template <class Slab>
inline void unpack_record(Slab slab, bt_rec* out) {
    uint32_t c[24];
    for (uint32_t k = 0; k < BT_REC_SLABS; ++k) std::memcpy(c + 4 * k, slab(k), 16);
    const uint32_t present = c[4] & 0xFFu, ok = (c[4] >> 8) & 0xFFu;
    const uint32_t v0 = (ok & BT_L_VLAN0) ? 1u : 0u, v1 = (ok & BT_L_VLAN1) ? 1u : 0u, ne = v0 + v1;
    const uint32_t m4 = (ok & BT_L_IPV4) ? ~0u : 0u, m6 = (ok & BT_L_IPV6) && !m4 ? ~0u : 0u;
    const uint32_t l4d = (ok & BT_L_TCP) ? 5u : (ok & (BT_L_UDP | BT_L_ICMP)) ? 2u : 0u;
    const uint32_t x0 = v0 ? c[5] : 0u, x1 = v1 ? c[6] : 0u;
    const uint32_t* L = c + 5 + ne;   // <= c + 7: L[0..16] stays inside c
    uint32_t r[24];
    r[0] = c[0]; r[1] = c[1]; r[2] = c[2]; r[3] = c[3];
    r[4] = (v0 ? (c[3] & 0xFFFFu) : 0u) | (x0 & 0xFFFF0000u);   // tpid0 == ethertype
    r[5] = (x0 & 0xFFFFu) | (x1 << 16);
    // the walk's offsets (R-WALK): L3 after the tags the walk attempted; L4 after the
    // IPv4 header (IHL) or the fixed 40-B IPv6 header
    const uint32_t o3 = 14u + ((present & BT_L_VLAN0) ? 4u : 0u) + ((present & BT_L_VLAN1) ? 4u : 0u);
    const uint32_t l3_off = (present & (BT_L_IPV4 | BT_L_IPV6)) ? o3 : 0u;
    const uint32_t b0 = L[0] & 0xFFu;
    const uint32_t l4_off = (m4 && (present & (BT_L_TCP | BT_L_UDP | BT_L_ICMP))) ? o3 + 4u * (b0 & 0x0Fu)
                          : (m6 && (present & (BT_L_TCP | BT_L_UDP))) ? o3 + 40u : 0u;
    r[6] = present | (ok << 8) | (l3_off << 16) | (l4_off << 24);
    // IPv4 in bt_rec's padded layout, or IPv6 as stored, or nothing
    const uint32_t v4[10] = {b0 | (b0 << 8) | (((L[0] >> 8) & 0xFFu) << 16) | (((L[0] >> 16) & 0xFFu) << 24),
                             (L[0] >> 24) | (L[1] << 16), (L[1] >> 16) | (L[2] << 16), L[2] >> 16, L[3], L[4],
                             0u, 0u, 0u, 0u};
    for (int j = 0; j < 10; ++j) r[7 + j] = (v4[j] & m4) | (L[j] & m6);
    const uint32_t* l4 = L + ((m4 & 5u) | (m6 & 10u));
    for (uint32_t j = 0; j < 5; ++j) r[17 + j] = j < l4d ? l4[j] : 0u;
    r[22] = ((c[4] >> 16) & 7u) | (((c[4] >> 19) & 0xFFu) << 8) | (((c[4] >> 27) & 7u) << 16);
    r[23] = 0;
    std::memcpy(out, r, sizeof(r));
}

}  // namespace

extern "C" {

// Tiled layout: slab k >= 2 of a record sits at its rank among the tile's records that
// need slab k. ns[] = the tile's slab counts, read from the full slab-1 region.
static void tile_slab_counts(const uint8_t* tile, uint32_t* ns) {
    for (uint32_t j = 0; j < 64; ++j) {
        bt_rec r;
        r.ok = tile[(64 + j) * 16 + 1];   // slab 1, dword 0, byte 1
        ns[j] = bt_record_slabs(&r);
    }
}

static void gather_tiled(const uint8_t* tile, const uint32_t* ns, uint32_t lane, bt_rec* out) {
    unpack_record([&](uint32_t k) {
        uint32_t slot = lane;
        if (k >= 2) {
            slot = 0;
            for (uint32_t j = 0; j < lane; ++j) slot += ns[j] > k;
        }
        return tile + ((size_t)k * 64 + slot) * 16;
    }, out);
}

// Records [lo, hi) of one tile (lane order): the slab-k ranks are running counts, so a
// whole tile unpacks in one pass.
static void unpack_tile(const uint8_t* tile, uint32_t lo, uint32_t hi, bt_rec* out) {
    uint32_t rank[BT_REC_SLABS] = {};
    for (uint32_t j = 0; j < hi; ++j) {
        bt_rec r;
        r.ok = tile[(64 + j) * 16 + 1];
        const uint32_t ns = bt_record_slabs(&r);
        uint32_t at[BT_REC_SLABS] = {j, j, rank[2], rank[3], rank[4], rank[5]};
        for (uint32_t k = 2; k < ns; ++k) ++rank[k];
        if (j >= lo) unpack_record([&](uint32_t k) { return tile + ((size_t)k * 64 + at[k]) * 16; }, out + j);
    }
}

void bt_record_gather(const void* records, uint32_t n_cap, uint32_t i, bt_rec* out) {
    const uint8_t* tile = static_cast<const uint8_t*>(records) + (size_t)(i / 64) * BT_REC_SLABS * 64 * 16;
    uint32_t ns[64];
    tile_slab_counts(tile, ns);
    gather_tiled(tile, ns, i % 64, out);
    (void)n_cap;
}

void bt_record_gather_planes(const void* planes, uint32_t n_cap, uint32_t i, bt_rec* out) {
    const uint8_t* p = static_cast<const uint8_t*>(planes);
    unpack_record([&](uint32_t k) { return p + ((size_t)k * n_cap + i) * 16; }, out);
}

int bt_record_unpack(bt_ctx* ctx, const void* records, uint32_t n_cap, uint32_t n, uint32_t planes, bt_rec* out,
                     uint64_t* slabs) {
    if ((!records || (!out && !slabs)) && n) return fail(BT_E_INVALID_ARGUMENT, "null records / out");
    std::atomic<uint64_t> total{0};
    const uint8_t* p = static_cast<const uint8_t*>(records);
    host_parallel(ctx, [&](unsigned w, unsigned T) {
        const uint32_t lo = (uint32_t)((uint64_t)n * w / T), hi = (uint32_t)((uint64_t)n * (w + 1) / T);
        uint64_t cnt = 0;
        bt_rec r;
        for (uint32_t i = lo; i < hi; ++i) {
            if (out) {
                if (planes) {
                    bt_record_gather_planes(records, n_cap, i, out + i);
                } else {   // the rest of i's tile in one pass
                    const uint32_t t = i / 64, e = std::min(hi, t * 64 + 64);
                    unpack_tile(p + (size_t)t * BT_REC_SLABS * 64 * 16, i % 64, e - t * 64, out + t * 64);
                    if (slabs)
                        for (uint32_t j = i; j < e; ++j) cnt += bt_record_slabs(out + j);
                    i = e - 1;
                    continue;
                }
                if (slabs) cnt += bt_record_slabs(out + i);
            } else {   // count only: the ok byte sits in slab 1
                const uint8_t* s1 = planes ? p + ((size_t)n_cap + i) * 16
                                           : p + (((size_t)(i / 64) * BT_REC_SLABS + 1) * 64 + (i % 64)) * 16;
                r.ok = s1[1];
                cnt += bt_record_slabs(&r);
            }
        }
        total += cnt;
    });
    if (slabs) *slabs = total.load();
    return BT_OK;
}

uint32_t bt_record_slabs(const bt_rec* r) {
    const uint32_t ok = r->ok;
    const uint32_t nd = 5u + ((ok & BT_L_VLAN0) ? 1u : 0u) + ((ok & BT_L_VLAN1) ? 1u : 0u) +
                        ((ok & BT_L_IPV4) ? 5u : (ok & BT_L_IPV6) ? 10u : 0u) +
                        ((ok & BT_L_TCP) ? 5u : (ok & (BT_L_UDP | BT_L_ICMP)) ? 2u : 0u);
    return (nd + 3u) >> 2;
}

}  // extern "C"
