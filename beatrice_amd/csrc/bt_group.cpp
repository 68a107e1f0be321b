// bt_group.cpp — one process driving several MI355X devices.
//
// The reference daemon is one process whose capture threads feed one plugin set
// (/root/reference/src/BeatriceContext.cpp:215-278, src/PluginManager.cpp:158-188); a
// deployed stage there must be able to use every GPU of the node without a launcher. A
// group is one bt_ctx per device (its own streams, pinned staging and host pool, placed on
// its device's NUMA node); the filter program is compiled once on the host and installed on
// every member; a batch is split into contiguous, 64-packet-aligned ranges balanced by what
// each packet costs the call (bt_group_cost: the bytes it stages, or reads over PCIe), each
// member runs its range on its own host thread, and the results land straight in the
// caller's arrays: records, decisions and verdict words at the range's offset (the ranges
// start on tile boundaries, so verdict words concatenate without shifts), pass indices in
// ascending order. There is no collective: packets are independent.
//
// Two ingest forms: host batches (frames anywhere in host memory, gathered by each member's
// host pool into its pinned staging) and mapped batches (bt_group_parse_filter_mapped: the
// frames sit in group-registered host memory — a UMEM, a TPACKET_V3 ring — and each member's
// kernels read its range in place over its own PCIe link, the only ingest that is not
// bounded by the host's CPUs).
#include <hip/hip_runtime_api.h>
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "bt_device.h"
#include "bt_hip_util.h"
#include "bt_host.h"
#include "bt_host_pool.h"

namespace {

constexpr uint32_t kTile = 64;
constexpr uint32_t kMaxPool = 16;   // a context's host pool has at most 16 workers

using bt::MemberThreads;   // bt_host_pool.h

// A host range registered with every member (bt_group_host_register).
struct Region {
    uint8_t* host = nullptr;
    uint64_t bytes = 0;
    std::vector<uint8_t*> dev;   // member k's alias
};

}  // namespace

struct bt_group {
    std::vector<bt_ctx*> members;
    // members that share a device (BT_OPT_GROUP_SHARED_DEVICE): the device part of a mapped
    // call runs one member at a time per device when `serial_shared` (BT_GROUP_SHARED_SERIAL)
    std::vector<std::shared_ptr<std::mutex>> dev_mu;   // per member, shared by members of one device
    bool serial_shared = false;
    std::shared_mutex prog_mu;   // exclusive: bt_group_filter_compile; shared: batches (every member
                                 // of one batch runs the same program)
    std::unique_ptr<MemberThreads> threads;   // members > 1
    std::shared_mutex reg_mu;    // regions (exclusive: register / unregister)
    std::vector<Region> regions;
    // mapped calls that want a pass list but gave no verdict words: the group's own
    // (registered, grown on demand; one such call at a time)
    std::mutex scratch_mu;
    uint64_t* scratch = nullptr;
    size_t scratch_words = 0;
    std::vector<uint8_t*> scratch_dev;
    // host batches: a call that finds another one in flight runs whole on the least busy
    // member (up to route_below packets; BT_GROUP_ROUTE_BELOW, 0 = always split) instead of
    // splitting, so concurrent callers spread over the members (and the lanes of a device
    // listed twice) rather than each paying every member's per-call cost; a lone call splits
    std::atomic<uint32_t> calls{0};
    std::unique_ptr<std::atomic<uint32_t>[]> busy;   // per member: call parts running on it
    std::atomic<uint32_t> rr{0};
    uint32_t route_below = 0;
};

namespace {

// packet cost = round_up(min(len, window), align) + fixed
inline uint64_t packet_cost(uint32_t len, const bt_split_cost& c) {
    uint64_t w = std::min(len, c.window);
    if (c.align > 1) w = (w + c.align - 1) / c.align * c.align;
    return w + c.fixed;
}

constexpr bt_split_cost kShardCost{128, 1, 8 + 96, 0};   // beatrice_amd/shard.py's default model

struct Range {
    uint32_t lo, hi;
};

// The split a group call uses: bt_group_split_cost's exact per-tile costs for up to kExactTiles
// tiles; for larger batches the cost of one tile in every S (the middle tile of each run of S,
// about kExactTiles samples) stands for its run, and each cut lands on the tile where the
// interpolated running cost reaches total * k / parts. Exact costs read every descriptor on
// one thread before any member starts: for 16M packets that took ~45 ms, against 22 ms for a
// whole zero-copy pass over them (e2e --group 2, profiles/r04); the sampled split reads 1/S.
constexpr uint32_t kExactTiles = 4096;

template <class LenAt>
uint64_t tile_cost(LenAt len, uint32_t n, uint32_t t, const bt_split_cost& c) {
    uint64_t s = 0;
    const uint32_t e = std::min(n, (t + 1) * kTile);
    for (uint32_t i = t * kTile; i < e; ++i) s += packet_cost(len(i), c);
    return s;
}

template <class LenAt>
std::vector<Range> split_by(LenAt len, uint32_t n, uint32_t parts, const bt_split_cost& cost) {
    std::vector<Range> r(parts, Range{n, n});
    r[0].lo = 0;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    if (parts == 1 || n == 0) {
        r[0].hi = n;
        return r;
    }
    const uint32_t S = ntiles <= kExactTiles ? 1u : (ntiles + kExactTiles - 1) / kExactTiles;
    const uint32_t G = (ntiles + S - 1) / S;   // runs of S tiles
    std::vector<double> cum(G);
    double run = 0;
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t t0 = g * S, t1 = std::min(ntiles, t0 + S);
        if (S == 1) {
            run += (double)tile_cost(len, n, t0, cost);
        } else {   // the run's middle tile (a whole one: the last tile may be partial) for all of it
            const uint32_t mid = std::min(t0 + (t1 - t0) / 2, ntiles >= 2 && n % kTile ? ntiles - 2 : ntiles - 1);
            run += (double)tile_cost(len, n, mid, cost) * (double)(t1 - t0);
        }
        cum[g] = run;
    }
    std::vector<uint32_t> b(parts + 1, 0);
    for (uint32_t k = 1; k < parts; ++k) {
        const double target = run * (double)k / (double)parts;
        const uint32_t g = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        uint32_t tile;   // the first tile whose running cost reaches the target, + 1 (shard.py's cut)
        if (g >= G) {
            tile = ntiles;
        } else {
            const uint32_t t0 = g * S, t1 = std::min(ntiles, t0 + S);
            const double before = g ? cum[g - 1] : 0.0, per = (cum[g] - before) / (double)(t1 - t0);
            const double need = per > 0 ? (target - before) / per : 0.0;
            tile = t0 + std::min(t1 - t0, (uint32_t)std::max(1.0, std::ceil(need)));
        }
        const uint64_t cut = std::min<uint64_t>((uint64_t)std::min(tile, ntiles) * kTile, n);
        b[k] = (uint32_t)std::max<uint64_t>(cut, b[k - 1]);
    }
    b[parts] = n;
    for (uint32_t k = 0; k < parts; ++k) r[k] = {b[k], b[k + 1]};
    return r;
}

// Runs fn(k) for every member on its own thread; returns the first failure (with its
// message moved to this thread's bt_last_error). An exception in a member's part (an
// allocation) becomes BT_E_INTERNAL there: nothing throws across the C-ABI or out of a
// member thread.
template <class Fn>
int run_members(bt_group* g, Fn fn) {
    const uint32_t m = (uint32_t)g->members.size();
    std::vector<int> rc(m, BT_OK);
    std::vector<std::string> msg(m);
    auto one = [&](uint32_t k) {
        try {
            rc[k] = fn(k);
            if (rc[k]) msg[k] = bt_last_error();
        } catch (const std::exception& e) {
            rc[k] = BT_E_INTERNAL;
            msg[k] = e.what();
        } catch (...) {
            rc[k] = BT_E_INTERNAL;
            msg[k] = "unknown exception";
        }
    };
    if (m == 1) {
        one(0);   // one device: no thread
    } else {
        g->threads->run(one);
    }
    for (uint32_t k = 0; k < m; ++k)
        if (rc[k]) {
            if (m == 1) return bt::set_error(rc[k], "%s", msg[k].c_str());
            return bt::set_error(rc[k], "group member %u (device %d): %s", k, bt::ctx_device(g->members[k]),
                                 msg[k].c_str());
        }
    return BT_OK;
}

// Holds a counter up for a scope.
struct Hold {
    std::atomic<uint32_t>& a;
    explicit Hold(std::atomic<uint32_t>& x) : a(x) { a.fetch_add(1, std::memory_order_acq_rel); }
    ~Hold() { a.fetch_sub(1, std::memory_order_acq_rel); }
};

// One host batch over the group: frames(ctx, lo, cnt, ...) runs packets [lo, lo + cnt).
template <class LenAt, class Frames>
int group_batch(bt_group* g, uint32_t n, LenAt len, Frames frames, bt_rec* records, uint64_t* verdict,
                uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    const uint32_t m = (uint32_t)g->members.size();
    const uint32_t others = g->calls.load(std::memory_order_acquire);
    Hold in_flight(g->calls);
    if (m > 1 && others > 0 && n <= g->route_below) {   // concurrent callers: whole calls, spread
        const uint32_t start = g->rr.fetch_add(1, std::memory_order_relaxed) % m;
        uint32_t k = start, least = UINT32_MAX;
        for (uint32_t j = 0; j < m; ++j) {
            const uint32_t c = (start + j) % m, v = g->busy[c].load(std::memory_order_relaxed);
            if (v < least) least = v, k = c;
        }
        Hold on(g->busy[k]);
        return frames(g->members[k], 0, n, records, verdict, decide, pass_idx, n_pass);
    }
    const bool want_filter = verdict || decide || pass_idx || n_pass;
    bt_split_cost cost{};
    (void)bt_group_cost(g, 0, records != nullptr, want_filter, 8, &cost);
    const std::vector<Range> r = split_by(len, n, m, cost);
    std::vector<uint32_t> npass(m, 0);
    const bool want_pass = pass_idx || n_pass;
    // member k lists its passes (indices relative to its range) at pass_idx + lo, inside its own
    // range of the caller's array (it has at most cnt of them)
    int rc = run_members(g, [&](uint32_t k) -> int {
        const uint32_t lo = r[k].lo, cnt = r[k].hi - r[k].lo;
        if (!cnt) return BT_OK;
        Hold on(g->busy[k]);
        return frames(g->members[k], lo, cnt, records ? records + lo : nullptr, verdict ? verdict + lo / kTile : nullptr,
                      decide ? decide + lo : nullptr, pass_idx ? pass_idx + lo : nullptr,
                      want_pass ? &npass[k] : nullptr);
    });
    if (rc) return rc;
    // then they move down to their place in the whole list, in member order (member k's place
    // starts at or below its range's start, so nothing unread is overwritten)
    uint32_t at = npass[0];
    for (uint32_t k = 1; k < m; ++k) {
        if (pass_idx) {
            const uint32_t lo = r[k].lo;
            for (uint32_t j = 0; j < npass[k]; ++j) pass_idx[at + j] = pass_idx[lo + j] + lo;
        }
        at += npass[k];
    }
    if (n_pass) *n_pass = at;
    return BT_OK;
}

// Member k's alias of host range [p, p + need) (group-registered); nullptr if none.
uint8_t* alias_of(const bt_group* g, uint32_t k, const void* p, uint64_t need) {
    const uint8_t* a = static_cast<const uint8_t*>(p);
    for (const Region& r : g->regions)
        if (a >= r.host && a < r.host + r.bytes) {
            if ((uint64_t)(a - r.host) + need > r.bytes) return nullptr;
            return r.dev[k] + (a - r.host);
        }
    return nullptr;
}

// The members' devices, in member order (bt::pin_acquire's device list: member k's alias of
// a registered range is aliases[k], taken on its own device).
std::vector<int> member_devices(const bt_group* g) {
    std::vector<int> d;
    for (bt_ctx* c : g->members) d.push_back(bt::ctx_device(c));
    return d;
}

// Indices of the set bits of verdict words [w0, w1) whose packet index is < n, written
// ascending from out (out == nullptr: counted only); returns how many.
uint32_t verdict_bits(const uint64_t* ver, uint32_t w0, uint32_t w1, uint32_t n, uint32_t* out) {
    uint32_t c = 0;
    for (uint32_t w = w0; w < w1; ++w) {
        uint64_t x = ver[w];
        if ((uint64_t)w * 64 + 64 > n) x &= (n & 63) ? (1ull << (n & 63)) - 1ull : ~0ull;
        if (!out) {
            c += (uint32_t)__builtin_popcountll(x);
            continue;
        }
        while (x) {
            out[c++] = w * 64 + (uint32_t)__builtin_ctzll(x);
            x &= x - 1;
        }
    }
    return c;
}

}  // namespace

extern "C" {

int bt_group_split(const uint32_t* lens, uint32_t n, uint32_t parts, uint32_t* bounds) {
    return bt_group_split_cost(lens, n, parts, &kShardCost, bounds);
}

static int split_cost_exact(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost,
                            uint32_t* bounds);

int bt_group_split_cost(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost,
                        uint32_t* bounds) {
    if (!bounds || !parts || !cost || (n && !lens)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / zero parts");
    try {
        return split_cost_exact(lens, n, parts, cost, bounds);
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_split_cost: %s", e.what());
    }
}

static int split_cost_exact(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost,
                            uint32_t* bounds) {
    bounds[0] = 0;
    if (parts == 1 || n == 0) {
        for (uint32_t k = 1; k <= parts; ++k) bounds[k] = n;
        return BT_OK;
    }
    // cumulative cost per tile; cut k at the first tile whose running total reaches
    // total * k / parts (numpy's searchsorted(side="left") + 1 in shard.py)
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    std::vector<uint64_t> cum(ntiles);
    uint64_t run = 0;
    for (uint32_t t = 0; t < ntiles; ++t) {
        const uint32_t e = std::min(n, (t + 1) * kTile);
        for (uint32_t i = t * kTile; i < e; ++i) run += packet_cost(lens[i], *cost);
        cum[t] = run;
    }
    const double total = (double)run;
    for (uint32_t k = 1; k < parts; ++k) {
        const double target = total * (double)k / (double)parts;
        const uint32_t i = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target,
                                                        [](uint64_t c, double t) { return (double)c < t; }) -
                                      cum.begin());
        const uint64_t cut = std::min<uint64_t>((uint64_t)std::min(i + 1, ntiles) * kTile, n);
        bounds[k] = (uint32_t)std::max<uint64_t>(cut, bounds[k - 1]);
    }
    bounds[parts] = n;
    return BT_OK;
}

int bt_group_split_plan(const uint32_t* lens, uint32_t n, uint32_t parts, const bt_split_cost* cost, uint32_t* bounds) {
    if (!bounds || !parts || !cost || (n && !lens)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / zero parts");
    try {
        const std::vector<Range> r = split_by([lens](uint32_t i) { return lens[i]; }, n, parts, *cost);
        for (uint32_t k = 0; k < parts; ++k) bounds[k] = r[k].lo;
        bounds[parts] = n;
        return BT_OK;
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_split_plan: %s", e.what());
    }
}

int bt_group_thread_budget(uint32_t members, uint32_t usable, uint32_t requested, uint32_t* per_member) {
    if (!members || !per_member) return bt::set_error(BT_E_INVALID_ARGUMENT, "zero members / null out");
    usable = std::max(usable, 1u);
    if (requested) *per_member = std::min(std::max(requested / members, 1u), 16u);
    else *per_member = std::min(std::max(usable / members, 1u), 16u);
    return BT_OK;
}

static int group_create(const int* devices, uint32_t n_devices, const bt_opts* opts, bt_group** out);

int bt_group_create(const int* devices, uint32_t n_devices, const bt_opts* opts, bt_group** out) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!out || !devices || !n_devices) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / no devices");
    try {
        return group_create(devices, n_devices, opts, out);
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_RESOURCE, "bt_group_create: %s", e.what());
    }
}

static int group_create(const int* devices, uint32_t n_devices, const bt_opts* opts, bt_group** out) {
    *out = nullptr;
    for (uint32_t i = 0; i < n_devices; ++i)
        for (uint32_t j = 0; j < i; ++j)
            if (devices[i] == devices[j] && !(opts && (opts->flags & BT_OPT_GROUP_SHARED_DEVICE)))
                return bt::set_error(BT_E_INVALID_ARGUMENT, "device %d listed twice (BT_OPT_GROUP_SHARED_DEVICE "
                                     "allows it, for tests on one GPU)", devices[i]);
    // one host-thread budget for the whole group, split across the members (an 8-device
    // group on a 16-CPU host had built 8 pools of 8 threads)
    bt_opts mo{};
    if (opts) mo = *opts;
    uint32_t requested = mo.host_threads;
    if (!requested) {
        const char* e = getenv("BT_HOST_THREADS");
        if (e && atoi(e) > 0) requested = (uint32_t)atoi(e);
    }
    (void)bt_group_thread_budget(n_devices, bt::usable_cpus(), requested, &mo.host_threads);
    auto* g = new bt_group();
    for (uint32_t i = 0; i < n_devices; ++i) {
        bt_ctx* c = nullptr;
        const int rc = bt_create(devices[i], &mo, &c);
        if (rc) {
            const std::string msg = bt_last_error();
            bt_group_destroy(g);
            return bt::set_error(rc, "group member %u (device %d): %s", i, devices[i], msg.c_str());
        }
        g->members.push_back(c);
    }
    {
        std::vector<std::pair<int, std::shared_ptr<std::mutex>>> by_dev;
        for (uint32_t i = 0; i < n_devices; ++i) {
            auto it = std::find_if(by_dev.begin(), by_dev.end(), [&](const auto& x) { return x.first == devices[i]; });
            if (it == by_dev.end()) {
                by_dev.emplace_back(devices[i], std::make_shared<std::mutex>());
                it = by_dev.end() - 1;
            }
            g->dev_mu.push_back(it->second);
        }
        const char* e = getenv("BT_GROUP_SHARED_SERIAL");
        g->serial_shared = e && atoi(e) != 0;
        const char* rb = getenv("BT_GROUP_ROUTE_BELOW");
        g->route_below = rb ? (uint32_t)strtoul(rb, nullptr, 10) : (1u << 20);
        g->busy = std::make_unique<std::atomic<uint32_t>[]>(n_devices);
        for (uint32_t i = 0; i < n_devices; ++i) g->busy[i].store(0, std::memory_order_relaxed);
    }
    if (n_devices > 1) {
        std::vector<const cpu_set_t*> pins;
        for (bt_ctx* c : g->members) pins.push_back(bt::ctx_pin(c));
        try {
            // each member thread starts on its member's device (every entry point it calls selects
            // the context's device too; this keeps any HIP call made there on the right one)
            std::vector<int> devs(devices, devices + n_devices);
            g->threads = std::make_unique<MemberThreads>(n_devices, pins,
                                                         [devs](uint32_t k) { (void)hipSetDevice(devs[k]); });
        } catch (const std::exception& e) {
            bt_group_destroy(g);
            return bt::set_error(BT_E_RESOURCE, "group threads: %s", e.what());
        }
    }
    *out = g;
    return BT_OK;
}

void bt_group_destroy(bt_group* g) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g) return;
    g->threads.reset();
    // the group's references on its registered pages (the last one waits for the devices)
    for (const Region& r : g->regions) (void)bt::pin_release(r.host, r.bytes);
    if (g->scratch) {
        (void)bt::pin_release(g->scratch, g->scratch_words * 8);
        free(g->scratch);
    }
    for (bt_ctx* c : g->members) bt_destroy(c);
    delete g;
}

uint32_t bt_group_size(const bt_group* g) { return g ? (uint32_t)g->members.size() : 0u; }

bt_ctx* bt_group_member(bt_group* g, uint32_t k) {
    return g && k < g->members.size() ? g->members[k] : nullptr;
}

int bt_group_filter_compile(bt_group* g, const bt_filter_desc* filters, uint32_t n) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    try {
        std::unique_lock<std::shared_mutex> lk(g->prog_mu);
        bt::CompiledProgram p;   // compiled once, installed on every device
        if (int rc = bt::compile_program(filters, n, bt::ctx_flags(g->members[0]), &p)) return rc;
        const int rc = run_members(g, [&](uint32_t k) { return bt::install_program(g->members[k], p); });
        return rc;
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_filter_compile: %s", e.what());
    }
}

int bt_group_cost(bt_group* g, int mapped, int records, int filters, uint32_t desc_bytes, bt_split_cost* out) {
    if (!g || !out) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    *out = bt_split_cost{};
    out->align = 16;
    if (mapped) {
        // filter-only: the lean first round reads frame bytes [kLeanLo, kLeanPcie) = [12, 38),
        // 26 B in two or three 16-B chunks by the frame's alignment: 32 + one chunk of slack
        constexpr uint32_t kLeanWindow = (bt::kLeanPcie - bt::kLeanLo + 15u) / 16u * 16u + 16u;
        static_assert(kLeanWindow == 48u, "bt_group_cost's documented lean window");
        out->window = records ? 128u : kLeanWindow;
        out->fixed = desc_bytes + (records ? 64u : 0u) + (filters ? 1u : 0u);
    } else {
        // the bytes the host pipeline copies per frame for member 0's installed program (32 /
        // 112 / 176), published by the context at install time: a program compiled on a member
        // directly (bt_group_member + bt_filter_compile) is seen too, and no member lock is taken
        out->window = bt::staged_window(g->members[0], records != 0);
        out->fixed = desc_bytes + (records ? (uint32_t)BT_REC_BYTES : 0u) + (filters ? 1u : 0u);
    }
    return BT_OK;
}

int bt_group_parse_filter(bt_group* g, const uint8_t* base, const bt_pkt_desc* desc, uint32_t n, bt_rec* records,
                          uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    if (n && (!base || !desc)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null packet buffer/descriptors");
    try {
        std::shared_lock<std::shared_mutex> lk(g->prog_mu);
        return group_batch(g, n, [desc](uint32_t i) { return (uint32_t)BT_DESC_LEN(desc[i]); },
                           [&](bt_ctx* c, uint32_t lo, uint32_t cnt, bt_rec* r, uint64_t* v, uint8_t* d, uint32_t* p,
                               uint32_t* np) { return bt_parse_filter(c, base, desc + lo, cnt, r, v, d, p, np); },
                           records, verdict, decide, pass_idx, n_pass);
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_parse_filter: %s", e.what());
    }
}

int bt_group_parse_filter_ptrs(bt_group* g, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                               bt_rec* records, uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx,
                               uint32_t* n_pass) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    if (n && (!frames || !lens)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null frame pointers/lengths");
    try {
        std::shared_lock<std::shared_mutex> lk(g->prog_mu);
        return group_batch(g, n, [lens](uint32_t i) { return lens[i]; },
                           [&](bt_ctx* c, uint32_t lo, uint32_t cnt, bt_rec* r, uint64_t* v, uint8_t* d, uint32_t* p,
                               uint32_t* np) { return bt_parse_filter_ptrs(c, frames + lo, lens + lo, cnt, r, v, d, p, np); },
                           records, verdict, decide, pass_idx, n_pass);
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_parse_filter_ptrs: %s", e.what());
    }
}

int bt_group_host_parallel(bt_group* g, void (*fn)(void*, uint32_t, uint32_t), void* user) {
    if (!g || !fn) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    try {
        const uint32_t m = (uint32_t)g->members.size();
        std::vector<uint32_t> base(m + 1, 0);
        for (uint32_t k = 0; k < m; ++k) base[k + 1] = base[k] + bt::pool_size(g->members[k]);
        const uint32_t total = base[m];
        return run_members(g, [&](uint32_t k) -> int {
            bt::host_parallel(g->members[k], [&](unsigned w, unsigned) { fn(user, base[k] + w, total); });
            return BT_OK;
        });
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_host_parallel: %s", e.what());
    }
}

int bt_group_host_register(bt_group* g, void* host, uint64_t bytes) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g || !host || !bytes) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / empty range");
    try {
        std::unique_lock<std::shared_mutex> lk(g->reg_mu);
        const uint8_t* a = static_cast<const uint8_t*>(host);
        for (const Region& r : g->regions)
            if (a < r.host + r.bytes && r.host < a + bytes)
                return bt::set_error(BT_E_INVALID_ARGUMENT, "range %p + %llu overlaps a registered range", host,
                                     (unsigned long long)bytes);
        // whole pages, in the process's one table (bt_pin.h): pages a context or another group
        // already holds in full are shared, a range that holds only some of them is refused
        const std::vector<int> devs = member_devices(g);
        Region r;
        r.host = static_cast<uint8_t*>(host);
        r.bytes = bytes;
        r.dev.assign(devs.size(), nullptr);
        if (int rc = bt::pin_acquire(host, bytes, devs.data(), (uint32_t)devs.size(), r.dev.data())) return rc;
        g->regions.push_back(std::move(r));
        return BT_OK;
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_host_register: %s", e.what());
    }
}

int bt_group_host_unregister(bt_group* g, void* host) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g || !host) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    std::unique_lock<std::shared_mutex> lk(g->reg_mu);
    auto it = std::find_if(g->regions.begin(), g->regions.end(), [&](const Region& r) { return r.host == host; });
    if (it == g->regions.end()) return bt::set_error(BT_E_INVALID_ARGUMENT, "%p is not a registered range", host);
    // the last reference on the pages waits for every device that holds an alias of them (the
    // queued kernels of every member that may read or write the range) before unregistering
    if (int rc = bt::pin_release(it->host, it->bytes)) return rc;
    g->regions.erase(it);
    for (bt_ctx* c : g->members) bt::ctx_forget_base(c);   // the address may come back as another kind
    return BT_OK;
}

int bt_group_parse_filter_mapped(bt_group* g, const bt_batch* b, const bt_outputs* o) {
    const bt::DeviceRestore keep_device;   // the caller's current device, restored on return
    if (!g || !b || !o) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    const uint32_t n = b->n;
    if (n && !b->base) return bt::set_error(BT_E_INVALID_ARGUMENT, "null packet buffer");
    if (!b->desc && b->stride == 0 && n) return bt::set_error(BT_E_INVALID_ARGUMENT, "fixed-stride mode needs stride > 0");
    if (b->desc_format > BT_DESC_XDP) return bt::set_error(BT_E_INVALID_ARGUMENT, "unknown desc_format %u", b->desc_format);
    if (b->desc && !b->bytes) return bt::set_error(BT_E_INVALID_ARGUMENT, "descriptor batch with bytes == 0");
    // fixed stride: the members' ranges are carved out of [base, base + n * stride), so a
    // smaller stated size is refused here, as a single context refuses it (run_device)
    if (!b->desc && b->bytes && b->bytes < (uint64_t)n * b->stride)
        return bt::set_error(BT_E_INVALID_ARGUMENT, "fixed-stride batch: bytes %llu < n * stride %llu",
                             (unsigned long long)b->bytes, (unsigned long long)n * b->stride);
    if (o->records && o->n_cap < n) return bt::set_error(BT_E_INVALID_ARGUMENT, "records n_cap %u < n %u", o->n_cap, n);
    const bool filter = o->verdict || o->decide || o->pass_idx || o->n_pass;
    const bool want_pass = o->pass_idx || o->n_pass;
    if (!n || (!filter && !o->records)) {
        if (o->n_pass) *o->n_pass = 0;
        return BT_OK;
    }
    try {
        std::shared_lock<std::shared_mutex> plk(g->prog_mu);
        std::shared_lock<std::shared_mutex> rlk(g->reg_mu);
        const uint32_t m = (uint32_t)g->members.size();
        const uint32_t flags = bt::ctx_flags(g->members[0]);
        const bool aos = (flags & BT_OPT_RECORDS_AOS) != 0;
        if (o->records && (flags & BT_OPT_RECORDS_PLANES) && m > 1)
            return bt::set_error(BT_E_INVALID_ARGUMENT, "plane-major records cannot be split across group members");
        const uint32_t dsz = !b->desc ? 0u : b->desc_format == BT_DESC_XDP ? 16u : 8u;
        // the split: by what each packet costs its member's PCIe link
        std::vector<Range> r;
        if (m == 1) {
            r.push_back({0, n});
        } else if (!b->desc) {   // fixed stride: equal cost, equal tile counts
            const uint32_t tiles = (n + kTile - 1) / kTile;
            for (uint32_t k = 0; k < m; ++k)
                r.push_back({std::min(n, (uint32_t)((uint64_t)tiles * k / m) * kTile),
                             std::min(n, (uint32_t)((uint64_t)tiles * (k + 1) / m) * kTile)});
        } else {
            const uint8_t* d = static_cast<const uint8_t*>(b->desc);
            bt_split_cost cost{};
            (void)bt_group_cost(g, 1, o->records != nullptr, filter, dsz, &cost);
            if (b->desc_format == BT_DESC_XDP)
                r = split_by([d](uint32_t i) {
                    uint32_t l;
                    std::memcpy(&l, d + (size_t)i * 16 + 8, 4);
                    return l;
                }, n, m, cost);
            else
                r = split_by([d](uint32_t i) { return (uint32_t)BT_DESC_LEN(reinterpret_cast<const uint64_t*>(d)[i]); },
                             n, m, cost);
        }
        // the verdict words the pass list is built from
        const uint32_t words = (n + 63) / 64;
        std::unique_lock<std::mutex> slk(g->scratch_mu, std::defer_lock);
        uint64_t* ver = o->verdict;
        std::vector<uint8_t*> ver_dev(m, nullptr);
        if (!ver && want_pass) {
            slk.lock();
            if (g->scratch_words < words) {
                if (g->scratch) {
                    if (int rc = bt::pin_release(g->scratch, g->scratch_words * 8)) return rc;
                    free(g->scratch);
                    g->scratch = nullptr;
                    g->scratch_words = 0;
                    g->scratch_dev.clear();
                }
                const size_t bytes = ((size_t)words * 8 + 4095) & ~(size_t)4095;
                void* p = nullptr;
                if (posix_memalign(&p, 4096, bytes) != 0) return bt::set_error(BT_E_RESOURCE, "scratch verdict words");
                const std::vector<int> devs = member_devices(g);
                std::vector<uint8_t*> al(devs.size(), nullptr);
                if (int rc = bt::pin_acquire(p, bytes, devs.data(), (uint32_t)devs.size(), al.data())) {
                    free(p);   // no half-made scratch for later calls
                    return rc;
                }
                g->scratch_dev = std::move(al);
                g->scratch = static_cast<uint64_t*>(p);
                g->scratch_words = bytes / 8;
            }
            ver = g->scratch;
            ver_dev = g->scratch_dev;
        }
        // every buffer the kernels touch must be group-registered
        auto need = [&](const void* p, uint64_t bytes, const char* what, uint32_t k, uint8_t** out) -> int {
            *out = nullptr;
            if (!p) return BT_OK;
            *out = alias_of(g, k, p, bytes);
            if (!*out)
                return bt::set_error(BT_E_INVALID_ARGUMENT, "%s (%p + %llu) is not inside a group-registered range", what,
                                     p, (unsigned long long)bytes);
            return BT_OK;
        };
        const uint64_t rec_bytes = aos ? (uint64_t)o->n_cap * BT_REC_BYTES
                                       : (flags & BT_OPT_RECORDS_PLANES) ? (uint64_t)o->n_cap * 16 * 6
                                                                          : ((uint64_t)o->n_cap + 63) / 64 * 6144;
        struct Member {
            bt_batch b{};
            bt_outputs o{};
        };
        std::vector<Member> mb(m);
        for (uint32_t k = 0; k < m; ++k) {
            const uint32_t lo = r[k].lo, cnt = r[k].hi - r[k].lo;
            uint8_t *base = nullptr, *desc = nullptr, *rec = nullptr, *dec = nullptr, *vw = nullptr;
            if (int rc = need(b->base, b->bytes ? b->bytes : (uint64_t)n * b->stride, "batch.base", k, &base)) return rc;
            if (int rc = need(b->desc, (uint64_t)n * dsz, "batch.desc", k, &desc)) return rc;
            if (int rc = need(o->records, rec_bytes, "out.records", k, &rec)) return rc;
            if (int rc = need(o->decide, n, "out.decide", k, &dec)) return rc;
            if (o->verdict) {
                if (int rc = need(o->verdict, (uint64_t)words * 8, "out.verdict", k, &vw)) return rc;
            } else if (ver) {
                vw = ver_dev[k];
            }
            Member& x = mb[k];
            x.b = *b;
            x.b.n = cnt;
            if (b->desc) {
                x.b.base = base;
                x.b.desc = desc + (size_t)lo * dsz;
            } else {
                x.b.base = base + (size_t)lo * b->stride;
                x.b.bytes = (b->bytes ? b->bytes : (uint64_t)n * b->stride) - (uint64_t)lo * b->stride;
            }
            if (rec) {
                x.o.records = aos ? rec + (size_t)lo * BT_REC_BYTES : rec + (size_t)(lo / kTile) * 6144;
                x.o.n_cap = (flags & BT_OPT_RECORDS_PLANES) ? o->n_cap : o->n_cap - lo;
            }
            x.o.decide = dec ? dec + lo : nullptr;
            x.o.verdict = vw ? reinterpret_cast<uint64_t*>(vw) + lo / kTile : nullptr;
        }
        // sparse frames (BT_OPT_MAPPED_GATHER_SPARSE): filter-only batches of packed
        // descriptors whose frames lie far apart are gathered on the host instead, where each
        // frame's window would be a separate small PCIe read (C4-like frames ~870 B apart:
        // host gather 409-460 against 257 Mpps in place)
        static const uint64_t gather_above = [] {
            const char* e = getenv("BT_MAPPED_GATHER_ABOVE");
            return e ? strtoull(e, nullptr, 10) : 512ull;
        }();
        const bool may_gather = (flags & BT_OPT_MAPPED_GATHER_SPARSE) && !o->records && b->desc &&
                                b->desc_format == BT_DESC_PACKED && !(b->flags & BT_BATCH_PREFIXES);
        auto sparse = [&](uint32_t lo, uint32_t hi) {   // mean spacing of ~64 sampled neighbours
            const uint64_t* d = static_cast<const uint64_t*>(b->desc);
            if (hi - lo < 2) return false;
            const uint32_t samples = std::min<uint32_t>(64, hi - lo - 1);
            uint64_t sum = 0;
            for (uint32_t j = 0; j < samples; ++j) {
                const uint32_t i = lo + (uint32_t)((uint64_t)(hi - lo - 1) * j / samples);
                const uint64_t a = BT_DESC_OFF(d[i]), c = BT_DESC_OFF(d[i + 1]);
                sum += c > a ? c - a : a - c;
            }
            return sum >= gather_above * samples;
        };
        // the host gather reads each frame at base + off directly: only when every frame of the
        // range lies inside the batch's bytes (the kernels clamp reads at `bytes` instead)
        auto in_bounds = [&](bt_ctx* c, uint32_t lo, uint32_t hi) {
            const uint64_t* d = static_cast<const uint64_t*>(b->desc);
            std::atomic<bool> ok{true};
            bt::host_parallel(c, [&](unsigned w, unsigned T) {
                const uint32_t a = lo + (uint32_t)((uint64_t)(hi - lo) * w / T);
                const uint32_t e = lo + (uint32_t)((uint64_t)(hi - lo) * (w + 1) / T);
                for (uint32_t i = a; i < e; ++i)
                    if (BT_DESC_OFF(d[i]) + BT_DESC_LEN(d[i]) > b->bytes) {
                        ok.store(false, std::memory_order_relaxed);
                        return;
                    }
            });
            return ok.load();
        };
        // phase 1: every member's kernels over its range, then its pass count (per pool worker)
        std::vector<std::vector<uint32_t>> cnt(m);
        int rc = run_members(g, [&](uint32_t k) -> int {
            const uint32_t lo = r[k].lo, hi = r[k].hi;
            if (lo == hi) return BT_OK;
            bt_ctx* c = g->members[k];
            if (may_gather && sparse(lo, hi) && in_bounds(c, lo, hi)) {   // host addresses: frames, outputs
                if (int e = bt_parse_filter(c, b->base, static_cast<const bt_pkt_desc*>(b->desc) + lo, hi - lo, nullptr,
                                            ver ? ver + lo / kTile : nullptr, o->decide ? o->decide + lo : nullptr,
                                            nullptr, nullptr))
                    return e;
            } else {
                std::unique_lock<std::mutex> dl(*g->dev_mu[k], std::defer_lock);
                if (g->serial_shared) dl.lock();
                if (int e = bt_parse_filter_device(c, &mb[k].b, &mb[k].o, nullptr)) return e;
                if (int e = bt_synchronize(c)) return e;
            }
            if (!want_pass) return BT_OK;
            const uint32_t w0 = lo / kTile, w1 = (hi + 63) / 64;
            std::vector<uint32_t>& ck = cnt[k];
            ck.assign(kMaxPool, 0);
            bt::host_parallel(c, [&](unsigned w, unsigned T) {
                const uint32_t a = w0 + (uint32_t)((uint64_t)(w1 - w0) * w / T);
                const uint32_t e = w0 + (uint32_t)((uint64_t)(w1 - w0) * (w + 1) / T);
                ck[w] = verdict_bits(ver, a, e, hi, nullptr);
            });
            return BT_OK;
        });
        if (rc) return rc;
        if (!want_pass) return BT_OK;
        // phase 2: each member writes its indices at its offset in the whole list
        std::vector<uint32_t> at(m + 1, 0);
        for (uint32_t k = 0; k < m; ++k) {
            uint32_t s = 0;
            for (uint32_t x : cnt[k]) s += x;
            at[k + 1] = at[k] + s;
        }
        if (o->pass_idx) {
            rc = run_members(g, [&](uint32_t k) -> int {
                const uint32_t lo = r[k].lo, hi = r[k].hi;
                if (lo == hi) return BT_OK;
                const uint32_t w0 = lo / kTile, w1 = (hi + 63) / 64;
                const std::vector<uint32_t>& ck = cnt[k];
                bt::host_parallel(g->members[k], [&](unsigned w, unsigned T) {
                    const uint32_t a = w0 + (uint32_t)((uint64_t)(w1 - w0) * w / T);
                    const uint32_t e = w0 + (uint32_t)((uint64_t)(w1 - w0) * (w + 1) / T);
                    uint32_t off = at[k];
                    for (unsigned j = 0; j < w; ++j) off += ck[j];
                    (void)verdict_bits(ver, a, e, hi, o->pass_idx + off);
                });
                return BT_OK;
            });
            if (rc) return rc;
        }
        if (o->n_pass) *o->n_pass = at[m];
        return BT_OK;
    } catch (const std::exception& e) {
        return bt::set_error(BT_E_INTERNAL, "bt_group_parse_filter_mapped: %s", e.what());
    }
}

}  // extern "C"
