// bt_group.cpp — one process driving several MI355X devices.
//
// The reference daemon is one process whose capture threads feed one plugin set
// (/root/reference/src/BeatriceContext.cpp:215-278, src/PluginManager.cpp:158-188); a
// deployed stage there must be able to use every GPU of the node without a launcher. A
// group is one bt_ctx per device (its own streams, pinned staging and host pool); the
// filter program is compiled once on the host and installed on every member; a batch
// is split into contiguous, 64-packet-aligned ranges balanced by the bytes each packet
// costs to stage (bt_group_split, the C++ form of beatrice_amd/shard.py:shard_bounds),
// each member runs its range on its own host thread, and the results land straight in
// the caller's arrays: records, decisions and verdict words at the range's offset (the
// ranges start on tile boundaries, so verdict words concatenate without shifts), pass
// indices offset by the range start and concatenated in order. There is no collective:
// packets are independent.
#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <condition_variable>
#include <functional>

#include "bt_host.h"

namespace {

// One thread per member after the first, kept for the group's life: member k's part of a batch
// runs on thread k (member 0 on the caller), so a batch costs no thread creation (a plugin's
// 64k-packet batches over 8 devices had spawned 7 threads per batch).
class MemberThreads {
public:
    explicit MemberThreads(uint32_t members) {
        for (uint32_t k = 1; k < members; ++k) th_.emplace_back([this, k] { loop(k); });
    }
    ~MemberThreads() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // fn(k) for every member k, concurrently; returns when all have
    void run(const std::function<void(uint32_t)>& fn) {
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            pending_ = (uint32_t)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

private:
    void loop(uint32_t k) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(uint32_t)>* f;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = fn_;
            }
            (*f)(k);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)>* fn_ = nullptr;
    uint32_t pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace

struct bt_group {
    std::vector<bt_ctx*> members;
    std::mutex mu;   // one batch at a time (each member serialises its own calls anyway)
    std::unique_ptr<MemberThreads> threads;   // members > 1
};

namespace {

constexpr uint32_t kTile = 64;

// What one packet costs a member: its staged header prefix (<= 128 B), its descriptor and
// its 96-B record (shard.py's cost model).
inline uint64_t packet_cost(uint32_t len) { return (uint64_t)std::min(len, 128u) + 8u + 96u; }

struct Range {
    uint32_t lo, hi;
};

std::vector<Range> split(const uint32_t* lens, uint32_t n, uint32_t parts) {
    std::vector<uint32_t> b(parts + 1, 0);
    bt_group_split(lens, n, parts, b.data());
    std::vector<Range> r(parts);
    for (uint32_t k = 0; k < parts; ++k) r[k] = {b[k], b[k + 1]};
    return r;
}

// Runs fn(k) for every member on its own thread; returns the first failure (with its
// message moved to this thread's bt_last_error).
template <class Fn>
int run_members(bt_group* g, Fn fn) {
    const uint32_t m = (uint32_t)g->members.size();
    if (m == 1) return fn(0u);   // one device: no thread
    std::vector<int> rc(m, BT_OK);
    std::vector<std::string> msg(m);
    g->threads->run([&](uint32_t k) {
        rc[k] = fn(k);
        if (rc[k]) msg[k] = bt_last_error();
    });
    for (uint32_t k = 0; k < m; ++k)
        if (rc[k]) return bt::set_error(rc[k], "group member %u (device %d): %s", k, bt::ctx_device(g->members[k]),
                                        msg[k].c_str());
    return BT_OK;
}

// One host batch over the group: frame(i) gives packet i's bytes and length.
template <class Frames>
int group_batch(bt_group* g, uint32_t n, const uint32_t* lens, Frames frames, bt_rec* records, uint64_t* verdict,
                uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    const uint32_t m = (uint32_t)g->members.size();
    const std::vector<Range> r = split(lens, n, m);
    std::vector<std::vector<uint32_t>> pidx(m);
    std::vector<uint32_t> npass(m, 0);
    const bool want_pass = pass_idx || n_pass;
    int rc = run_members(g, [&](uint32_t k) -> int {
        const uint32_t lo = r[k].lo, cnt = r[k].hi - r[k].lo;
        if (!cnt) return BT_OK;
        if (pass_idx) pidx[k].resize(cnt);
        return frames(g->members[k], lo, cnt, records ? records + lo : nullptr, verdict ? verdict + lo / kTile : nullptr,
                      decide ? decide + lo : nullptr, pass_idx ? pidx[k].data() : nullptr,
                      want_pass ? &npass[k] : nullptr);
    });
    if (rc) return rc;
    uint32_t at = 0;
    for (uint32_t k = 0; k < m; ++k) {
        if (pass_idx)
            for (uint32_t j = 0; j < npass[k]; ++j) pass_idx[at + j] = pidx[k][j] + r[k].lo;
        at += npass[k];
    }
    if (n_pass) *n_pass = at;
    return BT_OK;
}

}  // namespace

extern "C" {

int bt_group_split(const uint32_t* lens, uint32_t n, uint32_t parts, uint32_t* bounds) {
    if (!bounds || !parts || (n && !lens)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / zero parts");
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
        for (uint32_t i = t * kTile; i < e; ++i) run += packet_cost(lens[i]);
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

int bt_group_create(const int* devices, uint32_t n_devices, const bt_opts* opts, bt_group** out) {
    if (!out || !devices || !n_devices) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument / no devices");
    *out = nullptr;
    for (uint32_t i = 0; i < n_devices; ++i)
        for (uint32_t j = 0; j < i; ++j)
            if (devices[i] == devices[j] && !(opts && (opts->flags & BT_OPT_GROUP_SHARED_DEVICE)))
                return bt::set_error(BT_E_INVALID_ARGUMENT, "device %d listed twice (BT_OPT_GROUP_SHARED_DEVICE "
                                     "allows it, for tests on one GPU)", devices[i]);
    auto* g = new bt_group();
    for (uint32_t i = 0; i < n_devices; ++i) {
        bt_ctx* c = nullptr;
        const int rc = bt_create(devices[i], opts, &c);
        if (rc) {
            const std::string msg = bt_last_error();
            bt_group_destroy(g);
            return bt::set_error(rc, "group member %u (device %d): %s", i, devices[i], msg.c_str());
        }
        g->members.push_back(c);
    }
    if (n_devices > 1) g->threads = std::make_unique<MemberThreads>(n_devices);
    *out = g;
    return BT_OK;
}

void bt_group_destroy(bt_group* g) {
    if (!g) return;
    g->threads.reset();
    for (bt_ctx* c : g->members) bt_destroy(c);
    delete g;
}

uint32_t bt_group_size(const bt_group* g) { return g ? (uint32_t)g->members.size() : 0u; }

bt_ctx* bt_group_member(bt_group* g, uint32_t k) {
    return g && k < g->members.size() ? g->members[k] : nullptr;
}

int bt_group_filter_compile(bt_group* g, const bt_filter_desc* filters, uint32_t n) {
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    std::lock_guard<std::mutex> lk(g->mu);
    bt::CompiledProgram p;   // compiled once, installed on every device
    if (int rc = bt::compile_program(filters, n, bt::ctx_flags(g->members[0]), &p)) return rc;
    return run_members(g, [&](uint32_t k) { return bt::install_program(g->members[k], p); });
}

int bt_group_parse_filter(bt_group* g, const uint8_t* base, const bt_pkt_desc* desc, uint32_t n, bt_rec* records,
                          uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx, uint32_t* n_pass) {
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    if (n && (!base || !desc)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null packet buffer/descriptors");
    std::lock_guard<std::mutex> lk(g->mu);
    std::vector<uint32_t> lens(n);
    for (uint32_t i = 0; i < n; ++i) lens[i] = BT_DESC_LEN(desc[i]);
    return group_batch(g, n, lens.data(),
                       [&](bt_ctx* c, uint32_t lo, uint32_t cnt, bt_rec* r, uint64_t* v, uint8_t* d, uint32_t* p,
                           uint32_t* np) { return bt_parse_filter(c, base, desc + lo, cnt, r, v, d, p, np); },
                       records, verdict, decide, pass_idx, n_pass);
}

int bt_group_parse_filter_ptrs(bt_group* g, const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                               bt_rec* records, uint64_t* verdict, uint8_t* decide, uint32_t* pass_idx,
                               uint32_t* n_pass) {
    if (!g) return bt::set_error(BT_E_INVALID_ARGUMENT, "null group");
    if (n && (!frames || !lens)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null frame pointers/lengths");
    std::lock_guard<std::mutex> lk(g->mu);
    return group_batch(g, n, lens,
                       [&](bt_ctx* c, uint32_t lo, uint32_t cnt, bt_rec* r, uint64_t* v, uint8_t* d, uint32_t* p,
                           uint32_t* np) { return bt_parse_filter_ptrs(c, frames + lo, lens + lo, cnt, r, v, d, p, np); },
                       records, verdict, decide, pass_idx, n_pass);
}

}  // extern "C"
