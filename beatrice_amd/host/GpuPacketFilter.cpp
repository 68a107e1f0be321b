// GpuPacketFilter.cpp — see GpuPacketFilter.hpp. Reference behaviour cited as
// src/PacketFilter.cpp:<line> (Open-Sentra/beatrice).
#include "GpuPacketFilter.hpp"

#include "bt_slot_eval.h"

#include <algorithm>
#include <sys/mman.h>

#include <chrono>
#include <cerrno>
#include <cstdlib>
#include <exception>
#include <memory>
#include <regex>
#include <stdexcept>

namespace beatrice {
namespace gpu {

namespace {

const std::string kPassedReason = "Packet passed all filters";   // src/PacketFilter.cpp:102-105

uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

// A built-in slot on one packet: the kernels' own FilterIn / eval_slot (bt_slot_eval.h).
// 1 pass, 0 reject, 2 throw (PAYLOAD / HOST slots are the callers' before they get here).
int eval_builtin(const bt_filter_slot& s, const uint8_t* d, size_t len) {
    const uint32_t l = len > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)len;
    const bt::FilterIn x = bt::filter_in([d](uint32_t i) { return (uint32_t)d[i]; }, l);
    return (int)bt::eval_slot(s.kind, s.a, s.b, x);
}

// applyPayloadFilter (src/PacketFilter.cpp:288-321) for a non-empty, valid regex.
bool payload_match(const std::regex& re, const uint8_t* d, size_t len) {
    if (len < 34) return false;
    if (be16(d + 12) != 0x0800) return false;
    const size_t payloadOffset = 14 + (size_t)(d[14] & 0x0F) * 4;
    if (len <= payloadOffset) return false;
    std::string payload(reinterpret_cast<const char*>(d + payloadOffset), std::min(len - payloadOffset, size_t(100)));
    try {
        return std::regex_search(payload, re);
    } catch (const std::regex_error&) {
        return false;
    }
}

}  // namespace

std::vector<int> GpuPacketFilter::devicesFromEnv(int fallback) {
    std::vector<int> d;
    if (const char* e = std::getenv("BEATRICE_GPU_DEVICES")) {
        std::string s(e);
        size_t at = 0;
        while (at < s.size()) {
            const size_t comma = s.find(',', at);
            const std::string tok = s.substr(at, comma == std::string::npos ? std::string::npos : comma - at);
            if (!tok.empty()) {
                char* end = nullptr;
                errno = 0;
                const long v = std::strtol(tok.c_str(), &end, 10);
                if (end == tok.c_str() || *end || errno || v < 0 || v > 1 << 20)
                    throw std::runtime_error("GpuPacketFilter: BEATRICE_GPU_DEVICES: bad device \"" + tok + "\"");
                d.push_back((int)v);
            }
            if (comma == std::string::npos) break;
            at = comma + 1;
        }
    }
    if (d.empty()) d.push_back(fallback);
    return d;
}

GpuPacketFilter::GpuPacketFilter(int device, const bt_opts* opts) {
    // an explicit device is that device alone; only the default reads the environment
    open(device >= 0 ? std::vector<int>{device} : devicesFromEnv(0), opts);
}

GpuPacketFilter::GpuPacketFilter(const std::vector<int>& devices, const bt_opts* opts) { open(devices, opts); }

void GpuPacketFilter::open(const std::vector<int>& devices, const bt_opts* opts) {
    if (const char* e = std::getenv("BEATRICE_GPU_HOST_BELOW")) hostBelow_.store(std::strtoull(e, nullptr, 10));
    if (devices.empty()) throw std::invalid_argument("GpuPacketFilter: empty device list");
    if (bt_abi_version() < BT_ABI_VERSION)   // a libbeatrice_gpu.so older than this header
        throw std::runtime_error("GpuPacketFilter: libbeatrice_gpu.so has C-ABI version " +
                                 std::to_string(bt_abi_version()) + ", this adapter needs " +
                                 std::to_string(BT_ABI_VERSION));
    // a device listed more than once is that many lanes on it (contexts with their own staging,
    // streams and host threads): concurrent callers' device passes then overlap on the device
    bt_opts o{};
    if (opts) o = *opts;
    for (size_t i = 0; i < devices.size(); ++i)
        for (size_t j = 0; j < i; ++j)
            if (devices[i] == devices[j]) o.flags |= BT_OPT_GROUP_SHARED_DEVICE;
    if (bt_group_create(devices.data(), (uint32_t)devices.size(), &o, &group_) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    ctx_ = bt_group_member(group_, 0);
}

GpuPacketFilter::~GpuPacketFilter() { bt_group_destroy(group_); }

Result<void> GpuPacketFilter::addFilter(const std::string& name, const FilterConfig& config) {
    std::unique_lock<std::shared_mutex> lock(filtersMutex_);   // :19-31
    if (filters_.find(name) != filters_.end())
        return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Filter already exists: " + name);
    FilterEntry entry;
    entry.config = config;
    filters_[name] = entry;
    dirty_ = true;
    updateNeedsPackets();
    return Result<void>::success();
}

Result<void> GpuPacketFilter::removeFilter(const std::string& name) {
    std::unique_lock<std::shared_mutex> lock(filtersMutex_);   // :33-43
    auto it = filters_.find(name);
    if (it == filters_.end()) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Filter not found: " + name);
    filters_.erase(it);
    dirty_ = true;
    updateNeedsPackets();
    return Result<void>::success();
}

Result<void> GpuPacketFilter::setFilterEnabled(const std::string& name, bool enabled) {
    std::unique_lock<std::shared_mutex> lock(filtersMutex_);   // :45-55
    auto it = filters_.find(name);
    if (it == filters_.end()) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Filter not found: " + name);
    it->second.config.enabled = enabled;
    dirty_ = true;
    updateNeedsPackets();
    return Result<void>::success();
}

Result<void> GpuPacketFilter::setCustomFilter(const std::string& name, std::function<bool(const Packet&)> filterFunc) {
    std::unique_lock<std::shared_mutex> lock(filtersMutex_);   // :155-166
    auto it = filters_.find(name);
    if (it == filters_.end()) return Result<void>::error(ErrorCode::INVALID_ARGUMENT, "Filter not found: " + name);
    it->second.customFunc = std::move(filterFunc);
    dirty_ = true;
    updateNeedsPackets();
    return Result<void>::success();
}

void GpuPacketFilter::updateNeedsPackets() {
    bool any = false;
    for (const auto& [name, entry] : filters_)
        if (entry.config.enabled && entry.config.type == FilterType::CUSTOM && entry.customFunc) any = true;
    needsPackets_.store(any, std::memory_order_relaxed);
}

std::vector<std::string> GpuPacketFilter::getActiveFilters() const {
    std::shared_lock<std::shared_mutex> lock(filtersMutex_);   // :132-143
    std::vector<std::string> active;
    for (const auto& [name, entry] : filters_)
        if (entry.config.enabled) active.push_back(name);
    return active;
}

GpuPacketFilter::FilterStats GpuPacketFilter::getStats() const {
    std::lock_guard<std::mutex> lock(statsMutex_);
    return stats_;
}

void GpuPacketFilter::resetStats() {
    std::lock_guard<std::mutex> lock(statsMutex_);
    stats_ = FilterStats{};
}

void GpuPacketFilter::compileLocked() {
    // The reference's own ordering (:63-73): enabled entries in unordered_map iteration
    // order, then std::sort by priority (descending). Same container, same calls.
    std::vector<std::pair<std::string, FilterEntry*>> sortedFilters;
    for (auto& [name, entry] : filters_)
        if (entry.config.enabled) sortedFilters.emplace_back(name, &entry);
    std::sort(sortedFilters.begin(), sortedFilters.end(),
              [](const auto& a, const auto& b) { return a.second->config.priority > b.second->config.priority; });
    std::vector<bt_filter_desc> descs(sortedFilters.size());
    for (size_t i = 0; i < sortedFilters.size(); ++i) {
        const FilterConfig& c = sortedFilters[i].second->config;
        descs[i].type = static_cast<int32_t>(c.type);
        descs[i].expression = c.expression.c_str();
        descs[i].enabled = 1;
        descs[i].priority = c.priority;
        descs[i].has_custom_func = sortedFilters[i].second->customFunc ? 1 : 0;
    }
    if (bt_group_filter_compile(group_, descs.data(), (uint32_t)descs.size()) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    std::vector<bt_filter_slot> slots(BT_MAX_FILTERS);
    uint32_t m = 0;
    bt_filter_program(ctx_, slots.data(), BT_MAX_FILTERS, &m);
    program_.clear();
    rejectReason_.clear();
    uint32_t pool = 0;
    if (bt_filter_dfa_pool(ctx_, nullptr, 0, &pool) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    dfaPool_.assign(pool, 0);
    if (pool && bt_filter_dfa_pool(ctx_, dfaPool_.data(), pool, &pool) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    for (uint32_t k = 0; k < m; ++k) {
        const auto& src = sortedFilters[slots[k].source_index];
        program_.push_back(Slot{src.first, src.second, slots[k]});
        rejectReason_.push_back("Filter " + src.first + " rejected packet");   // :106-110
    }
    dirty_ = false;
}

std::shared_lock<std::shared_mutex> GpuPacketFilter::lockProgram() {
    for (;;) {
        {
            std::shared_lock<std::shared_mutex> rd(filtersMutex_);
            if (!dirty_) return rd;
        }
        std::unique_lock<std::shared_mutex> wr(filtersMutex_);
        if (dirty_) compileLocked();
    }
}

std::vector<std::string> GpuPacketFilter::evaluationOrder() {
    const auto lock = lockProgram();
    std::vector<std::string> names;
    for (const auto& s : program_) names.push_back(s.name);
    return names;
}

void GpuPacketFilter::rethrow(const Slot& s) const {
    // std::stoi's own exceptions (libstdc++: what() == "stoi")
    if (s.compiled.throw_kind == 2) throw std::out_of_range("stoi");
    throw std::invalid_argument("stoi");
}

uint32_t GpuPacketFilter::evalFrame(const uint8_t* d, size_t len) const {
    for (uint32_t s = 0; s < program_.size(); ++s) {
        const bt_filter_slot& c = program_[s].compiled;
        int r;
        if (c.kind == BT_K_HOST) return (BT_DECIDE_HOST << 6) | s;
        if (c.kind == BT_K_PAYLOAD) r = bt_payload_dfa_eval(dfaPool_.data() + c.a, d, (uint32_t)len) ? 1 : 0;
        else r = eval_builtin(c, d, len);
        if (r == 0) return (BT_DECIDE_REJECT << 6) | s;
        if (r == 2) return (BT_DECIDE_THROW << 6) | s;
    }
    return (BT_DECIDE_PASS << 6) | (program_.empty() ? 0u : (uint32_t)program_.size() - 1);
}

uint32_t GpuPacketFilter::resolveHost(const Packet& p, uint32_t first) {
    const uint8_t* d = p.data();
    const size_t len = p.length();
    for (uint32_t s = first; s < program_.size(); ++s) {
        const Slot& sl = program_[s];
        int r;
        if (sl.compiled.kind == BT_K_PAYLOAD) {   // the compiled DFA: regex_search's result
            r = bt_payload_dfa_eval(dfaPool_.data() + sl.compiled.a, d, (uint32_t)len) ? 1 : 0;
        } else if (sl.compiled.kind != BT_K_HOST) {
            r = eval_builtin(sl.compiled, d, len);
        } else if (sl.entry->config.type == FilterType::CUSTOM) {
            r = sl.entry->customFunc ? (sl.entry->customFunc(p) ? 1 : 0) : 1;   // :323-328
        } else {
            // PAYLOAD: the regex is valid (compile checked it); the reference constructs
            // it per packet, which cannot change regex_search's result.
            thread_local std::string last_expr;
            thread_local std::shared_ptr<std::regex> re;
            if (!re || last_expr != sl.entry->config.expression) {
                last_expr = sl.entry->config.expression;
                re = std::make_shared<std::regex>(last_expr);
            }
            r = payload_match(*re, d, len) ? 1 : 0;
        }
        if (r == 0) return (BT_DECIDE_REJECT << 6) | s;
        if (r == 2) return (BT_DECIDE_THROW << 6) | s;
    }
    return (BT_DECIDE_PASS << 6) | (program_.empty() ? 0u : (uint32_t)program_.size() - 1);
}

namespace {

// fn(lo, hi) over [0, n) split across the group's host threads (bt_group_host_parallel: every
// member's pool, so a group's whole host budget works on the batch's results).
template <class Fn>
void parallel_ranges(bt_group* group, size_t n, Fn&& fn) {
    struct U {
        Fn* fn;
        size_t n;
    } u{&fn, n};
    bt_group_host_parallel(group, [](void* p, uint32_t w, uint32_t T) {
        auto* x = static_cast<U*>(p);
        const size_t lo = x->n * w / T, hi = x->n * (w + 1) / T;
        if (lo < hi) (*x->fn)(lo, hi);
    }, &u);
}

// A batch's FilterResults are 136 B each (two strings and a hash map): 570 MB for 4M
// packets, whose first-touch page faults are most of their construction time. For large
// results ask for transparent huge pages on the (still unconstructed) storage.
void advise_huge(void* p, size_t bytes) {
    constexpr uintptr_t kHuge = uintptr_t(2) << 20;
    if (bytes < (size_t(64) << 20)) return;
    const uintptr_t a = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1), e = ((uintptr_t)p + bytes) & ~(kHuge - 1);
    if (e > a) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

// Faults the (still unconstructed) storage in on the host threads, one write per 4 KiB
// page, so the serial default construction that follows runs on resident memory instead
// of taking every page fault (and the zeroing behind it) on the calling thread.
void prefault(bt_group* group, void* p, size_t bytes) {
    if (bytes < (size_t(16) << 20)) return;
    auto* b = static_cast<volatile uint8_t*>(p);
    parallel_ranges(group, (bytes + 4095) / 4096, [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; ++k) b[k * 4096] = 0;
    });
}

// Counts a batch call in flight for its duration.
struct InFlight {
    std::atomic<int>& n;
    explicit InFlight(std::atomic<int>& c) : n(c) { n.fetch_add(1, std::memory_order_relaxed); }
    ~InFlight() { n.fetch_sub(1, std::memory_order_relaxed); }
};

}  // namespace

template <class Fn>
void GpuPacketFilter::forRanges(size_t n, Fn&& fn) {
    // small ranges on the caller: waking the host pool costs ~10-15 us, more than the work
    // (classify of 1-256 packets spent 15 us per call there, profiles/r04/surfaces)
    constexpr size_t kInlineBelow = 8192;
    if (n < kInlineBelow || inFlight_.load(std::memory_order_relaxed) > 1) {
        if (n) fn(size_t(0), n);
    } else {
        parallel_ranges(group_, n, [&](size_t lo, size_t hi) { fn(lo, hi); });
    }
}

void GpuPacketFilter::setTiming(double device_s, double host_s) {
    std::lock_guard<std::mutex> lock(statsMutex_);
    timing_.device_s = device_s;
    timing_.host_s = host_s;
}

void GpuPacketFilter::runFrames(const uint8_t* const* frames, const uint32_t* lens, uint32_t n,
                                std::vector<uint8_t>& decide, std::vector<bt_rec>* records) {
    decide.resize(n);
    if (!records && hostSmall(n)) {   // a device round trip costs more than the batch
        for (uint32_t i = 0; i < n; ++i) decide[i] = (uint8_t)evalFrame(frames[i], lens[i]);
        return;
    }
    if (records) records->resize(n);
    if (bt_group_parse_filter_ptrs(group_, frames, lens, n, records ? records->data() : nullptr, nullptr,
                                   decide.data(), nullptr, nullptr) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
}

void GpuPacketFilter::runBatch(const std::vector<Packet>& packets, std::vector<uint8_t>& decide,
                               std::vector<bt_rec>* records) {
    const uint32_t n = (uint32_t)packets.size();
    // the gather list, per calling thread and reused across its batches (written through
    // plain pointers: a thread_local named inside the lambda would be the pool thread's own)
    thread_local std::vector<const uint8_t*> ptrs;
    thread_local std::vector<uint32_t> lens;
    ptrs.resize(n);
    lens.resize(n);
    const uint8_t** P = ptrs.data();
    uint32_t* L = lens.data();
    forRanges(n, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            P[i] = packets[i].data();
            L[i] = (uint32_t)packets[i].length();
        }
    });
    runFrames(P, L, n, decide, records);
}

// The host's pass over a batch's decisions, in packet order: PAYLOAD / CUSTOM slots the
// device handed over are resumed here (serially: a CUSTOM callback is the caller's code),
// and the stats are tallied per deciding slot, to be applied once (flushTally). `onThrow`
// decides what a throwing packet does: stop the scan there (applyFilters / classify, which
// rethrow after the earlier packets' stats, as the reference's per-packet loop does) or
// record it and go on (classifyPerPacket).
struct GpuPacketFilter::Tally {
    uint64_t counted = 0, passed = 0;
    std::vector<uint64_t> rejected;
    size_t stop = 0;        // packets scanned (== n unless a throw stopped the scan)
    bool threw = false;     // packet `stop` throws: its filter's std::stoi exception ...
    std::exception_ptr ex;  // ... or the exception its CUSTOM callback threw
    // after the stats of the packets before it are applied, as the reference's per-packet
    // loop leaves them (src/PacketFilter.cpp:116, 121-130)
    void rethrowIfAny(const GpuPacketFilter& f, const uint8_t* decide) const {
        if (ex) std::rethrow_exception(ex);
        if (threw) f.rethrow(f.program_[decide[stop] & 63u]);
    }
};

// The same pass over a large batch on the context's host threads, when the device decided
// every packet (no HOST code; a part that meets one makes the caller fall back to the serial
// scan): each part tallies its range up to its first throw, and the parts are joined in
// order up to the first part that threw. Returns false to fall back. (The serial pass took
// 3.3 ns per packet, more than the device pass of a one-caller classify.)
bool GpuPacketFilter::scanParallel(size_t n, const uint8_t* decide, std::vector<uint32_t>* pass_idx,
                                   std::vector<uint32_t>* error_idx, Tally& t) {
    struct Part {
        uint64_t counted = 0, passed = 0;
        std::vector<uint64_t> rejected;
        size_t stop = 0;
        bool threw = false, host = false;
        std::vector<uint32_t> pass, err;
    };
    const size_t slots = program_.size() + 1;
    constexpr uint32_t kParts = 16;
    std::vector<Part> parts(kParts);
    struct U {
        const uint8_t* decide;
        size_t n, slots;
        bool want_pass, errors;
        std::vector<Part>* parts;
    } u{decide, n, slots, pass_idx != nullptr, error_idx != nullptr, &parts};
    auto run = [](void* x, uint32_t w, uint32_t T) {
        auto* u = static_cast<U*>(x);
        for (uint32_t k = w; k < kParts; k += T) {
            Part& p = (*u->parts)[k];
            p.rejected.assign(u->slots, 0);
            const size_t lo = u->n * k / kParts, hi = u->n * (k + 1) / kParts;
            p.stop = hi;
            for (size_t i = lo; i < hi; ++i) {
                const uint32_t d = u->decide[i], code = d >> 6;
                if (code == BT_DECIDE_HOST) {
                    p.host = true;
                    return;
                }
                if (code == BT_DECIDE_THROW) {
                    if (u->errors) {
                        p.err.push_back((uint32_t)i);
                        continue;
                    }
                    p.stop = i;
                    p.threw = true;
                    break;
                }
                ++p.counted;
                if (code == BT_DECIDE_PASS) {
                    ++p.passed;
                    if (u->want_pass) p.pass.push_back((uint32_t)i);
                } else {
                    ++p.rejected[d & 63u];
                }
            }
        }
    };
    if (bt_group_host_parallel(group_, run, &u) != BT_OK) return false;
    for (const Part& p : parts)
        if (p.host) return false;
    t.rejected.assign(slots, 0);
    for (const Part& p : parts) {
        t.counted += p.counted;
        t.passed += p.passed;
        for (size_t s = 0; s < slots; ++s) t.rejected[s] += p.rejected[s];
        if (pass_idx) pass_idx->insert(pass_idx->end(), p.pass.begin(), p.pass.end());
        if (error_idx) error_idx->insert(error_idx->end(), p.err.begin(), p.err.end());
        if (p.threw) {   // the reference's loop stops at the first throwing packet
            t.stop = p.stop;
            t.threw = true;
            return true;
        }
    }
    t.stop = n;
    return true;
}

template <class PacketAt>
GpuPacketFilter::Tally GpuPacketFilter::scan(size_t n, PacketAt packet, uint8_t* decide,
                                            std::vector<uint32_t>* pass_idx, std::vector<uint32_t>* error_idx,
                                            uint64_t* verdict) {
    Tally t;
    if (n >= 65536 && inFlight_.load(std::memory_order_relaxed) == 1) {
        if (scanParallel(n, decide, pass_idx, error_idx, t)) return t;
        t = Tally{};   // a HOST code: the serial pass resumes those packets in order
        if (pass_idx) pass_idx->clear();
        if (error_idx) error_idx->clear();
    }
    t.rejected.assign(program_.size() + 1, 0);
    std::unique_lock<std::mutex> host(hostMutex_, std::defer_lock);   // taken at the first host slot
    for (size_t i = 0; i < n; ++i) {
        uint32_t d = decide[i];
        if ((d >> 6) == BT_DECIDE_HOST) {
            if (!host.owns_lock()) host.lock();
            if (error_idx) {
                try {
                    d = resolveHost(packet(i), d & 63u);
                } catch (...) {   // a CUSTOM callback threw for this packet
                    d = (BT_DECIDE_THROW << 6) | (d & 63u);
                }
            } else {
                try {
                    d = resolveHost(packet(i), d & 63u);
                } catch (...) {
                    t.stop = i;
                    t.ex = std::current_exception();
                    return t;
                }
            }
            decide[i] = (uint8_t)d;
            if (verdict && (d >> 6) == BT_DECIDE_PASS) verdict[i / 64] |= 1ull << (i % 64);
        }
        const uint32_t code = d >> 6, slot = d & 63u;
        if (code == BT_DECIDE_THROW) {
            if (!error_idx) {
                t.stop = i;
                t.threw = true;
                return t;
            }
            error_idx->push_back((uint32_t)i);
            continue;
        }
        ++t.counted;
        if (code == BT_DECIDE_PASS) {
            ++t.passed;
            if (pass_idx) pass_idx->push_back((uint32_t)i);
        } else {
            ++t.rejected[slot];
        }
    }
    t.stop = n;
    return t;
}

// updateStats (src/PacketFilter.cpp:374-386) for every counted packet of the tally at once.
void GpuPacketFilter::flushTally(const Tally& t, std::chrono::microseconds per) {
    std::lock_guard<std::mutex> lock(statsMutex_);
    stats_.packetsProcessed += t.counted;
    stats_.packetsPassed += t.passed;
    stats_.packetsDropped += t.counted - t.passed;
    stats_.totalProcessingTime += per * (int64_t)t.counted;
    if (program_.empty()) {   // FilterResult::filterName stays "" (:102-111)
        if (t.counted) stats_.filterCounts[""] += t.counted;
        return;
    }
    if (t.passed) stats_.filterCounts[program_.back().name] += t.passed;
    for (size_t s = 0; s < program_.size(); ++s)
        if (t.rejected[s]) stats_.filterCounts[program_[s].name] += t.rejected[s];
}

std::vector<GpuPacketFilter::FilterResult> GpuPacketFilter::applyFilters(const std::vector<Packet>& packets) {
    std::vector<FilterResult> results;
    const auto lock = lockProgram();
    const InFlight busy(inFlight_);
    if (packets.empty()) return results;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint8_t> decide;
    runBatch(packets, decide);
    const auto per = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0) /
                     (int64_t)packets.size();
    const auto t1 = std::chrono::steady_clock::now();
    const double device_s = std::chrono::duration<double>(t1 - t0).count();
    const Tally t =
        scan(packets.size(), [&](size_t i) -> const Packet& { return packets[i]; }, decide.data(), nullptr, nullptr);
    // The FilterResults of the packets before any throw (:102-111), built on the host
    // threads from per-slot strings made once per program: the reference's vector is the
    // result either way, its strings are copied rather than concatenated per packet.
    results.reserve(t.stop);
    advise_huge(results.data(), t.stop * sizeof(FilterResult));
    if (inFlight_.load(std::memory_order_relaxed) == 1) prefault(group_, results.data(), t.stop * sizeof(FilterResult));
    results.resize(t.stop);
    forRanges(t.stop, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            FilterResult& r = results[i];
            const uint32_t code = decide[i] >> 6, slot = decide[i] & 63u;
            r.passed = code == BT_DECIDE_PASS;
            if (!program_.empty()) {
                if (r.passed) {
                    r.filterName = program_.back().name;
                    r.reason = kPassedReason;
                } else {
                    r.filterName = program_[slot].name;
                    r.reason = rejectReason_[slot];
                }
            }
            r.processingTime = per;
        }
    });
    flushTally(t, per);
    t.rethrowIfAny(*this, decide.data());   // earlier packets are counted
    setTiming(device_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    return results;
}

// updateStats (src/PacketFilter.cpp:374-386) for one packet.
void GpuPacketFilter::tallyOne(uint32_t d, std::chrono::microseconds t) {
    std::lock_guard<std::mutex> lock(statsMutex_);
    ++stats_.packetsProcessed;
    const bool pass = (d >> 6) == BT_DECIDE_PASS;
    if (pass) ++stats_.packetsPassed;
    else ++stats_.packetsDropped;
    stats_.totalProcessingTime += t;
    if (program_.empty()) {
        ++stats_.filterCounts[""];
        return;
    }
    ++stats_.filterCounts[pass ? program_.back().name : program_[d & 63u].name];
}

// One packet (src/PacketFilter.cpp:57-119): decided on the calling thread with the compiled
// program; the device would cost a round trip for one packet.
GpuPacketFilter::FilterResult GpuPacketFilter::applyFilters(const Packet& packet) {
    if (!hostSmall(1)) return applyFilters(std::vector<Packet>{packet}).front();
    const auto lock = lockProgram();
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t d = evalFrame(packet.data(), packet.length());
    if ((d >> 6) == BT_DECIDE_HOST) {
        std::lock_guard<std::mutex> host(hostMutex_);   // CUSTOM callbacks one at a time, as the reference
        d = resolveHost(packet, d & 63u);                // a throwing callback propagates, no stats (:116)
    }
    const uint32_t code = d >> 6, slot = d & 63u;
    if (code == BT_DECIDE_THROW) rethrow(program_[slot]);   // std::stoi's exception, before updateStats
    FilterResult r;
    r.passed = code == BT_DECIDE_PASS;
    if (!program_.empty()) {
        if (r.passed) {
            r.filterName = program_.back().name;
            r.reason = kPassedReason;
        } else {
            r.filterName = program_[slot].name;
            r.reason = rejectReason_[slot];
        }
    }
    r.processingTime = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0);
    tallyOne(d, r.processingTime);
    return r;
}

GpuPacketFilter::Verdicts GpuPacketFilter::classify(const std::vector<Packet>& packets) {
    Verdicts v;
    const auto lock = lockProgram();
    const InFlight busy(inFlight_);
    if (packets.empty()) return v;
    const auto t0 = std::chrono::steady_clock::now();
    runBatch(packets, v.decide);
    const auto per = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0) /
                     (int64_t)packets.size();
    const auto t1 = std::chrono::steady_clock::now();
    const double device_s = std::chrono::duration<double>(t1 - t0).count();
    const Tally t =
        scan(packets.size(), [&](size_t i) -> const Packet& { return packets[i]; }, v.decide.data(), &v.pass_idx, nullptr);
    flushTally(t, per);
    t.rethrowIfAny(*this, v.decide.data());
    setTiming(device_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    return v;
}

GpuPacketFilter::Verdicts GpuPacketFilter::classifyPerPacket(const std::vector<Packet>& packets, bool withRecords) {
    Verdicts v;
    const auto lock = lockProgram();
    const InFlight busy(inFlight_);
    if (packets.empty()) return v;
    const auto t0 = std::chrono::steady_clock::now();
    runBatch(packets, v.decide, withRecords ? &v.records : nullptr);
    const auto per = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0) /
                     (int64_t)packets.size();
    const auto t1 = std::chrono::steady_clock::now();
    const double device_s = std::chrono::duration<double>(t1 - t0).count();
    const Tally t = scan(packets.size(), [&](size_t i) -> const Packet& { return packets[i]; }, v.decide.data(),
                         &v.pass_idx, &v.error_idx);
    flushTally(t, per);
    setTiming(device_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    return v;
}

uint32_t GpuPacketFilter::stagedPrefixBytes(bool withRecords) {
    const auto lock = lockProgram();
    uint32_t b = 0;
    if (bt_host_stage_bytes(ctx_, withRecords ? 1 : 0, &b) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    return b;
}

GpuPacketFilter::Verdicts GpuPacketFilter::classifyPerPacket(const uint8_t* const* frames, const uint32_t* lens,
                                                             size_t n, bool withRecords,
                                                             const std::function<Packet(size_t)>& packetOf,
                                                             uint32_t readable) {
    Verdicts v;
    const auto lock = lockProgram();
    const InFlight busy(inFlight_);
    if (!n) return v;
    if (!frames || !lens || !packetOf) throw std::invalid_argument("GpuPacketFilter::classifyPerPacket: null argument");
    // prefixes too short for the program under this lock (a GPU PAYLOAD slot reads the
    // payload window): the packets' own bytes instead
    std::vector<Packet> own;
    std::vector<const uint8_t*> ownFrames;
    if (readable) {
        uint32_t need = 0;
        if (bt_host_stage_bytes(ctx_, withRecords ? 1 : 0, &need) != BT_OK)
            throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
        if (readable < need) {
            own.reserve(n);
            ownFrames.resize(n);
            for (size_t i = 0; i < n; ++i) {
                own.push_back(packetOf(i));
                ownFrames[i] = own.back().data();
            }
            frames = ownFrames.data();
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    runFrames(frames, lens, (uint32_t)n, v.decide, withRecords ? &v.records : nullptr);
    const auto per = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0) /
                     (int64_t)n;
    const auto t1 = std::chrono::steady_clock::now();
    const double device_s = std::chrono::duration<double>(t1 - t0).count();
    const Tally t = scan(n, [&](size_t i) { return packetOf(i); }, v.decide.data(), &v.pass_idx, &v.error_idx);
    flushTally(t, per);
    setTiming(device_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    return v;
}

std::vector<uint32_t> GpuPacketFilter::classifyMapped(const bt_batch& batch, const bt_outputs& out,
                                                     const std::function<Packet(uint32_t)>& packetOf) {
    std::vector<uint32_t> pass;
    const auto lock = lockProgram();
    const InFlight busy(inFlight_);
    if (!batch.n) return pass;
    if (!out.decide) throw std::invalid_argument("GpuPacketFilter::classifyMapped: decide required");
    const auto t0 = std::chrono::steady_clock::now();
    bt_outputs o = out;   // the pass list comes from the host's scan (after host slots)
    o.pass_idx = nullptr;
    o.n_pass = nullptr;
    if (bt_group_parse_filter_mapped(group_, &batch, &o) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter: ") + bt_last_error());
    const auto per = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0) /
                     (int64_t)batch.n;
    const auto t1 = std::chrono::steady_clock::now();
    const double device_s = std::chrono::duration<double>(t1 - t0).count();
    const Tally t = scan(batch.n, [&](size_t i) { return packetOf((uint32_t)i); }, out.decide, &pass, nullptr,
                         out.verdict);
    flushTally(t, per);
    t.rethrowIfAny(*this, out.decide);
    setTiming(device_s, std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    return pass;
}

void GpuPacketFilter::registerHost(void* p, size_t bytes) {
    if (bt_group_host_register(group_, p, bytes) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter::registerHost: ") + bt_last_error());
}

void GpuPacketFilter::unregisterHost(void* p) {
    if (bt_group_host_unregister(group_, p) != BT_OK)
        throw std::runtime_error(std::string("GpuPacketFilter::unregisterHost: ") + bt_last_error());
}

}  // namespace gpu
}  // namespace beatrice
