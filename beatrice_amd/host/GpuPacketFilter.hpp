// GpuPacketFilter.hpp — drop-in replacement for beatrice::PacketFilter
// (reference include/beatrice/PacketFilter.hpp:15-94) whose per-packet work runs on
// the MI355X through the C-ABI in include/beatrice_gpu.h.
//
// Same public interface, same nested types (it re-uses the reference's own
// FilterConfig / FilterResult / FilterStats / FilterType), same observable results:
//   * filters live in an std::unordered_map<std::string, ...> updated with the same
//     operations as the reference, and are ordered with the same std::sort call
//     (src/PacketFilter.cpp:63-73), so ties on priority resolve exactly as there;
//   * FilterResult.passed / filterName / reason match the reference (:102-111);
//   * an expression the reference's std::stoi would reject rethrows the same
//     std::invalid_argument / std::out_of_range at the same packet, after the stats
//     of the packets before it were updated (:116);
//   * PAYLOAD (std::regex) and CUSTOM (std::function) filters are evaluated here on
//     the host, with the reference's semantics, for the packets that reach them.
// processingTime is the amortised batch time (the reference's value is a wall clock).
// Threads: batch calls from several threads run concurrently on one filter (the compiled
// program is shared and immutable while they run; the device pass is serialised per
// device, each caller builds its own results); addFilter / removeFilter / setFilterEnabled
// / setCustomFilter wait for the calls in flight, as the reference's filtersMutex_ makes
// them (src/PacketFilter.cpp:19-61), and CUSTOM / PAYLOAD host resumption stays serial,
// as in the reference, which holds that mutex around every callback.
// Several devices: a device list (or BEATRICE_GPU_DEVICES=0,1,... for the default
// constructor) makes the filter drive a bt_group — the program compiled once, every batch
// split across the devices (include/beatrice_gpu.h, "several devices in one process").
#pragma once

#include <cstdint>
#include <functional>
#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "beatrice/PacketFilter.hpp"
#include "beatrice_gpu.h"

namespace beatrice {
namespace gpu {

class GpuPacketFilter {
public:
    using FilterType = beatrice::PacketFilter::FilterType;
    using FilterConfig = beatrice::PacketFilter::FilterConfig;
    using FilterResult = beatrice::PacketFilter::FilterResult;
    using FilterStats = beatrice::PacketFilter::FilterStats;

    // Throws std::runtime_error when no MI355X is available (no CPU fallback). device >= 0
    // drives that device alone; the default (kEnvDevices) drives BEATRICE_GPU_DEVICES (e.g.
    // "0,1,2,3") when set, else device 0.
    static constexpr int kEnvDevices = -1;
    explicit GpuPacketFilter(int device = kEnvDevices, const bt_opts* opts = nullptr);
    explicit GpuPacketFilter(const std::vector<int>& devices, const bt_opts* opts = nullptr);
    ~GpuPacketFilter();
    GpuPacketFilter(const GpuPacketFilter&) = delete;
    GpuPacketFilter& operator=(const GpuPacketFilter&) = delete;

    Result<void> addFilter(const std::string& name, const FilterConfig& config);
    Result<void> removeFilter(const std::string& name);
    Result<void> setFilterEnabled(const std::string& name, bool enabled);
    FilterResult applyFilters(const Packet& packet);
    std::vector<FilterResult> applyFilters(const std::vector<Packet>& packets);
    std::vector<std::string> getActiveFilters() const;
    FilterStats getStats() const;
    void resetStats();
    Result<void> setCustomFilter(const std::string& name, std::function<bool(const Packet&)> filterFunc);

    // GPU-native batch form: decision bytes (BT_DECIDE_*) with host-side filters already
    // resolved, plus the ordered indices of passing packets. Updates stats like
    // applyFilters; throws like it.
    struct Verdicts {
        std::vector<uint8_t> decide;     // (code << 6) | slot
        std::vector<uint32_t> pass_idx;  // ascending
        std::vector<uint32_t> error_idx; // classifyPerPacket only: packets whose evaluation threw
        std::vector<bt_rec> records;     // withRecords: each packet's parse record, from the same
                                         // kernel pass (the reference's parsePacket per walked layer)
    };
    Verdicts classify(const std::vector<Packet>& packets);

    // The same batch with the exceptions attributed per packet, as a per-packet caller
    // sees them: PluginManager::processPacket catches a plugin's exception for each
    // packet and goes on with the next one (src/PluginManager.cpp:158-171). A packet whose
    // evaluation would throw (a std::stoi expression past its gates, or a throwing CUSTOM
    // callback) is listed in error_idx with decide code BT_DECIDE_THROW and, as in the
    // reference, does not update the stats; every other packet is classified and counted.
    // Never throws for a filter; throws std::runtime_error if the device fails.
    // withRecords: the same kernel pass also parses every packet (Verdicts::records).
    Verdicts classifyPerPacket(const std::vector<Packet>& packets, bool withRecords = false);
    // The same over frames held by the caller (n pointers and lengths, e.g. a batch that keeps
    // only each Packet's bytes alive); packetOf(i) gives packet i for the host-side filters
    // (PAYLOAD regexes outside the GPU subset, CUSTOM callbacks), only for packets that reach one.
    // `readable` (0 = whole frames): frames[i] may hold only the first `readable` bytes of
    // packet i (lens[i] stays its true length), e.g. prefixes packed when the packets
    // arrived; enough when readable >= stagedPrefixBytes(withRecords), otherwise the call
    // reads the packets' own bytes through packetOf.
    Verdicts classifyPerPacket(const uint8_t* const* frames, const uint32_t* lens, size_t n, bool withRecords,
                               const std::function<Packet(size_t)>& packetOf, uint32_t readable = 0);
    // The bytes of each frame a batch call reads with the current program (bt_host_stage_bytes).
    uint32_t stagedPrefixBytes(bool withRecords);

    // Zero-copy form over frames in host memory every device of the filter reads in place (a
    // capture ring, an AF_XDP UMEM), registered once with registerHost. `batch` and `out` hold
    // HOST addresses: batch.base / batch.desc and out.decide (required) / out.verdict /
    // out.records must lie in registered ranges. The batch is split across the filter's
    // devices, each reading its range over its own PCIe link
    // (bt_group_parse_filter_mapped); then PAYLOAD / CUSTOM slots are resolved with
    // packetOf(i) (out.decide and out.verdict updated), the stats updated, and it throws like
    // classify. Returns the pass indices, ascending.
    std::vector<uint32_t> classifyMapped(const bt_batch& batch, const bt_outputs& out,
                                         const std::function<Packet(uint32_t)>& packetOf);
    // Page-locks a host range and maps it into every device of the filter
    // (bt_group_host_register); throws std::runtime_error. unregisterHost waits for the devices.
    void registerHost(void* p, size_t bytes);
    void unregisterHost(void* p);

    // Where the last batch call's time went (the latest to finish, when several threads call): the device pass (host gather, H2D, kernels,
    // D2H over every device of the group) and the host's work after it (PAYLOAD / CUSTOM
    // resumption, FilterResults, stats).
    struct BatchTiming {
        double device_s = 0, host_s = 0;
    };
    BatchTiming lastBatchTiming() const {
        std::lock_guard<std::mutex> lock(statsMutex_);
        return timing_;
    }

    // Whether an enabled CUSTOM filter with a callback is installed (the callback gets the whole Packet: a
    // caller that keeps only packets' bytes for classifyPerPacket(frames, ...) keeps the Packets
    // too while this holds).
    bool needsPackets() const { return needsPackets_.load(std::memory_order_relaxed); }

    // Small batches stay on the host: a single packet (applyFilters(const Packet&)) and batches
    // of fewer than hostBatchBelow() packets that ask for no records are decided on the calling
    // thread with the same compiled program — the device's own slot semantics (eval_builtin),
    // the compiled PAYLOAD DFAs (bt_payload_dfa_eval), CUSTOM callbacks and host regexes as for
    // any batch — instead of paying a device round trip (~0.1 ms per call whatever its size,
    // against ~0.5 us per packet for the reference, src/PacketFilter.cpp:57-119). Default:
    // BEATRICE_GPU_HOST_BELOW, else kHostBelowDefault; 0 sends every call to the device.
    // Measured (surface_bench single, profiles/r04/surfaces): classify() on the host costs
    // ~0.2 us + 7-12 ns per packet, on the device 23-35 us + ~9 ns per packet; 2048 keeps the
    // host's share of a batch's CPU time below the device pass's wall time.
    static constexpr size_t kHostBelowDefault = 2048;
    void setHostBatchBelow(size_t n) { hostBelow_.store(n, std::memory_order_relaxed); }
    size_t hostBatchBelow() const { return hostBelow_.load(std::memory_order_relaxed); }

    // Evaluation order of the enabled filters (names), as applyFilters uses it.
    std::vector<std::string> evaluationOrder();
    bt_ctx* context() const { return ctx_; }          // the first device's context
    bt_group* group() const { return group_; }
    uint32_t deviceCount() const { return bt_group_size(group_); }
    // The devices BEATRICE_GPU_DEVICES names ({fallback} when unset or empty).
    static std::vector<int> devicesFromEnv(int fallback);

private:
    struct FilterEntry {
        FilterConfig config;
        std::function<bool(const Packet&)> customFunc;
    };
    struct Slot {
        std::string name;
        FilterEntry* entry;
        bt_filter_slot compiled;
    };

    void compileLocked();
    // A shared hold on the compiled program (compiling it first if a mutator changed it).
    std::shared_lock<std::shared_mutex> lockProgram();
    // fn(lo, hi) over [0, n): on the context's host threads when this is the only batch
    // call in flight, else on the calling thread (concurrent callers are the parallelism,
    // and results freed by the caller are then allocated on its own thread)
    template <class Fn>
    void forRanges(size_t n, Fn&& fn);
    void setTiming(double device_s, double host_s);
    // host continuation for packets the device left at a PAYLOAD/CUSTOM slot
    uint32_t resolveHost(const Packet& p, uint32_t first_slot);
    // the device's decision for one frame, on the host: BT_DECIDE_HOST at the first CUSTOM /
    // host-regex slot (resolveHost continues there), as the kernel leaves it
    uint32_t evalFrame(const uint8_t* d, size_t len) const;
    bool hostSmall(size_t n) const { return n < hostBelow_.load(std::memory_order_relaxed); }
    void tallyOne(uint32_t decision, std::chrono::microseconds t);
    [[noreturn]] void rethrow(const Slot& s) const;
    void runBatch(const std::vector<Packet>& packets, std::vector<uint8_t>& decide, std::vector<bt_rec>* records = nullptr);
    void runFrames(const uint8_t* const* frames, const uint32_t* lens, uint32_t n, std::vector<uint8_t>& decide,
                   std::vector<bt_rec>* records);
    struct Tally;
    // packet(i) -> packet i (a reference or a value) for the host-side resumption
    // verdict (optional): the batch's verdict words, whose bits follow packets resolved on the host
    template <class PacketAt>
    Tally scan(size_t n, PacketAt packet, uint8_t* decide, std::vector<uint32_t>* pass_idx,
               std::vector<uint32_t>* error_idx, uint64_t* verdict = nullptr);
    bool scanParallel(size_t n, const uint8_t* decide, std::vector<uint32_t>* pass_idx,
                      std::vector<uint32_t>* error_idx, Tally& t);
    void flushTally(const Tally& t, std::chrono::microseconds per);

    void open(const std::vector<int>& devices, const bt_opts* opts);

    bt_group* group_ = nullptr;
    bt_ctx* ctx_ = nullptr;
    std::unordered_map<std::string, FilterEntry> filters_;
    mutable std::shared_mutex filtersMutex_;   // unique: mutators and compile; shared: batch calls
    std::mutex hostMutex_;                      // CUSTOM / PAYLOAD host resumption, one caller at a time
    std::atomic<int> inFlight_{0};              // batch calls running
    std::atomic<bool> needsPackets_{false};     // an enabled CUSTOM filter (updated by the mutators)
    void updateNeedsPackets();                  // filtersMutex_ held
    FilterStats stats_;
    mutable std::mutex statsMutex_;
    bool dirty_ = true;
    std::vector<Slot> program_;
    std::vector<std::string> rejectReason_;   // per slot: "Filter <name> rejected packet"
    std::vector<uint8_t> dfaPool_;            // the program's PAYLOAD DFAs (bt_filter_dfa_pool)
    std::atomic<size_t> hostBelow_{kHostBelowDefault};
    BatchTiming timing_;
};

}  // namespace gpu
}  // namespace beatrice
