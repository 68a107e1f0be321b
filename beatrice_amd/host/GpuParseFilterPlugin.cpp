// GpuParseFilterPlugin.cpp — an IPacketPlugin (reference include/beatrice/IPacketPlugin.hpp:9-33)
// that PluginManager::loadPlugin can dlopen (reference src/PluginManager.cpp:38-122):
// it batches the packets BeatriceContext hands to onPacket (src/BeatriceContext.cpp:188-193,
// 245-250) and classifies each batch on the MI355X with GpuPacketFilter.
//
// Configuration (environment, read in onStart):
//   BEATRICE_GPU_DEVICE    device index (default 0)
//   BEATRICE_GPU_DEVICES   device list "0,1,2,..." (overrides BEATRICE_GPU_DEVICE): every batch
//                          is split across the devices (bt_group, one process)
//   BEATRICE_GPU_RECORDS   1: the kernel pass also parses every packet; the sink gets each
//                          packet's bt_rec (gpu_verdict_batch.records)
//   BEATRICE_GPU_BATCH     packets per GPU batch (default 65536)
//   BEATRICE_GPU_FLUSH_US  a partial batch is classified at the latest this many
//                          microseconds after its first packet arrived, by the plugin's
//                          flush thread when no further packet comes (default 2000)
//   BEATRICE_GPU_FILTERS   ';'-separated  name|TYPE|priority|expression  entries, TYPE one of
//                          BPF PROTOCOL IP_RANGE PORT_RANGE PAYLOAD CUSTOM
//
// Results. Each packet is attributed on its own, as PluginManager::processPacket sees a
// per-packet plugin (src/PluginManager.cpp:158-171: an exception is caught per packet and
// the next packet goes on): a packet whose filter evaluation throws counts in
// getErrorCount(), the others are classified (GpuPacketFilter::classifyPerPacket).
// Downstream consumers get every batch's verdicts, in arrival order, through a verdict
// sink: C++ setVerdictSink(), or the C hook gpu_plugin_set_sink() for code that only has
// the IPacketPlugin* PluginManager created.
//
// Link with -Wl,-z,nodelete: ~PluginManager dlcloses handles before destroying plugins
// (src/PluginManager.cpp:26-34).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "GpuPacketFilter.hpp"
#include "beatrice/IPacketPlugin.hpp"
#include "beatrice_gpu_plugin.h"

namespace beatrice {
namespace gpu {

class GpuParseFilterPlugin : public IPacketPlugin {
public:
    using Sink = std::function<void(uint64_t seq, const std::vector<Packet>&, const GpuPacketFilter::Verdicts&)>;

    ~GpuParseFilterPlugin() override { stopFlusher(); }

    void onStart() override {
        stopFlusher();
        {
            std::lock_guard<std::mutex> g(gpu_mu_);
            batch_ = (size_t)std::max(1, env_int("BEATRICE_GPU_BATCH", 65536));
            records_ = env_int("BEATRICE_GPU_RECORDS", 0) != 0;
            flush_us_ = std::max(1, env_int("BEATRICE_GPU_FLUSH_US", 2000));
            filter_ = std::make_shared<GpuPacketFilter>(env_int("BEATRICE_GPU_DEVICE", 0));
            if (const char* spec = std::getenv("BEATRICE_GPU_FILTERS")) configure(spec);
        }
        {
            std::lock_guard<std::mutex> lk(flush_mu_);
            stop_ = false;
        }
        flusher_ = std::thread([this] { flushLoop(); });
    }

    void onStop() override {
        stopFlusher();
        flush();
        std::lock_guard<std::mutex> g(gpu_mu_);
        filter_.reset();
    }

    // onPacket runs on several context threads at once (src/BeatriceContext.cpp:215-278).
    // Each thread appends to its own shard of the pending batch (its lock is contended only
    // by the flush thread), so the threads do not serialise on one lock per packet: with a
    // single pending vector, 16 threads ran at 1.1 Mpps against 8.6 Mpps for one
    // (tools/surfaces, round 3). A full shard is classified outside its lock, by the thread
    // that filled it, while the others keep appending.
    void onPacket(Packet& packet) override {
        if (!enabled_) return;
        Shard& sh = shards_[shardOfThisThread()];
        std::vector<Packet> full;
        uint64_t seq = 0;
        bool armed = false;
        {
            std::lock_guard<std::mutex> lk(sh.mu);
            if (sh.pending.empty()) {
                sh.first.store(Clock::now().time_since_epoch().count(), std::memory_order_relaxed);
                armed = true;
            }
            sh.pending.push_back(packet);        // shares the immutable bytes, no copy
            if (sh.pending.size() >= batch_) seq = takeLocked(sh, full);
        }
        if (armed && full.empty()) {             // the flush thread arms this shard's deadline
            std::lock_guard<std::mutex> lk(flush_mu_);
            ++armed_;
            cv_.notify_one();
        }
        if (!full.empty()) classifyBatch(full, seq);
    }

    std::string getName() const override { return "gpu_parse_filter"; }
    std::string getVersion() const override { return "1.2.0"; }
    std::string getDescription() const override {
        return "MI355X parse + PacketFilter stage (gfx950 kernels behind the beatrice_gpu C-ABI)";
    }
    bool isEnabled() const override { return enabled_; }
    void setEnabled(bool e) override { enabled_ = e; }
    uint64_t getProcessedPacketCount() const override { return processed_; }
    uint64_t getErrorCount() const override { return errors_; }
    void resetStatistics() override {
        processed_ = passed_ = errors_ = 0;
        std::lock_guard<std::mutex> g(gpu_mu_);
        if (filter_) filter_->resetStats();
    }

    // Classifies every partial shard now (the flush thread does this on its own after
    // BEATRICE_GPU_FLUSH_US).
    void flush() {
        for (Shard& sh : shards_) {
            std::vector<Packet> full;
            uint64_t seq = 0;
            {
                std::lock_guard<std::mutex> lk(sh.mu);
                if (!sh.pending.empty()) seq = takeLocked(sh, full);
            }
            if (!full.empty()) classifyBatch(full, seq);
        }
    }

    void setVerdictSink(Sink s) {
        std::lock_guard<std::mutex> g(gpu_mu_);
        sink_ = std::move(s);
    }
    uint64_t passed() const { return passed_; }
    GpuPacketFilter* filter() { return filter_.get(); }

private:
    using Clock = std::chrono::steady_clock;
    static constexpr size_t kShards = 32;
    struct Shard {
        std::mutex mu;
        std::vector<Packet> pending;
        std::atomic<int64_t> first{0};   // arrival of the pending batch's first packet (ticks)
    };

    static int env_int(const char* k, int d) {
        const char* v = std::getenv(k);
        return v ? std::atoi(v) : d;
    }

    static size_t shardOfThisThread() {
        static std::atomic<size_t> next{0};
        thread_local const size_t mine = next.fetch_add(1, std::memory_order_relaxed) % kShards;
        return mine;
    }

    // Hands the shard's pending batch out with the next sequence number (sh.mu held).
    uint64_t takeLocked(Shard& sh, std::vector<Packet>& out) {
        out.swap(sh.pending);
        sh.pending.reserve(std::min<size_t>(batch_, 4096));
        sh.first.store(0, std::memory_order_relaxed);
        return next_seq_.fetch_add(1);
    }

    // The flush thread: sleeps until the earliest deadline (first packet + flush_us) of any
    // non-empty shard, or a stop, and classifies the shards still partial then.
    void flushLoop() {
        std::unique_lock<std::mutex> lk(flush_mu_);
        while (!stop_) {
            int64_t earliest = 0;
            for (Shard& sh : shards_) {
                const int64_t f = sh.first.load(std::memory_order_relaxed);
                if (f && (!earliest || f < earliest)) earliest = f;
            }
            if (!earliest) {
                const uint64_t seen = armed_;
                cv_.wait(lk, [&] { return stop_ || armed_ != seen; });
                continue;
            }
            const auto deadline = Clock::time_point(Clock::duration(earliest)) + std::chrono::microseconds(flush_us_);
            if (Clock::now() < deadline) {
                cv_.wait_until(lk, deadline);
                continue;
            }
            lk.unlock();
            const int64_t due = (Clock::now() - std::chrono::microseconds(flush_us_)).time_since_epoch().count();
            for (Shard& sh : shards_) {
                const int64_t f = sh.first.load(std::memory_order_relaxed);
                if (!f || f > due) continue;
                std::vector<Packet> full;
                uint64_t seq = 0;
                {
                    std::lock_guard<std::mutex> sl(sh.mu);
                    if (!sh.pending.empty()) seq = takeLocked(sh, full);
                }
                if (full.empty()) continue;
                try {
                    classifyBatch(full, seq);
                } catch (const std::exception&) {   // the device failed: nobody to throw to here
                    errors_ += full.size();
                }
            }
            lk.lock();
        }
    }

    void stopFlusher() {
        {
            std::lock_guard<std::mutex> lk(flush_mu_);
            stop_ = true;
        }
        cv_.notify_all();
        if (flusher_.joinable()) flusher_.join();
    }

    void configure(const std::string& spec) {
        std::stringstream ss(spec);
        std::string item;
        while (std::getline(ss, item, ';')) {
            if (item.empty()) continue;
            std::string parts[4];
            size_t pos = 0;
            for (int k = 0; k < 3; ++k) {
                size_t bar = item.find('|', pos);
                if (bar == std::string::npos) bar = item.size();
                parts[k] = item.substr(pos, bar - pos);
                pos = bar < item.size() ? bar + 1 : bar;
            }
            parts[3] = pos < item.size() ? item.substr(pos) : "";
            GpuPacketFilter::FilterConfig c;
            static const char* names[] = {"BPF", "PROTOCOL", "IP_RANGE", "PORT_RANGE", "PAYLOAD", "CUSTOM"};
            for (int t = 0; t < 6; ++t)
                if (parts[1] == names[t]) c.type = static_cast<GpuPacketFilter::FilterType>(t);
            c.priority = std::atoi(parts[2].c_str());
            c.expression = parts[3];
            filter_->addFilter(parts[0], c);
        }
    }

    // Batches are classified concurrently by the threads that took them (GpuPacketFilter
    // serialises only the device pass; each caller resumes host slots and builds its own
    // verdicts) and reach the sink in sequence order. With the whole call under one lock,
    // the onPacket threads whose shards filled queued behind each other's host work.
    void classifyBatch(const std::vector<Packet>& batch, uint64_t seq) {
        std::shared_ptr<GpuPacketFilter> f;
        {
            std::lock_guard<std::mutex> g(gpu_mu_);
            f = filter_;
        }
        struct Advance {   // waits for this batch's turn, then lets the next one go (also on a throw)
            GpuParseFilterPlugin* p;
            uint64_t seq;
            std::unique_lock<std::mutex> g;
            void turn() {
                if (g.owns_lock()) return;
                g = std::unique_lock<std::mutex>(p->gpu_mu_);
                p->order_cv_.wait(g, [&] { return p->done_seq_ == seq; });
            }
            ~Advance() {
                turn();
                ++p->done_seq_;
                p->order_cv_.notify_all();
            }
        } advance{this, seq, {}};
        if (!f) return;
        const auto v = f->classifyPerPacket(batch, records_);
        processed_ += batch.size();
        passed_ += v.pass_idx.size();
        errors_ += v.error_idx.size();
        advance.turn();
        if (sink_) sink_(seq, batch, v);
    }

    Shard shards_[kShards];
    std::mutex flush_mu_;              // stop_, armed_ (the flush thread's wake-ups)
    std::condition_variable cv_;
    uint64_t armed_ = 0;               // shards that went from empty to pending
    std::mutex gpu_mu_;                // filter_, sink_, done_seq_ (the sink's turn)
    std::condition_variable order_cv_;
    std::shared_ptr<GpuPacketFilter> filter_;   // a batch in flight holds its own reference
    size_t batch_ = 65536;
    int flush_us_ = 2000;
    bool records_ = false;
    std::atomic<uint64_t> next_seq_{0};
    uint64_t done_seq_ = 0;
    bool stop_ = true;
    std::thread flusher_;
    Sink sink_;
    std::atomic<bool> enabled_{true};
    std::atomic<uint64_t> processed_{0}, passed_{0}, errors_{0};
};

}  // namespace gpu
}  // namespace beatrice

extern "C" beatrice::IPacketPlugin* createPlugin() { return new beatrice::gpu::GpuParseFilterPlugin(); }

// C hooks (include/beatrice_gpu_plugin.h): flush a partial batch, read the pass counter,
// install a verdict sink.
extern "C" void gpu_plugin_flush(beatrice::IPacketPlugin* p) {
    static_cast<beatrice::gpu::GpuParseFilterPlugin*>(p)->flush();
}
extern "C" uint64_t gpu_plugin_passed(const beatrice::IPacketPlugin* p) {
    return static_cast<const beatrice::gpu::GpuParseFilterPlugin*>(p)->passed();
}
extern "C" void gpu_plugin_set_sink(beatrice::IPacketPlugin* p, gpu_verdict_sink_fn fn, void* user) {
    auto* g = static_cast<beatrice::gpu::GpuParseFilterPlugin*>(p);
    if (!fn) {
        g->setVerdictSink(nullptr);
        return;
    }
    g->setVerdictSink([fn, user](uint64_t seq, const std::vector<beatrice::Packet>& b,
                                 const beatrice::gpu::GpuPacketFilter::Verdicts& v) {
        std::vector<const uint8_t*> frames(b.size());
        std::vector<uint32_t> lens(b.size());
        for (size_t i = 0; i < b.size(); ++i) {
            frames[i] = b[i].data();
            lens[i] = (uint32_t)b[i].length();
        }
        gpu_verdict_batch c{seq, (uint32_t)b.size(), frames.data(), lens.data(), v.decide.data(),
                            v.pass_idx.data(), (uint32_t)v.pass_idx.size(), v.error_idx.data(),
                            (uint32_t)v.error_idx.size(), v.records.empty() ? nullptr : v.records.data()};
        fn(user, &c);
    });
}

extern "C" uint32_t gpu_batch_layers(const gpu_verdict_batch* b, uint32_t i, gpu_walked_layer* out, uint32_t cap) {
    if (!b || !b->records || i >= b->n) return 0;
    const bt_rec& r = b->records[i];
    gpu_walked_layer l[6];
    uint32_t k = 0;
    auto add = [&](const char* name, uint32_t off, int32_t tag, uint32_t bit) {
        l[k++] = {name, off, tag, (r.ok & bit) ? 1u : 0u};
    };
    add("ethernet", 0, -1, BT_L_ETH);   // the walk (DESIGN.md R-WALK), from the record's bitmaps
    if (r.present & BT_L_VLAN0) add("vlan", 12, 0, BT_L_VLAN0);
    if (r.present & BT_L_VLAN1) add("vlan", 16, 1, BT_L_VLAN1);
    if (r.present & BT_L_IPV4) add("ipv4", r.l3_off, -1, BT_L_IPV4);
    if (r.present & BT_L_IPV6) add("ipv6", r.l3_off, -1, BT_L_IPV6);
    if (r.present & BT_L_TCP) add("tcp", r.l4_off, -1, BT_L_TCP);
    if (r.present & BT_L_UDP) add("udp", r.l4_off, -1, BT_L_UDP);
    if (r.present & BT_L_ICMP) add("icmp", r.l4_off, -1, BT_L_ICMP);
    for (uint32_t j = 0; j < k && j < cap && out; ++j) out[j] = l[j];
    return k;
}

extern "C" int gpu_batch_format(const gpu_verdict_batch* b, uint32_t i, uint32_t fmt, char* out, uint64_t cap,
                                uint64_t* out_len) {
    if (!b || !b->records || i >= b->n) return BT_E_INVALID_ARGUMENT;
    return bt_format_records(nullptr, b->records + i, 1, fmt, out, cap, out_len, nullptr);
}
