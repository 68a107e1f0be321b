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
//   BEATRICE_GPU_WORKERS   classifier threads (default 2, at most 8)
//   BEATRICE_GPU_DEBUG     1: onStop prints where the classifier threads' time went
//   BEATRICE_GPU_PACK      1: pack header prefixes at onPacket time (HeldBatch; off by default:
//                          with frames that are not in the onPacket thread's cache it was
//                          slower, C3 from 16 threads 29 against 39-43 Mpps,
//                          profiles/r03/surfaces/ab_plugin_pack.jsonl)
//   BEATRICE_GPU_FILTERS   ';'-separated  name|TYPE|priority|expression  entries, TYPE one of
//                          BPF PROTOCOL IP_RANGE PORT_RANGE PAYLOAD CUSTOM
//
// Threads. onPacket appends to a per-thread shard of the pending batch; a full shard (or, from
// the plugin's flush thread, a partial one past its deadline) is queued for the plugin's
// classifier threads, which take the batches in order, run them through GpuPacketFilter and
// call the sink in order; at most 4 batches wait in the queue (onPacket blocks beyond that).
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
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
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

// A batch of packets the plugin holds until it is classified: each packet's bytes kept alive
// through a reference to them (Packet::getData) with the frame pointers and lengths the device
// pass reads (28 B per packet instead of a 216-B Packet copy, whose copy and destruction were
// most of onPacket's time), plus the whole Packets only while a CUSTOM filter (whose callback
// gets the Packet, metadata included) is installed.
//
// With BEATRICE_GPU_PACK=1 and a program that allows it (no GPU PAYLOAD slot), each packet's
// first W bytes (the bytes the device pass reads: 48 for verdicts, 112 with records,
// bt_host_stage_bytes) are also copied, at onPacket time, into `pre` (W bytes per packet, back
// to back): the classifier's gather then reads one sequential buffer instead of a cache miss
// per frame, and the copy moves to the onPacket threads (a gain only where they hold the
// frame in cache, e.g. right after the capture backend wrote it).
struct HeldBatch {
    std::vector<std::shared_ptr<const uint8_t[]>> keep;
    std::vector<const uint8_t*> frames;
    std::vector<uint32_t> lens;
    std::vector<Packet> packets;   // empty unless the batch started with a CUSTOM filter installed
    std::vector<uint8_t> pre;      // W bytes per packet when W != 0
    bool whole = false;
    uint32_t W = 0;

    size_t size() const { return frames.size(); }
    bool empty() const { return frames.empty(); }
    void push(const Packet& p) {
        keep.push_back(p.getData());
        frames.push_back(p.data());
        lens.push_back((uint32_t)p.length());
        if (whole) packets.push_back(p);
        if (W) {
            const size_t at = pre.size();
            pre.resize(at + W);
            std::memcpy(pre.data() + at, p.data(), std::min<size_t>(p.length(), W));
        }
    }
    void clear() {
        keep.clear();
        frames.clear();
        lens.clear();
        packets.clear();
        pre.clear();
        whole = false;
        W = 0;
    }
    void reserve(size_t n) {
        keep.reserve(n);
        frames.reserve(n);
        lens.reserve(n);
        if (W) pre.reserve(n * W);
    }
    size_t capacity() const { return frames.capacity(); }
    void swap(HeldBatch& o) {
        keep.swap(o.keep);
        frames.swap(o.frames);
        lens.swap(o.lens);
        packets.swap(o.packets);
        pre.swap(o.pre);
        std::swap(whole, o.whole);
        std::swap(W, o.W);
    }
    // appends o's packets (same `whole` mode and W; o is left empty)
    void append(HeldBatch& o) {
        if (empty()) {
            swap(o);
            return;
        }
        keep.insert(keep.end(), std::make_move_iterator(o.keep.begin()), std::make_move_iterator(o.keep.end()));
        frames.insert(frames.end(), o.frames.begin(), o.frames.end());
        lens.insert(lens.end(), o.lens.begin(), o.lens.end());
        packets.insert(packets.end(), std::make_move_iterator(o.packets.begin()), std::make_move_iterator(o.packets.end()));
        pre.insert(pre.end(), o.pre.begin(), o.pre.end());
        o.clear();
    }
    // packet i for the host-side filters: the held Packet, or one made from its bytes
    Packet packet(size_t i) const { return whole ? packets[i] : Packet(keep[i], lens[i]); }
};

class GpuParseFilterPlugin : public IPacketPlugin {
public:
    using Sink = std::function<void(uint64_t seq, const HeldBatch&, const GpuPacketFilter::Verdicts&)>;

    ~GpuParseFilterPlugin() override {
        stopFlusher();
        stopWorker();
    }

    void onStart() override {
        stopFlusher();
        stopWorker();
        {
            std::lock_guard<std::mutex> g(gpu_mu_);
            batch_ = (size_t)std::max(1, env_int("BEATRICE_GPU_BATCH", 65536));
            records_ = env_int("BEATRICE_GPU_RECORDS", 0) != 0;
            flush_us_ = std::max(1, env_int("BEATRICE_GPU_FLUSH_US", 2000));
            workers_ = std::min(8, std::max(1, env_int("BEATRICE_GPU_WORKERS", 2)));
            pack_ = env_int("BEATRICE_GPU_PACK", 0) != 0;
            // the plugin reads the device list: BEATRICE_GPU_DEVICES=0,1,... (a group), else
            // BEATRICE_GPU_DEVICE (one device, default 0)
            const std::vector<int> devs = GpuPacketFilter::devicesFromEnv(env_int("BEATRICE_GPU_DEVICE", 0));
            // one device: its host pool at 8 threads, not every usable CPU, since the onPacket
            // producers share the host (16 producers lost 5-15 % with a 16-thread pool,
            // profiles/r04/surfaces/ab_pool_8_16.jsonl); BT_HOST_THREADS overrides
            bt_opts o{};
            if (devs.size() == 1 && !std::getenv("BT_HOST_THREADS")) o.host_threads = std::min(8u, std::max(1u, bt_usable_cpus()));
            filter_ = std::make_shared<GpuPacketFilter>(devs, &o);
            if (const char* spec = std::getenv("BEATRICE_GPU_FILTERS")) configure(spec);
            whole_ = filter_->needsPackets();
            stage_ = stageWidth(*filter_);
        }
        {
            std::lock_guard<std::mutex> lk(flush_mu_);
            stop_ = false;
        }
        {
            std::lock_guard<std::mutex> lk(q_mu_);
            wstop_ = false;
        }
        for (int k = 0; k < workers_; ++k) classifiers_.emplace_back([this] { classifyLoop(); });
        flusher_ = std::thread([this] { flushLoop(); });
    }

    void onStop() override {
        stopFlusher();
        flush();
        stopWorker();
        if (env_int("BEATRICE_GPU_DEBUG", 0))   // where the classifier threads' time went
            std::fprintf(stderr,
                         "[gpu_parse_filter] %llu batches: classify %.1f ms (device pass %.1f), waiting for the "
                         "sink's turn %.1f ms, "
                         "sink %.1f ms (summed over %d classifier threads); onPacket blocked on a full queue %.1f ms\n",
                         (unsigned long long)prof_.batches.load(), prof_.classify_ns / 1e6, prof_.device_ns / 1e6,
                         prof_.turn_ns / 1e6,
                         prof_.sink_ns / 1e6, workers_, prof_.blocked_ns / 1e6);
        std::lock_guard<std::mutex> g(gpu_mu_);
        filter_.reset();
    }

    // onPacket runs on several context threads at once (src/BeatriceContext.cpp:215-278).
    // Each thread appends to its own shard of the pending batch (its lock is contended only
    // by the flush thread), so the threads do not serialise on one lock per packet: with a
    // single pending vector, 16 threads ran at 1.1 Mpps against 8.6 Mpps for one
    // (tools/surfaces, round 3). A full shard goes to the classifier thread's queue and the
    // thread goes on appending; it blocks only while kMaxQueued batches wait (backpressure).
    void onPacket(Packet& packet) override {
        if (!enabled_) return;
        Shard& sh = shards_[shardOfThisThread()];
        HeldBatch full;
        bool armed = false;
        {
            std::lock_guard<SpinLock> lk(sh.mu);
            if (sh.pending.empty()) {
                sh.first.store(Clock::now().time_since_epoch().count(), std::memory_order_relaxed);
                sh.pending.whole = wholePackets();
                sh.pending.W = stage_.load(std::memory_order_relaxed);
                armed = true;
            }
            sh.pending.push(packet);             // shares the immutable bytes, no copy
            if (sh.pending.size() >= batch_) takeLocked(sh, full);
        }
        if (armed && full.empty()) {             // the flush thread arms this shard's deadline
            std::lock_guard<std::mutex> lk(flush_mu_);
            ++armed_;
            cv_.notify_one();
        }
        if (!full.empty()) {
            enqueue(std::move(full));
            recycleOne();
        }
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

    // Classifies every partial shard now and returns when every batch queued so far has
    // reached the sink (the flush thread does the same on its own after BEATRICE_GPU_FLUSH_US).
    void flush() {
        takePartials(0);
        std::unique_lock<std::mutex> lk(q_mu_);
        const uint64_t upto = next_seq_;
        done_cv_.wait(lk, [&] { return done_seq_ >= upto || wstop_; });
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
    // One shard per 128 B (two lines, the adjacent-line prefetch pair): a shard's lock and
    // vector ends are written on every onPacket, and neighbouring shards in one line made
    // every append a cache-line transfer between two producer threads.
    // A shard's lock: taken on every onPacket by its producer and, rarely, by the flush thread
    // or a second producer (more than kShards threads): one atomic exchange and a release store
    // instead of a pthread mutex's two locked operations (same box, alternating builds, 3 pairs:
    // 16 producers C2 169-178 -> 182-192 Mpps, C3 154-167 -> 160-187; one producer +11..31 %;
    // profiles/r04/surfaces/ab_plugin_spinlock.jsonl). A waiter yields after a short spin, so a
    // holder preempted under the job's CPU quota is not spun against for a whole slice.
    struct SpinLock {
        std::atomic<bool> held{false};
        void lock() {
            for (unsigned spins = 0; held.exchange(true, std::memory_order_acquire);)
                while (held.load(std::memory_order_relaxed)) {
                    if (++spins < 64) __builtin_ia32_pause();
                    else std::this_thread::yield();
                }
        }
        void unlock() { held.store(false, std::memory_order_release); }
    };
    struct alignas(128) Shard {
        SpinLock mu;
        HeldBatch pending;
        std::atomic<int64_t> first{0};   // arrival of the pending batch's first packet (ticks)
    };

    static int env_int(const char* k, int d) {
        const char* v = std::getenv(k);
        return v ? std::atoi(v) : d;
    }

    // Whether new batches keep whole Packets: an enabled CUSTOM filter is installed. Read from
    // the filter at onStart and after every classified batch (a CUSTOM filter installed later
    // through filter() reaches the batches started after the next one; the packets of batches
    // already pending reach its callback as Packet(bytes, length)).
    bool wholePackets() const { return whole_.load(std::memory_order_relaxed); }

    // Prefix bytes new batches pack per packet: what the device pass reads with the current
    // program, when that is a header prefix (not with a GPU PAYLOAD slot, whose window the
    // device reads from the frame itself); only with BEATRICE_GPU_PACK=1.
    uint32_t stageWidth(GpuPacketFilter& f) const {
        if (!pack_) return 0;
        const uint32_t w = f.stagedPrefixBytes(records_);
        return w <= 112 ? w : 0u;
    }

    static size_t shardOfThisThread() {
        static std::atomic<size_t> next{0};
        thread_local const size_t mine = next.fetch_add(1, std::memory_order_relaxed) % kShards;
        return mine;
    }

    // Hands the shard's pending batch out (sh.mu held); the shard continues in a cleared
    // vector from the recycled ones when there is one (its capacity kept).
    void takeLocked(Shard& sh, HeldBatch& out) {
        out.swap(sh.pending);
        {
            std::lock_guard<std::mutex> lk(q_mu_);
            if (!clean_.empty()) {
                sh.pending.swap(clean_.back());
                clean_.pop_back();
            }
        }
        if (sh.pending.capacity() < std::min<size_t>(batch_, 4096)) sh.pending.reserve(std::min<size_t>(batch_, 4096));
        sh.first.store(0, std::memory_order_relaxed);
    }

    // Queues a batch for the classifier thread under the next sequence number; waits while
    // kMaxQueued batches are queued.
    void enqueue(HeldBatch&& batch) {
        const auto t0 = Clock::now();
        std::unique_lock<std::mutex> lk(q_mu_);
        space_cv_.wait(lk, [&] { return queue_.size() < kMaxQueued || wstop_; });
        prof_.blocked_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
        if (wstop_) {   // stopped (onStop raced with onPacket): nobody will classify it
            errors_ += batch.size();
            return;
        }
        queue_.push_back({next_seq_++, std::move(batch)});
        q_cv_.notify_one();
    }

    // The Packets of a classified batch are released by a producer thread, not by the
    // classifier (whose time bounds the plugin): one used vector is cleared here and kept,
    // with its capacity, for the next shard that fills.
    void recycleOne() {
        HeldBatch v;
        {
            std::lock_guard<std::mutex> lk(q_mu_);
            if (used_.empty()) return;
            v.swap(used_.back());
            used_.pop_back();
        }
        v.clear();
        std::lock_guard<std::mutex> lk(q_mu_);
        if (clean_.size() < kShards) clean_.push_back(std::move(v));
    }

    // A classifier thread: takes the queued batches in sequence order and classifies them
    // (with several classifier threads, one batch's device pass overlaps another's host
    // work: GpuPacketFilter serialises only the device pass); the sink gets them in order.
    void classifyLoop() {
        std::unique_lock<std::mutex> lk(q_mu_);
        for (;;) {
            q_cv_.wait(lk, [&] { return wstop_ || !queue_.empty(); });
            if (queue_.empty()) return;   // stopped and drained
            Queued q = std::move(queue_.front());
            queue_.pop_front();
            space_cv_.notify_one();
            lk.unlock();
            std::shared_ptr<GpuPacketFilter> f;
            {
                std::lock_guard<std::mutex> g(gpu_mu_);
                f = filter_;
            }
            GpuPacketFilter::Verdicts v;
            bool ok = false;
            const auto t0 = Clock::now();
            if (f) {
                try {
                    const HeldBatch& b = q.batch;
                    const uint8_t* const* frames = b.frames.data();
                    thread_local std::vector<const uint8_t*> packed;
                    if (b.W) {   // the packed prefixes stand in for the frames
                        packed.resize(b.size());
                        for (size_t i = 0; i < b.size(); ++i) packed[i] = b.pre.data() + i * b.W;
                        frames = packed.data();
                    }
                    v = f->classifyPerPacket(frames, b.lens.data(), b.size(), records_,
                                             [&b](size_t i) { return b.packet(i); }, b.W);
                    whole_ = f->needsPackets();
                    stage_ = stageWidth(*f);
                    ok = true;
                    prof_.device_ns += (uint64_t)(f->lastBatchTiming().device_s * 1e9);
                } catch (const std::exception&) {   // the device failed: nobody to throw to here
                    errors_ += q.batch.size();
                }
            }
            const auto t1 = Clock::now();
            lk.lock();
            done_cv_.wait(lk, [&] { return done_seq_ == q.seq; });   // the sink's turn
            lk.unlock();
            const auto t2 = Clock::now();
            if (ok) {
                processed_ += q.batch.size();
                passed_ += v.pass_idx.size();
                errors_ += v.error_idx.size();
                std::lock_guard<std::mutex> g(gpu_mu_);
                if (sink_) sink_(q.seq, q.batch, v);
            }
            const auto t3 = Clock::now();
            auto ns = [](Clock::duration d) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
            prof_.classify_ns += ns(t1 - t0);
            prof_.turn_ns += ns(t2 - t1);
            prof_.sink_ns += ns(t3 - t2);
            ++prof_.batches;
            lk.lock();
            done_seq_ = q.seq + 1;
            if (used_.size() < kMaxUsed && !queue_.empty()) {
                used_.push_back(std::move(q.batch));   // a producer releases it (recycleOne)
            } else {
                // the producers are not recycling (no full shards), or nothing else is queued
                // (traffic stopped: release now rather than hold the capture's buffers until
                // the next burst): the classifier releases this batch and the parked ones
                std::vector<HeldBatch> drop;
                if (queue_.empty()) drop.swap(used_);
                lk.unlock();
                q.batch.clear();
                drop.clear();
                lk.lock();
                // (handing the cleared vectors to clean_ here, capacity kept, was measured: no
                // gain at 8 / 16 producers and one producer 40 % slower, writing into lines the
                // classifier's core last held; profiles/r04/surfaces/ab_plugin_shard_align.jsonl)
            }
            done_cv_.notify_all();
        }
    }

    void stopWorker() {
        {
            std::lock_guard<std::mutex> lk(q_mu_);
            wstop_ = true;
        }
        q_cv_.notify_all();
        space_cv_.notify_all();
        for (auto& w : classifiers_) w.join();
        classifiers_.clear();
        std::lock_guard<std::mutex> lk(q_mu_);
        used_.clear();
        clean_.clear();
        done_cv_.notify_all();
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
            takePartials(Clock::now().time_since_epoch().count());
            lk.lock();
        }
    }

    // Queues the partial shards as few batches: when one shard is due (its first packet
    // arrived flush_us ago, or `now` == 0: an explicit flush), every non-empty shard's packets
    // go into one merged batch (up to 4 x the batch size each), so a flush tick costs one
    // device pass rather than one per onPacket thread (16 threads each flushing a few
    // thousand packets every tick spent most of the device time on per-call costs).
    void takePartials(int64_t now) {
        const int64_t due = now - std::chrono::duration_cast<Clock::duration>(std::chrono::microseconds(flush_us_)).count();
        bool any_due = now == 0;
        for (Shard& sh : shards_) {
            const int64_t f = sh.first.load(std::memory_order_relaxed);
            if (f && f <= due) any_due = true;
        }
        if (!any_due) return;
        HeldBatch merged[4];   // by `whole` mode and whether prefixes are packed (W is one value at a time)
        for (Shard& sh : shards_) {
            HeldBatch part;
            {
                std::lock_guard<SpinLock> sl(sh.mu);
                if (!sh.pending.empty()) takeLocked(sh, part);
            }
            if (part.empty()) continue;
            HeldBatch& m = merged[(part.whole ? 1 : 0) + (part.W ? 2 : 0)];
            if (!m.empty() && m.W != part.W) {   // the program changed between two shards
                enqueue(std::move(m));
                m.clear();
            }
            m.append(part);
            if (m.size() >= 4 * batch_) enqueue(std::move(m)), m.clear();
            if (part.capacity()) recycleEmpty(std::move(part));
        }
        for (HeldBatch& m : merged)
            if (!m.empty()) enqueue(std::move(m));
    }

    // a cleared vector set back into circulation
    void recycleEmpty(HeldBatch&& v) {
        v.clear();
        std::lock_guard<std::mutex> lk(q_mu_);
        if (clean_.size() < kShards) clean_.push_back(std::move(v));
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

    Shard shards_[kShards];
    std::mutex flush_mu_;              // stop_, armed_ (the flush thread's wake-ups)
    std::condition_variable cv_;
    uint64_t armed_ = 0;               // shards that went from empty to pending
    std::mutex gpu_mu_;                // filter_, sink_
    std::shared_ptr<GpuPacketFilter> filter_;   // a batch in flight holds its own reference
    std::atomic<bool> whole_{false};            // wholePackets()
    std::atomic<uint32_t> stage_{0};            // stageWidth() of the current program
    bool pack_ = true;                          // BEATRICE_GPU_PACK
    size_t batch_ = 65536;
    int flush_us_ = 2000;
    bool records_ = false;
    // the classifier thread's queue and the vectors recycled through it (q_mu_)
    static constexpr size_t kMaxQueued = 4;
    // classified batches waiting for a producer to release their packets: each still holds
    // its packets' buffers, so only a few (the capture's memory is not the plugin's to keep)
    static constexpr size_t kMaxUsed = 4;
    struct Queued {
        uint64_t seq;
        HeldBatch batch;
    };
    std::mutex q_mu_;
    std::condition_variable q_cv_, space_cv_, done_cv_;
    std::deque<Queued> queue_;
    std::vector<HeldBatch> used_, clean_;   // classified (bytes still held) / cleared
    uint64_t next_seq_ = 0, done_seq_ = 0;
    bool wstop_ = true;
    struct {
        std::atomic<uint64_t> batches{0}, classify_ns{0}, device_ns{0}, turn_ns{0}, sink_ns{0}, blocked_ns{0};
    } prof_;
    std::vector<std::thread> classifiers_;   // the classifier threads (BEATRICE_GPU_WORKERS)
    int workers_ = 2;
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
    g->setVerdictSink([fn, user](uint64_t seq, const beatrice::gpu::HeldBatch& b,
                                 const beatrice::gpu::GpuPacketFilter::Verdicts& v) {
        gpu_verdict_batch c{seq, (uint32_t)b.size(), b.frames.data(), b.lens.data(), v.decide.data(),
                            v.pass_idx.data(), (uint32_t)v.pass_idx.size(), v.error_idx.data(),
                            (uint32_t)v.error_idx.size(), v.records.empty() ? nullptr : v.records.data()};
        fn(user, &c);
    });
}

extern "C" uint32_t gpu_batch_layers(const gpu_verdict_batch* b, uint32_t i, gpu_walked_layer* out, uint32_t cap) {
    if (!b || !b->records || i >= b->n) return 0;
    const bt_rec& r = b->records[i];
    // a kernel record holds at most 5 layers; a caller's record may set every present bit (8)
    gpu_walked_layer l[8];
    uint32_t k = 0;
    auto add = [&](const char* name, uint32_t off, int32_t tag, uint32_t bit) {
        if (k < 8) l[k++] = {name, off, tag, (r.ok & bit) ? 1u : 0u};
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
