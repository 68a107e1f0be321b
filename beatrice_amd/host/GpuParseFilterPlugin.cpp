// GpuParseFilterPlugin.cpp — an IPacketPlugin (reference include/beatrice/IPacketPlugin.hpp:9-33)
// that PluginManager::loadPlugin can dlopen (reference src/PluginManager.cpp:38-122):
// it batches the packets BeatriceContext hands to onPacket (src/BeatriceContext.cpp:188-193,
// 245-250) and classifies each batch on the MI355X with GpuPacketFilter.
//
// Configuration (environment, read in onStart):
//   BEATRICE_GPU_DEVICE    device index (default 0)
//   BEATRICE_GPU_BATCH     packets per GPU batch (default 65536)
//   BEATRICE_GPU_FLUSH_US  flush a partial batch after this many microseconds (default 2000)
//   BEATRICE_GPU_FILTERS   ';'-separated  name|TYPE|priority|expression  entries, TYPE one of
//                          BPF PROTOCOL IP_RANGE PORT_RANGE PAYLOAD CUSTOM
// Link with -Wl,-z,nodelete: ~PluginManager dlcloses handles before destroying plugins
// (src/PluginManager.cpp:26-34).
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "GpuPacketFilter.hpp"
#include "beatrice/IPacketPlugin.hpp"

namespace beatrice {
namespace gpu {

class GpuParseFilterPlugin : public IPacketPlugin {
public:
    void onStart() override {
        std::lock_guard<std::mutex> g(gpu_mu_);
        std::lock_guard<std::mutex> lk(mu_);
        const int device = env_int("BEATRICE_GPU_DEVICE", 0);
        batch_ = (size_t)env_int("BEATRICE_GPU_BATCH", 65536);
        flush_us_ = env_int("BEATRICE_GPU_FLUSH_US", 2000);
        filter_ = std::make_unique<GpuPacketFilter>(device);
        if (const char* spec = std::getenv("BEATRICE_GPU_FILTERS")) configure(spec);
        pending_.reserve(batch_);
    }

    void onStop() override {
        flush();
        std::lock_guard<std::mutex> g(gpu_mu_);
        filter_.reset();
    }

    // onPacket may run on several context threads at once (src/BeatriceContext.cpp:215-278).
    // A full batch is swapped out under mu_ and classified outside it, so the other
    // threads keep appending to a fresh batch while the GPU works; gpu_mu_ sends the
    // batches to the device one at a time.
    void onPacket(Packet& packet) override {
        if (!enabled_) return;
        std::vector<Packet> full;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (pending_.empty()) first_ = std::chrono::steady_clock::now();
            pending_.push_back(packet);        // shares the immutable bytes, no copy
            const auto age =
                std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - first_);
            if (pending_.size() >= batch_ || age.count() >= flush_us_) {
                full.swap(pending_);
                pending_.reserve(batch_);
            }
        }
        if (!full.empty()) classifyBatch(full);
    }

    std::string getName() const override { return "gpu_parse_filter"; }
    std::string getVersion() const override { return "1.0.0"; }
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

    void flush() {
        std::vector<Packet> full;
        {
            std::lock_guard<std::mutex> lk(mu_);
            full.swap(pending_);
        }
        if (!full.empty()) classifyBatch(full);
    }
    uint64_t passed() const { return passed_; }
    GpuPacketFilter* filter() { return filter_.get(); }

private:
    static int env_int(const char* k, int d) {
        const char* v = std::getenv(k);
        return v ? std::atoi(v) : d;
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

    void classifyBatch(const std::vector<Packet>& batch) {
        std::lock_guard<std::mutex> g(gpu_mu_);
        if (!filter_) return;
        try {
            auto v = filter_->classify(batch);
            processed_ += batch.size();
            passed_ += v.pass_idx.size();
        } catch (const std::exception&) {
            // a filter expression the reference would throw on: count the batch as errors
            errors_ += batch.size();
        }
    }

    std::mutex mu_;        // pending_, first_
    std::mutex gpu_mu_;    // filter_ (one batch on the device at a time)
    std::unique_ptr<GpuPacketFilter> filter_;
    std::vector<Packet> pending_;
    std::chrono::steady_clock::time_point first_;
    size_t batch_ = 65536;
    int flush_us_ = 2000;
    std::atomic<bool> enabled_{true};
    std::atomic<uint64_t> processed_{0}, passed_{0}, errors_{0};
};

}  // namespace gpu
}  // namespace beatrice

extern "C" beatrice::IPacketPlugin* createPlugin() { return new beatrice::gpu::GpuParseFilterPlugin(); }

// Test/ops hooks (plain C): flush a partial batch, read the pass counter.
extern "C" void gpu_plugin_flush(beatrice::IPacketPlugin* p) {
    static_cast<beatrice::gpu::GpuParseFilterPlugin*>(p)->flush();
}
extern "C" uint64_t gpu_plugin_passed(const beatrice::IPacketPlugin* p) {
    return static_cast<const beatrice::gpu::GpuParseFilterPlugin*>(p)->passed();
}
