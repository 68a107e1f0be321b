// bt_host_pool.h — the context's host thread pool (beatrice_amd/csrc/bt_runtime.cpp) and a
// group's member threads (bt_group.cpp), in a header of their own so
// tests/cpp/test_host_pool.cpp can stress them under ThreadSanitizer on the CPU. Host code only.
#pragma once

#include <pthread.h>
#include <sched.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bt {

// Fixed pool of host threads for the host-batch pipeline's gather / drain copies.
// run(fn) executes fn(0) .. fn(T-1) once each, T = size(): the caller and whichever workers
// wake claim the indices from one counter, and the caller waits only for the indices already
// claimed. On a host whose CPUs are all busy (callers on every CPU, the plugin's onPacket
// threads) a worker may not be scheduled for a whole time slice; waiting for every worker to
// take its fixed share made each run as slow as the latest one to wake (0.45 ms per device
// pass of a 12k-packet batch), whereas here the caller does the unclaimed work.
class HostPool {
public:
    // pin (optional): the CPUs the workers run on, e.g. those of the device's NUMA node
    // (bt_runtime.cpp place_ctx); the caller, worker 0, stays where it is
    explicit HostPool(unsigned n, const cpu_set_t* pin = nullptr) {
        nthreads_ = n ? (n < 0xFFFFu ? n : 0xFFFFu) : 1;   // indices fit the claim word's 16 bits
        static const bool fixed = getenv("BT_POOL_FIXED") != nullptr;   // A/B: each worker its own index
        fixed_ = fixed;
        if (pin) pin_ = *pin;
        const bool pinned = pin != nullptr;
        for (unsigned i = 1; i < nthreads_; ++i)
            th_.emplace_back([this, i, pinned] {
                if (pinned) (void)pthread_setaffinity_np(pthread_self(), sizeof(pin_), &pin_);
                loop(i);
            });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    unsigned size() const { return nthreads_; }
    // runs fn(k) for every k in [0, count) and waits; count 0 (or above size()) = size().
    // With count < size() the run's indices are fewer than its threads: the workers that find
    // none left go back to sleep (the context's host pipeline runs a smaller share of the pool
    // while other callers wait for it, bt_runtime.cpp pipeline_share)
    void run(const std::function<void(unsigned)>& fn, unsigned count = 0) {
        const unsigned want = count && count < nthreads_ ? count : nthreads_;
        if (want == 1) { fn(0); return; }
        std::lock_guard<std::mutex> one_at_a_time(run_mu_);   // callers on several threads
        uint32_t g;
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            g = (uint32_t)++gen_;
            finished_ = 0;
            count_ = fixed_ ? nthreads_ : want;
            fixed_want_ = want;   // fixed mode: workers with id >= want finish without running fn
            // the run's index count travels in the claim word itself: a worker still holding the
            // previous run's generation must never pair it with this run's (larger) count
            claim_.store(((uint64_t)g << 32) | ((uint64_t)want << 16), std::memory_order_release);
        }
        // wake as many workers as the run has indices beyond the caller's (a worker that is not
        // asleep yet sees the new generation in its wait predicate; one left asleep joins a
        // later run): a share of the pool does not wake the rest of it for nothing
        if (fixed_ || want == nthreads_) {
            cv_.notify_all();
        } else {
            for (unsigned k = 1; k < want; ++k) cv_.notify_one();
        }
        if (fixed_) {
            fn(0);
            std::lock_guard<std::mutex> lk(m_);
            ++finished_;
        } else {
            execute(g, fn);
        }
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return finished_ == count_; });
        fn_ = nullptr;
    }

private:
    // claims indices of run g and runs them. The claim word is generation << 32 | count << 16 |
    // next index: the generation keeps a late worker from claiming in a later run with an
    // earlier run's function, and reading the count from the same word keeps it from claiming
    // index `count` of its own run while the next run is being set up (with the count in a
    // separate variable, a worker that read the old claim word and the next run's larger count
    // ran one index past its run, on a function object that may already be the next run's)
    void execute(uint32_t g, const std::function<void(unsigned)>& fn) {
        for (;;) {
            uint64_t c = claim_.load(std::memory_order_acquire);
            for (;;) {
                if ((uint32_t)(c >> 32) != g || (c & 0xFFFFu) >= ((c >> 16) & 0xFFFFu)) return;
                if (claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel)) break;
            }
            fn((unsigned)(c & 0xFFFFu));
            std::lock_guard<std::mutex> lk(m_);
            if (++finished_ == count_) done_.notify_one();
        }
    }
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f;
            uint32_t g;
            unsigned want;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                f = fn_;   // null when that run has already finished
                g = (uint32_t)gen_;
                want = fixed_want_;
            }
            if (!f) continue;
            if (fixed_) {   // round 2's pool: worker id runs index id, the caller waits for all
                if (id < want) (*f)(id);   // a run of fewer indices than threads: the rest only check in
                std::lock_guard<std::mutex> lk(m_);
                if (++finished_ == nthreads_) done_.notify_one();
            } else {
                execute(g, *f);
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* fn_ = nullptr;
    std::atomic<uint64_t> claim_{0};   // (generation << 32) | (count << 16) | next index
    unsigned finished_ = 0, nthreads_ = 1;
    unsigned fixed_want_ = 1;   // fixed mode: the current run's index count (under m_)
    std::atomic<unsigned> count_{1};   // indices of the current run (set under m_ before its claims open)
    bool fixed_ = false;
    cpu_set_t pin_{};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// The group's member threads (beatrice_amd/csrc/bt_group.cpp).
// One worker thread per member after the first, kept for the group's life, each with its own
// FIFO of calls: member k's part of a call runs on thread k (member 0's on the caller), so a
// call creates no thread, and calls from several threads queue per member instead of waiting
// for each other's whole batch (each member still runs one call at a time: its context
// serialises them).
class MemberThreads {
public:
    // on_start (optional) runs first on member k's thread (the group selects k's device there)
    MemberThreads(uint32_t members, const std::vector<const cpu_set_t*>& pins,
                  std::function<void(uint32_t)> on_start = nullptr)
        : q_(members), on_start_(std::move(on_start)) {
        for (uint32_t k = 1; k < members; ++k) {
            if (pins[k]) {
                q_[k].pin = *pins[k];
                q_[k].pinned = true;
            }
            q_[k].th = std::thread([this, k] { loop(k); });
        }
    }
    ~MemberThreads() {
        for (size_t k = 1; k < q_.size(); ++k) {
            {
                std::lock_guard<std::mutex> lk(q_[k].m);
                q_[k].stop = true;
            }
            q_[k].cv.notify_one();
            q_[k].th.join();
        }
    }
    // fn(k) for every member k, concurrently; returns when all have. fn must not throw.
    void run(const std::function<void(uint32_t)>& fn) {
        Call call;
        call.fn = &fn;
        call.pending = (uint32_t)q_.size() - 1;
        for (size_t k = 1; k < q_.size(); ++k) {
            {
                std::lock_guard<std::mutex> lk(q_[k].m);
                q_[k].jobs.push_back(&call);
            }
            q_[k].cv.notify_one();
        }
        fn(0);
        std::unique_lock<std::mutex> lk(call.m);
        call.cv.wait(lk, [&] { return call.pending == 0; });
    }

private:
    struct Call {
        const std::function<void(uint32_t)>* fn = nullptr;
        std::mutex m;
        std::condition_variable cv;
        uint32_t pending = 0;
    };
    struct Queue {
        std::mutex m;
        std::condition_variable cv;
        std::deque<Call*> jobs;
        bool stop = false;
        bool pinned = false;
        cpu_set_t pin{};
        std::thread th;
    };
    void loop(uint32_t k) {
        Queue& q = q_[k];
        if (q.pinned) (void)pthread_setaffinity_np(pthread_self(), sizeof(q.pin), &q.pin);
        if (on_start_) on_start_(k);
        for (;;) {
            Call* c;
            {
                std::unique_lock<std::mutex> lk(q.m);
                q.cv.wait(lk, [&] { return q.stop || !q.jobs.empty(); });
                if (q.jobs.empty()) return;   // stop, and nothing left
                c = q.jobs.front();
                q.jobs.pop_front();
            }
            (*c->fn)(k);
            std::lock_guard<std::mutex> lk(c->m);
            if (--c->pending == 0) c->cv.notify_one();
        }
    }
    std::vector<Queue> q_;
    std::function<void(uint32_t)> on_start_;
};

}  // namespace bt
