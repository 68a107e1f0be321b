// test_host_pool.cpp — the host thread pool of the runtime (beatrice_amd/csrc/bt_host_pool.h)
// under stress, built with -fsanitize=thread by tests/test_host_pool.py (CPU, no GPU):
//   * run(fn) calls fn(k) exactly once for every k in [0, size()), whichever threads claim
//     (run(fn, count): every k in [0, count), none past it)
//     them, and returns only after all of them have finished;
//   * runs from several caller threads at once (the pool serialises them);
//   * slow indices (a worker sleeping inside fn) and workers that wake late (runs of
//     microseconds back to back) never let an index run twice or a run return early;
//   * destruction with idle workers;
//   * the group's MemberThreads: concurrent callers, each call's fn(k) once per member.
// Prints "ALL OK" and exits 0, or names the first failure.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../beatrice_amd/csrc/bt_host_pool.h"

static int check(unsigned T, int runs) {
    bt::HostPool p(T);
    if (p.size() != T) return std::printf("FAIL size %u != %u\n", p.size(), T), 1;
    std::vector<std::atomic<int>> hits(T);
    for (int r = 0; r < runs; ++r) {
        for (auto& h : hits) h = 0;
        std::atomic<int> done{0};
        p.run([&](unsigned k) {
            hits[k].fetch_add(1);
            if ((r + (int)k) % 97 == 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
            done.fetch_add(1);
        });
        if (done.load() != (int)T) return std::printf("FAIL T=%u run %d returned with %d of %u done\n", T, r, done.load(), T), 1;
        for (unsigned k = 0; k < T; ++k)
            if (hits[k] != 1) return std::printf("FAIL T=%u run %d index %u ran %d times\n", T, r, k, hits[k].load()), 1;
    }
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < 4; ++c)
        callers.emplace_back([&] {
            for (int r = 0; r < runs / 4; ++r) {
                std::vector<int> h(T, 0);
                p.run([&](unsigned k) { h[k]++; });
                for (unsigned k = 0; k < T; ++k)
                    if (h[k] != 1) bad++;
            }
        });
    for (auto& t : callers) t.join();
    if (bad) return std::printf("FAIL T=%u concurrent callers: %d bad indices\n", T, bad.load()), 1;
    std::printf("ok   T=%u: %d runs, 4 concurrent callers\n", T, runs);
    return 0;
}

// run(fn, count): fn(k) exactly once for every k < count and never for k >= count, with runs of
// every count in [1, size()] in turn and from 4 callers at once (a context's host pipeline uses
// a share of its pool while other callers wait, bt_runtime.cpp pipeline_share).
static int check_counts(unsigned T, int runs) {
    bt::HostPool p(T);
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < 4; ++c)
        callers.emplace_back([&, c] {
            for (int r = 0; r < runs; ++r) {
                const unsigned cnt = 1 + (unsigned)((r * 7 + c) % (int)T);
                std::vector<int> h(T, 0);
                p.run([&](unsigned k) {
                    h[k]++;
                    if ((r + (int)k) % 89 == 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
                }, cnt);
                for (unsigned k = 0; k < T; ++k)
                    if (h[k] != (k < cnt ? 1 : 0)) bad++;
            }
        });
    for (auto& t : callers) t.join();
    if (bad) return std::printf("FAIL T=%u counted runs: %d bad indices\n", T, bad.load()), 1;
    std::printf("ok   T=%u: %d counted runs from 4 callers\n", T, 4 * runs);
    return 0;
}

// The group's member threads: run(fn) from several callers at once, each call's fn(k) exactly
// once for every member k, calls queued per member in arrival order, destruction while idle.
static int check_members(uint32_t m, int calls) {
    std::vector<const cpu_set_t*> pins(m, nullptr);
    bt::MemberThreads mt(m, pins);
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < 6; ++c)
        callers.emplace_back([&, c] {
            for (int r = 0; r < calls; ++r) {
                std::vector<int> h(m, 0);   // written by the member threads, read after run()
                std::atomic<int> in{0};
                mt.run([&](uint32_t k) {
                    h[k]++;
                    in.fetch_add(1);
                    if ((r + c + (int)k) % 61 == 0) std::this_thread::sleep_for(std::chrono::microseconds(30));
                });
                if (in.load() != (int)m) bad++;
                for (uint32_t k = 0; k < m; ++k)
                    if (h[k] != 1) bad++;
            }
        });
    for (auto& t : callers) t.join();
    if (bad) return std::printf("FAIL members=%u: %d bad calls\n", m, bad.load()), 1;
    std::printf("ok   members=%u: %d calls from 6 threads\n", m, 6 * calls);
    return 0;
}

int main() {
    int fails = 0;
    for (unsigned T : {1u, 2u, 3u, 8u, 16u}) fails += check(T, 4000);
    for (unsigned T : {2u, 8u, 16u}) fails += check_counts(T, 1500);
    for (uint32_t m : {2u, 3u, 8u}) fails += check_members(m, 1500);
    { bt::HostPool idle(8); }   // destroyed with every worker waiting
    { bt::MemberThreads idle(4, std::vector<const cpu_set_t*>(4, nullptr)); }
    std::printf(fails ? "FAILED\n" : "ALL OK\n");
    return fails ? 1 : 0;
}
