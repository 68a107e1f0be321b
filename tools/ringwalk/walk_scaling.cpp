// walk_scaling.cpp — host thread scaling of bt_ring_walk_tpv3 (no GPU needed):
// T std::threads each walk a disjoint contiguous range of a packed TPACKET_V3 ring.
//   walk_scaling <cfg 2|3|4> <frames> <block_bytes> <max_threads> [reg|pool]
// reg:  the ring is page-locked + mapped with bt_host_register first (GPU needed)
// pool: the walk runs through a context's host pool (bt_create host_threads = T)
// gather: walk vs the three header gathers through a pool of max_threads threads
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <string>

#include "beatrice_gpu_bench.h"

extern "C" uint64_t bt_synth_layout(int cfg, uint64_t n, uint64_t seed, uint64_t* desc);
extern "C" int bt_synth_fill(int cfg, uint64_t n, uint64_t seed, const uint64_t* desc, uint8_t* data, int nthreads);
extern "C" uint64_t bt_synth_tpv3_pack(const uint8_t* data, const uint64_t* desc, uint64_t n, uint64_t block_size,
                                       uint8_t* ring, uint64_t ring_blocks, uint64_t* ring_desc, uint64_t* blocks_used);

int main(int argc, char** argv) {
    const int cfg = atoi(argv[1]);
    const uint64_t n = strtoull(argv[2], nullptr, 0), bs = strtoull(argv[3], nullptr, 0);
    unsigned maxT = (unsigned)atoi(argv[4]);
    const std::string mode = argc > 5 ? argv[5] : "";
    std::vector<uint64_t> desc(n);
    std::vector<uint8_t> data(bt_synth_layout(cfg, n, 1, desc.data()));
    bt_synth_fill(cfg, n, 1, desc.data(), data.data(), 8);
    uint64_t used = 0;
    bt_synth_tpv3_pack(data.data(), desc.data(), n, bs, nullptr, 1ull << 40, nullptr, &used);
    std::vector<uint8_t> ring(used * bs);
    bt_synth_tpv3_pack(data.data(), desc.data(), n, bs, ring.data(), used, nullptr, &used);
    data.clear();
    data.shrink_to_fit();
    std::vector<bt_pkt_desc> out(n + 64);
    bt_tpv3_ring r{ring.data(), bs, (uint32_t)used, 0};
    std::vector<uint64_t> first(used + 1, 0);   // frames before block b (block header num_pkts)
    for (uint64_t b = 0; b < used; ++b)
        first[b + 1] = first[b] + *reinterpret_cast<const uint32_t*>(ring.data() + b * bs + 12);
    for (auto& d : out) d = 0;                  // fault the output in before timing
    bt_ctx* reg_ctx = nullptr;
    if (mode == "reg") {
        void* alias = nullptr;
        if (bt_create(0, nullptr, &reg_ctx) != BT_OK || bt_host_register(reg_ctx, ring.data(), ring.size(), &alias) != BT_OK) {
            printf("register failed: %s\n", bt_last_error());
            return 1;
        }
        printf("ring registered with the GPU\n");
    }
    if (mode == "gather") {
        // walk / gather into 128-B slots / dense gather, interleaved, through a
        // pool of maxT threads, 128 blocks per call; best of 5 rounds each
        bt_opts o{};
        o.host_threads = maxT;
        bt_ctx* c = nullptr;
        if (bt_create(0, &o, &c) != BT_OK) {
            printf("bt_create failed (%s): one thread, no pool\n", bt_last_error());
            c = nullptr;
            maxT = 1;
        }
        std::vector<uint8_t> slots((n + 64) * BT_PREFIX_SLOT + 64);
        uint8_t* sl = slots.data() + ((64 - ((uintptr_t)slots.data() & 63)) & 63);
        for (auto& x : slots) x = 0;
        const char* names[3] = {"walk", "gather 128-B slots", "gather dense"};
        double best[3] = {1e9, 1e9, 1e9};
        for (int rep = 0; rep < 5; ++rep)
            for (int m = 0; m < 3; ++m) {
                const auto t0 = std::chrono::steady_clock::now();
                for (uint64_t b0 = 0; b0 < used; b0 += 128) {
                    uint32_t nd = 0, nb = 0;
                    const uint32_t cap = (uint32_t)(n + 64 - first[b0]);
                    if (m == 0)
                        bt_ring_walk_tpv3(c, &r, (uint32_t)b0, 128, out.data() + first[b0], cap, &nd, &nb);
                    else if (m == 1)
                        bt_ring_gather_tpv3(c, &r, (uint32_t)b0, 128, sl + first[b0] * BT_PREFIX_SLOT, out.data() + first[b0],
                                            cap, &nd, &nb);
                    else
                        bt_ring_gather_dense_tpv3(c, &r, (uint32_t)b0, 128, sl + first[b0] * BT_PREFIX_SLOT,
                                                  out.data() + first[b0], nullptr, cap, &nd, &nb);
                }
                best[m] = std::min(best[m], std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
        for (int m = 0; m < 3; ++m) printf("cfg %d threads %u  %-28s %.1f Mpps\n", cfg, maxT, names[m], n / best[m] / 1e6);
        if (c) bt_destroy(c);
        return 0;
    }
    if (mode == "pool") {
        for (unsigned T = 1; T <= maxT; T *= 2) {
            bt_opts o{};
            o.host_threads = T;
            bt_ctx* c = nullptr;
            if (bt_create(0, &o, &c) != BT_OK) {
                printf("bt_create failed: %s\n", bt_last_error());
                return 1;
            }
            double best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                const auto t0 = std::chrono::steady_clock::now();
                for (uint64_t b0 = 0; b0 < used; b0 += 128) {
                    uint32_t nd = 0, nb = 0;
                    bt_ring_walk_tpv3(c, &r, (uint32_t)b0, 128, out.data() + first[b0], (uint32_t)(n + 64 - first[b0]), &nd, &nb);
                }
                best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            printf("pool %2u  %.1f Mpps  (%.3f s)\n", T, n / best / 1e6, best);
            bt_destroy(c);
        }
        return 0;
    }
    printf("cfg %d frames %lu blocks %lu hw threads %u\n", cfg, (unsigned long)n, (unsigned long)used,
           std::thread::hardware_concurrency());
    for (unsigned T = 1; T <= maxT; T *= 2) {
        double best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (unsigned w = 0; w < T; ++w)
                th.emplace_back([&, w] {
                    const uint32_t a = (uint32_t)(used * w / T), b = (uint32_t)(used * (w + 1) / T);
                    uint32_t nd = 0, nb = 0;
                    bt_ring_walk_tpv3(nullptr, &r, a, b - a, out.data() + first[a], (uint32_t)(first[b] - first[a]),
                                      &nd, &nb);
                });
            for (auto& t : th) t.join();
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        printf("threads %2u  %.1f Mpps  (%.3f s)\n", T, n / best / 1e6, best);
    }
    return 0;
}
