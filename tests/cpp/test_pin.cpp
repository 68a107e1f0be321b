// CPU test of the registered-page table (beatrice_amd/csrc/bt_pin.h) with a fake driver:
// no GPU, no HIP. The fake gives every device its own alias space (alias = ((device + 1) << 48)
// + host address), records which device was current at every call, and refuses a lock of a page
// that is already locked (what hipHostRegister does for a start inside a registered range),
// so the table's own page bookkeeping is what keeps one page from being locked twice.
//
// Cases: page rounding; a range inside a live span shares it (one lock, refs); a range that
// holds only some pages of a span is refused; the last release syncs every device that got an
// alias and then unlocks; a failed sync leaves the span registered; eight members on eight
// devices each get the alias of their own device, taken with their device current (the group's
// per-member lookup, bt_group.cpp); concurrent acquire / release from 8 threads.
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "bt_pin.h"

namespace {

int g_fail = 0;
#define CHECK(...)                                                      \
    do {                                                                \
        if (!(__VA_ARGS__)) {                                           \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #__VA_ARGS__); \
            ++g_fail;                                                   \
        }                                                               \
    } while (0)

struct FakeLog {
    std::mutex mu;
    std::set<uint64_t> locked_pages;
    std::vector<std::pair<uint64_t, uint64_t>> locks, unlocks_;
    std::vector<int> syncs;
    std::vector<std::pair<int, uint64_t>> alias_calls;   // (current device, page)
    bool fail_sync = false;
};

struct FakeDriver {
    FakeLog* log = nullptr;
    int cur = 0;
    std::string msg;
    int set_device(int d) {
        if (d < 0 || d >= 8) return msg = "no such device", 1;
        cur = d;
        return 0;
    }
    int lock(void* lo, uint64_t bytes) {
        std::lock_guard<std::mutex> lk(log->mu);
        const uint64_t a = (uint64_t)(uintptr_t)lo;
        if (a % bt::kPinPage || bytes % bt::kPinPage) return msg = "unaligned lock", 1;
        for (uint64_t p = a; p < a + bytes; p += bt::kPinPage)
            if (log->locked_pages.count(p)) return msg = "page already locked", 1;
        for (uint64_t p = a; p < a + bytes; p += bt::kPinPage) log->locked_pages.insert(p);
        log->locks.emplace_back(a, bytes);
        return 0;
    }
    int alias(void* lo, void** dev) {
        std::lock_guard<std::mutex> lk(log->mu);
        log->alias_calls.emplace_back(cur, (uint64_t)(uintptr_t)lo);
        *dev = reinterpret_cast<void*>(((uint64_t)(cur + 1) << 48) + (uint64_t)(uintptr_t)lo);
        return 0;
    }
    int sync(int d) {
        std::lock_guard<std::mutex> lk(log->mu);
        if (log->fail_sync) return msg = "sync failed", 1;
        log->syncs.push_back(d);
        return d != cur;   // the device being waited for must be the current one
    }
    int unlock(void* lo) {
        std::lock_guard<std::mutex> lk(log->mu);
        const uint64_t a = (uint64_t)(uintptr_t)lo;
        uint64_t bytes = 0;
        for (const auto& l : log->locks)
            if (l.first == a) bytes = l.second;
        if (!bytes) return msg = "unlock of an unlocked range", 1;
        for (uint64_t p = a; p < a + bytes; p += bt::kPinPage) log->locked_pages.erase(p);
        log->unlocks_.emplace_back(a, bytes);
        return 0;
    }
    std::string last() const { return msg; }
};

using Table = bt::PinTable<FakeDriver>;

const void* at(uint64_t a) { return reinterpret_cast<const void*>(a); }
uint64_t u(const uint8_t* p) { return (uint64_t)(uintptr_t)p; }

void basic() {
    FakeLog log;
    FakeDriver d;
    d.log = &log;
    Table t(d);
    const int dev0 = 0;
    uint8_t* al = nullptr;
    // page rounding: [0x10010, +100) locks the page 0x10000
    CHECK(t.acquire(at(0x10010), 100, &dev0, 1, &al) == Table::kOk);
    CHECK(log.locks.size() == 1 && log.locks[0] == std::make_pair<uint64_t, uint64_t>(0x10000, 4096));
    CHECK(u(al) == ((1ull << 48) + 0x10010));
    // a range inside the same page shares the span: no second lock
    uint8_t* al2 = nullptr;
    CHECK(t.acquire(at(0x10100), 50, &dev0, 1, &al2) == Table::kOk);
    CHECK(log.locks.size() == 1 && u(al2) == ((1ull << 48) + 0x10100));
    auto sp = t.spans();
    CHECK(sp.size() == 1 && sp[0].lo == 0x10000 && sp[0].hi == 0x11000 && sp[0].refs == 2);
    // a range that crosses into the next page holds only some of the span's pages: refused
    CHECK(t.acquire(at(0x10F00), 0x200, &dev0, 1, &al2) == Table::kRefused);
    CHECK(Table::error().find("shares a page") != std::string::npos);
    CHECK(log.locks.size() == 1);
    // a range ending inside the span from below: refused too
    CHECK(t.acquire(at(0xF000), 0x1100, &dev0, 1, &al2) == Table::kRefused);
    // the next page is free: a new span
    CHECK(t.acquire(at(0x11000), 4096, &dev0, 1, &al2) == Table::kOk);
    CHECK(log.locks.size() == 2 && t.spans().size() == 2);
    // alias of a sub-range on another device: taken with that device current
    uint8_t* a3 = nullptr;
    CHECK(t.alias(at(0x10020), 16, 3, &a3) == Table::kOk);
    CHECK(u(a3) == ((4ull << 48) + 0x10020));
    CHECK(!log.alias_calls.empty() && log.alias_calls.back() == std::make_pair(3, (uint64_t)0x10000));
    CHECK(t.alias(at(0x20000), 16, 0, &a3) == Table::kMissing);
    // releases: the first leaves the span, the last syncs devices 0 and 3 then unlocks
    CHECK(t.release(at(0x10100), 50) == Table::kOk);
    CHECK(log.unlocks_.empty() && log.syncs.empty());
    CHECK(t.release(at(0x10010), 100) == Table::kOk);
    CHECK(log.unlocks_.size() == 1 && log.unlocks_[0].first == 0x10000);
    CHECK((log.syncs == std::vector<int>{0, 3}));
    CHECK(log.locked_pages.count(0x10000) == 0 && log.locked_pages.count(0x11000) == 1);
    CHECK(t.release(at(0x10010), 100) == Table::kMissing);
    // a failed sync leaves the span registered (the caller may retry)
    log.fail_sync = true;
    CHECK(t.release(at(0x11000), 4096) == Table::kDriver);
    CHECK(t.spans().size() == 1 && t.spans()[0].refs == 1 && log.locked_pages.count(0x11000) == 1);
    log.fail_sync = false;
    CHECK(t.release(at(0x11000), 4096) == Table::kOk);
    CHECK(t.spans().empty() && log.locked_pages.empty());
    // the same pages can be registered again after the last release
    CHECK(t.acquire(at(0x10010), 100, &dev0, 1, &al) == Table::kOk && t.release(at(0x10010), 100) == Table::kOk);
}

void eight_members() {
    // a group over 8 devices: one lock; member k's alias is device k's, taken with device k
    // current; a sub-range's alias is the member's alias + the offset
    FakeLog log;
    FakeDriver d;
    d.log = &log;
    Table t(d);
    std::vector<int> devs = {0, 1, 2, 3, 4, 5, 6, 7};
    std::vector<uint8_t*> al(8, nullptr);
    const uint64_t base = 0x7f0000001010ull, n = 64ull << 20;
    CHECK(t.acquire(at(base), n, devs.data(), 8, al.data()) == Table::kOk);
    CHECK(log.locks.size() == 1 && log.locks[0].first == 0x7f0000001000ull &&
          log.locks[0].second == bt::PinTable<FakeDriver>::page_hi(base + n) - 0x7f0000001000ull);
    CHECK(log.alias_calls.size() == 8);
    for (int k = 0; k < 8; ++k) {
        CHECK(u(al[k]) == (((uint64_t)(k + 1) << 48) + base));
        CHECK(log.alias_calls[k].first == k);   // device k was current when its alias was taken
        uint8_t* s = nullptr;
        const uint64_t off = (uint64_t)k * (n / 8);
        CHECK(t.alias(at(base + off), n / 8, k, &s) == Table::kOk && u(s) == u(al[k]) + off);
    }
    CHECK(log.alias_calls.size() == 8);   // cached: no further driver calls
    // a second group of the same 8 devices registering the same UMEM shares it
    std::vector<uint8_t*> al2(8, nullptr);
    CHECK(t.acquire(at(base), n, devs.data(), 8, al2.data()) == Table::kOk && al2 == al && log.locks.size() == 1);
    CHECK(t.release(at(base), n) == Table::kOk && log.syncs.empty());
    CHECK(t.release(at(base), n) == Table::kOk);
    std::vector<int> synced = log.syncs;
    CHECK((synced == std::vector<int>{0, 1, 2, 3, 4, 5, 6, 7}));
    CHECK(log.locked_pages.empty());
}

void threads() {
    FakeLog log;
    FakeDriver d;
    d.log = &log;
    Table t(d);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int w = 0; w < 8; ++w)
        th.emplace_back([&, w] {
            const int dev = w;
            for (int i = 0; i < 2000; ++i) {
                const uint64_t a = 0x100000000ull + (uint64_t)((w * 2000 + i) % 64) * 4096 + 16;
                uint8_t* al = nullptr;
                const int rc = t.acquire(at(a), 100, &dev, 1, &al);
                if (rc != Table::kOk) { ++bad; continue; }
                if (u(al) >= (1ull << 48) && u(al) - a < (9ull << 48)) {
                    // alias of whichever device took it first: any of the 8
                } else {
                    ++bad;
                }
                if (t.release(at(a), 100) != Table::kOk) ++bad;
            }
        });
    for (auto& x : th) x.join();
    CHECK(bad.load() == 0);
    CHECK(t.spans().empty() && log.locked_pages.empty());
}

}  // namespace

int main() {
    basic();
    eight_members();
    threads();
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
