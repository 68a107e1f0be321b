// bt_pin.h — the process's registered host page spans (bt_host_register,
// bt_group_host_register, a group's scratch verdict words).
//
// hipHostRegister page-locks and maps whole pages whatever byte range it is given, and the
// registration is the process's, not a context's: every device can reach it through its own
// alias (hipHostGetDevicePointer after selecting the device). Round 5's registrations were
// byte ranges kept per owner (the context's list, each group's regions), so two live
// registrations could hold the same page through two HIP registrations, a context and a group
// could both register one UMEM, and no table said which pages were locked. This table is the
// one record of what is registered, in whole pages:
//   * a request is rounded out to the pages that hold it, [lo, hi);
//   * a request inside a live span's pages takes a reference on that span: no second HIP
//     registration, the alias is the span's alias + the offset (a context and a group sharing
//     a UMEM, an output array carved out of a registered arena);
//   * a request whose pages overlap a live span only in part is refused (BT_E_INVALID_ARGUMENT,
//     naming the span): one page is never locked twice, so releasing one registration never
//     unlocks or unmaps a page another one still covers;
//   * a span is unregistered when its last reference goes, after every device that was handed
//     an alias of it has finished its queued work.
// The HIP calls go through a Driver policy (bt_pin.cpp: the real one) so the bookkeeping and a
// group's per-member alias lookup run on the CPU in tests/cpp/test_pin.cpp with a fake driver
// that gives every device its own alias space.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace bt {

constexpr uint64_t kPinPage = 4096;

// Driver: int set_device(int d); int lock(void* lo, uint64_t bytes);
//         int alias(void* lo, void** dev);   (for the current device)
//         int sync(int d); int unlock(void* lo); std::string last();
// every int is 0 on success.
template <class Driver>
class PinTable {
public:
    struct Span {
        uint64_t lo = 0, hi = 0;   // page-aligned host range
        uint32_t refs = 0;
        std::vector<std::pair<int, uint8_t*>> alias;   // device -> alias of lo
    };
    enum { kOk = 0, kRefused = 1, kDriver = 2, kMissing = 3 };

    explicit PinTable(Driver d = Driver()) : drv_(std::move(d)) {}

    static uint64_t page_lo(uint64_t a) { return a & ~(kPinPage - 1); }
    static uint64_t page_hi(uint64_t a) { return (a + kPinPage - 1) & ~(kPinPage - 1); }

    // Takes a reference on the pages of [p, p + n) (registering them if no span holds them)
    // and, for each device of devs, writes the alias of p to dev_alias[i] (may be null).
    int acquire(const void* p, uint64_t n, const int* devs, uint32_t ndev, uint8_t** dev_alias) {
        std::lock_guard<std::mutex> lk(mu_);
        const uint64_t a = (uint64_t)(uintptr_t)p, lo = page_lo(a), hi = page_hi(a + n);
        Span* s = find_locked(lo);
        if (s && hi <= s->hi) {
            for (uint32_t i = 0; i < ndev; ++i) {
                uint8_t* d = nullptr;
                if (int rc = alias_locked(*s, devs[i], &d)) return rc;
                if (dev_alias) dev_alias[i] = d + (a - s->lo);
            }
            ++s->refs;
            return kOk;
        }
        // any live span overlapping [lo, hi) in part
        auto it = spans_.lower_bound(lo);
        if (it != spans_.begin()) {
            auto pv = std::prev(it);
            if (pv->second.hi > lo) return refuse(a, n, pv->second);
        }
        if (it != spans_.end() && it->second.lo < hi) return refuse(a, n, it->second);
        if (ndev == 0) return fail("no device to register [%p, +%llu) for", p, (unsigned long long)n);
        if (drv_.set_device(devs[0]) || drv_.lock(reinterpret_cast<void*>(lo), hi - lo))
            return fail("hipHostRegister of pages [%#llx, %#llx): %s", (unsigned long long)lo, (unsigned long long)hi,
                        drv_.last().c_str());
        Span ns;
        ns.lo = lo;
        ns.hi = hi;
        ns.refs = 1;
        for (uint32_t i = 0; i < ndev; ++i) {
            uint8_t* d = nullptr;
            if (int rc = alias_locked(ns, devs[i], &d)) {
                (void)drv_.unlock(reinterpret_cast<void*>(lo));
                return rc;
            }
            if (dev_alias) dev_alias[i] = d + (a - lo);
        }
        spans_.emplace(lo, std::move(ns));
        return kOk;
    }

    // The alias on device `dev` of [p, p + n), which must lie inside one live span.
    int alias(const void* p, uint64_t n, int dev, uint8_t** out) {
        std::lock_guard<std::mutex> lk(mu_);
        const uint64_t a = (uint64_t)(uintptr_t)p;
        Span* s = find_locked(page_lo(a));
        if (!s || a + n > s->hi) return fail_code(kMissing, "[%p, +%llu) is not inside a registered span", p, (unsigned long long)n);
        uint8_t* d = nullptr;
        if (int rc = alias_locked(*s, dev, &d)) return rc;
        *out = d + (a - s->lo);
        return kOk;
    }

    // Drops the reference acquire(p, n) took; the last one waits for every device holding an
    // alias and unregisters the span.
    int release(const void* p, uint64_t n) {
        std::lock_guard<std::mutex> lk(mu_);
        const uint64_t a = (uint64_t)(uintptr_t)p;
        Span* s = find_locked(page_lo(a));
        if (!s || page_hi(a + n) > s->hi) return fail_code(kMissing, "[%p, +%llu) is not registered", p, (unsigned long long)n);
        if (--s->refs) return kOk;
        for (const auto& x : s->alias)
            if (drv_.set_device(x.first) || drv_.sync(x.first)) {
                ++s->refs;   // still registered: the caller may retry
                return fail("device %d before unregistering [%#llx, %#llx): %s", x.first, (unsigned long long)s->lo,
                            (unsigned long long)s->hi,
                            drv_.last().c_str());
            }
        const uint64_t lo = s->lo;
        const int rc = drv_.unlock(reinterpret_cast<void*>(lo));
        spans_.erase(lo);
        if (rc) return fail("hipHostUnregister of pages at %#llx: %s", (unsigned long long)lo, drv_.last().c_str());
        return kOk;
    }

    // (lo, hi, refs) of every live span, ascending (tests, diagnostics).
    std::vector<Span> spans() const {
        std::lock_guard<std::mutex> lk(mu_);
        std::vector<Span> v;
        for (const auto& x : spans_) v.push_back(x.second);
        return v;
    }
    // The message of this thread's last failed call.
    static const std::string& error() { return err_; }
    Driver& driver() { return drv_; }

private:
    Span* find_locked(uint64_t lo_page) {
        auto it = spans_.upper_bound(lo_page);
        if (it == spans_.begin()) return nullptr;
        --it;
        return lo_page < it->second.hi ? &it->second : nullptr;
    }
    int alias_locked(Span& s, int dev, uint8_t** out) {
        for (const auto& x : s.alias)
            if (x.first == dev) {
                *out = x.second;
                return kOk;
            }
        void* d = nullptr;
        if (drv_.set_device(dev) || drv_.alias(reinterpret_cast<void*>(s.lo), &d) || !d)
            return fail("hipHostGetDevicePointer on device %d for pages at %#llx: %s", dev, (unsigned long long)s.lo,
                        drv_.last().c_str());
        s.alias.emplace_back(dev, static_cast<uint8_t*>(d));
        *out = static_cast<uint8_t*>(d);
        return kOk;
    }
    int refuse(uint64_t a, uint64_t n, const Span& s) {
        return fail_code(kRefused,
                         "host range [%#llx, +%llu) shares a page with the registered pages [%#llx, %#llx) but is not "
                         "inside them: register page-aligned buffers, or one range that covers both",
                         (unsigned long long)a, (unsigned long long)n, (unsigned long long)s.lo,
                         (unsigned long long)s.hi);
    }
    template <class... A>
    int fail(const char* fmt, A... a) {
        return fail_code(kDriver, fmt, a...);
    }
    template <class... A>
    int fail_code(int code, const char* fmt, A... a) {
        char buf[512];
        snprintf(buf, sizeof(buf), fmt, a...);
        err_ = buf;
        return code;
    }

    Driver drv_;
    mutable std::mutex mu_;
    std::map<uint64_t, Span> spans_;
    inline static thread_local std::string err_;
};

}  // namespace bt
