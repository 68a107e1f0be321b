// bt_pin.cpp — the process's one table of registered host pages (bt_pin.h) over HIP.
#include <hip/hip_runtime_api.h>

#include <string>

#include "bt_hip_util.h"
#include "bt_host.h"
#include "bt_pin.h"

namespace bt {
namespace {

struct HipPinDriver {
    hipError_t err = hipSuccess;
    int note(hipError_t e) {
        if (e != hipSuccess) {
            err = e;
            (void)hipGetLastError();
        }
        return e != hipSuccess;
    }
    int set_device(int d) { return note(hipSetDevice(d)); }
    // portable: every device may be handed an alias; mapped: kernels read it in place
    int lock(void* lo, uint64_t bytes) {
        return note(hipHostRegister(lo, bytes, hipHostRegisterPortable | hipHostRegisterMapped));
    }
    int alias(void* lo, void** dev) { return note(hipHostGetDevicePointer(dev, lo, 0)); }
    int sync(int) { return note(hipDeviceSynchronize()); }   // the device set_device selected
    int unlock(void* lo) { return note(hipHostUnregister(lo)); }
    std::string last() const { return hipGetErrorString(err); }
};

using Table = PinTable<HipPinDriver>;

Table& table() {
    static Table t;
    return t;
}

int translate(int rc) {
    if (rc == Table::kOk) return BT_OK;
    return set_error(rc == Table::kDriver ? BT_E_INTERNAL : BT_E_INVALID_ARGUMENT, "%s", Table::error().c_str());
}

}  // namespace

int pin_acquire(const void* host, uint64_t bytes, const int* devices, uint32_t n_devices, uint8_t** aliases) {
    const DeviceRestore keep;
    return translate(table().acquire(host, bytes, devices, n_devices, aliases));
}

int pin_alias(const void* host, uint64_t bytes, int device, uint8_t** alias) {
    const DeviceRestore keep;
    return translate(table().alias(host, bytes, device, alias));
}

int pin_release(const void* host, uint64_t bytes) {
    const DeviceRestore keep;
    return translate(table().release(host, bytes));
}

uint32_t pin_spans(uint64_t* lo_hi_refs, uint32_t cap) {
    const auto v = table().spans();
    for (uint32_t i = 0; i < cap && i < v.size(); ++i) {
        lo_hi_refs[3 * i] = v[i].lo;
        lo_hi_refs[3 * i + 1] = v[i].hi;
        lo_hi_refs[3 * i + 2] = v[i].refs;
    }
    return (uint32_t)v.size();
}

}  // namespace bt

extern "C" int bt_host_alias(const void* host, uint64_t bytes, int device, void** alias) {
    if (!host || !alias) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    uint8_t* a = nullptr;
    if (int rc = bt::pin_alias(host, bytes, device, &a)) return rc;
    *alias = a;
    return BT_OK;
}

extern "C" int bt_host_pins(uint64_t* lo_hi_refs, uint32_t cap, uint32_t* n) {
    if (!n || (cap && !lo_hi_refs)) return bt::set_error(BT_E_INVALID_ARGUMENT, "null argument");
    *n = bt::pin_spans(lo_hi_refs, cap);
    return BT_OK;
}
