// bt_hip_util.h — HIP helpers shared by the hipcc-compiled host units (bt_runtime.cpp,
// bt_group.cpp, bt_pin.cpp).
#pragma once

#include <hip/hip_runtime_api.h>

namespace bt {

// The C-ABI's entry points select their context's device (hipSetDevice) before they
// launch, allocate or wait. A host thread that drives several devices must find its own
// current device unchanged when the call returns, so every such entry point holds one of
// these: it records the calling thread's current device and restores it on the way out.
struct DeviceRestore {
    int dev = -1;
    DeviceRestore() {
        if (hipGetDevice(&dev) != hipSuccess) {
            dev = -1;
            (void)hipGetLastError();
        }
    }
    ~DeviceRestore() {
        int cur = -1;
        if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
    }
    DeviceRestore(const DeviceRestore&) = delete;
    DeviceRestore& operator=(const DeviceRestore&) = delete;
};

}  // namespace bt
