// bt_host.h — runtime services shared by the host-only translation units of
// libbeatrice_gpu.so (bt_ring.cpp): the thread-local error slot behind
// bt_last_error() and the context's host thread pool.
#pragma once

#include <functional>

#include "beatrice_gpu.h"

namespace bt {

// Sets bt_last_error() and returns `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Runs fn(worker, n_workers) on every worker of ctx's host pool (the caller is
// worker 0) and waits; with ctx == NULL it runs fn(0, 1) inline.
void host_parallel(bt_ctx* ctx, const std::function<void(unsigned, unsigned)>& fn);

}  // namespace bt
