// bt_bounds.h — the BT_DEBUG_BOUNDS build (make -C beatrice_amd/csrc debug).
//
// In that build every global access of the kernels whose address is not already bounded
// by a buffer descriptor is checked against the range the C-ABI promises for it
// (include/beatrice_gpu.h): header-window loads against the batch's `bytes`, record /
// decision / verdict stores against n_cap / n / ntiles, the compaction's pass_idx stores
// against n, the extractor's value / image stores and its direct frame reads. A failed
// check is counted in a per-module device log (the first one in detail, and printf'd),
// and the access is dropped (a load yields zero), so a bounds bug reports itself through
// the C-ABI instead of faulting the GPU: after every launch the debug runtime waits for
// the stream, reads the log and returns BT_E_INTERNAL naming the kernel, the site, the
// index and the limit. The release build compiles every check to `true`.
#pragma once

#include <stdint.h>

namespace bt {

struct BoundsLog {
    uint32_t count;        // failed checks since the last read
    uint32_t site;         // first failure: BoundsSite
    uint32_t block, lane;
    uint64_t index;        // the offending byte / element index
    uint64_t limit;        // the bound it broke (index must be < limit)
};

enum BoundsSite : uint32_t {
    kSiteFixedLoad = 1,    // fixed-stride tile load       [0, n * stride)
    kSiteRoundA,           // round-A header chunk         [0, bytes)
    kSiteRoundB,           // round-B header chunk         [0, bytes)
    kSitePayload,          // PAYLOAD window chunk         [0, bytes)
    kSiteRecord,           // record store (tile / slot)   records capacity
    kSiteDecide,           // decision byte                [0, n)
    kSiteVerdict,          // verdict word                 [0, ntiles)
    kSiteChunkSums,        // compaction chunk sum         [0, nchunks)
    kSitePassIdx,          // compaction pass index        [0, n)
    kSiteExLoad,           // extractor staging chunk      [0, bytes)
    kSiteExFrame,          // extractor direct frame read  [0, bytes)
    kSiteExValue,          // extractor value column       [0, n_fields * n_cap)
    kSiteExImage,          // extractor image byte         [0, n * span)
    kSiteExStatus,         // extractor status byte        [0, n)
    kSiteRingHdr,          // ring walk: block / frame header read [0, ring bytes)
    kSiteRingOut,          // ring walk: descriptor / prefix write  output capacity
};

inline const char* bounds_site_name(uint32_t s) {
    static const char* const names[] = {"?", "fixed-stride load", "round-A header chunk", "round-B header chunk",
                                        "PAYLOAD window chunk", "record store", "decision store", "verdict store",
                                        "chunk sum", "pass_idx store", "extractor staging load",
                                        "extractor frame read", "extractor value store", "extractor image store",
                                        "extractor status store", "ring header read", "ring output write"};
    return s < sizeof(names) / sizeof(names[0]) ? names[s] : "?";
}

#if defined(__HIPCC__)
#ifdef BT_DEBUG_BOUNDS
// true when idx < lim; otherwise logs (vector atomics and stores only) and returns false
__device__ __noinline__ inline bool bounds_fail(BoundsLog* log, uint32_t site, uint64_t idx, uint64_t lim) {
    const uint32_t old = atomicAdd(&log->count, 1u);
    if (old == 0u) {
        log->site = site;
        log->block = blockIdx.x;
        log->lane = threadIdx.x;
        log->index = idx;
        log->limit = lim;
        printf("BT_DEBUG_BOUNDS: site %u block %u thread %u index %llu limit %llu\n", site, blockIdx.x,
               threadIdx.x, (unsigned long long)idx, (unsigned long long)lim);
    }
    return false;
}
#define BT_IN(log, site, idx, lim) \
    ((uint64_t)(idx) < (uint64_t)(lim) ? true : ::bt::bounds_fail((log), (site), (uint64_t)(idx), (uint64_t)(lim)))
#else
#define BT_IN(log, site, idx, lim) true
#endif
#endif

}  // namespace bt
