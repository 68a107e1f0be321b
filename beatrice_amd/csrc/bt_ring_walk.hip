// bt_ring_walk.hip — the TPACKET_V3 frame-chain walk on the GPU.
//
// The host walker (bt_ring.cpp) follows every block's frame chain in host memory. Here the
// host only reads the taken blocks' headers (status, num_pkts, first frame offset: one
// line per block, bt_ring_walk_tpv3_gpu) and the GPU follows the chains through the
// device-visible ring (its bt_host_register alias): one lane per block, each hop reading
// the frame's tpacket3_hdr (tp_next_offset @0, tp_snaplen @12, tp_mac @24) and writing the
// frame's bt_pkt_desc straight into device memory, where the parse+filter kernels take it.
//
// Each hop is a dependent read through PCIe (≈ 1-2 µs), so a lane walks one block at that
// latency and the rate is the number of blocks in flight over it: the walk suits large
// batches of blocks. The hops also move the frame headers' lines across PCIe a second time
// (the parse reads the frame windows, which start 82 B later, in other lines): DESIGN.md
// §9.2 has the measurements against the host walker.
#include <hip/hip_runtime.h>

#include "bt_device.h"

namespace bt {

__device__ BoundsLog g_bounds_ring;

namespace {

__global__ __launch_bounds__(64) void bt_ring_walk_chains(RingWalkArgs a) {
    const uint32_t k = blockIdx.x * 64u + threadIdx.x;
    if (k >= a.count) return;
    const RingBlock rb = a.blocks[k];
    const uint8_t* blk = a.ring + (uint64_t)rb.block * a.block_size;
    const uint64_t base_off = (uint64_t)rb.block * a.block_size;
    bt_pkt_desc* out = a.desc + rb.start;
    uint64_t off = rb.first_off;
    uint32_t j = 0;
    bool ok = true;
    for (; j < rb.n; ++j) {
        // tpacket3_hdr (48 B, linux/if_packet.h) inside the block, as the host walker checks;
        // the kernel places frames 8-B aligned (a chain off 4-B alignment counts as malformed)
        if (off + 48u > a.block_size || (off & 3u)) {
            ok = false;
            break;
        }
        const uint32_t* h = reinterpret_cast<const uint32_t*>(blk + off);
        const uint32_t next = h[0], snap = h[3], mac = h[6] & 0xFFFFu;   // tp_next_offset, tp_snaplen, tp_mac
        if (off + mac + snap > a.block_size) {
            ok = false;
            break;
        }
        if (BT_IN(&g_bounds_ring, kSiteRingOut, rb.start + j, a.cap))
            out[j] = (base_off + off + mac) | ((uint64_t)(snap < 0xFFFFu ? snap : 0xFFFFu) << 48);
        if (j + 1u < rb.n) {
            if (next < 48u) {
                ok = false;
                ++j;
                break;
            }
            off += next;
        }
    }
    if (!ok) {
        // a chain that leaves its block: its remaining frames become empty descriptors (no
        // byte of them is read), and the block is reported
        for (; j < rb.n; ++j)
            if (BT_IN(&g_bounds_ring, kSiteRingOut, rb.start + j, a.cap)) out[j] = 0ull;
        if (a.bad) atomicMax(a.bad, rb.block + 1u);
    }
}

}  // namespace

int launch_ring_walk(const RingWalkArgs& a, void* stream) {
    if (!a.count) return BT_OK;
    hipLaunchKernelGGL(bt_ring_walk_chains, dim3((a.count + 63u) / 64u), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    return hipGetLastError() == hipSuccess ? BT_OK : BT_E_INTERNAL;
}

uint32_t bounds_take_ring(void* stream, BoundsLog* first) {
#ifdef BT_DEBUG_BOUNDS
    if (hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return 0;
    BoundsLog log{};
    if (hipMemcpyFromSymbol(&log, HIP_SYMBOL(g_bounds_ring), sizeof(log)) != hipSuccess) return 0;
    if (log.count) {
        const BoundsLog zero{};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_ring), &zero, sizeof(zero));
        if (first) *first = log;
    }
    return log.count;
#else
    (void)stream;
    (void)first;
    return 0;
#endif
}

}  // namespace bt
