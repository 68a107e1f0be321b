#!/usr/bin/env python3
"""End-to-end (host buffers in, host buffers out) rate of bt_parse_filter: frames start
in host memory (the AF_PACKET / AF_XDP ring of the north star), header prefixes are
gathered into pinned staging, copied H2D, parsed + filtered, and records / decisions
copied D2H, double-buffered over two streams. PCIe-inclusive; reported in DESIGN.md."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4"])
ap.add_argument("--packets", type=int, default=1 << 24)
ap.add_argument("--chunk", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--zero-copy", action="store_true",
                help="register the host capture (bt_host_register) and let the kernel read the "
                     "header windows over PCIe: no host gather (AF_XDP UMEM style)")
ap.add_argument("--tpacket", action="store_true",
                help="pack the capture into an AF_PACKET TPACKET_V3 ring image (kernel layout), register "
                     "it, and run ring -> walk (bt_ring_walk_tpv3, host pool) -> kernels reading frames "
                     "in place -> outputs in registered host memory, walking batch k+1 while batch k runs")
ap.add_argument("--gather", action="store_true",
                help="with --tpacket: the walker also copies each frame's header prefix into 128-B pinned "
                     "slots (bt_ring_gather_tpv3) and the kernels read the slots (BT_BATCH_PREFIXES)")
ap.add_argument("--dense", action="store_true",
                help="with --gather: each block's prefixes packed back to back (bt_ring_gather_dense_tpv3)")
ap.add_argument("--lean", action="store_true",
                help="with --gather: each frame's bytes 12..43 packed back to back (bt_ring_gather_lean_tpv3, "
                     "BT_BATCH_LEAN): verdict rows only")
ap.add_argument("--mix", type=int, default=0,
                help="with --gather: every N-th batch is walked and read in place instead (the host "
                     "gathers, the GPU reads the other batches' frames over PCIe itself)")
ap.add_argument("--gpu-walk", action="store_true",
                help="with --tpacket: the frame chains are walked on the GPU (bt_ring_walk_tpv3_gpu: the host "
                     "reads only the block headers), descriptors in device memory")
ap.add_argument("--host-gather", action="store_true",
                help="with --tpacket: walk each batch of blocks, then bt_parse_filter over the ring and those "
                     "descriptors (the host pipeline's prefetched gather -> H2D -> kernels -> D2H) instead of "
                     "the kernels reading the frames in place")
ap.add_argument("--ring-batch-blocks", type=int, default=128)
ap.add_argument("--flags", type=lambda x: int(x, 0), default=0, help="bt_opts.flags (A/B, e.g. 0x8000 no lean PCIe round A)")
ap.add_argument("--host-threads", type=int, default=0)
ap.add_argument("--data-node", default="none",
                help="'auto': move the capture onto the device's NUMA node (where the context pins its "
                     "gather threads) before timing, as a NUMA-aware capture allocates its ring; N: that node; "
                     "'none': where the generator's threads first touched it (the default)")
ap.add_argument("--group", type=int, default=0,
                help="drive a bt_group of N members (devices 0..N-1; members share device 0 when fewer GPUs "
                     "are visible, labelled 'shared device'): host gather (bt_group_parse_filter) and zero-copy "
                     "(bt_group_host_register + bt_group_parse_filter_mapped) rows, with host CPU-seconds per Mpkt")
ap.add_argument("--hugepages", action="store_true",
                help="with --data-node: ask for transparent huge pages for the bound capture mapping")
ap.add_argument("--register-outputs", action="store_true",
                help="host-gather rows (one context): register the output arrays (bt_host_register), so the "
                     "host pipeline copies them D2H in place instead of through its staging")
ap.add_argument("--fresh-outputs", action="store_true",
                help="host-gather rows: allocate the output arrays inside every call (rounds 1-4's form) "
                     "instead of once, as a capture loop reuses them")
a = ap.parse_args()
cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4}[a.config]
data, desc = synth.capture(cfg, a.packets)


from beatrice_amd.numa import page_nodes, place_on  # noqa: E402


def place(arr, node):
    out = place_on(arr, node, hugepages=a.hugepages)
    # registration is in whole pages: a capture that may be registered gets pages of its own
    return abi.host_copy(arr) if out is arr else out


def data_node_for(placement):
    if a.data_node == "none":
        return None
    return placement["numa_node"] if a.data_node == "auto" else int(a.data_node)


FILTERS = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
           {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
           {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]

if a.group:
    import numpy as np
    m = a.group
    shared = abi.device_count() < m
    devices = [0] * m if shared else list(range(m))
    grp = abi.Group(devices, host_chunk_packets=a.chunk, host_threads=a.host_threads,
                    flags=a.flags | (abi.OPT_GROUP_SHARED_DEVICE if shared else 0))
    grp.compile(FILTERS)
    data = place(data, data_node_for(grp.placement(0)))
    n = a.packets
    where = {"members": m, "devices": devices, "shared_device": shared, "usable_cpus": abi.usable_cpus(),
             "flags": a.flags,
             "placement": [grp.placement(k) for k in range(m)], "data_nodes": page_nodes(data),
             "numa_pin": os.environ.get("BT_NUMA_PIN", "1"), "shared_serial": os.environ.get("BT_GROUP_SHARED_SERIAL", "0"),
             "outputs": "fresh per call" if a.fresh_outputs else "allocated once"}

    def timed(fn):
        best, cpu = 1e9, 0.0
        fn()   # warm
        for _ in range(a.reps):
            c0, t0 = time.process_time(), time.perf_counter()
            fn()
            dt, dc = time.perf_counter() - t0, time.process_time() - c0
            if dt < best:
                best, cpu = dt, dc
        return best, cpu

    for mode in ("verdicts", "records+verdicts"):
        rec = mode != "verdicts"
        houts = None if a.fresh_outputs else abi.host_outputs(a.packets, records=rec)
        best, cpu = timed(lambda: grp.run_host(data, desc, records=rec, outs=houts))
        print(json.dumps({"config": a.config, "flags": a.flags, "mode": f"group {m}, host gather, {mode}",
                          "packets": n, "seconds": round(best, 4), "mpps": round(n / best / 1e6, 1),
                          "host_cpu_s_per_mpkt": round(cpu / (n / 1e6), 4), "cost_model": grp.cost(False, rec, True),
                          **where}), flush=True)
    tiles = (n + 63) // 64
    h_dec = abi.host_array(tiles * 64, np.uint8)
    h_ver = abi.host_array(tiles, np.uint64)
    desc = abi.host_copy(desc)
    for arr in (data, desc, h_dec, h_ver):
        grp.register(arr)
    for mode in ("verdicts", "records+verdicts"):
        rec = mode != "verdicts"
        h_rec = abi.host_array(tiles * 6144, np.uint8) if rec else None
        if rec:
            grp.register(h_rec)
        batch = abi.Batch(data.ctypes.data, desc.ctypes.data, 0, n, data.nbytes, abi.DESC_PACKED, 0)
        outs = abi.Outputs(h_rec.ctypes.data if rec else None, n, h_ver.ctypes.data, h_dec.ctypes.data, None, None)
        best, cpu = timed(lambda: grp.run_mapped(batch, outs))
        print(json.dumps({"config": a.config, "flags": a.flags, "mode": f"group {m}, zero-copy in and out, {mode}",
                          "packets": n, "seconds": round(best, 4), "mpps": round(n / best / 1e6, 1),
                          "host_cpu_s_per_mpkt": round(cpu / (n / 1e6), 4), "cost_model": grp.cost(True, rec, True),
                          **where}), flush=True)
        if rec:
            grp.unregister(h_rec)
    for arr in (data, desc, h_dec, h_ver):
        grp.unregister(arr)
    grp.close()
    sys.exit(0)
ctx = abi.Context(0, host_chunk_packets=a.chunk, host_threads=a.host_threads, flags=a.flags)
ctx.compile(FILTERS)
data = place(data, data_node_for(ctx.placement()))
if a.tpacket:
    import numpy as np
    ring, rdesc, used = synth.tpv3_ring(data, desc)
    del data
    ring = place(ring, data_node_for(ctx.placement()))
    bs, n = synth.TPV3_BLOCK, len(rdesc)
    B = a.ring_batch_blocks
    nbat = (used + B - 1) // B
    d_ring = ctx.register(ring)
    h_desc = abi.host_array(n + 64, np.uint64)
    d_desc = ctx.register(h_desc)
    if a.gather:
        slots = abi.host_array((n + 64) * abi.PREFIX_SLOT, np.uint8)
        d_slots = ctx.register(slots)
    if a.gpu_walk:
        g_desc = ctx.alloc(8 * (n + 64))
    for mode in ("verdicts",) if a.lean else ("verdicts", "records+verdicts"):
        rec = mode != "verdicts"
        tiles = (n + 63) // 64 + nbat + 1          # each batch starts its outputs on a fresh tile
        h_dec = abi.host_array(tiles * 64, np.uint8)
        h_ver = abi.host_array(tiles, np.uint64)
        h_rec = abi.host_array(tiles * 6144, np.uint8) if rec else None
        h_recs = np.zeros(n * 96, np.uint8) if rec and a.host_gather else None   # bt_rec, AoS
        d_dec, d_ver = ctx.register(h_dec), ctx.register(h_ver)
        d_rec = ctx.register(h_rec) if rec else None

        counts = []

        def one_pass(walk=True):
            start, tile = 0, 0
            for k in range(nbat):
                gathered = a.gather and not (a.mix and k % a.mix == a.mix - 1)
                if walk and gathered:
                    got, taken = abi.ring_gather_tpv3(ring, bs, used, slots, h_desc, first=k * B,
                                                      max_blocks=min(B, used - k * B), ctx=ctx, slot_base=start,
                                                      dense=a.dense, lean=a.lean)
                    cnt = len(got)
                    if len(counts) < nbat:
                        counts.append(cnt)
                elif walk and a.gpu_walk:
                    cnt, taken = abi.ring_walk_tpv3_gpu(ctx, ring, d_ring, bs, used, g_desc.ptr + 8 * start,
                                                        n + 64 - start, first=k * B, max_blocks=min(B, used - k * B))
                    if len(counts) < nbat:
                        counts.append(cnt)
                elif walk:
                    got, taken = abi.ring_walk_tpv3(ring, bs, used, first=k * B, max_blocks=min(B, used - k * B),
                                                    ctx=ctx, out=h_desc[start:])
                    cnt = len(got)
                    if len(counts) < nbat:
                        counts.append(cnt)
                else:
                    cnt = counts[k]
                if a.host_gather:   # synchronous: the host pipeline over the ring + this batch's descriptors
                    p = lambda arr, off: None if arr is None else arr.ctypes.data + off  # noqa: E731
                    rc = abi.lib().bt_parse_filter(ctx.h, ring.ctypes.data, h_desc.ctypes.data + 8 * start, cnt,
                                                   p(h_recs, 96 * start), p(h_ver, 8 * tile), p(h_dec, 64 * tile),
                                                   None, None)
                    assert rc == 0, abi.lib().bt_last_error()
                    start += cnt
                    tile += (cnt + 63) // 64
                    continue
                if gathered:
                    batch = abi.Batch(d_slots + abi.PREFIX_SLOT * start, d_desc + 8 * start, 0, cnt,
                                      abi.PREFIX_SLOT * cnt, abi.DESC_PACKED,
                                      abi.BATCH_PREFIXES | (abi.BATCH_LEAN if a.lean else 0))
                else:
                    dd = g_desc.ptr if a.gpu_walk else d_desc
                    batch = abi.Batch(d_ring, dd + 8 * start, 0, cnt, ring.nbytes, abi.DESC_PACKED, 0)
                outs = abi.Outputs(d_rec + 6144 * tile if rec else None, cnt, d_ver + 8 * tile, d_dec + 64 * tile,
                                   None, None)
                ctx.run_device(batch, outs)      # async: the next walk overlaps this batch
                start += cnt
                tile += (cnt + 63) // 64
            ctx.synchronize()
            return start

        best = 1e9
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            done = one_pass()
            best = min(best, time.perf_counter() - t0)
        assert done == n
        kbest = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            one_pass(walk=False)
            kbest = min(kbest, time.perf_counter() - t0)
        t0 = time.perf_counter()
        for k in range(nbat):
            if a.gpu_walk:
                abi.ring_walk_tpv3_gpu(ctx, ring, d_ring, bs, used, g_desc.ptr, n + 64, first=k * B,
                                       max_blocks=min(B, used - k * B))
                continue
            if a.gather and not (a.mix and k % a.mix == a.mix - 1):
                abi.ring_gather_tpv3(ring, bs, used, slots, h_desc, first=k * B, max_blocks=min(B, used - k * B),
                                     ctx=ctx, dense=a.dense, lean=a.lean)
            else:
                abi.ring_walk_tpv3(ring, bs, used, first=k * B, max_blocks=min(B, used - k * B), ctx=ctx,
                                   out=h_desc[:])
        ctx.synchronize()
        walk = time.perf_counter() - t0
        lens = synth.desc_len(rdesc)
        pcie = float(np.minimum(lens, 64).sum() + 8 * n)
        how = "tpacket_v3 ring, walk then host gather (bt_parse_filter), " if a.host_gather else \
            f"tpacket_v3 ring, lean gather (bytes 12..43) per block, every {a.mix}th batch in place, zero-copy, " \
            if a.gather and a.lean and a.mix else \
            "tpacket_v3 ring, lean gather (bytes 12..43) per block, zero-copy, " if a.gather and a.lean else \
            f"tpacket_v3 ring, header gather packed per block, every {a.mix}th batch in place, zero-copy, " \
            if a.gather and a.dense and a.mix else \
            "tpacket_v3 ring, header gather packed per block, zero-copy, " if a.gather and a.dense else \
            "tpacket_v3 ring, header gather into 128-B slots, zero-copy, " if a.gather else \
            "tpacket_v3 ring, chains walked on the GPU, zero-copy, " if a.gpu_walk else "tpacket_v3 ring, zero-copy, "
        print(json.dumps({"config": a.config, "flags": a.flags, "mode": how + mode, "packets": n,
                          "ring_blocks": used, "block_bytes": bs, "batch_blocks": B, "seconds": round(best, 4),
                          "mpps": round(n / best / 1e6, 1), "walk_only_mpps": round(n / walk / 1e6, 1),
                          "kernels_only_mpps": round(n / kbest / 1e6, 1),
                          "pcie_read_GBps": round(pcie / best / 1e9, 2),
                          "pcie_write_GBps": round(n * (1.125 + (96 if rec else 0)) / best / 1e9, 2)}), flush=True)
        for h in (h_dec, h_ver) + ((h_rec,) if rec else ()):
            ctx.unregister(h)
    ctx.unregister(h_desc)
    ctx.unregister(ring)
    if a.gpu_walk:
        g_desc.free()
    if a.gather:
        ctx.unregister(slots)
    sys.exit(0)

if a.zero_copy:
    import numpy as np
    desc = abi.host_copy(desc)
    d_data = ctx.register(data)
    d_desc = ctx.register(desc)
    n = a.packets
    for mode in ("verdicts", "records+verdicts"):
        rec = mode != "verdicts"
        run = abi.DeviceRun(ctx, np.zeros(256, np.uint8), None, n, stride=1, records=rec)
        run.batch = abi.Batch(d_data, d_desc, 0, n, data.nbytes, abi.DESC_PACKED, 0)
        # outputs come back to host memory: decisions + verdict words (+ records)
        h_dec = abi.host_array(n, np.uint8)
        h_ver = abi.host_array((n + 63) // 64, np.uint64)
        h_rec = abi.host_array(((n + 63) // 64) * 6144, np.uint8) if rec else None
        best = 1e9
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            run.run()
            run.d_dec.download(h_dec)
            run.d_ver.download(h_ver)
            if rec:
                run.d_rec.download(h_rec)
            best = min(best, time.perf_counter() - t0)
        lens = synth.desc_len(desc)
        pcie = float(np.minimum(lens, 64).sum() + 8 * n)
        print(json.dumps({"config": a.config, "flags": a.flags, "mode": "zero-copy in, D2H copy out, " + mode, "packets": n,
                          "seconds": round(best, 4), "mpps": round(n / best / 1e6, 1),
                          "pcie_read_GBps": round(pcie / best / 1e9, 2),
                          "d2h_GBps": round(n * (1.125 + (96 if rec else 0)) / best / 1e9, 2)}), flush=True)
        # fully zero-copy: the kernel writes decisions / verdicts / records into registered host memory
        d_dec, d_ver = ctx.register(h_dec), ctx.register(h_ver)
        d_rec = ctx.register(h_rec) if rec else None
        outs = abi.Outputs(d_rec, n, d_ver, d_dec, None, None)
        best = 1e9
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            ctx.run_device(run.batch, outs)
            ctx.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"config": a.config, "flags": a.flags, "mode": "zero-copy in and out, " + mode, "packets": n,
                          "seconds": round(best, 4), "mpps": round(n / best / 1e6, 1),
                          "pcie_read_GBps": round(pcie / best / 1e9, 2),
                          "pcie_write_GBps": round(n * (1.125 + (96 if rec else 0)) / best / 1e9, 2)}), flush=True)
        ctx.unregister(h_dec)
        ctx.unregister(h_ver)
        if rec:
            ctx.unregister(h_rec)
        run.free()
    ctx.unregister(desc)
    ctx.unregister(data)
    sys.exit(0)

for mode in ("verdicts", "records+verdicts"):
    rec = mode != "verdicts"
    ctx.run_host(data[: 1 << 20], desc[: 1 << 14], records=rec)     # warm pinned buffers
    houts = None if a.fresh_outputs else abi.host_outputs(a.packets, records=rec)
    regs = [houts[k] for k in ("records", "decide", "verdict") if houts and houts[k] is not None] \
        if a.register_outputs else []
    for arr in regs:
        ctx.register(arr)
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = ctx.run_host(data, desc, records=rec, outs=houts)
        best = min(best, time.perf_counter() - t0)
    for arr in regs:
        ctx.unregister(arr)
    lens = synth.desc_len(desc)
    if rec:
        staged = lens.clip(max=112)
    elif a.flags & abi.OPT_NO_LEAN_HOST:
        staged = lens.clip(max=48)
    else:   # filter-only: frame bytes 12..43
        staged = (lens.astype(np.int64) - 12).clip(min=0, max=32)
    h2d = float((((staged + 15) // 16) * 16).sum() + 8 * a.packets)
    d2h = a.packets * (1 + 1 / 8 + (96 if rec else 0))
    print(json.dumps({"config": a.config, "flags": a.flags, "mode": mode, "packets": a.packets, "seconds": round(best, 4),
                      "mpps": round(a.packets / best / 1e6, 1), "h2d_GBps": round(h2d / best / 1e9, 2),
                      "d2h_GBps": round(d2h / best / 1e9, 2), "n_pass": out["n_pass"], "data_nodes": page_nodes(data),
                      "placement": ctx.placement(), "numa_pin": os.environ.get("BT_NUMA_PIN", "1"),
                      "outputs": ("fresh per call" if a.fresh_outputs else "allocated once")
                      + (", registered" if regs else "")}), flush=True)
