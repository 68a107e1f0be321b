#!/usr/bin/env python3
"""Benchmark of the device-resident parse+filter hot path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--config c2f|c2|c3|c4] [--configs LIST|none]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

--gpus N without a launcher (WORLD_SIZE unset) starts the N rank processes itself, before
anything touches a GPU (subprocess, never exec), rank r on device r, rendezvous on
127.0.0.1; under a launcher --gpus must equal WORLD_SIZE. Every rank checks that the ranks
drive distinct devices (PCI bus ids) unless BT_BENCH_DEVICE pins them all to one device (a
multi-rank rehearsal on a 1-GPU box, reported as such in the line).

A step = one bt_parse_filter_device() pass over one synthetic 16M-packet batch that is
already resident in HBM (the reference's batch entry it replaces:
PacketFilter::applyFilters(const std::vector<Packet>&), src/PacketFilter.cpp:121-130,
plus ProtocolParser::parsePacket per walked layer, src/parser/ProtocolParser.cpp:69-95).

The headline (`value`) is the metric's 64-B case: "c2f" = 16,777,216 fixed 64-B
Eth/IPv4/UDP frames (BASELINE configs[1]'s frames), parsed into packed records (48 B
per packet on the device for untagged Eth/IPv4/UDP) AND filtered by C3's 5-tuple
PacketFilter set (PROTOCOL udp, IP_RANGE 10.0.0.0/8, PORT_RANGE 1000-2000) with ordered
pass-index compaction. The same run adds a `configs` object with one entry per other
BASELINE config, each with its own ms_per_step, Mpps, roofline and CPU baseline:
  c2  configs[1]: the same frames, parse-only
  c3  configs[2]: IMIX 64/512/1500 Eth/VLAN/IPv4/{TCP,UDP}, parse + filter + compaction
  c4  configs[3]: QinQ/IPv6/IHL+TCP options at 2-mod-4 offsets, parse + filter
  c1  configs[0]'s protocol: parser_example's user table (ProtocolParser::parsePacket(frame,
      ProtocolDefinition)) extracted on the GPU from the C2 frames, next to the
      reference's own parsePacket on the host CPUs
At N > 1 (C5, configs[4]) the entries are c3 (weak scaling: 16M IMIX packets per GPU)
and c3_strong (one 16M IMIX batch split into tile-aligned, byte-balanced shards); the
headline is weak scaling. Packet batches shard with no collective: the only cross-rank
traffic is the timing barrier and the gathers of the per-rank times, over gloo.

Captures are generated range by range on the host (bt_synth_fill_range) and streamed to
the device, so no rank holds a whole capture in host memory.

Timing: W untimed warm-up steps; then barrier + device sync, K steps, device sync +
barrier; each rank's clock runs from its release at the opening barrier to its closing sync
(the closing barrier's latency is reported, not counted); max over ranks. bt_time_device2 enqueues the K steps between one event pair and
waits by polling; its breakdown (enqueue / first event seen / last event seen / GPU span)
goes into the line. Steps with a compaction are pipelined (bt_parse_filter_device_async:
step i's compaction runs on a second stream beside step i+1's main kernel; two output
sets alternate, so no step rewrites a verdict buffer its predecessor's compaction still
reads); every step's outputs are complete when the timed region ends. The main kernel's
duration (roofline.kernel_ms) comes from a second pass of the same K steps with an event
pair recorded by every main kernel's own dispatch: those events cost the GPU ~9 us per
step (tools/calib/boundary.hip), so the timed region carries none.
The CPU baseline is the reference's own parser + PacketFilter (oracle/_ref, compiled
from the reference sources) on rank 0, on every host CPU the process may use
(affinity, bounded by the cgroup CPU quota when there is one), after all GPU timing.
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from beatrice_amd import abi, shard, synth  # noqa: E402

METRIC = "Mpps + achieved HBM GB/s, device-resident parse+filter, 64B and IMIX"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LINE = 128              # bytes per HBM access line (the FETCH_SIZE granule)

C3_FILTERS = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
              {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
              {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]

WORKLOADS = {
    "c2f": dict(cfg=synth.C2, fixed=True, parse=True, filters=C3_FILTERS,
                name="C2 frames + filter: 16M x 64B Eth/IPv4/UDP, fixed stride, parse + PacketFilter "
                     "(udp, 10.0.0.0/8, 1000-2000) + ordered compaction (metric's 64B parse+filter)"),
    "c2": dict(cfg=synth.C2, fixed=True, parse=True, filters=None,
               name="C2: 16M x 64B Eth/IPv4/UDP, fixed stride, parse-only (BASELINE configs[1])"),
    "c3": dict(cfg=synth.C3, fixed=False, parse=True, filters=C3_FILTERS,
               name="C3: 16M IMIX 64/512/1500 Eth/VLAN/IPv4/{TCP,UDP}, parse + PacketFilter "
                    "(udp, 10.0.0.0/8, 1000-2000) + ordered compaction (BASELINE configs[2])"),
    "c4": dict(cfg=synth.C4, fixed=False, parse=True, filters=C3_FILTERS,
               name="C4: 16M QinQ/IPv6/IHL+TCP options, 2-mod-4 offsets, parse + PacketFilter "
                    "(BASELINE configs[3])"),
}
# C3 with a GPU PAYLOAD slot first: applyPayloadFilter's regex_search over every
# IPv4 packet's <= 100-byte payload window (src/PacketFilter.cpp:288-321) before the 5-tuple set;
# random payloads never match, so every window is searched to its end (the worst case)
PAYLOAD_EXPR = "GET|POST"
WORKLOADS["c3_payload"] = dict(cfg=synth.C3, fixed=False, parse=True, payload=PAYLOAD_EXPR, traffic_key="c3_payload",
                               filters=[{"type": abi.PAYLOAD, "expr": PAYLOAD_EXPR, "priority": 9}] + C3_FILTERS,
                               name="C3 + PAYLOAD /GET|POST/ first: 16M IMIX, parse + PacketFilter (payload regex on "
                                    "every IPv4 packet's window, then udp, 10.0.0.0/8, 1000-2000) + ordered compaction")
# configs[0]'s protocol: examples/parser_example.cpp:18-43's CUSTOM_PROTO (header u32 @0,
# version u8 @4, length u16 @5, data BYTES[10] @7; all NETWORK byte order = 2), a user
# table for ProtocolParser::parsePacket(frame, ProtocolDefinition)
PARSER_EXAMPLE = [(0, 4, abi.FT_UINT32, 2), (4, 1, abi.FT_UINT8, 2), (5, 2, abi.FT_UINT16, 2), (7, 10, abi.FT_BYTES, 2)]
WORKLOADS["c1"] = dict(cfg=synth.C2, fixed=True, parse=False, filters=None, extract=PARSER_EXAMPLE,
                       name="C1's user protocol on the GPU: parser_example's CUSTOM_PROTO table (4 fields, span 17) "
                            "extracted from 16M x 64B frames, fixed stride: status, extractValue<T> values, field "
                            "bytes (ProtocolParser::parsePacket(frame, ProtocolDefinition), BASELINE configs[0])")
# the kernels and their launch shapes (bt_runtime.cpp's cache-policy bits are A/B flags)
KERNEL_SOURCES = ["beatrice_amd/csrc/bt_kernels.hip", "beatrice_amd/csrc/bt_device.h", "beatrice_amd/csrc/bt_slot_eval.h",
                  "beatrice_amd/csrc/bt_extract.hip"]


def kernel_source_sha() -> str:
    """Key of the committed PMC traffic figures: the sources that decide what the
    kernels load and store (tools/pmc_traffic.py writes the same key)."""
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


_IMPORTED = time.time()


def _process_start() -> float:
    """This process's start (wall clock), from the OS; bench.py's import time without psutil."""
    try:
        import psutil
        return psutil.Process().create_time()
    except Exception:
        return _IMPORTED


def host_cpus() -> dict:
    """CPUs this process may run on: the affinity set, bounded by the cgroup v2/v1 CPU
    quota when one is set (threads past the quota only time-share it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = int(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                p = int(fh.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return {"model": model, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "threads": threads}


def header_need(buf: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
    """Bytes from each frame's start that the layer walk + filters read: the kernel's
    header_end() (bt_kernels.hip) with its 38-B floor, at most the frame."""
    def b(k):
        return buf[off + k].astype(np.int64)
    et0, et1, et2 = b(12) << 8 | b(13), b(16) << 8 | b(17), b(20) << 8 | b(21)
    vl = lambda e: (e == 0x8100) | (e == 0x88A8)  # noqa: E731
    t0 = vl(et0)
    t1 = t0 & vl(et1)
    o3 = 14 + 4 * t0 + 4 * t1
    et = np.where(t1, et2, np.where(t0, et1, et0))
    ihl = np.where(t1, b(22), np.where(t0, b(18), b(14))) & 15
    v4end = o3 + 40 + np.where(ihl > 5, 4 * ihl - 20, 0)
    end = np.where(et == 0x0800, v4end, np.where(et == 0x86DD, o3 + 60, o3))
    return np.minimum(np.maximum(end, 38), ln)


def unique_lines(start: np.ndarray, nbytes: np.ndarray, prev_last: int = -1) -> tuple[int, int]:
    """Distinct 128-B lines the byte ranges [start, start + nbytes) touch, for ranges in
    ascending start order (a line shared by neighbouring frames counts once); prev_last
    carries the last line counted across calls. Returns (lines, new prev_last)."""
    live = nbytes > 0
    first = (start // LINE)[live]
    last = ((start + nbytes - 1) // LINE)[live]
    if len(first) == 0:
        return 0, prev_last
    before = np.maximum.accumulate(np.concatenate([[prev_last], last[:-1]]))
    new = last - np.maximum(first, before + 1) + 1
    return int(np.maximum(new, 0).sum()), int(max(prev_last, last.max()))


class Capture:
    """Per-rank capture streamed to the device, plus the statistics the roofline needs
    (computed per streamed range, so the capture is never whole on the host)."""

    def __init__(self, ctx, wl, n_total, seed, lo, hi, chunk=1 << 20):
        cfg = wl["cfg"]
        self.desc_full, _ = synth.layout(cfg, n_total, seed)
        off_full = synth.desc_off(self.desc_full)
        ln_full = synth.desc_len(self.desc_full)
        self.n = n = hi - lo
        # rebase to a 128-B-aligned start so every window keeps its line alignment
        base = (int(off_full[lo]) & ~(LINE - 1)) if n else 0
        nbytes = int(off_full[hi - 1] + ln_full[hi - 1]) - base if n else 16
        self.desc = synth.make_desc(off_full[lo:hi] - base, ln_full[lo:hi])
        self.stride = 64 if wl["fixed"] else 0
        filt = wl["filters"] is not None
        outs = wl.get("outputs") or ("records", "decide", "verdict", "pass_idx")   # A/B: --outputs
        self.run = abi.DeviceRun(ctx, None, None if wl["fixed"] else self.desc, n, stride=self.stride,
                                 records=wl["parse"] and "records" in outs, decide=filt and "decide" in outs,
                                 verdict=filt and "verdict" in outs, pass_idx=filt and "pass_idx" in outs,
                                 data_bytes=nbytes)
        self.win_bytes = 0        # sum of min(len, 128)
        self.need_lines = 0       # distinct 128-B lines of [off, off + header_need)
        need_last = -1
        self.payload_extra = 0    # PAYLOAD window bytes past 128 (only with --payload)
        i = lo - lo % synth.RNG_BLOCK
        while i < hi:
            j = min(hi, i + chunk)
            buf, b0, _ = synth.fill_range(cfg, seed, self.desc_full, i, j)
            s = max(i, lo)
            rel = off_full[s:j] - b0
            lens = ln_full[s:j]
            self.run.upload_data(buf[int(rel[0]):int(rel[-1] + lens[-1])], int(off_full[s]) - base)
            start = off_full[s:j] - base
            w = np.minimum(lens, 128)
            self.win_bytes += int(w.sum())
            k, need_last = unique_lines(start, header_need(buf, rel, lens), need_last)
            self.need_lines += k
            if wl.get("payload"):
                self.payload_extra += payload_extra_bytes(buf, rel, lens)
            i = j

    def cpu_sample(self, wl, seed, n_sample):
        """The first n_sample packets of the same capture, for the CPU baseline."""
        m = min(n_sample, len(self.desc_full))
        buf, b0, nb = synth.fill_range(wl["cfg"], seed, self.desc_full, 0, m)
        d = self.desc_full[:m]
        return buf[:nb + 16].copy(), synth.make_desc(synth.desc_off(d) - b0, synth.desc_len(d))


def payload_extra_bytes(buf, rel, lens) -> int:
    """Bytes a PAYLOAD slot reads beyond the 128-B header window: applyPayloadFilter's
    window is [14 + 4*IHL, +min(len - that, 100)) of IPv4 frames (src/PacketFilter.cpp:293-309)."""
    ok = lens >= 34
    ipv4 = ok & (buf[rel + 12] == 8) & (buf[rel + 13] == 0)
    po = 14 + (buf[rel + 14].astype(np.int64) & 15) * 4
    end = np.minimum(lens, po + 100)
    return int(np.where(ipv4 & (lens > po), np.maximum(0, end - 128), 0).sum())


def main_kernel_name(wl, flags: int = 0) -> str:
    """The main-kernel variant launch_main picks (bt_kernels.hip launch_t)."""
    no_pipe = os.environ.get("BT_NO_PIPE", "") not in ("", "0")
    layout = flags & (abi.OPT_RECORDS_AOS | abi.OPT_RECORDS_PLANES)
    nt_stores = not (flags & abi.OPT_CACHE_DEFAULT) or (flags & abi.OPT_NT_STORES)
    # a program with a GPU PAYLOAD slot runs the main kernel at its residency (launch_t's F == 2)
    gpu_payload = any(f["type"] == abi.PAYLOAD for f in (wl.get("filters") or [])) and \
        not (flags & abi.OPT_PAYLOAD_HOST)
    pipe = not (wl["fixed"] or no_pipe or layout or (flags & abi.OPT_NO_PREFETCH) or not nt_stores or gpu_payload)
    return "bt_parse_filter_pipe" if pipe else "bt_parse_filter_main"


def record_write_stats(run) -> tuple[int, int]:
    """(record bytes stored, 128-B lines they fill) from this run's tiled records: slabs
    0-1 at every slot (2 KiB per tile), slab k >= 2 packed to the front of its region."""
    rec = run.d_rec.download(np.zeros(run.d_rec.nbytes, np.uint8))
    nt = (run.n + 63) // 64
    ok = rec[: nt * 6 * 1024].reshape(nt, 6, 64, 16)[:, 1, :, 1].astype(np.int64)
    nd = 5 + ((ok & abi.L_VLAN0) != 0) + ((ok & abi.L_VLAN1) != 0) + \
        np.where(ok & abi.L_IPV4, 5, np.where(ok & abi.L_IPV6, 10, 0)) + \
        np.where(ok & abi.L_TCP, 5, np.where(ok & (abi.L_UDP | abi.L_ICMP), 2, 0))
    ns = (nd + 3) // 4
    live = (np.arange(nt * 64).reshape(nt, 64) < run.n)
    ns = np.where(live, ns, 0)
    stored = int(ns.sum()) * 16
    lines = nt * 2 * (1024 // LINE)
    for k in range(2, 6):
        cnt = (ns > k).sum(axis=1)
        lines += int(((cnt * 16 + LINE - 1) // LINE).sum())
    return stored, lines


def record_write_stats_planes(run) -> tuple[int, int]:
    """(record bytes stored, 128-B lines) for the plane-major layout: slab k of packet i at
    plane k, row i; a wave stores slab k for its live lanes when any of them needs it."""
    n = run.n
    rec = run.d_rec.download(np.zeros(run.d_rec.nbytes, np.uint8))
    ok = rec[n * 16: 2 * n * 16].reshape(n, 16)[:, 1].astype(np.int64)
    nd = 5 + ((ok & abi.L_VLAN0) != 0) + ((ok & abi.L_VLAN1) != 0) + \
        np.where(ok & abi.L_IPV4, 5, np.where(ok & abi.L_IPV6, 10, 0)) + \
        np.where(ok & abi.L_TCP, 5, np.where(ok & (abi.L_UDP | abi.L_ICMP), 2, 0))
    nt = (n + 63) // 64
    ns = np.zeros(nt * 64, np.int64)
    ns[:n] = (nd + 3) // 4
    ns = ns.reshape(nt, 64)
    live = np.minimum(64, n - np.arange(nt) * 64)
    planes = 2 + sum((ns > k).any(axis=1).astype(np.int64) for k in range(2, 6))
    stored = int((planes * live).sum()) * 16
    return stored, -(-stored // LINE)


def load_traffic(path, key, n):
    """Per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py), if the
    committed figure was measured on these kernel sources and this batch size."""
    if not os.path.exists(path):
        return None, "no profiles/traffic.json"
    try:
        with open(path) as fh:
            rec = json.load(fh).get(key)
    except (OSError, ValueError) as e:
        return None, f"unreadable: {e}"
    if not rec:
        return None, f"no PMC measurement for {key}"
    if rec.get("packets") != n:
        return None, f"measured at {rec.get('packets')} packets, not {n}"
    sha = kernel_source_sha()
    if rec.get("kernel_src_sha") != sha:
        return None, f"stale: measured on kernel sources {rec.get('kernel_src_sha')}, these are {sha}"
    return rec, os.path.relpath(path, ROOT)


def aggregate_roofline(ranks: list, world: int) -> dict:
    """The job's roofline over its N devices: the algorithmic bytes of every
    rank's main-kernel launch summed, over the slowest rank's kernel time, against N x the HBM
    peak ("frac"); and the same bytes over the slowest rank's whole step (compaction and
    launch gaps included, "frac_step"). At N = 1 it equals the line's own roofline."""
    algo = float(sum(r["algo"] for r in ranks))
    kms = max(r["main_ms"] for r in ranks)
    step = max(r["step_s"] for r in ranks)
    peak = HBM_PEAK_GBS * world
    ach = algo / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    ach_step = algo / step / 1e9 if step > 0 else 0.0
    return {"bound": "hbm", "devices": world, "unit": "GB/s", "peak": peak,
            "algorithmic_bytes": int(algo), "kernel_ms_max": round(kms, 4),
            "achieved": round(ach, 1), "frac": round(ach / peak, 4),
            "ms_per_step_max": round(step * 1e3, 4), "achieved_step": round(ach_step, 1),
            "frac_step": round(ach_step / peak, 4)}


def measure(name, wl, args, ctx, flags, dist, rank, world, strong):
    """GPU half of one workload: build, warm up, time K steps. Returns this rank's
    results (the CPU baseline and the cross-rank max are filled in by the caller)."""
    seed = synth.SEEDS[wl["cfg"]] + (0 if strong else rank)
    n_job = args.packets if strong else args.packets * world
    if strong:
        d_all, _ = synth.layout(wl["cfg"], args.packets, seed)
        lo, hi = shard.shard_bounds(synth.desc_len(d_all), world)[rank]
        n_total = args.packets
        del d_all
    else:
        lo, hi, n_total = 0, args.packets, args.packets
    cap = Capture(ctx, wl, n_total, seed, lo, hi)
    run, n = cap.run, cap.n
    filt = wl["filters"] is not None
    if filt:
        prog = ctx.compile(wl["filters"])
        if wl.get("payload") and abi.KINDS[prog[0].kind] != "PAYLOAD":
            sys.exit(f"--payload {wl['payload']!r} is not GPU-compilable (kind {abi.KINDS[prog[0].kind]})")
    # Steps with a compaction run pipelined (bt_parse_filter_device_async: each step's
    # compaction beside the next step's main kernel) over two alternating output sets.
    piped = filt and not args.no_pipeline
    mode = abi.TIME_PIPELINED if piped else 0
    outs = [run.outs, run.second_outputs()] if piped else [run.outs]
    timed_mode = mode | (abi.TIME_KERNEL_EVENTS if args.kernel_events_in_timed else 0)
    # One untimed step for the host-side bookkeeping below (pass count, stored record
    # bytes); the warm-up follows it, so the GPU goes from the warm-up straight into the
    # timed region instead of idling through seconds of host work (a first pass after
    # such an idle spell ran 3-5 % slower than a second one, profiles/r02/ab/warm_order.txt).
    run.run()
    n_pass = run.n_pass() if filt else 0
    if run.d_rec is None or not n:
        rec_bytes, rec_lines = 0, 0
    elif flags & abi.OPT_RECORDS_AOS:   # 96-B bt_rec per packet, contiguous
        rec_bytes = n * abi.BT_REC_BYTES
        rec_lines = -(-rec_bytes // LINE)
    elif flags & abi.OPT_RECORDS_PLANES:   # six 16-B planes, slab k stored when any lane of the tile needs it
        rec_bytes, rec_lines = record_write_stats_planes(run)
    else:
        rec_bytes, rec_lines = record_write_stats(run)
    # warm-up: one untimed pass of the K steps with the kernel events (creates the event
    # pairs the kernel pass uses), then the W warm-up steps in exactly the timed form, so
    # the timed pass repeats the launches the GPU ran last (with the kernel-event pass
    # last, a timed pass of 20 steps ran ~0.2 ms longer than 20 x its steady step)
    ctx.time_device2(run.batch, outs, args.steps, mode | abi.TIME_KERNEL_EVENTS)
    if args.warmup:
        ctx.time_device2(run.batch, outs, args.warmup, timed_mode)

    def barrier():
        if dist is not None:
            dist.barrier()

    # The K steps are bracketed by a barrier + device sync on both sides; each rank's clock runs
    # from its release at the opening barrier to its closing sync, and the line takes the max
    # over ranks. The closing barrier's own latency (gloo: ~0.1 ms at 2 ranks, ~0.4-0.6 ms at 8
    # on a busy host, against ~7 ms for 20 c2f steps) is reported in `timing`, not counted as
    # step time: ranks share no data, so it is not part of any rank's work.
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    tm = ctx.time_device2(run.batch, outs, args.steps, timed_mode)
    ta = time.perf_counter()
    ctx.synchronize()
    t1 = time.perf_counter()
    barrier()
    tb = time.perf_counter()
    step_s = (t1 - t0) / args.steps
    # The main kernel's duration: the same K steps again, each main kernel between an
    # event pair recorded by its own dispatch. Those events cost the GPU ~9 us per step
    # (tools/calib/boundary.hip), so they stay out of the timed region above. A PAYLOAD
    # program's main kernel fills every CU (bt_parse_filter_main at its residency), so in the
    # pipelined form its dispatch events also span the previous step's compaction blocks it
    # waits behind (1.35 ms between the events against 0.89 ms of kernel in the rocprofv3 trace
    # of the same run): its kernel pass runs the compaction after each kernel instead.
    kmode = 0 if wl.get("payload") else mode
    tk = tm if args.kernel_events_in_timed else ctx.time_device2(run.batch, outs if kmode else outs[:1], args.steps,
                                                                 kmode | abi.TIME_KERNEL_EVENTS)

    # algorithmic bytes of one main-kernel launch (SURVEY §8(d), R = the stored slabs):
    # min(len,128) header read + 8 B descriptor (0 for fixed stride) + R + 1 B decision
    # + 1/8 B verdict bit; the compaction kernels' pass_idx is not the main kernel's
    algo = cap.win_bytes + (0 if wl["fixed"] else 8 * n) + rec_bytes + (n * 1.125 if filt else 0)
    algo += cap.payload_extra
    # the 128-B-line floor of what the walk must touch: header lines + descriptors +
    # record lines + decisions + verdict words
    floor_read = cap.need_lines * LINE + (0 if wl["fixed"] else 8 * n)
    floor_write = rec_lines * LINE + ((n + (n + 63) // 64 * 8) if filt else 0)
    main_ms = tk.main_ms
    mine = {"step_s": step_s, "main_ms": main_ms, "n": n, "algo": algo, "pass": n_pass,
            "host_ms": 1e3 * (ta - t0), "tail_ms": 1e3 * (t1 - ta), "barrier_ms": 1e3 * (tb - t1)}
    ranks = [mine]
    if dist is not None:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    step_max = max(r["step_s"] for r in ranks)
    kms_max = max(r["main_ms"] for r in ranks)
    value = n_job / step_max / 1e6
    achieved = algo / (main_ms * 1e-3) / 1e9
    key = wl.get("traffic_key", name if not wl.get("payload") else None)
    traffic_rec, traffic_src = load_traffic(args.traffic_json, key, n) if key else (None, "PAYLOAD variant")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic_rec["traffic"] if traffic_rec else None,
            "traffic_source": traffic_src,
            "traffic_bytes_per_packet": round(traffic_rec["traffic"] / n, 2) if traffic_rec else None,
            "traffic_floor": floor_read + floor_write,
            "traffic_floor_bytes_per_packet": round((floor_read + floor_write) / max(n, 1), 2),
            "traffic_floor_read_per_packet": round(floor_read / max(n, 1), 2),
            "traffic_floor_write_per_packet": round(floor_write / max(n, 1), 2),
            "kernel": main_kernel_name(wl, flags), "kernel_ms": round(main_ms, 4),
            "kernel_ms_min": round(tk.main_min_ms, 4), "kernel_ms_max": round(tk.main_max_ms, 4),
            "algorithmic_bytes_per_packet": round(algo / max(n, 1), 2),
            "record_bytes_per_packet": round(rec_bytes / max(n, 1), 2),
            "kernel_mpps": round(n / (main_ms * 1e-3) / 1e6, 1),
            "gpu_span_ms_per_step": round(tm.span_ms / args.steps, 4)}
    if traffic_rec:
        roof["traffic_read_per_packet"] = traffic_rec.get("read_per_packet")
        roof["traffic_write_per_packet"] = traffic_rec.get("write_per_packet")
    timing = tm.as_dict()
    timing.update({"wall_ms": round(1e3 * step_s * args.steps, 4), "host_call_ms": round(mine["host_ms"], 4),
                   "tail_sync_ms": round(mine["tail_ms"], 4),
                   "closing_barrier_ms_max_over_ranks": round(max(r["barrier_ms"] for r in ranks), 4),
                   "wall_over_span": round(step_s * args.steps * 1e3 / tm.span_ms, 4) if tm.span_ms > 0 else None,
                   "pipelined": piped, "output_sets": len(outs),
                   "kernel_events_in_timed_region": bool(args.kernel_events_in_timed)})
    timing["kernel_pass"] = {k: v for k, v in tk.as_dict().items()
                             if k in ("span_ms", "main_ms", "main_min_ms", "main_max_ms", "lead_ms", "gap_ms")}
    timing["kernel_pass"]["ms_per_step"] = round(tk.span_ms / args.steps, 4)
    out = {"workload": wl["name"], "value": round(value, 2), "unit": "Mpps", "ms_per_step": round(step_max * 1e3, 4),
           "scaling": "strong" if strong else "weak", "packets_per_gpu": n, "packets_total": n_job,
           "pass_fraction": round(n_pass / n, 4) if filt and n else None, "roofline": roof,
           "roofline_aggregate": aggregate_roofline(ranks, world), "timing": timing}
    if world > 1:
        out["per_rank"] = [{"rank": i, "packets": r["n"], "ms_per_step": round(r["step_s"] * 1e3, 4),
                            "kernel_ms": round(r["main_ms"], 4),
                            "frac": round(r["algo"] / (r["main_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                           for i, r in enumerate(ranks)]
        out["kernel_ms_max_over_ranks"] = round(kms_max, 4)
    sample = cap.cpu_sample(wl, seed, args.cpu_sample) if rank == 0 and not args.no_cpu else None
    run.free()
    return out, sample


def measure_extract(name, wl, args, ctx, rank):
    """The user-protocol extractor (bt_extract_tile) over a device-resident capture: one
    step = one bt_extract_device pass over the batch (N=1 entry)."""
    seed = synth.SEEDS[wl["cfg"]] + rank
    cap = Capture(ctx, wl, args.packets, seed, 0, args.packets)
    n, fields = cap.n, wl["extract"]
    ex = abi.DeviceExtract(ctx, None, None, n, fields, batch=cap.run.batch)
    ex.run()
    ok = int((ex.fetch()[0] == 0).sum())   # host bookkeeping before the warm-up (see measure)
    for _ in range(args.warmup):
        ex.run()
    ex.time(args.steps)   # untimed: creates the per-launch event pairs
    ctx.synchronize()
    t0 = time.perf_counter()
    tm = ex.time(args.steps, abi.TIME_KERNEL_EVENTS if args.kernel_events_in_timed else 0)
    ctx.synchronize()
    t1 = time.perf_counter()
    step_s = (t1 - t0) / args.steps
    tk = tm if args.kernel_events_in_timed else ex.time(args.steps)   # the kernel pass (see measure)
    span, nf = ex.span, len(fields)
    # algorithmic bytes: the [0, span) prefix read + status byte + one u64 per field + the
    # span-byte image; the floor reads the 128-B lines of those prefixes
    lens = synth.desc_len(cap.desc)
    starts = synth.desc_off(cap.desc) if not wl["fixed"] else np.arange(n, dtype=np.int64) * cap.stride
    rd = int(np.minimum(lens, span).sum())
    lines, _ = unique_lines(starts, np.minimum(lens, span))
    wr = n * (1 + 8 * nf + span)
    algo = rd + wr
    floor = lines * LINE + sum(-(-b // LINE) * LINE for b in (n, 8 * nf * n, span * n))
    achieved = algo / (tk.main_ms * 1e-3) / 1e9
    traffic_rec, traffic_src = load_traffic(args.traffic_json, name, n)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic_rec["traffic"] if traffic_rec else None, "traffic_source": traffic_src,
            "traffic_bytes_per_packet": round(traffic_rec["traffic"] / n, 2) if traffic_rec else None,
            "traffic_floor": floor, "traffic_floor_bytes_per_packet": round(floor / n, 2),
            "kernel": "bt_extract_tile", "kernel_ms": round(tk.main_ms, 4),
            "kernel_ms_min": round(tk.main_min_ms, 4), "kernel_ms_max": round(tk.main_max_ms, 4),
            "algorithmic_bytes_per_packet": round(algo / n, 2), "kernel_mpps": round(n / (tk.main_ms * 1e-3) / 1e6, 1),
            "gpu_span_ms_per_step": round(tm.span_ms / args.steps, 4)}
    if traffic_rec:
        roof["traffic_read_per_packet"] = traffic_rec.get("read_per_packet")
        roof["traffic_write_per_packet"] = traffic_rec.get("write_per_packet")
    timing = tm.as_dict()
    timing.update({"wall_ms": round(1e3 * step_s * args.steps, 4),
                   "wall_over_span": round(step_s * args.steps * 1e3 / tm.span_ms, 4) if tm.span_ms > 0 else None,
                   "kernel_events_in_timed_region": bool(args.kernel_events_in_timed)})
    timing["kernel_pass"] = {k: v for k, v in tk.as_dict().items()
                             if k in ("span_ms", "main_ms", "main_min_ms", "main_max_ms", "lead_ms", "gap_ms")}
    timing["kernel_pass"]["ms_per_step"] = round(tk.span_ms / args.steps, 4)
    out = {"workload": wl["name"], "value": round(n / step_s / 1e6, 2), "unit": "Mpps",
           "ms_per_step": round(step_s * 1e3, 4), "scaling": "weak", "packets_per_gpu": n, "packets_total": n,
           "parsed_fraction": round(ok / n, 4), "table": [list(f) for f in fields], "span": span,
           "roofline": roof,
           "roofline_aggregate": aggregate_roofline([{"algo": algo, "main_ms": tk.main_ms, "step_s": step_s}], 1),
           "timing": timing,
           "published": "parser_example: 25 us to parse its one 17-byte packet (README.md:1110; BASELINE.md §1)"}
    sample = cap.cpu_sample(wl, seed, args.cpu_sample) if rank == 0 and not args.no_cpu else None
    ex.free()
    cap.run.free()
    return out, sample


def cpu_baseline_extract(sample, wl, seconds, cpus):
    """The reference's ProtocolParser::parsePacket(frame, ProtocolDefinition) (oracle/_ref)
    on the host CPUs over a bounded sample; the C restatement where _ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol  # checker/baseline only

    data, sub = sample
    threads = cpus["threads"]
    if ol.ref_available():
        done, el = ol.ref_bench_extract(data, sub, len(sub), wl["extract"], threads=threads, seconds=seconds)
        kind = "reference"
    else:
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < seconds:
            ol.oracle_extract(data, sub, len(sub), wl["extract"])
            done += len(sub)
        el, kind, threads = time.perf_counter() - t0, "port", 1
    return {"value": round(done / el / 1e6, 4), "unit": "Mpps", "cores": threads, "kind": kind,
            "cpu_model": cpus["model"], "affinity_cpus": cpus["affinity_cpus"],
            "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "sample": f"first {len(sub)} packets of the same capture, repeated for {el:.1f}s; "
                      f"ProtocolParser::parsePacket(frame, CUSTOM_PROTO) with metrics off; {threads} "
                      f"std::threads, per-thread parser instances, disjoint shards"}


def cpu_baseline(sample, wl, seconds, cpus):
    """The reference's own parser + PacketFilter (oracle/_ref) on the host CPUs, on a
    bounded sample of the same capture; the C oracle port where _ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol  # checker/baseline only

    data, sub = sample
    threads = cpus["threads"]
    filters = wl["filters"] or []
    if ol.ref_available():
        done, el = ol.ref_bench(data, sub, len(sub), filters, parse=wl["parse"], threads=threads, seconds=seconds)
        kind = "reference"
    else:
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < seconds:
            ol.oracle_run(data, sub, len(sub), filters if filters else None, parse=wl["parse"], threads=threads)
            done += len(sub)
        el = time.perf_counter() - t0
        kind = "port"
    what = ("ProtocolParser::parsePacket per walked layer" if wl["parse"] else "") + \
           (" + PacketFilter::applyFilters" if filters else "")
    return {"value": round(done / el / 1e6, 4), "unit": "Mpps", "cores": threads, "kind": kind,
            "cpu_model": cpus["model"], "affinity_cpus": cpus["affinity_cpus"],
            "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "sample": f"first {len(sub)} packets of the same capture, repeated for {el:.1f}s; "
                      f"{what.strip()}; {threads} std::threads (one per usable host CPU), per-thread "
                      f"instances, disjoint shards"}


def measure_group_ingest(n_dev: int, packets: int, reps: int = 5, shared: bool = False) -> dict:
    """The product's multi-GPU ingest, in one process: a bt_group over the job's n_dev devices
    reads one batch of frames in registered host memory (an AF_XDP UMEM / a capture ring's
    shape: frames back to back) in place, every device its range over its own PCIe link
    (bt_group_host_register + bt_group_parse_filter_mapped), C3's 5-tuple filter, decisions and
    verdict words written back into registered host memory. PCIe-inclusive, strong scaling (one
    batch split n_dev ways), never the line's `value`. Rank 0 runs it after every rank's
    device-resident timing, the other ranks waiting at a barrier.

    The capture is placed the way INTEGRATION.md §4 tells a deployment to allocate its ring or
    UMEM: each member's byte range of the batch on its device's NUMA node (the nodes the
    members' gather threads are pinned to), reported in `placement` / `data_nodes`.

    shared (a rank rehearsal on a 1-GPU box, BT_BENCH_DEVICE): the n_dev members share device 0
    (BT_OPT_GROUP_SHARED_DEVICE, one PCIe link), so the N > 1 code path runs end to end; its
    rates are one link's, not a scaling point."""
    import time as _time
    from beatrice_amd import numa
    visible = abi.device_count()
    if visible < (1 if shared else n_dev):
        return {"skipped": f"rank 0 sees {visible} device(s), the job has {n_dev}"}
    devs = [0] * n_dev if shared else list(range(n_dev))
    out = {"workload": "zero-copy ingest, one process, bt_group over the job's devices: frames in registered "
                       "host memory read in place over each device's PCIe link (bt_group_parse_filter_mapped), "
                       "C3's 5-tuple filter, decisions + verdict words back into host memory",
           "n_devices": n_dev, "packets": packets, "scaling": "strong", "pcie_inclusive": True, "unit": "Mpps",
           "members_share_one_device": shared}
    for name, cfg in (("c2", synth.C2), ("c3", synth.C3)):
        raw, desc = synth.capture(cfg, packets)
        grp = abi.Group(devs, flags=abi.OPT_GROUP_SHARED_DEVICE if shared else 0)
        held = []
        try:
            grp.compile(C3_FILTERS)
            # each member's range of frames on its device's node (the mapped call's split)
            bounds = abi.group_split(synth.desc_len(desc), n_dev, grp.cost(True, False, True), plan=True)
            nodes = [grp.placement(k)["numa_node"] for k in range(n_dev)]
            spans = numa.member_byte_ranges(synth.desc_off(desc), synth.desc_len(desc), bounds)
            data = numa.place_ranges(raw, [(lo, hi, nd) for (lo, hi), nd in zip(spans, nodes)])
            if data is raw:   # no NUMA information: pages of its own all the same
                data = abi.host_copy(raw)
            del raw
            data_nodes = [numa.page_nodes(data[lo:hi]) if hi > lo else [] for lo, hi in spans]
            tiles = (packets + 63) // 64
            # registration is in whole pages: every registered buffer on pages of its own
            desc = abi.host_copy(desc)
            dec = abi.host_array(tiles * 64)
            ver = abi.host_array(tiles, np.uint64)
            for a in (data, desc, dec, ver):
                grp.register(a)
                held.append(a)
            batch = abi.Batch(data.ctypes.data, desc.ctypes.data, 0, packets, data.nbytes, abi.DESC_PACKED, 0)
            outs = abi.Outputs(None, packets, ver.ctypes.data, dec.ctypes.data, None, None)
            grp.run_mapped(batch, outs)   # warm: first touches of the mapping on every device
            times = []
            for _ in range(reps):
                t0 = _time.perf_counter()
                grp.run_mapped(batch, outs)
                times.append(_time.perf_counter() - t0)
            bits = np.unpackbits(ver.view(np.uint8), bitorder="little")[:packets].astype(bool)
            consistent = bool(np.array_equal(bits, (dec[:packets] >> 6) == 0))
            med = sorted(times)[len(times) // 2]
            out[name] = {"value": round(packets / med / 1e6, 1), "best": round(packets / min(times) / 1e6, 1),
                         "ms_per_call": round(med * 1e3, 3), "pass_fraction": round(float(bits.mean()), 4),
                         "verdicts_match_decisions": consistent,
                         "placement": [grp.placement(k) for k in range(n_dev)],
                         "data_nodes": data_nodes, "member_nodes": nodes}
            if name == "c3":   # the same frames through the members' host gathers (bt_group_parse_filter)
                hout = abi.host_outputs(packets, records=False)   # reused, as a capture loop does
                grp.run_host(data, desc, records=False, outs=hout)
                ht = []
                for _ in range(reps):
                    t0 = _time.perf_counter()
                    h = grp.run_host(data, desc, records=False, outs=hout)
                    ht.append(_time.perf_counter() - t0)
                hm = sorted(ht)[len(ht) // 2]
                out["c3_host_gather"] = {
                    "value": round(packets / hm / 1e6, 1), "best": round(packets / min(ht) / 1e6, 1),
                    "ms_per_call": round(hm * 1e3, 3), "decisions_match_zero_copy": bool(np.array_equal(h["decide"], dec[:packets])),
                    # after the gathers: staging_node = where the members' pinned staging landed
                    # (-1 in the zero-copy entries above, which stage nothing)
                    "placement": [grp.placement(k) for k in range(n_dev)],
                    "workload": "C3 frames in ordinary host memory (each member's range on its device's NUMA node): "
                                "each member gathers its range's 48-B prefixes on its NUMA-pinned host threads into "
                                "pinned staging, H2D, kernels, decisions + verdicts + pass list back into output "
                                "arrays allocated once"}
        finally:
            for a in held:
                grp.unregister(a)
            grp.close()
        if n_dev == 1 and not shared:   # the ring stage of these frames (one device)
            try:
                out.setdefault("ring", {})[name] = measure_ring_stage(data, desc, nodes[0])
            except Exception as e:   # reported, never fatal to the line
                out.setdefault("ring", {})[name] = {"error": str(e)[:300]}
        del data, desc
    return out


def measure_ring_stage(data: np.ndarray, desc: np.ndarray, node: int, reps: int = 5) -> dict:
    """The TPACKET_V3 ring stage on device 0 (bt_ring_stage_tpv3, the call GpuTpacketStage's
    poll makes): the frames packed into a ring image laid out as the Linux kernel fills a
    PACKET_RX_RING (synth.tpv3_ring), placed on the device's NUMA node and registered once; each
    pass takes every block, the host walking (or lean-gathering) batch k+1 of 128 blocks while
    the GPU filters batch k over PCIe, decisions and verdict words back in registered host
    memory. PCIe-inclusive, never the line's `value`. Modes: in place (the stage's default), lean
    gather on every other batch, lean gather on every batch, every batch split (its last 40 of 128
    blocks read in place, the rest gathered), and adaptive (a batch gathered while the device is
    still busy, in place once it caught up; batches of 128 or 32 blocks)."""
    import time as _time
    from beatrice_amd import numa
    ring, rdesc, used = synth.tpv3_ring(data, desc)
    n = len(rdesc)
    placed = numa.place_ranges(ring, [(0, ring.nbytes, node)])   # pages of its own, as a ring mapping is
    ring = placed if placed is not ring else abi.host_copy(ring)
    del placed
    ctx = abi.Context(0, flags=abi.OPT_SPIN_SYNC)
    held = []
    out = {"workload": "TPACKET_V3 ring image (kernel layout) of the same frames, registered once: per pass every "
                       "block through bt_ring_stage_tpv3 (batches of 128 blocks, host walk of the next batch "
                       "overlapping the kernels of this one), C3's 5-tuple filter, decisions + verdict words into "
                       "registered host memory",
           "frames": n, "ring_blocks": used, "block_bytes": synth.TPV3_BLOCK, "ring_bytes": int(ring.nbytes),
           "unit": "Mpps", "pcie_inclusive": True}
    try:
        ctx.compile(C3_FILTERS)
        rd = abi.host_array(n + 64, np.uint64)
        dec = abi.host_array(n + 64)
        ver = abi.host_array((n + 127) // 64, np.uint64)
        slots = abi.host_array((n + 64) * abi.PREFIX_SLOT)
        for a in (ring, rd, dec, ver, slots):
            ctx.register(a)
            held.append(a)
        ref_dec = None
        for mode, kw in (("in_place", {}), ("lean_every_other", dict(gather=True, in_place_every=2)),
                         ("lean_all", dict(gather=True)), ("lean_split_40", dict(gather=True, in_place_blocks=40)),
                         ("adaptive", dict(gather="adaptive")), ("adaptive_32", dict(gather="adaptive", batch_blocks=32))):
            abi.ring_stage_tpv3(ctx, ring, synth.TPV3_BLOCK, used, rd, dec, ver, slots, **kw)   # warm
            times = []
            for _ in range(reps):
                t0 = _time.perf_counter()
                got, npass = abi.ring_stage_tpv3(ctx, ring, synth.TPV3_BLOCK, used, rd, dec, ver, slots, **kw)
                times.append(_time.perf_counter() - t0)
            bits = np.unpackbits(ver.view(np.uint8), bitorder="little")[:got].astype(bool)
            med = sorted(times)[len(times) // 2]
            ent = {"value": round(got / med / 1e6, 1), "best": round(got / min(times) / 1e6, 1),
                   "ms_per_pass": round(med * 1e3, 3), "frames": got, "pass_fraction": round(npass / max(got, 1), 4),
                   "verdicts_match_decisions": bool(np.array_equal(bits, (dec[:got] >> 6) == 0))}
            if ref_dec is None:
                ref_dec = dec[:got].copy()
            else:
                ent["decisions_match_in_place"] = bool(np.array_equal(dec[:got], ref_dec))
            out[mode] = ent
    finally:
        for a in held:
            ctx.unregister(a)
        ctx.close()
    return out


def group_ingest_isolated(n_dev: int, packets: int, timeout: int = 900, shared: bool = False) -> dict:
    """measure_group_ingest in a child process (N > 1): the group then drives every device of
    the node from one process, which only this entry does and which no 1-GPU box can rehearse;
    a failure there (an error, or a fault that would end the process) is reported in the
    line instead of ending rank 0 before it prints. A child process, never an exec."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--group-ingest-child", str(n_dev),
                            "--group-ingest-packets", str(packets)] + (["--group-ingest-shared"] if shared else []),
                           env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"group ingest child did not finish in {timeout} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"group ingest child exited {r.returncode}: {(r.stderr or r.stdout)[-300:]}"}
    out = json.loads(lines[-1])
    out["process"] = "child of rank 0"
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`--gpus n` with no launcher: run this script as n rank processes (RANK = LOCAL_RANK
    = r, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1) and return the worst exit code. This process
    never touches a GPU. A rank that fails ends the others (they would wait at a barrier)."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    worst = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                worst = worst or rc
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
                break
        time.sleep(0.1)
    return worst


def check_devices(ctx, dist, world) -> dict:
    """Every rank's (host, PCI bus id); distinct unless BT_BENCH_DEVICE pins all ranks to
    one device. Returns what the line reports about it."""
    import socket
    ordinal, bus = ctx.device_id()
    me = (socket.gethostname(), bus)
    ids = [me]
    if dist is not None:
        ids = [None] * world
        dist.all_gather_object(ids, me)
    distinct = len(set(ids))
    pinned = "BT_BENCH_DEVICE" in os.environ
    if distinct != world and not pinned:
        sys.exit(f"bench.py: {world} ranks drive only {distinct} distinct device(s) {sorted(set(ids))}; "
                 f"set BT_BENCH_DEVICE for a one-device rehearsal")
    return {"devices_distinct": distinct, "pci_bus_ids": [b for _, b in ids],
            "rehearsal_one_device": bool(pinned and world > 1)}


@contextlib.contextmanager
def stdout_to_stderr():
    """Point fd 1 at stderr for the duration (native libraries' prints included), so that
    rank 0's stdout holds nothing but the line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2f", choices=sorted(WORKLOADS), help="the headline workload")
    ap.add_argument("--configs", default="auto",
                    help="comma list of extra workloads for the `configs` object (suffix _strong: strong "
                         "scaling), 'none', or 'auto' (N=1: c2,c3,c4,c1,c3_payload; N>1: c3,c3_strong)")
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 18)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--grid-waves", type=int, default=0, help="persistent grid size in wavefronts (0 = auto)")
    ap.add_argument("--no-prefetch", action="store_true", help="A/B: disable the next-tile load prefetch")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="A/B: each step's compaction on the main stream (bt_parse_filter_device)")
    ap.add_argument("--kernel-events-in-timed", action="store_true",
                    help="A/B: time the main kernels inside the timed region (round 2's first form)")
    ap.add_argument("--flags", type=int, default=None, help="raw bt_opts.flags (A/B experiments)")
    ap.add_argument("--payload", default=None,
                    help="put a PAYLOAD regex FIRST in the headline's filter program (every IPv4 packet runs "
                         "the GPU DFA: worst case); reported in config, not the default workload")
    ap.add_argument("--strong", action="store_true", help="the headline as strong scaling (C5's other half)")
    ap.add_argument("--outputs", default=None,
                    help="A/B only: comma list of the headline's outputs (records,decide,verdict,pass_idx)")
    ap.add_argument("--group-ingest-packets", type=int, default=1 << 24,
                    help="packets of the in-process group zero-copy ingest entry (0 = skip it)")
    ap.add_argument("--group-ingest-child", type=int, default=0, help=argparse.SUPPRESS)   # internal
    ap.add_argument("--group-ingest-shared", action="store_true", help=argparse.SUPPRESS)  # internal
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    args = ap.parse_args()

    if args.group_ingest_child:   # group_ingest_isolated's child: only the group entry, one JSON line
        try:
            res = measure_group_ingest(args.group_ingest_child, args.group_ingest_packets,
                                       shared=args.group_ingest_shared)
        except Exception as e:   # reported, never fatal to the parent's line
            res = {"error": str(e)[:300]}
        print(json.dumps(res), flush=True)
        return

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} (the launcher's rank count)")
    if os.environ.get("BT_BENCH_SPAWN_CHECK"):   # tests: the launcher's env, no GPU touched
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}),
              flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        with stdout_to_stderr():   # gloo's "[Gloo] Rank r is connected to ..." lines: stdout is the JSON line's
            dist.init_process_group("gloo")
    flags = args.flags if args.flags is not None else (abi.OPT_NO_PREFETCH if args.no_prefetch else 0)
    flags |= abi.OPT_SPIN_SYNC   # host waits spin: no wake-up latency inside the timed region
    # BT_BENCH_DEVICE: put every rank on one device (multi-rank rehearsal on a 1-GPU box)
    device = int(os.environ.get("BT_BENCH_DEVICE", local))
    ctx = abi.Context(device, grid_waves=args.grid_waves, flags=flags)
    devices = check_devices(ctx, dist, world)

    head = dict(WORKLOADS[args.config])
    if args.outputs is not None:
        head.update(outputs=tuple(args.outputs.split(",")), name=head["name"] + f" [outputs: {args.outputs}]")
    if args.payload is not None:
        if not head["filters"]:
            sys.exit("--payload needs a filtering workload")
        head.update(filters=[{"type": abi.PAYLOAD, "expr": args.payload, "priority": 9}] + head["filters"],
                    name=head["name"] + f" + PAYLOAD /{args.payload}/ first", payload=args.payload)
    if args.configs == "auto":
        extra = ["c2", "c3", "c4", "c1", "c3_payload"] if world == 1 else ["c3", "c3_strong"]
    elif args.configs == "none":
        extra = []
    else:
        extra = [c for c in args.configs.split(",") if c]
    extra = [c for c in extra if c != args.config or (args.strong != c.endswith("_strong"))]

    results, samples = {}, {}
    jobs = [("__head__", args.config, head, args.strong)] + \
           [(c, c.replace("_strong", ""), dict(WORKLOADS[c.replace("_strong", "")]), c.endswith("_strong"))
            for c in extra]
    for key, name, wl, strong in jobs:
        if wl.get("extract"):
            res, sample = measure_extract(name, wl, args, ctx, rank)
        else:
            res, sample = measure(name, wl, args, ctx, flags, dist, rank, world, strong)
        results[key] = res
        samples[key] = (sample, wl)
    # the reference CPU parser + filter on rank 0, after every rank's GPU timing; at N > 1 the
    # other ranks wait at the barrier below meanwhile (north_star: "timed on the node's own host
    # cores ... in the same run", at every GPU count)
    cpus = host_cpus()
    if rank == 0 and not args.no_cpu:
        attach_cpu_baselines(results, samples, cpus, world,
                             lambda smp, wl, sec, c: (cpu_baseline_extract if wl.get("extract") else cpu_baseline)(
                                 smp, wl, sec, c),
                             args.cpu_seconds)

    # the product's multi-GPU ingest (one process, every device of the job), after every rank's
    # device-resident timing: the other ranks wait at a barrier meanwhile
    if dist is not None:
        dist.barrier()
    if rank == 0 and args.group_ingest_packets > 0 and args.configs != "none":
        try:
            results["zero_copy_group"] = (measure_group_ingest(world, args.group_ingest_packets) if world == 1
                                          else group_ingest_isolated(world, args.group_ingest_packets,
                                                                     shared=devices["rehearsal_one_device"]))
        except Exception as e:   # reported, never fatal to the line
            results["zero_copy_group"] = {"error": str(e)[:300]}
    if dist is not None:
        dist.barrier()

    if rank == 0:
        line = build_line(results, args, world, devices)
        # rank 0's process age at the line (imports, every entry, the CPU baselines and the
        # group entry): what to hold against the driver's per-run limit
        line["job_wall_s"] = round(time.time() - _process_start(), 1)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def attach_cpu_baselines(results: dict, samples: dict, cpus: dict, world: int, timer, seconds: float) -> None:
    """Rank 0's CPU baselines, one per workload entry: timer(sample, wl, seconds, cpus) runs the
    reference (oracle/_ref) on the host CPUs. A strong-scaling entry whose weak twin was timed
    on the same capture (rank 0's weak sample is the strong batch's first packets: same seed)
    quotes that figure; the headline also reports one thread per affinity CPU when a cgroup
    quota caps the threads. Every baseline states the job's GPU count beside it."""
    for key, (sample, wl) in samples.items():
        entry = results[key]
        if sample is None:
            entry["cpu_baseline"] = None
            continue
        twin = key.replace("_strong", "")
        if entry.get("scaling") == "strong" and key != "__head__" and \
                (results.get(twin) or {}).get("cpu_baseline"):
            entry["cpu_baseline"] = dict(results[twin]["cpu_baseline"], same_as=f"configs.{twin}")
            continue
        entry["cpu_baseline"] = timer(sample, wl, seconds, cpus)
        if key == "__head__" and cpus["affinity_cpus"] > cpus["threads"]:
            # the same on one thread per affinity CPU, past the cgroup quota: shows
            # whether the quota, not the thread count, bounds the reference
            wide = timer(sample, wl, max(1.0, seconds / 2), dict(cpus, threads=cpus["affinity_cpus"]))
            entry["cpu_baseline"]["all_affinity_threads"] = {
                "threads": wide["cores"], "value": wide["value"], "unit": wide["unit"]}
    for entry in results.values():
        if isinstance(entry.get("cpu_baseline"), dict):
            entry["cpu_baseline"]["n_gpus_in_job"] = world
            entry["cpu_baseline"]["timed"] = ("rank 0, after every rank's GPU timing" +
                                              (", the other ranks waiting at a barrier" if world > 1 else ""))


def build_line(results: dict, args, world: int, devices: dict) -> dict:
    """Rank 0's JSON line from the per-workload entries (results["__head__"] = the headline)."""
    results = dict(results)
    h = results.pop("__head__")
    line = {
        "metric": METRIC,
        "value": h["value"],
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["ms_per_step"],
        "higher_is_better": True,
        "scaling": h["scaling"],
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (beatrice_amd/csrc/bt_synth.cpp, seeded mt19937_64, streamed to HBM)",
        "config": {"workload": h["workload"], "packets_per_gpu": h["packets_per_gpu"],
                   "packets_total": h["packets_total"], "parallelism": f"batch split x{world}",
                   "pass_fraction": h.get("pass_fraction"), **devices},
        "roofline": h["roofline"],
        "roofline_aggregate": h.get("roofline_aggregate"),
        "cpu_baseline": h.get("cpu_baseline"),
        "timing": h["timing"],
    }
    if "per_rank" in h:
        line["per_rank"] = h["per_rank"]
    line["configs"] = results
    return line


if __name__ == "__main__":
    main()
