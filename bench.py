#!/usr/bin/env python3
"""Benchmark of the device-resident parse+filter hot path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4] [--packets P]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step = one bt_parse_filter_device() pass over one synthetic 16M-packet batch that
is already resident in HBM. Default workload (N=1): BASELINE.json configs[1] — C2,
16,777,216 fixed 64 B Eth/IPv4/UDP frames, parse-only (one packed record per packet:
64 B on the device for Eth/IPv4/UDP, unpacked to the 96-B bt_rec by the host).
`--config c3` runs configs[2] (IMIX parse + 5-tuple PacketFilter + ordered
compaction). Multi-GPU is weak scaling by default: every rank owns its own 16M-packet
batch on its own device (packet batches shard with no collective; the only cross-rank
traffic is the timing barrier and the max-reduction of the step time, over gloo).
`--strong` (C5's other half) splits one --packets batch into tile-aligned,
byte-balanced contiguous shards, one per rank.

Prints ONE JSON line on rank 0 with value = packets of all ranks / max step time,
the roofline of the main kernel (HIP events around every main-kernel launch inside the
timed region) and, at N=1, the same run's CPU baseline: the reference's own parser +
PacketFilter (oracle/_ref, compiled from the reference sources) on the host cores.
"""
from __future__ import annotations

import argparse
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

C3_FILTERS = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
              {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
              {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]

WORKLOADS = {
    "c2": dict(cfg=synth.C2, fixed=True, parse=True, filters=None,
               name="C2: 16M x 64B Eth/IPv4/UDP, fixed stride, parse-only (BASELINE configs[1])"),
    "c3": dict(cfg=synth.C3, fixed=False, parse=True, filters=C3_FILTERS,
               name="C3: 16M IMIX 64/512/1500 Eth/VLAN/IPv4/{TCP,UDP}, parse + PacketFilter "
                    "(udp, 10.0.0.0/8, 1000-2000) + ordered compaction (BASELINE configs[2])"),
    "c4": dict(cfg=synth.C4, fixed=False, parse=True, filters=C3_FILTERS,
               name="C4: 16M QinQ/IPv6/IHL+TCP options, 2-mod-4 offsets, parse + PacketFilter "
                    "(BASELINE configs[3])"),
}


def payload_extra_bytes(data: np.ndarray, desc: np.ndarray) -> float:
    """Bytes a PAYLOAD slot reads beyond the 128-B header window: applyPayloadFilter's
    window is [14 + 4*IHL, +min(len - that, 100)) of IPv4 frames (src/PacketFilter.cpp:293-309)."""
    off = synth.desc_off(desc).astype(np.int64)
    ln = synth.desc_len(desc).astype(np.int64)
    ok = ln >= 34
    idx = np.minimum(off + 14, len(data) - 1)
    ipv4 = ok & (data[np.minimum(off + 12, len(data) - 1)] == 8) & (data[np.minimum(off + 13, len(data) - 1)] == 0)
    po = 14 + (data[idx].astype(np.int64) & 15) * 4
    end = np.minimum(ln, po + 100)
    extra = np.where(ipv4 & (ln > po), np.maximum(0, end - 128), 0)
    return float(extra.sum())


def main_kernel_name(wl, flags: int = 0) -> str:
    """The main-kernel variant launch_main picks (bt_kernels.hip launch_t): descriptor
    mode with packed tiled records (or none) and non-temporal record stores runs the
    counted-wait pipeline unless BT_NO_PIPE is set or prefetch is off; everything else
    runs bt_parse_filter_main."""
    no_pipe = os.environ.get("BT_NO_PIPE", "") not in ("", "0")
    layout = flags & (abi.OPT_RECORDS_AOS | abi.OPT_RECORDS_PLANES)
    nt_stores = not (flags & abi.OPT_CACHE_DEFAULT) or (flags & abi.OPT_NT_STORES)
    pipe = not (wl["fixed"] or no_pipe or layout or (flags & abi.OPT_NO_PREFETCH) or not nt_stores)
    return "bt_parse_filter_pipe" if pipe else "bt_parse_filter_main"


def algorithmic_bytes(desc: np.ndarray, fixed: bool, rec_bytes: float, filt: bool) -> float:
    """Bytes the main kernel must move per launch (SURVEY.md §8(d) formula, R = the
    packed record's stored slabs, counted from this run's records):
    min(len,128) header read + 8 B descriptor (0 for fixed stride) + R
    + 1 B decision + 1/8 B verdict bit (the ordered pass-index list is written by the
    compaction kernels and is not counted here)."""
    n = len(desc)
    lens = synth.desc_len(desc)
    b = float(np.minimum(lens, 128).sum())
    if not fixed:
        b += 8.0 * n
    b += rec_bytes
    if filt:
        b += n * (1.0 + 1.0 / 8.0)
    return b


def cpu_baseline(data, desc, wl, n_sample, seconds):
    """The reference's own parser + PacketFilter (oracle/_ref) on the host cores, on a
    bounded sample of the same capture; falls back to the C oracle port."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol  # checker/baseline only

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(16, cores))
    sub = desc[:n_sample]
    filters = wl["filters"] or []
    if ol.ref_available():
        done, el = ol.ref_bench(data, sub, len(sub), filters, parse=wl["parse"], threads=threads,
                                seconds=seconds)
        kind = "reference"
    else:
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < seconds:
            ol.oracle_run(data, sub, len(sub), filters if filters else None, parse=wl["parse"],
                          threads=threads)
            done += len(sub)
        el = time.perf_counter() - t0
        kind = "port"
    what = ("ProtocolParser::parsePacket per walked layer" if wl["parse"] else "") + \
           (" + PacketFilter::applyFilters" if filters else "")
    return {"value": round(done / el / 1e6, 4), "unit": "Mpps", "cores": threads, "kind": kind,
            "sample": f"first {len(sub)} packets of the same capture, repeated for {el:.1f}s; "
                      f"{what.strip()}; {threads} std::threads, per-thread instances, disjoint shards"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-sample", type=int, default=1 << 18)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--grid-waves", type=int, default=0, help="persistent grid size in wavefronts (0 = auto)")
    ap.add_argument("--no-prefetch", action="store_true", help="A/B: disable the next-tile load prefetch")
    ap.add_argument("--flags", type=int, default=None, help="raw bt_opts.flags (A/B experiments)")
    ap.add_argument("--payload", default=None,
                    help="c3/c4: put a PAYLOAD regex FIRST in the filter program (every IPv4 packet runs the "
                         "GPU DFA: worst case); reported in config, not the default workload")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (C5): --packets is the whole job, split across the ranks in "
                         "tile-aligned, byte-balanced contiguous shards (beatrice_amd/shard.py)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 PMC passes (tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")
    wl = WORKLOADS[args.config]
    n_job = args.packets * (1 if args.strong else world)
    if args.strong:
        # every rank generates the same capture and keeps its own shard, rebased
        data, desc = synth.capture(wl["cfg"], args.packets, seed=synth.SEEDS[wl["cfg"]])
        lo, hi = shard.shard_bounds(synth.desc_len(desc), world)[rank]
        if wl["fixed"]:
            data, desc = np.ascontiguousarray(data[lo * 64:hi * 64]), desc[lo:hi]
        else:
            data, desc = shard.local_batch(data, desc, lo, hi)
    else:
        data, desc = synth.capture(wl["cfg"], args.packets, seed=synth.SEEDS[wl["cfg"]] + rank)
    n = len(desc)
    flags = args.flags if args.flags is not None else (abi.OPT_NO_PREFETCH if args.no_prefetch else 0)
    flags |= abi.OPT_SPIN_SYNC   # the timed region's end is not delayed by a sleeping host thread
    # BT_BENCH_DEVICE: put every rank on one device (multi-rank rehearsal on a 1-GPU box)
    device = int(os.environ.get("BT_BENCH_DEVICE", local))
    ctx = abi.Context(device, grid_waves=args.grid_waves, flags=flags)
    if args.payload is not None:
        if not wl["filters"]:
            sys.exit("--payload needs a filtering workload (c3 / c4)")
        wl = dict(wl, filters=[{"type": abi.PAYLOAD, "expr": args.payload, "priority": 9}] + wl["filters"],
                  name=wl["name"] + f" + PAYLOAD /{args.payload}/ first")
    if wl["filters"]:
        prog = ctx.compile(wl["filters"])
        if args.payload is not None and abi.KINDS[prog[0].kind] != "PAYLOAD":
            sys.exit(f"--payload {args.payload!r} is not GPU-compilable (kind {abi.KINDS[prog[0].kind]})")
    filt = wl["filters"] is not None
    run = abi.DeviceRun(ctx, data, None if wl["fixed"] else desc, n, stride=64 if wl["fixed"] else 0,
                        records=wl["parse"], decide=filt, verdict=filt, pass_idx=filt)
    for _ in range(args.warmup):
        run.run()
    ctx.time_device(run.batch, run.outs, args.steps)   # untimed: creates the per-launch event pairs
    n_pass = run.n_pass() if filt else 0
    rec_bytes = 16.0 * run.record_slabs() if wl["parse"] else 0.0   # packed records: slabs stored
    # Two more untimed steps right before the timed region: an idle GPU (host-side work
    # between warm-up and t0) was measured to start the first timed kernel up to ~27 ms
    # late in 3 of 8 processes, with the device-side span unchanged.
    for _ in range(2):
        run.run()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    ms_iter, main_ms = ctx.time_device(run.batch, run.outs, args.steps)
    ta = time.perf_counter()
    ctx.synchronize()
    barrier()
    t1 = time.perf_counter()
    if os.environ.get("BT_DEBUG_TIMING"):
        print(f"[bench] time_device {1e3 * (ta - t0):.3f} ms, sync+barrier {1e3 * (t1 - ta):.3f} ms", file=sys.stderr)
    step_s = (t1 - t0) / args.steps
    if dist is not None:
        import torch
        t = torch.tensor([step_s, main_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_s, main_ms = float(t[0]), float(t[1])
    value = n_job / step_s / 1e6

    algo = algorithmic_bytes(desc, wl["fixed"], rec_bytes, filt)
    if args.payload is not None:
        algo += payload_extra_bytes(data, desc)
    achieved = algo / (main_ms * 1e-3) / 1e9
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):   # rocprofv3 PMC passes of this kernel (tools/pmc_traffic.py)
        try:
            with open(args.traffic_json) as fh:
                rec = json.load(fh).get(args.config)
            if rec and rec.get("packets") == n:
                traffic = rec["traffic"]
                traffic_src = os.path.relpath(args.traffic_json, ROOT)
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(data, desc, wl, args.cpu_sample, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (beatrice_amd/csrc/bt_synth.cpp, seeded mt19937_64)",
            "config": {"workload": wl["name"], "packets_per_gpu": n, "packets_total": n_job,
                       "parallelism": f"batch split x{world}",
                       "pass_fraction": round(n_pass / n, 4) if filt else None},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": main_kernel_name(wl, flags), "kernel_ms": round(main_ms, 4),
                         "algorithmic_bytes_per_packet": round(algo / n, 2),
                         "record_bytes_per_packet": round(rec_bytes / n, 2),
                         "kernel_mpps": round(n / (main_ms * 1e-3) / 1e6, 1),
                         "gpu_span_ms_per_step": round(ms_iter, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    run.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
