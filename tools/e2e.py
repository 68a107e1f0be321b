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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4"])
ap.add_argument("--packets", type=int, default=1 << 24)
ap.add_argument("--chunk", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4}[a.config]
data, desc = synth.capture(cfg, a.packets)
ctx = abi.Context(0, host_chunk_packets=a.chunk)
ctx.compile([{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
             {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
             {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}])
for mode in ("verdicts", "records+verdicts"):
    rec = mode != "verdicts"
    ctx.run_host(data[: 1 << 20], desc[: 1 << 14], records=rec)     # warm pinned buffers
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = ctx.run_host(data, desc, records=rec)
        best = min(best, time.perf_counter() - t0)
    lens = synth.desc_len(desc)
    h2d = float((((lens.clip(max=112) + 15) // 16) * 16).sum() + 8 * a.packets)
    d2h = a.packets * (1 + 1 / 8 + (96 if rec else 0))
    print(json.dumps({"config": a.config, "mode": mode, "packets": a.packets, "seconds": round(best, 4),
                      "mpps": round(a.packets / best / 1e6, 1), "h2d_GBps": round(h2d / best / 1e9, 2),
                      "d2h_GBps": round(d2h / best / 1e9, 2), "n_pass": out["n_pass"]}), flush=True)
