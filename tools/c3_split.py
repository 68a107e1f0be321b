#!/usr/bin/env python3
"""C3 main-kernel time split: parse-only, filter-only, parse+filter (same capture)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402

cfg = {"c3": synth.C3, "c4": synth.C4}[sys.argv[1] if len(sys.argv) > 1 else "c3"]
n = 1 << 24
data, desc = synth.capture(cfg, n)
F = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3}, {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
     {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
ctx = abi.Context(0)
res = {}
for name, rec, filt in (("parse+filter", True, True), ("parse", True, False), ("filter", False, True)):
    ctx.compile(F if filt else [])
    run = abi.DeviceRun(ctx, data, desc, n, records=rec, decide=filt, verdict=filt, pass_idx=filt)
    for _ in range(3):
        run.run()
    ms, k = ctx.time_device(run.batch, run.outs, 20)
    res[name] = round(k, 4)
    run.free()
print(json.dumps(res))
