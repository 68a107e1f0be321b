#!/usr/bin/env python3
"""Plane-stride skew sweep: n_cap = n + skew records (plane k at rec + k*n_cap*16)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402
n = 1 << 24
data, desc = synth.capture(synth.C2, n)
ctx = abi.Context(0, grid_waves=int(os.environ.get("GW", "8192")), flags=int(os.environ.get("FLAGS", "0")))
d = ctx.alloc(data.nbytes + 512)
d.upload(data)
batch = abi.Batch(d.ptr, None, 64, n, data.nbytes)
res = {}
for rep in range(6):
    for skew in (0,):
        ncap = n + skew
        rec = ctx.alloc(ncap * 96)
        outs = abi.Outputs(rec.ptr, ncap, None, None, None, None)
        for _ in range(5):
            ctx.run_device(batch, outs)
        _, k = ctx.time_device(batch, outs, 30)
        res.setdefault(skew, []).append(round(k, 4))
        rec.free()
print(json.dumps({"gw": os.environ.get("GW", "8192"), "flags": os.environ.get("FLAGS", "0"), "kern_ms_by_skew": res}))
