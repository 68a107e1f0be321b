#!/usr/bin/env python3
"""Which allocation makes the first C2 run slow? MODE: default | recfirst | prealloc"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402
mode = os.environ.get("MODE", "default")
n = 1 << 24
data, desc = synth.capture(synth.C2, n)
ctx = abi.Context(0, grid_waves=8192)
scratch = ctx.alloc(4 << 30) if mode == "prealloc" else None
if scratch is not None:
    scratch.free()
out = []
for r in range(3):
    if mode == "recfirst":
        rec = ctx.alloc(n * 96)
        d = ctx.alloc(data.nbytes + 512)
    else:
        d = ctx.alloc(data.nbytes + 512)
        rec = ctx.alloc(n * 96)
    d.upload(data)
    batch = abi.Batch(d.ptr, None, 64, n, data.nbytes)
    outs = abi.Outputs(rec.ptr, n, None, None, None, None)
    for _ in range(5):
        ctx.run_device(batch, outs)
    ctx.time_device(batch, outs, 20)
    _, k = ctx.time_device(batch, outs, 50)
    out.append(round(k, 4))
    if r == 1:
        d.free(); rec.free()
print(json.dumps({"mode": mode, "flags": os.environ.get("BT_MALLOC_FLAGS", "0"), "kern_ms": out}))
