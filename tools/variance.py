#!/usr/bin/env python3
"""Run-to-run variance probe: C2 kernel time over fresh allocations in one process,
plus buffer addresses (HBM placement) and rocm-smi clocks between rounds."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n = 1 << 24
data, desc = synth.capture(synth.C2, n)
ctx = abi.Context(0, grid_waves=8192)
res = []
keep = []
for r in range(rounds):
    run = abi.DeviceRun(ctx, data, None, n, stride=64, records=True, decide=False, verdict=False, pass_idx=False)
    warm = int(os.environ.get("WARM", "3"))
    for _ in range(warm):
        run.run()
    ctx.time_device(run.batch, run.outs, 20)
    ms, kern = ctx.time_device(run.batch, run.outs, 20)
    ms2, kern2 = ctx.time_device(run.batch, run.outs, 200)
    res.append({"round": r, "warm": warm, "kern_ms": round(kern, 4), "kern_ms_next200": round(kern2, 4),
                "data": hex(run.d_data.ptr), "rec": hex(run.d_rec.ptr)})
    print(json.dumps(res[-1]), flush=True)
    if r % 2 == 0:
        keep.append(run)      # hold every other allocation so placements differ
    else:
        run.free()
clk = subprocess.run(["rocm-smi", "--showclocks", "--showtemp"], capture_output=True, text=True).stdout
print("\n".join(l for l in clk.splitlines() if "sclk" in l or "mclk" in l or "Temperature" in l))
