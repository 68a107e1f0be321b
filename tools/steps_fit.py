"""A/B tool: how a timed pass's GPU span grows with its step count K.

For one workload (bench.py's c2 / c2f at 16M packets), alternate timed passes of K steps (the
bench's own form: bt_time_device2 without per-kernel events, pipelined when filtering) over
several K, and fit span = a + b * K. `a` is a per-pass one-off (what a 20-step region pays on
top of 20 steady steps), `b` the steady step. Variants (--variant):
  sync     host sync between passes (the bench's form)
  idle     the GPU left idle for 2 ms before the timed pass (host sleep after the sync)
  prime    a 1-step untimed pass right before each timed pass (after the sync)

  python tools/steps_fit.py --config c2f --ks 5,10,20,40,80 --rounds 3 > out.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beatrice_amd import abi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2f")
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--ks", default="5,10,20,40,80")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="sync,idle,prime")
    args = ap.parse_args()
    ks = [int(x) for x in args.ks.split(",")]
    wl = dict(bench.WORKLOADS[args.config])
    ctx = abi.Context(0, flags=abi.OPT_SPIN_SYNC)
    cap = bench.Capture(ctx, wl, args.packets, synth.SEEDS[wl["cfg"]], 0, args.packets)
    run = cap.run
    filt = wl["filters"] is not None
    if filt:
        ctx.compile(wl["filters"])
    mode = abi.TIME_PIPELINED if filt else 0
    outs = [run.outs, run.second_outputs()] if filt else [run.outs]
    run.run()
    ctx.time_device2(run.batch, outs, max(ks), mode | abi.TIME_KERNEL_EVENTS)
    rows = {}
    for r in range(args.rounds):
        for v in args.variants.split(","):
            for k in ks:
                ctx.time_device2(run.batch, outs, 5, mode)      # warm-up in the timed form
                ctx.synchronize()
                if v == "idle":
                    time.sleep(0.002)
                if v == "prime":
                    ctx.time_device2(run.batch, outs, 1, mode)
                    ctx.synchronize()
                tm = ctx.time_device2(run.batch, outs, k, mode)
                rows.setdefault((v, k), []).append((tm.span_ms, tm.wall_ms))
                print(json.dumps({"round": r, "variant": v, "k": k, "span_ms": round(tm.span_ms, 4),
                                  "wall_ms": round(tm.wall_ms, 4)}), flush=True)
    tk = ctx.time_device2(run.batch, outs, 20, mode | abi.TIME_KERNEL_EVENTS)
    for v in args.variants.split(","):
        x = np.array(ks, float)
        y = np.array([np.median([s for s, _ in rows[(v, k)]]) for k in ks])
        w = np.array([np.median([s for _, s in rows[(v, k)]]) for k in ks])
        b, a = np.polyfit(x, y, 1)
        bw, aw = np.polyfit(x, w, 1)
        print(json.dumps({"fit": v, "config": args.config, "one_off_ms": round(a, 4), "step_ms": round(b, 5),
                          "wall_one_off_ms": round(aw, 4), "wall_step_ms": round(bw, 5),
                          "per_step_at": {str(k): round(yy / k, 5) for k, yy in zip(ks, y)},
                          "kernel_ms": round(tk.main_ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
