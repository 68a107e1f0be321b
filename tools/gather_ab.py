#!/usr/bin/env python3
"""In-process A/B of the host batch path (bt_parse_filter, filter-only: the host gather ->
pinned staging -> H2D -> kernels -> D2H pipeline) between two bt_opts flag sets.

Host-side rates drift with the box's other load by tens of percent within a minute, so the
two contexts run in ONE process on ONE capture (placed on the device's NUMA node), their calls
alternating A, B, A, B, ...; each reports the median and best of its calls.

  python tools/gather_ab.py --config c3 --flags-b 0x20000 --calls 12
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import abi, synth  # noqa: E402
from beatrice_amd.numa import page_nodes, place_on  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4"])
ap.add_argument("--packets", type=int, default=1 << 24)
ap.add_argument("--flags-a", type=lambda x: int(x, 0), default=0)
ap.add_argument("--flags-b", type=lambda x: int(x, 0), default=abi.OPT_NO_LEAN_HOST)
ap.add_argument("--calls", type=int, default=12, help="calls per side")
ap.add_argument("--records", action="store_true", help="records + verdicts instead of verdicts")
a = ap.parse_args()

FILTERS = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
           {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
           {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4}[a.config]
ctxs = {"a": abi.Context(0, flags=a.flags_a), "b": abi.Context(0, flags=a.flags_b)}
for c in ctxs.values():
    c.compile(FILTERS)
data, desc = synth.capture(cfg, a.packets)
data = place_on(data, ctxs["a"].placement()["numa_node"])
outs = {k: abi.host_outputs(a.packets, records=a.records) for k in ctxs}
res = {}
for k, c in ctxs.items():   # warm: pinned staging, first touches
    res[k] = c.run_host(data, desc, records=a.records, outs=outs[k])
same = bool((res["a"]["decide"] == res["b"]["decide"]).all() and res["a"]["n_pass"] == res["b"]["n_pass"])
times = {k: [] for k in ctxs}
for _ in range(a.calls):
    for k, c in ctxs.items():
        t0 = time.perf_counter()
        c.run_host(data, desc, records=a.records, outs=outs[k])
        times[k].append(time.perf_counter() - t0)
row = {"config": a.config, "packets": a.packets, "mode": "records+verdicts" if a.records else "verdicts",
       "calls": a.calls, "decisions_equal": same, "data_nodes": page_nodes(data), "placement": ctxs["a"].placement()}
for k in ctxs:
    t = sorted(times[k])
    row[k] = {"flags": hex(a.flags_a if k == "a" else a.flags_b), "mpps_median": round(a.packets / t[len(t) // 2] / 1e6, 1),
              "mpps_best": round(a.packets / t[0] / 1e6, 1)}
row["a_over_b_median"] = round(row["a"]["mpps_median"] / row["b"]["mpps_median"], 3)
print(json.dumps(row), flush=True)
