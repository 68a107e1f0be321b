#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (and its configs): value, step, kernel, frac."""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(path, "no JSON line")
        continue
    d = json.loads(lines[-1])

    def one(name, e):
        r = e.get("roofline") or {}
        c = e.get("cpu_baseline") or {}
        print(f"{path} {name}: {e['value']} Mpps step {e['ms_per_step']} ms kernel {r.get('kernel_ms')} "
              f"frac {r.get('frac')} traffic {r.get('traffic_bytes_per_packet')} cpu {c.get('value')}")

    print(f"{path}: n_gpus {d.get('n_gpus')} {d['config'].get('devices_distinct', '')}")
    one("head", d)
    for k, e in (d.get("configs") or {}).items():
        if "value" in e:
            one(k, e)
        else:   # the group ingest entry: one value per capture, or why it was skipped
            print(f"{path} {k}: " + ", ".join(f"{c} {v['value']} Mpps" for c, v in e.items()
                                               if isinstance(v, dict) and "value" in v)
                  + (e.get("skipped") or e.get("error") or ""))
