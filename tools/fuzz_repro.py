#!/usr/bin/env python3
"""Replays tests/test_gpu_fuzz.py::test_randomized_parity_sweep's draws up to one round and runs
that round's capture and program again through every entry form (the mapped one with 1, 2 and 3
members), REPEAT times each, against the oracle: which forms differ, and whether the difference
repeats.

  python tools/fuzz_repro.py --seed 0xB1A5 --round 3160 --repeat 5
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
from random_programs import random_programs  # noqa: E402
from test_gpu_fuzz import FORMS, _mapped  # noqa: E402

from beatrice_amd import abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xB1A5)
ap.add_argument("--round", type=int, required=True, help="0-based round (the `round N` of the failure message)")
ap.add_argument("--repeat", type=int, default=5)
a = ap.parse_args()

rng = np.random.default_rng(a.seed)
for r in range(a.round + 1):
    cfg = [synth.C2, synth.C3, synth.C4, synth.FUZZ][int(rng.integers(0, 4))]
    n = int(rng.choice([1, 63, 64, 65, 127, 4097, int(rng.integers(1, 70000))]))
    cap_seed = int(rng.integers(1, 1 << 30))
    prog_seed = int(rng.integers(1, 1 << 30))
    metric = rng.random() < 0.2
    form = FORMS[r % len(FORMS)] if r < len(FORMS) else FORMS[int(rng.integers(0, len(FORMS)))]
    records = bool(rng.random() < 0.4)
    m = None
    if form in ("mapped", "grouphost"):
        m = int(rng.integers(1, 4)) if form == "mapped" else int(rng.integers(2, 4))
prog = random_programs(prog_seed, 1)[0]
if metric:
    prog = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
            {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
            {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
data, desc = synth.capture(cfg, n, seed=cap_seed)
if data.nbytes < 64:
    data = np.concatenate([data, np.zeros(64, np.uint8)])
print(json.dumps({"round": a.round, "form": form, "members": m, "cfg": cfg, "n": n, "cap_seed": hex(cap_seed),
                  "records": records, "program": prog}), flush=True)
rec, dec, npass = ol.oracle_run(data, desc, n, prog, parse=records)
ctx = abi.Context(0)
ctx.compile(prog)
groups = {k: abi.Group([0] * k, flags=abi.OPT_GROUP_SHARED_DEVICE if k > 1 else 0) for k in (1, 2, 3)}
for g in groups.values():
    g.compile(prog)
try:
    for rep in range(a.repeat):
        runs = {"host": lambda: ctx.run_host(data, desc, records=records)}

        def device():
            r = abi.DeviceRun(ctx, data, desc, n, records=records)
            r.run()
            out = r.fetch()
            r.free()
            return out
        runs["device"] = device
        for k, g in groups.items():
            runs[f"mapped{k}"] = (lambda g=g: _mapped(g, data, desc, n, records))
        runs["grouphost2"] = lambda: groups[2].run_host(data, desc, records=records)
        res = {}
        for name, fn in runs.items():
            out = fn()
            bad = np.nonzero(out["decide"][:n] != dec)[0]
            res[name] = {"differ": int(len(bad)), "first": [int(x) for x in bad[:8]],
                         "got": [int(out["decide"][x]) for x in bad[:4]], "want": [int(dec[x]) for x in bad[:4]]}
        print(json.dumps({"repeat": rep, "results": res}), flush=True)
finally:
    for g in groups.values():
        g.close()
    ctx.close()
