"""Where the GPU PAYLOAD filter's time goes: one C3 capture on the device, the main kernel timed
(event pair from its own dispatch, bt_time_device2 with BT_TIME_KERNEL_EVENTS) under programs
that differ only in their PAYLOAD slot, alternating variants round by round in one process:

  base        C3's 5-tuple set, no PAYLOAD slot (the uniform-predicate path, F = 1)
  last        + PAYLOAD /GET|POST/ last: the per-kind path, the regex only for packets that pass
  first       PAYLOAD /GET|POST/ first (every IPv4 packet runs it; random payloads never match:
              the whole <= 100-byte window is walked) — the configuration the verdict quotes;
              the bit-parallel (Shift-And) form the compiler picks for it
  first_dfa   the same program with the slot compiled as a byte DFA (BT_OPT_PAYLOAD_DFA context)
  ua, ua_dfa  PAYLOAD /User-Agent: .*(bot|curl)/ first: 33 positions (the 64-bit state)
  dot         PAYLOAD /./ first: staged, then decided on the first byte
  caret       PAYLOAD /^/ first: the bit-parallel compiler folds it to "always" (no window read)
  caret_x     PAYLOAD /^x/ first: every window loaded and staged, the search over after one turn
  *_cache     the same under a BT_OPT_CACHE_DEFAULT context; *_nopf under BT_OPT_NO_PREFETCH;
              *_wide under BT_OPT_WIDE_ALWAYS
each with records (parse + filter) and without (filter only).

Usage: python tools/payload_ab.py [--packets N] [--steps K] [--rounds R] [--variants a,b]
Prints one JSON line per variant with the median main-kernel time over the rounds.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from beatrice_amd import abi, synth  # noqa: E402

C3 = bench.C3_FILTERS


def prog(kind, expr=None):
    if kind == "base":
        return C3
    pay = {"type": abi.PAYLOAD, "expr": expr, "priority": 9 if kind != "last" else 0}
    return C3 + [pay] if kind == "last" else [pay] + C3


VARIANTS = {"base": prog("base"), "last": prog("last", "GET|POST"), "first": prog("first", "GET|POST"),
            "first_dfa": prog("first", "GET|POST"), "ua": prog("first", "User-Agent: .*(bot|curl)"),
            "ua_dfa": prog("first", "User-Agent: .*(bot|curl)"), "dot": prog("first", "."),
            "caret": prog("first", "^"), "caret_x": prog("first", "^x"), "caret_x_dfa": prog("first", "^x"),
            "first_cache": prog("first", "GET|POST"), "caret_cache": prog("first", "^"),
            "base_cache": prog("base"), "first_nopf": prog("first", "GET|POST"), "base_nopf": prog("base"),
            "caret_x_nopf": prog("first", "^x"), "last_nopf": prog("last", "GET|POST"),
            "ua_nopf": prog("first", "User-Agent: .*(bot|curl)"), "first_wide": prog("first", "GET|POST"),
            "last_wide": prog("last", "GET|POST"), "caret_x_wide": prog("first", "^x")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--records", default="1,0")
    a = ap.parse_args()
    ctx = abi.Context(0)
    ctx_dfa = abi.Context(0, flags=abi.OPT_PAYLOAD_DFA)
    ctx_cache = abi.Context(0, flags=abi.OPT_CACHE_DEFAULT)   # *_cache: default cache policy (no NT loads/stores)
    ctx_nopf = abi.Context(0, flags=abi.OPT_NO_PREFETCH)      # *_nopf: the main kernel without the next-tile prefetch
    ctx_wide = abi.Context(0, flags=abi.OPT_WIDE_ALWAYS)      # *_wide: round A reads chunks 4..7 too
    wl = dict(bench.WORKLOADS["c3"], payload="GET|POST")
    cap = bench.Capture(ctx, wl, a.packets, synth.SEEDS[synth.C3], 0, a.packets)
    run = cap.run
    res = {}
    names = a.variants.split(",")
    for rnd in range(a.rounds):
        for v in names:
            c = ctx_dfa if v.endswith("_dfa") else ctx_cache if v.endswith("_cache") else \
                ctx_nopf if v.endswith("_nopf") else ctx_wide if v.endswith("_wide") else ctx
            p = c.compile(VARIANTS[v])
            for rec in (int(x) for x in a.records.split(",")):
                o = abi.Outputs(run.outs.records if rec else None, run.n, run.outs.verdict, run.outs.decide,
                                run.outs.pass_idx, run.outs.n_pass)
                c.time_device2(run.batch, [o], 2, abi.TIME_KERNEL_EVENTS)   # warm
                t = c.time_device2(run.batch, [o], a.steps, abi.TIME_KERNEL_EVENTS)
                if rnd == 0:   # every form decides the same as the first variant with a PAYLOAD slot
                    dec = np.empty(run.n, np.uint8)
                    abi.lib().bt_memcpy_d2h(c.h, dec.ctypes.data, run.outs.decide, run.n)
                    res[(v, rec, "dec")] = dec
                res.setdefault((v, rec), []).append(t.main_ms)
                if rnd == 0:
                    res[(v, rec, "kinds")] = [abi.KINDS[s.kind] for s in p]
            print(json.dumps({"round": rnd, "variant": v, "done": True}), file=sys.stderr, flush=True)
    for v in names:
        for rec in (int(x) for x in a.records.split(",")):
            ms = sorted(res[(v, rec)])
            print(json.dumps({"variant": v, "records": bool(rec), "packets": run.n, "kernel_ms_median": round(ms[len(ms) // 2], 4),
                              "kernel_ms_all": [round(x, 4) for x in ms], "kinds": res[(v, rec, "kinds")],
                              "decisions_equal_to_dfa_form": (bool(np.array_equal(res[(v, rec, "dec")],
                                                                                  res[(v + "_dfa", rec, "dec")]))
                                                              if (v + "_dfa", rec, "dec") in res else None),
                              "n_pass": int(np.count_nonzero((res[(v, rec, "dec")] >> 6) == 0)),
                              "mpps": round(run.n / (ms[len(ms) // 2] * 1e-3) / 1e6, 1),
                              "payload_extra_bytes_per_packet": round(cap.payload_extra / run.n, 2),
                              "header_window_bytes_per_packet": round(cap.win_bytes / run.n, 2)}), flush=True)
    run.free()
    ctx_dfa.close()
    ctx_cache.close()
    ctx.close()


if __name__ == "__main__":
    main()
