#!/usr/bin/env python3
"""SQ / GRBM counter passes of the main kernel (tools/gpu_r05.sh sq_pass) side by side.

    python3 tools/sq_summary.py OUTDIR CFG [CFG...]

Reads OUTDIR/sq_<cfg>_<pass>/**/*counter_collection.csv, keeps the main kernel's
dispatches (bt_parse_filter_* / bt_extract_tile), averages the counters over the last
half of them (the warm launches) and prints per-config totals, per-packet instruction
counts and the wave-cycle split (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES,
all in quad-cycles). The effective clock is GRBM_GUI_ACTIVE / 8 XCDs / kernel time.
"""
import csv
import glob
import os
import sys

PACKETS = 1 << 24


def load(out, cfg):
    per = {}
    for f in glob.glob(os.path.join(out, f"sq_{cfg}_*", "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.relpath(f, out).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "parse_filter_" not in k and "extract_tile" not in k:
                continue
            d = per.setdefault(tag, {}).setdefault(int(r["Dispatch_Id"]), {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    avg = {}
    for tag, disp in per.items():
        ids = sorted(disp)[len(disp) // 2:]
        for c in disp[ids[0]]:
            avg[c] = sum(disp[i].get(c, 0.0) for i in ids) / len(ids)
    return avg


def main():
    out, cfgs = sys.argv[1], sys.argv[2:]
    rows = {c: load(out, c) for c in cfgs}
    names = sorted({k for d in rows.values() for k in d})
    print(f"{'counter':24s}" + "".join(f"{c:>16s}" for c in cfgs) + ("   delta(first-last)" if len(cfgs) > 1 else ""))
    for n in names:
        vals = [rows[c].get(n) for c in cfgs]
        line = f"{n:24s}" + "".join(f"{v:16.4g}" if v is not None else f"{'-':>16s}" for v in vals)
        if len(cfgs) > 1 and None not in (vals[0], vals[-1]):
            line += f"   {vals[0] - vals[-1]:+.4g}"
        print(line)
    for c in cfgs:
        d = rows[c]
        wc = d.get("SQ_WAVE_CYCLES")
        if not wc:
            continue
        split = {k: d.get(k, 0.0) / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        per_wave_tile = {k: d[k] / (PACKETS / 64) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                             "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM",
                                                             "SQ_INSTS_BRANCH") if k in d}
        print(f"{c}: wave-cycle split " + " ".join(f"{k[3:]} {v:.3f}" for k, v in split.items()))
        print(f"{c}: instructions per 64-packet tile " + " ".join(f"{k[9:]} {v:.1f}" for k, v in per_wave_tile.items()))
        if "SQ_WAVES" in d and d["SQ_WAVES"]:
            print(f"{c}: waves {d['SQ_WAVES']:.0f}, quad-cycles per wave {wc / d['SQ_WAVES']:.0f}")


if __name__ == "__main__":
    main()
