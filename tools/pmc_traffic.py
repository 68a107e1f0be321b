#!/usr/bin/env python3
"""Per-launch HBM traffic of the main kernel (bt_parse_filter_main / _pipe; bt_extract_tile for c1) from
rocprofv3 PMC passes.

    python tools/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE --config c2 \
        [--out profiles/traffic.json]

Each DIR holds one `rocprofv3 --pmc <counter> --output-format csv` pass (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950: TCC slots). Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads exactly half the bytes
of a wide (16 B/lane) coalesced streaming read, so the corrected read traffic is 2x
FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane streaming stores. Both raw and
corrected numbers are written; `traffic` (what bench.py reports) is the corrected sum.
Each figure is keyed with bench.kernel_source_sha() of the sources it was measured on;
bench.py reports `traffic: null` (with the reason) when the key does not match.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (kernel_source_sha: the key bench.py checks the figure against)

KERNEL = "bt_parse_filter_"   # bt_parse_filter_main (fixed stride) or bt_parse_filter_pipe (descriptors)
KERNEL_OF = {"c1": "bt_extract_tile"}   # bench.py's user-protocol entry


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if KERNEL not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {d}")
    xs = sorted(vals.values())
    return xs[len(xs) // 2], len(xs)   # median over dispatches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "profiles", "traffic.json"))
    a = ap.parse_args()
    global KERNEL
    KERNEL = KERNEL_OF.get(a.config, KERNEL)
    fetch_kib, nf = per_dispatch(a.fetch, "FETCH_SIZE")
    write_kib, nw = per_dispatch(a.write, "WRITE_SIZE")
    fetch_b = fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    rec = {
        "unit": "bytes per launch",
        "packets": a.packets,
        "fetch_size_raw": fetch_b,
        "write_size_raw": write_b,
        "read_corrected": 2.0 * fetch_b,
        "write": write_b,
        "traffic": 2.0 * fetch_b + write_b,
        "traffic_per_packet": (2.0 * fetch_b + write_b) / a.packets,
        "read_per_packet": 2.0 * fetch_b / a.packets,
        "write_per_packet": write_b / a.packets,
        "kernel_src_sha": bench.kernel_source_sha(),
        "dispatches": [nf, nw],
        "note": "read = 2 x FETCH_SIZE (gfx950 wide-read correction, MI355X_MICROARCH.md HBM section)",
    }
    data = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            data = json.load(fh)
    data[a.config] = rec
    with open(a.out, "w") as fh:
        json.dump(data, fh, indent=1)
    print(json.dumps({a.config: rec}))


if __name__ == "__main__":
    main()
