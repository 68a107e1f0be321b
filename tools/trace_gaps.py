"""Median kernel durations and inter-kernel gaps from a rocprofv3 kernel trace (csv).

    python3 tools/trace_gaps.py <run_kernel_trace.csv> [min_count]
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(bt_\w+|k_\w+|copyBuffer\w*)", name)
    return m.group(1) if m else name[:30]


def main(path, min_count=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    durs, gaps = collections.defaultdict(list), collections.defaultdict(list)
    prev = None
    for r in rows:
        n = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        durs[n].append(e - s)
        if prev:
            gaps[(prev[0], n)].append(s - prev[1])
        prev = (n, e)
    med = lambda v: sorted(v)[len(v) // 2] / 1000.0
    for k, v in durs.items():
        if len(v) >= min_count:
            print(f"dur  {k:34s} n={len(v):4d} median {med(v):9.2f} us")
    for (a, b), v in gaps.items():
        if len(v) >= min_count:
            print(f"gap  {a:>20s} -> {b:20s} n={len(v):4d} median {med(v):7.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
