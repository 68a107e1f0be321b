"""Expected fetched bytes of fetch_calib's patterns at 64-B and 128-B granularity, vs
the FETCH_SIZE counter (KiB) per dispatch. Usage: analyze.py <counter_collection.csv>"""
import csv, sys
from collections import defaultdict

GIB = 1 << 30


def touched(rec, chunks, unaligned, gran):
    n = GIB // rec
    tot = 0
    for r in range(n):
        first = ((r * 2654435761) % (1 << 64) >> 7) % (rec // 16 - chunks) if unaligned else 0
        # the kernel computes (r * 2654435761u) in size_t arithmetic
        first = ((r * 2654435761) >> 7) % (rec // 16 - chunks) if unaligned else 0
        a = r * rec + first * 16
        b = a + chunks * 16
        tot += ((b + gran - 1) // gran - a // gran) * gran
    return tot


exp = {
    "p_stream": (GIB, GIB),
    "p_desc8": (GIB, GIB),
}
for name, rec, ch, un in (("p_seg<4, 512, false>", 512, 4, False), ("p_seg<4, 512, true>", 512, 4, True),
                          ("p_seg<7, 1024, true>", 1024, 7, True)):
    exp[name] = (touched(rec, ch, un, 64), touched(rec, ch, un, 128))

vals = defaultdict(list)
with open(sys.argv[1]) as fh:
    for row in csv.DictReader(fh):
        vals[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    kb = sorted(v)[len(v) // 2] * 1024 if c == "FETCH_SIZE" else sorted(v)[len(v) // 2]
    for name, (e64, e128) in exp.items():
        if name in k:
            print(f"{name:24s} {c:12s} counter={kb/1e6:9.1f} MB  touched@64B={e64/1e6:9.1f} MB  "
                  f"touched@128B={e128/1e6:9.1f} MB  ratio64={kb/e64:.3f} ratio128={kb/e128:.3f}")
