#!/usr/bin/env python3
"""Parse one hex-encoded frame on the GPU and print every walked layer's ParseResult,
the counterpart of the reference CLI's `beatrice parser --raw=HEX --format=F`
(src/beatrice_cli.cpp:1632-1666). The reference parses a single protocol there; this
prints the whole layer walk (DESIGN.md "R-WALK") in the reference's formatter text
(bt_format_records), plus the ProtocolDetector verdict.

    python tools/parse_raw.py --raw 0102030405060a0b0c0d0e0f0800450000... --format json
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beatrice_amd import abi  # noqa: E402

FORMATS = {"json": abi.FMT_JSON, "xml": abi.FMT_XML, "csv": abi.FMT_CSV, "human": abi.FMT_HUMAN}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--raw", required=True, help="frame bytes as hex")
    ap.add_argument("--format", default="human", choices=sorted(FORMATS))
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    # the CLI's hex decode: pairs of digits, a trailing odd digit dropped (:1637-1643)
    raw = a.raw[: len(a.raw) // 2 * 2]
    frame = np.frombuffer(bytes.fromhex(raw), np.uint8)
    data = np.zeros(max(16, (len(frame) + 15) // 16 * 16), np.uint8)
    data[: len(frame)] = frame
    desc = np.array([len(frame) << 48], np.uint64)
    ctx = abi.Context(a.device)
    try:
        ctx.compile([])
        out = ctx.run_host(data, desc, records=True, filters=False)
        rec = out["records"]
        sys.stdout.write(abi.format_records(rec, FORMATS[a.format], ctx=ctx).decode())
        r = np.ascontiguousarray(rec).reshape(-1).view(abi.REC_DTYPE)[0]
        print(f"detected: {abi.DETECT_NAMES[int(r['detect_code'])]!r}")
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
