"""Generates tests/golden/extract.npz + extract.json from the COMPILED REFERENCE: user-defined
protocol tables through ProtocolParser::parsePacket(frame, ProtocolDefinition)
(reference src/parser/ProtocolParser.cpp:97-110, 238-433), driven by
oracle/ref_harness.cpp:ref_extract.

Run in the build container (needs `make -C oracle ref`):

    python tests/golden/make_extract_golden.py

Tables:
  * parser_example: the reference's only known-answer test (examples/parser_example.cpp:18-43):
    CUSTOM_PROTO = header u32 @0, version u8 @4, length u16 @5 (NETWORK), data BYTES[10] @7,
    on its 17-byte packet (header 0x12345678, version 1, length 10, data aabbccddeeff11223344)
    and on every fuzz frame;
  * seeded random tables over every FieldType and Endianness, lengths both natural and not
    (a u8 of 5 bytes, a float of 3, a 20-byte u64 ...), offsets inside the 256-byte staged
    window and past it, and the empty table.
Frames: seeded random bytes, lengths 0..320. TIMESTAMP fields stay <= 5 bytes: the
reference formats every TIMESTAMP with localtime(), which returns NULL (and put_time
crashes) for values past its range. Only data goes into the fixture files.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from beatrice_amd import synth  # noqa: E402
import oracle_lib as ol  # noqa: E402

NATURAL = {0: 1, 1: 2, 2: 4, 3: 8, 4: 1, 5: 2, 6: 4, 7: 8, 8: 4, 9: 8, 12: 1, 13: 6, 14: 4, 15: 16, 16: 8}
PARSER_EXAMPLE = [(0, 4, 2, 2), (4, 1, 0, 2), (5, 2, 1, 2), (7, 10, 10, 2)]
PARSER_EXAMPLE_PACKET = bytes([0x12, 0x34, 0x56, 0x78, 0x01, 0x00, 0x0A, 0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF,
                               0x11, 0x22, 0x33, 0x44])


def random_table(rng, far=False):
    nf = int(rng.integers(1, 11))
    out = []
    for _ in range(nf):
        t = int(rng.integers(0, 18))
        if t == 16:
            ln = int(rng.integers(0, 6))
        elif t in NATURAL and rng.random() < 0.6:
            ln = NATURAL[t]
        else:
            ln = int(rng.integers(1 if t == 12 else 0, 21))
        o = int(rng.integers(200, 300)) if far and rng.random() < 0.5 else int(rng.integers(0, 80))
        out.append((o, ln, t, int(rng.integers(0, 4))))
    return out


def frames(rng, n):
    fs = [PARSER_EXAMPLE_PACKET]
    for i in range(n - 1):
        ln = int(rng.integers(0, 321)) if i % 4 else int(rng.integers(0, 40))
        fs.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
    return fs


def main():
    rng = np.random.default_rng(0x5EED00E7)
    fr = frames(rng, 600)
    data, desc = synth.pack_frames(fr, align=1)
    n = len(desc)
    tables = {"parser_example": PARSER_EXAMPLE, "empty": []}
    for k in range(36):
        tables[f"rand_{k}"] = random_table(rng, far=(k % 4 == 3))
    out = {"data": data, "desc": desc}
    for name, t in tables.items():
        st, val, fb = ol.ref_extract(data, desc, n, t)
        out[f"status__{name}"] = st
        out[f"values__{name}"] = val
        out[f"fb__{name}"] = fb
    np.savez_compressed(os.path.join(HERE, "extract.npz"), **out)
    with open(os.path.join(HERE, "extract.json"), "w") as fh:
        json.dump({"n": n, "seed": "0x5EED00E7", "tables": tables,
                   "what": "ref_extract (oracle/ref_harness.cpp) = ProtocolParser::parsePacket(frame, def) per frame; "
                           "frame 0 is parser_example's 17-byte packet"}, fh, indent=1)
    st, val, fb = out["status__parser_example"], out["values__parser_example"], out["fb__parser_example"]
    print("parser_example KAT:", st[0], hex(int(val[0, 0])), int(val[1, 0]), int(val[2, 0]), bytes(fb[0, 7:17]).hex())


if __name__ == "__main__":
    main()
