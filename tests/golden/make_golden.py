"""Generates the golden fixtures in tests/golden/ from the COMPILED REFERENCE.

Run in the build container (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py

For each capture it stores the inputs (frames + bt_pkt_desc) and the reference's
outputs: per-packet bt_rec records from the reference ProtocolParser walked layer by
layer (oracle/ref_harness.cpp:ref_parse) and, for every filter set in FILTER_SETS,
the per-packet PacketFilter::applyFilters(const Packet&) outcome (code, filterName
index). Nothing from /root/reference is copied: only data goes into the .npz files.
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

T = {"BPF": 0, "PROTOCOL": 1, "IP_RANGE": 2, "PORT_RANGE": 3, "PAYLOAD": 4, "CUSTOM": 5}


def single(t, exprs):
    return {f"{t.lower()}_{i}": [{"type": T[t], "expr": e}] for i, e in enumerate(exprs)}


QUIRK_EXPRS = {
    "BPF": ["", "tcp", "udp", "icmp", "not udp", "UDP", "tcp or udp", "xyz", "icmp and tcp"],
    "PROTOCOL": ["", "tcp", "udp", "icmp", "ip", "IP", "tcp ", "arp"],
    "IP_RANGE": ["", "10.0.0.0/8", "192.168.0.0/16", "10.0.0.0/0", "10.0.0.0/33", "10.0.0.0/-1",
                 "0.0.0.0/1", "128.0.0.0/1", "10.1.2.3", "10.1.2", "10.1.2.3.4", "266.0.0.0/8",
                 " 10.0.0.0/8", "10.0.0.0/8junk", "a.b.c.d/8", "10.0.0.0/x", "10..0.0/8",
                 "10.0.0.0/99999999999", "10.0.0.0/", "/8", "10.0.0.0/8/3", "10.0.0.0.", "-246.0.0.0/8",
                 "192.168.1.1/32"],
    "PORT_RANGE": ["", "1000-2000", "0-65535", "53", "2000-1000", "-5", "1000-", "66770", "1000-66770",
                   " 1000 - 2000", "abc", "99999999999", "0", "1000-2000-3000", "+1000-+2000"],
    "PAYLOAD": ["", "GET", "HTTP/1\\.1", "[", "^GET", "beatrice"],
}

FILTER_SETS = {
    # C3/C4 headline set: priorities 3/2/1
    "c3": [{"type": T["PROTOCOL"], "expr": "udp", "priority": 3},
           {"type": T["IP_RANGE"], "expr": "10.0.0.0/8", "priority": 2},
           {"type": T["PORT_RANGE"], "expr": "1000-2000", "priority": 1}],
    # a throwing filter behind a rejecting one: only packets that pass the first throw
    "throw_after": [{"type": T["PROTOCOL"], "expr": "tcp", "priority": 5},
                    {"type": T["PORT_RANGE"], "expr": "1000-", "priority": 1}],
    "throw_oor": [{"type": T["BPF"], "expr": "udp", "priority": 2},
                  {"type": T["IP_RANGE"], "expr": "10.0.0.0/99999999999", "priority": 1}],
    # disabled filters are skipped; order by priority, not insertion
    "mixed": [{"type": T["PORT_RANGE"], "expr": "0-1023", "priority": -1},
              {"type": T["BPF"], "expr": "tcp udp", "priority": 10},
              {"type": T["IP_RANGE"], "expr": "192.168.0.0/16", "priority": 4, "enabled": 0},
              {"type": T["IP_RANGE"], "expr": "192.168.0.0/17", "priority": 4},
              {"type": T["PROTOCOL"], "expr": "ip", "priority": 7}],
    # host-side filters in the chain
    "payload_mid": [{"type": T["PROTOCOL"], "expr": "tcp", "priority": 3},
                    {"type": T["PAYLOAD"], "expr": "GET", "priority": 2},
                    {"type": T["PORT_RANGE"], "expr": "0-2047", "priority": 1}],
    "custom": [{"type": T["CUSTOM"], "expr": "", "priority": 2, "custom": 1},
               {"type": T["CUSTOM"], "expr": "ignored", "priority": 1}],
    "unknown_type": [{"type": 9, "expr": "x", "priority": 1}],
    "empty": [],
}
for t, exprs in QUIRK_EXPRS.items():
    FILTER_SETS.update(single(t, exprs))

# PAYLOAD regexes for the GPU DFA: realistic application patterns and
# the corners of libstdc++'s ECMAScript semantics; a few stay on the host (\b, \1).
PAYLOAD_REGEXES = [
    "GET|POST", "^GET /", "HTTP/1\\.[01]", "Host: [a-z0-9.-]+\\.com", "User-Agent: .*(bot|curl)",
    "^\\x16\\x03[\\x00-\\x03]", "[\\x80-\\xff]{4,}", "\\d{3} [A-Z]", "\\r\\n\\r\\n", "^.{0,5}$",
    "^$", "a|", "[^]", "[]", "\\s+$", "(?:GET|HEAD) /[^ ]* HTTP", "x{0}y", "^[\\x00-\\x1f]",
    "passw(or)?d=", "\\bfoo", "(ab)\\1", "\\0", ".$", "[\\n\\r]",
]
FILTER_SETS.update({f"payload_re_{i}": [{"type": T["PAYLOAD"], "expr": e}] for i, e in enumerate(PAYLOAD_REGEXES)})
FILTER_SETS.update({
    # a GPU-resolvable PAYLOAD slot between built-in slots, and two of them in one program
    "payload_chain": [{"type": T["BPF"], "expr": "tcp", "priority": 4},
                      {"type": T["PAYLOAD"], "expr": "HTTP/1\\.[01]", "priority": 3},
                      {"type": T["PORT_RANGE"], "expr": "0-1023", "priority": 2},
                      {"type": T["PAYLOAD"], "expr": "Host: ", "priority": 1}],
    "payload_host_mix": [{"type": T["PAYLOAD"], "expr": "GET|POST", "priority": 3},
                         {"type": T["PAYLOAD"], "expr": "(GE)\\1?T", "priority": 2},
                         {"type": T["CUSTOM"], "expr": "", "priority": 1, "custom": 1}],
})


def http_frames(n=3000, seed=7):
    """Frames with application payloads for the PAYLOAD filter: HTTP requests and
    responses, TLS records, binary noise; IPv4 with IHL 5..15, TCP and UDP, frame lengths
    cutting the 100-byte window anywhere; some VLAN / IPv6 / short frames the filter's
    gates reject."""
    import random
    import struct
    rnd = random.Random(seed)
    texts = [b"GET /index.html HTTP/1.1\r\nHost: www.example.com\r\nUser-Agent: curl/8.0\r\n\r\n",
             b"POST /api/login HTTP/1.0\r\nHost: api.test.com\r\n\r\npassword=hunter2",
             b"HTTP/1.1 200 OK\r\nContent-Length: 12\r\n\r\nhello world!",
             b"HEAD /x HTTP/1.1\r\nUser-Agent: Googlebot\r\n\r\n",
             b"\x16\x03\x01\x02\x00\x01\x00\x01\xfc\x03\x03" + bytes(range(32)),
             b"passwd=secret&user=root", b"", b"x", b"\n", b"GEGET GT", b"404 Not Found\r\n"]
    out = []
    for i in range(n):
        kind = rnd.random()
        body = rnd.choice(texts)
        if rnd.random() < 0.3:
            body = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 140))) + body
        ihl = 5 if rnd.random() < 0.6 else rnd.randrange(5, 16)
        proto = 6 if rnd.random() < 0.7 else 17
        l4 = (struct.pack(">HHIIBBHHH", rnd.randrange(65536), rnd.choice([80, 443, 8080, 53]), i, 0, 0x50, 0x18,
                          1024, 0, 0) if proto == 6 else struct.pack(">HHHH", 5353, 53, 8 + len(body), 0))
        ip = bytes([0x40 | ihl, 0]) + struct.pack(">HHHBBH", 20 + len(l4) + len(body), i & 0xFFFF, 0, 64, proto, 0)
        ip += bytes([10, 1, i & 255, 7]) + bytes([192, 168, 1, 1]) + bytes(4 * (ihl - 5)) + l4 + body
        if kind < 0.05:
            f = b"\x01" * 12 + b"\x81\x00\x00\x05\x08\x00" + ip        # VLAN: gate fails
        elif kind < 0.08:
            f = b"\x01" * 12 + b"\x86\xdd" + ip                            # IPv6 EtherType
        else:
            f = b"\x02" * 12 + b"\x08\x00" + ip
        if rnd.random() < 0.25:
            f = f[: rnd.randrange(0, len(f) + 1)]                            # cut anywhere
        out.append(f)
    return out


def edge_frames():
    """Hand-built frames for the walk's and the filters' boundary cases."""
    import struct

    def eth(et, body=b"", dst=b"\x01\x02\x03\x04\x05\x06", src=b"\x0a\x0b\x0c\x0d\x0e\x0f"):
        return dst + src + struct.pack(">H", et) + body

    def ipv4(proto, l4=b"", ihl=5, src=b"\x0a\x01\x02\x03", dst=b"\xc0\xa8\x01\x01", opts=None):
        hdr = bytes([0x40 | ihl, 0x10]) + struct.pack(">HHHBBH", 20 + len(l4), 0x1234, 0x4000, 64, proto, 0xBEEF)
        hdr += src + dst
        if ihl > 5:
            hdr += (opts or bytes(range(1, 1 + 4 * (ihl - 5))))[: 4 * (ihl - 5)]
        return hdr + l4

    def udp(sp, dp, payload=b""):
        return struct.pack(">HHHH", sp, dp, 8 + len(payload), 0x55AA) + payload

    def tcp(sp, dp, doff=5, payload=b""):
        h = struct.pack(">HHIIBBHHH", sp, dp, 0x01020304, 0xA0B0C0D0, doff << 4, 0x18, 0xFFFF, 0x1111, 7)
        return h + bytes(4 * max(doff - 5, 0)) + payload

    def vlan(tpid, tci, inner_et, body):
        return struct.pack(">HH", tci, inner_et) + body, tpid

    def ipv6(nh, l4=b""):
        return struct.pack(">IHBB", 0x6ABCDEF1, len(l4), nh, 64) + bytes(range(16)) + bytes(range(16, 32)) + l4

    f = []
    base = eth(0x0800, ipv4(17, udp(1500, 53, b"GET / HTTP/1.1")))
    for n in range(0, 60):
        f.append(base[:n])                              # every truncation of a UDP frame
    tb = eth(0x0800, ipv4(6, tcp(1234, 1999, payload=b"GET x")))
    for n in (33, 34, 35, 41, 42, 43, 53, 54, 55):
        f.append(tb[:n])
    for ihl in range(0, 16):                            # every IHL, incl. < 5
        fr = bytearray(eth(0x0800, ipv4(6, tcp(80, 8080), ihl=max(ihl, 5))) + bytes(64))
        fr[14] = 0x40 | ihl
        f.append(bytes(fr))
    for doff in range(0, 16):
        f.append(eth(0x0800, ipv4(6, tcp(1000, 2000, doff=doff))) + bytes(8))
    # VLAN / QinQ, with truncations around the tag boundaries
    body4 = ipv4(17, udp(1000, 2000))
    inner = struct.pack(">HH", 0x0064, 0x0800) + body4
    q1 = eth(0x8100, inner)
    qq = eth(0x88A8, struct.pack(">HH", 0x00C8, 0x8100) + inner)
    q3 = eth(0x8100, struct.pack(">HH", 1, 0x8100) + struct.pack(">HH", 2, 0x8100) + inner)
    for fr in (q1, qq, q3):
        for n in (14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 37, 38, 41, 42, 45, 46, 49, 50, len(fr)):
            f.append(fr[:n])
    # IPv6 with TCP/UDP/other next headers, truncations
    for nh, l4 in ((6, tcp(443, 1500)), (17, udp(1000, 53)), (58, bytes(8)), (0, bytes(8))):
        fr = eth(0x86DD, ipv6(nh, l4))
        for n in (14, 20, 53, 54, 55, 61, 62, 73, 74, len(fr)):
            f.append(fr[:n])
        f.append(eth(0x8100, struct.pack(">HH", 5, 0x86DD) + ipv6(nh, l4)))
    # ICMP, ARP, odd EtherTypes, protocol 0
    f.append(eth(0x0800, ipv4(1, bytes([8, 0, 0xAB, 0xCD, 0, 1, 0, 2]) + bytes(20))))
    f.append(eth(0x0800, ipv4(1, bytes([8, 0, 0xAB, 0xCD, 0, 1]))))
    f.append(eth(0x0806, bytes(28)))
    f.append(eth(0x0800, ipv4(0, bytes(30))))
    f.append(eth(0x0800, ipv4(255, bytes(30))))
    f.append(eth(0x86DD, bytes(10)))
    # address / port boundary values for the filters
    for src, dst in ((b"\x0a\x00\x00\x00", b"\x0b\x00\x00\x00"), (b"\x09\xff\xff\xff", b"\x0a\xff\xff\xff"),
                     (b"\x80\x00\x00\x00", b"\x7f\xff\xff\xff"), (b"\xc0\xa8\x01\x01", b"\x01\x01\x01\x01"),
                     (b"\x0a\x01\x02\x03", b"\x00\x00\x00\x00"), (b"\x0a\x01\x02\x04", b"\x0a\x01\x02\x03")):
        f.append(eth(0x0800, ipv4(17, udp(53, 53), src=src, dst=dst)))
    for sp, dp in ((999, 2001), (1000, 5), (5, 2000), (2000, 1000), (0, 65535), (1234, 1), (53, 0)):
        f.append(eth(0x0800, ipv4(17, udp(sp, dp))))
        f.append(eth(0x0800, ipv4(6, tcp(sp, dp))))
    # a frame longer than 65535 is impossible in bt_pkt_desc; a long one near the cap
    f.append(eth(0x0800, ipv4(17, udp(1500, 1500, bytes(9000)))))
    # ProtocolDetector (ProtocolRegistry.cpp:353-487): its isIPv4/isIPv6 read the version
    # nibble of frame byte 0 (the destination MAC), so these frames put 0x4_/0x6_ there;
    # HTTP/DNS ports on either side, every length gate (14, 28, 34, 42, 54) and ARP
    for mac0 in (b"\x45", b"\x4f", b"\x60", b"\x6a", b"\x05"):
        dst = mac0 + b"\x00\x00\x00\x00\x01"
        for fr in (eth(0x0800, ipv4(6, tcp(80, 1234)), dst=dst), eth(0x0800, ipv4(6, tcp(1234, 80)), dst=dst),
                   eth(0x0800, ipv4(17, udp(53, 9)), dst=dst), eth(0x0800, ipv4(17, udp(9, 53)), dst=dst),
                   eth(0x0800, ipv4(1, bytes(8)), dst=dst), eth(0x86DD, ipv6(6, tcp(80, 80)), dst=dst),
                   eth(0x0806, bytes(28), dst=dst), eth(0x0800, ipv4(6, tcp(8080, 80)), dst=dst)):
            f.append(fr)
        for n in (13, 14, 27, 28, 33, 34, 41, 42, 53, 54):
            f.append(eth(0x0806 if n < 34 else 0x0800, ipv4(17 if n < 50 else 6,
                                                             udp(53, 53) if n < 50 else tcp(80, 80)), dst=dst)[:n])
    return f


def build():
    out = {}
    caps = {
        "c1": (synth.capture(synth.C2, 10000), "C1: 10k fixed 64 B Eth/IPv4/UDP"),
        "c3": (synth.capture(synth.C3, 4096), "C3: IMIX 64/512/1500, 25% 802.1Q"),
        "c4": (synth.capture(synth.C4, 2048), "C4: QinQ/IPv6/IHL+TCP options, 2-mod-4 offsets"),
        "fuzz": (synth.capture(synth.FUZZ, 8192), "fuzz: short/odd frames, byte mutations"),
        "edge": (synth.pack_frames(edge_frames(), align=4, shift=2), "edge: hand-built boundary frames"),
        "http": (synth.pack_frames(http_frames(), align=2, shift=0),
                 "http: application payloads (HTTP, TLS, noise) for PAYLOAD regexes, IHL 5..15, cut frames"),
    }
    manifest = {"filter_sets": FILTER_SETS, "captures": {}}
    for name, ((data, desc), what) in caps.items():
        n = len(desc)
        rec = ol.ref_parse(data, desc, n)
        arrays = {"data": data, "desc": desc, "rec": rec}
        payload_sets = [k for k in FILTER_SETS if k.startswith("payload_re_")] + ["payload_chain",
                                                                                   "payload_host_mix"]
        if name in ("edge", "fuzz"):
            sets = list(FILTER_SETS)
        elif name == "http":
            sets = ["c3", "payload_mid", "empty"] + [k for k in FILTER_SETS if k.startswith("payload_")]
        else:
            sets = ["c3", "mixed", "throw_after", "payload_mid", "custom", "empty"] + payload_sets[:6]
        for s in sets:
            code, src = ol.ref_filter(data, desc, n, FILTER_SETS[s])
            arrays[f"code__{s}"] = code
            arrays[f"src__{s}"] = src
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        manifest["captures"][name] = {"n": n, "what": what, "filter_sets": sets}
        print(name, n, "frames", data.nbytes, "bytes;", len(sets), "filter sets")
    path = os.path.join(HERE, "manifest.json")
    if os.path.exists(path):   # keep entries other generators own (make_ring_fixture.py: "rings")
        with open(path) as fh:
            old = json.load(fh)
        for k, v in old.items():
            manifest.setdefault(k, v)
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1)


if __name__ == "__main__":
    if not ol.ref_available():
        sys.exit("oracle/_ref/libbt_ref.so missing: make -C oracle ref (needs /root/reference)")
    build()
