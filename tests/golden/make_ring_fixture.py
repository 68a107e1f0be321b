"""Generates tests/golden/ring_lo.npz: a TPACKET_V3 RX ring image WRITTEN BY THE LINUX
KERNEL, plus the compiled reference's outputs for every frame in it.

Run as root in the build container (needs CAP_NET_RAW, /root/reference and
`make -C oracle ref`):

    python tests/golden/make_ring_fixture.py

It opens an AF_PACKET socket on `lo` with PACKET_VERSION = TPACKET_V3 and a
PACKET_RX_RING, then puts traffic on the loopback:
  * every frame of the `edge` golden capture and 256 C4 frames (QinQ / IPv6 / IPv4
    options), injected through a second AF_PACKET socket;
  * real UDP over IPv4 and IPv6, a TCP connection and ICMP echo on 127.0.0.1.
After the blocks retire (retire_blk_tov) the ring memory is saved as-is, together
with the ring geometry and, for each frame the ring holds (walked with
tests/ring_util.py), the reference ProtocolParser records and the reference
PacketFilter outcome for several filter sets. Only data is stored.
"""
from __future__ import annotations

import json
import mmap
import os
import socket
import struct
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from beatrice_amd import synth  # noqa: E402
import oracle_lib as ol  # noqa: E402
import ring_util  # noqa: E402
from make_golden import FILTER_SETS, edge_frames  # noqa: E402

SOL_PACKET, PACKET_RX_RING, PACKET_VERSION, TPACKET_V3 = 263, 5, 10, 2
ETH_P_ALL = 0x0003
BLOCK_SIZE, N_BLOCKS, FRAME_SIZE, RETIRE_MS = 1 << 17, 16, 2048, 20
SETS = ["c3", "mixed", "throw_after", "payload_mid", "custom", "empty", "bpf_1", "port_range_1", "ip_range_1"]


def open_ring():
    s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
    s.setsockopt(SOL_PACKET, PACKET_VERSION, TPACKET_V3)
    req = struct.pack("7I", BLOCK_SIZE, N_BLOCKS, FRAME_SIZE, BLOCK_SIZE * N_BLOCKS // FRAME_SIZE, RETIRE_MS, 0, 0)
    s.setsockopt(SOL_PACKET, PACKET_RX_RING, req)
    s.bind(("lo", ETH_P_ALL))
    m = mmap.mmap(s.fileno(), BLOCK_SIZE * N_BLOCKS, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    return s, m


def traffic():
    inj = socket.socket(socket.AF_PACKET, socket.SOCK_RAW)
    inj.bind(("lo", 0))
    frames = list(edge_frames())
    data, desc = synth.capture(synth.C4, 256, seed=11)
    for d in desc:
        off, ln = int(d) & ((1 << 48) - 1), int(d) >> 48
        frames.append(bytes(data[off:off + ln]))
    sent = 0
    for f in frames:
        try:
            inj.send(f)
            sent += 1
        except OSError:
            pass          # the device refuses some frames (e.g. shorter than the link header)
    inj.close()
    # real stack traffic
    u4 = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    for i, n in enumerate((0, 1, 18, 64, 200, 1400, 4000)):
        u4.sendto(bytes([i]) * n, ("127.0.0.1", 1000 + 100 * i))
    u4.close()
    u6 = socket.socket(socket.AF_INET6, socket.SOCK_DGRAM)
    for i in range(4):
        u6.sendto(b"v6" * (10 * i), ("::1", 1500 + i))
    u6.close()
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def serve():
        c, _ = srv.accept()
        c.sendall(c.recv(100) * 2)
        c.close()

    t = threading.Thread(target=serve)
    t.start()
    cl = socket.create_connection(srv.getsockname())
    cl.sendall(b"GET / HTTP/1.1\r\n\r\n")
    cl.recv(100)
    cl.close()
    t.join()
    srv.close()
    ic = socket.socket(socket.AF_INET, socket.SOCK_RAW, socket.IPPROTO_ICMP)
    for i in range(3):
        ic.sendto(struct.pack("!BBHHH", 8, 0, 0, 7, i) + b"ping", ("127.0.0.1", 0))
    ic.close()
    return sent, len(frames)


def refresh():
    """Re-derives the expected outputs of the saved ring from the compiled reference
    (after the record layout gained a column), without capturing a new ring."""
    path = os.path.join(HERE, "ring_lo.npz")
    old = np.load(path)
    arrays = {k: old[k] for k in old.files}
    n = len(arrays["desc"])
    arrays["rec"] = ol.ref_parse(arrays["ring"], arrays["desc"], n)
    for name in SETS:
        code, src = ol.ref_filter(arrays["ring"], arrays["desc"], n, FILTER_SETS[name])
        assert np.array_equal(code, arrays[f"code__{name}"]) and np.array_equal(src, arrays[f"src__{name}"]), name
    np.savez_compressed(path, **arrays)
    print(f"ring_lo: {n} frames, expected records refreshed")


def main():
    if not ol.ref_available():
        sys.exit("oracle/_ref/libbt_ref.so missing: make -C oracle ref (needs /root/reference)")
    if "--refresh" in sys.argv:
        return refresh()
    s, m = open_ring()
    sent, total = traffic()
    time.sleep(8 * RETIRE_MS / 1000)
    ring = np.frombuffer(m, dtype=np.uint8).copy()
    m.close()
    s.close()
    desc, taken = ring_util.walk_tpv3(ring, BLOCK_SIZE, N_BLOCKS)
    used = max(b for b, *_ in ring_util.frame_headers(ring, BLOCK_SIZE, N_BLOCKS)) + 1
    ring = ring[:used * BLOCK_SIZE]        # blocks after the last filled one are all zero
    n = len(desc)
    arrays = {"ring": ring, "geometry": np.array([BLOCK_SIZE, used], np.uint64), "desc": desc,
              "rec": ol.ref_parse(ring, desc, n)}
    for name in SETS:
        code, src = ol.ref_filter(ring, desc, n, FILTER_SETS[name])
        arrays[f"code__{name}"] = code
        arrays[f"src__{name}"] = src
    np.savez_compressed(os.path.join(HERE, "ring_lo.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json")) as fh:
        man = json.load(fh)
    man["rings"] = {"ring_lo": {"n": n, "blocks": used, "block_size": BLOCK_SIZE, "filter_sets": SETS,
                                "what": f"TPACKET_V3 ring on lo written by the kernel: {sent}/{total} injected "
                                        "frames (edge + C4) plus UDPv4/UDPv6/TCP/ICMP stack traffic"}}
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(man, fh, indent=1)
    print(f"ring_lo: {n} frames in {taken} of {used} blocks, injected {sent}/{total}")


if __name__ == "__main__":
    main()
