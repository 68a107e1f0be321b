"""C1 (BASELINE.json configs[0]): 10k synthetic 64-B Eth/IPv4/UDP frames sent over
AF_PACKET on the loopback interface, captured by a TPACKET_V3 RX ring, walked
(bt_ring_walk_tpv3) and run through the parser + PacketFilter on the CPU.

The reference's plumbing for this config is parser_example.cpp plus its AF_PACKET
backend. Here the frames are the `c1` golden capture, whose
records and filter outcomes come from the compiled reference; every captured copy of
every frame must give exactly those outputs. The oracle stands in for the device (this
is the CPU config), and the compiled reference itself is run on the captured frames as
well. An ETH_P_ALL socket on `lo` sees each frame twice (outgoing and incoming), so the
frames are matched by content."""
import mmap
import socket
import struct
import time

import numpy as np
import pytest

import oracle_lib as ol
import ring_util as ru
from beatrice_amd import abi, synth
from conftest import load_golden
from golden_util import compare_decisions


def _can_raw():
    try:
        socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3)).close()
        return True
    except (PermissionError, OSError):
        return False


@pytest.mark.skipif(not _can_raw(), reason="no CAP_NET_RAW: cannot open an AF_PACKET ring")
def test_c1_frames_over_loopback_ring():
    g, man = load_golden("c1")
    data, desc = g["data"], g["desc"]
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    frames = [bytes(data[o:o + n]) for o, n in zip(off, ln)]
    index = {f: i for i, f in enumerate(frames)}
    assert len(index) == len(frames) == 10000

    bs, nb = 1 << 20, 16
    rx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
    rx.setsockopt(263, 10, 2)                                                         # TPACKET_V3
    rx.setsockopt(263, 5, struct.pack("7I", bs, nb, 2048, bs * nb // 2048, 5, 0, 0))  # RX ring, 5 ms retire
    rx.bind(("lo", 3))
    m = mmap.mmap(rx.fileno(), bs * nb)
    tx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW)
    tx.bind(("lo", 0))
    try:
        for f in frames:
            tx.send(f)
        time.sleep(0.2)
        ring = np.frombuffer(m, dtype=np.uint8)
        cap, taken = abi.ring_walk_tpv3(ring, bs, nb)
        assert taken >= 1 and np.array_equal(cap, ru.walk_tpv3(ring, bs, nb)[0])
        img = np.array(ring[: taken * bs])          # a copy, so the ring can go back to the kernel
        abi.ring_release_tpv3(ring, bs, nb, 0, taken)
        del ring
    finally:
        m.close()
        tx.close()
        rx.close()

    coff, cln = synth.desc_off(cap), synth.desc_len(cap)
    got = [index.get(bytes(img[o:o + n]), -1) for o, n in zip(coff, cln)]
    mine = np.array([i for i in got if i >= 0])
    keep = np.array([k for k, i in enumerate(got) if i >= 0])
    assert set(mine.tolist()) == set(range(10000)), "frames lost between send and ring"
    cdesc = cap[keep]
    n = len(cdesc)
    # parser: the oracle and the compiled reference on the captured frames == the golden
    rec, _, _ = ol.oracle_run(img, cdesc, n, None, parse=True)
    assert np.array_equal(rec, g["rec"][mine])
    assert np.array_equal(ol.ref_parse(img, cdesc, n), g["rec"][mine])
    # PacketFilter: every filter set the golden holds for c1
    for s in man["captures"]["c1"]["filter_sets"]:
        filters = man["filter_sets"][s]
        _, dec, _ = ol.oracle_run(img, cdesc, n, filters, parse=False)
        compare_decisions(dec, g[f"code__{s}"][mine], g[f"src__{s}"][mine], filters, where=f"c1-loopback/{s}")
