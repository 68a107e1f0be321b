"""CPU: AF_PACKET TPACKET_V3 capture-ring ingest — the block walker
bt_ring_walk_tpv3 / bt_ring_release_tpv3 and the ring-image packer, against

  * tests/golden/ring_lo.npz, a ring WRITTEN BY THE LINUX KERNEL on `lo`
    (tests/golden/make_ring_fixture.py) with the compiled reference's records and
    PacketFilter outcomes for every frame in it;
  * tests/ring_util.walk_tpv3, a plain-Python restatement of the walk;
  * a live ring on `lo` when this process may open AF_PACKET sockets.

None of these need a GPU: the walker is host code (ctx = NULL)."""
import mmap
import os
import socket
import struct
import time

import numpy as np
import pytest

import oracle_lib as ol
import ring_util as ru
from beatrice_amd import abi, synth
from conftest import GOLDEN
from golden_util import compare_decisions


def _fixture():
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    bs, nb = (int(x) for x in g["geometry"])
    return g, bs, nb


def test_walk_kernel_ring_matches_python_walk():
    g, bs, nb = _fixture()
    ring = g["ring"].copy()
    desc, taken = abi.ring_walk_tpv3(ring, bs, nb)
    ref, ref_taken = ru.walk_tpv3(ring, bs, nb)
    assert taken == ref_taken == nb
    assert np.array_equal(desc, ref) and np.array_equal(desc, g["desc"])
    assert len(desc) > 900


def test_kernel_ring_layout_is_what_the_packer_writes():
    g, bs, nb = _fixture()
    assert ru.layout_violations(g["ring"], bs, nb) == []
    frames = np.array(g["ring"])
    ring, rdesc, used = synth.tpv3_ring(frames, g["desc"], block_size=bs)
    assert ru.layout_violations(ring, bs, used) == []
    assert np.array_equal(ru.walk_tpv3(ring, bs, used)[0], rdesc)


def test_oracle_on_kernel_ring_matches_reference():
    """The reference's own outputs on kernel-captured frames pin the oracle there too."""
    g, bs, nb = _fixture()
    import json
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    info = man["rings"]["ring_lo"]
    n = len(g["desc"])
    rec, _, _ = ol.oracle_run(g["ring"], g["desc"], n, None, parse=True)
    assert np.array_equal(rec, g["rec"])
    for s in info["filter_sets"]:
        filters = man["filter_sets"][s]
        _, dec, _ = ol.oracle_run(g["ring"], g["desc"], n, filters, parse=False)
        compare_decisions(dec, g[f"code__{s}"], g[f"src__{s}"], filters, where=f"ring_lo/{s}")


@pytest.mark.parametrize("cfg,block", [(synth.C2, 1 << 16), (synth.C3, 1 << 17), (synth.C4, 1 << 20)])
def test_packed_ring_round_trip(cfg, block):
    data, desc = synth.capture(cfg, 20000, seed=5)
    ring, rdesc, used = synth.tpv3_ring(data, desc, block_size=block)
    assert len(rdesc) == len(desc) and used > 1
    got, taken = abi.ring_walk_tpv3(ring, block, used)
    assert taken == used and np.array_equal(got, rdesc)
    off, ln = synth.desc_off(got), synth.desc_len(got)
    assert np.array_equal(ln, synth.desc_len(desc))
    src = synth.desc_off(desc)
    for i in np.random.default_rng(0).integers(0, len(desc), 300):
        assert bytes(ring[off[i]:off[i] + ln[i]]) == bytes(data[src[i]:src[i] + ln[i]])


def test_walk_limits_wrap_and_release():
    data, desc = synth.capture(synth.C3, 6000, seed=9)
    bs = 1 << 16
    ring, rdesc, used = synth.tpv3_ring(data, desc, block_size=bs)
    per_block = [npk for _, npk, _, _ in ru.frame_headers(ring, bs, used)]
    start = np.concatenate([[0], np.cumsum(per_block)])
    # max_blocks and cap stop at whole blocks
    d, t = abi.ring_walk_tpv3(ring, bs, used, first=0, max_blocks=3)
    assert t == 3 and np.array_equal(d, rdesc[:start[3]])
    d, t = abi.ring_walk_tpv3(ring, bs, used, first=0, cap=int(start[2]) + 1)
    assert t == 2 and len(d) == start[2]
    # starting mid-ring wraps round to block 0
    d, t = abi.ring_walk_tpv3(ring, bs, used, first=used - 2, max_blocks=4)
    assert t == 4 and np.array_equal(d, np.concatenate([rdesc[start[used - 2]:], rdesc[:start[2]]]))
    # released blocks belong to the kernel again: the walk stops there
    abi.ring_release_tpv3(ring, bs, used, 1, 2)
    d, t = abi.ring_walk_tpv3(ring, bs, used, first=0)
    assert t == 1 and len(d) == start[1]
    d, t = abi.ring_walk_tpv3(ring, bs, used, first=1)
    assert t == 0 and len(d) == 0
    assert np.all(ring.reshape(used, bs)[1:3, 8:12].view(np.uint32) == ru.TP_STATUS_KERNEL)


def test_malformed_ring_is_rejected():
    data, desc = synth.capture(synth.C2, 3000, seed=3)
    bs = 1 << 16
    ring, _, used = synth.tpv3_ring(data, desc, block_size=bs)
    _, _, _, frames = next(ru.frame_headers(ring, bs, used))
    bad = ring.copy()
    off = bs + frames[5][0]        # frame 5 of block 1 points far outside the block
    bad[off:off + 4] = np.frombuffer(struct.pack("<I", bs), np.uint8)
    with pytest.raises(abi.BtError, match="frame chain leaves the block"):
        abi.ring_walk_tpv3(bad, bs, used)
    bad = ring.copy()              # first-frame offset past the block
    bad[bs + 16:bs + 20] = np.frombuffer(struct.pack("<I", bs + 8), np.uint8)
    with pytest.raises(abi.BtError, match="first frame outside block"):
        abi.ring_walk_tpv3(bad, bs, used)
    with pytest.raises(abi.BtError):
        abi.ring_walk_tpv3(ring, bs, used, first=used)
    # the gathers walk the same chains and refuse the same rings
    n = len(desc) + 64
    for dense in (False, True):
        bad = ring.copy()
        bad[off:off + 4] = np.frombuffer(struct.pack("<I", bs), np.uint8)
        slots, out = np.zeros(n * abi.PREFIX_SLOT, np.uint8), np.zeros(n, np.uint64)
        with pytest.raises(abi.BtError, match="frame chain leaves the block"):
            abi.ring_gather_tpv3(bad, bs, used, slots, out, dense=dense)
    with pytest.raises(abi.BtError, match="16-B aligned"):
        abi.ring_gather_tpv3(ring, bs, used, np.zeros(n * abi.PREFIX_SLOT + 16, np.uint8)[1:], out, dense=True)
    with pytest.raises(ValueError):   # ring descriptors come with the packed gather only
        abi.ring_gather_tpv3(ring, bs, used, slots, out, dense=False, ring_out=np.zeros(n, np.uint64))


def _can_raw():
    try:
        socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3)).close()
        return True
    except (PermissionError, OSError):
        return False


@pytest.mark.skipif(not _can_raw(), reason="no CAP_NET_RAW: cannot open an AF_PACKET ring")
def test_live_ring_on_loopback():
    bs, nb = 1 << 16, 8
    s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
    s.setsockopt(263, 10, 2)                                           # PACKET_VERSION = TPACKET_V3
    s.setsockopt(263, 5, struct.pack("7I", bs, nb, 2048, bs * nb // 2048, 5, 0, 0))   # PACKET_RX_RING
    s.bind(("lo", 3))
    m = mmap.mmap(s.fileno(), bs * nb)
    try:
        u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        marks = [b"bt-ring-%04d" % i for i in range(50)]
        for i, mk in enumerate(marks):
            u.sendto(mk * (1 + i % 7), ("127.0.0.1", 4000 + i))
        u.close()
        time.sleep(0.1)
        ring = np.frombuffer(m, dtype=np.uint8)
        desc, taken = abi.ring_walk_tpv3(ring, bs, nb)
        assert taken >= 1 and np.array_equal(desc, ru.walk_tpv3(ring, bs, nb)[0])
        frames = [bytes(ring[o:o + n]) for o, n in zip(synth.desc_off(desc), synth.desc_len(desc))]
        for mk in marks:
            assert any(mk in f for f in frames), mk
        abi.ring_release_tpv3(ring, bs, nb, 0, taken)
        del ring
    finally:
        m.close()
        s.close()


@pytest.mark.skipif(not _can_raw(), reason="no CAP_NET_RAW: cannot open an AF_PACKET ring")
@pytest.mark.parametrize("rings", [2, 3])
def test_fanout_hash_rings_split_by_flow(rings):
    """Per-GPU ring sharding: `rings` TPACKET_V3 rings on lo in one
    PACKET_FANOUT_HASH group (TpacketV3Ring::Options::fanoutGroup, one ring per GPU worker).
    The c1 golden frames go out as UDP payloads over 40 flows (distinct source ports); every
    frame lands in exactly one ring and every flow in one ring, and the walker reads each ring
    as bt_ring_walk_tpv3 does. Only each datagram's receive copy (sll_pkttype PACKET_HOST) is
    counted: lo also hands the rings its transmit copy, whose hash is the sending socket's random
    tx hash, where a NIC's receive ring sees the receive copy alone."""
    import random
    from conftest import load_golden
    g, _ = load_golden("c1")
    frames = [bytes(g["data"][o:o + n]) for o, n in zip(synth.desc_off(g["desc"]), synth.desc_len(g["desc"]))][:200]
    bs, nb = 1 << 16, 16
    group = random.randint(1, 0xFFFF)
    socks, maps = [], []
    try:
        for _ in range(rings):
            s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(3))
            s.setsockopt(263, 10, 2)                                       # PACKET_VERSION = TPACKET_V3
            s.setsockopt(263, 5, struct.pack("7I", bs, nb, 2048, bs * nb // 2048, 5, 0, 0))   # PACKET_RX_RING
            s.bind(("lo", 3))
            s.setsockopt(263, 18, group | (0 << 16))                       # PACKET_FANOUT, PACKET_FANOUT_HASH
            socks.append(s)
            maps.append(mmap.mmap(s.fileno(), bs * nb))
        sinks = []   # listeners, so that no ICMP port-unreachable (quoting the payload) comes back
        for p in range(7):
            k = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            k.bind(("127.0.0.1", 0))
            sinks.append(k)
        ports = [k.getsockname()[1] for k in sinks]
        senders = []
        for f in range(40):
            u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            u.bind(("127.0.0.1", 0))
            senders.append(u)
        sent = {}
        for i, fr in enumerate(frames):
            f = i % 40
            mark = b"bt-fan-%03d-%02d|" % (i, f)
            senders[f].sendto(mark + fr, ("127.0.0.1", ports[f % 7]))
            sent[mark] = f
        for u in senders + sinks:
            u.close()
        time.sleep(0.2)
        where = {}   # mark -> set of rings
        for r, m in enumerate(maps):
            ring = np.frombuffer(m, dtype=np.uint8)
            desc, taken = abi.ring_walk_tpv3(ring, bs, nb)
            assert np.array_equal(desc, ru.walk_tpv3(ring, bs, nb)[0])
            buf = memoryview(m)
            j = 0
            for b in range(taken):   # each frame's sll_pkttype: tpacket3_hdr (48 B), then sockaddr_ll
                status, npk, off = struct.unpack_from("<III", buf, b * bs + 8)
                for _ in range(npk):
                    nxt = struct.unpack_from("<I", buf, b * bs + off)[0]
                    host = buf[b * bs + off + 48 + 10] == 0   # PACKET_HOST
                    o, n = int(synth.desc_off(desc[j:j + 1])[0]), int(synth.desc_len(desc[j:j + 1])[0])
                    fr = bytes(ring[o:o + n])
                    k = fr.find(b"bt-fan-")
                    if host and k >= 0 and n > 23 and fr[23] == 17:
                        where.setdefault(fr[k:k + 14], set()).add(r)
                    off += nxt
                    j += 1
            assert j == len(desc)
            del buf
            abi.ring_release_tpv3(ring, bs, nb, 0, taken)
            del ring
        missing = [m for m in sent if m not in where]
        assert not missing, f"{len(missing)} frames captured by no ring"
        assert all(len(v) == 1 for v in where.values()), "a frame landed in two rings"
        flow_rings = {}
        for m, f in sent.items():
            flow_rings.setdefault(f, set()).update(where[m])
        assert all(len(v) == 1 for v in flow_rings.values()), "a flow was split across rings"
        assert len({next(iter(v)) for v in flow_rings.values()}) > 1, "every flow hashed to one ring"
    finally:
        for m in maps:
            m.close()
        for s in socks:
            s.close()


CAPTURE_BIN = os.path.join(os.path.dirname(GOLDEN), "cpp", "test_capture")


@pytest.mark.skipif(not _can_raw(), reason="no CAP_NET_RAW: cannot open an AF_PACKET ring")
def test_cpp_backend_on_loopback():
    """GpuAfPacketBackend (ICaptureBackend drop-in) on a live TPACKET_V3 ring on lo."""
    import subprocess
    assert os.path.exists(CAPTURE_BIN), "tests/cpp/test_capture not built (make -C tests/cpp)"
    r = subprocess.run([CAPTURE_BIN, "backend"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("which", ["kernel_ring", "c2", "c3", "c4", "fuzz"])
def test_gather_prefixes_hold_every_byte_the_walk_reads(which):
    """bt_ring_gather_tpv3: the header prefixes in their 128-B slots (rest of each slot
    poisoned) give the oracle the same records and filter decisions as the whole frames
    in the ring, for every built-in filter set; descriptors keep the real lengths."""
    import json
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    if which == "kernel_ring":
        g, bs, nb = _fixture()
        ring, used = g["ring"].copy(), nb
    else:
        cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4, "fuzz": synth.FUZZ}[which]
        data, desc = synth.capture(cfg, 6000, seed=11)
        bs = 1 << 16
        ring, _, used = synth.tpv3_ring(data, desc, block_size=bs)
    wdesc, taken = abi.ring_walk_tpv3(ring, bs, used)
    n = len(wdesc)
    slots = np.full(n * abi.PREFIX_SLOT, 0xA5, np.uint8)
    out = np.zeros(n, np.uint64)
    gdesc, gtaken = abi.ring_gather_tpv3(ring, bs, used, slots, out)
    assert gtaken == taken and len(gdesc) == n
    assert np.array_equal(synth.desc_len(gdesc), synth.desc_len(wdesc))
    assert np.array_equal(synth.desc_off(gdesc), np.arange(n, dtype=np.uint64) * abi.PREFIX_SLOT)
    _same_as_ring(ring, wdesc, slots, gdesc, man)


def _same_as_ring(ring, wdesc, slots, gdesc, man):
    n = len(wdesc)
    rec_w, _, _ = ol.oracle_run(ring, wdesc, n, None, parse=True)
    rec_g, _, _ = ol.oracle_run(slots, gdesc, n, None, parse=True)
    assert np.array_equal(rec_g, rec_w)
    for s in ("c3", "mixed", "throw_after", "bpf_1", "port_range_1", "ip_range_1"):
        filters = man["filter_sets"][s]
        _, dw, _ = ol.oracle_run(ring, wdesc, n, filters, parse=False)
        _, dg, _ = ol.oracle_run(slots, gdesc, n, filters, parse=False)
        assert np.array_equal(dg, dw), s


@pytest.mark.parametrize("which", ["kernel_ring", "c2", "c3", "c4", "fuzz"])
def test_dense_gather_packs_each_block(which):
    """bt_ring_gather_dense_tpv3: each block's prefixes back to back from its first slot,
    16-B aligned, each holding the frame's first bytes (the walk's prefix), and the oracle
    gives the same records and decisions over them as over the ring."""
    import json
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    if which == "kernel_ring":
        g, bs, nb = _fixture()
        ring, used = g["ring"].copy(), nb
    else:
        cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4, "fuzz": synth.FUZZ}[which]
        data, desc = synth.capture(cfg, 6000, seed=12)
        bs = 1 << 16
        ring, _, used = synth.tpv3_ring(data, desc, block_size=bs)
    wdesc, taken = abi.ring_walk_tpv3(ring, bs, used)
    n = len(wdesc)
    slots = np.full(n * abi.PREFIX_SLOT, 0xA5, np.uint8)
    out, rout = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    gdesc, gtaken = abi.ring_gather_tpv3(ring, bs, used, slots, out, dense=True, ring_out=rout)
    assert gtaken == taken and len(gdesc) == n
    assert np.array_equal(rout, wdesc)   # the frames' own descriptors alongside
    lens = synth.desc_len(wdesc).astype(np.int64)
    assert np.array_equal(synth.desc_len(gdesc), synth.desc_len(wdesc))
    goff = synth.desc_off(gdesc).astype(np.int64)
    woff = synth.desc_off(wdesc).astype(np.int64)
    blk = woff // bs
    first = np.r_[True, blk[1:] != blk[:-1]]
    assert np.all(goff % 16 == 0)
    assert np.array_equal(goff[first], np.flatnonzero(first) * abi.PREFIX_SLOT)   # block k at j_k * slot
    step = np.diff(goff)[~first[1:]]
    assert np.all((step >= 0) & (step <= abi.PREFIX_SLOT) & (step % 16 == 0))
    # each prefix holds the frame's first bytes: up to the next prefix within the block
    nxt = np.r_[goff[1:], goff[-1] + abi.PREFIX_SLOT]
    room = np.where(np.r_[~first[1:], False], nxt - goff, abi.PREFIX_SLOT)
    for i in range(n):
        k = int(min(room[i], lens[i], 38))
        assert np.array_equal(slots[goff[i]:goff[i] + k], ring[woff[i]:woff[i] + k]), i
    _same_as_ring(ring, wdesc, slots, gdesc, man)


@pytest.mark.parametrize("which", ["kernel_ring", "c2", "c3", "c4", "fuzz"])
def test_lean_gather_packs_the_filter_bytes(which):
    """bt_ring_gather_lean_tpv3 (filter-only batches): 32 B per frame, each block's frames back
    to back after a 16-B pad at its first slot; frame i's descriptor points 12 B before its 32
    B, which hold the frame's bytes 12..43 (zeros past the frame); the oracle's decisions over
    them equal its decisions over the ring for the reference's filter sets."""
    import json
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    if which == "kernel_ring":
        g, bs, nb = _fixture()
        ring, used = g["ring"].copy(), nb
    else:
        cfg = {"c2": synth.C2, "c3": synth.C3, "c4": synth.C4, "fuzz": synth.FUZZ}[which]
        data, desc = synth.capture(cfg, 6000, seed=12)
        bs = 1 << 16
        ring, _, used = synth.tpv3_ring(data, desc, block_size=bs)
    wdesc, taken = abi.ring_walk_tpv3(ring, bs, used)
    n = len(wdesc)
    slots = np.full(n * abi.PREFIX_SLOT, 0xA5, np.uint8)
    out, rout = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    gdesc, gtaken = abi.ring_gather_tpv3(ring, bs, used, slots, out, lean=True, ring_out=rout)
    assert gtaken == taken and len(gdesc) == n and np.array_equal(rout, wdesc)
    assert np.array_equal(synth.desc_len(gdesc), synth.desc_len(wdesc))
    goff = synth.desc_off(gdesc).astype(np.int64) + 12   # where each frame's 32 B start
    woff = synth.desc_off(wdesc).astype(np.int64)
    lens = synth.desc_len(wdesc).astype(np.int64)
    blk = woff // bs
    first = np.r_[True, blk[1:] != blk[:-1]]
    assert np.array_equal(goff[first], np.flatnonzero(first) * abi.PREFIX_SLOT + 16)
    assert np.all(np.diff(goff)[~first[1:]] == 32)
    for i in range(n):
        want = np.zeros(32, np.uint8)
        k = int(max(0, min(lens[i] - 12, 32)))
        want[:k] = ring[woff[i] + 12:woff[i] + 12 + k]
        assert np.array_equal(slots[goff[i]:goff[i] + 32], want), i
    for s in ("c3", "mixed", "throw_after", "bpf_1", "port_range_1", "ip_range_1"):
        filters = man["filter_sets"][s]
        _, dw, _ = ol.oracle_run(ring, wdesc, n, filters, parse=False)
        _, dg, _ = ol.oracle_run(slots, gdesc, n, filters, parse=False)
        assert np.array_equal(dg, dw), s
