"""TPACKET_V3 ring helpers for the tests (test infrastructure, not product code).

`walk_tpv3` is a plain-Python restatement of the block walk that
beatrice_amd/csrc/bt_ring.cpp performs, written from the Linux uapi layout
(linux/if_packet.h: tpacket_block_desc / tpacket_hdr_v1 / tpacket3_hdr). It is the
checker for bt_ring_walk_tpv3 on the kernel-written fixture (tests/golden/ring_lo.npz).
"""
from __future__ import annotations

import struct

import numpy as np

TP_STATUS_KERNEL = 0
TP_STATUS_USER = 1
BLOCK_STATUS = 8          # offsetof(tpacket_block_desc, hdr.bh1.block_status)
BLOCK_NUM_PKTS = 12
BLOCK_FIRST = 16
FRAME_HDR = struct.Struct("<IIIIIIHH")   # next_offset sec nsec snaplen len status mac net


def walk_tpv3(ring: np.ndarray, block_size: int, n_blocks: int, first: int = 0, max_blocks: int | None = None,
              cap: int = 1 << 62):
    """Returns (descs as uint64 BT_DESC(offset, min(snaplen, 65535)), blocks taken)."""
    buf = memoryview(ring.view(np.uint8)).cast("B")
    out = []
    taken = 0
    lim = n_blocks if max_blocks is None else min(max_blocks, n_blocks)
    for k in range(lim):
        b = (first + k) % n_blocks
        base = b * block_size
        status, npk, off = struct.unpack_from("<III", buf, base + BLOCK_STATUS)
        if not status & TP_STATUS_USER or len(out) + npk > cap:
            break
        for j in range(npk):
            nxt, _, _, snap, _, _, mac, _ = FRAME_HDR.unpack_from(buf, base + off)
            out.append(((min(snap, 0xFFFF)) << 48) | (base + off + mac))
            off += nxt
        taken += 1
    return np.array(out, dtype=np.uint64), taken


def frame_headers(ring: np.ndarray, block_size: int, n_blocks: int):
    """Yields (block, num_pkts, offset_to_first, [(off, next, snaplen, len, mac), ...]) per ready block."""
    buf = memoryview(ring.view(np.uint8)).cast("B")
    for b in range(n_blocks):
        base = b * block_size
        status, npk, first = struct.unpack_from("<III", buf, base + BLOCK_STATUS)
        if not status & TP_STATUS_USER:
            continue
        frames, off = [], first
        for _ in range(npk):
            nxt, _, _, snap, ln, _, mac, _ = FRAME_HDR.unpack_from(buf, base + off)
            frames.append((off, nxt, snap, ln, mac))
            off += nxt
        yield b, npk, first, frames


def layout_violations(ring: np.ndarray, block_size: int, n_blocks: int):
    """The kernel's V3 layout rules (net/packet/af_packet.c with tp_reserve 0 and no
    block private area) that bt_synth_tpv3_pack reproduces; returns the broken ones."""
    bad = []
    buf = ring.tobytes()
    for b, npk, first, frames in frame_headers(ring, block_size, n_blocks):
        ver, o2p = struct.unpack_from("<II", buf, b * block_size)
        blk_len = struct.unpack_from("<I", buf, b * block_size + 20)[0]
        if ver != 2 or o2p != 48 or first != 48:
            bad.append((b, "block header", ver, o2p, first))
        for j, (off, nxt, snap, ln, mac) in enumerate(frames):
            want = 0 if j == npk - 1 else (mac + snap + 7) & ~7
            if mac != 82 or nxt != want or snap > ln:
                bad.append((b, j, off, nxt, snap, ln, mac))
        if frames:
            off, _, snap, _, mac = frames[-1]
            if blk_len != off + ((mac + snap + 7) & ~7):
                bad.append((b, "blk_len", blk_len))
    return bad


def umem_capture(frames_data, desc, chunk=2048, shuffle_seed=5):
    """An AF_XDP-style UMEM (anonymous mmap, numBuffers x bufferSize chunks, headroom 0,
    reference src/AF_XDPBackend.cpp:683-720) holding each frame at the start of a chunk,
    plus the RX ring's xdp_desc {addr, len, options} (shuffled chunk order, as after
    fill-ring recycling)."""
    import mmap

    from beatrice_amd import synth
    n = len(desc)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    assert ln.max() <= chunk
    mm = mmap.mmap(-1, n * chunk)
    umem = np.frombuffer(mm, dtype=np.uint8)
    order = np.random.default_rng(shuffle_seed).permutation(n)
    for i in range(n):
        c = order[i] * chunk
        umem[c:c + ln[i]] = frames_data[off[i]:off[i] + ln[i]]
    xdp = np.zeros((n, 2), np.uint64)
    xdp[:, 0] = order.astype(np.uint64) * chunk
    xdp[:, 1] = ln.astype(np.uint64)               # len in the low 32 bits, options = 0
    packed = synth.make_desc(order.astype(np.uint64) * chunk, ln)
    return mm, umem, xdp, packed
