"""Deterministic synthetic captures (ctypes over libbt_synth.so, csrc/bt_synth.cpp).

A capture is (data: uint8 ndarray, desc: uint64 ndarray of bt_pkt_desc). The configs
are the BASELINE.json ones: 2 = C1/C2 fixed 64 B Eth/IPv4/UDP,
3 = C3 IMIX, 4 = C4 QinQ/IPv6/options, 9 = fuzz.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

C2, C3, C4, FUZZ = 2, 3, 4, 9
SEEDS = {C2: 0x5EED0002, C3: 0x5EED0003, C4: 0x5EED0004, FUZZ: 0x5EED0009}

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libbt_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (make -C beatrice_amd/csrc)")
        L = ctypes.CDLL(path)
        L.bt_synth_layout.restype = ctypes.c_uint64
        L.bt_synth_layout.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.bt_synth_fill.restype = ctypes.c_int
        L.bt_synth_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int]
        L.bt_synth_fill_range.restype = ctypes.c_int
        L.bt_synth_fill_range.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_int]
        L.bt_synth_tpv3_pack.restype = ctypes.c_uint64
        L.bt_synth_tpv3_pack.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def capture(cfg: int, n: int, seed: int | None = None, threads: int | None = None):
    """Returns (data, desc) for n frames of config cfg."""
    if seed is None:
        seed = SEEDS[cfg]
    L = lib()
    desc = np.empty(n, dtype=np.uint64)
    nbytes = L.bt_synth_layout(cfg, n, seed, desc.ctypes.data)
    data = np.zeros(int(nbytes), dtype=np.uint8)
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    L.bt_synth_fill(cfg, n, seed, desc.ctypes.data, data.ctypes.data, threads)
    return data, desc


RNG_BLOCK = 65536   # frames per RNG block of bt_synth.cpp (fill ranges start on one)


def layout(cfg: int, n: int, seed: int | None = None):
    """(desc, data bytes) of a capture without filling it."""
    if seed is None:
        seed = SEEDS[cfg]
    desc = np.empty(n, dtype=np.uint64)
    nbytes = lib().bt_synth_layout(cfg, n, seed, desc.ctypes.data)
    return desc, int(nbytes)


FILL_PAD = 128   # zero bytes fill_range leaves after the last frame (over-reads of header math)


def fill_range(cfg: int, seed: int, desc: np.ndarray, lo: int, hi: int, threads: int | None = None):
    """Frames [lo, hi) of a capture (lo a multiple of RNG_BLOCK), identical to the same
    frames of capture(cfg, len(desc), seed). Returns (buf, b0, nbytes): frame i sits at
    buf[offset_i - b0], the frames span buf[:nbytes], and FILL_PAD zero bytes follow."""
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    off = desc_off(desc)
    b0 = int(off[lo]) if hi > lo else 0
    b1 = int(off[hi - 1] + desc_len(desc[hi - 1:hi])[0]) if hi > lo else 0
    buf = np.zeros(b1 - b0 + FILL_PAD, dtype=np.uint8)
    rc = lib().bt_synth_fill_range(cfg, len(desc), seed, desc.ctypes.data, lo, hi, buf.ctypes.data, b0, threads)
    if rc:
        raise ValueError(f"bt_synth_fill_range({lo}, {hi}) = {rc}")
    return buf, b0, b1 - b0


def desc_off(desc: np.ndarray) -> np.ndarray:
    return (desc & np.uint64(0xFFFFFFFFFFFF)).astype(np.int64)


def desc_len(desc: np.ndarray) -> np.ndarray:
    return (desc >> np.uint64(48)).astype(np.int64)


def make_desc(off, length) -> np.ndarray:
    off = np.asarray(off, dtype=np.uint64)
    length = np.asarray(length, dtype=np.uint64)
    return off | (length << np.uint64(48))


def pack_frames(frames, align: int = 1, shift: int = 0):
    """Packs a list of bytes objects into (data, desc); frame i starts at an offset
    that is `shift` past a multiple of `align`."""
    offs, lens, pos = [], [], 0
    for f in frames:
        pos = (pos + align - 1) // align * align + shift
        offs.append(pos)
        lens.append(len(f))
        pos += len(f)
    data = np.zeros((pos + 255) // 256 * 256 + 256, dtype=np.uint8)
    for o, f in zip(offs, frames):
        data[o:o + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    return data, make_desc(offs, lens)


TPV3_BLOCK = 1 << 20   # 1 MiB blocks: ~6.9k 64-B frames or ~680 1500-B frames per block


def tpv3_ring(data: np.ndarray, desc: np.ndarray, block_size: int = TPV3_BLOCK, n_blocks: int | None = None):
    """Packs a capture into a TPACKET_V3 RX-ring image laid out exactly as the kernel
    writes one (bt_synth_tpv3_pack). Returns (ring uint8, ring_desc uint64, blocks used);
    ring_desc[i] = BT_DESC(ring offset, snaplen) of packed frame i. With n_blocks None
    the ring is sized to hold every frame; otherwise packing stops when it is full."""
    L = lib()
    n = len(desc)
    if n_blocks is None:
        used = ctypes.c_uint64()
        L.bt_synth_tpv3_pack(data.ctypes.data, desc.ctypes.data, n, block_size, None, 1 << 40, None,
                             ctypes.byref(used))
        n_blocks = max(1, used.value)
    ring = np.zeros(n_blocks * block_size, dtype=np.uint8)
    ring_desc = np.empty(max(n, 1), dtype=np.uint64)
    used = ctypes.c_uint64()
    k = L.bt_synth_tpv3_pack(data.ctypes.data, desc.ctypes.data, n, block_size, ring.ctypes.data, n_blocks,
                             ring_desc.ctypes.data, ctypes.byref(used))
    return ring, ring_desc[:k], int(used.value)
