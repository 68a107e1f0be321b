"""NUMA placement of host capture memory (Linux, host only).

A capture backend that feeds a device allocates its ring / UMEM on the device's NUMA node
(INTEGRATION.md §4): the context pins its gather threads there, and a zero-copy read crosses
the device's own PCIe root. These helpers do the same for a numpy capture in the bench and
the tools: an anonymous mapping whose pages are bound (mbind(2), MPOL_BIND, before the first
touch) to one node, or to one node per byte range — a device group's members each read their
own range of one batch (bt_group_parse_filter_mapped), so each range goes on its member's node.
"""
from __future__ import annotations

import ctypes
import mmap

import numpy as np

_SYS_MBIND = 237        # x86-64
_SYS_MOVE_PAGES = 279
_MPOL_BIND = 2
_PAGE = 4096


def _mbind(addr: int, size: int, node: int) -> None:
    mask = (ctypes.c_ulong * 16)()
    mask[node // 64] |= 1 << (node % 64)
    libc = ctypes.CDLL(None, use_errno=True)
    if libc.syscall(_SYS_MBIND, ctypes.c_void_p(addr), ctypes.c_ulong(size), _MPOL_BIND, mask,
                    ctypes.c_ulong(16 * 64 + 1), 0) != 0:
        raise OSError(ctypes.get_errno(), "mbind")


def place_ranges(arr: np.ndarray, ranges: list[tuple[int, int, int]], hugepages: bool = False) -> np.ndarray:
    """A copy of `arr` whose byte range [lo, hi) of each (lo, hi, node) lies on NUMA node
    `node` (ranges rounded to pages; bytes no range covers follow the default policy). A node
    < 0 leaves its range unbound. Returns `arr` itself when no range names a node. With
    `hugepages` the mapping asks for transparent huge pages (madvise, before the first touch);
    off by default: same box, alternating, host-gather and zero-copy rates were level within
    their spread either way (profiles/r05/e2e/ab_hugepages.jsonl)."""
    if not any(node >= 0 for _, _, node in ranges):
        return arr
    size = (arr.nbytes + _PAGE - 1) & ~(_PAGE - 1)
    m = mmap.mmap(-1, max(size, _PAGE))
    if hugepages and hasattr(mmap, "MADV_HUGEPAGE"):
        try:
            m.madvise(mmap.MADV_HUGEPAGE)
        except OSError:
            pass   # THP off or unsupported: 4-KiB pages
    anchor = ctypes.c_char.from_buffer(m)
    addr = ctypes.addressof(anchor)
    for lo, hi, node in ranges:
        if node < 0:
            continue
        a = lo & ~(_PAGE - 1)
        b = min(size, (hi + _PAGE - 1) & ~(_PAGE - 1))
        if b > a:
            _mbind(addr + a, b - a, node)
    del anchor   # the ctypes view's export of the mapping ends here
    out = np.frombuffer(m, dtype=arr.dtype, count=arr.size)   # holds the mapping: freed with the array
    np.copyto(out, arr)
    return out


def place_on(arr: np.ndarray, node: int | None, hugepages: bool = False) -> np.ndarray:
    """A copy of `arr` on NUMA node `node` (None / < 0: `arr` itself)."""
    if node is None or node < 0:
        return arr
    return place_ranges(arr, [(0, arr.nbytes, node)], hugepages)


def page_nodes(arr: np.ndarray, samples: int = 8) -> list[int]:
    """NUMA nodes of a few of the array's pages (move_pages(2) query; -1 unknown, [] if the
    query itself fails)."""
    libc = ctypes.CDLL(None, use_errno=True)
    base, nb = arr.ctypes.data, arr.nbytes
    pages = (ctypes.c_void_p * samples)(*[(base + nb * i // samples) & ~(_PAGE - 1) for i in range(samples)])
    status = (ctypes.c_int * samples)()
    if libc.syscall(_SYS_MOVE_PAGES, 0, ctypes.c_ulong(samples), pages, None, status, 0) != 0:
        return []
    return sorted(set(int(x) for x in status))


def member_byte_ranges(off: np.ndarray, ln: np.ndarray, bounds: list[tuple[int, int]]) -> list[tuple[int, int]]:
    """Byte range [first frame's start, last frame's end) of each member's packet range."""
    out = []
    for lo, hi in bounds:
        if hi <= lo:
            out.append((0, 0))
        else:
            out.append((int(off[lo]), int(off[hi - 1]) + int(ln[hi - 1])))
    return out
