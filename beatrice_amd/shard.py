"""Batch sharding across GPUs: packets are independent units, so a
batch splits into contiguous packet ranges — one per rank/GPU — with no collective on
the data path. Bounds are multiples of 64 packets (one wavefront tile) so per-shard
verdict words concatenate without bit shifts, and are balanced by cumulative header
bytes (min(len, 128) + descriptor) so IMIX shards cost the same on each device.

The only cross-rank result is host-side: sum of pass counts, concatenated verdict
words / decision bytes, pass indices offset by the shard start.
"""
from __future__ import annotations

import numpy as np

TILE = 64


# The per-packet cost model: round_up(min(len, window), align) + fixed bytes. The default is
# the device-resident strong-scaling case (header window + descriptor + 96-B record in HBM);
# the in-process group weighs each call by what it moves (bt_group_cost, mirrored by
# group_cost below).
DEFAULT_COST = (128, 1, 8 + 96)


def packet_cost(lengths, cost=DEFAULT_COST) -> np.ndarray:
    window, align, fixed = cost
    w = np.minimum(np.asarray(lengths, dtype=np.int64), window)
    if align > 1:
        w = (w + align - 1) // align * align
    return w + fixed


def group_cost(mapped: bool, records: bool, filters: bool, desc_bytes: int = 8, stage_bytes: int | None = None):
    """bt_group_cost (include/beatrice_gpu.h): what one packet costs a group member.
    Host batches stage round_up(min(len, stage_bytes), 16) bytes (the bytes the host pipeline
    copies: 32 filter-only, frame bytes 12..43; 112 with records; 176 with a GPU PAYLOAD slot),
    copy its descriptor up and its 96-B bt_rec and decision byte back; mapped batches read the
    header window over the member's PCIe link (the lean 48 B filter-only, the walk's 128 with
    records) and write packed record slabs (~64 B) and the decision."""
    if mapped:
        return (128 if records else 48, 16, desc_bytes + (64 if records else 0) + (1 if filters else 0))
    if stage_bytes is None:
        stage_bytes = 112 if records else 32
    return (stage_bytes, 16, desc_bytes + (96 if records else 0) + (1 if filters else 0))


def member_threads(members: int, usable: int, requested: int = 0) -> int:
    """bt_group_thread_budget: host threads per group member. `requested` is the whole
    group's budget (split evenly, 1..16 each); auto gives usable / members, 1..16 each (a
    member's host pipeline takes at most 8 of them while other callers wait for it)."""
    usable = max(usable, 1)
    if requested:
        return min(max(requested // members, 1), 16)
    return min(max(usable // members, 1), 16)


def shard_bounds(lengths: np.ndarray, world: int, by_bytes: bool = True, cost=DEFAULT_COST):
    """Contiguous [lo, hi) packet ranges, one per rank, tile-aligned."""
    n = len(lengths)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    ntiles = (n + TILE - 1) // TILE
    if by_bytes:
        cost = packet_cost(lengths, cost)
        tile_cost = np.add.reduceat(cost, np.arange(0, n, TILE))
        cum = np.cumsum(tile_cost)
        targets = cum[-1] * np.arange(1, world) / world
        cuts = np.searchsorted(cum, targets, side="left") + 1
    else:
        cuts = (np.arange(1, world) * ntiles) // world
    cuts = np.clip(cuts, 0, ntiles)
    edges = [0] + [int(c) * TILE for c in cuts] + [n]
    edges = [min(e, n) for e in edges]
    for i in range(1, len(edges)):
        edges[i] = max(edges[i], edges[i - 1])
    return [(edges[i], edges[i + 1]) for i in range(world)]


def local_batch(data: np.ndarray, desc: np.ndarray, lo: int, hi: int):
    """The shard's own bytes and descriptors rebased to them (what one GPU receives)."""
    d = desc[lo:hi]
    if len(d) == 0:
        return np.zeros(256, np.uint8), d.copy()
    off = (d & np.uint64(0xFFFFFFFFFFFF)).astype(np.int64)
    ln = (d >> np.uint64(48)).astype(np.int64)
    base = int(off.min()) & ~15          # keep 16-B alignment of every window
    end = int((off + ln).max())
    local = np.ascontiguousarray(data[base:end + 16])
    rebased = (off - base).astype(np.uint64) | (ln.astype(np.uint64) << np.uint64(48))
    return local, rebased


def merge(parts, bounds, n: int):
    """parts[r]: dict with decide (n_r,), verdict (ceil(n_r/64),), pass_idx, n_pass
    (and optionally records (n_r, 96)) from rank r; returns the whole-batch result."""
    out = {"decide": np.zeros(n, np.uint8), "verdict": np.zeros((n + 63) // 64, np.uint64)}
    has_rec = all("records" in p for p in parts)
    if has_rec:
        out["records"] = np.zeros((n, 96), np.uint8)
    idx, npass = [], 0
    for p, (lo, hi) in zip(parts, bounds):
        m = hi - lo
        if m == 0:
            continue
        assert lo % TILE == 0
        out["decide"][lo:hi] = p["decide"][:m]
        nw = (m + 63) // 64
        out["verdict"][lo // 64: lo // 64 + nw] = p["verdict"][:nw]
        idx.append(np.asarray(p["pass_idx"], np.uint64) + lo)
        npass += int(p["n_pass"])
        if has_rec:
            out["records"][lo:hi] = p["records"][:m]
    out["pass_idx"] = np.concatenate(idx).astype(np.uint32) if idx else np.zeros(0, np.uint32)
    out["n_pass"] = npass
    return out
