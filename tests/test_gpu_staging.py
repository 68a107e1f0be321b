"""GPU: the host batch calls' prefix contract (bt_host_stage_bytes, include/beatrice_gpu.h).

bt_parse_filter_ptrs reads min(len, W) bytes from each frame pointer, W as
bt_host_stage_bytes reports it for the current program: 48 for filter-only calls, 112 with
records, 176 with a GPU PAYLOAD slot. A caller may therefore hand over, instead of the
frames, copies of their first W bytes packed back to back (as the plugin does with
BEATRICE_GPU_PACK=1) with the frames' true lengths. Records and decisions must then equal
the reference fixtures bit for bit."""
import ctypes

import numpy as np
import pytest

from beatrice_amd import abi
from conftest import load_golden
from golden_util import compare_decisions

pytestmark = pytest.mark.gpu


def _stage_bytes(ctx, with_records):
    b = ctypes.c_uint32(0)
    assert abi.lib().bt_host_stage_bytes(ctx.h, int(with_records), ctypes.byref(b)) == 0
    return b.value


def _packed(data, desc, w):
    """Each frame's first min(len, w) bytes at i * w of one buffer (the rest of its slot
    poisoned: no byte past the prefix may matter), plus the true lengths."""
    off, ln = desc & ((1 << 48) - 1), (desc >> 48).astype(np.uint32)
    n = len(desc)
    buf = np.full(n * w + 16, 0xA5, np.uint8)
    for i in range(n):
        m = min(int(ln[i]), w)
        buf[i * w:i * w + m] = data[int(off[i]):int(off[i]) + m]
    return buf, ln


def _run_ptrs(ctx, buf, w, lens, records):
    n = len(lens)
    ptrs = (ctypes.c_void_p * n)(*[buf.ctypes.data + i * w for i in range(n)])
    rec = np.zeros((n, abi.BT_REC_BYTES), np.uint8) if records else None
    dec = np.zeros(n, np.uint8)
    ver = np.zeros((n + 63) // 64, np.uint64)
    p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    rc = abi.lib().bt_parse_filter_ptrs(ctx.h, ptrs, lens.ctypes.data, n, p(rec), p(ver), p(dec), None, None)
    assert rc == 0, abi.lib().bt_last_error()
    return rec, dec


@pytest.mark.parametrize("cap", ["c3", "c4", "fuzz", "edge"])
def test_packed_prefixes_equal_the_frames(cap):
    g, man = load_golden(cap)
    filters = man["filter_sets"]["c3"]
    ctx = abi.Context(0, host_chunk_packets=4096)
    try:
        ctx.compile(filters)
        w_filter, w_rec = _stage_bytes(ctx, False), _stage_bytes(ctx, True)
        assert (w_filter, w_rec) == (48, 112)
        buf, lens = _packed(g["data"], g["desc"], w_filter)
        _, dec = _run_ptrs(ctx, buf, w_filter, lens, records=False)
        compare_decisions(dec, g["code__c3"], g["src__c3"], filters, where=f"packed48/{cap}")
        buf, lens = _packed(g["data"], g["desc"], w_rec)
        rec, dec2 = _run_ptrs(ctx, buf, w_rec, lens, records=True)
        assert np.array_equal(rec, g["rec"]), f"{cap}: records from 112-B prefixes differ from the reference"
        assert np.array_equal(dec2, dec)
    finally:
        ctx.close()


def test_stage_bytes_follow_the_program():
    ctx = abi.Context(0)
    try:
        ctx.compile([{"type": abi.PROTOCOL, "expr": "tcp", "priority": 2},
                     {"type": abi.PAYLOAD, "expr": "GET|POST", "priority": 1}])   # a GPU DFA slot
        assert _stage_bytes(ctx, False) == 176 and _stage_bytes(ctx, True) == 176
        ctx.compile([{"type": abi.PROTOCOL, "expr": "tcp", "priority": 2}])
        assert (_stage_bytes(ctx, False), _stage_bytes(ctx, True)) == (48, 112)
    finally:
        ctx.close()


@pytest.mark.parametrize("cap", ["c3", "c4", "fuzz", "edge"])
def test_lean_staging_equals_full_prefixes(cap):
    """Filter-only host batches stage bytes 12..43 of each frame (their descriptors point 12 B
    before the staged bytes; frames of <= 12 B stage nothing). Decisions, verdicts and the pass
    list equal the reference fixture and the 48-B staging kept for A/B (BT_OPT_NO_LEAN_HOST),
    over every frame length the fixtures hold (the edge capture truncates every layer)."""
    g, man = load_golden(cap)
    filters = man["filter_sets"]["c3"]
    lean, full = abi.Context(0, host_chunk_packets=4096), abi.Context(0, host_chunk_packets=4096,
                                                                      flags=abi.OPT_NO_LEAN_HOST)
    try:
        outs = []
        for ctx in (lean, full):
            ctx.compile(filters)
            outs.append(ctx.run_host(g["data"], g["desc"], records=False))
        compare_decisions(outs[0]["decide"], g["code__c3"], g["src__c3"], filters, where=f"lean/{cap}")
        for k in ("decide", "verdict", "pass_idx"):
            assert np.array_equal(outs[0][k], outs[1][k]), f"{cap}: {k} differs between lean and 48-B staging"
        lens = (g["desc"] >> 48).astype(np.int64)
        assert (lens <= 12).any() or cap != "edge", "the edge capture should hold frames of <= 12 B"
    finally:
        lean.close()
        full.close()


@pytest.mark.parametrize("cap", ["c3", "c4", "edge"])
@pytest.mark.parametrize("records", [False, True])
def test_registered_outputs_are_written_in_place(cap, records):
    """Host batch outputs inside a range registered with bt_host_register are copied D2H in
    place (no staging drain); the results equal the reference fixture and the staged form, also
    with several chunks (host_chunk_packets 1024) and with only some outputs registered."""
    g, man = load_golden(cap)
    filters = man["filter_sets"]["c3"]
    n = len(g["desc"])
    ctx = abi.Context(0, host_chunk_packets=1024)
    try:
        ctx.compile(filters)
        want = ctx.run_host(g["data"], g["desc"], records=records)
        def own_pages(a):   # each array on pages of its own (registrations may not share a page)
            import mmap
            m = mmap.mmap(-1, (a.nbytes + 4095) // 4096 * 4096 or 4096)
            return np.frombuffer(m, a.dtype, count=a.size).reshape(a.shape)

        for which in (("records", "decide", "verdict"), ("decide",), ("verdict",)):
            outs = {k: None if v is None else own_pages(v) for k, v in abi.host_outputs(n, records=records).items()}
            regs = [outs[k] for k in which if outs.get(k) is not None]
            for a in regs:
                ctx.register(a)
            try:
                got = ctx.run_host(g["data"], g["desc"], records=records, outs=outs)
            finally:
                for a in regs:
                    ctx.unregister(a)
            compare_decisions(got["decide"], g["code__c3"], g["src__c3"], filters, where=f"registered {which}/{cap}")
            for k in ("decide", "verdict", "pass_idx"):
                assert np.array_equal(got[k], want[k]), f"{cap} {which}: {k} differs from the staged form"
            if records:
                assert np.array_equal(got["records"], want["records"]), f"{cap} {which}: records differ"
    finally:
        ctx.close()
