"""GPU: host registration in whole pages (bt_host_register / bt_group_host_register over the
process's page table, beatrice_amd/csrc/bt_pin.h) and the mapped kernels reading what was
registered, deterministically, in the patterns round 5's one parity difference pointed at
(profiles/r05/tests/fuzz_mapped_difference.txt):

  * a small range at page P registered and unregistered, then a large range covering P
    registered over new contents, read by the mapped kernel;
  * two ranges that share a page: the second is refused, the first keeps working, and once the
    first is gone the second registers and reads right;
  * a context and a group registering the same UMEM share its pages; either one's release
    leaves the other reading right;
  * one arena registered and unregistered at the same addresses with other contents, sizes and
    offsets, round after round.
Every kernel result is compared with the oracle (tests/oracle_lib.py, pinned by the compiled
reference's goldens); outputs are poisoned (0xFF) before each call."""
import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth

pytestmark = pytest.mark.gpu
PAGE = abi.PAGE
PROG = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
        {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
        {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]


def pins():
    import ctypes
    buf = (ctypes.c_uint64 * (3 * 64))()
    n = ctypes.c_uint32(0)
    abi._check(abi.lib().bt_host_pins(buf, 64, ctypes.byref(n)))
    return [(buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(min(n.value, 64))]


def mapped_decide(grp, data, desc, n, dec, ver):
    """bt_group_parse_filter_mapped over buffers the caller registered; outputs poisoned first."""
    dec[:] = 0xFF
    ver[:] = 0xFFFFFFFFFFFFFFFF
    npass = np.zeros(1, np.uint32)
    grp.run_mapped(abi.Batch(data.ctypes.data, desc.ctypes.data, 0, n, data.nbytes, abi.DESC_PACKED, 0),
                   abi.Outputs(None, n, ver.ctypes.data, dec.ctypes.data, None, npass.ctypes.data))
    return dec[:n].copy(), int(npass[0])


def check(data, desc, n, got, npass, where):
    _, want, wpass = ol.oracle_run(data, desc, n, PROG, parse=False)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{where}: {len(bad)} decisions differ, first {bad[:8]}"
    assert npass == wpass, where


@pytest.fixture
def group1():
    g = abi.Group([0])
    g.compile(PROG)
    yield g
    g.close()


def test_page_table_rounds_shares_and_refuses():
    ctx = abi.Context(0)
    arena = abi.host_array(16 * PAGE)
    a0 = arena.ctypes.data
    try:
        before = pins()
        ctx.register(arena[100:5000])                    # pages 0-1
        assert [p for p in pins() if p not in before] == [(a0, a0 + 2 * PAGE, 1)]
        d_in = ctx.register(arena[200:300])              # inside them: shared
        assert [p for p in pins() if p not in before] == [(a0, a0 + 2 * PAGE, 2)]
        with pytest.raises(abi.BtError) as e:            # pages 1..2: only page 1 is held
            ctx.register(arena[6000:9000])
        assert e.value.code == 1 and "shares a page" in str(e.value)
        with pytest.raises(abi.BtError):                 # registered twice on one context
            ctx.register(arena[100:5000])
        ctx.register(arena[2 * PAGE:3 * PAGE])           # the next page alone: its own span
        assert len([p for p in pins() if p not in before]) == 2
        ctx.unregister(arena[100:5000])
        assert (a0, a0 + 2 * PAGE, 1) in pins()          # the shared range still holds them
        assert d_in
        ctx.unregister(arena[200:300])
        ctx.unregister(arena[2 * PAGE:3 * PAGE])
        assert [p for p in pins() if p not in before] == []
        with pytest.raises(abi.BtError):
            ctx.unregister(arena[200:300])
    finally:
        ctx.close()


def test_small_range_then_large_range_over_the_same_page(group1):
    """The verdict's pattern: register + unregister a small range at page P, write new
    contents, register a large range covering P, read it with the mapped kernel."""
    arena = abi.host_array(12 << 20)
    dec = abi.host_array(70000)
    ver = abi.host_array(1100, np.uint64)
    group1.register(dec)
    group1.register(ver)
    try:
        for k in range(6):
            data, desc = synth.capture(synth.C3, 20000 + 777 * k, seed=0x5000 + k)
            n = len(desc)
            off = 16 * (k % 4)                                    # the capture's start in the arena
            P = (9 + 5 * k) * PAGE                                # a page inside the capture
            small = arena[P + 48:P + 48 + 1000]
            group1.register(small)
            group1.unregister(small)
            view = arena[off:off + data.nbytes]
            view[:] = data
            d = abi.host_copy(desc)
            group1.register(view)
            group1.register(d)
            try:
                got, npass = mapped_decide(group1, view, d, n, dec, ver)
            finally:
                group1.unregister(d)
                group1.unregister(view)
            check(data, desc, n, got, npass, f"round {k}")
    finally:
        group1.unregister(ver)
        group1.unregister(dec)


def test_ranges_sharing_a_page(group1):
    """Two byte-disjoint ranges on one shared page: the second registration is refused while
    the first lives; the first reads right; once it is gone the second registers and reads
    right."""
    data, desc = synth.capture(synth.C3, 9000, seed=0x77)
    n = len(desc)
    cut = ((data.nbytes + PAGE) // PAGE) * PAGE + 1024           # mid-page
    arena = abi.host_array(2 * cut + PAGE)
    a, b = arena[:cut], arena[cut:2 * cut]
    a[:data.nbytes] = data
    b[:data.nbytes] = data
    d = abi.host_copy(desc)
    dec, ver = abi.host_array(9024), abi.host_array(141, np.uint64)
    for x in (d, dec, ver):
        group1.register(x)
    try:
        group1.register(a)
        with pytest.raises(abi.BtError) as e:
            group1.register(b)
        assert "shares a page" in str(e.value)
        got, npass = mapped_decide(group1, a[:data.nbytes], d, n, dec, ver)
        check(data, desc, n, got, npass, "first range")
        group1.unregister(a)
        group1.register(b)
        got, npass = mapped_decide(group1, b[:data.nbytes], d, n, dec, ver)
        check(data, desc, n, got, npass, "second range")
        group1.unregister(b)
    finally:
        for x in (ver, dec, d):
            group1.unregister(x)


def test_context_and_group_share_a_umem(group1):
    """One UMEM registered by a context (bt_host_register) and by a group: one lock, two
    references; each side reads right, before and after the other lets go."""
    ctx = abi.Context(0)
    ctx.compile(PROG)
    data, desc = synth.capture(synth.C3, 30000, seed=0x99)
    n = len(desc)
    umem, d = abi.host_copy(data), abi.host_copy(desc)
    dec, ver = abi.host_array(30016), abi.host_array(469, np.uint64)
    before = pins()
    try:
        alias = ctx.register(umem)
        d_alias = ctx.register(d)
        group1.register(umem)
        group1.register(d)
        for x in (dec, ver):
            group1.register(x)
        mine = [p for p in pins() if p not in before]
        assert any(p[2] == 2 for p in mine), mine                 # the UMEM's span: two references
        got, npass = mapped_decide(group1, umem, d, n, dec, ver)
        check(data, desc, n, got, npass, "group, both registered")
        group1.unregister(umem)
        group1.unregister(d)
        r = abi.DeviceRun(ctx, np.zeros(256, np.uint8), None, n, stride=1, records=False)
        r.batch = abi.Batch(alias, d_alias, 0, n, umem.nbytes, abi.DESC_PACKED, 0)
        r.run()
        out = r.fetch()
        r.free()
        check(data, desc, n, out["decide"], out["n_pass"], "context, after the group let go")
        ctx.unregister(d)
        ctx.unregister(umem)
        for x in (ver, dec):
            group1.unregister(x)
        assert [p for p in pins() if p not in before] == []
    finally:
        ctx.close()


def test_reused_addresses_round_after_round(group1):
    """One arena, the same start addresses registered and unregistered 24 times with other
    captures (C2 / C3 / C4 / fuzz), sizes and 16-B offsets; every round against the oracle."""
    rng = np.random.default_rng(0x5EED)
    arena = abi.host_array(48 << 20)
    for k in range(24):
        cfg = [synth.C2, synth.C3, synth.C4, synth.FUZZ][k % 4]
        n = int(rng.integers(1, 40000))
        data, desc = synth.capture(cfg, n, seed=int(rng.integers(1, 1 << 30)))
        if data.nbytes < 64:
            data = np.concatenate([data, np.zeros(64, np.uint8)])
        off = 16 * int(rng.integers(0, 256)) if k % 3 else 0
        view = arena[off:off + data.nbytes]
        view[:] = data
        d = abi.host_copy(desc)
        dec, ver = abi.host_array(max(n, 1) + 64), abi.host_array((n + 63) // 64 + 1, np.uint64)
        held = [view, d, dec, ver]
        for x in held:
            group1.register(x)
        try:
            got, npass = mapped_decide(group1, view, d, n, dec, ver)
        finally:
            for x in held:
                group1.unregister(x)
        check(data, desc, n, got, npass, f"round {k} cfg {cfg} n {n} off {off}")
