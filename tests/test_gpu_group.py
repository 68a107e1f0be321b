"""GPU: the in-process multi-device group (bt_group_*).

On the 1-GPU box the members share device 0 (BT_OPT_GROUP_SHARED_DEVICE); every member
still has its own context, streams, pinned staging and host threads, runs its range of the
batch concurrently with the others, and writes into the caller's arrays at its offset. The
merged outputs must equal the reference fixtures and the single-context run bit for bit."""
import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from conftest import load_golden
from golden_util import compare_decisions

pytestmark = pytest.mark.gpu


def _group(m, **kw):
    return abi.Group([0] * m, flags=abi.OPT_GROUP_SHARED_DEVICE | kw.pop("flags", 0), **kw)


@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("cap", ["c3", "c4", "edge"])
def test_group_matches_reference_fixture(cap, members):
    g, man = load_golden(cap)
    filters = man["filter_sets"]["c3"]
    grp = _group(members, host_chunk_packets=1024)
    try:
        grp.compile(filters)
        out = grp.run_host(g["data"], g["desc"])
    finally:
        grp.close()
    n = len(g["desc"])
    assert np.array_equal(out["records"], g["rec"])
    compare_decisions(out["decide"], g["code__c3"], g["src__c3"], filters, where=f"group{members}/{cap}")
    bits = np.unpackbits(out["verdict"].view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, (out["decide"] >> 6) == 0)
    assert np.array_equal(out["pass_idx"], np.nonzero(bits)[0].astype(np.uint32)) and out["n_pass"] == bits.sum()


def test_group_ptrs_equals_single_context_and_oracle():
    n = 200003
    data, desc = synth.capture(synth.C3, n, seed=0x6A)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    frames = [data[o:o + l].tobytes() for o, l in zip(off, ln)]
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1},
               {"type": abi.PAYLOAD, "expr": "[0-9]{2}", "priority": 0}]
    grp = _group(4)
    try:
        grp.compile(filters)           # compiled once (the PAYLOAD DFA too), installed on all four
        out = grp.run_ptrs(frames)
        out_nf = grp.run_ptrs(frames, filters=False)
    finally:
        grp.close()
    ctx = abi.Context(0)
    try:
        ctx.compile(filters)
        one = ctx.run_host(data, desc)
    finally:
        ctx.close()
    for k in ("records", "verdict", "decide", "pass_idx"):
        assert np.array_equal(out[k], one[k]), k
    assert out["n_pass"] == one["n_pass"]
    assert np.array_equal(out_nf["records"], one["records"])
    rec, _, _ = ol.oracle_run(data, desc, n)
    assert np.array_equal(out["records"], rec)


def test_group_edge_sizes_and_errors():
    grp = _group(3)
    try:
        grp.compile([{"type": abi.PROTOCOL, "expr": "tcp"}])
        for n in (0, 1, 64, 65, 129):     # fewer tiles than members: empty ranges
            data, desc = synth.capture(synth.FUZZ, max(n, 1), seed=n)
            desc = desc[:n]
            out = grp.run_host(data, np.ascontiguousarray(desc))
            rec, dec, npass = ol.oracle_run(data, desc, n, [{"type": abi.PROTOCOL, "expr": "tcp"}])
            assert np.array_equal(out["records"], rec) and np.array_equal(out["decide"], dec)
            assert out["n_pass"] == npass
        with pytest.raises(abi.BtError):   # a throwing program is still a compile error only
            grp.compile([{"type": abi.BPF, "expr": "udp", "priority": i} for i in range(65)])
    finally:
        grp.close()
    with pytest.raises(abi.BtError) as e:
        abi.Group([0, 0])                  # a device twice without the test flag
    assert "listed twice" in str(e.value)


# ---- zero-copy over the group (bt_group_host_register + bt_group_parse_filter_mapped) --------

C3_SET = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
          {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
          {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]


def _ptr(a):
    return None if a is None else a.ctypes.data


def _run_mapped(grp, base, desc, n, fmt=abi.DESC_PACKED, stride=0, records=True, verdict=True, pass_list=True,
                nbytes=None):
    """Registers the batch and the device-written outputs with the group, runs the mapped call,
    unregisters. Returns the outputs (records still in the tiled device layout)."""
    tiles = max(1, (n + 63) // 64)
    # every registered buffer on pages of its own (registration is in whole pages)
    base = abi.host_copy(base)
    desc = None if desc is None else abi.host_copy(desc)
    h_rec = abi.host_array(tiles * 6144) if records else None
    h_dec = abi.host_array(tiles * 64)
    h_ver = abi.host_array(tiles, np.uint64) if verdict else None
    pidx = np.full(max(n, 1), 0xFFFFFFFF, np.uint32)
    npass = np.zeros(1, np.uint32)
    held = [a for a in (base, desc, h_rec, h_dec, h_ver) if a is not None]
    for a in held:
        grp.register(a)
    try:
        batch = abi.Batch(_ptr(base), _ptr(desc), stride, n, base.nbytes if nbytes is None else nbytes, fmt, 0)
        outs = abi.Outputs(_ptr(h_rec), n, _ptr(h_ver), _ptr(h_dec), _ptr(pidx) if pass_list else None,
                           npass.ctypes.data)
        grp.run_mapped(batch, outs)
    finally:
        for a in held:
            grp.unregister(a)
    return {"rec_tiled": h_rec, "records": abi.untile_records(h_rec, n) if records else None,
            "decide": h_dec[:n], "verdict": h_ver, "pass_idx": pidx[:int(npass[0])] if pass_list else pidx[:0],
            "n_pass": int(npass[0])}


def _single_zero_copy(ctx, base, desc, n, fmt, filters):
    """The same batch through one context's bt_parse_filter_device (round 3's zero-copy path)."""
    ctx.compile(filters)
    tiles = max(1, (n + 63) // 64)
    h_rec = abi.host_array(tiles * 6144)
    h_dec = abi.host_array(tiles * 64)
    h_ver = abi.host_array(tiles, np.uint64)
    held = [abi.host_copy(base), abi.host_copy(desc), h_rec, h_dec, h_ver]
    base = held[0]
    dev = [ctx.register(a) for a in held]
    try:
        ctx.run_device(abi.Batch(dev[0], dev[1], 0, n, base.nbytes, fmt, 0),
                       abi.Outputs(dev[2], n, dev[4], dev[3], None, None))
        ctx.synchronize()
    finally:
        for a in held:
            ctx.unregister(a)
    return h_rec, h_dec[:n], h_ver


def _check_filter(out, dec, n):
    assert np.array_equal(out["decide"], dec)
    bits = (dec >> 6) == 0
    if out["verdict"] is not None:
        vb = np.unpackbits(out["verdict"].view(np.uint8), bitorder="little")
        assert np.array_equal(vb[:n].astype(bool), bits) and not vb[n:].any()
    exp = np.nonzero(bits)[0].astype(np.uint32)
    assert out["n_pass"] == len(exp)
    assert np.array_equal(out["pass_idx"], exp)


@pytest.mark.parametrize("members", [1, 2, 3])
def test_group_mapped_umem_xdp_equals_oracle_and_single_context(members):
    """SURVEY §8(f) rank 1 over several devices: an AF_XDP UMEM and its xdp_desc RX ring
    registered once with the group; each member reads its range of the ring in place."""
    from ring_util import umem_capture
    n = 40000
    data, desc = synth.capture(synth.C3, n, seed=0x51)
    mm, umem, xdp, packed = umem_capture(data, desc)
    grp = _group(members)
    try:
        grp.compile(C3_SET)
        out = _run_mapped(grp, umem, xdp, n, fmt=abi.DESC_XDP)
        nov = _run_mapped(grp, umem, xdp, n, fmt=abi.DESC_XDP, records=False, verdict=False)  # scratch verdict
        nop = _run_mapped(grp, umem, xdp, n, fmt=abi.DESC_XDP, records=False, pass_list=False)
    finally:
        grp.close()
    rec, dec, npass = ol.oracle_run(umem, packed, n, C3_SET)
    assert np.array_equal(out["records"], rec)
    _check_filter(out, dec, n)
    _check_filter(nov, dec, n)
    assert np.array_equal(nop["decide"], dec) and nop["n_pass"] == npass and not nop["pass_idx"].size
    ctx = abi.Context(0)
    try:
        s_rec, s_dec, s_ver = _single_zero_copy(ctx, umem, xdp, n, abi.DESC_XDP, C3_SET)
    finally:
        ctx.close()
    assert np.array_equal(out["rec_tiled"], s_rec), "tiled record bytes differ from the single-context run"
    assert np.array_equal(out["decide"], s_dec) and np.array_equal(out["verdict"], s_ver)
    del umem
    mm.close()


@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("cap", ["c4", "edge", "http"])
def test_group_mapped_fixture_matches_reference(cap, members):
    """The reference fixtures read in place by 2 / 3 members: records + decisions against the
    compiled reference, with a GPU PAYLOAD slot on the http capture."""
    g, man = load_golden(cap)
    sets = ["c3"] + (["payload_re_0", "payload_chain"] if cap == "http" else [])
    data, desc = np.ascontiguousarray(g["data"]), np.ascontiguousarray(g["desc"], dtype=np.uint64)
    n = len(desc)
    for s in sets:
        filters = man["filter_sets"][s]
        grp = _group(members)
        try:
            grp.compile(filters)
            out = _run_mapped(grp, data, desc, n)
        finally:
            grp.close()
        assert np.array_equal(out["records"], g["rec"])
        compare_decisions(out["decide"], g[f"code__{s}"], g[f"src__{s}"], filters, where=f"mapped{members}/{cap}/{s}")


@pytest.mark.parametrize("members", [2, 3])
def test_group_mapped_kernel_written_ring(members):
    """The kernel-written TPACKET_V3 ring (tests/golden/ring_lo.npz) registered with the group and
    walked into ring-relative descriptors: each member reads its frames in place."""
    import json
    import os
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    bs, nb = (int(x) for x in z["geometry"])
    ring = z["ring"].copy()
    desc, taken = abi.ring_walk_tpv3(ring, bs, nb)
    assert taken == nb and np.array_equal(desc, z["desc"])
    n = len(desc)
    for k, s in enumerate(man["rings"]["ring_lo"]["filter_sets"]):
        filters = man["filter_sets"][s]
        grp = _group(members)
        try:
            grp.compile(filters)
            out = _run_mapped(grp, ring, desc, n, records=(k == 0))
        finally:
            grp.close()
        if k == 0:
            assert np.array_equal(out["records"], z["rec"])
        compare_decisions(out["decide"], z[f"code__{s}"], z[f"src__{s}"], filters, where=f"ring_lo/mapped{members}/{s}")
        bits = np.unpackbits(out["verdict"].view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(bits, (out["decide"] >> 6) == 0)


def test_group_mapped_fixed_stride_and_edges():
    """Fixed-stride 64-B frames (C2) split evenly by tiles, n not a tile multiple, fewer tiles
    than members, n = 0."""
    grp = _group(3)
    try:
        grp.compile(C3_SET)
        for n in (0, 1, 65, 129, 100003):
            buf, desc = synth.capture(synth.C2, max(n, 1), seed=n + 1)
            assert np.array_equal(synth.desc_off(desc), np.arange(max(n, 1)) * 64)
            buf = np.ascontiguousarray(buf[:max(n, 1) * 64])
            out = _run_mapped(grp, buf, None, n, stride=64)
            if n == 0:
                assert out["n_pass"] == 0
                continue
            rec, dec, _ = ol.oracle_run(buf, desc[:n], n, C3_SET)
            assert np.array_equal(out["records"], rec), n
            _check_filter(out, dec, n)
        # a stated size below n * stride is refused before the split (a member past it would
        # otherwise get an underflowed bound and read past the registered range)
        buf, _ = synth.capture(synth.C2, 1000, seed=9)
        buf = np.ascontiguousarray(buf[:1000 * 64])
        for nbytes in (64, 999 * 64 + 63):
            with pytest.raises(abi.BtError) as e:
                _run_mapped(grp, buf, None, 1000, stride=64, nbytes=nbytes)
            assert "bytes" in str(e.value) and "n * stride" in str(e.value)
    finally:
        grp.close()


def test_group_mapped_refuses_unregistered_and_bad_layouts():
    grp = _group(2)
    data, desc = synth.capture(synth.C3, 1000, seed=3)
    data, desc = abi.host_copy(data), abi.host_copy(desc)
    try:
        grp.compile(C3_SET)
        dec = abi.host_array(1024)
        grp.register(data)
        grp.register(dec)
        with pytest.raises(abi.BtError) as e:    # descriptors not registered
            grp.run_mapped(abi.Batch(data.ctypes.data, desc.ctypes.data, 0, 1000, data.nbytes, 0, 0),
                           abi.Outputs(None, 0, None, dec.ctypes.data, None, None))
        assert "not inside a group-registered range" in str(e.value)
        with pytest.raises(abi.BtError):         # overlapping registration
            grp.register(data[16:])
        grp.unregister(dec)
        grp.unregister(data)
        with pytest.raises(abi.BtError):         # not registered any more
            grp.unregister(data)
    finally:
        grp.close()
    pl = _group(2, flags=abi.OPT_RECORDS_PLANES)
    try:
        pl.compile(C3_SET)
        with pytest.raises(abi.BtError) as e:
            _run_mapped(pl, data, desc, 1000)
        assert "plane-major" in str(e.value)
    finally:
        pl.close()


def test_group_placement_and_budget():
    """Every member reports its NUMA placement; the group's host threads are one budget."""
    grp = _group(4)
    try:
        per = abi.group_thread_budget(4, abi.usable_cpus())
        for k in range(4):
            p = grp.placement(k)
            assert p["pool_threads"] == per
            if p["pinned_cpus"]:
                assert p["numa_node"] >= 0 and p["pinned_cpus"] == len(abi.node_cpus(p["numa_node"]))
        assert grp.cost(True, False, True, 16) == (48, 16, 17)
        assert grp.cost(False, True, True, 8) == (112, 16, 105)
        assert grp.cost(False, False, True, 8) == (32, 16, 9)   # filter-only host batches stage bytes 12..43
    finally:
        grp.close()


def test_group_host_parallel_covers_every_member_thread():
    """bt_group_host_parallel: each worker index of the group's whole budget runs once."""
    import ctypes
    grp = _group(3, host_threads=12)
    try:
        seen = []
        total = []
        cb_t = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32)

        def cb(_u, w, T):
            seen.append(w)
            total.append(T)
        f = cb_t(cb)
        assert abi.lib().bt_group_host_parallel(grp.h, ctypes.cast(f, ctypes.c_void_p), None) == 0
        assert len(set(total)) == 1 and total[0] == 3 * abi.group_thread_budget(3, abi.usable_cpus(), 12)
        assert sorted(seen) == list(range(total[0]))
    finally:
        grp.close()


@pytest.mark.parametrize("members", [1, 2])
def test_group_mapped_sparse_frames_gathered_on_host(members, monkeypatch):
    """BT_OPT_MAPPED_GATHER_SPARSE: filter-only mapped batches whose frames lie far apart (C4,
    ~870 B) take each member's host gather, dense ones (C2) stay in place; the outputs are
    the same either way. BT_MAPPED_GATHER_ABOVE is read once per process, so the test uses the
    default threshold (512 B)."""
    for cfg, n in ((synth.C4, 30011), (synth.C2, 20000)):
        data, desc = synth.capture(cfg, n, seed=0x33)
        grp = _group(members, flags=abi.OPT_MAPPED_GATHER_SPARSE)
        try:
            grp.compile(C3_SET)
            out = _run_mapped(grp, data, desc, n, records=False)
            nov = _run_mapped(grp, data, desc, n, records=False, verdict=False)
        finally:
            grp.close()
        _, dec, _ = ol.oracle_run(data, desc, n, C3_SET)
        _check_filter(out, dec, n)
        _check_filter(nov, dec, n)


@pytest.mark.parametrize("members", [1, 2])
def test_group_mapped_sparse_gather_keeps_the_bytes_bound(members):
    """A frame that runs past batch.bytes: the host gather would read it at base + off
    directly, so the member whose range holds it stays on the kernels (which clamp reads at
    `bytes`); the outputs equal the same batch without the option."""
    n = 30011
    data, desc = synth.capture(synth.C4, n, seed=0x34)
    last = int(synth.desc_off(desc)[-1])
    nbytes = last + 20   # the last frame's window crosses the end of the batch
    outs = []
    for flags in (abi.OPT_MAPPED_GATHER_SPARSE, 0):
        grp = _group(members, flags=flags)
        try:
            grp.compile(C3_SET)
            outs.append(_run_mapped(grp, data, desc, n, records=False, nbytes=nbytes))
        finally:
            grp.close()
    a, b = outs
    assert np.array_equal(a["decide"], b["decide"]) and np.array_equal(a["verdict"], b["verdict"])
    assert np.array_equal(a["pass_idx"], b["pass_idx"])
    _, dec, _ = ol.oracle_run(data, desc, n - 1, C3_SET)   # every frame inside the bytes: the oracle's
    assert np.array_equal(a["decide"][:n - 1], dec)


def test_group_concurrent_callers_routed_whole():
    """Host batches from several threads at once: a call that finds another in flight runs
    whole on the least busy member (a device listed twice = two lanes on it) instead of being
    split; every caller's outputs still equal the oracle's."""
    import threading
    caps = [synth.capture(synth.C3, 20000 + 640 * k, seed=0x70 + k) for k in range(6)]
    exp = [ol.oracle_run(d, q, len(q), C3_SET) for d, q in caps]
    grp = _group(2)
    errors = []
    try:
        grp.compile(C3_SET)

        def caller(k):
            try:
                d, q = caps[k]
                for _ in range(4):
                    out = grp.run_host(d, q, records=(k % 2 == 0))
                    rec, dec, npass = exp[k]
                    assert np.array_equal(out["decide"], dec) and out["n_pass"] == npass
                    if k % 2 == 0:
                        assert np.array_equal(out["records"], rec)
            except Exception as e:   # reported from the main thread
                errors.append((k, repr(e)))
        th = [threading.Thread(target=caller, args=(k,)) for k in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th), "a caller hung"
    finally:
        grp.close()
    assert not errors, errors
