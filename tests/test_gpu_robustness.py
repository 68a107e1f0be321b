"""GPU: the C-ABI's bounds and ordering contract.

- a descriptor batch must state `bytes` (the readable size of base); a fixed-stride batch
  may not claim fewer than n * stride;
- descriptors whose frames run past `bytes` read zeros there, never past it (main kernel
  and the user-table extractor, whose fields past its 256-B window read memory directly);
- a download issued right after bt_parse_filter_device_async, without a synchronize, sees
  that call's pass list (the copies are ordered after the compaction stream);
- a PAYLOAD program recompiled while launches that read the previous DFA pool are queued
  on two different streams: every launch decides with the program it was launched with.
"""
import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth

pytestmark = pytest.mark.gpu

C3_SET = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
          {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
          {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]


def test_descriptor_batch_needs_bytes(gpu_ctx):
    data, desc = synth.capture(synth.C3, 1000, seed=3)
    gpu_ctx.compile(C3_SET)
    r = abi.DeviceRun(gpu_ctx, data, desc, 1000)
    try:
        r.batch.bytes = 0
        with pytest.raises(abi.BtError) as e:
            r.run()
        assert e.value.code == 1 and "bytes == 0" in str(e.value)
    finally:
        r.free()


def test_fixed_stride_bytes_too_small(gpu_ctx):
    data, _ = synth.capture(synth.C2, 1000, seed=3)
    gpu_ctx.compile(C3_SET)
    r = abi.DeviceRun(gpu_ctx, data, None, 1000, stride=64)
    try:
        r.batch.bytes = 64 * 1000 - 1
        with pytest.raises(abi.BtError) as e:
            r.run()
        assert e.value.code == 1
        r.batch.bytes = 0          # 0 = n * stride
        r.run()
        out = r.fetch()
        rec, dec, _ = ol.oracle_run(data, None, 1000, C3_SET, stride=64)
        assert np.array_equal(out["records"], rec) and np.array_equal(out["decide"], dec)
    finally:
        r.free()


def test_frames_past_bytes_read_zeros(gpu_ctx):
    """The last frames' descriptors claim bytes past the batch's `bytes`: those packets
    parse as if the bytes past it were zero; every other packet is unaffected."""
    n = 5000
    data, desc = synth.capture(synth.C4, n, seed=8)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    limit = int(off[n - 3]) + 20                   # cut inside frame n-3's Ethernet/VLAN headers
    d2 = synth.make_desc(off, np.where(np.arange(n) >= n - 3, 1500, ln))
    gpu_ctx.compile(C3_SET)
    r = abi.DeviceRun(gpu_ctx, data, d2, n)
    try:
        r.batch.bytes = limit
        r.run()
        out = r.fetch()
    finally:
        r.free()
    rec, dec, _ = ol.oracle_run(data, d2, n - 3, C3_SET)
    assert np.array_equal(out["records"][: n - 3], rec)
    assert np.array_equal(out["decide"][: n - 3], dec)


def test_extractor_far_field_past_bytes(gpu_ctx):
    """A table whose field lies past the 256-B staged window reads memory directly; a
    descriptor longer than the buffer gets zeros there, not bytes past `bytes`."""
    fields = [(0, 2, abi.FT_UINT16, 2), (600, 4, abi.FT_UINT32, 2)]
    buf = np.arange(4096, dtype=np.uint32).astype(np.uint8)
    desc = synth.make_desc([0, 1024, 2048], [1000, 1000, 3000])   # the last runs past 4096
    ex = abi.DeviceExtract(gpu_ctx, buf, desc, 3, fields)
    try:
        ex.batch.bytes = 2700
        ex.run()
        st, vals, _ = ex.fetch()
    finally:
        ex.free()
    assert list(st) == [0, 0, 0]
    exp = [int.from_bytes(bytes(buf[o + 600:o + 604]), "big") for o in (0, 1024)]
    assert list(vals[1][:2]) == exp
    # frame 2: bytes 2648..2651 are inside `bytes` (2700): read as they are
    assert vals[1][2] == int.from_bytes(bytes(buf[2648:2652]), "big")
    ex = abi.DeviceExtract(gpu_ctx, buf, desc, 3, fields)
    try:
        ex.batch.bytes = 2640          # a 16-B boundary before frame 2's field: it reads zeros
        ex.run()
        st, vals, _ = ex.fetch()
    finally:
        ex.free()
    assert list(st) == [0, 0, 0] and list(vals[1][:2]) == exp and vals[1][2] == 0


def test_download_after_async_without_synchronize(gpu_ctx):
    n = 300000
    data, desc = synth.capture(synth.C3, n, seed=12)
    gpu_ctx.compile(C3_SET)
    r = abi.DeviceRun(gpu_ctx, data, desc, n)
    try:
        gpu_ctx.run_device_async(r.batch, r.outs)
        # no synchronize: bt_memcpy_d2h is ordered after the compaction stream
        npass = int(r.d_npass.download(np.zeros(1, np.uint32))[0])
        pidx = r.d_pidx.download(np.zeros(max(npass, 1), np.uint32))[:npass]
    finally:
        gpu_ctx.synchronize()
        r.free()
    _, dec, exp_n = ol.oracle_run(data, desc, n, C3_SET, parse=False)
    assert npass == exp_n
    assert np.array_equal(pidx, np.nonzero((dec >> 6) == 0)[0].astype(np.uint32))


def test_context_device_identity(gpu_ctx):
    ordinal, bus = gpu_ctx.device_id()
    assert ordinal == gpu_ctx.device and len(bus) >= 7 and ":" in bus


def test_payload_recompile_with_launches_on_two_streams():
    """Launches reading DFA pool k on two caller streams, then two recompiles (the second
    writes pool k again): it must wait for both streams' launches, so each launch's
    decisions are those of the program it was launched with."""
    n = 1 << 20
    data, desc = synth.capture(synth.C3, n, seed=0x5EED)
    prog_a = [{"type": abi.PAYLOAD, "expr": "[A-Z][a-z]+", "priority": 2},
              {"type": abi.PROTOCOL, "expr": "tcp", "priority": 1}]
    prog_b = [{"type": abi.PAYLOAD, "expr": "HTTP", "priority": 2}]
    ctx = abi.Context(0)
    runs, streams = [], []
    try:
        prog = ctx.compile(prog_a)
        assert abi.KINDS[prog[0].kind] == "PAYLOAD"
        streams = [ctx.stream_create() for _ in range(2)]
        runs = [abi.DeviceRun(ctx, data, desc, n, records=False) for _ in range(2)]
        for r, s in zip(runs, streams):
            ctx.run_device(r.batch, r.outs, s)
        assert abi.KINDS[ctx.compile(prog_b)[0].kind] == "PAYLOAD"   # the other pool
        ctx.compile(prog_a)          # pool k again: waits for both streams' launches
        for s in streams:
            ctx.stream_synchronize(s)
        outs = [r.fetch() for r in runs]
    finally:
        for r in runs:
            r.free()
        for s in streams:
            ctx.stream_destroy(s)
        ctx.close()
    # the reference decisions: program A alone, one stream, no recompile (PAYLOAD slots are
    # the GPU DFA's; tests/test_gpu_payload.py pins those against the compiled reference)
    solo = abi.Context(0)
    try:
        solo.compile(prog_a)
        r = abi.DeviceRun(solo, data, desc, n, records=False)
        r.run()
        dec = r.fetch()["decide"]
        r.free()
    finally:
        solo.close()
    assert ((dec >> 6) == 0).any() and ((dec >> 6) == 1).any()
    for out in outs:
        assert np.array_equal(out["decide"], dec)
