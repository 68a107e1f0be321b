"""GPU: TPACKET_V3 capture-ring ingest end to end.

The ring (a kernel-written image from tests/golden/ring_lo.npz, or a capture packed
into the kernel's layout) is registered with the device; bt_ring_walk_tpv3 turns its
ready blocks into descriptors and the parse+filter kernels read the frames in place,
writing records / decisions / verdicts into registered host memory. Checked against
the compiled reference's outputs (fixture) and the oracle (synthetic rings), and
through the C++ stage (tests/cpp/test_capture) against the reference PacketFilter."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from conftest import GOLDEN
from golden_util import compare_decisions

pytestmark = pytest.mark.gpu
CAPTURE_BIN = os.path.join(os.path.dirname(GOLDEN), "cpp", "test_capture")


def _run_ring(ctx, ring, bs, nb, filters, records=True):
    """Register -> walk -> device run with outputs in registered host memory."""
    ring = abi.host_copy(ring)   # on pages of its own, as the kernel maps a ring
    desc, taken = abi.ring_walk_tpv3(ring, bs, nb, ctx=ctx)
    assert taken == nb
    n = len(desc)
    tiles = (n + 63) // 64
    # every registered buffer on pages of its own (registration is in whole pages)
    desc = abi.host_copy(desc)
    h_rec = abi.host_array(tiles * 6144)
    h_dec = abi.host_array(tiles * 64)
    h_ver = abi.host_array(tiles, np.uint64)
    ctx.compile(filters)
    held = [ring, desc, h_dec, h_ver] + ([h_rec] if records else [])
    dev = [ctx.register(a) for a in held]
    try:
        batch = abi.Batch(dev[0], dev[1], 0, n, ring.nbytes, abi.DESC_PACKED, 0)
        outs = abi.Outputs(dev[4] if records else None, n, dev[3], dev[2], None, None)
        ctx.run_device(batch, outs)
        ctx.synchronize()
    finally:
        for a in held:
            ctx.unregister(a)
    rec = abi.untile_records(h_rec, n) if records else None
    return desc, rec, h_dec[:n], h_ver


def test_kernel_written_ring_matches_reference(gpu_ctx):
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    bs, nb = (int(x) for x in g["geometry"])
    for k, s in enumerate(man["rings"]["ring_lo"]["filter_sets"]):
        filters = man["filter_sets"][s]
        ring = g["ring"].copy()
        desc, rec, dec, ver = _run_ring(gpu_ctx, ring, bs, nb, filters, records=(k == 0))
        assert np.array_equal(desc, g["desc"])
        if rec is not None:
            bad = np.nonzero((rec != g["rec"]).any(axis=1))[0]
            assert len(bad) == 0, f"{len(bad)} records differ from the reference, first {bad[:5]}"
        compare_decisions(dec, g[f"code__{s}"], g[f"src__{s}"], filters, where=f"ring_lo/{s}")
        bits = np.unpackbits(ver.view(np.uint8), bitorder="little")[:len(dec)].astype(bool)
        assert np.array_equal(bits, (dec >> 6) == 0)


@pytest.mark.parametrize("cfg", [synth.C3, synth.C4, synth.FUZZ])
def test_packed_ring_1m_matches_oracle(gpu_ctx, cfg):
    n = 1 << 20
    data, desc0 = synth.capture(cfg, n, seed=21)
    ring, rdesc, used = synth.tpv3_ring(data, desc0)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    desc, rec, dec, ver = _run_ring(gpu_ctx, ring, synth.TPV3_BLOCK, used, filters)
    assert np.array_equal(desc, rdesc)
    orec, odec, _ = ol.oracle_run(ring, desc, len(desc), filters)
    assert np.array_equal(rec, orec)
    assert np.array_equal(dec, odec)


def test_cpp_stage_on_kernel_written_ring(tmp_path):
    assert os.path.exists(CAPTURE_BIN), "tests/cpp/test_capture not built (make -C tests/cpp)"
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    bs, nb = (int(x) for x in g["geometry"])
    img = tmp_path / "ring.bin"
    g["ring"].tofile(img)
    r = subprocess.run([CAPTURE_BIN, "stage", str(img), str(bs), str(nb)], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


def test_cpp_stage_synthetic_ring():
    assert os.path.exists(CAPTURE_BIN), "tests/cpp/test_capture not built (make -C tests/cpp)"
    r = subprocess.run([CAPTURE_BIN, "stage-synth"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


def test_cpp_stage_per_gpu_fanout_rings():
    """Per-GPU ring sharding: a capture split by flow into 2 and 3 TPACKET_V3 ring
    images, one GpuPacketFilter + GpuTpacketStage per ring, drained concurrently, each ring's
    decisions equal to the reference PacketFilter's and every frame seen once."""
    assert os.path.exists(CAPTURE_BIN), "tests/cpp/test_capture not built (make -C tests/cpp)"
    r = subprocess.run([CAPTURE_BIN, "stage-fanout"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


def _run_gathered(ctx, ring, bs, nb, filters, dense=False, lean=False):
    """bt_ring_gather_tpv3 (dense: bt_ring_gather_dense_tpv3; lean: bt_ring_gather_lean_tpv3,
    filter-only, BT_BATCH_LEAN, no records) -> device run over the prefix slots
    (BT_BATCH_PREFIXES), slots and outputs in registered host memory."""
    wdesc, _ = abi.ring_walk_tpv3(ring, bs, nb, ctx=ctx)
    n = len(wdesc)
    slots = abi.host_array(n * abi.PREFIX_SLOT)   # own pages: registered below
    slots.fill(0xA5)                               # poison past each prefix
    gd = abi.host_array(n, np.uint64)
    desc, taken = abi.ring_gather_tpv3(ring, bs, nb, slots, gd, ctx=ctx, dense=dense, lean=lean)
    assert taken == nb and len(desc) == n
    tiles = (n + 63) // 64
    h_rec = abi.host_array(tiles * 6144)
    h_dec = abi.host_array(tiles * 64)
    h_ver = abi.host_array(tiles, np.uint64)
    ctx.compile(filters)
    held = [slots, gd, h_dec, h_ver, h_rec]
    dev = [ctx.register(a) for a in held]
    try:
        batch = abi.Batch(dev[0], dev[1], 0, n, slots.nbytes, abi.DESC_PACKED,
                          abi.BATCH_PREFIXES | (abi.BATCH_LEAN if lean else 0))
        ctx.run_device(batch, abi.Outputs(None if lean else dev[4], n, dev[3], dev[2], None, None))
        ctx.synchronize()
    finally:
        for a in held:
            ctx.unregister(a)
    return wdesc, None if lean else abi.untile_records(h_rec, n), h_dec[:n]


def test_lean_gather_decides_as_the_reference(gpu_ctx):
    """bt_ring_gather_lean_tpv3 + BT_BATCH_LEAN: the kernels read frame bytes 12..43 only and
    decide as the reference on the kernel-written ring (every filter set without PAYLOAD) and
    as the oracle on 1M-frame C3 / C4 / fuzz rings; asking such a batch for records, or
    extracting a user table from it, is refused."""
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    bs, nb = (int(x) for x in g["geometry"])
    for s in man["rings"]["ring_lo"]["filter_sets"]:
        filters = man["filter_sets"][s]
        if any(f["type"] == abi.PAYLOAD for f in filters):
            continue
        desc, _, dec = _run_gathered(gpu_ctx, g["ring"].copy(), bs, nb, filters, lean=True)
        assert np.array_equal(desc, g["desc"])
        compare_decisions(dec, g[f"code__{s}"], g[f"src__{s}"], filters, where=f"ring_lo/{s} lean")
    for cfg in (synth.C3, synth.C4, synth.FUZZ):
        data, desc0 = synth.capture(cfg, 1 << 20, seed=29)
        ring, _, used = synth.tpv3_ring(data, desc0)
        desc, _, dec = _run_gathered(gpu_ctx, ring, synth.TPV3_BLOCK, used, C3_SET, lean=True)
        _, odec, _ = ol.oracle_run(ring, desc, len(desc), C3_SET, parse=False)
        assert np.array_equal(dec, odec), cfg
    buf = gpu_ctx.alloc(4096)
    batch = abi.Batch(buf.ptr, buf.ptr + 2048, 0, 1, 2048, abi.DESC_PACKED, abi.BATCH_PREFIXES | abi.BATCH_LEAN)
    with pytest.raises(abi.BtError):
        gpu_ctx.run_device(batch, abi.Outputs(buf.ptr + 3072, 1, None, None, None, None))


@pytest.mark.parametrize("dense", [False, True])
def test_gathered_prefixes_match_reference(gpu_ctx, dense):
    """Header prefixes gathered by the walker give the kernels the reference's records
    and decisions on the kernel-written ring; a PAYLOAD slot is left to the host."""
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    bs, nb = (int(x) for x in g["geometry"])
    for s in man["rings"]["ring_lo"]["filter_sets"]:
        filters = man["filter_sets"][s]
        if any(f["type"] == abi.PAYLOAD for f in filters):
            continue
        desc, rec, dec = _run_gathered(gpu_ctx, g["ring"].copy(), bs, nb, filters, dense)
        assert np.array_equal(desc, g["desc"])
        assert np.array_equal(rec, g["rec"])
        compare_decisions(dec, g[f"code__{s}"], g[f"src__{s}"], filters, where=f"ring_lo/{s} gathered")
    pay = [{"type": abi.PROTOCOL, "expr": "tcp", "priority": 3}, {"type": abi.PAYLOAD, "expr": "GET", "priority": 2}]
    _, _, dec = _run_gathered(gpu_ctx, g["ring"].copy(), bs, nb, pay, dense)
    _, _, dref, _ = _run_ring(gpu_ctx, g["ring"].copy(), bs, nb, pay, records=False)
    code, slot = dec >> 6, dec & 63
    reached = ((dref >> 6) != 1) | ((dref & 63) == 1)   # packets the PAYLOAD slot decides
    assert np.all(code[reached] == 3) and np.array_equal(dec[~reached], dref[~reached])


@pytest.mark.parametrize("dense", [False, True])
@pytest.mark.parametrize("cfg", [synth.C3, synth.C4, synth.FUZZ])
def test_gathered_prefixes_1m_match_oracle(gpu_ctx, cfg, dense):
    data, desc0 = synth.capture(cfg, 1 << 20, seed=23)
    ring, _, used = synth.tpv3_ring(data, desc0)
    desc, rec, dec = _run_gathered(gpu_ctx, ring, synth.TPV3_BLOCK, used, C3_SET, dense)
    orec, odec, _ = ol.oracle_run(ring, desc, len(desc), C3_SET)
    assert np.array_equal(rec, orec)
    assert np.array_equal(dec, odec)


C3_SET = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
          {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
          {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]


# ---- the frame chains walked on the GPU (bt_ring_walk_tpv3_gpu) -------------------------

def _gpu_walk(ctx, ring, bs, nb, first=0, max_blocks=None):
    """Registered ring -> GPU walk into device descriptors -> (descriptors, taken, bad)."""
    import struct as _s
    d_ring = ctx.register(ring)
    cap = int(ring.nbytes // 64) + 64
    d_desc = ctx.alloc(8 * cap)
    d_bad = ctx.alloc(16)
    try:
        d_bad.zero()
        n, taken = abi.ring_walk_tpv3_gpu(ctx, ring, d_ring, bs, nb, d_desc.ptr, cap, first=first,
                                          max_blocks=max_blocks, bad_dev=d_bad.ptr)
        ctx.synchronize()
        desc = d_desc.download(np.zeros(max(n, 1), np.uint64))[:n]
        bad = int(_s.unpack("<I", d_bad.download(np.zeros(4, np.uint8)).tobytes())[0])
    finally:
        d_desc.free()
        d_bad.free()
        ctx.unregister(ring)
    return desc, taken, bad


def test_gpu_walk_of_kernel_written_ring_matches_reference(gpu_ctx):
    """The kernel-written ring (994 frames in 4 blocks, real stack traffic + edge frames):
    the GPU-walked descriptors equal the fixture's, and parse + filter over them in device
    memory gives the reference's records and decisions."""
    g = np.load(os.path.join(GOLDEN, "ring_lo.npz"))
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    bs, nb = (int(x) for x in g["geometry"])
    ring = g["ring"].copy()
    desc, taken, bad = _gpu_walk(gpu_ctx, ring, bs, nb)
    assert taken == nb and bad == 0
    assert np.array_equal(desc, g["desc"])
    s = man["rings"]["ring_lo"]["filter_sets"][0]
    filters = man["filter_sets"][s]
    gpu_ctx.compile(filters)
    r = abi.DeviceRun(gpu_ctx, ring, desc, len(desc))
    try:
        r.run()
        out = r.fetch()
    finally:
        r.free()
    assert np.array_equal(out["records"], g["rec"])
    compare_decisions(out["decide"], g[f"code__{s}"], g[f"src__{s}"], filters, where="ring_lo gpu walk")


@pytest.mark.parametrize("cfg", [synth.C2, synth.C3, synth.C4, synth.FUZZ])
def test_gpu_walk_equals_host_walk(gpu_ctx, cfg):
    data, desc0 = synth.capture(cfg, 1 << 18, seed=33)
    ring, rdesc, used = synth.tpv3_ring(data, desc0, block_size=1 << 18)
    host, taken_h = abi.ring_walk_tpv3(ring, 1 << 18, used, ctx=gpu_ctx)
    dev, taken, bad = _gpu_walk(gpu_ctx, ring, 1 << 18, used)
    assert taken == taken_h == used and bad == 0
    assert np.array_equal(dev, host) and np.array_equal(dev, rdesc)
    # a window of blocks that wraps past the ring's end, stopping at a block the kernel owns
    rng = np.random.default_rng(cfg)
    first = int(rng.integers(1, used))
    ring2 = ring.copy()
    owned = (first + 3) % used
    ring2[owned * (1 << 18) + 8:owned * (1 << 18) + 12] = 0        # TP_STATUS_KERNEL
    host, th = abi.ring_walk_tpv3(ring2, 1 << 18, used, first=first, ctx=gpu_ctx)
    dev, td, bad = _gpu_walk(gpu_ctx, ring2, 1 << 18, used, first=first)
    assert th == td == 3 and bad == 0 and np.array_equal(dev, host)


def test_gpu_walk_reports_a_malformed_block(gpu_ctx):
    import struct as _s
    import ring_util as ru
    data, desc = synth.capture(synth.C2, 3000, seed=3)
    bs = 1 << 16
    ring, rdesc, used = synth.tpv3_ring(data, desc, block_size=bs)
    _, _, _, frames = next(ru.frame_headers(ring, bs, used))
    bad_ring = ring.copy()
    off = bs + frames[5][0]                                      # frame 5 of block 1 leaves the block
    bad_ring[off:off + 4] = np.frombuffer(_s.pack("<I", bs), np.uint8)
    dev, taken, bad = _gpu_walk(gpu_ctx, bad_ring, bs, used)
    assert taken == used and bad == 2                            # block 1, reported as block + 1
    host_ok, _ = abi.ring_walk_tpv3(ring, bs, used)
    n0 = int(np.frombuffer(ring[12:16].tobytes(), np.uint32)[0])                   # block 0's frames
    n1 = int(np.frombuffer(ring[bs + 12:bs + 16].tobytes(), np.uint32)[0])
    assert np.array_equal(dev[:n0 + 6], host_ok[:n0 + 6])        # up to and including frame 5
    assert not dev[n0 + 6:n0 + n1].any()                         # the rest of block 1: empty
    assert np.array_equal(dev[n0 + n1:], host_ok[n0 + n1:])      # later blocks unaffected


BUILTIN_C3 = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
              {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
              {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]


def _stage(ctx, ring, bs, used, n, **kw):
    """bt_ring_stage_tpv3 over a ring image with every buffer registered on pages of its own."""
    ring = abi.host_copy(ring)
    desc = abi.host_array(n + 64, np.uint64)
    dec = abi.host_array(n + 64)
    ver = abi.host_array((n + 127) // 64, np.uint64)
    slots = abi.host_array((n + 64) * abi.PREFIX_SLOT) if kw.get("gather") else None
    held = [a for a in (ring, desc, dec, ver, slots) if a is not None]
    for a in held:
        ctx.register(a)
    try:
        got, npass = abi.ring_stage_tpv3(ctx, ring, bs, used, desc, dec, ver, slots, **kw)
    finally:
        for a in held:
            ctx.unregister(a)
    return ring, got, npass, desc[:got].copy(), dec[:got].copy(), ver.copy()


@pytest.mark.parametrize("cfg", [synth.C2, synth.C3, synth.C4, synth.FUZZ])
@pytest.mark.parametrize("mode", ["in_place", "lean_mix", "lean_all", "lean_split", "adaptive"])
def test_ring_stage_decides_as_the_oracle(gpu_ctx, cfg, mode):
    """The one-call ring stage (walk of batch k+1 overlapping the kernels of batch k; in place,
    lean gather on every other batch, lean gather on all): every frame of a 200k-frame ring in
    ring order, decisions against the oracle on the frames, verdict words and pass count from
    them, batches of 7 blocks so that batches start mid-tile."""
    n = 200_000
    data, desc0 = synth.capture(cfg, n, seed=33)
    ring, rdesc, used = synth.tpv3_ring(data, desc0)
    gpu_ctx.compile(BUILTIN_C3)
    kw = {"in_place": {}, "lean_mix": dict(gather=True, in_place_every=2), "lean_all": dict(gather=True),
          "lean_split": dict(gather=True, in_place_blocks=3), "adaptive": dict(gather="adaptive")}[mode]
    ring, got, npass, desc, dec, ver = _stage(gpu_ctx, ring, synth.TPV3_BLOCK, used, n, batch_blocks=7, **kw)
    assert got == len(rdesc) == n
    _, odec, onp = ol.oracle_run(ring, rdesc, n, BUILTIN_C3, parse=False)
    bad = np.nonzero(dec != odec)[0]
    assert len(bad) == 0, f"{len(bad)} decisions differ, first {bad[:5]}"
    bits = np.unpackbits(ver.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, (odec >> 6) == 0) and npass == onp
    if mode == "in_place":
        assert np.array_equal(desc, rdesc)


def test_ring_stage_stops_at_a_kernel_owned_block(gpu_ctx):
    """A block still owned by the kernel (TP_STATUS_KERNEL) ends the run there: the frames of
    the blocks before it are decided, nothing after it is read."""
    import ring_util as ru
    n = 20_000
    data, desc0 = synth.capture(synth.C3, n, seed=5)
    ring, rdesc, used = synth.tpv3_ring(data, desc0)
    stop = used // 2
    at = stop * synth.TPV3_BLOCK + ru.BLOCK_STATUS
    ring[at:at + 4] = np.frombuffer(np.uint32(ru.TP_STATUS_KERNEL).tobytes(), np.uint8)
    gpu_ctx.compile(BUILTIN_C3)
    ring, got, npass, desc, dec, ver = _stage(gpu_ctx, ring, synth.TPV3_BLOCK, used, n, batch_blocks=3)
    expect = len(abi.ring_walk_tpv3(ring, synth.TPV3_BLOCK, used, max_blocks=stop)[0])
    assert 0 < got == expect < n
    _, odec, _ = ol.oracle_run(ring, rdesc[:got], got, BUILTIN_C3, parse=False)
    assert np.array_equal(dec, odec)


def test_ring_stage_refuses_unregistered_buffers(gpu_ctx):
    n = 1000
    data, desc0 = synth.capture(synth.C2, n, seed=1)
    ring, _, used = synth.tpv3_ring(data, desc0)
    ring = abi.host_copy(ring)
    desc, dec = abi.host_array(n, np.uint64), abi.host_array(n)
    gpu_ctx.compile(BUILTIN_C3)
    with pytest.raises(abi.BtError, match="registered"):
        abi.ring_stage_tpv3(gpu_ctx, ring, synth.TPV3_BLOCK, used, desc, dec)
