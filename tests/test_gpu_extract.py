"""GPU: user-defined protocol extraction (bt_extract_tile, beatrice_amd/csrc/bt_extract.hip)
through the C-ABI — the drop-in for ProtocolParser::parsePacket(packet, ProtocolDefinition)
— against the compiled reference's goldens (tests/golden/extract.*: parser_example's KAT
and seeded random tables) and the C restatement on large seeded batches."""
import json
import os

import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "extract.json")) as _fh:
    MAN = json.load(_fh)
G = dict(np.load(os.path.join(GOLDEN, "extract.npz"), allow_pickle=False))


def run(ctx, data, desc, n, fields, stride=0, desc_format=abi.DESC_PACKED):
    r = abi.DeviceExtract(ctx, data, desc, n, fields, stride=stride, desc_format=desc_format)
    r.run()
    out = r.fetch()
    r.free()
    return out


def check_against_golden(name, st, val, img):
    t = MAN["tables"][name]
    n = MAN["n"]
    assert np.array_equal(st, G[f"status__{name}"]), f"{name}: status"
    assert np.array_equal(val, G[f"values__{name}"]), f"{name}: values"
    fb = ol.field_bytes_of_image(img, t) if img is not None else np.zeros((n, 0), np.uint8)
    assert np.array_equal(fb, G[f"fb__{name}"]), f"{name}: field bytes"


@pytest.mark.parametrize("name", list(MAN["tables"]))
def test_device_matches_reference(gpu_ctx, name):
    st, val, img = run(gpu_ctx, G["data"], G["desc"], MAN["n"], MAN["tables"][name])
    check_against_golden(name, st, val, img)


@pytest.mark.parametrize("name", ["parser_example", "rand_3", "rand_7", "empty"])
def test_host_list_matches_reference(gpu_ctx, name):
    off, ln = synth.desc_off(G["desc"]), synth.desc_len(G["desc"])
    frames = [G["data"][o:o + l].tobytes() for o, l in zip(off, ln)]
    st, val, img = gpu_ctx.extract_host(frames, MAN["tables"][name])
    check_against_golden(name, st, val, img if img.shape[1] else None)


def test_parser_example_known_answer(gpu_ctx):
    """examples/parser_example.cpp:18-43: the 17-byte CUSTOM_PROTO packet."""
    pkt = np.frombuffer(bytes([0x12, 0x34, 0x56, 0x78, 1, 0, 10, 0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF, 0x11, 0x22,
                               0x33, 0x44]), np.uint8)
    st, val, img = run(gpu_ctx, pkt, synth.make_desc([0], [17]), 1, MAN["tables"]["parser_example"])
    assert st[0] == 0 and int(val[0, 0]) == 0x12345678 and int(val[1, 0]) == 1 and int(val[2, 0]) == 10
    assert bytes(img[0, 7:17]).hex() == "aabbccddeeff11223344"
    # one byte short of getTotalLength(): PACKET_TOO_SHORT, no field
    st, val, img = run(gpu_ctx, pkt, synth.make_desc([0], [16]), 1, MAN["tables"]["parser_example"])
    assert st[0] == 9 and not val.any() and not img.any()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_seeded_tables_match_oracle(gpu_ctx, seed):
    """200k frames at 2-mod-4 offsets (ragged, n not a multiple of 64), random tables
    including fields past the 256-byte staged window."""
    rng = np.random.default_rng(seed)
    n = 200003
    data, desc = synth.capture(synth.FUZZ, n, seed=seed)
    for k in range(6):
        nf = int(rng.integers(1, 12))
        t = [(int(rng.integers(0, 300 if k % 2 else 60)), int(rng.integers(0, 12)), int(rng.integers(0, 18)),
              int(rng.integers(0, 4))) for _ in range(nf)]
        t = [(o, max(ln, 1) if ty == abi.FT_BOOLEAN else ln, ty, e) for o, ln, ty, e in t]
        st, val, img = run(gpu_ctx, data, desc, n, t)
        ost, oval, oimg, span = ol.oracle_extract(data, desc, n, t)
        assert np.array_equal(st, ost) and np.array_equal(val, oval), f"table {t}"
        assert np.array_equal(img, oimg), f"table {t}: image"


@pytest.mark.parametrize("mode", ["fixed", "xdp"])
def test_descriptor_forms(gpu_ctx, mode):
    n = 70001
    data, desc = synth.capture(synth.C2, n)
    t = [(0, 6, abi.FT_MAC, 2), (12, 2, abi.FT_UINT16, 2), (26, 4, abi.FT_IPV4, 2), (34, 2, abi.FT_UINT16, 0),
         (23, 1, abi.FT_INT8, 1), (30, 8, abi.FT_FLOAT64, 0), (36, 4, abi.FT_FLOAT32, 3)]
    ost, oval, oimg, _ = ol.oracle_extract(data, desc, n, t)
    if mode == "fixed":
        st, val, img = run(gpu_ctx, data, None, n, t, stride=64)
    else:
        xdp = np.zeros((n, 2), np.uint64)
        xdp[:, 0] = synth.desc_off(desc).astype(np.uint64)
        xdp[:, 1] = synth.desc_len(desc).astype(np.uint64)
        st, val, img = run(gpu_ctx, data, xdp, n, t, desc_format=abi.DESC_XDP)
    assert np.array_equal(st, ost) and np.array_equal(val, oval) and np.array_equal(img, oimg)


def test_edges(gpu_ctx):
    data, desc = synth.capture(synth.FUZZ, 1000, seed=9)
    # n = 0 and n = 1
    st, val, img = run(gpu_ctx, data, desc[:0], 0, [(0, 2, abi.FT_UINT16, 2)])
    assert len(st) == 0
    st, val, img = run(gpu_ctx, data, desc[:1], 1, [(0, 2, abi.FT_UINT16, 2)])
    ost, oval, _, _ = ol.oracle_extract(data, desc[:1], 1, [(0, 2, abi.FT_UINT16, 2)])
    assert np.array_equal(st, ost) and np.array_equal(val, oval)
    # a table no frame can reach (span > 65535): every packet PACKET_TOO_SHORT
    st, val, img = run(gpu_ctx, data, desc, 1000, [(70000, 4, abi.FT_UINT32, 2)])
    assert (st == 9).all() and not val.any() and img is None
    # the empty table: every packet SUCCESS with no field
    st, val, img = run(gpu_ctx, data, desc, 1000, [])
    assert (st == 0).all()
    with pytest.raises(abi.BtError):
        run(gpu_ctx, data, desc, 1000, [(0, 0, abi.FT_BOOLEAN, 0)])
    with pytest.raises(abi.BtError):
        run(gpu_ctx, data, desc, 1000, [(0, 1, abi.FT_UINT8, 0)] * 65)


def test_timed_extraction_matches_reference(gpu_ctx):
    """bt_time_extract_ex (bench.py's c1 entry): K timed launches leave the reference's
    outputs, and every launch has a positive, consistent event-pair duration."""
    name = "parser_example"
    r = abi.DeviceExtract(gpu_ctx, G["data"], G["desc"], MAN["n"], MAN["tables"][name])
    try:
        t = r.time(5)
        assert t.main_ms > 0 and 0 < t.main_min_ms <= t.main_ms <= t.main_max_ms <= t.span_ms
        check_against_golden(name, *r.fetch())
    finally:
        r.free()
    empty = abi.DeviceExtract(gpu_ctx, G["data"], G["desc"], 0, MAN["tables"][name])
    try:
        with pytest.raises(abi.BtError):
            empty.time(2)
    finally:
        empty.free()


def test_extract_over_a_parse_batch(gpu_ctx):
    """DeviceExtract over packets already on the device (a DeviceRun's batch, as the bench
    uses it): same results as the oracle, and the DeviceRun keeps its buffer."""
    n = 5000
    data, desc = synth.capture(synth.C2, n)
    fields = MAN["tables"]["parser_example"]
    run_ = abi.DeviceRun(gpu_ctx, data, None, n, stride=64, records=False, decide=False, verdict=False,
                         pass_idx=False)
    try:
        ex = abi.DeviceExtract(gpu_ctx, None, None, n, fields, batch=run_.batch)
        ex.run()
        st, val, img = ex.fetch()
        ex.free()
        est, evl, eimg, _ = ol.oracle_extract(data, None, n, fields, stride=64)
        assert np.array_equal(st, est) and np.array_equal(val, evl) and np.array_equal(img, eimg)
    finally:
        run_.free()
