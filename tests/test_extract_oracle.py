"""CPU: the C restatement of user-defined protocol extraction (oracle/bt_oracle.c
bto_extract) against the compiled reference's ProtocolParser::parsePacket(frame,
ProtocolDefinition) goldens (tests/golden/make_extract_golden.py), including the
reference's only known-answer test, examples/parser_example.cpp:18-43."""
import json
import os

import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi
from conftest import GOLDEN

with open(os.path.join(GOLDEN, "extract.json")) as _fh:
    MAN = json.load(_fh)
G = dict(np.load(os.path.join(GOLDEN, "extract.npz"), allow_pickle=False))


def test_parser_example_known_answer():
    # examples/parser_example.cpp:56-79 / README.md:1097-1126: header 0x12345678, version 1,
    # length 10, data aabbccddeeff11223344 — frame 0 of the fixture is that packet
    t = MAN["tables"]["parser_example"]
    st, val, img, span = ol.oracle_extract(G["data"], G["desc"][:1], 1, t)
    assert span == 17 and st[0] == 0
    assert int(val[0, 0]) == 0x12345678 and int(val[1, 0]) == 1 and int(val[2, 0]) == 10
    assert bytes(img[0, 7:17]).hex() == "aabbccddeeff11223344"
    assert G["status__parser_example"][0] == 0 and int(G["values__parser_example"][0, 0]) == 0x12345678
    assert bytes(G["fb__parser_example"][0, 7:17]).hex() == "aabbccddeeff11223344"


@pytest.mark.parametrize("name", list(MAN["tables"]))
def test_oracle_matches_reference(name):
    t = MAN["tables"][name]
    n = MAN["n"]
    st, val, img, span = ol.oracle_extract(G["data"], G["desc"], n, t)
    assert np.array_equal(st, G[f"status__{name}"]), name
    assert np.array_equal(val, G[f"values__{name}"]), name
    fb = ol.field_bytes_of_image(img, t) if span else np.zeros((n, 0), np.uint8)
    assert np.array_equal(fb, G[f"fb__{name}"]), name


def test_span_is_get_total_length():
    # getTotalLength (src/parser/FieldDefinition.cpp:31-46): the largest field end
    for t in MAN["tables"].values():
        want = max((o + ln for o, ln, _, _ in t), default=0)
        assert abi.proto_span(t) == want
    with pytest.raises(abi.BtError):   # BOOLEAN of length 0: the reference reads fieldData[0] of an empty vector
        abi.proto_span([(0, 0, abi.FT_BOOLEAN, 0)])
    assert abi.proto_span([(70000, 4, abi.FT_UINT32, 2)]) == 70004


@pytest.mark.parametrize("name", list(MAN["tables"]))
def test_host_extractor_matches_reference(name):
    """bt_extract_host (the product's small-batch path for GpuProtocolParser::parsePacket, no
    device) against the compiled reference's goldens: status, extractValue<T> bits and the
    field bytes of every frame."""
    import ctypes
    t = MAN["tables"][name]
    n = MAN["n"]
    data, desc = G["data"], G["desc"][:n]
    off, ln = (desc & np.uint64(0xFFFFFFFFFFFF)).astype(np.int64), (desc >> np.uint64(48)).astype(np.int64)
    bufs = [np.ascontiguousarray(data[o:o + l]) if l else np.zeros(1, np.uint8) for o, l in zip(off, ln)]
    ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    lens = ln.astype(np.uint32)
    arr, nf = abi.field_table(t)
    span = abi.proto_span(t)
    span = span if span <= 0xFFFF else 0
    st = np.zeros(n, np.uint8)
    val = np.zeros(max(1, nf * n), np.uint64)
    img = np.zeros(max(1, n * span), np.uint8)
    lib = abi.lib()
    rc = lib.bt_extract_host(ptrs, lens.ctypes.data, n, arr, nf, st.ctypes.data,
                             val.ctypes.data if nf else None, img.ctypes.data if span else None)
    assert rc == 0
    assert np.array_equal(st, G[f"status__{name}"]), name
    assert np.array_equal(val[:nf * n].reshape(nf, n), G[f"values__{name}"]), name
    fb = ol.field_bytes_of_image(img[:n * span].reshape(n, span), t) if span else np.zeros((n, 0), np.uint8)
    assert np.array_equal(fb, G[f"fb__{name}"]), name
