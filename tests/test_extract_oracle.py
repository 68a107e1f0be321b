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
