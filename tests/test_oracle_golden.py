"""CPU: the plain-C oracle (oracle/bt_oracle.c) against the golden fixtures generated
from the compiled reference (tests/golden/make_golden.py). This pins the oracle
before any GPU result is compared with it."""
import numpy as np
import pytest

import oracle_lib as ol
from conftest import load_golden
from golden_util import CAPTURES, compare_decisions


@pytest.mark.parametrize("cap", CAPTURES)
def test_oracle_records_match_reference(cap):
    g, _ = load_golden(cap)
    n = len(g["desc"])
    rec, _, _ = ol.oracle_run(g["data"], g["desc"], n, None, parse=True)
    bad = np.nonzero((rec != g["rec"]).any(axis=1))[0]
    assert len(bad) == 0, f"{cap}: {len(bad)} records differ, first {bad[:5]}"


@pytest.mark.parametrize("cap", CAPTURES)
def test_oracle_filters_match_reference(cap):
    g, man = load_golden(cap)
    n = len(g["desc"])
    for s in man["captures"][cap]["filter_sets"]:
        filters = man["filter_sets"][s]
        _, dec, _ = ol.oracle_run(g["data"], g["desc"], n, filters, parse=False)
        compare_decisions(dec, g[f"code__{s}"], g[f"src__{s}"], filters, where=f"{cap}/{s}")


def test_golden_covers_every_layer_and_status():
    """The fixtures exercise every layer kind, both statuses, and all decision codes."""
    present = np.zeros(256, bool)
    ok = np.zeros(256, bool)
    for cap in CAPTURES:
        g, _ = load_golden(cap)
        for bit in range(8):
            m = 1 << bit
            present[m] |= bool(np.any(g["rec"][:, 24] & m))
            ok[m] |= bool(np.any(g["rec"][:, 25] & m))
            # attempted but too short
            ok[m + 128 if m < 128 else 255] |= False
    for bit in range(8):
        assert present[1 << bit] and ok[1 << bit], f"layer bit {bit} never seen"
    g, _ = load_golden("edge")
    short = (g["rec"][:, 24] & ~g["rec"][:, 25]) & 0xFF
    for bit in range(7):   # every layer also seen with PACKET_TOO_SHORT
        assert np.any(short & (1 << bit)), f"layer bit {bit} never too short"
    codes = set()
    for s in ("port_range_5", "ip_range_17", "c3"):
        codes |= set(np.unique(g[f"code__{s}"]).tolist())
    assert {0, 1, 2, 3} <= codes
