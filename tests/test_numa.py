"""CPU: beatrice_amd/numa.py — a capture copied into memory bound to a NUMA node (whole, or
one node per member byte range, as bench.py's group-ingest entry places it) keeps its bytes,
and its pages report that node."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beatrice_amd import numa, synth  # noqa: E402


def _nodes():
    try:
        return sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))
    except OSError:
        return []


@pytest.mark.skipif(not _nodes(), reason="no NUMA topology in sysfs")
def test_place_on_node_keeps_bytes_and_binds_pages():
    node = _nodes()[0]
    a = np.random.default_rng(1).integers(0, 256, 3 * 4096 + 17, dtype=np.uint8)
    try:
        b = numa.place_on(a, node)
    except OSError as e:   # mbind refused (seccomp / no NUMA support): nothing to check here
        pytest.skip(f"mbind: {e}")
    assert b is not a and np.array_equal(a, b) and b.ctypes.data % 4096 == 0
    assert numa.page_nodes(b) in ([node], [-1], [])   # -1/[]: move_pages query not permitted
    assert numa.place_on(a, None) is a and numa.place_on(a, -1) is a


@pytest.mark.skipif(not _nodes(), reason="no NUMA topology in sysfs")
def test_place_ranges_per_member():
    node = _nodes()[-1]
    data, desc = synth.capture(synth.C3, 5000, seed=4)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    bounds = [(0, 2000), (2000, 5000)]
    spans = numa.member_byte_ranges(off, ln, bounds)
    assert spans[0][0] == off[0] and spans[1][1] == off[4999] + ln[4999] and spans[0][1] <= spans[1][0] + 4096
    try:
        placed = numa.place_ranges(data, [(lo, hi, node) for lo, hi in spans])
    except OSError as e:
        pytest.skip(f"mbind: {e}")
    assert np.array_equal(placed, data)
    assert numa.place_ranges(data, [(lo, hi, -1) for lo, hi in spans]) is data
    assert numa.member_byte_ranges(off, ln, [(3, 3)]) == [(0, 0)]
