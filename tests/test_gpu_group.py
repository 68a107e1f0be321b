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
