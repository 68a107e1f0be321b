"""Helpers to compare decision bytes with the golden PacketFilter outcomes."""
import numpy as np

CAPTURES = ["c1", "c3", "c4", "fuzz", "edge", "http"]


def eval_order(filters):
    """Enabled filters in evaluation order (stable priority-descending sort): the
    program slots of bt_filter_compile / the oracle."""
    en = [i for i, f in enumerate(filters) if f.get("enabled", 1)]
    return sorted(en, key=lambda i: -f_prio(filters[i]))


def f_prio(f):
    return int(f.get("priority", 0))


def has_ties(filters):
    pr = [f_prio(f) for f in filters if f.get("enabled", 1)]
    return len(pr) != len(set(pr))


def compare_decisions(decide, code, src, filters, where=""):
    """decide: bt decision bytes; code/src: golden per-packet reference outcome.
    Returns the indices of packets the device left to the host (HOST code)."""
    order = eval_order(filters)
    dcode = decide >> 6
    dslot = decide & 63
    host = np.nonzero(dcode == 3)[0]
    done = dcode != 3
    # the reference: 0 pass, 1 reject, 2/3 exception; ours: 0 pass, 1 reject, 2 throw
    exp_code = np.where(code >= 2, 2, code)
    bad = np.nonzero(done & (dcode != exp_code))[0]
    assert len(bad) == 0, f"{where}: decision code mismatch at {bad[:10]} ours={dcode[bad[:10]]} ref={code[bad[:10]]}"
    # filterName of the deciding filter (reference: name of rejecting / last filter)
    chk = done & (dcode != 2)
    if len(order):
        src_of_slot = np.array(order, dtype=np.int64)[dslot[chk]]
        exp = src[chk].astype(np.int64)
        bad = np.nonzero(src_of_slot != exp)[0]
        assert len(bad) == 0, f"{where}: deciding filter mismatch at {np.nonzero(chk)[0][bad[:10]]}"
    else:
        assert np.all(src[chk] == 255)
    # host-pending packets: the reference decided at or after the host slot
    if len(host):
        ref_done = (code[host] < 2)
        pos = {s: k for k, s in enumerate(order)}
        ref_slot = np.array([pos.get(int(s), -1) for s in src[host]])
        assert np.all(~ref_done | (ref_slot >= dslot[host])), f"{where}: host slot after the reference decision"
    return host
