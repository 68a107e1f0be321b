"""CPU: the host filter compiler (bt_filter_compile_host). Its programs are evaluated
by a numpy emulation of the device's eval_slot semantics and compared with the
reference PacketFilter outcomes stored in the golden fixtures — every quirk set."""
import numpy as np
import pytest

from beatrice_amd import abi, synth
from conftest import load_golden
from golden_util import compare_decisions, eval_order

K = {name: i for i, name in enumerate(abi.KINDS)}


def frame_fields(data, desc):
    off = synth.desc_off(desc)
    ln = synth.desc_len(desc)
    top = len(data) - 1

    def b(k):
        return np.where(ln > k, data[np.minimum(off + k, top)], 0).astype(np.uint32)

    def be16(k):
        return (b(k) << 8) | b(k + 1)

    def be32(k):
        return (be16(k) << 16) | be16(k + 2)

    f = {"len": ln, "gate": (ln >= 34) & (be16(12) == 0x0800), "proto": b(23), "src": be32(26),
         "dst": be32(30), "sport": be16(34), "dport": be16(36)}
    f["l4ok"] = ((f["proto"] == 6) & (ln >= 54)) | ((f["proto"] == 17) & (ln >= 42))
    return f


def emulate(slots, f):
    n = len(f["len"])
    code = np.zeros(n, np.uint8)
    slot = np.full(n, max(len(slots) - 1, 0), np.uint8)
    open_ = np.ones(n, bool)
    for i, s in enumerate(slots):
        k = s.kind
        g, p = f["gate"], f["proto"]
        if k == K["TRUE"]:
            r = np.ones(n, np.uint8)
        elif k == K["FALSE"]:
            r = np.zeros(n, np.uint8)
        elif k == K["BPF"]:
            r = g & (((s.a & 1) > 0) & (p == 6) | ((s.a & 2) > 0) & (p == 17) | ((s.a & 4) > 0) & (p == 1))
        elif k == K["PROTO_EQ"]:
            r = g & (p == s.a)
        elif k == K["PROTO_NZ"]:
            r = g & (p != 0)
        elif k == K["IP_MASK"]:
            r = g & (((f["src"] & s.b) == s.a) | ((f["dst"] & s.b) == s.a))
        elif k == K["PORT"]:
            inr = lambda x: (x >= s.a) & (x <= s.b)  # noqa: E731
            r = g & f["l4ok"] & (inr(f["sport"]) | inr(f["dport"]))
        elif k == K["IP_THROW"]:
            r = np.where(g, 2, 0)
        elif k == K["PORT_THROW"]:
            r = np.where(g & f["l4ok"], 2, 0)
        else:
            r = np.full(n, 3)
        r = np.asarray(r, np.uint8)
        hit = open_ & (r != 1)
        code[hit] = np.select([r[hit] == 0, r[hit] == 2], [1, 2], 3)
        slot[hit] = i
        open_ &= ~hit
    return (code << 6) | slot


@pytest.mark.parametrize("cap", ["edge", "fuzz", "c3", "c4"])
def test_compiled_programs_match_reference(cap):
    g, man = load_golden(cap)
    f = frame_fields(g["data"], g["desc"])
    for s in man["captures"][cap]["filter_sets"]:
        filters = man["filter_sets"][s]
        slots = abi.compile_host(filters)
        assert [x.source_index for x in slots] == eval_order(filters)
        compare_decisions(emulate(slots, f), g[f"code__{s}"], g[f"src__{s}"], filters, where=f"{cap}/{s}")


@pytest.mark.parametrize("expr,kind,a,b,throw", [
    ("10.0.0.0/8", "IP_MASK", 0x0A000000, 0xFF000000, 0),
    ("10.0.0.0/0", "IP_MASK", 0x0A000000, 0xFFFFFFFF, 0),      # x86 shift masking: /0 == /32
    ("10.0.0.0/33", "IP_MASK", 0x0, 0x80000000, 0),            # /33 == /1
    ("10.0.0.0/-1", "IP_MASK", 0x0A000000, 0xFFFFFFFE, 0),
    ("266.0.0.0/8", "IP_MASK", 0x0A000000, 0xFF000000, 0),     # uint8_t(stoi) wraps
    ("10.1.2", "FALSE", 0, 0, 0),
    ("a.b.c.d/8", "IP_THROW", 0, 0, 1),
    ("10.0.0.0/99999999999", "IP_THROW", 0, 0, 2),
])
def test_ip_range_quirks(expr, kind, a, b, throw):
    (s,) = abi.compile_host([{"type": abi.IP_RANGE, "expr": expr}])
    assert (abi.KINDS[s.kind], s.a, s.b, s.throw_kind) == (kind, a, b, throw)


@pytest.mark.parametrize("expr,kind,a,b,throw", [
    ("1000-2000", "PORT", 1000, 2000, 0),
    ("66770", "PORT", 1234, 1234, 0),
    ("2000-1000", "FALSE", 0, 0, 0),
    ("-5", "PORT_THROW", 0, 0, 1),
    ("99999999999", "PORT_THROW", 0, 0, 2),
    (" 1000 - 2000", "PORT", 1000, 2000, 0),
])
def test_port_range_quirks(expr, kind, a, b, throw):
    (s,) = abi.compile_host([{"type": abi.PORT_RANGE, "expr": expr}])
    assert (abi.KINDS[s.kind], s.a, s.b, s.throw_kind) == (kind, a, b, throw)


def test_other_kinds():
    kinds = [abi.KINDS[s.kind] for s in abi.compile_host([
        {"type": abi.BPF, "expr": "not udp", "priority": 9},
        {"type": abi.PROTOCOL, "expr": "ip", "priority": 8},
        {"type": abi.PROTOCOL, "expr": "IP", "priority": 7},
        {"type": abi.PAYLOAD, "expr": "GET", "priority": 6},
        {"type": abi.PAYLOAD, "expr": "[", "priority": 5},
        {"type": abi.CUSTOM, "expr": "", "priority": 4},
        {"type": abi.CUSTOM, "expr": "", "priority": 3, "custom": 1},
        {"type": abi.PORT_RANGE, "expr": "", "priority": 2},
        {"type": 17, "expr": "x", "priority": 1},
    ])]
    assert kinds == ["BPF", "PROTO_NZ", "FALSE", "HOST", "FALSE", "TRUE", "HOST", "TRUE", "FALSE"]
