"""ctypes access to the TEST-ONLY checkers under oracle/:

* libbt_oracle.so   — plain-C restatement (oracle/bt_oracle.c)
* _ref/libbt_ref.so — the reference's own parser + PacketFilter sources compiled
                      unmodified (oracle/Makefile), driven by oracle/ref_harness.cpp

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use these.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "libbt_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libbt_ref.so")

BPF, PROTOCOL, IP_RANGE, PORT_RANGE, PAYLOAD, CUSTOM = range(6)


class FilterSpec(ctypes.Structure):
    """bto_filter (oracle) == FilterSpec (ref harness) == bt_filter_desc layout."""
    _fields_ = [("type", ctypes.c_int32), ("expression", ctypes.c_char_p),
                ("enabled", ctypes.c_int32), ("priority", ctypes.c_int32),
                ("custom", ctypes.c_int32)]


def filter_array(filters):
    """filters: list of dicts {type, expr, enabled=1, priority=0, custom=0}."""
    arr = (FilterSpec * max(1, len(filters)))()
    keep = []
    for i, f in enumerate(filters):
        e = f.get("expr", "").encode()
        keep.append(e)
        arr[i] = FilterSpec(f["type"], e, int(f.get("enabled", 1)), int(f.get("priority", 0)),
                            int(f.get("custom", 0)))
    arr._keep = keep  # keep the bytes alive
    return arr


_oracle = None
_ref = None


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle/libbt_oracle.so missing: make -C oracle")
        L = ctypes.CDLL(ORACLE_SO)
        L.bto_extract.restype = ctypes.c_uint64
        L.bto_extract.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p]
        L.bto_run.restype = ctypes.c_uint64
        L.bto_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_int]
        _oracle = L
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        L = ctypes.CDLL(REF_SO)
        L.ref_parse.restype = ctypes.c_int
        L.ref_parse.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_void_p]
        L.ref_filter.restype = ctypes.c_int
        L.ref_filter.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.ref_filter_batch.restype = ctypes.c_int
        L.ref_filter_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.ref_extract.restype = ctypes.c_int
        L.ref_extract.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_uint64]
        L.ref_bench.restype = ctypes.c_uint64
        L.ref_bench.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
        L.ref_bench_extract.restype = ctypes.c_uint64
        L.ref_bench_extract.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_double)]
        L.ref_format.restype = ctypes.c_uint64
        L.ref_format.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
        _ref = L
    return _ref


def _ptr(a):
    return None if a is None else a.ctypes.data


def oracle_run(data, desc, n, filters=None, stride=0, parse=True, threads=8):
    """Returns (records[n,96] or None, decide[n] or None, passed)."""
    f = filter_array(filters or [])
    rec = np.zeros((n, 96), dtype=np.uint8) if parse else None
    dec = np.zeros(n, dtype=np.uint8) if filters is not None else None
    passed = oracle().bto_run(_ptr(data), _ptr(desc), stride, n, f if filters is not None else None,
                              len(filters or []), _ptr(rec), _ptr(dec), threads)
    return rec, dec, int(passed)


def ref_parse(data, desc, n, stride=0):
    rec = np.zeros((n, 96), dtype=np.uint8)
    bad = ref().ref_parse(_ptr(data), _ptr(desc), stride, n, _ptr(rec))
    assert bad == 0, f"reference returned unexpected ParseStatus for {bad} packets"
    return rec


def ref_format(data, desc, n, fmt, stride=0):
    """The reference ParseResult formatter text of every walked layer (oracle/ref_harness.cpp)."""
    need = ref().ref_format(_ptr(data), _ptr(desc), stride, n, fmt, None, 0)
    out = np.empty(max(1, need), np.uint8)
    ref().ref_format(_ptr(data), _ptr(desc), stride, n, fmt, out.ctypes.data, need)
    return out[:need].tobytes()


def ref_filter(data, desc, n, filters, stride=0):
    """Per-packet applyFilters(const Packet&): (code[n], src[n]); code 0 pass, 1 reject,
    2 invalid_argument, 3 out_of_range; src = index of filterName (255 = none)."""
    f = filter_array(filters)
    code = np.zeros(n, dtype=np.uint8)
    src = np.zeros(n, dtype=np.uint8)
    ref().ref_filter(_ptr(data), _ptr(desc), stride, n, f, len(filters), _ptr(code), _ptr(src))
    return code, src


def ref_bench(data, desc, n, filters, parse=True, threads=8, seconds=10.0, stride=0):
    f = filter_array(filters)
    el = ctypes.c_double(0)
    done = ref().ref_bench(_ptr(data), _ptr(desc), stride, n, f, len(filters), int(parse), threads,
                           seconds, ctypes.byref(el))
    return int(done), el.value


def ref_bench_extract(data, desc, n, fields, threads=8, seconds=5.0, stride=0):
    """CPU baseline: the compiled reference's parsePacket(frame, ProtocolDefinition) on
    `threads` threads for `seconds`. Returns (packets, elapsed seconds)."""
    t = table_array(fields)
    el = ctypes.c_double(0)
    done = ref().ref_bench_extract(_ptr(data), _ptr(desc), stride, n, t.ctypes.data, len(t), threads, seconds,
                                   ctypes.byref(el))
    return int(done), el.value


def table_array(fields):
    """fields: list of (offset, length, type, endianness) -> contiguous u64[nf, 4]."""
    return np.ascontiguousarray(np.asarray(fields, dtype=np.uint64).reshape(-1, 4))


def oracle_extract(data, desc, n, fields, stride=0):
    """C restatement (bto_extract): (status[n], values[nf, n], image[n, span], span)."""
    t = table_array(fields)
    nf = len(t)
    span = oracle().bto_extract(None, None, 0, 0, t.ctypes.data, nf, None, None, None)
    status = np.zeros(n, np.uint8)
    values = np.zeros((nf, n), np.uint64)
    image = np.zeros((n, max(span, 1)), np.uint8)
    oracle().bto_extract(_ptr(data), _ptr(desc), stride, n, t.ctypes.data, nf, status.ctypes.data,
                         values.ctypes.data, image.ctypes.data)
    return status, values, image[:, :span], int(span)


def ref_extract(data, desc, n, fields, stride=0):
    """The compiled reference's ProtocolParser::parsePacket(frame, ProtocolDefinition):
    (status[n], values[nf, n], field_bytes[n, sum(length)])."""
    t = table_array(fields)
    nf = len(t)
    fbw = int(t[:, 1].sum()) if nf else 0
    status = np.zeros(n, np.uint8)
    values = np.zeros((nf, n), np.uint64)
    fb = np.zeros((n, max(fbw, 1)), np.uint8)
    odd = ref().ref_extract(_ptr(data), _ptr(desc), stride, n, t.ctypes.data, nf, status.ctypes.data,
                            values.ctypes.data, fb.ctypes.data, max(fbw, 1))
    assert odd == 0, f"{odd} reference results with a partial field set"
    return status, values, fb[:, :fbw]


def field_bytes_of_image(image, fields):
    """The concatenated field bytes (ref_extract's layout) cut out of [0, span) images."""
    parts = [image[:, int(o):int(o) + int(ln)] for o, ln, _, _ in fields]
    return np.concatenate(parts, axis=1) if parts else np.zeros((len(image), 0), np.uint8)
