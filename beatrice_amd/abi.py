"""ctypes binding of the C-ABI in include/beatrice_gpu.h (libbeatrice_gpu.so).

This is the Python-side caller of the drop-in boundary, used by tests/ and bench.py;
the production caller is the C++ adapter in beatrice_amd/host/. There is no CPU
fallback: if the HIP library is missing or no GPU is visible, Context() raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BT_LIB_PATH") or os.path.join(HERE, "libbeatrice_gpu.so")

BT_REC_BYTES = 96
ABI_VERSION = 2     # include/beatrice_gpu.h BT_ABI_VERSION this binding is written against
BT_MAX_FILTERS = 64

# FilterType order (reference include/beatrice/PacketFilter.hpp:17-24)
BPF, PROTOCOL, IP_RANGE, PORT_RANGE, PAYLOAD, CUSTOM = range(6)
DECIDE_PASS, DECIDE_REJECT, DECIDE_THROW, DECIDE_HOST = range(4)
KINDS = ["TRUE", "FALSE", "BPF", "PROTO_EQ", "PROTO_NZ", "IP_MASK", "PORT", "IP_THROW", "PORT_THROW", "HOST",
         "PAYLOAD"]

L_ETH, L_VLAN0, L_VLAN1, L_IPV4, L_IPV6, L_TCP, L_UDP, L_ICMP = (1 << i for i in range(8))
# bt_rec.detect_code: reference ProtocolDetector::detectProtocol names (ProtocolRegistry.cpp:353-388)
DETECT_NAMES = ("unknown", "", "ethernet", "tcp", "udp", "icmp")

# numpy view of bt_rec (96 B, include/beatrice_gpu.h)
REC_DTYPE = np.dtype({
    "names": ["eth_dst", "eth_src", "ethertype", "pkt_len", "vlan_tpid", "vlan_tci", "present", "ok",
              "l3_off", "l4_off", "l3", "l4", "detect_code", "detect_is", "detect_is2", "reserved"],
    "formats": [("u1", 6), ("u1", 6), "<u2", "<u2", ("<u2", 2), ("<u2", 2), "u1", "u1", "u1", "u1",
                ("u1", 40), ("u1", 20), "u1", "u1", "u1", ("u1", 5)],
    "offsets": [0, 6, 12, 14, 16, 20, 24, 25, 26, 27, 28, 68, 88, 89, 90, 91],
    "itemsize": 96,
})


class BtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"beatrice_gpu error {code}: {msg}")
        self.code = code


class FilterDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("expression", ctypes.c_char_p), ("enabled", ctypes.c_int32),
                ("priority", ctypes.c_int32), ("has_custom_func", ctypes.c_int32)]


class FilterSlot(ctypes.Structure):
    _fields_ = [("source_index", ctypes.c_uint32), ("kind", ctypes.c_uint32), ("a", ctypes.c_uint32),
                ("b", ctypes.c_uint32), ("throw_kind", ctypes.c_int32)]


class Opts(ctypes.Structure):
    _fields_ = [("host_chunk_packets", ctypes.c_uint32), ("host_chunk_bytes", ctypes.c_uint32),
                ("grid_waves", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("host_threads", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 3)]


OPT_NO_PREFETCH = 0x1
OPT_TILE_BLOCKED = 0x2
OPT_RECORDS_AOS = 0x4
OPT_GRAPH = 0x8
OPT_RECORDS_PLANES = 0x10
OPT_NT_STORES = 0x20
OPT_NT_LOADS = 0x40
OPT_CACHE_DEFAULT = 0x80
OPT_SPIN_SYNC = 0x100
OPT_PAYLOAD_HOST = 0x200
OPT_WIDE_NEVER = 0x400
OPT_WIDE_ALWAYS = 0x800
OPT_PIPELINE = 0x2000
OPT_GROUP_SHARED_DEVICE = 0x4000
OPT_NO_LEAN_PCIE = 0x8000
OPT_MAPPED_GATHER_SPARSE = 0x10000
OPT_NO_LEAN_HOST = 0x20000
OPT_PAYLOAD_DFA = 0x40000
TIME_KERNEL_EVENTS = 0x1
TIME_PIPELINED = 0x2


DESC_PACKED, DESC_XDP = 0, 1


class Batch(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("stride", ctypes.c_uint32),
                ("n", ctypes.c_uint32), ("bytes", ctypes.c_uint64), ("desc_format", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class Outputs(ctypes.Structure):
    _fields_ = [("records", ctypes.c_void_p), ("n_cap", ctypes.c_uint32), ("verdict", ctypes.c_void_p),
                ("decide", ctypes.c_void_p), ("pass_idx", ctypes.c_void_p), ("n_pass", ctypes.c_void_p)]


class Timing(ctypes.Structure):
    """bt_timing (include/beatrice_gpu.h): bt_time_device_ex's breakdown."""
    _fields_ = [("span_ms", ctypes.c_float), ("main_ms", ctypes.c_float), ("main_min_ms", ctypes.c_float),
                ("main_max_ms", ctypes.c_float), ("lead_ms", ctypes.c_float), ("gap_ms", ctypes.c_float),
                ("enqueue_ms", ctypes.c_double), ("first_seen_ms", ctypes.c_double),
                ("last_seen_ms", ctypes.c_double), ("query_ms", ctypes.c_double), ("wall_ms", ctypes.c_double),
                ("spin_rc", ctypes.c_int32), ("device_flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 6)]

    def as_dict(self) -> dict:
        return {k: (round(getattr(self, k), 4) if isinstance(getattr(self, k), float) else getattr(self, k))
                for k, _ in self._fields_ if k != "reserved"}


class FieldDef(ctypes.Structure):
    """bt_field_def: one FieldDefinition of a user protocol table."""
    _fields_ = [("offset", ctypes.c_uint64), ("length", ctypes.c_uint64), ("type", ctypes.c_uint32),
                ("endianness", ctypes.c_uint32)]


class ExtractOut(ctypes.Structure):
    _fields_ = [("status", ctypes.c_void_p), ("values", ctypes.c_void_p), ("image", ctypes.c_void_p),
                ("n_cap", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


# FieldType (reference include/parser/FieldDefinition.hpp:16-35)
(FT_UINT8, FT_UINT16, FT_UINT32, FT_UINT64, FT_INT8, FT_INT16, FT_INT32, FT_INT64, FT_FLOAT32, FT_FLOAT64,
 FT_BYTES, FT_STRING, FT_BOOLEAN, FT_MAC, FT_IPV4, FT_IPV6, FT_TIMESTAMP, FT_CUSTOM) = range(18)


def field_table(fields):
    """fields: (offset, length, type, endianness) tuples -> (bt_field_def array, n)."""
    arr = (FieldDef * max(1, len(fields)))()
    for i, (o, ln, t, e) in enumerate(fields):
        arr[i] = FieldDef(int(o), int(ln), int(t), int(e))
    return arr, len(fields)


def proto_span(fields) -> int:
    arr, n = field_table(fields)
    span = ctypes.c_uint64(0)
    _check(lib().bt_proto_span(arr, n, ctypes.byref(span)))
    return span.value


class SplitCost(ctypes.Structure):
    """bt_split_cost: packet cost = round_up(min(len, window), align) + fixed."""
    _fields_ = [("window", ctypes.c_uint32), ("align", ctypes.c_uint32), ("fixed", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]

    def as_tuple(self):
        return (self.window, self.align, self.fixed)


class Placement(ctypes.Structure):
    """bt_placement: where a context's host work runs (bt_context_placement)."""
    _fields_ = [("numa_node", ctypes.c_int32), ("pinned_cpus", ctypes.c_uint32), ("pool_threads", ctypes.c_uint32),
                ("staging_node", ctypes.c_int32), ("reserved", ctypes.c_uint32 * 4)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class Tpv3Ring(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("block_size", ctypes.c_uint64), ("n_blocks", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class RingStageOpts(ctypes.Structure):
    """bt_ring_stage_opts (include/beatrice_gpu.h)."""
    _fields_ = [("batch_blocks", ctypes.c_uint32), ("gather", ctypes.c_uint32), ("in_place_every", ctypes.c_uint32),
                ("in_place_blocks", ctypes.c_uint32)]


EXPORTS = [
    "bt_abi_version", "bt_last_error", "bt_create", "bt_destroy", "bt_device_count", "bt_context_device",
    "bt_filter_compile",
    "bt_filter_program", "bt_filter_compile_host", "bt_reserve", "bt_parse_filter_device",
    "bt_parse_filter_device_async",
    "bt_parse_filter", "bt_parse_filter_ptrs", "bt_host_stage_bytes", "bt_host_register", "bt_host_unregister", "bt_dev_malloc", "bt_dev_free", "bt_memcpy_h2d", "bt_memcpy_d2h", "bt_memset_d",
    "bt_synchronize", "bt_host_parallel", "bt_stream_create", "bt_stream_synchronize", "bt_stream_destroy", "bt_time_device", "bt_time_device_ex", "bt_time_device2", "bt_proto_span", "bt_extract_device", "bt_extract", "bt_time_extract_ex", "bt_time_extract2", "bt_record_gather", "bt_record_gather_planes",
    "bt_ring_walk_tpv3", "bt_ring_release_tpv3", "bt_ring_walk_tpv3_gpu",
    "bt_payload_dfa_compile", "bt_payload_dfa_compile_ex", "bt_payload_dfa_search", "bt_payload_dfa_eval",
    "bt_format_records", "bt_format_records_to",
    "bt_record_unpack", "bt_record_slabs", "bt_ring_gather_tpv3", "bt_ring_gather_dense_tpv3",
    "bt_ring_gather_lean_tpv3", "bt_ring_stage_tpv3",
    "bt_group_create", "bt_group_destroy", "bt_group_size", "bt_group_member", "bt_group_filter_compile",
    "bt_group_parse_filter", "bt_group_parse_filter_ptrs", "bt_group_split",
    "bt_group_split_cost", "bt_group_cost", "bt_group_thread_budget", "bt_group_host_register",
    "bt_group_host_unregister", "bt_group_parse_filter_mapped", "bt_context_placement", "bt_node_cpus",
    "bt_usable_cpus", "bt_extract_host", "bt_filter_dfa_pool", "bt_group_split_plan",
    "bt_group_host_parallel",
]

DEST_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)   # bt_format_records_to's dest

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: the gfx950 extension was not built "
                           "(python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    sig = {
        "bt_abi_version": (ctypes.c_int, []),
        "bt_last_error": (ctypes.c_char_p, []),
        "bt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(Opts), ctypes.POINTER(vp)]),
        "bt_destroy": (None, [vp]),
        "bt_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "bt_context_device": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, u32]),
        "bt_filter_compile": (ctypes.c_int, [vp, ctypes.POINTER(FilterDesc), u32]),
        "bt_filter_program": (ctypes.c_int, [vp, ctypes.POINTER(FilterSlot), u32, ctypes.POINTER(u32)]),
        "bt_filter_compile_host": (ctypes.c_int, [ctypes.POINTER(FilterDesc), u32, ctypes.POINTER(FilterSlot),
                                                  u32, ctypes.POINTER(u32)]),
        "bt_reserve": (ctypes.c_int, [vp, u32]),
        "bt_parse_filter_device": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.POINTER(Outputs), vp]),
        "bt_parse_filter_device_async": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.POINTER(Outputs), vp,
                                                        vp]),
        "bt_parse_filter": (ctypes.c_int, [vp, vp, vp, u32, vp, vp, vp, vp, vp]),
        "bt_parse_filter_ptrs": (ctypes.c_int, [vp, vp, vp, u32, vp, vp, vp, vp, vp]),
        "bt_host_stage_bytes": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(u32)]),
        "bt_host_register": (ctypes.c_int, [vp, vp, u64, ctypes.POINTER(vp)]),
        "bt_host_unregister": (ctypes.c_int, [vp, vp]),
        "bt_dev_malloc": (ctypes.c_int, [vp, u64, ctypes.POINTER(vp)]),
        "bt_dev_free": (ctypes.c_int, [vp, vp]),
        "bt_memcpy_h2d": (ctypes.c_int, [vp, vp, vp, u64]),
        "bt_memcpy_d2h": (ctypes.c_int, [vp, vp, vp, u64]),
        "bt_memset_d": (ctypes.c_int, [vp, vp, ctypes.c_int, u64]),
        "bt_synchronize": (ctypes.c_int, [vp]),
        "bt_stream_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        "bt_stream_synchronize": (ctypes.c_int, [vp, vp]),
        "bt_stream_destroy": (ctypes.c_int, [vp, vp]),
        "bt_time_device": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.POINTER(Outputs), u32,
                                          ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
        "bt_time_device_ex": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.POINTER(Outputs), u32,
                                             ctypes.POINTER(Timing)]),
        "bt_time_device2": (ctypes.c_int, [vp, ctypes.POINTER(Batch), vp, u32, u32, u32, ctypes.POINTER(Timing)]),
        "bt_proto_span": (ctypes.c_int, [vp, u32, ctypes.POINTER(u64)]),
        "bt_extract_device": (ctypes.c_int, [vp, ctypes.POINTER(Batch), vp, u32, ctypes.POINTER(ExtractOut), vp]),
        "bt_extract": (ctypes.c_int, [vp, vp, vp, u32, vp, u32, vp, vp, vp]),
        "bt_extract_host": (ctypes.c_int, [vp, vp, u32, vp, u32, vp, vp, vp]),
        "bt_filter_dfa_pool": (ctypes.c_int, [vp, vp, u32, ctypes.POINTER(u32)]),
        "bt_time_extract_ex": (ctypes.c_int, [vp, ctypes.POINTER(Batch), vp, u32, ctypes.POINTER(ExtractOut), u32,
                                              ctypes.POINTER(Timing)]),
        "bt_time_extract2": (ctypes.c_int, [vp, ctypes.POINTER(Batch), vp, u32, ctypes.POINTER(ExtractOut), u32, u32,
                                            ctypes.POINTER(Timing)]),
        "bt_record_gather": (None, [vp, u32, u32, vp]),
        "bt_record_gather_planes": (None, [vp, u32, u32, vp]),
        "bt_ring_walk_tpv3": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), u32, u32, vp, u32,
                                             ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "bt_ring_release_tpv3": (ctypes.c_int, [ctypes.POINTER(Tpv3Ring), u32, u32]),
        "bt_ring_walk_tpv3_gpu": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), vp, u32, u32, vp, u32,
                                                 ctypes.POINTER(u32), ctypes.POINTER(u32), vp, vp]),
        "bt_ring_gather_tpv3": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), u32, u32, vp, vp, u32,
                                               ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "bt_ring_gather_dense_tpv3": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), u32, u32, vp, vp, vp, u32,
                                                     ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "bt_ring_gather_lean_tpv3": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), u32, u32, vp, vp, vp, u32,
                                                     ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "bt_ring_stage_tpv3": (ctypes.c_int, [vp, ctypes.POINTER(Tpv3Ring), u32, u32, ctypes.POINTER(RingStageOpts),
                                              vp, vp, vp, vp, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "bt_payload_dfa_compile": (ctypes.c_int, [ctypes.c_char_p, vp, u32, ctypes.POINTER(u32)]),
        "bt_payload_dfa_search": (ctypes.c_int, [vp, vp, u32]),
        "bt_payload_dfa_eval": (ctypes.c_int, [vp, vp, u32]),
        "bt_format_records": (ctypes.c_int, [vp, vp, u32, u32, vp, u64, ctypes.POINTER(u64), vp]),
        "bt_format_records_to": (ctypes.c_int, [vp, vp, u32, u32, DEST_FN, vp, ctypes.POINTER(u64), vp]),
        "bt_record_unpack": (ctypes.c_int, [vp, vp, u32, u32, u32, vp, ctypes.POINTER(u64)]),
        "bt_record_slabs": (u32, [vp]),
        "bt_group_create": (ctypes.c_int, [vp, u32, ctypes.POINTER(Opts), ctypes.POINTER(vp)]),
        "bt_group_destroy": (None, [vp]),
        "bt_group_size": (u32, [vp]),
        "bt_group_member": (vp, [vp, u32]),
        "bt_group_filter_compile": (ctypes.c_int, [vp, ctypes.POINTER(FilterDesc), u32]),
        "bt_group_parse_filter": (ctypes.c_int, [vp, vp, vp, u32, vp, vp, vp, vp, vp]),
        "bt_group_parse_filter_ptrs": (ctypes.c_int, [vp, vp, vp, u32, vp, vp, vp, vp, vp]),
        "bt_group_split": (ctypes.c_int, [vp, u32, u32, vp]),
        "bt_group_split_cost": (ctypes.c_int, [vp, u32, u32, ctypes.POINTER(SplitCost), vp]),
        "bt_group_split_plan": (ctypes.c_int, [vp, u32, u32, ctypes.POINTER(SplitCost), vp]),
        "bt_group_host_parallel": (ctypes.c_int, [vp, vp, vp]),
        "bt_group_cost": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32, ctypes.POINTER(SplitCost)]),
        "bt_group_thread_budget": (ctypes.c_int, [u32, u32, u32, ctypes.POINTER(u32)]),
        "bt_group_host_register": (ctypes.c_int, [vp, vp, u64]),
        "bt_group_host_unregister": (ctypes.c_int, [vp, vp]),
        "bt_group_parse_filter_mapped": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.POINTER(Outputs)]),
        "bt_context_placement": (ctypes.c_int, [vp, ctypes.POINTER(Placement)]),
        "bt_node_cpus": (ctypes.c_int, [ctypes.c_int, vp, u32, ctypes.POINTER(u32)]),
        "bt_usable_cpus": (u32, []),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):   # an older build under BT_LIB_PATH (A/B runs); tests check EXPORTS
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _ = i32
    have = L.bt_abi_version()
    if have < ABI_VERSION:
        msg = f"{LIB_PATH}: C-ABI version {have}, this binding needs {ABI_VERSION} (rebuild the library)"
        if not os.environ.get("BT_LIB_PATH"):
            raise RuntimeError(msg)
        import sys   # an older build under BT_LIB_PATH (A/B runs): what it lacks fails when called
        print(f"beatrice_amd.abi: warning: {msg}", file=sys.stderr)
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise BtError(rc, lib().bt_last_error().decode(errors="replace"))


def filter_descs(filters):
    """filters: list of dicts {type, expr, enabled=1, priority=0, custom=0}."""
    arr = (FilterDesc * max(1, len(filters)))()
    keep = []
    for i, f in enumerate(filters):
        e = f.get("expr", "").encode()
        keep.append(e)
        arr[i] = FilterDesc(f["type"], e, int(f.get("enabled", 1)), int(f.get("priority", 0)),
                            int(bool(f.get("custom", 0))))
    arr._keep = keep
    return arr


def compile_host(filters):
    """Host-only compile (no GPU needed): list of FilterSlot in evaluation order."""
    arr = filter_descs(filters)
    out = (FilterSlot * BT_MAX_FILTERS)()
    n = ctypes.c_uint32(0)
    _check(lib().bt_filter_compile_host(arr, len(filters), out, BT_MAX_FILTERS, ctypes.byref(n)))
    return [out[i] for i in range(n.value)]


FMT_JSON, FMT_XML, FMT_CSV, FMT_HUMAN = range(4)


def format_records_once(records: np.ndarray, fmt: int = FMT_JSON, ctx: "Context | None" = None) -> bytes:
    """bt_format_records_to: the same text as format_records, formatted once."""
    recs = np.ascontiguousarray(records).view(np.uint8).reshape(-1, 96)
    held = {}

    def dest(_user, nbytes):
        held["buf"] = np.empty(max(1, nbytes), np.uint8)
        return held["buf"].ctypes.data

    cb = DEST_FN(dest)
    need = ctypes.c_uint64(0)
    _check(lib().bt_format_records_to(ctx.h if ctx is not None else None, recs.ctypes.data, len(recs), fmt, cb,
                                      None, ctypes.byref(need), None))
    return held["buf"][:need.value].tobytes() if "buf" in held else b""


def format_records(records: np.ndarray, fmt: int = FMT_JSON, ctx: "Context | None" = None,
                   offsets: bool = False):
    """bt_format_records over host bt_rec (REC_DTYPE or (n, 96) u8): the reference
    ParseResult text of every walked layer. Returns bytes (and the n+1 packet offsets)."""
    recs = np.ascontiguousarray(records).view(np.uint8).reshape(-1, 96)
    n = len(recs)
    need = ctypes.c_uint64(0)
    h = ctx.h if ctx is not None else None
    _check(lib().bt_format_records(h, recs.ctypes.data, n, fmt, None, 0, ctypes.byref(need), None))
    out = np.empty(max(1, need.value), np.uint8)
    off = np.empty(n + 1, np.uint64) if offsets else None
    _check(lib().bt_format_records(h, recs.ctypes.data, n, fmt, out.ctypes.data, need.value, ctypes.byref(need),
                                   off.ctypes.data if offsets else None))
    text = out[:need.value].tobytes()
    return (text, off) if offsets else text


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().bt_device_count(ctypes.byref(n))
    return n.value


class DeviceBuffer:
    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p(0)
        _check(lib().bt_dev_malloc(ctx.h, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0):
        arr = np.ascontiguousarray(arr)
        assert offset >= 0 and offset + arr.nbytes <= self.nbytes
        _check(lib().bt_memcpy_h2d(self.ctx.h, self.ptr + offset, arr.ctypes.data, arr.nbytes))

    def download(self, arr: np.ndarray):
        assert arr.flags.c_contiguous and arr.nbytes <= self.nbytes
        _check(lib().bt_memcpy_d2h(self.ctx.h, arr.ctypes.data, self.ptr, arr.nbytes))
        return arr

    def zero(self):
        _check(lib().bt_memset_d(self.ctx.h, self.ptr, 0, self.nbytes))

    def free(self):
        """hipFree waits for the device, so an asynchronous kernel fault is reported here:
        raise it (a swallowed fault resurfaces at some later, unrelated call)."""
        if self.ptr:
            if not self.ctx.h:
                raise BtError(1, "DeviceBuffer.free after its context was closed")
            p, self.ptr = self.ptr, None
            _check(lib().bt_dev_free(self.ctx.h, p))

    def __del__(self):
        try:
            self.free()
        except Exception as e:   # cannot raise from a finaliser: say so loudly
            import sys
            print(f"beatrice_amd.abi: DeviceBuffer finaliser: {e}", file=sys.stderr, flush=True)


class Context:
    """One bt_ctx on one device."""

    def __init__(self, device: int = 0, host_chunk_packets: int = 0, grid_waves: int = 0, flags: int = 0,
                 host_threads: int = 0):
        opts = Opts()
        opts.host_threads = host_threads
        opts.host_chunk_packets = host_chunk_packets
        opts.grid_waves = grid_waves
        opts.flags = flags
        h = ctypes.c_void_p(0)
        _check(lib().bt_create(device, ctypes.byref(opts), ctypes.byref(h)))
        self.h = h.value
        self.device = device
        self.flags = flags

    def close(self):
        if self.h:
            lib().bt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_id(self) -> tuple[int, str]:
        """(HIP ordinal, PCI bus id) of the context's device (bt_context_device)."""
        d = ctypes.c_int(-1)
        bus = ctypes.create_string_buffer(64)
        _check(lib().bt_context_device(self.h, ctypes.byref(d), bus, 64))
        return d.value, bus.value.decode(errors="replace")

    def compile(self, filters):
        arr = filter_descs(filters)
        _check(lib().bt_filter_compile(self.h, arr, len(filters)))
        return self.program()

    def program(self):
        out = (FilterSlot * BT_MAX_FILTERS)()
        n = ctypes.c_uint32(0)
        _check(lib().bt_filter_program(self.h, out, BT_MAX_FILTERS, ctypes.byref(n)))
        return [out[i] for i in range(n.value)]

    def reserve(self, n: int):
        _check(lib().bt_reserve(self.h, n))

    def placement(self) -> dict:
        """bt_context_placement: NUMA node, pinned CPUs, pool size, staging node."""
        p = Placement()
        _check(lib().bt_context_placement(self.h, ctypes.byref(p)))
        return p.as_dict()

    def register(self, arr: np.ndarray) -> int:
        """Page-lock + map a host array (zero-copy); returns its device alias."""
        p = ctypes.c_void_p(0)
        _check(lib().bt_host_register(self.h, arr.ctypes.data, arr.nbytes, ctypes.byref(p)))
        return p.value

    def unregister(self, arr: np.ndarray):
        _check(lib().bt_host_unregister(self.h, arr.ctypes.data))

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def synchronize(self):
        _check(lib().bt_synchronize(self.h))

    def stream_create(self) -> int:
        """A caller-owned hipStream_t on the context's device (bt_stream_create)."""
        p = ctypes.c_void_p(0)
        _check(lib().bt_stream_create(self.h, ctypes.byref(p)))
        return p.value

    def stream_synchronize(self, stream: int):
        _check(lib().bt_stream_synchronize(self.h, stream))

    def stream_destroy(self, stream: int):
        _check(lib().bt_stream_destroy(self.h, stream))

    def run_device(self, batch: Batch, outs: Outputs, stream=None):
        _check(lib().bt_parse_filter_device(self.h, ctypes.byref(batch), ctypes.byref(outs), stream))

    def run_device_async(self, batch: Batch, outs: Outputs, stream=None, done_event=None):
        """bt_parse_filter_device_async: the compaction on the context's compaction stream;
        synchronize() (or done_event, a hipEvent_t) before reading pass_idx / n_pass."""
        _check(lib().bt_parse_filter_device_async(self.h, ctypes.byref(batch), ctypes.byref(outs), stream,
                                                  done_event))

    def time_device(self, batch: Batch, outs: Outputs, iters: int):
        a, b = ctypes.c_float(0), ctypes.c_float(0)
        _check(lib().bt_time_device(self.h, ctypes.byref(batch), ctypes.byref(outs), iters, ctypes.byref(a),
                                    ctypes.byref(b)))
        return a.value, b.value

    def time_device_ex(self, batch: Batch, outs: Outputs, iters: int) -> Timing:
        t = Timing()
        _check(lib().bt_time_device_ex(self.h, ctypes.byref(batch), ctypes.byref(outs), iters, ctypes.byref(t)))
        return t

    def time_device2(self, batch: Batch, outs, iters: int, mode: int) -> Timing:
        """bt_time_device2: outs = a list of Outputs (step i writes outs[i % len(outs)])."""
        arr = (Outputs * len(outs))(*outs)
        t = Timing()
        _check(lib().bt_time_device2(self.h, ctypes.byref(batch), ctypes.cast(arr, ctypes.c_void_p), len(outs), iters,
                                     mode, ctypes.byref(t)))
        return t

    def extract_host(self, frames, fields):
        """bt_extract over a list of frames (bytes): (status[n], values[nf, n], image[n, span])."""
        n = len(frames)
        bufs = [np.frombuffer(bytes(f), np.uint8) if len(f) else np.zeros(1, np.uint8) for f in frames]
        ptrs = (ctypes.c_void_p * max(1, n))(*[b.ctypes.data for b in bufs])
        lens = np.array([len(f) for f in frames], np.uint32)
        arr, nf = field_table(fields)
        span = proto_span(fields)
        span = span if span <= 0xFFFF else 0
        status = np.zeros(max(n, 1), np.uint8)
        values = np.zeros(max(1, nf * n), np.uint64)          # field-major, column stride n
        image = np.zeros(max(1, n * span), np.uint8)
        _check(lib().bt_extract(self.h, ptrs, lens.ctypes.data, n, arr, nf, status.ctypes.data,
                                values.ctypes.data if nf else None, image.ctypes.data if span else None))
        return status[:n], values[:nf * n].reshape(nf, n), image[:n * span].reshape(n, span)

    def run_host(self, data: np.ndarray, desc: np.ndarray, records=True, filters=True, outs: dict | None = None):
        """bt_parse_filter over host buffers. Returns dict of numpy outputs. `outs` (from
        host_outputs) reuses output arrays across calls, as a capture loop does."""
        n = len(desc)
        rec, ver, dec, pidx, npass = _host_outputs(n, records, filters, outs)
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        data = np.ascontiguousarray(data)
        desc = np.ascontiguousarray(desc, dtype=np.uint64)
        _check(lib().bt_parse_filter(self.h, p(data), p(desc), n, p(rec), p(ver), p(dec), p(pidx), p(npass)))
        out = {"records": rec, "verdict": ver, "decide": dec}
        if filters:
            out["pass_idx"] = pidx[: int(npass[0])]
            out["n_pass"] = int(npass[0])
        return out


PAGE = 4096


def host_array(shape, dtype=np.uint8) -> np.ndarray:
    """A zeroed array on pages of its own: an anonymous mapping, page-aligned and padded to
    whole pages, that lives as long as the array. Registration (Context.register,
    Group.register) is in whole pages and refuses a range that shares only some of its pages
    with a live registration, so buffers registered side by side (a capture, its
    descriptors, the outputs) are allocated this way, as a UMEM or a ring is."""
    import mmap
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    m = mmap.mmap(-1, max(PAGE, (n + PAGE - 1) // PAGE * PAGE))
    return np.frombuffer(m, dtype=dt, count=n // dt.itemsize).reshape(shape)


def host_copy(arr: np.ndarray) -> np.ndarray:
    """host_array holding a copy of arr."""
    out = host_array(arr.shape, arr.dtype)
    np.copyto(out, arr)
    return out


def host_outputs(n: int, records=True, filters=True) -> dict:
    """Output arrays for run_host calls of n packets, allocated and touched once (a capture
    loop reuses its outputs; fresh arrays would fault their pages in inside every call), each
    on pages of its own (host_array), so any of them may be registered."""
    o = {"records": host_array((n, BT_REC_BYTES), np.uint8) if records else None,
         "verdict": host_array((n + 63) // 64, np.uint64) if filters else None,
         "decide": host_array(n, np.uint8) if filters else None,
         "pass_idx": host_array(max(n, 1), np.uint32) if filters else None,
         "n_pass": host_array(1, np.uint32) if filters else None}
    for a in o.values():
        if a is not None:
            a.fill(0)   # first touch now, outside any timed call
    return o


def _host_outputs(n, records, filters, outs):
    """The output arrays of a run_host call: `outs` (from host_outputs) checked against what
    the call writes — the native side takes bare pointers, so a short or mistyped array would
    be written past its end — or fresh ones."""
    if outs is None:
        outs = host_outputs(n, records, filters)
    else:
        need = {"records": (bool(records), np.uint8, n * BT_REC_BYTES),
                "verdict": (bool(filters), np.uint64, (n + 63) // 64),
                "decide": (bool(filters), np.uint8, n),
                "pass_idx": (bool(filters), np.uint32, max(n, 1)),
                "n_pass": (bool(filters), np.uint32, 1)}
        for k, (want, dt, size) in need.items():
            a = outs.get(k)
            if (a is not None) != want:
                raise ValueError(f"outs[{k!r}]: {'required' if want else 'must be None'} for this call")
            if a is not None and (a.dtype != dt or not a.flags.c_contiguous or not a.flags.writeable or a.size < size):
                raise ValueError(f"outs[{k!r}]: need a writable contiguous {np.dtype(dt).name} array of at least "
                                 f"{size} elements, got {a.dtype} x {a.size}")
        # views of this call's part (arrays sized for a larger batch are reused as they are)
        outs = {k: None if outs.get(k) is None else outs[k].reshape(-1)[:size] for k, (_, _, size) in need.items()}
        if outs["records"] is not None:
            outs["records"] = outs["records"].reshape(n, BT_REC_BYTES)
    return outs["records"], outs["verdict"], outs["decide"], outs["pass_idx"], outs["n_pass"]


def group_split(lens: np.ndarray, parts: int, cost=None, plan=False) -> list[tuple[int, int]]:
    """bt_group_split (host only): the members' [lo, hi) packet ranges; cost = (window,
    align, fixed) selects bt_group_split_cost, plan=True bt_group_split_plan (what the
    group's calls use)."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    b = np.zeros(parts + 1, np.uint32)
    lp = lens.ctypes.data if len(lens) else None
    if cost is None:
        _check(lib().bt_group_split(lp, len(lens), parts, b.ctypes.data))
    else:
        c = SplitCost(*[int(x) for x in cost], 0)
        fn = lib().bt_group_split_plan if plan else lib().bt_group_split_cost
        _check(fn(lp, len(lens), parts, ctypes.byref(c), b.ctypes.data))
    return [(int(b[k]), int(b[k + 1])) for k in range(parts)]


def group_thread_budget(members: int, usable: int, requested: int = 0) -> int:
    """bt_group_thread_budget (host only): host threads per member."""
    out = ctypes.c_uint32(0)
    _check(lib().bt_group_thread_budget(members, usable, requested, ctypes.byref(out)))
    return out.value


def node_cpus(node: int) -> list[int]:
    """bt_node_cpus (host only): the CPUs of NUMA node `node` in this process's affinity set."""
    cpus = (ctypes.c_int32 * 4096)()
    n = ctypes.c_uint32(0)
    _check(lib().bt_node_cpus(node, cpus, 4096, ctypes.byref(n)))
    return [cpus[i] for i in range(min(n.value, 4096))]


def usable_cpus() -> int:
    return int(lib().bt_usable_cpus())


class Group:
    """bt_group: one context per device in this process."""

    def __init__(self, devices, host_chunk_packets: int = 0, flags: int = 0, host_threads: int = 0):
        opts = Opts()
        opts.host_chunk_packets = host_chunk_packets
        opts.flags = flags
        opts.host_threads = host_threads
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p(0)
        _check(lib().bt_group_create(devs, len(devices), ctypes.byref(opts), ctypes.byref(h)))
        self.h = h.value
        self.devices = list(devices)

    def close(self):
        if self.h:
            lib().bt_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return int(lib().bt_group_size(self.h))

    def member(self, k: int) -> int:
        return lib().bt_group_member(self.h, k)

    def placement(self, k: int) -> dict:
        p = Placement()
        _check(lib().bt_context_placement(self.member(k), ctypes.byref(p)))
        return p.as_dict()

    def cost(self, mapped: bool, records: bool, filters: bool, desc_bytes: int = 8):
        """bt_group_cost: the (window, align, fixed) model a call splits its batch by."""
        c = SplitCost()
        _check(lib().bt_group_cost(self.h, int(mapped), int(records), int(filters), desc_bytes, ctypes.byref(c)))
        return c.as_tuple()

    def register(self, arr: np.ndarray):
        """bt_group_host_register: page-lock + map a host array into every member's device."""
        _check(lib().bt_group_host_register(self.h, arr.ctypes.data, arr.nbytes))

    def unregister(self, arr: np.ndarray):
        _check(lib().bt_group_host_unregister(self.h, arr.ctypes.data))

    def run_mapped(self, batch: Batch, outs: Outputs):
        """bt_group_parse_filter_mapped: batch / outputs as host addresses in registered ranges."""
        _check(lib().bt_group_parse_filter_mapped(self.h, ctypes.byref(batch), ctypes.byref(outs)))

    def compile(self, filters):
        arr = filter_descs(filters)
        _check(lib().bt_group_filter_compile(self.h, arr, len(filters)))

    def run_host(self, data: np.ndarray, desc: np.ndarray, records=True, filters=True, outs: dict | None = None):
        """bt_group_parse_filter over host buffers (the same outputs as Context.run_host)."""
        return self._run(lambda *o: lib().bt_group_parse_filter(self.h, data.ctypes.data, desc.ctypes.data,
                                                                len(desc), *o),
                         len(desc), records, filters, keep=(np.ascontiguousarray(data),), outs=outs)

    def run_ptrs(self, frames, records=True, filters=True):
        """bt_group_parse_filter_ptrs over a list of frames (the std::vector<Packet> form)."""
        bufs = [np.frombuffer(bytes(f), np.uint8) if len(f) else np.zeros(1, np.uint8) for f in frames]
        ptrs = (ctypes.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])
        lens = np.array([len(f) for f in frames], np.uint32)
        return self._run(lambda *o: lib().bt_group_parse_filter_ptrs(self.h, ptrs, lens.ctypes.data, len(frames), *o),
                         len(frames), records, filters, keep=(bufs, lens))

    def _run(self, call, n, records, filters, keep=(), outs=None):
        rec, ver, dec, pidx, npass = _host_outputs(n, records, filters, outs)
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        _check(call(p(rec), p(ver), p(dec), p(pidx), p(npass)))
        del keep
        out = {"records": rec, "verdict": ver, "decide": dec}
        if filters:
            out["pass_idx"] = pidx[: int(npass[0])]
            out["n_pass"] = int(npass[0])
        return out


def ring_walk_tpv3(ring: np.ndarray, block_size: int, n_blocks: int, first: int = 0,
                   max_blocks: int | None = None, cap: int | None = None, ctx: "Context | None" = None,
                   out: np.ndarray | None = None):
    """bt_ring_walk_tpv3 over a TPACKET_V3 ring image / mmap'd ring held in `ring` (uint8).
    Returns (desc uint64[n], blocks taken); with `out` (contiguous uint64) the descriptors
    are written there and desc is a view of it. Host-only: ctx may be None (no GPU)."""
    L = lib()
    if ring.nbytes < block_size * n_blocks:
        raise ValueError("ring buffer smaller than block_size * n_blocks")
    if out is not None:
        if out.dtype != np.uint64 or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint64 array")
        cap = len(out) if cap is None else min(cap, len(out))
        desc = out
    else:
        if cap is None:
            cap = int(ring.nbytes // 96) + 1
        desc = np.empty(max(cap, 1), dtype=np.uint64)
    r = Tpv3Ring(ring.ctypes.data, block_size, n_blocks, 0)
    nd, nb = ctypes.c_uint32(), ctypes.c_uint32()
    _check(L.bt_ring_walk_tpv3(ctx.h if ctx else None, ctypes.byref(r), first,
                               n_blocks if max_blocks is None else max_blocks, desc.ctypes.data, cap,
                               ctypes.byref(nd), ctypes.byref(nb)))
    return desc[:nd.value], nb.value


PREFIX_SLOT = 128
BATCH_PREFIXES = 0x1
BATCH_LEAN = 0x2


def ring_gather_tpv3(ring: np.ndarray, block_size: int, n_blocks: int, slots: np.ndarray, out: np.ndarray,
                     first: int = 0, max_blocks: int | None = None, ctx: "Context | None" = None,
                     slot_base: int = 0, dense: bool = False, ring_out: np.ndarray | None = None,
                     lean: bool = False):
    """bt_ring_gather_tpv3: the walk of ring_walk_tpv3, plus every frame's header prefix
    copied into slots[(slot_base + i) * PREFIX_SLOT ...]; descriptors (written to
    out[slot_base:]) point into `slots`. dense=True: bt_ring_gather_dense_tpv3 (each block's
    prefixes back to back from its first slot; ring_out[slot_base:] gets the ring descriptors).
    lean=True: bt_ring_gather_lean_tpv3 (filter-only: each frame's bytes 12..43, packed after a
    16-B pad; run the batch with BATCH_PREFIXES | BATCH_LEAN). Returns (desc view, blocks taken)."""
    if slots.dtype != np.uint8 or not slots.flags.c_contiguous or out.dtype != np.uint64:
        raise ValueError("slots must be contiguous uint8, out uint64")
    if ring_out is not None and (not (dense or lean) or ring_out.dtype != np.uint64 or len(ring_out) < len(out)):
        raise ValueError("ring_out: uint64, as long as out, dense or lean gather only")
    cap = min(len(out) - slot_base, len(slots) // PREFIX_SLOT - slot_base)
    r = Tpv3Ring(ring.ctypes.data, block_size, n_blocks, 0)
    nd, nb = ctypes.c_uint32(), ctypes.c_uint32()
    args = (ctx.h if ctx else None, ctypes.byref(r), first, n_blocks if max_blocks is None else max_blocks,
            slots.ctypes.data + slot_base * PREFIX_SLOT, out.ctypes.data + 8 * slot_base)
    tail = (cap, ctypes.byref(nd), ctypes.byref(nb))
    if dense or lean:
        rd = None if ring_out is None else ring_out.ctypes.data + 8 * slot_base
        fn = lib().bt_ring_gather_lean_tpv3 if lean else lib().bt_ring_gather_dense_tpv3
        _check(fn(*args, rd, *tail))
    else:
        _check(lib().bt_ring_gather_tpv3(*args, *tail))
    return out[slot_base:slot_base + nd.value], nb.value


def ring_stage_tpv3(ctx: "Context", ring: np.ndarray, block_size: int, n_blocks: int, desc: np.ndarray,
                    decide: np.ndarray, verdict: np.ndarray | None = None, slots: np.ndarray | None = None,
                    first: int = 0, count: int | None = None, batch_blocks: int = 0, gather: bool = False,
                    in_place_every: int = 0, in_place_blocks: int = 0):
    """bt_ring_stage_tpv3: blocks [first, first + count) of a registered ring through the
    context's filter, walk of each batch overlapping the kernels of the one before. desc /
    decide (/ verdict, slots) are host arrays registered with ctx (abi.host_array + register).
    Returns (frames, passed)."""
    cap = min(len(desc), len(decide))
    if verdict is not None and len(verdict) * 64 < cap:
        raise ValueError("verdict: need ceil(cap / 64) words")
    if slots is not None and slots.nbytes < cap * PREFIX_SLOT:
        raise ValueError("slots: need cap * PREFIX_SLOT bytes")
    r = Tpv3Ring(ring.ctypes.data, block_size, n_blocks, 0)
    o = RingStageOpts(batch_blocks, 2 if gather == "adaptive" else int(bool(gather)), in_place_every, in_place_blocks)
    nd, npass = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().bt_ring_stage_tpv3(ctx.h, ctypes.byref(r), first, n_blocks if count is None else count, ctypes.byref(o),
                                    desc.ctypes.data, None if slots is None else slots.ctypes.data,
                                    decide.ctypes.data, None if verdict is None else verdict.ctypes.data, cap,
                                    ctypes.byref(nd), ctypes.byref(npass)))
    return nd.value, npass.value


def ring_walk_tpv3_gpu(ctx: "Context", ring: np.ndarray, ring_dev: int, block_size: int, n_blocks: int,
                       desc_dev: int, cap: int, first: int = 0, max_blocks: int | None = None,
                       bad_dev: int | None = None, stream=None):
    """bt_ring_walk_tpv3_gpu: the host reads the ready blocks' headers, a kernel walks
    their frame chains through ring_dev (the ring's registered alias) and writes the
    descriptors into desc_dev (device memory). Returns (descriptors, blocks taken); the
    descriptors are ready once the context stream (or `stream`) has run the walk."""
    r = Tpv3Ring(ring.ctypes.data, block_size, n_blocks, 0)
    nd, nb = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().bt_ring_walk_tpv3_gpu(ctx.h, ctypes.byref(r), ring_dev, first,
                                       n_blocks if max_blocks is None else max_blocks, desc_dev, cap,
                                       ctypes.byref(nd), ctypes.byref(nb), bad_dev, stream))
    return nd.value, nb.value


def ring_release_tpv3(ring: np.ndarray, block_size: int, n_blocks: int, first: int, count: int):
    r = Tpv3Ring(ring.ctypes.data, block_size, n_blocks, 0)
    _check(lib().bt_ring_release_tpv3(ctypes.byref(r), first, count))


def payload_dfa(expr: str):
    """bt_payload_dfa_compile: the DFA blob (bytes), None when the expression is outside
    the GPU subset (it stays on the host), or raises BtError if std::regex rejects it."""
    L = lib()
    e = expr.encode("latin-1")
    size = ctypes.c_uint32()
    rc = L.bt_payload_dfa_compile(e, None, 0, ctypes.byref(size))
    if rc == 11:
        return None
    if rc:
        raise BtError(rc, f"bt_payload_dfa_compile({expr!r}) = {rc}")
    buf = ctypes.create_string_buffer(size.value)
    _check(L.bt_payload_dfa_compile(e, buf, size.value, ctypes.byref(size)))
    return buf.raw


def payload_dfa_search(blob: bytes, s: bytes) -> bool:
    return bool(lib().bt_payload_dfa_search(blob, s, len(s)))


def payload_dfa_eval(blob: bytes, frame) -> bool:
    """applyPayloadFilter(frame) for the compiled (non-empty) expression, on the host."""
    f = bytes(frame)
    return bool(lib().bt_payload_dfa_eval(blob, f, len(f)))


def untile_records(buf: np.ndarray, n: int, planes: bool = False, ctx: "Context | None" = None,
                   n_cap: int | None = None) -> np.ndarray:
    """bt_rec[n] (AoS) from the packed device record layout (include/beatrice_gpu.h),
    unpacked by bt_record_unpack."""
    out = np.zeros((n, BT_REC_BYTES), np.uint8)
    buf = np.ascontiguousarray(buf)
    _check(lib().bt_record_unpack(ctx.h if ctx is not None else None, buf.ctypes.data,
                                  n if n_cap is None else n_cap, n, int(planes), out.ctypes.data, None))
    return out


def record_slabs(rec: np.ndarray) -> np.ndarray:
    """Slabs the packed device form of each bt_rec occupies (bt_record_slabs)."""
    ok = np.ascontiguousarray(rec).view(np.uint8).reshape(-1, BT_REC_BYTES)[:, 25].astype(np.int64)
    nd = 5 + ((ok & L_VLAN0) != 0) + ((ok & L_VLAN1) != 0) + \
        np.where(ok & L_IPV4, 5, np.where(ok & L_IPV6, 10, 0)) + \
        np.where(ok & L_TCP, 5, np.where(ok & (L_UDP | L_ICMP), 2, 0))
    return (nd + 3) // 4


def pack_records(rec: np.ndarray) -> np.ndarray:
    """numpy restatement of the kernel's packed record (parse_packet<true>; test helper):
    bt_rec[n] -> [n, 24] packed dwords, zero past each record's stored slabs."""
    r = np.ascontiguousarray(rec).view(np.uint8).reshape(-1, BT_REC_BYTES).view("<u4").astype(np.uint64)
    n = len(r)
    present, ok = r[:, 6] & 0xFF, (r[:, 6] >> 8) & 0xFF
    det = r[:, 22]
    ok4, ok6 = (ok & L_IPV4) != 0, (ok & L_IPV6) != 0
    c = np.zeros((n, 24), np.uint64)
    c[:, 0:4] = r[:, 0:4]
    c[:, 4] = present | (ok << 8) | ((det & 7) << 16) | (((det >> 8) & 0xFF) << 19) | (((det >> 16) & 7) << 27)
    ne = ((ok & L_VLAN0) != 0).astype(np.int64) + ((ok & L_VLAN1) != 0)
    x0 = (r[:, 5] & 0xFFFF) | (r[:, 4] & 0xFFFF0000)
    x1 = r[:, 5] >> 16
    v4 = np.stack([(r[:, 7] & 0xFF) | ((r[:, 7] >> 8) & 0xFF00) | ((r[:, 7] >> 8) & 0xFF0000) | ((r[:, 8] & 0xFF) << 24),
                   (r[:, 8] >> 16) | ((r[:, 9] & 0xFFFF) << 16), (r[:, 9] >> 16) | ((r[:, 10] & 0xFFFF) << 16),
                   r[:, 11], r[:, 12]], axis=1)
    l4 = r[:, 17:22]
    L = np.zeros((n, 15), np.uint64)
    L[ok4, 0:5] = v4[ok4]
    L[ok4, 5:10] = l4[ok4]
    L[ok6, 0:10] = r[ok6, 7:17]
    L[ok6, 10:15] = l4[ok6]
    for e in (0, 1, 2):
        m = ne == e
        if e >= 1:
            c[m, 5] = x0[m]
        if e == 2:
            c[m, 6] = x1[m]
        c[m, 5 + e:20 + e] = L[m]
    return c.astype(np.uint32)


def tile_packed(c: np.ndarray, nslab: np.ndarray, planes: bool = False, seed: int = 1) -> np.ndarray:
    """Test helper: packed records [n, 24] in the device layout (tiled, or plane-major
    with n_cap = n). Slabs a record does not store hold random bytes, as on the device."""
    n = len(c)
    nt = (n + 63) // 64
    rng = np.random.default_rng(seed)
    slabs = c.reshape(n, 6, 16 // 4).view(np.uint8).reshape(n, 6, 16).copy()
    keep = np.arange(6)[None, :] < nslab[:, None]
    if planes:   # whole-wave slabs, one slot per packet
        slabs[~keep] = rng.integers(0, 256, size=(int((~keep).sum()), 16), dtype=np.uint8)
        return np.ascontiguousarray(slabs.transpose(1, 0, 2)).reshape(-1)
    # tiled: slabs 0..1 at the packet's slot (zeros for a last tile's unused slots), slab
    # k >= 2 packed in packet order to the front of the tile's slab-k region
    t = rng.integers(0, 256, size=(nt, 6, 64, 16), dtype=np.uint8)
    t[:, 0:2] = 0
    for i in range(n):
        tt, lane = divmod(i, 64)
        t[tt, 0:2, lane] = slabs[i, 0:2]
    for tt in range(nt):
        idx = np.arange(tt * 64, min(n, tt * 64 + 64))
        for k in range(2, 6):
            sel = idx[nslab[idx] > k]
            t[tt, k, :len(sel)] = slabs[sel, k]
    return t.reshape(-1)


class DeviceRun:
    """Device-resident batch + outputs (the bench / parity path)."""

    def __init__(self, ctx: Context, data: np.ndarray | None, desc: np.ndarray | None, n: int, stride: int = 0,
                 records=True, decide=True, verdict=True, pass_idx=True, data_bytes: int | None = None):
        """data=None: the packet buffer (data_bytes long) is filled later with upload_data()."""
        self.ctx, self.n = ctx, n
        nbytes = int(data.nbytes) if data is not None else int(data_bytes)
        self.d_data = ctx.alloc((nbytes + 255) // 256 * 256 + 256)
        if data is not None:
            self.d_data.upload(data)
        self.d_desc = None
        if desc is not None:
            self.d_desc = ctx.alloc(max(8, desc.nbytes))
            self.d_desc.upload(np.ascontiguousarray(desc, dtype=np.uint64))
        self.batch = Batch(self.d_data.ptr, self.d_desc.ptr if self.d_desc else None, stride, n, nbytes)
        nt = (n + 63) // 64
        self.d_rec = ctx.alloc(max(16, nt * 64 * BT_REC_BYTES)) if records else None
        self.d_dec = ctx.alloc(max(16, n)) if decide else None
        self.d_ver = ctx.alloc(max(16, nt * 8)) if verdict else None
        self.d_pidx = ctx.alloc(max(16, n * 4)) if pass_idx else None
        self.d_npass = ctx.alloc(16) if pass_idx else None
        self.outs = Outputs(self.d_rec.ptr if self.d_rec else None, n,
                            self.d_ver.ptr if self.d_ver else None,
                            self.d_dec.ptr if self.d_dec else None,
                            self.d_pidx.ptr if self.d_pidx else None,
                            self.d_npass.ptr if self.d_npass else None)
        ctx.reserve(n)
        self.alt, self.alt_outs = None, None

    def upload_data(self, buf: np.ndarray, offset: int):
        """Bytes of the packet buffer from `offset` on (a capture streamed range by range)."""
        self.d_data.upload(buf, offset)

    def run(self):
        self.ctx.run_device(self.batch, self.outs)

    def fetch(self):
        n = self.n
        out = {}
        self.ctx.synchronize()
        if self.d_rec:
            buf = self.d_rec.download(np.zeros(self.d_rec.nbytes, np.uint8))
            if self.ctx.flags & OPT_RECORDS_AOS:   # bt_rec as is
                out["records"] = buf[: n * BT_REC_BYTES].reshape(n, BT_REC_BYTES)
            else:
                out["records"] = untile_records(buf, n, planes=bool(self.ctx.flags & OPT_RECORDS_PLANES))
        if self.d_dec:
            out["decide"] = self.d_dec.download(np.zeros(n, dtype=np.uint8))
        if self.d_ver:
            out["verdict"] = self.d_ver.download(np.zeros((n + 63) // 64, dtype=np.uint64))
        if self.d_pidx:
            npass = int(self.d_npass.download(np.zeros(1, dtype=np.uint32))[0])
            out["n_pass"] = npass
            out["pass_idx"] = self.d_pidx.download(np.zeros(max(npass, 1), dtype=np.uint32))[:npass]
        return out

    def record_slabs(self) -> int:
        """Total 16-B slabs the last run stored (packed records), counted on the host."""
        if not self.d_rec:
            return 0
        if not hasattr(lib(), "bt_record_unpack"):   # A/B against a build from before packed records
            return 6 * self.n
        self.ctx.synchronize()
        buf = self.d_rec.download(np.zeros(self.d_rec.nbytes, np.uint8))
        if self.ctx.flags & OPT_RECORDS_AOS:   # bt_rec as is: what the packed form would need
            return int(record_slabs(buf[: self.n * BT_REC_BYTES].reshape(self.n, BT_REC_BYTES)).sum())
        tot = ctypes.c_uint64(0)
        _check(lib().bt_record_unpack(self.ctx.h, buf.ctypes.data, self.n, self.n,
                                      int(bool(self.ctx.flags & OPT_RECORDS_PLANES)), None, ctypes.byref(tot)))
        return int(tot.value)

    def n_pass(self) -> int:
        self.ctx.synchronize()
        return int(self.d_npass.download(np.zeros(1, dtype=np.uint32))[0]) if self.d_npass else 0

    def second_outputs(self) -> Outputs:
        """A second output set of the same shape (records, decide, verdict, pass_idx,
        n_pass as this run has them), for pipelined steps that alternate two sets."""
        if self.alt is None:
            self.alt = [self.ctx.alloc(b.nbytes) if b is not None else None
                        for b in (self.d_rec, self.d_ver, self.d_dec, self.d_pidx, self.d_npass)]
            r, v, d, p, c = (b.ptr if b is not None else None for b in self.alt)
            self.alt_outs = Outputs(r, self.n, v, d, p, c)
        return self.alt_outs

    def free(self):
        for b in (self.d_data, self.d_desc, self.d_rec, self.d_dec, self.d_ver, self.d_pidx, self.d_npass,
                  *(self.alt or [])):
            if b is not None:
                b.free()


class DeviceExtract:
    """Device-resident batch for bt_extract_device (user protocol tables)."""

    def __init__(self, ctx: Context, data: np.ndarray | None, desc: np.ndarray | None, n: int, fields, stride: int = 0,
                 desc_format: int = DESC_PACKED, image=True, batch: Batch | None = None):
        """data / desc are uploaded; or `batch` names packets already on the device
        (e.g. a DeviceRun's), which this object then neither owns nor frees."""
        self.ctx, self.n = ctx, n
        self.fields = list(fields)
        self.span = proto_span(self.fields)
        self.d_data = self.d_desc = None
        if batch is not None:
            self.batch = batch
        else:
            self.d_data = ctx.alloc((data.nbytes + 255) // 256 * 256 + 256)
            self.d_data.upload(data)
            if desc is not None:
                self.d_desc = ctx.alloc(max(16, desc.nbytes))
                self.d_desc.upload(np.ascontiguousarray(desc))
            self.batch = Batch(self.d_data.ptr, self.d_desc.ptr if self.d_desc else None, stride, n,
                               int(data.nbytes), desc_format, 0)
        nf = len(self.fields)
        img = image and 0 < self.span <= 0xFFFF
        self.d_status = ctx.alloc(max(16, n))
        self.d_values = ctx.alloc(max(16, nf * n * 8)) if nf else None
        self.d_image = ctx.alloc(max(16, n * self.span)) if img else None
        self.out = ExtractOut(self.d_status.ptr, self.d_values.ptr if self.d_values else None,
                              self.d_image.ptr if self.d_image else None, n, 0)
        self.table, self.nf = field_table(self.fields)

    def run(self, stream=None):
        _check(lib().bt_extract_device(self.ctx.h, ctypes.byref(self.batch), self.table, self.nf,
                                       ctypes.byref(self.out), stream))

    def time(self, iters: int, mode: int = TIME_KERNEL_EVENTS) -> Timing:
        """bt_time_extract2: `iters` launches; with TIME_KERNEL_EVENTS each is timed from
        its own dispatch (main_ms), without them only the span is."""
        t = Timing()
        _check(lib().bt_time_extract2(self.ctx.h, ctypes.byref(self.batch), self.table, self.nf,
                                      ctypes.byref(self.out), iters, mode, ctypes.byref(t)))
        return t

    def fetch(self):
        self.ctx.synchronize()
        n, nf = self.n, len(self.fields)
        status = self.d_status.download(np.zeros(max(n, 1), np.uint8))[:n]
        values = self.d_values.download(np.zeros(max(1, nf * n), np.uint64))[:nf * n].reshape(nf, n) \
            if self.d_values else np.zeros((nf, n), np.uint64)
        image = self.d_image.download(np.zeros(max(16, n * self.span), np.uint8))[:n * self.span].reshape(n, self.span) \
            if self.d_image else None
        return status, values, image

    def free(self):
        for b in (self.d_data, self.d_desc, self.d_status, self.d_values, self.d_image):
            if b is not None:
                b.free()
