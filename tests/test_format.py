"""bt_format_records (beatrice_amd/csrc/bt_format.cpp) against the reference's own
ParseResult formatters (src/parser/ParserResult.cpp:214-349), run by the compiled
reference over the same frames (oracle/ref_harness.cpp:ref_format, per-field wall-clock
parseTime zeroed). CPU: records from the golden fixtures (which the reference wrote)."""
import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi
from conftest import load_golden

CAPTURES = ["edge", "fuzz", "c3", "c4", "http"]
FORMATS = {"json": abi.FMT_JSON, "xml": abi.FMT_XML, "csv": abi.FMT_CSV, "human": abi.FMT_HUMAN}

needs_ref = pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref not built (needs /root/reference)")


def _first_diff(a: bytes, b: bytes) -> str:
    i = next((k for k in range(min(len(a), len(b))) if a[k] != b[k]), min(len(a), len(b)))
    return f"first difference at byte {i}: ours {a[max(0, i - 60):i + 60]!r} vs reference {b[max(0, i - 60):i + 60]!r}"


@needs_ref
@pytest.mark.parametrize("cap", CAPTURES)
@pytest.mark.parametrize("fmt", list(FORMATS))
def test_format_matches_reference(cap, fmt):
    g, _ = load_golden(cap)
    n = min(len(g["desc"]), 3000)
    ours = abi.format_records(g["rec"][:n], FORMATS[fmt])
    want = ol.ref_format(g["data"], g["desc"], n, FORMATS[fmt])
    assert ours == want, _first_diff(ours, want)


@needs_ref
@pytest.mark.parametrize("fmt", list(FORMATS))
def test_single_pass_format_matches_reference(fmt):
    """bt_format_records_to (formatted once, placed where the caller's dest says) prints
    exactly the reference's text too; no records: dest gets 0 bytes."""
    g, _ = load_golden("fuzz")
    n = min(len(g["desc"]), 3000)
    ours = abi.format_records_once(g["rec"][:n], FORMATS[fmt])
    want = ol.ref_format(g["data"], g["desc"], n, FORMATS[fmt])
    assert ours == want, _first_diff(ours, want)
    assert abi.format_records_once(g["rec"][:0], FORMATS[fmt]) == b""


def test_format_offsets_and_sizes():
    g, _ = load_golden("c4")
    rec = g["rec"][:500]
    text, off = abi.format_records(rec, abi.FMT_JSON, offsets=True)
    assert off[0] == 0 and off[-1] == len(text) and np.all(np.diff(off.astype(np.int64)) > 0)
    # packet i's slice is exactly its layers, one JSON object per line
    for i in (0, 17, 499):
        chunk = text[int(off[i]):int(off[i + 1])].decode()
        lines = chunk.rstrip("\n").split("\n")
        assert all(s.startswith('{"status":') and s.endswith("}") for s in lines)
    # the empty batch and a too-small buffer
    assert abi.format_records(rec[:0], abi.FMT_CSV) == b""
    need = abi.ctypes.c_uint64(0)
    buf = np.empty(16, np.uint8)
    rc = abi.lib().bt_format_records(None, rec.ctypes.data, 1, abi.FMT_XML, buf.ctypes.data, 16,
                                     abi.ctypes.byref(need), None)
    assert rc != 0 and need.value > 16
    assert abi.lib().bt_format_records(None, rec.ctypes.data, 1, 7, None, 0, abi.ctypes.byref(need), None) != 0


@needs_ref
@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["c4", "fuzz"])
def test_gpu_records_format_like_reference(gpu_ctx, cap):
    """The whole path: frames -> gfx950 parse -> bt_format_records on the context's host
    threads == the reference's parsePacket(...).toJsonString() / toCsvString()."""
    g, _ = load_golden(cap)
    n = min(len(g["desc"]), 2000)
    gpu_ctx.compile([])
    r = abi.DeviceRun(gpu_ctx, g["data"], g["desc"], n, records=True, decide=False, verdict=False, pass_idx=False)
    r.run()
    rec = r.fetch()["records"]
    r.free()
    for fmt in (abi.FMT_JSON, abi.FMT_CSV):
        ours = abi.format_records(rec, fmt, ctx=gpu_ctx)
        want = ol.ref_format(g["data"], g["desc"], n, fmt)
        assert ours == want, _first_diff(ours, want)


@pytest.mark.gpu
def test_parse_raw_tool():
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    frame = ("0102030405060a0b0c0d0e0f0800" "4500001c12344000401100000a010203c0a80101" "05dc0035000855aa")
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "parse_raw.py"), "--raw", frame,
                          "--format", "json"], capture_output=True, text=True, timeout=120, check=True).stdout
    lines = out.strip().split("\n")
    assert [ln.split('"protocol_name":"')[1].split('"')[0] for ln in lines[:3]] == ["ethernet", "ipv4", "udp"]
    assert '"source_ip":{"type":"14","value":"10.1.2.3"' in lines[1]
    assert lines[3] == "detected: 'udp'"
