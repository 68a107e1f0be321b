"""CPU: the C-ABI library loads, exports every entry point include/beatrice_gpu.h (the
product) and include/beatrice_gpu_bench.h (tests and benchmarks) declare, keeps the two apart,
and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

from beatrice_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BT_E_INVALID_ARGUMENT = 1   # include/beatrice_gpu.h (beatrice::ErrorCode::INVALID_ARGUMENT)
HEADER = os.path.join(ROOT, "include", "beatrice_gpu.h")
BENCH_HEADER = os.path.join(ROOT, "include", "beatrice_gpu_bench.h")


def declared(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(bt_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_is_exported():
    names = declared() + declared(BENCH_HEADER)
    assert len(names) >= 19, names
    L = ctypes.CDLL(abi.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"not exported: {missing}"
    assert set(abi.EXPORTS) <= set(names)


def test_product_header_holds_no_harness_entry_points():
    """The drop-in contract is beatrice_gpu.h alone: raw device memory, streams
    and timing loops are the tests' and bench.py's (beatrice_gpu_bench.h)."""
    product, harness = set(declared()), set(declared(BENCH_HEADER))
    assert not product & harness
    for name in ("bt_dev_malloc", "bt_memcpy_h2d", "bt_stream_create", "bt_time_device2", "bt_time_extract2"):
        assert name in harness and name not in product
    for name in ("bt_create", "bt_filter_compile", "bt_parse_filter", "bt_parse_filter_device",
                 "bt_group_parse_filter_mapped", "bt_synchronize"):
        assert name in product


def test_abi_version_and_struct_sizes():
    assert abi.lib().bt_abi_version() == abi.ABI_VERSION == 2
    assert ctypes.sizeof(abi.SplitCost) == 16 and ctypes.sizeof(abi.Placement) == 32
    assert ctypes.sizeof(abi.Opts) == 32
    assert ctypes.sizeof(abi.Batch) == 40
    assert ctypes.sizeof(abi.Outputs) == 48
    assert ctypes.sizeof(abi.FilterDesc) == 32
    assert ctypes.sizeof(abi.FilterSlot) == 20
    assert abi.REC_DTYPE.itemsize == 96


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU visible")
def test_no_cpu_fallback_without_gpu():
    assert abi.device_count() == 0
    with pytest.raises(abi.BtError) as e:
        abi.Context(0)
    assert e.value.code == 2   # BT_E_INIT_FAILED == ErrorCode::INITIALIZATION_FAILED


def test_compile_rejects_more_than_64_enabled_filters():
    fs = [{"type": abi.BPF, "expr": "udp", "priority": i} for i in range(65)]
    with pytest.raises(abi.BtError):
        abi.compile_host(fs)
    fs[3]["enabled"] = 0
    assert len(abi.compile_host(fs)) == 64


def test_packed_records_round_trip():
    """The packed device record (include/beatrice_gpu.h): the numpy restatement of the
    kernel's pack_record, placed in the tiled and plane-major layouts with random bytes
    in the slabs a record does not store, unpacks (bt_record_gather / _planes /
    bt_record_unpack) to the reference's bt_rec on every golden capture."""
    import numpy as np
    from conftest import load_golden
    for cap in ("edge", "fuzz", "c3", "c4", "http"):
        g, _ = load_golden(cap)
        rec = g["rec"]
        n = len(rec)
        c = abi.pack_records(rec)
        ns = abi.record_slabs(rec)
        assert ns.min() >= 2 and ns.max() <= 6
        # every dword past a record's stored slabs is zero (nothing is lost by not storing it)
        assert not np.any(c[np.arange(24)[None, :] >= 4 * ns[:, None]])
        assert all(abi.lib().bt_record_slabs(rec[i].ctypes.data) == ns[i] for i in range(0, n, 97))
        tiled = abi.tile_packed(c, ns)
        assert np.array_equal(abi.untile_records(tiled, n), rec), cap
        planes = abi.tile_packed(c, ns, planes=True)
        assert np.array_equal(abi.untile_records(planes, n, planes=True), rec), cap
        out = np.zeros(96, np.uint8)
        for i in (0, 1, 63, 64, n - 1):
            abi.lib().bt_record_gather(tiled.ctypes.data, n, i, out.ctypes.data)
            assert np.array_equal(out, rec[i])
            abi.lib().bt_record_gather_planes(planes.ctypes.data, n, i, out.ctypes.data)
            assert np.array_equal(out, rec[i])
        tot = abi.ctypes.c_uint64(0)
        buf = np.zeros_like(rec)
        assert abi.lib().bt_record_unpack(None, tiled.ctypes.data, n, n, 0, buf.ctypes.data, abi.ctypes.byref(tot)) == 0
        assert tot.value == int(ns.sum()) and np.array_equal(buf, rec)


def _dynamic_symbols(path, defined=True):
    out = subprocess.run(["nm", "-D", "--defined-only" if defined else "--undefined-only", path],
                         capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_plugin_library_exports_the_plugin_abi():
    """libgpu_parse_filter_plugin.so: createPlugin (what PluginManager::loadPlugin dlsyms,
    /root/reference/src/PluginManager.cpp:67-68) and every C hook its header declares; linked
    -z nodelete (~PluginManager dlcloses before destroying plugins, :26-34); and the only
    reference symbol it takes from the host process is Packet's out-of-line constructor."""
    so = os.path.join(ROOT, "beatrice_amd", "libgpu_parse_filter_plugin.so")
    assert os.path.exists(so), "plugin not built"
    hdr = open(os.path.join(ROOT, "include", "beatrice_gpu_plugin.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    hooks = set(re.findall(r"\b(gpu_(?:plugin|batch)_[a-z_]+)\s*\(", hdr))
    assert {"gpu_plugin_set_sink", "gpu_plugin_flush", "gpu_batch_layers", "gpu_batch_format"} <= hooks
    defined = _dynamic_symbols(so)
    assert "createPlugin" in defined
    assert hooks <= defined, hooks - defined
    dyn = subprocess.run(["readelf", "-d", so], capture_output=True, text=True, check=True).stdout
    assert "NODELETE" in dyn
    undefined = {s for s in _dynamic_symbols(so, defined=False) if "8beatrice" in s and "3gpu" not in s}
    assert undefined <= {"_ZN8beatrice6PacketC1ESt10shared_ptrIA_KhEmNSt6chrono10time_pointINS5_3_V212steady_clock"
                         "ENS5_8durationIlSt5ratioILl1ELl1000000000EEEEEE"}, undefined


def test_host_stage_bytes_refuses_null_arguments():
    """bt_host_stage_bytes (no GPU needed to refuse): a null context or output is
    BT_E_INVALID_ARGUMENT, as every entry point of the C-ABI."""
    b = ctypes.c_uint32(7)
    assert abi.lib().bt_host_stage_bytes(None, 0, ctypes.byref(b)) == BT_E_INVALID_ARGUMENT
    assert abi.lib().bt_host_stage_bytes(None, 1, None) == BT_E_INVALID_ARGUMENT
    assert b.value == 7


def test_reused_host_outputs_are_checked_and_viewed_per_call():
    """run_host's `outs`: the native side takes bare pointers, so arrays too short, of the
    wrong type or missing are refused before the call; larger ones are reused as views."""
    import numpy as np
    o = abi.host_outputs(100)
    rec, ver, dec, pidx, npass = abi._host_outputs(70, True, True, o)
    assert rec.shape == (70, abi.BT_REC_BYTES) and rec.ctypes.data == o["records"].ctypes.data
    assert len(ver) == 2 and len(dec) == 70 and len(pidx) == 70 and len(npass) == 1
    for bad in (dict(o, decide=np.zeros(50, np.uint8)), dict(o, records=None),
                dict(o, verdict=np.zeros(2, np.int64)), dict(o, pass_idx=np.zeros(200, np.uint32)[::2])):
        with pytest.raises(ValueError):
            abi._host_outputs(100, True, True, bad)
    with pytest.raises(ValueError):   # records given to a filter-only call
        abi._host_outputs(10, False, True, o)


def test_reused_host_outputs_may_leave_out_unused_keys():
    """A caller-built `outs` may omit the arrays the call does not write (no 'records' for a
    filter-only call): the views are taken with .get, so that is not a KeyError."""
    import numpy as np
    o = abi.host_outputs(64, records=False)
    del o["records"]
    rec, ver, dec, pidx, npass = abi._host_outputs(64, False, True, o)
    assert rec is None and len(dec) == 64 and len(ver) == 1
    o2 = {"records": np.zeros((64, abi.BT_REC_BYTES), np.uint8)}   # parse-only: no filter keys at all
    rec, ver, dec, pidx, npass = abi._host_outputs(64, True, False, o2)
    assert rec.shape == (64, abi.BT_REC_BYTES) and ver is None and dec is None and pidx is None and npass is None
