"""CPU: the C-ABI library loads, exports every entry point include/beatrice_gpu.h
declares, and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from beatrice_amd import abi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "beatrice_gpu.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(bt_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def test_every_declared_symbol_is_exported():
    names = declared()
    assert len(names) >= 19, names
    L = ctypes.CDLL(abi.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, f"not exported: {missing}"
    assert set(abi.EXPORTS) <= set(names)


def test_abi_version_and_struct_sizes():
    assert abi.lib().bt_abi_version() == 1
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


def test_record_gather_matches_untile():
    """bt_record_gather (C) and abi.untile_records (numpy) agree on the tiled layout."""
    import numpy as np
    n = 200
    nt = (n + 63) // 64
    buf = (np.arange(nt * 6144, dtype=np.uint32) * 2654435761 >> 13).astype(np.uint8)
    aos = abi.untile_records(buf, n)
    out = np.zeros(96, np.uint8)
    for i in (0, 1, 63, 64, 130, 199):
        abi.lib().bt_record_gather(buf.ctypes.data, n, i, out.ctypes.data)
        assert np.array_equal(out, aos[i])
    planes = buf[: 6 * n * 16]
    aos_p = abi.untile_records(planes, n, planes=True)
    for i in (0, 77, 199):
        abi.lib().bt_record_gather_planes(planes.ctypes.data, n, i, out.ctypes.data)
        assert np.array_equal(out, aos_p[i])
