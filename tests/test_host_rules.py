"""CPU: host-code rules the round-3 faults taught, checked on the sources and
on the plugin's C hooks, no GPU needed.

1. A `thread_local` named inside a lambda that runs on another thread is that thread's own
   (empty) object, not the caller's: round 3's host SIGSEGV (a gather list declared
   thread_local in GpuPacketFilter::runBatch and indexed inside a forRanges lambda on a pool
   thread). Every lambda handed to a host-thread runner (forRanges, parallel_ranges,
   host_parallel, pipeline_run, pool run, the group's member threads) must not name one.
2. gpu_batch_layers writes at most 8 layers whatever bits a caller's record sets.
"""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = [os.path.join(ROOT, d, f) for d in ("beatrice_amd/host", "beatrice_amd/csrc")
           for f in sorted(os.listdir(os.path.join(ROOT, d))) if f.endswith((".cpp", ".hip", ".h", ".hpp"))]
RUNNERS = r"\b(forRanges|parallel_ranges|host_parallel|bt_host_parallel|pipeline_run|run_members|pool->run|threads->run)\s*\("


def _strip(src: str) -> str:
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r'"(?:\\.|[^"\\])*"', '""', src)


def _call_body(src: str, at: int) -> str:
    """The argument text of the call whose '(' is at or after `at` (balanced parentheses)."""
    i = src.index("(", at)
    depth = 0
    for j in range(i, len(src)):
        depth += src[j] == "("
        depth -= src[j] == ")"
        if depth == 0:
            return src[i:j + 1]
    return src[i:]


def test_no_thread_local_named_inside_host_thread_lambdas():
    bad = []
    for path in SOURCES:
        src = _strip(open(path).read())
        tl = set(re.findall(r"\bthread_local\b[^;=({]*?\b([A-Za-z_]\w*)\s*(?:[;={(]|$)", src, flags=re.M))
        if not tl:
            continue
        for m in re.finditer(RUNNERS, src):
            body = _call_body(src, m.start())
            if "[" not in body:   # no lambda in the call
                continue
            used = {n for n in tl if re.search(rf"\b{re.escape(n)}\b", body)}
            if used:
                line = src.count("\n", 0, m.start()) + 1
                bad.append(f"{os.path.relpath(path, ROOT)}:{line}: {m.group(1)} lambda names thread_local {sorted(used)}")
    assert not bad, "\n".join(bad)


def test_the_rule_catches_the_round3_pattern(tmp_path):
    """The check above flags the exact shape of round 3's bug."""
    src = _strip('''
        void f(size_t n) {
            thread_local std::vector<const uint8_t*> ptrs;
            ptrs.resize(n);
            forRanges(n, [&](size_t lo, size_t hi) { for (size_t i = lo; i < hi; ++i) ptrs[i] = nullptr; });
        }''')
    tl = set(re.findall(r"\bthread_local\b[^;=({]*?\b([A-Za-z_]\w*)\s*(?:[;={(]|$)", src, flags=re.M))
    assert tl == {"ptrs"}
    m = re.search(RUNNERS, src)
    assert m and "ptrs" in _call_body(src, m.start())


class _Batch(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_uint64), ("n", ctypes.c_uint32), ("frames", ctypes.c_void_p),
                ("lens", ctypes.c_void_p), ("decide", ctypes.c_void_p), ("pass_idx", ctypes.c_void_p),
                ("n_pass", ctypes.c_uint32), ("error_idx", ctypes.c_void_p), ("n_error", ctypes.c_uint32),
                ("records", ctypes.c_void_p)]


class _Layer(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("offset", ctypes.c_uint32), ("tag", ctypes.c_int32),
                ("parsed", ctypes.c_uint32)]


def test_gpu_batch_layers_bounded_for_any_record():
    so = os.path.join(ROOT, "beatrice_amd", "libgpu_parse_filter_plugin.so")
    assert os.path.exists(so), "plugin not built"
    L = ctypes.CDLL(so, mode=os.RTLD_LAZY | os.RTLD_GLOBAL)
    L.gpu_batch_layers.restype = ctypes.c_uint32
    L.gpu_batch_layers.argtypes = [ctypes.POINTER(_Batch), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    rec = np.zeros((3, 96), np.uint8)
    rec[0, 24] = 0xFF        # present: every BT_L_* bit
    rec[0, 25] = 0xFF        # ok
    rec[0, 26], rec[0, 27] = 14, 34
    rec[1, 24] = rec[1, 25] = 0x01 | 0x08 | 0x40   # Ethernet / IPv4 / UDP
    rec[1, 26], rec[1, 27] = 14, 34
    b = _Batch(0, 3, None, None, None, None, 0, None, 0, rec.ctypes.data)
    out = (_Layer * 16)()
    for k in range(16):
        out[k] = _Layer(b"guard", 0xDEAD, -7, 0xBEEF)
    n = L.gpu_batch_layers(ctypes.byref(b), 0, out, 16)
    assert n == 8
    assert [out[k].name.decode() for k in range(8)] == ["ethernet", "vlan", "vlan", "ipv4", "ipv6", "tcp", "udp", "icmp"]
    assert out[8].offset == 0xDEAD and out[8].name == b"guard"   # nothing written past what it reported
    for k in range(16):
        out[k] = _Layer(b"guard", 0xDEAD, -7, 0xBEEF)
    assert L.gpu_batch_layers(ctypes.byref(b), 1, out, 2) == 3           # cap bounds the writes, not the count
    assert [out[k].name.decode() for k in range(2)] == ["ethernet", "ipv4"] and out[2].offset == 0xDEAD
    assert L.gpu_batch_layers(ctypes.byref(b), 3, out, 16) == 0          # past n


def test_gpu_scripts_parse():
    """Every GPU-box script under tools/ is valid bash (a syntax error would only show on the
    box, after the queue and the box's start-up)."""
    import glob
    import subprocess
    scripts = sorted(glob.glob(os.path.join(ROOT, "tools", "*.sh")) + glob.glob(os.path.join(ROOT, "tools", "*", "*.sh")))
    assert scripts
    for sc in scripts:
        r = subprocess.run(["bash", "-n", sc], capture_output=True, text=True)
        assert r.returncode == 0, f"{sc}: {r.stderr}"
