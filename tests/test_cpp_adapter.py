"""GPU: the C++ drop-in layer (GpuPacketFilter / GpuProtocolParser / the IPacketPlugin)
against the reference's own compiled PacketFilter and ProtocolParser, side by side in
one process (tests/cpp/test_adapter.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_adapter")


@pytest.mark.gpu
def test_cpp_adapter_matches_reference():
    assert os.path.exists(BIN), "tests/cpp/test_adapter not built (make -C tests/cpp in the build container)"
    r = subprocess.run([BIN, os.path.join(ROOT, "beatrice_amd", "libgpu_parse_filter_plugin.so")],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "ALL OK" in r.stdout


@pytest.mark.gpu
def test_plugin_in_the_reference_pipeline():
    """tests/cpp/test_plugin.cpp: the plugin driven through PluginManager's call sequence
    from an in-memory capture backend — flush thread, per-packet errors, ordered verdict
    sink — against the reference PacketFilter."""
    b = os.path.join(ROOT, "tests", "cpp", "test_plugin")
    assert os.path.exists(b), "tests/cpp/test_plugin not built (make -C tests/cpp in the build container)"
    r = subprocess.run([b, os.path.join(ROOT, "beatrice_amd", "libgpu_parse_filter_plugin.so")],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "ALL OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["c3", "c4", "edge"])
def test_plugin_sink_records_equal_reference_goldens(cap, tmp_path):
    """BEATRICE_GPU_RECORDS=1: the plugin's sink hands out each packet's parse record from
    the same kernel pass; tests/cpp/test_plugin compares them with the golden records the
    compiled reference's ProtocolParser produced for the same frames."""
    import numpy as np
    from conftest import load_golden
    g, _ = load_golden(cap)
    paths = []
    for k in ("data", "desc", "rec"):
        p = tmp_path / f"{k}.bin"
        g[k].tofile(p)
        paths.append(str(p))
    b = os.path.join(ROOT, "tests", "cpp", "test_plugin")
    assert os.path.exists(b), "tests/cpp/test_plugin not built (make -C tests/cpp in the build container)"
    env = dict(os.environ, BT_PLUGIN_SO=os.path.join(ROOT, "beatrice_amd", "libgpu_parse_filter_plugin.so"))
    r = subprocess.run([b, "records", *paths], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "ALL OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("cap", ["c3", "c4", "edge"])
def test_small_calls_host_and_device_branches(cap, tmp_path):
    """Single-packet applyFilters / small batches / parsePacket(slice, name): the host branch
    (the compiled program and extractor on the calling thread) and the device branch
    (setHostBatchBelow(0)) against the compiled reference, on the golden captures."""
    import numpy as np
    from conftest import load_golden
    g, _ = load_golden(cap)
    desc = np.ascontiguousarray(g["desc"], dtype=np.uint64)
    data = np.ascontiguousarray(g["data"], dtype=np.uint8)
    path = tmp_path / f"{cap}.bin"
    with open(path, "wb") as fh:
        fh.write(np.uint64(len(desc)).tobytes())
        fh.write(desc.tobytes())
        fh.write(np.uint64(data.nbytes).tobytes())
        fh.write(data.tobytes())
    r = subprocess.run([BIN, "small", str(path), cap], capture_output=True, text=True, timeout=600, cwd=ROOT)
    print(r.stdout[-4000:])
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_adapter_randomized_against_reference():
    """`test_adapter fuzz`: random programs over every filter type (PAYLOAD regexes, CUSTOM
    callbacks that throw, the reference's expression quirks, ties, disabled filters) on random
    captures whose sizes straddle the host / device threshold and the staging chunk, through
    one- and two-lane filters: the vector form, single packets, classify and the stats equal
    the compiled reference PacketFilter's. BT_FUZZ_SECONDS long (default 10 s here)."""
    secs = os.environ.get("BT_FUZZ_SECONDS", "10")
    seed = os.environ.get("BT_FUZZ_SEED", "0xB1A5")   # fixed in the suite; "random": the binary picks
    args = [BIN, "fuzz", secs] + ([] if seed == "random" else [seed])
    # lines are passed on as they come (a long run keeps writing its progress)
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=ROOT)
    lines = []
    for line in p.stdout:
        print(line, end="", flush=True)
        lines.append(line)
    rc = p.wait(timeout=float(secs) + 300)
    out = "".join(lines[-60:])
    assert rc == 0 and "ALL OK" in out, out
