"""CPU: the runtime's host thread pool (beatrice_amd/csrc/bt_host_pool.h) under stress,
compiled here with ThreadSanitizer (tests/cpp/test_host_pool.cpp): every index of a run
exactly once, runs from several callers, late or slow workers; no data race reported. Run
twice: the claiming pool, and the fixed pool (BT_POOL_FIXED, worker id runs index id), whose
runs of fewer indices than threads must not call fn past the count."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("fixed", [False, True], ids=["claiming", "fixed"])
def test_host_pool_under_thread_sanitizer(tmp_path, fixed):
    exe = tmp_path / "test_host_pool"
    src = os.path.join(ROOT, "tests", "cpp", "test_host_pool.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-o", str(exe), src, "-lpthread"],
                   check=True)
    env = {k: v for k, v in os.environ.items() if k != "BT_POOL_FIXED"}
    if fixed:
        env["BT_POOL_FIXED"] = "1"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={**env, "TSAN_OPTIONS": "halt_on_error=1 exitcode=66"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ALL OK" in r.stdout
