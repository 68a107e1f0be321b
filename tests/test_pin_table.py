"""CPU: the process's table of registered host pages (beatrice_amd/csrc/bt_pin.h), the
bookkeeping behind bt_host_register / bt_group_host_register, run with a fake driver in place
of HIP (tests/cpp/test_pin.cpp): page rounding, shared and refused overlaps, the last release
waiting for every device that holds an alias, eight group members each getting their own
device's alias, concurrent callers (also under ThreadSanitizer)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_pin.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("flags", [["-O2"], ["-O1", "-g", "-fsanitize=thread"]], ids=["plain", "tsan"])
def test_pin_table(tmp_path, flags):
    exe = tmp_path / "test_pin"
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", *flags, "-I", os.path.join(ROOT, "beatrice_amd", "csrc"),
                    SRC, "-o", str(exe), "-lpthread"], check=True, timeout=120)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
