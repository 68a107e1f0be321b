"""Shared test setup.

Markers: `gpu` = needs an MI355X (run with `-m gpu` on the GPU box); everything else
runs on CPU. GPU tests are skipped only when no HIP device is visible at all; a missing
or broken gfx950 library makes them fail loudly instead.
"""
import json
import os
import sys

import numpy as np
import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
sys.path.insert(0, ROOT)
sys.path.insert(0, TESTS)

GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def _gpu_visible() -> bool:
    # /dev/kfd is what the HIP runtime opens; cheaper and side-effect free
    return os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)


def pytest_collection_modifyitems(config, items):
    if _gpu_visible():
        return
    skip = pytest.mark.skip(reason="no GPU visible (/dev/kfd)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


_cache = {}


def load_golden(name):
    if name not in _cache:
        with open(os.path.join(GOLDEN, "manifest.json")) as fh:
            man = json.load(fh)
        z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
        _cache[name] = ({k: z[k] for k in z.files}, man)
    return _cache[name]


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def gpu_ctx():
    from beatrice_amd import abi
    ctx = abi.Context(0)
    yield ctx
    ctx.close()
