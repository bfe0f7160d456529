import json
import os
import sys

# Load torch (and with it torch's bundled HIP runtime, libamdhip64.so.7) before
# libnydusgpu.so: both resolve the same SONAME, so the first loaded runtime
# serves the whole process ("One HIP runtime per process").
import torch  # noqa: F401

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "nydus-snapshotter_amd"), os.path.join(ROOT, "oracle"), GOLDEN, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_layers():
    with open(os.path.join(GOLDEN, "layers.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def tars():
    import layers
    return {k: fn() for k, fn in layers.LAYERS.items()}


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.lib()
    return oracle_py


def kat_input(n):
    return (np.arange(n, dtype=np.int64) % 251).astype(np.uint8).tobytes()
