"""Shared test setup.

Markers: `gpu` = needs a real MI355X (run with -m gpu on the GPU box).
The oracle (oracle/) is the checker; the product is reached only through the C ABI
(jpeg-encoder-and-decoder_amd/lib/libjpgx.so via the jpgx package).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "jpeg-encoder-and-decoder_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "libjpgx.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    if not os.path.exists(os.path.join(REPO, "oracle", "_build", "libcpuref.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def coef_sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a).astype("<i2")).tobytes()).hexdigest()


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="session")
def cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
