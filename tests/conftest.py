import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the GPU)")
    config.addinivalue_line("markers", "slow: long-running")
    # torch ships its own libamdhip64.so.7: load it before librio_gpu.so so that
    # one HIP runtime serves both (tests that hand torch device buffers to the ABI)
    markexpr = getattr(config.option, "markexpr", "") or ""
    if "gpu" in markexpr and "not gpu" not in markexpr:
        import torch  # noqa: F401


def pytest_collection_modifyitems(config, items):
    # the same when GPU test files are named without -m gpu
    if any(it.get_closest_marker("gpu") for it in items) and "not gpu" not in (config.option.markexpr or ""):
        import torch  # noqa: F401


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure only)."""
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


def golden_bytes(case):
    with open(os.path.join(GOLDEN, case["file"]), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def gpu_lib():
    """librio_gpu.so, built in-tree; a GPU test fails loudly when it is missing or
    was not built from this tree's sources (its build id, base_amd/build.py)."""
    from base_amd.recordio import gpu
    return gpu.load()


@pytest.fixture(scope="session")
def gpu_ctx(gpu_lib):
    from base_amd.recordio import gpu
    ctx = gpu.Context(0, max_span_bytes=64 << 20)
    yield ctx
    ctx.close()


def oracle_has_zstd(O):
    from base_amd.recordio.codecs import have_zstd, zstd_compress
    return have_zstd() and O.zstd_decompress(zstd_compress(b"probe", 1))[0] == 0


def run(cmd):
    return subprocess.run(cmd, capture_output=True, text=True)
