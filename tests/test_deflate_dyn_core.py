"""CPU check of the dynamic-Huffman DEFLATE core (base_amd/csrc/deflate_dyn.h)
against zlib: tests/native/deflate_dyn_check.cpp compiled with g++ and run;
every raw DEFLATE stream it builds (trees, header, codes) must inflate with
zlib to its input."""
import os
import subprocess

import pytest

from conftest import ROOT

ZINC, ZLIB = "/opt/conda/include", "/opt/conda/lib"


def test_deflate_dynamic_core_streams_inflate_with_zlib(tmp_path):
    if not os.path.exists(os.path.join(ZINC, "zlib.h")) and not os.path.exists("/usr/include/zlib.h"):
        pytest.skip("zlib headers absent")
    exe = str(tmp_path / "deflate_dyn_check")
    cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "base_amd", "csrc"), "-I", ZINC,
           os.path.join(ROOT, "tests", "native", "deflate_dyn_check.cpp"), "-L", ZLIB, "-lz",
           "-Wl,-rpath," + ZLIB, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "fails=0" in r.stdout, r.stdout[-3000:]
