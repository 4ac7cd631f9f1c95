"""CPU check of the GPU zstd encoder's core (base_amd/csrc/zstd_enc.h) against
libzstd: tests/native/zstd_enc_check.cpp compiled with g++ and run; every frame
it encodes must decode with ZSTD_decompress to its input."""
import os
import subprocess

import pytest

from conftest import ROOT

ZSTD_INC, ZSTD_LIB = "/opt/conda/include", "/opt/conda/lib"


def test_zstd_encoder_core_frames_decode_with_libzstd(tmp_path):
    if not os.path.exists(os.path.join(ZSTD_INC, "zstd.h")):
        pytest.skip("libzstd headers absent")
    exe = str(tmp_path / "zstd_enc_check")
    cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "base_amd", "csrc"), "-I", ZSTD_INC,
           os.path.join(ROOT, "tests", "native", "zstd_enc_check.cpp"), "-L", ZSTD_LIB, "-lzstd",
           "-Wl,-rpath," + ZSTD_LIB, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "fails=0" in r.stdout, r.stdout[-3000:]
