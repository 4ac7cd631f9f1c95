"""Build librio_gpu.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The library travels to the GPU box with the repo snapshot; nothing is JIT-built.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "base_amd", "csrc")
# RIO_BUILD_DIR: build an experiment variant elsewhere (load it with RIO_GPU_LIB)
OUT_DIR = os.environ.get("RIO_BUILD_DIR") or os.path.join(ROOT, "base_amd", "lib")
LIB = os.path.join(OUT_DIR, "librio_gpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RIO_OFFLOAD_ARCH", "gfx950")

SOURCES = ["kernels.hip", "blocks.hip", "crc.hip", "codec.hip", "codec_flate.hip", "codec_zstd.hip", "legacy.hip", "encode.hip", "deflate_enc.hip", "zstd_enc.hip",
           "pipeline.cpp", "messages.cpp", "scanner.cpp", "crc_tables.cpp"]
FLAGS = (["-DRIO_CHECKED"] if os.environ.get("RIO_CHECKED") else []) + (["-DRIO_FLSTAT"] if os.environ.get("RIO_FLSTAT") else []) + (["-DRIO_ZPROF"] if os.environ.get("RIO_ZPROF") else []) + os.environ.get("RIO_EXTRA_FLAGS", "").split() + ([f"-DRIO_FOLD_COPIES={os.environ['RIO_FOLD_COPIES']}"] if os.environ.get("RIO_FOLD_COPIES") else []) + ([f"-DRIO_CRC_WAVES={os.environ['RIO_CRC_WAVES']}"] if os.environ.get("RIO_CRC_WAVES") else []) + ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"),
         "-I", CSRC, "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]


def _obj(src: str) -> str:
    return os.path.join(OUT_DIR, "obj", src + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(ROOT, "include", "rio_gpu.h"))
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    # a change of compile flags (RIO_CHECKED, arch) rebuilds every object
    stamp = os.path.join(OUT_DIR, "obj", ".flags")
    flags_now = " ".join(FLAGS)
    if not os.path.exists(stamp) or open(stamp).read() != flags_now:
        for s in srcs:
            if os.path.exists(_obj(s)):
                os.remove(_obj(s))
        with open(stamp, "w") as f:
            f.write(flags_now)

    def compile_one(src):
        path = os.path.join(CSRC, src)
        obj = _obj(src)
        if not _stale(obj, [path] + headers):
            return None
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [HIPCC] + FLAGS + lang + ["-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
        return r.stderr

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for w in ex.map(compile_one, srcs):
            if w and verbose:
                print(w)
    objs = [_obj(s) for s in srcs]
    if _stale(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
