"""Build librio_gpu.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The library travels to the GPU box with the repo snapshot; nothing is JIT-built.

Build provenance: the library embeds a build id, a hash of every source under
base_amd/csrc, include/rio_gpu.h and the compile flags (`tree_build_id()`),
exported as rio_build_id(). `build()` rebuilds whenever the library's id is not
the tree's, and `check_lib()` (used by the loader, smoke(), bench.py and the
GPU tests) refuses a library whose id differs from the sources it ships with.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "base_amd", "csrc")
HEADER = os.path.join(ROOT, "include", "rio_gpu.h")
# RIO_BUILD_DIR: build an experiment variant elsewhere (load it with RIO_GPU_LIB)
OUT_DIR = os.environ.get("RIO_BUILD_DIR") or os.path.join(ROOT, "base_amd", "lib")
LIB = os.path.join(OUT_DIR, "librio_gpu.so")
DEFAULT_LIB = os.path.join(ROOT, "base_amd", "lib", "librio_gpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["kernels.hip", "blocks.hip", "crc.hip", "codec.hip", "codec_flate.hip", "codec_zstd.hip", "legacy.hip",
           "encode.hip", "deflate_enc.hip", "zstd_enc.hip", "pipeline.cpp", "messages.cpp", "scanner.cpp",
           "crc_tables.cpp", "sdma.cpp"]
# RIO_EXTRA_FLAGS: -D switches of ablation builds (tools/ablate.py); the product
# build has none, and any flag changes the build id
FLAGS = os.environ.get("RIO_EXTRA_FLAGS", "").split() + [
    "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
    "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result"]


def _obj(src: str) -> str:
    return os.path.join(OUT_DIR, "obj", src + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _inputs():
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h")))
    return [os.path.join(CSRC, f) for f in files] + [HEADER]


def tree_build_id(flags=None) -> str:
    """The build id of the sources in this tree: sha256 over every csrc file's
    name and bytes, the ABI header and the compile flags (paths made relative,
    so the id does not depend on where the tree lives)."""
    h = hashlib.sha256()
    for p in _inputs():
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    fl = FLAGS if flags is None else flags
    h.update(" ".join(x.replace(ROOT, ".") for x in fl).encode())
    return h.hexdigest()[:16]


_MARK = b"RIO_BUILD_ID="


def lib_build_id(path: str = LIB) -> str | None:
    """The build id a built library carries (the string rio_build_id() returns),
    read from the file's bytes: no dlopen, so a later load of a rebuilt library
    at the same path in this process is not handed the old one. None if the
    file is absent or has no id."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        blob = f.read()
    i = blob.find(_MARK)
    if i < 0:
        return None
    return blob[i + len(_MARK):i + len(_MARK) + 16].decode("ascii", "replace")


def check_lib(path: str = DEFAULT_LIB) -> str:
    """Refuse a library that was not built from this tree's sources and flags.
    Returns the build id."""
    want = tree_build_id()
    got = lib_build_id(path)
    if got != want:
        raise RuntimeError(f"{path}: build id {got} is not this tree's {want}: the library is stale -- "
                           "run __graft_entry__.build() (python -m base_amd.build)")
    return got


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    headers = [p for p in _inputs() if p.endswith(".h")]
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    # a change of compile flags rebuilds every object
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
    # the build id object: regenerated whenever the tree's id changes
    bid = tree_build_id()
    id_src = os.path.join(OUT_DIR, "obj", "build_id.cpp")
    text = ('// generated by base_amd/build.py: hash of the csrc sources, rio_gpu.h and the flags\n'
            'static const char kId[] = "RIO_BUILD_ID=%s";\n'
            'extern "C" const char *rio_build_id(void) { return kId + 13; }\n' % bid)
    if not os.path.exists(id_src) or open(id_src).read() != text:
        with open(id_src, "w") as f:
            f.write(text)
    id_obj = id_src + ".o"
    if _stale(id_obj, [id_src]):
        subprocess.check_call([HIPCC, "-O2", "-fPIC", "-c", id_src, "-o", id_obj])
    objs = [_obj(s) for s in srcs] + [id_obj]
    if _stale(LIB, objs) or lib_build_id(LIB) != bid:
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB + ".tmp"] + objs + [
            "-L/opt/rocm/lib", "-lhsa-runtime64", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
