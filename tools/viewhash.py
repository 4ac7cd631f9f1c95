"""Per-record hashes for the benchmarks' parity checks (tools/viewhash.c; test
infrastructure). build() compiles the helper with gcc into tools/_build/ (run by
__graft_entry__.build(); the .so travels to the GPU box with the tree)."""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "viewhash.c")
LIB = os.path.join(HERE, "_build", "libviewhash.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["gcc", "-O3", "-shared", "-fPIC", "-o", LIB, SRC])
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB)
        P, U64 = ctypes.c_void_p, ctypes.c_uint64
        L.view_hash.argtypes = [P, P, U64, P]
        L.buf_hash.argtypes = [P, P, U64, P]
        _lib = L
    return _lib


def hash_views(ptrs, lens, n: int):
    """Hashes of n views: ptrs / lens are ctypes arrays (c_void_p / c_uint64)."""
    import numpy as np
    out = np.empty(n, dtype=np.uint64)
    lib().view_hash(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p), n, out.ctypes.data)
    return out


def hash_records(records) -> "np.ndarray":
    """Hashes of a list of bytes records (the generator's)."""
    import numpy as np
    blob = b"".join(records)
    ends = np.cumsum(np.fromiter((len(r) for r in records), dtype=np.uint64, count=len(records)),
                     dtype=np.uint64)
    data = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8)
    out = np.empty(len(records), dtype=np.uint64)
    lib().buf_hash(data.ctypes.data, ends.ctypes.data, len(records), out.ctypes.data)
    return out
