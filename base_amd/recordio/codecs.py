"""Encode-side transformers used by the host Writer (recordioflate / recordiozstd).

Only compression lives here: it produces files for tests and the synthetic
benchmark. Decompression is the GPU path (base_amd/csrc). The encoders need not
be byte-identical to klauspost/compress or DataDog/zstd — only decode parity
matters.

- "flate N": raw DEFLATE (RFC 1951), like recordioflate.flateCompress
  (recordio/recordioflate/recordioflate.go:29-49). Level -1 -> 6, as
  flate.DefaultCompression. ``style="go"`` ends the stream the way Go's
  flate.Writer.Close does: data in non-final blocks, then an empty final stored
  block (01 00 00 ff ff).
- "zstd N": one zstd frame via ZSTD_compress, like compress/zstd.CompressLevel
  (compress/zstd/zstd_cgo.go:19-29); level < 0 -> 5 (DataDog default).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import zlib

_ZSTD = None


def _libzstd():
    global _ZSTD
    if _ZSTD is not None:
        return _ZSTD
    cands = ["/opt/conda/lib/libzstd.so.1", ctypes.util.find_library("zstd"),
             "libzstd.so.1"]
    for c in cands:
        if not c:
            continue
        try:
            lib = ctypes.CDLL(c)
        except OSError:
            continue
        lib.ZSTD_compressBound.restype = ctypes.c_size_t
        lib.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
        lib.ZSTD_compress.restype = ctypes.c_size_t
        lib.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_int]
        lib.ZSTD_isError.restype = ctypes.c_uint
        lib.ZSTD_isError.argtypes = [ctypes.c_size_t]
        lib.ZSTD_decompress.restype = ctypes.c_size_t
        lib.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                        ctypes.c_size_t]
        lib.ZSTD_versionNumber.restype = ctypes.c_uint
        _ZSTD = lib
        return lib
    raise RuntimeError("libzstd not found: zstd encode unavailable")


def zstd_version() -> int:
    return int(_libzstd().ZSTD_versionNumber())


def zstd_compress(data: bytes, level: int = 5) -> bytes:
    lib = _libzstd()
    if level < 0:
        level = 5
    src = bytes(data)
    cap = lib.ZSTD_compressBound(len(src))
    dst = ctypes.create_string_buffer(cap)
    n = lib.ZSTD_compress(dst, cap, src, len(src), level)
    if lib.ZSTD_isError(n):
        raise RuntimeError("ZSTD_compress failed")
    return dst.raw[:n]


def zstd_compress_ex(data: bytes, level: int = 5, checksum: bool = False, content_size: bool = True,
                     window_log: int = 0) -> bytes:
    """One frame with explicit frame parameters (ZSTD_compress2 over a CCtx):
    the content checksum (XXH64), the content-size field and the window log.
    Test helper: the recordio writer itself uses zstd_compress."""
    lib = _libzstd()
    if not hasattr(lib, "_cctx_ready"):
        lib.ZSTD_createCCtx.restype = ctypes.c_void_p
        lib.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
        lib.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
        lib.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.ZSTD_compress2.restype = ctypes.c_size_t
        lib.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_size_t]
        lib._cctx_ready = True
    cctx = lib.ZSTD_createCCtx()
    try:
        # zstd.h: ZSTD_c_compressionLevel 100, windowLog 101, contentSizeFlag 200, checksumFlag 201
        params = [(100, level if level >= 0 else 5), (200, int(content_size)), (201, int(checksum))]
        if window_log:
            params.append((101, window_log))
        for k, v in params:
            if lib.ZSTD_isError(lib.ZSTD_CCtx_setParameter(cctx, k, v)):
                raise RuntimeError("ZSTD_CCtx_setParameter(%d, %d) failed" % (k, v))
        src = bytes(data)
        cap = lib.ZSTD_compressBound(len(src))
        dst = ctypes.create_string_buffer(cap)
        n = lib.ZSTD_compress2(cctx, dst, cap, src, len(src))
        if lib.ZSTD_isError(n):
            raise RuntimeError("ZSTD_compress2 failed")
        return dst.raw[:n]
    finally:
        lib.ZSTD_freeCCtx(cctx)


def zstd_decompress_ref(data: bytes, cap: int) -> bytes:
    """libzstd decode (test/fixture helper only)."""
    lib = _libzstd()
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = lib.ZSTD_decompress(dst, cap, bytes(data), len(data))
    if lib.ZSTD_isError(n):
        raise RuntimeError("ZSTD_decompress failed")
    return dst.raw[:n]


def flate_compress(data: bytes, level: int = -1, style: str = "go") -> bytes:
    if level < 0:
        level = 6
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    if style == "go":
        out = c.compress(bytes(data)) + c.flush(zlib.Z_SYNC_FLUSH)
        return out + b"\x01\x00\x00\xff\xff"
    return c.compress(bytes(data)) + c.flush(zlib.Z_FINISH)


def parse_transformer(spec: str):
    """registry.go:54-64: split on the first space -> (name, config)."""
    toks = spec.split(" ", 1)
    return toks[0], (toks[1] if len(toks) > 1 else "")


def make_compressor(spec: str, flate_style: str = "go"):
    name, config = parse_transformer(spec)
    if name == "flate":
        level = int(config) if config else -1
        return lambda b: flate_compress(b, level, flate_style)
    if name == "zstd":
        level = int(config) if config else -1
        return lambda b: zstd_compress(b, level)
    raise KeyError(f"Transformer {spec} not found")


def have_zstd() -> bool:
    try:
        _libzstd()
        return True
    except RuntimeError:
        return False


__all__ = ["flate_compress", "zstd_compress", "make_compressor", "parse_transformer",
           "have_zstd", "zstd_version", "zstd_decompress_ref", "zstd_compress_ex"]
