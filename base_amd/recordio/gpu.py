"""ctypes binding of librio_gpu.so (include/rio_gpu.h) and the Python mirror of
the reference scanner surface:

    recordio.NewScanner(in, ScannerOpts)          -> NewScanner(src, ScannerOpts)
    recordio.NewShardScanner(in, opts, s, l, n)   -> NewShardScanner(src, opts, s, l, n)
    Scanner.{Header,Scan,Get,Err,Seek,Trailer,Version,Finish}

(recordio/scannerv2.go:100-235). Decoding runs in the HIP pipeline; this module
only moves views. Loading fails loudly when the library is missing — there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import threading
from typing import Callable, List, Optional, Tuple

from .format import Uint
from .writer import ItemLocation

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RIO_GPU_LIB") or os.path.join(_ROOT, "lib", "librio_gpu.so")  # (override: experiments)

RIO_CODEC_NONE, RIO_CODEC_FLATE, RIO_CODEC_ZSTD = 0, 1, 2
RIO_CODEC_CHAIN_FLAG = 0x10000


def codec_chain(*codecs: int) -> int:
    """RIO_CODEC_CHAIN of the header's transformer values t0, t1, ... (each
    RIO_CODEC_FLATE or RIO_CODEC_ZSTD; untransformed last to first)."""
    codes = 0
    for i, c in enumerate(codecs):
        codes |= c << (2 * i)
    return RIO_CODEC_CHAIN_FLAG | (len(codecs) << 8) | codes
RIO_STOP_MORE, RIO_STOP_EOF, RIO_STOP_ERROR = 0, 1, 2
RIO_ERR_CAPACITY = 98
RIO_ERR_LOCATION = 22  # "Invalid location ..." / no item at a location (scannerv2.go:348-361)
RIO_ERR_LEGACY = 20    # (no longer returned: v1 files decode natively)
RIO_ERR_V1_RECORD = 24  # v1 record header / read errors (deprecated/recordio.go:258-300)
RIO_ERR_V1_PACKED = 25  # v1 packed-record errors (deprecated/packer.go:214-272)
RIO_ERR_FALLBACK = 23  # transformer chain / name other than flate, zstd (registry.go:113-148)
U64_MAX = (1 << 64) - 1
ITEM_IN_RECORDS = 1 << 63  # RIO_ITEM_IN_RECORDS


class RioError(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("reserved", ctypes.c_int32), ("file_off", ctypes.c_uint64),
                ("a", ctypes.c_uint64), ("b", ctypes.c_uint64), ("c", ctypes.c_uint64),
                ("msg", ctypes.c_char * 512)]


RIO_CFG_ITEM_END = 1  # device results carry item_end (cumSize) + block_data / block_first_off
RIO_CFG_FLATE_NO_SPLIT = 2  # never split a flate block's copy pass (tuning / tests)
RIO_CFG_FLATE_TOK_ONLY = 4  # every flate block through the fallback Huffman pass, k_flate_tok (tests)
RIO_CFG_FLATE_ONE_WAVE = 16  # the one-wave Huffman pass on every span, not its 4-wave variant (tests)


def RIO_CFG_SPANS_AHEAD(n: int) -> int:
    """Scanners over the ctx decode up to n (0-2) spans ahead (default 2; above 2 is 2)."""
    return (min(max(int(n), 0), 2) + 1) << 8


class RioConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_int32), ("max_span_bytes", ctypes.c_uint64),
                ("max_out_bytes", ctypes.c_uint64), ("max_items", ctypes.c_uint64),
                ("flate_tok_limit", ctypes.c_uint64), ("flate_grid", ctypes.c_uint64)]


class RioBatch(ctypes.Structure):
    _fields_ = [("span", ctypes.c_void_p), ("records", ctypes.c_void_p), ("records_len", ctypes.c_uint64),
                ("item_off", ctypes.POINTER(ctypes.c_uint64)), ("item_len", ctypes.POINTER(ctypes.c_uint64)),
                ("n_items", ctypes.c_uint64),
                ("block_first_item", ctypes.POINTER(ctypes.c_uint64)),
                ("block_file_off", ctypes.POINTER(ctypes.c_uint64)), ("n_blocks", ctypes.c_uint64),
                ("consumed", ctypes.c_uint64), ("stop", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("in_bytes", ctypes.c_uint64), ("kernel_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("err", RioError),
                ("item_end", ctypes.POINTER(ctypes.c_uint64)), ("block_data", ctypes.POINTER(ctypes.c_uint64)),
                ("block_first_off", ctypes.POINTER(ctypes.c_uint64)),
                ("block_segment", ctypes.POINTER(ctypes.c_uint64)), ("err_segment", ctypes.c_int64)]


READ_AT = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_uint64)


class RioReader(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("read_at", READ_AT), ("size", ctypes.c_int64)]


class RioEncodeArgs(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("item_end", ctypes.c_void_p), ("n_items", ctypes.c_uint64),
                ("items_per_block", ctypes.c_uint64), ("codec", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("level", ctypes.c_int32), ("reserved", ctypes.c_int32)]


RIO_BLOCK_BODY, RIO_BLOCK_HEADER, RIO_BLOCK_TRAILER = 0, 1, 2


class RioStats(ctypes.Structure):
    _fields_ = [("spans", ctypes.c_uint64), ("h2d_bytes", ctypes.c_uint64), ("d2h_bytes", ctypes.c_uint64),
                ("device_ms", ctypes.c_double), ("span_cap", ctypes.c_uint64)]


class RioMemory(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_uint64)]


# every symbol include/rio_gpu.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "rio_open", "rio_close", "rio_last_error", "rio_abi_version", "rio_stream", "rio_codec_for_transformers",
    "rio_scan_span", "rio_scan_device", "rio_scan_device_async", "rio_sync", "rio_stage_times", "rio_decode_block",
    "rio_scanner_new", "rio_scanner_scan", "rio_scanner_get", "rio_scanner_next_batch", "rio_scanner_err",
    "rio_scanner_header_len", "rio_scanner_header_kv", "rio_scanner_trailer", "rio_scanner_seek",
    "rio_scanner_location", "rio_scanner_version", "rio_scanner_finish", "rio_scanner_gather",
    "rio_memory_reader", "rio_scan_v1_span", "rio_encode", "rio_encode_device", "rio_build_id",
    "rio_scan_device_segments_async", "rio_flate_split_blocks", "rio_ctx_stats",
]

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load librio_gpu.so; raises if it was not built (no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build() (there is no CPU fallback)")
        from .. import build as B
        B.check_lib(path)  # refuses a library not built from this tree's sources
        L = ctypes.CDLL(path)
        L.rio_build_id.restype = ctypes.c_char_p
        L.rio_ctx_stats.restype = ctypes.c_int
        L.rio_ctx_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(RioStats)]
        L.rio_flate_split_blocks.restype = ctypes.c_uint64
        L.rio_flate_split_blocks.argtypes = [ctypes.c_void_p]
        L.rio_scan_device_segments_async.restype = ctypes.c_int
        L.rio_scan_device_segments_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                     ctypes.c_int32]
        P, U64, I64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32
        L.rio_open.restype = P
        L.rio_open.argtypes = [ctypes.POINTER(RioConfig)]
        L.rio_close.argtypes = [P]
        L.rio_last_error.restype = ctypes.c_char_p
        L.rio_abi_version.restype = ctypes.c_int
        L.rio_stream.restype = P
        L.rio_stream.argtypes = [P]
        L.rio_codec_for_transformers.restype = ctypes.c_int
        L.rio_codec_for_transformers.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                                 ctypes.POINTER(I32), ctypes.POINTER(RioError)]
        L.rio_scan_span.restype = ctypes.c_int
        L.rio_scan_span.argtypes = [P, P, U64, U64, I32, U64, I32, ctypes.POINTER(RioBatch)]
        L.rio_scan_v1_span.restype = ctypes.c_int
        L.rio_scan_v1_span.argtypes = [P, P, U64, U64, I32, ctypes.POINTER(RioBatch)]
        L.rio_encode.restype = ctypes.c_int
        L.rio_encode.argtypes = [P, ctypes.POINTER(RioEncodeArgs), P, U64, ctypes.POINTER(U64), P,
                                 ctypes.POINTER(RioError)]
        L.rio_encode_device.restype = ctypes.c_int
        L.rio_encode_device.argtypes = [P, ctypes.POINTER(RioEncodeArgs), P, U64, ctypes.POINTER(U64), P,
                                        ctypes.POINTER(RioError)]
        L.rio_scan_device.restype = ctypes.c_int
        L.rio_scan_device.argtypes = [P, P, U64, U64, I32, U64, I32, ctypes.POINTER(RioBatch)]
        L.rio_scan_device_async.restype = ctypes.c_int
        L.rio_scan_device_async.argtypes = [P, P, U64, U64, I32]
        L.rio_sync.restype = ctypes.c_int
        L.rio_sync.argtypes = [P, ctypes.POINTER(RioBatch)]
        L.rio_stage_times.restype = ctypes.c_int
        L.rio_stage_times.argtypes = [P, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        L.rio_decode_block.restype = ctypes.c_int
        L.rio_decode_block.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.c_int, I32, P, U64, ctypes.POINTER(U64), ctypes.POINTER(RioError)]
        L.rio_scanner_new.restype = P
        L.rio_scanner_new.argtypes = [P, ctypes.POINTER(RioReader), ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.rio_scanner_scan.restype = ctypes.c_int
        L.rio_scanner_scan.argtypes = [P]
        L.rio_scanner_get.restype = ctypes.c_int
        L.rio_scanner_get.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(U64)]
        L.rio_scanner_next_batch.restype = I64
        L.rio_scanner_next_batch.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(U64), I64]
        L.rio_scanner_err.restype = ctypes.c_int
        L.rio_scanner_err.argtypes = [P, ctypes.POINTER(RioError)]
        L.rio_scanner_header_len.restype = ctypes.c_int
        L.rio_scanner_header_len.argtypes = [P]
        L.rio_scanner_header_kv.restype = ctypes.c_int
        L.rio_scanner_header_kv.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                            ctypes.POINTER(I32), ctypes.POINTER(I64),
                                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(U64)]
        L.rio_scanner_trailer.restype = ctypes.c_int
        L.rio_scanner_trailer.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(U64)]
        L.rio_scanner_seek.argtypes = [P, U64, I64]
        L.rio_scanner_location.argtypes = [P, ctypes.POINTER(U64), ctypes.POINTER(I64)]
        L.rio_scanner_version.restype = ctypes.c_int
        L.rio_scanner_version.argtypes = [P]
        L.rio_scanner_finish.restype = ctypes.c_int
        L.rio_scanner_finish.argtypes = [P, ctypes.POINTER(RioError)]
        L.rio_memory_reader.restype = RioReader
        L.rio_memory_reader.argtypes = [ctypes.POINTER(RioMemory)]
        L.rio_scanner_gather.restype = I64
        L.rio_scanner_gather.argtypes = [P, ctypes.POINTER(U64), ctypes.POINTER(I64), I64,
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(U64), ctypes.POINTER(RioError)]
        _lib = L
        return L


class RecordioError(Exception):
    """An error reported by the scanner; str() is the reference's message."""

    def __init__(self, code: int, msg: str, file_off: int = 0):
        super().__init__(msg)
        self.code = code
        self.file_off = file_off


def _err(e: RioError) -> RecordioError:
    return RecordioError(int(e.code), e.msg.decode(errors="replace"), int(e.file_off))


class Context:
    """One rio_ctx: a device, a HIP stream and fixed-capacity buffers."""

    def __init__(self, device: int = 0, max_span_bytes: int = 0, max_out_bytes: int = 0, max_items: int = 0,
                 item_end: bool = False, flate_tok_limit: int = 0, flate_grid: int = 0,
                 flate_split: bool = True, flate_tok_only: bool = False, spans_ahead: Optional[int] = None,
                 flate_one_wave: bool = False):
        self.L = load()
        flags = (RIO_CFG_ITEM_END if item_end else 0) | (0 if flate_split else RIO_CFG_FLATE_NO_SPLIT) | \
            (RIO_CFG_FLATE_TOK_ONLY if flate_tok_only else 0) | (RIO_CFG_FLATE_ONE_WAVE if flate_one_wave else 0) | \
            (0 if spans_ahead is None else RIO_CFG_SPANS_AHEAD(spans_ahead))
        cfg = RioConfig(device, flags, max_span_bytes, max_out_bytes, max_items, flate_tok_limit, flate_grid)
        self.item_end = item_end
        self.h = self.L.rio_open(ctypes.byref(cfg))
        if not self.h:
            raise RuntimeError("rio_open failed: " + self.L.rio_last_error().decode())
        self.device = device

    def close(self):
        if self.h:
            self.L.rio_close(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def scan_span(self, span: bytes, file_off: int = 0, is_file_end: bool = True, limit_off: int = U64_MAX,
                  codec: int = RIO_CODEC_NONE) -> RioBatch:
        out = RioBatch()
        buf = (ctypes.c_char * len(span)).from_buffer_copy(span) if not isinstance(span, ctypes.Array) else span
        rc = self.L.rio_scan_span(self.h, ctypes.addressof(buf), len(span), file_off, int(is_file_end), limit_off,
                                  codec, ctypes.byref(out))
        if rc != 0:
            raise RuntimeError("rio_scan_span: " + self.L.rio_last_error().decode())
        out._span_buf = buf  # item views point into it
        return out

    def scan_v1_span(self, span: bytes, file_off: int = 0, is_file_end: bool = True) -> RioBatch:
        """rio_scan_v1_span: the v1 (legacy) records of span (legacyscanner.go:84-117)."""
        out = RioBatch()
        buf = (ctypes.c_char * max(len(span), 1)).from_buffer_copy(bytes(span) or b"\0")
        rc = self.L.rio_scan_v1_span(self.h, ctypes.addressof(buf), len(span), file_off, int(is_file_end),
                                     ctypes.byref(out))
        if rc != 0:
            raise RuntimeError("rio_scan_v1_span: " + self.L.rio_last_error().decode())
        out._span_buf = buf
        return out

    def encode(self, items, items_per_block: int = 0, kind: int = RIO_BLOCK_BODY,
               codec: int = RIO_CODEC_NONE, level: int = 0):
        """rio_encode: the chunk stream of the blocks holding `items` (a list of
        bytes) and each block's offset in it (writerv2.go:388-442, chunk.go:100-141)."""
        import numpy as np
        n = len(items)
        lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=n)
        ends = np.cumsum(lens, dtype=np.uint64) if n else np.zeros(0, dtype=np.uint64)
        blob = b"".join(bytes(x) for x in items)
        return self.encode_arrays(blob, ends, items_per_block, kind, codec, level)

    def encode_arrays(self, blob, ends, items_per_block: int = 0, kind: int = RIO_BLOCK_BODY,
                      codec: int = RIO_CODEC_NONE, level: int = 0):
        """rio_encode over item bytes `blob` (buffer protocol) and exclusive ends."""
        import numpy as np
        ends = np.ascontiguousarray(ends, dtype=np.uint64)
        data = np.frombuffer(blob, dtype=np.uint8) if len(blob) else np.zeros(1, dtype=np.uint8)
        n = int(ends.size)
        per = items_per_block or 16385
        nb = (n + per - 1) // per
        a = RioEncodeArgs(data.ctypes.data, ends.ctypes.data if n else None, n, items_per_block, codec, kind,
                          level, 0)
        err = RioError()
        olen = ctypes.c_uint64()
        boff = np.zeros(max(nb, 1), dtype=np.uint64)
        cap = 32768 * (2 * nb + (len(blob) * 9 // 8 + 11 * (n + nb)) // 32740 + 2)  # >= the chunk stream
        for _ in range(2):
            out = np.empty(cap, dtype=np.uint8)
            rc = self.L.rio_encode(self.h, ctypes.byref(a), out.ctypes.data, cap, ctypes.byref(olen),
                                   boff.ctypes.data, ctypes.byref(err))
            if rc != RIO_ERR_CAPACITY or olen.value <= cap:
                break
            cap = olen.value  # the exact size, once
        if rc < 0:
            raise RuntimeError("rio_encode: " + self.L.rio_last_error().decode())
        if rc != 0:
            raise _err(err)
        return out[:olen.value].tobytes(), [int(x) for x in boff[:nb]]

    def scan_host_ptr(self, host_ptr: int, nbytes: int, file_off: int = 0, is_file_end: bool = True,
                      limit_off: int = U64_MAX, codec: int = RIO_CODEC_NONE) -> RioBatch:
        """rio_scan_span over caller-owned host memory at host_ptr (pinned or
        pageable); item views point into it, so it must outlive the batch."""
        out = RioBatch()
        rc = self.L.rio_scan_span(self.h, host_ptr, nbytes, file_off, int(is_file_end), limit_off, codec,
                                  ctypes.byref(out))
        if rc != 0:
            raise RuntimeError("rio_scan_span: " + self.L.rio_last_error().decode())
        return out

    def scan_device_async(self, dev_ptr: int, nbytes: int, file_off: int = 0, codec: int = RIO_CODEC_NONE):
        rc = self.L.rio_scan_device_async(self.h, dev_ptr, nbytes, file_off, codec)
        if rc != 0:
            raise RuntimeError("rio_scan_device_async: " + self.L.rio_last_error().decode())

    def scan_device_segments_async(self, dev_ptr: int, nbytes: int, seg_end, seg_file_off,
                                   codec: int = RIO_CODEC_NONE):
        """rio_scan_device_segments_async: nseg file bodies back to back at
        dev_ptr (segment s = bytes [seg_end[s-1], seg_end[s]), starting at byte
        seg_file_off[s] of its file); rio_sync's results carry block_segment and
        block_file_off per block."""
        n = len(seg_end)
        e = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in seg_end])
        f = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in seg_file_off])
        rc = self.L.rio_scan_device_segments_async(self.h, dev_ptr, nbytes, e, f, n, codec)
        if rc != 0:
            raise RuntimeError("rio_scan_device_segments_async: " + self.L.rio_last_error().decode())

    def sync(self) -> RioBatch:
        out = RioBatch()
        if self.L.rio_sync(self.h, ctypes.byref(out)) != 0:
            raise RuntimeError("rio_sync: " + self.L.rio_last_error().decode())
        return out

    def stats(self) -> dict:
        """rio_ctx_stats: host spans scanned, bytes copied in and out, device ms,
        and the span the device buffers are sized for now."""
        st = RioStats()
        self.L.rio_ctx_stats(self.h, ctypes.byref(st))
        return {"spans": int(st.spans), "h2d_bytes": int(st.h2d_bytes), "d2h_bytes": int(st.d2h_bytes),
                "device_ms": float(st.device_ms), "span_cap": int(st.span_cap)}

    def flate_split_blocks(self) -> int:
        """Flate blocks of the last completed run copied as segments (split copy pass)."""
        return int(self.L.rio_flate_split_blocks(self.h))

    def stage_times(self):
        """Device ms of the last run: [parse path, codec, k_crc, chunk meta+scans, total]."""
        ms = (ctypes.c_float * 5)()
        n = self.L.rio_stage_times(self.h, ms, 5)
        return [float(ms[i]) for i in range(n)]

    def decode_block(self, payloads, codec: int, cap: int = -1) -> bytes:
        """rio_decode_block, the TransformFunc analogue (recordio.go:12): the
        untransformed block of one block's chunk payloads. Raises RecordioError
        with the codec's error (or RIO_ERR_CAPACITY when cap is too small)."""
        n = len(payloads)
        bufs = [(ctypes.c_char * max(len(p), 1)).from_buffer_copy(bytes(p) or b"\0") for p in payloads]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in bufs])
        lens = (ctypes.c_uint32 * max(n, 1))(*[len(p) for p in payloads])
        if cap < 0:
            cap = max(64 << 10, 16 * sum(len(p) for p in payloads))
        for _ in range(2):
            scratch = ctypes.create_string_buffer(max(cap, 1))
            olen = ctypes.c_uint64()
            err = RioError()
            rc = self.L.rio_decode_block(self.h, ptrs, lens, n, codec, scratch, cap, ctypes.byref(olen),
                                         ctypes.byref(err))
            if rc < 0:
                raise RuntimeError("rio_decode_block: " + self.L.rio_last_error().decode())
            if rc == RIO_ERR_CAPACITY and olen.value > cap:
                cap = olen.value  # like scratch[:cap] too small in the reference: grow once
                continue
            if rc != 0:
                raise _err(err)
            return scratch.raw[:olen.value]
        raise _err(err)

    def scan_device(self, dev_ptr: int, nbytes: int, file_off: int = 0, is_file_end: bool = True,
                    codec: int = RIO_CODEC_NONE) -> RioBatch:
        out = RioBatch()
        rc = self.L.rio_scan_device(self.h, dev_ptr, nbytes, file_off, int(is_file_end), U64_MAX, codec,
                                    ctypes.byref(out))
        if rc != 0:
            raise RuntimeError("rio_scan_device: " + self.L.rio_last_error().decode())
        return out


def batch_items(b: RioBatch) -> List[bytes]:
    """Materialise the items of a host batch (rio_scan_span) as bytes."""
    items = []
    if b.n_items == 0:
        return items
    for i in range(b.n_items):
        o, n = b.item_off[i], b.item_len[i]
        if o & ITEM_IN_RECORDS:
            items.append(ctypes.string_at(b.records + (o & ~ITEM_IN_RECORDS), n) if n else b"")
        else:
            items.append(ctypes.string_at(b.span + o, n) if n else b"")
    return items


def build_id() -> str:
    """rio_build_id() of the loaded library (the tree hash it was built from)."""
    return load().rio_build_id().decode()


def _hip():
    """The process's HIP runtime (the one librio_gpu.so bound: torch's, when imported first)."""
    return ctypes.CDLL("libamdhip64.so.7")


def dev_to_host(ptr: int, nbytes: int) -> bytes:
    """Copy nbytes of device memory to host (test / tooling helper)."""
    if nbytes == 0:
        return b""
    buf = ctypes.create_string_buffer(nbytes)
    H = _hip()
    H.hipDeviceSynchronize()
    rc = H.hipMemcpy(buf, ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed: {rc}")
    return buf.raw


def _dev_u64(ptr, n: int):
    import numpy as np
    return np.frombuffer(dev_to_host(ctypes.cast(ptr, ctypes.c_void_p).value, 8 * n), dtype=np.uint64)


def item_end_views(b: RioBatch):
    """(off, len) item views of an item-end batch (RIO_CFG_ITEM_END), in the
    item_off convention (bit 63: in records), from item_end, block_data,
    block_first_off and block_first_item -- the consumer rule of rio_gpu.h."""
    import numpy as np
    n, nb = int(b.n_items), int(b.n_blocks)
    end = _dev_u64(b.item_end, n).astype(np.int64)
    first = _dev_u64(b.block_first_item, nb + 1).astype(np.int64)
    data = _dev_u64(b.block_data, nb)
    foff = _dev_u64(b.block_first_off, nb).astype(np.int64)
    blk = np.repeat(np.arange(nb), np.diff(first))
    start_in_blk = np.concatenate([[True], np.diff(blk) != 0]) if n else np.zeros(0, bool)
    prev = np.concatenate([[0], end[:-1]]) if n else end
    prev = np.where(start_in_blk, 0, prev)
    s = foff[blk] + prev
    e = foff[blk] + end
    ln = (e - s).astype(np.uint64)
    in_rec = (data[blk] >> np.uint64(63)).astype(bool)
    D = (data[blk] & np.uint64((1 << 63) - 1)).astype(np.int64)
    k = s // 32740
    chunked = D + k * 32768 + 28 + s % 32740
    cross = (~in_rec) & (e - s > 0) & ((e - 1) // 32740 != k)
    off = np.where(in_rec, D + s, chunked).astype(np.uint64)
    off[cross | in_rec] |= np.uint64(ITEM_IN_RECORDS)
    return off, ln


def device_batch_items(b: RioBatch, span_host: bytes) -> List[bytes]:
    """Items of a device batch (rio_scan_device) as bytes; span_host is the span's host copy."""
    import numpy as np
    n = int(b.n_items)
    if n == 0:
        return []
    if b.item_end:
        off, ln = item_end_views(b)
        rec = dev_to_host(b.records, int(b.records_len)) if b.records_len else b""
        out = []
        for o, k in zip(off.tolist(), ln.tolist()):
            if o & ITEM_IN_RECORDS:
                o &= ~ITEM_IN_RECORDS
                out.append(rec[o:o + k])
            else:
                out.append(span_host[o:o + k])
        return out
    off = np.frombuffer(dev_to_host(ctypes.cast(b.item_off, ctypes.c_void_p).value, 8 * n), dtype=np.uint64)
    ln = np.frombuffer(dev_to_host(ctypes.cast(b.item_len, ctypes.c_void_p).value, 8 * n), dtype=np.uint64)
    rec = dev_to_host(b.records, int(b.records_len)) if b.records_len else b""
    out = []
    for o, k in zip(off.tolist(), ln.tolist()):
        if o & ITEM_IN_RECORDS:
            o &= ~ITEM_IN_RECORDS
            out.append(rec[o:o + k])
        else:
            out.append(span_host[o:o + k])
    return out


@dataclasses.dataclass
class ScannerOpts:
    """scannerv2.go:100-111."""
    LegacyTransform: Optional[Callable] = None
    Unmarshal: Optional[Callable] = None


_default_ctx = {}


def default_context(device: int = 0) -> Context:
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device)
        _default_ctx[device] = ctx
    return ctx


class _BytesReader:
    def __init__(self, data):
        self.data = memoryview(data).cast("B") if not isinstance(data, bytes) else data
        self.size = len(data)
        self._keep = (ctypes.c_char * self.size).from_buffer_copy(bytes(self.data)) if self.size else None

        def read_at(user, buf, n, off):
            if off >= self.size:
                return 0
            k = min(n, self.size - off)
            ctypes.memmove(buf, ctypes.addressof(self._keep) + off, k)
            return k
        self.cb = READ_AT(read_at)


class MemorySource:
    """A file held in host memory, read by the library's own reader
    (rio_memory_reader): no Python callback on the read path. `buf` is any
    object with the buffer protocol (bytes, bytearray, numpy array, pinned
    torch tensor via .numpy()); it is kept alive here."""

    def __init__(self, buf):
        import numpy as np
        self._arr = np.frombuffer(buf, dtype=np.uint8)
        self.size = int(self._arr.size)
        self.mem = RioMemory(self._arr.ctypes.data if self.size else None, self.size)


class _FileReader:
    """io.ReaderAt over a file object: os.pread for a plain OS file (raw or
    buffered io.FileIO), else seek + read under a lock (the scanner's
    read-ahead thread and the caller's thread -- Trailer, Gather -- may read at
    once). Wrappers such as gzip.GzipFile or bz2.BZ2File expose the descriptor
    of the compressed file underneath, so they are read through their own
    seek + read, never pread."""

    def __init__(self, f):
        import io
        self.f = f
        f.seek(0, os.SEEK_END)
        self.size = f.tell()
        self._lock = threading.Lock()
        raw = f
        if isinstance(f, (io.BufferedReader, io.BufferedRandom)):
            raw = f.raw
        self._fd = None
        if isinstance(raw, io.FileIO):
            try:
                self._fd = raw.fileno()
            except (OSError, ValueError):
                self._fd = None

        def read_at(user, buf, n, off):
            try:
                if self._fd is not None:
                    b = os.pread(self._fd, n, off)
                else:
                    with self._lock:
                        self.f.seek(off)
                        b = self.f.read(n)
            except Exception:
                return -1
            ctypes.memmove(buf, b, len(b))
            return len(b)
        self.cb = READ_AT(read_at)


class Scanner:
    """Mirror of the recordio.Scanner interface (scannerv2.go:120-161).

    Every scanner owns its staging and result buffers (the C scanner does), so
    scanners sharing one Context never see each other's records. v1 (legacy)
    files decode natively (Version() == 1, legacyscanner.go). A file this
    library does not decode -- a transformer chain / other registered
    transformer (RIO_ERR_FALLBACK) -- reports that code from Err(); the Go shim
    hands such files to recordio.NewShardScanner."""

    def __init__(self, src, opts: ScannerOpts = None, start: int = 0, limit: int = 1, nshard: int = 1,
                 ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self.L = self.ctx.L
        self.opts = opts or ScannerOpts()
        self.unmarshal = self.opts.Unmarshal or (lambda b: b)
        if isinstance(src, MemorySource):  # rio_memory_reader: reads are a memcpy in C (any thread)
            self._rd = src
            self._rr = self.L.rio_memory_reader(ctypes.byref(src.mem))
        else:
            self._rd = _BytesReader(src) if isinstance(src, (bytes, bytearray, memoryview)) else _FileReader(src)
            self._rr = RioReader(None, self._rd.cb, self._rd.size)
        self.h = self.L.rio_scanner_new(self.ctx.h, ctypes.byref(self._rr), start, limit, nshard)
        self._item = None
        self._err = None

    def Header(self) -> List[Tuple[str, object]]:
        out = []
        for i in range(self.L.rio_scanner_header_len(self.h)):
            key = ctypes.c_char_p()
            typ = ctypes.c_int32()
            ival = ctypes.c_int64()
            sval = ctypes.c_void_p()
            slen = ctypes.c_uint64()
            self.L.rio_scanner_header_kv(self.h, i, ctypes.byref(key), ctypes.byref(typ), ctypes.byref(ival),
                                         ctypes.byref(sval), ctypes.byref(slen))
            t = typ.value
            if t == 1:
                v = bool(ival.value)
            elif t == 2:
                v = int(ival.value)
            elif t == 3:
                v = Uint(ival.value & 0xFFFFFFFFFFFFFFFF)
            else:
                v = ctypes.string_at(sval.value, slen.value).decode(errors="surrogateescape") if slen.value else ""
            out.append((key.value.decode(errors="surrogateescape"), v))
        return out

    def Scan(self) -> bool:
        if self._err is not None:  # errors.Once: the first error is sticky (scannerv2.go:242)
            return False
        if not self.L.rio_scanner_scan(self.h):
            return False
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        self.L.rio_scanner_get(self.h, ctypes.byref(p), ctypes.byref(n))
        raw = ctypes.string_at(p.value, n.value) if n.value else b""
        try:
            self._item = self.unmarshal(raw)
        except Exception as e:  # scannerv2.go:396-399
            self._err = e
            return False
        return True

    def ScanBatch(self, max_items: int = 1 << 16) -> List[bytes]:
        """Batched Scan+Get (rio_scanner_next_batch): raw item bytes."""
        ptrs = (ctypes.c_void_p * max_items)()
        lens = (ctypes.c_uint64 * max_items)()
        n = self.L.rio_scanner_next_batch(self.h, ptrs, lens, max_items)
        return [ctypes.string_at(ptrs[i], lens[i]) if lens[i] else b"" for i in range(n)]

    def Get(self):
        return self._item

    def Location(self) -> ItemLocation:
        b = ctypes.c_uint64()
        i = ctypes.c_int64()
        self.L.rio_scanner_location(self.h, ctypes.byref(b), ctypes.byref(i))
        return ItemLocation(b.value, i.value)

    def Err(self) -> Optional[Exception]:
        if self._err is not None:
            return self._err
        e = RioError()
        if self.L.rio_scanner_err(self.h, ctypes.byref(e)) != 0:
            return _err(e)
        return None

    def Seek(self, loc: ItemLocation):
        self.L.rio_scanner_seek(self.h, loc.Block, loc.Item)

    def Gather(self, locs: List[ItemLocation]) -> List[bytes]:
        """rio_scanner_gather: the raw items at locs (as Seek + Scan + Get each),
        their blocks decoded as one batch. Raises RecordioError (with .index,
        the first failing location, and .items, those before it) on the error
        Seek / Scan would set there. The scan position is untouched."""
        n = len(locs)
        blocks = (ctypes.c_uint64 * max(n, 1))(*[int(x.Block) for x in locs])
        items = (ctypes.c_int64 * max(n, 1))(*[int(x.Item) for x in locs])
        ptrs = (ctypes.c_void_p * max(n, 1))()
        lens = (ctypes.c_uint64 * max(n, 1))()
        e = RioError()
        k = self.L.rio_scanner_gather(self.h, blocks, items, n, ptrs, lens, ctypes.byref(e))
        if k < 0:
            raise ValueError("rio_scanner_gather: bad arguments")
        got = [ctypes.string_at(ptrs[i], lens[i]) if lens[i] else b"" for i in range(k)]
        if k < n:
            err = _err(e)
            err.index = k
            err.items = got
            raise err
        return got

    def Trailer(self) -> Optional[bytes]:
        p = ctypes.c_void_p()
        n = ctypes.c_uint64()
        if not self.L.rio_scanner_trailer(self.h, ctypes.byref(p), ctypes.byref(n)):
            return None
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def Version(self) -> int:
        return self.L.rio_scanner_version(self.h)

    def Finish(self) -> Optional[Exception]:
        err = self.Err()
        if self.h:
            self.L.rio_scanner_finish(self.h, None)
            self.h = None
        return err

    def __del__(self):  # pragma: no cover
        try:
            if self.h:
                self.L.rio_scanner_finish(self.h, None)
        except Exception:
            pass


def NewScanner(src, opts: ScannerOpts = None, ctx: Optional[Context] = None) -> Scanner:
    """recordio.NewScanner (scannerv2.go:200)."""
    return Scanner(src, opts, 0, 1, 1, ctx)


def NewShardScanner(src, opts: ScannerOpts, start: int, limit: int, nshard: int,
                    ctx: Optional[Context] = None) -> Scanner:
    """recordio.NewShardScanner (scannerv2.go:211)."""
    return Scanner(src, opts, start, limit, nshard, ctx)
