"""GPU writer: recordio.NewWriter / Writer (recordio/writerv2.go:47-587) with
the block serialisation, chunk framing and CRC32 on the GPU (rio_encode,
SURVEY.md §8(f) 1).

Same state machine, header order and bytes as the reference for the none
transformer; "flate" blocks are valid DEFLATE streams and "zstd" blocks valid
zstd frames of the same payloads (GPU-encoded, deflate_enc.hip / zstd_enc.hip),
so they decode to the same records. The reference serialises each block on a goroutine as it fills
(MaxItems + 1 items, writerv2.go:315, 366-368) and writes blocks in sequence;
here the items between two block-ending calls (Flush, SetTrailer, Finish) are
kept and encoded by one rio_encode call -- once a run holds `batch_bytes`, its
whole blocks are encoded early -- so thousands of blocks go through one launch.
The Index callback runs after a block's location is known, as in the
reference (writerv2.go:458-470: after serialisation, before the write)."""
from __future__ import annotations

import dataclasses
from typing import Optional

from . import format as F
from . import gpu
from .writer import ItemLocation, WriterOpts, _has_trailer

_INITIAL, _BODY, _TRAILER, _FINISHED = range(4)


class GpuWriter:
    def __init__(self, out, opts: WriterOpts = None, ctx: Optional[gpu.Context] = None,
                 batch_bytes: int = 64 << 20):
        opts = dataclasses.replace(opts) if opts is not None else WriterOpts()
        if opts.Marshal is None:
            opts.Marshal = lambda v: bytes(v)
        if opts.MaxItems == 0:
            opts.MaxItems = F.DEFAULT_PACKED_ITEMS
        opts.MaxItems = min(opts.MaxItems, F.MAX_PACKED_ITEMS)
        # transformers: none, or one "flate" / "flate N" (recordioflate.go:31-52: N = 0
        # stored blocks, 1 fixed Huffman, otherwise dynamic Huffman per 32 KiB, the
        # smaller of dynamic / fixed) or "zstd" / "zstd N" (recordiozstd.go:31-52)
        self.codec, self.level = gpu.RIO_CODEC_NONE, 0
        if opts.Transformers:
            name, _, arg = opts.Transformers[0].partition(" ")
            if len(opts.Transformers) != 1 or name not in ("flate", "zstd"):
                raise ValueError("GpuWriter encodes none or one flate / zstd transformer (got %r)"
                                 % (opts.Transformers,))
            self.codec = gpu.RIO_CODEC_FLATE if name == "flate" else gpu.RIO_CODEC_ZSTD
            self.level = int(arg) if arg.strip() else -1
        self.opts = opts
        self.out = out
        self.ctx = ctx or gpu.default_context()
        self.batch_bytes = batch_bytes
        self.n_written = 0
        self.err: Optional[Exception] = None
        self.header = []
        self.state = _BODY if opts.SkipHeader else _INITIAL
        if not opts.SkipHeader:
            for t in opts.Transformers:
                self.header.append((F.KEY_TRANSFORMER, t))
        if opts.KeyTrailer:
            self.header.append((F.KEY_TRAILER, True))
        self.run_objs = []   # the current run's objects
        self.run_items = []  # ... and their marshalled bytes
        self.run_bytes = 0

    def _write(self, data: bytes):
        self.out.write(data)
        self.n_written += len(data)

    def _encode_run(self, n: int):
        """Encode the first n items of the run (whole blocks unless the run ends)."""
        if n == 0:
            return
        objs, items = self.run_objs[:n], self.run_items[:n]
        del self.run_objs[:n], self.run_items[:n]
        self.run_bytes -= sum(len(x) for x in items)
        per = self.opts.MaxItems + 1
        data, boff = self.ctx.encode(items, per, gpu.RIO_BLOCK_BODY, self.codec, self.level)
        base = self.n_written
        if self.opts.Index is not None:
            for i, v in enumerate(objs):
                self.opts.Index(ItemLocation(base + boff[i // per], i % per), v)
        self._write(data)

    def _flush_header(self):
        data, _ = self.ctx.encode([F.marshal_header(self.header)], 1, gpu.RIO_BLOCK_HEADER)
        self._write(data)

    def AddHeader(self, key: str, value):
        if self.state != _INITIAL:
            raise RuntimeError(f"AddHeader: wrong state: {self.state}")
        self.header.append((key, value))

    def Append(self, v):
        if self.state == _INITIAL:
            self._flush_header()
            self.state = _BODY
        elif self.state != _BODY:
            raise RuntimeError(f"Append: wrong state: {self.state}")
        b = bytes(self.opts.Marshal(v))
        self.run_objs.append(v)
        self.run_items.append(b)
        self.run_bytes += len(b)
        per = self.opts.MaxItems + 1
        if self.run_bytes >= self.batch_bytes and len(self.run_items) >= per:
            self._encode_run(len(self.run_items) // per * per)

    def Flush(self):
        if self.state == _INITIAL:
            return
        if self.state != _BODY:
            raise RuntimeError(f"Flush: wrong state: {self.state}")
        self._encode_run(len(self.run_items))

    def SetTrailer(self, data: bytes):
        if not _has_trailer(self.header):  # writerv2.go:512-514
            raise RuntimeError("settrailer: Key 'trailer' must be set to true")
        if self.state == _INITIAL:
            self._flush_header()
        elif self.state == _BODY:
            self._encode_run(len(self.run_items))
        else:
            raise RuntimeError(f"SetTrailer: wrong state: {self.state}")
        self.state = _TRAILER
        enc, _ = self.ctx.encode([bytes(data)], 1, gpu.RIO_BLOCK_TRAILER, self.codec, self.level)
        self._write(enc)

    def Err(self):
        return self.err

    def Finish(self):
        if self.state == _INITIAL:
            self._flush_header()
            self.state = _BODY
        if self.state == _BODY:
            self._encode_run(len(self.run_items))
        elif self.state != _TRAILER:
            raise RuntimeError("Finish: wrong state")
        self.state = _FINISHED
        return self.err


def NewWriter(out, opts: WriterOpts = None, ctx: Optional[gpu.Context] = None) -> GpuWriter:
    return GpuWriter(out, opts, ctx)
