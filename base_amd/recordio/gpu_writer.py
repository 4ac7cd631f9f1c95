"""GPU writer: recordio.NewWriter / Writer (recordio/writerv2.go:47-587) with
the block serialisation, chunk framing and CRC32 on the GPU (rio_encode,
SURVEY.md §8(f) 1).

Same state machine, header order and bytes as the reference for the none
transformer; "flate" blocks are valid DEFLATE streams and "zstd" blocks valid
zstd frames of the same payloads (GPU-encoded, deflate_enc.hip / zstd_enc.hip),
so they decode to the same records. The reference serialises each block on a goroutine as it fills
(MaxItems + 1 items, writerv2.go:315, 366-368) and writes blocks in sequence;
here the items between two block-ending calls (Flush, SetTrailer, Finish) are
kept and encoded by rio_encode calls of up to `batch_bytes` of whole blocks
each -- once a run holds `batch_bytes`, its whole blocks are encoded early -- so
thousands of blocks go through one launch. Errors stick as the reference's
errors.Once does: an unknown transformer name or a config that does not parse
(NewWriter sets them on err, writerv2.go:318-320), or a flate level outside
[-2, 9] (the first transformed block), stops every later write and is reported
by Err() / Finish(). Transformer chains (2-4 of flate / zstd) encode in one
rio_encode call per batch (RIO_CODEC_CHAIN: each stage re-reads the previous
stage's payloads).
The Index callback runs after a block's location is known, as in the
reference (writerv2.go:458-470: after serialisation, before the write)."""
from __future__ import annotations

import dataclasses
import re
from typing import Optional

from . import format as F
from . import gpu
from .writer import ItemLocation, WriterOpts, _has_trailer

_INITIAL, _BODY, _TRAILER, _FINISHED = range(4)
_ATOI = re.compile(r"[+-]?[0-9]+\Z")


def _atoi(config: str) -> int:
    """Go's strconv.Atoi (decimal, optional sign), as recordioflate.Init and
    recordiozstd.parseConfig parse a transformer's config
    (recordioflate.go:76-81, recordiozstd.go:19-25)."""
    if not _ATOI.match(config):
        raise RuntimeError('strconv.Atoi: parsing "%s": invalid syntax' % config)
    v = int(config)
    if not -(1 << 63) <= v < (1 << 63):
        raise RuntimeError('strconv.Atoi: parsing "%s": value out of range' % config)
    return v


class GpuWriter:
    def __init__(self, out, opts: WriterOpts = None, ctx: Optional[gpu.Context] = None,
                 batch_bytes: int = 64 << 20):
        opts = dataclasses.replace(opts) if opts is not None else WriterOpts()
        if opts.Marshal is None:
            opts.Marshal = lambda v: bytes(v)
        if opts.MaxItems == 0:
            opts.MaxItems = F.DEFAULT_PACKED_ITEMS
        opts.MaxItems = min(opts.MaxItems, F.MAX_PACKED_ITEMS)
        self.opts = opts
        self.out = out
        self.ctx = ctx or gpu.default_context()
        self.batch_bytes = batch_bytes
        self.n_written = 0
        self.err: Optional[Exception] = None
        # transformers (registry.go:75-111, applied in order at writerv2.go:432-441):
        # none, or 1-4 of "flate" / "flate N" (recordioflate.go:31-52: N = 0 stored
        # blocks, 1 fixed Huffman, otherwise dynamic Huffman per 32 KiB, the smaller
        # of dynamic / fixed) and "zstd" / "zstd N" (recordiozstd.go:31-52); two or
        # more are one RIO_CODEC_CHAIN encode, stage k transforming stage k - 1's
        # output. As NewWriter does (writerv2.go:318-320), a name the registry does
        # not hold or a config that does not parse is set on err, not raised.
        self.codec, self.level = gpu.RIO_CODEC_NONE, 0
        self.stages = []  # (codec, level) per transformer
        for t in opts.Transformers:
            name, _, arg = t.partition(" ")  # registry.go:54-64: split on the first space
            if name not in ("flate", "zstd"):
                self._set_err(RuntimeError("Transformer %s not found" % t))
                break
            level = -1
            if arg:
                try:  # strconv.Atoi of the config (recordioflate.go:76-81, recordiozstd.go:19-25)
                    level = _atoi(arg)
                except RuntimeError as e:
                    self._set_err(e)
                    break
            self.stages.append((gpu.RIO_CODEC_FLATE if name == "flate" else gpu.RIO_CODEC_ZSTD, level))
        if self.err is None and len(self.stages) > 4:
            self._set_err(RuntimeError("GpuWriter: at most 4 transformers encode on the GPU (got %d)"
                                       % len(self.stages)))
        if self.err is None and len(self.stages) == 1:
            self.codec, self.level = self.stages[0]
        elif self.err is None and self.stages:
            self.codec = gpu.codec_chain(*[c for c, _ in self.stages])
            self.level = 0
            for k, (_, lv) in enumerate(self.stages):  # stage k's level: a signed byte (rio_gpu.h)
                self.level |= (max(-128, min(127, lv)) & 0xFF) << (8 * k)
            if self.level >= 1 << 31:
                self.level -= 1 << 32  # (int32)
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

    def _set_err(self, e):
        if self.err is None:  # errors.Once: the first error sticks
            self.err = e

    def _transform_err(self):
        """The error klauspost's flate.NewWriter returns on the first block a
        transform runs on (recordioflate.go:31-34: levels outside
        [HuffmanOnly, BestCompression] = [-2, 9]); in a chain, the first flate
        stage that has one (the stages run in order)."""
        for codec, level in self.stages:
            if codec == gpu.RIO_CODEC_FLATE and not -2 <= level <= 9:
                return RuntimeError("flate: invalid compression level %d: want value in range [-2, 9]" % level)
        return None

    def _write(self, data: bytes):
        if self.err is None:  # flushBlock writes only while no error is set (writerv2.go:491-495)
            self.out.write(data)
            self.n_written += len(data)

    def _encode_blocks(self, items, per: int, kind: int):
        """rio_encode of whole blocks; the error sticks (serializeBlock's fq.err.Set)."""
        if self.err is None and kind != gpu.RIO_BLOCK_HEADER:
            e = self._transform_err()
            if e is not None:
                self._set_err(e)
        if self.err is not None:
            return None, None
        try:
            return self.ctx.encode(items, per, kind, self.codec if kind != gpu.RIO_BLOCK_HEADER else
                                   gpu.RIO_CODEC_NONE, self.level)
        except gpu.RecordioError as e:
            self._set_err(e)
            return None, None

    def _encode_run(self, n: int):
        """Encode the first n items of the run (whole blocks unless the run ends),
        one rio_encode call per group of whole blocks of at most batch_bytes (a
        single larger block alone). The run keeps its items until they are
        encoded (or the writer's error is set)."""
        per = self.opts.MaxItems + 1
        done = 0
        while done < n:
            # whole blocks while the group stays within batch_bytes (at least one)
            end, nbytes = done, 0
            while end < n:
                blk = self.run_items[end:min(end + per, n)]
                b = sum(len(x) for x in blk)
                if end > done and nbytes + b > self.batch_bytes:
                    break
                nbytes += b
                end = min(end + per, n)
            objs, items = self.run_objs[done:end], self.run_items[done:end]
            data, boff = self._encode_blocks(items, per, gpu.RIO_BLOCK_BODY)
            base = self.n_written
            if self.opts.Index is not None:  # called even after an error, as flushBlock does
                for i, v in enumerate(objs):
                    off = base + boff[i // per] if boff is not None else base
                    self.opts.Index(ItemLocation(off, i % per), v)
            if data is not None:
                self._write(data)
            done = end
        del self.run_objs[:n], self.run_items[:n]
        self.run_bytes = sum(len(x) for x in self.run_items)

    def _flush_header(self):
        data, _ = self._encode_blocks([F.marshal_header(self.header)], 1, gpu.RIO_BLOCK_HEADER)
        if data is not None:
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
        enc, _ = self._encode_blocks([bytes(data)], 1, gpu.RIO_BLOCK_TRAILER)
        if enc is not None:
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
