"""Host-side v2 recordio Writer (the encode side).

Mirrors recordio.NewWriter / WriterOpts / Writer (recordio/writerv2.go:47-587)
with the same state machine, header ordering and block layout, but runs
synchronously: the reference's async flush goroutines only reorder work, the
bytes on disk are the same sequence (writerv2.go:447-489 writes in flushSeq
order). It exists to produce test fixtures and the synthetic benchmark files.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional

from . import format as F
from .codecs import make_compressor


@dataclasses.dataclass(frozen=True)
class ItemLocation:
    """writerv2.go:33-39."""
    Block: int
    Item: int


@dataclasses.dataclass
class WriterOpts:
    """writerv2.go:47-109 (MaxFlushParallelism accepted and ignored)."""
    Marshal: Optional[Callable] = None
    Index: Optional[Callable] = None
    Transformers: List[str] = dataclasses.field(default_factory=list)
    MaxItems: int = 0
    MaxFlushParallelism: int = 0
    KeyTrailer: bool = False
    SkipHeader: bool = False
    # Not in the reference: how "flate" terminates its stream ("go" = Writer.Close style).
    FlateStyle: str = "go"


_INITIAL, _BODY, _TRAILER, _FINISHED = range(4)


class Writer:
    def __init__(self, out, opts: WriterOpts = None):
        opts = dataclasses.replace(opts) if opts is not None else WriterOpts()
        if opts.Marshal is None:
            opts.Marshal = lambda v: bytes(v)
        if opts.MaxItems == 0:
            opts.MaxItems = F.DEFAULT_PACKED_ITEMS
        opts.MaxItems = min(opts.MaxItems, F.MAX_PACKED_ITEMS)
        self.opts = opts
        self.out = out
        self.n_written = 0
        self.err: Optional[Exception] = None
        self.header = []
        self.state = _INITIAL
        if opts.SkipHeader:
            self.state = _BODY
        else:
            for t in opts.Transformers:
                self.header.append((F.KEY_TRANSFORMER, t))
        if opts.KeyTrailer:
            self.header.append((F.KEY_TRAILER, True))
        self.cur: Optional[list] = None
        comps = []
        try:
            comps = [make_compressor(t, opts.FlateStyle) for t in opts.Transformers]
        except KeyError as e:  # registry.go:58
            self._set_err(RuntimeError(e.args[0]))

        def transform(b: bytes) -> bytes:
            for c in comps:  # Transformers[0] first (writerv2.go:66-72)
                b = c(b)
            return b
        self.transform = transform

    def _set_err(self, e):
        if self.err is None:
            self.err = e

    def _write_block(self, magic: bytes, payload: bytes):
        data = F.chunk_block(magic, payload)
        self.out.write(data)
        self.n_written += len(data)

    def _flush_header(self):
        self._write_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header(self.header)]))

    def _flush_body(self):
        objs, self.cur = self.cur, None
        items = [bytes(self.opts.Marshal(v)) for v in objs]
        payload = self.transform(F.packed_block_payload(items))
        offset = self.n_written
        if self.err is None:
            self._write_block(F.MAGIC_PACKED, payload)
        if self.opts.Index is not None:
            for i, v in enumerate(objs):
                self.opts.Index(ItemLocation(offset, i), v)

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
        if self.cur is None:
            self.cur = []
        self.cur.append(v)
        # a block's object slice has capacity MaxItems + 1 and is flushed when
        # full (writerv2.go:315, 366-368): MaxItems + 1 items per block
        if len(self.cur) >= self.opts.MaxItems + 1:
            self._flush_body()

    def Flush(self):
        if self.state == _INITIAL:
            return
        if self.state != _BODY:
            raise RuntimeError(f"Flush: wrong state: {self.state}")
        if self.cur is not None:
            self._flush_body()

    def Wait(self):
        pass

    def SetTrailer(self, data: bytes):
        if not _has_trailer(self.header):  # writerv2.go:512-514
            raise RuntimeError("settrailer: Key 'trailer' must be set to true")
        if self.state == _INITIAL:
            self._flush_header()
        elif self.state == _BODY:
            if self.cur is not None:
                self._flush_body()
        else:
            raise RuntimeError(f"SetTrailer: wrong state: {self.state}")
        self.state = _TRAILER
        payload = self.transform(F.packed_block_payload([bytes(data)]))
        self._write_block(F.MAGIC_TRAILER, payload)

    def Err(self):
        return self.err

    def Finish(self):
        if self.state == _INITIAL:
            self._flush_header()
            self.state = _BODY
        if self.state == _BODY:
            if self.cur is not None:
                self._flush_body()
        elif self.state != _TRAILER:
            raise RuntimeError("Finish: wrong state")
        self.state = _FINISHED
        return self.err


def _has_trailer(header) -> bool:
    """ParsedHeader.HasTrailer (header.go:242-254): the first 'trailer' key decides."""
    for k, v in header:
        if k != F.KEY_TRAILER:
            continue
        return v is True
    return False


def NewWriter(out, opts: WriterOpts = None) -> Writer:
    return Writer(out, opts)


def write_file(records, opts: WriterOpts = None, header=(), trailer: Optional[bytes] = None,
               flush_every: int = 0) -> bytes:
    """Convenience: records -> recordio bytes (flush_every = records per block)."""
    import io
    buf = io.BytesIO()
    opts = dataclasses.replace(opts) if opts is not None else WriterOpts()
    if trailer is not None:
        opts.KeyTrailer = True
    w = Writer(buf, opts)
    for k, v in header:
        w.AddHeader(k, v)
    for i, r in enumerate(records):
        w.Append(r)
        if flush_every and (i % flush_every) == flush_every - 1:
            w.Flush()
    if trailer is not None:
        w.SetTrailer(trailer)
    err = w.Finish()
    if err is not None:
        raise err
    return buf.getvalue()
