"""On-disk constants and small codecs of the v2 recordio format.

Host-side helpers shared by the writer (encode side) and the scanner mirror.
Every constant cites the reference line it restates.
"""
from __future__ import annotations

import zlib

# recordio/internal/chunk.go:20-29
CHUNK_HEADER_SIZE = 28
CHUNK_SIZE = 32 << 10
MAX_CHUNK_PAYLOAD = CHUNK_SIZE - CHUNK_HEADER_SIZE  # 32740

# recordio/internal/magic.go:15-36
MAGIC_LEGACY_UNPACKED = bytes([0xFC, 0xAE, 0x95, 0x31, 0xF0, 0xD9, 0xBD, 0x20])
MAGIC_PACKED = bytes([0x2E, 0x76, 0x47, 0xEB, 0x34, 0x07, 0x3C, 0x2E])
MAGIC_HEADER = bytes([0xD9, 0xE1, 0xD9, 0x5C, 0xC2, 0x16, 0x04, 0xF7])
MAGIC_TRAILER = bytes([0xFE, 0xBA, 0x1A, 0xD7, 0xCB, 0xDF, 0x75, 0x3A])
MAGIC_INVALID = bytes([0xE4, 0xE7, 0x9A, 0xC1, 0xB3, 0xF6, 0xB7, 0xA2])

# recordio/writerv2.go:17-30
DEFAULT_FLUSH_PARALLELISM = 8
MAX_FLUSH_PARALLELISM = 128
MAX_PACKED_ITEMS = 10 * 1024 * 1024
DEFAULT_PACKED_ITEMS = 16 * 1024

# recordio/header.go:16-25, 39-45
KEY_TRAILER = "trailer"
KEY_TRANSFORMER = "transformer"
HEADER_TYPE_BOOL = 1
HEADER_TYPE_INT = 2
HEADER_TYPE_UINT = 3
HEADER_TYPE_STRING = 4

# chunk.go:77-82: padding pattern of the last chunk of a block
_PAD = (b"\xde\xad\xbe\xef" * ((MAX_CHUNK_PAYLOAD + 3) // 4))[:MAX_CHUNK_PAYLOAD]


class Uint(int):
    """An unsigned header value (Go uint*), kept distinct from a signed int."""

    def __repr__(self) -> str:  # pragma: no cover - cosmetic
        return f"Uint({int(self)})"


def put_uvarint(v: int) -> bytes:
    """encoding/binary.PutUvarint."""
    if v < 0:
        raise ValueError("uvarint of negative value")
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def put_varint(v: int) -> bytes:
    """encoding/binary.PutVarint (zigzag)."""
    ux = (v << 1) & 0xFFFFFFFFFFFFFFFF
    if v < 0:
        ux ^= 0xFFFFFFFFFFFFFFFF
    return put_uvarint(ux)


def uvarint(buf, pos: int = 0):
    """encoding/binary.Uvarint of Go 1.13-1.15 (go.mod:3; CI ci.yml:17).

    Returns (value, n): n > 0 bytes consumed; n == 0 buffer too small;
    n < 0 overflow (-(index of the terminating byte + 1)).
    """
    x = 0
    s = 0
    i = 0
    n = len(buf) - pos
    while i < n:
        b = buf[pos + i]
        if b < 0x80:
            if i > 9 or (i == 9 and b > 1):
                return 0, -(i + 1)
            return (x | (b << s)) & 0xFFFFFFFFFFFFFFFF, i + 1
        x |= (b & 0x7F) << s
        s += 7
        i += 1
    return 0, 0


def crc32_ieee(data) -> int:
    """hash/crc32 IEEE (magic.go:39)."""
    return zlib.crc32(data) & 0xFFFFFFFF


def marshal_header(kvs) -> bytes:
    """ParsedHeader.marshal (header.go:200-209) with headerEncoder (49-136)."""
    out = bytearray()

    def put_uint(v):
        out.append(HEADER_TYPE_UINT)
        out.extend(put_uvarint(v))

    def put_string(s):
        b = s.encode() if isinstance(s, str) else bytes(s)
        out.append(HEADER_TYPE_STRING)
        put_uint(len(b))
        out.extend(b)

    put_uint(len(kvs))
    for key, value in kvs:
        put_string(key)
        if isinstance(value, bool):
            out.append(HEADER_TYPE_BOOL)
            out.append(1 if value else 0)
        elif isinstance(value, Uint):
            put_uint(int(value))
        elif isinstance(value, int):
            out.append(HEADER_TYPE_INT)
            out.extend(put_varint(value))
        elif isinstance(value, (str, bytes)):
            put_string(value)
        else:
            raise TypeError(f"illegal header type {type(value).__name__}")
    return bytes(out)


def packed_block_payload(items) -> bytes:
    """generatePackedHeaderv2 + item bytes (writerv2.go:388-401, 404-441)."""
    hdr = bytearray(put_uvarint(len(items)))
    for it in items:
        hdr.extend(put_uvarint(len(it)))
    return bytes(hdr) + b"".join(bytes(it) for it in items)


def chunk_block(magic: bytes, payload: bytes) -> bytes:
    """ChunkWriter.Write (chunk.go:100-141): split into 32 KiB chunks."""
    out = bytearray()
    n = len(payload)
    # Go's (len-1)/Max + 1 truncates toward zero, so an empty payload is 1 chunk.
    total = (n - 1) // MAX_CHUNK_PAYLOAD + 1 if n > 0 else 1
    pos = 0
    for index in range(total):
        part = payload[pos:pos + MAX_CHUNK_PAYLOAD]
        pos += len(part)
        tail = (0).to_bytes(4, "little") + len(part).to_bytes(4, "little") + \
            total.to_bytes(4, "little") + index.to_bytes(4, "little")
        crc = crc32_ieee(tail + part)
        out += magic + crc.to_bytes(4, "little") + tail + part
        if index == total - 1:
            out += _PAD[:MAX_CHUNK_PAYLOAD - len(part)]
    return bytes(out)


# ------------------------------------------------------------------ v1 (legacy)
# recordio/deprecated/recordio.go:80-86: 8-byte magic, u64 size, crc32 of size
LEGACY_HEADER_SIZE = 20
MAX_READ_RECORD_SIZE = 1 << 29  # recordio/internal/magic.go:33
# recordio/deprecated/packed.go:18-24
LEGACY_DEFAULT_PACKED_ITEMS = 16 * 1024
LEGACY_DEFAULT_PACKED_BYTES = 16 * 1024 * 1024


def legacy_record(magic: bytes, payload: bytes) -> bytes:
    """One v1 record: marshalHeader (deprecated/recordio.go:316-322) + payload."""
    size = len(payload).to_bytes(8, "little")
    return magic + size + crc32_ieee(size).to_bytes(4, "little") + bytes(payload)


def legacy_packed_payload(items) -> bytes:
    """Packer.Pack (deprecated/packer.go:85-133), no transform: crc32 of the
    varint header, item count, item sizes, then the items."""
    hdr = put_uvarint(len(items)) + b"".join(put_uvarint(len(p)) for p in items)
    return crc32_ieee(hdr).to_bytes(4, "little") + hdr + b"".join(bytes(p) for p in items)


def legacy_unpacked_file(items) -> bytes:
    """NewLegacyWriter + Write per item (deprecated/recordio.go:132-142)."""
    return b"".join(legacy_record(MAGIC_LEGACY_UNPACKED, p) for p in items)


def legacy_packed_file(items, max_items: int = LEGACY_DEFAULT_PACKED_ITEMS,
                       max_bytes: int = LEGACY_DEFAULT_PACKED_BYTES) -> bytes:
    """NewLegacyPackedWriter + Write per item + Flush (deprecated/packed.go:
    119-200): a record is flushed before an item that would exceed max_items
    or max_bytes."""
    out, cur, nbytes = [], [], 0
    for p in items:
        if len(p) > max_bytes:
            raise ValueError(f"buffer is too large {len(p)} > {max_bytes}")
        if cur and (nbytes + len(p) > max_bytes or len(cur) + 1 > max_items):
            out.append(legacy_record(MAGIC_PACKED, legacy_packed_payload(cur)))
            cur, nbytes = [], 0
        cur.append(p)
        nbytes += len(p)
    if cur:
        out.append(legacy_record(MAGIC_PACKED, legacy_packed_payload(cur)))
    return b"".join(out)
