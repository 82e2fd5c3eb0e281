"""TEST INFRASTRUCTURE ONLY (imported by tests/, __graft_entry__.smoke() and bench.py's checks):
the reference's compression framing for the deflate family, with Python's zlib as the
RFC 1951 inflater/deflater.

Reference (read as text): repo/compression/compressor.go:67-72 (compressionHeader: 4-byte
big-endian header ID), :107-119 (verifyCompressionHeader), compressor_deflate.go:42-78
(Compress = header || flate stream; Decompress = header check, then flate.NewReader),
compression_ids.go:28-30 (IDs), repo/content/content_manager_lock_free.go:64-73 (keep the
compressed form only when it is shorter than the content).

The reference encodes with github.com/klauspost/compress/flate (not vendored, Go absent), so
encoder bytes are not comparable; parity for a compressor is the round trip through an
independent RFC 1951 inflater (zlib here, flate.NewReader in the reference), the header, and the
reference's own test properties (compressor_test.go:15-87: all-zero input shrinks, random input
does not, another compressor's reader rejects the stream).  The gzip family (compressor_gzip.go,
compressor_pgzip.go) is the same stream in an RFC 1952 member.
"""
from __future__ import annotations

import zlib

# compression_ids.go:8-30 (every registered ID; the device encodes the deflate ones)
HEADER_IDS = {
    "gzip": 0x1000, "gzip-best-speed": 0x1001, "gzip-best-compression": 0x1002,
    "zstd": 0x1100, "zstd-fastest": 0x1101, "zstd-better-compression": 0x1102, "zstd-best-compression": 0x1103,
    "s2-default": 0x1200, "s2-better": 0x1201, "s2-parallel-4": 0x1202, "s2-parallel-8": 0x1203,
    "pgzip": 0x1300, "pgzip-best-speed": 0x1301, "pgzip-best-compression": 0x1302,
    "lz4": 0x1400,
    "deflate-default": 0x1500, "deflate-best-speed": 0x1501, "deflate-best-compression": 0x1502,
}
DEFLATE_LEVELS = {"deflate-best-speed": 1, "deflate-default": 6, "deflate-best-compression": 9}
# compressor_gzip.go / compressor_pgzip.go: the same DEFLATE levels inside a gzip member (RFC 1952);
# gzip.NewReader / pgzip.NewReader accept any valid member.
GZIP_LEVELS = {"gzip": 6, "gzip-best-speed": 1, "gzip-best-compression": 9,
               "pgzip": 6, "pgzip-best-speed": 1, "pgzip-best-compression": 9}
LEVELS = {**DEFLATE_LEVELS, **GZIP_LEVELS}


def _wbits(name: str) -> int:
    return 31 if name in GZIP_LEVELS else -15


def header(name: str) -> bytes:
    return HEADER_IDS[name].to_bytes(4, "big")


def compress(name: str, data: bytes) -> bytes:
    """A reference-format stream from zlib's deflater (for ratio comparison, not byte parity)."""
    co = zlib.compressobj(LEVELS[name], zlib.DEFLATED, _wbits(name))
    return header(name) + co.compress(data) + co.flush()


def decompress(name: str, blob: bytes) -> bytes:
    """deflateCompressor.Decompress(withHeader=true): header check, then a raw inflate that must
    consume the whole stream (flate.NewReader reads to the final block).  gzip/pgzip names: the
    member's header, CRC-32 and ISIZE are checked as gzip.NewReader does (zlib, wbits 31)."""
    if blob[:4] != header(name):
        raise ValueError(f"invalid compression header, expected {header(name).hex()} but got {blob[:4].hex()}")
    d = zlib.decompressobj(_wbits(name))
    out = d.decompress(blob[4:]) + d.flush()
    if not d.eof:
        raise ValueError("truncated deflate stream")
    if d.unused_data:
        raise ValueError(f"{len(d.unused_data)} bytes after the final block")
    return out


def kept_header_id(name: str, data_len: int, blob_len: int) -> int:
    """content_manager_lock_free.go:64-73: NoCompression (0) unless the stream is shorter."""
    return HEADER_IDS[name] if blob_len < data_len else 0
