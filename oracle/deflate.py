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
# compressor_s2.go:20-23: s2.NewWriter streams; the decoder is oracle/s2_oracle.c (restated from the
# Snappy framing + block formats; klauspost/compress is not vendored), format parity only.
S2_NAMES = ("s2-better", "s2-default", "s2-parallel-4", "s2-parallel-8")
# compressor_zstd.go:15-18: klauspost zstd.NewWriter at SpeedFastest / SpeedDefault / SpeedBetterCompression /
# SpeedBestCompression (roughly zstd levels 1 / 3 / 7 / 11); the reader is zstd.NewReader.  The oracle's
# independent RFC 8878 decoder is the system libzstd (libzstd.so.1, the C reference implementation).
ZSTD_LEVELS = {"zstd": 3, "zstd-best-compression": 11, "zstd-better-compression": 7, "zstd-fastest": 1}
ZSTD_NAMES = tuple(ZSTD_LEVELS)
_ZSTD = None


def _zstd():
    global _ZSTD
    if _ZSTD is None:
        import ctypes as C
        L = C.CDLL("libzstd.so.1")
        L.ZSTD_decompress.restype = C.c_size_t
        L.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.ZSTD_compress.restype = C.c_size_t
        L.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int]
        L.ZSTD_compressBound.restype = C.c_size_t
        L.ZSTD_compressBound.argtypes = [C.c_size_t]
        L.ZSTD_isError.restype = C.c_uint
        L.ZSTD_isError.argtypes = [C.c_size_t]
        L.ZSTD_getErrorName.restype = C.c_char_p
        L.ZSTD_getErrorName.argtypes = [C.c_size_t]
        L.ZSTD_getFrameContentSize.restype = C.c_ulonglong
        L.ZSTD_getFrameContentSize.argtypes = [C.c_char_p, C.c_size_t]
        _ZSTD = L
    return _ZSTD


def zstd_decode(stream: bytes) -> bytes:
    """zstd.NewReader over whole frames (every block checked; trailing bytes rejected)."""
    import ctypes as C
    L = _zstd()
    cap = L.ZSTD_getFrameContentSize(stream, len(stream))
    if cap >= (1 << 63):  # unknown (0xFF..FF) or error (0xFF..FE): the device always writes the size
        raise ValueError("zstd frame without a content size")
    out = C.create_string_buffer(max(int(cap), 1))
    n = L.ZSTD_decompress(out, int(cap), stream, len(stream))
    if L.ZSTD_isError(n):
        raise ValueError(f"invalid zstd stream: {L.ZSTD_getErrorName(n).decode()}")
    return out.raw[:n]


def zstd_encode(data: bytes, level: int) -> bytes:
    import ctypes as C
    L = _zstd()
    cap = L.ZSTD_compressBound(len(data))
    out = C.create_string_buffer(cap)
    n = L.ZSTD_compress(out, cap, data, len(data), level)
    if L.ZSTD_isError(n):
        raise ValueError(L.ZSTD_getErrorName(n).decode())
    return out.raw[:n]


def s2_decode(stream: bytes) -> bytes:
    """s2.NewReader over a framed stream: stream identifier, CRC-32C of every chunk checked."""
    import ctypes as C

    from oracle import coracle
    L = coracle.lib()
    L.orc_s2_decode.restype = C.c_int64
    L.orc_s2_decode.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_int64]
    cap = 4 * len(stream) + (1 << 16)
    while True:
        out = C.create_string_buffer(cap)
        n = L.orc_s2_decode(stream, len(stream), out, cap)
        if n == -11 or n == -6:  # a block larger than the room left: retry bigger
            cap *= 8
            continue
        if n < 0:
            raise ValueError(f"invalid S2 stream (oracle error {n})")
        return out.raw[:n]


def s2_encode(data: bytes) -> bytes:
    """A plain S2 stream writer (for the oracle's own round-trip properties, not byte parity with
    s2.NewWriter): stream identifier, 64 KiB framing chunks, greedy 4-byte-hash LZ77 emitting
    Snappy literal / copy-2 elements (the subset the device emits too)."""
    import struct
    out = [b"\xff\x06\x00\x00S2sTwO"]
    for c0 in range(0, len(data), 1 << 16):
        blk = data[c0:c0 + (1 << 16)]
        n = len(blk)
        body = bytearray()
        v = n
        while True:
            body.append((v & 127) | (128 if v >= 128 else 0))
            v >>= 7
            if not v:
                break
        tab, i, lit = {}, 0, 0

        def literal(a, b):
            while a < b:
                k = min(b - a, 65536)
                body.extend(bytes([61 << 2]) + struct.pack("<H", k - 1) + blk[a:a + k])
                a += k
        while i + 4 <= n:
            key = blk[i:i + 4]
            q = tab.get(key, -1)
            tab[key] = i
            if q >= 0:
                m = 4
                while i + m < n and blk[q + m] == blk[i + m]:
                    m += 1
                literal(lit, i)
                left = m
                while left:
                    k = min(left, 64)
                    body.extend(bytes([2 | ((k - 1) << 2)]) + struct.pack("<H", i - q))
                    left -= k
                i += m
                lit = i
            else:
                i += 1
        literal(lit, n)
        c = crc32c(blk)
        masked = (((c >> 15) | (c << 17)) + 0xa282ead8) & 0xFFFFFFFF
        payload = struct.pack("<I", masked) + bytes(body)
        out.append(b"\x00" + struct.pack("<I", len(payload))[:3] + payload)
    return b"".join(out)


def s2_decode_snappy(stream: bytes) -> bytes:
    """A second, independent reader for the S2 streams the device writes: the framing format is
    parsed here and every compressed chunk's block is decoded by Google's Snappy library (through
    pyarrow's codec), which the device's blocks must satisfy since they use only Snappy elements
    (literals, copy-1, copy-2; no S2 repeat codes).  CRCs are checked by `s2_decode`, not here."""
    import pyarrow as pa

    codec = pa.Codec("snappy")
    out, i = [], 0
    while i < len(stream):
        if i + 4 > len(stream):
            raise ValueError("truncated chunk header")
        t = stream[i]
        n = int.from_bytes(stream[i + 1:i + 4], "little")
        body = stream[i + 4:i + 4 + n]
        if len(body) != n:
            raise ValueError("truncated chunk")
        if t == 0xFF:
            if body != b"S2sTwO":
                raise ValueError(f"bad stream identifier {body!r}")
        elif t == 0x00:
            blk = body[4:]
            size, shift, j = 0, 0, 0
            while True:  # the block's uvarint uncompressed length
                b = blk[j]
                size |= (b & 0x7F) << shift
                shift += 7
                j += 1
                if b < 0x80:
                    break
            out.append(codec.decompress(blk, decompressed_size=size, asbytes=True))
        elif t == 0x01:
            out.append(body[4:])
        elif t < 0x80:
            raise ValueError(f"reserved chunk type {t:#x}")
        i += 4 + n
    return b"".join(out)


def crc32c(data: bytes) -> int:
    import ctypes as C

    from oracle import coracle
    L = coracle.lib()
    L.orc_crc32c.restype = C.c_uint32
    L.orc_crc32c.argtypes = [C.c_char_p, C.c_int64]
    return int(L.orc_crc32c(data, len(data)))


def _wbits(name: str) -> int:
    return 31 if name in GZIP_LEVELS else -15


def header(name: str) -> bytes:
    return HEADER_IDS[name].to_bytes(4, "big")


def compress(name: str, data: bytes) -> bytes:
    """A reference-format stream from zlib's deflater, libzstd, or the oracle's S2 writer (for ratio
    comparison and the oracle's own properties, not byte parity)."""
    if name in S2_NAMES:
        return header(name) + s2_encode(data)
    if name in ZSTD_NAMES:
        return header(name) + zstd_encode(data, ZSTD_LEVELS[name])
    co = zlib.compressobj(LEVELS[name], zlib.DEFLATED, _wbits(name))
    return header(name) + co.compress(data) + co.flush()


def decompress(name: str, blob: bytes) -> bytes:
    """deflateCompressor.Decompress(withHeader=true): header check, then a raw inflate that must
    consume the whole stream (flate.NewReader reads to the final block).  gzip/pgzip names: the
    member's header, CRC-32 and ISIZE are checked as gzip.NewReader does (zlib, wbits 31)."""
    if blob[:4] != header(name):
        raise ValueError(f"invalid compression header, expected {header(name).hex()} but got {blob[:4].hex()}")
    if name in S2_NAMES:
        return s2_decode(blob[4:])
    if name in ZSTD_NAMES:
        return zstd_decode(blob[4:])
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
