"""CPU: the compression oracle (oracle/deflate.py) and the library's compression registry.
The oracle's framing follows repo/compression/compressor.go:67-119 and compressor_deflate.go;
its inflater is Python's zlib (an independent RFC 1951 implementation).  The header IDs are
compression_ids.go:8-30 and the names compressor_*.go's RegisterCompressor calls."""
import zlib

import numpy as np
import pytest

from kopia_amd import _lib
from kopia_amd import compression as kc
from oracle import deflate

DEFLATE = ["deflate-best-compression", "deflate-best-speed", "deflate-default"]
GZIP = ["gzip", "gzip-best-compression", "gzip-best-speed", "pgzip", "pgzip-best-compression", "pgzip-best-speed"]
S2 = list(deflate.S2_NAMES)
ZSTD = ["zstd", "zstd-best-compression", "zstd-better-compression", "zstd-fastest"]
DEVICE = DEFLATE + GZIP + S2 + ZSTD  # the library's registry order (sorted within each family)


def test_header_ids_match_reference():
    # compression_ids.go:28-30
    assert deflate.HEADER_IDS["deflate-default"] == 0x1500
    assert deflate.HEADER_IDS["deflate-best-speed"] == 0x1501
    assert deflate.HEADER_IDS["deflate-best-compression"] == 0x1502
    assert len(set(deflate.HEADER_IDS.values())) == len(deflate.HEADER_IDS)
    # compression_ids.go:8-10, 19-21 (gzip, pgzip)
    assert [deflate.HEADER_IDS[n] for n in GZIP] == [0x1000, 0x1002, 0x1001, 0x1300, 0x1302, 0x1301]


def test_library_registry():
    assert kc.SupportedAlgorithms() == DEVICE
    for name in DEVICE:
        assert kc.HeaderID(name) == deflate.HEADER_IDS[name]
    with pytest.raises(_lib.KcdcError):
        kc.HeaderID("lz4")  # registered in the reference (deprecated), not encoded on the device
    with pytest.raises(_lib.KcdcError):
        kc.Compressor("no-such-compressor")


def test_bound():
    """4-byte header ID + final block (2) + a gzip member's header and trailer (18), plus the
    input and 5 bytes per 512-byte segment (a stored block's header)."""
    assert kc.compress_bound(0) == 24
    assert kc.compress_bound(1) == 30
    assert kc.compress_bound(512) == 24 + 512 + 5
    assert kc.compress_bound(513) == 24 + 513 + 10
    assert kc.compress_bound(1 << 20) == 24 + (1 << 20) + 5 * 2048


@pytest.mark.parametrize("name", DEVICE)
def test_oracle_round_trip_and_properties(name):
    """compressor_test.go:15-87 on the oracle: zeros shrink, random does not, other headers fail."""
    zeros = bytes(10000)
    blob = deflate.compress(name, zeros)
    assert len(blob) < len(zeros)
    assert deflate.decompress(name, blob) == zeros
    for other in DEVICE:
        if other != name:
            with pytest.raises(ValueError):
                deflate.decompress(other, blob)
    rnd = np.random.default_rng(1).integers(0, 256, 10000, dtype=np.uint8).tobytes()
    blob = deflate.compress(name, rnd)
    assert len(blob) >= len(rnd)
    assert deflate.kept_header_id(name, len(rnd), len(blob)) == 0
    assert deflate.decompress(name, blob) == rnd


def test_oracle_rejects_truncated_and_trailing():
    blob = deflate.compress("deflate-default", b"abc" * 100)
    with pytest.raises(ValueError):
        deflate.decompress("deflate-default", blob[:-1])
    with pytest.raises(ValueError):
        deflate.decompress("deflate-default", blob + b"\x00")


def test_sync_flush_segments_concatenate():
    """The device format: fixed-Huffman or stored segments, each ending byte-aligned (a sync
    flush), then an empty final block 03 00 -- one valid RFC 1951 stream."""
    parts = [b"hello " * 50, bytes(300), np.random.default_rng(2).integers(0, 256, 200, dtype=np.uint8).tobytes()]
    stream = b""
    for p in parts:
        co = zlib.compressobj(6, zlib.DEFLATED, -15, 9, zlib.Z_FIXED)
        seg = co.compress(p) + co.flush(zlib.Z_SYNC_FLUSH)
        assert seg.endswith(b"\x00\x00\xff\xff")
        stream += seg
    stream += b"\x03\x00"
    assert deflate.decompress("deflate-default", deflate.header("deflate-default") + stream) == b"".join(parts)


def _s2_chunk(block: bytes, data: bytes, kind: int = 0) -> bytes:
    import struct
    c = deflate.crc32c(data)
    m = (((c >> 15) | (c << 17)) + 0xa282ead8) & 0xFFFFFFFF
    body = struct.pack("<I", m) + (block if kind == 0 else data)
    return bytes([kind]) + struct.pack("<I", len(body))[:3] + body


def test_s2_oracle_decoder():
    """oracle/s2_oracle.c (the S2 compressors' reader, restated from the Snappy framing and block
    formats): CRC-32C check value, literals of every length form, copy-1/-2/-4, uncompressed and
    padding chunks decode; a wrong CRC, a missing stream identifier and an S2 repeat code are
    rejected."""
    import struct
    assert deflate.crc32c(b"123456789") == 0xE3069283  # CRC-32C (Castagnoli) check value
    sid = b"\xff\x06\x00\x00S2sTwO"
    lit = bytes(range(256)) * 2
    block = bytes([0x80, 0x04])  # uvarint 512 + 15 + 64 = 591 -> filled below
    data = lit[:300] + lit[:300][-4:] * 3 + lit[:64]
    body = bytes([61 << 2]) + struct.pack("<H", 299) + lit[:300]       # literal, 2-byte length
    body += bytes([1 | ((8 - 4) << 2) | (0 << 5), 4])                  # copy-1: len 8, offset 4
    body += bytes([3 | ((4 - 1) << 2)]) + struct.pack("<I", 4)         # copy-4: len 4, offset 4
    body += bytes([2 | ((64 - 1) << 2)]) + struct.pack("<H", 312)      # copy-2: len 64, offset 312
    n = len(data)
    block = bytes([n & 127 | 128, n >> 7]) + body
    stream = sid + _s2_chunk(block, data) + b"\xfe\x02\x00\x00\x00\x00" + _s2_chunk(b"", b"raw!", 1)
    assert deflate.s2_decode(stream) == data + b"raw!"
    with pytest.raises(ValueError):
        deflate.s2_decode(stream[10:])  # no stream identifier
    bad = bytearray(stream)
    bad[14] ^= 1  # the masked CRC of the first chunk
    with pytest.raises(ValueError):
        deflate.s2_decode(bytes(bad))
    rep = bytes([8, 3 << 2]) + b"abcd" + bytes([1 | (0 << 2), 0])      # copy-1 offset 0 (S2 repeat)
    with pytest.raises(ValueError):
        deflate.s2_decode(sid + _s2_chunk(rep, b"abcdabcd"))


def test_s2_snappy_reader_agrees_with_the_oracle_reader():
    """The second S2 reader (`deflate.s2_decode_snappy`: the framing parsed in Python, each block
    decoded by Google's Snappy library through pyarrow) against the C oracle reader, over the
    oracle's own S2 writer on text-like, periodic, zero and random data."""
    pytest.importorskip("pyarrow")
    rng = np.random.default_rng(9)
    words = [b"kopia", b"snapshot", b"content", b" ", b"\n", b"index"]
    text = b"".join(words[int(k)] for k in rng.integers(0, len(words), 60000))
    for data in (text, bytes(100000), (b"0123456789" * 20000), rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()):
        stream = deflate.s2_encode(data)
        assert deflate.s2_decode(stream) == data
        assert deflate.s2_decode_snappy(stream) == data
