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
DEVICE = DEFLATE + GZIP  # the library's registry order (sorted names)


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
        kc.HeaderID("zstd-fastest")  # registered in the reference, not encoded on the device
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
