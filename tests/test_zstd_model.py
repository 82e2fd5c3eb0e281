"""CPU: the host model of the span-level zstd layout (tools/zstd_span_model.py), which the device
writer (kcdc_compress.hip zstd_emit_kernel) restates, decodes through the system libzstd: blocks
of 16 segments with the span's Huffman code carried once and Treeless after, compressed FSE
tables carried once and Repeat_Mode after, and the FSE-compressed Huffman weights description
(two interleaved states, as zstd's HUF_compressWeights)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

zm = pytest.importorskip("zstd_span_model")


def test_fse_compressed_weights_decode():
    zm.check_fse_weights(seed=11)


def test_span_level_blocks_decode():
    from compress_bench import mixed
    data = bytes(mixed(96 << 10, 5))
    for G in (16, 64):
        blob = zm.encode_chunk_t(data, G)
        assert zm.zstd_decode(blob) == data
        assert len(blob) < 0.5 * len(data)
