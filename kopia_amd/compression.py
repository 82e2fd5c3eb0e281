"""Content compression of chunks on the GPU (C ABI: include/kcdc.h, kcdc_compress_*),
mirroring Kopia's compression package for the deflate, gzip, pgzip and s2 compressors
(repo/compression/compressor.go: Compressor, HeaderID, ByName; compressor_deflate.go,
compressor_gzip.go, compressor_pgzip.go, compressor_s2.go; compression_ids.go) and the content manager's keep-or-drop rule
(repo/content/content_manager_lock_free.go:42-73: the compressed form is kept only when it is
shorter than the content, else the header ID is NoCompression = 0).
No CPU fallback for the byte path: the library must be loaded."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

NoCompression = 0  # repo/content/content_manager.go:37
compressionHeaderSize = 4  # compressor.go:15


def SupportedAlgorithms() -> list[str]:
    arr = (C.c_char_p * 64)()
    n = _lib.lib().kcdc_compression_algorithms(arr, 64)
    return [arr[i].decode() for i in range(n)]


def HeaderID(name: str) -> int:
    return _lib.check(_lib.lib().kcdc_compression_header_id(name.encode()))


def compress_bound(length: int) -> int:
    return int(_lib.lib().kcdc_compress_bound(int(length)))


def compressed_layout(lengths):
    """Offsets and total size of an output buffer with room for every chunk's bound."""
    bounds = np.array([compress_bound(int(n)) for n in np.asarray(lengths, dtype=np.int64)], dtype=np.int64)
    offs = np.concatenate(([0], np.cumsum(bounds)[:-1])).astype(np.int64) if len(bounds) else np.zeros(0, np.int64)
    return offs, max(int(bounds.sum()), 1)


class Compressor:
    """ByName[name] for the GPU: the batch form of Compress (plus the content manager's rule)."""

    def __init__(self, name: str):
        if name not in SupportedAlgorithms():
            raise _lib.KcdcError(_lib.KCDC_ENOENT, f"unknown compression algorithm: {name}")
        self.name = name
        self.header_id = HeaderID(name)

    def HeaderID(self) -> int:
        return self.header_id

    def compress_chunks_device(self, data_ptr: int, offsets, lengths, d_out, out_offsets, device, stream=None):
        """Compress chunk i = [offsets[i], +lengths[i]) of the device bytes at data_ptr into d_out
        (a device uint8 tensor) at out_offsets[i] (room for compress_bound(lengths[i]) bytes).
        Returns device tensors (out_lens int64, header_ids int32): header_ids[i] is this
        compressor's ID when the compressed form is shorter than the chunk, else 0.
        Asynchronous on `stream`."""
        import torch
        n = len(offsets)
        if stream is None:
            stream = torch.cuda.current_stream(device)
        lens = np.asarray(lengths, dtype=np.int64)
        # Temporaries are allocated and filled on `stream` itself (the kernels run there), and
        # out_lens / ids need no fill: the frame kernel writes every entry.
        with torch.cuda.stream(stream):
            out_lens = torch.empty(max(n, 1), dtype=torch.int64, device=device)
            ids = torch.empty(max(n, 1), dtype=torch.int32, device=device)
            if n == 0:
                return out_lens[:0], ids[:0]
            d_offs = torch.as_tensor(np.asarray(offsets, dtype=np.int64)).to(device)
            d_lens = torch.as_tensor(lens).to(device)
            d_oo = torch.as_tensor(np.asarray(out_offsets, dtype=np.int64)).to(device)
            wb = int(_lib.lib().kcdc_compress_workspace_size(int(lens.sum()), n))
            work = torch.empty(max(wb, 1), dtype=torch.uint8, device=device)
        _lib.check(_lib.lib().kcdc_compress_chunks_device(
            self.name.encode(), C.c_void_p(data_ptr), d_offs.data_ptr(), d_lens.data_ptr(), n, d_out.data_ptr(),
            d_oo.data_ptr(), out_lens.data_ptr(), ids.data_ptr(), work.data_ptr(), work.numel(),
            C.c_void_p(stream.cuda_stream)))
        out_lens._kcdc_keep = (d_offs, d_lens, d_oo, work)  # alive until the caller syncs
        return out_lens[:n], ids[:n]
