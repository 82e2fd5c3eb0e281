"""Content hashes of chunks on the GPU (C ABI: include/kcdc.h, kcdc_hash_*), mirroring
Kopia's hashing registry for the keyed BLAKE2 family (repo/hashing/hashing.go:41-101,
blake_hashes.go:8-13): a hash function of a chunk is HashFunc(output, data) keyed with the
repository's HMAC secret, truncated to 16 or 32 bytes.  Many chunks per launch: one lane
per chunk.  No CPU fallback: the library must be loaded."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

DefaultAlgorithm = "BLAKE2B-256-128"  # repo/hashing/hashing.go:51


def SupportedAlgorithms() -> list[str]:
    arr = (C.c_char_p * 16)()
    n = _lib.lib().kcdc_hash_algorithms(arr, 16)
    return [arr[i].decode() for i in range(n)]


def hash_size(name: str) -> int:
    return _lib.check(_lib.lib().kcdc_hash_size(name.encode()))


def chunk_table(stream_offsets, cut_lists):
    """(offsets, lens) of every chunk of streams laid out at stream_offsets (bytes from a
    common base), from their cut lists (chunk end offsets, the last one = stream length)."""
    offs, lens = [], []
    for base, cuts in zip(stream_offsets, cut_lists):
        c = np.asarray(cuts, dtype=np.int64)
        starts = np.concatenate(([0], c[:-1])) if c.size else c
        offs.append(int(base) + starts)
        lens.append(c - starts)
    if not offs:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(offs).astype(np.int64), np.concatenate(lens).astype(np.int64)


def hash_chunks_device(name: str, data_ptr: int, offsets, lengths, key: bytes, device, stream=None,
                       order: bool = True):
    """Hash chunk i = [offsets[i], offsets[i] + lengths[i]) of the device bytes at data_ptr.
    offsets/lengths: host arrays (int64).  Returns a device uint8 tensor [n, hash_size]
    (asynchronous on `stream`).  order: process chunks by descending length."""
    import torch
    n = len(offsets)
    size = hash_size(name)
    stride = (size + 3) & ~3
    out = torch.empty((max(n, 1), stride), dtype=torch.uint8, device=device)
    if n == 0:
        return out[:0, :size]
    lens = np.asarray(lengths, dtype=np.int64)
    d_offs = torch.as_tensor(np.asarray(offsets, dtype=np.int64)).to(device)
    d_lens = torch.as_tensor(lens).to(device)
    d_order = None
    if order:
        d_order = torch.as_tensor(np.argsort(-lens, kind="stable").astype(np.int32)).to(device)
    if stream is None:
        stream = torch.cuda.current_stream(device)
    _lib.check(_lib.lib().kcdc_hash_chunks_device(
        name.encode(), C.c_void_p(data_ptr), d_offs.data_ptr(), d_lens.data_ptr(),
        d_order.data_ptr() if d_order is not None else None, n, bytes(key), len(key), out.data_ptr(), stride,
        C.c_void_p(stream.cuda_stream)))
    out._kcdc_keep = (d_offs, d_lens, d_order)  # alive until the caller syncs
    return out[:, :size]
