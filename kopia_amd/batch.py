"""Batch (hot-path) entry points over the C ABI, for device-resident torch tensors
and for host buffers.  PyTorch is used only for device memory and streams."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .splitter import cut_capacity


@dataclass
class DeviceBatch:
    """Device-resident batch layout: streams at arbitrary device addresses."""
    ptrs: "torch.Tensor"       # int64 [n] device pointers (on device)
    lens: "torch.Tensor"       # int64 [n] (on device)
    cut_base: "torch.Tensor"   # int64 [n] (on device)
    cuts: "torch.Tensor"       # int64 [cap] (on device)
    counts: "torch.Tensor"     # int64 [n] (on device)
    cap: int
    n: int


def make_device_batch(name: str, ptr_list, len_list, device) -> DeviceBatch:
    import torch
    n = len(ptr_list)
    caps = np.array([cut_capacity(name, int(L)) for L in len_list], dtype=np.int64)
    base = np.zeros(n, dtype=np.int64)
    if n > 1:
        base[1:] = np.cumsum(caps)[:-1]
    cap = int(caps.sum()) if n else 0
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64)).to(device)
    return DeviceBatch(ptrs=t(ptr_list), lens=t(len_list), cut_base=t(base),
                       cuts=torch.zeros(max(cap, 1), dtype=torch.int64, device=device),
                       counts=torch.zeros(max(n, 1), dtype=torch.int64, device=device), cap=cap, n=n)


def split_batch_device(name: str, b: DeviceBatch, stream=None) -> None:
    """Launch the splitter on the batch (asynchronous on `stream`, torch's current stream if None)."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(b.cuts.device)
    _lib.check(_lib.lib().kcdc_split_batch_device(
        name.encode(), b.ptrs.data_ptr(), b.lens.data_ptr(), b.n, b.cuts.data_ptr(), b.cap,
        b.cut_base.data_ptr(), b.counts.data_ptr(), C.c_void_p(stream.cuda_stream)))


def check_counts(counts: np.ndarray) -> None:
    """Raise if the launch that produced `counts` failed on the device (KCDC_COUNT_FAILED)."""
    if counts.size and (counts.view(np.uint64) == np.uint64(_lib.COUNT_FAILED)).any():
        raise _lib.KcdcError(_lib.KCDC_EIO, "batch launch failed on the device (KCDC_COUNT_FAILED)")


def read_cuts(b: DeviceBatch) -> list[np.ndarray]:
    """Copy cut lists back (host); raises on capacity overflow."""
    cuts = b.cuts.cpu().numpy()
    counts = b.counts.cpu().numpy()[:b.n]
    base = b.cut_base.cpu().numpy()
    check_counts(counts)
    out = []
    for i in range(b.n):
        capi = (base[i + 1] if i + 1 < b.n else b.cap) - base[i]
        if counts[i] > capi:
            raise _lib.KcdcError(_lib.KCDC_EOVERFLOW, f"stream {i}: {counts[i]} cuts > capacity {capi}")
        out.append(cuts[base[i]:base[i] + counts[i]].copy())
    return out


def split_batch_host(name: str, streams, device: int = 0) -> list[np.ndarray]:
    """Host buffers in, cut lists out (H2D + kernel + D2H inside the library)."""
    arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else np.ascontiguousarray(s)
            for s in streams]
    n = len(arrs)
    lens = np.array([a.size for a in arrs], dtype=np.uint64)
    caps = np.array([cut_capacity(name, int(L)) for L in lens], dtype=np.uint64)
    base = np.zeros(n, dtype=np.uint64)
    if n > 1:
        base[1:] = np.cumsum(caps)[:-1]
    cap = int(caps.sum())
    cuts = np.zeros(max(cap, 1), dtype=np.uint64)
    counts = np.zeros(max(n, 1), dtype=np.uint64)
    ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    _lib.check(_lib.lib().kcdc_split_batch_host(
        name.encode(), C.cast(ptrs, C.c_void_p), lens.ctypes.data, n, cuts.ctypes.data, cap, base.ctypes.data,
        counts.ctypes.data, device))
    return [cuts[int(base[i]):int(base[i]) + int(counts[i])].astype(np.int64) for i in range(n)]


def split_batch_host_devices(name: str, streams, devices=None) -> list[np.ndarray]:
    """split_batch_host over a device set (None or []: every device; repeats allowed): the streams
    are spread over the devices by bytes (lpt_assign), each device splits its share."""
    arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else np.ascontiguousarray(s)
            for s in streams]
    n = len(arrs)
    lens = np.array([a.size for a in arrs], dtype=np.uint64)
    caps = np.array([cut_capacity(name, int(L)) for L in lens], dtype=np.uint64)
    base = np.zeros(n, dtype=np.uint64)
    if n > 1:
        base[1:] = np.cumsum(caps)[:-1]
    cap = int(caps.sum())
    cuts = np.zeros(max(cap, 1), dtype=np.uint64)
    counts = np.zeros(max(n, 1), dtype=np.uint64)
    ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    devs = list(devices or [])
    darr = (C.c_int * max(len(devs), 1))(*devs)
    _lib.check(_lib.lib().kcdc_split_batch_host_devices(
        name.encode(), C.cast(darr, C.c_void_p) if devs else None, len(devs), C.cast(ptrs, C.c_void_p),
        lens.ctypes.data, n, cuts.ctypes.data, cap, base.ctypes.data, counts.ctypes.data))
    return [cuts[int(base[i]):int(base[i]) + int(counts[i])].astype(np.int64) for i in range(n)]


def lpt_assign(lens, ndev: int) -> np.ndarray:
    """kcdc_lpt_assign: device position of every stream (largest first to the least loaded)."""
    a = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    out = np.zeros(max(a.size, 1), dtype=np.uint32)
    _lib.check(_lib.lib().kcdc_lpt_assign(a.ctypes.data, a.size, ndev, out.ctypes.data))
    return out[:a.size]


def fill_prng(data: "torch.Tensor", stream_len: int, nstreams: int, stride: int, seed: int, first_sid: int = 0,
              stream=None) -> None:
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(data.device)
    assert data.numel() * data.element_size() >= stride * (nstreams - 1) + stream_len
    _lib.check(_lib.lib().kcdc_fill_prng(data.data_ptr(), stride, stream_len, nstreams, seed, first_sid,
                                         C.c_void_p(stream.cuda_stream)))


def split_long_device(name: str, data_ptr: int, length: int, device, stream=None):
    """Exact intra-stream parallel CDC of ONE device-resident stream (config 3).
    Returns (cuts tensor on device, count tensor on device); cuts[:count] valid."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(device)
    cap = cut_capacity(name, length)
    ws_bytes = int(_lib.lib().kcdc_long_workspace_bytes(name.encode(), length))
    ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=device)
    cuts = torch.zeros(max(cap, 1), dtype=torch.int64, device=device)
    count = torch.zeros(1, dtype=torch.int64, device=device)
    _lib.check(_lib.lib().kcdc_split_long_device(
        name.encode(), data_ptr, length, cuts.data_ptr(), cap, count.data_ptr(), ws.data_ptr(), ws.numel(),
        C.c_void_p(stream.cuda_stream)))
    return cuts, count, ws


def read_long(cuts, count) -> np.ndarray:
    n = int(count.item())
    if n > cuts.numel():
        raise _lib.KcdcError(_lib.KCDC_EOVERFLOW, f"{n} cuts > capacity {cuts.numel()}")
    return cuts[:n].cpu().numpy()


def split_files_device(name: str, ptr_list, len_list, device, stream=None):
    """Streams of any sizes (config 5): each goes to the batch or the long-stream path,
    whichever finishes it sooner (kcdc_split_files_device).  Asynchronous on `stream`.
    Returns (cuts, counts, cut_base, cap) with cuts/counts on the device."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(device)
    n = len(ptr_list)
    lens = np.ascontiguousarray(np.asarray(len_list, dtype=np.uint64))
    caps = np.array([cut_capacity(name, int(L)) for L in lens], dtype=np.uint64)
    base = np.zeros(max(n, 1), dtype=np.uint64)
    if n > 1:
        base[1:n] = np.cumsum(caps)[:-1]
    cap = int(caps.sum()) if n else 0
    ptrs = np.ascontiguousarray(np.asarray(ptr_list, dtype=np.uint64))
    cuts = torch.zeros(max(cap, 1), dtype=torch.int64, device=device)
    counts = torch.zeros(max(n, 1), dtype=torch.int64, device=device)
    _lib.check(_lib.lib().kcdc_split_files_device(
        name.encode(), ptrs.ctypes.data, lens.ctypes.data, n, cuts.data_ptr(), cap, base.ctypes.data,
        counts.data_ptr(), C.c_void_p(stream.cuda_stream)))
    return cuts, counts, base[:n].astype(np.int64), cap


def read_files(cuts, counts, base, cap) -> list[np.ndarray]:
    """Cut lists of split_files_device (host); raises on capacity overflow."""
    c = cuts.cpu().numpy()
    k = counts.cpu().numpy()[:len(base)]
    check_counts(k)
    out = []
    for i in range(len(base)):
        capi = (base[i + 1] if i + 1 < len(base) else cap) - base[i]
        if k[i] > capi:
            raise _lib.KcdcError(_lib.KCDC_EOVERFLOW, f"stream {i}: {k[i]} cuts > capacity {capi}")
        out.append(c[base[i]:base[i] + k[i]].copy())
    return out


def gorand_read(seed: int, n: int) -> np.ndarray:
    """Go ``rand.New(rand.NewSource(seed)).Read`` of n bytes (the library's host restatement;
    input generator of ``kopia benchmark splitter``)."""
    out = np.empty(max(n, 1), dtype=np.uint8)
    _lib.check(_lib.lib().kcdc_gorand_read(seed, out.ctypes.data, n))
    return out[:n]
