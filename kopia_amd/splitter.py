"""Python mirror of Kopia's ``repo/splitter`` package over the native C ABI.

Reference surface (kopia/kopia):
  type Splitter interface { NextSplitPoint([]byte) int; MaxSegmentSize() int; Reset(); Close() }
                                              repo/splitter/splitter.go:20-29
  type Factory func() Splitter                repo/splitter/splitter.go:45
  SupportedAlgorithms() []string              repo/splitter/splitter.go:32-42
  GetFactory(name) Factory                    repo/splitter/splitter.go:84-86 (nil if unknown)
  DefaultAlgorithm                            repo/splitter/splitter.go:89

Every split decision is made by the gfx950 kernels behind libkcdc.so; this
module only marshals arguments.  Method names keep the Go spelling so tests
read like repo/splitter/splitter_test.go.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Callable, Optional

from . import _lib

DefaultAlgorithm: str = "DYNAMIC-4M-BUZHASH"


def SupportedAlgorithms() -> list[str]:
    L = _lib.lib()
    n = L.kcdc_supported_algorithms(None, 0)
    arr = (C.c_char_p * n)()
    L.kcdc_supported_algorithms(arr, n)
    return [x.decode() for x in arr]


def lookup(name: str) -> Optional[_lib.AlgoInfo]:
    info = _lib.AlgoInfo()
    rc = _lib.lib().kcdc_lookup(name.encode(), C.byref(info))
    return info if rc == 0 else None


def custom_algorithm(kind: str, avg: int) -> str:
    """Name for an unregistered parameterisation (the reference tests' direct
    factory calls, e.g. newBuzHash32SplitterFactory(32), splitter_test.go:30)."""
    k = {"fixed": _lib.KIND_FIXED, "buzhash": _lib.KIND_BUZHASH, "rabinkarp": _lib.KIND_RABINKARP}[kind]
    r = _lib.lib().kcdc_custom_algorithm(k, avg)
    if not r:
        raise _lib.KcdcError(_lib.KCDC_EINVAL, _lib.last_error())
    return r.decode()


def max_segment_size(name: str) -> int:
    return _lib.check(_lib.lib().kcdc_max_segment_size(name.encode()))


def cut_capacity(name: str, stream_len: int) -> int:
    return int(_lib.lib().kcdc_cut_capacity(name.encode(), stream_len))


class Splitter:
    """One GPU-backed splitter handle (not thread-safe, like the reference)."""

    def __init__(self, name: str, device: int = 0):
        h = _lib.lib().kcdc_splitter_new(name.encode(), device)
        if not h:
            raise _lib.KcdcError(_lib.KCDC_EINVAL, _lib.last_error())
        self._h = h
        self.name = name

    def NextSplitPoint(self, b) -> int:
        mv = memoryview(b).cast("B")
        n = mv.nbytes
        if n == 0:
            buf = None
        elif mv.readonly:
            buf = C.c_char_p(mv.tobytes())
        else:
            buf = (C.c_char * n).from_buffer(mv)
        r = _lib.lib().kcdc_splitter_next(self._h, C.cast(buf, C.c_void_p) if buf is not None else None, n)
        if r < -1:
            raise _lib.KcdcError(int(r), _lib.last_error())
        return int(r)

    def MaxSegmentSize(self) -> int:
        return int(_lib.lib().kcdc_splitter_max_segment_size(self._h))

    def Reset(self) -> None:
        _lib.lib().kcdc_splitter_reset(self._h)

    def Close(self) -> None:
        if self._h:
            _lib.lib().kcdc_splitter_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.Close()
        except Exception:
            pass


class SplitterGroup:
    """kcdc_group: handles for concurrent object writers whose GPU scans share launches
    (one wave per pending NextSplitPoint call).  Each handle is used by one thread at a
    time, like any Splitter; different handles may be called from different threads."""

    def __init__(self, name: str, device: int = 0, max_batch: int = 0, max_wait_us: int = 0):
        g = _lib.lib().kcdc_group_new(name.encode(), device, max_batch, max_wait_us)
        if not g:
            raise _lib.KcdcError(_lib.KCDC_EINVAL, _lib.last_error())
        self._g = g
        self.name = name
        self._close_mu = threading.Lock()

    def splitter(self) -> Splitter:
        h = _lib.lib().kcdc_group_splitter(self._g)
        if not h:
            raise _lib.KcdcError(_lib.KCDC_EINVAL, _lib.last_error())
        s = Splitter.__new__(Splitter)
        s._h = h
        s.name = self.name
        return s

    def close(self) -> None:
        """Free the group; splitters still open keep working, and the last one to close
        releases it.  Safe to call from several threads (the handle is swapped out under a
        lock, so it is freed once); close() must not race splitter()."""
        with self._close_mu:
            g, self._g = self._g, None
        if g:
            _lib.lib().kcdc_group_free(g)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


Factory = Callable[[], Splitter]


def GetFactory(name: str, device: int = 0) -> Optional[Factory]:
    if lookup(name) is None:
        return None
    return lambda: Splitter(name, device)
