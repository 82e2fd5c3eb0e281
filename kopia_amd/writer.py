"""Batching object writers (include/kcdc.h "batching object writers").

Kopia's objectWriter.Write (repo/object/object_writer.go:113-139) asks its Splitter for a
cut after every 64 KiB slice.  Here a writer only stages the slice; a batcher ships every
writer's staged bytes to the GPU in one round and the cuts come back later, as final chunk
end offsets.  The sequence of cuts equals one NextSplitPoint pass over the whole object.

    b = WriterBatcher("DYNAMIC-4M-BUZHASH")
    w = b.open()
    w.write(slice)            # any slicing
    ready = w.cuts()          # final cuts so far (flush those chunks)
    rest = w.finish()         # Close/Result: the remaining cuts, ending at the object size
    w.close(); b.close()
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class BatchedWriter:
    """One object's writer (a Splitter's place in objectWriter)."""

    def __init__(self, batcher: "WriterBatcher", size_hint: int = 0):
        self._b = batcher
        self._h = _lib.lib().kcdc_bw_open_hint(batcher._h, size_hint)
        if not self._h:
            raise _lib.KcdcError(_lib.KCDC_EINVAL, _lib.last_error())
        self._buf = np.zeros(1024, dtype=np.uint64)
        batcher._writers.add(self)

    @property
    def device(self) -> int:
        """Position of this writer's device in the batcher's device list."""
        return int(_lib.check(_lib.lib().kcdc_bw_device(self._h)))

    def write(self, data) -> None:
        a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
        _lib.check(_lib.lib().kcdc_bw_write(self._h, a.ctypes.data, a.size))

    def cuts(self) -> list[int]:
        """Final cut offsets found since the last call (non-blocking)."""
        out: list[int] = []
        while True:
            k = _lib.lib().kcdc_bw_cuts(self._h, self._buf.ctypes.data, self._buf.size)
            if k < 0:
                _lib.check(int(k))
            out.extend(int(x) for x in self._buf[:k])
            if k < self._buf.size:
                return out

    def finish(self) -> list[int]:
        """Split the rest (blocks) and return the remaining cuts, the last one = the object size."""
        _lib.check(_lib.lib().kcdc_bw_finish(self._h))
        return self.cuts()

    def close(self) -> None:
        if self._h:
            _lib.lib().kcdc_bw_free(self._h)
            self._h = None
            self._b._writers.discard(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WriterBatcher:
    """kcdc_bw_batcher: one per repository splitter name, over one device or a device set
    (`devices`: device indices, repeats allowed; [] = every device)."""

    def __init__(self, name: str, device: int = 0, round_bytes: int = 0, max_wait_us: int = 0,
                 devices: list[int] | None = None):
        import weakref
        self.name = name
        self._writers = weakref.WeakSet()
        if devices is None:
            self._h = _lib.lib().kcdc_bw_batcher_new(name.encode(), device, round_bytes, max_wait_us)
        else:
            arr = (C.c_int * max(len(devices), 1))(*devices)
            self._h = _lib.lib().kcdc_bw_batcher_new_devices(name.encode(), arr if devices else None, len(devices),
                                                            round_bytes, max_wait_us)
        if not self._h:
            raise _lib.KcdcError(_lib.KCDC_ENODEV, _lib.last_error())

    def open(self, size_hint: int = 0) -> BatchedWriter:
        return BatchedWriter(self, size_hint)

    @property
    def ndevices(self) -> int:
        return int(_lib.lib().kcdc_bw_batcher_devices(self._h))

    def rounds(self) -> int:
        return int(_lib.lib().kcdc_bw_rounds(self._h))

    def close(self) -> None:
        """Free every writer still open (their objects are abandoned), then the batcher."""
        if self._h:
            for w in list(self._writers):
                w.close()
            _lib.lib().kcdc_bw_batcher_free(self._h)
            self._h = None
