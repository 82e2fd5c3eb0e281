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

    def cuts_ids(self) -> list[tuple[int, bytes]]:
        """Final cuts found since the last call with their chunks' content hashes (batchers built
        with hash=...): (cut, digest) in cut order, non-blocking."""
        n = self._buf.size
        ids = np.zeros(n * 32, dtype=np.uint8)
        size = self._b.hash_size
        out: list[tuple[int, bytes]] = []
        while True:
            k = _lib.lib().kcdc_bw_cuts_ids(self._h, self._buf.ctypes.data, ids.ctypes.data, 32, n)
            if k < 0:
                _lib.check(int(k))
            out.extend((int(self._buf[i]), ids[32 * i:32 * i + size].tobytes()) for i in range(k))
            if k < n:
                return out

    def finish(self) -> list[int]:
        """Split the rest (blocks) and return the remaining cuts, the last one = the object size."""
        _lib.check(_lib.lib().kcdc_bw_finish(self._h))
        return self.cuts()

    def finish_ids(self) -> list[tuple[int, bytes]]:
        """finish() for batchers with content IDs: the remaining (cut, digest) pairs."""
        _lib.check(_lib.lib().kcdc_bw_finish(self._h))
        return self.cuts_ids()

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
                 devices: list[int] | None = None, hash: str | None = None, key: bytes = b""):
        import weakref
        self.name = name
        self.hash_size = 0
        self._writers = weakref.WeakSet()
        if devices is None:
            self._h = _lib.lib().kcdc_bw_batcher_new(name.encode(), device, round_bytes, max_wait_us)
        else:
            arr = (C.c_int * max(len(devices), 1))(*devices)
            self._h = _lib.lib().kcdc_bw_batcher_new_devices(name.encode(), arr if devices else None, len(devices),
                                                            round_bytes, max_wait_us)
        if not self._h:
            raise _lib.KcdcError(_lib.KCDC_ENODEV, _lib.last_error())
        if hash is not None:
            kb = (C.c_uint8 * max(len(key), 1)).from_buffer_copy(key or b"\0")
            rc = _lib.lib().kcdc_bw_batcher_hash(self._h, hash.encode(), kb, len(key))
            if rc != 0:
                _lib.lib().kcdc_bw_batcher_free(self._h)
                self._h = None
                _lib.check(rc)
            self.hash_size = int(_lib.check(_lib.lib().kcdc_hash_size(hash.encode())))

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
