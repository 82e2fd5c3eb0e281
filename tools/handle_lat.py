"""Per-call latency of a private streaming handle whose every call reaches the test range
(random bytes, huge max: nearly every call scans its whole slice and finds nothing), with the
resident scan server on and off.  Not a parity test (tests/test_gpu_server.py is)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from kopia_amd import _lib
    from kopia_amd import splitter as ks
    L = _lib.lib()
    name = "DYNAMIC-8M-BUZHASH"  # min 4 MiB: first skip it, then every call scans
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    out = []
    for slice_kib in (64, 256, 1024):
        for off in (0, 1):
            L.kcdc_test_set(_lib.TEST_NO_SERVER, off)
            s = ks.GetFactory(name)()
            mv = memoryview(data)
            s.NextSplitPoint(mv[:(4 << 20) - 1])  # the fast path: no GPU
            i, calls, t_gpu = (4 << 20) - 1, 0, 0.0
            S = slice_kib << 10
            while i + S <= len(data) and calls < 300:
                t0 = time.perf_counter()
                r = s.NextSplitPoint(mv[i:i + S])
                t_gpu += time.perf_counter() - t0
                calls += 1
                if r != -1:
                    s.Close()
                    s = ks.GetFactory(name)()
                    s.NextSplitPoint(mv[i:i + (4 << 20) - 1]) if i + (4 << 20) < len(data) else None
                    i += 4 << 20
                    continue
                i += S
            s.Close()
            out.append({"slice_kib": slice_kib, "server": not off, "calls": calls,
                        "us_per_call": round(t_gpu / calls * 1e6, 1),
                        "gb_s": round(calls * S / t_gpu / 1e9, 3)})
    L.kcdc_test_set(_lib.TEST_NO_SERVER, 0)
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
