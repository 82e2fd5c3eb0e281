"""GPU: the resident scan server behind private streaming handles (kcdc_splitter_next ->
server_scan_first, kcdc_kernels.hip scan_server_kernel).  Cuts must be identical with the
server on and off and equal the oracle's, across the server's idle exit and relaunch, scratch
growth to whole-chunk slices, and concurrent handles (the busy server falls back to a launch)."""
import threading
import time

import numpy as np
import pytest

from kopia_amd import _lib
from kopia_amd import splitter as ks
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def _feed(name, data, slices):
    s = ks.GetFactory(name)()
    cuts, i, k = [], 0, 0
    n = len(data)
    mv = memoryview(data)
    while i < n:
        num = min(slices[k % len(slices)], n - i)
        k += 1
        r = s.NextSplitPoint(mv[i:i + num])
        if r == -1:
            i += num
            continue
        i += r
        cuts.append(i)
    if not cuts or cuts[-1] != n:
        cuts.append(n)
    s.Close()
    return cuts


@pytest.fixture
def server(request):
    L = _lib.lib()
    yield L
    L.kcdc_test_set(_lib.TEST_NO_SERVER, 0)


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-1M-RABINKARP", "DYNAMIC-128K-BUZHASH"])
def test_server_on_off_oracle(gpu, server, name):
    data = coracle.gen_stream(SEED, 11, 24 << 20).tobytes()
    want = coracle.split_stream(name, np.frombuffer(data, np.uint8)).tolist()
    for off in (0, 1):
        server.kcdc_test_set(_lib.TEST_NO_SERVER, off)
        before = server.kcdc_test_server_requests()
        assert _feed(name, data, [64 << 10, 1000, 300000, 7]) == want, ("no_server", off)
        served = server.kcdc_test_server_requests() - before
        assert (served > 0) if off == 0 else (served == 0), (off, served)  # the path under test ran


def test_server_idle_relaunch(gpu, server):
    """The server exits after ~2 ms without requests; later calls relaunch it transparently."""
    name = "DYNAMIC-128K-BUZHASH"
    data = coracle.gen_stream(SEED, 12, 4 << 20).tobytes()
    want = coracle.split_stream(name, np.frombuffer(data, np.uint8)).tolist()
    s = ks.GetFactory(name)()
    cuts, i = [], 0
    mv = memoryview(data)
    while i < len(data):
        num = min(96 << 10, len(data) - i)
        r = s.NextSplitPoint(mv[i:i + num])
        time.sleep(0.004)  # past the idle limit: every call finds the server gone
        if r == -1:
            i += num
            continue
        i += r
        cuts.append(i)
    s.Close()
    if not cuts or cuts[-1] != len(data):
        cuts.append(len(data))
    assert cuts == want
    assert server.kcdc_test_server_requests() > 0


def test_server_scratch_growth(gpu, server):
    """Slices from 1 KiB up to whole 16 MiB (more than max_size): the server's scratch grows
    (the running server is drained first)."""
    name = "DYNAMIC-8M-BUZHASH"
    data = coracle.gen_stream(SEED, 13, 64 << 20).tobytes()
    want = coracle.split_stream(name, np.frombuffer(data, np.uint8)).tolist()
    assert _feed(name, data, [1 << 10, 64 << 10, 5 << 20, 16 << 20]) == want


def test_server_concurrent_handles(gpu, server):
    """Eight writers with private handles at once: with more than one private handle open the
    scans are launched side by side instead of queueing on the one-workgroup server; every
    writer's cuts equal the oracle's."""
    name = "DYNAMIC-1M-BUZHASH"
    streams = [coracle.gen_stream(SEED, 20 + w, 12 << 20).tobytes() for w in range(8)]
    wants = [coracle.split_stream(name, np.frombuffer(d, np.uint8)).tolist() for d in streams]
    got = [None] * 8

    def run(w):
        got[w] = _feed(name, streams[w], [64 << 10, 33333])

    th = [threading.Thread(target=run, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == wants
