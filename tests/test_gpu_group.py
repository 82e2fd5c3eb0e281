"""GPU: grouped streaming handles (kcdc_group) under concurrent writers.

Mirrors Kopia's upload: many object writers (snapshot/upload/upload.go:769-782), each
driving its own Splitter with NextSplitPoint over slices (repo/object/object_writer.go:
120-136).  Every writer's chunk boundaries must equal the oracle's for its stream,
whatever the interleaving of the calls that shared a launch."""
import threading
import time

import numpy as np
import pytest

from kopia_amd import splitter as ks
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def write_object(s, data: np.ndarray, slices) -> list:
    """objectWriter.Write over successive slices, then Result(): chunk end offsets."""
    cuts, pos, chunk_start = [], 0, 0
    for k in slices:
        d = data[pos:pos + k]
        base = pos
        pos += len(d)
        while len(d):
            n = s.NextSplitPoint(d)
            if n < 0:
                break
            base += n
            cuts.append(base)
            chunk_start = base
            d = d[n:]
        if pos >= len(data):
            break
    if chunk_start < len(data):
        cuts.append(len(data))
    return cuts


def slice_plan(rng, total, mode):
    out, acc = [], 0
    while acc < total:
        k = 64 << 10 if mode == "64k" else int(rng.integers(1, 256 << 10))
        out.append(k)
        acc += k
    return out


@pytest.mark.parametrize("name", ["DYNAMIC-128K-BUZHASH", "DYNAMIC-128K-RABINKARP", "DYNAMIC-1M-BUZHASH"])
@pytest.mark.parametrize("wait_us", [0, 200])
def test_group_concurrent_writers_match_oracle(name, wait_us):
    nw, L = 12, 6 << 20
    streams = [coracle.gen_stream(SEED, 500 + i, L + 977 * i) for i in range(nw)]
    want = [coracle.split_stream(name, d).tolist() for d in streams]
    g = ks.SplitterGroup(name, 0, max_batch=64, max_wait_us=wait_us)
    got = [None] * nw
    errs = []

    def run(i):
        try:
            rng = np.random.default_rng(i)
            s = g.splitter()
            got[i] = write_object(s, streams[i], slice_plan(rng, len(streams[i]), "64k" if i % 2 else "rand"))
            s.Close()
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(nw)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    g.close()
    assert not errs, errs
    for i in range(nw):
        assert got[i] == want[i], (name, i)


def test_group_throughput_vs_private_handles():
    """Reported, not asserted: 16 writers x 64 KiB slices, grouped vs private handles."""
    name, nw, L = "DYNAMIC-4M-BUZHASH", 16, 24 << 20
    streams = [coracle.gen_stream(SEED, 900 + i, L) for i in range(nw)]
    plans = [[64 << 10] * (L // (64 << 10))] * nw

    def timed(make):
        res = [None] * nw

        def run(i):
            s = make()
            res[i] = write_object(s, streams[i], plans[i])
            s.Close()
        th = [threading.Thread(target=run, args=(i,)) for i in range(nw)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0, res

    g = ks.SplitterGroup(name, 0, max_batch=64, max_wait_us=50)
    tg, rg = timed(g.splitter)
    g.close()
    tp, rp = timed(lambda: ks.Splitter(name))
    assert rg == rp
    print(f"\n{nw} writers x {L >> 20} MiB in 64 KiB slices: grouped {nw * L / tg / 1e9:.2f} GB/s, "
          f"private handles {nw * L / tp / 1e9:.2f} GB/s")


def test_group_freed_before_its_handles():
    """kcdc_group_free with a handle still open defers to that handle's Close; the handle keeps
    working in the meantime."""
    name = "DYNAMIC-128K-BUZHASH"
    data = coracle.gen_stream(SEED, 77, 3 << 20)
    g = ks.SplitterGroup(name, 0)
    s = g.splitter()
    g.close()
    assert write_object(s, data, slice_plan(np.random.default_rng(3), len(data), "64k")) == \
        coracle.split_stream(name, data).tolist()
    s.Close()


def test_group_freed_then_many_handles_close_concurrently():
    """kcdc_group_free with 16 handles open, then 16 threads each write an object through
    their handle and Close it at the same time: the last closer tears the group down while
    the others are still closing (the release path must not touch the group after its
    unlock).  Every writer's cuts equal the oracle's."""
    name, nw = "DYNAMIC-128K-BUZHASH", 16
    streams = [coracle.gen_stream(SEED, 1200 + i, (1 << 20) + 4099 * i) for i in range(nw)]
    want = [coracle.split_stream(name, d).tolist() for d in streams]
    for rep in range(3):
        g = ks.SplitterGroup(name, 0, max_batch=64, max_wait_us=100)
        hs = [g.splitter() for _ in range(nw)]
        g.close()
        got, errs = [None] * nw, []
        go = threading.Barrier(nw)

        def run(i):
            try:
                got[i] = write_object(hs[i], streams[i], slice_plan(np.random.default_rng(rep * 100 + i),
                                                                    len(streams[i]), "64k"))
                go.wait(timeout=60)  # every writer done: close all at once
                hs[i].Close()
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,)) for i in range(nw)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs, errs
        assert got == want
