"""GPU: batching object writers (kcdc_bw_*) against the oracle.

Concurrent writers feed their objects in 64 KiB slices (snapshot/upload/upload.go:394-407),
random 1-1000 B slices, or whole; the final cuts they collect while writing plus the ones
finish() returns must equal one sequential pass of the reference splitter over each object
(oracle/cdc_oracle.c restates repo/splitter/splitter_buzhash32.go:26-67 and
splitter_rabinkarp64.go:26-67, pinned by TestSplitterStability)."""
import threading

import numpy as np
import pytest

from kopia_amd import _lib
from kopia_amd import splitter as ks
from kopia_amd.writer import WriterBatcher
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


def _feed(w, data, mode, rng):
    got = []
    pos = 0
    while pos < data.size:
        if mode == "64k":
            k = 64 << 10
        elif mode == "rand":
            k = int(rng.integers(1, 1001))
        else:
            k = data.size
        w.write(data[pos:pos + k])
        pos += k
        if rng.random() < 0.05:
            got.extend(w.cuts())
    got.extend(w.finish())
    return got


def _run(name, sizes, modes, round_bytes=0, wait_us=0, sid0=0, devices=None, hints=False):
    b = WriterBatcher(name, round_bytes=round_bytes, max_wait_us=wait_us, devices=devices)
    datas = [coracle.gen_stream(SEED, sid0 + i, int(n)) for i, n in enumerate(sizes)]
    got = [None] * len(sizes)
    placed = [None] * len(sizes)
    errs = []

    def work(i):
        try:
            w = b.open(size_hint=int(sizes[i]) if hints else 0)
            placed[i] = w.device
            got[i] = _feed(w, datas[i], modes[i % len(modes)], np.random.default_rng(i))
            w.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(sizes))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    rounds = b.rounds()
    b.close()
    assert not errs, errs
    for i, d in enumerate(datas):
        want = coracle.split_stream(name, d).tolist()
        assert got[i] == want, f"writer {i} ({modes[i % len(modes)]}, {d.size} B): {len(got[i])} vs {len(want)} cuts"
    if devices is not None:
        _run.placed = placed
    return rounds


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-128K-BUZHASH", "DYNAMIC-1M-RABINKARP",
                                  "DYNAMIC-128K-RABINKARP"])
def test_concurrent_writers_parity(gpu, name):
    rng = np.random.default_rng(11)
    avg = ks.GetFactory(name)().MaxSegmentSize() // 2
    sizes = [int(rng.integers(0, 6 * avg)) for _ in range(12)] + [0, 1, 63, 64, avg // 2 - 1, avg // 2, 2 * avg]
    _run(name, sizes, ["64k", "rand", "whole"])


def test_sixty_four_writers_64k_slices(gpu):
    """The uploader's shape: 64 concurrent writers, 64 KiB slices, several rounds."""
    rounds = _run("DYNAMIC-4M-BUZHASH", [12 << 20] * 48 + [int(x) for x in range(1 << 20, 17 << 20, 1 << 20)],
                  ["64k", "64k", "64k", "rand"], round_bytes=64 << 20)
    assert rounds >= 4


@pytest.mark.parametrize("name", ["DYNAMIC-1M-BUZHASH", "DYNAMIC-1M-RABINKARP"])
def test_objects_one_after_another_reuse_arenas(gpu, name):
    """An uploader opens a writer per object: a freed writer's arenas go to the next one
    (kcdc_bw_free/kcdc_bw_open).  Long objects first, then short ones whose arena still holds the
    previous object's bytes beyond their end, then long again: every object's cuts exact."""
    b = WriterBatcher(name, round_bytes=8 << 20)
    sizes = [9 << 20, 7 << 20, 3000, 0, 65, 1 << 20, (1 << 20) + 17, 5 << 20, 200_000, 11 << 20]
    try:
        for rep in range(2):
            for i, n in enumerate(sizes):
                d = coracle.gen_stream(SEED, 500 + 16 * rep + i, n)
                w = b.open()
                got = _feed(w, d, ["64k", "rand", "whole"][i % 3], np.random.default_rng(i))
                w.close()
                assert got == coracle.split_stream(name, d).tolist(), f"object {rep}/{i} ({n} B)"
    finally:
        b.close()


def test_device_set_two_logical_devices(gpu):
    """kcdc_bw_batcher_new_devices over [0, 0]: two device batchers (own round threads, streams
    and arenas) on the one GPU, 64 writers with size hints spread over both, every object's cuts
    exact (snapshot/upload/upload.go:769-782 drives NumCPU writers; the shim binds every GPU)."""
    rng = np.random.default_rng(21)
    sizes = [int(x) for x in rng.integers(1 << 20, 24 << 20, 64)]
    rounds = _run("DYNAMIC-4M-BUZHASH", sizes, ["64k", "64k", "rand"], round_bytes=64 << 20, devices=[0, 0],
                  hints=True)
    placed = _run.placed
    assert sorted(set(placed)) == [0, 1]
    load = [sum(s for s, p in zip(sizes, placed) if p == d) for d in (0, 1)]
    assert min(load) > 0.6 * max(load), load
    assert rounds >= 4


def test_device_set_rabinkarp_and_all_devices(gpu):
    """The device set with a Rabin-Karp name, and devices=[] (every device of the box)."""
    rng = np.random.default_rng(22)
    sizes = [int(x) for x in rng.integers(0, 6 << 20, 12)]
    _run("DYNAMIC-1M-RABINKARP", sizes, ["64k", "rand"], devices=[0, 0, 0])
    _run("DYNAMIC-1M-BUZHASH", sizes, ["64k"], devices=[])


def test_tiny_rounds_carry_the_tail(gpu):
    """1 MiB rounds force every chunk to span many rounds (device tail carried over)."""
    rounds = _run("DYNAMIC-4M-BUZHASH", [20 << 20, 9 << 20, 3 << 20], ["64k", "rand"], round_bytes=1 << 20,
                  wait_us=50)
    assert rounds >= 20


def test_kat_rows_through_writers(gpu):
    """TestSplitterStability parameterisations (splitter_test.go:30-39) with random slicing."""
    kat = coracle.gorand_read(5, 5_000_000)
    rows = [(1, "buzhash", 32, (124235, 16, 64)), (1, "buzhash", 2048, (1924, 1024, 4096)),
            (2, "rabinkarp", 1024, (3771, 512, 2048))]
    for kind, oname, avg, want in rows:
        name = _lib.lib().kcdc_custom_algorithm(kind, avg).decode()
        b = WriterBatcher(name, round_bytes=1 << 20, max_wait_us=100)
        w = b.open()
        got = _feed(w, kat, "rand" if avg == 2048 else "64k", np.random.default_rng(avg))
        w.close()
        b.close()
        assert got == coracle.split_stream_kind(oname, avg, kat).tolist()
        split = got[:-1]  # the KAT counts NextSplitPoint hits; the last entry is the stream's end
        sizes = np.diff([0] + split)
        assert (len(split), int(sizes.min()), int(sizes.max())) == want


def _aligned_candidate_stops(cuts, limit):
    """Cut positions c at which a round's region can end so that the next round's resume tile
    starts exactly at c: the coordinate of c in the next round's stream (c - tail_pos + tail_pos
    mod 16, tail_pos = previous cut - 64) is a multiple of 128."""
    stops, prev = [], 0
    for c in cuts[:-1]:
        tail = max(prev - 64, 0)
        if (c - (tail & ~15)) % 128 == 0 and c - prev > 0:
            stops.append(c)
            if len(stops) == limit:
                break
        prev = c
    return stops


def test_region_ending_on_a_candidate(gpu):
    """A round whose region ends right after a candidate: its last cut equals the region end, so
    the batcher keeps it open, and the next round must test that last byte again.  Before the fix
    (kcdc_writer.cpp resume) a resume tile starting at the region end skipped it and two
    chunks merged.  Every write here ends at such a cut and is shipped as a round of its own."""
    import time
    kat = coracle.gorand_read(5, 5_000_000)
    for kind, oname, avg in [(1, "buzhash", 32), (1, "buzhash", 1024), (2, "rabinkarp", 32),
                             (2, "rabinkarp", 1024)]:
        name = _lib.lib().kcdc_custom_algorithm(kind, avg).decode()
        want = coracle.split_stream_kind(oname, avg, kat).tolist()
        stops = _aligned_candidate_stops(want, 120)
        assert len(stops) >= 20, (name, len(stops))
        b = WriterBatcher(name, round_bytes=64 << 20, max_wait_us=20)
        w = b.open()
        got, pos = [], 0
        for c in stops + [kat.size]:
            r0 = b.rounds()
            w.write(kat[pos:c])
            pos = c
            t0 = time.monotonic()
            while b.rounds() == r0 and time.monotonic() - t0 < 5:
                time.sleep(0.0002)
            time.sleep(0.001)
            got.extend(w.cuts())
        got.extend(w.finish())
        rounds = b.rounds()
        w.close()
        b.close()
        assert rounds >= len(stops), (name, rounds, len(stops))
        assert got == want, f"{name}: {len(got)} vs {len(want)} cuts, first diff at " + str(
            next((i for i, (x, y) in enumerate(zip(got, want)) if x != y), None))


def test_errors(gpu):
    b = WriterBatcher("DYNAMIC-4M-BUZHASH")
    w = b.open()
    w.write(bytes(1000))
    assert w.finish() == [1000]
    with pytest.raises(_lib.KcdcError):
        w.write(b"x")
    w.close()
    b.close()
    with pytest.raises(_lib.KcdcError):
        WriterBatcher("NO-SUCH-SPLITTER")


# ---- content IDs (kcdc_bw_batcher_hash / kcdc_bw_cuts_ids): every final chunk named on the device
# as the content manager names what the object writer flushes (object_writer.go:186-227 ->
# content_manager.go:812, hashing.go:78-101), checked against hashlib / the hash oracle.
KEY = bytes(range(7, 39))  # a 32-byte repository HMAC secret


def _feed_ids(w, data, mode, rng):
    got = []
    pos = 0
    while pos < data.size:
        k = 64 << 10 if mode == "64k" else int(rng.integers(1, 1001)) if mode == "rand" else data.size
        w.write(data[pos:pos + k])
        pos += k
        if rng.random() < 0.05:
            got.extend(w.cuts_ids())
    got.extend(w.finish_ids())
    return got


def _run_ids(name, sizes, modes, hash_name="BLAKE2B-256-128", key=KEY, round_bytes=0, sid0=0):
    from oracle import hashes
    b = WriterBatcher(name, round_bytes=round_bytes, hash=hash_name, key=key)
    datas = [coracle.gen_stream(SEED, sid0 + i, int(n)) for i, n in enumerate(sizes)]
    got = [None] * len(sizes)
    errs = []

    def work(i):
        try:
            w = b.open()
            got[i] = _feed_ids(w, datas[i], modes[i % len(modes)], np.random.default_rng(i))
            w.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(sizes))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    rounds = b.rounds()
    b.close()
    assert not errs, errs
    for i, d in enumerate(datas):
        want = coracle.split_stream(name, d).tolist()
        assert [c for c, _ in got[i]] == want, f"writer {i}: cuts"
        prev = 0
        for c, h in got[i]:
            assert h == hashes.kopia_hash(hash_name, key, d[prev:c].tobytes()), f"writer {i}: chunk [{prev}, {c})"
            prev = c
    return rounds


def test_ids_sixty_four_writers(gpu):
    """The uploader's shape with content IDs on: 64 writers in 64 KiB slices, BLAKE2B-256-128 (the
    repository default), every chunk's ID equal to hashlib's keyed BLAKE2b truncated to 16 bytes."""
    rounds = _run_ids("DYNAMIC-4M-BUZHASH", [12 << 20] * 48 + [int(x) for x in range(1 << 20, 17 << 20, 1 << 20)],
                      ["64k", "64k", "64k", "rand"], round_bytes=64 << 20)
    assert rounds >= 4


@pytest.mark.parametrize("hash_name", ["BLAKE2B-256", "BLAKE2S-128", "BLAKE2S-256", "BLAKE3-256-128",
                                       "HMAC-SHA256-128"])
def test_ids_every_kind(gpu, hash_name):
    """Sliced chains (BLAKE2b, BLAKE2s) and whole-chunk steps (BLAKE3, HMAC-SHA256), with empty,
    tiny and block-edge objects."""
    rng = np.random.default_rng(31)
    sizes = [int(x) for x in rng.integers(0, 5 << 20, 6)] + [0, 1, 127, 128, 129, 64 << 10]
    _run_ids("DYNAMIC-1M-BUZHASH", sizes, ["64k", "rand", "whole"], hash_name=hash_name, round_bytes=8 << 20)


def test_ids_kat_rows_and_rabinkarp(gpu):
    """The KAT parameterisations' many small chunks (TestSplitterStability, splitter_test.go:30-39)
    and a Rabin-Karp name, with an unkeyed and a 64-byte key."""
    kat = coracle.gorand_read(5, 5_000_000)
    from oracle import hashes
    for kind, avg, key in [(1, 2048, b""), (2, 1024, bytes(range(64)))]:
        name = _lib.lib().kcdc_custom_algorithm(kind, avg).decode()
        b = WriterBatcher(name, round_bytes=1 << 20, max_wait_us=100, hash="BLAKE2B-256-128", key=key)
        w = b.open()
        got = _feed_ids(w, kat, "rand", np.random.default_rng(avg))
        w.close()
        b.close()
        want = coracle.split_stream_kind("buzhash" if kind == 1 else "rabinkarp", avg, kat).tolist()
        assert [c for c, _ in got] == want
        prev = 0
        for c, h in got:
            assert h == hashes.kopia_hash("BLAKE2B-256-128", key, kat[prev:c].tobytes())
            prev = c


def test_ids_errors(gpu):
    b = WriterBatcher("DYNAMIC-4M-BUZHASH", hash="BLAKE2B-256-128", key=KEY)
    w = b.open()
    w.write(bytes(1000))
    with pytest.raises(_lib.KcdcError):
        w.cuts()  # cuts come with their IDs when IDs are on
    assert [c for c, _ in w.finish_ids()] == [1000]
    w.close()
    with pytest.raises(_lib.KcdcError):  # IDs must be chosen before the first writer opens
        _lib.check(_lib.lib().kcdc_bw_batcher_hash(b._h, b"BLAKE2B-256-128", None, 0))
    b.close()
    with pytest.raises(_lib.KcdcError):
        WriterBatcher("FIXED-4M", hash="BLAKE2B-256-128", key=KEY)
    with pytest.raises(_lib.KcdcError):
        WriterBatcher("DYNAMIC-4M-BUZHASH", hash="NO-SUCH-HASH", key=KEY)


@pytest.mark.parametrize("hash_name", ["BLAKE2B-256-128", "BLAKE3-256-128"])
def test_ids_ring_wraps_under_backpressure(gpu, hash_name):
    """An ID ring far smaller than the data (KCDC_TEST_ID_RING = 24 MiB): chunks wrap around its
    end, rounds wait for ring space while the hash thread names the chains ahead of them, and chain
    slots are reused; every ID must still match hashlib's, in order.  Small averages (many chunks,
    many publishes) and one long object whose chunks reach the 2 MiB maximum."""
    lib = _lib.lib()
    assert lib.kcdc_test_set(_lib.TEST_ID_RING, 24 << 20) == 0
    try:
        sizes = [24 << 20] * 6 + [int(x) for x in np.random.default_rng(3).integers(1, 8 << 20, 10)]
        _run_ids("DYNAMIC-1M-BUZHASH", sizes, ["64k", "rand"], hash_name=hash_name, round_bytes=4 << 20, sid0=900)
    finally:
        lib.kcdc_test_set(_lib.TEST_ID_RING, 0)
