"""Host-side checks of the product library (CPU only, no GPU needed): it loads,
exports every symbol include/kcdc.h declares, its registry matches the
reference's, and its independently derived hash tables match the golden ones."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden
from kopia_amd import _lib
from kopia_amd import splitter as ks
from oracle import splitter_ref as ref


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "kcdc.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(kcdc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), f"libkcdc.so does not export {s}"
    assert sorted(_lib.exported_symbols()) == syms


def test_supported_algorithms_match_reference():
    assert ks.SupportedAlgorithms() == ref.supported_algorithms()
    assert _lib.lib().kcdc_default_algorithm().decode() == ref.DEFAULT_ALGORITHM == ks.DefaultAlgorithm


@pytest.mark.parametrize("name", ref.supported_algorithms())
def test_lookup_params(name):
    kind, size = ref.REGISTRY[name]
    info = ks.lookup(name)
    assert info is not None
    assert info.kind == {"fixed": 0, "buzhash": 1, "rabinkarp": 2}[kind]
    assert info.avg == size
    if kind == "fixed":
        assert (info.min_size, info.max_size, info.mask) == (size, size, 0)
    else:
        assert (info.min_size, info.max_size, info.mask) == (size // 2, 2 * size, size - 1)
    # pooled(...) everywhere except the two legacy names (splitter.go:75-80)
    assert info.pooled == (0 if name in ("FIXED", "DYNAMIC") else 1)
    assert ks.max_segment_size(name) == (size if kind == "fixed" else 2 * size)


def test_max_segment_invariants():
    """gather chunk allocator (internal/gather/gather_write_buffer_chunk_test.go:69-81)
    and gRPC message limit (repo/grpc_repository_client_test.go:14-26)."""
    for name in ks.SupportedAlgorithms():
        m = ks.max_segment_size(name)
        assert m <= (16 << 20) + 128 - 128
        assert m <= (20 << 20) - 1024


def test_unknown_name():
    assert ks.GetFactory("nosuchsplitter") is None
    assert ks.lookup("nosuchsplitter") is None
    with pytest.raises(_lib.KcdcError):
        ks.max_segment_size("nosuchsplitter")


def test_custom_algorithm_names():
    a = ks.custom_algorithm("buzhash", 32)
    assert a == ks.custom_algorithm("buzhash", 32)
    assert a not in ks.SupportedAlgorithms()
    assert ks.max_segment_size(a) == 64
    assert ks.max_segment_size(ks.custom_algorithm("fixed", 1000)) == 1000
    with pytest.raises(_lib.KcdcError):
        ks.custom_algorithm("buzhash", 1000)  # not a power of two


def test_cut_capacity():
    assert ks.cut_capacity("DYNAMIC-4M-BUZHASH", 4 << 20) == 3
    assert ks.cut_capacity("FIXED-1M", 1441792) == 2


def test_tables_match_golden():
    buz = (C.c_uint32 * 256)()
    pol = C.c_uint64()
    out = (C.c_uint64 * 256)()
    mod = (C.c_uint64 * 256)()
    assert _lib.lib().kcdc_tables(buz, C.byref(pol), out, mod) == 0
    g = golden("tables.json")
    assert [f"{x:08x}" for x in buz] == g["buzhash"]
    assert hex(pol.value) == g["rabin_pol"]
    assert [f"{x:016x}" for x in out] == g["rabin_out"]
    assert [f"{x:016x}" for x in mod] == g["rabin_mod"]


def test_gpu_entry_points_fail_loudly_without_device():
    if _lib.lib().kcdc_device_count() > 0:
        pytest.skip("a gfx950 device is present")
    # no silent CPU fallback: a dynamic splitter cannot be created without the GPU
    with pytest.raises(_lib.KcdcError):
        ks.Splitter("DYNAMIC-4M-BUZHASH")
    data = np.zeros(10, dtype=np.uint8)
    from kopia_amd import batch
    with pytest.raises(_lib.KcdcError):
        batch.split_batch_host("DYNAMIC-4M-BUZHASH", [data])


def test_fixed_streaming_handle_needs_no_device():
    """FIXED reads no data (splitter_fixed.go:15-26): pure host arithmetic."""
    s = ks.GetFactory("FIXED-128K")()
    data = bytes(300000)
    assert s.MaxSegmentSize() == 128 << 10
    assert s.NextSplitPoint(data[:100000]) == -1
    assert s.NextSplitPoint(data[100000:]) == (128 << 10) - 100000
    s.Close()


def test_group_needs_device_and_rolling_name():
    """kcdc_group_new: unknown names and FIXED are refused; without a gfx950 device it fails
    loudly (no CPU fallback)."""
    L = _lib.lib()
    assert not L.kcdc_group_new(b"NO-SUCH-SPLITTER", 0, 0, 0)
    assert not L.kcdc_group_new(b"FIXED-4M", 0, 0, 0)
    if L.kcdc_device_count() == 0:
        with pytest.raises(_lib.KcdcError):
            ks.SplitterGroup("DYNAMIC-4M-BUZHASH")


def test_fixed_batched_writer_needs_no_device():
    """kcdc_bw_* with a FIXED name: cuts every chunkLength (splitter_fixed.go:15-26), the trailing
    chunk at finish, whatever the slicing; no device involved."""
    from kopia_amd.writer import WriterBatcher
    b = WriterBatcher("FIXED-128K")
    w = b.open()
    rng = np.random.default_rng(3)
    n, got = 0, []
    while n < 1_000_000:
        k = int(rng.integers(1, 70000))
        w.write(bytes(k))
        n += k
        got.extend(w.cuts())
    got.extend(w.finish())
    w.close()
    b.close()
    step = 128 << 10
    assert got == list(range(step, n + 1, step)) + ([n] if n % step else [])


def test_product_build_has_no_wrong_output_ablations():
    """The timing ablations (KCDC_EXP_COMPONLY / _MEMONLY, KCDC_RK_ABL, KCDC_CRYPT_ABL) make the
    kernels cut or encrypt wrongly; the shipped library must have none compiled in."""
    v = _lib.lib().kcdc_version().decode()
    assert v.endswith("ablations=none"), v


def _greedy(hints, writes, ndev):
    """The batcher's assignment rule: each new writer goes to the device with the least load,
    load = sum over its open writers of max(size hint, bytes written) (ties: the lowest index)."""
    load = [0] * ndev
    got = []
    for h, wr in zip(hints, writes):
        d = min(range(ndev), key=lambda i: (load[i], i))
        got.append(d)
        load[d] += max(h, wr)
    return got


def test_writer_device_assignment():
    """kcdc_bw_batcher_new_devices: writers land on the least-loaded device of the set, by size
    hint and bytes written (host logic; FIXED names read no data, so no GPU is involved)."""
    from kopia_amd.writer import WriterBatcher
    rng = np.random.default_rng(3)
    hints = [int(x) for x in rng.integers(0, 50 << 20, 40)]
    writes = [int(x) for x in rng.integers(0, 50 << 20, 40)]
    hints[5] = 0
    b = WriterBatcher("FIXED-4M", devices=[0, 0, 0])
    assert b.ndevices == 3
    ws, devs = [], []
    for h, wr in zip(hints, writes):
        w = b.open(size_hint=h)
        devs.append(w.device)
        w.write(bytes(wr))  # counts toward the device's load beyond the hint
        ws.append(w)
    assert devs == _greedy(hints, writes, 3)
    # freeing writers returns their load: the next writer goes to the emptied device
    for i, w in enumerate(ws):
        if devs[i] == 1:
            w.close()
    assert b.open(size_hint=1).device == 1
    b.close()  # closes the remaining writers first
    assert all(w._h is None for w in ws)


def test_writer_batcher_free_fails_late_calls():
    """Writers outlive their batcher only for free(): a call after batcher_free fails cleanly."""
    from kopia_amd.writer import WriterBatcher
    lib = _lib.lib()
    b = WriterBatcher("FIXED-1M")
    h = lib.kcdc_bw_open(b._h)
    assert lib.kcdc_bw_write(h, bytes(10).__class__(b"x" * 10), 10) == 0
    lib.kcdc_bw_batcher_free(b._h)
    b._h = None
    assert lib.kcdc_bw_write(h, b"y", 1) == _lib.KCDC_EINVAL
    lib.kcdc_bw_free(h)


def test_writer_calls_racing_batcher_free():
    """A writer call that races kcdc_bw_batcher_free returns KCDC_OK or KCDC_EINVAL and never touches
    the freed batcher: the batcher's lifetime state is refcounted by its writers (kcdc_writer.cpp
    BwCtl), so a call starting during or after the free sees `closing` in memory that outlives the
    batcher.  Threads hammer write / cuts / finish on FIXED writers (host logic, no GPU) while the
    batcher is freed; every writer is freed after."""
    import threading
    from kopia_amd.writer import WriterBatcher
    lib = _lib.lib()
    for rep in range(20):
        b = WriterBatcher("FIXED-128K")
        hs = [lib.kcdc_bw_open(b._h) for _ in range(6)]
        assert all(hs)
        codes, stop = [], threading.Event()
        buf = b"z" * 5000
        out = (C.c_uint64 * 64)()

        def hammer(h, k):
            got = []
            i = 0
            while not stop.is_set() and i < 4000:
                op = (i + k) % 3
                if op == 0:
                    rc = lib.kcdc_bw_write(h, buf, len(buf))
                elif op == 1:
                    rc = lib.kcdc_bw_cuts(h, out, 64)
                    rc = 0 if rc >= 0 else rc
                else:
                    rc = lib.kcdc_bw_device(h)
                    rc = 0 if rc >= 0 else rc
                got.append(rc)
                i += 1
            codes.append(got)

        th = [threading.Thread(target=hammer, args=(h, k)) for k, h in enumerate(hs)]
        for t in th:
            t.start()
        lib.kcdc_bw_batcher_free(b._h)
        b._h = None
        stop.set()
        for t in th:
            t.join()
        for h in hs:
            assert lib.kcdc_bw_write(h, b"y", 1) == _lib.KCDC_EINVAL
            assert lib.kcdc_bw_finish(h) == _lib.KCDC_EINVAL
            lib.kcdc_bw_free(h)
        flat = [c for g in codes for c in g]
        assert set(flat) <= {0, _lib.KCDC_EINVAL}, set(flat)
