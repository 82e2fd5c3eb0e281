"""The batch kernel's persistent work queue: failures are loud, and progress does not
depend on every workgroup of the persistent grid being resident at once.

Reference contract: NextSplitPoint has no error channel (repo/splitter/splitter.go:25),
so the library must never hand back a cut list it did not finish (kcdc.h,
KCDC_COUNT_FAILED)."""
import ctypes as C

import numpy as np
import pytest

from kopia_amd import _lib, batch
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961
NAME = "DYNAMIC-4M-BUZHASH"


class knob:
    def __init__(self, key, value):
        self.key, self.value = key, value

    def __enter__(self):
        assert _lib.lib().kcdc_test_set(self.key, self.value) == 0

    def __exit__(self, *exc):
        _lib.lib().kcdc_test_set(self.key, 0)


def _streams(gpu, ns, L, first_sid=0):
    import torch
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=first_sid)
    return data, batch.make_device_batch(NAME, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, gpu)


def _oracle(ns, L, first_sid=0):
    cuts, counts = coracle.split_prng_streams(NAME, SEED, np.arange(first_sid, first_sid + ns), L, nthreads=16)
    return [cuts[i, :counts[i]] for i in range(ns)]


def test_failed_launch_is_reported(gpu):
    """A launch marked failed on the device (test hook) sets every count to
    KCDC_COUNT_FAILED: the device path raises on read, the host path returns EIO."""
    import torch
    ns, L = 64, 1 << 20
    data, b = _streams(gpu, ns, L)
    with knob(_lib.TEST_FORCE_ERROR, 1):
        batch.split_batch_device(NAME, b)
        torch.cuda.synchronize()
        counts = b.counts.cpu().numpy()[:ns].view(np.uint64)
        assert (counts == np.uint64(_lib.COUNT_FAILED)).all()
        with pytest.raises(_lib.KcdcError) as e:
            batch.read_cuts(b)
        assert e.value.code == _lib.KCDC_EIO
        # sub-MiB streams: the host path routes them through the batch kernel (larger ones
        # that would be a batch's tail take the long path, which has no work queue)
        host = data[: 4 * L].cpu().numpy()
        with pytest.raises(_lib.KcdcError) as e:
            batch.split_batch_host(NAME, [host[i * (L // 4):(i + 1) * (L // 4)] for i in range(16)])
        assert e.value.code == _lib.KCDC_EIO
    # the next launch is clean again
    batch.split_batch_device(NAME, b)
    torch.cuda.synchronize()
    got = batch.read_cuts(b)
    want = _oracle(ns, L)
    assert all(np.array_equal(got[i], want[i]) for i in range(ns))


def test_waiting_wave_give_up_loses_nothing(gpu):
    """One 1 GiB stream among 2047 tiny ones: one wave scans it for tens of ms while every
    other wave waits on a queue that does not move.  With a 1000-poll cap the waiting waves
    give up (the queue header counts them); they hold no stream, so the result is still
    exact -- a give-up can only ever cost a stream that a waiting wave held a ticket for."""
    import torch
    big, small, ns = 1 << 30, 64 << 10, 2048
    data = torch.empty(big + (ns - 1) * small, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, big, 1, big, SEED, first_sid=0)
    batch.fill_prng(data[big:], small, ns - 1, small, SEED, first_sid=1)
    ptrs = [data.data_ptr()] + [data.data_ptr() + big + i * small for i in range(ns - 1)]
    b = batch.make_device_batch(NAME, ptrs, [big] + [small] * (ns - 1), gpu)
    cuts, counts = coracle.split_prng_streams(NAME, SEED, [0], big, nthreads=1)
    for cap in (1000, 0):
        with knob(_lib.TEST_SPIN_CAP, cap), knob(_lib.TEST_NO_STEAL, 1):
            batch.split_batch_device(NAME, b)
            torch.cuda.synchronize()
            giveups = _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_GIVEUPS))
            assert _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_DONE)) == ns
        assert (giveups > 0) == (cap != 0), (cap, giveups)
        got = batch.read_cuts(b)
        np.testing.assert_array_equal(got[0], cuts[0, :counts[0]])
        assert all(g.tolist() == [small] for g in got[1:])  # shorter than min: one chunk


def test_give_up_holding_a_ticket_is_reported(gpu):
    """A 1-poll cap: waves give up as soon as the entry behind their ticket is not yet
    written, which loses the stream a yielding wave then writes there.  Every launch must
    then be exact or raise KCDC_EIO (its lost streams' counts stay KCDC_COUNT_FAILED) --
    never a silently partial cut list.  At least one launch must lose a stream."""
    import torch
    ns, L = 4096, 4 << 20  # (min size is 2 MiB: shorter streams never queue a yield)
    _data, b = _streams(gpu, ns, L)
    want = _oracle(ns, L)
    failed = 0
    for _ in range(4):
        with knob(_lib.TEST_SPIN_CAP, 1), knob(_lib.TEST_NO_STEAL, 1):
            batch.split_batch_device(NAME, b)
            torch.cuda.synchronize()
            giveups = _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_GIVEUPS))
            done = _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_DONE))
        counts = b.counts.cpu().numpy()[:ns].view(np.uint64)
        lost = int((counts == np.uint64(_lib.COUNT_FAILED)).sum())
        assert lost == ns - done, (lost, done)
        if lost:
            failed += 1
            assert giveups > 0
            with pytest.raises(_lib.KcdcError) as e:
                batch.read_cuts(b)
            assert e.value.code == _lib.KCDC_EIO
        else:
            got = batch.read_cuts(b)
            assert all(np.array_equal(got[i], want[i]) for i in range(ns))
        # streams that did finish are exact either way
        ok = np.nonzero(counts != np.uint64(_lib.COUNT_FAILED))[0]
        cuts = b.cuts.cpu().numpy().view(np.uint64)
        base = b.cut_base.cpu().numpy().view(np.uint64)
        for i in ok[:: max(1, len(ok) // 64)]:
            c = int(counts[i])
            assert np.array_equal(cuts[int(base[i]):int(base[i]) + c], want[i])
    assert failed > 0, "a 1-poll cap never lost a stream: the test does not exercise the failure path"


def _beside_occupier(gpu, nwg, usec):
    """Run a 4096 x 4 MiB launch on one stream while a kernel on another stream holds
    `nwg` CUs for `usec`; returns (cut lists, batch end, occupier end) in ms after start."""
    import time

    import torch
    ns, L = 4096, 4 << 20
    _data, b = _streams(gpu, ns, L)
    batch.split_batch_device(NAME, b)  # warm (tables, workspaces)
    torch.cuda.synchronize()
    # the batch on a high-priority stream: two default-priority streams may share a hardware
    # queue (HIP assigns them round-robin as a process creates streams), which would serialise
    # the batch behind the occupier whatever the kernel does
    sa, sb = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu, priority=-1)
    t0 = torch.cuda.Event(enable_timing=True)
    ea = torch.cuda.Event(enable_timing=True)
    eb = torch.cuda.Event(enable_timing=True)
    t0.record(sa)
    sb.wait_event(t0)
    _lib.check(_lib.lib().kcdc_test_occupy(nwg, usec, C.c_void_p(sa.cuda_stream)))
    ea.record(sa)
    time.sleep(0.005)  # the occupier is resident before the batch is dispatched
    batch.split_batch_device(NAME, b, sb)
    eb.record(sb)
    torch.cuda.synchronize()
    return batch.read_cuts(b), t0.elapsed_time(eb), t0.elapsed_time(ea)


def test_batch_beside_occupying_kernel_steals(gpu):
    """Half the CUs are held for 300 ms: the batch's workgroups there cannot start, their
    preassigned streams are requeued by waiting waves, and the launch finishes (with
    every stream bit-exact) long before the occupier does."""
    got, t_batch, t_occ = _beside_occupier(gpu, 128, 300_000)
    want = _oracle(4096, 4 << 20)
    bad = [i for i in range(4096) if not np.array_equal(got[i], want[i])]
    assert not bad, f"{len(bad)} streams differ, first {bad[:5]}"
    assert t_occ > 250.0, t_occ
    assert t_batch < 0.5 * t_occ, (t_batch, t_occ)


def test_batch_beside_occupying_kernel_no_steal(gpu):
    """Without stealing the same launch waits for the occupied CUs (no deadlock, no
    give-up) and is still exact."""
    with knob(_lib.TEST_NO_STEAL, 1):
        got, t_batch, t_occ = _beside_occupier(gpu, 128, 100_000)
    want = _oracle(4096, 4 << 20)
    assert all(np.array_equal(got[i], want[i]) for i in range(4096))
    assert t_batch >= 0.9 * t_occ, (t_batch, t_occ)


def test_highest_device_index(gpu):
    """Per-device state (tables, queue workspaces, host staging) on the highest visible
    device; with several devices, device 0 and the last one in the same process agree."""
    import torch
    ndev = torch.cuda.device_count()
    ns, L = 256, 4 << 20
    want = _oracle(ns, L, first_sid=7)
    for d in sorted({0, ndev - 1}):
        dev = torch.device("cuda", d)
        with torch.cuda.device(dev):
            _data, b = _streams(dev, ns, L, first_sid=7)
            batch.split_batch_device(NAME, b)
            torch.cuda.synchronize(dev)
            got = batch.read_cuts(b)
        assert all(np.array_equal(got[i], want[i]) for i in range(ns)), f"device {d}"
        host = [coracle.gen_stream(SEED, 7 + i, L) for i in range(4)]
        hc = batch.split_batch_host(NAME, host, device=d)
        assert all(np.array_equal(hc[i], want[i]) for i in range(4)), f"device {d} host path"
