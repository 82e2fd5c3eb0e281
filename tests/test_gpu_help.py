"""GPU: intra-region help in the batch kernels (split_batch_pipe_kernel for buzhash,
split_batch_rk_kernel for Rabin-Karp).

Waves with no stream of their own claim far tiles of other waves' regions and post each tile's
first candidate; an owner whose next claim fails takes the region's cut from those posts.  The
cut must still be exactly the reference's: the first candidate in [s + min - 1, s + max - 1],
else the forced cut (repo/splitter/splitter_buzhash32.go:26-67, splitter_rabinkarp64.go:26-67), checked here against the C
oracle (oracle/cdc_oracle.c, pinned by TestSplitterStability) on launches where helpers do most
of the scanning -- few long streams, many regions per stream, small and custom averages,
misaligned streams, dense candidates -- and with help switched off (KCDC_TEST_NO_HELP) for A/B
parity."""
import numpy as np
import pytest

from kopia_amd import _lib, batch
from oracle import coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961


class knob:
    def __init__(self, key, value):
        self.key, self.value = key, value

    def __enter__(self):
        assert _lib.lib().kcdc_test_set(self.key, self.value) == 0

    def __exit__(self, *exc):
        _lib.lib().kcdc_test_set(self.key, 0)


def _helped(name, ns=4096):
    """Whether waiting waves help this launch (launch_split_batch's policy):
    averages of 1 MiB and up for both kinds, and Rabin-Karp launches with fewer streams than the
    grid's waves (2,048 on MI355X)."""
    avg = _lib.lib().kcdc_max_segment_size(name.encode()) // 2  # max = 2 x avg (splitter_buzhash32.go:73-86)
    return avg >= (1 << 20) or ("RABINKARP" in name and ns < 2048)


def _split(name, data, offs, lens, gpu):
    import torch
    b = batch.make_device_batch(name, [data.data_ptr() + int(o) for o in offs], [int(x) for x in lens], gpu)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize()
    helps = _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_HELPS))
    return batch.read_cuts(b), helps


def _check(name, host, offs, lens, got):
    for i, (o, L) in enumerate(zip(offs, lens)):
        want = coracle.split_stream(name, host[int(o):int(o) + int(L)])
        assert got[i].tolist() == want.tolist(), f"{name} stream {i} ({L} B at +{o}): {len(got[i])} vs {len(want)} cuts"


@pytest.mark.parametrize("name,ns,mib", [("DYNAMIC-4M-BUZHASH", 4, 64), ("DYNAMIC-4M-BUZHASH", 24, 16),
                                         ("DYNAMIC-8M-BUZHASH", 3, 96), ("DYNAMIC-1M-BUZHASH", 8, 40),
                                         ("DYNAMIC-128K-BUZHASH", 6, 24), ("DYNAMIC-4M-RABINKARP", 4, 64),
                                         ("DYNAMIC-4M-RABINKARP", 24, 16), ("DYNAMIC-1M-RABINKARP", 8, 40),
                                         ("DYNAMIC-128K-RABINKARP", 6, 24)])
def test_few_long_streams(gpu, name, ns, mib):
    """Fewer streams than waves: almost every tile of every region is a helper's."""
    import torch
    L = mib << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=100)
    got, helps = _split(name, data, [i * L for i in range(ns)], [L] * ns, gpu)
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(100, 100 + ns), L, nthreads=16)
    for i in range(ns):
        assert got[i].tolist() == cuts[i, :counts[i]].tolist(), f"{name} stream {i}"
    assert helps > 0 or not _helped(name, ns), "no tile was helped"


@pytest.mark.parametrize("name", ["DYNAMIC-2M-BUZHASH", "DYNAMIC-2M-RABINKARP"])
def test_ragged_misaligned_streams(gpu, name):
    """Odd lengths at odd offsets (coordinates with a nonzero head), including lengths that end
    inside a helper's tile and regions of exactly kHelpMinTiles tiles."""
    import torch
    rng = np.random.default_rng(5)
    lens = [int(x) for x in rng.integers(3 << 20, 30 << 20, 10)] + [(1 << 20) + 3 * (128 << 10) - 1, 5 << 20, 1, 0]
    offs = np.concatenate(([7], 7 + np.cumsum(np.asarray(lens) + 13)[:-1])).astype(np.int64)
    total = int(offs[-1] + lens[-1] + 64)
    host = coracle.gen_stream(SEED, 9, total)
    data = torch.from_numpy(host).to(gpu)
    got, helps = _split(name, data, offs, lens, gpu)
    _check(name, host, offs, lens, got)
    assert helps > 0 or not _helped(name, len(lens))


@pytest.mark.parametrize("kind", ["buzhash", "rabinkarp"])
def test_custom_small_averages(gpu, kind):
    """Custom averages (the TestSplitterStability parameterisations, splitter_test.go:30-52):
    small tiles, many regions, regions of few tiles."""
    import torch
    kat = coracle.gorand_read(5, 5_000_000)
    data = torch.from_numpy(kat).to(gpu)
    for avg in (1024, 2048, 32 << 10, 64 << 10):
        name = _lib.lib().kcdc_custom_algorithm(coracle.KIND[kind], avg).decode()
        offs = [0, 1_000_003, 2_500_001]
        lens = [1_000_003, 1_500_000, 2_499_999]
        got, _ = _split(name, data, offs, lens, gpu)
        for i, (o, L) in enumerate(zip(offs, lens)):
            assert got[i].tolist() == coracle.split_stream_kind(kind, avg, kat[o:o + L]).tolist(), (avg, i)


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP"])
def test_dense_and_periodic(gpu, name):
    """All-zero data (every position a candidate: cuts every min) and a periodic pattern (one
    candidate phase) through helped launches."""
    import torch
    L = 40 << 20
    zeros = np.zeros(L, np.uint8)
    pat = np.tile(np.arange(1, 12, dtype=np.uint8), L // 11 + 1)[:L]
    host = np.concatenate([zeros, pat])
    data = torch.from_numpy(host).to(gpu)
    got, _ = _split(name, data, [0, L], [L, L], gpu)
    _check(name, host, [0, L], [L, L], got)


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP"])
def test_help_off_is_identical(gpu, name):
    """The same batch with help switched off (KCDC_TEST_NO_HELP) cuts identically and posts no help."""
    import torch
    ns, L = 12, 24 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=7)
    offs = [i * L for i in range(ns)]
    on, helps_on = _split(name, data, offs, [L] * ns, gpu)
    with knob(_lib.TEST_NO_HELP, 1):
        off, helps_off = _split(name, data, offs, [L] * ns, gpu)
    assert (helps_on > 0 or not _helped(name, ns)) and helps_off == 0
    assert [x.tolist() for x in on] == [x.tolist() for x in off]


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP"])
def test_config2_shape_with_tail_help(gpu, name):
    """A config-2-shaped batch (512 x 4 MiB here): help happens only in the batch's tail, every
    stream bit-exact."""
    import torch
    ns, L = 512, 4 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=3000)
    got, helps = _split(name, data, [i * L for i in range(ns)], [L] * ns, gpu)
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(3000, 3000 + ns), L, nthreads=16)
    bad = [i for i in range(ns) if got[i].tolist() != cuts[i, :counts[i]].tolist()]
    assert not bad, bad[:8]


@pytest.mark.parametrize("name", ["DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP"])
@pytest.mark.parametrize("ns", [2304, 4096])
def test_many_streams_with_yields(gpu, name, ns):
    """More streams than launch waves (2,048): visits yield, waves wait on tickets and take help
    tasks while they hold them.  Round 4's Rabin-Karp port lost streams exactly here (a held ticket
    never re-presented after a help task: DESIGN.md §2.1c).  Every stream must come back exact, no
    wave may give up, help must happen, and the held-ticket audit (the ticket's register copy
    against its memory copy at the end of every help task) must be clean."""
    import torch
    L = 4 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=0)
    got, helps = _split(name, data, [i * L for i in range(ns)], [L] * ns, gpu)
    lib = _lib.lib()
    assert lib.kcdc_test_queue_stat(_lib.STAT_GIVEUPS) == 0
    assert lib.kcdc_test_queue_stat(_lib.STAT_DONE) == ns
    assert lib.kcdc_test_queue_stat(_lib.STAT_TICKET_AUDIT) == 0
    assert helps > 0
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
    bad = [i for i in range(ns) if got[i].tolist() != cuts[i, :counts[i]].tolist()]
    assert not bad, bad[:8]


@pytest.mark.parametrize("name", ["DYNAMIC-128K-BUZHASH", "DYNAMIC-512K-RABINKARP"])
def test_forced_help_below_policy(gpu, name):
    """Below 1 MiB the policy keeps help off; forced on (KCDC_TEST_NO_HELP = 2)
    the protocol must still cut exactly: small averages mean many regions per tile and owners
    closing regions while helpers scan them."""
    import torch
    ns, L = 2304, 1 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=11)
    with knob(_lib.TEST_NO_HELP, 2):
        got, helps = _split(name, data, [i * L for i in range(ns)], [L] * ns, gpu)
        giveups = _lib.lib().kcdc_test_queue_stat(_lib.STAT_GIVEUPS)
    assert helps > 0 and giveups == 0
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(11, 11 + ns), L, nthreads=16)
    bad = [i for i in range(ns) if got[i].tolist() != cuts[i, :counts[i]].tolist()]
    assert not bad, bad[:8]


def _ring_balance():
    lib = _lib.lib()
    tickets = _lib.check(lib.kcdc_test_queue_stat(_lib.STAT_TICKETS))
    entries = _lib.check(lib.kcdc_test_queue_stat(_lib.STAT_ENTRIES))
    waves = _lib.check(lib.kcdc_test_queue_stat(_lib.STAT_WAVES))
    return tickets, entries, waves


@pytest.mark.parametrize("name,lane_cap", [("DYNAMIC-4M-BUZHASH", 0), ("DYNAMIC-2M-BUZHASH", 0),
                                           ("DYNAMIC-2M-BUZHASH", 1024), ("DYNAMIC-4M-RABINKARP", 0)])
def test_every_reserved_entry_is_written(gpu, name, lane_cap):
    """Round-5 regression: a HELP task whose wave had spent its own visit's budget reserved a ring
    entry (the yield path's atomic) and never wrote it, so the wave that took that entry's ticket
    waited to the end of the launch -- ~1,200 of 2,048 waves per config-2 launch at 2M.  With
    1 KiB lanes at 2M (regions of 49 tiles, yields every 8) the orphans outnumbered the waves:
    every wave ended up holding an orphan ticket, the real entries behind them were never taken,
    and the launch lost the streams still queued (profiles/r05/orphan_entries/).  Now every wave
    exits holding exactly one ticket no entry was written for (the last stream's tombstone may
    leave one fewer), and the 1 KiB geometry splits bit-exact launch after launch, each launch
    bounded by a small spin cap so a regression fails fast instead of spinning."""
    import torch
    ns, L = 4096, 4 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, 0)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, gpu)
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
    want = [cuts[i, :counts[i]].tolist() for i in range(ns)]
    with knob(_lib.TEST_LANE_CAP, lane_cap), knob(_lib.TEST_SPIN_CAP, 200000):
        for launch in range(6):
            batch.split_batch_device(name, b)
            torch.cuda.synchronize()
            tickets, entries, waves = _ring_balance()
            assert waves - 1 <= tickets - entries <= waves, (launch, tickets, entries, waves)
            assert _lib.check(_lib.lib().kcdc_test_queue_stat(_lib.STAT_GIVEUPS)) == 0, launch
            got = batch.read_cuts(b)
            bad = [i for i in range(ns) if got[i].tolist() != want[i]]
            assert not bad, f"launch {launch}: {len(bad)} streams differ, first {bad[:5]}"


@pytest.mark.parametrize("name,lane_cap", [("DYNAMIC-128K-BUZHASH", 256), ("DYNAMIC-128K-BUZHASH", 4096),
                                           ("DYNAMIC-2M-BUZHASH", 256), ("DYNAMIC-2M-BUZHASH", 4096)])
def test_forced_help_in_other_geometries(gpu, name, lane_cap):
    """Help forced on in tile geometries the default rule never picks (KCDC_TEST_LANE_CAP): 16 KiB
    tiles give 128K regions of ~8 tiles and 2M regions of up to ~190 (only those of <= 128 tiles
    take help); 256 KiB tiles leave 128K regions too short to publish.  Every stream exact and the ring balanced, launch after launch
    (tools/geometry_sweep.py runs the full grid: profiles/r05/geometry_sweep/)."""
    import torch
    ns, L = 4096, 4 << 20
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, 0)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, gpu)
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(ns), L, nthreads=16)
    want = [cuts[i, :counts[i]].tolist() for i in range(ns)]
    with knob(_lib.TEST_LANE_CAP, lane_cap), knob(_lib.TEST_NO_HELP, 2), knob(_lib.TEST_SPIN_CAP, 200000):
        for launch in range(3):
            batch.split_batch_device(name, b)
            torch.cuda.synchronize()
            tickets, entries, waves = _ring_balance()
            assert waves - 1 <= tickets - entries <= waves, (launch, tickets, entries, waves)
            got = batch.read_cuts(b)
            bad = [i for i in range(ns) if got[i].tolist() != want[i]]
            assert not bad, f"launch {launch}: {len(bad)} streams differ, first {bad[:5]}"
