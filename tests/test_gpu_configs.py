"""GPU: BASELINE.json configs 3, 4 and 5 at their stated per-GPU sizes, bit-exact against
the oracle.  Large: each test moves tens of GiB through HBM and runs the
oracle over the same bytes on the host's cores.

* config 3: one 64 GiB stream through the exact intra-stream path (kcdc_split_long_device)
  vs one sequential streaming-oracle pass (NextSplitPoint over 256 MiB slices).
* config 4: one GPU's shard of the 8-GPU job, 8192 x 8 MiB, every stream vs the oracle.
* config 5: rank 0 of the 8-rank LPT plan over 256 GiB of Zipf-sized files (4 KiB..1 GiB,
  32 GiB on this GPU) through kcdc_split_files_device, every file vs the oracle.
Reference intent: snapshot/upload/upload.go:166-209 (big files), splitter_buzhash32.go:26-67."""
import numpy as np
import pytest

from kopia_amd import batch
from kopia_amd import dist as kd
from kopia_amd import splitter as ks
from oracle import coracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
SEED = 0x6B6F706961


def test_config3_64gib_stream(gpu):
    import torch
    name, L = "DYNAMIC-4M-BUZHASH", 64 << 30
    data = torch.empty(L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, 1, L, SEED, 0)
    cuts, count, _ws = batch.split_long_device(name, data.data_ptr(), L, gpu)
    torch.cuda.synchronize()
    got = batch.read_long(cuts, count)
    del data, cuts, _ws
    torch.cuda.empty_cache()
    want, _s = coracle.split_prng_stream_blocks(name, SEED, 0, L)
    assert got.size == want.size and got[-1] == L
    np.testing.assert_array_equal(got, want)


def test_config4_shard_8192x8mib(gpu):
    import torch
    name, ns, L = "DYNAMIC-4M-BUZHASH", 8192, 8 << 20
    rank = 3  # any rank's shard: stream ids rank*8192 ..
    data = torch.empty(ns * L, dtype=torch.uint8, device=gpu)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=rank * ns)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, gpu)
    batch.split_batch_device(name, b)
    torch.cuda.synchronize()
    got = batch.read_cuts(b)
    del data
    torch.cuda.empty_cache()
    cuts, counts = coracle.split_prng_streams(name, SEED, np.arange(rank * ns, (rank + 1) * ns), L, nthreads=16)
    bad = [i for i in range(ns) if not np.array_equal(got[i], cuts[i, :counts[i]])]
    assert not bad, f"{len(bad)} of {ns} streams differ, first {bad[:5]}"


@pytest.mark.parametrize("name", ks.SupportedAlgorithms())  # "across all registered splitter variants"
def test_config5_full_lpt_rank(gpu, name):
    import torch
    sizes = kd.zipf_sizes(256 << 30)
    mine = sorted(kd.lpt_plan(sizes, 8)[0], key=lambda i: (int(sizes[i]), i))
    lens = [int(sizes[i]) for i in mine]
    assert max(lens) == 1 << 30 and sum(lens) >= 31 << 30
    total = sum(lens)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    data = torch.empty(total, dtype=torch.uint8, device=gpu)
    k = 0
    while k < len(lens):  # file i's bytes are counter-PRNG stream i; one fill per run of ids
        e = k
        while e < len(lens) and lens[e] == lens[k] and mine[e] == mine[k] + (e - k):
            e += 1
        batch.fill_prng(data[int(offs[k]):], lens[k], e - k, lens[k], SEED, first_sid=int(mine[k]))
        k = e
    cuts, counts, base, cap = batch.split_files_device(name, [data.data_ptr() + int(o) for o in offs], lens, gpu)
    got = batch.read_files(cuts, counts, base, cap)
    del data
    torch.cuda.empty_cache()
    bad = []
    for sz in sorted(set(lens)):  # the oracle per size class (same bytes: stream id = file index)
        ks_ = [k for k in range(len(lens)) if lens[k] == sz]
        want, cnt = coracle.split_prng_streams(name, SEED, [mine[k] for k in ks_], sz, nthreads=16)
        bad += [mine[k] for j, k in enumerate(ks_) if not np.array_equal(got[k], want[j, :cnt[j]])]
    assert not bad, f"{len(bad)} of {len(lens)} files differ ({name}), first {bad[:5]}"
