#!/usr/bin/env python3
"""Splitter throughput benchmark (BASELINE.json metric) for the MI355X CDC splitter.

Workload (BASELINE.json configs[1]): per GPU, 4096 independent 4 MiB streams of
counter-PRNG bytes resident in HBM, split with the default algorithm
DYNAMIC-4M-BUZHASH (repo/splitter/splitter.go:89).  One *step* = one launch of
the batch splitter over all 4096 streams (the whole 16 GiB shard); cut lists stay
in HBM.  For N > 1 GPUs every rank splits its own shard (stream ids offset by
rank): weak scaling, no collective on the data path (the only collectives are
the timing barrier and the max-over-ranks of the elapsed time).

Prints ONE JSON line on rank 0 (the driver's contract).  Extra keys:
  roofline     — dominant kernel's algorithmic bytes / kernel time vs HBM peak
  cpu_baseline — the oracle's C restatement of the reference Go loop timed on
                 this host (rank 0, N=1 only)
  host_inclusive_gib_s — H2D + kernel + D2H rate through kcdc_split_batch_host
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from kopia_amd import _lib, batch  # noqa: E402
from kopia_amd import dist as kd  # noqa: E402
from kopia_amd import splitter as ks  # noqa: E402

METRIC = "splitter throughput GiB/s (device-resident) at 1/2/4/8 GPU; boundaries bit-exact"
SEED = 0x6B6F706961
# dominant kernel per splitter kind (kcdc_kernels.hip launch_split_batch)
BATCH_KERNEL = {0: "kcdc::dev::split_fixed_kernel", 1: "kcdc::dev::split_batch_pipe_kernel<true>",
                2: "kcdc::dev::split_batch_kernel<rabinkarp>"}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
GiB = float(1 << 30)


def rolled_bytes(cuts: np.ndarray, min_size: int) -> int:
    """Bytes the reference loop must read for one stream:
    per chunk [s,e): (e-s) - max(min(min-1, e-s) - 64, 0)."""
    if cuts.size == 0:
        return 0
    lens = np.diff(np.concatenate(([0], cuts)))
    fastp = np.minimum(min_size - 1, lens)
    return int(np.sum(lens - np.maximum(fastp - 64, 0)))


def load_pmc_traffic(kernel_prefix: str):
    """Measured HBM bytes per launch from a committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get(kernel_prefix, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(name: str, ns: int, L: int, gpu_cuts: list, nthreads: int, min_seconds: float = 10.0):
    """Rank 0, N=1: the C restatement of the reference Go loop (oracle/, "port"),
    timed on host cores over a sample of the same workload; also checks that the
    GPU cut lists of the sample are bit-identical."""
    from oracle import coracle  # oracle import confined to this leg
    t0 = time.time()
    streams = [None] * ns
    # generate the sample (not timed), then time only the split
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(nthreads) as ex:
        for i, s in enumerate(ex.map(lambda i: coracle.gen_stream(SEED, i, L), range(ns))):
            streams[i] = s
    gen_s = time.time() - t0
    coracle.split_batch(name, streams[:8], nthreads=nthreads)  # warm
    # repeat whole passes over the sample until >= min_seconds of wall time
    t0 = time.perf_counter()
    want = coracle.split_batch(name, streams, nthreads=nthreads)
    passes = 1
    while time.perf_counter() - t0 < min_seconds:
        coracle.split_batch(name, streams, nthreads=nthreads)
        passes += 1
    dt = time.perf_counter() - t0
    mism = sum(1 for i in range(ns) if not np.array_equal(want[i], gpu_cuts[i]))
    return {"value": round(passes * ns * L / GiB / dt, 3), "unit": "GiB/s", "cores": nthreads, "kind": "port",
            "sample": f"{ns} x {L >> 20} MiB counter-PRNG streams (stream ids 0..{ns - 1}, same bytes as GPU rank 0), "
                      f"{name}, C restatement of repo/splitter/splitter_buzhash32.go:26-67 (oracle/cdc_oracle.c), "
                      f"{nthreads} threads, {passes} passes, {dt:.2f}s wall",
            "sample_parity_mismatches": mism, "gen_seconds": round(gen_s, 2)}, streams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--splitter", default="DYNAMIC-4M-BUZHASH")
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--stream-mib", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5],
                    help="BASELINE.json config: 2 = 4096 x 4 MiB/GPU (default), 3 = one 64 GiB stream "
                         "(exact tiled CDC), 4 = 8192 x 8 MiB/GPU, 5 = Zipf-sized files, LPT over ranks")
    ap.add_argument("--long-gib", type=int, default=64, help="config 3 stream size")
    ap.add_argument("--files-gib", type=int, default=32, help="config 5 bytes per GPU (256 GiB over 8 GPUs)")
    ap.add_argument("--all-names", action="store_true", help="config 5: also time every registered name")
    args = ap.parse_args()
    if args.config == 4:
        args.streams, args.stream_mib = 8192, 8
    if args.config == 3:
        return bench_long(args)
    if args.config == 5:
        return bench_files(args)

    rank, world, local = kd.env_rank_world()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    name, ns, L = args.splitter, args.streams, args.stream_mib << 20
    info = ks.lookup(name)
    assert info is not None, name
    data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=rank * ns)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        batch.split_batch_device(name, b, stream)
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        batch.split_batch_device(name, b, stream)
        e1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = kd.max_over_ranks(time.perf_counter() - t0, dev)
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))

    cuts = batch.read_cuts(b)
    alg_bytes = sum(rolled_bytes(c, int(info.min_size)) for c in cuts)  # per launch, this rank
    total_bytes = ns * L * world * args.steps
    value = total_bytes / GiB / elapsed

    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"config{args.config}: {ns} x {args.stream_mib} MiB independent streams per GPU "
                               f"(counter-PRNG bytes, HBM-resident), {name}",
                   "splitter": name, "streams_per_gpu": ns, "stream_bytes": L, "global_streams": ns * world,
                   "parallelism": f"stream-sharded x{world}, no data-path collectives"},
    }
    # Roofline: algorithmic bytes = 1 byte per ingested stream byte, so
    # `achieved` = stream bytes / kernel time.  A skip-aware kernel reads only the bytes the
    # reference loop rolls (min-size fast path), so `frac` can exceed 1; the physical HBM
    # figure is `traffic` (rocprofv3 FETCH_SIZE, calibrated) / kernel time.
    traffic = load_pmc_traffic("split_batch")  # key written by tools/pmc_traffic.py
    kern_s = kern_ms * 1e-3
    achieved = ns * L / kern_s / 1e9
    out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                       "kernel": BATCH_KERNEL[int(info.kind)], "kernel_ms": round(kern_ms, 4),
                       "algorithmic_bytes_per_launch": ns * L,
                       "algorithmic_bytes_def": "1 byte per ingested stream byte (SURVEY.md §8d): "
                                                f"{ns} streams x {L} B per launch",
                       "hbm_gbs_measured": round(traffic / kern_s / 1e9, 1) if traffic else None,
                       "hbm_frac_measured": round(traffic / kern_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                       "rolled_bytes_per_launch": alg_bytes,
                       "rolled_gbs": round(alg_bytes / kern_s / 1e9, 1)}
    out["cut_stats"] = {"chunks": int(sum(c.size for c in cuts)),
                        "rolled_fraction": round(alg_bytes / (ns * L), 4)}

    if rank == 0 and world == 1 and not args.no_host_inclusive:
        # host-inclusive: pageable host buffers -> H2D -> kernel -> D2H (kcdc_split_batch_host)
        nh = min(ns, 1024)
        host = data[: nh * L].cpu().numpy()
        views = [host[i * L:(i + 1) * L] for i in range(nh)]
        batch.split_batch_host(name, views[:4], device=local)
        t0 = time.perf_counter()
        hc = batch.split_batch_host(name, views, device=local)
        dt = time.perf_counter() - t0
        assert all(np.array_equal(hc[i], cuts[i]) for i in range(nh))
        out["host_inclusive_gib_s"] = round(nh * L / GiB / dt, 3)
        del host, views

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nthreads = min(16, os.cpu_count() or 1)
        sample = min(ns, max(1, (16 << 30) // L))  # bounded host sample (<= 16 GiB)
        base, _ = cpu_baseline(name, sample, L, cuts, nthreads)
        out["cpu_baseline"] = base

    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def bench_long(args):
    """Config 3: ONE long stream (default 64 GiB) split exactly by the tiled candidate
    scan + device resolver; cut set checked against the per-wave sequential path.
    Single GPU (the stream does not shard across ranks in this mode)."""
    rank, world, local = kd.env_rank_world()
    assert world == 1, "config 3 is a single-GPU configuration"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    name, L = args.splitter, args.long_gib << 30
    data = torch.empty(L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, 1, L, SEED, first_sid=0)
    stream = torch.cuda.current_stream(dev)
    cuts, count, ws = batch.split_long_device(name, data.data_ptr(), L, dev, stream)
    torch.cuda.synchronize(dev)
    steps = max(1, min(args.steps, 10))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        _c, _n, _w = batch.split_long_device(name, data.data_ptr(), L, dev, stream)
        e1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    got = batch.read_long(cuts, count)
    # independent check: the per-wave sequential batch path on the same bytes
    b = batch.make_device_batch(name, [data.data_ptr()], [L], dev)
    batch.split_batch_device(name, b, stream)
    torch.cuda.synchronize(dev)
    seq = batch.read_cuts(b)[0]
    out = {"metric": METRIC, "value": round(L * steps / GiB / elapsed, 3), "unit": "GiB/s", "n_gpus": 1,
           "steps": steps, "warmup": 1, "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"config3: one {args.long_gib} GiB stream, exact intra-stream tiled CDC, {name}",
                      "splitter": name, "stream_bytes": L, "parallelism": "single GPU, 128 KiB segments/wave"},
           "kernel_ms_events": round(ms, 3), "cuts": int(got.size),
           "identical_to_sequential_path": bool(np.array_equal(got, seq))}
    print(json.dumps(out), flush=True)


def bench_files(args):
    """Config 5: file sizes from a Zipf law over 19 classes 4 KiB..1 GiB
    (s = 1.1, fixed seed), files_gib x world bytes in total, LPT-balanced over the ranks;
    every rank splits its files with kcdc_split_files_device (each file through the batch
    or the long path).  Weak scaling, no data-path collective.  FIXED names read no data."""
    rank, world, local = kd.env_rank_world()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    sizes = kd.zipf_sizes(args.files_gib * world << 30)
    mine = sorted(kd.lpt_plan(sizes, world)[rank], key=lambda i: int(sizes[i]))
    lens = [int(sizes[i]) for i in mine]
    total = sum(lens)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if lens else np.zeros(0, np.int64)
    # runs of equal sizes are contiguous (sorted): one fill per run, file ids = global indices
    k = 0
    while k < len(lens):
        e = k
        while e < len(lens) and lens[e] == lens[k] and mine[e] == mine[k] + (e - k):
            e += 1
        batch.fill_prng(data[int(offs[k]):], lens[k], e - k, lens[k], SEED, first_sid=int(mine[k]))
        k = e
    ptrs = [data.data_ptr() + int(o) for o in offs]
    stream = torch.cuda.current_stream(dev)

    def run(name, steps, warmup):
        for _ in range(warmup):
            batch.split_files_device(name, ptrs, lens, dev, stream)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        res = None
        for _ in range(steps):
            res = batch.split_files_device(name, ptrs, lens, dev, stream)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        return kd.max_over_ranks(time.perf_counter() - t0, dev), res

    name = args.splitter
    steps = max(1, min(args.steps, 10))
    elapsed, res = run(name, steps, max(1, min(args.warmup, 2)))
    out = {"metric": METRIC, "value": round(total * world * steps / GiB / elapsed, 3), "unit": "GiB/s",
           "n_gpus": world, "steps": steps, "warmup": max(1, min(args.warmup, 2)),
           "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"config5: Zipf(s=1.1) file sizes over 4 KiB..1 GiB, {args.files_gib} GiB per GPU, "
                                  f"LPT over {world} rank(s), {name}",
                      "splitter": name, "files_this_rank": len(lens), "bytes_this_rank": total,
                      "largest_file": max(lens) if lens else 0,
                      "parallelism": f"LPT file sharding x{world}, no data-path collectives"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # cpu_baseline leg: the oracle's C restatement timed on a sample of this rank's files
        # (the 64 smallest and the 2 largest), which also checks the GPU cuts of the sample
        from oracle import coracle  # oracle import confined to this leg
        got = batch.read_files(*res)
        pick = sorted(set(range(min(64, len(lens)))) | set(range(0, len(lens), 8)) |
                      set(range(max(0, len(lens) - 2), len(lens))))
        host = [data[int(offs[i]):int(offs[i]) + lens[i]].cpu().numpy() for i in pick]
        nthreads = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        want = coracle.split_batch(name, host, nthreads=nthreads)
        dt = time.perf_counter() - t0
        sb = sum(lens[i] for i in pick)
        out["cpu_baseline"] = {
            "value": round(sb / GiB / dt, 3), "unit": "GiB/s", "cores": nthreads, "kind": "port",
            "sample": f"{len(pick)} files of this rank (64 smallest, every 8th, 2 largest; {sb >> 20} MiB), {name}, "
                      f"oracle/cdc_oracle.c, {nthreads} threads, {dt:.2f}s wall",
            "sample_parity_mismatches": sum(1 for j, i in enumerate(pick) if not np.array_equal(got[i], want[j]))}
    if args.all_names:
        out["per_name_gib_s"] = {}
        for nm in ks.SupportedAlgorithms():
            el, _ = run(nm, 2, 1)
            out["per_name_gib_s"][nm] = round(total * world * 2 / GiB / el, 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
