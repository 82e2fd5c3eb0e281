#!/usr/bin/env python3
"""Splitter throughput benchmark (BASELINE.json metric) for the MI355X CDC splitter.

Workload (BASELINE.json configs[1]): per GPU, 4096 independent 4 MiB streams of
counter-PRNG bytes resident in HBM, split with the default algorithm
DYNAMIC-4M-BUZHASH (repo/splitter/splitter.go:89).  One *step* = one launch of
the batch splitter over all 4096 streams (the whole 16 GiB shard); cut lists stay
in HBM.  For N > 1 GPUs every rank splits its own shard (stream ids offset by
rank): weak scaling, no collective on the data path.  The only inter-process
traffic is the timing barrier and the max/gather of per-rank timings, over gloo
(CPU) -- no RCCL.

Launch: under torch.distributed.run (RANK/WORLD_SIZE/LOCAL_RANK set) each process
is one rank; without RANK, `--gpus N` spawns N fresh rank processes itself (before
anything touches a GPU in this process), the way `kopia benchmark splitter
--parallel` runs N splitters at once (cli/command_benchmark.go:67-82).

Prints ONE JSON line on rank 0 (the driver's contract).  Extra keys:
  roofline     — the dominant kernel: rolled (algorithmic) bytes / kernel time vs
                 HBM peak, plus the rocprofv3-measured physical HBM rate
  cpu_baseline — the oracle's C restatement of the reference Go loop on this host's
                 cores, 1 thread and all usable threads (rank 0, N=1 only)
  host_inclusive_gib_s — host buffers -> H2D -> kernel -> D2H (kcdc_split_batch_host)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "splitter throughput GiB/s (device-resident) at 1/2/4/8 GPU; boundaries bit-exact"
SEED = 0x6B6F706961
# the pipelined launch: init_ring_kernel, the splitter kernel, check_queue_kernel
BATCH_KERNEL = {0: "kcdc::dev::split_fixed_kernel", 1: "kcdc::dev::split_batch_pipe_kernel<true>",
                2: "kcdc::dev::split_batch_rk_kernel"}  # rocprofv3 names
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
# SIMD VALU-busy fraction of the byte-pass kernels, measured with rocprofv3 SQ counters
# (profiles/r02/aes/pmc_sq.csv, profiles/r02/crypt/pmc_sq.csv): the reason the legs sit below HBM.
AES_VALU_BUSY = 0.60
CHACHA_VALU_BUSY = 0.83
GiB = float(1 << 30)


# ----------------------------------------------------------------- ranks
def env_rank_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


class Comm:
    """Timing barrier and scalar/object reductions over gloo (CPU): no RCCL anywhere."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj) -> list:
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(rank: int, world: int, port: int, argv: list, entry: str):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    mod = sys.modules[__name__]
    getattr(mod, entry)(argv)


def spawn_ranks(world: int, argv: list, entry: str = "main") -> None:
    """Run `entry(argv)` in `world` fresh processes (spawn start method, so nothing of this
    process -- which has not touched a GPU -- is inherited); returns when all exit."""
    import torch.multiprocessing as mp
    mp.start_processes(_child, args=(world, _free_port(), argv, entry), nprocs=world, join=True,
                       start_method="spawn")


def aggregate(per_rank: list, steps: int) -> dict:
    """Whole-job numbers from every rank's {bytes_per_step, elapsed_s}: value = all ranks'
    bytes / the slowest rank's time (weak scaling), plus each rank's own rate."""
    elapsed = max(r["elapsed_s"] for r in per_rank)
    total = sum(r["bytes_per_step"] for r in per_rank) * steps
    return {"value": round(total / GiB / elapsed, 3), "elapsed_s": elapsed,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "per_gpu_gib_s": [round(r["bytes_per_step"] * steps / GiB / r["own_s"], 3) for r in per_rank]}


# ------------------------------------------------------------- roofline
def rolled_bytes(cuts: np.ndarray, min_size: int) -> int:
    """Bytes the reference loop must roll for one stream:
    per chunk [s,e): (e-s) - max(min(min-1, e-s) - 64, 0).  The reference's fast path
    (splitter_buzhash32.go:29-40) never reads the rest, and neither does the kernel."""
    if cuts.size == 0:
        return 0
    lens = np.diff(np.concatenate(([0], cuts)))
    fastp = np.minimum(min_size - 1, lens)
    return int(np.sum(lens - np.maximum(fastp - 64, 0)))


def load_pmc_traffic(kernel: str, config: str):
    """Measured HBM bytes per launch of `kernel` on `config` from a committed rocprofv3
    --pmc FETCH_SIZE summary (profiles/pmc_traffic.json, tools/pmc_traffic.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None
    e = d.get(f"{kernel}|{config}")
    return e.get("hbm_bytes_per_launch") if e else None


def roofline(kernel: str, config: str, kern_ms: float, rolled: int, stream_bytes: int) -> dict:
    kern_s = kern_ms * 1e-3
    achieved = rolled / kern_s / 1e9
    traffic = load_pmc_traffic(kernel, config)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
            "kernel_ms": round(kern_ms, 4), "algorithmic_bytes_per_launch": rolled,
            "algorithmic_bytes_def": "rolled bytes R: the bytes the reference loop reads, per chunk [s,e) "
                                     "(e-s) - max(min(min-1,e-s) - 64, 0) (SURVEY.md §8d), summed over the "
                                     "launch's cut lists",
            "hbm_gbs_measured": round(traffic / kern_s / 1e9, 1) if traffic else None,
            "hbm_frac_measured": round(traffic / kern_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
            "traffic_source": "profiles/pmc_traffic.json[" + f"{kernel}|{config}" + "] (FETCH_SIZE x 1024 x 2)",
            "stream_bytes_per_launch": stream_bytes,
            "stream_gbs": round(stream_bytes / kern_s / 1e9, 1)} | valu_note(kernel, config)


# Rabin-Karp's limiter: the hot loop is throughput-bound on VALU issue
# and the LDS array together, neither saturated (profiles/r06/rk_counters, rk_final: LDS array busy
# 58.5 % of the CU's cycles, VALU ~64 % of each SIMD's at the measured per-class issue costs of
# tools/valu_rate.hip), the per-byte chain's latency a 5 % term (ablations of the hot loop alone,
# tools/rk_loop.hip, profiles/r06/rk_loop/rk_loop2.log: 1.555 ms for config 2's rolled bytes with
# the round-6 address forms).  The floors are the busy fractions times the kernel's 2.15 ms.
RK_HOT_LOOP_MS = {"config2-rk": 1.555}
RK_VALU_FLOOR_MS = {"config2-rk": 1.38}
RK_LDS_FLOOR_MS = {"config2-rk": 1.26}


def valu_note(kernel: str, config: str) -> dict:
    hot = RK_HOT_LOOP_MS.get(config)
    if not hot:
        return {}
    return {"limited_by": "VALU issue and the LDS array together (co-bound; chain latency ~5 %)",
            "hot_loop_alone_ms": hot, "valu_floor_ms": RK_VALU_FLOOR_MS[config],
            "lds_floor_ms": RK_LDS_FLOOR_MS[config],
            "hot_loop_source": "profiles/r06/rk_loop/rk_loop2.log (tools/rk_loop.hip, round-6 replica)"}


def h2d_rates(host: np.ndarray, dev) -> dict:
    """The PCIe H2D ceiling of the host-inclusive path, measured on this box: plain copies of
    the same host bytes (pageable, as kcdc_split_batch_host receives them) and of a pinned
    buffer, 1 GiB at a time."""
    import torch
    n = min(host.size, 1 << 30)
    src = torch.from_numpy(host[:n])
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    pinned.copy_(src)
    res = {}
    for key, t in (("pageable", src), ("pinned", pinned)):
        dst.copy_(t)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(3):
            dst.copy_(t, non_blocking=True)
        torch.cuda.synchronize(dev)
        res[key] = round(3 * n / GiB / (time.perf_counter() - t0), 3)
    del pinned, dst
    return res


# --------------------------------------------------------- CPU baseline
def host_cpu_info() -> dict:
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    logical = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = logical
    quota = None
    try:  # cgroup v2 CPU quota ("max 100000" = unlimited)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    threads = usable if quota is None else max(1, min(usable, int(quota + 0.5)))
    return {"cpu_model": model, "logical_cores": logical, "affinity_cpus": usable, "cgroup_cpu_quota": quota,
            "threads_all": threads}


def _time_passes(fn, min_seconds: float) -> tuple[int, float]:
    t0 = time.perf_counter()
    fn()
    passes = 1
    while time.perf_counter() - t0 < min_seconds:
        fn()
        passes += 1
    return passes, time.perf_counter() - t0


def ref_loop(name: str) -> str:
    """The reference loop a name's CPU baseline restates."""
    return ("repo/splitter/splitter_rabinkarp64.go:26-67" if "RABINKARP" in name
            else "repo/splitter/splitter_fixed.go:15-26" if name.startswith("FIXED")
            else "repo/splitter/splitter_buzhash32.go:26-67")


def cpu_baseline(name: str, ns: int, L: int, gpu_cuts: list) -> dict:
    """Rank 0, N=1: the C restatement of the reference Go loop (oracle/cdc_oracle.c, "port")
    timed on this host with 1 thread and with every usable thread, on disjoint streams of
    the same workload (`--parallel`, cli/command_benchmark.go:67-82); also checks the GPU
    cut lists of the whole sample bit-for-bit."""
    from oracle import coracle  # oracle import confined to this leg
    import concurrent.futures as cf
    info = host_cpu_info()
    nt = info["threads_all"]
    t0 = time.time()
    streams = [None] * ns
    with cf.ThreadPoolExecutor(nt) as ex:
        for i, s in enumerate(ex.map(lambda i: coracle.gen_stream(SEED, i, L), range(ns))):
            streams[i] = s
    gen_s = time.time() - t0
    want = coracle.split_batch(name, streams, nthreads=nt)  # parity reference (untimed)
    mism = sum(1 for i in range(ns) if not np.array_equal(want[i], gpu_cuts[i]))
    one = streams[: max(1, min(ns, (512 << 20) // L))]
    p1, d1 = _time_passes(lambda: coracle.split_batch(name, one, nthreads=1), 8.0)
    pa, da = _time_passes(lambda: coracle.split_batch(name, streams, nthreads=nt), 8.0)
    r1 = p1 * len(one) * L / GiB / d1
    ra = pa * ns * L / GiB / da
    return {"value": round(ra, 3), "unit": "GiB/s", "cores": nt, "logical_cores": info["logical_cores"],
            "kind": "port", "threads_1": round(r1, 3), "threads_all": round(ra, 3), "threads_all_n": nt,
            "cpu_model": info["cpu_model"], "affinity_cpus": info["affinity_cpus"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"],
            "sample": f"{ns} x {L >> 20} MiB counter-PRNG streams (ids 0..{ns - 1}, the GPU's bytes), {name}; "
                      f"C restatement of {ref_loop(name)} (oracle/cdc_oracle.c); "
                      f"1 thread: {len(one)} streams x {p1} passes in {d1:.1f}s; {nt} threads (every usable CPU of "
                      f"this process): {pa} passes in {da:.1f}s",
            "sample_parity_mismatches": mism, "gen_seconds": round(gen_s, 2)}


def cpu_config1(seconds_cap: float = 12.0) -> dict:
    """Config 1 on the host: `kopia benchmark splitter --data-size 256MiB --block-count 1
    --rand-seed 42` (cli/command_benchmark_splitters.go:64-131) through the oracle, one
    thread, every registered name, GB/s base-10 as the command prints them."""
    from oracle import coracle
    from kopia_amd import splitter as ks
    buf = coracle.gorand_read(42, 256 << 20)
    out, t_all = {}, time.perf_counter()
    for nm in ks.SupportedAlgorithms():
        t0 = time.perf_counter()
        coracle.split_stream(nm, buf)
        out[nm] = round(buf.size / 1e9 / (time.perf_counter() - t0), 3)
        if time.perf_counter() - t_all > seconds_cap:
            out["_truncated"] = True
            break
    return out


# ------------------------------------------------------------- configs
def warm_up(fn, min_steps: int, min_s: float, dev) -> tuple[int, float]:
    """Untimed warm-up: at least `min_steps` calls of fn and at least `min_s` seconds (the chip's
    clock ramps over ~10 config-2 launches after idle, profiles/r03/buz/ramp.log)."""
    import torch
    n, t0 = 0, time.perf_counter()
    while n < min_steps or time.perf_counter() - t0 < min_s:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    return n, time.perf_counter() - t0


def bench_batch(args, comm: Comm):
    """Configs 2 and 4: `streams` x `stream_mib` per GPU, one batch launch per step."""
    import torch
    from kopia_amd import batch
    from kopia_amd import splitter as ks
    rank, world = comm.rank, comm.world
    local = env_rank_world()[2]
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    name, ns, L = args.splitter, args.streams, args.stream_mib << 20
    info = ks.lookup(name)
    assert info is not None, name
    data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, ns, L, SEED, first_sid=rank * ns)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    # W untimed steps, continued until the warm-up has lasted --warmup-min-s: after idle the
    # chip's clock ramps over ~10 launches (1.6-1.7 ms -> 1.35 ms; profiles/r03/buz/ramp.log),
    # so a 5-step warm-up leaves the first timed launches on the ramp.
    warm_steps, warm_s = warm_up(lambda: batch.split_batch_device(name, b, stream), args.warmup, args.warmup_min_s, dev)

    # One event pair around the K launches (on the launch stream): the average launch duration,
    # init kernel and inter-launch gaps included.  An event pair per launch put ~9 us of timing
    # packets between consecutive launches (kernel traces, profiles/r03/launch_gaps/).
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        batch.split_batch_device(name, b, stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    own = time.perf_counter() - t0
    comm.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / args.steps

    cuts = batch.read_cuts(b)
    rolled = sum(rolled_bytes(c, int(info.min_size)) for c in cuts)
    per = comm.gather({"bytes_per_step": ns * L, "elapsed_s": elapsed, "own_s": own, "kernel_ms": kern_ms,
                       "rolled": rolled})
    agg = aggregate(per, args.steps)
    # traffic is looked up per (kernel, config) and measured for the 4M names only: another
    # average gets its own key (no FETCH pass: traffic null rather than another name's bytes)
    cfg = f"config{args.config}" + ("-rk" if int(info.kind) == 2 else "")
    if name not in ("DYNAMIC-4M-BUZHASH", "DYNAMIC-4M-RABINKARP"):
        cfg += "-" + name
    if (ns, args.stream_mib) not in ((4096, 4), (8192, 8)):  # another shape: its own key, too
        cfg += f"-{ns}x{args.stream_mib}MiB"
    out = {
        "metric": METRIC, "value": agg["value"], "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_steps_run": warm_steps, "warmup_s": round(warm_s, 3),
        "ms_per_step": agg["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"{cfg}: {ns} x {args.stream_mib} MiB independent streams per GPU "
                               f"(counter-PRNG bytes, HBM-resident), {name}",
                   "splitter": name, "streams_per_gpu": ns, "stream_bytes": L, "global_streams": ns * world,
                   "parallelism": f"stream-sharded x{world}, no data-path collectives (gloo timing only)"},
        "per_gpu_gib_s": agg["per_gpu_gib_s"],
    }
    out["roofline"] = roofline(BATCH_KERNEL[int(info.kind)], cfg, kern_ms, rolled, ns * L)
    if "hot_loop_alone_ms" in out["roofline"]:
        out["roofline"]["hot_loop_frac"] = round(out["roofline"]["hot_loop_alone_ms"] / kern_ms, 3)
    out["cut_stats"] = {"chunks": int(sum(c.size for c in cuts)), "rolled_fraction": round(rolled / (ns * L), 4)}

    if args.hash and rank == 0 and world == 1:
        out["hash"] = bench_hash(args, data, ns, L, cuts, dev)
    if args.encrypt and args.hash and rank == 0 and world == 1 and args.pipeline_slots > 0:
        out["pipeline"] = bench_pipeline(args, data, ns, L, cuts, dev)
    if args.encrypt and rank == 0 and world == 1:
        out["encrypt"] = bench_encrypt(args, data, ns, L, cuts, dev)
        out["encrypt_aes"] = bench_encrypt(args, data, ns, L, cuts, dev, "AES256-GCM-HMAC-SHA256")

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
        out["h2d_gib_s"] = h2d_rates(host, dev)
        out["host_inclusive_vs_pageable_h2d"] = round(out["host_inclusive_gib_s"] / out["h2d_gib_s"]["pageable"], 3)
        del host, views

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(name, ns, L, cuts)
        if args.config == 2:
            out["cpu_baseline"]["config1_gb_s_1thread"] = cpu_config1()
    return out


def bench_hash(args, data, ns: int, L: int, cuts: list, dev) -> dict:
    """§8f #2: keyed BLAKE2 content hash of every chunk the split produced
    (repo/content/content_manager.go:812, repo/hashing/hashing.go:78-101), on the device.
    A chunk is one sequential BLAKE2 chain (a quad of lanes), so two figures: the batch alone
    (its 5,7xx chunks: bounded by the longest chunk) and `--hash-inflight` batches' chunk
    tables in one launch (the pipelined upload case: many chunks in flight; the same bytes are
    re-read and re-hashed per table, 16 GiB each).  Each beside the one-lane-per-chunk kernel.
    CPU baseline: hashlib, one thread."""
    import hashlib
    import torch
    from kopia_amd import _lib
    from kopia_amd import hashing as kh
    name, key = args.hash, bytes(range(32))
    offs, lens = kh.chunk_table([i * L for i in range(ns)], cuts)
    total = int(lens.sum())

    def timed(o, ln, reps):
        kh.hash_chunks_device(name, data.data_ptr(), o, ln, key, dev)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            out = kh.hash_chunks_device(name, data.data_ptr(), o, ln, key, dev)
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps, out

    ms1, out = timed(offs, lens, 3)  # auto: a quad of lanes per chunk at this chunk count
    L = _lib.lib()
    L.kcdc_test_set(_lib.TEST_HASH_LANES, 1)
    ms1_lane, _ = timed(offs, lens, 1)  # one lane per chunk, for comparison
    L.kcdc_test_set(_lib.TEST_HASH_LANES, 0)
    # parity of a sample against the oracle (hashlib, RFC 7693; tests/test_hash_oracle.py)
    host = None
    bad = 0
    pick = list(range(0, len(offs), max(1, len(offs) // 48)))
    got = out.cpu().numpy()
    fn, nn, keep = {"BLAKE2B-256-128": (hashlib.blake2b, 32, 16), "BLAKE2B-256": (hashlib.blake2b, 32, 32),
                    "BLAKE2S-128": (hashlib.blake2s, 16, 16), "BLAKE2S-256": (hashlib.blake2s, 32, 32)}[name]
    for i in pick:
        chunk = data[int(offs[i]):int(offs[i] + lens[i])].cpu().numpy().tobytes()
        bad += fn(chunk, key=key, digest_size=nn).digest()[:keep] != got[i].tobytes()
    R = args.hash_inflight
    msR, _ = timed(np.tile(offs, R), np.tile(lens, R), 1)
    L.kcdc_test_set(_lib.TEST_HASH_LANES, 1)
    msR1, _ = timed(np.tile(offs, R), np.tile(lens, R), 1)  # one lane per chunk, for comparison
    L.kcdc_test_set(_lib.TEST_HASH_LANES, 0)
    sample = data[: 256 << 20].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    fn(sample, key=key, digest_size=nn).digest()
    cpu = len(sample) / GiB / (time.perf_counter() - t0)
    return {"algo": name, "batch_chunks": int(len(offs)), "batch_bytes": total, "largest_chunk": int(lens.max()),
            "batch_ms": round(ms1, 3), "batch_gib_s": round(total / GiB / (ms1 * 1e-3), 2),
            "batch_kernel": "4 lanes per chunk" if len(offs) <= (1 << 20) else "1 lane per chunk",
            "batch_1lane_ms": round(ms1_lane, 3),
            "inflight_tables": R, "inflight_chunks": int(R * len(offs)), "inflight_ms": round(msR, 3),
            "inflight_gib_s": round(R * total / GiB / (msR * 1e-3), 2),
            "inflight_kernel": "4 lanes per chunk" if R * len(offs) <= (1 << 20) else "1 lane per chunk",
            "inflight_1lane_ms": round(msR1, 3),
            "sample_parity_mismatches": int(bad), "sample_chunks": len(pick),
            "cpu_hashlib_1thread_gib_s": round(cpu, 3)}


def bench_pipeline(args, data, ns: int, L: int, cuts: list, dev, algo: str = "AES256-GCM-HMAC-SHA256") -> dict:
    """The upload path's device stages over K batches: split -> chunk table (built on the device
    from the cut lists, no host round trip) -> content hash (Kopia's default BLAKE2B-256-128, and
    `--pipeline-hash`) -> seal keyed by the content IDs (Kopia's default AES256-GCM-HMAC-SHA256;
    content_manager.go:812, content_manager_lock_free.go:42-73).  The K splits run first, one
    after another and alone on the GPU (so every launch of the split kernel in this process has
    the same duration and the rocprof average matches the bench's), then each batch's table ->
    hash -> seal runs on stream i % slots, so the batches' hash and seal kernels overlap -- the
    per-chunk hash is one dependent chain per chunk and fills the GPU only with many chunks in
    flight.  Value: the stream bytes of all K batches over the wall time of both phases; each
    stage alone on one batch for comparison.  Parity: a sample of the last batch's digests and
    sealed chunks against the oracle."""
    import ctypes as C
    import torch
    from kopia_amd import _lib, batch
    from kopia_amd import encryption as ke
    from kopia_amd import hashing as kh
    lib = _lib.lib()
    name = args.splitter
    S, K = args.pipeline_slots, args.pipeline_batches
    hashes = [kh.DefaultAlgorithm] + ([args.pipeline_hash] if args.pipeline_hash != kh.DefaultAlgorithm else [])
    secret = ke.derive_key(bytes(range(64, 96)))
    key = bytes(range(32))
    ptrs = [data.data_ptr() + i * L for i in range(ns)]
    bats = [batch.make_device_batch(name, ptrs, [L] * ns, dev) for _ in range(K)]
    cap_per = bats[0].cap // ns
    nent = ns * cap_per
    starts = torch.arange(ns, dtype=torch.int64, device=dev) * L
    jidx = torch.arange(cap_per, dtype=torch.int64, device=dev).view(1, -1)
    nonces = torch.randint(0, 256, (12 * nent,), dtype=torch.uint8, device=dev)
    work_bytes = int(lib.kcdc_crypt_workspace_size(nent))
    split_stream = torch.cuda.current_stream(dev)

    class Slot:
        def __init__(self):
            self.stream = torch.cuda.Stream(dev)
            self.digest = torch.empty((nent, 32), dtype=torch.uint8, device=dev)
            self.sealed = torch.empty(ns * L + 32 * nent, dtype=torch.uint8, device=dev)
            self.status = torch.empty(nent, dtype=torch.int32, device=dev)
            self.work = torch.empty(work_bytes, dtype=torch.uint8, device=dev)

    slots = [Slot() for _ in range(S)]

    def stage_table(sl, b):  # cut lists -> (offsets, lengths, order, sealed offsets) on the device
        with torch.cuda.stream(sl.stream):
            c = b.cuts[:nent].view(ns, cap_per)
            prev = torch.cat([torch.zeros((ns, 1), dtype=torch.int64, device=dev), c[:, :-1]], dim=1)
            valid = jidx < b.counts[:ns].view(-1, 1)
            sl.lens = torch.where(valid, c - prev, torch.zeros_like(c)).reshape(-1).contiguous()
            sl.offs = (starts.view(-1, 1) + torch.where(valid, prev, torch.zeros_like(prev))).reshape(-1).contiguous()
            sl.order = torch.argsort(sl.lens, descending=True).to(torch.int32)
            slen = ((sl.lens + 28 + 3) // 4) * 4
            sl.oo = (torch.cumsum(slen, 0) - slen).contiguous()

    def stage_hash(sl, hname):
        _lib.check(lib.kcdc_hash_chunks_device(hname.encode(), C.c_void_p(data.data_ptr()), sl.offs.data_ptr(),
                                               sl.lens.data_ptr(), sl.order.data_ptr(), nent, key, len(key),
                                               sl.digest.data_ptr(), 32, C.c_void_p(sl.stream.cuda_stream)))

    def stage_seal(sl, hname):
        hs = kh.hash_size(hname)
        _lib.check(lib.kcdc_encrypt_chunks_device(
            algo.encode(), secret, len(secret), C.c_void_p(data.data_ptr()), sl.offs.data_ptr(), sl.lens.data_ptr(),
            nent, C.c_void_p(sl.digest.data_ptr() + hs - 16), 16, 32, nonces.data_ptr(), sl.sealed.data_ptr(),
            sl.oo.data_ptr(), sl.status.data_ptr(), sl.work.data_ptr(), work_bytes, C.c_void_p(sl.stream.cuda_stream)))

    def run(hname):
        for b in bats:  # phase 1: the splits, alone
            batch.split_batch_device(name, b, split_stream)
        done = torch.cuda.Event()
        done.record(split_stream)
        for sl in slots:
            sl.stream.wait_event(done)
        for i, b in enumerate(bats):  # phase 2: hash and seal of the batches, overlapped
            sl = slots[i % S]
            stage_table(sl, b)
            stage_hash(sl, hname)
            stage_seal(sl, hname)

    res = {"slots": S, "batches": K, "encrypt": algo, "chunk_table_entries": nent,
           "valid_chunks": int(sum(c.size for c in cuts))}
    for hname in hashes:
        run(hname)  # warm
        torch.cuda.synchronize(dev)
        alone = {}
        sl, b0 = slots[0], bats[0]
        for stage, fn, st in (("split", lambda: batch.split_batch_device(name, b0, sl.stream), sl.stream),
                              ("table", lambda: stage_table(sl, b0), sl.stream),
                              ("hash", lambda: stage_hash(sl, hname), sl.stream),
                              ("seal", lambda: stage_seal(sl, hname), sl.stream)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            alone[stage] = round(e0.elapsed_time(e1), 3)
        t0 = time.perf_counter()
        run(hname)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        st = torch.stack([s_.status for s_ in slots]).cpu().numpy()
        res[hname] = {"ms_per_batch": round(dt / K * 1e3, 3), "gib_s": round(K * ns * L / GiB / dt, 1),
                      "stages_alone_ms": alone, "serial_sum_ms": round(sum(alone.values()), 3),
                      "status_nonzero": int((st != 0).sum())}
    # parity of the last batch (its slot), on a sample: digest and sealed bytes against the oracle
    from oracle import aesgcm, openssl_aead
    from oracle.hashes import kopia_hash
    seal_ref = openssl_aead.Sealer(algo).kopia_encrypt if openssl_aead.available() else aesgcm.kopia_encrypt
    sl = slots[(K - 1) % S]
    hname = hashes[-1]
    hs = kh.hash_size(hname)
    offs, lens, oo = sl.offs.cpu().numpy(), sl.lens.cpu().numpy(), sl.oo.cpu().numpy()
    dig = sl.digest.cpu().numpy()
    nz = np.nonzero(lens)[0]
    pick = nz[:: max(1, len(nz) // 6)]
    nh = nonces.cpu().numpy().tobytes()
    bad = 0
    for i in pick:
        chunk = data[int(offs[i]):int(offs[i] + lens[i])].cpu().numpy().tobytes()
        d = kopia_hash(hname, key, chunk)
        bad += dig[i, :hs].tobytes() != d
        want = seal_ref(secret, d[hs - 16:], nh[12 * i:12 * i + 12], chunk)
        bad += sl.sealed[int(oo[i]):int(oo[i]) + len(want)].cpu().numpy().tobytes() != want
    res["sample_parity_mismatches"] = int(bad)
    res["sample_chunks"] = int(len(pick))
    return res


def bench_encrypt(args, data, ns: int, L: int, cuts: list, dev, algo: str = "CHACHA20-POLY1305-HMAC-SHA256") -> dict:
    """§8f #4: `algo` (CHACHA20-POLY1305-HMAC-SHA256, or AES256-GCM-HMAC-SHA256, Kopia's default)
    of every chunk the split produced, keyed by its
    content ID (BLAKE2B-256-128 on the device), as content_manager_lock_free.go:178-182 does.
    Times seal (and open) of the whole batch: 4 launches each (key/power table, unit scan,
    byte pass, tag).  Algorithmic HBM bytes: every plaintext byte read once and every sealed
    byte written once (open: the reverse).  Parity: a spread sample against oracle/aead.py."""
    import torch
    from kopia_amd import encryption as ke
    from kopia_amd import hashing as kh
    from oracle import aead, aesgcm
    oracle = aesgcm if algo == ke.Aes256Gcm else aead
    offs, lens = kh.chunk_table([i * L for i in range(ns)], cuts)
    n, total = len(offs), int(lens.sum())
    ids = kh.hash_chunks_device(kh.DefaultAlgorithm, data.data_ptr(), offs, lens, bytes(range(32)), dev).contiguous()
    master = bytes(range(64, 96))
    enc = ke.Encryptor(algo, master)
    nonces = bytes(np.random.default_rng(5).integers(0, 256, 12 * n, dtype=np.uint8))
    oo, sealed_total = ke.sealed_layout(lens)
    out = torch.empty(sealed_total, dtype=torch.uint8, device=dev)
    po, plain_total = ke.plain_layout(lens + 28)
    plain = torch.empty(plain_total, dtype=torch.uint8, device=dev)
    reps = 5

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            st = fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps, st

    seal_ms, st = timed(lambda: enc.encrypt_chunks_device(data.data_ptr(), offs, lens, ids, 16, out, oo, dev,
                                                          nonces=nonces))
    assert not st.cpu().numpy().any()
    open_ms, st2 = timed(lambda: enc.decrypt_chunks_device(out.data_ptr(), oo, lens + 28, ids, 16, plain, po, dev))
    assert not st2.cpu().numpy().any()
    secret, idh = aead.derive_key(master), ids.cpu().numpy()
    pick = list(range(0, n, max(1, n // (8 if algo != ke.Aes256Gcm else 4))))
    bad = 0
    t0 = time.perf_counter()
    for i in pick:
        chunk = data[int(offs[i]):int(offs[i] + lens[i])].cpu().numpy().tobytes()
        want = oracle.kopia_encrypt(secret, idh[i].tobytes(), nonces[12 * i:12 * i + 12], chunk)
        bad += out[int(oo[i]):int(oo[i]) + len(want)].cpu().numpy().tobytes() != want
        bad += plain[int(po[i]):int(po[i] + lens[i])].cpu().numpy().tobytes() != chunk
    oracle_s = time.perf_counter() - t0
    alg = 2 * total + 28 * n
    valu_busy = AES_VALU_BUSY if algo == ke.Aes256Gcm else CHACHA_VALU_BUSY
    return {"algo": algo, "chunks": n, "plaintext_bytes": total,
            "seal_ms": round(seal_ms, 3), "seal_gib_s": round(total / GiB / (seal_ms * 1e-3), 1),
            "open_ms": round(open_ms, 3), "open_gib_s": round(total / GiB / (open_ms * 1e-3), 1),
            # Against HBM: the algorithmic bytes are the plaintext read plus the sealed output
            # written.  The bound that holds the kernel below it is vector ALU work (no AES or
            # carry-less multiply instructions on gfx950; ChaCha20 is ~990 VALU per 64-byte lane
            # block): the SIMDs' measured VALU-busy fraction is the explanation.
            "roofline": {"bound": "hbm", "achieved": round(alg / (seal_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg / (seal_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
                         "traffic": None, "algorithmic_bytes": alg,
                         "limited_by": "VALU", "valu_busy_measured": valu_busy,
                         "timed": "all 4 seal launches (rocprof splits them)"},
            "sample_parity_mismatches": int(bad), "sample_chunks": len(pick),
            "cpu_baseline": cpu_aead_baseline(algo, secret, data, offs, lens, idh, nonces)}


def cpu_aead_baseline(algo, secret, data, offs, lens, idh, nonces) -> dict:
    """The same seal (HMAC-SHA256 key per content + AEAD) by OpenSSL's EVP through ctypes, the
    C-speed stand-in for the reference's Go crypto (oracle/openssl_aead.py; it re-seals the
    reference's ciphertext samples byte for byte, tests/test_aead_oracle.py), on the chunks of
    the batch's first 2 GiB, 1 thread and every usable thread."""
    from oracle import openssl_aead as osl  # oracle import confined to this leg
    if not osl.available():
        return {"value": None, "note": "libcrypto.so.3 not loadable on this host"}
    info = host_cpu_info()
    lim = 2 << 30
    sel = [i for i in range(len(offs)) if int(offs[i] + lens[i]) <= lim]
    host = data[:lim].cpu().numpy()
    so, sl = offs[sel], lens[sel]
    sid = [idh[i].tobytes() for i in sel]
    sn = b"".join(nonces[12 * i:12 * i + 12] for i in sel)
    r1 = osl.seal_rate(algo, secret, host, so[: max(1, len(sel) // 4)], sl[: max(1, len(sel) // 4)], sid, sn, 1)
    ra = osl.seal_rate(algo, secret, host, so, sl, sid, sn, info["threads_all"])
    g1, ga = r1["bytes"] / GiB / r1["seconds"], ra["bytes"] / GiB / ra["seconds"]
    return {"value": round(ga, 2), "unit": "GiB/s", "cores": info["threads_all"], "kind": "library",
            "threads_1": round(g1, 2), "threads_all": round(ga, 2), "threads_all_n": info["threads_all"],
            "cpu_model": info["cpu_model"],
            "sample": f"{len(sel)} chunks ({ra['bytes'] / GiB:.2f} GiB) of this batch sealed by OpenSSL {algo} "
                      f"(EVP + HMAC-SHA256 key per content); 1 thread on a quarter of them"}


def bench_long(args, comm: Comm):
    """Config 3: ONE long stream (default 64 GiB) split exactly by the tiled candidate
    scan + device resolver.  Single GPU (on N ranks each splits its own stream)."""
    import torch
    from kopia_amd import batch
    from kopia_amd import splitter as ks
    local = env_rank_world()[2]
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    name, L = args.splitter, args.long_gib << 30
    info = ks.lookup(name)
    data = torch.empty(L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, 1, L, SEED, first_sid=comm.rank)
    stream = torch.cuda.current_stream(dev)
    cuts, count, ws = batch.split_long_device(name, data.data_ptr(), L, dev, stream)
    torch.cuda.synchronize(dev)
    warm_steps, warm_s = warm_up(lambda: batch.split_long_device(name, data.data_ptr(), L, dev, stream), 1,
                                 args.warmup_min_s, dev)
    steps = max(1, min(args.steps, 10))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    comm.barrier()
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        _c, _n, _w = batch.split_long_device(name, data.data_ptr(), L, dev, stream)
        e1.record(stream)
    torch.cuda.synchronize(dev)
    own = time.perf_counter() - t0
    comm.barrier()
    elapsed = time.perf_counter() - t0
    ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    got = batch.read_long(cuts, count)
    per = comm.gather({"bytes_per_step": L, "elapsed_s": elapsed, "own_s": own})
    agg = aggregate(per, steps)
    out = {"metric": METRIC, "value": agg["value"], "unit": "GiB/s", "n_gpus": comm.world, "steps": steps,
           "warmup": 1, "warmup_steps_run": warm_steps + 1, "warmup_s": round(warm_s, 3), "ms_per_step": agg["ms_per_step"], "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"config3: one {args.long_gib} GiB stream per GPU, exact intra-stream tiled CDC, "
                                  f"{name}", "splitter": name, "stream_bytes": L,
                      "parallelism": "128 KiB segments per wave; one stream per GPU"},
           "per_gpu_gib_s": agg["per_gpu_gib_s"], "kernel_ms_events": round(ms, 3), "cuts": int(got.size)}
    # the long path scans every byte: its algorithmic bytes are the stream bytes
    rk = int(info.kind) == 2
    out["roofline"] = roofline("kcdc::dev::cand_scan_rk_kernel" if rk else "kcdc::dev::cand_scan_dma_kernel<true>",
                               "config3" + ("-rk" if rk else ""), ms, L, L)
    out["roofline"]["algorithmic_bytes_def"] = "every stream byte (the full-scan candidate pass reads each once)"
    if comm.rank == 0 and comm.world == 1 and not args.no_cpu_baseline:
        # the oracle's single sequential pass over the same bytes: the streaming splitter fed
        # 256 MiB slices generated ahead on other threads (only the split is timed)
        from oracle import coracle
        want, split_s = coracle.split_prng_stream_blocks(name, SEED, 0, L)
        out["oracle_parity"] = bool(np.array_equal(got, want))
        out["cpu_baseline"] = {"value": round(L / GiB / split_s, 3), "unit": "GiB/s",
                               "cores": 1, "logical_cores": host_cpu_info()["logical_cores"],
                               "cpu_model": host_cpu_info()["cpu_model"],
                               "kind": "port", "threads_1": round(L / GiB / split_s, 3),
                               "sample": f"the whole {args.long_gib} GiB stream, one sequential NextSplitPoint pass of "
                                         f"oracle/cdc_oracle.c over 256 MiB slices (bytes generated ahead on other "
                                         f"threads, untimed), {name}"}
    return out


def bench_files(args, comm: Comm):
    """Config 5: file sizes from a Zipf law over 19 classes 4 KiB..1 GiB
    (s = 1.1, fixed seed), files_gib x world bytes in total, LPT-balanced over the ranks;
    every rank splits its files with kcdc_split_files_device (each file through the batch
    or the long path).  Weak scaling, no data-path collective.  FIXED names read no data."""
    import torch
    from kopia_amd import batch
    from kopia_amd import dist as kd
    from kopia_amd import splitter as ks
    rank, world = comm.rank, comm.world
    local = env_rank_world()[2]
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sizes = kd.zipf_sizes(args.files_gib * world << 30)
    mine = sorted(kd.lpt_plan(sizes, world)[rank], key=lambda i: int(sizes[i]))
    lens = [int(sizes[i]) for i in mine]
    total = sum(lens)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if lens else np.zeros(0, np.int64)
    k = 0
    while k < len(lens):  # runs of equal sizes are contiguous (sorted): one fill per run
        e = k
        while e < len(lens) and lens[e] == lens[k] and mine[e] == mine[k] + (e - k):
            e += 1
        batch.fill_prng(data[int(offs[k]):], lens[k], e - k, lens[k], SEED, first_sid=int(mine[k]))
        k = e
    ptrs = [data.data_ptr() + int(o) for o in offs]
    stream = torch.cuda.current_stream(dev)

    ev = {}

    def run(name, steps, warmup):
        warm_up(lambda: batch.split_files_device(name, ptrs, lens, dev, stream), warmup, args.warmup_min_s, dev)
        comm.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        res = None
        e0.record(stream)
        for _ in range(steps):
            res = batch.split_files_device(name, ptrs, lens, dev, stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        own = time.perf_counter() - t0
        ev["step_ms"] = e0.elapsed_time(e1) / steps
        comm.barrier()
        return time.perf_counter() - t0, own, res

    name = args.splitter
    steps = max(1, min(args.steps, 10))
    elapsed, own, res = run(name, steps, max(1, min(args.warmup, 2)))
    step_ms = ev["step_ms"]
    agg = aggregate(comm.gather({"bytes_per_step": total, "elapsed_s": elapsed, "own_s": own}), steps)
    out = {"metric": METRIC, "value": agg["value"], "unit": "GiB/s", "n_gpus": world, "steps": steps,
           "warmup": max(1, min(args.warmup, 2)), "ms_per_step": agg["ms_per_step"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"config5: Zipf(s=1.1) file sizes over 4 KiB..1 GiB, {args.files_gib} GiB per GPU, "
                                  f"LPT over {world} rank(s), {name}",
                      "splitter": name, "files_this_rank": len(lens), "bytes_this_rank": total,
                      "largest_file": max(lens) if lens else 0,
                      "parallelism": f"LPT file sharding x{world}, no data-path collectives"},
           "per_gpu_gib_s": agg["per_gpu_gib_s"]}
    got = batch.read_files(*res)
    info = ks.lookup(name)
    if int(info.kind) != 0:  # FIXED names read no data: no roofline
        # The step's kernels (batch kernel for the small files, the long path's scan/prefix/resolve
        # for the large ones, kcdc_split_files_device) timed together with one event pair on the
        # launch stream: rolled bytes R summed over every file's cut list / the step's device time.
        rolled = sum(rolled_bytes(c, int(info.min_size)) for c in got)
        out["roofline"] = roofline("kcdc_split_files_device step (batch + long-path kernels)",
                                   "config5" + ("-rk" if int(info.kind) == 2 else ""), step_ms, rolled, total)
        out["roofline"]["kernel_def"] = ("every kernel of one kcdc_split_files_device call, one HIP event pair around "
                                         "the K steps on the launch stream")
        out["cut_stats"] = {"chunks": int(sum(c.size for c in got)), "rolled_fraction": round(rolled / max(total, 1), 4)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # cpu_baseline leg: the oracle's C restatement on a sample of this rank's files
        # (the 64 smallest, every 8th and the 2 largest), which also checks their GPU cuts
        from oracle import coracle
        pick = sorted(set(range(min(64, len(lens)))) | set(range(0, len(lens), 8)) |
                      set(range(max(0, len(lens) - 2), len(lens))))
        host = [data[int(offs[i]):int(offs[i]) + lens[i]].cpu().numpy() for i in pick]
        nt = host_cpu_info()["threads_all"]
        t0 = time.perf_counter()
        want = coracle.split_batch(name, host, nthreads=nt)
        dt = time.perf_counter() - t0
        sb = sum(lens[i] for i in pick)
        out["cpu_baseline"] = {
            "value": round(sb / GiB / dt, 3), "unit": "GiB/s", "cores": nt,
            "logical_cores": host_cpu_info()["logical_cores"], "kind": "port", "threads_all_n": nt,
            "sample": f"{len(pick)} files of this rank (64 smallest, every 8th, 2 largest; {sb >> 20} MiB), {name}, "
                      f"oracle/cdc_oracle.c, {nt} threads, {dt:.2f}s wall",
            "sample_parity_mismatches": sum(1 for j, i in enumerate(pick) if not np.array_equal(got[i], want[j]))}
    if args.all_names:
        out["per_name_gib_s"] = {}
        for nm in ks.SupportedAlgorithms():
            el, _own, _ = run(nm, 2, 1)
            out["per_name_gib_s"][nm] = round(total * world * 2 / GiB / el, 2)
    return out


def multirank_check(argv):
    """tests/test_gpu_multirank.py: the N>1 path on the device.  Every rank (its GPU: LOCAL_RANK
    modulo the visible devices, so two ranks may share the one GPU of a test box) splits its
    disjoint static shard of config-2-shaped streams through libkcdc and computes the config-5
    LPT plan on its own; rank 0 writes what the ranks gathered over gloo to argv[0].
    argv: out_path, streams per rank, MiB per stream, splitter name."""
    import hashlib

    import torch

    from kopia_amd import batch
    from kopia_amd import dist as kd
    out_path, per, mib, name = argv[0], int(argv[1]), int(argv[2]), argv[3]
    rank, world, local = env_rank_world()
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    comm = Comm(rank, world)
    try:
        L = mib << 20
        ids = kd.static_shard(rank, world, per)
        data = torch.empty(per * L, dtype=torch.uint8, device=dev)
        batch.fill_prng(data, L, per, L, SEED, int(ids[0]))
        b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(per)], [L] * per, dev)
        batch.split_batch_device(name, b)
        torch.cuda.synchronize(dev)
        cuts = batch.read_cuts(b)
        plan = kd.lpt_plan(kd.zipf_sizes(1 << 36), world)
        digest = hashlib.sha256(json.dumps(plan).encode()).hexdigest()
        comm.barrier()
        got = comm.gather({"rank": rank, "device": str(dev), "ids": [int(i) for i in ids],
                           "cuts": [c.tolist() for c in cuts], "plan": digest, "mine": len(plan[rank])})
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(got, f)
    finally:
        comm.close()


def launcher_selftest(argv):
    """Spawn + gloo timing/aggregation without a GPU (tests/test_bench_launcher.py): every
    rank reports made-up timings, rank 0 writes the aggregate to argv[0]."""
    rank, world, _ = env_rank_world()
    comm = Comm(rank, world)
    try:
        comm.barrier()
        per = comm.gather({"bytes_per_step": (rank + 1) << 30, "elapsed_s": 1.0 + rank, "own_s": 0.5 + rank})
        mx = comm.max(float(rank))
        if rank == 0:
            with open(argv[0], "w") as f:
                json.dump({"agg": aggregate(per, 2), "max": mx, "world": world}, f)
    finally:
        comm.close()


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-min-s", type=float, default=0.3,
                    help="keep taking untimed warm-up steps until this many seconds have passed "
                         "(the clock ramps after idle); 0: exactly --warmup steps")
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
    ap.add_argument("--hash", default="BLAKE2B-256-128", help="configs 2/4, one GPU: also hash every chunk on "
                    "the device with this content hash (§8f #2; default Kopia's BLAKE2B-256-128)")
    ap.add_argument("--no-hash", action="store_true", help="skip the content-hash leg")
    ap.add_argument("--pipeline-slots", type=int, default=3, help="split->hash->seal batches in flight (0: skip)")
    ap.add_argument("--pipeline-batches", type=int, default=12, help="batches through the overlapped pipeline")
    ap.add_argument("--pipeline-hash", default="BLAKE3-256-128", help="second hash timed through the pipeline")
    ap.add_argument("--encrypt", action="store_true", default=True,
                    help="configs 2/4, one GPU: also seal/open every chunk with CHACHA20-POLY1305-HMAC-SHA256 "
                         "(§8f #4; on by default)")
    ap.add_argument("--no-encrypt", action="store_true", help="skip the encryption leg")
    ap.add_argument("--hash-inflight", type=int, default=24, help="--hash: chunk tables per launch, throughput figure")
    args = ap.parse_args(argv)
    if args.no_hash:
        args.hash = None
    if args.no_encrypt:
        args.encrypt = False
    if args.config == 4:
        args.streams, args.stream_mib = 8192, 8
    return args


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rank, world, _local = env_rank_world()
    if "RANK" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, argv)  # this process never touches a GPU
    comm = Comm(rank, world)
    try:
        fn = {2: bench_batch, 4: bench_batch, 3: bench_long, 5: bench_files}[args.config]
        out = fn(args, comm)
        if rank == 0:
            print(json.dumps(out), flush=True)
    finally:
        comm.close()


if __name__ == "__main__":
    main()
