"""Deflate compression throughput on the device (kcdc_compress_chunks_device) with the output
inflated back through zlib on a sample, the ratio beside zlib's (fixed Huffman and level 6),
and a 1-thread zlib rate on the host.  Inputs:
  random   config-2 bytes (uniform PRNG; every segment is stored), 16 GiB in DYNAMIC-4M chunks
  pattern  the reference benchmark's 1..10 pattern and zeros (compressor_test.go:92-93)
  mixed    random / zero / periodic / word-salad stretches (tests/test_gpu_compress.py)
Usage: python tools/compress_bench.py [--gib 16] [--name deflate-default] [--iters 5]"""
import argparse
import json
import os
import sys
import time
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kopia_amd import _lib  # noqa: E402
from kopia_amd import compression as kc  # noqa: E402
from oracle import deflate  # noqa: E402


def mixed(nbytes, seed):
    rng = np.random.default_rng(seed)
    words = [b"kopia", b"snapshot", b"content", b"chunk", b"the", b"of", b"blob", b"index", b" ", b"\n"]
    out, size = [], 0
    while size < nbytes:
        kind = int(rng.integers(0, 4))
        n = int(rng.integers(1, 20000))
        if kind == 0:
            s = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            s = bytes(n)
        elif kind == 2:
            p = rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
            s = (p * (n // len(p) + 1))[:n]
        else:
            s = b"".join(words[int(k)] for k in rng.integers(0, len(words), n // 4 + 1))[:n]
        out.append(s)
        size += len(s)
    return np.frombuffer(b"".join(out)[:nbytes], np.uint8).copy()


def run(name, d, offs, lens, iters, dev):
    n = len(offs)
    oo, total = kc.compressed_layout(lens)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    comp = kc.Compressor(name)
    d_offs = torch.as_tensor(np.asarray(offs, np.int64)).to(dev)
    d_lens = torch.as_tensor(np.asarray(lens, np.int64)).to(dev)
    d_oo = torch.as_tensor(oo).to(dev)
    ol = torch.zeros(n, dtype=torch.int64, device=dev)
    ids = torch.zeros(n, dtype=torch.int32, device=dev)
    wb = int(_lib.lib().kcdc_compress_workspace_size(int(np.sum(lens)), n))
    work = torch.empty(wb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)

    def once():
        _lib.check(_lib.lib().kcdc_compress_chunks_device(
            name.encode(), d.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, out.data_ptr(), d_oo.data_ptr(),
            ol.data_ptr(), ids.data_ptr(), work.data_ptr(), wb, st.cuda_stream))

    once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        once()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, out, oo, ol.cpu().numpy(), ids.cpu().numpy(), comp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--name", default="deflate-default")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    total = int(args.gib * (1 << 30))
    res = {"name": args.name, "device_time_excludes_h2d": True}
    chunk = 4 << 20
    for kind in ["random", "pattern", "mixed"]:
        if args.only and kind != args.only:
            continue
        if kind == "random":
            d = torch.empty(total, dtype=torch.uint8, device=dev)
            _lib.check(_lib.lib().kcdc_fill_prng(d.data_ptr(), total, total, 1, 0x6B6F706961, 0, None))
            torch.cuda.synchronize()
            nbytes = total
        else:
            base = (np.tile(np.arange(1, 11, dtype=np.uint8), (64 << 20) // 10 + 1)[:64 << 20] if kind == "pattern"
                    else mixed(64 << 20, 9))
            if kind == "pattern":
                base[32 << 20:] = 0
            reps = max(1, total // base.size // 4)  # 1/4 of --gib: host-built data is uploaded once
            d = torch.from_numpy(base).to(dev).repeat(reps)
            nbytes = d.numel()
        rng = np.random.default_rng(1)
        lens, pos = [], 0
        while pos < nbytes:  # ~4 MiB chunks (DYNAMIC-4M's range)
            L = min(int(rng.integers(chunk // 2, 2 * chunk)), nbytes - pos)
            lens.append(L)
            pos += L
        offs = np.concatenate(([0], np.cumsum(lens)[:-1])).astype(np.int64)
        ms, out, oo, ol, ids, comp = run(args.name, d, offs, lens, args.iters, dev)
        # Inflate a sample of the chunks back through zlib.
        host_out = out.cpu().numpy()
        sample = list(range(0, len(lens), max(1, len(lens) // 16)))
        for i in sample:
            src = d[int(offs[i]):int(offs[i]) + lens[i]].cpu().numpy().tobytes()
            assert deflate.decompress(args.name, host_out[oo[i]:oo[i] + ol[i]].tobytes()) == src, (kind, i)
        ratio = float(np.sum(ol)) / nbytes
        one = d[:min(nbytes, 16 << 20)].cpu().numpy().tobytes()
        t0 = time.perf_counter()
        z6 = len(zlib.compress(one, 6))
        cpu_s = time.perf_counter() - t0
        co = zlib.compressobj(6, zlib.DEFLATED, -15, 9, zlib.Z_FIXED)
        zf = len(co.compress(one) + co.flush())
        res[kind] = {
            "bytes": nbytes, "chunks": len(lens), "ms": round(ms, 3), "GiB_s": round(nbytes / ms / 1e6 / 1.073741824, 1),
            "ratio": round(ratio, 4), "kept_compressed": int((ids != 0).sum()),
            "zlib_level6_ratio_16MiB": round(z6 / len(one), 4), "zlib_fixed_huffman_ratio_16MiB": round(zf / len(one), 4),
            "zlib_level6_1thread_MiB_s": round(len(one) / cpu_s / (1 << 20), 1),
            "inflated_sample_chunks": len(sample),
        }
        print(json.dumps({kind: res[kind]}), flush=True)
        del d, out
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
