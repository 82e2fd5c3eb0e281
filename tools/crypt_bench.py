"""Seal/open timing of a device encryptor (--algo) over a synthetic chunk table (A/B of
library builds via KCDC_LIB (with KCDC_ALLOW_VARIANT_LIB=1); not a parity test -- tests/test_gpu_crypt.py is)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--avg-mib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--algo", default="CHACHA20-POLY1305-HMAC-SHA256")
    args = ap.parse_args()
    import torch
    from kopia_amd import encryption as ke
    dev = torch.device("cuda", 0)
    total = int(args.gib * (1 << 30))
    rng = np.random.default_rng(1)
    avg = int(args.avg_mib * (1 << 20))
    lens = []
    while sum(lens) < total - 2 * avg:
        lens.append(int(rng.integers(avg // 2, avg * 2)))
    lens = np.array(lens, np.int64)
    offs = np.concatenate(([3], 3 + np.cumsum(lens)[:-1])).astype(np.int64)  # misaligned
    data = torch.randint(0, 256, (int(offs[-1] + lens[-1] + 8),), dtype=torch.uint8, device=dev)
    ids = torch.randint(0, 256, (len(lens), 16), dtype=torch.uint8, device=dev)
    enc = ke.Encryptor(args.algo, bytes(range(32)))
    oo, st_total = ke.sealed_layout(lens)
    out = torch.empty(st_total, dtype=torch.uint8, device=dev)
    po, pt_total = ke.plain_layout(lens + 28)
    plain = torch.empty(pt_total, dtype=torch.uint8, device=dev)
    nonces = bytes(12 * len(lens))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    seal = timed(lambda: enc.encrypt_chunks_device(data.data_ptr(), offs, lens, ids, 16, out, oo, dev, nonces=nonces))
    opn = timed(lambda: enc.decrypt_chunks_device(out.data_ptr(), oo, lens + 28, ids, 16, plain, po, dev))
    b = int(lens.sum())
    print(json.dumps({"lib": os.environ.get("KCDC_LIB", "default"), "chunks": len(lens), "bytes": b,
                      "seal_ms": round(seal, 3), "seal_gib_s": round(b / (1 << 30) / seal * 1e3, 1),
                      "open_ms": round(opn, 3), "open_gib_s": round(b / (1 << 30) / opn * 1e3, 1),
                      "seal_hbm_frac": round((2 * b) / (seal * 1e-3) / 8e12, 3)}))


if __name__ == "__main__":
    main()
