"""Content-hash timing on a synthetic chunk table shaped like one config-2 batch (A/B of
library builds via KCDC_LIB (with KCDC_ALLOW_VARIANT_LIB=1); parity is tests/test_gpu_hash.py)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kopia_amd import hashing as kh
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    lens = rng.integers(2 << 20, 6 << 20, 5700).astype(np.int64)
    lens[0] = 4 << 20
    offs = np.concatenate(([0], np.cumsum(lens)[:-1])).astype(np.int64)
    data = torch.randint(0, 256, (int(lens.sum()) + 64,), dtype=torch.uint8, device=dev)
    key = bytes(range(32))
    out = {}
    names = sys.argv[1:] or kh.SupportedAlgorithms()
    for name in names:
        kh.hash_chunks_device(name, data.data_ptr(), offs, lens, key, dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            kh.hash_chunks_device(name, data.data_ptr(), offs, lens, key, dev)
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) / 3, 2)
    total = int(lens.sum())
    print(json.dumps({"lib": os.environ.get("KCDC_LIB", "default"), "ms": out, "chunks": len(lens),
                      "bytes": total, "gib_s": {k: round(total / 2**30 / (v * 1e-3), 1) for k, v in out.items()},
                      "largest": int(lens.max())}))


if __name__ == "__main__":
    main()
