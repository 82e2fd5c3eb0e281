"""Saves the zstd chunks of the ragged-chunks test case that libzstd rejects (diagnosis aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_compress import _compress, _mixed  # noqa: E402
from oracle import deflate  # noqa: E402

out_dir = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "zstd"
os.makedirs(out_dir, exist_ok=True)
host = _mixed(24 << 20, 11)
rng = np.random.default_rng(12)
edge = [0, 1, 2, 3, 4, 5, 7, 8, 255, 511, 512, 513, 1023, 1024, 1025, 4096, 32767, 32768, 32769,
        65535, 65536, 65537, 100000, (1 << 20) + 3]
lens = edge + [int(x) for x in rng.integers(0, 300000, 200)]
offs = [int(rng.integers(0, host.size - L)) for L in lens]
out, oo, ol, ids = _compress(name, host, offs, lens, torch.device("cuda:0"))
bad = 0
for i, (o, n) in enumerate(zip(offs, lens)):
    blob = out[oo[i]:oo[i] + ol[i]].tobytes()
    exp = host[o:o + n].tobytes()
    try:
        ok = deflate.decompress(name, blob) == exp
    except ValueError:
        ok = False
    if not ok:
        if bad < 6:
            np.savez(os.path.join(out_dir, f"fail_{i}.npz"), blob=np.frombuffer(blob, np.uint8),
                     exp=np.frombuffer(exp, np.uint8))
        bad += 1
print("chunks", len(lens), "bad", bad)
