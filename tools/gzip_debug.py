"""Debug aid: device gzip members of a few chunks, their CRC-32 / ISIZE trailers against zlib."""
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kopia_amd import compression as kc
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    host = np.concatenate([np.zeros(10000, np.uint8), rng.integers(0, 256, 10000, dtype=np.uint8),
                           np.arange(70001, dtype=np.uint8), np.zeros(1, np.uint8)])
    offs, lens = [0, 10000, 20000, 1, 20003], [10000, 10000, 40000, 513, 0]
    d = torch.from_numpy(host).to(dev)
    oo, total = kc.compressed_layout(lens)
    out = torch.zeros(total, dtype=torch.uint8, device=dev)
    ol, ids = kc.Compressor("gzip").compress_chunks_device(d.data_ptr(), offs, lens, out, oo, dev)
    torch.cuda.synchronize()
    o, ol = out.cpu().numpy(), ol.cpu().numpy()
    for i, (a, n) in enumerate(zip(offs, lens)):
        blob = o[oo[i]:oo[i] + ol[i]].tobytes()
        crc = int.from_bytes(blob[-8:-4], "little")
        print(i, n, "len", ol[i], "dev crc", hex(crc), "zlib", hex(zlib.crc32(host[a:a + n].tobytes())),
              "isize", int.from_bytes(blob[-4:], "little"), "hdr", blob[:14].hex())


if __name__ == "__main__":
    main()
