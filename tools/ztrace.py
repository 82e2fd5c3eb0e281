"""Phase times of zstd_emit_kernel (the span-level zstd writer) from a KCDC_TRACE build.

Runs one zstd compression of the mixed bench data through build/libkcdc_trace.so, reads lane
0's s_memtime stamps (descriptor words 64.. of each span: kcdc_compress.hip KCDC_ZSTAMP) back
from the workspace, and prints each phase's mean cycles per span.
usage: KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 python tools/ztrace.py [MiB] [name]
(a deflate name: the parse and plan cycles of lz_spans_kernel<deflate> instead)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from compress_bench import mixed  # noqa: E402
from kopia_amd import _lib  # noqa: E402
from kopia_amd import compression as kc  # noqa: E402

SLOT, SPAN, DESC_WORDS = 576, 32768, 288
PHASES = ["stage+seq copy+carry", "literal/code counts", "huffman", "fse tables", "stream bits",
          "fse pass", "decision", "literal writes+move", "headers+merge"]


def a256(x):
    return (x + 255) & ~255


def ws(n, spans):  # kcdc_compress.hip comp_ws
    crc = a256((n + 1) * 4)
    span_crc = a256(crc + n * 4)
    seglen = a256(span_crc + spans * 4)
    span_bytes = a256(seglen + spans * 64 * 4)
    span_pos = a256(span_bytes + spans * 4)
    slots = a256(span_pos + (spans + 1) * 8)
    desc = a256(slots + spans * 64 * SLOT)
    return desc, a256(desc + spans * 4 * DESC_WORDS)


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    name = sys.argv[2] if len(sys.argv) > 2 else "zstd"
    dev = torch.device("cuda:0")
    host = mixed(mib << 20, 9)
    d = torch.from_numpy(host).to(dev)
    lens = [4 << 20] * (host.size // (4 << 20))
    offs = np.arange(len(lens), dtype=np.int64) * (4 << 20)
    n = len(lens)
    oo, total = kc.compressed_layout(lens)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    d_offs = torch.as_tensor(offs).to(dev)
    d_lens = torch.as_tensor(np.asarray(lens, np.int64)).to(dev)
    d_oo = torch.as_tensor(oo).to(dev)
    ol = torch.zeros(n, dtype=torch.int64, device=dev)
    ids = torch.zeros(n, dtype=torch.int32, device=dev)
    wb = int(_lib.lib().kcdc_compress_workspace_size(int(sum(lens)), n))
    work = torch.zeros(wb, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().kcdc_compress_chunks_device(
        name.encode(), d.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, out.data_ptr(), d_oo.data_ptr(),
        ol.data_ptr(), ids.data_ptr(), work.data_ptr(), wb, None))
    torch.cuda.synchronize()
    fixed = ws(n, 0)[1]
    per = 64 * (SLOT + 4) + 4 + 4 + 8 + 4 * DESC_WORDS
    ms = (wb - fixed) // per
    while ms > 0 and ws(n, ms)[1] > wb:
        ms -= 1
    desc_off = ws(n, ms)[0]
    spans = sum((L + SPAN - 1) // SPAN for L in lens)
    w = work.cpu().numpy()
    desc = w[desc_off:desc_off + spans * 4 * DESC_WORDS].view(np.uint32).reshape(spans, DESC_WORDS)
    if name.startswith("deflate"):  # lz_spans_kernel<deflate>: u32 stamps at words 281..287
        tw = desc[:, 281:288].astype(np.int64)
        dd = (np.diff(tw, axis=1) % (1 << 32)).astype(np.float64)
        names = ["parse", "plan: counts", "plan: code lengths", "plan: header", "plan: segment bits",
                 "plan: layout and descriptor"]
        out = {"name": name, "spans": int(spans), "ratio": float(ol.sum().item()) / host.size}
        dyn = tw[:, 3] != 0  # spans with a dynamic code (the other spans skip stamps 3)
        for i, n in enumerate(names):
            rows = dyn if i in (2, 3) else np.ones(len(dd), bool)
            out[n] = round(float(dd[rows, i].mean()), 1) if rows.any() else None
        out["dynamic_spans"] = int(dyn.sum())
        print(json.dumps(out, indent=1))
        return
    st = desc[:, 64:84].copy().view(np.uint64).astype(np.int64)  # [spans, 10]
    dt = np.diff(st, axis=1)
    res = {"spans": int(spans), "ratio": float(ol.sum().item()) / host.size,
           "total_cycles_mean": float((st[:, 9] - st[:, 0]).mean())}
    for i, name in enumerate(PHASES):
        res[name] = {"mean": round(float(dt[:, i].mean()), 1), "p90": float(np.percentile(dt[:, i], 90))}
    seqs = desc[:, :64].astype(np.int64).sum(axis=1)
    res["sequences_per_span_mean"] = float(seqs.mean())
    # the FSE phase against the longest block's sequence count: cycles per chained sequence
    mx = desc[:, :64].astype(np.int64).reshape(spans, 4, 16).sum(axis=2).max(axis=1)
    fse = dt[:, PHASES.index("fse pass")].astype(np.float64)
    a, b0 = np.polyfit(mx.astype(np.float64), fse, 1)
    res["fse_cycles_per_sequence_fit"] = {"slope": round(float(a), 1), "intercept": round(float(b0), 1),
                                          "longest_block_mean": float(mx.mean())}
    sub = desc[:, 92:96].copy().view(np.uint64).astype(np.int64)  # huffman: lengths done, weights table done
    hs = sub[:, 0] > 0
    if hs.any():
        res["huffman_split"] = {"spans_with_code": int(hs.sum()),
                                "lengths": round(float((sub[hs, 0] - st[hs, 2]).mean()), 1),
                                "codes+weights_table": round(float((sub[hs, 1] - sub[hs, 0]).mean()), 1),
                                "weights_encode": round(float((st[hs, 3] - sub[hs, 1]).mean()), 1)}
    bud = desc[:, 84:92].astype(np.int64).sum(axis=0)
    names = ["raw_blocks", "literal_sections", "sequence_bitstreams", "table_descriptions", "huffman_trees",
             "headers", "coded_literals", "coded_sequences"]
    res["bytes_per_span"] = {n: round(float(v) / spans, 1) for n, v in zip(names, bud)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
