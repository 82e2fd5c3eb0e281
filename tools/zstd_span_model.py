"""Host model of the span-level zstd block layout (round 6), checked against the system libzstd.

The device encoder (kopia_amd/csrc/kcdc_compress.hip) parses a chunk in 32 KiB spans of 64
512-byte segments (one lane each).  Until round 6 every segment was its own zstd block: a block
header, a literals header and a sequences header with its FSE states per 512 bytes.  This model
restates the bitstream layout of the alternative -- one block per G segments, the span's Huffman
literal code carried by its first block and reused by the others (Treeless), the literals in one
or four Huffman streams, the block's sequences through the predefined FSE tables, and repeat
offset 1 for a match at the previous match's distance -- and measures the ratio of each layout on
the same parse, every frame decoded by libzstd.  It is a design check for the device code, not a
test oracle (the tests decode the device's frames with libzstd directly).

usage: python tools/zstd_span_model.py [MiB]
"""
import heapq
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle.deflate import zstd_decode, zstd_encode  # noqa: E402

SEG, SPAN = 512, 32768

# ---------------------------------------------------------------- predefined FSE tables (RFC 8878)
LL_NORM = [4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
           -1, -1, -1, -1]
ML_NORM = [1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
           1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1]
OF_NORM = [1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1]


class Fse:
    """The encoder side of a predefined table, as kcdc_compress.hip's FseTab."""

    def __init__(self, norm, al):
        size = 1 << al
        sym, nb, base = [0] * size, [0] * size, [0] * size
        nxt = [0] * len(norm)
        high = size - 1
        for s, n in enumerate(norm):
            if n == -1:
                sym[high] = s
                high -= 1
                nxt[s] = 1
            else:
                nxt[s] = n
        pos, step = 0, (size >> 1) + (size >> 3) + 3
        for s, n in enumerate(norm):
            for _ in range(max(n, 0)):
                sym[pos] = s
                pos = (pos + step) & (size - 1)
                while pos > high:
                    pos = (pos + step) & (size - 1)
        self.enc = [[0] * size for _ in norm]
        self.first = [0] * len(norm)
        for u in range(size):
            s = sym[u]
            ns = nxt[s]
            nxt[s] += 1
            hb = ns.bit_length() - 1
            nb[u] = al - hb
            base[u] = (ns << (al - hb)) - size
            self.first[s] = u
            for t in range(base[u], base[u] + (1 << nb[u])):
                self.enc[s][t] = u
        self.nb, self.base = nb, base


FLL, FML, FOF = Fse(LL_NORM, 6), Fse(ML_NORM, 6), Fse(OF_NORM, 5)


def ll_code(ll):
    if ll < 16:
        return ll, 0, 0
    if ll < 64:
        base = [16, 18, 20, 22, 24, 28, 32, 40, 48]
        bits = [1, 1, 1, 1, 2, 2, 3, 3, 4]
        c = max(i for i in range(9) if base[i] <= ll)
        return 16 + c, bits[c], ll - base[c]
    h = ll.bit_length() - 1
    return h + 19, h, ll - (1 << h)


def ml_code(ml):
    m = ml - 3
    if m < 32:
        return m, 0, 0
    if ml < 131:
        base = [35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99]
        bits = [1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5]
        c = max(i for i in range(11) if base[i] <= ml)
        return 32 + c, bits[c], ml - base[c]
    h = m.bit_length() - 1
    return h + 36, h, m - (1 << h)


class BitW:
    def __init__(self):
        self.out, self.bb, self.nb = bytearray(), 0, 0

    def put(self, v, n):
        self.bb |= (v & ((1 << n) - 1)) << self.nb
        self.nb += n
        while self.nb >= 8:
            self.out.append(self.bb & 255)
            self.bb >>= 8
            self.nb -= 8

    def close(self):  # end marker, then pad to a byte
        self.put(1, 1)
        if self.nb:
            self.put(0, 8 - self.nb)
        return bytes(self.out)


def sequences_section(seqs):
    """seqs: (ll, ml, offset_value) in order.  Predefined modes; backwards as zstd_seqs."""
    n = len(seqs)
    hdr = bytearray([n] if n < 128 else [128 + (n >> 8), n & 255])
    if n == 0:
        return bytes(hdr)
    hdr.append(0)  # Predefined_Mode x 3
    w = BitW()
    sLL = sML = sOF = 0
    for k in range(n - 1, -1, -1):
        ll, ml, ov = seqs[k]
        llc, llb, llx = ll_code(ll)
        mlc, mlb, mlx = ml_code(ml)
        ofc = ov.bit_length() - 1
        ofx = ov - (1 << ofc)
        if k == n - 1:
            sLL, sML, sOF = FLL.first[llc], FML.first[mlc], FOF.first[ofc]
        else:
            for f, sym, attr in ((FOF, ofc, "sOF"), (FML, mlc, "sML"), (FLL, llc, "sLL")):
                s = {"sOF": sOF, "sML": sML, "sLL": sLL}[attr]
                ns = f.enc[sym][s]
                w.put(s - f.base[ns], f.nb[ns])
                if attr == "sOF":
                    sOF = ns
                elif attr == "sML":
                    sML = ns
                else:
                    sLL = ns
        w.put(llx, llb)
        w.put(mlx, mlb)
        w.put(ofx, ofc)
    w.put(sML, 6)
    w.put(sOF, 5)
    w.put(sLL, 6)
    return bytes(hdr) + w.close()


# ---------------------------------------------------------------- Huffman literals
def huff_lengths(freq, maxb=11):
    """Length-limited Huffman code lengths (package-merge)."""
    syms = [s for s in range(256) if freq[s]]
    if len(syms) < 2:
        return None
    items = sorted((freq[s], [s]) for s in syms)
    lens = [0] * 256
    pk = list(items)
    for _ in range(maxb - 1):
        merged = []
        for i in range(0, len(pk) - 1, 2):
            merged.append((pk[i][0] + pk[i + 1][0], pk[i][1] + pk[i + 1][1]))
        pk = sorted(items + merged, key=lambda t: t[0])
    for _, ss in pk[:2 * len(syms) - 2]:
        for s in ss:
            lens[s] += 1
    return lens


def huff_table(lens):
    """zstd canonical codes (by weight ascending, then symbol) and the direct-weights description."""
    top = max(s for s in range(256) if lens[s])
    if top > 128:
        return None
    maxb = max(lens)
    w = [maxb + 1 - lens[s] if lens[s] else 0 for s in range(256)]
    num = [0] * (maxb + 2)
    for s in range(top + 1):
        if w[s]:
            num[w[s]] += 1
    start, acc = [0] * (maxb + 2), 0
    for wt in range(1, maxb + 1):
        start[wt] = acc >> (wt - 1)
        acc += num[wt] << (wt - 1)
    codes = {}
    for s in range(top + 1):
        if w[s]:
            codes[s] = (start[w[s]], lens[s])
            start[w[s]] += 1
    desc = bytearray([127 + top])
    for j in range(0, top, 2):
        w0 = w[j]
        w1 = w[j + 1] if j + 1 < top else 0
        desc.append((w0 << 4) | w1)
    return codes, bytes(desc)


def huff_stream(lits, codes):
    w = BitW()
    for c in reversed(lits):
        v, n = codes[c]
        w.put(v, n)
    return w.close()


def literals_section(lits, codes, desc):
    """Raw when codes is None; else Compressed (desc given) or Treeless (desc None)."""
    n = len(lits)
    if codes is None:
        if n < 32:
            return bytes([n << 3]) + bytes(lits)
        if n < 4096:
            return bytes([0b0100 | ((n & 15) << 4), n >> 4]) + bytes(lits)
        return bytes([0b1100 | ((n & 15) << 4), (n >> 4) & 255, n >> 12]) + bytes(lits)
    typ = 2 if desc else 3
    tree = desc or b""
    if n <= 1023:
        body = tree + huff_stream(lits, codes)
        sf, streams = 0, 1
    else:
        q = (n + 3) // 4
        parts = [lits[0:q], lits[q:2 * q], lits[2 * q:3 * q], lits[3 * q:]]
        ss = [huff_stream(p, codes) for p in parts]
        jump = b"".join(len(s).to_bytes(2, "little") for s in ss[:3])
        body = tree + jump + b"".join(ss)
        streams = 4
    c = len(body)
    if streams == 1:
        if c > 1023:
            return None
        v = typ | (0 << 2) | (n << 4) | (c << 14)
        return v.to_bytes(3, "little") + body
    if n <= 1023 and c <= 1023:
        v = typ | (1 << 2) | (n << 4) | (c << 14)
        return v.to_bytes(3, "little") + body
    if n <= 16383 and c <= 16383:
        v = typ | (2 << 2) | (n << 4) | (c << 18)
        return v.to_bytes(4, "little") + body
    v = typ | (3 << 2) | (n << 4) | (c << 22)
    return v.to_bytes(5, "little") + body


# ---------------------------------------------------------------- a parse like the device's
def parse_span(span):
    """Per 512-byte segment: greedy matches (>= 4 bytes, inside the segment), candidates the
    previous match's distance and the most recent position of the 4-byte hash in the span.
    Returns per segment [(ll, ml, dist), ...] and its trailing literal count."""
    last = {}
    segs = []
    for x0 in range(0, len(span), SEG):
        xe = min(len(span), x0 + SEG)
        seqs, x, lit, last_d = [], x0, x0, 0
        while x + 4 <= xe:
            key = span[x:x + 4]
            best, bd = 0, 0
            cands = []
            if last_d and x - last_d >= 0:
                cands.append(x - last_d)
            if key in last:
                cands.append(last[key])
            for c in cands:
                n = 0
                while x + n < xe and span[c + n] == span[x + n] and n < 65535:
                    n += 1
                if n > best or (n == best and n and x - c < bd):
                    best, bd = n, x - c
            last[key] = x
            if best >= 4:
                seqs.append((x - lit, best, bd))
                for y in range(x + 1, min(x + best, xe - 3)):
                    last[span[y:y + 4]] = y
                last_d = bd
                x += best
                lit = x
            else:
                x += 1
        segs.append((seqs, xe - lit))
    return segs


def frame_header(n):
    fcs = 1 if n < 256 else 2 if n < 65536 + 256 else 4
    flag = {1: 0, 2: 1, 4: 2}[fcs]
    v = n - 256 if fcs == 2 else n
    return b"\x28\xb5\x2f\xfd" + bytes([(flag << 6) | 0x20]) + v.to_bytes(fcs, "little")


def encode_chunk(data, G, rep, huff=True):
    """One frame: blocks of G segments (G = 1: the round-5 layout, minus its raw fallbacks)."""
    out = bytearray(frame_header(len(data)))
    for s0 in range(0, len(data), SPAN):
        span = data[s0:s0 + SPAN]
        segs = parse_span(span)
        # the span's literals (for its one Huffman code)
        freq = [0] * 256
        seg_lits = []
        for i, (seqs, tail) in enumerate(segs):
            x = i * SEG
            lits = []
            for ll, ml, _ in seqs:
                lits += span[x:x + ll]
                x += ll + ml
            lits += span[x:x + tail]
            seg_lits.append(lits)
            for c in lits:
                freq[c] += 1
        codes = desc = None
        if huff:
            lens = huff_lengths(freq)
            t = huff_table(lens) if lens else None
            if t:
                codes, desc = t
        span_out = bytearray()
        prev_off = None  # the first sequence of a span never uses a repeat offset
        carry = 0
        for g0 in range(0, len(segs), G):
            lits, seqs = [], []
            for i in range(g0, min(g0 + G, len(segs))):
                sq, tail = segs[i]
                lits += seg_lits[i]
                for k, (ll, ml, d) in enumerate(sq):
                    ll2 = ll + (carry if k == 0 else 0)
                    ov = 1 if rep and ll2 > 0 and d == prev_off else d + 3
                    seqs.append((ll2, ml, ov))
                    prev_off = d
                # literals pending since the block's last sequence (an all-literal segment adds all)
                carry = (tail if sq else carry + len(seg_lits[i]))
            carry = 0  # a block's trailing literals are its last literals
            ls = literals_section(lits, codes, desc) if codes else None
            coded = ls is not None
            if ls is None:
                ls = literals_section(lits, None, None)
            body = ls + sequences_section(seqs)
            raw = span[g0 * SEG:min(len(span), (g0 + G) * SEG)]
            if len(body) >= len(raw):  # a Raw_Block (it carries no table: the next block may)
                out_blk = ((len(raw) << 3) | 0).to_bytes(3, "little") + bytes(raw)
            else:
                out_blk = ((len(body) << 3) | (2 << 1)).to_bytes(3, "little") + body
                if coded:
                    desc = None  # later blocks reuse the table (Treeless)
            span_out += out_blk
        out += span_out
    out += b"\x01\x00\x00"  # last block: empty Raw_Block
    return bytes(out)


def main():
    from compress_bench import mixed
    mib = float(sys.argv[1]) if len(sys.argv) > 1 else 1
    data = mixed(int(mib * (1 << 20)), 9)
    data = bytes(data) if not isinstance(data, bytes) else data
    print(f"{len(data)} bytes of mixed data; zstd -3 ratio {len(zstd_encode(data, 3)) / len(data):.4f}")
    chunk = 4 << 20
    for G, rep in ((1, False), (8, False), (16, False), (64, False), (16, True), (64, True)):
        tot = 0
        for c0 in range(0, len(data), chunk):
            blob = encode_chunk(data[c0:c0 + chunk], G, rep)
            assert zstd_decode(blob) == data[c0:c0 + chunk], (G, rep)
            tot += len(blob)
        print(f"blocks of {G:2d} segments, repeat offsets {'on ' if rep else 'off'}: ratio {tot / len(data):.4f}")


if __name__ == "__main__" and len(sys.argv) <= 2 and (len(sys.argv) < 2 or sys.argv[1] != "fseweights"):
    main()


def stats(mib=1):
    """Where a span-level frame's bytes go: literals vs sequences, and what ideal (order-0
    entropy) codes for the LL / ML / OF symbols would cost against the predefined tables."""
    import math
    from compress_bench import mixed
    data = bytes(mixed(int(mib * (1 << 20)), 9))
    cnt = {"LL": {}, "ML": {}, "OF": {}}
    extra = 0
    nseq = nrep = nlit = 0
    for s0 in range(0, len(data), SPAN):
        prev = None
        for sq, tail in parse_span(data[s0:s0 + SPAN]):
            for ll, ml, d in sq:
                ov = 1 if (ll > 0 and d == prev) else d + 3
                nrep += ov == 1
                prev = d
                llc, llb, _ = ll_code(ll)
                mlc, mlb, _ = ml_code(ml)
                ofc = ov.bit_length() - 1
                for k, c in (("LL", llc), ("ML", mlc), ("OF", ofc)):
                    cnt[k][c] = cnt[k].get(c, 0) + 1
                extra += llb + mlb + ofc
                nseq += 1
                nlit += ll
            nlit += tail
    ent = 0.0
    for k, h in cnt.items():
        n = sum(h.values())
        ent += sum(-c * math.log2(c / n) for c in h.values())
    # the predefined-table cost: the bits the FSE states emit (sequences_section minus extras)
    pre = 0
    for s0 in range(0, len(data), SPAN):
        seqs = []
        prev = None
        carry = 0
        for sq, tail in parse_span(data[s0:s0 + SPAN]):
            for k, (ll, ml, d) in enumerate(sq):
                ll2 = ll + (carry if k == 0 else 0)
                seqs.append((ll2, ml, 1 if (ll2 > 0 and d == prev) else d + 3))
                prev = d
            carry = tail if sq else carry
        pre += 8 * len(sequences_section(seqs))
    print(f"{len(data)} B: {nseq} sequences ({nrep} repeat offsets), {nlit} literals; sequence bits: "
          f"predefined tables {pre} (extra bits {extra}), order-0 entropy of the codes {ent:.0f} + extras")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "stats":
    stats(float(sys.argv[1]))


# ---------------------------------------------------------------- compressed FSE tables (round 6)
LL_MAXLOG, ML_MAXLOG, OF_MAXLOG = 9, 9, 8


def normalize(counts, al):
    """counts -> normalized counts summing to 2^al, every used symbol >= 1 (no 'less than 1'
    symbols: a simple, valid normalization; zstd's FSE_normalizeCount is one of many)."""
    total = sum(counts)
    size = 1 << al
    norm = [0] * len(counts)
    for s, c in enumerate(counts):
        if c:
            norm[s] = max(1, (c * size + total // 2) // total)
    diff = size - sum(norm)
    order = sorted((s for s in range(len(counts)) if counts[s]), key=lambda s: -norm[s])
    i = 0
    while diff != 0:  # give to / take from the largest entries (never below 1)
        s = order[i % len(order)]
        if diff > 0:
            norm[s] += 1
            diff -= 1
        elif norm[s] > 1:
            norm[s] -= 1
            diff += 1
        i += 1
    return norm


def write_ncount(norm, al):
    """FSE table description (RFC 8878 §4.1.1), as zstd's FSE_writeNCount."""
    out = bytearray()
    bs, bc = (al - 5), 4
    remaining, threshold, nbits = (1 << al) + 1, 1 << al, al + 1
    sym, prev0 = 0, False
    n = len(norm)
    while sym < n and remaining > 1:
        if prev0:
            start = sym
            while sym < n and norm[sym] == 0:
                sym += 1
            while sym >= start + 24:
                start += 24
                bs |= 0xFFFF << bc
                bc += 16
            while sym >= start + 3:
                start += 3
                bs |= 3 << bc
                bc += 2
            bs |= (sym - start) << bc
            bc += 2
        count = norm[sym]
        sym += 1
        mx = (2 * threshold - 1) - remaining
        remaining -= abs(count)
        count += 1
        if count >= threshold:
            count += mx
        bs |= count << bc
        bc += nbits
        if count < mx:
            bc -= 1
        prev0 = count == 1
        assert remaining >= 1
        while remaining < threshold:
            nbits -= 1
            threshold >>= 1
    assert remaining == 1
    nbytes = (bc + 7) // 8
    return (bs & ((1 << (8 * nbytes)) - 1)).to_bytes(nbytes, "little")


class CTable:
    """zstd's FSE_buildCTable (state values in [size, 2 size))."""

    def __init__(self, norm, al):
        size = 1 << al
        n = len(norm)
        high = size - 1
        cumul = [0] * (n + 1)
        tsym = [0] * size
        for u in range(1, n + 1):
            if norm[u - 1] == -1:
                cumul[u] = cumul[u - 1] + 1
                tsym[high] = u - 1
                high -= 1
            else:
                cumul[u] = cumul[u - 1] + norm[u - 1]
        pos, step = 0, (size >> 1) + (size >> 3) + 3
        for s in range(n):
            for _ in range(max(norm[s], 0)):
                tsym[pos] = s
                pos = (pos + step) & (size - 1)
                while pos > high:
                    pos = (pos + step) & (size - 1)
        self.st = [0] * size
        c = list(cumul)
        for u in range(size):
            s = tsym[u]
            self.st[c[s]] = size + u
            c[s] += 1
        self.dnb, self.dfs = [0] * n, [0] * n
        total = 0
        for s in range(n):
            f = norm[s]
            if f == 0:
                self.dnb[s] = ((al + 1) << 16) - size
            elif f in (-1, 1):
                self.dnb[s] = (al << 16) - size
                self.dfs[s] = total - 1
                total += 1
            else:
                mbo = al - ((f - 1).bit_length() - 1)  # tableLog - highbit(f - 1)
                self.dnb[s] = (mbo << 16) - (f << mbo)
                self.dfs[s] = total - f
                total += f
        self.al = al

    def init(self, s):
        nbo = (self.dnb[s] + (1 << 15)) >> 16
        v = (nbo << 16) - self.dnb[s]
        return self.st[(v >> nbo) + self.dfs[s]]

    def enc(self, w, v, s):
        nbo = (v + self.dnb[s]) >> 16
        w.put(v, nbo)
        return self.st[(v >> nbo) + self.dfs[s]]


def table_log(nseq, nsyms, maxlog):
    al = max(5, min(maxlog, nseq.bit_length() - 1))
    while (1 << al) < nsyms + 1 and al < maxlog:
        al += 1
    return al


def seq_codes(seqs):
    return [(ll_code(ll)[0], ml_code(ml)[0], ov.bit_length() - 1) for ll, ml, ov in seqs]


def span_tables(all_seqs):
    """The span's three compressed tables from its symbol counts: (modes-byte bits, description,
    CTables)."""
    codes = seq_codes(all_seqs)
    tabs = []
    for k, (nsym, maxlog, norm_pre, al_pre) in enumerate(((36, LL_MAXLOG, LL_NORM, 6), (29, OF_MAXLOG, OF_NORM, 5),
                                                          (53, ML_MAXLOG, ML_NORM, 6))):
        idx = {0: 0, 1: 2, 2: 1}[k]  # LL, OF, ML from (llc, mlc, ofc)
        cnt = [0] * nsym
        for c in codes:
            cnt[c[idx]] += 1
        used = sum(1 for x in cnt if x)
        al = table_log(len(codes), used, maxlog)
        norm = normalize(cnt, al)
        # trim trailing zeros: the description stops at the last used symbol
        last = max(s for s in range(nsym) if norm[s])
        tabs.append((write_ncount(norm[:last + 1], al), CTable(norm, al)))
    return tabs


def sequences_section_t(seqs, tabs, send):
    """seqs in order through the span's tables; send: the tables are described here (Compressed
    mode) else reused (Repeat mode)."""
    n = len(seqs)
    hdr = bytearray([n] if n < 128 else [128 + (n >> 8), n & 255])
    if n == 0:
        return bytes(hdr)
    (dLL, tLL), (dOF, tOF), (dML, tML) = tabs
    mode = 2 if send else 3
    hdr.append((mode << 6) | (mode << 4) | (mode << 2))
    if send:
        hdr += dLL + dOF + dML
    w = BitW()
    codes = seq_codes(seqs)
    for k in range(n - 1, -1, -1):
        ll, ml, ov = seqs[k]
        llc, llb, llx = ll_code(ll)
        mlc, mlb, mlx = ml_code(ml)
        ofc = ov.bit_length() - 1
        if k == n - 1:
            sML, sOF, sLL = tML.init(mlc), tOF.init(ofc), tLL.init(llc)
        else:
            sOF = tOF.enc(w, sOF, ofc)
            sML = tML.enc(w, sML, mlc)
            sLL = tLL.enc(w, sLL, llc)
        w.put(llx, llb)
        w.put(mlx, mlb)
        w.put(ov - (1 << ofc), ofc)
    w.put(sML, tML.al)
    w.put(sOF, tOF.al)
    w.put(sLL, tLL.al)
    return bytes(hdr) + w.close()


def encode_chunk_t(data, G):
    """Blocks of G segments with the span's Huffman code and compressed FSE tables, both carried
    by the span's first compressed block (with sequences) and reused by the later ones."""
    out = bytearray(frame_header(len(data)))
    for s0 in range(0, len(data), SPAN):
        span = data[s0:s0 + SPAN]
        segs = parse_span(span)
        freq = [0] * 256
        seg_lits = []
        for i, (seqs, tail) in enumerate(segs):
            x = i * SEG
            lits = []
            for ll, ml, _ in seqs:
                lits += span[x:x + ll]
                x += ll + ml
            lits += span[x:x + tail]
            seg_lits.append(lits)
            for c in lits:
                freq[c] += 1
        codes = desc = None
        lens = huff_lengths(freq)
        t = huff_table(lens) if lens else None
        if t:
            codes, desc = t
        blocks = []
        for g0 in range(0, len(segs), G):
            # a block's first sequence names its offset: the block before it may become a
            # Raw_Block, which leaves the decoder's repeat offsets where the last compressed one did
            lits, seqs, carry, prev_off = [], [], 0, None
            for i in range(g0, min(g0 + G, len(segs))):
                sq, tail = segs[i]
                lits += seg_lits[i]
                for k, (ll, ml, d) in enumerate(sq):
                    ll2 = ll + (carry if k == 0 else 0)
                    seqs.append((ll2, ml, 1 if (ll2 > 0 and d == prev_off) else d + 3))
                    prev_off = d
                carry = tail if sq else carry + len(seg_lits[i])
            blocks.append((lits, seqs, span[g0 * SEG:min(len(span), (g0 + G) * SEG)]))
        all_seqs = [q for _, sq, _ in blocks for q in sq]
        tabs = span_tables(all_seqs) if all_seqs else None
        sent = False
        for lits, seqs, raw in blocks:
            ls = literals_section(lits, codes, desc) if codes else None
            coded = ls is not None
            if ls is None:
                ls = literals_section(lits, None, None)
            send = bool(seqs) and not sent
            body = ls + (sequences_section_t(seqs, tabs, send) if seqs else bytes([0]))
            if len(body) >= len(raw):
                out += ((len(raw) << 3) | 0).to_bytes(3, "little") + bytes(raw)
            else:
                out += ((len(body) << 3) | (2 << 1)).to_bytes(3, "little") + body
                if coded:
                    desc = None
                if send:
                    sent = True
    out += b"\x01\x00\x00"
    return bytes(out)


def main_t(mib):
    from compress_bench import mixed
    data = bytes(mixed(int(mib * (1 << 20)), 9))
    chunk = 4 << 20
    for G in (16, 32, 64):
        tot = 0
        for c0 in range(0, len(data), chunk):
            blob = encode_chunk_t(data[c0:c0 + chunk], G)
            assert zstd_decode(blob) == data[c0:c0 + chunk], G
            tot += len(blob)
        print(f"compressed tables, blocks of {G:2d} segments: ratio {tot / len(data):.4f}")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "tables":
    main_t(float(sys.argv[1]))


# ---------------------------------------------------------------- FSE-compressed Huffman weights (round 6)
def huff_desc_fse(lens):
    """The tree description with FSE-compressed weights (RFC 8878 §4.2.1.2), as zstd's
    HUF_compressWeights: weights of symbols 0..top-1 (the last one's is implied), one table
    (accuracy log 5), two interleaved states written backwards; None when it does not apply."""
    top = max(s for s in range(256) if lens[s])
    maxb = max(lens)
    w = [maxb + 1 - lens[s] if lens[s] else 0 for s in range(top)]
    cnt = [0] * 12
    for x in w:
        cnt[x] += 1
    if top < 3 or max(cnt) == top:
        return None
    norm = normalize(cnt, 5)
    last = max(s for s in range(12) if norm[s])
    nc = write_ncount(norm[:last + 1], 5)
    t = CTable(norm, 5)
    bw = BitW()
    i = top
    if top & 1:
        i -= 1; s1 = t.init(w[i])
        i -= 1; s2 = t.init(w[i])
        i -= 1; s1 = t.enc(bw, s1, w[i])
    else:
        i -= 1; s2 = t.init(w[i])
        i -= 1; s1 = t.init(w[i])
    two = True
    while i > 0:
        i -= 1
        if two:
            s2 = t.enc(bw, s2, w[i])
        else:
            s1 = t.enc(bw, s1, w[i])
        two = not two
    bw.put(s2, 5)
    bw.put(s1, 5)
    body = nc + bw.close()
    if len(body) >= 128:
        return None
    return bytes([len(body)]) + body


def check_fse_weights(seed=3):
    """Literal-only blocks whose code has literals above 128 (no direct weights possible), each
    frame decoded by libzstd."""
    import random
    rnd = random.Random(seed)
    for trial in range(200):
        nsym = rnd.randint(3, 256)
        syms = rnd.sample(range(256), nsym)
        lits = [rnd.choice(syms) for _ in range(rnd.randint(50, 1000))]
        lits += [max(syms)]
        freq = [0] * 256
        for c in lits:
            freq[c] += 1
        lens = huff_lengths(freq)
        if lens is None:
            continue
        desc = huff_desc_fse(lens)
        if desc is None:
            continue
        codes, _ = huff_table_any(lens)
        ls = literals_section(lits, codes, desc)
        if ls is None:
            continue
        body = ls + bytes([0])
        blob = frame_header(len(lits)) + ((len(body) << 3) | (2 << 1) | 1).to_bytes(3, "little") + body
        assert zstd_decode(blob) == bytes(lits), trial
    print("fse weights: ok")


def huff_table_any(lens):
    """huff_table's codes without its top <= 128 limit."""
    top = max(s for s in range(256) if lens[s])
    maxb = max(lens)
    w = [maxb + 1 - lens[s] if lens[s] else 0 for s in range(256)]
    num = [0] * (maxb + 2)
    for s in range(top + 1):
        if w[s]:
            num[w[s]] += 1
    start, acc = [0] * (maxb + 2), 0
    for wt in range(1, maxb + 1):
        start[wt] = acc >> (wt - 1)
        acc += num[wt] << (wt - 1)
    codes = {}
    for s in range(top + 1):
        if w[s]:
            codes[s] = (start[w[s]], lens[s])
            start[w[s]] += 1
    return codes, None


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "fseweights":
    check_fse_weights()
