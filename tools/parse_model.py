"""Host model of the device LZ77 parse (kcdc_compress.hip lz_spans_kernel) on the compression
bench's word-salad data: 512-byte segments in 32 KiB spans, fixed-Huffman bit costs, greedy
matches from a chosen candidate set (lane table, the span's first occurrence, previous segments'
tables, a short chain, lazy matching).  Prints the ratio per strategy; zlib with
fixed codes gets 0.217 on the same data.  A model, not the kernel: no literal-skip heuristic."""
import numpy as np, math
rng=np.random.default_rng(9)
words=[b"kopia",b"snapshot",b"content",b"chunk",b"the",b"of",b"blob",b"index",b" ",b"\n"]
n=256<<10
D=b"".join(words[int(k)] for k in rng.integers(0,len(words),n//4+1))[:n]
SEG=512; SPAN=32768
def lcode_bits(L):
    # fixed huffman: length codes 257..279 7 bits, 280..285 8 bits + extra
    if L<=10: e=0; code=257+L-3
    elif L==258: e=0; code=285
    else:
        e=int(math.log2((L-3)))-2 if L>10 else 0
        code=265 if L<19 else (269 if L<35 else (273 if L<67 else (277 if L<131 else 281)))
        e = 1 if L<19 else 2 if L<35 else 3 if L<67 else 4 if L<131 else 5
    return (7 if code<=279 else 8)+e
def dbits(d):
    e=0 if d<=4 else int(math.log2(d-1))-1
    return 5+e
def lit_bits(b): return 8 if b<144 else 9
def h4(x): return int.from_bytes(D[x:x+4],'little')
def mlen(q,x,xe):
    L=0
    while x+L<xe and L<258 and D[q+L]==D[x+L]: L+=1
    return L
def run(strategy, hbits=6, prevsegs=0, chain=0, minlen=4, lazy=False):
    total=0
    for s0 in range(0,n,SPAN):
        span=D[s0:s0+SPAN]
        # first occurrence per 11-bit hash in span
        first={}
        lasts=[]  # per segment: full last-occurrence dict (hash6)
        for sg in range(0,len(span),SEG):
            d={}
            for x in range(s0+sg, min(s0+sg+SEG, s0+len(span))-3):
                d[(h4(x)*0x1E35A7BD & 0xffffffff)>>(32-hbits)]=x
            lasts.append(d)
        for x in range(s0, s0+len(span)-3):
            k=(h4(x)*0x1E35A7BD & 0xffffffff)>>21
            first.setdefault(k,x)
        for si,sg in enumerate(range(0,len(span),SEG)):
            x0=s0+sg; xe=min(x0+SEG, s0+len(span))
            tab={}; hist={}
            bits=3+7+35
            x=x0; lit=x0
            def best(xx):
                hv=(h4(xx)*0x1E35A7BD)&0xffffffff; h=hv>>(32-hbits)
                cands=[]
                if h in tab: cands.append(tab[h])
                if chain: cands += hist.get(hv>>21,[])[-chain:]
                if strategy>=1:
                    f=first.get(hv>>21)
                    if f is not None and f<xx: cands.append(f)
                for j in range(1,prevsegs+1):
                    if si-j>=0 and h in lasts[si-j]: cands.append(lasts[si-j][h])
                tab[h]=xx
                hist.setdefault(hv>>21,[]).append(xx)
                bl,bq=0,0
                for q in cands:
                    if q<xx and xx-q<=32768:
                        L=mlen(q,xx,xe)
                        if L>bl: bl,bq=L,q
                return bl,bq
            while x+4<=xe:
                L,q=best(x)
                if L>=minlen and lazy and L<32 and x+5<=xe:
                    L2,q2=best(x+1)
                    if L2>L+1:
                        bits+=lit_bits(D[x]); x+=1; L,q=L2,q2
                if L>=minlen:
                    for b in D[lit:x]: bits+=lit_bits(b)
                    bits+=lcode_bits(L)+dbits(x-q); x+=L; lit=x
                else: x+=1
            for b in D[lit:xe]: bits+=lit_bits(b)
            total+=min(bits/8, (xe-x0)+5)
    return total/n
print('lane table only', round(run(0),3))
print('+first (current default)', round(run(1),3))
print('+first, 8-bit lane table', round(run(1,hbits=8),3))
print('+first +prev1', round(run(1,prevsegs=1),3))
print('+first +prev3', round(run(1,prevsegs=3),3))
print('+first +prev3 lazy', round(run(1,prevsegs=3,lazy=True),3))
print('+first +chain4 (own seg)', round(run(1,chain=4),3))
print('+first +prev3 +chain4 lazy', round(run(1,prevsegs=3,chain=4,lazy=True),3))
print('minlen3 +first +prev3 +chain4', round(run(1,prevsegs=3,chain=4,minlen=3),3))
