// Kopia content compression on gfx950: the deflate family.
//
// What the reference does per content (repo/content/content_manager_lock_free.go:42-73,
// repo/compression/compressor.go:67-72, compressor_deflate.go:14-62):
//   out = BE32(header ID) || raw DEFLATE stream (RFC 1951) of the content
// and the content is stored uncompressed (header ID 0, NoCompression) when len(out) >= len(in).
// The stream is written by github.com/klauspost/compress/flate (not vendored); readers accept
// any valid RFC 1951 stream, so what must match is the format, not the encoder's choices.
//
// Device layout: a chunk is cut into 32 KiB spans (one 64-lane wave each) and a span into
// 512-byte segments (one lane each).  The wave stages its span in LDS (segment l at a
// 516-byte stride, so lanes at equal offsets hit distinct banks), and every lane runs a
// greedy LZ77 over its own segment with a 128-entry hash table of its own (lane-minor u16
// columns: conflict free).  A lane emits one fixed-Huffman block (BTYPE 01) for its segment
// and ends it with an empty stored block (zlib's sync flush: 3 bits, pad, 00 00 FF FF), so
// every segment's output is a whole number of bytes and segments concatenate by a byte
// prefix sum.  A segment whose block is not smaller than a stored copy becomes a stored
// block (5 + n bytes, copied from the input by the finish kernel).  The stream ends with an
// empty final fixed block (03 00).
//
// Kernels, in stream order: span_count (spans per chunk), span_scan (prefix), deflate_spans
// (LZ77 + bits), deflate_finish (per chunk: scan of segment lengths, header, concatenation).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "kcdc_internal.h"

namespace kcdc {
namespace compdev {

constexpr uint32_t kSeg = 512;                  // bytes per lane segment
constexpr uint32_t kSpan = 64 * kSeg;           // bytes per wave span (<= the 32 KiB window)
constexpr uint32_t kSlot = kSeg + 64;           // scratch bytes per segment (the encoder stops at kSeg + 8)
constexpr uint32_t kStored = 0x80000000u;       // segment length flag: emit a stored block
constexpr uint32_t kHashBits = 7;
constexpr uint32_t kLdsWords = 8320;            // >= (4 * 2049 + 1) + 65: the staged span + 1 word of read-ahead

struct CompArgs {
    const uint8_t* in;
    const uint64_t* in_offs;
    const uint64_t* in_lens;
    uint8_t* out;
    const uint64_t* out_offs;
    uint64_t* out_lens;
    uint32_t* ids;
    uint32_t* spans;    // [n + 1]: spans per chunk, then their exclusive prefix
    uint32_t* seglen;   // [max_spans * 64]
    uint8_t* slots;     // [max_spans * 64 * kSlot]
    uint32_t n;
    uint32_t max_spans;
    uint32_t header_id;
    uint32_t skip;      // literal-run skip shift of the match search (level)
};

__global__ __launch_bounds__(256) void span_count_kernel(CompArgs a) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c < a.n) a.spans[c] = static_cast<uint32_t>((a.in_lens[c] + kSpan - 1) / kSpan);
}

// Exclusive prefix of spans[0..n) in place; spans[n] = total.  One workgroup.
__global__ __launch_bounds__(1024) void span_scan_kernel(uint32_t n, uint32_t* spans) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t b = static_cast<uint64_t>(n) * t / 1024u, e = static_cast<uint64_t>(n) * (t + 1) / 1024u;
    uint32_t s = 0;
    for (uint64_t i = b; i < e; i++) s += spans[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint64_t i = b; i < e; i++) {
        const uint32_t u = spans[i];
        spans[i] = run;
        run += u;
    }
    if (t == 1023u) spans[n] = part[1023];
}

// LDS dword index of staged word k: one pad dword per 128 words (a 512-byte segment).
__device__ __forceinline__ uint32_t pw(uint32_t k) { return k + (k >> 7); }

struct Bits {
    uint64_t bb;
    uint32_t nb;
    uint32_t* op;
    __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
        bb |= static_cast<uint64_t>(v) << nb;
        nb += n;
        if (nb >= 32u) {
            *op++ = static_cast<uint32_t>(bb);  // vector store
            bb >>= 32;
            nb -= 32u;
        }
    }
};
// Huffman codes go MSB-first into the LSB-first bit stream (RFC 1951 §3.1.1).
__device__ __forceinline__ uint32_t rev(uint32_t code, uint32_t n) { return __builtin_bitreverse32(code) >> (32u - n); }

// Fixed literal/length code (RFC 1951 §3.2.6).
__device__ __forceinline__ void put_lit(Bits& w, uint32_t b) {
    if (b < 144u)
        w.put(rev(0x30u + b, 8), 8);
    else
        w.put(rev(0x190u + (b - 144u), 9), 9);
}
__device__ __forceinline__ void put_match(Bits& w, uint32_t len, uint32_t dist) {
    uint32_t sym, eb = 0, ev = 0;
    const uint32_t l = len - 3u;
    if (len == 258u) {
        sym = 285u;
    } else if (l < 8u) {
        sym = 257u + l;
    } else {
        const uint32_t nb = 31u - __builtin_clz(l);
        eb = nb - 2u;
        sym = 257u + 4u * (nb - 1u) + ((l >> eb) & 3u);
        ev = l & ((1u << eb) - 1u);
    }
    if (sym < 280u)
        w.put(rev(sym - 256u, 7), 7);
    else
        w.put(rev(0xC0u + (sym - 280u), 8), 8);
    if (eb) w.put(ev, eb);
    const uint32_t d = dist - 1u;
    uint32_t dc = d, deb = 0, dev = 0;
    if (d >= 4u) {
        const uint32_t nb = 31u - __builtin_clz(d);
        deb = nb - 1u;
        dc = 2u * nb + ((d >> deb) & 1u);
        dev = d & ((1u << deb) - 1u);
    }
    w.put(rev(dc, 5), 5);
    if (deb) w.put(dev, deb);
}

// One wave per span: blockIdx.x = global span index.
__global__ __launch_bounds__(64) void deflate_spans_kernel(CompArgs a) {
    __shared__ uint32_t L[kLdsWords];
    __shared__ uint16_t tab[(1u << kHashBits) * 64u];
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    // The chunk: the last c with spans[c] <= b (empty chunks share their prefix with the next).
    uint32_t lo = 0, hi = a.n;  // spans[lo] <= b < spans[hi]
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.spans[mid] <= b) lo = mid; else hi = mid;
    }
    const uint32_t c = lo;
    const uint32_t u = b - a.spans[c];
    const uint64_t len = a.in_lens[c];
    const uint64_t sb = static_cast<uint64_t>(u) * kSpan;
    const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
    // Stage [A0, A0 + 16 ng) with A0 = A & ~15: every 16-byte granule holds a byte of the span.
    const uint8_t* A = a.in + a.in_offs[c] + sb;
    const uint32_t d = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(A) & 15u);
    const uint4* G = reinterpret_cast<const uint4*>(A - d);
    const uint32_t ng = (d + span_len + 15u) >> 4;
    for (uint32_t g = lane; g < ng; g += 64u) {
        const uint4 v = G[g];
        const uint32_t k = 4u * g;
        L[pw(k)] = v.x;
        L[pw(k + 1)] = v.y;
        L[pw(k + 2)] = v.z;
        L[pw(k + 3)] = v.w;
    }
    {
        uint64_t* t64 = reinterpret_cast<uint64_t*>(tab);
        for (uint32_t i = lane; i < (1u << kHashBits) * 16u; i += 64u) t64[i] = ~0ull;
    }
    __syncthreads();
    const uint8_t* Lb = reinterpret_cast<const uint8_t*>(L);
    auto ld32 = [&](uint32_t x) -> uint32_t {
        const uint32_t q = x + d, k = q >> 2;
        return __builtin_amdgcn_alignbit(L[pw(k + 1)], L[pw(k)], 8u * (q & 3u));
    };
    auto byte = [&](uint32_t x) -> uint32_t {
        const uint32_t q = x + d;
        return Lb[4u * pw(q >> 2) + (q & 3u)];
    };

    const uint32_t slot = b * 64u + lane;
    const uint32_t x0 = kSeg * lane;
    if (x0 >= span_len) {
        a.seglen[slot] = 0u;
        return;
    }
    const uint32_t xe = span_len - x0 < kSeg ? span_len : x0 + kSeg;
    const uint32_t seg_len = xe - x0;
    uint32_t* base = reinterpret_cast<uint32_t*>(a.slots + static_cast<uint64_t>(slot) * kSlot);
    const uint32_t limit = seg_len + 8u;  // bytes flushed before giving up on the fixed block
    Bits w{0ull, 0u, base};
    bool over = false;
    w.put(2u, 3);  // BFINAL 0, BTYPE 01
    uint32_t x = x0, lit = x0;
    auto literals = [&](uint32_t e) {
        for (uint32_t q = lit; q < e; q++) {
            put_lit(w, byte(q));
            if (4u * static_cast<uint32_t>(w.op - base) > limit) {
                over = true;
                break;
            }
        }
    };
    while (!over && x + 4u <= xe) {
        const uint32_t v = ld32(x);
        const uint32_t h = (v * 0x1E35A7BDu) >> (32u - kHashBits);
        const uint32_t cand = tab[h * 64u + lane];
        tab[h * 64u + lane] = static_cast<uint16_t>(x);
        if (cand >= x0 && cand < x && ld32(cand) == v) {
            const uint32_t maxlen = xe - x < 258u ? xe - x : 258u;
            uint32_t n = 4;
            bool done = false;
            while (n + 4u <= maxlen) {
                const uint32_t diff = ld32(x + n) ^ ld32(cand + n);
                if (diff) {
                    n += static_cast<uint32_t>(__builtin_ctz(diff)) >> 3;
                    done = true;
                    break;
                }
                n += 4u;
            }
            if (!done)
                while (n < maxlen && byte(x + n) == byte(cand + n)) n++;
            literals(x);
            if (over) break;
            put_match(w, n, x - cand);
            if (4u * static_cast<uint32_t>(w.op - base) > limit) {
                over = true;
                break;
            }
            x += n;
            lit = x;
        } else {
            x += 1u + ((x - lit) >> a.skip);
        }
    }
    if (!over) literals(xe);
    uint32_t bytes = 0;
    if (!over) {
        w.put(0u, 7);  // end of block (256: seven zero bits)
        w.put(0u, 3);  // empty stored block: BFINAL 0, BTYPE 00 ...
        w.nb = (w.nb + 7u) & ~7u;  // ... padded to a byte
        w.put(0x0000u, 16);
        w.put(0xFFFFu, 16);
        bytes = 4u * static_cast<uint32_t>(w.op - base) + (w.nb >> 3);
        if (w.nb) *w.op = static_cast<uint32_t>(w.bb);
        if (bytes >= seg_len + 5u) over = true;
    }
    a.seglen[slot] = over ? (kStored | seg_len) : bytes;
}

// One workgroup per chunk: concatenates its segments behind the header ID and ends the
// stream with an empty final fixed block.
__global__ __launch_bounds__(256) void deflate_finish_kernel(CompArgs a) {
    __shared__ uint32_t pos[256];
    __shared__ uint32_t wsum[4];
    const uint32_t c = blockIdx.x, t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans) {  // workspace smaller than the chunks need: no output
        if (t == 0) {
            a.out_lens[c] = 0ull;
            a.ids[c] = 0u;
        }
        return;
    }
    const uint64_t s0 = static_cast<uint64_t>(a.spans[c]) * 64u;
    const uint32_t ns = (a.spans[c + 1] - a.spans[c]) * 64u;
    uint8_t* dst = a.out + a.out_offs[c];
    const uint8_t* src_in = a.in + a.in_offs[c];
    uint64_t carry = 4;
    for (uint32_t base = 0; base < ns; base += 256u) {
        const uint32_t i = base + t;
        const uint32_t Lr = i < ns ? a.seglen[s0 + i] : 0u;
        const uint32_t eff = (Lr & kStored) ? 5u + (Lr & ~kStored) : Lr;
        // Block exclusive scan of eff.
        uint32_t incl = eff;
        for (uint32_t o = 1; o < 64u; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63u) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (uint32_t k = 0; k < 4u; k++) {
            if (k < wv) before += wsum[k];
            tot += wsum[k];
        }
        pos[t] = before + incl - eff;
        __syncthreads();
        for (uint32_t j = wv; j < 256u && base + j < ns; j += 4u) {
            const uint32_t Lj = a.seglen[s0 + base + j];
            uint8_t* o = dst + carry + pos[j];
            if (Lj & kStored) {
                const uint32_t m = Lj & ~kStored;
                if (lane < 5u) {
                    const uint32_t hdr = lane == 0 ? 0u : lane == 1 ? (m & 255u) : lane == 2 ? (m >> 8)
                                       : lane == 3 ? (~m & 255u) : ((~m >> 8) & 255u);
                    o[lane] = static_cast<uint8_t>(hdr);
                }
                const uint8_t* s = src_in + static_cast<uint64_t>(base + j) * kSeg;
                for (uint32_t q = lane; q < m; q += 64u) o[5u + q] = s[q];
            } else {
                const uint8_t* s = a.slots + (s0 + base + j) * kSlot;
                for (uint32_t q = lane; q < Lj; q += 64u) o[q] = s[q];
            }
        }
        carry += tot;
        __syncthreads();
    }
    if (t < 4u) dst[t] = static_cast<uint8_t>(a.header_id >> (8u * (3u - t)));
    if (t == 4u) dst[carry] = 0x03u;  // BFINAL 1, BTYPE 01, end of block
    if (t == 5u) dst[carry + 1] = 0x00u;
    if (t == 0) {
        const uint64_t out_len = carry + 2u;
        a.out_lens[c] = out_len;
        a.ids[c] = out_len < a.in_lens[c] ? a.header_id : 0u;  // content_manager_lock_free.go:64
    }
}

}  // namespace compdev

namespace {

struct CompAlgo {
    const char* name;
    uint32_t header_id;  // repo/compression/compression_ids.go:28-30
    uint32_t skip;
};
// repo/compression/compressor_deflate.go:14-16
constexpr CompAlgo kCompAlgos[] = {
    {"deflate-best-compression", 0x1502u, 7u},
    {"deflate-best-speed", 0x1501u, 4u},
    {"deflate-default", 0x1500u, 5u},
};

const CompAlgo* find_comp(const char* name) {
    if (!name) return nullptr;
    for (const CompAlgo& a : kCompAlgos)
        if (std::strcmp(a.name, name) == 0) return &a;
    return nullptr;
}

uint64_t align256c(uint64_t x) { return (x + 255u) & ~uint64_t(255); }

struct CompWs {
    uint64_t spans, seglen, slots, total;
};
CompWs comp_ws(uint32_t n, uint64_t max_spans) {
    CompWs l{};
    l.spans = 0;
    l.seglen = align256c((uint64_t(n) + 1u) * 4u);
    l.slots = align256c(l.seglen + max_spans * 64u * 4u);
    l.total = align256c(l.slots + max_spans * 64u * compdev::kSlot);
    return l;
}

}  // namespace
}  // namespace kcdc

using namespace kcdc;

extern "C" int kcdc_compression_algorithms(const char** names, int cap) {
    const int n = static_cast<int>(sizeof(kCompAlgos) / sizeof(kCompAlgos[0]));
    for (int i = 0; i < n && i < cap; i++) names[i] = kCompAlgos[i].name;
    return n;
}

extern "C" int64_t kcdc_compression_header_id(const char* name) {
    const CompAlgo* a = find_comp(name);
    return a ? static_cast<int64_t>(a->header_id)
             : set_error(-2, std::string("unknown compression algorithm: ") + (name ? name : "(null)"));
}

extern "C" uint64_t kcdc_compress_bound(uint64_t len) {
    return 6u + len + 5u * ((len + compdev::kSeg - 1) / compdev::kSeg);
}

extern "C" uint64_t kcdc_compress_workspace_size(uint64_t total_bytes, uint32_t nchunks) {
    return comp_ws(nchunks, total_bytes / compdev::kSpan + nchunks).total;
}

extern "C" int kcdc_compress_chunks_device(const char* name, const uint8_t* d_data, const uint64_t* d_offsets,
                                           const uint64_t* d_lens, uint32_t nchunks, uint8_t* d_out,
                                           const uint64_t* d_out_offsets, uint64_t* d_out_lens,
                                           uint32_t* d_header_ids, void* d_work, uint64_t work_bytes, void* stream) {
    const CompAlgo* al = find_comp(name);
    if (!al) return set_error(-2, std::string("unknown compression algorithm: ") + (name ? name : "(null)"));
    if (nchunks == 0) return 0;
    if (!d_data || !d_offsets || !d_lens || !d_out || !d_out_offsets || !d_out_lens || !d_header_ids || !d_work)
        return set_error(-22, "null argument");
    // The largest span count this workspace holds (the kernels check the real count against it).
    const uint64_t fixed = comp_ws(nchunks, 0).total;
    if (work_bytes < fixed) return set_error(-22, "workspace too small (kcdc_compress_workspace_size)");
    uint64_t max_spans = (work_bytes - fixed) / (64u * (compdev::kSlot + 4u));
    while (max_spans > 0 && comp_ws(nchunks, max_spans).total > work_bytes) max_spans--;
    if (max_spans > 0x7fffffffull) max_spans = 0x7fffffffull;
    compdev::CompArgs a{};
    a.in = d_data;
    a.in_offs = d_offsets;
    a.in_lens = d_lens;
    a.out = d_out;
    a.out_offs = d_out_offsets;
    a.out_lens = d_out_lens;
    a.ids = d_header_ids;
    const CompWs l = comp_ws(nchunks, max_spans);
    uint8_t* w = static_cast<uint8_t*>(d_work);
    a.spans = reinterpret_cast<uint32_t*>(w + l.spans);
    a.seglen = reinterpret_cast<uint32_t*>(w + l.seglen);
    a.slots = w + l.slots;
    a.n = nchunks;
    a.max_spans = static_cast<uint32_t>(max_spans);
    a.header_id = al->header_id;
    a.skip = al->skip;
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compdev::span_count_kernel, dim3((nchunks + 255u) / 256u), dim3(256), 0, st, a);
    hipLaunchKernelGGL(compdev::span_scan_kernel, dim3(1), dim3(1024), 0, st, nchunks, a.spans);
    if (max_spans > 0)
        hipLaunchKernelGGL(compdev::deflate_spans_kernel, dim3(static_cast<uint32_t>(max_spans)), dim3(64), 0, st, a);
    hipLaunchKernelGGL(compdev::deflate_finish_kernel, dim3(nchunks), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("compression kernel launch: ") + hipGetErrorString(e));
}
