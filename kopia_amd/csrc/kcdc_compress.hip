// Kopia content compression on gfx950: the deflate family (deflate, gzip,
// pgzip), S2 (s2-default/-better/-parallel-4/-8: Snappy elements in S2's framing format,
// compressor_s2.go:20-23) and Zstandard (zstd, -fastest, -better-, -best-compression: RFC 8878
// frames, compressor_zstd.go:15-18).  All three share the span/segment layout and the LZ77 parse
// below; they differ in how a segment's literals and matches are written (lz_spans_kernel<FMT>).
//
// What the reference does per content (repo/content/content_manager_lock_free.go:42-73,
// repo/compression/compressor.go:67-72, compressor_deflate.go:14-62):
//   out = BE32(header ID) || raw DEFLATE stream (RFC 1951) of the content
// and the content is stored uncompressed (header ID 0, NoCompression) when len(out) >= len(in).
// The stream is written by github.com/klauspost/compress/flate (not vendored); readers accept
// any valid RFC 1951 stream, so what must match is the format, not the encoder's choices.
//
// Device layout: a chunk is cut into 32 KiB spans (one 64-lane wave each) and a span into
// 512-byte segments (one lane each).  The wave stages its span in LDS (segment l at a 516-byte
// stride, so lanes at equal offsets hit distinct banks) and every lane runs a greedy LZ77 parse
// over its own segment (lz_spans_kernel<FMT>).  Candidates per position: the lane's 64-entry hash
// table (lane-minor u16 columns); with effort >= 1 also the previous match's distance (a repeat
// candidate), the 32 nearest distances at the segment's first position, the three previous lanes'
// latest entries and the span's first occurrence of the hash (a table built by LDS atomic min);
// among equally long matches the nearest wins; the default level adds one-step lazy matching.
// How a segment's matches are written depends on the format:
//   deflate  the parse leaves tokens; deflate_plan builds one plan per span (literal/length and
//            distance histograms, code lengths <= 15 bits, the dynamic header, every segment's
//            exact size under the dynamic and the fixed code) and picks stored / fixed / dynamic
//            blocks; deflate_emit_kernel writes each segment's bits at its planned bit offset, a
//            span ends byte-aligned (deflate_stored_kernel copies stored spans);
//   S2       Snappy elements (literal runs, copy-1/copy-2) in S2's framing format, one framed
//            chunk per span with the masked CRC-32C of its bytes (crc_spans_kernel<true>);
//   zstd     one Compressed_Block per segment: literals Huffman-coded with one code per span
//            (the first saving segment carries the tree, later ones are Treeless) or raw, the
//            sequences through the predefined FSE tables, written backwards (zstd_seqs).
// A segment that would not beat a stored copy is stored.  Segments join by a byte prefix sum
// (span_pos), deflate_copy_kernel places them, deflate_frame_kernel writes the header ID, the
// format's frame (gzip member with CRC-32 and ISIZE, zstd frame header, final empty block) and
// the kept-or-dropped ID (NoCompression when the output is not smaller).
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
constexpr int kFmtDeflate = 0;                  // RFC 1951 (deflate, gzip, pgzip)
constexpr int kFmtS2 = 1;                       // S2 / Snappy block elements in the S2 framing format
constexpr uint32_t kS2StoredHdr = 3;            // a stored S2 segment: one literal, tag 61 + 2-byte length
constexpr uint32_t kS2ChunkHdr = 8;             // framing chunk: type 0x00, 3-byte length, masked CRC-32C
constexpr uint32_t kS2StreamId = 10;            // ff 06 00 00 "S2sTwO" (s2.NewWriter's stream identifier)
constexpr int kFmtZstd = 2;                     // Zstandard frame (RFC 8878): one compressed block per segment
constexpr uint32_t kZOff = 3;                   // a zstd segment's bytes start at slot + 3 (see lz_spans_kernel)
constexpr uint32_t kZStoredHdr = 3;             // a stored zstd segment: Raw_Block header
#ifndef KCDC_DEFLATE_HASH_BITS
#define KCDC_DEFLATE_HASH_BITS 6  // per-lane match table entries (log2); LDS = 33 KiB span + 128 B << bits
#endif
constexpr uint32_t kHashBits = KCDC_DEFLATE_HASH_BITS;
// Span-wide table: for every 11-bit hash, the FIRST position of the span with that hash (an LDS
// atomic min over all lanes before the parse).  A lane's own table only sees its 512-byte segment;
// this one offers a match anywhere earlier in the span (<= 32 KiB back, inside the window).
// Simulated on the mixed data (tools/compress_bench.py): ratio 0.362 -> 0.339 against zlib-6 0.270.
// LDS: 33 KiB span + 8 KiB lane tables + 8 KiB span table = 49.7 KiB: three waves per CU, as before.
constexpr uint32_t kFirstBits = 11;
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
    uint32_t* span_bytes;  // [max_spans]: output bytes of each span's segments
    uint64_t* span_pos;    // [max_spans + 1]: their exclusive prefix over all chunks
    uint8_t* slots;     // [max_spans * 64 * kSlot]
    uint32_t* desc;     // [max_spans * kDescWords]: deflate, each span's plan
    uint32_t n;
    uint32_t max_spans;
    uint32_t header_id;
    uint32_t skip;      // literal-run skip shift of the match search (level)
    uint32_t effort;    // 0: the lane's own table only; 1: + the span-wide first-occurrence table,
                        // previous segments' tables, lazy matching of short matches; 2: lazy < 32 B
    uint32_t gzip;      // 1: the stream sits in a gzip member (RFC 1952): gzip, pgzip
    uint32_t fmt;       // kFmtDeflate or kFmtS2
    uint32_t* crc;      // [n]: per chunk, XOR of its spans' shifted raw CRC-32s (atomic)
    uint32_t* span_crc; // [max_spans]: S2, each span's raw CRC-32C
    uint32_t x2n[32];   // x^(2^k) mod P, CRC-32's reflected polynomial (zlib x2n_table)
    uint32_t x2nc[32];  // the same for CRC-32C (Castagnoli, S2 framing)
};

__global__ __launch_bounds__(256) void span_count_kernel(CompArgs a) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c < a.n) {
        a.spans[c] = static_cast<uint32_t>((a.in_lens[c] + kSpan - 1) / kSpan);
        a.crc[c] = 0u;
    }
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
// Byte x / the 4 bytes at x of a span staged at byte offset d (the source's misalignment).
__device__ __forceinline__ uint32_t st_byte(const uint32_t* L, uint32_t d, uint32_t x) {
    const uint32_t q = x + d;
    return reinterpret_cast<const uint8_t*>(L)[4u * pw(q >> 2) + (q & 3u)];
}
__device__ __forceinline__ uint32_t st_ld32(const uint32_t* L, uint32_t d, uint32_t x) {
    const uint32_t q = x + d, k = q >> 2;
    return __builtin_amdgcn_alignbit(L[pw(k + 1)], L[pw(k)], 8u * (q & 3u));
}
// Stage the span_len bytes at A into L: the 16-byte granules [A & ~15, ...) holding them, at
// staged word pw(k); returns d = A & 15.
__device__ __forceinline__ uint32_t stage_span(uint32_t* L, const uint8_t* A, uint32_t span_len, uint32_t lane,
                                                uint32_t nt = 64u) {
    const uint32_t d = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(A) & 15u);
    const uint4* G = reinterpret_cast<const uint4*>(A - d);
    const uint32_t ng = (d + span_len + 15u) >> 4;
    for (uint32_t g = lane; g < ng; g += nt) {
        const uint4 v = G[g];
        const uint32_t k = 4u * g;
        L[pw(k)] = v.x;
        L[pw(k + 1)] = v.y;
        L[pw(k + 2)] = v.z;
        L[pw(k + 3)] = v.w;
    }
    return d;
}

// ---------------------------------------------------------------- Zstandard sequences (RFC 8878)
// The sequences of a block go through FSE with the predefined distributions (Symbol_Compression_Modes
// = Predefined_Mode for literal lengths, offsets and match lengths, RFC 8878 §3.1.1.3.2.2).  The
// decoding tables are built exactly as the RFC's FSE table construction (spread with step
// (size >> 1) + (size >> 3) + 3, "less than 1" symbols at the top); the encoder uses, per symbol, the
// cell whose [baseline, baseline + 2^bits) holds the next state (a symbol's cells cover every state
// once).  All compile-time: no table upload.
template <int NS, int AL>
struct FseTab {
    static constexpr int kSize = 1 << AL;
    uint8_t sym[kSize], nb[kSize], base[kSize];
    uint8_t enc[NS][kSize];  // enc[s][next state] = the cell of symbol s that reaches it
    uint8_t first[NS];       // some cell of s (the last sequence's state is free)
    constexpr FseTab(const int8_t (&norm)[NS]) : sym{}, nb{}, base{}, enc{}, first{} {
        int next[NS] = {};
        int high = kSize - 1;
        for (int s = 0; s < NS; s++) {
            if (norm[s] == -1) {
                sym[high--] = static_cast<uint8_t>(s);
                next[s] = 1;
            } else {
                next[s] = norm[s];
            }
        }
        int pos = 0;
        const int step = (kSize >> 1) + (kSize >> 3) + 3;
        for (int s = 0; s < NS; s++)
            for (int i = 0; i < norm[s]; i++) {
                sym[pos] = static_cast<uint8_t>(s);
                do pos = (pos + step) & (kSize - 1);
                while (pos > high);
            }
        for (int u = 0; u < kSize; u++) {
            const int s = sym[u];
            const int ns = next[s]++;
            int hb = 0;
            while ((2 << hb) <= ns) hb++;
            nb[u] = static_cast<uint8_t>(AL - hb);
            base[u] = static_cast<uint8_t>((ns << (AL - hb)) - kSize);
            first[s] = static_cast<uint8_t>(u);
            for (int t = base[u]; t < base[u] + (1 << nb[u]); t++) enc[s][t] = static_cast<uint8_t>(u);
        }
    }
};
constexpr int8_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int8_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int8_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                -1, -1, -1, -1, -1};
__device__ const FseTab<36, 6> kFseLL(kLLNorm);
__device__ const FseTab<53, 6> kFseML(kMLNorm);
__device__ const FseTab<29, 5> kFseOF(kOFNorm);

// Literal length -> (code, extra bits, extra value); RFC 8878 Literals_Length_Code table: codes
// 16..24 cover 16..63 in groups of 1, 2, 3, 4 extra bits (bases 16, 24, 32, 48), from 64 the
// code is 19 + log2.  Branch-free within each range (the FSE writer's serial loop runs it).
__device__ __forceinline__ void ll_code(uint32_t ll, uint32_t& code, uint32_t& nbx, uint32_t& x) {
    const uint32_t g = ll >> 3;
    const uint32_t nb = g == 2u ? 1u : g == 3u ? 2u : g < 6u ? 3u : 4u;
    const uint32_t base = nb == 1u ? 16u : nb == 2u ? 24u : nb == 3u ? 32u : 48u;
    const uint32_t c0 = nb == 1u ? 16u : nb == 2u ? 20u : nb == 3u ? 22u : 24u;
    const uint32_t h = 31u - static_cast<uint32_t>(__builtin_clz(ll | 1u));
    if (ll < 16u) {
        code = ll;
        nbx = 0;
        x = 0;
    } else if (ll < 64u) {
        code = c0 + ((ll - base) >> nb);
        nbx = nb;
        x = (ll - base) & ((1u << nb) - 1u);
    } else {
        code = h + 19u;
        nbx = h;
        x = ll - (1u << h);
    }
}
// Match length (>= 3) -> (code, extra bits, extra value); Match_Length_Code table: m = ml - 3,
// codes 32..42 cover m 32..127 in groups of 1..5 extra bits (bases 32, 40, 48, 64, 96), from 128
// the code is 36 + log2.
__device__ __forceinline__ void ml_code(uint32_t ml, uint32_t& code, uint32_t& nbx, uint32_t& x) {
    const uint32_t m = ml - 3u, g = m >> 3;
    const uint32_t nb = g == 4u ? 1u : g == 5u ? 2u : g < 8u ? 3u : g < 12u ? 4u : 5u;
    const uint32_t base = nb == 1u ? 32u : nb == 2u ? 40u : nb == 3u ? 48u : nb == 4u ? 64u : 96u;
    const uint32_t c0 = nb == 1u ? 32u : nb == 2u ? 36u : nb == 3u ? 38u : nb == 4u ? 40u : 42u;
    const uint32_t h = 31u - static_cast<uint32_t>(__builtin_clz(m | 1u));
    if (m < 32u) {
        code = m;
        nbx = 0;
        x = 0;
    } else if (m < 128u) {
        code = c0 + ((m - base) >> nb);
        nbx = nb;
        x = (m - base) & ((1u << nb) - 1u);
    } else {
        code = h + 36u;
        nbx = h;
        x = m - (1u << h);
    }
}

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

// A deflate match's symbols (RFC 1951 §3.2.5): length symbol 257..285 with its extra bits,
// distance symbol 0..29 with its extra bits.
struct MatchSyms {
    uint32_t ls, eb, ev, ds, deb, dev;
};
__device__ __forceinline__ MatchSyms match_syms(uint32_t len, uint32_t dist) {
    MatchSyms m{0u, 0u, 0u, 0u, 0u, 0u};
    const uint32_t l = len - 3u;
    if (len == 258u) {
        m.ls = 285u;
    } else if (l < 8u) {
        m.ls = 257u + l;
    } else {
        const uint32_t nb = 31u - __builtin_clz(l);
        m.eb = nb - 2u;
        m.ls = 257u + 4u * (nb - 1u) + ((l >> m.eb) & 3u);
        m.ev = l & ((1u << m.eb) - 1u);
    }
    const uint32_t d = dist - 1u;
    m.ds = d;
    if (d >= 4u) {
        const uint32_t nb = 31u - __builtin_clz(d);
        m.deb = nb - 1u;
        m.ds = 2u * nb + ((d >> m.deb) & 1u);
        m.dev = d & ((1u << m.deb) - 1u);
    }
    return m;
}

// ---------------------------------------------------------------- deflate blocks of a span
// The parse (lz_spans_kernel<kFmtDeflate>) leaves each segment's matches as tokens in its slot
// ((literal run << 23) | (length - 3) << 15 | (distance - 1): a segment holds <= 128) and marks
// the segment stored when a fixed code would not beat a stored copy (random data).  The span's
// coded segments then share ONE code: per maximal run of coded segments one Huffman block,
// BTYPE 10 with a dynamic code built from the span's symbol counts (default and
// best-compression) or BTYPE 01 with the fixed code (best-speed, or when smaller for the span);
// per run of stored segments one stored block; a span whose coded form is not smaller than a
// stored copy is one stored block.  A span ends byte aligned (a coded run last: an empty stored
// block, zlib's sync flush), so spans concatenate by a byte prefix as before.  The plan (block
// type, code lengths, header bits, every segment's bit offset) goes to the span's descriptor;
// deflate_emit_kernel writes the bits straight to the chunk's place.
// The reference's encoder (klauspost/compress/flate, compressor_deflate.go:14-16) chooses
// between the same three block types per block; readers accept any valid RFC 1951 stream.
constexpr uint32_t kNLit = 286, kNDist = 30, kNSym = kNLit + kNDist;
constexpr uint32_t kHdrWords = 72;  // a dynamic header: <= 5 + 5 + 4 + 19 * 3 + 316 * 7 bits
// Descriptor words per span: [0, 64) each segment's bit offset in the span's output; [64, 128)
// its info (class 1 coded / 2 stored, bit 2 first of its run, bit 3 last of its run, bit 4 the
// span's last segment, bits 16.. a stored run's length at its first segment); [128, 208) the code
// lengths (bytes: 286 literal/length, 30 distance); [208, 280) the dynamic header's bits; [280]
// the mode (0 one stored block, 1 fixed, 2 dynamic) | header bits << 8.
constexpr uint32_t kDescOff = 0, kDescInfo = 64, kDescLens = 128, kDescHdr = 208, kDescMode = 280;
constexpr uint32_t kDescWords = 288;
static_assert(kDescHdr + kHdrWords <= kDescMode && kDescMode < kDescWords, "descriptor layout");
constexpr uint32_t kModeStored = 0, kModeFixed = 1, kModeDynamic = 2;
constexpr uint32_t kClsCoded = 1, kClsStored = 2;

// Fixed code lengths (RFC 1951 §3.2.6); s >= 286: distance symbols.
__device__ __forceinline__ uint32_t fixed_len(uint32_t s) {
    return s < 144u ? 8u : s < 256u ? 9u : s < 280u ? 7u : s < kNLit ? 8u : 5u;
}

// Orders one wave's LDS accesses across its lanes (a wave's LDS instructions complete in order):
// the barrier for wave-collective helpers that also run inside multi-wave workgroups.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Canonical codes (RFC 1951 §3.2.2) of the n code lengths len[] (LDS bytes), bit-reversed for the
// LSB-first stream: out[s] = rev(code) | length << 16 (0 for unused symbols).  Wave-collective:
// symbols in 64-wide groups, a symbol's rank among the equal lengths before it by ballot.
__device__ void canon_codes(const uint8_t* len, uint32_t n, uint32_t* out, uint32_t lane) {
    uint32_t cnt[16];
#pragma unroll
    for (int j = 0; j < 16; j++) cnt[j] = 0u;
    for (uint32_t k = 0; k < n; k += 64u) {
        const uint32_t l = k + lane < n ? len[k + lane] : 0u;
#pragma unroll
        for (int j = 1; j < 16; j++) cnt[j] += static_cast<uint32_t>(__popcll(__ballot(l == static_cast<uint32_t>(j))));
    }
    uint32_t next[16];
    next[0] = 0u;
    uint32_t code = 0u;
#pragma unroll
    for (int j = 1; j < 16; j++) {
        code = (code + (j > 1 ? cnt[j - 1] : 0u)) << 1;
        next[j] = code;
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    for (uint32_t k = 0; k < n; k += 64u) {
        const uint32_t l = k + lane < n ? len[k + lane] : 0u;
        uint32_t c = 0u;
#pragma unroll
        for (int j = 1; j < 16; j++) {
            const uint64_t m = __ballot(l == static_cast<uint32_t>(j));
            if (l == static_cast<uint32_t>(j)) c = next[j] + static_cast<uint32_t>(__popcll(m & lt));
            next[j] += static_cast<uint32_t>(__popcll(m));
        }
        if (k + lane < n) out[k + lane] = l ? (rev(c, l) | (l << 16)) : 0u;
    }
}

// Code lengths (<= maxb bits) of a minimum-redundancy code for the n <= 512 counts cnt[] (LDS,
// each < 2^23), into len[] (LDS bytes); unused symbols get 0, a single used symbol 1.  The wave
// sorts the used symbols by (count, symbol) (a bitonic sort of count << 9 | symbol keys over the
// next power of two >= n, unused keys last); lane 0 then runs Moffat and Katajainen's in-place
// construction ("In-place calculation of minimum-redundancy codes", WADS 1995) over the sorted
// counts and, if a depth exceeds maxb, clamps the depths and moves leaves down until the Kraft sum
// is exactly 1 (the zlib/miniz limiting heuristic).  Scratch (LDS): sa[max(64, pow2 >= n)] (may
// alias cnt: the counts are read first), ss[n], num[33].  Wave-collective.
__device__ void huff_lengths(const uint32_t* cnt, uint32_t n, uint32_t maxb, uint8_t* len, uint32_t* sa, uint16_t* ss,
                             uint32_t* num, uint32_t lane) {
    uint32_t P = 64u;
    while (P < n) P <<= 1;
    uint32_t key[8];
    uint32_t used = 0u;
#pragma unroll
    for (uint32_t t = 0; t < 8u; t++) {
        const uint32_t s = lane + 64u * t;
        const uint32_t c = s < n && 64u * t < P ? cnt[s] : 0u;
        key[t] = c ? ((c << 9) | s) : 0xFFFFFFFFu;
        used += static_cast<uint32_t>(__popcll(__ballot(c != 0u)));
    }
    wave_sync();
#pragma unroll
    for (uint32_t t = 0; t < 8u; t++) {
        const uint32_t s = lane + 64u * t;
        if (64u * t < P) sa[s] = key[t];
        if (s < n) len[s] = 0u;
    }
    wave_sync();
    for (uint32_t kk = 2; kk <= P; kk <<= 1)
        for (uint32_t j = kk >> 1; j > 0u; j >>= 1) {
            for (uint32_t i = lane; i < P; i += 64u) {
                const uint32_t pi = i ^ j;
                if (pi > i) {
                    const uint32_t x = sa[i], y = sa[pi];
                    if ((x > y) == ((i & kk) == 0u)) {
                        sa[i] = y;
                        sa[pi] = x;
                    }
                }
            }
            wave_sync();
        }
    for (uint32_t r = lane; r < used; r += 64u) {  // the sorted counts in sa[], their symbols in ss[]
        const uint32_t x = sa[r];
        ss[r] = static_cast<uint16_t>(x & 511u);
        sa[r] = x >> 9;
    }
    wave_sync();
    if (lane == 0 && used == 1u) len[ss[0]] = 1u;
    if (used < 2u) {
        wave_sync();
        return;
    }
    const int m = static_cast<int>(used);
    uint32_t* A = sa;
    if (lane == 0) {
        // Phase 1 (lane 0): the internal nodes' weights, two queues (internal nodes from A[root],
        // leaves from A[leaf]); the next weights of both queues are kept in registers and their
        // loads issued a step ahead (a node's weight is final once built, leaves are never written).
        const uint32_t kInf = 0xFFFFFFFFu;
        uint32_t r0 = A[0] + A[1];  // weight of node root; r1: of node root + 1 once built
        A[0] = r0;
        uint32_t r1 = 0u;
        int root = 0, leaf = 2;
        uint32_t l0 = leaf < m ? A[leaf] : kInf, l1 = leaf + 1 < m ? A[leaf + 1] : kInf;
        auto take_root = [&](int next) -> uint32_t {
            const uint32_t w = r0;
            A[root] = static_cast<uint32_t>(next);  // consumed: its parent
            root++;
            r0 = r1;
            r1 = root + 1 < next ? A[root + 1] : 0u;
            return w;
        };
        auto take_leaf = [&]() -> uint32_t {
            const uint32_t w = l0;
            leaf++;
            l0 = l1;
            l1 = leaf + 1 < m ? A[leaf + 1] : kInf;
            return w;
        };
        for (int next = 1; next < m - 1; next++) {
            const uint32_t w1 = (leaf >= m || r0 < l0) ? take_root(next) : take_leaf();
            const uint32_t w2 = (leaf >= m || (root < next && r0 < l0)) ? take_root(next) : take_leaf();
            const uint32_t w = w1 + w2;
            A[next] = w;
            if (root == next) r0 = w;
            else if (root + 1 == next) r1 = w;
        }
        // Phase 2: parent pointers to depths, downwards (a parent's depth is final before its
        // children's; the parent pointer is read an iteration ahead, the previous depth forwarded)
        A[m - 2] = 0u;
        if (m >= 3) {
            uint32_t dprev = 0u, p = A[m - 3];
            for (int i = m - 3; i >= 0; i--) {
                const uint32_t pn = i > 0 ? A[i - 1] : 0u;
                const uint32_t di = (p == static_cast<uint32_t>(i + 1) ? dprev : A[p]) + 1u;
                A[i] = di;
                dprev = di;
                p = pn;
            }
        }
        // Phase 3: depths to leaf depths (the node at A[root] read a step ahead)
        int avbl = 1, usedc = 0, dpth = 0, next = m - 1;
        root = m - 2;
        uint32_t ar = A[root], an = root > 0 ? A[root - 1] : 0u;
        while (avbl > 0) {
            while (root >= 0 && static_cast<int>(ar) == dpth) {
                usedc++;
                root--;
                ar = an;
                an = root > 0 ? A[root - 1] : 0u;
            }
            while (avbl > usedc) {
                A[next--] = static_cast<uint32_t>(dpth);
                avbl--;
            }
            avbl = 2 * usedc;
            dpth++;
            usedc = 0;
        }
    }
    wave_sync();
    // A[i]: depth of the i-th least frequent symbol (non-increasing in i); the depths' histogram
    if (lane < 33u) num[lane] = 0u;
    wave_sync();
    uint32_t maxd = 0u;
    for (int i = static_cast<int>(lane); i < m; i += 64) {
        const uint32_t dd = A[i] < 32u ? A[i] : 32u;
        atomicAdd(&num[dd], 1u);
        maxd = dd > maxd ? dd : maxd;
    }
    for (uint32_t o = 32; o > 0; o >>= 1) maxd = max(maxd, static_cast<uint32_t>(__shfl_xor(maxd, static_cast<int>(o), 64)));
    wave_sync();
    if (lane == 0 && maxd > maxb) {
        for (uint32_t l = maxb + 1u; l <= 32u; l++) {
            num[maxb] += num[l];
            num[l] = 0u;
        }
        uint32_t total = 0u;
        for (uint32_t l = 1; l <= maxb; l++) total += num[l] << (maxb - l);
        while (total != (1u << maxb)) {
            num[maxb]--;
            for (uint32_t l = maxb - 1u; l > 0u; l--)
                if (num[l]) {
                    num[l]--;
                    num[l + 1u] += 2u;
                    break;
                }
            total--;
        }
    }
    wave_sync();
    // lengths: the least frequent symbols take the longest (sorted index i -> its length's bucket)
    for (int i = static_cast<int>(lane); i < m; i += 64) {
        uint32_t l = maxb, acc = num[maxb];
        while (static_cast<uint32_t>(i) >= acc && l > 1u) {
            l--;
            acc += num[l];
        }
        len[ss[i]] = static_cast<uint8_t>(l);
    }
    wave_sync();
}

// The bit layout of a span's output for one code (hb = block header bits incl. the 3-bit BTYPE
// header, eob = the end-of-block code's length): each segment's bit offset and info (see the
// descriptor), the total in bits (a multiple of 8).  cls/bits/slen per segment, nseg segments.
// One lane; deflate_emit_kernel writes exactly these bits.
__device__ uint32_t deflate_layout(const uint32_t* cls, const uint32_t* bits, const uint32_t* slen, uint32_t nseg,
                                   uint32_t hb, uint32_t eob, uint32_t* boff, uint32_t* info) {
    uint32_t pos = 0u;
    for (uint32_t j = 0; j < nseg; j++) {
        const uint32_t c = cls[j];
        const bool first = j == 0u || cls[j - 1u] != c, end = j + 1u == nseg, last = end || cls[j + 1u] != c;
        uint32_t inf = c | (first ? 4u : 0u) | (last ? 8u : 0u) | (end ? 16u : 0u);
        if (boff) boff[j] = pos;
        if (c == kClsCoded) {
            pos += (first ? hb : 0u) + bits[j] + (last ? eob : 0u);
            if (end) pos = ((pos + 3u + 7u) & ~7u) + 32u;  // sync flush: 000, pad, 00 00 FF FF
        } else {
            if (first) {
                uint32_t run = 0u;
                for (uint32_t k = j; k < nseg && cls[k] == kClsStored; k++) run += slen[k];
                inf |= run << 16;
                pos = ((pos + 3u + 7u) & ~7u) + 32u;  // BFINAL 0, BTYPE 00, pad, LEN, NLEN
            }
            pos += 8u * slen[j];
        }
        if (info) info[j] = inf;
    }
    return pos;
}

__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Bits OR-ed into an LDS word buffer from any bit offset (neighbouring segments share words).
struct OrBits {
    uint64_t bb;
    uint32_t nb;
    uint32_t wa;
    uint32_t* buf;
    __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
        bb |= static_cast<uint64_t>(v) << nb;
        nb += n;
        if (nb >= 32u) {
            atomicOr(&buf[wa++], static_cast<uint32_t>(bb));
            bb >>= 32;
            nb -= 32u;
        }
    }
    __device__ __forceinline__ void pad() { put(0u, (8u - (nb & 7u)) & 7u); }
    __device__ __forceinline__ void flush() {
        if (nb) atomicOr(&buf[wa], static_cast<uint32_t>(bb));
    }
};

// The dynamic block header (RFC 1951 §3.2.7) for the code lengths len[0..316): HLIT, HDIST,
// HCLEN, the code-length code's lengths in the permuted order, then the literal/length and
// distance lengths (one sequence) run-length coded with 16 (the previous length 3-6 times), 17
// (3-10 zeros) and 18 (11-138 zeros) through that code (lengths <= 7, at least two used symbols:
// inflaters reject an incomplete code-length code).  Bits to hdr[] (LDS words); returns their
// count.  Wave-parallel: the runs start where a length differs from the one before (a ballot per
// 64 positions), each run's lane emits its symbols at its offset (a prefix over the runs in order),
// and every symbol's code goes to its bit offset (a prefix over the symbols), OR-ed into hdr.
// Scratch (LDS): cl[316] (symbol | extra << 8), clcnt[19], cllen[20], clcode[19], misc[4] and
// huff_lengths' sa/ss/num.  Wave-collective.
__device__ uint32_t dyn_header(const uint8_t* len, uint32_t* hdr, uint16_t* cl, uint32_t* clcnt, uint8_t* cllen,
                               uint32_t* clcode, uint32_t* sa, uint16_t* ss, uint32_t* num, uint32_t* misc,
                               uint32_t lane) {
    uint32_t hlit = 257u, hdist = 1u;  // the last used literal/length and distance codes
    for (uint32_t k = 0; k < kNLit; k += 64u) {
        const uint64_t m = __ballot(k + lane < kNLit && len[k + lane] != 0u);
        if (m) hlit = max(hlit, k + 64u - static_cast<uint32_t>(__builtin_clzll(m)));
    }
    {
        const uint64_t m = __ballot(lane < kNDist && len[kNLit + lane] != 0u);
        if (m) hdist = max(hdist, 64u - static_cast<uint32_t>(__builtin_clzll(m)));
    }
    const uint32_t nt = hlit + hdist;
    auto at = [&](uint32_t i) -> uint32_t { return i < hlit ? len[i] : len[kNLit + i - hlit]; };
    if (lane < 19u) clcnt[lane] = 0u;
    for (uint32_t j = lane; j < kHdrWords; j += 64u) hdr[j] = 0u;
    uint64_t S[5];  // run starts, per 64 positions
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const uint32_t i = 64u * static_cast<uint32_t>(c) + lane;
        S[c] = __ballot(i < nt && (i == 0u || at(i) != at(i - 1u)));
    }
    wave_sync();
    auto emit = [&](uint32_t v, uint32_t r, auto f) {  // the symbols of a run of r lengths v
        if (v == 0u) {
            while (r >= 11u) {
                const uint32_t k = r < 138u ? r : 138u;
                f(18u, k - 11u);
                r -= k;
            }
            if (r >= 3u) {
                f(17u, r - 3u);
                r = 0u;
            }
        } else {
            f(v, 0u);
            r--;
            while (r >= 3u) {
                const uint32_t k = r < 6u ? r : 6u;
                f(16u, k - 3u);
                r -= k;
            }
        }
        for (; r > 0u; r--) f(v, 0u);
    };
    uint32_t base = 0;  // symbols of the runs before this group of positions
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const uint32_t i = 64u * static_cast<uint32_t>(c) + lane;
        const bool st = (S[c] >> lane) & 1ull;
        uint32_t r = 0, v = 0, cnt = 0;
        if (st) {
            uint32_t nx = nt;  // the next run's start
            const uint64_t above = lane < 63u ? (S[c] >> (lane + 1u)) << (lane + 1u) : 0ull;
            if (above) {
                nx = 64u * static_cast<uint32_t>(c) + static_cast<uint32_t>(__builtin_ctzll(above));
            } else {
                for (int c2 = c + 1; c2 < 5; c2++)
                    if (S[c2]) {
                        nx = 64u * static_cast<uint32_t>(c2) + static_cast<uint32_t>(__builtin_ctzll(S[c2]));
                        break;
                    }
            }
            r = nx - i;
            v = at(i);
            emit(v, r, [&](uint32_t, uint32_t) { cnt++; });
        }
        uint32_t incl = cnt;
        for (uint32_t o = 1; o < 64u; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (st) {
            uint32_t o = base + incl - cnt;
            emit(v, r, [&](uint32_t sy, uint32_t x) {
                cl[o++] = static_cast<uint16_t>(sy | (x << 8));
                atomicAdd(&clcnt[sy], 1u);
            });
        }
        base += static_cast<uint32_t>(__shfl(incl, 63, 64));
    }
    const uint32_t ncl = base;
    wave_sync();
    if (lane == 0) {
        uint32_t nz = 0;
        for (uint32_t j = 0; j < 19u; j++) nz += clcnt[j] != 0u;
        if (nz < 2u) {
            if (clcnt[0] == 0u) clcnt[0] = 1u;
            else clcnt[1] = 1u;
        }
    }
    wave_sync();
    huff_lengths(clcnt, 19u, 7u, cllen, sa, ss, num, lane);
    canon_codes(cllen, 19u, clcode, lane);
    wave_sync();
    uint32_t hclen = 19u;
    {
        const uint32_t l = lane < 19u ? cllen[kClOrder[lane]] : 0u;
        const uint64_t m = __ballot(l != 0u);
        hclen = m ? 64u - static_cast<uint32_t>(__builtin_clzll(m)) : 0u;
        hclen = hclen < 4u ? 4u : hclen;
    }
    if (lane == 0) {
        OrBits w{0ull, 0u, 0u, hdr};
        w.put(hlit - 257u, 5);
        w.put(hdist - 1u, 5);
        w.put(hclen - 4u, 4);
        for (uint32_t i = 0; i < hclen; i++) w.put(cllen[kClOrder[i]], 3);
        w.flush();
    }
    uint32_t pos = 14u + 3u * hclen;
    for (uint32_t k0 = 0; k0 < ncl; k0 += 64u) {  // each symbol's code (and extra bits) at its offset
        const uint32_t k = k0 + lane;
        uint32_t sy = 0, x = 0, c = 0, nbits = 0;
        if (k < ncl) {
            sy = cl[k] & 31u;
            x = cl[k] >> 8;
            c = clcode[sy];
            nbits = (c >> 16) + (sy == 16u ? 2u : sy == 17u ? 3u : sy == 18u ? 7u : 0u);
        }
        uint32_t incl = nbits;
        for (uint32_t o = 1; o < 64u; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (k < ncl) {
            const uint32_t p0 = pos + incl - nbits;
            OrBits w{0ull, p0 & 31u, p0 >> 5, hdr};
            w.put(c & 0xFFFFu, c >> 16);
            if (sy >= 16u) w.put(x, sy == 16u ? 2u : sy == 17u ? 3u : 7u);
            w.flush();
        }
        pos += static_cast<uint32_t>(__shfl(incl, 63, 64));
    }
    wave_sync();
    return pos;
}

// S2 framing header of span b: 0x00, 3-byte LE length of (CRC + block), then the masked CRC
// (written by the copy kernel) and the block's uvarint uncompressed length.
__device__ __forceinline__ uint32_t uvarint_len(uint32_t v) { return v < 128u ? 1u : v < 16384u ? 2u : 3u; }

// The chunk of global span b: the last c with spans[c] <= b (empty chunks share their prefix
// with the next).
__device__ __forceinline__ uint32_t span_chunk(const CompArgs& a, uint32_t b) {
    uint32_t lo = 0, hi = a.n;  // spans[lo] <= b < spans[hi]
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.spans[mid] <= b) lo = mid; else hi = mid;
    }
    return lo;
}

// Walk a coded segment's tokens: lit(x) per literal byte position, match(x, len, dist) per match.
template <typename FL, typename FM>
__device__ __forceinline__ void walk_tokens(const uint32_t* tok, uint32_t nm, uint32_t x0, uint32_t xe, FL lit, FM match) {
    uint32_t x = x0;
    for (uint32_t k = 0; k < nm; k++) {
        const uint32_t t = tok[k];
        for (const uint32_t e = x + (t >> 23); x < e; x++) lit(x);
        const uint32_t n = ((t >> 15) & 255u) + 3u;
        match(x, n, (t & 0x7FFFu) + 1u);
        x += n;
    }
    for (; x < xe; x++) lit(x);
}

// KCDC_TRACE builds (tools/ztrace.py with a deflate name): lane 0's s_memtime (low 32 bits) at the
// deflate span's phase ends, descriptor words 281.. (after the plan's mode word)
#ifdef KCDC_TRACE
#define KCDC_DSTAMP(i)                                                                              \
    do {                                                                                          \
        if (threadIdx.x == 0)                                                                     \
            a.desc[static_cast<uint64_t>(blockIdx.x) * kDescWords + 281u + (i)] =                  \
                static_cast<uint32_t>(__builtin_amdgcn_s_memtime());                              \
    } while (0)
#else
#define KCDC_DSTAMP(i) \
    do {               \
    } while (0)
#endif

// The span's deflate plan (see "deflate blocks of a span"), after the parse: symbol counts of the
// coded segments, the dynamic code and its header (effort >= 1), every segment's size under the
// dynamic and the fixed code, the cheapest of dynamic / fixed / one stored block, and the layout
// to the span's descriptor; span_bytes[b] = the span's output bytes.  S: 2048 words of LDS
// scratch (the match tables, free once every lane's parse is done).
__device__ __forceinline__ void deflate_plan(const CompArgs& a, uint32_t b, uint32_t lane, uint32_t span_len,
                                             uint32_t x0, uint32_t word, uint32_t nm, uint32_t* hist, uint32_t* S,
                                             const uint32_t* L, uint32_t d) {
    __syncthreads();  // every lane's parse is done
    uint32_t* sa = S;                                      // [0, 288)
    uint16_t* ss = reinterpret_cast<uint16_t*>(S + 288);   // 286 u16
    uint8_t* lens = reinterpret_cast<uint8_t*>(S + 432);   // 316 bytes
    uint32_t* hdr = S + 512;                               // kHdrWords
    uint32_t* clcnt = S + 584;                             // 19
    uint8_t* cllen = reinterpret_cast<uint8_t*>(S + 604);  // 19 bytes
    uint32_t* clcode = S + 612;                            // 19
    uint16_t* cl = reinterpret_cast<uint16_t*>(S + 640);   // 316 u16
    uint32_t *lcls = S + 800, *lbd = S + 864, *lbf = S + 928, *llen = S + 992;  // per segment
    uint32_t *boff = S + 1056, *info = S + 1120;
    uint32_t* num = S + 1184;                              // 33
    uint32_t* misc = S + 1220;                             // 8
    const uint32_t seg_len = x0 < span_len ? min(kSeg, span_len - x0) : 0u, xe = x0 + seg_len;
    const bool coded = seg_len && !(word & kStored);
    const uint32_t* tok = reinterpret_cast<const uint32_t*>(a.slots + (static_cast<uint64_t>(b) * 64u + lane) * kSlot);
    const uint64_t cm = __ballot(coded);
    const bool dynamic = cm != 0ull && a.effort >= 1u;
    if (dynamic && coded)
        walk_tokens(tok, nm, x0, xe, [&](uint32_t x) { atomicAdd(&hist[st_byte(L, d, x)], 1u); },
                    [&](uint32_t, uint32_t n, uint32_t dist) {
                        const MatchSyms m = match_syms(n, dist);
                        atomicAdd(&hist[m.ls], 1u);
                        atomicAdd(&hist[kNLit + m.ds], 1u);
                    });
    __syncthreads();
    KCDC_DSTAMP(2);
    uint32_t hb = 0;
    if (dynamic) {
        if (lane == 0) {
            hist[256] = 1u;  // end of block
            uint32_t nz = 0;  // >= 2 distance codes: inflaters take no incomplete code but a single 1-bit one
            for (uint32_t j = 0; j < kNDist; j++) nz += hist[kNLit + j] != 0u;
            if (nz < 2u) {
                if (hist[kNLit] == 0u) hist[kNLit] = 1u;
                if (hist[kNLit + 1] == 0u) hist[kNLit + 1] = 1u;
            }
        }
        __syncthreads();
        huff_lengths(hist, kNLit, 15u, lens, S + 1232, ss, num, lane);  // (512 words: free from 1228)
        huff_lengths(hist + kNLit, kNDist, 15u, lens + kNLit, sa, ss, num, lane);
        KCDC_DSTAMP(3);
        hb = dyn_header(lens, hdr, cl, clcnt, cllen, clcode, sa, ss, num, misc, lane);
    }
    KCDC_DSTAMP(4);
    uint32_t bd = 0, bf = 0;  // the segment's bits under the dynamic / the fixed code
    if (coded)
        walk_tokens(tok, nm, x0, xe,
                    [&](uint32_t x) {
                        const uint32_t v = st_byte(L, d, x);
                        if (dynamic) bd += lens[v];
                        bf += fixed_len(v);
                    },
                    [&](uint32_t, uint32_t n, uint32_t dist) {
                        const MatchSyms m = match_syms(n, dist);
                        if (dynamic) bd += lens[m.ls] + lens[kNLit + m.ds] + m.eb + m.deb;
                        bf += fixed_len(m.ls) + 5u + m.eb + m.deb;
                    });
    lcls[lane] = coded ? kClsCoded : seg_len ? kClsStored : 0u;
    lbd[lane] = bd;
    lbf[lane] = bf;
    llen[lane] = seg_len;
    __syncthreads();
    KCDC_DSTAMP(5);
    const uint32_t nseg = (span_len + kSeg - 1u) / kSeg;
    if (lane == 0) {
        uint32_t mode = kModeStored, bits = 8u * (span_len + 5u);
        if (cm) {
            const uint32_t tf = deflate_layout(lcls, lbf, llen, nseg, 3u, 7u, nullptr, nullptr);
            if (tf < bits) {
                mode = kModeFixed;
                bits = tf;
            }
            if (dynamic) {
                const uint32_t td = deflate_layout(lcls, lbd, llen, nseg, 3u + hb, lens[256], nullptr, nullptr);
                if (td < bits) {
                    mode = kModeDynamic;
                    bits = td;
                }
            }
            if (mode == kModeDynamic)
                deflate_layout(lcls, lbd, llen, nseg, 3u + hb, lens[256], boff, info);
            else if (mode == kModeFixed)
                deflate_layout(lcls, lbf, llen, nseg, 3u, 7u, boff, info);
        }
        misc[4] = mode;
        misc[5] = bits;
    }
    __syncthreads();
    const uint32_t mode = misc[4];
    uint32_t* desc = a.desc + static_cast<uint64_t>(b) * kDescWords;
    if (mode != kModeStored) {
        a.seglen[b * 64u + lane] = nm;
        desc[kDescOff + lane] = lane < nseg ? boff[lane] : 0u;
        desc[kDescInfo + lane] = lane < nseg ? info[lane] : 0u;
    }
    if (mode == kModeDynamic) {
        for (uint32_t k = lane; k < 80u; k += 64u) desc[kDescLens + k] = k < 79u ? S[432 + k] : 0u;
        for (uint32_t k = lane; k < (hb + 31u) / 32u; k += 64u) desc[kDescHdr + k] = hdr[k];
    }
    if (lane == 0) {
        desc[kDescMode] = mode | (hb << 8);
        a.span_bytes[b] = misc[5] >> 3;
    }
}

// A zstd sequence word: literal length, match length (4..512) and distance (15 bits) in 32 bits.
// Inside a 512-byte segment ll + (ml - 4) <= 508, so the pair fits a 9-bit field A and an 8-bit
// field B: ml - 4 < 256 as (A, B) = (ll, ml - 4); a longer match (then ll <= 252) as
// (508 - ll, 511 - (ml - 4)), told apart by A + B > 508 (no short pair sums past 508).
__device__ __forceinline__ uint32_t zseq_word(uint32_t ll, uint32_t ml, uint32_t dist) {
    const uint32_t t = ml - 4u;
    const bool lng = t >= 256u;
    return ((lng ? 508u - ll : ll) << 23) | ((lng ? 511u - t : t) << 15) | dist;
}
__device__ __forceinline__ uint32_t zseq_ll(uint32_t v) {
    const uint32_t A = v >> 23, B = (v >> 15) & 255u;
    return A + B > 508u ? 508u - A : A;
}
__device__ __forceinline__ uint32_t zseq_ml(uint32_t v) {
    const uint32_t A = v >> 23, B = (v >> 15) & 255u;
    return (A + B > 508u ? 511u - B : B) + 4u;
}

// The sequences section of a segment's zstd block at sb8 + o (RFC 8878 §3.1.1.3.2):
// Number_of_Sequences, Symbol_Compression_Modes = 0 (all Predefined), then the FSE bitstream written
// backwards from the last sequence (zstd's ZSTD_encodeSequences order), closed by the 1-bit end
// marker.  The sequences are read from the slot's words 143 - k (the parse keeps them at the slot's
// end); the writer must stay below the words not yet read and inside the segment's size, else
// kZOver (rare: costly sequences).  write = false: the size only, nothing stored.
constexpr uint32_t kZOver = 0xFFFFFFFFu;
__device__ uint32_t zstd_seqs(uint8_t* sb8, uint32_t o, uint32_t nseq, uint32_t seg_len, bool write) {
    const uint32_t* words = reinterpret_cast<const uint32_t*>(sb8);
    uint32_t pos = o;
    uint64_t bb = 0;
    uint32_t nb = 0;
    auto put = [&](uint32_t v, uint32_t n) {
        bb |= static_cast<uint64_t>(v) << nb;
        nb += n;
        while (nb >= 8u) {
            if (write) sb8[pos] = static_cast<uint8_t>(bb);
            pos++;
            bb >>= 8;
            nb -= 8u;
        }
    };
    if (nseq < 128u) {
        put(nseq, 8);
    } else {
        put(128u + (nseq >> 8), 8);
        put(nseq & 255u, 8);
    }
    if (nseq) {
        put(0u, 8);  // Predefined_Mode x 3
        uint32_t sLL = 0, sML = 0, sOF = 0;
        for (int k = static_cast<int>(nseq) - 1; k >= 0; k--) {
            if (pos + 8u > 4u * (144u - static_cast<uint32_t>(k) - 1u) || pos > seg_len + 2u) return kZOver;
            const uint32_t v = words[143u - static_cast<uint32_t>(k)];
            const uint32_t ll = zseq_ll(v), ml = zseq_ml(v), ov = (v & 0x7FFFu) + 3u;
            uint32_t llc, llb, llx, mlc, mlb, mlx;
            ll_code(ll, llc, llb, llx);
            ml_code(ml, mlc, mlb, mlx);
            const uint32_t ofc = 31u - __builtin_clz(ov), ofx = ov - (1u << ofc);
            if (k == static_cast<int>(nseq) - 1) {
                sLL = kFseLL.first[llc];
                sML = kFseML.first[mlc];
                sOF = kFseOF.first[ofc];
            } else {  // the decoder's updates after sequence k: LL, ML, OF -> written OF, ML, LL
                const uint32_t nOF = kFseOF.enc[ofc][sOF];
                put(sOF - kFseOF.base[nOF], kFseOF.nb[nOF]);
                sOF = nOF;
                const uint32_t nML = kFseML.enc[mlc][sML];
                put(sML - kFseML.base[nML], kFseML.nb[nML]);
                sML = nML;
                const uint32_t nLL = kFseLL.enc[llc][sLL];
                put(sLL - kFseLL.base[nLL], kFseLL.nb[nLL]);
                sLL = nLL;
            }
            put(llx, llb);  // the decoder reads offset, match length, literal length extras
            put(mlx, mlb);
            put(ofx, ofc);
        }
        put(sML, 6);  // initial states, read LL, OF, ML
        put(sOF, 5);
        put(sLL, 6);
        put(1u, 1);  // end marker
        if (nb) put(0u, 8u - nb);
    }
    return pos - o;
}

// ---------------------------------------------------------------- zstd: span-level blocks (effort >= 1)
// The parse leaves each segment's sequences in its slot (word 143 - k: literal length << 23 |
// (match length - 4) << 15 | distance) and their count in the span's descriptor.  zstd_emit_kernel
// (one workgroup per span) then writes the span as kZBlks Compressed_Blocks, runs of segments of
// about equal sequence counts (RFC 8878 §3.1.1.2), all sharing the span's codes:
//   literals   one Huffman code for the span (<= 11 bits, direct weights: the largest literal
//              must be <= 128), its tree carried by the span's first compressed block that uses it
//              (Compressed_Literals_Block), the later ones Treeless; 1 stream up to 1023 literals,
//              else 4 (jump table); a block whose raw literals are smaller keeps them raw;
//   sequences  three FSE tables (literal length, offset, match length codes) normalized from the
//              span's code counts and described once (Symbol_Compression_Mode 2, the first
//              compressed block with sequences), Repeat_Mode (3) in the later blocks; offset
//              value 1 (repeat offset 1) for a match at the previous sequence's distance in the
//              same block (a block's first sequence names its offset: a Raw_Block before it
//              leaves the decoder's repeat offsets at the last compressed block's);
//   fallback   a block whose body is not smaller than its bytes is a Raw_Block (it carries no
//              table: the next compressed block does).
// Segments are the parse's unit, blocks the coding unit: a segment's literals before its first
// sequence join the previous sequence's (the block's carry).  Literal streams are written by all
// lanes at once (each lane its literals' bits at its offset in the stream; bytes shared by two
// lanes go through per-lane edge records merged by the block's leader); the sequences bitstream
// by the block's leader lane, backwards (ZSTD_encodeSequences order), after a counting pass (the
// raw-or-compressed choice needs the exact size first).  Block k goes to the slots of its first
// segment (its segments' kSlot bytes each, > 512); its seglen word is its size, 0 for the
// other segments (deflate_copy_kernel skips them).  tools/zstd_span_model.py is the host model of
// this layout (libzstd-decoded; mixed data 0.327 per-segment -> 0.281 span-level).
// The reference (klauspost/compress/zstd, compressor_zstd.go:15-18) writes the same block types
// (Huffman literals with table reuse, FSE-compressed or repeated sequence tables, raw fallback).
constexpr uint32_t kZBlks = 4;                     // blocks per span (one per wave of zstd_emit_kernel)
#ifndef KCDC_ZSEGW
#define KCDC_ZSEGW 4
#endif
constexpr uint32_t kZSegW = KCDC_ZSEGW;            // a segment's cost in the block split, in sequences
constexpr uint32_t kZMaxSeq = kSpan / 4;           // a sequence covers >= 4 bytes
constexpr uint32_t kZDesc = 80;                    // a table description: <= 53 x 10 bits + 4 + 2 bytes
constexpr uint32_t kZNone = 0xFFFFFFFFu;

struct ZTab {          // FSE encoding table (RFC 8878 §4.1; zstd's FSE_buildCTable formulation)
    uint16_t st[512];  // next state, by (state >> bits) + dfs; states in [size, 2 size)
    uint2 dd[53];      // per symbol: x = dnb = (bits << 16) - (count << bits) (output bits =
                       // (state + dnb) >> 16), y = dfs = cumulative count before s - count of s
    uint32_t al;       // Accuracy_Log
};

// One field's table from the span's code counts (total nseq).  Wave-collective, lane = symbol:
// Accuracy_Log from the sequence count (log2 - 2 as zstd's FSE_optimalTableLog, 5..maxlog, >= used
// + 1 cells); counts rounded to 2^al with
// every used symbol >= 1 (the rounding surplus to the largest entry, a deficit taken from the
// largest one at a time); the encoding table (the RFC's spread puts cumulative cell j at
// j * step mod size, so each symbol's lane walks the states in order and keeps those whose
// j = state * step^-1 is one of its cells); lane 0 writes the description (RFC 8878 §4.1.1, as
// zstd's FSE_writeNCount) into desc and returns its bytes.  norm: nsym shorts of LDS.
__device__ uint32_t zstd_table(const uint32_t* cnt, uint32_t nsym, uint32_t maxlog, uint32_t nseq, uint16_t* tst,
                               uint2* tdd, uint32_t* tal, int16_t* norm, uint8_t* desc, uint32_t lane) {
    const uint32_t cs = lane < nsym ? cnt[lane] : 0u;
    const uint64_t um = __ballot(cs != 0u);
    const uint32_t used = static_cast<uint32_t>(__popcll(um));
    const uint32_t last = 63u - static_cast<uint32_t>(__builtin_clzll(um));
    uint32_t al = nseq > 4u ? 29u - static_cast<uint32_t>(__builtin_clz(nseq - 1u)) : 0u;  // log2(n) - 2, as zstd
    al = al < 5u ? 5u : al > maxlog ? maxlog : al;
    while ((1u << al) < used + 1u && al < maxlog) al++;
    const uint32_t size = 1u << al;
    uint32_t v = cs ? (cs * size + nseq / 2u) / nseq : 0u;
    if (cs && v == 0u) v = 1u;
    uint32_t sum = v;
    for (uint32_t o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, static_cast<int>(o), 64);
    int32_t diff = static_cast<int32_t>(size) - static_cast<int32_t>(sum);
    while (diff != 0) {  // size >= used + 1: while the sum is over, the largest entry is > 1
        uint32_t mx = v;
        for (uint32_t o = 32; o > 0; o >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, static_cast<int>(o), 64)));
        const uint32_t am = static_cast<uint32_t>(__builtin_ctzll(__ballot(v == mx)));
        if (diff > 0) {
            if (lane == am) v += static_cast<uint32_t>(diff);
            diff = 0;
        } else {
            if (lane == am) v--;
            diff++;
        }
    }
    if (lane < nsym) norm[lane] = static_cast<int16_t>(v);
    uint32_t incl = v;
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const uint32_t cum = incl - v;
    if (lane < nsym) {
        uint2 e;
        if (v == 0u) {
            e = make_uint2(((al + 1u) << 16) - size, 0u);
        } else if (v == 1u) {
            e = make_uint2((al << 16) - size, cum - 1u);
        } else {
            const uint32_t mbo = al - (31u - static_cast<uint32_t>(__builtin_clz(v - 1u)));
            e = make_uint2((mbo << 16) - (v << mbo), cum - v);
        }
        tdd[lane] = e;
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3u, mask = size - 1u;  // step is odd
    uint32_t inv = step;  // Newton: step * inv == 1 (mod 2^32)
    for (int i = 0; i < 5; i++) inv *= 2u - step * inv;
    if (v) {
        uint32_t r = cum;
        for (uint32_t u = 0; u < size; u++)
            if (((u * inv) & mask) - cum < v) tst[r++] = static_cast<uint16_t>(size + u);
    }
    if (lane == 0) *tal = al;
    wave_sync();
    if (lane != 0) return 0u;
    // description: Accuracy_Log - 5, then each count + 1 in a variable number of bits, runs of
    // zero counts after a zero as 2-bit repeat flags (16 bits = 24 zeros)
    uint64_t bb = 0;
    uint32_t nb = 0, o = 0;
    auto put = [&](uint32_t x, uint32_t n) {
        bb |= static_cast<uint64_t>(x) << nb;
        nb += n;
        while (nb >= 8u) {
            desc[o++] = static_cast<uint8_t>(bb);
            bb >>= 8;
            nb -= 8u;
        }
    };
    put(al - 5u, 4);
    int32_t remaining = static_cast<int32_t>(size) + 1;
    int32_t threshold = static_cast<int32_t>(size);
    uint32_t nbits = al + 1u, sym = 0;
    bool prev0 = false;
    while (sym <= last && remaining > 1) {
        if (prev0) {
            uint32_t start = sym;
            while (sym <= last && norm[sym] == 0) sym++;
            while (sym >= start + 24u) {
                start += 24u;
                put(0xFFFFu, 16);
            }
            while (sym >= start + 3u) {
                start += 3u;
                put(3u, 2);
            }
            put(sym - start, 2);
        }
        int32_t count = norm[sym++];
        const int32_t mx = (2 * threshold - 1) - remaining;
        remaining -= count;
        count += 1;
        if (count >= threshold) count += mx;
        put(static_cast<uint32_t>(count), count < mx ? nbits - 1u : nbits);
        prev0 = count == 1;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
    }
    if (nb) put(0u, 8u - nb);
    return o;
}
__device__ __forceinline__ uint32_t zstd_table(const uint32_t* cnt, uint32_t nsym, uint32_t maxlog, uint32_t nseq,
                                               ZTab& t, int16_t* norm, uint8_t* desc, uint32_t lane) {
    return zstd_table(cnt, nsym, maxlog, nseq, t.st, t.dd, &t.al, norm, desc, lane);
}

// The predefined distribution of field f (0 LL, 1 OF, 2 ML; RFC 8878 §3.1.1.3.2.2) as an encoding
// table: the "less than 1" symbols (-1) take one cell each at the top, the others are spread with
// the RFC's step skipping those cells.  One lane; tsym: 64 bytes of scratch.
__device__ int32_t zstd_pre_norm(uint32_t f, uint32_t s) {
    return f == 0u ? (s < 36u ? kLLNorm[s] : 0) : f == 1u ? (s < 29u ? kOFNorm[s] : 0) : (s < 53u ? kMLNorm[s] : 0);
}
__device__ void zstd_pre_table(uint32_t f, ZTab& t, uint8_t* tsym) {
    const uint32_t al = f == 1u ? 5u : 6u, size = 1u << al, n = f == 0u ? 36u : f == 1u ? 29u : 53u;
    uint32_t high = size - 1u;
    for (uint32_t s = 0; s < n; s++)
        if (zstd_pre_norm(f, s) == -1) tsym[high--] = static_cast<uint8_t>(s);
    const uint32_t step = (size >> 1) + (size >> 3) + 3u, mask = size - 1u;
    uint32_t pos = 0;
    for (uint32_t s = 0; s < n; s++)
        for (int32_t i = 0; i < zstd_pre_norm(f, s); i++) {
            tsym[pos] = static_cast<uint8_t>(s);
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    uint32_t total = 0;
    for (uint32_t s = 0; s < n; s++) {  // running slots in dd[].x first
        t.dd[s].x = total;
        const int32_t v = zstd_pre_norm(f, s);
        total += v == -1 ? 1u : static_cast<uint32_t>(v);
    }
    for (uint32_t u = 0; u < size; u++) t.st[t.dd[tsym[u]].x++] = static_cast<uint16_t>(size + u);
    total = 0;
    for (uint32_t s = 0; s < 53u; s++) {
        const int32_t v = zstd_pre_norm(f, s);
        if (v == 0) {
            t.dd[s] = make_uint2(((al + 1u) << 16) - size, 0u);
        } else if (v == -1 || v == 1) {
            t.dd[s] = make_uint2((al << 16) - size, total - 1u);
            total += 1u;
        } else {
            const uint32_t fv = static_cast<uint32_t>(v);
            const uint32_t mbo = al - (31u - static_cast<uint32_t>(__builtin_clz(fv - 1u)));
            t.dd[s] = make_uint2((mbo << 16) - (fv << mbo), total - fv);
            total += fv;
        }
    }
    t.al = al;
}

// Sequence i's offset value (RFC 8878 §3.1.2.5) from its word v, the two before it (pv, ppv), its
// literal length ll and the previous one's llp (both with carries); blk0: the block's first sequence.
// Repeat offset 1 is always the previous sequence's distance: offset value 1 when ll > 0.  With
// ll = 0, offset value 1 names repeat offset 2, which is this distance when the previous two
// sequences had it and the previous one had ll = 0 (then it was either explicit, pushing the one
// before it to second place, or itself repeat offset 2, which swaps the first two).  A block's
// first sequences name their offsets: the history before the block is not known here.
__device__ __forceinline__ uint32_t zstd_ov(uint32_t i, uint32_t blk0, uint32_t v, uint32_t pv, uint32_t ppv,
                                            uint32_t ll, uint32_t llp) {
    const uint32_t dist = v & 0x7FFFu;
    const bool same1 = i > blk0 && (pv & 0x7FFFu) == dist;
    if (same1 && ll > 0u) return 1u;
    if (same1 && ll == 0u && llp == 0u && i >= blk0 + 2u && (ppv & 0x7FFFu) == dist) return 1u;
    return dist + 3u;
}

// A block of the span: [3-byte header][literals section][sequences section]; offsets from the block.
struct ZBlk {
    uint32_t raw;        // input bytes
    uint32_t nl, ns;     // literals, sequences
    uint32_t q;          // literals per Huffman stream (the last takes the rest)
    uint32_t nstr;       // Huffman streams: 1 or 4
    uint32_t fbits;      // the sequences bitstream's bits (with the end marker); kZNone: too long
    uint32_t fscr;       // where the bitstream was written first (16-byte aligned address)
    uint32_t sbits[4];   // each Huffman stream's bits (with the end marker)
    uint32_t role;       // kZr*
    uint32_t body;       // bytes after the block header
    uint32_t lh;         // the literals header's bytes
    uint32_t lit0;       // where the raw literals / the first Huffman stream start
    uint32_t soff[4];    // where each Huffman stream starts
    uint32_t seq0;       // where the sequences section starts
    uint32_t sh;         // the sequences section's header bytes (count, modes, descriptions)
};
constexpr uint32_t kZrCoded = 1, kZrHuff = 2, kZrTree = 4, kZrTables = 8;

// KCDC_TRACE builds (tools/ztrace.py): thread 0's s_memtime at the phase ends, descriptor words 64..
#ifdef KCDC_TRACE
#define KCDC_ZSTAMP(i)                                                                                  \
    do {                                                                                              \
        if (tid == 0)                                                                                 \
            reinterpret_cast<uint64_t*>(a.desc + static_cast<uint64_t>(b) * kDescWords + 64u)[i] =   \
                __builtin_amdgcn_s_memtime();                                                         \
    } while (0)
#else
#define KCDC_ZSTAMP(i) \
    do {               \
    } while (0)
#endif

// One workgroup of 4 waves per span (zstd, effort >= 1), after lz_spans_kernel<kFmtZstd>.  Wave 0
// does the per-segment work (lane = segment); waves 1..3 build the three FSE tables while wave 0
// builds the Huffman code; each wave's lane 0 writes one block's sequences bitstream (the serial
// part: four SIMDs instead of one).
__global__ __launch_bounds__(256) void zstd_emit_kernel(CompArgs a) {
    __shared__ uint32_t L[kLdsWords];
    __shared__ uint32_t seqw[kZMaxSeq];
    // H: the literal counts and the Huffman scratch, then the weights' FSE table
    __shared__ uint32_t H[256 + 256 + 128];
    uint32_t* hist = H;
    uint32_t* sa = H + 256;
    uint16_t* ss = reinterpret_cast<uint16_t*>(H + 512);
    __shared__ uint32_t zc[256];           // Huffman code | bits << 16
    __shared__ uint8_t lens[256];
    __shared__ uint32_t num[40];
    __shared__ uint32_t fcnt[36 + 53 + 32];  // LL, ML, OF code counts
    __shared__ ZTab tab[3];                  // LL, OF, ML (the description's order)
    __shared__ int16_t fnorm[3][64];
    __shared__ uint8_t fdesc[3][kZDesc];
    __shared__ uint32_t fdlen[3];
    __shared__ uint32_t fmode[3];            // each field's Symbol_Compression_Mode in the carrier block
    __shared__ uint32_t ln_off[65], ln_nseq[64], ln_len[64], ln_nlit[64], ln_carry[64], ln_p[64], ln_prev[64];
    __shared__ uint32_t ln_bits[64 * 4];
    __shared__ uint16_t pbits[64 * 4 * 4];   // per lane, part (wave) and stream: the part's literal bits
    __shared__ ZBlk blk[kZBlks];
    __shared__ uint32_t misc[2];             // [0]: the tree description's bytes (0: no Huffman), [1]: longest code
    __shared__ uint8_t hdesc[128];           // the Huffman tree description (RFC 8878 §4.2.1)
    __shared__ uint32_t llut[64], mlut[128];  // code | extra bits << 8 | baseline << 16 (ml: of ml - 3)
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const bool w0 = wv == 0u;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    const uint32_t c = span_chunk(a, b);
    const uint32_t u = b - a.spans[c];
    const uint64_t len = a.in_lens[c];
    const uint64_t sb = static_cast<uint64_t>(u) * kSpan;
    const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
    KCDC_ZSTAMP(0);
    const uint32_t d = stage_span(L, a.in + a.in_offs[c] + sb, span_len, tid, 256u);
    const uint32_t x0 = kSeg * lane;
    const uint32_t seg_len = x0 < span_len ? min(kSeg, span_len - x0) : 0u, xe = x0 + seg_len;
    const uint32_t nseq = seg_len ? a.desc[static_cast<uint64_t>(b) * kDescWords + lane] : 0u;
    hist[tid] = 0u;
    ln_bits[tid] = 0u;
    if (tid < 36u + 53u + 32u) fcnt[tid] = 0u;
    if (w0) {
        uint32_t cc, nn, xx;
        ll_code(lane, cc, nn, xx);
        llut[lane] = cc | (nn << 8) | ((lane - xx) << 16);
        for (uint32_t m = lane; m < 128u; m += 64u) {
            ml_code(m + 3u, cc, nn, xx);
            mlut[m] = cc | (nn << 8) | ((m - xx) << 16);
        }
    }
    // the span's sequences in order (lane-major), each lane's literal count and trailing literals
    uint32_t incl = nseq;
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const uint32_t off = incl - nseq;
    // The blocks: runs of segments of about equal cost (a sequence is a step of its block's
    // serial FSE chain, a segment with data 4 besides), each at least one segment; cut where a
    // segment's middle passes each quarter of the span's cost.
    const uint32_t cost = nseq + (seg_len ? kZSegW : 0u);
    const uint32_t ci = incl + kZSegW * static_cast<uint32_t>(__popcll(__ballot(seg_len != 0u) & ((2ull << lane) - 1ull)));
    const uint32_t ctot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ci), 63));
    const uint32_t mid2 = 2u * ci - cost;  // twice the segment's middle
    uint32_t b1 = static_cast<uint32_t>(__popcll(__ballot(2u * mid2 <= ctot)));
    uint32_t b2 = static_cast<uint32_t>(__popcll(__ballot(2u * mid2 <= 2u * ctot)));
    uint32_t b3 = static_cast<uint32_t>(__popcll(__ballot(2u * mid2 <= 3u * ctot)));
    b1 = min(max(b1, 1u), 61u);
    b2 = min(max(b2, b1 + 1u), 62u);
    b3 = min(max(b3, b2 + 1u), 63u);
    auto bsel = [&](uint32_t i) -> uint32_t { return i == 0u ? 0u : i == 1u ? b1 : i == 2u ? b2 : i == 3u ? b3 : 64u; };
    const uint32_t k = (lane >= b1 ? 1u : 0u) + (lane >= b2 ? 1u : 0u) + (lane >= b3 ? 1u : 0u);
    const uint32_t lead = bsel(k), bend = bsel(k + 1u);  // the lane's block: its first lane, one past its last
    const uint32_t* sq = reinterpret_cast<const uint32_t*>(a.slots + (static_cast<uint64_t>(b) * 64u + lane) * kSlot);
    uint32_t covered = 0, matched = 0;
    for (uint32_t j = 0; j < (w0 ? nseq : 0u); j++) {  // (wave 0: the others use the LDS copies)
        const uint32_t v = sq[143u - j];
        seqw[off + j] = v;
        const uint32_t ml = zseq_ml(v);
        covered += zseq_ll(v) + ml;
        matched += ml;
    }
    const uint32_t nlit = seg_len - matched, tail = seg_len - covered;
    // the lane's first literal's index in its block
    uint32_t pin = nlit;
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(pin, o, 64);
        if (lane - lead >= o) pin += y;
    }
    // the nearest earlier segment with sequences (0 if none: never followed past a block's first)
    const uint64_t nz = __ballot(nseq != 0u) & ((1ull << lane) - 1ull);
    if (w0) {
        ln_off[lane] = off;
        if (lane == 63u) ln_off[64] = incl;
        ln_nseq[lane] = nseq;
        ln_prev[lane] = nz ? 63u - static_cast<uint32_t>(__builtin_clzll(nz)) : 0u;
        ln_len[lane] = seg_len;
        ln_nlit[lane] = nlit;
        ln_carry[lane] = tail;  // (becomes the carry below)
        ln_p[lane] = pin - nlit;
    }
    __syncthreads();
    if (tid == 0) {  // literals pending before each segment's first sequence, within its block
        uint32_t cy = 0;
        for (uint32_t j = 0; j < 64u; j++) {
            if (j == 0u || j == b1 || j == b2 || j == b3) cy = 0u;
            const uint32_t t = ln_carry[j];
            ln_carry[j] = cy;
            cy = ln_nseq[j] ? t : cy + ln_len[j];
        }
    }
    __syncthreads();
    KCDC_ZSTAMP(1);
    // The four waves share the counting passes: wave w takes the lane's literals at bytes
    // [x0 + 128 w, x0 + 128 (w + 1)) of its segment (lits_part: f(value, index in the block)) and
    // its sequences j = w mod 4.
    const uint32_t plo = x0 + 128u * wv, phi = plo + 128u;
    auto lits_part = [&](auto f) {
        uint32_t idx = ln_p[lane];  // the block index of the first literal at or after plo
        auto run = [&](uint32_t x, uint32_t e) {
            const uint32_t a0 = max(x, plo), e0 = min(e, phi);
            idx += (a0 > x ? min(a0, e) - x : 0u);
            if (a0 >= e0) return;
            uint32_t y = a0;
            for (; y + 4u <= e0; y += 4u) {
                const uint32_t w = st_ld32(L, d, y);
                f(w & 255u, idx);
                f((w >> 8) & 255u, idx + 1u);
                f((w >> 16) & 255u, idx + 2u);
                f(w >> 24, idx + 3u);
                idx += 4u;
            }
            for (; y < e0; y++) f(st_byte(L, d, y), idx++);
            idx += e > e0 ? e - e0 : 0u;
        };
        uint32_t x = x0;
        for (uint32_t j = 0; j < nseq && x < phi; j++) {
            const uint32_t v = seqw[off + j], ll = zseq_ll(v);
            run(x, x + ll);
            x += ll + zseq_ml(v);
        }
        if (x < phi) run(x, xe);
    };
    // the codes of the lane's sequences: the carry joins the first literal length; offset value 1
    // for the previous sequence's distance (same block, literal length > 0), else distance + 3
    {
        lits_part([&](uint32_t v, uint32_t) { atomicAdd(&hist[v], 1u); });
        const uint32_t blk0 = ln_off[lead];
        const uint32_t cy = ln_carry[lane];
        for (uint32_t j = wv; j < nseq; j += 4u) {
            const uint32_t i = off + j, v = seqw[i];
            const uint32_t ll = zseq_ll(v) + (j == 0u ? cy : 0u);
            const uint32_t pv = seqw[i > blk0 ? i - 1u : i], ppv = seqw[i > blk0 + 1u ? i - 2u : i];
            const uint32_t lp = j ? lane : ln_prev[lane];  // the segment of sequence i - 1
            const uint32_t llp = zseq_ll(pv) + (i > blk0 && i - 1u == ln_off[lp] ? ln_carry[lp] : 0u);
            const uint32_t ov = zstd_ov(i, blk0, v, pv, ppv, ll, llp);
            uint32_t llc, llb, llx, mlc, mlb, mlx;
            ll_code(ll, llc, llb, llx);
            ml_code(zseq_ml(v), mlc, mlb, mlx);
            atomicAdd(&fcnt[llc], 1u);
            atomicAdd(&fcnt[36u + mlc], 1u);
            atomicAdd(&fcnt[89u + 31u - static_cast<uint32_t>(__builtin_clz(ov))], 1u);
        }
    }
    __syncthreads();
    KCDC_ZSTAMP(2);
    // The span's Huffman code and its description (RFC 8878 §4.2.1): the weights of symbols
    // 0..top-1 (the last one's is implied) FSE-compressed (zstd's HUF_compressWeights: one table,
    // two interleaved states) when that is smaller or when top > 128, else direct 4-bit weights.
    // No Huffman literals when neither applies (e.g. all weights equal: random bytes).
    uint32_t used = 0, top = 0;
    for (uint32_t i = 0; i < 256u; i += 64u) {
        const uint64_t m = __ballot(hist[i + lane] != 0u);
        used += static_cast<uint32_t>(__popcll(m));
        if (m) top = i + 63u - static_cast<uint32_t>(__builtin_clzll(m));
    }
    // Worth a code at all?  The literals' order-0 entropy against 8 bits each: a span whose
    // literals are near-uniform (random data) would save less than a description costs.
    float ent = 0.f;
    uint32_t nl_span = 0;
    for (uint32_t i = lane; i < 256u; i += 64u) {
        const uint32_t cv = hist[i];
        nl_span += cv;
        ent += cv ? static_cast<float>(cv) * __log2f(static_cast<float>(cv)) : 0.f;
    }
    for (uint32_t o = 32; o > 0; o >>= 1) {
        nl_span += static_cast<uint32_t>(__shfl_xor(nl_span, static_cast<int>(o), 64));
        ent += __shfl_xor(ent, static_cast<int>(o), 64);
    }
    // bits = N log2 N - sum c log2 c; a Huffman code is within ~3 % of it here
    const float hbits = nl_span ? static_cast<float>(nl_span) * __log2f(static_cast<float>(nl_span)) - ent : 0.f;
    const bool try_huff = used >= 2u && 1.02f * hbits / 8.f + 24.f < static_cast<float>(nl_span);
    const uint32_t nseq_span = ln_off[64];
    __syncthreads();  // every wave has read the counts (wave 0 reuses their space below)
    if (w0 && try_huff) {
        huff_lengths(hist, 256u, 11u, lens, sa, ss, num, lane);
        KCDC_ZSTAMP(14);
        // codes: by weight ascending (longest first), then symbol (RFC 8878 §4.2.1.4); each
        // weight's codes start where the lighter weights' end, ranks within a weight by ballot
        uint32_t maxb = 0;
        for (uint32_t i = lane; i <= top; i += 64u) maxb = max(maxb, static_cast<uint32_t>(lens[i]));
        for (uint32_t o = 32; o > 0; o >>= 1) maxb = max(maxb, static_cast<uint32_t>(__shfl_xor(maxb, static_cast<int>(o), 64)));
        uint32_t start[12];
        {
            uint32_t acc = 0;  // in 2^(w-1) cells
#pragma unroll
            for (uint32_t w = 1; w < 12u; w++) {
                uint32_t cw = 0;
                for (uint32_t i = 0; i <= top; i += 64u) {
                    const uint32_t l = i + lane <= top ? lens[i + lane] : 0u;
                    cw += static_cast<uint32_t>(__popcll(__ballot(l && maxb + 1u - l == w)));
                }
                start[w] = w <= maxb ? acc >> (w - 1u) : 0u;
                acc += w <= maxb ? cw << (w - 1u) : 0u;
            }
        }
        const uint64_t lt = (1ull << lane) - 1ull;
        for (uint32_t i = 0; i <= top; i += 64u) {
            const uint32_t sy = i + lane, l = sy <= top ? lens[sy] : 0u, w = l ? maxb + 1u - l : 0u;
            uint32_t code = 0;
#pragma unroll
            for (uint32_t j = 1; j < 12u; j++) {
                const uint64_t m = __ballot(w == j);
                if (w == j) code = start[j] + static_cast<uint32_t>(__popcll(m & lt));
                start[j] += static_cast<uint32_t>(__popcll(m));
            }
            if (sy <= top) zc[sy] = l ? (code | (l << 16)) : 0u;
        }
        if (lane == 0) misc[1] = maxb;
        // the weights' table in H (the counts there are spent): 32 states, 12 symbols
        uint16_t* wst = reinterpret_cast<uint16_t*>(H);
        uint2* wdd = reinterpret_cast<uint2*>(H + 16);
        uint32_t* wal = H + 40;
        int16_t* wnorm = reinterpret_cast<int16_t*>(H + 48);
        uint32_t* wcnt = H + 64;
        if (lane < 16u) wcnt[lane] = 0u;
        wave_sync();
        auto wt = [&](uint32_t sy) -> uint32_t { return lens[sy] ? maxb + 1u - lens[sy] : 0u; };
        for (uint32_t sy = lane; sy < top; sy += 64u) atomicAdd(&wcnt[wt(sy)], 1u);
        wave_sync();
        uint32_t wmax = lane < 12u ? wcnt[lane] : 0u;
        for (uint32_t o = 32; o > 0; o >>= 1) wmax = max(wmax, static_cast<uint32_t>(__shfl_xor(wmax, static_cast<int>(o), 64)));
        const bool fse_ok = top >= 3u && wmax < top;  // >= 2 distinct weights (one value: an RLE case)
        const uint32_t nc = fse_ok ? zstd_table(wcnt, 12u, 5u, top, wst, wdd, wal, wnorm, hdesc + 1, lane) : 0u;
        KCDC_ZSTAMP(15);
        if (lane == 0) {
            const uint32_t direct = top <= 128u ? 1u + (top + 1u) / 2u : 0u;
            uint32_t fsz = 0;
            if (fse_ok) {  // backwards, two states (FSE_compress_usingCTable): the decoder reads state 1 first
                uint64_t bb = 0;
                uint32_t nb = 0, o = 1u + nc;
                auto put = [&](uint32_t x, uint32_t n) {
                    bb |= static_cast<uint64_t>(x) << nb;
                    nb += n;
                    while (nb >= 8u) {
                        if (o < 128u) hdesc[o] = static_cast<uint8_t>(bb);
                        o++;
                        bb >>= 8;
                        nb -= 8u;
                    }
                };
                auto initw = [&](uint32_t sy) -> uint32_t {
                    const uint2 e = wdd[sy];
                    const uint32_t nbo = (e.x + (1u << 15)) >> 16;
                    const uint32_t s0 = (nbo << 16) - e.x;
                    return wst[(s0 >> nbo) + e.y];
                };
                auto encw = [&](uint32_t& st, uint32_t sy) {
                    const uint2 e = wdd[sy];
                    const uint32_t nbo = (st + e.x) >> 16;
                    put(st & ((1u << nbo) - 1u), nbo);
                    st = wst[(st >> nbo) + e.y];
                };
                uint32_t i = top, s1, s2;
                if (top & 1u) {
                    s1 = initw(wt(--i));
                    s2 = initw(wt(--i));
                    encw(s1, wt(--i));
                } else {
                    s2 = initw(wt(--i));
                    s1 = initw(wt(--i));
                }
                for (bool two = true; i > 0u; two = !two) encw(two ? s2 : s1, wt(--i));
                const uint32_t wa = *wal;
                put(s2 & ((1u << wa) - 1u), wa);
                put(s1 & ((1u << wa) - 1u), wa);
                put(1u, 1);  // end marker
                if (nb) put(0u, 8u - nb);
                if (o < 128u) fsz = o;
            }
            uint32_t tsz = 0;
            if (fsz && (!direct || fsz < direct)) {
                hdesc[0] = static_cast<uint8_t>(fsz - 1u);  // < 128: FSE-compressed weights of that size
                tsz = fsz;
            } else if (direct) {  // direct weights: W = maxb + 1 - bits (0: unused), high nibble first
                hdesc[0] = static_cast<uint8_t>(127u + top);
                for (uint32_t j = 0; 2u * j < top; j++)
                    hdesc[1u + j] = static_cast<uint8_t>((wt(2u * j) << 4) | (2u * j + 1u < top ? wt(2u * j + 1u) : 0u));
                tsz = direct;
            }
            misc[0] = tsz;
        }
    }
    if (!w0 && nseq_span) {  // the LL, OF, ML tables, one per wave (at the same time as the Huffman code)
        const uint32_t t = wv - 1u;
        const uint32_t* cn = fcnt + (t == 0u ? 0u : t == 1u ? 89u : 36u);
        const uint32_t ns = t == 0u ? 36u : t == 1u ? 32u : 53u;
        const uint32_t r = zstd_table(cn, ns, t == 1u ? 8u : 9u, nseq_span, tab[t], fnorm[t], fdesc[t], lane);
        // The mode of least estimated cost (the FSE cost of a symbol ~ log2(size / count)):
        // Compressed (the table above and its description), Predefined (no description) or RLE
        // (one symbol: one byte, no state bits).
        const uint32_t cs = lane < ns ? cn[lane] : 0u;
        const int32_t pn = static_cast<int32_t>(zstd_pre_norm(t, lane));
        const float alc = static_cast<float>(tab[t].al), alp = t == 1u ? 5.f : 6.f;
        float cc = cs ? static_cast<float>(cs) * (alc - __log2f(static_cast<float>(fnorm[t][lane]))) : 0.f;
        float cp = cs ? (pn == 0 ? 1e30f : static_cast<float>(cs) * (alp - __log2f(pn == -1 ? 1.f : static_cast<float>(pn)))) : 0.f;
        for (uint32_t o = 32; o > 0; o >>= 1) {
            cc += __shfl_xor(cc, static_cast<int>(o), 64);
            cp += __shfl_xor(cp, static_cast<int>(o), 64);
        }
        const uint64_t um = __ballot(cs != 0u);
        const uint32_t rb = static_cast<uint32_t>(__shfl(static_cast<int>(r), 0, 64));
        if (lane == 0) {
            uint32_t mode = 2u;
            if (__popcll(um) == 1) {  // RLE: state 1 forever, no bits
                const uint32_t sy = static_cast<uint32_t>(__builtin_ctzll(um));
                tab[t].st[0] = 1u;
                tab[t].st[1] = 1u;
                tab[t].dd[sy] = make_uint2(0u, 0u);
                tab[t].al = 0u;
                fdesc[t][0] = static_cast<uint8_t>(sy);
                fdlen[t] = 1u;
                mode = 1u;
            } else if (cp <= cc + 8.f * static_cast<float>(rb)) {
                zstd_pre_table(t, tab[t], fdesc[t]);
                fdlen[t] = 0u;
                mode = 0u;
            } else {
                fdlen[t] = r;
            }
            fmode[t] = mode;
        }
    }
    __syncthreads();
    KCDC_ZSTAMP(3);
    KCDC_ZSTAMP(4);
    const uint32_t tsz = try_huff ? misc[0] : 0u;  // the tree description's bytes
    const bool huff = tsz != 0u;
    // literal streams: each lane's bits per stream of its block
    uint32_t nl_blk = 0;
    for (uint32_t j = lead; j < bend; j++) nl_blk += ln_nlit[j];
    const uint32_t nstr = nl_blk > 1023u ? 4u : 1u;
    const uint32_t qn = nstr == 4u ? (nl_blk + 3u) / 4u : (nl_blk ? nl_blk : 1u);
    if (huff && ln_nlit[lane]) {  // (the four waves, each its part of the lane's literals)
        uint32_t bits[4] = {0u, 0u, 0u, 0u};
        uint32_t q = 4u, nextb = 0u;  // the stream of the part's first literal, then by boundary
        lits_part([&](uint32_t v, uint32_t idx) {
            if (q == 4u) {
                q = nstr == 1u ? 0u : min(idx / qn, 3u);
                nextb = nstr == 1u ? kZNone : (q + 1u) * qn;
            }
            if (idx == nextb && q < 3u) {
                q++;
                nextb += qn;
            }
            const uint32_t nbq = zc[v] >> 16;
            bits[0] += q == 0u ? nbq : 0u;
            bits[1] += q == 1u ? nbq : 0u;
            bits[2] += q == 2u ? nbq : 0u;
            bits[3] += q == 3u ? nbq : 0u;
        });
        for (uint32_t q = 0; q < 4u; q++)
            if (bits[q]) atomicAdd(&ln_bits[lane * 4u + q], bits[q]);
        for (uint32_t q = 0; q < 4u; q++) pbits[(lane * 4u + wv) * 4u + q] = static_cast<uint16_t>(bits[q]);
    } else {
        for (uint32_t q = 0; q < 4u; q++) pbits[(lane * 4u + wv) * 4u + q] = 0u;
    }
    __syncthreads();
    KCDC_ZSTAMP(5);
    const uint32_t ns_blk = ln_off[bend] - ln_off[lead];
    const uint32_t tdesc = nseq_span ? fdlen[0] + fdlen[1] + fdlen[2] : 0u;
    uint8_t* R = a.slots + (static_cast<uint64_t>(b) * 64u + lead) * kSlot + kZOff;  // the block's bytes
    uint32_t* Sw = reinterpret_cast<uint32_t*>(a.slots + (static_cast<uint64_t>(b) * 64u + lead) * kSlot);  // its dwords
    if (w0 && lane == lead) {
        ZBlk& B = blk[k];
        uint32_t raw = 0;
        for (uint32_t j = lead; j < bend; j++) raw += ln_len[j];
        B.raw = raw;
        B.nl = nl_blk;
        B.ns = ns_blk;
        B.q = qn;
        B.nstr = nstr;
        uint32_t lit = (nl_blk < 32u ? 1u : nl_blk < 4096u ? 2u : 3u) + nl_blk;  // raw literals
        for (uint32_t q = 0; q < 4u; q++) {
            uint32_t s = 0;
            for (uint32_t j = lead; j < bend; j++) s += ln_bits[j * 4u + q];
            B.sbits[q] = s + 1u;
        }
        if (huff && nl_blk) {  // the Huffman section with the tree: a bound on any literals section chosen
            uint32_t cs = tsz + (nstr == 4u ? 6u : 0u);
            for (uint32_t q = 0; q < nstr; q++) cs += (B.sbits[q] + 7u) / 8u;
            lit = min(lit, 5u + cs);
        }
        // The bitstream goes first to a scratch place above any layout the choices below can
        // give (then moves down); a stream that would not fit the block's bytes from there makes
        // the block raw: it exceeds the block's own size (the literals bound above is at most the
        // tree's bytes over the section chosen).
        B.fscr = ((3u + 3u + lit + 3u + tdesc + kZOff + 15u) & ~15u) - kZOff;
        B.fbits = 0u;
    }
    __syncthreads();
    if (blk[wv].ns) {  // wave wv: block wv's sequences bitstream
        // Backwards from the block's last sequence (ZSTD_encodeSequences order), 64 at a time: the
        // wave's lanes derive 64 sequences' codes, extras and table entries at once (independent
        // of the states), then lane 0 runs the state chain over them, reading each lane's values
        // with readlane: per sequence the chain is the three state steps and the bit packing.
        ZBlk& B = blk[wv];
        const uint32_t lead = bsel(wv), end = bsel(wv + 1u), fs = B.fscr;
        uint8_t* R = a.slots + (static_cast<uint64_t>(b) * 64u + lead) * kSlot + kZOff;
        uint32_t* dst = reinterpret_cast<uint32_t*>(R + fs);
        const uint32_t region = (end - lead) * kSlot - kZOff;  // the block's bytes
        // words (the chain stops within 7 of it); a block whose scratch starts too high is raw
        const uint32_t lim = fs + 96u <= region ? (region - fs - 40u) / 4u : 0u;
        const ZTab &tLL = tab[0], &tOF = tab[1], &tML = tab[2];
        const uint32_t i0 = ln_off[lead], i1 = ln_off[end];
        uint64_t bb = 0;       // lane 0: the bit writer
        uint32_t nb = 0, o = 0;
        uint32_t sLL = 0, sML = 0, sOF = 0;  // lane 0: the states
        bool over = lim == 0u;
        // val < 2^n, n <= 63, with nb < 32 before: both words of the low 64 bits are stored, the
        // cursor moves by the full words, the rest stays (bits past 64 come from the high part)
        auto put64 = [&](uint64_t val, uint32_t n) {
            const uint64_t low = bb | (val << nb);
            const uint64_t high = nb ? (val >> (64u - nb)) : 0ull;
            const uint32_t tot = nb + n;
            dst[o] = static_cast<uint32_t>(low);
            dst[o + 1u] = static_cast<uint32_t>(low >> 32);
            o += tot >> 5;
            bb = tot >= 64u ? high : tot >= 32u ? (low >> 32) : low;
            nb = tot & 31u;
        };
        auto put = [&](uint32_t x, uint32_t n) {  // x < 2^n; the current word is stored every time
            bb |= static_cast<uint64_t>(x) << nb;
            nb += n;
            dst[o] = static_cast<uint32_t>(bb);
            const bool full = nb >= 32u;
            o += full ? 1u : 0u;
            bb = full ? bb >> 32 : bb;
            nb -= full ? 32u : 0u;
        };
        for (uint32_t hi = i1; hi > i0 && !over; hi = hi > i0 + 64u ? hi - 64u : i0) {
            const uint32_t cnt = min(64u, hi - i0);
            // lane t: sequence hi - 1 - t
            const uint32_t idx = hi - 1u - min(lane, cnt - 1u);
            uint32_t cy = 0, cyp = 0;  // its (and the previous one's) segment's carry when it is the segment's first
            for (uint32_t sg = lead; sg < end; sg++) {
                const uint32_t lo = ln_off[sg], hs = ln_off[sg + 1u];
                if (lo < hs && idx == lo) cy = ln_carry[sg];
                if (lo < hs && idx > i0 && idx - 1u == lo) cyp = ln_carry[sg];
            }
            const uint32_t v = seqw[idx], pv = seqw[idx > i0 ? idx - 1u : idx];
            const uint32_t ppv = seqw[idx > i0 + 1u ? idx - 2u : idx];
            const uint32_t ll = zseq_ll(v) + cy, m = zseq_ml(v) - 3u;
            const uint32_t ov = zstd_ov(idx, i0, v, pv, ppv, ll, zseq_ll(pv) + cyp);
            const uint32_t tl = llut[min(ll, 63u)], hl = 31u - static_cast<uint32_t>(__builtin_clz(ll | 1u));
            const uint32_t tm = mlut[min(m, 127u)], hm = 31u - static_cast<uint32_t>(__builtin_clz(m));
            const bool bl = ll >= 64u, bm = m >= 128u;
            const uint32_t llc = bl ? hl + 19u : (tl & 255u);
            const uint32_t llb = bl ? hl : ((tl >> 8) & 255u);
            const uint32_t llx = ll - (bl ? (1u << hl) : (tl >> 16));
            const uint32_t mlc = bm ? hm + 36u : (tm & 255u);
            const uint32_t mlb = bm ? hm : ((tm >> 8) & 255u);
            const uint32_t mlx = m - (bm ? (1u << hm) : (tm >> 16));
            const uint32_t ofc = 31u - static_cast<uint32_t>(__builtin_clz(ov));
            const uint32_t x1 = llx | (mlx << llb), n1 = llb + mlb, x2 = ov - (1u << ofc);
            const uint2 eLL = tLL.dd[llc], eML = tML.dd[mlc], eOF = tOF.dd[ofc];
            // packed for the chain: dnb (< 2^20) | (dfs + 512) << 20; x1 (< 2^22: a literal length < 2^15
            // and a match length < 2^9) | n1 << 22; x2 | ofc << 16
            uint32_t pLL = eLL.x | ((eLL.y + 512u) << 20), pML = eML.x | ((eML.y + 512u) << 20);
            uint32_t pOF = eOF.x | ((eOF.y + 512u) << 20), xa = x1 | (n1 << 22), xb = x2 | (ofc << 16);
            // every lane's values are read across lanes below: keep them computed here, by all
            asm volatile("" : "+v"(pLL), "+v"(pML), "+v"(pOF), "+v"(xa), "+v"(xb));
            if (lane == 0) {
                uint32_t t = 0;
                if (hi == i1) {  // the block's last sequence: the initial states
                    auto init = [&](const ZTab& tb, uint2 e) -> uint32_t {
                        const uint32_t nbo = (e.x + (1u << 15)) >> 16;
                        const uint32_t s0 = (nbo << 16) - e.x;
                        return tb.st[(s0 >> nbo) + e.y];
                    };
                    sML = init(tML, eML);
                    sOF = init(tOF, eOF);
                    sLL = init(tLL, eLL);
                    put(x1, n1);  // the decoder reads offset, match length, literal length extras
                    put(x2, ofc);
                    t = 1;
                }
                for (; t < cnt; t++) {  // each earlier sequence: state bits (OF, ML, LL), extras
                    const int tt = static_cast<int>(t);
                    const uint32_t qOF = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pOF), tt));
                    const uint32_t qML = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pML), tt));
                    const uint32_t qLL = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pLL), tt));
                    const uint32_t ya = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(xa), tt));
                    const uint32_t yb = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(xb), tt));
                    const uint32_t dOF = qOF & 0xFFFFFu, fOF = (qOF >> 20) - 512u;
                    const uint32_t dML = qML & 0xFFFFFu, fML = (qML >> 20) - 512u;
                    const uint32_t dLL = qLL & 0xFFFFFu, fLL = (qLL >> 20) - 512u;
                    const uint32_t nOF = (sOF + dOF) >> 16, nML = (sML + dML) >> 16, nLL = (sLL + dLL) >> 16;
                    const uint32_t bits = (sOF & ((1u << nOF) - 1u)) | ((sML & ((1u << nML) - 1u)) << nOF) |
                                          ((sLL & ((1u << nLL) - 1u)) << (nOF + nML));
                    sOF = tOF.st[(sOF >> nOF) + fOF];
                    sML = tML.st[(sML >> nML) + fML];
                    sLL = tLL.st[(sLL >> nLL) + fLL];
                    // the sequence's <= 63 bits (states <= 26, extras <= 22 + 15) as one value
                    const uint32_t ns = nOF + nML + nLL, n1s = ya >> 22;
                    const uint64_t val = static_cast<uint64_t>(bits) | (static_cast<uint64_t>(ya & 0x3FFFFFu) << ns) |
                                         (static_cast<uint64_t>(yb & 0xFFFFu) << (ns + n1s));
                    put64(val, ns + n1s + (yb >> 16));
                    if (o > lim) {
                        over = true;
                        break;
                    }
                }
            }
            over = __builtin_amdgcn_readfirstlane(over ? 1 : 0) != 0;
        }
        if (lane == 0) {
            if (!over) {
                const uint32_t am = tML.al, ao = tOF.al, ala = tLL.al;  // initial states, read LL, OF, ML
                put((sML & ((1u << am) - 1u)) | ((sOF & ((1u << ao) - 1u)) << am), am + ao);
                put(sLL & ((1u << ala) - 1u), ala);
                put(1u, 1);  // end marker
            }
            B.fbits = over ? kZNone : 32u * o + nb;
        }
    }
    __syncthreads();
    KCDC_ZSTAMP(6);
    if (tid == 0) {  // each block: raw or compressed, which carries the tree / the tables; sizes
        bool tree_sent = false, tables_sent = false;
        uint32_t bytes = 0;
        for (uint32_t kb = 0; kb < kZBlks; kb++) {
            ZBlk& B = blk[kb];
            B.role = 0u;
            B.body = 0u;
            if (B.raw == 0u) continue;
            const uint32_t n = B.nl;
            const uint32_t rawlh = n < 32u ? 1u : n < 4096u ? 2u : 3u;
            uint32_t lit = rawlh + n, lh = rawlh, use = 0u;
            if (huff && n) {
                uint32_t cs = (tree_sent ? 0u : tsz) + (B.nstr == 4u ? 6u : 0u);
                for (uint32_t q = 0; q < B.nstr; q++) cs += (B.sbits[q] + 7u) / 8u;
                const uint32_t hlh = B.nstr == 1u ? (cs <= 1023u ? 3u : 0u) : (n <= 16383u && cs <= 16383u ? 4u : 5u);
                if (hlh && hlh + cs < lit) {
                    lit = hlh + cs;
                    lh = hlh;
                    use = kZrHuff | (tree_sent ? 0u : kZrTree);
                }
            }
            const bool tables = B.ns && !tables_sent;
            const uint32_t sh = B.ns == 0u ? 1u : (B.ns < 128u ? 1u : 2u) + 1u + (tables ? tdesc : 0u);
            const uint32_t body = B.fbits == kZNone ? kZNone : lit + sh + (B.fbits + 7u) / 8u;
            if (body < B.raw) {
                B.role = kZrCoded | use | (tables ? kZrTables : 0u);
                B.body = body;
                B.lh = lh;
                B.sh = sh;
                uint32_t o = 3u + lh + ((use & kZrTree) ? tsz : 0u);
                if ((use & kZrHuff) && B.nstr == 4u) o += 6u;
                B.lit0 = o;
                if (use & kZrHuff) {
                    for (uint32_t q = 0; q < B.nstr; q++) {
                        B.soff[q] = o;
                        o += (B.sbits[q] + 7u) / 8u;
                    }
                } else {
                    o += n;
                }
                B.seq0 = o;
                if (use & kZrHuff) tree_sent = true;
                if (B.ns) tables_sent = true;
                bytes += 3u + body;
            } else {
                bytes += kZStoredHdr + B.raw;
            }
        }
        a.span_bytes[b] = bytes;
#ifdef KCDC_TRACE
        {  // the span's byte budget (tools/ztrace.py): words 84.. of its descriptor
            uint32_t* tw = a.desc + static_cast<uint64_t>(b) * kDescWords + 84u;
            uint32_t st[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // raw blocks' bytes, literal sections,
            // sequence bitstreams, table descriptions, trees, headers (block + literals + sequences), literals, sequences
            for (uint32_t kb = 0; kb < kZBlks; kb++) {
                const ZBlk& B = blk[kb];
                if (B.raw == 0u) continue;
                if (!(B.role & kZrCoded)) {
                    st[0] += B.raw + 3u;
                    continue;
                }
                st[1] += B.seq0 - 3u - B.lh - ((B.role & kZrTree) ? tsz : 0u);
                st[2] += B.ns ? (B.fbits + 7u) / 8u : 0u;
                st[3] += (B.role & kZrTables) ? tdesc : 0u;
                st[4] += (B.role & kZrTree) ? tsz : 0u;
                st[5] += 3u + B.lh + (B.ns ? B.sh - ((B.role & kZrTables) ? tdesc : 0u) : 1u);
                st[6] += B.nl;
                st[7] += B.ns;
            }
            for (uint32_t i = 0; i < 8u; i++) tw[i] = st[i];
        }
#endif
    }
    __syncthreads();
    KCDC_ZSTAMP(7);
    const ZBlk& B = blk[k];
    // Huffman streams are OR-ed together where parts share a byte: their bytes start at zero
    for (uint32_t kb = 0; kb < kZBlks; kb++) {
        const ZBlk& Z = blk[kb];
        if ((Z.role & (kZrCoded | kZrHuff)) != (kZrCoded | kZrHuff)) continue;
        uint32_t* Sk = reinterpret_cast<uint32_t*>(a.slots + (static_cast<uint64_t>(b) * 64u + bsel(kb)) * kSlot);
        for (uint32_t w = ((kZOff + Z.soff[0]) >> 2) + tid; w < (kZOff + Z.seq0 + 3u) >> 2; w += 256u) Sk[w] = 0u;
    }
    __syncthreads();
    // The literals, each wave its part of every lane's literals (bytes [x0 + 128 w, + 128) of the
    // segment): raw at their index, or Huffman bits at their offset in their stream (each stream
    // holds its literals last to first: a part starts after the bits of the block's later lanes
    // and of its lane's later parts).  Bytes a part fully covers are stored; its partial first
    // and last bytes are OR-ed in (global atomics on the dword), as are the streams' end markers.
    if (B.role & kZrCoded) {
        if (!(B.role & kZrHuff)) {
            lits_part([&](uint32_t v, uint32_t idx) { R[B.lit0 + idx] = static_cast<uint8_t>(v); });
        } else if (ln_nlit[lane]) {
            uint32_t bo[4];
            for (uint32_t q = 0; q < 4u; q++) {
                uint32_t sum = 0;
                for (uint32_t j = lane + 1u; j < bend; j++) sum += ln_bits[j * 4u + q];
                for (uint32_t w = wv + 1u; w < 4u; w++) sum += pbits[(lane * 4u + w) * 4u + q];
                bo[q] = sum;
            }
            auto or_byte = [&](uint32_t q, uint32_t bi, uint32_t v) {  // (slot bases are 4-byte aligned)
                const uint32_t y = kZOff + B.soff[q] + bi;
                atomicOr(Sw + (y >> 2), v << (8u * (y & 3u)));
            };
            uint32_t idx = ln_p[lane] + ln_nlit[lane], q = 4u, qlo = 0u;  // idx: one past the next literal back
            uint64_t bb = 0;
            uint32_t nb = 0, bi = 0, b0 = 0;
            auto close = [&]() {  // the part's last byte in stream q, when partial
                if (q < 4u && nb) or_byte(q, bi, static_cast<uint32_t>(bb & 255u));
            };
            auto lit = [&](uint32_t y) {  // the literal at byte y, block index idx - 1
                idx--;
                if (q == 4u || idx < qlo) {
                    close();
                    q = B.nstr == 1u ? 0u : min(idx / B.q, 3u);
                    qlo = B.nstr == 1u ? 0u : q * B.q;
                    b0 = bo[q];
                    bi = b0 >> 3;
                    nb = b0 & 7u;
                    bb = 0;
                }
                const uint32_t cw = zc[st_byte(L, d, y)];
                bb |= static_cast<uint64_t>(cw & 0xFFFFu) << nb;
                nb += cw >> 16;
                while (nb >= 8u) {
                    const uint32_t v = static_cast<uint32_t>(bb & 255u);
                    if (bi == (b0 >> 3) && (b0 & 7u))
                        or_byte(q, bi, v);  // shared with the part before
                    else
                        R[B.soff[q] + bi] = static_cast<uint8_t>(v);
                    bi++;
                    bb >>= 8;
                    nb -= 8u;
                }
            };
            auto run_back = [&](uint32_t x, uint32_t e) {  // the run [x, e), last to first
                if (e > phi) idx -= e - max(x, phi);
                for (uint32_t y = min(e, phi); y > max(x, plo); y--) lit(y - 1u);
                if (x < plo) idx -= min(e, plo) - x;
            };
            uint32_t xm = x0;
            for (uint32_t j = 0; j < nseq; j++) {
                const uint32_t v = seqw[off + j];
                xm += zseq_ll(v) + zseq_ml(v);
            }
            run_back(xm, xe);  // the trailing literals, then each sequence's, backwards
            for (uint32_t j = nseq; j-- > 0u && xm > plo;) {
                const uint32_t v = seqw[off + j];
                xm -= zseq_ml(v);
                const uint32_t ll = zseq_ll(v);
                run_back(xm - ll, xm);
                xm -= ll;
            }
            close();
        }
        if (w0 && lane == lead && (B.role & kZrHuff))
            for (uint32_t q = 0; q < B.nstr; q++) {
                const uint32_t mb = B.sbits[q] - 1u;  // the end marker: the stream's highest bit
                {
                    const uint32_t y = kZOff + B.soff[q] + (mb >> 3);
                    atomicOr(Sw + (y >> 2), (1u << (mb & 7u)) << (8u * (y & 3u)));
                }
            }
    }
    {  // block wv's sequences bitstream down to its place, by wave wv (above the literals; dst <=
       // src: 1024-byte steps, each read before it is written, never overlap an unread byte)
        const ZBlk& Z = blk[wv];
        if ((Z.role & kZrCoded) && Z.ns) {
            uint8_t* Rw = a.slots + (static_cast<uint64_t>(b) * 64u + bsel(wv)) * kSlot + kZOff;
            const uint32_t n = (Z.fbits + 7u) / 8u;
            const uint8_t* src = Rw + Z.fscr;
            uint8_t* dst = Rw + Z.seq0 + Z.sh;
            const uint32_t t = lane * 16u;
            for (uint32_t o = 0; o < n; o += 1024u) {
                const uint4 w = *reinterpret_cast<const uint4*>(src + o + t);
                const uint32_t wv4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (uint32_t j = 0; j < 16u; j++)
                    if (o + t + j < n) dst[o + t + j] = static_cast<uint8_t>(wv4[j >> 2] >> (8u * (j & 3u)));
            }
        }
    }
    __syncthreads();
    KCDC_ZSTAMP(8);
    if (w0 && lane == lead && (B.role & kZrCoded)) {
        const uint32_t hdr = (B.body << 3) | (2u << 1);  // Compressed_Block, not the last
        R[0] = static_cast<uint8_t>(hdr);
        R[1] = static_cast<uint8_t>(hdr >> 8);
        R[2] = static_cast<uint8_t>(hdr >> 16);
        const uint32_t n = B.nl;
        if (B.role & kZrHuff) {
            const uint32_t typ = (B.role & kZrTree) ? 2u : 3u;  // Compressed / Treeless_Literals_Block
            const uint64_t cs = B.seq0 - 3u - B.lh, nn = n;
            const uint64_t lh = B.nstr == 1u ? (typ | (nn << 4) | (cs << 14))
                               : B.lh == 4u ? (typ | (2u << 2) | (nn << 4) | (cs << 18))
                                            : (typ | (3u << 2) | (nn << 4) | (cs << 22));
            for (uint32_t i = 0; i < B.lh; i++) R[3u + i] = static_cast<uint8_t>(lh >> (8u * i));
            uint32_t o = 3u + B.lh;
            if (B.role & kZrTree)
                for (uint32_t i = 0; i < tsz; i++) R[o++] = hdesc[i];
            if (B.nstr == 4u)
                for (uint32_t q = 0; q < 3u; q++) {
                    const uint32_t sz = (B.sbits[q] + 7u) / 8u;
                    R[o++] = static_cast<uint8_t>(sz);
                    R[o++] = static_cast<uint8_t>(sz >> 8);
                }
        } else {
            const uint32_t rh = n < 32u ? (n << 3) : n < 4096u ? (0x4u | (n << 4)) : (0xCu | (n << 4));
            for (uint32_t i = 0; i < B.lh; i++) R[3u + i] = static_cast<uint8_t>(rh >> (8u * i));
        }
        uint32_t o = B.seq0;
        const uint32_t ns = B.ns;
        if (ns < 128u) {
            R[o++] = static_cast<uint8_t>(ns);
        } else {
            R[o++] = static_cast<uint8_t>(128u + (ns >> 8));
            R[o++] = static_cast<uint8_t>(ns);
        }
        if (ns) {
            // each field's mode in the carrier (0 Predefined, 1 RLE, 2 FSE_Compressed), else Repeat_Mode
            const bool tb = (B.role & kZrTables) != 0u;
            R[o++] = static_cast<uint8_t>(((tb ? fmode[0] : 3u) << 6) | ((tb ? fmode[1] : 3u) << 4) |
                                          ((tb ? fmode[2] : 3u) << 2));
            if (B.role & kZrTables)
                for (uint32_t t = 0; t < 3u; t++)
                    for (uint32_t i = 0; i < fdlen[t]; i++) R[o++] = fdesc[t][i];
        }
    }
    if (w0)
        a.seglen[b * 64u + lane] = lane != lead || B.raw == 0u ? 0u : (B.role & kZrCoded) ? 3u + B.body : (kStored | B.raw);
    __syncthreads();
    KCDC_ZSTAMP(9);
}

// One wave per span: blockIdx.x = global span index.  FMT: kFmtDeflate or kFmtS2 (the parse is
// shared; the emitters differ: fixed-Huffman bits closed by a sync flush, or Snappy tags).
template <int FMT>
__global__ __launch_bounds__(64) void lz_spans_kernel(CompArgs a) {
    __shared__ uint32_t L[kLdsWords];
    __shared__ uint16_t tab[(1u << kHashBits) * 64u];
    __shared__ uint32_t ftab[1u << kFirstBits];
    __shared__ uint32_t hist[FMT == kFmtDeflate ? kNSym : 1];  // deflate: the span's symbol counts
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    const uint32_t c = span_chunk(a, b);
    const uint32_t u = b - a.spans[c];
    const uint64_t len = a.in_lens[c];
    const uint64_t sb = static_cast<uint64_t>(u) * kSpan;
    const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
#ifdef KCDC_TRACE
    if (FMT == kFmtDeflate) KCDC_DSTAMP(0);
#endif
    // Stage [A0, A0 + 16 ng) with A0 = A & ~15: every 16-byte granule holds a byte of the span.
    const uint32_t d = stage_span(L, a.in + a.in_offs[c] + sb, span_len, lane);
    {
        uint64_t* t64 = reinterpret_cast<uint64_t*>(tab);
        for (uint32_t i = lane; i < (1u << kHashBits) * 16u; i += 64u) t64[i] = ~0ull;
        for (uint32_t i = lane; i < (1u << kFirstBits); i += 64u) ftab[i] = ~0u;
        if constexpr (FMT == kFmtDeflate)
            for (uint32_t i = lane; i < kNSym; i += 64u) hist[i] = 0u;
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
    constexpr uint32_t kMul = 0x1E35A7BDu;
    if (a.effort >= 1u) {  // every position's 4-byte hash: the span's first occurrence (LDS atomic min)
        const uint32_t e = span_len >= 3u ? span_len - 3u : 0u;
        for (uint32_t x = x0; x < x0 + kSeg && x < e; x++)
            atomicMin(&ftab[(ld32(x) * kMul) >> (32u - kFirstBits)], x);
        __syncthreads();
    }
    uint32_t word = 0;  // the segment's length word (0: past the span's end)
    uint32_t nm = 0;    // deflate: the segment's match tokens; zstd: its sequences
    if (x0 < span_len) word = [&]() -> uint32_t {
    const uint32_t xe = span_len - x0 < kSeg ? span_len : x0 + kSeg;
    const uint32_t seg_len = xe - x0;
    uint32_t* base = reinterpret_cast<uint32_t*>(a.slots + static_cast<uint64_t>(slot) * kSlot);
    const uint32_t limit = seg_len + 8u;  // bytes flushed before giving up on the segment
    // zstd: block header at bytes 3..5, Raw literals header at 6..7, the literals from byte 8; the
    // sequences (4 bytes each) are kept from the slot's end downwards (8 + literals + 4 sequences
    // <= 8 + seg_len: a sequence covers >= 4 input bytes, so the two never meet).
    Bits w{0ull, 0u, FMT == kFmtZstd ? base + 2 : base};
    bool over = false;
    uint32_t nseq = 0;
    uint32_t fb = 3;  // deflate: the segment's size as one fixed-code block (bits), the stored/coded test
    uint32_t x = x0, lit = x0;
    auto literals = [&](uint32_t e) {
        if constexpr (FMT == kFmtZstd)
            if (a.effort >= 1u) return;  // zstd_emit_kernel takes the literals from the input
        if constexpr (FMT == kFmtS2) {  // one literal element: tag (n-1) << 2 | 0, 60: +1 byte, 61: +2
            if (e == lit) return;
            const uint32_t m = e - lit - 1u;
            if (m < 60u) {
                w.put(m << 2, 8);
            } else if (m < 256u) {
                w.put(60u << 2, 8);
                w.put(m, 8);
            } else {
                w.put(61u << 2, 8);
                w.put(m, 16);
            }
        }
        if constexpr (FMT == kFmtDeflate) {
            for (uint32_t q = lit; q < e; q++) fb += byte(q) < 144u ? 8u : 9u;
            over = fb > 8u * limit;
            return;
        }
        for (uint32_t q = lit; q < e; q++) {
            w.put(byte(q), 8);
            if (4u * static_cast<uint32_t>(w.op - base) > limit) {
                over = true;
                break;
            }
        }
    };
    // S2 copies (Snappy tags, no S2 repeat codes): copy1 for lengths 4..11 at offsets < 2048,
    // else copy2 (lengths 1..64, 16-bit offsets: a span is 32 KiB); longer matches are split.
    auto s2_copy = [&](uint32_t n, uint32_t off) {
        while (n > 0u) {
            const uint32_t k = n > 64u ? (n - 64u < 4u ? 60u : 64u) : n;  // keep the rest >= 4
            if (k >= 4u && k <= 11u && off < 2048u) {
                w.put(1u | ((k - 4u) << 2) | ((off >> 8) << 5), 8);
                w.put(off & 255u, 8);
            } else {
                w.put(2u | ((k - 1u) << 2), 8);
                w.put(off, 16);
            }
            n -= k;
        }
    };
    // Length of the match of x against an earlier q (>= 4 when the first 4 bytes agree), <= maxlen.
    auto match_len = [&](uint32_t q, uint32_t xx, uint32_t v) -> uint32_t {
        if (q >= xx || ld32(q) != v) return 0u;
        const uint32_t cap = FMT == kFmtDeflate ? 258u : kSeg;  // S2 copies and zstd matches: the segment
        const uint32_t maxlen = xe - xx < cap ? xe - xx : cap;
        uint32_t n = 4;
        while (n + 4u <= maxlen) {
            const uint32_t diff = ld32(xx + n) ^ ld32(q + n);
            if (diff) return n + (static_cast<uint32_t>(__builtin_ctz(diff)) >> 3);
            n += 4u;
        }
        while (n < maxlen && byte(xx + n) == byte(q + n)) n++;
        return n;
    };
    // Best match at xx: the lane table's latest candidate (inside the segment) and, with effort
    // >= 1, the span's first occurrence (anywhere earlier in the span), the previous lanes' latest
    // entries and the previous match's distance (a repeat candidate, zstd's repcode idea: periodic
    // and structured data repeat their distances).  Among equally long matches the nearest wins
    // (fewer distance extra bits).  Updates the lane table.
    uint32_t last_d = 0;  // the previous match's distance (0: none yet)
    auto best_at = [&](uint32_t xx, uint32_t& q) -> uint32_t {
        const uint32_t v = ld32(xx);
        const uint32_t hv = v * kMul;
        const uint32_t h = hv >> (32u - kHashBits);
        const uint32_t c1 = tab[h * 64u + lane];
        tab[h * 64u + lane] = static_cast<uint16_t>(xx);
        uint32_t n = 0;
        q = c1;
        // effort >= 1: the repeat distance first (periodic data: nearest, and usually full length)
        if (a.effort >= 1u && last_d && last_d <= xx) {
            n = match_len(xx - last_d, xx, v);
            if (n) q = xx - last_d;
        }
        if (c1 >= x0 && (n == 0u || c1 != q)) {
            const uint32_t m = match_len(c1, xx, v);
            if (m > n || (m == n && m && c1 > q)) {
                n = m;
                q = c1;
            }
        }
        if (a.effort >= 1u) {
            // candidates nearest first; none is tried once a match reaches the longest possible
            const uint32_t full = min(xe - xx, FMT == kFmtDeflate ? 258u : kSeg);
            auto offer = [&](uint32_t c) {  // longer, or as long and nearer
                if (n >= full) return;
                const uint32_t m = match_len(c, xx, v);
                if (m > n || (m == n && m && c > q)) {
                    n = m;
                    q = c;
                }
            };
            // a segment's first position: its own table is empty, so probe the 32 nearest
            // distances (a period up to 32 then costs its distance, not one to a far occurrence);
            // the 32 bytes before it are read once and compared from registers
            if (xx == x0 && xx >= 32u && n < full) {
                uint32_t w[9];
#pragma unroll
                for (int i = 0; i < 9; i++) w[i] = ld32(xx - 32u + 4u * i);  // bytes xx-32 .. xx+3
                uint32_t kmin = 0;  // the nearest distance whose 4 bytes agree (then one match_len)
#pragma unroll
                for (uint32_t k = 32; k >= 1u; k--) {
                    const uint32_t o = 32u - k;  // byte offset of xx - k in w
                    const uint32_t cv = (o & 3u) ? __builtin_amdgcn_alignbit(w[(o >> 2) + 1], w[o >> 2], 8u * (o & 3u))
                                                 : w[o >> 2];
                    kmin = cv == v ? k : kmin;
                }
                if (kmin) offer(xx - kmin);
            }
            // the latest candidates of the three previous segments (their lanes' tables: any entry
            // is an earlier position of this hash, whatever those lanes have reached; a host model
            // of the parse on the mixed bench data: 1 segment back -0.7 % bytes, 3 back -1.4 %)
            for (uint32_t k = 1; k <= 3u && k <= lane; k++) {
                const uint32_t c3 = tab[h * 64u + lane - k];
                if (c3 != 0xFFFFu && c3 != q) offer(c3);
            }
            const uint32_t c2 = ftab[hv >> (32u - kFirstBits)];  // the span's first occurrence: farthest
            if (c2 != c1) offer(c2);
        }
        return n;
    };
    while (!over && x + 4u <= xe) {
        uint32_t cand;
        uint32_t n = best_at(x, cand);
        // lazy: a longer match one byte later wins (default: for matches under 8 bytes, the short
        // word repeats of text; best-compression: under 32)
        if (n && a.effort >= 1u && n < (a.effort >= 2u ? 32u : 8u) && x + 5u <= xe) {
            uint32_t c2;
            const uint32_t n2 = best_at(x + 1u, c2);
            if (n2 > n + 1u) {
                x += 1u;
                n = n2;
                cand = c2;
            }
        }
        if (n) {
            literals(x);
            if (over) break;
            if constexpr (FMT == kFmtS2) {
                s2_copy(n, x - cand);
            } else if constexpr (FMT == kFmtZstd) {  // (literal length, match length - 4, offset)
                base[143u - nseq] = zseq_word(x - lit, n, x - cand);
                nseq++;
            } else {  // deflate token; the fixed code's cost
                base[nm++] = ((x - lit) << 23) | ((n - 3u) << 15) | (x - cand - 1u);
                const MatchSyms m = match_syms(n, x - cand);
                fb += (m.ls < 280u ? 7u : 8u) + m.eb + 5u + m.deb;
                if (fb > 8u * limit) over = true;
            }
            if (4u * static_cast<uint32_t>(w.op - base) > limit) {
                over = true;
                break;
            }
            last_d = x - cand;
            x += n;
            lit = x;
        } else {
            x += 1u + ((x - lit) >> a.skip);
        }
    }
    if constexpr (FMT == kFmtZstd) {
        if (a.effort >= 1u) {  // zstd_emit_kernel codes the span (the sequences stay in the slot)
            nm = nseq;
            return seg_len;
        }
        if (!over) literals(xe);  // the block's last literals (no sequence)
        if (over) return kStored | seg_len;
        const uint32_t nlit = 4u * static_cast<uint32_t>(w.op - (base + 2)) + (w.nb >> 3);
        if (w.nb) *w.op = static_cast<uint32_t>(w.bb);
        uint8_t* sb8 = reinterpret_cast<uint8_t*>(base);
        // zstd-fastest: one block per segment, the sequences section after the raw literals
        const uint32_t qs = zstd_seqs(sb8, 8u + nlit, nseq, seg_len, true);
        if (qs == kZOver) return kStored | seg_len;
        const uint32_t total = 5u + nlit + qs;  // block header + literals section + sequences section
        if (total >= seg_len + kZStoredHdr) return kStored | seg_len;
        const uint32_t hdr = ((total - 3u) << 3) | (2u << 1);  // Compressed_Block, not the last
        sb8[3] = static_cast<uint8_t>(hdr);
        sb8[4] = static_cast<uint8_t>(hdr >> 8);
        sb8[5] = static_cast<uint8_t>(hdr >> 16);
        sb8[6] = static_cast<uint8_t>(0x04u | ((nlit & 15u) << 4));  // Raw_Literals_Block, 2-byte size
        sb8[7] = static_cast<uint8_t>(nlit >> 4);
        return total;
    }
    if constexpr (FMT == kFmtS2) {
        if (!over) {  // exact size with the pending literal: worse than one stored literal -> stored
            const uint32_t m = xe - lit;
            const uint32_t bytes = 4u * static_cast<uint32_t>(w.op - base) + (w.nb >> 3) + m +
                                   (m == 0u ? 0u : m <= 60u ? 1u : m <= 256u ? 2u : 3u);
            if (bytes >= seg_len + kS2StoredHdr) over = true;
        }
        if (!over) literals(xe);
        uint32_t bytes = 0;
        if (!over) {
            bytes = 4u * static_cast<uint32_t>(w.op - base) + (w.nb >> 3);
            if (w.nb) *w.op = static_cast<uint32_t>(w.bb);
            if (bytes >= seg_len + kS2StoredHdr) over = true;
        }
        return over ? (kStored | seg_len) : bytes;
    }
    if (!over) {
        // The block's size with the pending literals, counted 4 bytes at a time (a fixed literal
        // is 8 bits, 9 from 0x90): a segment that would not beat a stored copy (random data) is
        // stored; the others share the span's code (deflate_plan).
        uint32_t a0 = lit, nine = 0;
        for (; a0 < xe && ((a0 + d) & 3u); a0++) nine += byte(a0) >= 144u;
        for (; a0 + 4u <= xe; a0 += 4u) {
            const uint32_t v = L[pw((a0 + d) >> 2)];
            nine += __builtin_popcount(v & 0x80808080u & ((v << 1) | (v << 2) | (v << 3)));
        }
        for (; a0 < xe; a0++) nine += byte(a0) >= 144u;
        const uint32_t bits = fb + 8u * (xe - lit) + nine + 10u;
        if (((bits + 7u) >> 3) + 4u >= seg_len + 5u) over = true;
    }
    return over ? (kStored | seg_len) : seg_len;
    }();
    if constexpr (FMT == kFmtDeflate) {
#ifdef KCDC_TRACE
        __syncthreads();
        KCDC_DSTAMP(1);
#endif
        deflate_plan(a, b, lane, span_len, x0, word, nm, hist, reinterpret_cast<uint32_t*>(tab), L, d);
#ifdef KCDC_TRACE
        __syncthreads();
        KCDC_DSTAMP(6);
#endif
        return;
    }
    if constexpr (FMT == kFmtZstd)
        if (a.effort >= 1u) {
            a.desc[static_cast<uint64_t>(b) * kDescWords + lane] = nm;
            return;
        }
    a.seglen[slot] = word;
    // The span's output bytes (stored segments: 5 + n, S2: 3 + n; S2 adds the framing header).
    const uint32_t shdr = FMT == kFmtS2 ? kS2StoredHdr : FMT == kFmtZstd ? kZStoredHdr : 5u;
    uint32_t eff = (word & kStored) ? shdr + (word & ~kStored) : word;
    for (uint32_t o = 32; o > 0; o >>= 1) eff += __shfl_xor(eff, o, 64);
    if (FMT == kFmtS2) eff += kS2ChunkHdr + uvarint_len(span_len);
    if (lane == 0) a.span_bytes[b] = eff;
}

// Exclusive prefix (64-bit) of span_bytes[0..total) into span_pos[0..total]; one workgroup.
__global__ __launch_bounds__(1024) void span_pos_kernel(CompArgs a) {
    __shared__ uint64_t part[1024];
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans) return;
    const uint32_t t = threadIdx.x;
    const uint64_t b = static_cast<uint64_t>(total) * t / 1024u, e = static_cast<uint64_t>(total) * (t + 1) / 1024u;
    uint64_t s = 0;
    for (uint64_t i = b; i < e; i++) s += a.span_bytes[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0ull;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - s;
    for (uint64_t i = b; i < e; i++) {
        a.span_pos[i] = run;
        run += a.span_bytes[i];
    }
    if (t == 1023u) a.span_pos[total] = part[1023];
}

// ------------------------------------------------------------------ CRC-32 (gzip trailer)
// crc32(A || B) = crc32(A) * x^(8|B|) ^ crc32(B) in GF(2)[x] / P (zlib's crc32_combine), and the
// raw CRC (register 0, no final XOR) ignores leading zero bytes.  So a chunk is cut into 32 KiB
// spans counted back from its END (bytes before the chunk read as zeros), one wave per span,
// 512 bytes per lane; lanes combine in a 6-level tree with the constants x^(2^(12+j)), the span
// is scaled by x^(8 * 32768 * spans after it), and the chunk's word takes the XOR (atomic, order
// free).  The frame kernel adds crc32 of len zero bytes (the init / final-XOR terms).
constexpr uint32_t kCrcPoly = 0xEDB88320u;   // CRC-32 (gzip), reflected
constexpr uint32_t kCrc32cPoly = 0x82F63B78u; // CRC-32C (Castagnoli: the S2 / Snappy framing), reflected
__host__ __device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly = kCrcPoly) {
    uint32_t p = 0;  // a * b mod P (reflected)
    for (int i = 31; i >= 0; i--) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b >> 1) ^ (poly & (0u - (b & 1u)));
    }
    return p;
}

// S2 = false: gzip's CRC-32 of each chunk, its 32 KiB spans counted back from the chunk's end.
// S2 = true: the CRC-32C of each S2 span on its own (a framing chunk's checksum), lanes counted
// back from the span's end; raw register value to span_crc[b].
constexpr uint32_t kCrcWaves = 4;
template <bool S2>
__global__ __launch_bounds__(64 * kCrcWaves) void crc_spans_kernel(CompArgs a) {
    constexpr uint32_t poly = S2 ? kCrc32cPoly : kCrcPoly;
    __shared__ uint32_t tab[256 * 32];  // 32 copies: lane l reads copy l & 31 (conflict free)
    for (uint32_t x = threadIdx.x; x < 256u; x += 64u * kCrcWaves) {
        uint32_t r = x;
        for (int k = 0; k < 8; k++) r = (r >> 1) ^ (poly & (0u - (r & 1u)));
        for (uint32_t c = 0; c < 32u; c++) tab[32u * x + ((c + x) & 31u)] = r;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t b = blockIdx.x * kCrcWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    uint32_t lo = 0, hi = a.n;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.spans[mid] <= b) lo = mid; else hi = mid;
    }
    const uint32_t c = lo;
    const uint32_t s = b - a.spans[c], ns = a.spans[c + 1] - a.spans[c];
    int64_t len = static_cast<int64_t>(a.in_lens[c]);
    int64_t p0 = len - static_cast<int64_t>(kSpan) * (ns - s) + static_cast<int64_t>(kSeg) * lane;
    const uint8_t* in = a.in + a.in_offs[c];
    if (S2) {  // the span alone: [s kSpan, s kSpan + span_len) as a message of its own
        const int64_t sb = static_cast<int64_t>(s) * kSpan;
        len = len - sb < static_cast<int64_t>(kSpan) ? len - sb : static_cast<int64_t>(kSpan);
        in += sb;
        p0 = len - static_cast<int64_t>(kSpan) + static_cast<int64_t>(kSeg) * lane;
    }
    // 16-byte granules from the aligned address below the segment; m16 is wave-uniform (lanes
    // are 512 bytes apart).  A granule is read only when it holds a byte of the chunk.
    const uint32_t m16 = static_cast<uint32_t>((reinterpret_cast<uintptr_t>(in) + static_cast<uint64_t>(p0 & 15)) & 15u);
    const uint8_t* gb = in + p0 - m16;
    auto granule = [&](int64_t g) -> uint4 {
        const int64_t o = p0 - static_cast<int64_t>(m16) + 16 * g;
        return (o + 16 > 0 && o < len) ? *reinterpret_cast<const uint4*>(gb + 16 * g) : make_uint4(0u, 0u, 0u, 0u);
    };
    const uint32_t q4 = m16 >> 2, sh = 8u * (m16 & 3u);
    const uint32_t sel = lane & 31u;
    uint32_t r = 0;
    uint4 cur = granule(0);
    for (int j = 0; j < static_cast<int>(kSeg / 16u); j++) {
        const uint4 nxt = granule(j + 1);
        const uint32_t c8[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
        uint32_t w4[4];
        // words q4 .. q4 + 4 of the pair, shifted by sh bits (q4 uniform: one branch)
        if (q4 == 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) w4[i] = __builtin_amdgcn_alignbit(c8[i + 1], c8[i], sh);
        } else if (q4 == 1) {
#pragma unroll
            for (int i = 0; i < 4; i++) w4[i] = __builtin_amdgcn_alignbit(c8[i + 2], c8[i + 1], sh);
        } else if (q4 == 2) {
#pragma unroll
            for (int i = 0; i < 4; i++) w4[i] = __builtin_amdgcn_alignbit(c8[i + 3], c8[i + 2], sh);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) w4[i] = __builtin_amdgcn_alignbit(c8[i + 4], c8[i + 3], sh);
        }
        cur = nxt;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t pos = p0 + 16 * j + 4 * i;  // bytes before the chunk read as 0
            uint32_t w = w4[i];
            if (pos < 0) w = pos <= -4 ? 0u : (w & (0xFFFFFFFFu << (8u * static_cast<uint32_t>(-pos))));
            r ^= w;
#pragma unroll
            for (int t = 0; t < 4; t++) r = (r >> 8) ^ tab[32u * (r & 255u) + sel];
        }
    }
    // lanes 2i, 2i+1, ...: left * x^(8 * right bytes) ^ right, right = 512 * 2^j bytes
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const uint32_t right = __shfl_down(r, 1u << j, 64);
        if (((lane >> j) & 1u) == 0u) r = multmodp(r, S2 ? a.x2nc[12 + j] : a.x2n[12 + j], poly) ^ right;
    }
    if (S2) {
        if (lane == 0) a.span_crc[b] = r;
        return;
    }
    if (lane == 0) {
        uint32_t after = ns - 1u - s;  // whole spans after this one: x^(8 * 32768 * after)
        for (int bit = 0; after; bit++, after >>= 1)
            if (after & 1u) r = multmodp(r, a.x2n[18 + bit]);
        atomicXor(&a.crc[c], r);
    }
}

// n bytes from src to dst, both at any alignment, by one wave: byte stores for dst's partial
// head and tail words, aligned dword stores (from two aligned loads + alignbit) in between.
// Only aligned source words holding a byte of [src, src + n) are read.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane) {
    const uint32_t head = min(n, static_cast<uint32_t>((4u - (reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u));
    if (lane < head) dst[lane] = src[lane];
    const uint32_t m = (n - head) >> 2;
    uint32_t* __restrict__ dw = reinterpret_cast<uint32_t*>(dst + head);
    const uint8_t* s0 = src + head;
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(s0) & 3u);
    const uint32_t* __restrict__ sw = reinterpret_cast<const uint32_t*>(s0 - sh);
    // 8 words per lane in flight per round (loads first, then stores): one dependent load per
    // 256 bytes left a copy latency-bound at the emit kernel's two waves per CU
    constexpr uint32_t kU = 8;
    uint32_t i = lane;
    for (; i + 64u * (kU - 1u) < m; i += 64u * kU) {
        uint32_t w0[kU], w1[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            w0[u] = sw[i + 64u * u];
            w1[u] = sh ? sw[i + 64u * u + 1u] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) dw[i + 64u * u] = __builtin_amdgcn_alignbit(w1[u], w0[u], 8u * sh);
    }
    for (; i < m; i += 64u) {
        const uint32_t w0 = sw[i];
        const uint32_t w1 = sh ? sw[i + 1] : 0u;
        dw[i] = __builtin_amdgcn_alignbit(w1, w0, 8u * sh);
    }
    const uint32_t done = head + 4u * m;
    if (lane < n - done) dst[done + lane] = src[done + lane];
}

// Zstandard frame header of a chunk of `len` bytes (RFC 8878 §3.1.1.1): magic, Frame_Header_Descriptor
// with Single_Segment_flag (the window is the content) and the smallest Frame_Content_Size field;
// no checksum, no dictionary.  Returns its size; writes it when dst is set.
__device__ __forceinline__ uint32_t zstd_frame_header(uint64_t len, uint8_t* dst) {
    const uint32_t fcs = len < 256u ? 1u : len < 65536u + 256u ? 2u : len < (1ull << 32) ? 4u : 8u;
    if (dst) {
        const uint8_t magic[4] = {0x28u, 0xB5u, 0x2Fu, 0xFDu};
        for (int i = 0; i < 4; i++) dst[i] = magic[i];
        const uint32_t flag = fcs == 1u ? 0u : fcs == 2u ? 1u : fcs == 4u ? 2u : 3u;
        dst[4] = static_cast<uint8_t>((flag << 6) | 0x20u);
        const uint64_t v = fcs == 2u ? len - 256u : len;
        for (uint32_t i = 0; i < fcs; i++) dst[5 + i] = static_cast<uint8_t>(v >> (8u * i));
    }
    return 5u + fcs;
}

// One wave per span: its segments' bytes to their places in the chunk's stream.
__global__ __launch_bounds__(64) void deflate_copy_kernel(CompArgs a) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    uint32_t lo = 0, hi = a.n;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.spans[mid] <= b) lo = mid; else hi = mid;
    }
    const uint32_t c = lo;
    const uint32_t u = b - a.spans[c];
    uint8_t* dst = a.out + a.out_offs[c] + 4u + (a.gzip ? 10u : 0u) + (a.fmt == kFmtS2 ? kS2StreamId : 0u) +
                   (a.fmt == kFmtZstd ? zstd_frame_header(a.in_lens[c], nullptr) : 0u) +
                   (a.span_pos[b] - a.span_pos[a.spans[c]]);
    const uint8_t* in = a.in + a.in_offs[c] + static_cast<uint64_t>(u) * kSpan;
    const uint32_t word = a.seglen[b * 64u + lane];
    const bool s2 = a.fmt == kFmtS2, zs = a.fmt == kFmtZstd;
    const uint32_t eff = (word & kStored) ? (s2 ? kS2StoredHdr : zs ? kZStoredHdr : 5u) + (word & ~kStored) : word;
    if (s2) {  // framing chunk header: 0x00, length, masked CRC-32C of the span, uvarint(span length)
        const uint64_t len = a.in_lens[c], sb = static_cast<uint64_t>(u) * kSpan;
        const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
        const uint32_t vl = uvarint_len(span_len);
        if (lane == 0) {
            const uint32_t clen = a.span_bytes[b] - 4u;  // CRC + block
            uint32_t z = 0x80000000u;  // standard CRC-32C = raw ^ (~0 x^(8 n) mod P) ^ ~0
            for (uint32_t n = span_len, bit = 0; n; bit++, n >>= 1)
                if (n & 1u) z = multmodp(z, a.x2nc[(3 + bit) & 31], kCrc32cPoly);
            const uint32_t crc = a.span_crc[b] ^ multmodp(z, 0xFFFFFFFFu, kCrc32cPoly) ^ 0xFFFFFFFFu;
            const uint32_t masked = ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
            uint8_t h[11] = {0x00u, static_cast<uint8_t>(clen), static_cast<uint8_t>(clen >> 8),
                             static_cast<uint8_t>(clen >> 16), static_cast<uint8_t>(masked),
                             static_cast<uint8_t>(masked >> 8), static_cast<uint8_t>(masked >> 16),
                             static_cast<uint8_t>(masked >> 24), 0u, 0u, 0u};
            uint32_t v = span_len;
            for (uint32_t i = 0; i < vl; i++, v >>= 7) h[8 + i] = static_cast<uint8_t>((v & 127u) | (i + 1 < vl ? 128u : 0u));
            for (uint32_t i = 0; i < 8u + vl; i++) dst[i] = h[i];
        }
        dst += kS2ChunkHdr + vl;
    }
    uint32_t incl = eff;
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const uint32_t pos = incl - eff;
    for (uint32_t j = 0; j < 64u; j++) {
        const uint32_t wj = __shfl(word, j, 64), pj = __shfl(pos, j, 64);
        if (wj == 0u) continue;  // past the chunk's end, or inside a zstd block of segments
        uint8_t* o = dst + pj;
        if ((wj & kStored) && zs) {  // Raw_Block: header (size << 3 | 0), then the bytes
            const uint32_t m = wj & ~kStored;
            if (lane < kZStoredHdr) o[lane] = static_cast<uint8_t>((m << 3) >> (8u * lane));
            wave_copy(o + kZStoredHdr, in + j * kSeg, m, lane);
        } else if ((wj & kStored) && s2) {  // one literal: tag 61 (length - 1 in 2 bytes)
            const uint32_t m = wj & ~kStored;
            if (lane < kS2StoredHdr)
                o[lane] = static_cast<uint8_t>(lane == 0 ? 61u << 2 : lane == 1 ? ((m - 1u) & 255u) : ((m - 1u) >> 8));
            wave_copy(o + kS2StoredHdr, in + j * kSeg, m, lane);
        } else if (wj & kStored) {
            const uint32_t m = wj & ~kStored;
            if (lane < 5u) {
                const uint32_t hdr = lane == 0 ? 0u : lane == 1 ? (m & 255u) : lane == 2 ? (m >> 8)
                                   : lane == 3 ? (~m & 255u) : ((~m >> 8) & 255u);
                o[lane] = static_cast<uint8_t>(hdr);  // stored block: BFINAL 0, BTYPE 00, LEN, NLEN
            }
            wave_copy(o + 5, in + j * kSeg, m, lane);
        } else {
            wave_copy(o, a.slots + (static_cast<uint64_t>(b) * 64u + j) * kSlot + (zs ? kZOff : 0u), wj, lane);
        }
    }
}

// One wave per span (deflate, gzip, pgzip): the span's blocks as its plan says (deflate_plan),
// assembled in LDS (segments OR their bits in from their bit offsets), then copied to the
// chunk's stream.  A stored span is copied from the input directly.
constexpr uint32_t kOutWords = 8200;  // >= (32768 + 4) / 4 + 2: a coded span is smaller than stored
__global__ __launch_bounds__(64) void deflate_emit_kernel(CompArgs a) {
    __shared__ uint32_t L[kLdsWords];
    __shared__ uint32_t ob[kOutWords];
    __shared__ uint32_t ctab[kNSym];
    __shared__ uint32_t lensw[80];
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    const uint32_t c = span_chunk(a, b);
    const uint32_t u = b - a.spans[c];
    const uint64_t len = a.in_lens[c], sb = static_cast<uint64_t>(u) * kSpan;
    const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
    uint8_t* dst = a.out + a.out_offs[c] + 4u + (a.gzip ? 10u : 0u) + (a.span_pos[b] - a.span_pos[a.spans[c]]);
    const uint8_t* in = a.in + a.in_offs[c] + sb;
    const uint32_t* desc = a.desc + static_cast<uint64_t>(b) * kDescWords;
    const uint32_t mw = desc[kDescMode], mode = mw & 255u, hb = mw >> 8;
    if (mode == kModeStored) return;  // deflate_stored_kernel
    const uint32_t nbytes = a.span_bytes[b];
    const uint32_t d = stage_span(L, in, span_len, lane);
    uint8_t* lens = reinterpret_cast<uint8_t*>(lensw);
    for (uint32_t k = lane; k < 80u; k += 64u) lensw[k] = mode == kModeDynamic ? desc[kDescLens + k] : 0u;
    for (uint32_t k = lane; k < (nbytes + 3u) / 4u + 2u; k += 64u) ob[k] = 0u;
    __syncthreads();
    // The fixed code is canonical over all 288 literal/length symbols (RFC 1951 §3.2.6: 286 and 287
    // take part in the construction though never sent), so its 9-bit literals start at 0x190; the
    // distance lengths then sit at byte 288 (ctab[286..287] are overwritten by the distance codes).
    const uint32_t lit_n = mode == kModeFixed ? kNLit + 2u : kNLit;
    uint8_t* dlens = lens + lit_n;
    if (mode == kModeFixed)
        for (uint32_t s = lane; s < lit_n + kNDist; s += 64u)
            lens[s] = static_cast<uint8_t>(s < lit_n ? (s < kNLit ? fixed_len(s) : 8u) : 5u);
    __syncthreads();
    canon_codes(lens, lit_n, ctab, lane);
    canon_codes(dlens, kNDist, ctab + kNLit, lane);
    __syncthreads();
    const uint32_t x0 = kSeg * lane;
    if (x0 < span_len) {
        const uint32_t xe = span_len - x0 < kSeg ? span_len : x0 + kSeg;
        const uint32_t inf = desc[kDescInfo + lane], bo = desc[kDescOff + lane];
        OrBits w{0ull, bo & 31u, bo >> 5, ob};
        if ((inf & 3u) == kClsCoded) {
            if (inf & 4u) {  // a run's first segment: the block header
                w.put(mode == kModeDynamic ? 4u : 2u, 3);  // BFINAL 0, BTYPE 10 / 01
                if (mode == kModeDynamic) {
                    for (uint32_t k = 0; k < hb / 32u; k++) w.put(desc[kDescHdr + k], 32);
                    if (hb & 31u) w.put(desc[kDescHdr + hb / 32u], hb & 31u);
                }
            }
            const uint32_t* tok = reinterpret_cast<const uint32_t*>(a.slots + (static_cast<uint64_t>(b) * 64u + lane) * kSlot);
            const uint32_t nm = a.seglen[b * 64u + lane];  // the segment's tokens
            walk_tokens(tok, nm, x0, xe,
                        [&](uint32_t x) {
                            const uint32_t cw = ctab[st_byte(L, d, x)];
                            w.put(cw & 0xFFFFu, cw >> 16);
                        },
                        [&](uint32_t, uint32_t n, uint32_t dist) {
                            const MatchSyms m = match_syms(n, dist);
                            const uint32_t cl = ctab[m.ls], cd = ctab[kNLit + m.ds];
                            w.put(cl & 0xFFFFu, cl >> 16);
                            w.put(m.ev, m.eb);
                            w.put(cd & 0xFFFFu, cd >> 16);
                            w.put(m.dev, m.deb);
                        });
            if (inf & 8u) {  // a run's last segment: end of block
                const uint32_t ce = ctab[256];
                w.put(ce & 0xFFFFu, ce >> 16);
            }
            if (inf & 16u) {  // the span's end: an empty stored block (sync flush)
                w.put(0u, 3);
                w.pad();
                w.put(0u, 16);
                w.put(0xFFFFu, 16);
            }
        } else {
            if (inf & 4u) {  // a stored run: BFINAL 0, BTYPE 00, pad, LEN, NLEN
                const uint32_t run = inf >> 16;
                w.put(0u, 3);
                w.pad();
                w.put(run, 16);
                w.put(~run & 0xFFFFu, 16);
            }
            uint32_t x = x0;
            for (; x + 4u <= xe; x += 4u) w.put(st_ld32(L, d, x), 32);
            for (; x < xe; x++) w.put(st_byte(L, d, x), 8);
        }
        w.flush();
    }
    __syncthreads();
    wave_copy(dst, reinterpret_cast<const uint8_t*>(ob), nbytes, lane);
}

// One wave per span whose plan is one stored block (random data): BFINAL 0, BTYPE 00, LEN, NLEN,
// the bytes.  Apart from deflate_emit_kernel, whose 67 KiB of LDS allow two waves per CU: at that
// occupancy the copy of an incompressible batch ran at ~130 GB/s.
__global__ __launch_bounds__(64) void deflate_stored_kernel(CompArgs a) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans || b >= total) return;
    const uint32_t* desc = a.desc + static_cast<uint64_t>(b) * kDescWords;
    if ((desc[kDescMode] & 255u) != kModeStored) return;
    const uint32_t c = span_chunk(a, b);
    const uint32_t u = b - a.spans[c];
    const uint64_t len = a.in_lens[c], sb = static_cast<uint64_t>(u) * kSpan;
    const uint32_t span_len = static_cast<uint32_t>(len - sb < kSpan ? len - sb : kSpan);
    uint8_t* dst = a.out + a.out_offs[c] + 4u + (a.gzip ? 10u : 0u) + (a.span_pos[b] - a.span_pos[a.spans[c]]);
    if (lane < 5u) {
        const uint32_t m = span_len;
        const uint32_t h = lane == 0 ? 0u : lane == 1 ? (m & 255u) : lane == 2 ? (m >> 8)
                         : lane == 3 ? (~m & 255u) : ((~m >> 8) & 255u);
        dst[lane] = static_cast<uint8_t>(h);
    }
    wave_copy(dst + 5, a.in + a.in_offs[c] + sb, span_len, lane);
}

// One thread per chunk: header ID, the empty final block (03 00), the length and the ID kept.
__global__ __launch_bounds__(256) void deflate_frame_kernel(CompArgs a) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    if (c >= a.n) return;
    const uint32_t total = a.spans[a.n];
    if (total > a.max_spans) {  // workspace smaller than the chunks need: no output
        a.out_lens[c] = 0ull;
        a.ids[c] = 0u;
        return;
    }
    uint8_t* dst = a.out + a.out_offs[c];
    const uint64_t body = a.span_pos[a.spans[c + 1]] - a.span_pos[a.spans[c]];
    for (uint32_t t = 0; t < 4u; t++) dst[t] = static_cast<uint8_t>(a.header_id >> (8u * (3u - t)));
    uint64_t out_len;
    if (a.fmt == kFmtZstd) {  // frame header, the segments' blocks, a last empty Raw_Block (01 00 00)
        const uint32_t fh = zstd_frame_header(a.in_lens[c], dst + 4);
        uint8_t* e = dst + 4 + fh + body;
        e[0] = 0x01u;
        e[1] = 0x00u;
        e[2] = 0x00u;
        out_len = 4u + fh + body + 3u;
    } else if (a.fmt == kFmtS2) {  // the stream identifier chunk, then the spans' framing chunks
        const uint8_t id[kS2StreamId] = {0xffu, 6u, 0u, 0u, 'S', '2', 's', 'T', 'w', 'O'};
        for (uint32_t t = 0; t < kS2StreamId; t++) dst[4 + t] = id[t];
        out_len = 4u + kS2StreamId + body;
    } else if (a.gzip) {
        // RFC 1952 member: ID1 ID2 CM=8 FLG=0 MTIME=0 XFL OS=255, the stream, CRC32, ISIZE.  XFL as
        // Go's compress/gzip (and klauspost/pgzip) Writer sets it from the level: 2 for
        // BestCompression, 4 for BestSpeed, else 0 (effort 2 / 0 / 1 here).
        const uint8_t xfl = a.effort == 2u ? 2u : a.effort == 0u ? 4u : 0u;
        const uint8_t gz[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, xfl, 0xff};
        for (uint32_t t = 0; t < 10u; t++) dst[4 + t] = gz[t];
        uint8_t* e = dst + 14 + body;
        e[0] = 0x03u;
        e[1] = 0x00u;
        const uint64_t len = a.in_lens[c];
        uint32_t z = 0x80000000u;  // x^(8 len) mod P = product of x^(2^(3+bit)) over len's bits
        uint64_t n = len;
        for (int bit = 0; n; bit++, n >>= 1)
            if (n & 1u) z = multmodp(z, a.x2n[(3 + bit) & 31]);
        const uint32_t crc = a.crc[c] ^ multmodp(z, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        const uint32_t isize = static_cast<uint32_t>(len);
        for (uint32_t t = 0; t < 4u; t++) {
            e[2 + t] = static_cast<uint8_t>(crc >> (8u * t));
            e[6 + t] = static_cast<uint8_t>(isize >> (8u * t));
        }
        out_len = body + 24u;
    } else {
        dst[4 + body] = 0x03u;  // BFINAL 1, BTYPE 01, end of block
        dst[5 + body] = 0x00u;
        out_len = body + 6u;
    }
    a.out_lens[c] = out_len;
    a.ids[c] = out_len < a.in_lens[c] ? a.header_id : 0u;  // content_manager_lock_free.go:64
}

}  // namespace compdev

namespace {

struct CompAlgo {
    const char* name;
    uint32_t header_id;  // repo/compression/compression_ids.go:8-10, 19-21, 28-30
    uint32_t skip;       // literal-run skip shift: larger = fewer positions skipped
    uint32_t effort;     // match search (CompArgs::effort)
    uint32_t gzip;
    uint32_t fmt = compdev::kFmtDeflate;
};
// compressor_deflate.go:14-16, compressor_gzip.go:15-17, compressor_pgzip.go:16-18 (sorted names).
// pgzip's writer splits its input into independently compressed blocks; gzip and pgzip readers
// accept any valid member, so both families carry the same device stream.  The levels differ in
// search effort: best-speed = the lane's own table; default = + the span's first occurrences, the
// three previous segments' tables and lazy matching of matches under 8 bytes; best-compression =
// lazy matching under 32 bytes and no literal-run skipping to speak of.
constexpr CompAlgo kCompAlgos[] = {
    {"deflate-best-compression", 0x1502u, 8u, 2u, 0u},
    {"deflate-best-speed", 0x1501u, 4u, 0u, 0u},
    {"deflate-default", 0x1500u, 5u, 1u, 0u},
    {"gzip", 0x1000u, 5u, 1u, 1u},
    {"gzip-best-compression", 0x1002u, 8u, 2u, 1u},
    {"gzip-best-speed", 0x1001u, 4u, 0u, 1u},
    {"pgzip", 0x1300u, 5u, 1u, 1u},
    {"pgzip-best-compression", 0x1302u, 8u, 2u, 1u},
    {"pgzip-best-speed", 0x1301u, 4u, 0u, 1u},
    // compressor_s2.go:20-23: s2.NewWriter's stream (framing chunks of Snappy-compatible blocks, which
    // s2.NewReader decodes); the parallel variants differ only in the writer's goroutines.
    {"s2-better", 0x1201u, 8u, 2u, 0u, compdev::kFmtS2},
    {"s2-default", 0x1200u, 5u, 1u, 0u, compdev::kFmtS2},
    {"s2-parallel-4", 0x1202u, 5u, 1u, 0u, compdev::kFmtS2},
    {"s2-parallel-8", 0x1203u, 5u, 1u, 0u, compdev::kFmtS2},
    // compressor_zstd.go:15-18: zstd.NewWriter frames (zstd.NewReader decodes any RFC 8878 frame);
    // zstd-best-compression is registered deprecated (decompression of old data), still encodable.
    {"zstd", 0x1100u, 5u, 1u, 0u, compdev::kFmtZstd},
    {"zstd-best-compression", 0x1103u, 8u, 2u, 0u, compdev::kFmtZstd},
    {"zstd-better-compression", 0x1102u, 8u, 2u, 0u, compdev::kFmtZstd},
    {"zstd-fastest", 0x1101u, 4u, 0u, 0u, compdev::kFmtZstd},
};

const CompAlgo* find_comp(const char* name) {
    if (!name) return nullptr;
    for (const CompAlgo& a : kCompAlgos)
        if (std::strcmp(a.name, name) == 0) return &a;
    return nullptr;
}

uint64_t align256c(uint64_t x) { return (x + 255u) & ~uint64_t(255); }

struct CompWs {
    uint64_t spans, crc, span_crc, seglen, span_bytes, span_pos, slots, desc, total;
};
constexpr uint64_t kPerSpan = 64u * (compdev::kSlot + 4u) + 4u + 4u + 8u + 4u * compdev::kDescWords;
CompWs comp_ws(uint32_t n, uint64_t max_spans) {
    CompWs l{};
    l.spans = 0;
    l.crc = align256c((uint64_t(n) + 1u) * 4u);
    l.span_crc = align256c(l.crc + uint64_t(n) * 4u);
    l.seglen = align256c(l.span_crc + max_spans * 4u);
    l.span_bytes = align256c(l.seglen + max_spans * 64u * 4u);
    l.span_pos = align256c(l.span_bytes + max_spans * 4u);
    l.slots = align256c(l.span_pos + (max_spans + 1u) * 8u);
    l.desc = align256c(l.slots + max_spans * 64u * compdev::kSlot);
    l.total = align256c(l.desc + max_spans * 4u * compdev::kDescWords);
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

extern "C" uint64_t kcdc_compress_bound(uint64_t len) {  // + 18: a gzip member's header and trailer (>= zstd's 13 + 3)
    return 24u + len + 5u * ((len + compdev::kSeg - 1) / compdev::kSeg);
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
    uint64_t max_spans = (work_bytes - fixed) / kPerSpan;
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
    a.span_bytes = reinterpret_cast<uint32_t*>(w + l.span_bytes);
    a.span_pos = reinterpret_cast<uint64_t*>(w + l.span_pos);
    a.slots = w + l.slots;
    a.desc = reinterpret_cast<uint32_t*>(w + l.desc);
    a.n = nchunks;
    a.max_spans = static_cast<uint32_t>(max_spans);
    a.header_id = al->header_id;
    a.skip = al->skip;
    a.effort = al->effort;
    a.gzip = al->gzip;
    a.fmt = al->fmt;
    a.crc = reinterpret_cast<uint32_t*>(w + l.crc);
    a.span_crc = reinterpret_cast<uint32_t*>(w + l.span_crc);
    {
        uint32_t p = 1u << 30, q = 1u << 30;  // x^1
        for (int k = 0; k < 32; k++) {
            a.x2n[k] = p;
            a.x2nc[k] = q;
            p = compdev::multmodp(p, p);
            q = compdev::multmodp(q, q, compdev::kCrc32cPoly);
        }
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compdev::span_count_kernel, dim3((nchunks + 255u) / 256u), dim3(256), 0, st, a);
    hipLaunchKernelGGL(compdev::span_scan_kernel, dim3(1), dim3(1024), 0, st, nchunks, a.spans);
    if (max_spans > 0) {
        const dim3 grid(static_cast<uint32_t>(max_spans));
        const dim3 cgrid(static_cast<uint32_t>((max_spans + compdev::kCrcWaves - 1) / compdev::kCrcWaves));
        if (a.fmt == compdev::kFmtS2) {
            hipLaunchKernelGGL(compdev::lz_spans_kernel<compdev::kFmtS2>, grid, dim3(64), 0, st, a);
            hipLaunchKernelGGL(compdev::crc_spans_kernel<true>, cgrid, dim3(64 * compdev::kCrcWaves), 0, st, a);
        } else if (a.fmt == compdev::kFmtZstd) {
            hipLaunchKernelGGL(compdev::lz_spans_kernel<compdev::kFmtZstd>, grid, dim3(64), 0, st, a);
            if (a.effort >= 1u) hipLaunchKernelGGL(compdev::zstd_emit_kernel, grid, dim3(256), 0, st, a);
        } else {
            hipLaunchKernelGGL(compdev::lz_spans_kernel<compdev::kFmtDeflate>, grid, dim3(64), 0, st, a);
        }
        hipLaunchKernelGGL(compdev::span_pos_kernel, dim3(1), dim3(1024), 0, st, a);
        if (a.fmt == compdev::kFmtDeflate) {
            hipLaunchKernelGGL(compdev::deflate_emit_kernel, grid, dim3(64), 0, st, a);
            hipLaunchKernelGGL(compdev::deflate_stored_kernel, grid, dim3(64), 0, st, a);
        } else
            hipLaunchKernelGGL(compdev::deflate_copy_kernel, grid, dim3(64), 0, st, a);
        if (a.gzip)
            hipLaunchKernelGGL(compdev::crc_spans_kernel<false>, cgrid, dim3(64 * compdev::kCrcWaves), 0, st, a);
    }
    hipLaunchKernelGGL(compdev::deflate_frame_kernel, dim3((nchunks + 255u) / 256u), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("compression kernel launch: ") + hipGetErrorString(e));
}
