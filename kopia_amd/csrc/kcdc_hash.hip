// Keyed BLAKE2 content hashes of many chunks on gfx950.
//
// Kopia names every chunk by a keyed hash of its bytes before it is packed
// (repo/content/content_manager.go:812 -> repo/hashing/hashing.go:78-101):
//   BLAKE2B-256-128  blake2b.New256(secret), digest truncated to 16 bytes (the default,
//                    repo/hashing/hashing.go:51, blake_hashes.go:11)
//   BLAKE2B-256      blake2b.New256(secret), 32 bytes              (blake_hashes.go:12)
//   BLAKE2S-128      blake2s.New128(secret), 16 bytes              (blake_hashes.go:9)
//   BLAKE2S-256      blake2s.New256(secret), 32 bytes              (blake_hashes.go:10)
// The algorithms are RFC 7693 (golang.org/x/crypto/blake2b, blake2s, go.mod of the
// reference; not vendored): the key is padded to one block and hashed first.
//
// A BLAKE2 message is compressed block after block, so one chunk is one sequential chain.
// The kernel gives each chunk one lane (the whole state in VGPRs, rounds fully unrolled)
// and relies on many chunks in flight for throughput; lanes of a wave should get chunks of
// similar length (d_order, e.g. by descending length), since a wave runs until its longest
// chunk is done.  DESIGN.md §2.5 has the arithmetic.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>

#include "kcdc_internal.h"

namespace kcdc {
namespace hashdev {

struct HashKey {
    uint32_t w[16];  // key bytes, little-endian words, zero padded (one BLAKE2b block = 128 B)
    uint32_t kk;     // key length in bytes
};

// Message permutations (RFC 7693 §2.7), compile-time constants: the unrolled rounds index registers.
constexpr uint8_t kSig[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

constexpr uint64_t kIV64[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                               0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                               0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
constexpr uint32_t kIV32[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

// 64-bit rotate right by a constant on the two 32-bit halves: two independent v_alignbit (a
// rotate by 32 is a register swap); the shift-or form compiled to ~5 dependent instructions.
template <int N>
__device__ __forceinline__ uint64_t rotr64(uint64_t x) {
    const uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32);
    uint32_t nlo, nhi;
    if constexpr (N == 32) {
        nlo = hi;
        nhi = lo;
    } else if constexpr (N < 32) {
        nlo = __builtin_amdgcn_alignbit(hi, lo, N);
        nhi = __builtin_amdgcn_alignbit(lo, hi, N);
    } else {
        nlo = __builtin_amdgcn_alignbit(lo, hi, N - 32);
        nhi = __builtin_amdgcn_alignbit(hi, lo, N - 32);
    }
    return (static_cast<uint64_t>(nhi) << 32) | nlo;
}
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

// Words [0, nw) of the block at p (take valid bytes, the rest zero), from 4-byte-aligned
// loads that never leave the chunk's aligned words (a chunk may start at any byte).
template <int NW>
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t take, uint32_t (&d)[NW]) {
    if (take == 0) {  // the empty message's one block: nothing to read
#pragma unroll
        for (int i = 0; i < NW; i++) d[i] = 0;
        return;
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t mis = static_cast<uint32_t>(a & 3u);
    const __attribute__((address_space(1))) uint32_t* w =
        reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(a - mis);  // global, not flat
    // Word i loads from min(i, last word holding a block byte): no branches (a guarded load
    // per word became 17-33 divergent branches per block), and never past the chunk's last
    // aligned word (allocations end on 4-byte boundaries).  Excess words are masked below.
    const uint32_t lw = (take + mis - 1) >> 2;
    uint32_t x[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; i++) x[i] = w[min(static_cast<uint32_t>(i), lw)];
#pragma unroll
    for (int i = 0; i < NW; i++) d[i] = mis ? __builtin_amdgcn_alignbit(x[i + 1], x[i], 8 * mis) : x[i];
    if (take < 4u * NW) {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const int32_t keep = static_cast<int32_t>(take) - 4 * i;  // valid bytes of word i
            d[i] &= keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * keep));
        }
    }
}

// ------------------------------------------------------------------ BLAKE2b
__device__ __forceinline__ void g64(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t x, uint64_t y) {
    a = a + b + x;
    d = rotr64<32>(d ^ a);
    c = c + d;
    b = rotr64<24>(b ^ c);
    a = a + b + y;
    d = rotr64<16>(d ^ a);
    c = c + d;
    b = rotr64<63>(b ^ c);
}

__device__ __forceinline__ void compress64(uint64_t (&h)[8], const uint32_t (&mw)[32], uint64_t t, bool last) {
    uint64_t m[16], v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = static_cast<uint64_t>(mw[2 * i]) | (static_cast<uint64_t>(mw[2 * i + 1]) << 32);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        v[i] = h[i];
        v[i + 8] = kIV64[i];
    }
    v[12] ^= t;  // the counter's high word is 0: chunks are < 2^64 bytes
    if (last) v[14] = ~v[14];
#pragma unroll
    for (int r = 0; r < 12; r++) {
        g64(v[0], v[4], v[8], v[12], m[kSig[r][0]], m[kSig[r][1]]);
        g64(v[1], v[5], v[9], v[13], m[kSig[r][2]], m[kSig[r][3]]);
        g64(v[2], v[6], v[10], v[14], m[kSig[r][4]], m[kSig[r][5]]);
        g64(v[3], v[7], v[11], v[15], m[kSig[r][6]], m[kSig[r][7]]);
        g64(v[0], v[5], v[10], v[15], m[kSig[r][8]], m[kSig[r][9]]);
        g64(v[1], v[6], v[11], v[12], m[kSig[r][10]], m[kSig[r][11]]);
        g64(v[2], v[7], v[8], v[13], m[kSig[r][12]], m[kSig[r][13]]);
        g64(v[3], v[4], v[9], v[14], m[kSig[r][14]], m[kSig[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

__global__ __launch_bounds__(256) void blake2b_chunks_kernel(const uint8_t* data, const uint64_t* offs,
                                                             const uint64_t* lens, const uint32_t* order, uint32_t n,
                                                             HashKey key, uint32_t nn, uint32_t out_len,
                                                             uint32_t out_stride, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = order ? order[i] : i;
    const uint64_t len = lens[c];
    const uint8_t* p = data + offs[c];
    uint64_t h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = kIV64[j];
    h[0] ^= 0x01010000ull ^ (static_cast<uint64_t>(key.kk) << 8) ^ nn;
    uint64_t t = 0;
    if (key.kk) {  // the key, zero padded, is the first block (RFC 7693 §3.3)
        uint32_t kb[32];
#pragma unroll
        for (int j = 0; j < 32; j++) kb[j] = j < 16 ? key.w[j] : 0u;
        t = 128;
        compress64(h, kb, t, len == 0);
    }
    const uint64_t nblk = len ? (len + 127) / 128 : (key.kk ? 0 : 1);
    // Block b+1's loads are issued before block b is compressed: one block of compression
    // (~2,500 VALU) hides the memory latency that otherwise every block paid in full.
    auto take_of = [&](uint64_t b) -> uint32_t {
        const uint64_t rem = len - 128 * b;
        return rem < 128 ? static_cast<uint32_t>(rem) : 128u;
    };
    uint32_t cur[32], nxt[32];
    if (nblk) load_block<32>(p, take_of(0), cur);
    for (uint64_t b = 0; b < nblk; b++) {
        if (b + 1 < nblk) load_block<32>(p + 128 * (b + 1), take_of(b + 1), nxt);
        t += take_of(b);
        compress64(h, cur, t, b + 1 == nblk);
#pragma unroll
        for (int j = 0; j < 32; j++) cur[j] = nxt[j];
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if (8u * j < out_len) o[2 * j] = static_cast<uint32_t>(h[j]);
        if (8u * j + 4u < out_len) o[2 * j + 1] = static_cast<uint32_t>(h[j] >> 32);
    }
}

// ------------------------------------------------------------------ BLAKE2s
__device__ __forceinline__ void g32(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
    a = a + b + x;
    d = rotr32(d ^ a, 16);
    c = c + d;
    b = rotr32(b ^ c, 12);
    a = a + b + y;
    d = rotr32(d ^ a, 8);
    c = c + d;
    b = rotr32(b ^ c, 7);
}

__device__ __forceinline__ void compress32(uint32_t (&h)[8], const uint32_t (&m)[16], uint64_t t, bool last) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        v[i] = h[i];
        v[i + 8] = kIV32[i];
    }
    v[12] ^= static_cast<uint32_t>(t);
    v[13] ^= static_cast<uint32_t>(t >> 32);
    if (last) v[14] = ~v[14];
#pragma unroll
    for (int r = 0; r < 10; r++) {
        g32(v[0], v[4], v[8], v[12], m[kSig[r][0]], m[kSig[r][1]]);
        g32(v[1], v[5], v[9], v[13], m[kSig[r][2]], m[kSig[r][3]]);
        g32(v[2], v[6], v[10], v[14], m[kSig[r][4]], m[kSig[r][5]]);
        g32(v[3], v[7], v[11], v[15], m[kSig[r][6]], m[kSig[r][7]]);
        g32(v[0], v[5], v[10], v[15], m[kSig[r][8]], m[kSig[r][9]]);
        g32(v[1], v[6], v[11], v[12], m[kSig[r][10]], m[kSig[r][11]]);
        g32(v[2], v[7], v[8], v[13], m[kSig[r][12]], m[kSig[r][13]]);
        g32(v[3], v[4], v[9], v[14], m[kSig[r][14]], m[kSig[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

__global__ __launch_bounds__(256) void blake2s_chunks_kernel(const uint8_t* data, const uint64_t* offs,
                                                             const uint64_t* lens, const uint32_t* order, uint32_t n,
                                                             HashKey key, uint32_t nn, uint32_t out_len,
                                                             uint32_t out_stride, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = order ? order[i] : i;
    const uint64_t len = lens[c];
    const uint8_t* p = data + offs[c];
    uint32_t h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = kIV32[j];
    h[0] ^= 0x01010000u ^ (key.kk << 8) ^ nn;
    uint64_t t = 0;
    if (key.kk) {
        uint32_t kb[16];
#pragma unroll
        for (int j = 0; j < 16; j++) kb[j] = j < 8 ? key.w[j] : 0u;
        t = 64;
        compress32(h, kb, t, len == 0);
    }
    const uint64_t nblk = len ? (len + 63) / 64 : (key.kk ? 0 : 1);
    auto take_of = [&](uint64_t b) -> uint32_t {
        const uint64_t rem = len - 64 * b;
        return rem < 64 ? static_cast<uint32_t>(rem) : 64u;
    };
    uint32_t cur[16], nxt[16];  // block b+1 in flight while block b is compressed
    if (nblk) load_block<16>(p, take_of(0), cur);
    for (uint64_t b = 0; b < nblk; b++) {
        if (b + 1 < nblk) load_block<16>(p + 64 * (b + 1), take_of(b + 1), nxt);
        t += take_of(b);
        compress32(h, cur, t, b + 1 == nblk);
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (4u * j < out_len) o[j] = h[j];
}

// ------------------------------------------------------------------ four lanes per chunk
// One BLAKE2 compression has 4-way parallelism: the four G functions of a column step (and of
// a diagonal step) are independent.  Here a quad of lanes shares one chunk: lane q holds column
// q of the working state (v[q], v[4+q], v[8+q], v[12+q]) and h[q], h[4+q].  Before the
// diagonal step rows b, c, d are rotated across the quad by 1, 2, 3 lanes (DPP quad_perm),
// and back after it.  The block's message words sit in LDS (128 or 64 bytes per quad); each
// lane reads the 4 it needs per round through a per-lane table of sigma indices.  The chain
// per block is ~1/3 of the one-lane kernel's, at ~1.3x its total VALU: for launches with too
// few chunks to fill the GPU (one split batch: ~5,700 chunks).
template <int CTRL>
__device__ __forceinline__ uint32_t qperm32(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint64_t qperm(uint64_t x) {
    return static_cast<uint64_t>(qperm32<CTRL>(static_cast<uint32_t>(x))) |
           (static_cast<uint64_t>(qperm32<CTRL>(static_cast<uint32_t>(x >> 32))) << 32);
}
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
    return qperm32<CTRL>(x);
}
constexpr int kQRot1 = 0x39;  // quad_perm [1,2,3,0]: lane q reads lane q+1
constexpr int kQRot2 = 0x4E;  // [2,3,0,1]
constexpr int kQRot3 = 0x93;  // [3,0,1,2]

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool B64>
__global__ __launch_bounds__(256) void blake2_chunks_x4_kernel(const uint8_t* data, const uint64_t* offs,
                                                               const uint64_t* lens, const uint32_t* order, uint32_t n,
                                                               HashKey key, uint32_t nn, uint32_t out_len,
                                                               uint32_t out_stride, uint8_t* out) {
    using W = typename std::conditional<B64, uint64_t, uint32_t>::type;
    constexpr int R = B64 ? 12 : 10;
    constexpr uint32_t BB = B64 ? 128 : 64;  // block bytes
    constexpr int NW = BB / 4;               // dwords per block
    constexpr int PER = NW / 4;              // dwords each lane loads
    __shared__ __attribute__((aligned(16))) uint32_t msg[4][16][NW];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, q = lane & 3u;
    uint32_t* M = msg[wv][lane >> 2];
    const uint32_t gi = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const bool live = gi < n;
    const uint32_t c = live ? (order ? order[gi] : gi) : 0u;
    const uint64_t len = live ? lens[c] : 0u;
    const uint8_t* p = data + (live ? offs[c] : 0u);

    // sigma indices this lane needs per round: column pair, diagonal pair (4 nibbles)
    uint32_t sidx[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint8_t* sg = kSig[r];
        const uint32_t v0 = sg[0] | (sg[1] << 4) | (sg[8] << 8) | (sg[9] << 12);
        const uint32_t v1 = sg[2] | (sg[3] << 4) | (sg[10] << 8) | (sg[11] << 12);
        const uint32_t v2 = sg[4] | (sg[5] << 4) | (sg[12] << 8) | (sg[13] << 12);
        const uint32_t v3 = sg[6] | (sg[7] << 4) | (sg[14] << 8) | (sg[15] << 12);
        sidx[r] = q == 0 ? v0 : q == 1 ? v1 : q == 2 ? v2 : v3;
    }
    auto iv = [](uint32_t i) -> W {
        if constexpr (B64)
            return i == 0 ? kIV64[0] : i == 1 ? kIV64[1] : i == 2 ? kIV64[2] : i == 3 ? kIV64[3]
                 : i == 4 ? kIV64[4] : i == 5 ? kIV64[5] : i == 6 ? kIV64[6] : kIV64[7];
        else return i == 0 ? kIV32[0] : i == 1 ? kIV32[1] : i == 2 ? kIV32[2] : i == 3 ? kIV32[3]
                   : i == 4 ? kIV32[4] : i == 5 ? kIV32[5] : i == 6 ? kIV32[6] : kIV32[7];
    };
    auto mword = [&](uint32_t k) -> W {
        if constexpr (B64) {
            const uint2 v = *reinterpret_cast<const uint2*>(M + 2 * k);
            return static_cast<uint64_t>(v.x) | (static_cast<uint64_t>(v.y) << 32);
        } else {
            return M[k];
        }
    };
    auto g = [](W& a, W& b, W& cc, W& d, W x, W y) {
        if constexpr (B64) g64(a, b, cc, d, x, y);
        else g32(a, b, cc, d, x, y);
    };
    const W ivq = iv(q), ivq4 = iv(4 + q);
    W h0 = ivq, h1 = ivq4;  // h[q], h[4+q]
    if (q == 0) h0 ^= static_cast<W>(0x01010000u ^ (key.kk << 8) ^ nn);
    auto compress = [&](uint64_t t, bool last) {
        W a = h0, b = h1, cc = ivq, d = ivq4;
        if (q == 0) d ^= static_cast<W>(t);
        if constexpr (!B64) {
            if (q == 1) d ^= static_cast<W>(t >> 32);
        }
        if (q == 2 && last) d = ~d;
        // the message words of round r + 1 are read from LDS during round r: the chain never
        // waits for them (4 LDS reads per round were on the critical path)
        W mx = mword(sidx[0] & 15u), my = mword((sidx[0] >> 4) & 15u);
        W dx = mword((sidx[0] >> 8) & 15u), dy = mword(sidx[0] >> 12);
#pragma unroll
        for (int r = 0; r < R; r++) {
            W nmx = mx, nmy = my, ndx = dx, ndy = dy;
            if (r + 1 < R) {
                const uint32_t sn = sidx[r + 1];
                nmx = mword(sn & 15u);
                nmy = mword((sn >> 4) & 15u);
                ndx = mword((sn >> 8) & 15u);
                ndy = mword(sn >> 12);
            }
            g(a, b, cc, d, mx, my);
            b = qperm<kQRot1>(b);
            cc = qperm<kQRot2>(cc);
            d = qperm<kQRot3>(d);
            g(a, b, cc, d, dx, dy);
            b = qperm<kQRot3>(b);
            cc = qperm<kQRot2>(cc);
            d = qperm<kQRot1>(d);
            mx = nmx;
            my = nmy;
            dx = ndx;
            dy = ndy;
        }
        h0 ^= a ^ cc;
        h1 ^= b ^ d;
    };
    uint64_t t = 0;
    if (live && key.kk) {  // the key block (RFC 7693 §3.3)
        if (q == 0) {
#pragma unroll
            for (int j = 0; j < NW; j++) M[j] = j < 16 ? key.w[j] : 0u;
        }
        wave_lds_fence();
        t = BB;
        compress(t, len == 0);
        wave_lds_fence();
    }
    const uint64_t nblk = !live ? 0 : len ? (len + BB - 1) / BB : (key.kk ? 0 : 1);
    for (uint64_t blk = 0; blk < nblk; blk++) {
        const uint64_t rem = len - BB * blk;
        const uint32_t take = rem < BB ? static_cast<uint32_t>(rem) : BB;
        // this lane's quarter of the block: bytes [4 PER q, 4 PER q + 4 PER)
        const int32_t part = static_cast<int32_t>(take) - static_cast<int32_t>(4 * PER * q);
        uint32_t w[PER];
        load_block<PER>(p + BB * blk + 4 * PER * q, part <= 0 ? 0u : static_cast<uint32_t>(part), w);
#pragma unroll
        for (int j = 0; j < PER; j++) M[PER * q + j] = w[j];
        wave_lds_fence();
        t += take;
        compress(t, blk + 1 == nblk);
        wave_lds_fence();
    }
    if (!live) return;
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
    constexpr uint32_t WB = sizeof(W);
    if (WB * q < out_len) {
        o[(WB / 4) * q] = static_cast<uint32_t>(h0);
        if constexpr (B64) o[2 * q + 1] = static_cast<uint32_t>(static_cast<uint64_t>(h0) >> 32);
    }
    if (WB * (4 + q) < out_len) {
        o[(WB / 4) * (4 + q)] = static_cast<uint32_t>(h1);
        if constexpr (B64) o[2 * (4 + q) + 1] = static_cast<uint32_t>(static_cast<uint64_t>(h1) >> 32);
    }
}

}  // namespace hashdev

int& test_hash_lanes() {  // kcdc_test_set(KCDC_TEST_HASH_LANES): 0 auto, 1 or 4 lanes per chunk
    static int v = 0;
    return v;
}

namespace {
struct HashAlgo {
    const char* name;
    bool b64;       // BLAKE2b (else BLAKE2s)
    uint32_t nn;    // digest length parameter
    uint32_t out;   // bytes kept (truncation)
};
// repo/hashing/blake_hashes.go:8-13 (registered names and their truncation)
constexpr HashAlgo kHashAlgos[] = {
    {"BLAKE2B-256-128", true, 32, 16},
    {"BLAKE2B-256", true, 32, 32},
    {"BLAKE2S-128", false, 16, 16},
    {"BLAKE2S-256", false, 32, 32},
};
const HashAlgo* find_hash(const char* name) {
    if (!name) return nullptr;
    for (const HashAlgo& h : kHashAlgos)
        if (std::strcmp(h.name, name) == 0) return &h;
    return nullptr;
}
}  // namespace
}  // namespace kcdc

using namespace kcdc;

extern "C" int kcdc_hash_algorithms(const char** names, int cap) {
    const int n = static_cast<int>(sizeof(kHashAlgos) / sizeof(kHashAlgos[0]));
    for (int i = 0; i < n && i < cap; i++) names[i] = kHashAlgos[i].name;
    return n;
}

extern "C" int kcdc_hash_size(const char* name) {
    const HashAlgo* h = find_hash(name);
    return h ? static_cast<int>(h->out) : set_error(-2, std::string("unknown hash: ") + (name ? name : "(null)"));
}

extern "C" int kcdc_hash_chunks_device(const char* name, const uint8_t* d_data, const uint64_t* d_offsets,
                                       const uint64_t* d_lens, const uint32_t* d_order, uint32_t nchunks,
                                       const uint8_t* key, uint32_t key_len, uint8_t* d_out, uint32_t out_stride,
                                       void* stream) {
    const HashAlgo* h = find_hash(name);
    if (!h) return set_error(-2, std::string("unknown hash: ") + (name ? name : "(null)"));
    // blake2b.New256 / blake2s.New*: at most 64 / 32 key bytes; BLAKE2s-128 needs a key
    // (golang.org/x/crypto/blake2s New128 rejects an empty one), as CreateHashFunc reports.
    if (key_len > (h->b64 ? 64u : 32u) || (key_len && !key)) return set_error(-22, "hash key too long");
    if (!h->b64 && h->nn == 16 && key_len == 0) return set_error(-22, "BLAKE2S-128 requires a key");
    if (out_stride < h->out || out_stride % 4) return set_error(-22, "out_stride must be >= the hash size and a multiple of 4");
    if (nchunks == 0) return 0;
    if (!d_data || !d_offsets || !d_lens || !d_out) return set_error(-22, "null argument");
    hashdev::HashKey k{};
    k.kk = key_len;
    for (uint32_t i = 0; i < key_len; i++) k.w[i / 4] |= static_cast<uint32_t>(key[i]) << (8 * (i % 4));
    hipStream_t st = static_cast<hipStream_t>(stream);
    // Four lanes per chunk unless the launch holds over 2^20 chunks (64 waves per SIMD, where
    // the one-lane kernel's ~25 % lower VALU per block would matter).  Measured on config-2
    // chunk tables: 5,705 chunks 84 vs 540 ms, 136,920 chunks 263 vs 630 ms (one lane per
    // chunk leaves a dependent chain per lane with too few waves to interleave).
    const int forced = test_hash_lanes();
    const bool x4 = forced ? forced == 4 : nchunks <= (1u << 20);
    if (x4) {
        const dim3 grid4((4ull * nchunks + 255) / 256), block4(256);
        if (h->b64)
            hipLaunchKernelGGL(hashdev::blake2_chunks_x4_kernel<true>, grid4, block4, 0, st, d_data, d_offsets, d_lens,
                               d_order, nchunks, k, h->nn, h->out, out_stride, d_out);
        else
            hipLaunchKernelGGL(hashdev::blake2_chunks_x4_kernel<false>, grid4, block4, 0, st, d_data, d_offsets, d_lens,
                               d_order, nchunks, k, h->nn, h->out, out_stride, d_out);
        const hipError_t e4 = hipGetLastError();
        return e4 == hipSuccess ? 0 : set_error(-5, std::string("hash kernel launch: ") + hipGetErrorString(e4));
    }
    const dim3 grid((nchunks + 255) / 256), block(256);
    if (h->b64)
        hipLaunchKernelGGL(hashdev::blake2b_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    else
        hipLaunchKernelGGL(hashdev::blake2s_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("hash kernel launch: ") + hipGetErrorString(e));
}
