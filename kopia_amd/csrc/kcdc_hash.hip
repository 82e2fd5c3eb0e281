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

// Prefetch for 16-byte aligned chunks (the resumable chains): a lane's quarter of a block is
// issued as dwordx4 loads and only masked when its block is used, so the loads stay in flight
// while earlier blocks compress.  (load_block consumes its loads at once: the "next block"
// prefetch of round 5's first chain kernel waited a memory round trip every block, ~2.5 us.)
// Loads are unconditional (a conditional load leaves the waitcnt pass unsure at the join, and it
// waits for everything there): a vector with no bytes of the chunk reads the chunk's first 16
// bytes instead (`safe`), which the mask discards.
template <int NW>
__device__ __forceinline__ void load_aligned(const uint8_t* p, uint32_t take, const uint8_t* safe, uint32_t (&x)[NW]) {
    static_assert(NW % 4 == 0, "whole dwordx4 vectors");
    typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) u32x4v gu32x4;
#pragma unroll
    for (int v = 0; v < NW / 4; v++) {
        const uint8_t* a = take > 16u * v ? p + 16 * v : safe;
        const u32x4v r = *reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(a));
        x[4 * v] = r.x;
        x[4 * v + 1] = r.y;
        x[4 * v + 2] = r.z;
        x[4 * v + 3] = r.w;
    }
}
template <int NW>
__device__ __forceinline__ void mask_take(uint32_t take, uint32_t (&d)[NW]) {
    if (take < 4u * NW) {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            const int32_t keep = static_cast<int32_t>(take) - 4 * i;
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
    // this lane's quarter of block blk: bytes [4 PER q, 4 PER q + 4 PER)
    auto take_of = [&](uint64_t blk) -> uint32_t {
        const uint64_t rem = len - BB * blk;
        return rem < BB ? static_cast<uint32_t>(rem) : BB;
    };
    auto load_quarter = [&](uint64_t blk, uint32_t (&w)[PER]) {
        const int32_t part = static_cast<int32_t>(take_of(blk)) - static_cast<int32_t>(4 * PER * q);
        load_block<PER>(p + BB * blk + 4 * PER * q, part <= 0 ? 0u : static_cast<uint32_t>(part), w);
    };
    // Block blk+1's quarter is loaded while block blk is compressed (round 5): the chain no longer
    // waits a global-memory round trip per block.
    uint32_t w[PER], wn[PER];
    if (nblk) load_quarter(0, w);
    for (uint64_t blk = 0; blk < nblk; blk++) {
        if (blk + 1 < nblk) load_quarter(blk + 1, wn);
#pragma unroll
        for (int j = 0; j < PER; j++) M[PER * q + j] = w[j];
        wave_lds_fence();
        t += take_of(blk);
        compress(t, blk + 1 == nblk);
        wave_lds_fence();
#pragma unroll
        for (int j = 0; j < PER; j++) w[j] = wn[j];
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

// ------------------------------------------------------------------ resumable chains (writers)
// The batching object writers (kcdc_bw_*, kcdc_writer.cpp) name every final chunk as it is cut.
// A BLAKE2 chunk is one chain of dependent compressions (~32,768 for a 4 MiB chunk), far longer
// than a writer round, so the chains advance in slices: each launch moves every active chain by
// at most max_blocks blocks, from its state in device memory (HashChain), one quad of lanes per
// chain as in blake2_chunks_x4_kernel.  A chain's first slice also runs the key block; its last
// writes the digest to slot `out`.  Chunks stay where the writer copied them until their chain ends.
// A step is one launch and no copies: the active list may be host-mapped pinned memory, an entry
// with kChainNew set takes its record (src, len, out) from `fresh` (host-mapped: the host wrote it)
// and stores it into `chains` for the later slices, and `out` may be host-mapped too.  (One small
// hipMemcpyAsync each way per step queued behind the writers' PCIe gathers on the copy engines.)
// The message words' LDS addresses are the same for every block (lane and round only): computed
// once, 48 VGPRs (recomputing them was 144 of the block's 928 instructions).
// Workgroups of 4 waves, one per SIMD: a wave issues ~800 instructions per block for its 16 chains
// and runs alone at ~7 cycles per instruction; three waves per SIMD (12-wave workgroups) measured
// 8.2 ms per 2,048-block step against 5.1 (profiles/r05/writer_ids/), so the SIMD's issue, not the
// chain's latency, is what a second wave would share.
constexpr int kChainWaves = 4;
template <bool B64>
__global__ __launch_bounds__(kChainWaves * 64) void blake2_chain_step_kernel(HashChain* chains, const HashChain* fresh,
                                                                const uint32_t* active, uint32_t n,
                                                                uint64_t max_blocks, HashKey key, uint32_t nn,
                                                                uint32_t out_len, uint32_t out_stride, uint8_t* out) {
    using W = typename std::conditional<B64, uint64_t, uint32_t>::type;
    constexpr int R = B64 ? 12 : 10;
    constexpr uint32_t BB = B64 ? 128 : 64;
    constexpr int NW = BB / 4;
    constexpr int PER = NW / 4;
    __shared__ __attribute__((aligned(16))) uint32_t msg[kChainWaves][16][NW];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, q = lane & 3u;
    uint32_t* M = msg[wv][lane >> 2];
    const uint32_t gi = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    const bool live = gi < n;
    const uint32_t ent = live ? active[gi] : 0u;
    const bool is_new = (ent & kChainNew) != 0u;
    const uint32_t slot = ent & ~kChainNew;
    HashChain* ch = chains + slot;
    const HashChain* rec = is_new ? fresh + slot : ch;
    const uint64_t len = live ? rec->len : 0u;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(live ? rec->src : 0u);
    const uint64_t next0 = !live ? 0u : is_new ? ~0ull : ch->next;
    const uint32_t oslot = live ? rec->out : 0u;
    if (live && is_new && q == 0) {  // the record, for the chain's later slices
        ch->src = reinterpret_cast<uint64_t>(p);
        ch->len = len;
        ch->out = oslot;
    }
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
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) const u32x2 lds_u2;
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    const uint32_t mbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint32_t*)(M)));
    uint32_t maddr[R][4];  // byte addresses of the 4 words this lane reads in round r
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            maddr[r][j] = mbase + (B64 ? 8u : 4u) * ((sidx[r] >> (4 * j)) & 15u);
            asm volatile("" : "+v"(maddr[r][j]));  // opaque: kept in a register, not recomputed per block
        }
    auto mword = [&](uint32_t addr) -> W {
        if constexpr (B64) {
            const u32x2 v = *reinterpret_cast<lds_u2*>(addr);
            return static_cast<uint64_t>(v.x) | (static_cast<uint64_t>(v.y) << 32);
        } else {
            return *reinterpret_cast<lds_u32*>(addr);
        }
    };
    auto g = [](W& a, W& b, W& cc, W& d, W x, W y) {
        if constexpr (B64) g64(a, b, cc, d, x, y);
        else g32(a, b, cc, d, x, y);
    };
    const W ivq = iv(q), ivq4 = iv(4 + q);
    W h0, h1;
    auto compress = [&](uint64_t t, bool last) {
        W a = h0, b = h1, cc = ivq, d = ivq4;
        if (q == 0) d ^= static_cast<W>(t);
        if constexpr (!B64) {
            if (q == 1) d ^= static_cast<W>(t >> 32);
        }
        if (q == 2 && last) d = ~d;
        W mx = mword(maddr[0][0]), my = mword(maddr[0][1]);
        W dx = mword(maddr[0][2]), dy = mword(maddr[0][3]);
#pragma unroll
        for (int r = 0; r < R; r++) {
            W nmx = mx, nmy = my, ndx = dx, ndy = dy;
            if (r + 1 < R) {
                nmx = mword(maddr[r + 1][0]);
                nmy = mword(maddr[r + 1][1]);
                ndx = mword(maddr[r + 1][2]);
                ndy = mword(maddr[r + 1][3]);
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
    const uint64_t nblk = len ? (len + BB - 1) / BB : (key.kk ? 0 : 1);
    uint64_t next = next0;
    if (next == ~0ull) {  // a new chain: the parameter block, then the key block (RFC 7693 §3.3)
        h0 = ivq;
        h1 = ivq4;
        if (q == 0) h0 ^= static_cast<W>(0x01010000u ^ (key.kk << 8) ^ nn);
        if (live && key.kk) {
            if (q == 0) {
#pragma unroll
                for (int j = 0; j < NW; j++) M[j] = j < 16 ? key.w[j] : 0u;
            }
            wave_lds_fence();
            compress(BB, len == 0);
            wave_lds_fence();
        }
        next = 0;
    } else {
        h0 = static_cast<W>(live ? ch->h[q] : 0u);
        h1 = static_cast<W>(live ? ch->h[4 + q] : 0u);
    }
    const uint64_t end = !live ? next : nblk - next < max_blocks ? nblk : next + max_blocks;
    auto take_of = [&](uint64_t blk) -> uint32_t {
        const uint64_t rem = len - BB * blk;
        return rem < BB ? static_cast<uint32_t>(rem) : BB;
    };
    uint64_t t = (key.kk ? BB : 0) + (next * BB < len ? next * BB : len);
    // Blocks blk+1 and blk+2 are in flight (unmasked) while block blk is compressed: beside the
    // writers' gathers and splits a load takes about as long as one compression.  The chunk
    // starts 16-byte aligned (launch_hash_chains' contract; the writers' ring copies realign).
    constexpr int kAhead = 3;
    auto part_of = [&](uint64_t blk) -> uint32_t {
        const int32_t part = static_cast<int32_t>(take_of(blk)) - static_cast<int32_t>(4 * PER * q);
        return part <= 0 ? 0u : static_cast<uint32_t>(part);
    };
    uint32_t w[kAhead][PER];
    // block indices past the slice's end load the slice's last block again (never used)
    auto pre = [&](uint64_t b, uint32_t (&r)[PER]) {
        const uint64_t bb = b < end ? b : end - 1;
        load_aligned<PER>(p + BB * bb + 4 * PER * q, part_of(bb), p, r);
    };
    static_assert(kAhead == 3, "the block loop below is unrolled over three buffers");
    // one block: prefetch blk + 2 into `fill`, compress blk from `use` (the buffers rotate by
    // unrolling, not by copies: a register copy of an in-flight load waits for it)
    auto step = [&](uint32_t (&use)[PER], uint32_t (&fill)[PER], uint64_t blk) {
        pre(blk + kAhead - 1, fill);
        uint32_t cur[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) cur[j] = use[j];
        mask_take<PER>(part_of(blk), cur);
#pragma unroll
        for (int j = 0; j < PER; j++) M[PER * q + j] = cur[j];
        wave_lds_fence();
        t += take_of(blk);
        compress(t, blk + 1 == nblk);
        wave_lds_fence();
    };
    if (next < end) {
        pre(next, w[0]);
        pre(next + 1, w[1]);
    }
    for (uint64_t blk = next; blk < end;) {
        step(w[0], w[2], blk);
        if (++blk >= end) break;
        step(w[1], w[0], blk);
        if (++blk >= end) break;
        step(w[2], w[1], blk);
        ++blk;
    }
    if (!live) return;
    if (end < nblk) {  // the chain goes on in a later slice
        ch->h[q] = static_cast<uint64_t>(h0);
        ch->h[4 + q] = static_cast<uint64_t>(h1);
        if (q == 0) ch->next = end;
        return;
    }
    if (q == 0) ch->next = nblk;
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(oslot) * out_stride);
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

// ------------------------------------------------------------------ HMAC-SHA256 / HMAC-SHA224
// repo/hashing/sha_hashes.go:10-12: hmac.New(sha256.New | sha256.New224, secret), truncated.
// HMAC(K, m) = H(K0 ^ opad || H(K0 ^ ipad || m)) (RFC 2104, FIPS 198-1): the host compresses the
// two key blocks once (ShaMid), so a chunk costs its own blocks plus one outer block.  One lane
// per chunk: SHA-256's 64 rounds are one dependent chain (FIPS 180-4), no intra-block width.
constexpr uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

struct ShaMid {
    uint32_t in[8];   // state after the K0 ^ ipad block
    uint32_t out[8];  // state after the K0 ^ opad block
};

__host__ __device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// One SHA-256 block (big-endian words already assembled in w).
__host__ __device__ __forceinline__ void sha256_block(uint32_t (&h)[8], uint32_t (&w)[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int r = 0; r < 64; r++) {
        if (r >= 16) {
            const uint32_t x = w[(r - 15) & 15], y = w[(r - 2) & 15];
            w[r & 15] += (ror32(x, 7) ^ ror32(x, 18) ^ (x >> 3)) + w[(r - 7) & 15] + (ror32(y, 17) ^ ror32(y, 19) ^ (y >> 10));
        }
        const uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + kK256[r] + w[r & 15];
        const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

// DW = digest words of the inner hash (8: SHA-256, 7: SHA-224).
template <int DW>
__global__ __launch_bounds__(256) void hmac_sha256_kernel(const uint8_t* data, const uint64_t* offs, const uint64_t* lens,
                                                          const uint32_t* order, uint32_t n, ShaMid mid, uint32_t out_len,
                                                          uint32_t out_stride, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = order ? order[i] : i;
    const uint64_t len = lens[c];
    const uint8_t* p = data + offs[c];
    uint32_t h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = mid.in[j];
    const uint64_t nfull = len / 64;
    const uint32_t rem = static_cast<uint32_t>(len % 64);
    uint32_t cur[16], nxt[16];
    load_block<16>(p, nfull ? 64u : rem, cur);
    for (uint64_t b = 0; b < nfull; b++) {  // block b+1 (or the tail) in flight while b is compressed
        load_block<16>(p + 64 * (b + 1), b + 1 < nfull ? 64u : rem, nxt);
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = bswap32(cur[j]);
        sha256_block(h, cur);
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = nxt[j];
    }
    // tail: rem bytes, 0x80, zeros, the 64-bit bit length of ipad block + message
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if (static_cast<uint32_t>(j) == (rem >> 2)) cur[j] |= 0x80u << (8 * (rem & 3u));
        cur[j] = bswap32(cur[j]);
    }
    const uint64_t bits = (len + 64) * 8;
    if (rem >= 56) {
        sha256_block(h, cur);
#pragma unroll
        for (int j = 0; j < 16; j++) cur[j] = 0;
    }
    cur[14] = static_cast<uint32_t>(bits >> 32);
    cur[15] = static_cast<uint32_t>(bits);
    sha256_block(h, cur);
    // outer: K0 ^ opad (in mid.out) then the inner digest, 0x80, length (64 + 4 DW) * 8
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = j < DW ? h[j] : j == DW ? 0x80000000u : 0u;
    w[15] = (64u + 4u * DW) * 8u;
    uint32_t o2[8];
#pragma unroll
    for (int j = 0; j < 8; j++) o2[j] = mid.out[j];
    sha256_block(o2, w);
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (4u * j < out_len) o[j] = bswap32(o2[j]);
}

// ------------------------------------------------------------------ HMAC-SHA3-224 / -256
// repo/hashing/sha_hashes.go:13-14: hmac.New(sha3.New224 | sha3.New256, secret); the HMAC block
// is the sponge rate (144 / 136 bytes, FIPS 202; Go's sha3 BlockSize()).  The host absorbs the two
// key blocks (KeccakMid); one lane per chunk runs Keccak-f[1600] on 25 x 64-bit lanes held as
// 50 VGPR halves (rotations by constants are v_alignbit pairs, chi is v_bitop3).
struct KeccakMid {
    uint64_t in[25];
    uint64_t out[25];
};

constexpr uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull, 0x000000000000808Bull,
    0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull, 0x000000000000008Aull, 0x0000000000000088ull,
    0x0000000080008009ull, 0x000000008000000Aull, 0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull,
    0x8000000000008003ull, 0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
// rho offsets and pi destinations by lane index x + 5 y (FIPS 202 §3.2.2-3.2.3)
constexpr int kKeccakRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
// pi: B[y, 2x + 3y] = rot(A[x, y]) -> destination index of source lane x + 5 y
// pi: B[y, 2x + 3y] = rot(A[x, y], rho[x, y]): source lane x + 5 y -> destination y + 5 ((2x + 3y) mod 5)
constexpr int keccak_pi_dst(int s) { return (s / 5) + 5 * ((2 * (s % 5) + 3 * (s / 5)) % 5); }

// rotate left by n (a constant once the rounds are unrolled): v_alignbit pairs
__device__ __forceinline__ uint64_t rotl64n(uint64_t x, int n) {
    const uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32);
    uint32_t nlo, nhi;
    if (n == 0) return x;
    if (n == 32) {
        nlo = hi;
        nhi = lo;
    } else if (n < 32) {
        nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - n);
        nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - n);
    } else {
        nhi = __builtin_amdgcn_alignbit(lo, hi, 64 - n);
        nlo = __builtin_amdgcn_alignbit(hi, lo, 64 - n);
    }
    return (static_cast<uint64_t>(nhi) << 32) | nlo;
}

__device__ __forceinline__ void keccak_f(uint64_t (&s)[25]) {
#pragma unroll
    for (int r = 0; r < 24; r++) {
        uint64_t C[5], D[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
#pragma unroll
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rotl64n(C[(x + 1) % 5], 1);
#pragma unroll
        for (int k = 0; k < 25; k++) B[keccak_pi_dst(k)] = rotl64n(s[k] ^ D[k % 5], kKeccakRho[k]);
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
#pragma unroll
            for (int x = 0; x < 5; x++) s[y + x] = B[y + x] ^ (~B[y + (x + 1) % 5] & B[y + (x + 2) % 5]);
        }
        s[0] ^= kKeccakRC[r];
    }
}

// RATE: sponge rate in bytes; DB: digest bytes of the inner hash.
template <int RATE, int DB>
__global__ __launch_bounds__(256) void hmac_sha3_kernel(const uint8_t* data, const uint64_t* offs, const uint64_t* lens,
                                                        const uint32_t* order, uint32_t n, KeccakMid mid, uint32_t out_len,
                                                        uint32_t out_stride, uint8_t* out) {
    constexpr int NW = RATE / 4;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = order ? order[i] : i;
    const uint64_t len = lens[c];
    const uint8_t* p = data + offs[c];
    uint64_t s[25];
#pragma unroll
    for (int j = 0; j < 25; j++) s[j] = mid.in[j];
    const uint64_t nfull = len / RATE;
    const uint32_t rem = static_cast<uint32_t>(len % RATE);
    uint32_t cur[NW], nxt[NW];
    load_block<NW>(p, nfull ? static_cast<uint32_t>(RATE) : rem, cur);
    auto absorb = [&](const uint32_t (&w)[NW]) {
#pragma unroll
        for (int j = 0; j < NW / 2; j++) s[j] ^= static_cast<uint64_t>(w[2 * j]) | (static_cast<uint64_t>(w[2 * j + 1]) << 32);
        keccak_f(s);
    };
    for (uint64_t b = 0; b < nfull; b++) {
        load_block<NW>(p + static_cast<uint64_t>(RATE) * (b + 1), b + 1 < nfull ? static_cast<uint32_t>(RATE) : rem, nxt);
        absorb(cur);
#pragma unroll
        for (int j = 0; j < NW; j++) cur[j] = nxt[j];
    }
    // pad10*1 with the SHA-3 domain bits: 0x06 after the message, 0x80 in the block's last byte
#pragma unroll
    for (int j = 0; j < NW; j++) {
        if (static_cast<uint32_t>(j) == (rem >> 2)) cur[j] |= 0x06u << (8 * (rem & 3u));
        if (j == NW - 1) cur[j] |= 0x80000000u;
    }
    absorb(cur);
    // outer: the inner digest's DB bytes (little-endian lanes of s), then its padding
    uint32_t w[NW];
#pragma unroll
    for (int j = 0; j < NW; j++) {
        const uint32_t half = (j & 1) ? static_cast<uint32_t>(s[j / 2] >> 32) : static_cast<uint32_t>(s[j / 2]);
        w[j] = 4 * j < DB ? half : 0u;
        if (4 * j == DB) w[j] = 0x06u;
        if (j == NW - 1) w[j] |= 0x80000000u;
    }
#pragma unroll
    for (int j = 0; j < 25; j++) s[j] = mid.out[j];
    absorb(w);
    uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (4u * j < out_len) o[j] = (j & 1) ? static_cast<uint32_t>(s[j / 2] >> 32) : static_cast<uint32_t>(s[j / 2]);
}

// ------------------------------------------------------------------ BLAKE3 keyed hash
// repo/hashing/blake3_hashes.go:10-27: blake3.NewKeyed(key) (github.com/zeebo/blake3, not
// vendored), key = the 32-byte secret, or DeriveKey("kopia blake3 derived key v1", secret) for a
// shorter one (host side, kcdc_hash_chunks_device).  BLAKE3 (the published spec): 1 KiB chunks
// hashed independently (16 blocks, a 7-round BLAKE2s-like compression, counter = chunk index),
// CVs merged in a left-complete binary tree of PARENT nodes; ROOT marks the last compression.
// One wave per content: a round takes up to 256 chunks (4 per lane, in order), then merges their
// CVs level by level in LDS; the level leftovers (odd counts) are the round's subtrees.  Full
// rounds' 256-chunk subtrees go on a per-wave stack and merge as in the sequential algorithm;
// the last round's subtrees are appended, and the stack is folded right to left at the end.
// A merge is the ROOT when it covers every chunk of the content.
constexpr uint32_t kB3ChunkStart = 1, kB3ChunkEnd = 2, kB3Parent = 4, kB3Root = 8, kB3Keyed = 16;
constexpr int kB3Perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
struct B3Sched {
    int s[7][16];
    constexpr B3Sched() : s{} {
        for (int i = 0; i < 16; i++) s[0][i] = i;
        for (int r = 1; r < 7; r++)
            for (int i = 0; i < 16; i++) s[r][i] = s[r - 1][kB3Perm[i]];
    }
};
constexpr B3Sched kB3S{};

struct B3Key {
    uint32_t k[8];
};

// Compression -> the 8-word chaining value (v[i] ^ v[i + 8]).
__host__ __device__ __forceinline__ void b3_compress(const uint32_t (&cv)[8], const uint32_t (&m)[16], uint64_t t,
                                                     uint32_t blen, uint32_t flags, uint32_t (&out)[8]) {
    uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7], kIV32[0], kIV32[1], kIV32[2], kIV32[3],
                      static_cast<uint32_t>(t), static_cast<uint32_t>(t >> 32), blen, flags};
    auto g = [](uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
        a = a + b + x;
        d = ror32(d ^ a, 16);
        c = c + d;
        b = ror32(b ^ c, 12);
        a = a + b + y;
        d = ror32(d ^ a, 8);
        c = c + d;
        b = ror32(b ^ c, 7);
    };
#pragma unroll
    for (int r = 0; r < 7; r++) {
#define S3(i) m[kB3S.s[r][i]]
        g(v[0], v[4], v[8], v[12], S3(0), S3(1));
        g(v[1], v[5], v[9], v[13], S3(2), S3(3));
        g(v[2], v[6], v[10], v[14], S3(4), S3(5));
        g(v[3], v[7], v[11], v[15], S3(6), S3(7));
        g(v[0], v[5], v[10], v[15], S3(8), S3(9));
        g(v[1], v[6], v[11], v[12], S3(10), S3(11));
        g(v[2], v[7], v[8], v[13], S3(12), S3(13));
        g(v[3], v[4], v[9], v[14], S3(14), S3(15));
#undef S3
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = v[i] ^ v[i + 8];
}

constexpr int kB3PerLane = 4;                     // chunks per lane per round
constexpr int kB3Round = 64 * kB3PerLane;         // chunks per round
constexpr int kB3Stack = 48;                      // per-wave stack entries (2^48 rounds: never full)
constexpr int kB3Waves = 4;                       // waves (contents) per workgroup

struct B3Wave {
    uint32_t x[kB3Round][8];   // the round's CVs, merged level by level in place
    uint32_t st[kB3Stack][8];  // the stack's subtree CVs, left to right
};

__global__ __launch_bounds__(64 * kB3Waves) void blake3_keyed_kernel(const uint8_t* data, const uint64_t* offs,
                                                                     const uint64_t* lens, const uint32_t* order,
                                                                     uint32_t n, B3Key key, uint32_t out_len,
                                                                     uint32_t out_stride, uint8_t* out) {
    __shared__ B3Wave sw[kB3Waves];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t gi = blockIdx.x * kB3Waves + wv;
    if (gi >= n) return;  // wave-uniform
    B3Wave& W = sw[wv];
    const uint32_t c = order ? order[gi] : gi;
    const uint64_t len = lens[c];
    const uint8_t* p = data + offs[c];
    const uint64_t nch = len ? (len + 1023) / 1024 : 1;
    uint32_t kcv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) kcv[j] = key.k[j];
    // chunk ch's CV (ROOT on its last block when it is the content's only chunk)
    auto chunk_cv = [&](uint64_t ch, uint32_t (&cv)[8]) {
        const uint64_t base = ch * 1024;
        const uint64_t clen64 = len - base < 1024 ? len - base : 1024;
        const uint32_t clen = static_cast<uint32_t>(clen64);
        const uint32_t nb = clen ? (clen + 63) / 64 : 1;
#pragma unroll
        for (int j = 0; j < 8; j++) cv[j] = kcv[j];
        uint32_t cur[16], nxt[16];
        load_block<16>(p + base, clen < 64 ? clen : 64u, cur);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t take = clen - 64 * b < 64 ? clen - 64 * b : 64u;
            if (b + 1 < nb) {
                const uint32_t tn = clen - 64 * (b + 1);
                load_block<16>(p + base + 64 * (b + 1), tn < 64 ? tn : 64u, nxt);
            }
            const uint32_t fl = kB3Keyed | (b == 0 ? kB3ChunkStart : 0u) |
                                (b + 1 == nb ? (kB3ChunkEnd | (nch == 1 ? kB3Root : 0u)) : 0u);
            uint32_t o[8];
            b3_compress(cv, cur, ch, take, fl, o);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                cv[j] = o[j];
                cur[j] = nxt[j];
                cur[j + 8] = nxt[j + 8];
            }
        }
    };
    auto parent = [&](const uint32_t* l, const uint32_t* r, bool root, uint32_t (&o)[8]) {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            m[j] = l[j];
            m[j + 8] = r[j];
        }
        b3_compress(kcv, m, 0, 64, kB3Keyed | kB3Parent | (root ? kB3Root : 0u), o);
    };
    if (nch == 1) {
        if (lane == 0) {
            uint32_t cv[8];
            chunk_cv(0, cv);
            uint32_t* o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (4u * j < out_len) o[j] = cv[j];
        }
        return;
    }
    uint32_t* const o = reinterpret_cast<uint32_t*>(out + static_cast<uint64_t>(c) * out_stride);
    uint32_t sdepth = 0;  // entries on the wave's stack (W.st), wave-uniform
    const uint64_t rounds = (nch + kB3Round - 1) / kB3Round;
    for (uint64_t rd = 0; rd < rounds; rd++) {
        const uint64_t c0 = rd * kB3Round;
        const uint32_t cnt = static_cast<uint32_t>(nch - c0 < static_cast<uint64_t>(kB3Round) ? nch - c0 : kB3Round);
        for (int q = 0; q < kB3PerLane; q++) {  // lane: chunks [4 lane, 4 lane + 4) of the round
            const uint32_t k = kB3PerLane * lane + q;
            if (k < cnt) {
                uint32_t cv[8];
                chunk_cv(c0 + k, cv);
#pragma unroll
                for (int j = 0; j < 8; j++) W.x[k][j] = cv[j];
            }
        }
        wave_lds_fence();
        // level L holds floor(cnt / 2^L) items at stride 2^L; an odd count leaves its last item
        // (slot (count - 1) 2^L) as one of the round's subtrees
        uint32_t count = cnt, stride = 1;
        bool lower_left = false;  // a lower level left a subtree over
        while (count > 1) {
            const uint32_t pairs = count / 2;
            const bool whole = cnt == nch && count == 2 && !lower_left;  // this merge covers the content
            for (uint32_t pr = lane; pr < pairs; pr += 64) {
                uint32_t h[8];
                parent(W.x[2 * pr * stride], W.x[(2 * pr + 1) * stride], whole, h);
#pragma unroll
                for (int j = 0; j < 8; j++) W.x[2 * pr * stride][j] = h[j];
            }
            wave_lds_fence();
            if (whole) {  // the content is one power-of-two round: x[0] is the root's output
                if (lane < 8 && 4u * lane < out_len) o[lane] = W.x[0][lane];
                return;
            }
            lower_left = lower_left || (count & 1u);
            count = pairs;
            stride *= 2;
        }
        if (c0 + cnt < nch) {
            // a full, non-final round: its 256-chunk subtree (slot 0) goes on the stack, merging
            // equal sizes as the sequential algorithm does (rounds done = rd + 1, while even);
            // never the root, since chunks remain
            if (lane < 8) W.st[sdepth][lane] = W.x[0][lane];
            sdepth++;
            wave_lds_fence();
            for (uint64_t t = rd + 1; (t & 1u) == 0; t >>= 1) {
                uint32_t h[8];
                parent(W.st[sdepth - 2], W.st[sdepth - 1], false, h);
                wave_lds_fence();
                if (lane == 0) {
#pragma unroll
                    for (int j = 0; j < 8; j++) W.st[sdepth - 2][j] = h[j];
                }
                sdepth--;
                wave_lds_fence();
            }
            continue;
        }
        // the final round: append its subtrees left to right (highest level first), then fold
        // the stack right to left; the last merge is the root
        for (int L = 31; L >= 0; L--) {
            const uint32_t cL = cnt >> L;
            if (cL & 1u) {
                if (lane < 8) W.st[sdepth][lane] = W.x[(cL - 1) << L][lane];
                sdepth++;
            }
        }
        wave_lds_fence();
        uint32_t acc[8];
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = W.st[sdepth - 1][j];
        for (int e = static_cast<int>(sdepth) - 2; e >= 0; e--) {
            uint32_t h[8];
            parent(W.st[e], acc, e == 0, h);
#pragma unroll
            for (int j = 0; j < 8; j++) acc[j] = h[j];
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (4u * j < out_len) o[j] = acc[j];
        }
    }
}

}  // namespace hashdev

int& test_hash_lanes() {  // kcdc_test_set(KCDC_TEST_HASH_LANES): 0 auto, 1 or 4 lanes per chunk
    static int v = 0;
    return v;
}

namespace {
enum class HashKind { Blake2b, Blake2s, HmacSha256, HmacSha224, HmacSha3_224, HmacSha3_256, Blake3 };
struct HashAlgo {
    const char* name;
    HashKind kind;
    uint32_t nn;   // BLAKE2 digest length parameter
    uint32_t out;  // bytes kept (truncation)
};
// repo/hashing/{blake_hashes.go:8-13, blake3_hashes.go:24-27, sha_hashes.go:9-15}: every registered
// name, in the order hashing.SupportedAlgorithms() returns them (sort.Strings, hashing.go:40-49)
constexpr HashAlgo kHashAlgos[] = {
    {"BLAKE2B-256", HashKind::Blake2b, 32, 32},
    {"BLAKE2B-256-128", HashKind::Blake2b, 32, 16},
    {"BLAKE2S-128", HashKind::Blake2s, 16, 16},
    {"BLAKE2S-256", HashKind::Blake2s, 32, 32},
    {"BLAKE3-256", HashKind::Blake3, 32, 32},
    {"BLAKE3-256-128", HashKind::Blake3, 32, 16},
    {"HMAC-SHA224", HashKind::HmacSha224, 0, 28},
    {"HMAC-SHA256", HashKind::HmacSha256, 0, 32},
    {"HMAC-SHA256-128", HashKind::HmacSha256, 0, 16},
    {"HMAC-SHA3-224", HashKind::HmacSha3_224, 0, 28},
    {"HMAC-SHA3-256", HashKind::HmacSha3_256, 0, 32},
};
const HashAlgo* find_hash(const char* name) {
    if (!name) return nullptr;
    for (const HashAlgo& h : kHashAlgos)
        if (std::strcmp(h.name, name) == 0) return &h;
    return nullptr;
}

// ---- host-side key preparation (per launch, a few blocks): HMAC midstates, BLAKE3 key derivation
constexpr uint32_t kSha256IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
constexpr uint32_t kSha224IV[8] = {0xc1059ed8u, 0x367cd507u, 0x3070dd17u, 0xf70e5939u,
                                   0xffc00b31u, 0x68581511u, 0x64f98fa7u, 0xbefa4fa4u};

void sha256_block_bytes(uint32_t (&h)[8], const uint8_t* b) {
    uint32_t w[16];
    for (int j = 0; j < 16; j++)
        w[j] = (uint32_t(b[4 * j]) << 24) | (uint32_t(b[4 * j + 1]) << 16) | (uint32_t(b[4 * j + 2]) << 8) | b[4 * j + 3];
    hashdev::sha256_block(h, w);
}

// SHA-256 / SHA-224 of a short message (a long HMAC key): FIPS 180-4 padding.
void sha2_host(bool is224, const uint8_t* m, size_t n, uint8_t* digest) {
    uint32_t h[8];
    for (int j = 0; j < 8; j++) h[j] = is224 ? kSha224IV[j] : kSha256IV[j];
    size_t i = 0;
    for (; i + 64 <= n; i += 64) sha256_block_bytes(h, m + i);
    uint8_t blk[128] = {};
    const size_t r = n - i;
    std::memcpy(blk, m + i, r);
    blk[r] = 0x80;
    const size_t tot = r < 56 ? 64 : 128;
    const uint64_t bits = static_cast<uint64_t>(n) * 8;
    for (int j = 0; j < 8; j++) blk[tot - 1 - j] = static_cast<uint8_t>(bits >> (8 * j));
    sha256_block_bytes(h, blk);
    if (tot == 128) sha256_block_bytes(h, blk + 64);
    const int dw = is224 ? 7 : 8;
    for (int j = 0; j < dw; j++)
        for (int k = 0; k < 4; k++) digest[4 * j + k] = static_cast<uint8_t>(h[j] >> (24 - 8 * k));
}

void keccak_f_host(uint64_t (&s)[25]) {
    for (int r = 0; r < 24; r++) {
        uint64_t C[5], D[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ ((C[(x + 1) % 5] << 1) | (C[(x + 1) % 5] >> 63));
        for (int k = 0; k < 25; k++) {
            const uint64_t v = s[k] ^ D[k % 5];
            const int rho = hashdev::kKeccakRho[k];
            B[hashdev::keccak_pi_dst(k)] = rho ? (v << rho) | (v >> (64 - rho)) : v;
        }
        for (int y = 0; y < 25; y += 5)
            for (int x = 0; x < 5; x++) s[y + x] = B[y + x] ^ (~B[y + (x + 1) % 5] & B[y + (x + 2) % 5]);
        s[0] ^= hashdev::kKeccakRC[r];
    }
}
void keccak_absorb_block(uint64_t (&s)[25], const uint8_t* b, size_t rate) {
    for (size_t j = 0; j < rate / 8; j++) {
        uint64_t w = 0;
        for (int k = 0; k < 8; k++) w |= static_cast<uint64_t>(b[8 * j + k]) << (8 * k);
        s[j] ^= w;
    }
    keccak_f_host(s);
}
// SHA3-224 / SHA3-256 of a short message (a long HMAC key): FIPS 202.
void sha3_host(size_t rate, size_t db, const uint8_t* m, size_t n, uint8_t* digest) {
    uint64_t s[25] = {};
    size_t i = 0;
    for (; i + rate <= n; i += rate) keccak_absorb_block(s, m + i, rate);
    uint8_t blk[200] = {};
    std::memcpy(blk, m + i, n - i);
    blk[n - i] ^= 0x06;
    blk[rate - 1] ^= 0x80;
    keccak_absorb_block(s, blk, rate);
    for (size_t k = 0; k < db; k++) digest[k] = static_cast<uint8_t>(s[k / 8] >> (8 * (k % 8)));
}

// HMAC key block K0 (RFC 2104 / FIPS 198-1): the key, hashed first when longer than the block.
void hmac_k0(const HashAlgo& h, const uint8_t* key, uint32_t key_len, size_t block, uint8_t* k0) {
    std::memset(k0, 0, block);
    if (key_len <= block) {
        if (key_len) std::memcpy(k0, key, key_len);
        return;
    }
    switch (h.kind) {
        case HashKind::HmacSha256: sha2_host(false, key, key_len, k0); break;
        case HashKind::HmacSha224: sha2_host(true, key, key_len, k0); break;
        case HashKind::HmacSha3_224: sha3_host(144, 28, key, key_len, k0); break;
        default: sha3_host(136, 32, key, key_len, k0); break;
    }
}

// BLAKE3 (host, short inputs): the hash of `m` under key words `kw` and mode flags `mode`
// (KEYED_HASH, DERIVE_KEY_CONTEXT, DERIVE_KEY_MATERIAL); recursive left-complete tree.
void b3_words(const uint8_t* b, uint32_t len, uint32_t (&m)[16]) {
    for (int j = 0; j < 16; j++) {
        m[j] = 0;
        for (int k = 0; k < 4; k++)
            if (4u * j + k < len) m[j] |= static_cast<uint32_t>(b[4 * j + k]) << (8 * k);
    }
}
void b3_chunk_host(const uint32_t (&kw)[8], const uint8_t* m, size_t n, uint64_t ctr, uint32_t mode, bool root,
                   uint32_t (&cv)[8]) {
    for (int j = 0; j < 8; j++) cv[j] = kw[j];
    const size_t nb = n ? (n + 63) / 64 : 1;
    for (size_t b = 0; b < nb; b++) {
        const uint32_t take = static_cast<uint32_t>(n - 64 * b < 64 ? n - 64 * b : 64);
        uint32_t w[16], o[8];
        b3_words(m + 64 * b, take, w);
        const uint32_t fl = mode | (b == 0 ? hashdev::kB3ChunkStart : 0u) |
                            (b + 1 == nb ? (hashdev::kB3ChunkEnd | (root ? hashdev::kB3Root : 0u)) : 0u);
        hashdev::b3_compress(cv, w, ctr, take, fl, o);
        for (int j = 0; j < 8; j++) cv[j] = o[j];
    }
}
void b3_subtree_host(const uint32_t (&kw)[8], const uint8_t* m, size_t n, uint64_t ctr0, uint32_t mode, bool root,
                     uint32_t (&cv)[8]) {
    const size_t nch = n ? (n + 1023) / 1024 : 1;
    if (nch == 1) return b3_chunk_host(kw, m, n, ctr0, mode, root, cv);
    size_t left = 1;
    while (2 * left < nch) left *= 2;  // the largest power of two below nch chunks
    uint32_t l[8], r[8], w[16];
    b3_subtree_host(kw, m, 1024 * left, ctr0, mode, false, l);
    b3_subtree_host(kw, m + 1024 * left, n - 1024 * left, ctr0 + left, mode, false, r);
    for (int j = 0; j < 8; j++) {
        w[j] = l[j];
        w[8 + j] = r[j];
    }
    hashdev::b3_compress(kw, w, 0, 64, mode | hashdev::kB3Parent | (root ? hashdev::kB3Root : 0u), cv);
}
constexpr uint32_t kB3DeriveContext = 32, kB3DeriveMaterial = 64;
// blake3.DeriveKey(context, material, out[:32])
void b3_derive_key(const char* context, const uint8_t* material, size_t n, uint32_t (&key)[8]) {
    uint32_t iv[8], ck[8];
    for (int j = 0; j < 8; j++) iv[j] = hashdev::kIV32[j];
    b3_subtree_host(iv, reinterpret_cast<const uint8_t*>(context), std::strlen(context), 0, kB3DeriveContext, true, ck);
    b3_subtree_host(ck, material, n, 0, kB3DeriveMaterial, true, key);
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
    const bool blake2 = h->kind == HashKind::Blake2b || h->kind == HashKind::Blake2s;
    if (key_len && !key) return set_error(-22, "null key");
    if (blake2) {
        // blake2b.New256 / blake2s.New*: at most 64 / 32 key bytes; BLAKE2s-128 needs a key
        // (golang.org/x/crypto/blake2s New128 rejects an empty one), as CreateHashFunc reports.
        if (key_len > (h->kind == HashKind::Blake2b ? 64u : 32u)) return set_error(-22, "hash key too long");
        if (h->kind == HashKind::Blake2s && h->nn == 16 && key_len == 0)
            return set_error(-22, "BLAKE2S-128 requires a key");
    }
    if (out_stride < h->out || out_stride % 4) return set_error(-22, "out_stride must be >= the hash size and a multiple of 4");
    if (nchunks == 0) return 0;
    if (!d_data || !d_offsets || !d_lens || !d_out) return set_error(-22, "null argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 block(256), grid((nchunks + 255) / 256);
    auto launched = [&]() {
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : set_error(-5, std::string("hash kernel launch: ") + hipGetErrorString(e));
    };
    switch (h->kind) {
        case HashKind::HmacSha256:
        case HashKind::HmacSha224: {
            const bool is224 = h->kind == HashKind::HmacSha224;
            uint8_t k0[64], pad[64];
            hmac_k0(*h, key, key_len, 64, k0);
            hashdev::ShaMid mid{};
            for (int j = 0; j < 8; j++) mid.in[j] = mid.out[j] = is224 ? kSha224IV[j] : kSha256IV[j];
            for (int j = 0; j < 64; j++) pad[j] = k0[j] ^ 0x36u;
            sha256_block_bytes(mid.in, pad);
            for (int j = 0; j < 64; j++) pad[j] = k0[j] ^ 0x5cu;
            sha256_block_bytes(mid.out, pad);
            if (is224)
                hipLaunchKernelGGL(hashdev::hmac_sha256_kernel<7>, grid, block, 0, st, d_data, d_offsets, d_lens, d_order,
                                   nchunks, mid, h->out, out_stride, d_out);
            else
                hipLaunchKernelGGL(hashdev::hmac_sha256_kernel<8>, grid, block, 0, st, d_data, d_offsets, d_lens, d_order,
                                   nchunks, mid, h->out, out_stride, d_out);
            return launched();
        }
        case HashKind::HmacSha3_224:
        case HashKind::HmacSha3_256: {
            const bool is224 = h->kind == HashKind::HmacSha3_224;
            const size_t rate = is224 ? 144 : 136;
            uint8_t k0[144], pad[144];
            hmac_k0(*h, key, key_len, rate, k0);
            hashdev::KeccakMid mid{};
            for (size_t j = 0; j < rate; j++) pad[j] = k0[j] ^ 0x36u;
            keccak_absorb_block(mid.in, pad, rate);
            for (size_t j = 0; j < rate; j++) pad[j] = k0[j] ^ 0x5cu;
            keccak_absorb_block(mid.out, pad, rate);
            if (is224)
                hipLaunchKernelGGL((hashdev::hmac_sha3_kernel<144, 28>), grid, block, 0, st, d_data, d_offsets, d_lens,
                                   d_order, nchunks, mid, h->out, out_stride, d_out);
            else
                hipLaunchKernelGGL((hashdev::hmac_sha3_kernel<136, 32>), grid, block, 0, st, d_data, d_offsets, d_lens,
                                   d_order, nchunks, mid, h->out, out_stride, d_out);
            return launched();
        }
        case HashKind::Blake3: {
            // blake3_hashes.go:10-22: a secret under 32 bytes is stretched with DeriveKey; otherwise
            // its first 32 bytes are the key
            hashdev::B3Key k{};
            if (key_len < 32) {
                b3_derive_key("kopia blake3 derived key v1", key, key_len, k.k);
            } else {
                for (int j = 0; j < 8; j++)
                    k.k[j] = uint32_t(key[4 * j]) | (uint32_t(key[4 * j + 1]) << 8) | (uint32_t(key[4 * j + 2]) << 16) |
                             (uint32_t(key[4 * j + 3]) << 24);
            }
            const dim3 g3((nchunks + hashdev::kB3Waves - 1) / hashdev::kB3Waves), b3(64 * hashdev::kB3Waves);
            hipLaunchKernelGGL(hashdev::blake3_keyed_kernel, g3, b3, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                               k, h->out, out_stride, d_out);
            return launched();
        }
        default: break;
    }
    hashdev::HashKey k{};
    k.kk = key_len;
    for (uint32_t i = 0; i < key_len; i++) k.w[i / 4] |= static_cast<uint32_t>(key[i]) << (8 * (i % 4));
    const bool b64 = h->kind == HashKind::Blake2b;
    // Four lanes per chunk unless the launch holds over 2^20 chunks (64 waves per SIMD, where
    // the one-lane kernel's ~25 % lower VALU per block would matter).  Measured on config-2
    // chunk tables: 5,705 chunks 84 vs 540 ms, 136,920 chunks 263 vs 630 ms (one lane per
    // chunk leaves a dependent chain per lane with too few waves to interleave).
    const int forced = test_hash_lanes();
    const bool x4 = forced ? forced == 4 : nchunks <= (1u << 20);
    if (x4) {
        const dim3 grid4((4ull * nchunks + 255) / 256), block4(256);
        if (b64)
            hipLaunchKernelGGL(hashdev::blake2_chunks_x4_kernel<true>, grid4, block4, 0, st, d_data, d_offsets, d_lens,
                               d_order, nchunks, k, h->nn, h->out, out_stride, d_out);
        else
            hipLaunchKernelGGL(hashdev::blake2_chunks_x4_kernel<false>, grid4, block4, 0, st, d_data, d_offsets, d_lens,
                               d_order, nchunks, k, h->nn, h->out, out_stride, d_out);
        return launched();
    }
    if (b64)
        hipLaunchKernelGGL(hashdev::blake2b_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    else
        hipLaunchKernelGGL(hashdev::blake2s_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    return launched();
}

namespace kcdc {
int hash_chain_kind(const char* name, uint32_t* out_len) {
    const HashAlgo* h = find_hash(name);
    if (!h) return set_error(-2, std::string("unknown hash: ") + (name ? name : "(null)"));
    if (out_len) *out_len = h->out;
    return h->kind == HashKind::Blake2b ? 1 : h->kind == HashKind::Blake2s ? 2 : 3;
}

int launch_hash_chains(const char* name, const uint8_t* key, uint32_t key_len, HashChain* d_chains,
                       const HashChain* fresh, const uint32_t* d_active, uint32_t nactive, uint64_t max_blocks,
                       uint8_t* d_digests, uint32_t digest_stride, void* stream) {
    const HashAlgo* h = find_hash(name);
    if (!h || (h->kind != HashKind::Blake2b && h->kind != HashKind::Blake2s))
        return set_error(-22, "resumable chains: BLAKE2 names only");
    if (key_len > (h->kind == HashKind::Blake2b ? 64u : 32u)) return set_error(-22, "hash key too long");
    if (h->kind == HashKind::Blake2s && h->nn == 16 && key_len == 0) return set_error(-22, "BLAKE2S-128 requires a key");
    if (nactive == 0) return 0;
    hashdev::HashKey k{};
    k.kk = key_len;
    for (uint32_t i = 0; i < key_len; i++) k.w[i / 4] |= static_cast<uint32_t>(key[i]) << (8 * (i % 4));
    hipStream_t st = static_cast<hipStream_t>(stream);
    constexpr unsigned kT = hashdev::kChainWaves * 64;
    const dim3 block(kT), grid(static_cast<unsigned>((4ull * nactive + kT - 1) / kT));
    if (h->kind == HashKind::Blake2b)
        hipLaunchKernelGGL(hashdev::blake2_chain_step_kernel<true>, grid, block, 0, st, d_chains, fresh, d_active, nactive,
                           max_blocks, k, h->nn, h->out, digest_stride, d_digests);
    else
        hipLaunchKernelGGL(hashdev::blake2_chain_step_kernel<false>, grid, block, 0, st, d_chains, fresh, d_active, nactive,
                           max_blocks, k, h->nn, h->out, digest_stride, d_digests);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("hash chain launch: ") + hipGetErrorString(e));
}
}  // namespace kcdc
