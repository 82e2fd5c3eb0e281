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

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

// Words [0, nw) of the block at p (take valid bytes, the rest zero), from 4-byte-aligned
// loads that never leave the chunk's aligned words (a chunk may start at any byte).
template <int NW>
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t take, uint32_t (&d)[NW]) {
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
    d = rotr64(d ^ a, 32);
    c = c + d;
    b = rotr64(b ^ c, 24);
    a = a + b + y;
    d = rotr64(d ^ a, 16);
    c = c + d;
    b = rotr64(b ^ c, 63);
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

}  // namespace hashdev

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
    const dim3 grid((nchunks + 255) / 256), block(256);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (h->b64)
        hipLaunchKernelGGL(hashdev::blake2b_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    else
        hipLaunchKernelGGL(hashdev::blake2s_chunks_kernel, grid, block, 0, st, d_data, d_offsets, d_lens, d_order, nchunks,
                           k, h->nn, h->out, out_stride, d_out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("hash kernel launch: ") + hipGetErrorString(e));
}
