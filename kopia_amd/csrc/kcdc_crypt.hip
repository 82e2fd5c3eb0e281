// Kopia content encryption on gfx950: CHACHA20-POLY1305-HMAC-SHA256 (this
// header) and AES256-GCM-HMAC-SHA256, Kopia's default (the section "AES256-GCM-HMAC-SHA256"
// below: T-table AES-CTR and table-driven GHASH, same four-launch shape).
//
// What the reference does per content (repo/encryption/chacha20_poly1305_hmac_sha256_encryptor.go:24-80,
// aead_helpers.go:12-45, encryption.go:80-92, repo/content/content_manager_lock_free.go:178-182):
//   secret = HKDF-SHA256(masterKey, salt "encryption", info "", 32)        (once per repository)
//   iv     = last 16 bytes of the content hash (content ID)
//   key    = HMAC-SHA256(secret, iv)
//   output = nonce(12, crypto/rand) || ChaCha20-Poly1305.Seal(key, nonce, plaintext, aad = iv)
// The arithmetic is RFC 8439 (golang.org/x/crypto/chacha20poly1305; not vendored).
//
// Device layout: a chunk is cut into 4 KiB units; one wave owns one unit at a time
// (64 lanes x one 64-byte ChaCha20 block each).  Plaintext is loaded coalesced into LDS,
// each lane XORs its own keystream block, and the ciphertext goes back out coalesced.
// Poly1305 is a polynomial in r, so it is evaluated in parallel: each lane runs Horner
// over its 4 sixteen-byte blocks, the lane sums are scaled by r^e from a per-chunk table of
// powers of r and reduced across the wave, and the unit sum is scaled by r^Q (Q = its
// distance from the end of the message) and added into a per-chunk accumulator.  No byte
// of a chunk is visited twice and no chunk runs serially.  DESIGN.md §2.6 has the layout.
//
// Kernels, in stream order: crypt_prep (HMAC key, one-time Poly1305 key, power table),
// unit_scan (units per chunk -> prefix), crypt_units (the byte pass), crypt_finish (tag).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "kcdc_internal.h"

namespace kcdc {
namespace cryptdev {

constexpr uint32_t kUnit = 4096;                      // bytes per wave step
constexpr uint32_t kTabT = 0, kTabA = 256, kTabB = 320, kTabC = 384, kTabN = 448;  // r^a, r^256b, r^16384c, r^(2^20)d
constexpr uint64_t kMaxLen = (1ull << 30) - 64;       // exponents stay below 2^26
constexpr uint32_t kM26 = 0x3FFFFFFu;

struct Fe {  // element of GF(2^130 - 5), radix 2^26, limbs not fully reduced
    uint32_t v[5];
};

struct HmacMid {  // SHA-256 states after the (key ^ ipad) and (key ^ opad) blocks
    uint32_t in[8], out[8];
};

struct ChunkKey {  // 128 bytes per chunk
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t s[4];
    uint32_t r[5];
    uint32_t len_lo, len_hi;  // plaintext length
    uint32_t pad[10];
};
static_assert(sizeof(ChunkKey) == 128, "ChunkKey layout");

// ------------------------------------------------------------------ SHA-256 (host + device)
constexpr uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
constexpr uint32_t kSha256IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__host__ __device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__host__ __device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

__host__ __device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], const uint32_t (&m)[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = m[i];
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        if (i >= 16) {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            w[i & 15] += (ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3)) + w[(i - 7) & 15] +
                         (ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10));
        }
        const uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[i] + w[i & 15];
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

// ------------------------------------------------------------------ ChaCha20 (RFC 8439 §2.3)
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

#define KCDC_QR(a, b, c, d) \
    a += b;                 \
    d = rotl32(d ^ a, 16);  \
    c += d;                 \
    b = rotl32(b ^ c, 12);  \
    a += b;                 \
    d = rotl32(d ^ a, 8);   \
    c += d;                 \
    b = rotl32(b ^ c, 7);

__device__ __forceinline__ void chacha20_block(const uint32_t (&k)[8], uint32_t ctr, const uint32_t (&nc)[3],
                                               uint32_t (&o)[16]) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                             k[4],        k[5],        k[6],        k[7],        ctr,  nc[0], nc[1], nc[2]};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = in[i];
#pragma unroll
    for (int r = 0; r < 10; r++) {
        KCDC_QR(x[0], x[4], x[8], x[12]);
        KCDC_QR(x[1], x[5], x[9], x[13]);
        KCDC_QR(x[2], x[6], x[10], x[14]);
        KCDC_QR(x[3], x[7], x[11], x[15]);
        KCDC_QR(x[0], x[5], x[10], x[15]);
        KCDC_QR(x[1], x[6], x[11], x[12]);
        KCDC_QR(x[2], x[7], x[8], x[13]);
        KCDC_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = x[i] + in[i];
}
#undef KCDC_QR

// ------------------------------------------------------------------ GF(2^130 - 5) (RFC 8439 §2.5)
__device__ __forceinline__ Fe fe_zero() { return Fe{{0u, 0u, 0u, 0u, 0u}}; }
__device__ __forceinline__ Fe fe_one() { return Fe{{1u, 0u, 0u, 0u, 0u}}; }

// Inputs: limbs < 2^27 + 2^12 (a), normalized (b).  Output: limbs < 2^26 except v[1] < 2^26 + 2^11.
__device__ __forceinline__ Fe fe_mul(const Fe& a, const Fe& b) {
    const uint32_t s1 = b.v[1] * 5u, s2 = b.v[2] * 5u, s3 = b.v[3] * 5u, s4 = b.v[4] * 5u;
    auto m = [](uint32_t x, uint32_t y) { return static_cast<uint64_t>(x) * y; };
    uint64_t d0 = m(a.v[0], b.v[0]) + m(a.v[1], s4) + m(a.v[2], s3) + m(a.v[3], s2) + m(a.v[4], s1);
    uint64_t d1 = m(a.v[0], b.v[1]) + m(a.v[1], b.v[0]) + m(a.v[2], s4) + m(a.v[3], s3) + m(a.v[4], s2);
    uint64_t d2 = m(a.v[0], b.v[2]) + m(a.v[1], b.v[1]) + m(a.v[2], b.v[0]) + m(a.v[3], s4) + m(a.v[4], s3);
    uint64_t d3 = m(a.v[0], b.v[3]) + m(a.v[1], b.v[2]) + m(a.v[2], b.v[1]) + m(a.v[3], b.v[0]) + m(a.v[4], s4);
    uint64_t d4 = m(a.v[0], b.v[4]) + m(a.v[1], b.v[3]) + m(a.v[2], b.v[2]) + m(a.v[3], b.v[1]) + m(a.v[4], b.v[0]);
    Fe r;
    d1 += d0 >> 26;
    r.v[0] = static_cast<uint32_t>(d0) & kM26;
    d2 += d1 >> 26;
    r.v[1] = static_cast<uint32_t>(d1) & kM26;
    d3 += d2 >> 26;
    r.v[2] = static_cast<uint32_t>(d2) & kM26;
    d4 += d3 >> 26;
    r.v[3] = static_cast<uint32_t>(d3) & kM26;
    const uint64_t t = (d4 >> 26) * 5u + r.v[0];  // 2^130 = 5 (mod p)
    r.v[4] = static_cast<uint32_t>(d4) & kM26;
    r.v[0] = static_cast<uint32_t>(t) & kM26;
    r.v[1] += static_cast<uint32_t>(t >> 26);
    return r;
}

__device__ __forceinline__ Fe fe_add(const Fe& a, const Fe& b) {
    Fe r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}

// One carry pass: limbs < 2^31 in, < 2^26 out (v[1] < 2^26 + 2^7).
__device__ __forceinline__ Fe fe_carry(Fe a) {
    uint32_t c;
    c = a.v[0] >> 26;
    a.v[0] &= kM26;
    a.v[1] += c;
    c = a.v[1] >> 26;
    a.v[1] &= kM26;
    a.v[2] += c;
    c = a.v[2] >> 26;
    a.v[2] &= kM26;
    a.v[3] += c;
    c = a.v[3] >> 26;
    a.v[3] &= kM26;
    a.v[4] += c;
    c = a.v[4] >> 26;
    a.v[4] &= kM26;
    a.v[0] += c * 5u;
    c = a.v[0] >> 26;
    a.v[0] &= kM26;
    a.v[1] += c;
    return a;
}

// A 16-byte block (little-endian words) plus 2^128.
__device__ __forceinline__ Fe fe_block(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    Fe m;
    m.v[0] = w0 & kM26;
    m.v[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & kM26;
    m.v[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & kM26;
    m.v[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & kM26;
    m.v[4] = (w3 >> 8) | (1u << 24);
    return m;
}

// r^q from the chunk's power table, q < 2^26 (q = a + 256 b + 16384 c + 2^20 d).
__device__ __forceinline__ Fe fe_pow_tab(const Fe* tab, uint32_t q) {
    Fe p = tab[kTabT + (q & 255u)];
    if ((q >> 8) & 63u) p = fe_mul(p, tab[kTabA + ((q >> 8) & 63u)]);
    if ((q >> 14) & 63u) p = fe_mul(p, tab[kTabB + ((q >> 14) & 63u)]);
    if ((q >> 20) & 63u) p = fe_mul(p, tab[kTabC + ((q >> 20) & 63u)]);
    return p;
}

// (h mod p + s) mod 2^128 (RFC 8439 §2.5.1 final step).
__device__ __forceinline__ void fe_tag(Fe h, const uint32_t (&s)[4], uint32_t (&tag)[4]) {
    h = fe_carry(fe_carry(h));
    uint32_t g[5], c;
    g[0] = h.v[0] + 5u;
    c = g[0] >> 26;
    g[0] &= kM26;
#pragma unroll
    for (int i = 1; i < 4; i++) {
        g[i] = h.v[i] + c;
        c = g[i] >> 26;
        g[i] &= kM26;
    }
    g[4] = h.v[4] + c - (1u << 26);
    const uint32_t keep_g = (g[4] >> 31) - 1u;  // all ones when h >= p
#pragma unroll
    for (int i = 0; i < 5; i++) h.v[i] = (h.v[i] & ~keep_g) | (g[i] & keep_g);
    const uint32_t w0 = h.v[0] | (h.v[1] << 26);
    const uint32_t w1 = (h.v[1] >> 6) | (h.v[2] << 20);
    const uint32_t w2 = (h.v[2] >> 12) | (h.v[3] << 14);
    const uint32_t w3 = (h.v[3] >> 18) | (h.v[4] << 8);
    uint64_t f = static_cast<uint64_t>(w0) + s[0];
    tag[0] = static_cast<uint32_t>(f);
    f = static_cast<uint64_t>(w1) + s[1] + (f >> 32);
    tag[1] = static_cast<uint32_t>(f);
    f = static_cast<uint64_t>(w2) + s[2] + (f >> 32);
    tag[2] = static_cast<uint32_t>(f);
    f = static_cast<uint64_t>(w3) + s[3] + (f >> 32);
    tag[3] = static_cast<uint32_t>(f);
}

__device__ __forceinline__ uint32_t load_le32_bytes(const uint8_t* p) {
    return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) | (static_cast<uint32_t>(p[2]) << 16) |
           (static_cast<uint32_t>(p[3]) << 24);
}

__device__ __forceinline__ uint32_t keep_mask(int64_t keep) {  // low `keep` bytes of a word
    return keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * keep));
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct CryptArgs {
    uint32_t n;
    const uint8_t* in;          // seal: plaintext base; open: sealed base
    const uint64_t* in_offs;
    const uint64_t* in_lens;    // seal: plaintext lengths; open: sealed lengths
    uint8_t* out;               // seal: sealed base; open: plaintext base
    const uint64_t* out_offs;   // multiples of 4
    const uint8_t* ivs;         // iv_len bytes per chunk at ivs + i * iv_stride (the content ID)
    uint32_t iv_len;            // 1..64
    uint32_t iv_stride;
    const uint8_t* nonces;      // seal: 12 bytes per chunk
    int32_t* status;            // per chunk: 0, or a negative errno
    ChunkKey* keys;
    Fe* tabs;                   // kTabN powers of r per chunk
    unsigned long long* acc;    // 5 limb sums per chunk
    uint32_t* units;            // n + 1: units per chunk, then their exclusive prefix
    HmacMid mid;
};

// HMAC-SHA256(secret, id) from the secret's midstates: the per-content key of both encryptors
// (chacha20_poly1305_hmac_sha256_encryptor.go:24-48, aes256_gcm_hmac_sha256_encryptor.go:24-47).
__device__ __forceinline__ void hmac_key(const HmacMid& mid, const uint8_t* ivp, uint32_t il, uint32_t (&key)[8]) {
    // HMAC-SHA256(secret, id): after the (key ^ ipad) block, id || 0x80 || 0.. || bit length
    // fills one block (id <= 55 bytes) or two; the outer hash is digest || pad (96 bytes).
    
    uint32_t blk[32];
#pragma unroll
    for (int j = 0; j < 32; j++) blk[j] = 0;
#pragma unroll
    for (uint32_t i = 0; i < 65; i++) {
        const uint32_t b = i < il ? static_cast<uint32_t>(ivp[i < 64 ? i : 63]) : (i == il ? 0x80u : 0u);
        blk[i >> 2] |= b << (24 - 8 * (i & 3));
    }
    const bool two = il > 55u;
    const uint32_t bits = (64u + il) * 8u;
    if (two) blk[31] = bits;
    else blk[15] = bits;
    uint32_t h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = mid.in[j];
    {
        uint32_t b0[16];
#pragma unroll
        for (int j = 0; j < 16; j++) b0[j] = blk[j];
        sha256_compress(h, b0);
        if (two) {
#pragma unroll
            for (int j = 0; j < 16; j++) b0[j] = blk[16 + j];
            sha256_compress(h, b0);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) blk[j] = h[j];
    blk[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; j++) blk[j] = 0;
    blk[15] = 96u * 8u;
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = mid.out[j];
    {
        uint32_t b0[16];
#pragma unroll
        for (int j = 0; j < 16; j++) b0[j] = blk[j];
        sha256_compress(h, b0);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) key[j] = bswap32(h[j]);
}

// One wave per chunk: key, one-time Poly1305 key, power table; every lane computes the
// (wave-uniform) key schedule and then its own table entries.
template <bool kOpen>
__global__ __launch_bounds__(256) void crypt_prep_kernel(CryptArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (c >= a.n) return;
    const uint64_t in_len = a.in_lens[c];
    const bool bad = kOpen ? (in_len < 28u || in_len - 28u > kMaxLen) : in_len > kMaxLen;
    const uint64_t len = bad ? 0 : (kOpen ? in_len - 28u : in_len);
    const uint8_t* ivp = a.ivs + static_cast<uint64_t>(c) * a.iv_stride;
    const uint8_t* np = kOpen ? a.in + a.in_offs[c] : a.nonces + 12ull * c;
    uint32_t nonce[3] = {0u, 0u, 0u};
    if (!(kOpen && bad)) {
#pragma unroll
        for (int j = 0; j < 3; j++) nonce[j] = load_le32_bytes(np + 4 * j);
    }
    uint32_t key[8];
    hmac_key(a.mid, ivp, a.iv_len, key);
    uint32_t ks[16];
    chacha20_block(key, 0u, nonce, ks);  // block 0 -> Poly1305 one-time key (RFC 8439 §2.6)
    const uint32_t r0 = ks[0] & 0x0FFFFFFFu, r1 = ks[1] & 0x0FFFFFFCu, r2 = ks[2] & 0x0FFFFFFCu, r3 = ks[3] & 0x0FFFFFFCu;
    Fe r;
    r.v[0] = r0 & kM26;
    r.v[1] = __builtin_amdgcn_alignbit(r1, r0, 26) & kM26;
    r.v[2] = __builtin_amdgcn_alignbit(r2, r1, 20) & kM26;
    r.v[3] = __builtin_amdgcn_alignbit(r3, r2, 14) & kM26;
    r.v[4] = r3 >> 8;
    uint32_t rec[32];
#pragma unroll
    for (int j = 0; j < 8; j++) rec[j] = key[j];
#pragma unroll
    for (int j = 0; j < 3; j++) rec[8 + j] = nonce[j];
#pragma unroll
    for (int j = 0; j < 4; j++) rec[11 + j] = ks[4 + j];
#pragma unroll
    for (int j = 0; j < 5; j++) rec[15 + j] = r.v[j];
    rec[20] = static_cast<uint32_t>(len);
    rec[21] = static_cast<uint32_t>(len >> 32);
#pragma unroll
    for (int j = 22; j < 32; j++) rec[j] = 0;
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < 32; j++)
        if (lane == static_cast<uint32_t>(j)) mine = rec[j];
    if (lane < 32u) reinterpret_cast<uint32_t*>(a.keys + c)[lane] = mine;

    // Power table: lane l writes r^l, r^(64+l), r^(128+l), r^(192+l), r^(256 l), r^(16384 l), r^(2^20 l).
    Fe* tab = a.tabs + static_cast<uint64_t>(c) * kTabN;
    auto pow_lane = [&](Fe base, Fe& base_out) {  // base^lane, and base^64
        Fe p = fe_one();
#pragma unroll
        for (int b = 0; b < 6; b++) {
            const Fe q = fe_mul(p, base);
            if ((lane >> b) & 1u) p = q;
            base = fe_mul(base, base);
        }
        base_out = base;
        return p;
    };
    Fe r64, r16384, r2_20, unused;
    const Fe t0 = pow_lane(r, r64);
    const Fe r128 = fe_mul(r64, r64);
    const Fe r256 = fe_mul(r128, r128);
    tab[kTabT + lane] = t0;
    tab[kTabT + 64 + lane] = fe_mul(t0, r64);
    const Fe t128 = fe_mul(t0, r128);
    tab[kTabT + 128 + lane] = t128;
    tab[kTabT + 192 + lane] = fe_mul(t128, r64);
    tab[kTabA + lane] = pow_lane(r256, r16384);
    tab[kTabB + lane] = pow_lane(r16384, r2_20);
    tab[kTabC + lane] = pow_lane(r2_20, unused);
    if (lane < 5u) a.acc[5ull * c + lane] = 0ull;
    if (lane == 0) {
        a.units[c] = static_cast<uint32_t>((len + kUnit - 1) / kUnit);
        a.status[c] = bad ? (kOpen && in_len < 28u ? -22 : -27) : 0;  // EINVAL / EFBIG
    }
    if (!kOpen && lane < 3u) reinterpret_cast<uint32_t*>(a.out + a.out_offs[c])[lane] = nonce[lane];
}

// Exclusive prefix of units[0..n) in place; units[n] = total.  One workgroup.
__global__ __launch_bounds__(1024) void unit_scan_kernel(uint32_t n, uint32_t* units) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t b = static_cast<uint64_t>(n) * t / 1024u, e = static_cast<uint64_t>(n) * (t + 1) / 1024u;
    uint32_t s = 0;
    for (uint64_t i = b; i < e; i++) s += units[i];
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
        const uint32_t u = units[i];
        units[i] = run;
        run += u;
    }
    if (t == 1023u) units[n] = part[1023];
}

// LDS word index of unit word i: 16-byte slot s = i/4 lives at slot s ^ ((s >> 4) & 3), so
// both the coalesced view (lane l, word 64k + l) and the lane-own view (lane l, slots
// 4l..4l+3) are free of bank conflicts.
__device__ __forceinline__ uint32_t swz(uint32_t i) {
    const uint32_t s = i >> 2;
    return ((s ^ ((s >> 4) & 3u)) << 2) | (i & 3u);
}

// LDS-DMA (buffer_load_dwordx4 ... lds): 64 lanes x 16 bytes -> LDS bytes [m0, m0 + 1 KiB),
// lane d at m0 + 16 d.  Inline asm, so the compiler's waitcnt pass never waits on it; every
// read of a slot follows an explicit s_waitcnt.  nt: each source byte is read once.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(const_cast<void*>(p)))));
}
__device__ __forceinline__ void dma16(const u32x4& d, uint32_t m0, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds" ::"s"(m0), "v"(voff),
                 "s"(d)
                 : "memory");
}

// Slot layout (4 KiB + one 16-byte tail granule per unit): the unit's aligned 16-byte
// granule g sits at position pos(g) = g with its low 2 bits XORed by (g >> 4) & 3, so lane
// l's reads of granules 4l..4l+4 and the coalesced word view (swz) are both conflict free.
constexpr uint32_t kSlotBytes = kUnit + 32;

// The byte pass: persistent waves, each over a contiguous range of (chunk, unit) pairs.
// Unit u+1 is fetched into the wave's other LDS slot by DMA while unit u's keystream is
// computed, so the ~1,000 VALU of ChaCha20 per lane hide the HBM latency.
// Poly1305 over a run of consecutive full units of one chunk stays per lane: lane l holds
// blocks 4l..4l+3 of every unit, 253 blocks apart from one unit to the next, so it runs
// Horner as acc = acc r^253 + m0, then acc r + m1..m3.  The run is folded into the chunk
// sum (lane l scaled by r^(4(63-l)), reduced across the wave, scaled by r^Q) only when the
// chunk or the wave's range ends, or at the chunk's partial last unit.
constexpr int kCryptWaves = 4;  // waves per SIMD: 127 VGPRs, no VGPR spills; seal 3.08-3.12 vs 3.17-3.20 ms at 3
template <bool kOpen>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kCryptWaves, kCryptWaves))) void crypt_units_kernel(
    CryptArgs a, const ChunkKey* __restrict__ keys, const uint32_t* __restrict__ units,
    const uint64_t* __restrict__ in_offs, const uint64_t* __restrict__ out_offs, const Fe* __restrict__ tabs,
    uint8_t* __restrict__ out, unsigned long long* __restrict__ acc) {
    // The arrays come as separate __restrict__ arguments: the output stores then cannot
    // clobber them, so their wave-uniform reads are scalar loads.  As vector loads every one
    // carried a vmcnt wait that drained the in-flight prefetch and the previous stores.
    __shared__ __attribute__((aligned(16))) uint8_t lds[4][2][kSlotBytes];
    // wave index made visibly uniform: the unit walk, the chunk record and its key stay in SGPRs
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t total = units[a.n];
    const uint64_t W = static_cast<uint64_t>(gridDim.x) * 4u, w = static_cast<uint64_t>(blockIdx.x) * 4u + wv;
    uint32_t u = static_cast<uint32_t>(total * w / W);
    const uint32_t u1 = static_cast<uint32_t>(total * (w + 1) / W);
    if (u >= u1) return;
    uint32_t lo = 0, hi = a.n;  // units[lo] <= u < units[hi]
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (units[mid] <= u) lo = mid;
        else hi = mid;
    }
    const uint32_t slot_addr[2] = {lds_addr(lds[wv][0]), lds_addr(lds[wv][1])};
    const uint32_t hdr_in = kOpen ? 12u : 0u, hdr_out = kOpen ? 0u : 12u;

    // DMA of unit uq of chunk cq into slot sl; returns the unit's start offset in its first granule.
    auto issue = [&](uint32_t cq, uint32_t uq, uint32_t sl) -> uint32_t {
        const ChunkKey& k = keys[cq];
        const uint64_t lq = static_cast<uint64_t>(k.len_lo) | (static_cast<uint64_t>(k.len_hi) << 32);
        const uintptr_t chunk = reinterpret_cast<uintptr_t>(a.in + in_offs[cq] + hdr_in);
        const uintptr_t src = chunk + static_cast<uint64_t>(uq) * kUnit;
        const uintptr_t b16 = src & ~uintptr_t(15);
        uint64_t nrec = ((chunk + lq + 15u) & ~uintptr_t(15)) - b16;  // granules holding chunk bytes
        if (nrec > kUnit + 16u) nrec = kUnit + 16u;
        u32x4 d;
        d.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b16));
        d.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b16 >> 32) & 0xFFFFu);  // stride 0
        d.z = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nrec));
        d.w = 0x00020000u;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t p = 64u * i + lane;
            dma16(d, slot_addr[sl] + 1024u * i, 16u * ((p & ~3u) | ((p & 3u) ^ ((p >> 4) & 3u))));
        }
        if (lane == 0) dma16(d, slot_addr[sl] + kUnit, 16u * 256u);  // tail granule -> position 256
        return static_cast<uint32_t>(src & 15u);
    };

    uint32_t c = lo;
    uint64_t nct = 0;        // 16-byte blocks of chunk c
    Fe accum = fe_zero();    // chunk c's share from this wave, scaled to the message end
    Fe run = fe_zero();      // this lane's Horner value over the current run of full units
    uint32_t run_end = ~0u;  // unit index (within chunk c) of the run's last unit; ~0u: no run

    auto wave_sum = [&](Fe h) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            Fe o;
#pragma unroll
            for (int j = 0; j < 5; j++) o.v[j] = __shfl_xor(h.v[j], off, 64);
            h = fe_carry(fe_add(h, o));
        }
        return h;
    };
    auto fold_run = [&]() {
        if (run_end == ~0u) return;
        const Fe* tab = tabs + static_cast<uint64_t>(c) * kTabN;
        const Fe h = wave_sum(fe_mul(run, tab[kTabT + 4u * (63u - lane)]));
        const uint32_t q = static_cast<uint32_t>(nct + 1u - (static_cast<uint64_t>(run_end) * 256u + 255u));
        accum = fe_carry(fe_add(accum, fe_mul(h, fe_pow_tab(tab, q))));
        run = fe_zero();
        run_end = ~0u;
    };
    auto flush = [&]() {
        unsigned long long* dst = acc + 5ull * c;
#pragma unroll
        for (uint32_t j = 0; j < 5; j++)
            if (lane == j) atomicAdd(dst + j, static_cast<unsigned long long>(accum.v[j]));
        accum = fe_zero();
    };

    uint32_t sl = 0;
    uint32_t mis = issue(c, u - units[c], 0);
    uint32_t cn = c;  // chunk of unit u + 1
    bool prev_full = false;  // the previous iteration was a full unit (16 stores, no other vector memory op)
    for (; u < u1; u++, sl ^= 1u) {
        bool exact = prev_full;
        if (units[c + 1] <= u) {
            fold_run();
            flush();
            exact = false;
            do c++;
            while (units[c + 1] <= u);
        }
        // 1. prefetch unit u + 1 into the other slot (its previous unit's reads are done)
        const bool more = u + 1u < u1;
        uint32_t mis_next = 0;
        if (more) {
            if (cn < c) cn = c;
            while (units[cn + 1] <= u + 1u) cn++;
            mis_next = issue(cn, u + 1u - units[cn], sl ^ 1u);
        }
        const ChunkKey& ck = keys[c];
        const uint64_t len = static_cast<uint64_t>(ck.len_lo) | (static_cast<uint64_t>(ck.len_hi) << 32);
        nct = (len + 15u) >> 4;
        const uint32_t uu = u - units[c];
        const uint64_t ub = static_cast<uint64_t>(uu) * kUnit;
        const uint32_t rem = static_cast<uint32_t>(len - ub < kUnit ? len - ub : kUnit);
        const bool full = rem == kUnit;
        uint32_t* dst = reinterpret_cast<uint32_t*>(out + out_offs[c] + hdr_out + ub);

        // 2. this lane's keystream block (counter 1 + byte offset / 64), under the DMAs
        uint32_t ks[16];
        {
            uint32_t kk[8], nc[3];
#pragma unroll
            for (int j = 0; j < 8; j++) kk[j] = ck.key[j];
#pragma unroll
            for (int j = 0; j < 3; j++) nc[j] = ck.nonce[j];
            chacha20_block(kk, 1u + uu * 64u + lane, nc, ks);
        }
        // 3. wait for this unit's DMA (only the prefetch may stay in flight), read this lane's
        //    bytes [64 lane + mis, +64) from granules 4 lane .. 4 lane + 4
        //    In steady state exactly the previous unit's 16 stores and the 5 prefetch DMAs
        //    were issued after this unit's DMA; otherwise wait for everything but the prefetch.
        if (exact) {
            if (more) asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else {
            if (more) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        uint8_t* S = lds[wv][sl];
        const uint32_t sw = (lane >> 2) & 3u;
        uint32_t q[20];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint4 g = *reinterpret_cast<const uint4*>(S + 16u * (4u * lane + (t ^ sw)));
            q[4 * t] = g.x;
            q[4 * t + 1] = g.y;
            q[4 * t + 2] = g.z;
            q[4 * t + 3] = g.w;
        }
        {
            const uint32_t l1 = lane + 1u;
            const uint4 g = *reinterpret_cast<const uint4*>(S + 16u * (4u * l1 + ((l1 >> 2) & 3u)));
            q[16] = g.x;
            q[17] = g.y;
            q[18] = g.z;
            q[19] = g.w;
        }
        uint32_t d[16], res[16];
        {
            const uint32_t sh = 8u * (mis & 3u);
            switch (mis >> 2) {  // wave-uniform word offset
#define KCDC_FUNNEL(W0)                                                                         \
    case W0:                                                                                    \
        _Pragma("unroll") for (int j = 0; j < 16; j++) d[j] =                                   \
            __builtin_amdgcn_alignbit(q[j + W0 + 1 < 20 ? j + W0 + 1 : 19], q[j + W0], sh); \
        break;
                KCDC_FUNNEL(0)
                KCDC_FUNNEL(1)
                KCDC_FUNNEL(2)
                default:
                    KCDC_FUNNEL(3)
#undef KCDC_FUNNEL
            }
        }
        if (!full) {  // zero past the chunk end (the granules hold whatever follows it)
#pragma unroll
            for (int j = 0; j < 16; j++) d[j] &= keep_mask(static_cast<int64_t>(rem) - 64 * static_cast<int64_t>(lane) - 4 * j);
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
            res[j] = d[j] ^ ks[j];
            if (!full) res[j] &= keep_mask(static_cast<int64_t>(rem) - 64 * static_cast<int64_t>(lane) - 4 * j);
        }
        // 4. result -> this slot in the lane-own layout (every lane has read its granules)
        wave_lds_sync();
#pragma unroll
        for (int t = 0; t < 4; t++)
            *reinterpret_cast<uint4*>(S + 16u * (4u * lane + (t ^ sw))) =
                make_uint4(res[4 * t], res[4 * t + 1], res[4 * t + 2], res[4 * t + 3]);

        // 5. Poly1305 over this unit's ciphertext blocks (zero padded to 16 bytes)
        const uint32_t* m = kOpen ? d : res;
        Fe r;
#pragma unroll
        for (int j = 0; j < 5; j++) r.v[j] = ck.r[j];
        const Fe* tab = tabs + static_cast<uint64_t>(c) * kTabN;
        if (full) {
            run = fe_add(fe_mul(run, tab[kTabT + 253u]), fe_block(m[0], m[1], m[2], m[3]));
#pragma unroll
            for (int t = 1; t < 4; t++)
                run = fe_add(fe_mul(run, r), fe_block(m[4 * t], m[4 * t + 1], m[4 * t + 2], m[4 * t + 3]));
            run_end = uu;
        } else {
            // the chunk's last unit: lanes past the end add nothing; the unit sum is relative
            // to its last block j_end, whose exponent is Nct + 1 - j_end
            fold_run();
            const uint32_t nreal = (rem + 15u) >> 4, j0 = 4u * lane;
            Fe hl = fe_zero();
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const Fe nx = fe_add(fe_mul(hl, r), fe_block(m[4 * t], m[4 * t + 1], m[4 * t + 2], m[4 * t + 3]));
                if (j0 + t < nreal) hl = nx;
            }
            if (j0 < nreal) hl = fe_mul(hl, tab[kTabT + (nreal - 1u - min(j0 + 3u, nreal - 1u))]);
            else hl = fe_zero();
            hl = wave_sum(hl);
            const uint32_t qe = static_cast<uint32_t>(nct + 1u - (static_cast<uint64_t>(uu) * 256u + nreal - 1u));
            accum = fe_carry(fe_add(accum, fe_mul(hl, fe_pow_tab(tab, qe))));
        }
        wave_lds_sync();

        // 6. coalesced store; the zero tail of a partial last word stays inside the tag
        //    (seal) or the 4-byte padding of the plaintext slot (open)
        const uint32_t* Sw = reinterpret_cast<const uint32_t*>(S);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t i = 64u * k + lane;
            if (full || 4u * i < rem) dst[i] = Sw[swz(i)];
        }
        wave_lds_sync();
        mis = mis_next;
        prev_full = full;
    }
    fold_run();
    flush();
}

// One lane per chunk: add the AAD and length blocks, finish the tag, write or check it.
template <bool kOpen>
__global__ __launch_bounds__(256) void crypt_finish_kernel(CryptArgs a) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.n || a.status[c] != 0) return;
    const ChunkKey& ck = a.keys[c];
    const uint64_t len = static_cast<uint64_t>(ck.len_lo) | (static_cast<uint64_t>(ck.len_hi) << 32);
    const uint64_t nct = (len + 15u) >> 4;
    const Fe* tab = a.tabs + static_cast<uint64_t>(c) * kTabN;
    Fe h;
    {
        uint64_t l[5];
#pragma unroll
        for (int j = 0; j < 5; j++) l[j] = a.acc[5ull * c + j];
        for (int pass = 0; pass < 2; pass++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                l[j + 1] += l[j] >> 26;
                l[j] &= kM26;
            }
            l[0] += (l[4] >> 26) * 5u;
            l[4] &= kM26;
        }
#pragma unroll
        for (int j = 0; j < 5; j++) h.v[j] = static_cast<uint32_t>(l[j]);
        h = fe_carry(h);
    }
    // AAD = the content ID, zero padded to 16-byte blocks: block i of na has exponent Nct + 1 + na - i
    const uint8_t* ivp = a.ivs + static_cast<uint64_t>(c) * a.iv_stride;
    const uint32_t il = a.iv_len, na = (il + 15u) >> 4;
    for (uint32_t i = 0; i < na; i++) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            w[j] = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t at = 16u * i + 4u * j + b;
                if (at < il) w[j] |= static_cast<uint32_t>(ivp[at]) << (8 * b);
            }
        }
        const Fe m = fe_block(w[0], w[1], w[2], w[3]);
        h = fe_carry(fe_add(h, fe_mul(m, fe_pow_tab(tab, static_cast<uint32_t>(nct + 1u + na - i)))));
    }
    Fe r;
#pragma unroll
    for (int j = 0; j < 5; j++) r.v[j] = ck.r[j];
    const Fe lens = fe_block(il, 0u, static_cast<uint32_t>(len), static_cast<uint32_t>(len >> 32));
    h = fe_carry(fe_add(h, fe_mul(lens, r)));
    uint32_t s[4], tag[4];
#pragma unroll
    for (int j = 0; j < 4; j++) s[j] = ck.s[j];
    fe_tag(h, s, tag);
    if (kOpen) {
        const uint8_t* tp = a.in + a.in_offs[c] + 12u + len;
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) diff |= load_le32_bytes(tp + 4 * j) ^ tag[j];
        a.status[c] = diff ? -74 : 0;  // EBADMSG
    } else {
        uint8_t* tp = a.out + a.out_offs[c] + 12u + len;
#pragma unroll
        for (int j = 0; j < 16; j++) tp[j] = static_cast<uint8_t>(tag[j >> 2] >> (8 * (j & 3)));
    }
}

// ------------------------------------------------------------------ AES256-GCM-HMAC-SHA256
// repo/encryption/aes256_gcm_hmac_sha256_encryptor.go:24-65 (key = HMAC-SHA256(secret, id);
// AES-256-GCM from Go's crypto/cipher, 12-byte nonce, aad = id), aead_helpers.go:12-75.
// NIST SP 800-38D: J0 = nonce || 1, block j of the text uses counter j + 2, the tag is
// GHASH_H(aad, text) ^ E(J0).  AES is the big-endian T-table form (FIPS-197 §5.1 with
// SubBytes/ShiftRows/MixColumns folded into four 256-word tables), the tables derived on the
// device from GF(2^8) inverses.  GHASH elements are 4 big-endian words: bit 31 of w[0] is the
// coefficient of x^0.
//
// Byte pass layout: a chunk of c 16-byte blocks is padded at the FRONT with pre zero blocks to
// U whole 4 KiB units (256 blocks), so every unit is full and zero blocks before the text
// leave GHASH unchanged.  A segment is 64 units counted back from the end (the first may be
// shorter), one wave.  Lane l owns the blocks
// v = l (mod 64): CTR + GHASH Horner with the one multiplier M = H^64 (4-bit tables per nibble
// position in LDS); at the segment end lane l's sum is scaled by H^(63-l), the wave XORs the
// lanes, scales by H^(16384 (segments after)), and XORs that into the chunk's accumulator.
constexpr uint32_t kGcmSegUnits = 64;               // units per segment (one wave)
constexpr uint32_t kGcmHp = 12;                     // H^(16384 * 2^i): chunks < 2^30 B

struct GcmKey {  // per chunk, 1664 bytes
    uint32_t rk[60];
    uint32_t h[4], h64[4], ej0[4];
    uint32_t nonce[3];  // big-endian words
    uint32_t len_lo, len_hi;
    uint32_t pre, nseg;
    uint32_t pad[3];
    uint32_t acc[4];           // XOR of the segments' scaled sums (atomic)
    uint32_t hp[kGcmHp][4];    // H^(16384 * 2^i)
    uint32_t hl[64][4];        // H^l
    uint32_t pad2[26];
};
static_assert(sizeof(GcmKey) == 1664, "GcmKey layout");

__device__ __forceinline__ uint32_t xt8(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x11Bu : 0u)) & 0xFFu; }
__device__ __forceinline__ uint32_t gmul8(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        r ^= (b & 1u) ? a : 0u;
        a = xt8(a);
        b >>= 1;
    }
    return r;
}
// FIPS-197 §5.1.1: S(x) = affine(x^254).
__device__ __forceinline__ uint32_t aes_sbox_entry(uint32_t x) {
    uint32_t p = 1, b = x;
#pragma unroll
    for (int i = 0; i < 8; i++) {  // x^254: bits 1..7 of 254
        if ((254u >> i) & 1u) p = gmul8(p, b);
        b = gmul8(b, b);
    }
    uint32_t out = 0x63u;
#pragma unroll
    for (int k = 0; k < 5; k++) out ^= ((p << k) | (p >> (8 - k))) & 0xFFu;
    return out;
}

// Te0[x] = {2S, S, S, 3S} big-endian, Te1 = ror8(Te0); Te2 = ror16(Te0), Te3 = ror16(Te1) are one
// v_alignbit each.  Row x (256 bytes) holds 32 copies of Te0[x] then 32 of Te1[x]: lane l reads
// copy l & 31, so the 32 lanes of a ds_read_b32 group hit 32 distinct banks (one shared table
// was 60 % bank-conflict cycles), and the byte address (x << 8) | lane offset is ONE v_perm of
// the state word.  Kernels keep the table first in their LDS so the base folds
// into the ds_read offset.  Sb[x] = S for the key schedule.
// Te0 + Te1 rows of 256 B, 32 replicas each (one v_perm address; a Te0-only 32 KiB table fits 12
// waves but spills at 168 VGPRs: 333/306 vs 409 GiB/s, profiles/r02/aes/ab_narrow_table.log).
struct alignas(256) AesTabs {
    uint32_t te[256 * 64];
    uint32_t sb[256];
};
__device__ __forceinline__ void aes_tabs_build(AesTabs& t, uint32_t tid, uint32_t nthreads) {
    for (uint32_t x = tid; x < 256u; x += nthreads) {
        const uint32_t sx = aes_sbox_entry(x), s2 = xt8(sx), s3 = s2 ^ sx;
        const uint32_t w = (s2 << 24) | (sx << 16) | (sx << 8) | s3, w1 = ror32(w, 8);
#pragma unroll 8
        for (uint32_t c = 0; c < 64u; c++) {
            const uint32_t cc = (c + x) & 63u;  // lanes start on different banks
            t.te[64u * x + cc] = (cc & 32u) ? w1 : w;
        }
        t.sb[x] = sx;
    }
}
// LDS byte address of a table entry: byte k of s in address byte 1, the lane's copy offset
// (in byte 0 of `off`: 4 (lane & 31), + 128 for Te1) in byte 0.
template <int k>
__device__ __forceinline__ uint32_t te_at(const AesTabs& t, uint32_t s, uint32_t off) {
    const uint32_t byte = __builtin_amdgcn_perm(s, off, 0x0C0C0000u | ((4u + k) << 8));
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(t.te) + byte);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// gcm_prep's table: two blocks per chunk do not need the replicated rows (2 KiB, more
// workgroups per CU).
struct AesSmall {
    uint32_t te0[256];
    uint32_t sb[256];
};
__device__ __forceinline__ void aes_small_build(AesSmall& t, uint32_t tid, uint32_t nthreads) {
    for (uint32_t x = tid; x < 256u; x += nthreads) {
        const uint32_t sx = aes_sbox_entry(x), s2 = xt8(sx), s3 = s2 ^ sx;
        t.te0[x] = (s2 << 24) | (sx << 16) | (sx << 8) | s3;
        t.sb[x] = sx;
    }
}
template <typename RK>
__device__ __forceinline__ void aes256_block_small(const AesSmall& t, const RK& rk, uint32_t (&s)[4]) {
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return t.te0[a >> 24] ^ ror32(t.te0[(b >> 16) & 255u], 8) ^ ror32(t.te0[(c >> 8) & 255u], 16) ^
               ror32(t.te0[d & 255u], 24) ^ k;
    };
#pragma unroll
    for (int r = 1; r < 14; r++) {
        const uint32_t t0 = col(s0, s1, s2, s3, rk[4 * r]), t1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
        const uint32_t t2 = col(s2, s3, s0, s1, rk[4 * r + 2]), t3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return ((t.sb[a >> 24] << 24) | (t.sb[(b >> 16) & 255u] << 16) | (t.sb[(c >> 8) & 255u] << 8) | t.sb[d & 255u]) ^ k;
    };
    s[0] = fin(s0, s1, s2, s3, rk[56]);
    s[1] = fin(s1, s2, s3, s0, rk[57]);
    s[2] = fin(s2, s3, s0, s1, rk[58]);
    s[3] = fin(s3, s0, s1, s2, rk[59]);
}

template <typename Tabs>
__device__ __forceinline__ void aes256_expand(const Tabs& t, const uint32_t (&key)[8], uint32_t (&rk)[60]) {
#pragma unroll
    for (int i = 0; i < 8; i++) rk[i] = key[i];
    uint32_t rcon = 1;
#pragma unroll
    for (int i = 8; i < 60; i++) {
        uint32_t x = rk[i - 1];
        if (i % 8 == 0) {
            x = (t.sb[(x >> 16) & 255u] << 24) | (t.sb[(x >> 8) & 255u] << 16) | (t.sb[x & 255u] << 8) | t.sb[x >> 24];
            x ^= rcon << 24;
            rcon = xt8(rcon);
        } else if (i % 8 == 4) {
            x = (t.sb[x >> 24] << 24) | (t.sb[(x >> 16) & 255u] << 16) | (t.sb[(x >> 8) & 255u] << 8) | t.sb[x & 255u];
        }
        rk[i] = rk[i - 8] ^ x;
    }
}

// One block in place; o0 / o1 = the lane's Te0 / Te1 copy offsets (4 (lane & 31), + 128).
template <typename RK>
__device__ __forceinline__ void aes256_block(const AesTabs& t, uint32_t o0, uint32_t o1, const RK& rk, uint32_t (&s)[4]) {
    uint32_t s0 = s[0] ^ rk[0], s1 = s[1] ^ rk[1], s2 = s[2] ^ rk[2], s3 = s[3] ^ rk[3];
    auto col = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        const uint32_t t0 = te_at<3>(t, a, o0), t1 = te_at<2>(t, b, o1);
        const uint32_t t2 = ror32(te_at<1>(t, c, o0), 16), t3 = ror32(te_at<0>(t, d, o1), 16);
        return xor3(xor3(t0, t1, t2), t3, k);
    };
#pragma unroll
    for (int r = 1; r < 14; r++) {
        const uint32_t t0 = col(s0, s1, s2, s3, rk[4 * r]);
        const uint32_t t1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
        const uint32_t t2 = col(s2, s3, s0, s1, rk[4 * r + 2]);
        const uint32_t t3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    // Last round: S(x) is byte 2 and byte 1 of Te0[x]; two v_perm assemble the column.
    auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        const uint32_t ea = te_at<3>(t, a, o0), eb = te_at<2>(t, b, o0), ec = te_at<1>(t, c, o0), ed = te_at<0>(t, d, o0);
        return xor3(__builtin_amdgcn_perm(ea, eb, 0x06020C0Cu), __builtin_amdgcn_perm(ec, ed, 0x0C0C0501u), k);
    };
    s[0] = fin(s0, s1, s2, s3, rk[56]);
    s[1] = fin(s1, s2, s3, s0, rk[57]);
    s[2] = fin(s2, s3, s0, s1, rk[58]);
    s[3] = fin(s3, s0, s1, s2, rk[59]);
}

// z = x * y in GCM's field (bit-serial, 128 steps).
__device__ __forceinline__ void gf_mul(const uint32_t (&x)[4], const uint32_t (&y)[4], uint32_t (&z)[4]) {
    uint32_t v0 = y[0], v1 = y[1], v2 = y[2], v3 = y[3];
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t xw = x[w];
#pragma unroll 8
        for (int b = 31; b >= 0; b--) {
            const uint32_t m = 0u - ((xw >> b) & 1u);
            z0 ^= v0 & m;
            z1 ^= v1 & m;
            z2 ^= v2 & m;
            z3 ^= v3 & m;
            const uint32_t red = 0xE1000000u & (0u - (v3 & 1u));
            v3 = __builtin_amdgcn_alignbit(v2, v3, 1);
            v2 = __builtin_amdgcn_alignbit(v1, v2, 1);
            v1 = __builtin_amdgcn_alignbit(v0, v1, 1);
            v0 = (v0 >> 1) ^ red;
        }
    }
    z[0] = z0;
    z[1] = z1;
    z[2] = z2;
    z[3] = z3;
}
__device__ __forceinline__ void gf_mul_in(uint32_t (&x)[4], const uint32_t (&y)[4]) {
    uint32_t z[4];
    gf_mul(x, y, z);
#pragma unroll
    for (int j = 0; j < 4; j++) x[j] = z[j];
}
__device__ __forceinline__ void gf_one(uint32_t (&x)[4]) {
    x[0] = 0x80000000u;
    x[1] = x[2] = x[3] = 0u;
}
// 32 bits -> 64 with a zero between neighbours (bit i -> bit 2i).
__device__ __forceinline__ uint64_t spread32(uint32_t v) {
    uint64_t x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}
// x = x^2.  Squaring is linear over GF(2): in the natural order (bit i = coefficient of x^i, the
// bit reverse of GCM's words) it spreads bit i to 2i, and the upper 128 bits fold back through
// x^128 = x^7 + x^2 + x + 1.  ~100 VALU against ~1,300 for gf_mul.
__device__ __forceinline__ void gf_sqr_in(uint32_t (&x)[4]) {
    uint64_t lo0 = spread32(__builtin_bitreverse32(x[0])), lo1 = spread32(__builtin_bitreverse32(x[1]));
    uint64_t hi0 = spread32(__builtin_bitreverse32(x[2])), hi1 = spread32(__builtin_bitreverse32(x[3]));
    // natural order: coefficients 0..127 in (lo1:lo0), 128..255 in (hi1:hi0); fold hi * (1 + x + x^2 + x^7)
    auto fold = [&](uint64_t h0, uint64_t h1, int k, uint64_t& o0, uint64_t& o1, uint64_t& over) {
        o0 ^= h0 << k;
        o1 ^= (h1 << k) | (k ? (h0 >> (64 - k)) : 0ull);
        over ^= k ? (h1 >> (64 - k)) : 0ull;
    };
    uint64_t over = 0;
    fold(hi0, hi1, 0, lo0, lo1, over);
    fold(hi0, hi1, 1, lo0, lo1, over);
    fold(hi0, hi1, 2, lo0, lo1, over);
    fold(hi0, hi1, 7, lo0, lo1, over);
    // over: coefficients 128..134 -> times (1 + x + x^2 + x^7) lands below 2^14
    lo0 ^= over ^ (over << 1) ^ (over << 2) ^ (over << 7);
    x[0] = __builtin_bitreverse32(static_cast<uint32_t>(lo0));
    x[1] = __builtin_bitreverse32(static_cast<uint32_t>(lo0 >> 32));
    x[2] = __builtin_bitreverse32(static_cast<uint32_t>(lo1));
    x[3] = __builtin_bitreverse32(static_cast<uint32_t>(lo1 >> 32));
}
// x = y^e (square and multiply)
__device__ __forceinline__ void gf_pow(const uint32_t (&y)[4], uint64_t e, uint32_t (&x)[4]) {
    gf_one(x);
    uint32_t b[4] = {y[0], y[1], y[2], y[3]};
    while (e) {
        if (e & 1u) gf_mul_in(x, b);
        e >>= 1;
        if (e) gf_sqr_in(b);
    }
}

__device__ __forceinline__ void gcm_layout(uint64_t len, uint32_t& pre, uint32_t& nseg) {
    const uint64_t c = (len + 15u) >> 4;
    const uint64_t u = (c + 255u) >> 8;
    pre = static_cast<uint32_t>(u * 256u - c);
    nseg = static_cast<uint32_t>((u + kGcmSegUnits - 1u) / kGcmSegUnits);
}

// One wave per chunk: HMAC key, key schedule, H, E(J0), powers of H; the nonce for seal.
template <bool kOpen>
__global__ __launch_bounds__(256) void gcm_prep_kernel(CryptArgs a, GcmKey* keys) {
    __shared__ AesSmall t;
    aes_small_build(t, threadIdx.x, 256u);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (c >= a.n) return;
    const uint64_t in_len = a.in_lens[c];
    const bool bad = kOpen ? (in_len < 28u || in_len - 28u > kMaxLen) : in_len > kMaxLen;
    const uint64_t len = bad ? 0 : (kOpen ? in_len - 28u : in_len);
    const uint8_t* ivp = a.ivs + static_cast<uint64_t>(c) * a.iv_stride;
    const uint8_t* np = kOpen ? a.in + a.in_offs[c] : a.nonces + 12ull * c;
    uint32_t nonce[3] = {0u, 0u, 0u};  // little-endian words as stored
    if (!(kOpen && bad)) {
#pragma unroll
        for (int j = 0; j < 3; j++) nonce[j] = load_le32_bytes(np + 4 * j);
    }
    uint32_t key[8];
    hmac_key(a.mid, ivp, a.iv_len, key);  // big-endian words of the digest after bswap below
#pragma unroll
    for (int j = 0; j < 8; j++) key[j] = bswap32(key[j]);
    uint32_t rk[60];
    aes256_expand(t, key, rk);
    uint32_t h[4] = {0u, 0u, 0u, 0u};
    aes256_block_small(t, rk, h);
    uint32_t ej0[4] = {bswap32(nonce[0]), bswap32(nonce[1]), bswap32(nonce[2]), 1u};
    aes256_block_small(t, rk, ej0);
    GcmKey& k = keys[c];
    // Lane l: H^l, and for l < 12 H^(16384 * 2^l) = H^(2^(14 + l)); lane 0 also H^64.
    uint32_t p[4];
    gf_pow(h, lane, p);
#pragma unroll
    for (int j = 0; j < 4; j++) k.hl[lane][j] = p[j];
    if (lane < kGcmHp) {
        uint32_t q[4] = {h[0], h[1], h[2], h[3]};
        for (uint32_t i = 0; i < 14u + lane; i++) gf_sqr_in(q);
#pragma unroll
        for (int j = 0; j < 4; j++) k.hp[lane][j] = q[j];
    }
    uint32_t pre, nseg;
    gcm_layout(len, pre, nseg);
    if (lane == 0) {
        uint32_t q[4] = {h[0], h[1], h[2], h[3]};
        for (int i = 0; i < 6; i++) gf_sqr_in(q);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            k.h[j] = h[j];
            k.h64[j] = q[j];
            k.ej0[j] = ej0[j];
            k.acc[j] = 0u;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) k.nonce[j] = bswap32(nonce[j]);
        k.len_lo = static_cast<uint32_t>(len);
        k.len_hi = static_cast<uint32_t>(len >> 32);
        k.pre = pre;
        k.nseg = nseg;
        a.units[c] = nseg;
        a.status[c] = bad ? (kOpen && in_len < 28u ? -22 : -27) : 0;  // EINVAL / EFBIG
    }
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < 60; j++)
        if (lane == static_cast<uint32_t>(j)) mine = rk[j];
    if (lane < 60u) k.rk[lane] = mine;
    if (!kOpen && lane < 3u) reinterpret_cast<uint32_t*>(a.out + a.out_offs[c])[lane] = nonce[lane];
}

// GHASH tables of one wave: tab[k][n] = (nibble n at position k) * M, position k = bits 4k..4k+3
// of the big-endian 128-bit value (k = 0: the low bits of w[3]).
struct alignas(256) GcmWave {
    alignas(256) uint32_t tab[32][16][4];  // 16-byte aligned rows: ds_read_b128, banks mod 64
    uint32_t p[128][4];  // M * x^i
};

__device__ __forceinline__ void gcm_tab_build(GcmWave& g, const uint32_t (&m)[4], uint32_t lane) {
    uint32_t v0 = m[0], v1 = m[1], v2 = m[2], v3 = m[3];
    for (uint32_t i = 0; i < 128u; i++) {
        if ((i & 63u) == lane) {
            g.p[i][0] = v0;
            g.p[i][1] = v1;
            g.p[i][2] = v2;
            g.p[i][3] = v3;
        }
        const uint32_t red = 0xE1000000u & (0u - (v3 & 1u));
        v3 = __builtin_amdgcn_alignbit(v2, v3, 1);
        v2 = __builtin_amdgcn_alignbit(v1, v2, 1);
        v1 = __builtin_amdgcn_alignbit(v0, v1, 1);
        v0 = (v0 >> 1) ^ red;
    }
    wave_lds_sync();
#pragma unroll
    for (uint32_t q = 0; q < 8u; q++) {
        const uint32_t e = lane + 64u * q, kk = e >> 4, n = e & 15u;
        uint32_t z[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (uint32_t b = 0; b < 4u; b++)
            if ((n >> b) & 1u) {
                const uint32_t i = 127u - 4u * kk - b;
#pragma unroll
                for (int j = 0; j < 4; j++) z[j] ^= g.p[i][j];
            }
#pragma unroll
        for (int j = 0; j < 4; j++) g.tab[kk][n][j] = z[j];
    }
    wave_lds_sync();
}

// x = x * M through the wave's tables (two entries per 3-input XOR).
__device__ __forceinline__ void gcm_tab_mul(const GcmWave& g, uint32_t (&x)[4]) {
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t xw = x[3 - w];  // positions 8w .. 8w+7 live in word 3 - w
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
            const uint4 e = *reinterpret_cast<const uint4*>(g.tab[8 * w + q][(xw >> (4 * q)) & 15u]);
            const uint4 f = *reinterpret_cast<const uint4*>(g.tab[8 * w + q + 1][(xw >> (4 * q + 4)) & 15u]);
            z0 = xor3(z0, e.x, f.x);
            z1 = xor3(z1, e.y, f.y);
            z2 = xor3(z2, e.z, f.z);
            z3 = xor3(z3, e.w, f.w);
        }
    }
    x[0] = z0;
    x[1] = z1;
    x[2] = z2;
    x[3] = z3;
}

constexpr int kGcmSimdWaves = 2;  // waves per SIMD the register budget is sized for
constexpr int kGcmRb = 2;         // AES blocks in flight per lane (rows of a unit per batch)
constexpr uint32_t kGcmWaves = 8;  // waves per workgroup: 64 KiB table + 8 GHASH tables = 146 KiB
struct GcmLds {
    AesTabs t;  // first: at LDS address 0
    GcmWave gw[kGcmWaves];
};
template <bool kOpen>
__global__ __launch_bounds__(64 * kGcmWaves) __attribute__((amdgpu_waves_per_eu(kGcmSimdWaves, kGcmSimdWaves))) void gcm_units_kernel(
    CryptArgs a, const GcmKey* __restrict__ keys, GcmKey* acc_keys, const uint32_t* __restrict__ segp) {
    __shared__ GcmLds L;
    aes_tabs_build(L.t, threadIdx.x, 64u * kGcmWaves);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t o0 = 4u * (lane & 31u), o1 = o0 + 128u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    GcmWave& g = L.gw[wv];
    const uint32_t total = segp[a.n];
    const uint32_t nw = gridDim.x * kGcmWaves;
    uint32_t cur = 0xFFFFFFFFu;
    for (uint32_t s = blockIdx.x * kGcmWaves + wv; s < total; s += nw) {
        uint32_t lo = 0, hi = a.n;  // segp[lo] <= s < segp[hi]
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (segp[mid] <= s) lo = mid;
            else hi = mid;
        }
        const uint32_t c = lo;
        const GcmKey& k = keys[c];
        if (c != cur) {
            wave_lds_sync();
            const uint32_t m[4] = {k.h64[0], k.h64[1], k.h64[2], k.h64[3]};
            gcm_tab_build(g, m, lane);
            cur = c;
        }
        const uint64_t len = static_cast<uint64_t>(k.len_lo) | (static_cast<uint64_t>(k.len_hi) << 32);
        const uint32_t pre = k.pre, nseg = k.nseg;
        const uint64_t nblk = (len + 15u) >> 4;
        const uint32_t units = static_cast<uint32_t>((nblk + pre) >> 8);
        const uint32_t sl = s - segp[c];
        // Segments end at 64-unit steps from the chunk's end: only the first is partial, so every
        // segment after this one holds exactly 16384 blocks.
        const uint32_t u1 = units - kGcmSegUnits * (nseg - 1u - sl);
        const uint32_t u0 = u1 > kGcmSegUnits ? u1 - kGcmSegUnits : 0u;
        const uint8_t* inb = a.in + a.in_offs[c] + (kOpen ? 12u : 0u);
        uint8_t* outb = a.out + a.out_offs[c] + (kOpen ? 0u : 12u);
        const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(inb) & 3u);
        const uint32_t* inw = reinterpret_cast<const uint32_t*>(inb - mis);
        uint32_t* outw = reinterpret_cast<uint32_t*>(outb);
        uint32_t acc[4] = {0u, 0u, 0u, 0u};
        for (uint32_t u = u0; u < u1; u++)
#pragma unroll
        for (int rb = 0; rb < 4; rb += kGcmRb) {
            uint32_t st[kGcmRb][4];
            int64_t jb[kGcmRb];
#pragma unroll
            for (int r = 0; r < kGcmRb; r++) {
                const int64_t j = static_cast<int64_t>(256u * u + 64u * (rb + r) + lane) - pre;
                jb[r] = j;
                st[r][0] = k.nonce[0];
                st[r][1] = k.nonce[1];
                st[r][2] = k.nonce[2];
                st[r][3] = static_cast<uint32_t>(j + 2);
            }
#pragma unroll
            for (int r = 0; r < kGcmRb; r++) aes256_block(L.t, o0, o1, k.rk, st[r]);
#pragma unroll
            for (int r = 0; r < kGcmRb; r++) {
                const int64_t j = jb[r];
                const int64_t rem = j >= 0 ? static_cast<int64_t>(len) - 16 * j : 0;
                const uint32_t hiB = rem <= 0 ? 0u : rem >= 16 ? 16u : static_cast<uint32_t>(rem);
                uint32_t d[4] = {0u, 0u, 0u, 0u};
                if (hiB) {
                    const uint64_t w0 = 4ull * static_cast<uint64_t>(j);  // word index of the block in inw
                    uint32_t w[5];
#pragma unroll
                    for (uint32_t q = 0; q < 5u; q++) w[q] = (4u * q < mis + hiB) ? inw[w0 + q] : 0u;
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        d[q] = __builtin_amdgcn_alignbit(w[q + 1], w[q], 8u * mis) & keep_mask(static_cast<int64_t>(hiB) - 4 * q);
                }
                uint32_t o[4], gin[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    o[q] = (d[q] ^ bswap32(st[r][q])) & keep_mask(static_cast<int64_t>(hiB) - 4 * q);
                    gin[q] = bswap32(kOpen ? d[q] : o[q]);
                }
                if (hiB) {
                    uint32_t* ow = outw + 4ull * static_cast<uint64_t>(j);
#pragma unroll
                    for (uint32_t q = 0; q < 4u; q++) {
                        if (4u * q + 4u <= hiB) ow[q] = o[q];
                        else if (4u * q < hiB) {
                            uint8_t* ob = reinterpret_cast<uint8_t*>(ow + q);
                            for (uint32_t b = 0; b < hiB - 4u * q; b++) ob[b] = static_cast<uint8_t>(o[q] >> (8 * b));
                        }
                    }
                }
                gcm_tab_mul(g, acc);
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] ^= gin[q];
            }
        }
        // Lane l's last block is 63 - l blocks before the segment's end.
        {
            const uint32_t hl[4] = {k.hl[63u - lane][0], k.hl[63u - lane][1], k.hl[63u - lane][2], k.hl[63u - lane][3]};
            gf_mul_in(acc, hl);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) acc[q] ^= __shfl_xor(acc[q], off, 64);
        }
        uint32_t after = nseg - 1u - sl;  // whole segments after this one
        for (uint32_t i = 0; after; i++, after >>= 1)
            if (after & 1u) {
                const uint32_t hp[4] = {k.hp[i][0], k.hp[i][1], k.hp[i][2], k.hp[i][3]};
                gf_mul_in(acc, hp);
            }
        if (lane < 4u) {
            uint32_t mine = acc[0];
#pragma unroll
            for (int q = 1; q < 4; q++)
                if (lane == static_cast<uint32_t>(q)) mine = acc[q];
            atomicXor(&acc_keys[c].acc[lane], mine);
        }
    }
}

// One lane per chunk: AAD, text sum, length block, tag.
template <bool kOpen>
__global__ __launch_bounds__(256) void gcm_finish_kernel(CryptArgs a, const GcmKey* keys) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.n || a.status[c] != 0) return;
    const GcmKey& k = keys[c];
    const uint64_t len = static_cast<uint64_t>(k.len_lo) | (static_cast<uint64_t>(k.len_hi) << 32);
    const uint32_t h[4] = {k.h[0], k.h[1], k.h[2], k.h[3]};
    const uint8_t* ivp = a.ivs + static_cast<uint64_t>(c) * a.iv_stride;
    const uint32_t il = a.iv_len;
    uint32_t x[4] = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < il; i += 16u) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t w = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t at = i + 4u * q + b;
                w = (w << 8) | (at < il ? static_cast<uint32_t>(ivp[at]) : 0u);
            }
            x[q] ^= w;
        }
        gf_mul_in(x, h);
    }
    uint32_t hc[4];
    gf_pow(h, (len + 15u) >> 4, hc);
    gf_mul_in(x, hc);
    uint32_t sc[4] = {k.acc[0], k.acc[1], k.acc[2], k.acc[3]};
    gf_mul_in(sc, h);
    const uint64_t abits = 8ull * il, cbits = 8ull * len;
    x[0] ^= sc[0] ^ static_cast<uint32_t>(abits >> 32);
    x[1] ^= sc[1] ^ static_cast<uint32_t>(abits);
    x[2] ^= sc[2] ^ static_cast<uint32_t>(cbits >> 32);
    x[3] ^= sc[3] ^ static_cast<uint32_t>(cbits);
    gf_mul_in(x, h);
    uint32_t tag[4];
#pragma unroll
    for (int q = 0; q < 4; q++) tag[q] = bswap32(x[q] ^ k.ej0[q]);  // little-endian words of the tag bytes
    if (kOpen) {
        const uint8_t* tp = a.in + a.in_offs[c] + 12u + len;
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) diff |= load_le32_bytes(tp + 4 * j) ^ tag[j];
        a.status[c] = diff ? -74 : 0;  // EBADMSG
    } else {
        uint8_t* tp = a.out + a.out_offs[c] + 12u + len;
#pragma unroll
        for (int j = 0; j < 16; j++) tp[j] = static_cast<uint8_t>(tag[j >> 2] >> (8 * (j & 3)));
    }
}

// Open: a chunk that fails its check hands back no plaintext, as Go's Open returns nil on a bad
// tag (aeadOpenPrefixedWithNonce, repo/encryption/aes256_gcm_hmac_sha256_encryptor.go:49-56,
// aead_helpers.go).  The byte pass has already written the unauthenticated plaintext, so the
// chunk's output slot (sealed length - 28 bytes) is zeroed.  One wave per chunk; the wave of a
// chunk that opened cleanly exits at once.
__global__ __launch_bounds__(256) void open_mask_kernel(CryptArgs a) {
    const uint32_t c = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (c >= a.n || a.status[c] == 0) return;
    const uint64_t in_len = a.in_lens[c];
    if (in_len <= 28u) return;  // too short: nothing was written
    const uint64_t len = in_len - 28u;
    uint8_t* p = a.out + a.out_offs[c];  // a multiple of 4
    const uint64_t nq = len / 16u;
    u32x4* pq = reinterpret_cast<u32x4*>(p);
    const u32x4 z = {0u, 0u, 0u, 0u};
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
        for (uint64_t i = lane; i < nq; i += 64u) pq[i] = z;
        for (uint64_t i = 16u * nq + lane; i < len; i += 64u) p[i] = 0;
    } else {
        uint32_t* pw = reinterpret_cast<uint32_t*>(p);
        const uint64_t nw = len / 4u;
        for (uint64_t i = lane; i < nw; i += 64u) pw[i] = 0u;
        for (uint64_t i = 4u * nw + lane; i < len; i += 64u) p[i] = 0;
    }
}

}  // namespace cryptdev

namespace {
using cryptdev::ChunkKey;
using cryptdev::Fe;
using cryptdev::kTabN;

struct CryptAlgo {
    const char* name;
    uint32_t overhead;
};
// repo/encryption/chacha20_poly1305_hmac_sha256_encryptor.go:16,67 (name, Overhead())
// aes256_gcm_hmac_sha256_encryptor.go:15,67-69,72 (AES256-GCM-HMAC-SHA256, Overhead() = 28)
constexpr CryptAlgo kCryptAlgos[] = {{"AES256-GCM-HMAC-SHA256", 28}, {"CHACHA20-POLY1305-HMAC-SHA256", 28}};

const CryptAlgo* find_crypt(const char* name) {
    if (!name) return nullptr;
    for (const CryptAlgo& a : kCryptAlgos)
        if (std::strcmp(a.name, name) == 0) return &a;
    return nullptr;
}

uint64_t align256(uint64_t x) { return (x + 255u) & ~uint64_t(255); }

struct WsLayout {
    uint64_t keys, tabs, acc, units, status_off, total;
};
WsLayout ws_layout(uint32_t n) {
    WsLayout l{};
    l.keys = 0;
    l.tabs = align256(l.keys + uint64_t(n) * sizeof(ChunkKey));
    l.acc = align256(l.tabs + uint64_t(n) * kTabN * sizeof(Fe));
    l.units = align256(l.acc + uint64_t(n) * 5u * 8u);
    l.total = align256(l.units + (uint64_t(n) + 1u) * 4u);
    return l;
}

int units_grid(int* err) {
    static thread_local int cached_dev = -1, cached_grid = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return *err = set_error(-5, "hipGetDevice failed"), 0;
    if (dev != cached_dev) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return *err = set_error(-5, "device attribute query failed"), 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, cryptdev::crypt_units_kernel<false>, 256, 0) != hipSuccess ||
            per <= 0)
            per = 2;
        cached_grid = cus * per;
        cached_dev = dev;
    }
    return cached_grid;
}

int gcm_grid(int* err) {
    static thread_local int cached_dev = -1, cached_grid = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return *err = set_error(-5, "hipGetDevice failed"), 0;
    if (dev != cached_dev) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return *err = set_error(-5, "device attribute query failed"), 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, cryptdev::gcm_units_kernel<false>, 64 * cryptdev::kGcmWaves, 0) != hipSuccess ||
            per <= 0)
            per = 2;
        cached_grid = cus * per;
        cached_dev = dev;
    }
    return cached_grid;
}

template <bool kOpen>
int crypt_run(const char* name, const uint8_t* secret, uint32_t secret_len, const uint8_t* d_in,
              const uint64_t* d_in_offs, const uint64_t* d_in_lens, uint32_t n, const uint8_t* d_ivs, uint32_t iv_len,
              uint32_t iv_stride,
              const uint8_t* d_nonces, uint8_t* d_out, const uint64_t* d_out_offs, int32_t* d_status, void* d_work,
              uint64_t work_bytes, void* stream) {
    if (!find_crypt(name)) return set_error(-2, std::string("unknown encryption algorithm: ") + (name ? name : "(null)"));
    if (!secret || secret_len == 0 || secret_len > 64)
        return set_error(-22, "secret must be 1..64 bytes (the HKDF-derived key is 32)");
    if (iv_len == 0 || iv_len > 64) return set_error(-22, "content ID (iv) must be 1..64 bytes");
    if (iv_stride < iv_len && n > 1) return set_error(-22, "iv_stride must be >= iv_len");
    if (n == 0) return 0;
    if (!d_in || !d_in_offs || !d_in_lens || !d_ivs || !d_out || !d_out_offs || !d_status || !d_work ||
        (!kOpen && !d_nonces))
        return set_error(-22, "null argument");
    const WsLayout l = ws_layout(n);
    if (work_bytes < l.total) return set_error(-22, "workspace too small (kcdc_crypt_workspace_size)");
    int err = 0;
    const int grid = units_grid(&err);
    if (err) return err;

    cryptdev::CryptArgs a{};
    a.n = n;
    a.in = d_in;
    a.in_offs = d_in_offs;
    a.in_lens = d_in_lens;
    a.out = d_out;
    a.out_offs = d_out_offs;
    a.ivs = d_ivs;
    a.iv_len = iv_len;
    a.iv_stride = iv_stride;
    a.nonces = d_nonces;
    a.status = d_status;
    uint8_t* w = static_cast<uint8_t*>(d_work);
    a.keys = reinterpret_cast<ChunkKey*>(w + l.keys);
    a.tabs = reinterpret_cast<Fe*>(w + l.tabs);
    a.acc = reinterpret_cast<unsigned long long*>(w + l.acc);
    a.units = reinterpret_cast<uint32_t*>(w + l.units);
    // HMAC midstates (RFC 2104) for the repository secret, once per call on the host.
    {
        uint32_t ib[16], ob[16];
        uint8_t kb[64] = {};
        std::memcpy(kb, secret, secret_len);
        for (int j = 0; j < 16; j++) {
            uint32_t x = 0;
            for (int b = 0; b < 4; b++) x = (x << 8) | kb[4 * j + b];
            ib[j] = x ^ 0x36363636u;
            ob[j] = x ^ 0x5c5c5c5cu;
        }
        for (int j = 0; j < 8; j++) a.mid.in[j] = a.mid.out[j] = cryptdev::kSha256IV[j];
        cryptdev::sha256_compress(a.mid.in, ib);
        cryptdev::sha256_compress(a.mid.out, ob);
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (std::strcmp(name, "AES256-GCM-HMAC-SHA256") == 0) {
        static_assert(sizeof(cryptdev::GcmKey) <= sizeof(ChunkKey) + kTabN * sizeof(Fe), "GcmKey fits the ChaCha slots");
        cryptdev::GcmKey* gk = reinterpret_cast<cryptdev::GcmKey*>(w + l.keys);
        const int ggrid = gcm_grid(&err);
        if (err) return err;
        hipLaunchKernelGGL(cryptdev::gcm_prep_kernel<kOpen>, dim3((n + 3u) / 4u), dim3(256), 0, st, a, gk);
        hipLaunchKernelGGL(cryptdev::unit_scan_kernel, dim3(1), dim3(1024), 0, st, n, a.units);
        hipLaunchKernelGGL(cryptdev::gcm_units_kernel<kOpen>, dim3(ggrid), dim3(64 * cryptdev::kGcmWaves), 0, st, a, gk, gk, a.units);
        hipLaunchKernelGGL(cryptdev::gcm_finish_kernel<kOpen>, dim3((n + 255u) / 256u), dim3(256), 0, st, a, gk);
        if (kOpen) hipLaunchKernelGGL(cryptdev::open_mask_kernel, dim3((n + 3u) / 4u), dim3(256), 0, st, a);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : set_error(-5, std::string("encryption kernel launch: ") + hipGetErrorString(e));
    }
    hipLaunchKernelGGL(cryptdev::crypt_prep_kernel<kOpen>, dim3((n + 3u) / 4u), dim3(256), 0, st, a);
    hipLaunchKernelGGL(cryptdev::unit_scan_kernel, dim3(1), dim3(1024), 0, st, n, a.units);
    hipLaunchKernelGGL(cryptdev::crypt_units_kernel<kOpen>, dim3(grid), dim3(256), 0, st, a, a.keys, a.units, a.in_offs,
                       a.out_offs, a.tabs, a.out, a.acc);
    hipLaunchKernelGGL(cryptdev::crypt_finish_kernel<kOpen>, dim3((n + 255u) / 256u), dim3(256), 0, st, a);
    if (kOpen) hipLaunchKernelGGL(cryptdev::open_mask_kernel, dim3((n + 3u) / 4u), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error(-5, std::string("encryption kernel launch: ") + hipGetErrorString(e));
}
}  // namespace
}  // namespace kcdc

using namespace kcdc;

extern "C" int kcdc_encryption_algorithms(const char** names, int cap) {
    const int n = static_cast<int>(sizeof(kCryptAlgos) / sizeof(kCryptAlgos[0]));
    for (int i = 0; i < n && i < cap; i++) names[i] = kCryptAlgos[i].name;
    return n;
}

extern "C" int kcdc_encryption_overhead(const char* name) {
    const CryptAlgo* a = find_crypt(name);
    return a ? static_cast<int>(a->overhead)
             : set_error(-2, std::string("unknown encryption algorithm: ") + (name ? name : "(null)"));
}

extern "C" uint64_t kcdc_crypt_workspace_size(uint32_t nchunks) { return ws_layout(nchunks).total; }

extern "C" int kcdc_encrypt_chunks_device(const char* name, const uint8_t* secret, uint32_t secret_len,
                                          const uint8_t* d_data, const uint64_t* d_offsets, const uint64_t* d_lens,
                                          uint32_t nchunks, const uint8_t* d_ivs, uint32_t iv_len, uint32_t iv_stride,
                                          const uint8_t* d_nonces, uint8_t* d_out, const uint64_t* d_out_offsets,
                                          int32_t* d_status, void* d_work, uint64_t work_bytes, void* stream) {
    return crypt_run<false>(name, secret, secret_len, d_data, d_offsets, d_lens, nchunks, d_ivs, iv_len, iv_stride,
                            d_nonces, d_out, d_out_offsets, d_status, d_work, work_bytes, stream);
}

extern "C" int kcdc_decrypt_chunks_device(const char* name, const uint8_t* secret, uint32_t secret_len,
                                          const uint8_t* d_sealed, const uint64_t* d_offsets,
                                          const uint64_t* d_sealed_lens, uint32_t nchunks, const uint8_t* d_ivs,
                                          uint32_t iv_len, uint32_t iv_stride, uint8_t* d_out,
                                          const uint64_t* d_out_offsets,
                                          int32_t* d_status, void* d_work, uint64_t work_bytes, void* stream) {
    return crypt_run<true>(name, secret, secret_len, d_sealed, d_offsets, d_sealed_lens, nchunks, d_ivs, iv_len, iv_stride,
                           nullptr, d_out, d_out_offsets, d_status, d_work, work_bytes, stream);
}

namespace kcdc {
// Timing ablations of the encryption byte pass (wrong output); none in the product build.
const char* ablations_crypt() { return ""; }  // none left in the source (round 4)
}  // namespace kcdc
