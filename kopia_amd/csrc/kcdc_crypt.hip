// Kopia content encryption on gfx950: CHACHA20-POLY1305-HMAC-SHA256.
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

__device__ __forceinline__ uint32_t fe_limb(const Fe& a, uint32_t i) {  // register select, no scratch
    uint32_t r = a.v[0];
#pragma unroll
    for (uint32_t j = 1; j < 5; j++)
        if (i == j) r = a.v[j];
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
    const uint8_t* ivs;         // 16 bytes per chunk at ivs + i * iv_stride
    uint32_t iv_stride;
    const uint8_t* nonces;      // seal: 12 bytes per chunk
    int32_t* status;            // per chunk: 0, or a negative errno
    ChunkKey* keys;
    Fe* tabs;                   // kTabN powers of r per chunk
    unsigned long long* acc;    // 5 limb sums per chunk
    uint32_t* units;            // n + 1: units per chunk, then their exclusive prefix
    HmacMid mid;
};

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
    uint32_t blk[16];
#pragma unroll
    for (int j = 0; j < 4; j++) blk[j] = bswap32(load_le32_bytes(ivp + 4 * j));
    uint32_t nonce[3] = {0u, 0u, 0u};
    if (!(kOpen && bad)) {
#pragma unroll
        for (int j = 0; j < 3; j++) nonce[j] = load_le32_bytes(np + 4 * j);
    }
    // HMAC-SHA256(secret, iv): inner block = iv || pad (80 bytes hashed), outer = digest || pad (96 bytes).
    blk[4] = 0x80000000u;
#pragma unroll
    for (int j = 5; j < 15; j++) blk[j] = 0;
    blk[15] = 80u * 8u;
    uint32_t h[8];
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = a.mid.in[j];
    sha256_compress(h, blk);
#pragma unroll
    for (int j = 0; j < 8; j++) blk[j] = h[j];
    blk[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; j++) blk[j] = 0;
    blk[15] = 96u * 8u;
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = a.mid.out[j];
    sha256_compress(h, blk);
    uint32_t key[8];
#pragma unroll
    for (int j = 0; j < 8; j++) key[j] = bswap32(h[j]);
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

// The byte pass: persistent waves, each over a contiguous range of (chunk, unit) pairs.
template <bool kOpen>
__global__ __launch_bounds__(256) void crypt_units_kernel(CryptArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4][1024];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t* L = lds[wv];
    const uint32_t total = a.units[a.n];
    const uint64_t W = static_cast<uint64_t>(gridDim.x) * 4u, w = static_cast<uint64_t>(blockIdx.x) * 4u + wv;
    uint32_t u = static_cast<uint32_t>(total * w / W);
    const uint32_t u1 = static_cast<uint32_t>(total * (w + 1) / W);
    if (u >= u1) return;
    uint32_t lo = 0, hi = a.n;  // units[lo] <= u < units[hi]
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.units[mid] <= u) lo = mid;
        else hi = mid;
    }
    uint32_t c = lo;
    Fe accum = fe_zero();
    auto flush = [&](uint32_t cc) {
        if (lane < 5u) atomicAdd(a.acc + 5ull * cc + lane, static_cast<unsigned long long>(fe_limb(accum, lane)));
        accum = fe_zero();
    };
    for (; u < u1; u++) {
        if (a.units[c + 1] <= u) {
            flush(c);
            do c++;
            while (a.units[c + 1] <= u);
        }
        const ChunkKey& ck = a.keys[c];
        const uint64_t len = static_cast<uint64_t>(ck.len_lo) | (static_cast<uint64_t>(ck.len_hi) << 32);
        const uint32_t uu = u - a.units[c];
        const uint64_t ub = static_cast<uint64_t>(uu) * kUnit;
        const uint32_t rem = static_cast<uint32_t>(len - ub < kUnit ? len - ub : kUnit);
        const uint8_t* src = a.in + a.in_offs[c] + (kOpen ? 12u : 0u) + ub;
        uint32_t* dst = reinterpret_cast<uint32_t*>(a.out + a.out_offs[c] + (kOpen ? 0u : 12u) + ub);

        // 1. coalesced load (any byte alignment, never past the unit's last aligned word) -> LDS
        {
            const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
            const uint32_t mis = static_cast<uint32_t>(sa & 3u);
            const __attribute__((address_space(1))) uint32_t* ws =
                reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(sa - mis);
            const uint32_t lw = (rem + mis - 1u) >> 2;
            uint32_t x[16], y[16];
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t i = 64u * k + lane;
                x[k] = ws[min(i, lw)];
                y[k] = ws[min(i + 1u, lw)];
            }
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t i = 64u * k + lane;
                const uint32_t v = mis ? __builtin_amdgcn_alignbit(y[k], x[k], 8u * mis) : x[k];
                L[swz(i)] = v & keep_mask(static_cast<int64_t>(rem) - 4 * static_cast<int64_t>(i));
            }
        }
        wave_lds_sync();

        // 2. lane-own 64 bytes: keystream XOR
        uint32_t ks[16];
        uint32_t kk[8], nc[3];
#pragma unroll
        for (int j = 0; j < 8; j++) kk[j] = ck.key[j];
#pragma unroll
        for (int j = 0; j < 3; j++) nc[j] = ck.nonce[j];
        chacha20_block(kk, 1u + uu * 64u + lane, nc, ks);
        const uint32_t sw = (lane >> 2) & 3u;
        uint32_t d[16], res[16];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint4 q = *reinterpret_cast<const uint4*>(L + ((4u * lane + (t ^ sw)) << 2));
            d[4 * t] = q.x;
            d[4 * t + 1] = q.y;
            d[4 * t + 2] = q.z;
            d[4 * t + 3] = q.w;
        }
#pragma unroll
        for (int j = 0; j < 16; j++)
            res[j] = (d[j] ^ ks[j]) & keep_mask(static_cast<int64_t>(rem) - 64 * static_cast<int64_t>(lane) - 4 * j);
        wave_lds_sync();
#pragma unroll
        for (int t = 0; t < 4; t++)
            *reinterpret_cast<uint4*>(L + ((4u * lane + (t ^ sw)) << 2)) =
                make_uint4(res[4 * t], res[4 * t + 1], res[4 * t + 2], res[4 * t + 3]);

        // 3. Poly1305 over the ciphertext blocks of this unit (zero padded to 16 bytes)
        {
            const uint32_t* m = kOpen ? d : res;
            Fe r;
#pragma unroll
            for (int j = 0; j < 5; j++) r.v[j] = ck.r[j];
            const uint32_t nreal = (rem + 15u) >> 4, j0 = 4u * lane;
            Fe hl = fe_zero();
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const Fe nx = fe_add(fe_mul(hl, r), fe_block(m[4 * t], m[4 * t + 1], m[4 * t + 2], m[4 * t + 3]));
                if (j0 + t < nreal) hl = nx;
            }
            const Fe* tab = a.tabs + static_cast<uint64_t>(c) * kTabN;
            if (j0 < nreal) {
                const uint32_t jl = min(j0 + 3u, nreal - 1u);
                hl = fe_mul(hl, tab[kTabT + (nreal - 1u - jl)]);
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                Fe o;
#pragma unroll
                for (int j = 0; j < 5; j++) o.v[j] = __shfl_xor(hl.v[j], off, 64);
                hl = fe_carry(fe_add(hl, o));
            }
            // unit sum is relative to its last block j_end; that block's exponent is Nct + 1 - j_end
            const uint64_t nct = (len + 15u) >> 4;
            const uint32_t q = static_cast<uint32_t>(nct + 1u - (static_cast<uint64_t>(uu) * 256u + nreal - 1u));
            hl = fe_mul(hl, fe_pow_tab(tab, q));
            accum = fe_carry(fe_add(accum, hl));
        }
        wave_lds_sync();

        // 4. coalesced store; the zero tail of a partial last word stays inside the tag
        //    (seal) or the 4-byte padding of the plaintext slot (open)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t i = 64u * k + lane;
            if (4u * i < rem) dst[i] = L[swz(i)];
        }
        wave_lds_sync();
    }
    flush(c);
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
    const uint8_t* ivp = a.ivs + static_cast<uint64_t>(c) * a.iv_stride;
    const Fe aad = fe_block(load_le32_bytes(ivp), load_le32_bytes(ivp + 4), load_le32_bytes(ivp + 8),
                            load_le32_bytes(ivp + 12));
    h = fe_carry(fe_add(h, fe_mul(aad, fe_pow_tab(tab, static_cast<uint32_t>(nct + 2u)))));
    Fe r;
#pragma unroll
    for (int j = 0; j < 5; j++) r.v[j] = ck.r[j];
    const Fe lens = fe_block(16u, 0u, static_cast<uint32_t>(len), static_cast<uint32_t>(len >> 32));
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
constexpr CryptAlgo kCryptAlgos[] = {{"CHACHA20-POLY1305-HMAC-SHA256", 28}};

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

template <bool kOpen>
int crypt_run(const char* name, const uint8_t* secret, uint32_t secret_len, const uint8_t* d_in,
              const uint64_t* d_in_offs, const uint64_t* d_in_lens, uint32_t n, const uint8_t* d_ivs, uint32_t iv_stride,
              const uint8_t* d_nonces, uint8_t* d_out, const uint64_t* d_out_offs, int32_t* d_status, void* d_work,
              uint64_t work_bytes, void* stream) {
    if (!find_crypt(name)) return set_error(-2, std::string("unknown encryption algorithm: ") + (name ? name : "(null)"));
    if (!secret || secret_len == 0 || secret_len > 64)
        return set_error(-22, "secret must be 1..64 bytes (the HKDF-derived key is 32)");
    if (iv_stride < 16 && n > 1) return set_error(-22, "iv_stride must be >= 16");
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
    hipLaunchKernelGGL(cryptdev::crypt_prep_kernel<kOpen>, dim3((n + 3u) / 4u), dim3(256), 0, st, a);
    hipLaunchKernelGGL(cryptdev::unit_scan_kernel, dim3(1), dim3(1024), 0, st, n, a.units);
    hipLaunchKernelGGL(cryptdev::crypt_units_kernel<kOpen>, dim3(grid), dim3(256), 0, st, a);
    hipLaunchKernelGGL(cryptdev::crypt_finish_kernel<kOpen>, dim3((n + 255u) / 256u), dim3(256), 0, st, a);
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
                                          uint32_t nchunks, const uint8_t* d_ivs, uint32_t iv_stride,
                                          const uint8_t* d_nonces, uint8_t* d_out, const uint64_t* d_out_offsets,
                                          int32_t* d_status, void* d_work, uint64_t work_bytes, void* stream) {
    return crypt_run<false>(name, secret, secret_len, d_data, d_offsets, d_lens, nchunks, d_ivs, iv_stride, d_nonces,
                            d_out, d_out_offsets, d_status, d_work, work_bytes, stream);
}

extern "C" int kcdc_decrypt_chunks_device(const char* name, const uint8_t* secret, uint32_t secret_len,
                                          const uint8_t* d_sealed, const uint64_t* d_offsets,
                                          const uint64_t* d_sealed_lens, uint32_t nchunks, const uint8_t* d_ivs,
                                          uint32_t iv_stride, uint8_t* d_out, const uint64_t* d_out_offsets,
                                          int32_t* d_status, void* d_work, uint64_t work_bytes, void* stream) {
    return crypt_run<true>(name, secret, secret_len, d_sealed, d_offsets, d_sealed_lens, nchunks, d_ivs, iv_stride,
                           nullptr, d_out, d_out_offsets, d_status, d_work, work_bytes, stream);
}
