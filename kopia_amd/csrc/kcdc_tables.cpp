// Rolling-hash constants for the Kopia splitters, derived at library init.
//
// The reference splitters (repo/splitter/splitter_buzhash32.go:4,
// splitter_rabinkarp64.go:4) call github.com/chmduquesne/rollinghash
// v4.0.0+incompatible (go.mod:13), whose tables come from Go's math/rand seeded
// with 1.  Rather than embedding magic numbers, the library re-derives them:
//   * Go math/rand rngSource: additive lagged Fibonacci x_n = x_{n-607} + x_{n-273}
//     (mod 2^64), seeded through `seedrand` and XORed with rngCooked, where
//     rngCooked is itself the generator state after 7.8e12 steps from srand(1).
//     We reach that state by polynomial jump-ahead modulo z^607 - z^334 - 1.
//   * buzhash32 byte table: 256 distinct uint32(Int63()) draws from NewSource(1).
//   * Rabin-Karp: first irreducible degree-53 polynomial drawn from
//     rand.New(NewSource(1)) as 8-byte little-endian reads (Ben-Or test), and the
//     out/mod roll tables derived from it.
// tests/test_lib_host.py checks every table against the oracle's golden values.
#include "kcdc_internal.h"

#include <cstring>
#include <mutex>
#include <set>
#include <vector>

namespace kcdc {
namespace {

constexpr int kLen = 607;
constexpr int kTap = 273;
constexpr int32_t kInt32Max = 2147483647;

int32_t seedrand(int32_t x) {
    const int32_t hi = x / 44488, lo = x % 44488;
    x = 48271 * lo - 3399 * hi;
    if (x < 0) x += kInt32Max;
    return x;
}

void seed_vector(int64_t seed, int sh0, int sh1, const uint64_t* cooked, uint64_t* vec) {
    seed %= kInt32Max;
    if (seed < 0) seed += kInt32Max;
    if (seed == 0) seed = 89482311;
    int32_t x = static_cast<int32_t>(seed);
    for (int i = -20; i < kLen; i++) {
        x = seedrand(x);
        if (i >= 0) {
            uint64_t u = static_cast<uint64_t>(static_cast<int64_t>(x)) << sh0;
            x = seedrand(x);
            u ^= static_cast<uint64_t>(static_cast<int64_t>(x)) << sh1;
            x = seedrand(x);
            u ^= static_cast<uint64_t>(static_cast<int64_t>(x));
            if (cooked) u ^= cooked[i];
            vec[i] = u;
        }
    }
}

// r = a*b mod (z^607 - z^334 - 1), coefficients mod 2^64.
void polymulmod(const uint64_t* a, const uint64_t* b, uint64_t* r) {
    std::vector<uint64_t> t(2 * kLen - 1, 0);
    for (int i = 0; i < kLen; i++) {
        const uint64_t ai = a[i];
        if (!ai) continue;
        uint64_t* ti = t.data() + i;
        for (int j = 0; j < kLen; j++) ti[j] += ai * b[j];
    }
    for (int i = 2 * kLen - 2; i >= kLen; i--) {  // z^i = z^(i-607) + z^(i-273)
        const uint64_t c = t[i];
        t[i - kLen] += c;
        t[i - kTap] += c;
    }
    std::memcpy(r, t.data(), kLen * sizeof(uint64_t));
}

// State of gen_cooked.go after srand(1) and 7.8e12 vrand() steps.
void compute_rng_cooked(uint64_t* cooked) {
    uint64_t v0[kLen];
    seed_vector(1, 20, 10, nullptr, v0);
    // Step n >= 1 writes y_n = y_{n-607} + y_{n-273} to slot (334-n) mod 607;
    // the initial slots are y_n for n in [-606, 0].  u_k = y_{k-606}.
    uint64_t u0[kLen];
    for (int k = 0; k < kLen; k++) u0[k] = v0[(940 - k) % kLen];
    const uint64_t N = 7800000000000ull;
    std::vector<uint64_t> res(kLen, 0), base(kLen, 0), tmp(kLen);
    res[0] = 1;
    base[1] = 1;
    for (uint64_t e = N; e; e >>= 1) {
        if (e & 1) { polymulmod(res.data(), base.data(), tmp.data()); res.swap(tmp); }
        if (e > 1) { polymulmod(base.data(), base.data(), tmp.data()); base.swap(tmp); }
    }
    for (int k = 0; k < kLen; k++) {  // y_{N-606+k} = u_{N+k}
        uint64_t y = 0;
        for (int j = 0; j < kLen; j++) y += res[j] * u0[j];
        const int64_t n = static_cast<int64_t>(N % kLen) - 606 + k;  // slot only needs n mod 607
        cooked[((334 - n) % kLen + kLen) % kLen] = y;
        const uint64_t c = res[kLen - 1];  // res *= z
        for (int j = kLen - 1; j > 0; j--) res[j] = res[j - 1];
        res[0] = c;
        res[334] += c;
    }
}

struct GoRand {
    uint64_t vec[kLen];
    int tap = 0, feed = kLen - kTap;
    int pos = 0;
    int64_t val = 0;
    GoRand(int64_t seed, const uint64_t* cooked) { seed_vector(seed, 40, 20, cooked, vec); }
    uint64_t uint64() {
        if (--tap < 0) tap += kLen;
        if (--feed < 0) feed += kLen;
        const uint64_t x = vec[feed] + vec[tap];
        vec[feed] = x;
        return x;
    }
    int64_t int63() { return static_cast<int64_t>(uint64() & 0x7FFFFFFFFFFFFFFFull); }
    void read(uint8_t* p, uint64_t n) {  // rand.go read(): 7 bytes per Int63
        for (uint64_t i = 0; i < n; i++) {
            if (pos == 0) { val = int63(); pos = 7; }
            p[i] = static_cast<uint8_t>(val);
            val >>= 8;
            pos--;
        }
    }
};

// ---- GF(2) polynomial helpers for the Rabin polynomial (degree <= 63) ----
int gf2_deg(uint64_t x) { return x ? 63 - __builtin_clzll(x) : -1; }
uint64_t gf2_mod(uint64_t x, uint64_t m) {
    const int dm = gf2_deg(m);
    for (int d = gf2_deg(x); d >= dm; d = gf2_deg(x)) x ^= m << (d - dm);
    return x;
}
uint64_t gf2_mulmod(uint64_t a, uint64_t b, uint64_t m) {  // a, b < 2^deg(m)
    const int dm = gf2_deg(m);
    uint64_t r = 0;
    a = gf2_mod(a, m);
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (gf2_deg(a) >= dm) a ^= m;
    }
    return r;
}
uint64_t gf2_gcd(uint64_t a, uint64_t b) {
    while (b) { const uint64_t t = gf2_mod(a, b); a = b; b = t; }
    return a;
}
bool irreducible(uint64_t f) {  // Ben-Or
    const int d = gf2_deg(f);
    uint64_t xp = 2;
    for (int i = 1; i <= d / 2; i++) {
        xp = gf2_mulmod(xp, xp, f);
        if (gf2_gcd(f, xp ^ 2) != 1) return false;
    }
    return true;
}

Tables g_tables;
std::once_flag g_once;

void build_tables() {
    std::vector<uint64_t> cooked(kLen);
    compute_rng_cooked(cooked.data());
    std::memcpy(g_tables.cooked, cooked.data(), sizeof(g_tables.cooked));
    {  // buzhash32: GenerateHashes(1)
        GoRand r(1, cooked.data());
        std::set<uint32_t> used;
        for (int i = 0; i < 256; i++) {
            uint32_t x = static_cast<uint32_t>(r.int63());
            while (used.count(x)) x = static_cast<uint32_t>(r.int63());
            used.insert(x);
            g_tables.buz[i] = x;
        }
    }
    {  // rabinkarp64: RandomPolynomial(1)
        GoRand r(1, cooked.data());
        uint64_t f = 0;
        for (int tries = 0; tries < 1000000; tries++) {
            uint8_t b[8];
            r.read(b, 8);
            f = 0;
            for (int k = 7; k >= 0; k--) f = (f << 8) | b[k];
            f &= (1ull << 54) - 1;
            f |= (1ull << 53) | 1ull;
            if (irreducible(f)) break;
        }
        g_tables.rk_pol = f;
        const int k = gf2_deg(f);
        g_tables.rk_shift = k - 8;
        uint64_t xw = 1;  // x^(8*63) mod P
        for (int i = 0; i < 8 * (kWindow - 1); i++) {
            xw <<= 1;
            if (gf2_deg(xw) >= k) xw ^= f;
        }
        for (uint64_t b = 0; b < 256; b++) {
            g_tables.rk_out[b] = gf2_mulmod(b, xw, f);
            g_tables.rk_mod[b] = gf2_mod(b << k, f) | (b << k);
        }
    }
}

}  // namespace

const Tables& tables() {
    std::call_once(g_once, build_tables);
    return g_tables;
}

void gorand_read(int64_t seed, uint8_t* p, uint64_t n) {
    GoRand r(seed, tables().cooked);
    r.read(p, n);
}

}  // namespace kcdc
