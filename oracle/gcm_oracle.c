/* ORACLE / TEST INFRASTRUCTURE ONLY: GHASH (NIST SP 800-38D §6.4) in C for the test suite's
 * large AES256-GCM-HMAC-SHA256 chunks, where the pure-Python GHASH of oracle/aesgcm.py is too
 * slow.  Same 4-bit table method as aesgcm.ghash (tests/test_aesgcm_oracle.py checks the two
 * agree and pins aesgcm against the published GCM vectors).  Never linked by the product. */
#include <stdint.h>
#include <string.h>

typedef struct { uint64_t hi, lo; } be128;  /* big-endian halves: bit 63 of hi = x^0 */

static be128 load(const uint8_t* p) {
    be128 r = {0, 0};
    for (int i = 0; i < 8; i++) r.hi = (r.hi << 8) | p[i];
    for (int i = 8; i < 16; i++) r.lo = (r.lo << 8) | p[i];
    return r;
}

static be128 mulx(be128 v) {
    const uint64_t red = (v.lo & 1u) ? 0xE100000000000000ull : 0;
    v.lo = (v.lo >> 1) | (v.hi << 63);
    v.hi = (v.hi >> 1) ^ red;
    return v;
}

/* out = GHASH_H(data), data = nblocks 16-byte blocks (already padded). */
void oracle_ghash(const uint8_t* h16, const uint8_t* data, uint64_t nblocks, uint8_t* out16) {
    static be128 p[128], tab[32][16];
    be128 v = load(h16);
    for (int i = 0; i < 128; i++) { p[i] = v; v = mulx(v); }
    for (int k = 0; k < 32; k++)
        for (int n = 0; n < 16; n++) {
            be128 z = {0, 0};
            for (int t = 0; t < 4; t++)
                if ((n >> t) & 1) { z.hi ^= p[127 - 4 * k - t].hi; z.lo ^= p[127 - 4 * k - t].lo; }
            tab[k][n] = z;
        }
    be128 x = {0, 0};
    for (uint64_t b = 0; b < nblocks; b++) {
        const be128 d = load(data + 16 * b);
        x.hi ^= d.hi;
        x.lo ^= d.lo;
        be128 z = {0, 0};
        for (int k = 0; k < 16; k++) {
            const be128 e = tab[k][(x.lo >> (4 * k)) & 15], f = tab[16 + k][(x.hi >> (4 * k)) & 15];
            z.hi ^= e.hi ^ f.hi;
            z.lo ^= e.lo ^ f.lo;
        }
        x = z;
    }
    for (int i = 0; i < 8; i++) { out16[i] = (uint8_t)(x.hi >> (56 - 8 * i)); out16[8 + i] = (uint8_t)(x.lo >> (56 - 8 * i)); }
}
