// ORACLE / TEST INFRASTRUCTURE ONLY: BLAKE3 restated from its published specification (the
// BLAKE3 paper, "BLAKE3: one function, fast everywhere", 2020), for the BLAKE3-256 and
// BLAKE3-256-128 content hashes (repo/hashing/blake3_hashes.go:10-27 -> github.com/zeebo/blake3,
// not vendored; Go is absent).  Streaming form: a chunk state absorbs 64-byte blocks, completed
// chunk chaining values go on a stack that merges pairs whenever the chunk count allows, and the
// finalisation folds the stack right to left (the device kernel instead merges level by level;
// the two constructions must agree).  Pinned by published BLAKE3 vectors (tests/test_hash_oracle.py).
#include <stdint.h>
#include <string.h>

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const int PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8, KEYED_HASH = 16, DERIVE_CTX = 32, DERIVE_MAT = 64 };

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void gmix(uint32_t* v, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    v[a] += v[b] + x; v[d] = rotr(v[d] ^ v[a], 16);
    v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 12);
    v[a] += v[b] + y; v[d] = rotr(v[d] ^ v[a], 8);
    v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 7);
}

// compression: returns the 16-word state; the chaining value is its first 8 words
static void compress(const uint32_t cv[8], const uint8_t block[64], uint64_t ctr, uint32_t blen, uint32_t flags,
                     uint32_t out[16]) {
    uint32_t m[16], v[16], t[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) | ((uint32_t)block[4 * i + 2] << 16) |
               ((uint32_t)block[4 * i + 3] << 24);
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = IV[i];
    v[12] = (uint32_t)ctr; v[13] = (uint32_t)(ctr >> 32); v[14] = blen; v[15] = flags;
    for (int r = 0; r < 7; r++) {
        gmix(v, 0, 4, 8, 12, m[0], m[1]);   gmix(v, 1, 5, 9, 13, m[2], m[3]);
        gmix(v, 2, 6, 10, 14, m[4], m[5]);  gmix(v, 3, 7, 11, 15, m[6], m[7]);
        gmix(v, 0, 5, 10, 15, m[8], m[9]);  gmix(v, 1, 6, 11, 12, m[10], m[11]);
        gmix(v, 2, 7, 8, 13, m[12], m[13]); gmix(v, 3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) { out[i] = v[i] ^ v[i + 8]; out[i + 8] = v[i + 8] ^ cv[i]; }
}

typedef struct {
    uint32_t key[8], flags;
    uint32_t cv[8];          // current chunk
    uint64_t chunk;          // its counter
    uint8_t buf[64];
    uint32_t buflen, blocks; // bytes in buf, blocks compressed in this chunk
    uint32_t stack[54][8];
    int depth;
} hasher;

static void init(hasher* h, const uint32_t key[8], uint32_t flags) {
    memset(h, 0, sizeof *h);
    memcpy(h->key, key, 32);
    memcpy(h->cv, key, 32);
    h->flags = flags;
}

static void parent_cv(const hasher* h, const uint32_t l[8], const uint32_t r[8], uint32_t flags, uint32_t out[8]) {
    uint8_t blk[64];
    uint32_t o[16];
    for (int i = 0; i < 8; i++)
        for (int k = 0; k < 4; k++) { blk[4 * i + k] = (uint8_t)(l[i] >> (8 * k)); blk[32 + 4 * i + k] = (uint8_t)(r[i] >> (8 * k)); }
    compress(h->key, blk, 0, 64, h->flags | PARENT | flags, o);
    memcpy(out, o, 32);
}

static void update(hasher* h, const uint8_t* p, int64_t n) {
    while (n > 0) {
        if (h->buflen == 64) {  // a full buffered block and more input: it is not the message's last
            uint32_t o[16];
            if (h->blocks == 15) {  // the chunk's 16th block: finish the chunk, push, merge
                uint32_t cv[8];
                compress(h->cv, h->buf, h->chunk, 64, h->flags | CHUNK_END, o);
                memcpy(cv, o, 32);
                for (uint64_t total = h->chunk + 1; (total & 1) == 0; total >>= 1) {
                    parent_cv(h, h->stack[h->depth - 1], cv, 0, cv);
                    h->depth--;
                }
                memcpy(h->stack[h->depth++], cv, 32);
                h->chunk++;
                memcpy(h->cv, h->key, 32);
                h->blocks = 0;
            } else {
                compress(h->cv, h->buf, h->chunk, 64, h->flags | (h->blocks == 0 ? CHUNK_START : 0), o);
                memcpy(h->cv, o, 32);
                h->blocks++;
            }
            h->buflen = 0;
        }
        const uint32_t k = (uint32_t)(n < (int64_t)(64 - h->buflen) ? n : (int64_t)(64 - h->buflen));
        memcpy(h->buf + h->buflen, p, k);
        h->buflen += k;
        p += k;
        n -= k;
    }
}

static void finish(hasher* h, uint8_t out[32]) {
    uint32_t o[16], cv[8];
    const uint32_t fl = h->flags | (h->blocks == 0 ? CHUNK_START : 0) | CHUNK_END;
    uint8_t pad[64] = {0};  // the final block, zero padded
    memcpy(pad, h->buf, h->buflen);
    if (h->depth == 0) {
        compress(h->cv, pad, h->chunk, h->buflen, fl | ROOT, o);
    } else {
        compress(h->cv, pad, h->chunk, h->buflen, fl, o);
        memcpy(cv, o, 32);
        for (int d = h->depth - 1; d >= 0; d--) {
            if (d == 0) {
                uint8_t blk[64];
                for (int i = 0; i < 8; i++)
                    for (int k = 0; k < 4; k++) {
                        blk[4 * i + k] = (uint8_t)(h->stack[0][i] >> (8 * k));
                        blk[32 + 4 * i + k] = (uint8_t)(cv[i] >> (8 * k));
                    }
                compress(h->key, blk, 0, 64, h->flags | PARENT | ROOT, o);
            } else {
                parent_cv(h, h->stack[d], cv, 0, cv);
            }
        }
    }
    for (int i = 0; i < 8; i++)
        for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(o[i] >> (8 * k));
}

static void words(const uint8_t* b, uint32_t w[8]) {
    for (int i = 0; i < 8; i++)
        w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}

// key == NULL: the plain hash; else the keyed hash under the 32-byte key.  32-byte output.
void orc_blake3(const uint8_t* key, const uint8_t* msg, int64_t n, uint8_t* out) {
    hasher h;
    uint32_t kw[8];
    if (key) { words(key, kw); init(&h, kw, KEYED_HASH); } else init(&h, IV, 0);
    update(&h, msg, n);
    finish(&h, out);
}

// derive_key(context, material) -> 32 bytes
void orc_blake3_derive_key(const char* context, const uint8_t* material, int64_t n, uint8_t* out) {
    hasher h;
    uint8_t ck[32];
    uint32_t kw[8];
    init(&h, IV, DERIVE_CTX);
    update(&h, (const uint8_t*)context, (int64_t)strlen(context));
    finish(&h, ck);
    words(ck, kw);
    init(&h, kw, DERIVE_MAT);
    update(&h, material, n);
    finish(&h, out);
}
