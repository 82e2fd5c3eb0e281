// ORACLE / TEST INFRASTRUCTURE ONLY: an independent decoder for the S2 stream format that
// Kopia's s2 compressors write (repo/compression/compressor_s2.go:20-23 -> s2.NewWriter of
// github.com/klauspost/compress, not vendored; Go is absent).  Restated from the published
// formats: the Snappy framing format (chunk = type byte, 3-byte little-endian length, payload;
// 0xff stream identifier "sNaPpY" or S2's "S2sTwO"; 0x00 compressed / 0x01 uncompressed data
// with a masked CRC-32C of the uncompressed bytes; 0xfe padding and 0x80-0xfd skippable) and
// the Snappy block format (uvarint length, then literal / copy-1 / copy-2 / copy-4 elements).
// S2's block extensions (repeat offsets) are rejected: the device encoder emits none, so a
// stream that uses one is a bug.  There are no S2 vectors in the reference (its test is a
// round trip, compressor_test.go), so parity is "format, unpinned": every device stream must
// decode here, CRCs included, to the original bytes.
#include <stdint.h>
#include <string.h>

static uint32_t crc32c_tab[256];
static int crc32c_ready;

static void crc32c_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t r = i;
        for (int k = 0; k < 8; k++) r = (r >> 1) ^ (0x82F63B78u & (0u - (r & 1u)));
        crc32c_tab[i] = r;
    }
    crc32c_ready = 1;
}

uint32_t orc_crc32c(const uint8_t* p, int64_t n) {
    if (!crc32c_ready) crc32c_init();
    uint32_t c = 0xFFFFFFFFu;
    for (int64_t i = 0; i < n; i++) c = (c >> 8) ^ crc32c_tab[(c ^ p[i]) & 255u];
    return c ^ 0xFFFFFFFFu;
}

static uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// One Snappy block -> out[0..cap); returns its length or < 0.
static int64_t snappy_block(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
    int64_t i = 0, o = 0;
    uint64_t want = 0;
    for (int shift = 0;; shift += 7) {  // uvarint
        if (i >= n || shift > 28) return -10;
        const uint8_t b = in[i++];
        want |= (uint64_t)(b & 127u) << shift;
        if (!(b & 128u)) break;
    }
    if ((int64_t)want > cap) return -11;
    while (i < n) {
        const uint8_t tag = in[i++];
        uint64_t len, off = 0;
        switch (tag & 3u) {
            case 0: {
                len = (tag >> 2) + 1u;
                if (len > 60) {
                    const int nb = (int)len - 60;  // 1..4 length bytes
                    if (i + nb > n) return -12;
                    len = 0;
                    for (int k = 0; k < nb; k++) len |= (uint64_t)in[i + k] << (8 * k);
                    len += 1;
                    i += nb;
                }
                if (i + (int64_t)len > n || o + (int64_t)len > (int64_t)want) return -13;
                memcpy(out + o, in + i, len);
                i += (int64_t)len;
                o += (int64_t)len;
                continue;
            }
            case 1:
                if (i >= n) return -14;
                len = 4u + ((tag >> 2) & 7u);
                off = ((uint64_t)(tag >> 5) << 8) | in[i++];
                break;
            case 2:
                if (i + 2 > n) return -14;
                len = 1u + (tag >> 2);
                off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
                i += 2;
                break;
            default:
                if (i + 4 > n) return -14;
                len = 1u + (tag >> 2);
                off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8) | ((uint64_t)in[i + 2] << 16) |
                      ((uint64_t)in[i + 3] << 24);
                i += 4;
                break;
        }
        if (off == 0 || (int64_t)off > o) return -15;  // S2 repeat codes are not expected
        if (o + (int64_t)len > (int64_t)want) return -16;
        for (uint64_t k = 0; k < len; k++, o++) out[o] = out[o - (int64_t)off];
    }
    return o == (int64_t)want ? o : -17;
}

// A whole framed stream -> out; returns the decoded length or a negative error.
int64_t orc_s2_decode(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
    int64_t i = 0, o = 0;
    int seen_id = 0;
    while (i < n) {
        if (i + 4 > n) return -1;
        const uint8_t type = in[i];
        const int64_t len = (int64_t)in[i + 1] | ((int64_t)in[i + 2] << 8) | ((int64_t)in[i + 3] << 16);
        const uint8_t* p = in + i + 4;
        if (i + 4 + len > n) return -2;
        i += 4 + len;
        if (type == 0xffu) {
            if (len != 6 || (memcmp(p, "S2sTwO", 6) != 0 && memcmp(p, "sNaPpY", 6) != 0)) return -3;
            seen_id = 1;
            continue;
        }
        if (!seen_id) return -4;
        if (type == 0x00u || type == 0x01u) {
            if (len < 4) return -5;
            const uint32_t crc = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
            int64_t k;
            if (type == 0x00u) {
                k = snappy_block(p + 4, len - 4, out + o, cap - o);
                if (k < 0) return k;
            } else {
                k = len - 4;
                if (o + k > cap) return -6;
                memcpy(out + o, p + 4, k);
            }
            if (mask_crc(orc_crc32c(out + o, k)) != crc) return -7;
            o += k;
        } else if (type >= 0x02u && type <= 0x7fu) {
            return -8;  // reserved unskippable
        }  // 0x80..0xfe: skippable / padding
    }
    return seen_id ? o : -9;
}
