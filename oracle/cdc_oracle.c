/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called
 * from the product library (kopia_amd/libkcdc.so).  Used by tests/ as the
 * parity checker and by bench.py's cpu_baseline leg as the "port" CPU baseline.
 *
 * Plain-C restatement of Kopia's CDC splitters, following the reference loop
 * structure line by line (including the min-size fast path), so that timing it
 * is a fair stand-in for the Go splitter (Go is not installed):
 *
 *   buzhash32Splitter.NextSplitPoint   repo/splitter/splitter_buzhash32.go:26-67
 *   rabinKarp64Splitter.NextSplitPoint repo/splitter/splitter_rabinkarp64.go:26-67
 *   fixedSplitter.NextSplitPoint       repo/splitter/splitter_fixed.go:15-26
 *   Reset (64-zero window)             splitter_buzhash32.go:20-24, splitter_rabinkarp64.go:20-24
 *   rollinghash Roll/Sum32/Sum64       github.com/chmduquesne/rollinghash v4.0.0 (go.mod:13; not vendored)
 *   Go math/rand rngSource/Read        (Go stdlib; restated in oracle/gorand.py, tables passed in)
 *
 * Tables (buzhash byte hashes, Rabin out/mod tables, Go rngCooked) are produced
 * by oracle/gorand.py + oracle/rollinghash.py and passed in by the caller.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define WINDOW 64

/* ------------------------------------------------------------------ tables */
static uint32_t g_buz[256];
static uint64_t g_rk_out[256];
static uint64_t g_rk_mod[256];
static int g_rk_shift = 45;

void orc_set_tables(const uint32_t* buz, const uint64_t* rk_out, const uint64_t* rk_mod, int rk_shift) {
    memcpy(g_buz, buz, sizeof g_buz);
    memcpy(g_rk_out, rk_out, sizeof g_rk_out);
    memcpy(g_rk_mod, rk_mod, sizeof g_rk_mod);
    g_rk_shift = rk_shift;
}

/* ---------------------------------------------------------------- splitter */
enum { K_FIXED = 0, K_BUZ = 1, K_RK = 2 };

typedef struct {
    int kind;
    /* fixed */
    int64_t cur, chunk_length;
    /* rolling */
    uint8_t window[WINDOW];
    int oldest;
    uint32_t sum32;
    uint64_t val64;
    uint64_t mask;
    int64_t count, min_size, max_size;
} orc_splitter;

static inline uint32_t rotl32(uint32_t x, unsigned k) {
    k &= 31u;
    return k ? (x << k) | (x >> (32u - k)) : x;
}

void orc_reset(orc_splitter* s) {
    if (s->kind == K_FIXED) { s->cur = 0; return; }
    memset(s->window, 0, WINDOW);  /* Write(make([]byte, 64)) */
    s->oldest = 0;
    s->sum32 = 0;   /* buzhash of 64 zeros = 0 (each rotation of T[0] twice) */
    s->val64 = 0;   /* rabin of 64 zeros = 0 */
    s->count = 0;
}

void orc_init(orc_splitter* s, int kind, int64_t size) {
    memset(s, 0, sizeof *s);
    s->kind = kind;
    if (kind == K_FIXED) { s->chunk_length = size; return; }
    /* newBuzHash32SplitterFactory :73-86 / newRabinKarp64SplitterFactory :73-83 */
    s->mask = (uint64_t)(size - 1);
    s->max_size = size * 2;
    s->min_size = size / 2;
    orc_reset(s);
}

orc_splitter* orc_new(int kind, int64_t size) {
    orc_splitter* s = (orc_splitter*)malloc(sizeof *s);
    orc_init(s, kind, size);
    return s;
}
void orc_free(orc_splitter* s) { free(s); }

static inline void roll_buz(orc_splitter* s, uint8_t c) {
    uint8_t leave = s->window[s->oldest];
    s->window[s->oldest] = c;
    if (++s->oldest >= WINDOW) s->oldest = 0;
    s->sum32 = rotl32(s->sum32, 1) ^ rotl32(g_buz[leave], WINDOW % 32) ^ g_buz[c];
}

static inline void roll_rk(orc_splitter* s, uint8_t c) {
    uint8_t leave = s->window[s->oldest];
    s->window[s->oldest] = c;
    if (++s->oldest >= WINDOW) s->oldest = 0;
    uint64_t v = s->val64 ^ g_rk_out[leave];
    unsigned idx = (unsigned)(v >> g_rk_shift) & 0xFFu;
    v = (v << 8) | c;
    s->val64 = v ^ g_rk_mod[idx];
}

/* NextSplitPoint: returns n in 1..len (cut after n bytes) or -1. */
int64_t orc_next(orc_splitter* s, const uint8_t* b, int64_t len) {
    if (s->kind == K_FIXED) {  /* splitter_fixed.go:15-26 */
        int64_t n = s->chunk_length - s->cur;
        if (len < n) { s->cur += len; return -1; }
        s->cur = 0;
        return n;
    }
    int64_t fast = 0;
    int64_t left = s->min_size - s->count - 1;
    if (left > 0) {  /* :29-40 until minSize, only hash the last 64 bytes */
        fast = left < len ? left : len;
        int64_t i = fast - WINDOW > 0 ? fast - WINDOW : 0;
        if (s->kind == K_BUZ) for (; i < fast; i++) roll_buz(s, b[i]);
        else                  for (; i < fast; i++) roll_rk(s, b[i]);
        s->count += fast;
        b += fast;
        len -= fast;
    }
    left = s->max_size - s->count;
    if (left > 0) {  /* :42-58 */
        int64_t fp = left < len ? left : len;
        if (s->kind == K_BUZ) {
            uint32_t m = (uint32_t)s->mask;
            for (int64_t i = 0; i < fp; i++) {
                roll_buz(s, b[i]);
                s->count++;
                if ((s->sum32 & m) == 0) { s->count = 0; return fast + i + 1; }
            }
        } else {
            for (int64_t i = 0; i < fp; i++) {
                roll_rk(s, b[i]);
                s->count++;
                if ((s->val64 & s->mask) == 0) { s->count = 0; return fast + i + 1; }
            }
        }
        fast += fp;
    }
    if (s->count >= s->max_size) { s->count = 0; return fast; }  /* :60-64 */
    return -1;
}

int64_t orc_max_segment(const orc_splitter* s) {
    return s->kind == K_FIXED ? s->chunk_length : s->max_size;
}

/* ------------------------------------------------------------------ feeders
 * Return chunk END offsets (absolute, 1-based "after byte n") as reported by
 * the splitter; the trailing remainder is NOT appended (it is not a split
 * point).  Modes mirror repo/splitter/splitter_test.go:
 *   0 getSplitPoints (:118-143)  1 getSplitPointsByteByByte (:145-171)
 *   2 getSplitPointsRandomSlices (:173-211; slice sizes 1..1000 from a
 *     splitmix64 sequence seeded by `seed` — the reference uses the global
 *     Go rand, whose values do not matter: only slicing invariance does). */
static inline uint64_t splitmix_next(uint64_t* st) {
    uint64_t z = (*st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int64_t orc_feed(orc_splitter* s, const uint8_t* data, int64_t n, int mode, uint64_t seed,
                 int64_t* cuts, int64_t cap) {
    int64_t cnt = 0;
    if (mode == 0) {
        int64_t pos = 0;
        while (pos < n) {
            int64_t k = orc_next(s, data + pos, n - pos);
            if (k < 0) break;
            pos += k;
            if (cnt < cap) cuts[cnt] = pos;
            cnt++;
        }
    } else if (mode == 1) {
        for (int64_t i = 0; i < n; i++) {
            if (orc_next(s, data + i, 1) == -1) continue;
            if (cnt < cap) cuts[cnt] = i + 1;
            cnt++;
        }
    } else {
        uint64_t st = seed;
        for (int64_t i = 0; i < n;) {
            int64_t num = (int64_t)(splitmix_next(&st) % 1000u) + 1;
            if (i + num > n) num = n - i;
            int64_t k = orc_next(s, data + i, num);
            if (k == -1) { i += num; continue; }
            if (cnt < cap) cuts[cnt] = i + k;
            cnt++;
            i += k;
        }
    }
    return cnt;
}

/* Whole-stream split with the trailing remainder appended, i.e. the list of
 * chunk end offsets whose last entry is n (cli/command_benchmark_splitters.go:88-101).
 * Empty stream -> 0 entries. */
int64_t orc_split_stream(int kind, int64_t size, const uint8_t* data, int64_t n, int64_t* cuts, int64_t cap) {
    orc_splitter s;
    orc_init(&s, kind, size);
    int64_t cnt = 0, pos = 0;
    while (pos < n) {
        int64_t k = orc_next(&s, data + pos, n - pos);
        pos = k < 0 ? n : pos + k;  /* k < 0: trailing remainder is one more chunk */
        if (cnt < cap) cuts[cnt] = pos;
        cnt++;
    }
    return cnt;
}

/* ------------------------------------------------------- Go math/rand bytes */
void orc_gorand_read(int64_t seed, const uint64_t* cooked, uint8_t* out, int64_t n) {
    /* rng.go Seed (shifts 40/20, cooked XOR) + rand.go read (7 bytes per Int63) */
    const int64_t M = 2147483647;
    uint64_t vec[607];
    int64_t s = seed % M;
    if (s < 0) s += M;
    if (s == 0) s = 89482311;
    int32_t x = (int32_t)s;
#define SEEDRAND(v) do { int32_t hi_ = (v) / 44488, lo_ = (v) % 44488; (v) = 48271 * lo_ - 3399 * hi_; if ((v) < 0) (v) += 2147483647; } while (0)
    for (int i = -20; i < 607; i++) {
        SEEDRAND(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 40;
            SEEDRAND(x);
            u ^= (uint64_t)(int64_t)x << 20;
            SEEDRAND(x);
            u ^= (uint64_t)(int64_t)x;
            u ^= cooked[i];
            vec[i] = u;
        }
    }
#undef SEEDRAND
    int tap = 0, feed = 607 - 273;
    int pos = 0;
    uint64_t val = 0;
    for (int64_t i = 0; i < n; i++) {
        if (pos == 0) {
            if (--tap < 0) tap += 607;
            if (--feed < 0) feed += 607;
            uint64_t y = vec[feed] + vec[tap];
            vec[feed] = y;
            val = y & 0x7FFFFFFFFFFFFFFFull;
            pos = 7;
        }
        out[i] = (uint8_t)val;
        val >>= 8;
        pos--;
    }
}

/* ------------------------------------------------- counter PRNG stream data
 * Synthetic stream bytes for configs 2-5 (BASELINE.json): 64-bit word j of
 * stream `sid` = mix64(key + (j+1)*golden), key = mix64(seed ^ mix64(sid + c)).
 * The GPU generator in kopia_amd/csrc/kcdc_kernels.hip computes the same words. */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_gen_stream(uint64_t seed, uint64_t sid, uint64_t offset, uint8_t* out, int64_t n) {
    uint64_t key = mix64(seed ^ mix64(sid + 0x632BE59BD9B4E019ull));
    int64_t i = 0;
    while (i < n) {
        uint64_t pos = offset + (uint64_t)i;
        uint64_t j = pos >> 3;
        uint64_t w = mix64(key + (j + 1) * 0x9E3779B97F4A7C15ull);
        unsigned b = (unsigned)(pos & 7u);
        for (; b < 8 && i < n; b++, i++) out[i] = (uint8_t)(w >> (8 * b));
    }
}

/* ---------------------------------------------------- threaded batch split */
typedef struct {
    int kind; int64_t size;
    const uint8_t* const* ptrs; const int64_t* lens;
    int64_t* cuts; const int64_t* cut_base; const int64_t* caps; int64_t* counts;
    int64_t nstreams;
    /* prng mode */
    int prng; uint64_t seed; const uint64_t* sids; int64_t stream_len;
    int64_t next; pthread_mutex_t mu;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    uint8_t* buf = NULL;
    if (j->prng) buf = (uint8_t*)malloc((size_t)j->stream_len);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t i = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->nstreams) break;
        const uint8_t* d;
        int64_t n;
        if (j->prng) {
            orc_gen_stream(j->seed, j->sids[i], 0, buf, j->stream_len);
            d = buf; n = j->stream_len;
        } else {
            d = j->ptrs[i]; n = j->lens[i];
        }
        j->counts[i] = orc_split_stream(j->kind, j->size, d, n, j->cuts + j->cut_base[i], j->caps[i]);
    }
    free(buf);
    return NULL;
}

static void run_batch(batch_job* j, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_mutex_init(&j->mu, NULL);
    j->next = 0;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j->mu);
}

void orc_split_batch(int kind, int64_t size, const uint8_t* const* ptrs, const int64_t* lens, int64_t nstreams,
                     int64_t* cuts, const int64_t* cut_base, const int64_t* caps, int64_t* counts, int nthreads) {
    batch_job j;
    memset(&j, 0, sizeof j);
    j.kind = kind; j.size = size; j.ptrs = ptrs; j.lens = lens; j.cuts = cuts;
    j.cut_base = cut_base; j.caps = caps; j.counts = counts; j.nstreams = nstreams;
    run_batch(&j, nthreads);
}

void orc_split_prng_streams(int kind, int64_t size, uint64_t seed, const uint64_t* sids, int64_t nstreams,
                            int64_t stream_len, int64_t* cuts, const int64_t* cut_base, const int64_t* caps,
                            int64_t* counts, int nthreads) {
    batch_job j;
    memset(&j, 0, sizeof j);
    j.kind = kind; j.size = size; j.prng = 1; j.seed = seed; j.sids = sids; j.stream_len = stream_len;
    j.cuts = cuts; j.cut_base = cut_base; j.caps = caps; j.counts = counts; j.nstreams = nstreams;
    run_batch(&j, nthreads);
}

/* Bytes the reference loop actually rolls for one stream given its cut list
 * (SURVEY.md §8d): per chunk [s,e): (e-s) - max(min(min-1, e-s) - 64, 0). */
int64_t orc_rolled_bytes(int64_t min_size, const int64_t* cuts, int64_t ncuts) {
    int64_t s = 0, r = 0;
    for (int64_t i = 0; i < ncuts; i++) {
        int64_t len = cuts[i] - s;
        int64_t fastp = min_size - 1 < len ? min_size - 1 : len;
        int64_t skip = fastp - WINDOW > 0 ? fastp - WINDOW : 0;
        r += len - skip;
        s = cuts[i];
    }
    return r;
}
